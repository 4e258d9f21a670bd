%% vmq_reg_gpu_batcher — one of vmq_reg_gpu_view's fold/4 batchers.
%%
%% vmq_reg_trie:fold/4 runs in every caller's process, on every scheduler,
%% against read_concurrency ETS tables (vmq_reg_trie.erl:59-66, 136-137).
%% The GPU view keeps that concurrency: vmq_reg_gpu_view starts one batcher
%% per scheduler, a caller goes to the batcher of the scheduler it runs on,
%% and each batcher turns the fold requests queued in its mailbox into one
%% vmqg_nif:match/4 call on a dirty CPU scheduler.  Those calls run in
%% parallel — topic preparation and result terms under the view's read lock,
%% only the device call itself taking turns (c_src/vmqg_batch.c,
%% vmqgb_view_*) — so the batchers add up instead of queueing behind one
%% process.
%%
%% Liveness: a batcher only ever receives fold requests, and every callback
%% returns a 0 timeout while requests are pending, so a pending request is
%% flushed as soon as the mailbox is drained, whatever arrives in between.
-module(vmq_reg_gpu_batcher).
-behaviour(gen_server).

-export([start_link/2]).
-export([init/1,
         handle_call/3,
         handle_cast/2,
         handle_info/2,
         terminate/2,
         code_change/3]).

%% a batch goes to the GPU when it holds this many publishes, or when the
%% batcher's mailbox has no more fold requests queued behind it
-define(MAX_BATCH, 4096).

-record(state, {ctx,           % vmqg_nif view resource
                batch,         % this batcher's vmqg_nif batch resource
                mode=ranges,   % ranges | records (app env gpu_reg_view_output)
                pending=[],    % [{From, MP, Topic}], newest first (Topic: the word list fold/4 got)
                npending=0}).

start_link(Ctx, Mode) ->
    gen_server:start_link(?MODULE, [Ctx, Mode], []).

init([Ctx, Mode]) ->
    {ok, Batch} = vmqg_nif:batch_new(Ctx),
    {ok, #state{ctx=Ctx, batch=Batch, mode=Mode}}.

handle_call({match, MP, Topic}, From, #state{pending=P, npending=N} = State) ->
    State1 = State#state{pending=[{From, MP, Topic} | P], npending=N + 1},
    case N + 1 >= ?MAX_BATCH of
        true -> noreply(flush(State1));
        false -> noreply(State1)
    end;
handle_call(_Request, _From, State) ->
    reply(ok, State).

handle_cast(_Msg, State) ->
    noreply(State).

handle_info(timeout, State) ->
    noreply(flush(State));
handle_info(_Info, State) ->
    noreply(State).

terminate(_Reason, #state{pending=P}) ->
    [gen_server:reply(From, {error, shutdown}) || {From, _, _} <- P],
    ok.

code_change(_OldVsn, State, _Extra) ->
    {ok, State}.

%%%===================================================================
%%% Internal functions
%%%===================================================================

%% a 0 timeout whenever requests are pending: flushed once the mailbox is empty
noreply(#state{npending=0} = State) -> {noreply, State};
noreply(State) -> {noreply, State, 0}.

reply(Reply, #state{npending=0} = State) -> {reply, Reply, State};
reply(Reply, State) -> {reply, Reply, State, 0}.

%% One NIF call for every queued fold request (dirty CPU scheduler: word
%% lookups, the GPU match, term construction), then one reply per caller.
flush(#state{pending=[]} = State) ->
    State;
flush(#state{ctx=Ctx, batch=B, mode=Mode, pending=P} = State) ->
    Batch = lists:reverse(P),
    Results = vmqg_nif:match(Ctx, B, [{MP, T} || {_, MP, T} <- Batch], Mode),
    lists:foreach(fun({{From, _, _}, Res}) -> gen_server:reply(From, Res) end,
                  lists:zip(Batch, Results)),
    State#state{pending=[], npending=0}.
