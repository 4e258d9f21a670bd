%% vmq_reg_gpu_view — a vmq_reg_view backed by libvmqgpu (MI355X).
%%
%% Drop-in for vmq_reg_trie (apps/vmq_server/src/vmq_reg_trie.erl): same
%% exports for the view behaviour (vmq_reg_view.erl:20-27) and the registry
%% supervisor (vmq_reg_sup.erl:86-87, 128-129), same event source
%% (vmq_reg:subscribe_subscriber_changes/0, vmq_reg.erl:618-619), same
%% initial fold (vmq_reg:fold_subscriptions/2, vmq_reg_trie.erl:145-149) and
%% the same event replay after `subscribers_loaded` (:198-205).
%%
%% What changes is where fold/4 is answered.  vmq_reg_trie walks ETS in the
%% caller's process, on every scheduler at once (read_concurrency tables,
%% vmq_reg_trie.erl:136-137); here the callers on each scheduler are
%% collected by that scheduler's batcher (vmq_reg_gpu_batcher, one per
%% scheduler), each batcher matches its batch with one NIF call on a dirty
%% scheduler (vmqg_nif:match/4) — the batchers' calls run in parallel, only
%% the device call itself takes turns — and each caller then runs its
%% FoldFun over its own entries in its own process — FoldFun has side
%% effects (vmq_queue:enqueue, cluster forward, vmq_reg.erl:327-353) and is
%% called exactly as vmq_reg_trie calls it, FoldFun(Entry, SubscriberId,
%% Acc) (vmq_reg_trie.erl:83, 97).  A caller blocks on its own call, so the
%% order of one publisher's publishes is kept (vmq_in_order_delivery_SUITE).
%%
%% This gen_server owns the view: the NIF resource, the batchers, the
%% subscriber-change events (applied as writers: no match reads the tables
%% while an apply changes them) and the initial load.  It never queues a
%% fold request, so no event can delay one.
%%
%% Events are coalesced: vmq_reg_trie applies each subscriber event with a
%% few ETS inserts in its gen_server (vmq_reg_trie.erl:198-210, 240-251); here
%% an apply is a write-lock section plus a table patch upload, so on each
%% event the view drains the further subscriber events already in its
%% mailbox (a selective receive with a 0 timeout, up to ?MAX_COALESCE) and
%% applies the group with ONE vmqg_nif:apply_many/2.  The group is applied
%% in arrival order, each event's deletes before its adds, which is what
%% applying the events one after the other does; under load the groups grow
%% with the backlog, so the view keeps up with config D's 100k changes/s.
%%
%% Install: reg_views = [vmq_reg_trie, vmq_reg_gpu_view] (shadow) or
%% default_reg_view = vmq_reg_gpu_view (vmq_server.schema:115-137).  The NIF
%% (c_src/vmqg_nif.c) and priv/libvmqgpu.so come from this repository.
%%
%% Not compiled in this repository's image (no OTP); its C core
%% (c_src/vmqg_batch.c, the batchers' locking protocol included) is compiled
%% and tested (tests/test_nif_layer.py, tools/nif_harness.c).
-module(vmq_reg_gpu_view).
-behaviour(gen_server).
-behaviour(vmq_reg_view).

-export([start_link/0,
         fold/4,
         stats/0]).

%% gen_server callbacks
-export([init/1,
         handle_call/3,
         handle_cast/2,
         handle_info/2,
         terminate/2,
         code_change/3]).

-define(SERVER, ?MODULE).
%% subscriber events applied per vmqg_nif:apply_many/2 at most
-define(MAX_COALESCE, 10000).

-record(state, {ctx,                    % vmqg_nif resource (vmqg_ctx + term tables)
                batchers,               % tuple of vmq_reg_gpu_batcher pids
                event_handler,
                status=init,
                event_queue=queue:new()}).

%%%===================================================================
%%% API
%%%===================================================================
start_link() ->
    gen_server:start_link({local, ?SERVER}, ?MODULE, [], []).

%% vmq_reg_view callback (vmq_reg_view.erl:20-25; called by vmq_reg:publish/5,
%% vmq_reg.erl:260, and vmq_cluster_com:process/2, vmq_cluster_com.erl:156).
fold({MP, _} = SubscriberId, Topic, FoldFun, Acc) when is_list(Topic) ->
    TopicBin = iolist_to_binary(lists:join(<<"/">>, Topic)),
    Batchers = persistent_term:get({?MODULE, batchers}),
    Batcher = element(erlang:system_info(scheduler_id) rem tuple_size(Batchers) + 1, Batchers),
    case gen_server:call(Batcher, {match, MP, TopicBin}, infinity) of
        {ok, Entries} ->
            lists:foldl(fun(Entry, AccAcc) -> FoldFun(Entry, SubscriberId, AccAcc) end,
                        Acc, Entries);
        {error, Reason} ->
            error({vmq_reg_gpu_view, Reason})
    end.

%% stats/0 as vmq_reg_trie:stats/0 (vmq_reg_trie.erl:101-112):
%% {NrOfSubs + NrOfRemoteSubs, Memory}, memory being the device arena.
stats() ->
    case persistent_term:get({?MODULE, ctx}, undefined) of
        undefined -> {0, 0};
        Ctx -> vmqg_nif:stats(Ctx)
    end.

%%%===================================================================
%%% gen_server callbacks
%%%===================================================================
init([]) ->
    Device = application:get_env(vmq_server, gpu_reg_view_device, 0),
    {ok, Ctx} = vmqg_nif:create(#{device => Device, local_node => node()}),
    persistent_term:put({?MODULE, ctx}, Ctx),
    %% fold/4 batchers, one per scheduler (linked: they die with the view)
    Mode = application:get_env(vmq_server, gpu_reg_view_output, records),
    Batchers = list_to_tuple(
                 [begin {ok, Pid} = vmq_reg_gpu_batcher:start_link(Ctx, Mode), Pid end
                  || _ <- lists:seq(1, erlang:system_info(schedulers))]),
    persistent_term:put({?MODULE, batchers}, Batchers),
    Self = self(),
    spawn_link(
      fun() ->
              %% initialize_trie/2 (vmq_reg_trie.erl:305-316), batched
              ok = vmq_reg:fold_subscriptions(
                     fun({MP, Topic, {SubscriberId, SubInfo, Node}}, ok) ->
                             vmqg_nif:add_init(Ctx, MP, Topic, SubscriberId, SubInfo, Node)
                     end, ok),
              ok = vmqg_nif:flush_init(Ctx),
              Self ! subscribers_loaded
      end),
    EventHandler = vmq_reg:subscribe_subscriber_changes(),
    {ok, #state{ctx=Ctx, batchers=Batchers, event_handler=EventHandler}}.

handle_call({event, Event}, _From, State) ->
    %% used only for testing/microbenchmarking, as vmq_reg_trie.erl:167-170
    {reply, ok, handle_events([Event], State)};
handle_call(_Request, _From, State) ->
    {reply, ok, State}.

handle_cast(_Msg, State) ->
    {noreply, State}.

handle_info(subscribers_loaded, #state{event_queue=Q} = State) ->
    %% the events queued during the initial load, replayed in order (:198-205)
    State1 = replay(queue:to_list(Q), State#state{status=ready}),
    {Subs, _} = stats(),
    lager:info("loaded ~p subscriptions into ~p", [Subs, ?MODULE]),
    {noreply, State1#state{event_queue=undefined}};
handle_info(Event, #state{status=init, event_queue=Q} = State) ->
    {noreply, State#state{event_queue=queue:in(Event, Q)}};
handle_info(Event, State) ->
    {noreply, handle_events([Event | drain_events(?MAX_COALESCE - 1, [])], State)}.

terminate(_Reason, _State) ->
    persistent_term:erase({?MODULE, batchers}),
    persistent_term:erase({?MODULE, ctx}),
    ok.

code_change(_OldVsn, State, _Extra) ->
    {ok, State}.

%%%===================================================================
%%% Internal functions
%%%===================================================================

%% The subscriber events already in the mailbox, oldest first (a selective
%% receive keeps their relative order; other messages stay where they are).
%% The shapes are the metadata events vmq_subscriber_db's handler converts
%% (vmq_subscriber_db.erl:56-71).
drain_events(0, Acc) ->
    lists:reverse(Acc);
drain_events(N, Acc) ->
    receive
        {updated, {vmq, subscriber}, _, _, _} = E -> drain_events(N - 1, [E | Acc]);
        {deleted, {vmq, subscriber}, _, _} = E -> drain_events(N - 1, [E | Acc])
    after 0 ->
        lists:reverse(Acc)
    end.

replay([], State) ->
    State;
replay(Events, State) ->
    {Group, Rest} = case length(Events) > ?MAX_COALESCE of
                        true -> lists:split(?MAX_COALESCE, Events);
                        false -> {Events, []}
                    end,
    replay(Rest, handle_events(Group, State)).

%% handle_event/2 (vmq_reg_trie.erl:240-251) for a group of events: the same
%% diff per event, the same order (deletes, then adds; event after event);
%% the NIF turns the whole group into one vmqg_apply_ops.  If the group is
%% refused (a malformed change: nothing was applied) the events are applied
%% one by one, so only the offending one fails, as it would alone.
handle_events(Events, #state{ctx=Ctx, event_handler=Handler} = State) ->
    AllChanges = lists:foldr(fun(E, Acc) ->
                                     case event_changes(Handler, E) of
                                         ignore -> Acc;
                                         C -> [C | Acc]
                                     end
                             end, [], Events),
    case AllChanges of
        [] ->
            ok;
        Changes ->
            case vmqg_nif:apply_many(Ctx, Changes) of
                ok ->
                    ok;
                {error, _} ->
                    lists:foreach(fun({SubscriberId, Ch}) ->
                                          ok = vmqg_nif:apply(Ctx, SubscriberId, Ch)
                                  end, Changes)
            end
    end,
    State.

%% {SubscriberId, [{Kind, Topic, SubInfo, Node}]} of one event, or ignore
event_changes(Handler, Event) ->
    case Handler(Event) of
        {delete, SubscriberId, Subscriptions} ->
            Removed = vmq_subscriber:get_changes(Subscriptions),
            {SubscriberId, changes(del, Removed)};
        {update, SubscriberId, OldValue, NewValue} ->
            {ToRemove, ToAdd} = vmq_subscriber:get_changes(OldValue, NewValue),
            {SubscriberId, changes(del, ToRemove) ++ changes(add, ToAdd)};
        ignore ->
            ignore
    end.

%% [{Node, [{Topic, SubInfo}]}] (vmq_subscriber:get_changes/1,2) in the
%% order vmq_subscriber:fold/3 (vmq_subscriber.erl:184-196) visits it ->
%% [{Kind, Topic, SubInfo, Node}]
changes(Kind, Changes) ->
    lists:reverse(
      vmq_subscriber:fold(fun({Topic, SubInfo, Node}, Acc) -> [{Kind, Topic, SubInfo, Node} | Acc] end,
                          [], Changes)).
