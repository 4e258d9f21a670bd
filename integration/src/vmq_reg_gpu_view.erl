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
%% subscriber-change events (applied as the one writer: the batchers never
%% wait for an apply, an apply's host half runs beside their device rounds,
%% and every fold answers from the tables of one epoch) and the initial load.
%% It never queues a fold request, so no event can delay one.
%%
%% Events are coalesced: vmq_reg_trie applies each subscriber event with a
%% few ETS inserts in its gen_server (vmq_reg_trie.erl:198-210, 240-251); here
%% an apply is a host-table update plus a patch upload, so the view applies
%% a window of events with ONE vmqg_nif:apply_many/2: from the first event,
%% the subscriber events that arrive within ?WINDOW_MS ms or until there are
%% ?WINDOW_EVENTS of them, plus whatever backlog is already queued (up to
%% ?MAX_COALESCE; selective receive).  The group is applied in arrival order,
%% each event's deletes before its adds, which is what applying the events
%% one after the other does; config D's 100k changes/s become ~100 applies/s
%% of 1,000 events, each visible to folds within a few ms.
%%
%% Install: reg_views = [vmq_reg_trie, vmq_reg_gpu_view] (shadow) or
%% default_reg_view = vmq_reg_gpu_view (vmq_server.schema:115-137).  The NIF
%% (c_src/vmqg_nif.c) and priv/libvmqgpu.so come from this repository.
%%
%% OTP: the reference supports 18.0+ and is tested on 19.3, 20.3 and 21.1
%% (rebar.config:2, .travis.yml).  This module and the batcher use only
%% gen_server, ets (named table, read_concurrency), queue, lists:foldl /
%% foldr / reverse / split / zip, application:get_env/3,
%% erlang:system_info(scheduler_id | schedulers), spawn_link, selective
%% receive, os:timestamp/0 — all older than OTP 18 (no persistent_term, no
%% lists:join, no maps-only API).  The NIF reschedules itself onto dirty schedulers when
%% the emulator has them (vmqg_nif.c, load/3).
%%
%% Not compiled in this repository's image (no OTP); its C core
%% (c_src/vmqg_batch.c, the batchers' locking protocol included) is compiled
%% and tested (tests/test_nif_layer.py, tools/nif_harness.c), and the NIF
%% glue runs over an erl_nif test double (tests/c/nif_mock_check.c).
-module(vmq_reg_gpu_view).
-behaviour(gen_server).
-behaviour(vmq_reg_view).

-export([start_link/0,
         fold/4,
         stats/0,
         shadow_stats/0,
         fallbacks/0]).

%% gen_server callbacks
-export([init/1,
         handle_call/3,
         handle_cast/2,
         handle_info/2,
         terminate/2,
         code_change/3]).

-define(SERVER, ?MODULE).
%% subscriber events applied per vmqg_nif:apply_many/2 at most: a backlog
%% goes out in slices of this many (each lands within ~1 ms of host stage, so
%% the first events of a backlog do not wait for the last)
-define(MAX_COALESCE, 1000).
%% the coalescing window: an apply waits at most this long after its first
%% event for more, or until it has this many
-define(WINDOW_MS, 2).
-define(WINDOW_EVENTS, 1000).
%% shadow-compare counters (public: every fold caller bumps them)
-define(SHADOW, vmq_reg_gpu_view_shadow).
%% a fold the device refuses as busy (applies kept rewriting the records its
%% round read) is asked again this many times
-define(MATCH_RETRIES, 3).
%% an apply whose upload failed stays pending in the library; the commit is
%% retried after this many ms (and by the next apply)
-define(COMMIT_RETRY_MS, 100).
%% reclamation of dropped terms / words waits for the batchers' grace periods
%% and runs in the writer: at every apply, and at least this often when
%% subscriptions are quiet (vmqg_nif:commit/1 with nothing pending)
-define(RECLAIM_MS, 1000).

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
%% Topic goes to the NIF as the word list it is (vmq_reg_trie:fold/4 walks it
%% as given, vmq_reg_trie.erl:59-66: a plugin publish is not validated,
%% vmq_reg.erl:572-594) — '+' / '#' words, words holding '/', [] included.
fold(SubscriberId, Topic, FoldFun, Acc) when is_list(Topic) ->
    Entries = entries(SubscriberId, Topic),
    shadow(SubscriberId, Topic, Entries),
    lists:foldl(fun(Entry, AccAcc) -> FoldFun(Entry, SubscriberId, AccAcc) end, Acc, Entries).

%% The FoldFun entries of one publish.  vmq_reg_trie:fold/4 has no failure
%% mode (vmq_reg_trie.erl:59-98), so neither may this: a match the device
%% refuses as busy is asked again; any other refusal (device, nomem) is
%% answered by vmq_reg_trie when it runs beside this view (reg_views =
%% [vmq_reg_trie, vmq_reg_gpu_view]: a CPU copy of the same tables, fed the
%% same events) and counted (fallbacks/0); only a view with no CPU copy
%% raises, as it has no answer to give.
entries(SubscriberId, Topic) ->
    entries(SubscriberId, Topic, ?MATCH_RETRIES).

entries({MP, _} = SubscriberId, Topic, Retries) ->
    case match(MP, Topic) of
        {ok, Entries} -> Entries;
        {error, busy} when Retries > 0 -> entries(SubscriberId, Topic, Retries - 1);
        {error, Reason} -> cpu_fold(SubscriberId, Topic, Reason)
    end.

match(MP, Topic) ->
    Batchers = ets:lookup_element(?MODULE, batchers, 2),
    Batcher = element(erlang:system_info(scheduler_id) rem tuple_size(Batchers) + 1, Batchers),
    gen_server:call(Batcher, {match, MP, Topic}, infinity).

cpu_fold(SubscriberId, Topic, Reason) ->
    case whereis(vmq_reg_trie) of
        undefined ->
            error({vmq_reg_gpu_view, Reason});
        _ ->
            ets:update_counter(?SHADOW, fallbacks, 1),
            Collect = fun(E, _, A) -> [E | A] end,
            lists:reverse(vmq_reg_trie:fold(SubscriberId, Topic, Collect, []))
    end.

%% Shadow compare.  With reg_views = [vmq_reg_trie, vmq_reg_gpu_view] both
%% views receive every subscriber event (vmq_reg_sup.erl:42-47, 86-87), so
%% vmq_reg_trie is a live oracle: app env gpu_reg_view_shadow = N > 0 folds
%% one publish in N through vmq_reg_trie:fold/4 as well and compares the
%% entry multisets (FoldFun argument lists, sorted).  A difference is folded
%% once more on both views before it counts (an event may have reached one
%% view's tables and not yet the other's); mismatches are counted and logged
%% with the topic, and shadow_stats/0 returns {Sampled, Mismatched}.  The
%% caller's own FoldFun always runs over the GPU view's entries.
shadow(SubscriberId, Topic, Entries) ->
    case ets:lookup(?SHADOW, every) of
        [{every, N}] when N > 0 ->
            case rand:uniform(N) of
                1 -> shadow_compare(SubscriberId, Topic, Entries);
                _ -> ok
            end;
        _ ->
            ok
    end.

shadow_compare({MP, _} = SubscriberId, Topic, Entries) ->
    Collect = fun(E, _, A) -> [E | A] end,
    Trie = lists:sort(vmq_reg_trie:fold(SubscriberId, Topic, Collect, [])),
    ets:update_counter(?SHADOW, sampled, 1),
    case lists:sort(Entries) of
        Trie ->
            ok;
        _ ->
            Gpu2 = lists:sort(entries(SubscriberId, Topic)),
            case lists:sort(vmq_reg_trie:fold(SubscriberId, Topic, Collect, [])) of
                Gpu2 ->
                    ok;
                Trie2 ->
                    ets:update_counter(?SHADOW, mismatched, 1),
                    lager:warning("~p: fold of ~p on ~p differs from vmq_reg_trie: ~p entries vs ~p",
                                  [?MODULE, Topic, MP, length(Gpu2), length(Trie2)])
            end
    end.

shadow_stats() ->
    case catch ets:lookup(?SHADOW, sampled) of
        [{sampled, S}] -> {S, ets:lookup_element(?SHADOW, mismatched, 2)};
        _ -> {0, 0}
    end.

%% folds answered by vmq_reg_trie because the device refused them
fallbacks() ->
    case catch ets:lookup_element(?SHADOW, fallbacks, 2) of
        N when is_integer(N) -> N;
        _ -> 0
    end.

%% stats/0 as vmq_reg_trie:stats/0 (vmq_reg_trie.erl:101-112):
%% {NrOfSubs + NrOfRemoteSubs, Memory}, memory being the device arena.  Like
%% vmq_reg_trie's info/2 (:114-118) it answers 0s while the view is down.
stats() ->
    case catch ets:lookup_element(?MODULE, ctx, 2) of
        {'EXIT', _} -> {0, 0};
        Ctx -> vmqg_nif:stats(Ctx)
    end.

%%%===================================================================
%%% gen_server callbacks
%%%===================================================================
init([]) ->
    Device = application:get_env(vmq_server, gpu_reg_view_device, 0),
    %% gpu_reg_view_devices = [D0, D1, ...]: the tables on D0 and a replica of
    %% them on each further GPU (SURVEY §8e); scheduler k's batcher matches
    %% on device k mod N (vmqgb_view_bind in the NIF's batch_new/1)
    Devices = application:get_env(vmq_server, gpu_reg_view_devices, [Device]),
    {ok, Ctx} = vmqg_nif:create(#{device => hd(Devices), devices => Devices, local_node => node()}),
    %% kernel knobs (include/vmqg.h vmqg_set_option), [{Name, Value}]
    lists:foreach(fun({Name, Value}) ->
                          case vmqg_nif:set_option(Ctx, Name, Value) of
                              ok -> ok;
                              {error, R} -> lager:warning("~p: option ~p = ~p refused: ~p", [?MODULE, Name, Value, R])
                          end
                  end, application:get_env(vmq_server, gpu_reg_view_options, [])),
    %% the callers' lookups: a read_concurrency table this process owns
    %% (gone with it), as vmq_reg_trie's tables are (vmq_reg_trie.erl:136-143)
    ?MODULE = ets:new(?MODULE, [named_table, protected, {read_concurrency, true}]),
    true = ets:insert(?MODULE, {ctx, Ctx}),
    ?SHADOW = ets:new(?SHADOW, [named_table, public, {write_concurrency, true}, {read_concurrency, true}]),
    true = ets:insert(?SHADOW, [{every, application:get_env(vmq_server, gpu_reg_view_shadow, 0)},
                                {sampled, 0}, {mismatched, 0}, {fallbacks, 0}]),
    %% fold/4 batchers, one per scheduler (linked: they die with the view)
    %% ranges (the default): the device returns {record off, count} per key and
    %% the entries are built straight from the pinned record table of the
    %% match's epoch; records: each batch gets its own copy of its records first
    Mode = application:get_env(vmq_server, gpu_reg_view_output, ranges),
    Batchers = list_to_tuple(
                 [begin {ok, Pid} = vmq_reg_gpu_batcher:start_link(Ctx, Mode), Pid end
                  || _ <- lists:seq(1, erlang:system_info(schedulers))]),
    true = ets:insert(?MODULE, {batchers, Batchers}),
    Self = self(),
    spawn_link(
      fun() ->
              %% initialize_trie/2 (vmq_reg_trie.erl:305-316), batched.  It
              %% has no failure mode, so neither has this load: a
              %% subscription the view cannot hold (past a limit: logged) is
              %% skipped and the load goes on; an upload that failed stays
              %% pending and is retried (retry_commit)
              Skipped = vmq_reg:fold_subscriptions(
                          fun({MP, Topic, {SubscriberId, SubInfo, Node}}, N) ->
                                  case vmqg_nif:add_init(Ctx, MP, Topic, SubscriberId, SubInfo, Node) of
                                      ok ->
                                          N;
                                      {error, device} ->
                                          Self ! retry_commit,
                                          N;
                                      {error, Reason} ->
                                          lager:warning("~p: subscription ~p of ~p not loaded: ~p",
                                                        [?MODULE, Topic, SubscriberId, Reason]),
                                          N + 1
                                  end
                          end, 0),
              case vmqg_nif:flush_init(Ctx) of
                  ok -> ok;
                  {error, device} -> Self ! retry_commit;
                  {error, Reason} -> exit({vmqg_load_failed, Reason})
              end,
              Self ! {subscribers_loaded, Skipped}
      end),
    EventHandler = vmq_reg:subscribe_subscriber_changes(),
    erlang:send_after(?RECLAIM_MS, self(), reclaim),
    {ok, #state{ctx=Ctx, batchers=Batchers, event_handler=EventHandler}}.

handle_call({event, Event}, _From, State) ->
    %% used only for testing/microbenchmarking, as vmq_reg_trie.erl:167-170
    {reply, ok, handle_events([Event], State)};
handle_call(_Request, _From, State) ->
    {reply, ok, State}.

handle_cast(_Msg, State) ->
    {noreply, State}.

handle_info({subscribers_loaded, Skipped}, #state{event_queue=Q} = State) ->
    %% the events queued during the initial load, replayed in order (:198-205)
    State1 = replay(queue:to_list(Q), State#state{status=ready}),
    {Subs, _} = stats(),
    lager:info("loaded ~p subscriptions into ~p (~p skipped)", [Subs, ?MODULE, Skipped]),
    {noreply, State1#state{event_queue=undefined}};
handle_info(reclaim, #state{ctx=Ctx} = State) ->
    _ = vmqg_nif:commit(Ctx),   % runs the reclamation that is due (c_src/vmqg_batch.c grace periods)
    erlang:send_after(?RECLAIM_MS, self(), reclaim),
    {noreply, State};
handle_info(retry_commit, #state{ctx=Ctx} = State) ->
    %% changes of an apply whose upload failed: pending in the library until
    %% a commit goes through (this one, or the next apply's)
    case vmqg_nif:commit(Ctx) of
        ok ->
            ok;
        {error, Reason} ->
            lager:warning("~p: commit failed (~p), retrying", [?MODULE, Reason]),
            erlang:send_after(?COMMIT_RETRY_MS, self(), retry_commit)
    end,
    {noreply, State};
handle_info(Event, #state{status=init, event_queue=Q} = State) ->
    {noreply, State#state{event_queue=queue:in(Event, Q)}};
handle_info(Event, State) ->
    Deadline = now_ms() + ?WINDOW_MS,
    {noreply, handle_events([Event | drain_events(?MAX_COALESCE - 1, ?WINDOW_EVENTS - 1, Deadline, [])], State)}.

terminate(_Reason, _State) ->
    ok.

code_change(_OldVsn, State, _Extra) ->
    {ok, State}.

%%%===================================================================
%%% Internal functions
%%%===================================================================

%% The window's subscriber events, oldest first (a selective receive keeps
%% their relative order; other messages stay where they are): while fewer
%% than W have come, wait for the next until Deadline; then only take what
%% is already queued, N at most.  The shapes are the metadata events
%% vmq_subscriber_db's handler converts (vmq_subscriber_db.erl:56-71).
drain_events(0, _W, _Deadline, Acc) ->
    lists:reverse(Acc);
drain_events(N, W, Deadline, Acc) ->
    Timeout = case W > 0 of
                  true -> erlang:max(0, Deadline - now_ms());
                  false -> 0
              end,
    receive
        {updated, {vmq, subscriber}, _, _, _} = E -> drain_events(N - 1, W - 1, Deadline, [E | Acc]);
        {deleted, {vmq, subscriber}, _, _} = E -> drain_events(N - 1, W - 1, Deadline, [E | Acc])
    after Timeout ->
        lists:reverse(Acc)
    end.

now_ms() ->
    {M, S, U} = os:timestamp(),
    (M * 1000000 + S) * 1000 + U div 1000.

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
%% the NIF turns the whole group into one vmqg_apply_ops.  vmq_reg_trie's
%% handler cannot fail, so this one never stops the view:
%%   - refused before anything is applied (invalid_topic: a malformed change;
%%     limit: a change past the node / mountpoint id space): the events are
%%     applied one by one, so only the offending event is skipped (logged),
%%     as it would be alone;
%%   - device: the group is applied on the host and pending in the library
%%     (folds answer from the previous tables meanwhile); a timer retries the
%%     commit, and the next apply ships it too — nothing is lost;
%%   - nomem: the group may be partly applied and cannot be replayed (that
%%     would apply its first part twice); logged, the view keeps answering,
%%     and the shadow compare (or a restart) is what shows the difference.
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
                {error, Refused} when Refused =:= invalid_topic; Refused =:= limit ->
                    lists:foreach(fun(C) -> apply_one(Ctx, C) end, Changes);
                {error, Reason} ->
                    apply_failed(Reason, length(Changes))
            end
    end,
    State.

apply_one(Ctx, {SubscriberId, Ch}) ->
    case vmqg_nif:apply(Ctx, SubscriberId, Ch) of
        ok ->
            ok;
        {error, Refused} when Refused =:= invalid_topic; Refused =:= limit ->
            lager:warning("~p: event of ~p skipped: ~p (~p)", [?MODULE, SubscriberId, Refused, Ch]);
        {error, Reason} ->
            apply_failed(Reason, 1)
    end.

apply_failed(device, _N) ->
    erlang:send_after(?COMMIT_RETRY_MS, self(), retry_commit);
apply_failed(Reason, N) ->
    lager:error("~p: applying ~p subscriber events failed: ~p", [?MODULE, N, Reason]).

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
