%% vmqg_nif — NIF stubs of c_src/vmqg_nif.c (libvmqgpu behind vmq_reg_gpu_view).
-module(vmqg_nif).
-export([create/1, apply/3, apply_many/2, add_init/6, flush_init/1, batch_new/1, match/4, stats/1,
         commit/1, set_option/3, counts/1]).
-on_load(init/0).

init() ->
    Priv = case code:priv_dir(vmq_server) of
               {error, _} -> "priv";
               Dir -> Dir
           end,
    erlang:load_nif(filename:join(Priv, "vmqg_nif"), 0).

%% #{device => integer(), local_node => node()} -> {ok, Ctx} | {error, term()}
create(_Opts) -> erlang:nif_error(nif_not_loaded).
%% Ctx, SubscriberId, [{add | del, Topic, SubInfo, Node}] -> ok | {error, term()}
apply(_Ctx, _SubscriberId, _Changes) -> erlang:nif_error(nif_not_loaded).
%% Ctx, [{SubscriberId, [{add | del, Topic, SubInfo, Node}]}] -> ok | {error, term()}
%% (a group of events as one apply; nothing applied on error)
apply_many(_Ctx, _EventChanges) -> erlang:nif_error(nif_not_loaded).
%% Ctx, MP, Topic, SubscriberId, SubInfo, Node -> ok | {error, term()}
add_init(_Ctx, _MP, _Topic, _SubscriberId, _SubInfo, _Node) -> erlang:nif_error(nif_not_loaded).
flush_init(_Ctx) -> erlang:nif_error(nif_not_loaded).
%% Ctx -> {ok, Batch}: a batcher's own publish batch
batch_new(_Ctx) -> erlang:nif_error(nif_not_loaded).
%% Ctx, Batch, [{MP, Topic}], records | ranges -> [{ok, [Entry]} | {error, term()}]
%% (Topic: the word list vmq_reg_view:fold/4 got, used as given)
match(_Ctx, _Batch, _Publishes, _Mode) -> erlang:nif_error(nif_not_loaded).
%% Ctx -> {NrOfSubs, DeviceBytes}
stats(_Ctx) -> erlang:nif_error(nif_not_loaded).
%% Ctx -> ok | {error, term()}: ships changes left pending by an apply whose
%% upload failed ({error, device}: they are kept, not lost)
commit(_Ctx) -> erlang:nif_error(nif_not_loaded).
%% Ctx -> [{atom(), non_neg_integer()}]: live terms, ids, tables and memory
counts(_Ctx) -> erlang:nif_error(nif_not_loaded).
%% Ctx, atom(), integer() -> ok | {error, term()} (vmqg_set_option)
set_option(_Ctx, _Name, _Value) -> erlang:nif_error(nif_not_loaded).
%% Errors: {error, invalid_topic | limit | nomem | device | busy | internal}
%% (c_src/vmqg_nif.c error_term/2).
