/*
 * vmqg_nif.c — the erl_nif glue of vmq_reg_gpu_view (src/vmq_reg_gpu_view.erl)
 * over libvmqgpu (include/vmqg.h).
 *
 * Only term <-> id conversion lives here; batching, matching with the
 * overflow retry, the fold and the op batches are vmqg_batch.c (plain C,
 * compiled and unit-tested in this repository: tests/test_nif_layer.py,
 * tools/nif_harness.c).  This file is written against the documented
 * erl_nif API of OTP 19.3 .. 21 (the releases the reference is tested on,
 * .travis.yml: the newest calls are enif_term_to_binary, OTP 19.0, and
 * enif_schedule_nif / enif_system_info's dirty_scheduler_support, OTP
 * 17.3); OTP is not in this image, so it is compiled and run over an
 * erl_nif test double (tests/c/mock_erl_nif, tests/c/nif_mock_check.c).
 *
 * Build (in apps/vmq_server, rebar3 port_specs or a Makefile):
 *   cc -O2 -fPIC -shared -I$ERTS/include -I<repo>/include -I<repo>/integration/c_src \
 *      vmqg_nif.c vmqg_batch.c -L<priv> -lvmqgpu -o priv/vmqg_nif.so
 *
 * Terms and their ids (one resource per view):
 *   mountpoint (string)          -> vmqg mountpoint id    (interner `mps`)
 *   node atom                    -> node id; node() is 0   (interner `nodes`)
 *   SubscriberId {MP, ClientId}  -> subscriber id         (interner `subs`)
 *   SubInfo (QoS | {QoS, Map})   -> subinfo id            (interner `infos`)
 *   $share group binary          <- its word id           (`groups`, by word id)
 * Terms are keyed by their external term format (enif_term_to_binary) and
 * kept as copies in the resource's own environment, so building an entry is
 * an enif_make_copy, never a decode.
 *
 * Concurrency (vmqgb_view, vmqg_batch.c): vmq_reg_gpu_view runs one batcher
 * process per scheduler; each calls match/4 with its own batch resource, and
 * those calls run in parallel on dirty CPU schedulers — preparing the
 * publishes and building the result terms without a lock and without ever
 * waiting for a writer, only the device call itself taking turns — as
 * vmq_reg_trie:fold/4 runs in every caller's process (vmq_reg_trie.erl:59-66,
 * read_concurrency tables with one writer :136-137); the device calls of all
 * batchers are combined (vmqgb_view_match).  apply/3, apply_many/2,
 * add_init/6 and flush_init/1 (the subscription changes and the term tables
 * they intern) are writers, one at a time: the term tables only grow, in
 * chunks that never move, so readers index them while a writer adds.  Every
 * NIF that can wait for a lock or the device is a dirty one.
 */
#include <erl_nif.h>
#include <stdint.h>
#include <string.h>

#include "vmqg.h"
#include "vmqg_batch.h"

/* Terms by id, TS_CHUNK ids per chunk.  A chunk owns a process-independent
 * environment holding its terms (enif_make_copy) and is published whole
 * (release) before any result can carry one of its ids; readers (batchers
 * folding) index it without a lock while the writer adds terms.  Ids are
 * reused once their terms are dropped (the view's grace period has passed),
 * so a chunk's environment accumulates dead copies: when they outnumber the
 * live ones the writer copies the live terms into a fresh chunk, publishes
 * it, and frees the old one after another grace period (vmqgb_view_defer). */
#define TS_CHUNK_BITS 14
#define TS_CHUNK (1u << TS_CHUNK_BITS)
#define TS_CHUNKS (1u << 18)      /* ids < 2^32 */
typedef struct {
  ErlNifEnv* env;                 /* owns the chunk's stored terms */
  uint32_t live, dead;            /* terms stored / dead copies in env */
  ERL_NIF_TERM t[TS_CHUNK];
} ts_chunk;

typedef struct {
  ts_chunk** dir;                 /* TS_CHUNKS chunk pointers */
  uint64_t live, chunks, compactions;
} term_store;

typedef struct vmqg_res vmqg_res;
struct vmqg_res {
  vmqg_ctx* ctx;                  /* the primary (host engine + its device tables) */
  vmqg_ctx* replicas[VMQGB_MAX_LANES];   /* devices => [D0, D1, ...]: replicas on D1, ... */
  int nreplicas;
  vmqgb_view* view;               /* batchers (readers) vs. table changes (writers) */
  ErlNifMutex* mp_mu;             /* the mountpoint interner: batchers look up, writers add */
  vmqgb_interner *mps, *nodes, *subs, *infos;
  term_store node_t, sub_t, info_t, group_t;   /* group_t indexed by word id */
  vmqgb_ops ops;                  /* apply/3 and add_init/6 accumulation (under the write lock) */
  uint64_t terms_dropped;
};

typedef struct {                  /* one batcher's batch (batch_new/1) */
  vmqg_res* owner;                /* kept alive while the batch lives */
  vmqgb_batch b;
} vmqg_bres;

static ErlNifResourceType* RES;
static ErlNifResourceType* BRES;
static ERL_NIF_TERM a_ok, a_error, a_invalid_topic, a_device, a_nomem, a_badarg, a_limit, a_busy, a_internal,
    a_records, a_ranges;

/* ------------------------------------------------------------ helpers */
static int store_init(term_store* s) {
  s->dir = (ts_chunk**)enif_alloc(TS_CHUNKS * sizeof(ts_chunk*));
  if (!s->dir) return 0;
  memset(s->dir, 0, TS_CHUNKS * sizeof(ts_chunk*));
  s->live = s->chunks = s->compactions = 0;
  return 1;
}

static void chunk_free(ts_chunk* c) {
  if (!c) return;
  enif_free_env(c->env);
  enif_free(c);
}

static void store_free(term_store* s) {
  if (s->dir)
    for (size_t c = 0; c < TS_CHUNKS; c++) chunk_free(s->dir[c]);
  enif_free(s->dir);
}

static ts_chunk* chunk_new(void) {
  ts_chunk* c = (ts_chunk*)enif_alloc(sizeof(ts_chunk));
  if (!c) return NULL;
  memset(c, 0, sizeof(*c));
  c->env = enif_alloc_env();
  if (!c->env) { enif_free(c); return NULL; }
  return c;
}

/* the writer only */
static int store_put(term_store* s, size_t id, ERL_NIF_TERM t) {
  if (!s->dir || (id >> TS_CHUNK_BITS) >= TS_CHUNKS) return 0;
  ts_chunk* ch = s->dir[id >> TS_CHUNK_BITS];
  if (!ch) {
    if (!(ch = chunk_new())) return 0;
    __atomic_store_n(&s->dir[id >> TS_CHUNK_BITS], ch, __ATOMIC_RELEASE);
    s->chunks++;
  }
  ERL_NIF_TERM* slot = &ch->t[id & (TS_CHUNK - 1)];
  if (*slot) ch->dead++; else { ch->live++; s->live++; }   /* a group word's term replaced */
  *slot = enif_make_copy(ch->env, t);
  return 1;
}

/* readers: an id from a match result (stored before the apply that made it reachable) */
static ERL_NIF_TERM store_get(const term_store* s, uint32_t id) {
  const ts_chunk* ch = __atomic_load_n(&s->dir[id >> TS_CHUNK_BITS], __ATOMIC_ACQUIRE);
  return ch ? ch->t[id & (TS_CHUNK - 1)] : 0;
}

/* The writer: when id's chunk holds more dead copies than live terms (and
 * at least 1,024), its live terms are copied into a fresh chunk, which is
 * published; the old chunk is returned for the caller to free after a
 * grace period (readers may still index it). */
static ts_chunk* store_compact(term_store* s, uint32_t id) {
  ts_chunk* ch = s->dir[id >> TS_CHUNK_BITS];
  if (!ch || ch->dead < 1024 || ch->dead <= ch->live) return NULL;
  ts_chunk* nc = chunk_new();
  if (!nc) return NULL;   /* stays as it is: only memory */
  for (uint32_t i = 0; i < TS_CHUNK; i++)
    if (ch->t[i]) { nc->t[i] = enif_make_copy(nc->env, ch->t[i]); nc->live++; }
  __atomic_store_n(&s->dir[id >> TS_CHUNK_BITS], nc, __ATOMIC_RELEASE);
  s->compactions++;
  return ch;
}

/* the writer, after a grace period: id's term is dead (its copy stays in
 * the chunk's environment until the chunk is compacted: store_compact) */
static ts_chunk* store_drop(term_store* s, uint32_t id) {
  ts_chunk* ch = s->dir[id >> TS_CHUNK_BITS];
  if (!ch || !ch->t[id & (TS_CHUNK - 1)]) return NULL;
  ch->t[id & (TS_CHUNK - 1)] = 0;
  ch->live--;
  ch->dead++;
  s->live--;
  return store_compact(s, id);
}

/* id of a term (created on first sight, possibly a reused id), its copy
 * stored under the id */
static int term_id(vmqgb_interner* in, term_store* st, ErlNifEnv* env, ERL_NIF_TERM t, uint32_t* id) {
  ErlNifBinary b;
  if (!enif_term_to_binary(env, t, &b)) return 0;
  int created = 0;
  *id = vmqgb_intern_ex(in, b.data, b.size, &created);
  enif_release_binary(&b);
  if (*id == VMQG_NONE) return 0;
  if (st && created) return store_put(st, *id, t);
  return 1;
}

/* ------------------------------------------------------- term reclamation */
/* SubscriberId / SubInfo terms no record holds any more (vmqg_released_ids
 * after each stage): taken out of the interner at once — a later
 * subscription of the same term gets a fresh id — and, once the view's grace
 * period has passed (no batcher can still fold a record naming them),
 * dropped from the store and their ids made reusable.  Memory thus follows
 * the live subscriptions, as vmq_reg_trie's ETS rows do
 * (vmq_reg_trie.erl:472-496). */
typedef struct {
  vmqg_res* r;
  uint32_t kind, n;
  uint32_t ids[];
} drop_batch;

static void chunk_retire_fn(void* arg, uint64_t u) { (void)u; chunk_free((ts_chunk*)arg); }

static void drop_terms_fn(void* arg, uint64_t u) {
  (void)u;
  drop_batch* d = (drop_batch*)arg;
  vmqg_res* r = d->r;
  vmqgb_interner* in = d->kind ? r->infos : r->subs;
  term_store* st = d->kind ? &r->info_t : &r->sub_t;
  for (uint32_t i = 0; i < d->n; i++) {
    ts_chunk* old = store_drop(st, d->ids[i]);
    if (old) vmqgb_view_defer(r->view, chunk_retire_fn, old, 0, 0);   /* after readers of it leave (if the
                                                                         defer cannot allocate, it is kept) */
    vmqgb_interner_release(in, d->ids[i]);
    r->terms_dropped++;
  }
  enif_free(d);
}

static void stage_hook(void* arg, vmqgb_view* v) {
  vmqg_res* r = (vmqg_res*)arg;
  for (uint32_t kind = 0; kind < 2; kind++) {
    const uint32_t* ids = NULL;
    size_t n = 0;
    if (vmqg_released_ids(r->ctx, kind, &ids, &n) || !n) continue;
    vmqgb_interner* in = kind ? r->infos : r->subs;
    drop_batch* d = (drop_batch*)enif_alloc(sizeof(drop_batch) + n * sizeof(uint32_t));
    if (!d) continue;   /* the terms stay: only memory */
    d->r = r; d->kind = kind; d->n = 0;
    for (size_t i = 0; i < n; i++)
      if (vmqgb_interner_remove(in, ids[i]) == 0) d->ids[d->n++] = ids[i];
    if (!d->n || vmqgb_view_defer(v, drop_terms_fn, d, 0, 1)) enif_free(d);
  }
}

/* the mountpoint interner is shared with the batchers' lookups */
static int mp_id(vmqg_res* r, ErlNifEnv* env, ERL_NIF_TERM t, uint32_t* id) {
  enif_mutex_lock(r->mp_mu);
  const int ok = term_id(r->mps, NULL, env, t, id);
  enif_mutex_unlock(r->mp_mu);
  return ok;
}

/* {error, Reason}: invalid_topic (a malformed change or Topic: nothing
 * applied), limit (a change past VMQG_MAX_NODES nodes or VMQG_MAX_MOUNTPOINTS
 * mountpoints: nothing applied), nomem, device (an apply whose upload failed
 * stays pending and lands with the next commit; a match that failed), busy
 * (applies kept rewriting what a match read: retry), internal (anything
 * else).  vmq_reg_gpu_view tells them apart. */
static ERL_NIF_TERM error_term(ErlNifEnv* env, int rc) {
  ERL_NIF_TERM r = rc == VMQG_E_INVAL ? a_invalid_topic : rc == VMQG_E_NOMEM ? a_nomem
                 : rc == VMQG_E_DEVICE ? a_device : rc == VMQG_E_LIMIT ? a_limit
                 : rc == VMQG_E_STATE ? a_busy : a_internal;
  return enif_make_tuple2(env, a_error, r);
}

static void res_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  vmqg_res* r = (vmqg_res*)obj;
  vmqgb_view_free(r->view);   /* its rounds, before the contexts they ran on */
  r->view = NULL;
  for (int k = 0; k < r->nreplicas; k++) vmqg_destroy(r->replicas[k]);
  if (r->ctx) vmqg_destroy(r->ctx);
  vmqgb_interner_free(r->mps); vmqgb_interner_free(r->nodes);
  vmqgb_interner_free(r->subs); vmqgb_interner_free(r->infos);
  term_store* ts[4] = {&r->node_t, &r->sub_t, &r->info_t, &r->group_t};
  for (int i = 0; i < 4; i++) store_free(ts[i]);
  vmqgb_ops_free(&r->ops);
  if (r->mp_mu) enif_mutex_destroy(r->mp_mu);
}

static void bres_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  vmqg_bres* br = (vmqg_bres*)obj;
  vmqgb_batch_free(&br->b);
  if (br->owner) enif_release_resource(br->owner);
}

static vmqg_res* get_res(ErlNifEnv* env, ERL_NIF_TERM t) {
  vmqg_res* r = NULL;
  return enif_get_resource(env, t, RES, (void**)&r) ? r : NULL;
}

/* ------------------------------------------------------------- create/1 */
/* create(#{device => D, local_node => node()[, devices => [D0, D1, ...]]})
 * -> {ok, Ctx} | {error, _} (vmq_reg_trie:init/1, vmq_reg_trie.erl:135-151).
 * devices: the primary on D0 and a replica of its tables on each further
 * device (the same device may repeat); the view spreads the batchers over
 * them (the trie replicated, publish batches sharded). */
static ERL_NIF_TERM nif_create(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  ERL_NIF_TERM v;
  int device = 0;
  if (enif_get_map_value(env, argv[0], enif_make_atom(env, "device"), &v)) enif_get_int(env, v, &device);
  ERL_NIF_TERM local;
  if (!enif_get_map_value(env, argv[0], enif_make_atom(env, "local_node"), &local)) return enif_make_badarg(env);
  vmqg_res* r = (vmqg_res*)enif_alloc_resource(RES, sizeof(vmqg_res));
  memset(r, 0, sizeof(*r));
  r->mps = vmqgb_interner_new(); r->nodes = vmqgb_interner_new();
  r->subs = vmqgb_interner_new(); r->infos = vmqgb_interner_new();
  r->mp_mu = enif_mutex_create("vmqg_mp");
  if (!r->mp_mu || !store_init(&r->node_t) || !store_init(&r->sub_t) || !store_init(&r->info_t) ||
      !store_init(&r->group_t)) {
    enif_release_resource(r);
    return error_term(env, VMQG_E_NOMEM);
  }
  vmqgb_ops_init(&r->ops);
  uint32_t id;
  term_id(r->mps, NULL, env, enif_make_string(env, "", ERL_NIF_LATIN1), &id);   /* "" is mountpoint 0 */
  term_id(r->nodes, &r->node_t, env, local, &id);                               /* node() is node 0 */
  vmqg_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.device = device;
  cfg.local_node = 0;
  cfg.max_nodes = VMQG_MAX_NODES;
  cfg.max_mountpoints = 1024;   /* the initial root range: more mountpoints grow it (no limit below
                                   VMQG_MAX_MOUNTPOINTS, as vmq_reg_trie has none) */
  int devs[VMQGB_MAX_LANES], ndev = 0;
  ERL_NIF_TERM dl;
  if (enif_get_map_value(env, argv[0], enif_make_atom(env, "devices"), &dl)) {
    ERL_NIF_TERM h, t = dl;
    while (enif_get_list_cell(env, t, &h, &t)) {
      if (ndev == VMQGB_MAX_LANES || !enif_get_int(env, h, &devs[ndev])) { enif_release_resource(r); return enif_make_badarg(env); }
      ndev++;
    }
    if (ndev) cfg.device = devs[0];
  }
  int err = 0;
  r->ctx = vmqg_create(&cfg, &err);
  if (r->ctx && !(r->view = vmqgb_view_new(r->ctx))) err = VMQG_E_NOMEM;
  for (int k = 1; r->view && !err && k < ndev; k++) {
    vmqg_config rc = cfg;
    rc.device = devs[k];
    rc.flags = VMQG_CFG_REPLICA;
    vmqg_ctx* x = vmqg_create(&rc, &err);
    if (!x) break;
    r->replicas[r->nreplicas++] = x;
    err = vmqgb_view_add_replica(r->view, x);
  }
  if (err && r->ctx) { vmqgb_view_free(r->view); r->view = NULL; }
  if (r->view) vmqgb_view_set_stage_hook(r->view, stage_hook, r);
  ERL_NIF_TERM ret = r->ctx && r->view ? enif_make_tuple2(env, a_ok, enif_make_resource(env, r)) : error_term(env, err);
  enif_release_resource(r);
  return ret;
}

/* ------------------------------------------------------------------ ops */
/* One {Kind, Topic, SubInfo, Node} change of SubscriberId into r->ops. */
static int add_change(ErlNifEnv* env, vmqg_res* r, uint32_t kind, ERL_NIF_TERM sid, ERL_NIF_TERM topic,
                      ERL_NIF_TERM subinfo, ERL_NIF_TERM node) {
  int arity;
  const ERL_NIF_TERM* sid_el;
  if (!enif_get_tuple(env, sid, &arity, &sid_el) || arity != 2) return VMQG_E_INVAL;
  uint32_t mp, sub, info, nd;
  /* the id spaces checked here, change by change, so that one change past a
   * limit is refused alone (the library would refuse its whole op batch) */
  if (!mp_id(r, env, sid_el[0], &mp) || !term_id(r->nodes, &r->node_t, env, node, &nd)) return VMQG_E_NOMEM;
  if (mp >= VMQG_MAX_MOUNTPOINTS || nd >= VMQG_MAX_NODES) return VMQG_E_LIMIT;
  if (!term_id(r->subs, &r->sub_t, env, sid, &sub) || !term_id(r->infos, &r->info_t, env, subinfo, &info))
    return VMQG_E_NOMEM;
  unsigned len;
  if (!enif_get_list_length(env, topic, &len) || len == 0 || len > 65536) return VMQG_E_INVAL;
  /* word pointers on the heap: a topic of 65,535 bytes has ~32k levels,
   * far more than a scheduler's stack holds */
  const uint8_t** wp = (const uint8_t**)enif_alloc(len * sizeof(*wp));
  size_t* wl = (size_t*)enif_alloc(len * sizeof(*wl));
  if (!wp || !wl) { enif_free(wp); enif_free(wl); return VMQG_E_NOMEM; }
  ERL_NIF_TERM group = 0, head, tail = topic;
  int rc = 0;
  for (unsigned i = 0; i < len; i++) {
    ErlNifBinary b;
    enif_get_list_cell(env, tail, &head, &tail);
    if (!enif_inspect_binary(env, head, &b)) { rc = VMQG_E_INVAL; break; }
    wp[i] = b.data;
    wl[i] = b.size;
    if (i == 1) group = head;
  }
  const size_t w0 = r->ops.nwords;
  if (!rc) rc = vmqgb_ops_add(&r->ops, r->ctx, kind, mp, wp, wl, len, nd, sub, info);
  enif_free(wp);
  enif_free(wl);
  if (rc) return rc;
  /* $share/Group/...: remember the group binary under its word id (decoding
   * kind-B entries) — unless it is there already: a word id released and
   * reused for another word gets its new binary, the old copy becomes dead */
  if (len >= 3 && r->ops.words[w0] == VMQG_WORD_SHARE) {
    const uint32_t gw = r->ops.words[w0 + 1];
    const ERL_NIF_TERM have = store_get(&r->group_t, gw);
    ErlNifBinary hb, gb;
    if (!have || !enif_inspect_binary(env, have, &hb) || !enif_inspect_binary(env, group, &gb) || hb.size != gb.size ||
        memcmp(hb.data, gb.data, gb.size) != 0) {
      store_put(&r->group_t, gw, group);
      ts_chunk* old = store_compact(&r->group_t, gw);
      if (old) vmqgb_view_defer(r->view, chunk_retire_fn, old, 0, 0);
    }
  }
  return 0;
}

/* The changes of one subscriber event: [{add | del, Topic, SubInfo, Node}]
 * in vmq_subscriber:fold/3 order (deletes first), into r->ops. */
static int add_changes(ErlNifEnv* env, vmqg_res* r, ERL_NIF_TERM sid, ERL_NIF_TERM changes) {
  ERL_NIF_TERM head, tail = changes;
  const ERL_NIF_TERM a_add = enif_make_atom(env, "add");
  while (enif_get_list_cell(env, tail, &head, &tail)) {
    int arity;
    const ERL_NIF_TERM* el;
    if (!enif_get_tuple(env, head, &arity, &el) || arity != 4) return VMQG_E_INVAL;
    const uint32_t kind = enif_is_identical(el[0], a_add) ? VMQG_OP_ADD : VMQG_OP_DEL;
    const int rc = add_change(env, r, kind, sid, el[1], el[2], el[3]);
    if (rc) return rc;
  }
  return 0;
}

/* Under the write lock: applies the pending add_init ops (they keep their
 * order before anything applied after them); their failure is returned. */
static int flush_pending(vmqg_res* r) {
  if (!r->ops.n) return 0;
  const int rc = vmqgb_view_apply_ops(r->view, &r->ops, NULL);
  vmqgb_ops_reset(&r->ops);
  return rc;
}

/* apply(Ctx, SubscriberId, [{add | del, Topic, SubInfo, Node}]) -> ok | {error, _}
 * (handle_event/2, vmq_reg_trie.erl:240-277) */
static ERL_NIF_TERM nif_apply(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqg_res* r = get_res(env, argv[0]);
  if (!r) return enif_make_badarg(env);
  vmqgb_view_write_begin(r->view);
  int rc = flush_pending(r);
  if (!rc) rc = add_changes(env, r, argv[1], argv[2]);
  if (!rc) rc = vmqgb_view_apply_ops(r->view, &r->ops, NULL);
  vmqgb_ops_reset(&r->ops);
  vmqgb_view_write_end(r->view);
  return rc ? error_term(env, rc) : a_ok;
}

/* apply_many(Ctx, [{SubscriberId, Changes}]) -> ok | {error, _}: the events
 * vmq_reg_gpu_view drained from its mailbox, in arrival order, as ONE
 * vmqg_apply_ops (one write-lock section, one patch upload).  Applying the
 * concatenation is applying them one after the other: every event's deletes
 * precede its adds, and events keep their order (vmq_reg_trie.erl:240-251).
 * An invalid change rejects the whole call with nothing applied (the view
 * then applies the events one by one to isolate it). */
static ERL_NIF_TERM nif_apply_many(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqg_res* r = get_res(env, argv[0]);
  if (!r) return enif_make_badarg(env);
  vmqgb_view_write_begin(r->view);
  int rc = flush_pending(r);
  ERL_NIF_TERM head, tail = argv[1];
  while (!rc && enif_get_list_cell(env, tail, &head, &tail)) {
    int arity;
    const ERL_NIF_TERM* el;
    if (!enif_get_tuple(env, head, &arity, &el) || arity != 2) { rc = VMQG_E_INVAL; break; }
    rc = add_changes(env, r, el[0], el[1]);
  }
  if (!rc) rc = vmqgb_view_apply_ops(r->view, &r->ops, NULL);
  vmqgb_ops_reset(&r->ops);
  vmqgb_view_write_end(r->view);
  return rc ? error_term(env, rc) : a_ok;
}

/* add_init(Ctx, MP, Topic, SubscriberId, SubInfo, Node) -> ok: one
 * initialize_trie/2 tuple (vmq_reg_trie.erl:305-316), applied in batches.
 * Only the table lock: interning terms and words never waits for a device
 * call; the device mutex is taken for the apply every 65,536 changes. */
static ERL_NIF_TERM nif_add_init(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqg_res* r = get_res(env, argv[0]);
  if (!r) return enif_make_badarg(env);
  vmqgb_view_write_begin(r->view);
  int rc = add_change(env, r, VMQG_OP_ADD, argv[3], argv[2], argv[4], argv[5]);
  if (!rc && r->ops.n >= 65536) rc = flush_pending(r);
  vmqgb_view_write_end(r->view);
  return rc ? error_term(env, rc) : a_ok;
}

static ERL_NIF_TERM nif_flush_init(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqg_res* r = get_res(env, argv[0]);
  if (!r) return enif_make_badarg(env);
  vmqgb_view_write_begin(r->view);
  const int rc = flush_pending(r);
  vmqgb_view_write_end(r->view);
  return rc ? error_term(env, rc) : a_ok;
}

/* commit(Ctx) -> ok | {error, _}: ships changes still pending after an apply
 * whose upload failed ({error, device}): vmq_reg_gpu_view retries on a timer,
 * so a transient device error delays changes and loses none. */
static ERL_NIF_TERM nif_commit(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqg_res* r = get_res(env, argv[0]);
  if (!r) return enif_make_badarg(env);
  const int rc = vmqgb_view_commit(r->view, NULL);
  return rc ? error_term(env, rc) : a_ok;
}

/* set_option(Ctx, Name, Value) -> ok | {error, _}: vmqg_set_option (kernel
 * knobs from app env; "fail_commits" for tests) under the writer and device
 * locks */
static ERL_NIF_TERM nif_set_option(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqg_res* r = get_res(env, argv[0]);
  char name[64];
  ErlNifSInt64 value;
  if (!r || enif_get_atom(env, argv[1], name, sizeof name, ERL_NIF_LATIN1) <= 0 || !enif_get_int64(env, argv[2], &value))
    return enif_make_badarg(env);
  const int rc = vmqgb_view_set_option(r->view, name, (int64_t)value);
  return rc ? error_term(env, rc) : a_ok;
}

/* ---------------------------------------------------------------- match */
typedef struct {
  ErlNifEnv* env;
  vmqg_res* r;
  ERL_NIF_TERM* out;
  size_t n;
} fold_acc;

/* FoldFun argument term of one entry (vmq_reg_trie.erl:68-98) */
static int make_entry(void* accp, const vmqgb_entry* e) {
  fold_acc* acc = (fold_acc*)accp;
  vmqg_res* r = acc->r;
  ErlNifEnv* env = acc->env;
  ERL_NIF_TERM t;
  if (e->kind == VMQG_EMIT_LOCAL) {          /* {SubscriberId, SubInfo} */
    t = enif_make_tuple2(env, enif_make_copy(env, store_get(&r->sub_t, e->subscriber)),
                         enif_make_copy(env, store_get(&r->info_t, e->subinfo)));
  } else if (e->kind == VMQG_EMIT_GROUP) {   /* {Node, Group, SubscriberId, SubInfo} */
    t = enif_make_tuple4(env, enif_make_copy(env, store_get(&r->node_t, e->node)),
                         enif_make_copy(env, store_get(&r->group_t, e->group)),
                         enif_make_copy(env, store_get(&r->sub_t, e->subscriber)),
                         enif_make_copy(env, store_get(&r->info_t, e->subinfo)));
  } else {                                   /* Node */
    t = enif_make_copy(env, store_get(&r->node_t, e->node));
  }
  acc->out[acc->n++] = t;
  return 0;
}

/* a run of consecutive records (vmqgb_fold_spans): one term each, in order */
static int make_entries(void* accp, const vmqg_emit* run, size_t n) {
  for (size_t j = 0; j < n; j++) {
    const vmqgb_entry e = {run[j].kind_node >> 24, run[j].kind_node & 0xFFFFFFu, run[j].group, run[j].subscriber,
                           run[j].subinfo};
    make_entry(accp, &e);
  }
  return 0;
}

/* batch_new(Ctx) -> {ok, Batch}: a batcher's own publish batch */
static ERL_NIF_TERM nif_batch_new(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqg_res* r = get_res(env, argv[0]);
  if (!r) return enif_make_badarg(env);
  vmqg_bres* br = (vmqg_bres*)enif_alloc_resource(BRES, sizeof(vmqg_bres));
  memset(br, 0, sizeof(*br));
  if (vmqgb_batch_init(&br->b, 4096)) { enif_release_resource(br); return error_term(env, VMQG_E_NOMEM); }
  vmqgb_view_bind(r->view, &br->b);   /* batcher k's publishes go to device context k mod N */
  enif_keep_resource(r);
  br->owner = r;
  ERL_NIF_TERM t = enif_make_resource(env, br);
  enif_release_resource(br);
  return enif_make_tuple2(env, a_ok, t);
}

/* match(Ctx, Batch, [{MP, Topic}], records | ranges) -> [{ok, Entries} | {error, Reason}]
 * (fold/4 for a batch of callers, vmq_reg_trie.erl:59-98); dirty CPU.
 * Topic is the word list fold/4 was given, used as given (no join, no
 * split, no validate_topic: a plugin publish reaches fold/4 unvalidated,
 * vmq_reg.erl:572-594): each element one dictionary lookup, an element that
 * is not a binary equal to no filter word, [] the root alone.
 * Batchers run this concurrently and never wait for a writer: the prepare
 * reads the lock-free dictionary, the batch joins the view's combining
 * submitter for the device call (vmqgb_view_match), and the terms are built
 * from the batch's own records (records mode) or from the record table of
 * its epoch pinned until the end (ranges). */
static ERL_NIF_TERM nif_match(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqg_res* r = get_res(env, argv[0]);
  vmqg_bres* br = NULL;
  unsigned n;
  if (!r || !enif_get_resource(env, argv[1], BRES, (void**)&br) || br->owner != r ||
      !enif_get_list_length(env, argv[2], &n))
    return enif_make_badarg(env);
  const int ranges = enif_is_identical(argv[3], a_ranges);
  vmqgb_batch* b = &br->b;
  const size_t m = n ? n : 1;
  long* idx = (long*)enif_alloc(m * sizeof(long));
  ERL_NIF_TERM* res = (ERL_NIF_TERM*)enif_alloc(m * sizeof(ERL_NIF_TERM));
  ERL_NIF_TERM* topics = (ERL_NIF_TERM*)enif_alloc(m * sizeof(ERL_NIF_TERM));
  uint32_t* cnt = (uint32_t*)enif_alloc(m * sizeof(uint32_t));
  uint32_t* mps = (uint32_t*)enif_alloc(m * sizeof(uint32_t));
  if (!idx || !res || !topics || !cnt || !mps) {
    enif_free(idx); enif_free(res); enif_free(topics); enif_free(cnt); enif_free(mps);
    return enif_make_badarg(env);
  }
  /* pass 1: each publish's Topic list and length, and its mountpoint id; the
   * MP of the previous publish is reused when identical (one term_to_binary
   * per distinct mountpoint run, not per publish) */
  ERL_NIF_TERM head, tail = argv[2], last_mp = 0;
  uint32_t last_id = VMQG_NONE;
  size_t total = 0;
  for (unsigned i = 0; i < n; i++) {
    int arity;
    const ERL_NIF_TERM* el;
    unsigned len = 0;
    enif_get_list_cell(env, tail, &head, &tail);
    idx[i] = 0;
    cnt[i] = 0;
    mps[i] = 0;
    if (!enif_get_tuple(env, head, &arity, &el) || arity != 2 || !enif_get_list_length(env, el[1], &len)) {
      idx[i] = VMQG_E_INVAL;   /* fold/4's is_list(Topic) guard (vmq_reg_trie.erl:60) */
      continue;
    }
    topics[i] = el[1];
    cnt[i] = len;
    total += len;
    if (!last_mp || !enif_is_identical(el[0], last_mp)) {
      ErlNifBinary mpb;
      last_mp = el[0];
      last_id = VMQG_NONE;   /* an unknown mountpoint has no subscriptions: an id no root ever takes */
      if (enif_term_to_binary(env, el[0], &mpb)) {
        uint32_t id;
        enif_mutex_lock(r->mp_mu);
        if (vmqgb_lookup(r->mps, mpb.data, mpb.size, &id) == 0) last_id = id;
        enif_mutex_unlock(r->mp_mu);
        enif_release_binary(&mpb);
      }
    }
    mps[i] = last_id;
  }
  /* pass 2: every word's bytes (valid for this call) */
  const uint8_t** wp = (const uint8_t**)enif_alloc((total ? total : 1) * sizeof(*wp));
  size_t* wl = (size_t*)enif_alloc((total ? total : 1) * sizeof(size_t));
  if (!wp || !wl) {
    enif_free(wp); enif_free(wl);
    enif_free(idx); enif_free(res); enif_free(topics); enif_free(cnt); enif_free(mps);
    return enif_make_badarg(env);
  }
  size_t k = 0;
  for (unsigned i = 0; i < n; i++) {
    if (idx[i]) continue;
    ERL_NIF_TERM wt = topics[i], w;
    while (enif_get_list_cell(env, wt, &w, &wt)) {
      ErlNifBinary wb;
      if (enif_inspect_binary(env, w, &wb)) { wp[k] = wb.data; wl[k] = wb.size; }
      else { wp[k] = NULL; wl[k] = VMQGB_NOT_BINARY; }   /* equals no filter word */
      k++;
    }
  }
  vmqgb_batch_reset(b);
  vmqgb_view_enter(r->view, b);   /* word ids from here to the fold: the grace period's reader */
  /* the batched prepare: rejected terms keep their error, the others are
   * prepared together */
  {
    unsigned q = 0;
    for (unsigned i = 0; i < n; i++)
      if (idx[i] == 0) { mps[q] = mps[i]; cnt[q] = cnt[i]; q++; }
    long* sub = (long*)enif_alloc((q ? q : 1) * sizeof(long));
    const int prc = sub ? vmqgb_batch_add_word_lists(b, r->ctx, q, mps, cnt, wp, wl, sub) : VMQG_E_NOMEM;
    unsigned j = 0;
    for (unsigned i = 0; i < n; i++)
      if (idx[i] == 0) idx[i] = prc ? prc : sub[j++];
    enif_free(sub);
  }
  enif_free(wp);
  enif_free(wl);
  const vmqg_emit* recs = NULL;
  uint64_t nrecs = 0;
  const int rc = vmqgb_view_match(r->view, b, ranges, &recs, &nrecs);
  __atomic_thread_fence(__ATOMIC_ACQUIRE);   /* the term tables as of the results' epoch */
  for (unsigned i = 0; i < n; i++) {
    if (idx[i] < 0 || rc) { res[i] = error_term(env, idx[i] < 0 ? (int)idx[i] : rc); continue; }
    size_t cnt = 0;
    if (b->out_ranges) {
      for (uint64_t k = b->offsets[idx[i]]; k < b->offsets[idx[i] + 1]; k++) cnt += b->rng[k].count ? b->rng[k].count : 1;
    } else {
      cnt = vmqgb_count_of(b, (size_t)idx[i]);
    }
    fold_acc acc = {env, r, (ERL_NIF_TERM*)enif_alloc((cnt ? cnt : 1) * sizeof(ERL_NIF_TERM)), 0};
    if (i + VMQGB_PREFETCH_AHEAD < n && idx[i + VMQGB_PREFETCH_AHEAD] >= 0)
      vmqgb_prefetch_entries(b, b->out_ranges, recs, nrecs, (size_t)idx[i + VMQGB_PREFETCH_AHEAD]);
    const int frc = vmqgb_fold_spans(b, b->out_ranges, recs, nrecs, (size_t)idx[i], make_entries, &acc);
    /* a fold that stops early (a range beyond the table) is this publish's error, never a partial list */
    res[i] = frc ? error_term(env, frc) : enif_make_tuple2(env, a_ok, enif_make_list_from_array(env, acc.out, (unsigned)acc.n));
    enif_free(acc.out);
  }
  vmqgb_view_release(r->view, b);
  ERL_NIF_TERM list = enif_make_list_from_array(env, res, n);
  enif_free(res); enif_free(idx); enif_free(topics); enif_free(cnt); enif_free(mps);
  return list;
}

/* counts(Ctx) -> [{Name, N}]: what the view holds now — live terms and
 * ids, the library's live tables and memory (the reclamation's evidence;
 * vmq_metrics can report them) */
static ERL_NIF_TERM nif_counts(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqg_res* r = get_res(env, argv[0]);
  if (!r) return enif_make_badarg(env);
  vmqg_stats_t st;
  vmqgb_view_write_begin(r->view);
  const uint64_t v[] = {vmqgb_live(r->subs), vmqgb_live(r->infos), vmqgb_live(r->nodes), vmqgb_live(r->mps),
                        r->sub_t.live, r->info_t.live, r->sub_t.chunks + r->info_t.chunks + r->group_t.chunks,
                        r->sub_t.compactions + r->info_t.compactions, r->terms_dropped};
  uint64_t runs = 0;
  int waiting = 0;
  vmqgb_view_grace_stats(r->view, &runs, &waiting);
  vmqgb_view_write_end(r->view);
  const int rc = vmqgb_view_ctx_stats(r->view, &st);
  if (rc) return error_term(env, rc);
  const char* names[] = {"subscriber_ids", "subinfo_ids", "node_ids", "mountpoint_ids", "subscriber_terms",
                         "subinfo_terms", "term_chunks", "term_compactions", "terms_dropped",
                         "words", "paths", "keys", "topics", "host_bytes", "device_bytes", "subs",
                         "deferred_runs", "deferred_lists_waiting"};
  const uint64_t w[] = {st.words, st.paths, st.keys, st.topics, st.host_bytes, st.device_bytes, st.subs,
                        runs, (uint64_t)waiting};
  ERL_NIF_TERM items[18];
  for (int i = 0; i < 18; i++)
    items[i] = enif_make_tuple2(env, enif_make_atom(env, names[i]), enif_make_uint64(env, i < 9 ? v[i] : w[i - 9]));
  return enif_make_list_from_array(env, items, 18);
}

/* stats(Ctx) -> {NrOfSubs + NrOfRemoteSubs, DeviceBytes} (vmq_reg_trie.erl:101-112) */
static ERL_NIF_TERM nif_stats(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqg_res* r = get_res(env, argv[0]);
  if (!r) return enif_make_badarg(env);
  vmqg_stats_t st;
  const int rc = vmqgb_view_ctx_stats(r->view, &st);   /* writer mutex, then device mutex (the apply's order) */
  if (rc) return error_term(env, rc);
  return enif_make_tuple2(env, enif_make_uint64(env, st.subs), enif_make_uint64(env, st.device_bytes));
}

/* Dirty schedulers: every call that can wait for the table lock or the
 * device runs on one (add_init applies a 65,536-op batch: host engine +
 * upload).  The table registers plain NIFs that reschedule themselves with
 * enif_schedule_nif (erl_nif 2.7, OTP 17.3+), dirty when the emulator has
 * dirty schedulers — the default from OTP 20; OTP 19.3 only when built with
 * --enable-dirty-schedulers — and on the calling scheduler otherwise, so
 * the library loads on every OTP the reference supports (19.3, 20.3, 21.1,
 * .travis.yml).  Dirty flags in the table itself would refuse the load on
 * an emulator without them. */
static int g_dirty;

#define RESCHEDULE(name, impl, kind)                                                    \
  static ERL_NIF_TERM name(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {        \
    return enif_schedule_nif(env, #impl, g_dirty ? (kind) : 0, impl, argc, argv);       \
  }
RESCHEDULE(d_create, nif_create, ERL_NIF_DIRTY_JOB_IO_BOUND)
RESCHEDULE(d_apply, nif_apply, ERL_NIF_DIRTY_JOB_CPU_BOUND)
RESCHEDULE(d_apply_many, nif_apply_many, ERL_NIF_DIRTY_JOB_CPU_BOUND)
RESCHEDULE(d_add_init, nif_add_init, ERL_NIF_DIRTY_JOB_CPU_BOUND)
RESCHEDULE(d_flush_init, nif_flush_init, ERL_NIF_DIRTY_JOB_CPU_BOUND)
RESCHEDULE(d_match, nif_match, ERL_NIF_DIRTY_JOB_CPU_BOUND)
RESCHEDULE(d_stats, nif_stats, ERL_NIF_DIRTY_JOB_CPU_BOUND)
RESCHEDULE(d_commit, nif_commit, ERL_NIF_DIRTY_JOB_CPU_BOUND)
RESCHEDULE(d_counts, nif_counts, ERL_NIF_DIRTY_JOB_CPU_BOUND)
RESCHEDULE(d_set_option, nif_set_option, ERL_NIF_DIRTY_JOB_CPU_BOUND)

static int load(ErlNifEnv* env, void** priv, ERL_NIF_TERM info) {
  (void)priv; (void)info;
  ErlNifSysInfo si;
  enif_system_info(&si, sizeof si);
  g_dirty = si.dirty_scheduler_support != 0;
  RES = enif_open_resource_type(env, NULL, "vmqg_ctx", res_dtor, ERL_NIF_RT_CREATE, NULL);
  BRES = enif_open_resource_type(env, NULL, "vmqg_batch", bres_dtor, ERL_NIF_RT_CREATE, NULL);
  a_ok = enif_make_atom(env, "ok");
  a_error = enif_make_atom(env, "error");
  a_invalid_topic = enif_make_atom(env, "invalid_topic");
  a_device = enif_make_atom(env, "device");
  a_nomem = enif_make_atom(env, "nomem");
  a_badarg = enif_make_atom(env, "badarg");
  a_limit = enif_make_atom(env, "limit");
  a_busy = enif_make_atom(env, "busy");
  a_internal = enif_make_atom(env, "internal");
  a_records = enif_make_atom(env, "records");
  a_ranges = enif_make_atom(env, "ranges");
  return RES && BRES ? 0 : 1;
}

static ErlNifFunc funcs[] = {
    {"create", 1, d_create, 0},
    {"apply", 3, d_apply, 0},
    {"apply_many", 2, d_apply_many, 0},
    {"add_init", 6, d_add_init, 0},
    {"flush_init", 1, d_flush_init, 0},
    {"batch_new", 1, nif_batch_new, 0},
    {"match", 4, d_match, 0},
    {"stats", 1, d_stats, 0},
    {"commit", 1, d_commit, 0},
    {"counts", 1, d_counts, 0},
    {"set_option", 3, d_set_option, 0},
};

ERL_NIF_INIT(vmqg_nif, funcs, load, NULL, NULL, NULL)
