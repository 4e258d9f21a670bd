/*
 * vmqr_nif.c — erl_nif glue of the retained-message matcher (include/vmqr.h)
 * behind vmq_retain_srv.
 *
 * Replaces, in apps/vmq_server/src/vmq_retain_srv.erl:
 *   insert/3 (:68-71), delete/2 (:63-66), the init fold of the metadata
 *   store (:129-138)                       -> apply/2 (vmqr_apply)
 *   match_fold/4 (:75-99), for a batch     -> match/2 (vmqr_match_batch)
 *   stats/0 (:101-113)                     -> stats/1 (vmqr_stats)
 * The #retain_msg{} payloads stay in Erlang, keyed by the integer message
 * id the caller passes to insert (vmq_retain_ids in INTEGRATION.md).
 *
 * Terms: a mountpoint (string) -> a dense mountpoint id (an interner keyed by
 * its external term format); a topic / filter is its word list, each word
 * one dictionary id ("+" / "#" the reserved ones).  Retained topics intern
 * their words (create); a filter's unseen words map to VMQG_WORD_UNKNOWN
 * (they equal no retained word).  One mutex per context: vmqr contexts are
 * not re-entrant (vmqr.h).
 *
 * Written against the erl_nif API of OTP 19.3 .. 21 (as vmqg_nif.c:
 * enif_term_to_binary, enif_schedule_nif / dirty_scheduler_support); OTP is
 * not in this image: compiled and run over the erl_nif test double
 * (tests/c/mock_erl_nif, tests/c/retain_nif_check.c).
 */
#include <erl_nif.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>

#include "vmqg_batch.h"
#include "vmqr.h"

typedef struct {
  vmqr_ctx* ctx;
  pthread_mutex_t mu;
  vmqgb_interner* mps;
} vmqr_res;

static ErlNifResourceType* RES;
static ERL_NIF_TERM a_ok, a_error, a_insert, a_delete, a_badarg, a_nomem, a_device, a_limit;
static int g_dirty;

static ERL_NIF_TERM error_term(ErlNifEnv* env, int rc) {
  ERL_NIF_TERM r = rc == VMQG_E_NOMEM ? a_nomem : rc == VMQG_E_DEVICE ? a_device : rc == VMQG_E_LIMIT ? a_limit : a_badarg;
  return enif_make_tuple2(env, a_error, r);
}

static void res_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  vmqr_res* r = (vmqr_res*)obj;
  if (r->ctx) vmqr_destroy(r->ctx);
  vmqgb_interner_free(r->mps);
  pthread_mutex_destroy(&r->mu);
}

static vmqr_res* get_res(ErlNifEnv* env, ERL_NIF_TERM t) {
  vmqr_res* r = NULL;
  return enif_get_resource(env, t, RES, (void**)&r) ? r : NULL;
}

/* mountpoint id of MP; create: intern it (a retained topic: the library
 * grows its per-mountpoint lists), else VMQG_NONE for an unseen one (it
 * holds nothing) */
static int mp_id(ErlNifEnv* env, vmqr_res* r, ERL_NIF_TERM mp, int create, uint32_t* id) {
  ErlNifBinary b;
  if (!enif_term_to_binary(env, mp, &b)) return VMQG_E_NOMEM;
  int rc = 0;
  if (create) {
    *id = vmqgb_intern(r->mps, b.data, b.size);
    if (*id == VMQG_NONE) rc = VMQG_E_NOMEM;
    else if (*id >= VMQG_MAX_MOUNTPOINTS) rc = VMQG_E_LIMIT;
  } else if (vmqgb_lookup(r->mps, b.data, b.size, id) != 0) {
    *id = VMQG_NONE;
  }
  enif_release_binary(&b);
  return rc;
}

/* a word list's ids into *ids (grown by the caller's buffer); create as vmqr_intern_words */
typedef struct {
  uint32_t* v;
  size_t n, cap;
} u32vec;

static int vec_push(u32vec* w, uint32_t x) {
  if (w->n == w->cap) {
    size_t c = w->cap ? 2 * w->cap : 256;
    uint32_t* nv = (uint32_t*)enif_realloc(w->v, c * sizeof(uint32_t));
    if (!nv) return 0;
    w->v = nv;
    w->cap = c;
  }
  w->v[w->n++] = x;
  return 1;
}

static int topic_ids(ErlNifEnv* env, vmqr_res* r, ERL_NIF_TERM topic, int create, u32vec* out, uint32_t* nwords) {
  unsigned len;
  if (!enif_get_list_length(env, topic, &len)) return VMQG_E_INVAL;
  ERL_NIF_TERM h, t = topic;
  *nwords = len;
  while (enif_get_list_cell(env, t, &h, &t)) {
    ErlNifBinary wb;
    uint32_t id = VMQG_WORD_UNKNOWN;
    if (enif_inspect_binary(env, h, &wb)) {
      const uint64_t offs[2] = {0, wb.size};
      static const uint8_t none[1] = {0};
      const int rc = vmqr_intern_words(r->ctx, wb.size ? wb.data : none, offs, 1, create, &id);
      if (rc) return rc;
    } else if (create) {
      return VMQG_E_INVAL;   /* a retained topic is validated words (vmq_reg:publish/4) */
    }
    if (!vec_push(out, id)) return VMQG_E_NOMEM;
  }
  return 0;
}

/* create(#{device => D}) -> {ok, Ctx} | {error, _}  (vmq_retain_srv:init/1 :128-138) */
static ERL_NIF_TERM nif_create(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  ERL_NIF_TERM v;
  int device = 0;
  if (enif_get_map_value(env, argv[0], enif_make_atom(env, "device"), &v)) enif_get_int(env, v, &device);
  vmqr_res* r = (vmqr_res*)enif_alloc_resource(RES, sizeof(vmqr_res));
  memset(r, 0, sizeof(*r));
  pthread_mutex_init(&r->mu, NULL);
  r->mps = vmqgb_interner_new();
  uint32_t id;
  mp_id(env, r, enif_make_string(env, "", ERL_NIF_LATIN1), 1, &id);   /* "" is mountpoint 0 */
  vmqr_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.device = device;
  cfg.max_mountpoints = 1024;   /* the initial range: more mountpoints grow it */
  int err = 0;
  r->ctx = r->mps ? vmqr_create(&cfg, &err) : NULL;
  if (!r->mps) err = VMQG_E_NOMEM;
  ERL_NIF_TERM ret = r->ctx ? enif_make_tuple2(env, a_ok, enif_make_resource(env, r)) : error_term(env, err);
  enif_release_resource(r);
  return ret;
}

/* apply(Ctx, [{insert, MP, Topic, Id} | {delete, MP, Topic}]) -> ok | {error, _}:
 * the ops in order as one vmqr_apply (insert replaces: an ets set, :68-71) */
static ERL_NIF_TERM nif_apply(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqr_res* r = get_res(env, argv[0]);
  unsigned n;
  if (!r || !enif_get_list_length(env, argv[1], &n)) return enif_make_badarg(env);
  vmqr_op* ops = (vmqr_op*)enif_alloc((n ? n : 1) * sizeof(vmqr_op));
  u32vec w = {NULL, 0, 0};
  if (!ops) return error_term(env, VMQG_E_NOMEM);
  pthread_mutex_lock(&r->mu);
  int rc = 0;
  ERL_NIF_TERM h, t = argv[1];
  for (unsigned i = 0; !rc && i < n; i++) {
    enif_get_list_cell(env, t, &h, &t);
    int ar;
    const ERL_NIF_TERM* el;
    if (!enif_get_tuple(env, h, &ar, &el) || ar < 3) { rc = VMQG_E_INVAL; break; }
    const int ins = enif_is_identical(el[0], a_insert);
    if (!(ins && ar == 4) && !(enif_is_identical(el[0], a_delete) && ar == 3)) { rc = VMQG_E_INVAL; break; }
    uint32_t mp, nw;
    unsigned msg = 0;
    if (ins && !enif_get_uint(env, el[3], &msg)) { rc = VMQG_E_INVAL; break; }
    if ((rc = mp_id(env, r, el[1], 1, &mp))) break;
    const size_t off = w.n;
    if ((rc = topic_ids(env, r, el[2], 1, &w, &nw))) break;
    if (nw == 0) { rc = VMQG_E_INVAL; break; }
    ops[i] = (vmqr_op){ins ? VMQR_OP_INSERT : VMQR_OP_DELETE, mp, (uint32_t)off, nw, (uint32_t)msg, 0};
  }
  if (!rc) rc = vmqr_apply(r->ctx, ops, n, w.v, w.n);
  pthread_mutex_unlock(&r->mu);
  enif_free(ops);
  enif_free(w.v);
  return rc ? error_term(env, rc) : a_ok;
}

/* match(Ctx, [{MP, Filter}]) -> [[Id]] | {error, _}: match_fold/4 (:75-99)
 * for a batch of filters — per filter the message ids of the retained
 * topics it matches (an ets set has no order: the ids are sorted) */
/* Sorts n message ids: insertion sort for a short span, else an LSD radix
 * sort (8-bit digits, a digit on which every id agrees is skipped) through
 * tmp (n entries) — O(n), since one '#' filter may match every retained
 * message (match_fold/4 walks the whole table, vmq_retain_srv.erl:75-99). */
static void sort_ids(uint32_t* a, size_t n, uint32_t* tmp) {
  if (n <= 32) {
    for (size_t i = 1; i < n; i++)
      for (size_t j = i; j > 0 && a[j - 1] > a[j]; j--) { const uint32_t x = a[j]; a[j] = a[j - 1]; a[j - 1] = x; }
    return;
  }
  uint32_t *src = a, *dst = tmp;
  for (int shift = 0; shift < 32; shift += 8) {
    size_t cnt[257] = {0};
    for (size_t i = 0; i < n; i++) cnt[((src[i] >> shift) & 255u) + 1]++;
    if (cnt[((src[0] >> shift) & 255u) + 1] == n) continue;   /* one bucket: the digit orders nothing */
    for (int d = 0; d < 256; d++) cnt[d + 1] += cnt[d];
    for (size_t i = 0; i < n; i++) dst[cnt[(src[i] >> shift) & 255u]++] = src[i];
    uint32_t* x = src; src = dst; dst = x;
  }
  if (src != a) memcpy(a, src, n * sizeof(uint32_t));
}

static ERL_NIF_TERM nif_match(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqr_res* r = get_res(env, argv[0]);
  unsigned n;
  if (!r || !enif_get_list_length(env, argv[1], &n)) return enif_make_badarg(env);
  vmqg_pub* f = (vmqg_pub*)enif_alloc((n ? n : 1) * sizeof(vmqg_pub));
  uint64_t* offs = (uint64_t*)enif_alloc((n + 1) * sizeof(uint64_t));
  u32vec w = {NULL, 0, 0};
  uint32_t* out = NULL;
  size_t cap = 1024, got = 0;
  int rc = f && offs ? 0 : VMQG_E_NOMEM;
  pthread_mutex_lock(&r->mu);
  ERL_NIF_TERM h, t = argv[1];
  for (unsigned i = 0; !rc && i < n; i++) {
    enif_get_list_cell(env, t, &h, &t);
    int ar;
    const ERL_NIF_TERM* el;
    uint32_t mp, nw;
    if (!enif_get_tuple(env, h, &ar, &el) || ar != 2) { rc = VMQG_E_INVAL; break; }
    if ((rc = mp_id(env, r, el[0], 0, &mp))) break;
    const size_t off = w.n;
    if ((rc = topic_ids(env, r, el[1], 0, &w, &nw))) break;
    f[i] = (vmqg_pub){mp, (uint32_t)off, nw, 0};
  }
  while (!rc) {
    uint32_t* nb = (uint32_t*)enif_realloc(out, cap * sizeof(uint32_t));
    if (!nb) { rc = VMQG_E_NOMEM; break; }
    out = nb;
    rc = vmqr_match_batch(r->ctx, f, n, w.v, w.n, out, cap, &got, offs);
    if (rc == VMQG_E_OVERFLOW && got > cap) { cap = got; rc = 0; continue; }
    break;
  }
  pthread_mutex_unlock(&r->mu);
  ERL_NIF_TERM ret;
  if (rc) {
    ret = error_term(env, rc);
  } else {
    ERL_NIF_TERM* lists = (ERL_NIF_TERM*)enif_alloc((n ? n : 1) * sizeof(ERL_NIF_TERM));
    ERL_NIF_TERM* ids = (ERL_NIF_TERM*)enif_alloc((got ? got : 1) * sizeof(ERL_NIF_TERM));
    uint64_t span = 0;
    for (unsigned i = 0; i < n; i++) if (offs[i + 1] - offs[i] > span) span = offs[i + 1] - offs[i];
    uint32_t* tmp = span > 32 ? (uint32_t*)enif_alloc(span * sizeof(uint32_t)) : NULL;
    if (span > 32 && !tmp) { enif_free(lists); lists = NULL; }
    for (unsigned i = 0; lists && ids && i < n; i++) {
      const uint64_t lo = offs[i], hi = offs[i + 1];
      sort_ids(out + lo, (size_t)(hi - lo), tmp);   /* a '#' filter can match every retained message */
      for (uint64_t k = lo; k < hi; k++) ids[k] = enif_make_uint(env, out[k]);
      lists[i] = enif_make_list_from_array(env, ids + lo, (unsigned)(hi - lo));
    }
    ret = lists && ids ? enif_make_list_from_array(env, lists, n) : error_term(env, VMQG_E_NOMEM);
    enif_free(lists);
    enif_free(ids);
    enif_free(tmp);
  }
  enif_free(f);
  enif_free(offs);
  enif_free(w.v);
  enif_free(out);
  return ret;
}

/* stats(Ctx) -> {Retained, DeviceBytes}  (stats/0, :101-113) */
static ERL_NIF_TERM nif_stats(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqr_res* r = get_res(env, argv[0]);
  if (!r) return enif_make_badarg(env);
  vmqr_stats_t st;
  pthread_mutex_lock(&r->mu);
  const int rc = vmqr_stats(r->ctx, &st);
  pthread_mutex_unlock(&r->mu);
  if (rc) return error_term(env, rc);
  return enif_make_tuple2(env, enif_make_uint64(env, st.retained), enif_make_uint64(env, st.device_bytes));
}

/* dirty rescheduling as in vmqg_nif.c (loads on OTP 19.3 .. 21) */
#define RESCHEDULE(name, impl, kind)                                              \
  static ERL_NIF_TERM name(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) { \
    return enif_schedule_nif(env, #impl, g_dirty ? (kind) : 0, impl, argc, argv); \
  }
RESCHEDULE(d_create, nif_create, ERL_NIF_DIRTY_JOB_IO_BOUND)
RESCHEDULE(d_apply, nif_apply, ERL_NIF_DIRTY_JOB_CPU_BOUND)
RESCHEDULE(d_match, nif_match, ERL_NIF_DIRTY_JOB_CPU_BOUND)
RESCHEDULE(d_stats, nif_stats, ERL_NIF_DIRTY_JOB_CPU_BOUND)

static int load(ErlNifEnv* env, void** priv, ERL_NIF_TERM info) {
  (void)priv; (void)info;
  ErlNifSysInfo si;
  enif_system_info(&si, sizeof si);
  g_dirty = si.dirty_scheduler_support != 0;
  RES = enif_open_resource_type(env, NULL, "vmqr_ctx", res_dtor, ERL_NIF_RT_CREATE, NULL);
  a_ok = enif_make_atom(env, "ok");
  a_error = enif_make_atom(env, "error");
  a_insert = enif_make_atom(env, "insert");
  a_delete = enif_make_atom(env, "delete");
  a_badarg = enif_make_atom(env, "badarg");
  a_nomem = enif_make_atom(env, "nomem");
  a_device = enif_make_atom(env, "device");
  a_limit = enif_make_atom(env, "limit");
  return RES ? 0 : 1;
}

static ErlNifFunc funcs[] = {
    {"create", 1, d_create, 0},
    {"apply", 2, d_apply, 0},
    {"match", 2, d_match, 0},
    {"stats", 1, d_stats, 0},
};

ERL_NIF_INIT(vmqr_nif, funcs, load, NULL, NULL, NULL)
