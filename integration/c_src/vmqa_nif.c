/*
 * vmqa_nif.c — erl_nif glue of the ACL checker (include/vmqa.h) behind
 * vmq_acl.
 *
 * Replaces, in apps/vmq_acl/src/vmq_acl.erl:
 *   the six ets tables after load_from_list/1 / load_from_file/1
 *   (:114-144; the parser, parse_acl_line/2 and in/3, stays in Erlang)
 *                                            -> load/2 (vmqa_load)
 *   check/4 (:179-204) with topic/3 + subst/5 (:206-217), for a batch
 *                                            -> check/2 (vmqa_check_batch)
 * auth_on_subscribe/3 checks all its topics in one call (:78-85).
 *
 * Terms: rule words and users are interned by the context's dictionary
 * ("%u" / "%c" / "%m" are the reserved ids); in a check, a string the
 * dictionary does not hold (a client id, a topic word no rule has, the
 * mountpoint) gets a batch-local id >= VMQA_EPHEMERAL, one per distinct
 * string within the call, so subst/5's substitutions compare exactly as
 * the reference compares terms.  A user other than a binary (`undefined`)
 * is VMQA_NO_USER: no user table, and substituted for %u it equals no word.
 * A check of an empty topic, or one whose first word is not a binary, has
 * no check/4 clause: its result is {error, function_clause}.  One mutex per
 * context (vmqa contexts are not re-entrant).
 *
 * Written against the erl_nif API of OTP 19.3 .. 21 (as vmqg_nif.c); OTP is
 * not in this image: compiled and run over the erl_nif test double
 * (tests/c/mock_erl_nif, tests/c/acl_nif_check.c).
 */
#include <erl_nif.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>

#include "vmqa.h"
#include "vmqg_batch.h"

typedef struct {
  vmqa_ctx* ctx;
  pthread_mutex_t mu;
} vmqa_res;

static ErlNifResourceType* RES;
static ERL_NIF_TERM a_ok, a_error, a_read, a_write, a_all, a_user, a_pattern, a_true, a_false, a_badarg,
    a_nomem, a_device, a_function_clause;
static int g_dirty;

static ERL_NIF_TERM error_term(ErlNifEnv* env, int rc) {
  ERL_NIF_TERM r = rc == VMQG_E_NOMEM ? a_nomem : rc == VMQG_E_DEVICE ? a_device : a_badarg;
  return enif_make_tuple2(env, a_error, r);
}

static void res_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  vmqa_res* r = (vmqa_res*)obj;
  if (r->ctx) vmqa_destroy(r->ctx);
  pthread_mutex_destroy(&r->mu);
}

static vmqa_res* get_res(ErlNifEnv* env, ERL_NIF_TERM t) {
  vmqa_res* r = NULL;
  return enif_get_resource(env, t, RES, (void**)&r) ? r : NULL;
}

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

static int word_id(vmqa_res* r, const uint8_t* p, size_t n, int create, uint32_t* id) {
  static const uint8_t none[1] = {0};
  const uint64_t offs[2] = {0, n};
  return vmqa_intern_words(r->ctx, n ? p : none, offs, 1, create, id);
}

/* a check's string -> its dictionary id, or the call's ephemeral id for it */
static int check_id(vmqa_res* r, vmqgb_interner* eph, const uint8_t* p, size_t n, uint32_t* id) {
  int rc = word_id(r, p, n, 0, id);
  if (rc) return rc;
  if (*id == VMQG_WORD_UNKNOWN) {
    const uint32_t e = vmqgb_intern(eph, p, n);
    if (e == VMQG_NONE) return VMQG_E_NOMEM;
    *id = VMQA_EPHEMERAL + e;
  }
  return 0;
}

/* create(#{device => D}) -> {ok, Ctx} | {error, _}  (vmq_acl:init/0 :105-112) */
static ERL_NIF_TERM nif_create(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  ERL_NIF_TERM v;
  int device = 0;
  if (enif_get_map_value(env, argv[0], enif_make_atom(env, "device"), &v)) enif_get_int(env, v, &device);
  vmqa_res* r = (vmqa_res*)enif_alloc_resource(RES, sizeof(vmqa_res));
  memset(r, 0, sizeof(*r));
  pthread_mutex_init(&r->mu, NULL);
  vmqa_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.device = device;
  int err = 0;
  r->ctx = vmqa_create(&cfg, &err);
  ERL_NIF_TERM ret = r->ctx ? enif_make_tuple2(env, a_ok, enif_make_resource(env, r)) : error_term(env, err);
  enif_release_resource(r);
  return ret;
}

/* load(Ctx, [{read | write, all | user | pattern, User, Words}]) -> ok |
 * {error, _}: the six tables as load_from_list/1 left them (duplicates
 * absorbed, as by an ets set) */
static ERL_NIF_TERM nif_load(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqa_res* r = get_res(env, argv[0]);
  unsigned n;
  if (!r || !enif_get_list_length(env, argv[1], &n)) return enif_make_badarg(env);
  vmqa_rule* rules = (vmqa_rule*)enif_alloc((n ? n : 1) * sizeof(vmqa_rule));
  u32vec w = {NULL, 0, 0};
  if (!rules) return error_term(env, VMQG_E_NOMEM);
  pthread_mutex_lock(&r->mu);
  int rc = 0;
  ERL_NIF_TERM h, t = argv[1];
  for (unsigned i = 0; !rc && i < n; i++) {
    enif_get_list_cell(env, t, &h, &t);
    int ar;
    const ERL_NIF_TERM* el;
    if (!enif_get_tuple(env, h, &ar, &el) || ar != 4) { rc = VMQG_E_INVAL; break; }
    const uint32_t type = enif_is_identical(el[0], a_read) ? VMQA_READ : enif_is_identical(el[0], a_write) ? VMQA_WRITE : 0;
    const uint32_t table = enif_is_identical(el[1], a_all) ? VMQA_TABLE_ALL
                         : enif_is_identical(el[1], a_user) ? VMQA_TABLE_USER
                         : enif_is_identical(el[1], a_pattern) ? VMQA_TABLE_PATTERN : 99u;
    if (!type || table == 99u) { rc = VMQG_E_INVAL; break; }
    uint32_t user = 0;
    if (table == VMQA_TABLE_USER) {
      ErlNifBinary ub;
      if (!enif_inspect_binary(env, el[2], &ub)) { rc = VMQG_E_INVAL; break; }
      if ((rc = word_id(r, ub.data, ub.size, 1, &user))) break;
    }
    const size_t off = w.n;
    ERL_NIF_TERM wh, wt = el[3];
    while (!rc && enif_get_list_cell(env, wt, &wh, &wt)) {
      ErlNifBinary wb;
      uint32_t id;
      if (!enif_inspect_binary(env, wh, &wb)) { rc = VMQG_E_INVAL; break; }
      if ((rc = word_id(r, wb.data, wb.size, 1, &id))) break;
      if (!vec_push(&w, id)) rc = VMQG_E_NOMEM;
    }
    if (!rc && w.n == off) rc = VMQG_E_INVAL;
    rules[i] = (vmqa_rule){type, table, user, (uint32_t)off, (uint32_t)(w.n - off), 0};
  }
  if (!rc) rc = vmqa_load(r->ctx, rules, n, w.v, w.n);
  pthread_mutex_unlock(&r->mu);
  enif_free(rules);
  enif_free(w.v);
  return rc ? error_term(env, rc) : a_ok;
}

/* check(Ctx, [{read | write, Topic, User, MP, ClientId}]) -> [true | false |
 * {error, function_clause}]: check/4 per request (MP the mountpoint string,
 * list_to_binary'd by topic/3, :206-207) */
static ERL_NIF_TERM nif_check(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqa_res* r = get_res(env, argv[0]);
  unsigned n;
  if (!r || !enif_get_list_length(env, argv[1], &n)) return enif_make_badarg(env);
  vmqa_req* reqs = (vmqa_req*)enif_alloc((n ? n : 1) * sizeof(vmqa_req));
  uint8_t* ok = (uint8_t*)enif_alloc(n ? n : 1);
  uint8_t* bad = (uint8_t*)enif_alloc(n ? n : 1);   /* no check/4 clause */
  u32vec w = {NULL, 0, 0};
  vmqgb_interner* eph = vmqgb_interner_new();
  int rc = reqs && ok && bad && eph ? 0 : VMQG_E_NOMEM;
  if (!rc) pthread_mutex_lock(&r->mu);
  ERL_NIF_TERM h, t = argv[1];
  size_t k = 0;   /* requests passed to the device */
  for (unsigned i = 0; !rc && i < n; i++) {
    enif_get_list_cell(env, t, &h, &t);
    int ar;
    const ERL_NIF_TERM* el;
    ErlNifBinary mpb, cb, ub, first;
    bad[i] = 0;
    if (!enif_get_tuple(env, h, &ar, &el) || ar != 5) { rc = VMQG_E_INVAL; break; }
    const uint32_t type = enif_is_identical(el[0], a_read) ? VMQA_READ : enif_is_identical(el[0], a_write) ? VMQA_WRITE : 0;
    if (!type) { rc = VMQG_E_INVAL; break; }
    ERL_NIF_TERM wh, wt = el[1];
    if (!enif_get_list_cell(env, wt, &wh, &wt) || !enif_inspect_binary(env, wh, &first)) { bad[i] = 1; continue; }
    if (!enif_inspect_iolist_as_binary(env, el[3], &mpb) || !enif_inspect_binary(env, el[4], &cb)) {
      rc = VMQG_E_INVAL;
      break;
    }
    vmqa_req q = {type, VMQA_NO_USER, 0, 0, (uint32_t)w.n, 0};
    if (enif_inspect_binary(env, el[2], &ub) && (rc = check_id(r, eph, ub.data, ub.size, &q.user))) break;
    if ((rc = check_id(r, eph, cb.data, cb.size, &q.client)) || (rc = check_id(r, eph, mpb.data, mpb.size, &q.mountpoint)))
      break;
    uint32_t id;
    if ((rc = check_id(r, eph, first.data, first.size, &id))) break;
    if (!vec_push(&w, id)) { rc = VMQG_E_NOMEM; break; }
    while (!rc && enif_get_list_cell(env, wt, &wh, &wt)) {
      ErlNifBinary wb;
      if (enif_inspect_binary(env, wh, &wb)) rc = check_id(r, eph, wb.data, wb.size, &id);
      else id = 0xFFFFFFF0u;   /* not a binary: equals no rule word (an ephemeral id no string gets) */
      if (!rc && !vec_push(&w, id)) rc = VMQG_E_NOMEM;
    }
    q.nwords = (uint32_t)(w.n - q.word_off);
    reqs[k++] = q;
  }
  if (!rc && k) rc = vmqa_check_batch(r->ctx, reqs, k, w.v, w.n, ok);
  if (reqs && ok && bad && eph) pthread_mutex_unlock(&r->mu);
  ERL_NIF_TERM ret;
  if (rc) {
    ret = error_term(env, rc);
  } else {
    ERL_NIF_TERM* res = (ERL_NIF_TERM*)enif_alloc((n ? n : 1) * sizeof(ERL_NIF_TERM));
    size_t j = 0;
    for (unsigned i = 0; res && i < n; i++)
      res[i] = bad[i] ? enif_make_tuple2(env, a_error, a_function_clause) : ok[j++] ? a_true : a_false;
    ret = res ? enif_make_list_from_array(env, res, n) : error_term(env, VMQG_E_NOMEM);
    enif_free(res);
  }
  enif_free(reqs);
  enif_free(ok);
  enif_free(bad);
  enif_free(w.v);
  vmqgb_interner_free(eph);
  return ret;
}

/* stats(Ctx) -> {Rules, Users, DeviceBytes} */
static ERL_NIF_TERM nif_stats(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  vmqa_res* r = get_res(env, argv[0]);
  if (!r) return enif_make_badarg(env);
  vmqa_stats_t st;
  pthread_mutex_lock(&r->mu);
  const int rc = vmqa_stats(r->ctx, &st);
  pthread_mutex_unlock(&r->mu);
  if (rc) return error_term(env, rc);
  const ERL_NIF_TERM el[3] = {enif_make_uint64(env, st.rules), enif_make_uint64(env, st.users),
                              enif_make_uint64(env, st.device_bytes)};
  return enif_make_tuple_from_array(env, el, 3);
}

/* dirty rescheduling as in vmqg_nif.c (loads on OTP 19.3 .. 21) */
#define RESCHEDULE(name, impl, kind)                                              \
  static ERL_NIF_TERM name(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) { \
    return enif_schedule_nif(env, #impl, g_dirty ? (kind) : 0, impl, argc, argv); \
  }
RESCHEDULE(d_create, nif_create, ERL_NIF_DIRTY_JOB_IO_BOUND)
RESCHEDULE(d_load, nif_load, ERL_NIF_DIRTY_JOB_CPU_BOUND)
RESCHEDULE(d_check, nif_check, ERL_NIF_DIRTY_JOB_CPU_BOUND)
RESCHEDULE(d_stats, nif_stats, ERL_NIF_DIRTY_JOB_CPU_BOUND)

static int load(ErlNifEnv* env, void** priv, ERL_NIF_TERM info) {
  (void)priv; (void)info;
  ErlNifSysInfo si;
  enif_system_info(&si, sizeof si);
  g_dirty = si.dirty_scheduler_support != 0;
  RES = enif_open_resource_type(env, NULL, "vmqa_ctx", res_dtor, ERL_NIF_RT_CREATE, NULL);
  a_ok = enif_make_atom(env, "ok");
  a_error = enif_make_atom(env, "error");
  a_read = enif_make_atom(env, "read");
  a_write = enif_make_atom(env, "write");
  a_all = enif_make_atom(env, "all");
  a_user = enif_make_atom(env, "user");
  a_pattern = enif_make_atom(env, "pattern");
  a_true = enif_make_atom(env, "true");
  a_false = enif_make_atom(env, "false");
  a_badarg = enif_make_atom(env, "badarg");
  a_nomem = enif_make_atom(env, "nomem");
  a_device = enif_make_atom(env, "device");
  a_function_clause = enif_make_atom(env, "function_clause");
  return RES ? 0 : 1;
}

static ErlNifFunc funcs[] = {
    {"create", 1, d_create, 0},
    {"load", 2, d_load, 0},
    {"check", 2, d_check, 0},
    {"stats", 1, d_stats, 0},
};

ERL_NIF_INIT(vmqa_nif, funcs, load, NULL, NULL, NULL)
