/*
 * erl_nif_mock.c — the TEST DOUBLE behind tests/c/mock_erl_nif/erl_nif.h: a
 * minimal term model (atoms, integers, binaries, tuples, lists, maps,
 * resources) with the documented semantics of the enif_* calls
 * integration/c_src/vmqg_nif.c makes, plus mock_* constructors and a printer
 * for the check program.  Terms are immutable cells never freed (a check
 * program's lifetime); the resource refcounts and destructors are real, so
 * the NIF's keep/release pairs are exercised.
 */
#include "erl_nif.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { T_ATOM, T_INT, T_BIN, T_TUPLE, T_NIL, T_CONS, T_MAP, T_RES };

typedef struct cell {
  int type;
  int64_t i;                 /* T_INT */
  size_t n;                  /* T_BIN bytes, T_TUPLE / T_MAP arity */
  unsigned char* bytes;      /* T_BIN, T_ATOM (NUL-terminated name) */
  ERL_NIF_TERM* el;          /* T_TUPLE elements; T_MAP keys then values; T_CONS head, tail */
  void* res;                 /* T_RES */
} cell;

/* an environment owns the cells copied into it (enif_make_copy) and frees
 * them with itself: a NIF that reads a term of a freed environment reads
 * freed memory (ASan / the test's cell count see it) */
struct enif_environment_t { struct cell** owned; size_t n, cap; };
static long env_cells;   /* cells owned by live environments (mock_env_cells) */
struct enif_resource_type_t { ErlNifResourceDtor* dtor; char name[64]; };

typedef struct { ErlNifResourceType* type; long refs; } res_hdr;

static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
static cell nil_cell = {T_NIL, 0, 0, NULL, NULL, NULL};

static cell* C(ERL_NIF_TERM t) { return (cell*)t; }
static ERL_NIF_TERM T(cell* c) { return (ERL_NIF_TERM)c; }

static cell* new_cell(int type) {
  cell* c = (cell*)calloc(1, sizeof(cell));
  c->type = type;
  return c;
}

void* enif_alloc(size_t size) { return malloc(size ? size : 1); }
void* enif_realloc(void* ptr, size_t size) { return realloc(ptr, size ? size : 1); }
void enif_free(void* ptr) { free(ptr); }
ErlNifEnv* enif_alloc_env(void) { return (ErlNifEnv*)calloc(1, sizeof(ErlNifEnv)); }
void enif_free_env(ErlNifEnv* env) {
  if (!env) return;
  for (size_t i = 0; i < env->n; i++) {
    free(env->owned[i]->bytes);
    free(env->owned[i]->el);
    free(env->owned[i]);
  }
  __atomic_fetch_sub(&env_cells, (long)env->n, __ATOMIC_RELAXED);
  free(env->owned);
  free(env);
}
long mock_env_cells(void) { return __atomic_load_n(&env_cells, __ATOMIC_RELAXED); }

/* atoms are interned: one cell per name */
static cell** atoms;
static size_t natoms;
ERL_NIF_TERM enif_make_atom(ErlNifEnv* env, const char* name) {
  (void)env;
  pthread_mutex_lock(&mu);
  for (size_t i = 0; i < natoms; i++)
    if (!strcmp((const char*)atoms[i]->bytes, name)) { pthread_mutex_unlock(&mu); return T(atoms[i]); }
  cell* c = new_cell(T_ATOM);
  c->bytes = (unsigned char*)strdup(name);
  c->n = strlen(name);
  atoms = (cell**)realloc(atoms, (natoms + 1) * sizeof(cell*));
  atoms[natoms++] = c;
  pthread_mutex_unlock(&mu);
  return T(c);
}

static ERL_NIF_TERM make_tuple(size_t n, const ERL_NIF_TERM* el) {
  cell* c = new_cell(T_TUPLE);
  c->n = n;
  c->el = (ERL_NIF_TERM*)malloc((n ? n : 1) * sizeof(ERL_NIF_TERM));
  memcpy(c->el, el, n * sizeof(ERL_NIF_TERM));
  return T(c);
}
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv* env, ERL_NIF_TERM a, ERL_NIF_TERM b) {
  (void)env;
  const ERL_NIF_TERM e[2] = {a, b};
  return make_tuple(2, e);
}
ERL_NIF_TERM enif_make_tuple4(ErlNifEnv* env, ERL_NIF_TERM a, ERL_NIF_TERM b, ERL_NIF_TERM c, ERL_NIF_TERM d) {
  (void)env;
  const ERL_NIF_TERM e[4] = {a, b, c, d};
  return make_tuple(4, e);
}
static ERL_NIF_TERM cons(ERL_NIF_TERM h, ERL_NIF_TERM t) {
  cell* c = new_cell(T_CONS);
  c->el = (ERL_NIF_TERM*)malloc(2 * sizeof(ERL_NIF_TERM));
  c->el[0] = h;
  c->el[1] = t;
  return T(c);
}
ERL_NIF_TERM enif_make_list_from_array(ErlNifEnv* env, const ERL_NIF_TERM arr[], unsigned cnt) {
  (void)env;
  ERL_NIF_TERM l = T(&nil_cell);
  for (unsigned i = cnt; i-- > 0;) l = cons(arr[i], l);
  return l;
}
static ERL_NIF_TERM make_int(int64_t v) {
  cell* c = new_cell(T_INT);
  c->i = v;
  return T(c);
}
ERL_NIF_TERM enif_make_string(ErlNifEnv* env, const char* s, ErlNifCharEncoding enc) {
  (void)env; (void)enc;
  ERL_NIF_TERM l = T(&nil_cell);
  for (size_t i = strlen(s); i-- > 0;) l = cons(make_int((unsigned char)s[i]), l);
  return l;
}
ERL_NIF_TERM enif_make_uint64(ErlNifEnv* env, uint64_t i) { (void)env; return make_int((int64_t)i); }
ERL_NIF_TERM enif_make_uint(ErlNifEnv* env, unsigned i) { (void)env; return make_int((int64_t)i); }
ERL_NIF_TERM enif_make_tuple_from_array(ErlNifEnv* env, const ERL_NIF_TERM arr[], unsigned cnt) {
  (void)env;
  return make_tuple(cnt, arr);
}
ERL_NIF_TERM enif_make_badarg(ErlNifEnv* env) { return enif_make_atom(env, "$badarg_exception"); }
static cell* owned_cell(ErlNifEnv* e, int type) {
  cell* c = new_cell(type);
  if (e->n == e->cap) {
    e->cap = e->cap ? 2 * e->cap : 64;
    e->owned = (cell**)realloc(e->owned, e->cap * sizeof(cell*));
  }
  e->owned[e->n++] = c;
  __atomic_fetch_add(&env_cells, 1, __ATOMIC_RELAXED);
  return c;
}
/* a deep copy owned by dst_env (atoms, [] and resources are shared, as in OTP) */
ERL_NIF_TERM enif_make_copy(ErlNifEnv* dst_env, ERL_NIF_TERM src_term) {
  const cell* a = C(src_term);
  if (!dst_env || a->type == T_ATOM || a->type == T_NIL || a->type == T_RES) return src_term;
  cell* c = owned_cell(dst_env, a->type);
  c->i = a->i;
  c->n = a->n;
  if (a->type == T_BIN) {
    c->bytes = (unsigned char*)malloc(a->n ? a->n : 1);
    memcpy(c->bytes, a->bytes, a->n);
  }
  const size_t k = a->type == T_TUPLE ? a->n : a->type == T_MAP ? 2 * a->n : a->type == T_CONS ? 2 : 0;
  if (k || a->type == T_TUPLE) {
    c->el = (ERL_NIF_TERM*)malloc((k ? k : 1) * sizeof(ERL_NIF_TERM));
    for (size_t i = 0; i < k; i++) c->el[i] = enif_make_copy(dst_env, a->el[i]);
  }
  return T(c);
}
ERL_NIF_TERM enif_make_resource(ErlNifEnv* env, void* obj) {
  (void)env;
  cell* c = new_cell(T_RES);
  c->res = obj;
  enif_keep_resource(obj);   /* the term holds a reference (never dropped: terms are not collected) */
  return T(c);
}

int enif_get_int(ErlNifEnv* env, ERL_NIF_TERM term, int* ip) {
  (void)env;
  if (C(term)->type != T_INT) return 0;
  *ip = (int)C(term)->i;
  return 1;
}
int enif_get_int64(ErlNifEnv* env, ERL_NIF_TERM term, ErlNifSInt64* ip) {
  (void)env;
  if (C(term)->type != T_INT) return 0;
  *ip = C(term)->i;
  return 1;
}
int enif_get_atom(ErlNifEnv* env, ERL_NIF_TERM atom, char* buf, unsigned size, ErlNifCharEncoding encoding) {
  (void)env; (void)encoding;
  if (C(atom)->type != T_ATOM || C(atom)->n + 1 > size) return 0;
  memcpy(buf, C(atom)->bytes, C(atom)->n);
  buf[C(atom)->n] = 0;
  return (int)C(atom)->n + 1;
}
int enif_get_uint(ErlNifEnv* env, ERL_NIF_TERM term, unsigned* ip) {
  (void)env;
  if (C(term)->type != T_INT || C(term)->i < 0 || C(term)->i > 0xFFFFFFFFll) return 0;
  *ip = (unsigned)C(term)->i;
  return 1;
}
int enif_get_tuple(ErlNifEnv* env, ERL_NIF_TERM term, int* arity, const ERL_NIF_TERM** array) {
  (void)env;
  if (C(term)->type != T_TUPLE) return 0;
  *arity = (int)C(term)->n;
  *array = C(term)->el;
  return 1;
}
int enif_get_list_length(ErlNifEnv* env, ERL_NIF_TERM term, unsigned* len) {
  (void)env;
  unsigned n = 0;
  for (cell* c = C(term);; c = C(c->el[1])) {
    if (c->type == T_NIL) { *len = n; return 1; }
    if (c->type != T_CONS) return 0;
    n++;
  }
}
int enif_get_list_cell(ErlNifEnv* env, ERL_NIF_TERM list, ERL_NIF_TERM* head, ERL_NIF_TERM* tail) {
  (void)env;
  if (C(list)->type != T_CONS) return 0;
  *head = C(list)->el[0];
  *tail = C(list)->el[1];
  return 1;
}
int enif_get_map_value(ErlNifEnv* env, ERL_NIF_TERM map, ERL_NIF_TERM key, ERL_NIF_TERM* value) {
  (void)env;
  cell* m = C(map);
  if (m->type != T_MAP) return 0;
  for (size_t i = 0; i < m->n; i++)
    if (enif_is_identical(m->el[i], key)) { *value = m->el[m->n + i]; return 1; }
  return 0;
}
int enif_inspect_binary(ErlNifEnv* env, ERL_NIF_TERM t, ErlNifBinary* bin) {
  (void)env;
  if (C(t)->type != T_BIN) return 0;
  bin->size = C(t)->n;
  bin->data = C(t)->bytes;
  bin->ref_bin = NULL;
  return 1;
}

/* iolist flattening (binaries, bytes, nested lists) */
static int iolist_put(cell* c, unsigned char** buf, size_t* n, size_t* cap) {
  if (c->type == T_BIN) {
    if (*n + c->n > *cap) { *cap = (*n + c->n) * 2 + 16; *buf = (unsigned char*)realloc(*buf, *cap); }
    memcpy(*buf + *n, c->bytes, c->n);
    *n += c->n;
    return 1;
  }
  for (;; c = C(c->el[1])) {
    if (c->type == T_NIL) return 1;
    if (c->type != T_CONS) return 0;
    cell* h = C(c->el[0]);
    if (h->type == T_INT) {
      if (h->i < 0 || h->i > 255) return 0;
      if (*n + 1 > *cap) { *cap = *cap * 2 + 16; *buf = (unsigned char*)realloc(*buf, *cap); }
      (*buf)[(*n)++] = (unsigned char)h->i;
    } else if (!iolist_put(h, buf, n, cap)) {
      return 0;
    }
  }
}
int enif_inspect_iolist_as_binary(ErlNifEnv* env, ERL_NIF_TERM term, ErlNifBinary* bin) {
  if (C(term)->type == T_BIN) return enif_inspect_binary(env, term, bin);
  unsigned char* buf = NULL;
  size_t n = 0, cap = 0;
  if (!iolist_put(C(term), &buf, &n, &cap)) { free(buf); return 0; }
  bin->size = n;
  bin->data = buf ? buf : (unsigned char*)calloc(1, 1);   /* owned by the "env": never freed here */
  bin->ref_bin = NULL;
  return 1;
}

int enif_is_identical(ERL_NIF_TERM lhs, ERL_NIF_TERM rhs) {
  cell *a = C(lhs), *b = C(rhs);
  if (a == b) return 1;
  if (a->type != b->type) return 0;
  switch (a->type) {
    case T_ATOM: return 0;   /* interned */
    case T_INT: return a->i == b->i;
    case T_BIN: return a->n == b->n && !memcmp(a->bytes, b->bytes, a->n);
    case T_NIL: return 1;
    case T_RES: return a->res == b->res;
    case T_CONS: return enif_is_identical(a->el[0], b->el[0]) && enif_is_identical(a->el[1], b->el[1]);
    case T_TUPLE: case T_MAP: {
      const size_t k = a->type == T_MAP ? 2 * a->n : a->n;
      if (a->n != b->n) return 0;
      for (size_t i = 0; i < k; i++) if (!enif_is_identical(a->el[i], b->el[i])) return 0;
      return 1;
    }
  }
  return 0;
}

/* a deterministic, injective encoding (not the external term format: only
 * equality of encodings matters to the NIF, which keys its interners on it) */
static void enc(cell* c, unsigned char** buf, size_t* n, size_t* cap) {
  unsigned char hdr[17];
  size_t hl = 0;
  hdr[hl++] = (unsigned char)c->type;
  uint64_t v = c->type == T_INT ? (uint64_t)c->i : c->type == T_RES ? (uint64_t)(uintptr_t)c->res : (uint64_t)c->n;
  memcpy(hdr + hl, &v, 8);
  hl += 8;
  if (*n + hl + c->n + 16 > *cap) { *cap = (*n + hl + c->n) * 2 + 64; *buf = (unsigned char*)realloc(*buf, *cap); }
  memcpy(*buf + *n, hdr, hl);
  *n += hl;
  if (c->type == T_BIN || c->type == T_ATOM) { memcpy(*buf + *n, c->bytes, c->n); *n += c->n; }
  if (c->type == T_TUPLE) for (size_t i = 0; i < c->n; i++) enc(C(c->el[i]), buf, n, cap);
  if (c->type == T_MAP) for (size_t i = 0; i < 2 * c->n; i++) enc(C(c->el[i]), buf, n, cap);
  if (c->type == T_CONS) { enc(C(c->el[0]), buf, n, cap); enc(C(c->el[1]), buf, n, cap); }
}
int enif_term_to_binary(ErlNifEnv* env, ERL_NIF_TERM term, ErlNifBinary* bin) {
  (void)env;
  unsigned char* buf = NULL;
  size_t n = 0, cap = 0;
  enc(C(term), &buf, &n, &cap);
  bin->size = n;
  bin->data = buf;
  bin->ref_bin = buf;
  return 1;
}
void enif_release_binary(ErlNifBinary* bin) {
  free(bin->ref_bin);
  bin->ref_bin = NULL;
}

ErlNifResourceType* enif_open_resource_type(ErlNifEnv* env, const char* module_str, const char* name,
                                            ErlNifResourceDtor* dtor, ErlNifResourceFlags flags,
                                            ErlNifResourceFlags* tried) {
  (void)env; (void)module_str; (void)flags;
  ErlNifResourceType* t = (ErlNifResourceType*)calloc(1, sizeof(*t));
  t->dtor = dtor;
  snprintf(t->name, sizeof t->name, "%s", name);
  if (tried) *tried = ERL_NIF_RT_CREATE;
  return t;
}
void* enif_alloc_resource(ErlNifResourceType* type, size_t size) {
  res_hdr* h = (res_hdr*)calloc(1, sizeof(res_hdr) + size + 16);
  h->type = type;
  h->refs = 1;
  return (void*)(h + 1);
}
void enif_keep_resource(void* obj) {
  pthread_mutex_lock(&mu);
  ((res_hdr*)obj - 1)->refs++;
  pthread_mutex_unlock(&mu);
}
void enif_release_resource(void* obj) {
  res_hdr* h = (res_hdr*)obj - 1;
  pthread_mutex_lock(&mu);
  const long r = --h->refs;
  pthread_mutex_unlock(&mu);
  if (r == 0) {
    if (h->type->dtor) h->type->dtor(NULL, obj);
    free(h);
  }
}
int enif_get_resource(ErlNifEnv* env, ERL_NIF_TERM term, ErlNifResourceType* type, void** objp) {
  (void)env;
  cell* c = C(term);
  if (c->type != T_RES || ((res_hdr*)c->res - 1)->type != type) return 0;
  *objp = c->res;
  return 1;
}

void enif_system_info(ErlNifSysInfo* sip, size_t si_size) {
  memset(sip, 0, si_size);
  sip->nif_major_version = 2;
  sip->nif_minor_version = 11;   /* OTP 19 */
  sip->dirty_scheduler_support = getenv("MOCK_NO_DIRTY") ? 0 : 1;
}
ERL_NIF_TERM enif_schedule_nif(ErlNifEnv* env, const char* fun_name, int flags,
                               ERL_NIF_TERM (*fp)(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]), int argc,
                               const ERL_NIF_TERM argv[]) {
  (void)fun_name;
  if (flags & ~(ERL_NIF_DIRTY_JOB_IO_BOUND | ERL_NIF_DIRTY_JOB_CPU_BOUND)) return enif_make_badarg(env);
  return fp(env, argc, argv);
}

/* ---- for the check program ---------------------------------------------- */
ERL_NIF_TERM mock_make_binary(const void* data, size_t n) {
  cell* c = new_cell(T_BIN);
  c->n = n;
  c->bytes = (unsigned char*)malloc(n ? n : 1);
  if (n) memcpy(c->bytes, data, n);
  return T(c);
}
ERL_NIF_TERM mock_make_int(int64_t v) { return make_int(v); }
ERL_NIF_TERM mock_make_map(size_t n, const ERL_NIF_TERM* keys, const ERL_NIF_TERM* vals) {
  cell* c = new_cell(T_MAP);
  c->n = n;
  c->el = (ERL_NIF_TERM*)malloc((2 * n + 1) * sizeof(ERL_NIF_TERM));
  memcpy(c->el, keys, n * sizeof(ERL_NIF_TERM));
  memcpy(c->el + n, vals, n * sizeof(ERL_NIF_TERM));
  return T(c);
}
ERL_NIF_TERM mock_make_tuple(size_t n, const ERL_NIF_TERM* el) { return make_tuple(n, el); }
int mock_is_list(ERL_NIF_TERM t) { return C(t)->type == T_CONS || C(t)->type == T_NIL; }

/* Erlang-ish text: atoms bare, binaries <<"..">>, strings as lists of ints */
void mock_print(FILE* f, ERL_NIF_TERM t) {
  cell* c = C(t);
  switch (c->type) {
    case T_ATOM: fputs((const char*)c->bytes, f); break;
    case T_INT: fprintf(f, "%lld", (long long)c->i); break;
    case T_BIN:
      fputs("<<\"", f);
      for (size_t i = 0; i < c->n; i++) {
        const unsigned char ch = c->bytes[i];
        if (ch >= 0x20 && ch < 0x7f && ch != '"' && ch != '\\') fputc(ch, f);
        else fprintf(f, "\\x%02x", ch);
      }
      fputs("\">>", f);
      break;
    case T_NIL: fputs("[]", f); break;
    case T_RES: fputs("#Ref", f); break;
    case T_TUPLE:
      fputc('{', f);
      for (size_t i = 0; i < c->n; i++) { if (i) fputc(',', f); mock_print(f, c->el[i]); }
      fputc('}', f);
      break;
    case T_MAP:
      fputs("#{", f);
      for (size_t i = 0; i < c->n; i++) {
        if (i) fputc(',', f);
        mock_print(f, c->el[i]);
        fputs("=>", f);
        mock_print(f, c->el[c->n + i]);
      }
      fputc('}', f);
      break;
    case T_CONS:
      fputc('[', f);
      for (int first = 1; c->type == T_CONS; c = C(c->el[1]), first = 0) {
        if (!first) fputc(',', f);
        mock_print(f, c->el[0]);
      }
      fputc(']', f);
      break;
  }
}

const char* mock_atom_name(ERL_NIF_TERM t) { return C(t)->type == T_ATOM ? (const char*)C(t)->bytes : NULL; }

/* mutexes: pthread mutexes, as the emulator's on Linux */
struct enif_mutex_t { pthread_mutex_t m; };
ErlNifMutex* enif_mutex_create(char* name) {
  (void)name;
  ErlNifMutex* x = (ErlNifMutex*)calloc(1, sizeof(ErlNifMutex));
  if (x && pthread_mutex_init(&x->m, NULL) != 0) { free(x); return NULL; }
  return x;
}
void enif_mutex_destroy(ErlNifMutex* mtx) { if (mtx) { pthread_mutex_destroy(&mtx->m); free(mtx); } }
void enif_mutex_lock(ErlNifMutex* mtx) { pthread_mutex_lock(&mtx->m); }
void enif_mutex_unlock(ErlNifMutex* mtx) { pthread_mutex_unlock(&mtx->m); }
