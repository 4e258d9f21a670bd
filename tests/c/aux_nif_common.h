/* Shared plumbing of the retained / ACL NIF checks (tests/c/retain_nif_check.c,
 * tests/c/acl_nif_check.c): the NIF's ErlNifFunc table called for real over
 * the erl_nif test double (tests/c/mock_erl_nif). */
#ifndef AUX_NIF_COMMON_H
#define AUX_NIF_COMMON_H
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "erl_nif.h"

ErlNifEntry* nif_init(void);
ERL_NIF_TERM mock_make_binary(const void* data, size_t n);
ERL_NIF_TERM mock_make_int(int64_t v);
ERL_NIF_TERM mock_make_map(size_t n, const ERL_NIF_TERM* keys, const ERL_NIF_TERM* vals);
ERL_NIF_TERM mock_make_tuple(size_t n, const ERL_NIF_TERM* el);
const char* mock_atom_name(ERL_NIF_TERM t);
void mock_print(FILE* f, ERL_NIF_TERM t);

static ErlNifEntry* E;
static ErlNifEnv* env;

static ERL_NIF_TERM call(const char* name, int argc, const ERL_NIF_TERM* argv) {
  for (int i = 0; i < E->num_of_funcs; i++)
    if (!strcmp(E->funcs[i].name, name) && (int)E->funcs[i].arity == argc) return E->funcs[i].fptr(env, argc, argv);
  fprintf(stderr, "no NIF %s/%d\n", name, argc);
  exit(3);
}

/* "a/b/+" -> [<<"a">>, <<"b">>, <<"+">>] (empty levels kept); "!" -> [] */
static ERL_NIF_TERM words_term(const char* f) {
  if (!strcmp(f, "!")) return enif_make_list_from_array(env, NULL, 0);
  ERL_NIF_TERM w[256];
  unsigned n = 0;
  const char* s = f;
  for (;;) {
    const char* e = strchr(s, '/');
    const size_t l = e ? (size_t)(e - s) : strlen(s);
    w[n++] = mock_make_binary(s, l);
    if (!e || n == 256) break;
    s = e + 1;
  }
  return enif_make_list_from_array(env, w, n);
}

/* "-" is the empty mountpoint */
static ERL_NIF_TERM mp_term(const char* mp) { return enif_make_string(env, mp[0] == '-' ? "" : mp, ERL_NIF_LATIN1); }

static ERL_NIF_TERM create_ctx(int device) {
  ERL_NIF_TERM k[1] = {enif_make_atom(env, "device")};
  ERL_NIF_TERM v[1] = {mock_make_int(device)};
  const ERL_NIF_TERM arg = mock_make_map(1, k, v);
  const ERL_NIF_TERM r = call("create", 1, &arg);
  int ar;
  const ERL_NIF_TERM* el;
  if (!enif_get_tuple(env, r, &ar, &el) || ar != 2 || strcmp(mock_atom_name(el[0]) ? mock_atom_name(el[0]) : "", "ok")) {
    fprintf(stderr, "create: ");
    mock_print(stderr, r);
    fputc('\n', stderr);
    exit(4);
  }
  return el[1];
}

static void start(const char* name) {
  E = nif_init();
  env = enif_alloc_env();
  if (strcmp(E->name, name) || E->load(env, NULL, 0) != 0) { fprintf(stderr, "load failed\n"); exit(3); }
}
#endif
