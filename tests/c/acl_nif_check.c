/* Runs the ACL NIF glue (integration/c_src/vmqa_nif.c) through its
 * ErlNifFunc table over the erl_nif test double; tests/test_nif_layer.py
 * compares the verdicts with oracle/vmq_acl_oracle.cpp.
 *
 * usage: acl_nif_check <script> <out>; script lines:
 *   N <device>                                   create(#{device => D})
 *   R <read|write> <all|user|pattern> <user|-> <words>   a table row
 *   L                                            load(Ctx, the rows) -> "L <result>"
 *   C <read|write> <topic|!> <user|~> <mp|-> <client>    a check ("~" user: undefined)
 *   K                                            check(Ctx, every check so far) -> "K <n>", then "<i> <verdict>" */
#define _GNU_SOURCE
#include "aux_nif_common.h"

int main(int argc, char** argv) {
  if (argc != 3) { fprintf(stderr, "usage: %s <script> <out>\n", argv[0]); return 2; }
  FILE* in = fopen(argv[1], "r");
  FILE* out = fopen(argv[2], "w");
  if (!in || !out) { perror("open"); return 2; }
  start("vmqa_nif");
  ERL_NIF_TERM ctx = 0, *rows = NULL, *checks = NULL;
  size_t nr = 0, nc = 0;
  char* line = NULL;
  size_t lcap = 0;
  ssize_t ln;
  while ((ln = getline(&line, &lcap, in)) > 0) {
    if (line[ln - 1] == '\n') line[--ln] = 0;
    char ty[16], table[16], user[256], words[4096], mp[64], client[256];
    if (line[0] == 'N') {
      ctx = create_ctx(atoi(line + 2));
    } else if (line[0] == 'R') {
      if (sscanf(line + 2, "%15s %15s %255s %4095s", ty, table, user, words) != 4) return 5;
      const ERL_NIF_TERM el[4] = {enif_make_atom(env, ty), enif_make_atom(env, table),
                                  !strcmp(user, "-") ? enif_make_atom(env, "all") : mock_make_binary(user, strlen(user)),
                                  words_term(words)};
      rows = (ERL_NIF_TERM*)realloc(rows, (nr + 1) * sizeof(ERL_NIF_TERM));
      rows[nr++] = mock_make_tuple(4, el);
    } else if (line[0] == 'L') {
      const ERL_NIF_TERM args[2] = {ctx, enif_make_list_from_array(env, rows, (unsigned)nr)};
      fprintf(out, "L ");
      mock_print(out, call("load", 2, args));
      fputc('\n', out);
      nr = 0;
    } else if (line[0] == 'C') {
      if (sscanf(line + 2, "%15s %4095s %255s %63s %255s", ty, words, user, mp, client) != 5) return 6;
      const ERL_NIF_TERM el[5] = {enif_make_atom(env, ty), words_term(words),
                                  !strcmp(user, "~") ? enif_make_atom(env, "undefined") : mock_make_binary(user, strlen(user)),
                                  mp_term(mp), mock_make_binary(client, strlen(client))};
      checks = (ERL_NIF_TERM*)realloc(checks, (nc + 1) * sizeof(ERL_NIF_TERM));
      checks[nc++] = mock_make_tuple(5, el);
    } else if (line[0] == 'K') {
      const ERL_NIF_TERM args[2] = {ctx, enif_make_list_from_array(env, checks, (unsigned)nc)};
      const ERL_NIF_TERM r = call("check", 2, args);
      unsigned n = 0;
      if (!enif_get_list_length(env, r, &n)) { fprintf(out, "K error "); mock_print(out, r); fputc('\n', out); continue; }
      fprintf(out, "K %u\n", n);
      ERL_NIF_TERM h, t = r;
      for (unsigned i = 0; i < n; i++) {
        enif_get_list_cell(env, t, &h, &t);
        fprintf(out, "%u ", i);
        mock_print(out, h);
        fputc('\n', out);
      }
    }
  }
  fclose(out);
  return 0;
}
