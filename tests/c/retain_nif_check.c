/* Runs the retained-store NIF glue (integration/c_src/vmqr_nif.c) through its
 * ErlNifFunc table over the erl_nif test double; tests/test_nif_layer.py
 * compares the printed message ids with oracle/vmq_retain_oracle.cpp.
 *
 * usage: retain_nif_check <script> <out>; script lines:
 *   N <device>              create(#{device => D})
 *   I <mp> <topic> <id>     an {insert, MP, Topic, Id} op
 *   D <mp> <topic>          a {delete, MP, Topic} op
 *   A                       apply(Ctx, the ops since the last A) -> "A <result>"
 *   Q <mp> <filter>         a filter ("!" the empty list)
 *   M                       match(Ctx, every filter so far) -> "M <n>", then "<i> <ids...>"
 *   T                       stats(Ctx) -> "T <retained>" */
#define _GNU_SOURCE
#include "aux_nif_common.h"

int main(int argc, char** argv) {
  if (argc != 3) { fprintf(stderr, "usage: %s <script> <out>\n", argv[0]); return 2; }
  FILE* in = fopen(argv[1], "r");
  FILE* out = fopen(argv[2], "w");
  if (!in || !out) { perror("open"); return 2; }
  start("vmqr_nif");
  ERL_NIF_TERM ctx = 0, *ops = NULL, *filters = NULL;
  size_t nops = 0, nf = 0;
  char* line = NULL;
  size_t lcap = 0;
  ssize_t ln;
  while ((ln = getline(&line, &lcap, in)) > 0) {
    if (line[ln - 1] == '\n') line[--ln] = 0;
    char mp[64], topic[4096];
    unsigned id;
    if (line[0] == 'N') {
      ctx = create_ctx(atoi(line + 2));
    } else if (line[0] == 'I' || line[0] == 'D') {
      const int ins = line[0] == 'I';
      if (ins ? sscanf(line + 2, "%63s %4095s %u", mp, topic, &id) != 3 : sscanf(line + 2, "%63s %4095s", mp, topic) != 2)
        return 5;
      const ERL_NIF_TERM el[4] = {enif_make_atom(env, ins ? "insert" : "delete"), mp_term(mp), words_term(topic),
                                  mock_make_int(ins ? id : 0)};
      ops = (ERL_NIF_TERM*)realloc(ops, (nops + 1) * sizeof(ERL_NIF_TERM));
      ops[nops++] = mock_make_tuple(ins ? 4 : 3, el);
    } else if (line[0] == 'A') {
      const ERL_NIF_TERM args[2] = {ctx, enif_make_list_from_array(env, ops, (unsigned)nops)};
      fprintf(out, "A ");
      mock_print(out, call("apply", 2, args));
      fputc('\n', out);
      nops = 0;
    } else if (line[0] == 'Q') {
      if (sscanf(line + 2, "%63s %4095s", mp, topic) != 2) return 6;
      const ERL_NIF_TERM el[2] = {mp_term(mp), words_term(topic)};
      filters = (ERL_NIF_TERM*)realloc(filters, (nf + 1) * sizeof(ERL_NIF_TERM));
      filters[nf++] = mock_make_tuple(2, el);
    } else if (line[0] == 'M') {
      const ERL_NIF_TERM args[2] = {ctx, enif_make_list_from_array(env, filters, (unsigned)nf)};
      const ERL_NIF_TERM r = call("match", 2, args);
      unsigned n = 0;
      if (!enif_get_list_length(env, r, &n)) { fprintf(out, "M error "); mock_print(out, r); fputc('\n', out); continue; }
      fprintf(out, "M %u\n", n);
      ERL_NIF_TERM h, t = r;
      for (unsigned i = 0; i < n; i++) {
        enif_get_list_cell(env, t, &h, &t);
        fprintf(out, "%u", i);
        ERL_NIF_TERM ih, it = h;
        while (enif_get_list_cell(env, it, &ih, &it)) {
          int v = -1;
          enif_get_int(env, ih, &v);
          fprintf(out, " %d", v);
        }
        fputc('\n', out);
      }
    } else if (line[0] == 'T') {
      const ERL_NIF_TERM r = call("stats", 1, &ctx);
      int ar, v = -1;
      const ERL_NIF_TERM* el;
      if (enif_get_tuple(env, r, &ar, &el) && ar == 2) enif_get_int(env, el[0], &v);
      fprintf(out, "T %d\n", v);
    }
  }
  fclose(out);
  return 0;
}
