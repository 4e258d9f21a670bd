/* Runs the vmq_reg_gpu_view NIF glue (integration/c_src/vmqg_nif.c) for
 * real, through its ErlNifFunc table, over the erl_nif test double
 * (tests/c/mock_erl_nif): create/1, add_init/6 + flush_init/1 (the initial
 * load), apply/3 and apply_many/2 (the view's coalesced subscriber events),
 * batch_new/1, match/4 in both modes, stats/1 — the term <-> id glue that
 * cannot be built against OTP here.  tests/test_nif_layer.py compares the
 * printed FoldFun entries with the oracle.
 *
 * usage: nif_mock_check <script> <out>; script lines:
 *   N <device> [<lanes>]                create(#{device => D, local_node => 'n0@h'[, devices => [D x lanes]]})
 *   I <node> <mp> <client> <qos> <filter>   add_init(Ctx, MP, Topic, {MP, Client}, QoS, Node)
 *   F                                   flush_init(Ctx)
 *   V <mp> <client>                     opens an event of SubscriberId {MP, Client}
 *   C <add|del> <node> <qos> <filter>   a change of the open event ("!" filter: [] , an invalid topic)
 *   A                                   apply_many(Ctx, the events since the last A / S)
 *   S                                   apply(Ctx, SubscriberId, Changes) per event since the last A / S
 *   P <mp> <topic>                      a publish: its Topic word list (split on '/'; "%2F" a '/'
 *                                       inside a word, "~x" the atom x, "!" the empty list)
 *   M <records|ranges>                  match(Ctx, Batch, every publish so far, Mode)
 *   T                                   stats(Ctx)
 *   Y <rounds> <per_round> <every>      churn cycles: per round, <per_round> new subscribers
 *                                       (unique client ids and topic words: dev/<u>/state,
 *                                       all/<u>/#, $share/g<r%5>/jobs/<u>) in one
 *                                       apply_many, then all of them deleted in another;
 *                                       every <every> rounds "Y <round> peak <counts>" and
 *                                       "Y <round> empty <counts>" (counts/1 + the mock's
 *                                       environment cells)
 *   X <name> <value>                    set_option(Ctx, name, value)
 *   R                                   commit(Ctx)
 * output: "A <result>", "S <result>...", "T <subs>", "M <n>" then per
 * publish "<i> ok <entries>" (A,<mp>,<client>,<qos> | B,<node>,<group>,<mp>,
 * <client>,<qos> | C,<node>, space separated) or "<i> error <reason>". */
#define _GNU_SOURCE
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
long mock_env_cells(void);
void mock_print(FILE* f, ERL_NIF_TERM t);

static ErlNifEntry* E;
static ErlNifEnv* env;

static ERL_NIF_TERM call(const char* name, int argc, const ERL_NIF_TERM* argv) {
  for (int i = 0; i < E->num_of_funcs; i++)
    if (!strcmp(E->funcs[i].name, name) && (int)E->funcs[i].arity == argc) return E->funcs[i].fptr(env, argc, argv);
  fprintf(stderr, "no NIF %s/%d\n", name, argc);
  exit(3);
}

static ERL_NIF_TERM mp_term(const char* mp) { return enif_make_string(env, mp[0] == '-' ? "" : mp, ERL_NIF_LATIN1); }
/* "a/b/+" -> [<<"a">>, <<"b">>, <<"+">>] (empty levels kept) */
static ERL_NIF_TERM topic_term(const char* f) {
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
/* a publish's Topic list: words split on '/', "%2F" a '/' inside a word,
 * a word "~name" the atom name (a list element that is not a binary), "!"
 * the empty list */
static ERL_NIF_TERM pub_topic_term(const char* f) {
  if (!strcmp(f, "!")) return enif_make_list_from_array(env, NULL, 0);
  ERL_NIF_TERM w[256];
  unsigned n = 0;
  const char* s = f;
  for (;;) {
    const char* e = strchr(s, '/');
    const size_t l = e ? (size_t)(e - s) : strlen(s);
    char buf[4096];
    size_t k = 0;
    for (size_t i = 0; i < l && k < sizeof buf; i++) {
      if (s[i] == '%' && i + 2 < l + 0 && s[i + 1] == '2' && (s[i + 2] == 'F' || s[i + 2] == 'f')) { buf[k++] = '/'; i += 2; }
      else buf[k++] = s[i];
    }
    if (k && buf[0] == '~') { buf[k] = 0; w[n++] = enif_make_atom(env, buf + 1); }
    else w[n++] = mock_make_binary(buf, k);
    if (!e || n == 256) break;
    s = e + 1;
  }
  return enif_make_list_from_array(env, w, n);
}
static ERL_NIF_TERM sid_term(const char* mp, const char* client) {
  const ERL_NIF_TERM el[2] = {mp_term(mp), mock_make_binary(client, strlen(client))};
  return mock_make_tuple(2, el);
}
static ERL_NIF_TERM node_term(unsigned node) {
  char b[32];
  snprintf(b, sizeof b, "n%u@h", node);
  return enif_make_atom(env, b);
}

static void print_chars(FILE* f, ERL_NIF_TERM t) {   /* a charlist / binary as text ("-" when empty) */
  ErlNifBinary b;
  if (!enif_inspect_iolist_as_binary(env, t, &b) || b.size == 0) { fputc('-', f); return; }
  fwrite(b.data, 1, b.size, f);
}
static void print_sid(FILE* f, ERL_NIF_TERM sid) {
  int ar;
  const ERL_NIF_TERM* el;
  enif_get_tuple(env, sid, &ar, &el);
  print_chars(f, el[0]);
  fputc(',', f);
  print_chars(f, el[1]);
}
static void print_entry(FILE* f, ERL_NIF_TERM e) {
  int ar, q = 0;
  const ERL_NIF_TERM* el;
  if (mock_atom_name(e)) { fprintf(f, " C,%s", mock_atom_name(e)); return; }
  enif_get_tuple(env, e, &ar, &el);
  if (ar == 2) {
    fputs(" A,", f);
    print_sid(f, el[0]);
    enif_get_int(env, el[1], &q);
    fprintf(f, ",%d", q);
  } else {
    fprintf(f, " B,%s,", mock_atom_name(el[0]));
    print_chars(f, el[1]);
    fputc(',', f);
    print_sid(f, el[2]);
    enif_get_int(env, el[3], &q);
    fprintf(f, ",%d", q);
  }
}

int main(int argc, char** argv) {
  if (argc != 3) { fprintf(stderr, "usage: %s <script> <out>\n", argv[0]); return 2; }
  FILE* in = fopen(argv[1], "r");
  FILE* out = fopen(argv[2], "w");
  if (!in || !out) { perror("open"); return 2; }
  E = nif_init();
  env = enif_alloc_env();
  if (strcmp(E->name, "vmqg_nif") || E->load(env, NULL, 0) != 0) { fprintf(stderr, "load failed\n"); return 3; }
  ERL_NIF_TERM ctx = 0, batch = 0;
  ERL_NIF_TERM* events = NULL;       /* {SubscriberId, Changes} */
  ERL_NIF_TERM* changes = NULL;
  size_t nev = 0, nch = 0;
  ERL_NIF_TERM cur_sid = 0;
  ERL_NIF_TERM* pubs = NULL;
  size_t npubs = 0;
  char* line = NULL;
  size_t lcap = 0;
  ssize_t ln;
  const ERL_NIF_TERM ok = enif_make_atom(env, "ok");
#define CLOSE_EVENT()                                                                               \
  do {                                                                                              \
    if (cur_sid) {                                                                                  \
      const ERL_NIF_TERM ev[2] = {cur_sid, enif_make_list_from_array(env, changes, (unsigned)nch)}; \
      events = (ERL_NIF_TERM*)realloc(events, (nev + 1) * sizeof(ERL_NIF_TERM));                    \
      events[nev++] = mock_make_tuple(2, ev);                                                       \
      nch = 0;                                                                                      \
      cur_sid = 0;                                                                                  \
    }                                                                                               \
  } while (0)
  while ((ln = getline(&line, &lcap, in)) > 0) {
    if (line[ln - 1] == '\n') line[--ln] = 0;
    char a1[64], a2[256], a3[64], topic[4096];
    int d, node, qos;
    if (line[0] == 'N') {
      int lanes = 1;
      sscanf(line + 2, "%d %d", &d, &lanes);
      ERL_NIF_TERM dev[16];
      for (int i = 0; i < lanes && i < 16; i++) dev[i] = mock_make_int(d);
      ERL_NIF_TERM k[3] = {enif_make_atom(env, "device"), enif_make_atom(env, "local_node"), enif_make_atom(env, "devices")};
      ERL_NIF_TERM v[3] = {mock_make_int(d), node_term(0), enif_make_list_from_array(env, dev, (unsigned)(lanes < 16 ? lanes : 16))};
      const ERL_NIF_TERM arg = mock_make_map(lanes > 1 ? 3 : 2, k, v);
      const ERL_NIF_TERM r = call("create", 1, &arg);
      int ar;
      const ERL_NIF_TERM* el;
      if (!enif_get_tuple(env, r, &ar, &el) || ar != 2 || !enif_is_identical(el[0], ok)) {
        fprintf(stderr, "create: ");
        mock_print(stderr, r);
        fputc('\n', stderr);
        return 4;
      }
      ctx = el[1];
      ERL_NIF_TERM rb = call("batch_new", 1, &ctx);
      if (lanes > 1) rb = call("batch_new", 1, &ctx);   /* batches are bound round robin: this one to lane 1 */
      enif_get_tuple(env, rb, &ar, &el);
      batch = el[1];
    } else if (line[0] == 'I') {
      if (sscanf(line + 2, "%d %63s %255s %d %4095s", &node, a1, a2, &qos, topic) != 5) return 5;
      const ERL_NIF_TERM args[6] = {ctx, mp_term(a1), topic_term(topic), sid_term(a1, a2), mock_make_int(qos), node_term((unsigned)node)};
      const ERL_NIF_TERM r = call("add_init", 6, args);
      if (!enif_is_identical(r, ok)) { fprintf(out, "I "); mock_print(out, r); fputc('\n', out); }
    } else if (line[0] == 'F') {
      const ERL_NIF_TERM r = call("flush_init", 1, &ctx);
      fprintf(out, "F ");
      mock_print(out, r);
      fputc('\n', out);
    } else if (line[0] == 'V') {
      CLOSE_EVENT();
      if (sscanf(line + 2, "%63s %255s", a1, a2) != 2) return 6;
      cur_sid = sid_term(a1, a2);
    } else if (line[0] == 'C') {
      if (sscanf(line + 2, "%63s %d %d %4095s", a3, &node, &qos, topic) != 4) return 7;
      const ERL_NIF_TERM el[4] = {enif_make_atom(env, a3), topic_term(topic), mock_make_int(qos), node_term((unsigned)node)};
      changes = (ERL_NIF_TERM*)realloc(changes, (nch + 1) * sizeof(ERL_NIF_TERM));
      changes[nch++] = mock_make_tuple(4, el);
    } else if (line[0] == 'A' || line[0] == 'S') {
      CLOSE_EVENT();
      if (line[0] == 'A') {
        const ERL_NIF_TERM args[2] = {ctx, enif_make_list_from_array(env, events, (unsigned)nev)};
        const ERL_NIF_TERM r = call("apply_many", 2, args);
        fprintf(out, "A ");
        mock_print(out, r);
        fputc('\n', out);
      } else {
        fprintf(out, "S");
        for (size_t i = 0; i < nev; i++) {
          int ar;
          const ERL_NIF_TERM* el;
          enif_get_tuple(env, events[i], &ar, &el);
          const ERL_NIF_TERM args[3] = {ctx, el[0], el[1]};
          fputc(' ', out);
          mock_print(out, call("apply", 3, args));
        }
        fputc('\n', out);
      }
      nev = 0;
    } else if (line[0] == 'P') {
      if (sscanf(line + 2, "%63s %4095s", a1, topic) != 2) return 8;
      const ERL_NIF_TERM el[2] = {mp_term(a1), pub_topic_term(topic)};
      pubs = (ERL_NIF_TERM*)realloc(pubs, (npubs + 1) * sizeof(ERL_NIF_TERM));
      pubs[npubs++] = mock_make_tuple(2, el);
    } else if (line[0] == 'M') {
      if (sscanf(line + 2, "%63s", a1) != 1) return 9;
      const ERL_NIF_TERM args[4] = {ctx, batch, enif_make_list_from_array(env, pubs, (unsigned)npubs), enif_make_atom(env, a1)};
      const ERL_NIF_TERM r = call("match", 4, args);
      unsigned n = 0;
      if (!enif_get_list_length(env, r, &n) || n != npubs) { fprintf(stderr, "match: bad result\n"); return 10; }
      fprintf(out, "M %u\n", n);
      ERL_NIF_TERM h, t = r;
      for (unsigned i = 0; i < n; i++) {
        enif_get_list_cell(env, t, &h, &t);
        int ar;
        const ERL_NIF_TERM* el;
        enif_get_tuple(env, h, &ar, &el);
        if (enif_is_identical(el[0], ok)) {
          fprintf(out, "%u ok", i);
          ERL_NIF_TERM eh, et = el[1];
          while (enif_get_list_cell(env, et, &eh, &et)) print_entry(out, eh);
        } else {
          fprintf(out, "%u error %s", i, mock_atom_name(el[1]) ? mock_atom_name(el[1]) : "?");
        }
        fputc('\n', out);
      }
    } else if (line[0] == 'Y') {
      int rounds = 0, per = 0, every = 1;
      if (sscanf(line + 2, "%d %d %d", &rounds, &per, &every) != 3 || per < 1 || every < 1) return 12;
      ERL_NIF_TERM* ev = (ERL_NIF_TERM*)malloc((size_t)per * sizeof(ERL_NIF_TERM));
      ERL_NIF_TERM* del = (ERL_NIF_TERM*)malloc((size_t)per * sizeof(ERL_NIF_TERM));
      const ERL_NIF_TERM a_add = enif_make_atom(env, "add"), a_del = enif_make_atom(env, "del");
      for (int rd = 0; rd < rounds; rd++) {
        for (int i = 0; i < per; i++) {
          char u[48], cid[48], grp[16];
          snprintf(u, sizeof u, "u%d_%d", rd, i);
          snprintf(cid, sizeof cid, "client_%d_%d", rd, i);
          snprintf(grp, sizeof grp, "g%d", rd % 5);
          const ERL_NIF_TERM sid = sid_term("-", cid);
          const ERL_NIF_TERM t1[3] = {mock_make_binary("dev", 3), mock_make_binary(u, strlen(u)), mock_make_binary("state", 5)};
          const ERL_NIF_TERM t2[3] = {mock_make_binary("all", 3), mock_make_binary(u, strlen(u)), mock_make_binary("#", 1)};
          const ERL_NIF_TERM t3[4] = {mock_make_binary("$share", 6), mock_make_binary(grp, strlen(grp)),
                                      mock_make_binary("jobs", 4), mock_make_binary(u, strlen(u))};
          const ERL_NIF_TERM tops[3] = {enif_make_list_from_array(env, t1, 3), enif_make_list_from_array(env, t2, 3),
                                        enif_make_list_from_array(env, t3, 4)};
          ERL_NIF_TERM ca[3], cd[3];
          for (int k = 0; k < 3; k++) {
            const ERL_NIF_TERM el[4] = {a_add, tops[k], mock_make_int(k % 3), node_term(i % 9 == 0 ? 2u : 0u)};
            const ERL_NIF_TERM eld[4] = {a_del, tops[k], mock_make_int(k % 3), node_term(i % 9 == 0 ? 2u : 0u)};
            ca[k] = mock_make_tuple(4, el);
            cd[k] = mock_make_tuple(4, eld);
          }
          const ERL_NIF_TERM e1[2] = {sid, enif_make_list_from_array(env, ca, 3)};
          const ERL_NIF_TERM e2[2] = {sid, enif_make_list_from_array(env, cd, 3)};
          ev[i] = mock_make_tuple(2, e1);
          del[i] = mock_make_tuple(2, e2);
        }
        for (int ph = 0; ph < 2; ph++) {
          const ERL_NIF_TERM args[2] = {ctx, enif_make_list_from_array(env, ph ? del : ev, (unsigned)per)};
          const ERL_NIF_TERM r = call("apply_many", 2, args);
          if (!enif_is_identical(r, ok)) { fprintf(out, "Y %d apply ", rd); mock_print(out, r); fputc('\n', out); }
          if ((rd + 1) % every == 0 || rd == 0) {
            fprintf(out, "Y %d %s", rd, ph ? "empty" : "peak");
            const ERL_NIF_TERM cl = call("counts", 1, &ctx);
            ERL_NIF_TERM h, t = cl;
            while (enif_get_list_cell(env, t, &h, &t)) {
              int ar;
              const ERL_NIF_TERM* el;
              ErlNifSInt64 x = 0;
              enif_get_tuple(env, h, &ar, &el);
              enif_get_int64(env, el[1], &x);
              fprintf(out, " %s=%lld", mock_atom_name(el[0]), (long long)x);
            }
            fprintf(out, " env_cells=%ld\n", mock_env_cells());
          }
        }
      }
      free(ev);
      free(del);
    } else if (line[0] == 'X') {
      long long v;
      if (sscanf(line + 2, "%63s %lld", a1, &v) != 2) return 11;
      const ERL_NIF_TERM args[3] = {ctx, enif_make_atom(env, a1), mock_make_int(v)};
      fprintf(out, "X ");
      mock_print(out, call("set_option", 3, args));
      fputc('\n', out);
    } else if (line[0] == 'R') {
      fprintf(out, "R ");
      mock_print(out, call("commit", 1, &ctx));
      fputc('\n', out);
    } else if (line[0] == 'T') {
      const ERL_NIF_TERM r = call("stats", 1, &ctx);
      int ar, subs = -1;
      const ERL_NIF_TERM* el;
      if (enif_get_tuple(env, r, &ar, &el) && ar == 2) enif_get_int(env, el[0], &subs);
      fprintf(out, "T %d\n", subs);
    }
  }
  fclose(out);
  return 0;
}
