/* GPU check of the NIF's C core (integration/c_src/vmqg_batch.c) driven the
 * way vmqg_nif.c drives it: batcher threads, each with its own batch (no
 * lock: prepare, device call through the combining submitter, fold),
 * subscription changes as writers beside them — against the oracle
 * (tests/test_nif_layer.py compares the output).
 *
 * usage: batch_gpu_check <script> <out>
 * script lines (fields separated by one space; the topic/filter is the rest
 * of the line):
 *   S <node> <sub> <info> <mp> <filter>   subscribe   (vmqgb_ops_add_filter)
 *   U <node> <sub> <info> <mp> <filter>   unsubscribe
 *   A                                     apply the pending changes (vmqgb_view_apply)
 *   P <mp> <topic>                        a publish (raw topic bytes)
 *   M <records|ranges> <threads> <batch>  match every publish so far with
 *                                         <threads> batchers of <batch>
 *                                         publishes, concurrently with
 *                                         nothing else; writes to <out>:
 *                                         "M <n>" then per publish
 *                                         "<i> <rc> <kind>,<node>,<group>,<sub>,<info> ..." in output order
 *   C <records|ranges> <threads> <batch> <rounds>
 *                                         the same while a writer thread
 *                                         re-applies S/U pairs of filter
 *                                         "zz/<k>" (no publish matches them)
 *                                         <rounds> times: the matches
 *                                         must not change
 *   X S|U <node> <sub> <info> <mp> <filter>
 *                                         a change of the current churn group
 *   G                                     ends a churn group
 *   W <records|ranges> <threads> <batch> <passes>
 *                                         batchers match every publish
 *                                         over and over (at least <passes>
 *                                         times) while a
 *                                         writer applies the churn groups one
 *                                         apply each, ~1 ms apart: changes
 *                                         that DO alter the answers, some
 *                                         bringing words that publishes
 *                                         already hold.  Writes "W <e0>
 *                                         <groups> <lines>", then per group
 *                                         "g <k> <epoch after>", then per
 *                                         matched publish "<i> <epoch> <rc>
 *                                         entries..." (the epoch its batch's
 *                                         answer is from; the test compares
 *                                         it with the oracle at that epoch),
 *                                         then "v <rounds> <stale rematches>
 *                                         <batches>"; the groups are then
 *                                         forgotten (the next X opens anew)
 *   R <n>                                 adds n replica contexts on device 0
 *                                         as lanes of the view (vmqgb_view_add_replica;
 *                                         batchers are bound round robin); after
 *                                         every apply the lanes' arena digests
 *                                         are compared (the last line of <out>:
 *                                         "H <applies checked> <mismatches>"),
 *                                         and each "v" line ends with the rounds
 *                                         per lane
 * group is the $share group's text ("-" for none).
 * Exit 0 after writing everything; non-zero with a message otherwise. */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vmqg_batch.h"

typedef struct { uint32_t mp; char* topic; size_t len; } pub_t;

static vmqg_ctx* ctx;
static vmqgb_view* view;
static pub_t* pubs;
static size_t npubs, pcap;
static char** gname;     /* group text by word id */
static size_t gcap;
static vmqg_ctx* replicas[VMQGB_MAX_LANES];
static int nreplicas, forced;
static uint64_t digests_checked, digests_mismatched;

/* with replicas: every lane's arena digest equals the primary's (writer mutex held) */
static void check_digests(void) {
  if (!nreplicas) return;
  uint64_t d[VMQGB_MAX_LANES];
  const int n = vmqgb_view_lanes(view);
  digests_checked++;
  if (vmqgb_view_digests(view, d, n)) { digests_mismatched++; return; }
  for (int k = 1; k < n; k++) if (d[k] != d[0]) { digests_mismatched++; return; }
}

typedef struct { char* buf; size_t n, cap; } sbuf;

typedef struct {
  int tid, T, ranges;
  size_t B;
  char** lines;          /* per publish: its output line (M / C) */
  int passes;            /* W: passes at least, and until the writer is done */
  sbuf* wout;            /* W: this batcher's output lines */
  int err;
} bt_t;

static void sput(sbuf* s, const char* t) {
  const size_t l = strlen(t);
  if (s->n + l + 1 > s->cap) {
    s->cap = (s->n + l + 1) * 2;
    s->buf = (char*)realloc(s->buf, s->cap);
  }
  memcpy(s->buf + s->n, t, l + 1);
  s->n += l;
}

static int put_entry(void* acc, const vmqgb_entry* e) {
  sbuf* s = (sbuf*)acc;
  char t[160];
  const char* g = e->group < gcap && gname[e->group] ? gname[e->group] : "-";
  snprintf(t, sizeof t, " %u,%u,%s,%u,%u", e->kind, e->kind == VMQG_EMIT_REMOTE || e->kind == VMQG_EMIT_GROUP ? e->node : 0u,
           e->kind == VMQG_EMIT_GROUP ? g : "-", e->kind == VMQG_EMIT_REMOTE ? 0u : e->subscriber,
           e->kind == VMQG_EMIT_REMOTE ? 0u : e->subinfo);
  sput(s, t);
  return 0;
}

static volatile int writer_done;

/* one batch of publishes [lo, lo + n) exactly as vmqg_nif.c's match/4: the
 * batched prepare, the combined device call, the fold, the release (no lock
 * anywhere); one output line per publish */
static int one_batch(bt_t* a, vmqgb_batch* b, long* idx, size_t lo, size_t n, char** lines, sbuf* wout) {
  vmqgb_batch_reset(b);
  vmqgb_view_enter(view, b);   /* as vmqg_nif.c: the reader section covers the prepare */
  const uint8_t** tp = (const uint8_t**)malloc(n * sizeof(*tp));
  size_t* tl = (size_t*)malloc(n * sizeof(size_t));
  uint32_t* mp = (uint32_t*)malloc(n * sizeof(uint32_t));
  for (size_t i = 0; i < n; i++) {
    tp[i] = (const uint8_t*)pubs[lo + i].topic;
    tl[i] = pubs[lo + i].len;
    mp[i] = pubs[lo + i].mp;
  }
  const int prc = vmqgb_batch_add_many(b, ctx, n, mp, tp, tl, idx);
  free(tp); free(tl); free(mp);
  if (prc) return prc;
  const vmqg_emit* recs = NULL;
  uint64_t nrecs = 0;
  const int rc = vmqgb_view_match(view, b, a->ranges, &recs, &nrecs);
  for (size_t i = 0; i < n; i++) {
    sbuf s = {0, 0, 0};
    char h[64];
    int frc = idx[i] < 0 ? (int)idx[i] : rc;
    sput(&s, "");
    if (!frc) frc = b->out_ranges ? vmqgb_fold_ranges(b, recs, nrecs, (size_t)idx[i], put_entry, &s)
                              : vmqgb_fold(b, (size_t)idx[i], put_entry, &s);
    if (wout) snprintf(h, sizeof h, "%zu %llu %d", lo + i, (unsigned long long)b->epoch, frc);
    else snprintf(h, sizeof h, "%zu %d", lo + i, frc);
    sbuf line = {0, 0, 0};
    sput(&line, h);
    if (!frc) sput(&line, s.buf);
    free(s.buf);
    if (wout) { sput(wout, line.buf); sput(wout, "\n"); free(line.buf); }
    else lines[lo + i] = line.buf;
  }
  vmqgb_view_release(view, b);
  return 0;
}

/* one batcher: batches t, t + T, ... (W: pass after pass) */
static void* batcher(void* p) {
  bt_t* a = (bt_t*)p;
  vmqgb_batch b;
  if (vmqgb_batch_init(&b, a->B)) { a->err = VMQG_E_NOMEM; return NULL; }
  vmqgb_view_bind(view, &b);   /* as the NIF's batch_new: batcher k on lane k mod N */
  long* idx = (long*)malloc(a->B * sizeof(long));
  for (int pass = 0; !a->err; pass++) {
    if (a->wout ? (pass >= a->passes && writer_done) : pass >= 1) break;
    for (size_t lo = (size_t)a->tid * a->B; lo < npubs && !a->err; lo += (size_t)a->T * a->B) {
      const size_t n = lo + a->B <= npubs ? a->B : npubs - lo;
      const int rc = one_batch(a, &b, idx, lo, n, a->lines, a->wout);
      if (rc) a->err = rc;
    }
  }
  free(idx);
  vmqgb_batch_free(&b);
  return NULL;
}

typedef struct { int rounds, err; } churn_t;

static void* churner(void* p) {   /* a writer: S/U pairs nobody's publishes match */
  churn_t* c = (churn_t*)p;
  vmqgb_ops ops;
  vmqgb_ops_init(&ops);
  for (int r = 0; r < c->rounds && !c->err; r++) {
    char f[32];
    const int l = snprintf(f, sizeof f, "zz/%d", r % 97);
    const uint32_t kind = (r / 97) % 2 ? VMQG_OP_DEL : VMQG_OP_ADD;
    vmqgb_view_write_begin(view);
    int rc = vmqgb_ops_add_filter(&ops, ctx, kind, 0, (const uint8_t*)f, (size_t)l, 0, 900000 + (uint32_t)(r % 97), 0);
    if (!rc) rc = vmqgb_view_apply_ops(view, &ops, NULL);
    if (!rc) check_digests();
    vmqgb_view_write_end(view);
    if (rc) c->err = rc;
  }
  vmqgb_ops_free(&ops);
  return NULL;
}

static int run_match(FILE* out, int ranges, int T, size_t B, int churn_rounds) {
  char** lines = (char**)calloc(npubs ? npubs : 1, sizeof(char*));
  bt_t* a = (bt_t*)calloc((size_t)T, sizeof(bt_t));
  pthread_t* th = (pthread_t*)calloc((size_t)T, sizeof(pthread_t));
  pthread_t cw;
  churn_t cc = {churn_rounds, 0};
  if (churn_rounds) pthread_create(&cw, NULL, churner, &cc);
  for (int t = 0; t < T; t++) {
    a[t] = (bt_t){t, T, ranges, B, lines, 0, NULL, 0};
    pthread_create(&th[t], NULL, batcher, &a[t]);
  }
  int err = 0;
  for (int t = 0; t < T; t++) { pthread_join(th[t], NULL); if (a[t].err) err = a[t].err; }
  if (churn_rounds) { pthread_join(cw, NULL); if (cc.err) err = cc.err; }
  if (!err) {
    fprintf(out, "M %zu\n", npubs);
    for (size_t i = 0; i < npubs; i++) { fprintf(out, "%s\n", lines[i] ? lines[i] : "missing"); free(lines[i]); }
  }
  free(lines); free(a); free(th);
  return err;
}

/* "<node> <sub> <info> <mp> <filter>" of an S/U/X line into ops (interning
 * its words: callers hold the view's write lock when batchers run) */
static int add_change_line(vmqgb_ops* ops, const char* rest, uint32_t kind) {
  unsigned node, sub, info, mp;
  int off = 0;
  if (sscanf(rest, "%u %u %u %u %n", &node, &sub, &info, &mp, &off) < 4) return VMQG_E_INVAL;
  const char* f = rest + off;
  const size_t fl = strlen(f);
  if (fl > 7 && memcmp(f, "$share/", 7) == 0) {   /* remember the group's text by its word id */
    const char* g = f + 7;
    const char* e = strchr(g, '/');
    uint64_t offs[2] = {0, (uint64_t)(e - g)};
    uint32_t wid;
    if (vmqg_intern_words(ctx, (const uint8_t*)g, offs, 1, 1, &wid)) return VMQG_E_INVAL;
    if (wid >= gcap) return VMQG_E_LIMIT;   /* gname is sized once: batchers read it concurrently */
    if (!gname[wid]) gname[wid] = strndup(g, (size_t)(e - g));
  }
  return vmqgb_ops_add_filter(ops, ctx, kind, mp, (const uint8_t*)f, fl, node, sub, info);
}

/* W: the churn groups, applied by a writer while batchers match */
static char*** groups;           /* groups[k]: NULL-terminated change lines ("S ..." / "U ...") */
static size_t ngroups;

typedef struct { uint64_t* epochs; int err; } wr_t;

static void* group_writer(void* p) {
  wr_t* w = (wr_t*)p;
  vmqgb_ops ops;
  vmqgb_ops_init(&ops);
  for (size_t k = 0; k < ngroups && !w->err; k++) {
    struct timespec ts = {0, 1000000};
    nanosleep(&ts, NULL);
    vmqgb_view_write_begin(view);
    for (char** l = groups[k]; *l && !w->err; l++)
      if (add_change_line(&ops, *l + 2, (*l)[0] == 'S' ? VMQG_OP_ADD : VMQG_OP_DEL)) w->err = VMQG_E_INVAL;
    if (!w->err) w->err = vmqgb_view_apply_ops(view, &ops, &w->epochs[k]);
    if (!w->err) check_digests();
    vmqgb_ops_reset(&ops);
    vmqgb_view_write_end(view);
  }
  writer_done = 1;
  vmqgb_ops_free(&ops);
  return NULL;
}

static int run_w(FILE* out, int ranges, int T, size_t B, int passes) {
  uint64_t e0 = 0;
  vmqg_epoch(ctx, &e0);
  bt_t* a = (bt_t*)calloc((size_t)T, sizeof(bt_t));
  sbuf* wo = (sbuf*)calloc((size_t)T, sizeof(sbuf));
  pthread_t* th = (pthread_t*)calloc((size_t)T, sizeof(pthread_t));
  pthread_t cw;
  wr_t w = {(uint64_t*)calloc(ngroups + 1, sizeof(uint64_t)), 0};
  writer_done = 0;
  for (int t = 0; t < T; t++) {
    a[t] = (bt_t){t, T, ranges, B, NULL, passes, &wo[t], 0};
    sput(&wo[t], "");
    pthread_create(&th[t], NULL, batcher, &a[t]);
  }
  pthread_create(&cw, NULL, group_writer, &w);
  int err = 0;
  pthread_join(cw, NULL);
  if (w.err) err = w.err;
  for (int t = 0; t < T; t++) { pthread_join(th[t], NULL); if (a[t].err) err = a[t].err; }
  if (!err) {
    size_t lines = 0;
    for (int t = 0; t < T; t++) for (size_t i = 0; i < wo[t].n; i++) lines += wo[t].buf[i] == '\n';
    fprintf(out, "W %llu %zu %zu\n", (unsigned long long)e0, ngroups, lines);
    for (size_t k = 0; k < ngroups; k++) fprintf(out, "g %zu %llu\n", k, (unsigned long long)w.epochs[k]);
    for (int t = 0; t < T; t++) fputs(wo[t].buf, out);
  }
  for (int t = 0; t < T; t++) free(wo[t].buf);
  free(a); free(wo); free(th); free(w.epochs);
  return err;
}

int main(int argc, char** argv) {
  if (argc != 3) { fprintf(stderr, "usage: %s <script> <out>\n", argv[0]); return 2; }
  FILE* in = fopen(argv[1], "r");
  FILE* out = fopen(argv[2], "w");
  if (!in || !out) { perror("open"); return 2; }
  vmqg_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.device = 0;
  cfg.max_nodes = VMQG_MAX_NODES;
  int err = 0;
  ctx = vmqg_create(&cfg, &err);
  if (!ctx) { fprintf(stderr, "vmqg_create: %d\n", err); return 3; }
  view = vmqgb_view_new(ctx);
  gcap = 1u << 20;   /* group names by word id, sized once (batchers read it while a writer adds) */
  gname = (char**)calloc(gcap, sizeof(char*));
  vmqgb_ops ops;
  vmqgb_ops_init(&ops);
  char* line = NULL;
  int group_open = 0;
  size_t lcap = 0;
  ssize_t ln;
  while ((ln = getline(&line, &lcap, in)) > 0) {
    if (line[ln - 1] == '\n') line[--ln] = 0;
    if (line[0] == 'S' || line[0] == 'U') {
      if (add_change_line(&ops, line + 2, line[0] == 'S' ? VMQG_OP_ADD : VMQG_OP_DEL)) {
        fprintf(stderr, "bad change: %s\n", line);
        return 6;
      }
    } else if (line[0] == 'G') {
      group_open = 0;
    } else if (line[0] == 'X') {
      if (!group_open) {   /* the first X after a G (or the start) opens a group */
        groups = (char***)realloc(groups, (ngroups + 1) * sizeof(char**));
        groups[ngroups] = (char**)calloc(1, sizeof(char*));
        ngroups++;
        group_open = 1;
      }
      char** g = groups[ngroups - 1];
      size_t k = 0;
      while (g[k]) k++;
      g = (char**)realloc(g, (k + 2) * sizeof(char*));
      g[k] = strdup(line + 2);
      g[k + 1] = NULL;
      groups[ngroups - 1] = g;
    } else if (line[0] == 'R') {
      int n = 0;
      if (sscanf(line + 2, "%d", &n) != 1 || n < 1 || n >= VMQGB_MAX_LANES) return 12;
      for (int k = 0; k < n; k++) {
        vmqg_config rc = cfg;
        rc.flags = VMQG_CFG_REPLICA;
        vmqg_ctx* x = vmqg_create(&rc, &err);
        if (!x || (err = vmqgb_view_add_replica(view, x))) { fprintf(stderr, "replica: %d\n", err); return 13; }
        replicas[nreplicas++] = x;
      }
    } else if (line[0] == 'F') {   /* F n: the next n range pins answer E_STATE (the ranges fallback) */
      long n = 0;
      if (sscanf(line + 2, "%ld", &n) != 1 || vmqgb_view_set_option(view, "force_pin_state", n)) return 14;
      forced = 1;
    } else if (line[0] == 'A') {
      vmqgb_view_write_begin(view);
      const int rc = vmqgb_view_apply_ops(view, &ops, NULL);
      if (!rc) check_digests();
      vmqgb_view_write_end(view);
      if (rc) { fprintf(stderr, "apply: %d\n", rc); return 7; }
    } else if (line[0] == 'P') {
      unsigned mp;
      int off = 0;
      if (sscanf(line + 2, "%u %n", &mp, &off) < 1) return 8;
      if (npubs == pcap) { pcap = pcap ? 2 * pcap : 1024; pubs = (pub_t*)realloc(pubs, pcap * sizeof(pub_t)); }
      pubs[npubs].mp = mp;
      pubs[npubs].topic = strdup(line + 2 + off);
      pubs[npubs].len = strlen(pubs[npubs].topic);
      npubs++;
    } else if (line[0] == 'W') {
      char mode[16];
      int T = 1, passes = 1;
      size_t B = 1;
      if (sscanf(line + 2, "%15s %d %zu %d", mode, &T, &B, &passes) < 4 || T < 1 || T > 64 || B < 1) return 9;
      vmqgb_view_stats s0, s1;
      vmqgb_view_get_stats(view, &s0);
      const int rc = run_w(out, strcmp(mode, "ranges") == 0, T, B, passes);
      if (rc) { fprintf(stderr, "W: %d\n", rc); return 11; }
      vmqgb_view_get_stats(view, &s1);
      fprintf(out, "v %llu %llu %llu", (unsigned long long)(s1.rounds - s0.rounds),
              (unsigned long long)(s1.stale_rematches - s0.stale_rematches),
              (unsigned long long)(s1.round_batches - s0.round_batches));
      for (int k = 0; k < vmqgb_view_lanes(view); k++)
        fprintf(out, " %llu", (unsigned long long)(s1.lane_rounds[k] - s0.lane_rounds[k]));
      fputc('\n', out);
      for (size_t k = 0; k < ngroups; k++) { for (char** l = groups[k]; *l; l++) free(*l); free(groups[k]); }
      ngroups = 0;
      group_open = 0;
    } else if (line[0] == 'M' || line[0] == 'C') {
      char mode[16];
      int T = 1, rounds = 0;
      size_t B = 1;
      if (sscanf(line + 2, "%15s %d %zu %d", mode, &T, &B, &rounds) < 3 || T < 1 || T > 64 || B < 1) return 9;
      const int rc = run_match(out, strcmp(mode, "ranges") == 0, T, B, line[0] == 'C' ? rounds : 0);
      if (rc) { fprintf(stderr, "match: %d\n", rc); return 10; }
    }
  }
  if (nreplicas) fprintf(out, "H %llu %llu\n", (unsigned long long)digests_checked, (unsigned long long)digests_mismatched);
  if (forced) {
    vmqgb_view_stats vs;
    vmqgb_view_get_stats(view, &vs);
    fprintf(out, "F %llu\n", (unsigned long long)vs.ranges_fallbacks);
  }
  fclose(out);
  vmqgb_view_free(view);
  for (int k = 0; k < nreplicas; k++) vmqg_destroy(replicas[k]);
  vmqg_destroy(ctx);
  return 0;
}
