/* GPU check of the NIF's C core (integration/c_src/vmqg_batch.c) driven the
 * way vmqg_nif.c drives it: batcher threads, each with its own batch, under
 * the view's locking protocol (read lock: prepare, device call, fold; the
 * device call serialised), subscription changes as writers — against the
 * oracle (tests/test_nif_layer.py compares the output).
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

typedef struct {
  int tid, T, ranges;
  size_t B;
  char** lines;          /* per publish: its output line */
  int err;
} bt_t;

typedef struct { char* buf; size_t n, cap; } sbuf;

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

/* one batcher, exactly as vmqg_nif.c's match/4: batches t, t + T, ... */
static void* batcher(void* p) {
  bt_t* a = (bt_t*)p;
  vmqgb_batch b;
  if (vmqgb_batch_init(&b, a->B)) { a->err = VMQG_E_NOMEM; return NULL; }
  long* idx = (long*)malloc(a->B * sizeof(long));
  for (size_t lo = (size_t)a->tid * a->B; lo < npubs; lo += (size_t)a->T * a->B) {
    const size_t n = lo + a->B <= npubs ? a->B : npubs - lo;
    vmqgb_view_read_begin(view);
    vmqgb_batch_reset(&b);
    for (size_t i = 0; i < n; i++)
      idx[i] = vmqgb_batch_add(&b, ctx, pubs[lo + i].mp, (const uint8_t*)pubs[lo + i].topic, pubs[lo + i].len);
    const vmqg_emit* recs = NULL;
    uint64_t nrecs = 0;
    const int rc = vmqgb_view_match(view, &b, a->ranges, &recs, &nrecs);
    for (size_t i = 0; i < n; i++) {
      sbuf s = {0, 0, 0};
      char h[64];
      int frc = idx[i] < 0 ? (int)idx[i] : rc;
      sput(&s, "");
      if (!frc) frc = a->ranges ? vmqgb_fold_ranges(&b, recs, nrecs, (size_t)idx[i], put_entry, &s)
                                : vmqgb_fold(&b, (size_t)idx[i], put_entry, &s);
      snprintf(h, sizeof h, "%zu %d", lo + i, frc);
      sbuf line = {0, 0, 0};
      sput(&line, h);
      if (!frc) sput(&line, s.buf);
      free(s.buf);
      a->lines[lo + i] = line.buf;
    }
    vmqgb_view_read_end(view);
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
    if (!rc) rc = vmqgb_ops_apply(&ops, ctx, NULL);
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
    a[t] = (bt_t){t, T, ranges, B, lines, 0};
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
  vmqgb_ops ops;
  vmqgb_ops_init(&ops);
  char* line = NULL;
  size_t lcap = 0;
  ssize_t ln;
  while ((ln = getline(&line, &lcap, in)) > 0) {
    if (line[ln - 1] == '\n') line[--ln] = 0;
    if (line[0] == 'S' || line[0] == 'U') {
      unsigned node, sub, info, mp;
      int off = 0;
      if (sscanf(line + 2, "%u %u %u %u %n", &node, &sub, &info, &mp, &off) < 4) { fprintf(stderr, "bad: %s\n", line); return 4; }
      const char* f = line + 2 + off;
      const size_t fl = strlen(f);
      if (fl > 7 && memcmp(f, "$share/", 7) == 0) {   /* remember the group's text by its word id */
        const char* g = f + 7;
        const char* e = strchr(g, '/');
        uint64_t offs[2] = {0, (uint64_t)(e - g)};
        uint32_t wid;
        if (vmqg_intern_words(ctx, (const uint8_t*)g, offs, 1, 1, &wid)) return 5;
        if (wid >= gcap) {
          size_t nc = gcap ? gcap : 64;
          while (nc <= wid) nc *= 2;
          gname = (char**)realloc(gname, nc * sizeof(char*));
          memset(gname + gcap, 0, (nc - gcap) * sizeof(char*));
          gcap = nc;
        }
        if (!gname[wid]) gname[wid] = strndup(g, (size_t)(e - g));
      }
      if (vmqgb_ops_add_filter(&ops, ctx, line[0] == 'S' ? VMQG_OP_ADD : VMQG_OP_DEL, mp, (const uint8_t*)f, fl, node,
                               sub, info)) { fprintf(stderr, "add_filter failed: %s\n", line); return 6; }
    } else if (line[0] == 'A') {
      const int rc = vmqgb_view_apply(view, &ops, NULL);
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
    } else if (line[0] == 'M' || line[0] == 'C') {
      char mode[16];
      int T = 1, rounds = 0;
      size_t B = 1;
      if (sscanf(line + 2, "%15s %d %zu %d", mode, &T, &B, &rounds) < 3 || T < 1 || T > 64 || B < 1) return 9;
      const int rc = run_match(out, strcmp(mode, "ranges") == 0, T, B, line[0] == 'C' ? rounds : 0);
      if (rc) { fprintf(stderr, "match: %d\n", rc); return 10; }
    }
  }
  fclose(out);
  vmqgb_view_free(view);
  vmqg_destroy(ctx);
  return 0;
}
