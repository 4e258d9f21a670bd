/*
 * nif_harness.c — times the host half of the drop-in path the NIF runs
 * (integration/c_src/vmqg_nif.c over vmqg_batch.c), on config C's shape:
 * 1,000,000 devices/{d}/telemetry/# + 64 devices/+/telemetry/#, publishes
 * devices/{d}/telemetry/m{k} as raw topic bytes, d uniform in [0, 1.25M).
 *
 Threading exactly as the NIF's (vmqg_nif.c match/4 under
 * vmq_reg_gpu_batcher): T batcher threads, each with its own batch of B
 * publishes, each batch under the view's read lock (vmqgb_view_*):
 *   prepare  vmqg_prepare_publish on raw topics (vmq_topic:validate_topic +
 *            word lookup), into the batcher's batch
 *   match    vmqgb_view_match: vmqgb_match (records: H2D + kernels + D2H of
 *            every record) or vmqgb_match_ranges (D2H of {record off, count}
 *            entries only); the device call is the only serialised step
 *   fold     every FoldFun argument of every publish (the NIF builds one term
 *            per entry here; the harness sums the ids)
 * and once more with a writer applying config D's 100k changes/s (write
 * lock) while 16 batchers run.  Prints one JSON line per configuration.
 * Needs a GPU.  argv[1]: seconds per configuration (default 3).
 *
 * build: gcc -O2 -std=gnu11 -pthread -Iinclude -Iintegration/c_src tools/nif_harness.c \
 *        integration/c_src/vmqg_batch.c -Lvernemq_amd -l:libvmqgpu.so \
 *        -Wl,-rpath,'$ORIGIN/../../vernemq_amd' -o tools/bin/nif_harness
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "vmqg_batch.h"

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

static uint64_t sm_state = 0xC;
static uint64_t splitmix(void) {
  uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static vmqg_ctx* ctx;
static vmqgb_view* view;
static char* topics;            /* NPUB topics, 40 bytes each, NUL padded */
static uint16_t* tlen;
static size_t NPUB;

static int sum_entry(void* acc, const vmqgb_entry* e) {
  uint64_t* s = (uint64_t*)acc;
  s[0] += e->subscriber ^ e->subinfo ^ e->node;
  s[1]++;
  return 0;
}

/* ------------------------------------------------------------ batchers */
/* One batcher thread = one vmq_reg_gpu_batcher process and its match/4 NIF
 * call (integration/c_src/vmqg_nif.c): its own batch, the view's read lock
 * around prepare, the device call (serialised by the view) and the fold. */
typedef struct {
  int tid, T, ranges;
  size_t B;
  double t_end;
  uint64_t pubs, entries, sum, batches;
  double t_prep, t_match, t_fold;
  int err;
} bt_t;

static void* batcher(void* p) {
  bt_t* a = (bt_t*)p;
  vmqgb_batch b;
  vmqgb_batch_init(&b, a->B);
  uint64_t acc[2] = {0, 0};
  size_t lo = ((size_t)a->tid * a->B * 7919) % NPUB;
  while (now() < a->t_end) {
    const double t0 = now();
    vmqgb_view_read_begin(view);
    vmqgb_batch_reset(&b);
    for (size_t i = 0; i < a->B; i++) {
      if (i && i % VMQGB_YIELD_EVERY == 0) vmqgb_view_yield(view);
      const size_t q = (lo + i) % NPUB;
      if (vmqgb_batch_add(&b, ctx, 0, (const uint8_t*)topics + q * 40, tlen[q]) < 0) { a->err = 1; break; }
    }
    lo = (lo + (size_t)a->T * a->B) % NPUB;
    const double t1 = now();
    const vmqg_emit* recs = NULL;
    uint64_t nrecs = 0;
    int rc = vmqgb_view_match(view, &b, a->ranges, &recs, &nrecs);
    const double t2 = now();
    for (size_t i = 0; !rc && i < b.n; i++) {
      if (!a->ranges && i && i % VMQGB_YIELD_EVERY == 0) vmqgb_view_yield(view);   /* records: copies */
      rc = a->ranges ? vmqgb_fold_ranges(&b, recs, nrecs, i, sum_entry, acc) : vmqgb_fold(&b, i, sum_entry, acc);
    }
    vmqgb_view_read_end(view);
    const double t3 = now();
    if (rc || a->err) { a->err = rc ? rc : a->err; break; }
    a->pubs += b.n;
    a->batches++;
    a->t_prep += t1 - t0; a->t_match += t2 - t1; a->t_fold += t3 - t2;
  }
  a->sum = acc[0];
  a->entries = acc[1];
  vmqgb_batch_free(&b);
  return NULL;
}

/* config D's churn rate on this shape: a writer applying `ops` subscription
 * changes every `period` seconds (half adds, half deletes of extra device
 * filters that no publish matches) while the batchers run */
typedef struct { double t_end, period; int ops; uint64_t applied; double t_apply; int err; } churn_t;

static void* churner(void* p) {
  churn_t* c = (churn_t*)p;
  vmqgb_ops ops;
  vmqgb_ops_init(&ops);
  uint32_t k = 0;
  double next = now();
  while (now() < c->t_end && !c->err) {
    while (now() < next) { struct timespec ts = {0, 200000}; nanosleep(&ts, NULL); }
    next += c->period;
    vmqgb_ops_reset(&ops);
    for (int i = 0; i < c->ops; i++, k++) {
      char f[48];
      const uint32_t slot = k % 20000;
      const int l = snprintf(f, sizeof f, "churn/%u/telemetry/#", slot);
      const uint32_t kind = (k / 20000) % 2 ? VMQG_OP_DEL : VMQG_OP_ADD;
      if (vmqgb_ops_add_filter(&ops, ctx, kind, 0, (const uint8_t*)f, (size_t)l, 0, 2000000 + slot, 1)) { c->err = 1; break; }
    }
    const double t0 = now();
    if (!c->err && vmqgb_view_apply(view, &ops, NULL)) c->err = 2;
    c->t_apply += now() - t0;
    c->applied += (uint64_t)c->ops;
  }
  vmqgb_ops_free(&ops);
  return NULL;
}

int main(int argc, char** argv) {
  const size_t NDEV = 1000000, NWILD = 64;
  NPUB = (size_t)1 << 20;
  const double secs = argc > 1 ? atof(argv[1]) : 3.0;
  const int threads_list[] = {1, 4, 8, 16, 32};
  const size_t batch_list[] = {1024, 4096};
  vmqg_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.device = 0;
  cfg.hint_edges = cfg.hint_paths = 3 * NDEV + 1024;
  cfg.hint_keys = cfg.hint_records = NDEV + 1024;
  int err = 0;
  ctx = vmqg_create(&cfg, &err);
  if (!ctx) { fprintf(stderr, "vmqg_create: %d\n", err); return 1; }
  view = vmqgb_view_new(ctx);
  /* subscriptions through the NIF's op layer: subscriber ids from an interner */
  vmqgb_interner* subs = vmqgb_interner_new();
  vmqgb_ops ops;
  vmqgb_ops_init(&ops);
  char buf[64];
  double t0 = now();
  for (size_t d = 0; d < NDEV + NWILD; d++) {
    const int ln = d < NDEV ? snprintf(buf, sizeof buf, "c%zu", d) : snprintf(buf, sizeof buf, "w%zu", d - NDEV);
    const uint32_t sid = vmqgb_intern(subs, buf, (size_t)ln);
    char f[64];
    const int fl = d < NDEV ? snprintf(f, sizeof f, "devices/%zu/telemetry/#", d) : snprintf(f, sizeof f, "devices/+/telemetry/#");
    if (vmqgb_ops_add_filter(&ops, ctx, VMQG_OP_ADD, 0, (const uint8_t*)f, (size_t)fl, 0, sid, (uint32_t)(d % 3))) return 2;
    if (ops.n == 65536 || d + 1 == NDEV + NWILD) {
      if (vmqgb_view_apply(view, &ops, NULL)) { fprintf(stderr, "apply failed\n"); return 3; }
    }
  }
  const double load_s = now() - t0;
  /* raw publish topics */
  topics = (char*)calloc(NPUB, 40);
  tlen = (uint16_t*)calloc(NPUB, sizeof(uint16_t));
  for (size_t i = 0; i < NPUB; i++) {
    const uint64_t r = splitmix();
    tlen[i] = (uint16_t)snprintf(topics + i * 40, 40, "devices/%llu/telemetry/m%llu",
                                 (unsigned long long)(r % (NDEV + NDEV / 4)), (unsigned long long)((r >> 40) % 16));
  }
  fprintf(stderr, "loaded %zu subscriptions in %.1fs\n", NDEV + NWILD, load_s);
  uint64_t checksum = 0;
  for (int churn = 0; churn < 2; churn++) {
    for (int mode = 0; mode < 2; mode++) {
      for (size_t ti = 0; ti < sizeof threads_list / sizeof threads_list[0]; ti++) {
        for (size_t bi = 0; bi < sizeof batch_list / sizeof batch_list[0]; bi++) {
          const int T = threads_list[ti];
          const size_t B = batch_list[bi];
          if (churn && (T != 16 || B != 4096)) continue;   /* churn: the shipped shape only */
          bt_t a[64];
          pthread_t th[64], cw;
          churn_t cc = {0, 0.01, 1000, 0, 0, 0};   /* 100k ops/s: config D's 1 %/s of 10M */
          const double tstart = now(), t_end = tstart + secs;
          cc.t_end = t_end;
          if (churn) pthread_create(&cw, NULL, churner, &cc);
          for (int t = 0; t < T; t++) {
            memset(&a[t], 0, sizeof a[t]);
            a[t].tid = t; a[t].T = T; a[t].ranges = mode; a[t].B = B; a[t].t_end = t_end;
            pthread_create(&th[t], NULL, batcher, &a[t]);
          }
          uint64_t pubs = 0, ents = 0, nb = 0;
          double tp = 0, tm = 0, tf = 0;
          for (int t = 0; t < T; t++) {
            pthread_join(th[t], NULL);
            if (a[t].err) { fprintf(stderr, "batcher %d failed: %d\n", t, a[t].err); return 4; }
            pubs += a[t].pubs; ents += a[t].entries; nb += a[t].batches; checksum += a[t].sum;
            tp += a[t].t_prep; tm += a[t].t_match; tf += a[t].t_fold;
          }
          if (churn) { pthread_join(cw, NULL); if (cc.err) { fprintf(stderr, "churn failed\n"); return 5; } }
          const double el = now() - tstart;
          printf("{\"threading\": \"vmqg_nif batchers (vmqgb_view)\", \"mode\": \"%s\", \"batchers\": %d, "
                 "\"batch\": %zu, \"seconds\": %.2f, \"publishes\": %llu, \"entries\": %llu, \"publishes_per_s\": %.4g, "
                 "\"entries_per_s\": %.4g, \"per_batch_ms\": {\"prepare\": %.3f, \"match\": %.3f, \"fold\": %.3f}, "
                 "\"churn_ops_per_s\": %.4g, \"apply_ms_per_batch\": %.3f, \"load_s\": %.1f}\n",
                 mode ? "ranges" : "records", T, B, el, (unsigned long long)pubs, (unsigned long long)ents, pubs / el,
                 ents / el, nb ? tp * 1e3 / nb : 0, nb ? tm * 1e3 / nb : 0, nb ? tf * 1e3 / nb : 0,
                 churn ? cc.applied / el : 0.0, churn && cc.applied ? cc.t_apply * 1e3 / (cc.applied / cc.ops) : 0.0,
                 load_s);
          fflush(stdout);
        }
      }
    }
  }
  fprintf(stderr, "checksum %llu\n", (unsigned long long)checksum);
  vmqgb_view_free(view);
  vmqg_destroy(ctx);
  return 0;
}
