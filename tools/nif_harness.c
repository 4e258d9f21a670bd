/*
 * nif_harness.c — times the host half of the drop-in path the NIF runs
 * (integration/c_src/vmqg_nif.c over vmqg_batch.c), on config C's shape:
 * 1,000,000 devices/{d}/telemetry/# + 64 devices/+/telemetry/#, publishes
 * devices/{d}/telemetry/m{k} as raw topic bytes, d uniform in [0, 1.25M).
 *
 * Per batch of B publishes (the fold/4 callers one NIF call serves):
 *   prepare  vmqg_prepare_publish on raw topics (vmq_topic:validate_topic +
 *            word lookup), T threads each into a thread-local batch, merged
 *   match    vmqgb_match (records, H2D + kernels + D2H of every record) or
 *            vmqgb_match_ranges (D2H of {record off, count} entries only)
 *   fold     every FoldFun argument of every publish, T threads (the NIF
 *            builds one term per entry here; the harness sums the ids)
 * Prints one JSON line per (mode, threads, batch).  Needs a GPU.
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

/* ------------------------------------------------------------ worker pool */
typedef struct {
  int nthreads;
  pthread_barrier_t start, done;
  int stage;          /* 1 prepare, 2 fold (records), 3 fold (ranges), 0 exit */
  size_t lo;          /* first publish of the batch */
  size_t n;           /* publishes in the batch */
} pool_t;

static pool_t pool;
static vmqg_ctx* ctx;
static char* topics;            /* NPUB topics, 40 bytes each, NUL padded */
static uint16_t* tlen;
static vmqgb_batch* local;      /* per thread */
static vmqgb_batch main_batch;
static const vmqg_emit* recs;
static uint64_t nrecs;
static uint64_t sums[64];
static uint64_t entries[64];

static int sum_entry(void* acc, const vmqgb_entry* e) {
  uint64_t* s = (uint64_t*)acc;
  s[0] += e->subscriber ^ e->subinfo ^ e->node;
  s[1]++;
  return 0;
}

static void work(int tid) {
  const size_t per = (pool.n + pool.nthreads - 1) / pool.nthreads;
  const size_t a = tid * per, b = a + per < pool.n ? a + per : pool.n;
  if (pool.stage == 1) {
    vmqgb_batch_reset(&local[tid]);
    for (size_t i = a; i < b; i++) {
      const size_t p = pool.lo + i;
      if (vmqgb_batch_add(&local[tid], ctx, 0, (const uint8_t*)topics + p * 40, tlen[p]) < 0) abort();
    }
  } else {
    uint64_t acc[2] = {0, 0};
    for (size_t i = a; i < b; i++) {
      if (pool.stage == 2) vmqgb_fold(&main_batch, i, sum_entry, acc);
      else vmqgb_fold_ranges(&main_batch, recs, nrecs, i, sum_entry, acc);
    }
    sums[tid] += acc[0];
    entries[tid] += acc[1];
  }
}

static void* worker(void* arg) {
  const int tid = (int)(intptr_t)arg;
  for (;;) {
    pthread_barrier_wait(&pool.start);
    if (pool.stage == 0) return NULL;
    work(tid);
    pthread_barrier_wait(&pool.done);
  }
}

static void run_stage(int stage) {   /* the caller is thread 0 */
  pool.stage = stage;
  pthread_barrier_wait(&pool.start);
  work(0);
  pthread_barrier_wait(&pool.done);
}

int main(int argc, char** argv) {
  const size_t NDEV = 1000000, NWILD = 64, NPUB = (size_t)1 << 20;
  int threads_list[2] = {1, 16};
  size_t batch_list[2] = {4096, 65536};
  (void)argc; (void)argv;
  vmqg_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.device = 0;
  cfg.hint_edges = cfg.hint_paths = 3 * NDEV + 1024;
  cfg.hint_keys = cfg.hint_records = NDEV + 1024;
  int err = 0;
  ctx = vmqg_create(&cfg, &err);
  if (!ctx) { fprintf(stderr, "vmqg_create: %d\n", err); return 1; }
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
      if (vmqgb_ops_apply(&ops, ctx, NULL)) { fprintf(stderr, "apply failed\n"); return 3; }
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
  local = (vmqgb_batch*)calloc(64, sizeof(vmqgb_batch));
  for (int t = 0; t < 64; t++) vmqgb_batch_init(&local[t], 65536);
  vmqgb_batch_init(&main_batch, 65536);
  fprintf(stderr, "loaded %zu subscriptions in %.1fs\n", NDEV + NWILD, load_s);
  for (int mode = 0; mode < 2; mode++) {
    for (int ti = 0; ti < 2; ti++) {
      const int T = threads_list[ti];
      pool.nthreads = T;
      pthread_barrier_init(&pool.start, NULL, (unsigned)T);
      pthread_barrier_init(&pool.done, NULL, (unsigned)T);
      pthread_t th[64];
      for (int t = 1; t < T; t++) pthread_create(&th[t], NULL, worker, (void*)(intptr_t)t);
      for (int bi = 0; bi < 2; bi++) {
        const size_t B = batch_list[bi];
        double t_prep = 0, t_match = 0, t_fold = 0;
        uint64_t n_entries = 0;
        memset(entries, 0, sizeof entries);
        const double tstart = now();
        for (size_t lo = 0; lo < NPUB; lo += B) {
          pool.lo = lo;
          pool.n = lo + B <= NPUB ? B : NPUB - lo;
          double a = now();
          run_stage(1);
          vmqgb_batch_reset(&main_batch);
          for (int t = 0; t < T; t++) vmqgb_batch_append(&main_batch, &local[t]);
          double b = now();
          int rc = mode == 0 ? vmqgb_match(&main_batch, ctx) : vmqgb_match_ranges(&main_batch, ctx);
          if (!rc && mode == 1) rc = vmqg_records(ctx, &recs, &nrecs);
          if (rc) { fprintf(stderr, "match failed: %d\n", rc); return 4; }
          double c = now();
          run_stage(mode == 0 ? 2 : 3);
          double d = now();
          t_prep += b - a; t_match += c - b; t_fold += d - c;
        }
        const double total = now() - tstart;
        for (int t = 0; t < T; t++) n_entries += entries[t];
        printf("{\"mode\": \"%s\", \"threads\": %d, \"batch\": %zu, \"publishes\": %zu, \"entries\": %llu, "
               "\"publishes_per_s\": %.4g, \"prepare_publishes_per_s\": %.4g, \"match_publishes_per_s\": %.4g, "
               "\"fold_entries_per_s\": %.4g, \"seconds\": {\"prepare\": %.3f, \"match\": %.3f, \"fold\": %.3f}, "
               "\"load_s\": %.1f}\n",
               mode == 0 ? "records" : "ranges", T, B, NPUB, (unsigned long long)n_entries, NPUB / total,
               NPUB / t_prep, NPUB / t_match, n_entries / t_fold, t_prep, t_match, t_fold, load_s);
        fflush(stdout);
      }
      pool.stage = 0;
      if (T > 1) pthread_barrier_wait(&pool.start);
      for (int t = 1; t < T; t++) pthread_join(th[t], NULL);
      pthread_barrier_destroy(&pool.start);
      pthread_barrier_destroy(&pool.done);
    }
  }
  uint64_t s = 0;
  for (int t = 0; t < 64; t++) s += sums[t];
  fprintf(stderr, "checksum %llu\n", (unsigned long long)s);
  vmqg_destroy(ctx);
  return 0;
}
