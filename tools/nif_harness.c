/*
 * nif_harness.c — times the host half of the drop-in path the NIF runs
 * (integration/c_src/vmqg_nif.c over vmqg_batch.c), on config C's shape:
 * 1,000,000 devices/{d}/telemetry/# + 64 devices/+/telemetry/#, publishes
 * devices/{d}/telemetry/m{k} as raw topic bytes, d uniform in [0, 1.25M).
 *
 * Threading exactly as the NIF's (vmqg_nif.c match/4 under
 * vmq_reg_gpu_batcher): T batcher threads, each with its own batch of B
 * publishes, no lock anywhere on their path (vmqgb_view_*):
 *   prepare  vmqgb_batch_add_word_lists on the Topic word lists fold/4 is
 *            handed (one dictionary lookup per word; the lists are split
 *            once at start-up, as the Erlang side hands them over split)
 *   match    vmqgb_view_match: the combining submitter (batches queued at
 *            once matched as one device call, rounds pipelined)
 *   fold     every FoldFun argument of every publish (the NIF builds one term
 *            per entry here; the harness sums the ids)
 * Sections (argv[2..], default all):
 *   scale    1..48 batchers, records and ranges
 *   devrec   records copied by the device over PCIe (vmqgb_view_set_device_records)
 *   (VMQGB_RECLAIM=0: dropped rows kept, for an A/B of reclamation)
 *   churn    subscriber events at 100k/s (config D's 1 %/s of 10M) while 16
 *            and 32 batchers run, applied the way the Erlang view applies
 *            them (vmq_reg_gpu_view's drain_events + vmqg_nif:apply_many):
 *            "coalesced" = the events of a window — from the first event
 *            queued, 2 ms or 1,000 events, whichever comes first — in one
 *            apply; the events unsubscribe and resubscribe real
 *            devices/{d}/telemetry/# filters, so they change answers
 *   churn1   the same with one apply per event ("single": round 3's view)
 *   load     initialize_trie while matching: a writer interning new
 *            subscriptions as vmqg_nif:add_init does (the writer mutex, an
 *            apply every 65,536) while 16 batchers run
 * Prints one JSON line per configuration.  Needs a GPU.  argv[1]: seconds
 * per configuration (default 3).  VMQGB_REPLICAS=n adds n replica contexts
 * on device 0 as lanes of the view (batchers spread over them).
 *
 * build: see tools/Makefile (gcc -O2 -pthread ... integration/c_src/vmqg_batch.c -l:libvmqgpu.so)
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
static size_t* tlen;
static const uint8_t** tptr;
static uint32_t* tmp0;           /* mountpoint 0 for every publish */
static uint32_t* wcnt;           /* publish i: its word list, words [woff[i], woff[i] + wcnt[i]) */
static size_t* woff;
static const uint8_t** wptr;
static size_t* wlen;
static size_t NPUB;
static const size_t NDEV = 1000000, NWILD = 64;

static int sum_entry(void* acc, const vmqgb_entry* e) {
  uint64_t* s = (uint64_t*)acc;
  s[0] += e->subscriber ^ e->subinfo ^ e->node;
  s[1]++;
  return 0;
}

/* the same per-entry work over a run of records (vmqgb_fold_spans) */
static int sum_span(void* acc, const vmqg_emit* r, size_t n) {
  uint64_t* s = (uint64_t*)acc;
  uint64_t x = 0;
  for (size_t j = 0; j < n; j++) x += r[j].subscriber ^ r[j].subinfo ^ (r[j].kind_node & 0xFFFFFFu);
  s[0] += x;
  s[1] += n;
  return 0;
}
static int fold_spans = 1;   /* 0: one callback per entry (vmqgb_fold / vmqgb_fold_ranges) */

/* ------------------------------------------------------------ batchers */
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
  vmqgb_view_bind(view, &b);   /* batcher k on device context k mod N, as the NIF's batch_new */
  long* idx = (long*)malloc(a->B * sizeof(long));
  uint64_t acc[2] = {0, 0};
  size_t lo = ((size_t)a->tid * a->B * 7919) % NPUB;
  while (now() < a->t_end) {
    const double t0 = now();
    vmqgb_batch_reset(&b);
    vmqgb_view_enter(view, &b);   /* as vmqg_nif.c: the reader section covers the prepare */
    if (lo + a->B > NPUB) lo = 0;
    if (vmqgb_batch_add_word_lists(&b, ctx, a->B, tmp0 + lo, wcnt + lo, wptr + woff[lo], wlen + woff[lo], idx))
      a->err = 1;
    lo = (lo + (size_t)a->T * a->B) % NPUB;
    const double t1 = now();
    const vmqg_emit* recs = NULL;
    uint64_t nrecs = 0;
    int rc = a->err ? 0 : vmqgb_view_match(view, &b, a->ranges, &recs, &nrecs);
    const double t2 = now();
    for (size_t i = 0; !rc && i < b.n; i++) {
      if (fold_spans) {
        vmqgb_prefetch_entries(&b, b.out_ranges, recs, nrecs, i + VMQGB_PREFETCH_AHEAD);
        rc = vmqgb_fold_spans(&b, b.out_ranges, recs, nrecs, i, sum_span, acc);
      }
      else rc = b.out_ranges ? vmqgb_fold_ranges(&b, recs, nrecs, i, sum_entry, acc) : vmqgb_fold(&b, i, sum_entry, acc);
    }
    vmqgb_view_release(view, &b);
    const double t3 = now();
    if (rc || a->err) { a->err = rc ? rc : a->err; break; }
    a->pubs += b.n;
    a->batches++;
    a->t_prep += t1 - t0; a->t_match += t2 - t1; a->t_fold += t3 - t2;
  }
  a->sum = acc[0];
  a->entries = acc[1];
  free(idx);
  vmqgb_batch_free(&b);
  return NULL;
}

/* ------------------------------------------------------------- churn */
/* subscriber events: device d's devices/{d}/telemetry/# unsubscribed, later
 * subscribed again (one change per event, as a one-topic SUBSCRIBE /
 * UNSUBSCRIBE makes), produced at `rate` per second with their due times */
typedef struct { uint32_t d, kind; double t; } event_t;
typedef struct {
  double t_end, rate;
  int coalesce;                 /* 0: one apply per event; 1: a window's events in one apply */
  pthread_mutex_t mu;
  event_t* q;
  size_t cap, head, tail;       /* ring */
  uint64_t produced, applied, applies, max_group;
  double lag_sum, lag_max, wait_max, apply_sum;
  double* lags;                 /* sample of lags for percentiles */
  size_t nlags, lags_cap;
  size_t max_backlog;
  int err;
} churn_t;

static void* producer(void* p) {
  churn_t* c = (churn_t*)p;
  const double t0 = now();
  uint64_t k = 0;
  while (now() < c->t_end && !c->err) {
    const double due = now();
    const uint64_t want = (uint64_t)((due - t0) * c->rate);
    pthread_mutex_lock(&c->mu);
    for (; k < want; k++) {
      const size_t used = c->tail - c->head;
      if (used == c->cap) break;   /* the writer fell too far behind: stop producing (reported as backlog) */
      event_t* e = &c->q[c->tail % c->cap];
      /* a rotating window of 20,000 devices: unsubscribe them, then resubscribe */
      e->d = (uint32_t)((k % 20000) * 50);
      e->kind = (k / 20000) % 2 ? VMQG_OP_ADD : VMQG_OP_DEL;
      e->t = t0 + (double)k / c->rate;
      c->tail++;
      c->produced++;
      if (c->tail - c->head > c->max_backlog) c->max_backlog = c->tail - c->head;
    }
    pthread_mutex_unlock(&c->mu);
    struct timespec ts = {0, 200000};
    nanosleep(&ts, NULL);
  }
  return NULL;
}

static void* applier(void* p) {   /* the vmq_reg_gpu_view gen_server */
  churn_t* c = (churn_t*)p;
  vmqgb_ops ops;
  vmqgb_ops_init(&ops);
  event_t* grp = (event_t*)malloc(10000 * sizeof(event_t));
  char f[64];
  while (now() < c->t_end && !c->err) {
    pthread_mutex_lock(&c->mu);
    size_t n = c->tail - c->head;
    /* the window: 2 ms after its first event, or 1,000 events (vmq_reg_gpu_view) */
    if (c->coalesce && n && n < 1000 && now() - c->q[c->head % c->cap].t < 0.002) n = 0;
    if (!c->coalesce && n > 1) n = 1;
    if (n > 1000) n = 1000;   /* one apply takes at most 1,000 events: a backlog goes out in slices (vmq_reg_gpu_view ?MAX_COALESCE) */
    for (size_t i = 0; i < n; i++) grp[i] = c->q[(c->head + i) % c->cap];
    c->head += n;
    pthread_mutex_unlock(&c->mu);
    if (!n) { struct timespec ts = {0, 50000}; nanosleep(&ts, NULL); continue; }
    const double t0 = now();
    vmqgb_view_write_begin(view);   /* interning is the writer's (the NIF's add_change) */
    const double t1 = now();
    for (size_t i = 0; i < n; i++) {
      const int l = snprintf(f, sizeof f, "devices/%u/telemetry/#", grp[i].d);
      if (vmqgb_ops_add_filter(&ops, ctx, grp[i].kind, 0, (const uint8_t*)f, (size_t)l, 0, grp[i].d, grp[i].d % 3)) {
        c->err = 1;
        break;
      }
    }
    const int rc = c->err ? 0 : vmqgb_view_apply_ops(view, &ops, NULL);
    vmqgb_ops_reset(&ops);
    vmqgb_view_write_end(view);
    const double t2 = now();
    if (rc) { c->err = 2; break; }
    if (t1 - t0 > c->wait_max) c->wait_max = t1 - t0;
    c->apply_sum += t2 - t0;
    c->applies++;
    c->applied += n;
    if (n > c->max_group) c->max_group = n;
    for (size_t i = 0; i < n; i++) {
      const double lag = t2 - grp[i].t;
      c->lag_sum += lag;
      if (lag > c->lag_max) c->lag_max = lag;
      if (c->nlags < c->lags_cap) c->lags[c->nlags++] = lag;
    }
  }
  free(grp);
  vmqgb_ops_free(&ops);
  return NULL;
}

static int cmp_d(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

/* ------------------------------------------------------------- load */
/* initialize_trie while matching: vmqg_nif:add_init's locking (table lock
 * per subscription, the device mutex only for the apply of every 65,536) */
typedef struct { double t_end; uint64_t added, applies; double wait_max; int err; } load_t;

static void* loader(void* p) {
  load_t* L = (load_t*)p;
  vmqgb_ops ops;
  vmqgb_ops_init(&ops);
  char f[64];
  uint64_t k = 0;
  while (now() < L->t_end && !L->err) {
    const double t0 = now();
    vmqgb_view_write_begin(view);
    const double w = now() - t0;
    if (w > L->wait_max) L->wait_max = w;
    const int l = snprintf(f, sizeof f, "fleet/%llu/telemetry/#", (unsigned long long)k);
    if (vmqgb_ops_add_filter(&ops, ctx, VMQG_OP_ADD, 0, (const uint8_t*)f, (size_t)l, 0, 3000000 + (uint32_t)k, 1))
      L->err = 1;
    if (!L->err && ops.n >= 65536) {
      if (vmqgb_view_apply_ops(view, &ops, NULL)) L->err = 2;
      vmqgb_ops_reset(&ops);
      L->applies++;
    }
    vmqgb_view_write_end(view);
    k++;
  }
  vmqgb_view_write_begin(view);
  if (ops.n && vmqgb_view_apply_ops(view, &ops, NULL)) L->err = 2;
  vmqgb_view_write_end(view);
  L->added = k;
  vmqgb_ops_free(&ops);
  return NULL;
}

/* ----------------------------------------------------------------- run */
static uint64_t checksum;

/* the cgroup's CPU throttling (cgroup v2 cpu.stat): a quota-bound run stalls
 * every thread for the rest of a 100 ms period */
static void cpu_throttle(uint64_t* periods, uint64_t* usec) {
  *periods = *usec = 0;
  FILE* f = fopen("/sys/fs/cgroup/cpu.stat", "r");
  if (!f) return;
  char k[64];
  unsigned long long x;
  while (fscanf(f, "%63s %llu", k, &x) == 2) {
    if (!strcmp(k, "nr_throttled")) *periods = x;
    if (!strcmp(k, "throttled_usec")) *usec = x;
  }
  fclose(f);
}

static int run(const char* section, int T, size_t B, int ranges, double secs, churn_t* cc, load_t* ld) {
  bt_t a[64];
  pthread_t th[64], cw[2];
  vmqgb_view_stats s0, s1;
  vmqgb_view_reset_stats(view);
  vmqgb_view_get_stats(view, &s0);
  vmqg_stats_t e0, e1;
  vmqg_stats(ctx, &e0);
  uint64_t thr0, thu0, thr1, thu1;
  cpu_throttle(&thr0, &thu0);
  const double tstart = now(), t_end = tstart + secs;
  if (cc) {
    cc->t_end = t_end;
    pthread_create(&cw[0], NULL, producer, cc);
    pthread_create(&cw[1], NULL, applier, cc);
  }
  if (ld) { ld->t_end = t_end; pthread_create(&cw[0], NULL, loader, ld); }
  for (int t = 0; t < T; t++) {
    memset(&a[t], 0, sizeof a[t]);
    a[t].tid = t; a[t].T = T; a[t].ranges = ranges; a[t].B = B; a[t].t_end = t_end;
    pthread_create(&th[t], NULL, batcher, &a[t]);
  }
  uint64_t pubs = 0, ents = 0, nb = 0;
  double tp = 0, tm = 0, tf = 0;
  int err = 0;
  for (int t = 0; t < T; t++) {
    pthread_join(th[t], NULL);
    if (a[t].err) { fprintf(stderr, "batcher %d failed: %d\n", t, a[t].err); err = 4; }
    pubs += a[t].pubs; ents += a[t].entries; nb += a[t].batches; checksum += a[t].sum;
    tp += a[t].t_prep; tm += a[t].t_match; tf += a[t].t_fold;
  }
  if (cc) { pthread_join(cw[0], NULL); pthread_join(cw[1], NULL); if (cc->err) { fprintf(stderr, "churn failed %d\n", cc->err); err = 5; } }
  if (ld) { pthread_join(cw[0], NULL); if (ld->err) { fprintf(stderr, "load failed %d\n", ld->err); err = 6; } }
  const double el = now() - tstart;
  vmqgb_view_get_stats(view, &s1);
  vmqg_stats(ctx, &e1);
  cpu_throttle(&thr1, &thu1);
  const uint64_t rounds = s1.rounds - s0.rounds;
  printf("{\"section\": \"%s\", \"mode\": \"%s\", \"fold\": \"%s\", \"batchers\": %d, \"batch\": %zu, \"seconds\": %.2f, "
         "\"publishes\": %llu, \"entries\": %llu, \"publishes_per_s\": %.4g, \"entries_per_s\": %.4g, "
         "\"per_batch_ms\": {\"prepare\": %.3f, \"match\": %.3f, \"fold\": %.3f}, "
         "\"rounds\": %llu, \"publishes_per_round\": %.0f, \"batches_per_round\": %.2f, "
         "\"expanded_batches\": %llu, \"device_record_batches\": %llu, \"state_retries\": %llu, "
         "\"stale_rematches\": %llu, \"overflow_retries\": %llu",
         section, ranges ? "ranges" : "records", fold_spans ? "spans" : "entries", T, B, el, (unsigned long long)pubs, (unsigned long long)ents,
         pubs / el, ents / el, nb ? tp * 1e3 / nb : 0, nb ? tm * 1e3 / nb : 0, nb ? tf * 1e3 / nb : 0,
         (unsigned long long)rounds, rounds ? (double)(s1.round_publishes - s0.round_publishes) / rounds : 0.0,
         rounds ? (double)(s1.round_batches - s0.round_batches) / rounds : 0.0,
         (unsigned long long)(s1.expanded_batches - s0.expanded_batches),
         (unsigned long long)(s1.device_record_batches - s0.device_record_batches),
         (unsigned long long)(s1.state_retries - s0.state_retries),
         (unsigned long long)(s1.stale_rematches - s0.stale_rematches),
         (unsigned long long)(s1.overflow_retries - s0.overflow_retries));
  if (cc) {
    qsort(cc->lags, cc->nlags, sizeof(double), cmp_d);
    const double p50 = cc->nlags ? cc->lags[cc->nlags / 2] : 0, p99 = cc->nlags ? cc->lags[(size_t)(cc->nlags * 0.99)] : 0;
    printf(", \"churn\": {\"delivery\": \"%s\", \"events_per_s_offered\": %.4g, \"events_applied_per_s\": %.4g, "
           "\"applies\": %llu, \"mean_events_per_apply\": %.1f, \"max_events_per_apply\": %llu, "
           "\"backlog_at_end\": %llu, \"max_backlog\": %zu, \"lag_ms\": {\"p50\": %.3f, \"p99\": %.3f, \"max\": %.3f}, "
           "\"max_write_lock_wait_ms\": %.3f, \"mean_apply_section_ms\": %.3f, "
           "\"writer_ms\": {\"stage_mean\": %.3f, \"stage_max\": %.3f, \"device_wait_mean\": %.3f, "
           "\"device_wait_max\": %.3f, \"commit_mean\": %.3f, \"commit_max\": %.3f}, "
           "\"reader_buffer_waits\": %llu, \"reader_buffer_wait_ms\": %.3f}",
           cc->coalesce ? "coalesced" : "single", cc->produced / el, cc->applied / el, (unsigned long long)cc->applies,
           cc->applies ? (double)cc->applied / cc->applies : 0.0, (unsigned long long)cc->max_group,
           (unsigned long long)(cc->produced - cc->applied), cc->max_backlog, p50 * 1e3, p99 * 1e3, cc->lag_max * 1e3,
           cc->wait_max * 1e3, cc->applies ? cc->apply_sum * 1e3 / cc->applies : 0.0,
           s1.applies ? s1.stage_ns * 1e-6 / s1.applies : 0.0, s1.stage_max_ns * 1e-6,
           s1.applies ? s1.dev_wait_ns * 1e-6 / s1.applies : 0.0, s1.dev_wait_max_ns * 1e-6,
           s1.applies ? s1.commit_ns * 1e-6 / s1.applies : 0.0, s1.commit_max_ns * 1e-6,
           (unsigned long long)(e1.reader_waits - e0.reader_waits), (e1.reader_wait_ns - e0.reader_wait_ns) * 1e-6);
  }
  if (ld)
    printf(", \"load\": {\"subscriptions_added_per_s\": %.4g, \"applies\": %llu, \"max_write_lock_wait_ms\": %.3f}",
           ld->added / el, (unsigned long long)ld->applies, ld->wait_max * 1e3);
  printf(", \"lanes\": %d, \"lane_rounds\": [", vmqgb_view_lanes(view));
  for (int k = 0; k < vmqgb_view_lanes(view); k++)
    printf("%s%llu", k ? ", " : "", (unsigned long long)(s1.lane_rounds[k] - s0.lane_rounds[k]));
  printf("], \"follow_ms_mean\": %.3f, \"follow_failures\": %llu",
         s1.applies ? s1.follow_ns * 1e-6 / s1.applies : 0.0, (unsigned long long)s1.follow_failures);
  printf(", \"rebuilds\": %llu, \"cpu_throttled\": {\"periods\": %llu, \"ms\": %.1f}, \"build\": \"%s\"}\n",
         (unsigned long long)(e1.rebuilds - e0.rebuilds), (unsigned long long)(thr1 - thr0), (thu1 - thu0) * 1e-3,
         vmqg_build_id());
  fflush(stdout);
  return err;
}

static int want(int argc, char** argv, const char* s) {
  if (argc <= 2) return 1;
  for (int i = 2; i < argc; i++) if (!strcmp(argv[i], s)) return 1;
  return 0;
}

int main(int argc, char** argv) {
  NPUB = (size_t)1 << 20;
  const double secs = argc > 1 ? atof(argv[1]) : 3.0;
  vmqg_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.device = 0;
  cfg.hint_edges = cfg.hint_paths = 3 * NDEV + 1024;
  cfg.hint_keys = cfg.hint_records = NDEV + 1024;
  int err = 0;
  ctx = vmqg_create(&cfg, &err);
  if (!ctx) { fprintf(stderr, "vmqg_create: %d\n", err); return 1; }
  view = vmqgb_view_new(ctx);
  if (getenv("VMQGB_RECLAIM")) vmqg_set_option(ctx, "reclaim", atoi(getenv("VMQGB_RECLAIM")));   /* A/B of reclamation */
  /* subscriptions through the NIF's op layer; subscriber id = device index
   * (c{d}), the wildcard subscribers after them */
  vmqgb_ops ops;
  vmqgb_ops_init(&ops);
  double t0 = now();
  for (size_t d = 0; d < NDEV + NWILD; d++) {
    char f[64];
    const int fl = d < NDEV ? snprintf(f, sizeof f, "devices/%zu/telemetry/#", d) : snprintf(f, sizeof f, "devices/+/telemetry/#");
    vmqgb_view_write_begin(view);
    if (vmqgb_ops_add_filter(&ops, ctx, VMQG_OP_ADD, 0, (const uint8_t*)f, (size_t)fl, 0, (uint32_t)d, (uint32_t)(d % 3))) return 2;
    if ((ops.n == 65536 || d + 1 == NDEV + NWILD) && vmqgb_view_apply_ops(view, &ops, NULL)) {
      fprintf(stderr, "apply failed\n");
      return 3;
    }
    vmqgb_view_write_end(view);
  }
  const double load_s = now() - t0;
  /* VMQGB_REPLICAS=n: n replica contexts on device 0 as more lanes of the
   * view (the multi-GPU drop-in, rehearsed on one GPU) */
  const int nrep = getenv("VMQGB_REPLICAS") ? atoi(getenv("VMQGB_REPLICAS")) : 0;
  for (int k = 0; k < nrep; k++) {
    vmqg_config rc = cfg;
    rc.flags = VMQG_CFG_REPLICA;
    vmqg_ctx* x = vmqg_create(&rc, &err);
    if (!x || (err = vmqgb_view_add_replica(view, x))) { fprintf(stderr, "replica: %d\n", err); return 1; }
  }
  /* raw publish topics */
  topics = (char*)calloc(NPUB, 40);
  tlen = (size_t*)calloc(NPUB, sizeof(size_t));
  tptr = (const uint8_t**)calloc(NPUB, sizeof(*tptr));
  tmp0 = (uint32_t*)calloc(NPUB, sizeof(uint32_t));
  for (size_t i = 0; i < NPUB; i++) {
    const uint64_t r = splitmix();
    tlen[i] = (size_t)snprintf(topics + i * 40, 40, "devices/%llu/telemetry/m%llu",
                               (unsigned long long)(r % (NDEV + NDEV / 4)), (unsigned long long)((r >> 40) % 16));
    tptr[i] = (const uint8_t*)topics + i * 40;
  }
  /* the word lists fold/4 is handed (split once, as the Erlang side passes them) */
  wcnt = (uint32_t*)calloc(NPUB, sizeof(uint32_t));
  woff = (size_t*)calloc(NPUB + 1, sizeof(size_t));
  wptr = (const uint8_t**)calloc(NPUB * 4, sizeof(*wptr));
  wlen = (size_t*)calloc(NPUB * 4, sizeof(size_t));
  size_t nw = 0;
  for (size_t i = 0; i < NPUB; i++) {
    woff[i] = nw;
    size_t st = 0;
    for (size_t j = 0; j <= tlen[i]; j++)
      if (j == tlen[i] || tptr[i][j] == '/') { wptr[nw] = tptr[i] + st; wlen[nw] = j - st; nw++; st = j + 1; }
    wcnt[i] = (uint32_t)(nw - woff[i]);
  }
  woff[NPUB] = nw;
  fprintf(stderr, "loaded %zu subscriptions in %.1fs\n", NDEV + NWILD, load_s);
  int rc = 0;
  if (want(argc, argv, "scale")) {
    const int threads_list[] = {1, 8, 16, 24, 32, 48};
    for (int mode = 0; mode < 2 && !rc; mode++)
      for (size_t ti = 0; ti < sizeof threads_list / sizeof threads_list[0] && !rc; ti++)
        rc = run("scale", threads_list[ti], 4096, mode, secs, NULL, NULL);
    /* the per-entry callback (the round-3 fold) beside it; bigger batches */
    fold_spans = 0;
    for (int mode = 0; mode < 2 && !rc; mode++) rc = run("scale", 16, 4096, mode, secs, NULL, NULL);
    fold_spans = 1;
    for (int mode = 0; mode < 2 && !rc; mode++)
      for (int T = 16; T <= 32 && !rc; T += 16) rc = run("scale", T, 16384, mode, secs, NULL, NULL);
  }
  if (want(argc, argv, "inflight")) {   /* three rounds in the kernels at once instead of two */
    vmqgb_view_set_inflight(view, 3);
    for (int mode = 0; mode < 2 && !rc; mode++)
      for (int T = 16; T <= 32 && !rc; T += 16) rc = run("inflight3", T, 4096, mode, secs, NULL, NULL);
    vmqgb_view_set_inflight(view, 2);
  }
  if (want(argc, argv, "devrec") && !rc) {
    vmqgb_view_set_device_records(view, 1);
    rc = run("devrec", 16, 4096, 0, secs, NULL, NULL);
    if (!rc) rc = run("devrec", 32, 4096, 0, secs, NULL, NULL);
    vmqgb_view_set_device_records(view, 0);
  }
  {
    /* "churn": the windowed applies; "churn1" (named only): one apply per event */
    for (int co = 0; co < 2 && !rc; co++)
      if (co == 1 ? want(argc, argv, "churn") : argc > 2 && want(argc, argv, "churn1"))
      for (int mode = 0; mode < 2 && !rc; mode++)
        for (int T = 16; T <= 32 && !rc; T += 16) {
          churn_t cc;
          memset(&cc, 0, sizeof cc);
          pthread_mutex_init(&cc.mu, NULL);
          cc.rate = 100000;
          cc.coalesce = co;
          cc.cap = 1u << 21;
          cc.q = (event_t*)malloc(cc.cap * sizeof(event_t));
          cc.lags_cap = 1u << 22;
          cc.lags = (double*)malloc(cc.lags_cap * sizeof(double));
          rc = run("churn", T, 4096, mode, secs, &cc, NULL);
          free(cc.q);
          free(cc.lags);
          /* resubscribe what the run left unsubscribed (the next run starts from the full set) */
          vmqgb_view_write_begin(view);
          for (uint32_t k = 0; k < 20000; k++) {
            char f[64];
            const int l = snprintf(f, sizeof f, "devices/%u/telemetry/#", k * 50);
            vmqgb_ops_add_filter(&ops, ctx, VMQG_OP_DEL, 0, (const uint8_t*)f, (size_t)l, 0, k * 50, (k * 50) % 3);
            vmqgb_ops_add_filter(&ops, ctx, VMQG_OP_ADD, 0, (const uint8_t*)f, (size_t)l, 0, k * 50, (k * 50) % 3);
          }
          if (vmqgb_view_apply_ops(view, &ops, NULL)) rc = 7;
          vmqgb_view_write_end(view);
        }
  }
  if (want(argc, argv, "load") && !rc) {
    for (int mode = 0; mode < 2 && !rc; mode++) {
      load_t ld;
      memset(&ld, 0, sizeof ld);
      rc = run("load", 16, 4096, mode, secs, NULL, &ld);
    }
  }
  fprintf(stderr, "checksum %llu\n", (unsigned long long)checksum);
  vmqgb_ops_free(&ops);
  vmqgb_view_free(view);
  vmqg_destroy(ctx);
  return rc;
}
