/* The reader / writer contract of include/vmqg.h (ABI 6) on a host-engine
 * context, no GPU: reader threads prepare word lists and pin the readers'
 * record table while one writer interns new words and applies changes that
 * rewrite records.  Checked:
 *   - a word the writer interned is, to every reader, either not there yet
 *     or there with its one id, and there for sure once the dictionary
 *     generation counts it (vmqg_dict_generation);
 *   - a record table pinned for epoch E (vmqg_records_pin) holds exactly the
 *     records of epoch E for a key the writer rewrites at every apply (its 64
 *     records all carry the SubInfo of that apply: no torn or mixed table),
 *     and stays so until unpinned while the writer keeps applying;
 *   - readers are never refused a pin of the current epoch;
 * then the view's writer-side calls beside each other (applies, some with a
 * failed commit, commit retries, stats polls): no change lost.
 * tests/test_nif_layer.py also runs it built with -fsanitize=thread.
 * Prints "ok" and exits 0; otherwise a message and non-zero. */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vmqg_batch.h"

#define NWORDS 40000
#define NSUB 64
#define SUB0 1000u

static vmqg_ctx* ctx;
static _Atomic int done;
static uint32_t expect_id[NWORDS];          /* written by the writer before it bumps `published` */
static volatile uint32_t published;          /* words whose ids are in expect_id */
static volatile uint64_t info_of_epoch[1u << 16];   /* the SubInfo the key's records carry at each epoch */
static uint64_t key_off = ~0ull;             /* the rewritten key's record range [key_off, +NSUB) */
static _Atomic int failed;
static uint64_t total_pins;

#define FAIL(...) do { fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); failed = 1; } while (0)

static int word_name(char* buf, uint32_t k) { return snprintf(buf, 32, "w%u", k); }

static void* writer(void* p) {
  (void)p;
  vmqgb_ops ops;
  vmqgb_ops_init(&ops);
  uint32_t k = 0, round = 0;
  while (!failed && k < NWORDS) {
    /* a few new words: subscriptions on them (interning is the writer's) */
    for (int j = 0; j < 64 && k < NWORDS; j++, k++) {
      char f[48];
      int l = snprintf(f, sizeof f, "n/");
      l += word_name(f + l, k);
      if (vmqgb_ops_add_filter(&ops, ctx, VMQG_OP_ADD, 0, (const uint8_t*)f, (size_t)l, 0, 5000 + k, 1)) {
        FAIL("add n/w%u", k);
        break;
      }
      expect_id[k] = ops.words[ops.nwords - 1];
    }
    /* the key x/# rewritten: every subscriber's SubInfo round -> round + 1 */
    for (uint32_t s = 0; s < NSUB; s++) {
      vmqgb_ops_add_filter(&ops, ctx, VMQG_OP_DEL, 0, (const uint8_t*)"x/#", 3, 0, SUB0 + s, round);
      vmqgb_ops_add_filter(&ops, ctx, VMQG_OP_ADD, 0, (const uint8_t*)"x/#", 3, 0, SUB0 + s, round + 1);
    }
    uint64_t e0 = 0, e = 0;
    vmqg_epoch(ctx, &e0);
    info_of_epoch[(e0 + 1) & 0xFFFF] = round + 1;   /* before the apply: readers may pin it at once */
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    if (vmqgb_ops_apply(&ops, ctx, &e) || e != e0 + 1) { FAIL("apply %u", round); break; }
    round++;
    __atomic_store_n(&published, k, __ATOMIC_RELEASE);
  }
  vmqgb_ops_free(&ops);
  done = 1;
  return NULL;
}

static void* reader(void* p) {
  const uintptr_t tid = (uintptr_t)p;
  uint64_t rng = 0x9E3779B97F4A7C15ull * (tid + 1);
  uint64_t pins = 0, refused = 0;
  while (!done && !failed) {
    /* dictionary: 16 publishes [n, w<j>] for random j among the published and just beyond */
    const uint32_t pub = __atomic_load_n(&published, __ATOMIC_ACQUIRE);
    char names[16][32];
    const uint8_t* wp[32];
    size_t wl[32];
    uint32_t mps[16], cnt[16], js[16];
    for (int i = 0; i < 16; i++) {
      rng = rng * 6364136223846793005ull + 1442695040888963407ull;
      js[i] = (uint32_t)((rng >> 33) % (pub + 64 < NWORDS ? pub + 64 : NWORDS));
      const int l = word_name(names[i], js[i]);
      wp[2 * i] = (const uint8_t*)"n"; wl[2 * i] = 1;
      wp[2 * i + 1] = (const uint8_t*)names[i]; wl[2 * i + 1] = (size_t)l;
      mps[i] = 0;
      cnt[i] = 2;
    }
    vmqg_pub P[16];
    uint32_t W[32];
    size_t nw = 0;
    if (vmqg_prepare_word_lists(ctx, 16, mps, cnt, wp, wl, P, W, 32, &nw) || nw != 32) { FAIL("prepare"); break; }
    for (int i = 0; i < 16; i++) {
      const uint32_t id = W[2 * i + 1], j = js[i];
      if (j < pub && id != expect_id[j]) FAIL("w%u: id %u, interned as %u", j, id, expect_id[j]);
      /* the writer makes a word findable, then counts it in the generation
       * (a reader that missed it read an older generation and prepares the
       * publish again): an id found now is inside the generation once that
       * store lands, a few instructions later */
      if (id != VMQG_WORD_UNKNOWN) {
        uint64_t g = vmqg_dict_generation(ctx);
        for (int spin = 0; g <= id && spin < (1 << 22); spin++) g = vmqg_dict_generation(ctx);
        if (g <= id) FAIL("w%u: id %u past the generation", j, id);
      }
    }
    /* records: pin the current epoch, check the key, keep the pin a while */
    uint64_t e = 0;
    vmqg_epoch(ctx, &e);
    const vmqg_emit* recs = NULL;
    uint64_t n = 0;
    uint32_t pin = 0;
    const int rc = vmqg_records_pin(ctx, e, &recs, &n, &pin);
    if (rc) { refused++; continue; }
    pins++;
    const uint64_t want = info_of_epoch[e & 0xFFFF];
    for (int pass = 0; pass < 3 && !failed; pass++) {
      uint32_t seen = 0;
      for (uint64_t r = key_off; r < key_off + NSUB && r < n; r++) {
        const vmqg_emit x = recs[r];
        if (x.subscriber >= SUB0 && x.subscriber < SUB0 + NSUB) {
          seen++;
          if (x.subinfo != want) FAIL("epoch %llu: record %llu has SubInfo %u, want %llu (pass %d)",
                                      (unsigned long long)e, (unsigned long long)r, x.subinfo,
                                      (unsigned long long)want, pass);
        }
      }
      if (seen != NSUB) FAIL("epoch %llu: %u of the key's records in its range", (unsigned long long)e, seen);
      for (volatile int spin = 0; spin < 20000; spin++) {}
    }
    vmqg_records_unpin(ctx, pin);
  }
  __atomic_fetch_add(&total_pins, pins, __ATOMIC_RELAXED);
  if (refused > pins / 2 + 16) FAIL("reader %lu: %llu refusals for %llu pins", (unsigned long)tid,
                                    (unsigned long long)refused, (unsigned long long)pins);
  return NULL;
}

/* phase 2: the view's writer-side entry points beside each other — applies
 * (some of whose commits are made to fail: fail_commits), commit retries and
 * stats polls (vmqgb_view_ctx_stats: writer mutex, then device mutex) */
static _Atomic int done2;
#define ROUNDS2 3000

static void* view_writer(void* p) {
  vmqgb_view* v = (vmqgb_view*)p;
  vmqgb_ops ops;
  vmqgb_ops_init(&ops);
  for (uint32_t r = 0; r < ROUNDS2 && !failed; r++) {
    char f[32];
    const int l = snprintf(f, sizeof f, "y/%u", r);
    if (r % 50 == 7 && vmqgb_view_set_option(v, "fail_commits", 1)) FAIL("set_option");
    vmqgb_view_write_begin(v);
    if (vmqgb_ops_add_filter(&ops, ctx, VMQG_OP_ADD, 0, (const uint8_t*)f, (size_t)l, 0, 9000 + r, 1)) FAIL("add y");
    const int rc = vmqgb_view_apply_ops(v, &ops, NULL);
    vmqgb_view_write_end(v);
    if (rc && rc != VMQG_E_DEVICE) FAIL("apply y/%u: %d", r, rc);
  }
  vmqgb_ops_free(&ops);
  done2 = 1;
  return NULL;
}

static void* view_committer(void* p) {
  vmqgb_view* v = (vmqgb_view*)p;
  while (!done2 && !failed) {
    const int rc = vmqgb_view_commit(v, NULL);
    if (rc && rc != VMQG_E_DEVICE) FAIL("commit: %d", rc);
  }
  return NULL;
}

static void* view_stats(void* p) {
  vmqgb_view* v = (vmqgb_view*)p;
  uint64_t last = 0;
  while (!done2 && !failed) {
    vmqg_stats_t st;
    if (vmqgb_view_ctx_stats(v, &st)) FAIL("stats");
    if (st.subs < last) FAIL("stats: subs went back %llu -> %llu", (unsigned long long)last, (unsigned long long)st.subs);
    last = st.subs;
  }
  return NULL;
}

int main(void) {
  vmqg_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.device = -1;
  cfg.max_nodes = VMQG_MAX_NODES;
  int err = 0;
  ctx = vmqg_create(&cfg, &err);
  if (!ctx) { fprintf(stderr, "vmqg_create: %d\n", err); return 2; }
  vmqgb_ops ops;
  vmqgb_ops_init(&ops);
  for (uint32_t s = 0; s < NSUB; s++)
    vmqgb_ops_add_filter(&ops, ctx, VMQG_OP_ADD, 0, (const uint8_t*)"x/#", 3, 0, SUB0 + s, 0);
  uint64_t e = 0;
  if (vmqgb_ops_apply(&ops, ctx, &e)) { fprintf(stderr, "load\n"); return 3; }
  info_of_epoch[e & 0xFFFF] = 0;
  if (vmqg_set_option(ctx, "reader_records", 1)) { fprintf(stderr, "reader_records\n"); return 4; }
  /* the key's range: where its records are now (rewrites stay in it: 64 in, 64 out) */
  const vmqg_emit* recs = NULL;
  uint64_t n = 0;
  if (vmqg_records(ctx, &recs, &n)) return 5;
  uint64_t lo = ~0ull, hi = 0;
  for (uint64_t r = 0; r < n; r++)
    if (recs[r].subscriber >= SUB0 && recs[r].subscriber < SUB0 + NSUB && recs[r].kind_node >> 24 == VMQG_EMIT_LOCAL) {
      if (r < lo) lo = r;
      if (r > hi) hi = r;
    }
  if (hi - lo + 1 != NSUB) { fprintf(stderr, "key range %llu..%llu\n", (unsigned long long)lo, (unsigned long long)hi); return 6; }
  key_off = lo;
  pthread_t w, rd[6];
  for (uintptr_t t = 0; t < 6; t++) pthread_create(&rd[t], NULL, reader, (void*)t);
  pthread_create(&w, NULL, writer, NULL);
  pthread_join(w, NULL);
  for (int t = 0; t < 6; t++) pthread_join(rd[t], NULL);
  if (!failed) {
    vmqgb_view* v = vmqgb_view_new(ctx);
    vmqg_stats_t s0, s1;
    if (!v || vmqgb_view_ctx_stats(v, &s0)) FAIL("view");
    pthread_t pw, pc, ps;
    pthread_create(&ps, NULL, view_stats, v);
    pthread_create(&pc, NULL, view_committer, v);
    pthread_create(&pw, NULL, view_writer, v);
    pthread_join(pw, NULL);
    pthread_join(pc, NULL);
    pthread_join(ps, NULL);
    if (vmqgb_view_commit(v, NULL)) FAIL("final commit");   /* a pending failed commit goes out */
    if (vmqgb_view_ctx_stats(v, &s1) || s1.subs != s0.subs + ROUNDS2)
      FAIL("view phase: subs %llu, want %llu", (unsigned long long)s1.subs, (unsigned long long)s0.subs + ROUNDS2);
    vmqgb_view_free(v);
  }
  vmqgb_ops_free(&ops);
  vmqg_destroy(ctx);
  if (failed) return 1;
  if (total_pins < 1000) { fprintf(stderr, "only %llu pins\n", (unsigned long long)total_pins); return 1; }
  printf("ok\n");
  return 0;
}
