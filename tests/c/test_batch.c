/* CPU unit test of the NIF's pure-C layer (integration/c_src/vmqg_batch.c)
 * over a host-engine-only libvmqgpu context (device -1: no GPU needed).
 * Prints "ok" and exits 0, or names the failed check. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vmqg_batch.h"

#define CHECK(c) do { if (!(c)) { printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)

static int collect(void* acc, const vmqgb_entry* e) {
  vmqgb_entry** p = (vmqgb_entry**)acc;
  **p = *e;
  (*p)++;
  return 0;
}

typedef struct { vmqgb_entry* p; int runs; } span_acc;
static int collect_span(void* accp, const vmqg_emit* r, size_t n) {
  span_acc* a = (span_acc*)accp;
  for (size_t j = 0; j < n; j++) {
    const vmqgb_entry e = {r[j].kind_node >> 24, r[j].kind_node & 0xFFFFFFu, r[j].group, r[j].subscriber, r[j].subinfo};
    *a->p++ = e;
  }
  a->runs++;
  return 0;
}

int main(void) {
  /* interner: dense ids, both directions, growth past the first table */
  vmqgb_interner* t = vmqgb_interner_new();
  CHECK(t);
  char buf[32];
  for (int i = 0; i < 5000; i++) {
    snprintf(buf, sizeof buf, "term-%d", i);
    CHECK(vmqgb_intern(t, buf, strlen(buf)) == (uint32_t)i);
  }
  CHECK(vmqgb_intern(t, "term-42", 7) == 42);
  CHECK(vmqgb_intern(t, "", 0) == 5000);          /* the empty binary is a term too */
  uint32_t id = 0;
  CHECK(vmqgb_lookup(t, "term-4999", 9, &id) == 0 && id == 4999);
  CHECK(vmqgb_lookup(t, "nope", 4, &id) == -1);
  size_t len = 0;
  const uint8_t* b = vmqgb_bytes(t, 1234, &len);
  CHECK(b && len == 9 && memcmp(b, "term-1234", 9) == 0);
  CHECK(vmqgb_count(t) == 5001);
  vmqgb_interner_free(t);

  /* a host-only context: ops through the layer, publishes prepared */
  vmqg_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.device = -1;
  int err = 0;
  vmqg_ctx* ctx = vmqg_create(&cfg, &err);
  CHECK(ctx && err == 0);
  vmqgb_ops ops;
  vmqgb_ops_init(&ops);
  CHECK(vmqgb_ops_add_filter(&ops, ctx, VMQG_OP_ADD, 0, (const uint8_t*)"a/+/c", 5, 0, 1, 0) == 0);
  CHECK(vmqgb_ops_add_filter(&ops, ctx, VMQG_OP_ADD, 0, (const uint8_t*)"a//c", 4, 0, 2, 1) == 0);
  CHECK(vmqgb_ops_add_filter(&ops, ctx, VMQG_OP_ADD, 0, (const uint8_t*)"$share/g/a/#", 12, 1, 3, 2) == 0);
  CHECK(ops.n == 3 && ops.ops[1].nwords == 3 && ops.ops[2].nwords == 4);
  CHECK(ops.words[ops.ops[0].word_off + 1] == VMQG_WORD_PLUS);
  CHECK(ops.words[ops.ops[2].word_off] == VMQG_WORD_SHARE);
  uint64_t epoch = 0;
  CHECK(vmqgb_ops_apply(&ops, ctx, &epoch) == 0 && epoch == 1 && ops.n == 0);
  vmqg_stats_t st;
  CHECK(vmqg_stats(ctx, &st) == 0 && st.subs == 3);

  vmqgb_batch b1, b2;
  CHECK(vmqgb_batch_init(&b1, 4) == 0 && vmqgb_batch_init(&b2, 4) == 0);
  CHECK(vmqgb_batch_add(&b1, ctx, 0, (const uint8_t*)"a/b/c", 5) == 0);
  CHECK(vmqgb_batch_add(&b1, ctx, 0, (const uint8_t*)"a/+/c", 5) == VMQG_E_INVAL);   /* no '+' in publish */
  CHECK(vmqgb_batch_add(&b1, ctx, 0, (const uint8_t*)"", 0) == VMQG_E_INVAL);
  CHECK(vmqgb_batch_add(&b2, ctx, 0, (const uint8_t*)"$SYS/x", 6) == 0);
  /* a topic with more words than the batch has room for grows the buffer */
  static uint8_t longt[4001];
  for (int i = 0; i < 4001; i++) longt[i] = (i % 2) ? '/' : 'a';
  CHECK(vmqgb_batch_add(&b2, ctx, 0, longt, 4001) == 1);
  CHECK(b2.pubs[1].nwords == 2001);
  CHECK(b1.n == 1 && b1.pubs[0].nwords == 3 && b1.words[1] == VMQG_WORD_UNKNOWN);
  CHECK(b2.pubs[0].flags == (VMQG_PUB_DOLLAR | VMQG_PUB_UNKNOWN));   /* "$SYS", "x": no filter has them */
  CHECK(b1.pubs[0].flags == VMQG_PUB_UNKNOWN && b1.n_unk == 1 && b2.n_unk == 1);   /* the long topic is all "a": known */
  CHECK(vmqgb_batch_append(&b1, &b2) == 0);
  CHECK(b1.n == 3 && b1.pubs[1].word_off == 3 && b1.pubs[2].word_off == 5 && b1.nwords == 3 + 2 + 2001);
  CHECK(b1.n_unk == 2 && b1.unk[3] == 1);   /* the appended batch's unknown publishes follow */

  /* the batched prepare agrees with the one-topic form, rejects per topic */
  {
    const char* ts[6] = {"a/b/c", "a//c", "a/+/c", "$SYS/x", "/a", "q/#"};
    const uint8_t* tp[6];
    size_t tl[6];
    uint32_t mps[6] = {0, 0, 0, 0, 3, 0};
    long idx[6];
    for (int i = 0; i < 6; i++) { tp[i] = (const uint8_t*)ts[i]; tl[i] = strlen(ts[i]); }
    vmqgb_batch bm, bs;
    CHECK(vmqgb_batch_init(&bm, 1) == 0 && vmqgb_batch_init(&bs, 1) == 0);
    CHECK(vmqgb_batch_add_many(&bm, ctx, 6, mps, tp, tl, idx) == 0);
    CHECK(idx[0] == 0 && idx[1] == 1 && idx[2] == VMQG_E_INVAL && idx[3] == 2 && idx[4] == 3 && idx[5] == VMQG_E_INVAL);
    for (int i = 0; i < 6; i++) if (idx[i] >= 0) CHECK(vmqgb_batch_add(&bs, ctx, mps[i], tp[i], tl[i]) >= 0);
    CHECK(bm.n == 4 && bs.n == 4 && bm.nwords == bs.nwords);
    CHECK(memcmp(bm.pubs, bs.pubs, 4 * sizeof(vmqg_pub)) == 0 && memcmp(bm.words, bs.words, bm.nwords * 4) == 0);
    CHECK(bm.pubs[1].flags == 0 && bm.pubs[3].mountpoint == 3 && bm.words[4] != VMQG_WORD_UNKNOWN);   /* "a//c" known */
    /* a word interned after the prepare: recheck finds it, updates the ids */
    CHECK(vmqgb_batch_recheck(&bm, ctx) == 0);
    CHECK(vmqgb_ops_add_filter(&ops, ctx, VMQG_OP_ADD, 0, (const uint8_t*)"a/b/#", 5, 0, 4, 0) == 0);
    CHECK(vmqgb_batch_recheck(&bm, ctx) == 1 && bm.words[1] != VMQG_WORD_UNKNOWN && !(bm.pubs[0].flags & VMQG_PUB_UNKNOWN));
    CHECK(vmqgb_batch_recheck(&bm, ctx) == 0);
    CHECK(vmqgb_ops_apply(&ops, ctx, &epoch) == 0 && epoch == 2);
    vmqgb_batch_free(&bm);
    vmqgb_batch_free(&bs);
  }
  /* the view on a host-only context: no pipeline, the device call refused */
  {
    vmqgb_view* v = vmqgb_view_new(ctx);
    CHECK(v != NULL);
    vmqgb_batch bv;
    CHECK(vmqgb_batch_init(&bv, 4) == 0);
    CHECK(vmqgb_batch_add(&bv, ctx, 0, (const uint8_t*)"a/b/c", 5) == 0);
    const vmqg_emit* r0 = NULL;
    uint64_t n0 = 0;
    CHECK(vmqgb_view_match(v, &bv, 0, NULL, NULL) == VMQG_E_DEVICE);
    CHECK(vmqgb_view_match(v, &bv, 1, &r0, &n0) == VMQG_E_DEVICE);
    vmqgb_view_release(v, &bv);
    vmqgb_view_stats vs;
    vmqgb_view_get_stats(v, &vs);
    CHECK(vs.rounds == 0);
    vmqgb_batch_free(&bv);
    vmqgb_view_free(v);
  }
  /* a host-only context refuses to match (no CPU fallback) */
  CHECK(vmqgb_match(&b1, ctx) == VMQG_E_DEVICE);
  CHECK(vmqgb_match_ranges(&b1, ctx) == VMQG_E_DEVICE);

  /* the fold over records / over ranges gives the same entries */
  const vmqg_emit recs[4] = {{(VMQG_EMIT_LOCAL << 24) | 0, VMQG_NONE, 10, 1},
                             {(VMQG_EMIT_LOCAL << 24) | 0, VMQG_NONE, 11, 2},
                             {(VMQG_EMIT_GROUP << 24) | 2, 77, 12, 0},
                             {(VMQG_EMIT_LOCAL << 24) | 0, VMQG_NONE, 13, 0}};
  b1.n = 2;
  b1.offsets = b1.offs_buf = (uint64_t*)realloc(b1.offs_buf, 3 * sizeof(uint64_t));
  b1.offsets[0] = 0; b1.offsets[1] = 3; b1.offsets[2] = 4;
  b1.out = (vmqg_emit*)realloc(b1.out, 4 * sizeof(vmqg_emit));
  b1.out[0] = recs[1]; b1.out[1] = recs[2]; b1.out[2] = (vmqg_emit){(VMQG_EMIT_REMOTE << 24) | 70, VMQG_NONE, VMQG_NONE, VMQG_NONE};
  b1.out[3] = recs[3];
  vmqgb_entry got[8], *p = got;
  CHECK(vmqgb_fold(&b1, 0, collect, &p) == 0 && p - got == 3);
  CHECK(got[0].kind == VMQG_EMIT_LOCAL && got[0].subscriber == 11 && got[0].subinfo == 2);
  CHECK(got[1].kind == VMQG_EMIT_GROUP && got[1].node == 2 && got[1].group == 77);
  CHECK(got[2].kind == VMQG_EMIT_REMOTE && got[2].node == 70);
  b1.rng = b1.rng_buf = (vmqg_range*)realloc(b1.rng_buf, 3 * sizeof(vmqg_range));
  b1.rng[0] = (vmqg_range){1, 2};    /* records 1, 2 */
  b1.rng[1] = (vmqg_range){70, 0};   /* remote node 70 */
  b1.rng[2] = (vmqg_range){3, 1};
  b1.offsets[0] = 0; b1.offsets[1] = 2; b1.offsets[2] = 3;
  vmqgb_entry got2[8], *q = got2;
  CHECK(vmqgb_fold_ranges(&b1, recs, 4, 0, collect, &q) == 0 && q - got2 == 3);
  CHECK(memcmp(got, got2, 3 * sizeof(vmqgb_entry)) == 0);
  q = got2;
  CHECK(vmqgb_fold_ranges(&b1, recs, 4, 1, collect, &q) == 0 && q - got2 == 1 && got2[0].subscriber == 13);
  CHECK(vmqgb_fold_ranges(&b1, recs, 3, 1, collect, &q) == VMQG_E_STATE);   /* range past the table */
  /* runs of records: the same entries in the same order, one call per range / per publish */
  vmqgb_entry got3[8];
  span_acc sa = {got3, 0};
  CHECK(vmqgb_fold_spans(&b1, 1, recs, 4, 0, collect_span, &sa) == 0 && sa.p - got3 == 3 && sa.runs == 2);
  CHECK(memcmp(got, got3, 3 * sizeof(vmqgb_entry)) == 0);
  sa.p = got3;
  CHECK(vmqgb_fold_spans(&b1, 1, recs, 3, 1, collect_span, &sa) == VMQG_E_STATE);
  b1.offsets[0] = 0; b1.offsets[1] = 3; b1.offsets[2] = 4;   /* records mode again */
  sa.p = got3; sa.runs = 0;
  CHECK(vmqgb_fold_spans(&b1, 0, NULL, 0, 0, collect_span, &sa) == 0 && sa.p - got3 == 3 && sa.runs == 1);
  CHECK(memcmp(got, got3, 3 * sizeof(vmqgb_entry)) == 0);
  CHECK(vmqgb_fold_spans(&b1, 0, NULL, 0, 2, collect_span, &sa) == VMQG_E_INVAL);
  vmqgb_batch_free(&b1);
  vmqgb_batch_free(&b2);
  vmqgb_ops_free(&ops);
  vmqg_destroy(ctx);
  printf("ok\n");
  return 0;
}
