/*
 * vmqg_batch.h — the pure-C half of the vmq_reg_gpu_view NIF (vmqg_nif.c).
 *
 * Everything the NIF does besides converting Erlang terms lives here, in
 * plain C99 over the libvmqgpu C ABI (include/vmqg.h), so it is compiled and
 * tested without OTP (tests/test_nif_layer.py, tools/nif_harness.c):
 *
 *   - interners: Erlang terms (SubscriberId, SubInfo, node, mountpoint, group
 *     name — the NIF passes their external-term-format bytes) <-> dense
 *     uint32 ids, both directions;
 *   - publish batches: raw topics of concurrent fold/4 callers split by
 *     vmqg_prepare_publish (vmq_topic:validate_topic(publish, T),
 *     vmq_topic.erl:82-112) into one vmqg_pub / word-id batch;
 *   - matching with the overflow retry of vmqg_match_batch /
 *     vmqg_match_ranges (the output buffer grows to *out_n);
 *   - the fold: per publish, the FoldFun arguments in output order
 *     (vmq_reg_trie.erl:83, :97), from records or from ranges expanded over
 *     the record table (vmqg_records);
 *   - subscription ops: {Topic words, Node, SubscriberId, SubInfo} changes
 *     (deletes before adds, vmq_reg_trie.erl:245-248) -> vmqg_op batches.
 *
 *   - the view: the locking protocol the NIF runs fold/4 callers under
 *     (vmqgb_view_*), so that every batcher prepares its batch and folds its
 *     results in parallel — as vmq_reg_trie:fold/4 runs in every caller's
 *     process against read_concurrency tables (vmq_reg_trie.erl:59-66,
 *     136-137) — and only the device call is serialised.
 *
 * Threading: an interner or a batch is owned by one thread at a time.
 * vmqgb_batch_add only reads the context's dictionary (vmqg_prepare_publish),
 * so per-thread batches may be filled concurrently while no other call
 * modifies the context; vmqgb_batch_append merges them for one match call.
 * vmqgb_view: readers (a batch's prepare, device call and fold) share the
 * tables; a writer (vmqg_apply_ops, through vmqgb_view_apply) excludes them
 * and is not starved by them; device calls take turns.
 */
#ifndef VMQG_BATCH_H
#define VMQG_BATCH_H

#include <stddef.h>
#include <stdint.h>

#include "vmqg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- term <-> id --------------------------------------------------- */
typedef struct vmqgb_interner vmqgb_interner;

vmqgb_interner* vmqgb_interner_new(void);
void vmqgb_interner_free(vmqgb_interner* t);
/* id of `bytes`, created when new (ids are dense from 0) */
uint32_t vmqgb_intern(vmqgb_interner* t, const void* bytes, size_t len);
/* 0 and *id when present, -1 when not */
int vmqgb_lookup(const vmqgb_interner* t, const void* bytes, size_t len, uint32_t* id);
const uint8_t* vmqgb_bytes(const vmqgb_interner* t, uint32_t id, size_t* len);
uint32_t vmqgb_count(const vmqgb_interner* t);

/* ---- publish batches ------------------------------------------------ */
typedef struct vmqgb_batch {
  vmqg_pub* pubs;
  uint32_t* words;
  size_t n, cap, nwords, wcap;
  /* match output */
  uint64_t* offsets;    /* n + 1 */
  vmqg_emit* out;       /* records mode */
  size_t out_cap, out_n;
  vmqg_range* rng;      /* range mode */
  size_t rng_cap, rng_n;
  uint64_t epoch;       /* table epoch of the last match (vmqg_epoch): ranges index that epoch's records */
} vmqgb_batch;

int vmqgb_batch_init(vmqgb_batch* b, size_t cap_hint);
void vmqgb_batch_reset(vmqgb_batch* b);   /* keeps the buffers */
void vmqgb_batch_free(vmqgb_batch* b);
/* Adds one publish (raw topic bytes).  Returns its index in the batch, or a
 * negative VMQG_E_* (VMQG_E_INVAL: validate_topic rejects the topic). */
long vmqgb_batch_add(vmqgb_batch* b, vmqg_ctx* ctx, uint32_t mountpoint, const uint8_t* topic, size_t len);
/* Appends every publish of src (per-thread batches -> one match call). */
int vmqgb_batch_append(vmqgb_batch* dst, const vmqgb_batch* src);

/* vmqg_match_batch / vmqg_match_ranges with the output grown on
 * VMQG_E_OVERFLOW; the outputs stay in the batch. */
int vmqgb_match(vmqgb_batch* b, vmqg_ctx* ctx);
int vmqgb_match_ranges(vmqgb_batch* b, vmqg_ctx* ctx);

/* ---- the fold -------------------------------------------------------- */
/* One FoldFun argument: kind VMQG_EMIT_LOCAL {SubscriberId, SubInfo},
 * VMQG_EMIT_GROUP {Node, Group, SubscriberId, SubInfo}, VMQG_EMIT_REMOTE Node. */
typedef struct vmqgb_entry {
  uint32_t kind, node, group, subscriber, subinfo;
} vmqgb_entry;
/* return non-zero to stop the fold (returned by vmqgb_fold*) */
typedef int (*vmqgb_fold_fn)(void* acc, const vmqgb_entry* e);

size_t vmqgb_count_of(const vmqgb_batch* b, size_t i);   /* records mode: entries of publish i */
int vmqgb_fold(const vmqgb_batch* b, size_t i, vmqgb_fold_fn fn, void* acc);
/* range mode, expanded over the context's record table */
int vmqgb_fold_ranges(const vmqgb_batch* b, const vmqg_emit* recs, uint64_t nrecs, size_t i, vmqgb_fold_fn fn,
                      void* acc);

/* ---- subscription ops -------------------------------------------------- */
typedef struct vmqgb_ops {
  vmqg_op* ops;
  uint32_t* words;
  size_t n, cap, nwords, wcap;
} vmqgb_ops;

int vmqgb_ops_init(vmqgb_ops* o);
void vmqgb_ops_reset(vmqgb_ops* o);
void vmqgb_ops_free(vmqgb_ops* o);
/* One {Topic, SubInfo, Node} change of subscriber `sub`: kind VMQG_OP_ADD /
 * VMQG_OP_DEL; the topic as subscribed ("$share", Group prefix included),
 * its words interned into the context's dictionary. */
int vmqgb_ops_add(vmqgb_ops* o, vmqg_ctx* ctx, uint32_t kind, uint32_t mountpoint, const uint8_t* const* words,
                  const size_t* lens, uint32_t nwords, uint32_t node, uint32_t sub, uint32_t subinfo);
/* Splits a subscription filter on '/' (vmq_topic:validate_topic(subscribe,
 * T) has accepted it on the Erlang side) and adds it as above. */
int vmqgb_ops_add_filter(vmqgb_ops* o, vmqg_ctx* ctx, uint32_t kind, uint32_t mountpoint, const uint8_t* filter,
                         size_t len, uint32_t node, uint32_t sub, uint32_t subinfo);
int vmqgb_ops_apply(vmqgb_ops* o, vmqg_ctx* ctx, uint64_t* epoch);

/* ---- the view: concurrent batchers over one context ------------------- */
typedef struct vmqgb_view vmqgb_view;

vmqgb_view* vmqgb_view_new(vmqg_ctx* ctx);
void vmqgb_view_free(vmqgb_view* v);   /* does not destroy the context */
vmqg_ctx* vmqgb_view_ctx(vmqgb_view* v);
/* A batcher's critical section: read_begin, vmqgb_batch_add for each of its
 * publishes, vmqgb_view_match, the fold, read_end.  Any number of batchers
 * at once; vmqgb_view_match serialises only the device call. */
void vmqgb_view_read_begin(vmqgb_view* v);
void vmqgb_view_read_end(vmqgb_view* v);
/* Lets a waiting writer in and takes the read lock back: a batcher calls it
 * every VMQGB_YIELD_EVERY publishes while it prepares a batch, and while it
 * folds a records-mode batch (ids only ever grow, so what it prepared or
 * matched stays valid), so an apply waits for one slice of a batch, not for
 * every reader's whole batch. */
void vmqgb_view_yield(vmqgb_view* v);
#define VMQGB_YIELD_EVERY 512
/* Called under the read lock, returns under it: vmqgb_match or
 * vmqgb_match_ranges (ranges != 0) with the device to itself; in range mode
 * also the record table of the match's epoch (vmqg_records_at) for
 * vmqgb_fold_ranges.  In records mode the lock is let go while the batch
 * waits for the device (an apply may land between its prepare and its
 * match: word and term ids only ever grow); range mode keeps it, as its
 * entries index the host record table. */
int vmqgb_view_match(vmqgb_view* v, vmqgb_batch* b, int ranges, const vmqg_emit** recs, uint64_t* nrecs);
/* Table changes (vmqg_apply_ops, the term tables of the caller): writers;
 * write_begin takes the device mutex as well (after the table lock). */
void vmqgb_view_write_begin(vmqgb_view* v);
void vmqgb_view_write_end(vmqgb_view* v);
int vmqgb_view_apply(vmqgb_view* v, vmqgb_ops* o, uint64_t* epoch);   /* write_begin, apply, write_end */

#ifdef __cplusplus
}
#endif
#endif /* VMQG_BATCH_H */
