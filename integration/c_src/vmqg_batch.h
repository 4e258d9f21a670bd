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
 *   - the view: how the NIF runs fold/4 callers (vmqgb_view_*): every
 *     batcher prepares its batch and folds its results in parallel, without
 *     a lock and without waiting for writers — as vmq_reg_trie:fold/4 runs in
 *     every caller's process against read_concurrency tables with one writer
 *     (vmq_reg_trie.erl:59-66, 136-137) — and only device calls take turns.
 *
 * Threading: an interner or a batch is owned by one thread at a time.
 * vmqgb_batch_add* only reads the context's dictionary (a reader call of
 * include/vmqg.h, safe beside the one writer), so batches are filled
 * concurrently with each other and with table changes; vmqgb_batch_append
 * merges them for one match call.  vmqgb_view: batchers never take a lock
 * the writer holds; writers (interning, vmqgb_view_apply_ops) take turns on
 * the view's writer mutex; the host half of an apply runs beside the device
 * rounds, only its upload takes a turn at the device.
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
/* the same; *created = 1 when the key was not there (a new or reused id) */
uint32_t vmqgb_intern_ex(vmqgb_interner* t, const void* bytes, size_t len, int* created);
/* 0 and *id when present, -1 when not */
int vmqgb_lookup(const vmqgb_interner* t, const void* bytes, size_t len, uint32_t* id);
const uint8_t* vmqgb_bytes(const vmqgb_interner* t, uint32_t id, size_t* len);
uint32_t vmqgb_count(const vmqgb_interner* t);   /* ids handed out so far (a bound: reused ids count once) */
uint32_t vmqgb_live(const vmqgb_interner* t);    /* keys interned now */
/* Takes key `id` out (later interns of its bytes get another id); the id
 * stays reserved until vmqgb_interner_release makes it reusable — after the
 * readers that could still hold it are gone (the caller's grace period). */
int vmqgb_interner_remove(vmqgb_interner* t, uint32_t id);
int vmqgb_interner_release(vmqgb_interner* t, uint32_t id);

/* ---- publish batches ------------------------------------------------ */
typedef struct vmqgb_batch {
  vmqg_pub* pubs;
  uint32_t* words;
  size_t n, cap, nwords, wcap;
  /* match output: publish i's entries are out[offsets[i] .. offsets[i+1])
   * (records) or rng[...] (ranges).  offsets / rng may point into the view's
   * pipeline buffers after vmqgb_view_match (ranges mode) until
   * vmqgb_view_release or the batch's next match. */
  uint64_t* offsets;    /* n + 1 */
  vmqg_emit* out;       /* records mode (owned) */
  size_t out_cap, out_n;
  vmqg_range* rng;      /* range mode */
  size_t rng_cap, rng_n;
  uint64_t epoch;       /* table epoch the results are from (vmqg_epoch): ranges index that epoch's records */
  /* owned storage behind offsets / rng */
  uint64_t* offs_buf;
  size_t offs_cap;
  vmqg_range* rng_buf;
  /* publishes prepared with a word the dictionary did not know (VMQG_PUB_UNKNOWN):
   * their raw topics (or word lists), so they can be prepared again if the
   * dictionary grew before their match (vmqg_dict_generation) */
  uint64_t dict_gen;
  uint32_t* unk;        /* publish index, raw offset, raw length (| VMQGB_RAW_WORDS): 3 per entry */
  size_t n_unk, unk_cap;
  uint8_t* raw;
  size_t raw_n, raw_cap;
  void* lease;          /* the view pipeline round the outputs point into */
  uint32_t rec_pin;     /* range mode: the record table pinned for the fold (vmqg_records_pin) */
  int rec_pinned;
  uint32_t stale_rematches;   /* matches repeated because a publish's unknown word became known */
  unsigned lane;        /* the view context its matches go to (vmqgb_view_bind; 0: the primary) */
  int in_reader;        /* inside a reader section of the view (vmqgb_view_enter .. _release) */
  unsigned reader_era;
  int out_ranges;       /* set by vmqgb_view_match: 1 the results are ranges, 0 records (a
                           ranges request falls back to records when applies keep rewriting
                           the record slots its rounds index) */
} vmqgb_batch;

/* unk raw length flag: the raw bytes are a word list ({u32 len, bytes} per
 * word, len 0xFFFFFFFF for a non-binary element), not a topic to split */
#define VMQGB_RAW_WORDS 0x80000000u

int vmqgb_batch_init(vmqgb_batch* b, size_t cap_hint);
void vmqgb_batch_reset(vmqgb_batch* b);   /* keeps the buffers */
void vmqgb_batch_free(vmqgb_batch* b);
/* Adds one publish (raw topic bytes).  Returns its index in the batch, or a
 * negative VMQG_E_* (VMQG_E_INVAL: validate_topic rejects the topic). */
long vmqgb_batch_add(vmqgb_batch* b, vmqg_ctx* ctx, uint32_t mountpoint, const uint8_t* topic, size_t len);
/* Adds n publishes at once (vmqg_prepare_publishes: the dictionary probes of
 * a block of topics overlap).  idx_out[i] = index in the batch or a negative
 * VMQG_E_* for topic i, as vmqgb_batch_add.  Returns 0 or VMQG_E_NOMEM. */
int vmqgb_batch_add_many(vmqgb_batch* b, vmqg_ctx* ctx, size_t n, const uint32_t* mountpoints,
                         const uint8_t* const* topics, const size_t* lens, long* idx_out);
/* Adds n publishes given as Topic word lists, the form vmq_reg_trie:fold/4
 * takes (vmq_reg_trie.erl:59-66): publish i has counts[i] words (0 allowed),
 * word k of the call is words[k][0 .. lens[k]) — vmqg_prepare_word_lists, no
 * split, no validation.  lens[k] == VMQGB_NOT_BINARY marks a list element that
 * is not a binary: it equals no filter word (VMQG_WORD_UNKNOWN).  idx_out[i] =
 * index in the batch.  Returns 0 or VMQG_E_NOMEM (the batch unchanged). */
#define VMQGB_NOT_BINARY ((size_t)-1)
int vmqgb_batch_add_word_lists(vmqgb_batch* b, vmqg_ctx* ctx, size_t n, const uint32_t* mountpoints,
                               const uint32_t* counts, const uint8_t* const* words, const size_t* lens,
                               long* idx_out);
/* Appends every publish of src (per-thread batches -> one match call). */
int vmqgb_batch_append(vmqgb_batch* dst, const vmqgb_batch* src);
/* Prepares the publishes holding unknown words again if the dictionary grew
 * since they were prepared.  Returns 1 if a word id
 * changed (the batch must be matched again), 0 if not, or a VMQG_E_*. */
int vmqgb_batch_recheck(vmqgb_batch* b, vmqg_ctx* ctx);

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
/* The same FoldFun arguments in the same order, handed over as runs of
 * consecutive 16-B records (vmqg_emit: kind << 24 | node, group, subscriber,
 * subinfo): one call per publish in records mode, one per key range in range
 * mode (a remote node: a run of one record built on the stack).  `recs` /
 * `nrecs`: the record table of the batch's epoch in range mode, ignored in
 * records mode.  One indirect call per run instead of per entry. */
typedef int (*vmqgb_span_fn)(void* acc, const vmqg_emit* run, size_t n);
int vmqgb_fold_spans(const vmqgb_batch* b, int ranges, const vmqg_emit* recs, uint64_t nrecs, size_t i,
                     vmqgb_span_fn fn, void* acc);
/* Range mode: starts loading the first record of each of publish i's key
 * ranges (a publish's own subscribers sit at a random place of the record
 * table: one cache miss per range otherwise).  A fold loop calls it for
 * publish i + VMQGB_PREFETCH_AHEAD before folding publish i.  No-op in
 * records mode and past the batch. */
void vmqgb_prefetch_entries(const vmqgb_batch* b, int ranges, const vmqg_emit* recs, uint64_t nrecs, size_t i);
#define VMQGB_PREFETCH_AHEAD 16

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
void vmqgb_view_free(vmqgb_view* v);   /* does not destroy the contexts */
/* Multi-GPU (the trie replicated, publish batches spread over
 * the GPUs): a replica context (VMQG_CFG_REPLICA, any device) becomes one
 * more lane of the view.  It follows the primary after every commit
 * (vmqg_replica_follow: the commit's patches, or the whole image) under the
 * writer mutex, and batches bound to it (vmqgb_view_bind) are matched on it
 * — their rounds run beside the other lanes', each lane with its own device
 * mutex, queue and rounds; ranges index the primary's record table of the
 * same epoch.  Call before batchers start.  VMQG_E_STATE on a view without a
 * device, VMQG_E_LIMIT past VMQGB_MAX_LANES. */
int vmqgb_view_add_replica(vmqgb_view* v, vmqg_ctx* replica);
int vmqgb_view_lanes(vmqgb_view* v);
/* A batcher's batch bound to a lane, round robin over the lanes (the NIF
 * binds each batcher's batch once: one batcher per scheduler, so scheduler
 * k's publishes go to context k mod N). */
void vmqgb_view_bind(vmqgb_view* v, vmqgb_batch* b);
/* Grace periods.  A batcher's reader section runs from vmqgb_view_enter
 * (before its prepare: word ids are looked up there) to vmqgb_view_release
 * (after its fold: term ids are read there); vmqgb_view_match enters if the
 * batch has not.  Writer-side work that frees what readers may still hold —
 * the dictionary's retired words (vmqg_dict_release), the caller's terms
 * (its stage hook) — is deferred: vmqgb_view_defer(after_commit = 1) waits
 * for a commit that shipped the current stage to every lane, then for every
 * reader section open at that point to end; after_commit = 0 skips the
 * commit.  Deferred work runs in the writer (its mutex held): at applies,
 * commits, and vmqgb_view_reclaim.  The view itself queues the word release
 * after every commit. */
void vmqgb_view_enter(vmqgb_view* v, vmqgb_batch* b);
int vmqgb_view_defer(vmqgb_view* v, void (*fn)(void* arg, uint64_t u), void* arg, uint64_t u, int after_commit);
void vmqgb_view_reclaim(vmqgb_view* v);   /* writer mutex held */
/* fn(arg, v) after every stage that applied ops (writer mutex held, before
 * the commit): the NIF collects vmqg_released_ids there */
void vmqgb_view_set_stage_hook(vmqgb_view* v, void (*fn)(void* arg, vmqgb_view* v), void* arg);
void vmqgb_view_grace_stats(vmqgb_view* v, uint64_t* runs, int* waiting);
/* Device-arena digests of the lanes (out[k], k < n): tests check that every
 * replica's tables are the primary's byte for byte.  Takes each lane's
 * device mutex; call with the writer mutex held (between applies). */
int vmqgb_view_digests(vmqgb_view* v, uint64_t* out, int n);
vmqg_ctx* vmqgb_view_ctx(vmqgb_view* v);
/* A batcher's sequence: vmqgb_batch_add* for its publishes, vmqgb_view_match,
 * the fold, vmqgb_view_release.  Any number of batchers at once, no lock
 * held in between, alongside writers.
 *
 * The device side is a combining, pipelined submitter: a batcher queues its
 * prepared batch; whichever waiting batcher finds the pipeline free takes
 * every batch queued at that moment and matches them as ONE device call
 * (vmqg_hbatch_*: one H2D, one launch sequence, one D2H), then hands each
 * batch its slice.  Up to two such rounds (vmqgb_view_set_inflight) are in
 * the kernels at once and up to VMQGB_ROUNDS exist, so round k+1's inputs are
 * copied and matched while round k's results come back and round k-1's are
 * folded.  The device works in range mode ({record off, count} per key: 16 B
 * per config-C publish over PCIe instead of 1,040 B of records); a
 * records-mode batch is expanded from the readers' record table of its
 * round's epoch (vmqg_records_pin) into the batch's own buffer (byte-identical
 * to what the device would have copied; if two applies have rewritten record
 * slots since, the batch is matched again with device-side records). */
#define VMQGB_ROUNDS 6
#define VMQGB_MAX_LANES 16   /* device contexts of one view: the primary + replicas */
#define VMQGB_ROUND_MAX (1u << 17)   /* publishes per combined round */
/* The batch's results (offsets + out in records mode, offsets + rng in range
 * mode) — every publish's answer from the tables of one epoch, b->epoch —
 * and, in range mode, the record table of that epoch, pinned until
 * vmqgb_view_release, for vmqgb_fold_ranges / _spans.  If the dictionary grew
 * after the batch was prepared and a publish's unknown word is known now, the
 * batch is prepared and matched again (vmqgb_batch_recheck). */
int vmqgb_view_match(vmqgb_view* v, vmqgb_batch* b, int ranges, const vmqg_emit** recs, uint64_t* nrecs);
/* Ends the batch's use of the pipeline buffers its range-mode results point
 * into and of its pinned record table (also done by its next
 * vmqgb_view_match). */
void vmqgb_view_release(vmqgb_view* v, vmqgb_batch* b);
/* Table changes (the word dictionary, the caller's term tables, the apply):
 * writers, one at a time (write_begin / write_end: the view's writer mutex;
 * batchers never take it).  vmqgb_view_apply_ops stages the apply's host
 * half with no other lock (vmqg_apply_stage: matches keep running) and takes
 * the device mutex only for its upload (vmqg_apply_commit). */
void vmqgb_view_write_begin(vmqgb_view* v);
void vmqgb_view_write_end(vmqgb_view* v);
int vmqgb_view_apply_ops(vmqgb_view* v, vmqgb_ops* o, uint64_t* epoch);   /* inside write_begin/end */
int vmqgb_view_apply(vmqgb_view* v, vmqgb_ops* o, uint64_t* epoch);       /* write_begin, apply, write_end */
/* Retries a commit that failed (VMQG_E_DEVICE): the pending changes are
 * shipped as a whole image; 0 when nothing is pending. */
int vmqgb_view_commit(vmqgb_view* v, uint64_t* epoch);
/* vmqg_stats under the writer and the device mutex (the fields the writer
 * and the device calls update) */
int vmqgb_view_ctx_stats(vmqgb_view* v, vmqg_stats_t* out);
/* vmqg_set_option under both mutexes, on every lane's context; the batch
 * layer's own "force_pin_state" n (tests) makes the next n range-mode record
 * pins answer VMQG_E_STATE, so the ranges mode's fallback to device records
 * (after three refused pins) can be exercised */
int vmqgb_view_set_option(vmqgb_view* v, const char* name, int64_t value);
/* Knobs and counters of the submitter (tools/nif_harness.c reports them). */
void vmqgb_view_set_device_records(vmqgb_view* v, int on);   /* records over PCIe instead of host expansion */
void vmqgb_view_set_inflight(vmqgb_view* v, int n);          /* rounds in the kernels at once: 1..VMQGB_ROUNDS-1 (2) */
typedef struct vmqgb_view_stats {
  uint64_t rounds, round_publishes, round_batches, max_round_publishes;
  uint64_t expanded_batches, device_record_batches, state_retries, stale_rematches;
  uint64_t overflow_retries, ranges_fallbacks;
  uint64_t lane_rounds[VMQGB_MAX_LANES];   /* rounds per device context */
  uint64_t follow_ns, follow_failures;      /* replicas brought to each commit */
  /* the writer's applies (vmqgb_view_apply_ops): host stage, wait for the
   * device mutex, commit — sums and maxima, ns */
  uint64_t applies, stage_ns, stage_max_ns, dev_wait_ns, dev_wait_max_ns, commit_ns, commit_max_ns;
} vmqgb_view_stats;
void vmqgb_view_get_stats(vmqgb_view* v, vmqgb_view_stats* out);
void vmqgb_view_reset_stats(vmqgb_view* v);

#ifdef __cplusplus
}
#endif
#endif /* VMQG_BATCH_H */
