/*
 * vmqr.h — C ABI of libvmqgpu's retained-message matcher: the MI355X
 * restatement of VerneMQ's retained store and its match_fold/4 (the
 * "which retained messages does this new subscription receive" query).
 *
 * Drop-in boundary (paths relative to the reference checkout):
 *   apps/vmq_server/src/vmq_retain_srv.erl:63-66   delete/2          -> vmqr_apply (VMQR_OP_DELETE)
 *   apps/vmq_server/src/vmq_retain_srv.erl:68-71   insert/3          -> vmqr_apply (VMQR_OP_INSERT)
 *   apps/vmq_server/src/vmq_retain_srv.erl:75-99   match_fold/4      -> vmqr_match_batch / _device
 *   apps/vmq_server/src/vmq_retain_srv.erl:101-113 stats/0           -> vmqr_stats
 *   apps/vmq_server/src/vmq_retain_srv.erl:129-138 init fold of the metadata store -> bulk vmqr_apply
 * Callers that stay unchanged: vmq_reg:publish/4 retain set/delete
 * (vmq_reg.erl:274-313), vmq_reg:deliver_retained/5 (:383-417, the FoldFun
 * builds the #vmq_msg{} and enqueues), vmq_retain_info (:40-58).
 *
 * Semantics reproduced exactly: the store is an ets set keyed {MP, Topic}
 * (insert replaces the value of an existing key); for a filter with a
 * wildcard (has_wildcard/1, :239-242: a '+' anywhere, or '#' as the LAST
 * word) match_fold folds over every entry of the same MP whose topic
 * satisfies vmq_topic:match/2 (vmq_topic.erl:53-65) — no '$' rule — and for
 * any other filter over the one entry with exactly that key.  The order in
 * which ets:foldl visits a set is unspecified, so a filter's matches are a
 * set (returned in an unspecified order).
 *
 * Payloads (#retain_msg{} records) stay with the caller: a retained entry
 * carries an opaque uint32 message id.  Mountpoints are dense uint32 ids;
 * topic words are interned by the context's own dictionary
 * (vmqr_intern_words) so retained topics and filters share one id space,
 * '+' and '#' being VMQG_WORD_PLUS / VMQG_WORD_HASH.
 *
 * Conventions as in vmqg.h: 0 / negative VMQG_E_* status, caller-owned
 * buffers, one context is not re-entrant, apply and match calls on one
 * context are ordered on its stream.
 */
#ifndef VMQR_H
#define VMQR_H

#include "vmqg.h"

#ifdef __cplusplus
extern "C" {
#endif

#define VMQR_OP_INSERT 1u   /* vmq_retain_srv:insert/3  (ets:insert, replaces) */
#define VMQR_OP_DELETE 2u   /* vmq_retain_srv:delete/2  (ets:delete)            */

typedef struct vmqr_config {
  int32_t device;            /* HIP device ordinal; -1 = host tables only        */
  uint32_t max_mountpoints;  /* initial range (0 = 1024): a retained topic on a mountpoint id past it grows it, up to VMQG_MAX_MOUNTPOINTS; VMQG_NONE in a filter matches nothing */
  uint64_t hint_topics;      /* sizing hint (retained entries); 0 = grow         */
} vmqr_config;

/* One retained-store mutation: {MP, Topic} (word ids in `words`) -> msg. */
typedef struct vmqr_op {
  uint32_t kind;        /* VMQR_OP_INSERT | VMQR_OP_DELETE                  */
  uint32_t mountpoint;
  uint32_t word_off;    /* index of the first word id in `words`            */
  uint32_t nwords;      /* >= 1                                             */
  uint32_t msg;         /* opaque message id (insert)                       */
  uint32_t reserved;
} vmqr_op;

typedef struct vmqr_stats_s {
  uint64_t retained;        /* ets:info(?RETAIN_CACHE, size)               */
  uint64_t device_bytes;    /* retained arena on the device                 */
  uint64_t partitions;      /* {MP, first word} row lists                   */
  uint64_t epoch;           /* apply batches applied                        */
  uint64_t rebuilds;        /* full re-layouts                              */
  uint64_t words;           /* interned words                               */
} vmqr_stats_t;

typedef struct vmqr_ctx vmqr_ctx;

vmqr_ctx* vmqr_create(const vmqr_config* cfg, int* err);
void vmqr_destroy(vmqr_ctx* ctx);

/* As vmqg_intern_words: create != 0 adds unseen words (retained topics),
 * create == 0 maps them to VMQG_WORD_UNKNOWN (filters). */
int vmqr_intern_words(vmqr_ctx* ctx, const uint8_t* bytes, const uint64_t* offs, uint32_t n, int create,
                      uint32_t* ids_out);

/* Applies inserts / deletes in order, then pushes the table patches to the
 * device (stream-ordered before later matches).  The batch is validated
 * first; an invalid op rejects the whole batch unchanged. */
int vmqr_apply(vmqr_ctx* ctx, const vmqr_op* ops, size_t n, const uint32_t* words, size_t nwords);

/* match_fold/4 for a batch of filters (vmqg_pub records: mountpoint, word
 * range; flags ignored).  offsets[0..n] delimits each filter's message ids
 * in out; total > out_cap returns VMQG_E_OVERFLOW with *out_n = total and
 * offsets valid.  Synchronous. */
int vmqr_match_batch(vmqr_ctx* ctx, const vmqg_pub* filters, size_t n, const uint32_t* words, size_t nwords,
                     uint32_t* out, size_t out_cap, size_t* out_n, uint64_t* offsets);

/* Device-buffer form (pointers on the context's device, work on `stream`,
 * NULL = the legacy default stream as in vmqg_match_device; no
 * synchronisation); errors latch for vmqr_match_status. */
int vmqr_match_device(vmqr_ctx* ctx, const vmqg_pub* d_filters, uint32_t n, const uint32_t* d_words,
                      uint32_t* d_out, uint64_t out_cap, uint64_t* d_offsets, void* stream);
int vmqr_match_status(vmqr_ctx* ctx, void* stream);

/* Streams: device calls take the caller's stream (NULL = the legacy default
 * stream).  The context orders its work across streams by recording an event
 * on the stream it last queued on when the next call comes on another one;
 * so a stream passed to any entry point must stay alive until the next call
 * on the context, or be released first with vmqr_release_stream (records that
 * event now; no-op if the context's last work is not on it). */
int vmqr_release_stream(vmqr_ctx* ctx, void* stream);

int vmqr_stats(vmqr_ctx* ctx, vmqr_stats_t* out);

/* Canonical dump of ?RETAIN_CACHE: one line "mp#M [w,...] -> msg#N" per
 * entry, sorted.  Owned by the context until its next call. */
int vmqr_dump(vmqr_ctx* ctx, const char** text, size_t* len);

/* Tuning knob (results unchanged): "walk_rows_hint" = rows of the flattened
 * walk the first look-back allocation covers (grown on demand: a batch that
 * walks more reports VMQG_E_FRONTIER once and succeeds when run again). */
int vmqr_set_option(vmqr_ctx* ctx, const char* name, int64_t value);

/* Average duration (ns) of the timed calls' kernels: count_ns = plan + filter
 * scan, emit_ns = the one-pass walk. */
int vmqr_set_timing(vmqr_ctx* ctx, int enable);
int vmqr_kernel_times(vmqr_ctx* ctx, double* count_ns, double* emit_ns, uint64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* VMQR_H */
