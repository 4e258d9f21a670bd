/*
 * vmqg.h — C ABI of libvmqgpu, the MI355X-native subscription matcher that
 * sits behind VerneMQ's `vmq_reg_view` behaviour.
 *
 * Drop-in boundary (all paths relative to the reference checkout):
 *   apps/vmq_server/src/vmq_reg_view.erl:20-27   -callback fold/4, fold/5
 *   apps/vmq_server/src/vmq_reg_trie.erl:59-98    fold/4 (what vmqg_match_* replaces)
 *   apps/vmq_server/src/vmq_reg_trie.erl:240-277  handle_event / handle_add_event /
 *                                                 handle_delete_event (what vmqg_apply_ops replaces)
 *   apps/vmq_server/src/vmq_reg_trie.erl:305-316  initialize_trie/2 (bulk vmqg_apply_ops)
 *   apps/vmq_server/src/vmq_reg_trie.erl:101-118  stats/0 (vmqg_stats)
 *
 * The Erlang side (a `vmq_reg_gpu_view` gen_server + erl_nif shim, see
 * INTEGRATION.md) keeps every Erlang term <-> integer id table: mountpoints,
 * nodes, SubscriberIds and SubInfos are opaque uint32 ids to this library.
 * Topic words are interned by the library's own dictionary (vmqg_intern_words)
 * so that subscription filters and publish topics share one id space.
 *
 * Conventions: every call returns 0 (VMQG_OK) or a negative VMQG_E_* code; no
 * exception crosses the ABI.  The caller owns every buffer; the library never
 * keeps a caller pointer after a call returns.  Separate contexts (one per
 * GPU) are independent.  vmqg_apply_ops and the match calls on one context
 * are ordered on the context's stream, so a match batch observes either all
 * or none of an apply batch (epoch semantics).
 *
 * Concurrency on one context (ABI 6; vmq_reg_trie's tables are read_concurrency
 * ETS with one writer, vmq_reg_trie.erl:136-137).  Three roles:
 *   readers  any number at once, never waiting, alongside everything below:
 *            vmqg_prepare_publish / _publishes / _word_lists,
 *            vmqg_intern_words with create = 0, vmqg_dict_generation,
 *            vmqg_records_pin / _unpin;
 *   writer   one at a time: vmqg_intern_words with create = 1 and
 *            vmqg_apply_stage — these run alongside the readers and alongside
 *            device calls;
 *   device   one at a time (the caller's lock): the match calls, the hbatch
 *            calls, vmqg_apply_commit, vmqg_match_status, the option and
 *            timing calls.
 * vmqg_apply_ops (stage + commit) is both writer and device.  Any other call
 * (stats, dump, replica calls) wants the context to itself.
 */
#ifndef VMQG_H
#define VMQG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VMQG_ABI_VERSION 7

/* ---- status codes ---------------------------------------------------- */
#define VMQG_OK 0
#define VMQG_E_INVAL (-1)     /* malformed argument / op                      */
#define VMQG_E_OVERFLOW (-2)  /* output buffer too small: *out_n = required    */
#define VMQG_E_NOMEM (-3)     /* host or device allocation failed             */
#define VMQG_E_DEVICE (-4)    /* no device / HIP runtime error                */
#define VMQG_E_FRONTIER (-5)  /* a publish exceeded the device scratch (internal; vmqg_match_batch /
                                 vmqg_match_ranges retry with a larger stack) */
#define VMQG_E_LIMIT (-6)     /* a configured limit (nodes, mountpoints, ids)  */
#define VMQG_E_STATE (-7)     /* call not valid for this context kind          */

/* ---- reserved ids ---------------------------------------------------- */
#define VMQG_WORD_PLUS 0u       /* <<"+">>      */
#define VMQG_WORD_HASH 1u       /* <<"#">>      */
#define VMQG_WORD_SHARE 2u      /* <<"$share">> */
#define VMQG_WORD_UNKNOWN 0xFFFFFFFFu  /* publish word never seen in a filter */
#define VMQG_NONE 0xFFFFFFFFu

#define VMQG_MAX_NODES 4096u    /* cluster nodes (vmq_trie_remote_subs / node lists are unbounded in
                                   the reference; 4,096 is this library's node-id space)            */
#define VMQG_MAX_MOUNTPOINTS (1u << 24)   /* mountpoint ids: the roots grow on demand up to this many
                                            (vmq_reg_trie has no limit: a mountpoint is part of every
                                            key, vmq_reg_trie.erl:60, 279-281, 320)                  */

/* ---- configuration --------------------------------------------------- */
#define VMQG_CFG_REPLICA 1u     /* no host engine: device tables arrive as
                                   images/patches from a primary context */

typedef struct vmqg_config {
  int32_t device;            /* HIP device ordinal; -1 = host engine only     */
  uint32_t local_node;       /* node id that plays node() (< max_nodes)       */
  uint32_t max_nodes;        /* <= VMQG_MAX_NODES (0 = VMQG_MAX_NODES)        */
  uint32_t max_mountpoints;  /* initial root range (0 = 1024): mountpoint ids  */
                             /* are dense; an op on an id past the range grows */
                             /* it (a re-layout), up to VMQG_MAX_MOUNTPOINTS;  */
                             /* a publish on VMQG_NONE (an unknown mountpoint) */
                             /* matches nothing                                */
  uint32_t flags;            /* VMQG_CFG_*                                    */
  uint32_t reserved;
  uint64_t hint_edges;       /* sizing hints; 0 = small defaults, tables grow */
  uint64_t hint_paths;
  uint64_t hint_keys;
  uint64_t hint_records;
  uint64_t hint_exact;
} vmqg_config;

/* ---- subscription deltas --------------------------------------------- */
#define VMQG_OP_ADD 1u   /* handle_add_event/2     vmq_reg_trie.erl:253-264 */
#define VMQG_OP_DEL 2u   /* handle_delete_event/2  vmq_reg_trie.erl:266-277 */

/* One {Topic, SubInfo, Node} of a vmq_subscriber change list, in the order
 * vmq_subscriber:fold/3 visits it (vmq_subscriber.erl:184-196): all deletes
 * of an event before its adds (vmq_reg_trie.erl:245-248).  The topic is the
 * word-id list exactly as subscribed, "$share"/Group prefix included. */
typedef struct vmqg_op {
  uint32_t kind;        /* VMQG_OP_ADD | VMQG_OP_DEL                        */
  uint32_t mountpoint;  /* MP of the SubscriberId                           */
  uint32_t word_off;    /* index of the first word id in `words`            */
  uint32_t nwords;      /* >= 1                                             */
  uint32_t node;        /* node the subscription lives on                   */
  uint32_t subscriber;  /* SubscriberId id (opaque)                         */
  uint32_t subinfo;     /* SubInfo id (opaque)                              */
  uint32_t reserved;
} vmqg_op;

/* ---- publishes and matches ------------------------------------------- */
#define VMQG_PUB_DOLLAR 1u   /* first topic word starts with '$' (MQTT-4.7.2-1) */
#define VMQG_PUB_UNKNOWN 2u  /* set by vmqg_prepare_publish*: a word was not in the dictionary
                                (VMQG_WORD_UNKNOWN); ignored by the match */

typedef struct vmqg_pub {
  uint32_t mountpoint;
  uint32_t word_off;    /* index of the first word id in `words`            */
  uint32_t nwords;      /* >= 0: fold/4 answers an empty Topic list too       */
  uint32_t flags;       /* VMQG_PUB_*                                       */
} vmqg_pub;
/* Word ids of a publish are looked up, not validated: VMQG_WORD_PLUS /
 * VMQG_WORD_HASH in a publish are the literal words "+" / "#", matched as
 * vmq_reg_trie:trie_match/4 matches them (the W probe of [W, <<"+">>] takes
 * the "+" edge, so a "+" word walks it twice, vmq_reg_trie.erl:366-375), and
 * the `{Topic, node()}` candidate finds a wildcard filter's own local key
 * (:62, :257-260).  VMQG_WORD_UNKNOWN matches only "+" and "#" edges. */

#define VMQG_EMIT_LOCAL 1u   /* {SubscriberId, SubInfo}               */
#define VMQG_EMIT_GROUP 2u   /* {Node, Group, SubscriberId, SubInfo}  */
#define VMQG_EMIT_REMOTE 3u  /* Node                                  */

/* One FoldFun argument (vmq_reg_trie.erl:83, :97).  16 bytes. */
typedef struct vmqg_emit {
  uint32_t kind_node;   /* kind << 24 | node                               */
  uint32_t group;       /* group word id (kind 2) else VMQG_NONE           */
  uint32_t subscriber;  /* kinds 1, 2                                      */
  uint32_t subinfo;     /* kinds 1, 2                                      */
} vmqg_emit;

typedef struct vmqg_stats_s {
  uint64_t subs;            /* NrOfSubs + NrOfRemoteSubs (vmq_reg_trie.erl:101-112) */
  uint64_t device_bytes;    /* device arena size (router_memory analogue)   */
  uint64_t trie_edges;      /* |vmq_trie|                                   */
  uint64_t trie_nodes;      /* |vmq_trie_node|                              */
  uint64_t trie_topics;     /* |vmq_trie_topic|                             */
  uint64_t subs_objects;    /* |vmq_trie_subs|                              */
  uint64_t fanout_objects;  /* |vmq_trie_subs_fanout|                       */
  uint64_t remote_keys;     /* |vmq_trie_remote_subs|                       */
  uint64_t epoch;           /* apply batches applied                        */
  uint64_t rebuilds;        /* full device-image rebuilds                   */
  uint64_t paths;           /* interned trie paths (host)                   */
  uint64_t words;           /* interned words                               */
  uint64_t deferred_tier1;  /* publishes of the last checked match batch walked */
  uint64_t deferred_tier2;  /* by a whole wave (LDS stack) / of those, again with a global stack */
  uint64_t ops_applied;     /* vmqg_apply_ops: ops applied so far               */
  uint64_t apply_host_ns;   /*   time inside vmqg_apply_ops, of which:           */
  uint64_t apply_upload_ns; /*   staging + enqueueing the patches, of which:      */
  uint64_t apply_wait_ns;   /*   waiting for a staging buffer (back-pressure:     */
                            /*   the host ran 4 batches ahead of the GPU)        */
  uint64_t patch_bytes;     /*   patch bytes shipped to the device               */
  uint64_t image_bytes;     /*   full-image bytes shipped (re-layouts)           */
  uint64_t max_depth;       /* deepest trie path (levels)                       */
  /* ABI 3: how the last checked match batch was served                        */
  uint64_t many_key;        /* wide publishes: more keys than the spill slots   */
                            /* hold, written wave-wide by the EMIT tail launch  */
                            /* from their candidates (no walk)                  */
  uint64_t retried;         /* publishes the one-lane fast pass could not hold, */
                            /* retried four lanes per publish (the rest of them */
                            /* are the deferred_tier1 walks)                    */
  uint64_t wave_entries;    /* entries (records or ranges) written by the EMIT  */
                            /* wave-tier launch (the whole-wave walks)          */
  uint64_t wide_entries;    /* entries the EMIT tail wrote for wide publishes    */
  /* ABI 4: batch-wide dedupe of the last checked match batch                   */
  uint64_t dedup;           /* publishes whose (MP, topic) another publish of   */
                            /* the batch walked: listed as its duplicates       */
  uint64_t dedup_walked;    /* of those, walked after all (representative       */
                            /* deferred, or a fingerprint collision)            */
  uint64_t error_bits;      /* device error bits the last check collected: 2 a  */
                            /* frontier stack overflowed or none was free, 4    */
                            /* output overflow, 8 count mismatch, 16 look-back  */
  /* ABI 6: the readers' record buffers (vmqg_records_pin)                       */
  uint64_t reader_waits;    /* stages that waited for readers to leave a buffer */
  uint64_t reader_wait_ns;  /*   ... and how long in all                         */
  /* ABI 7: reclamation (the host tables follow the live set, as ETS does)      */
  uint64_t keys;            /* live subscriber-list keys (`paths`: live paths)   */
  uint64_t topics;          /* live (MP, Topic) terms                           */
  uint64_t words_retired;   /* words nothing holds, awaiting vmqg_dict_release  */
  uint64_t words_released;  /* words dropped by vmqg_dict_release so far         */
  uint64_t host_bytes;      /* the engine's tables on the host: mirror, path /   */
                            /* key / topic arrays, indexes, dictionary, readers' */
                            /* record copies (not the per-key value lists)       */
} vmqg_stats_t;

/* ---- lifecycle ------------------------------------------------------- */
typedef struct vmqg_ctx vmqg_ctx;

int vmqg_abi_version(void);

/* "vmqg-build:<16 hex>": sha256 of the sources and flags the library was
 * compiled from (profiles/ summaries carry it; bench.py compares them). */
const char* vmqg_build_id(void);

/* Creates a context.  With cfg->device >= 0 the device arena is allocated on
 * that HIP device; device = -1 gives a host-engine-only context (tables are
 * maintained and can be dumped, every match call returns VMQG_E_DEVICE).
 * *err receives the status when NULL is returned.
 *   Replaces: vmq_reg_trie:start_link/0 + init/1 (vmq_reg_trie.erl:56-57, 135-151). */
vmqg_ctx* vmqg_create(const vmqg_config* cfg, int* err);
void vmqg_destroy(vmqg_ctx* ctx);

/* ---- words ------------------------------------------------------------ */
/* Interns n words (word i = bytes[offs[i] .. offs[i+1])).  create != 0 adds
 * unseen words (subscription filters); create == 0 maps unseen words to
 * VMQG_WORD_UNKNOWN (publish topics).  "+", "#", "$share" always map to the
 * reserved ids. */
int vmqg_intern_words(vmqg_ctx* ctx, const uint8_t* bytes, const uint64_t* offs, uint32_t n,
                      int create, uint32_t* ids_out);

/* Splits a publish topic by vmq_topic:validate_topic(publish, T)
 * (vmq_topic.erl:82-112) and looks its words up.  Writes at most cap word ids
 * to words_out and fills *pub (word_off = 0, flags = VMQG_PUB_DOLLAR when the
 * first word starts with '$').  Returns VMQG_E_INVAL for a topic the
 * reference rejects. */
int vmqg_prepare_publish(vmqg_ctx* ctx, uint32_t mountpoint, const uint8_t* topic, size_t len,
                         uint32_t* words_out, uint32_t cap, vmqg_pub* pub);

/* Batched vmqg_prepare_publish (ABI 4): n topics at once, their dictionary
 * probes software-pipelined (a block of topics' lookups is prefetched before
 * any is resolved) — the per-publish host cost of a fold/4 batch.  Topic i is
 * topics[i][0 .. lens[i]) of mountpoint mountpoints[i].  rc_out[i] = 0 or
 * VMQG_E_INVAL (validate_topic rejects it: pubs_out[i] is zeroed and it has no
 * words); pubs_out[i].word_off indexes words_out.  A topic of len bytes has at
 * most len + 1 words: with wcap >= sum(lens[i] + 1) the call cannot overflow;
 * otherwise it may return VMQG_E_OVERFLOW (outputs undefined).  *nwords_out =
 * word ids written.  Same read-only contract as vmqg_prepare_publish. */
int vmqg_prepare_publishes(vmqg_ctx* ctx, size_t n, const uint32_t* mountpoints, const uint8_t* const* topics,
                           const size_t* lens, vmqg_pub* pubs_out, int32_t* rc_out, uint32_t* words_out,
                           size_t wcap, size_t* nwords_out);

/* Publishes given as Topic word lists, the form vmq_reg_trie:fold/4 takes
 * (vmq_reg_trie.erl:59-66; plugin publishes reach it unvalidated,
 * vmq_reg.erl:572-594): no split, no validation.  Publish i has counts[i]
 * words (0 allowed); word k of the batch is words[k][0 .. lens[k]), in
 * publish order.  Each word is one dictionary lookup: "+" / "#" give their
 * reserved ids, a word no filter has (one holding a '/', say) gives
 * VMQG_WORD_UNKNOWN.  flags: VMQG_PUB_DOLLAR when the first word starts with
 * '$', VMQG_PUB_UNKNOWN as vmqg_prepare_publishes.  words_out receives
 * sum(counts) ids (VMQG_E_OVERFLOW if wcap is smaller); pubs_out[i].word_off
 * indexes it.  Same read-only contract as vmqg_prepare_publish (ABI 5). */
int vmqg_prepare_word_lists(vmqg_ctx* ctx, size_t n, const uint32_t* mountpoints, const uint32_t* counts,
                            const uint8_t* const* words, const size_t* lens, vmqg_pub* pubs_out,
                            uint32_t* words_out, size_t wcap, size_t* nwords_out);

/* ---- reclamation (ABI 7) ---------------------------------------------
 * vmq_reg_trie's tables hold only what live subscriptions need (rows are
 * deleted with their last value, vmq_reg_trie.erl:417-441, 472-539).  Here a
 * trie path, an (MP, Topic) term and a subscriber-list key nothing holds any
 * more are dropped at the end of the stage that emptied them (their ids
 * reused).  Two kinds of ids are shared with the caller's readers and are
 * released only through the caller's grace periods:
 *   words          a word no path, topic or $share key holds is retired at the
 *                  stage end; vmqg_dict_grace_token (a writer call) takes a
 *                  token, and once every reader that was running then has
 *                  finished — every vmqg_prepare_* / vmqg_intern_words lookup
 *                  call, and every publish prepared before it is matched and
 *                  folded — vmqg_dict_release(token) drops the words retired
 *                  before the token (their ids reusable).  Without release
 *                  calls no word is dropped.
 *   SubscriberId / SubInfo ids (the caller's): vmqg_released_ids lists those
 *                  the last stage's ops named, or whose last record it
 *                  removed, that no record holds now (kind 0 subscribers, 1
 *                  SubInfos; valid until the next stage).  The caller drops
 *                  their terms once matches of earlier epochs are folded. */
uint64_t vmqg_dict_grace_token(vmqg_ctx* ctx);
int vmqg_dict_release(vmqg_ctx* ctx, uint64_t token);
int vmqg_released_ids(vmqg_ctx* ctx, uint32_t kind, const uint32_t** ids, size_t* n);

/* Words interned so far: grows whenever a filter brings a new word.  A
 * publish prepared with VMQG_PUB_UNKNOWN before the dictionary grew may name
 * a word that has subscriptions now, so it must be prepared again before it
 * is matched on newer tables (integration/c_src/vmqg_batch.c does).  Safe to
 * call concurrently with writers (an atomic read). */
uint64_t vmqg_dict_generation(vmqg_ctx* ctx);

/* ---- deltas --------------------------------------------------------- */
/* Applies a batch of subscribe/unsubscribe ops with the exact semantics of
 * vmq_reg_trie's event handlers, including the reference's structural
 * behaviour under churn, then pushes the resulting
 * table patches to the device (stream-ordered before later matches).  The
 * batch is validated first; an invalid op rejects the whole batch unchanged.
 *   Replaces: handle_event/2 (vmq_reg_trie.erl:240-277), initialize_trie/2 (:305-316). */
int vmqg_apply_ops(vmqg_ctx* ctx, const vmqg_op* ops, size_t n, const uint32_t* words,
                   size_t nwords, uint64_t* epoch_out);

/* vmqg_apply_ops in its two halves (ABI 6), so that the host work of an apply
 * does not hold up matching:
 *   vmqg_apply_stage   the host half (the state machine, the host mirror, the
 *                      patch list, the readers' record buffer): a writer call,
 *                      run while match calls are queued and running (they
 *                      read only the device tables); VMQG_E_STATE if the
 *                      previous stage is not committed yet.  A rejected batch
 *                      (validation) stages nothing.
 *   vmqg_apply_commit  the device half: ships the staged patches (or image)
 *                      on the context stream; matches queued after it see the
 *                      new tables, *epoch_out = their epoch.  A device call.
 *                      No-op when nothing is staged.  If the upload fails
 *                      (VMQG_E_DEVICE / VMQG_E_NOMEM) the stage stays pending:
 *                      the epoch does not move, matches keep answering from
 *                      the tables the device holds, the next commit (retry)
 *                      ships the whole image, and a further vmqg_apply_stage
 *                      adds to the pending one instead of returning
 *                      VMQG_E_STATE — no change is lost. */
int vmqg_apply_stage(vmqg_ctx* ctx, const vmqg_op* ops, size_t n, const uint32_t* words, size_t nwords);
int vmqg_apply_commit(vmqg_ctx* ctx, uint64_t* epoch_out);

/* ---- matching -------------------------------------------------------- */
/* Host-buffer match of npub publishes.  offsets[0..npub] receives the
 * exclusive prefix of per-publish emission counts (offsets[npub] = total);
 * publish i's emissions are out[offsets[i] .. offsets[i+1]).  If total >
 * out_cap, returns VMQG_E_OVERFLOW with *out_n = total (offsets valid).
 * Synchronous.  Emission multiset per publish == vmq_reg_trie:fold/4's.
 *   Replaces: vmq_reg_trie:fold/4 (vmq_reg_trie.erl:59-98) for a batch. */
int vmqg_match_batch(vmqg_ctx* ctx, const vmqg_pub* pubs, size_t npub, const uint32_t* words,
                     size_t nwords, vmqg_emit* out, size_t out_cap, size_t* out_n,
                     uint64_t* offsets);

/* Device-buffer match: every pointer is device memory of the context's
 * device; work is enqueued on `stream` (a hipStream_t; NULL = the legacy
 * default stream itself, hipStreamLegacy, so a caller on the default stream
 * needs no extra synchronisation) and the call returns without
 * synchronising.  Table changes (patches, images) queued on any
 * stream land before the match.  d_offsets needs
 * npub + 1 entries.  Overflow / scratch errors are latched on the device and
 * reported by the next vmqg_match_status(). */
int vmqg_match_device(vmqg_ctx* ctx, const vmqg_pub* d_pubs, uint32_t npub,
                      const uint32_t* d_words, vmqg_emit* d_out, uint64_t out_cap,
                      uint64_t* d_offsets, void* stream);

/* Synchronises `stream` (NULL = the legacy default stream), after the
 * match calls queued on any stream, and returns the status latched by every
 * vmqg_match_device / vmqg_match_ranges_device call since the previous
 * vmqg_match_status (VMQG_OK, VMQG_E_OVERFLOW, VMQG_E_FRONTIER,
 * VMQG_E_DEVICE), then clears it: an error of any call in a pipelined
 * sequence is reported, not only the last call's. */
int vmqg_match_status(vmqg_ctx* ctx, void* stream);

/* Streams: device calls take the caller's stream (NULL = the legacy default
 * stream).  The context orders its work across streams by recording an event
 * on the stream it last queued on when the next call comes on another one;
 * so a stream passed to any entry point must stay alive until the next call
 * on the context, or be released first with vmqg_release_stream (records that
 * event now; no-op if the context's last work is not on it). */
int vmqg_release_stream(vmqg_ctx* ctx, void* stream);

/* ---- range mode ------------------------------------------------------ */
/* Range-mode matching returns, instead of copies of the records, one 8-byte
 * entry per non-empty subscriber-list key (`lookup_subs/1`,
 * vmq_reg_trie.erl:87-94) and per remote node: count > 0 — the records
 * [off, off + count) of the context's record table (vmqg_records); count ==
 * 0 — the remote node `off` (kind C, once per publish as fold_/5 :78-84).
 * Expanding the ranges in order gives the same emission multiset as
 * vmqg_match_batch; a publish with 65 emissions in config C is 2 entries.
 *   Replaces: vmq_reg_trie:fold/4 (:59-98) for a batch, FoldFun-side expansion. */
typedef struct vmqg_range {
  uint32_t off;    /* record index, or node id when count == 0 */
  uint32_t count;
} vmqg_range;

/* Host-buffer range match: offsets[0..npub] = exclusive prefix of the
 * per-publish entry counts; VMQG_E_OVERFLOW with *out_n = total when
 * out_cap is too small.  Synchronous. */
int vmqg_match_ranges(vmqg_ctx* ctx, const vmqg_pub* pubs, size_t npub, const uint32_t* words,
                      size_t nwords, vmqg_range* out, size_t out_cap, size_t* out_n,
                      uint64_t* offsets);

/* Device-buffer range match (as vmqg_match_device). */
int vmqg_match_ranges_device(vmqg_ctx* ctx, const vmqg_pub* d_pubs, uint32_t npub,
                             const uint32_t* d_words, vmqg_range* d_out, uint64_t out_cap,
                             uint64_t* d_offsets, void* stream);

/* Host view of the record table the ranges index (the host mirror of the
 * device arena's records, byte-identical at the last vmqg_apply_ops).  Valid
 * until the next vmqg_apply_ops on the context; primary contexts only. */
int vmqg_records(vmqg_ctx* ctx, const vmqg_emit** recs, uint64_t* n);

/* Epoch-safe expansion (ABI 3).  vmqg_epoch: the table epoch a match queued
 * now sees (the number of vmqg_apply_ops batches applied; a device match is
 * stream-ordered after every apply made before it is queued, and before every
 * apply made after).  vmqg_records_at: the record table for range results
 * of `epoch` — VMQG_E_STATE when a later vmqg_apply_ops has rewritten a
 * record slot or re-laid out the arena, so the ranges could index changed
 * records (lookup_subs/1 never returns a stale list, vmq_reg_trie.erl:87-94):
 * the caller matches again.  Appends to fresh slots are conservative
 * refusals too. */
int vmqg_epoch(vmqg_ctx* ctx, uint64_t* epoch);
int vmqg_records_at(vmqg_ctx* ctx, uint64_t epoch, const vmqg_emit** recs, uint64_t* n);

/* Concurrent expansion (ABI 6): readers' copies of the record table, kept by
 * vmqg_apply_stage once vmqg_set_option(ctx, "reader_records", 1) turned them
 * on (primary contexts).  vmqg_records_pin returns a record table valid for
 * range results of `epoch` and a pin that keeps it unchanged until
 * vmqg_records_unpin; never waits.  Two copies are kept (left-right): the
 * writer updates the one no reader is pinned on, so a pin of the current or
 * the previous apply's epoch succeeds; VMQG_E_STATE for an older epoch whose
 * records have since changed (the caller matches again).  A reader call. */
int vmqg_records_pin(vmqg_ctx* ctx, uint64_t epoch, const vmqg_emit** recs, uint64_t* n, uint32_t* pin);
void vmqg_records_unpin(vmqg_ctx* ctx, uint32_t pin);

/* ---- pipelined host-buffer matching (ABI 4) ---------------------------- */
/* vmqg_match_batch is one synchronous round trip.  A host that matches many
 * batches back to back (the NIF's combining submitter, integration/c_src/
 * vmqg_batch.c) keeps several in flight instead: an hbatch owns pinned host
 * and device buffers for one batch, and its three phases are separate calls
 *   submit   H2D of the inputs (on the hbatch's own copy stream), then the
 *            match and the D2H of its offsets on the context's stream;
 *            returns at once.  Needs the context to itself (like every call
 *            that changes or reads device tables): callers serialise it with
 *            vmqg_apply_ops and the other match calls.
 *   offsets  waits for the match; *total = entries.  VMQG_E_OVERFLOW when the
 *            output did not fit (the hbatch's output grows to *total for the
 *            next submit: submit again), VMQG_E_FRONTIER likewise (the next
 *            submit uses a larger wave-tier stack).
 *   entries  D2H of the entries on the hbatch's copy stream; waits.
 * offsets and entries touch only the hbatch: they may run while another
 * thread submits the next batch (its H2D and kernels overlap this batch's
 * D2H).  Results are those of the table epoch *epoch (vmqg_epoch at submit).
 * Each submit also collects and clears the error bits its own match latched,
 * so hbatches in flight never report each other's errors (and a
 * vmqg_match_status afterwards does not see them). */
typedef struct vmqg_hbatch vmqg_hbatch;
vmqg_hbatch* vmqg_hbatch_new(vmqg_ctx* ctx);
void vmqg_hbatch_free(vmqg_hbatch* hb);
/* pinned input buffers with room for npub publishes and nwords word ids */
int vmqg_hbatch_inputs(vmqg_hbatch* hb, size_t npub, size_t nwords, vmqg_pub** pubs, uint32_t** words);
/* ranges != 0: vmqg_match_ranges semantics (8-B entries), else vmqg_match_batch (16-B records) */
int vmqg_hbatch_submit(vmqg_ctx* ctx, vmqg_hbatch* hb, size_t npub, size_t nwords, int ranges);
int vmqg_hbatch_offsets(vmqg_hbatch* hb, const uint64_t** offsets, uint64_t* total, uint64_t* epoch);
int vmqg_hbatch_entries(vmqg_hbatch* hb, const void** entries);

/* ---- introspection --------------------------------------------------- */
int vmqg_stats(vmqg_ctx* ctx, vmqg_stats_t* out);

/* Canonical text dump of the six logical tables (one line per ETS object,
 * sorted; ids printed as mp#N / node#N / sub#N / info#N).  *text is owned by
 * the context and valid until the next call on it. */
int vmqg_dump(vmqg_ctx* ctx, const char** text, size_t* len);

/* Tuning knobs of the match kernels (no effect on results):
 *   "fast_g"    0 | 1 | 2 | 4  lanes per publish in the fast tier (1: one lane per
 *                          publish in COUNT, two in EMIT over the same 64-publish
 *                          chunks; default 0 = auto: 1 from 262,144 publishes a
 *                          call, 2 below — a small batch needs the waves)
 *   "nt_stores" 0 | 1      non-temporal stores for emitted records (default 1)
 *   "trieless"  0 | 1      tables without any wildcard / $share filter: COUNT is
 *                          one exact-table probe per publish, four publishes per
 *                          lane in flight (default 1; 0: the general walk)
 *   "fused"     0 | 1      trie-less tables: COUNT, the offset scan and EMIT in one
 *                          launch, tiles chained by look-back (default 1; 0: the
 *                          three trie-less launches)
 *   "exact_one" 0 | 1      a topic of <= 3 words with one local record keeps the
 *                          record in its exact slot, so the trie-less match
 *                          writes it without reading the record table (default
 *                          1; applies to slots written from then on)
 *   "root_flags" 0 | 1     a walk starts from its root's cached child flags, so a
 *                          mountpoint without wildcard / $share filters walks
 *                          nothing (default 1; 0: the root's three probes)
 *   "count_bpc", "emit_bpc" 0..32  fast-tier grid cap, blocks per CU (0 = 8;
 *                          defaults 5 and 16)
 *   "dedupe"    0 | 1 | 2  batch-wide dedupe of repeated (MP, topic) publishes in
 *                          COUNT: off, on (a claim and a classify pass, COUNT
 *                          walks one representative per topic, a fix-up pass
 *                          gives the duplicates its result), or auto (2, the
 *                          default: on while more than half the publishes of
 *                          the last deduped call repeated another; while off,
 *                          whole calls are probed deduped — the first call,
 *                          then after 64, 128, ... up to 8,192 calls while the
 *                          probes keep finding distinct topics — and a call of
 *                          fewer than 256 publishes is never probed)
 *   "dd_g"      1 | 4      dedupe on: lanes per representative in COUNT (default 4)
 *   "groups"    0 | 1      records mode: publishes of >= 128 records grouped by what
 *                          they emit and written group by group by the EMIT tail
 *                          (default 0: it loses its A/B)
 *   "exfilter"  0 | 1 | 2  exact-topic lookups behind the 1-bit-per-slot filter:
 *                          off, on, or auto (2, the default: on the first call
 *                          and every 64th, 4,096 sampled publishes' filter bits
 *                          decide the next calls — on while fewer than half pass)
 *   "heavy_min" 0..2^30    records mode: publishes of >= that many records from
 *                          <= 2 keys are copied by the EMIT tail on the XCD their
 *                          first key hashes to (0, the default: off)
 *   "reader_records" 1     keep the readers' record buffers (vmqg_records_pin);
 *                          a writer call, made before readers start
 *   "fail_commits" 0..1000 test hook: the next n commits fail with VMQG_E_DEVICE
 *                          before touching the device (the recovery path above) */
int vmqg_set_option(vmqg_ctx* ctx, const char* name, int64_t value);

/* Average duration (ns) of the match kernels over the last
 * vmqg_match_device calls made with timing enabled (vmqg_set_timing):
 * vmqg_kernel_times gives the fast-tier COUNT and EMIT launches;
 * vmqg_kernel_times_ex all five launches of a call, stage_ns[5] =
 * {COUNT fast tier, COUNT wave tier, scan, EMIT fast tier, EMIT wave tier}. */
#define VMQG_TIMED_STAGES 5
int vmqg_set_timing(vmqg_ctx* ctx, int enable);
int vmqg_kernel_times(vmqg_ctx* ctx, double* count_ns, double* emit_ns, uint64_t* launches);
int vmqg_kernel_times_ex(vmqg_ctx* ctx, double* stage_ns, uint64_t* launches);

/* ---- replication (one primary, N device replicas) --------------------- */
/* Device arena of the context: pointer, byte size and the layout descriptor
 * (opaque, VMQG_LAYOUT_BYTES long) a replica needs to interpret it. */
#define VMQG_LAYOUT_BYTES 256
int vmqg_arena(vmqg_ctx* ctx, void** d_ptr, uint64_t* bytes, uint8_t* layout_out);

/* Primary side: copy the host mirror of the arena (byte-identical to the
 * device image) to host memory dst (cap >= bytes from vmqg_arena). */
int vmqg_export_image(vmqg_ctx* ctx, void* dst, uint64_t cap);

/* Replica side: adopt `layout` and copy a full arena image from device memory
 * d_src (same device as ctx) on `stream`. */
int vmqg_replica_load(vmqg_ctx* ctx, const uint8_t* layout, const void* d_src, void* stream);

/* Patches produced by the last vmqg_apply_ops on a primary: host bytes
 * (records of 24 bytes) valid until the next apply; *full_image = 1 when the
 * apply re-laid out the arena (replicas must reload the full image instead). */
int vmqg_last_patches(vmqg_ctx* ctx, const void** host_ptr, uint64_t* bytes, int* full_image);

/* Replica side: adopt the fields of the primary's layout that change without
 * a re-layout (the trie depth that sizes the wave tier's stack); every
 * region must match the replica's (else VMQG_E_STATE: reload the image). */
int vmqg_replica_sync_layout(vmqg_ctx* ctx, const uint8_t* layout);

/* Replica side: apply patch records already in device memory on `stream`
 * (after every match already queued on the context; matches queued later, on
 * any stream, see them).  Asynchronous. */
int vmqg_apply_patches_device(vmqg_ctx* ctx, const void* d_patches, uint64_t bytes, void* stream);

/* Replica side, one call per primary apply (ABI 7): brings the replica to the
 * primary's committed tables — the primary's last patch list when the
 * replica holds the epoch before it and that apply shipped patches, else the
 * whole image from the primary's host mirror — on the replica's own stream,
 * after the matches already queued on it.  The replica then reports the
 * primary's epoch (vmqg_epoch), so its range results index the primary's
 * record table of that epoch (vmqg_records_pin on the primary).  VMQG_E_STATE
 * while the primary's stage is pending after a failed commit (the replica
 * keeps its older tables; call again after the commit).  A device call on the
 * replica that reads the primary's writer state: made by the primary's writer
 * (after its commit, before its next stage).  Replaces, for contexts in one
 * process, the RCCL image / patch broadcast of vernemq_amd/dist.py. */
int vmqg_replica_follow(vmqg_ctx* replica, vmqg_ctx* primary);

/* Digest of the device arena's bytes (a device call; tests compare a
 * replica's with its primary's after every apply). */
int vmqg_arena_digest(vmqg_ctx* ctx, uint64_t* digest);

#ifdef __cplusplus
}
#endif
#endif /* VMQG_H */
