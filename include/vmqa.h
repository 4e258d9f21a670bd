/*
 * vmqa.h — C ABI of libvmqgpu's ACL checker: the MI355X restatement of
 * VerneMQ's file-based ACL plugin check (the auth_on_publish /
 * auth_on_subscribe hooks every publish and subscribe passes through).
 *
 * Drop-in boundary (paths relative to the reference checkout):
 *   apps/vmq_acl/src/vmq_acl.erl:128-144 load_from_list/1 (+ load_from_file/1
 *       :114-126): the host parses the lines (parse_acl_line/2 :146-177,
 *       in/3 :219-231) and hands the resulting six tables to  -> vmqa_load
 *   apps/vmq_acl/src/vmq_acl.erl:179-204 check/4 (check_all_acl,
 *       check_user_acl, check_pattern_acl; topic/3 + subst/5 :206-217)
 *                                                             -> vmqa_check_batch / _device
 *   apps/vmq_acl/src/vmq_acl.erl:78-93 auth_on_subscribe/3, auth_on_publish/6
 *       (+ the _m5 variants :95-99): one check per topic; the host folds
 *       the verdicts (all topics of a subscribe must pass)
 * Callers that stay unchanged: vmq_plugin's hook dispatch
 * (vmq_auth_on_publish / vmq_auth_on_subscribe) and vmq_acl_reloader.
 *
 * Semantics reproduced exactly: a check of type READ (subscribe) or WRITE
 * (publish) passes when vmq_topic:match(Topic, Rule) (vmq_topic.erl:53-65,
 * clause order kept: the checked topic's own '+'/'#' words — subscribe
 * filters — meet a rule's words by equality first) holds for a rule of that
 * type in the `all` table, in the requesting user's table, or in the
 * pattern table after %u / %c / %m in the rule are replaced by the user,
 * client id and mountpoint.  An `undefined` user (VMQA_NO_USER) has no user
 * table and, substituted for %u, equals no word.
 *
 * Word ids: rule words are interned by the context's dictionary
 * (vmqa_intern_words, '+', '#', '$share', '%u', '%c', '%m' reserved as ids
 * 0..5).  A check batch may also carry ids >= VMQA_EPHEMERAL for strings
 * absent from the dictionary (topic words, user names, client ids,
 * mountpoints): the caller assigns them per batch so that equal ids mean
 * equal strings; they equal no rule word.
 *
 * Conventions as in vmqg.h: 0 / negative VMQG_E_* status, caller-owned
 * buffers, one context is not re-entrant, load and check calls on one
 * context are ordered on its stream.
 */
#ifndef VMQA_H
#define VMQA_H

#include "vmqg.h"

#ifdef __cplusplus
extern "C" {
#endif

#define VMQA_READ 1u            /* auth_on_subscribe: t(read, ...)  */
#define VMQA_WRITE 2u           /* auth_on_publish:   t(write, ...) */
#define VMQA_TABLE_ALL 0u       /* vmq_acl_{read,write}_all        */
#define VMQA_TABLE_USER 1u      /* vmq_acl_{read,write}_user       */
#define VMQA_TABLE_PATTERN 2u   /* vmq_acl_{read,write}_pattern    */
#define VMQA_WORD_USER 3u       /* "%u" (?USER_SUP)                */
#define VMQA_WORD_CLIENT 4u     /* "%c" (?CLIENT_SUP)              */
#define VMQA_WORD_MOUNTPOINT 5u /* "%m" (?MOUNTPOINT_SUP)          */
#define VMQA_NO_USER 0xFFFFFFFEu     /* the user `undefined`      */
#define VMQA_EPHEMERAL 0x80000000u   /* first batch-local word id */

typedef struct vmqa_config {
  int32_t device;       /* HIP device ordinal; -1 = host tables only */
  uint32_t reserved;
} vmqa_config;

/* One table row: {Topic, 1} / {{User, Topic}, 1}.  24 bytes. */
typedef struct vmqa_rule {
  uint32_t type;        /* VMQA_READ | VMQA_WRITE                          */
  uint32_t table;       /* VMQA_TABLE_*                                    */
  uint32_t user;        /* word id of the user (VMQA_TABLE_USER)           */
  uint32_t word_off;    /* index of the first word id in `words`           */
  uint32_t nwords;      /* >= 1                                            */
  uint32_t reserved;
} vmqa_rule;

/* One check/4 call.  24 bytes. */
typedef struct vmqa_req {
  uint32_t type;        /* VMQA_READ | VMQA_WRITE                          */
  uint32_t user;        /* word id, or VMQA_NO_USER                        */
  uint32_t client;      /* word id of the client id                        */
  uint32_t mountpoint;  /* word id of the mountpoint string                */
  uint32_t word_off;    /* the checked topic: index of its first word id   */
  uint32_t nwords;      /* >= 1 (check/4 has no clause for an empty topic) */
} vmqa_req;

typedef struct vmqa_stats_s {
  uint64_t rules;          /* rows of the six tables                      */
  uint64_t users;          /* users with a table                          */
  uint64_t device_bytes;   /* the tables on the device                    */
  uint64_t loads;          /* vmqa_load calls                             */
  uint64_t words;          /* interned words                              */
} vmqa_stats_t;

typedef struct vmqa_ctx vmqa_ctx;

vmqa_ctx* vmqa_create(const vmqa_config* cfg, int* err);
void vmqa_destroy(vmqa_ctx* ctx);

/* As vmqg_intern_words: create != 0 adds unseen words (rules), create == 0
 * maps them to VMQG_WORD_UNKNOWN (the caller then assigns VMQA_EPHEMERAL
 * ids). */
int vmqa_intern_words(vmqa_ctx* ctx, const uint8_t* bytes, const uint64_t* offs, uint32_t n, int create,
                      uint32_t* ids_out);

/* Replaces the six tables with `rules` (duplicates allowed, as an ets set
 * absorbs them) and uploads them.  Invalid rows reject the call unchanged. */
int vmqa_load(vmqa_ctx* ctx, const vmqa_rule* rules, size_t n, const uint32_t* words, size_t nwords);

/* check/4 for a batch: allowed[i] = 1 when request i passes, else 0.
 * Synchronous. */
int vmqa_check_batch(vmqa_ctx* ctx, const vmqa_req* reqs, size_t n, const uint32_t* words, size_t nwords,
                     uint8_t* allowed);

/* Device-buffer form (pointers on the context's device, work on `stream`,
 * NULL = the legacy default stream as in vmqg_match_device; no
 * synchronisation); errors latch for vmqa_check_status. */
int vmqa_check_device(vmqa_ctx* ctx, const vmqa_req* d_reqs, uint32_t n, const uint32_t* d_words,
                      uint8_t* d_allowed, void* stream);
int vmqa_check_status(vmqa_ctx* ctx, void* stream);

/* Streams: device calls take the caller's stream (NULL = the legacy default
 * stream).  The context orders its work across streams by recording an event
 * on the stream it last queued on when the next call comes on another one;
 * so a stream passed to any entry point must stay alive until the next call
 * on the context, or be released first with vmqa_release_stream (records that
 * event now; no-op if the context's last work is not on it). */
int vmqa_release_stream(vmqa_ctx* ctx, void* stream);

int vmqa_stats(vmqa_ctx* ctx, vmqa_stats_t* out);

/* Average duration (ns) of the check kernel over the timed calls. */
int vmqa_set_timing(vmqa_ctx* ctx, int enable);
int vmqa_kernel_times(vmqa_ctx* ctx, double* check_ns, uint64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* VMQA_H */
