/*
 * vmqs.h — C ABI of libvmqgpu's shared-subscription dispatcher: the MI355X
 * restatement of what VerneMQ does with the `$share` members a publish's
 * fold collected.
 *
 * Drop-in boundary (paths relative to the reference checkout):
 *   apps/vmq_server/src/vmq_reg.erl:257-261   publish/5: fold, then
 *       vmq_shared_subscriptions:publish(Msg, SGPolicy, SubscriberGroups)
 *   apps/vmq_server/src/vmq_reg.erl:341-346, 373-378  the fold fun collects
 *       kind-B entries {Node, Group, SubscriberId, SubInfo} into a map
 *       Group -> [{Node, SubscriberId, SubInfo}] (add_to_subscriber_group)
 *   apps/vmq_server/src/vmq_shared_subscriptions.erl:18-106  publish/3:
 *       per group, filter_subscribers/2 by policy (:90-106), one random
 *       order (:27-28), the first ONLINE member takes the message
 *       (publish_online :46-63); when none is online, the members found
 *       offline/draining are tried in reverse order (publish_any :65-73);
 *       members whose queue is missing are skipped (:54-60, :75-78)
 *                                                   -> vmqs_select_batch / _device
 *
 * Input: the emission array of a match batch exactly as vmqg_match_* left it
 * (vmqg_emit records, per-publish offsets), so dispatch runs on the device
 * right after the match without the records leaving HBM.  Output: one byte
 * per record, 1 on the kind-B record whose subscriber receives the message
 * for its group, 0 elsewhere; and per publish the number of groups that
 * reached nobody ({error, no_subscribers}).
 *
 * Randomness.  The reference orders a group by rand:uniform() per list
 * element (:27-28), so only the distribution is reference behaviour: each
 * collected entry is equally likely to come first, and a member collected k
 * times (the Q2 multiplicity) is k times as likely.  This
 * library draws the element keys from a counter-based generator instead:
 * key = vmqs_key(seed, pub_seq + i, p) for the record at position p of
 * publish i's segment (see below), ties broken by position.  The choice is
 * therefore a pure function of (records, states, policy, seed, pub_seq) and
 * is bit-exact against the CPU restatement; the distribution matches the
 * reference's.
 *
 * Queue states come from a device-resident table indexed by SubscriberId
 * id (vmqs_set_states), the host's view of vmq_reg:get_queue_pid /
 * vmq_queue status for local and remote members.  Ids never set are
 * VMQS_ONLINE.
 *
 * Conventions as in vmqg.h: 0 / negative VMQG_E_* status, caller-owned
 * buffers, one context is not re-entrant, calls on one context are ordered
 * on its stream.
 */
#ifndef VMQS_H
#define VMQS_H

#include "vmqg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* shared_subscription_policy (vmq_server.schema:1472; filter_subscribers/2) */
#define VMQS_POLICY_RANDOM 0u        /* all members                            */
#define VMQS_POLICY_PREFER_LOCAL 1u  /* local members if any, else all          */
#define VMQS_POLICY_LOCAL_ONLY 2u    /* local members only                      */

/* queue state of a member as publish_/3 meets it */
#define VMQS_NOT_FOUND 0u   /* no queue: {error, not_found}, skipped             */
#define VMQS_ONLINE 1u      /* enqueue(online) succeeds                          */
#define VMQS_OFFLINE 2u     /* {error, offline}: kept for publish_any            */
#define VMQS_DRAINING 3u    /* {error, draining}: kept for publish_any           */

#define VMQS_MAX_SEGMENT (1u << 24)   /* records per publish the keys can order  */

typedef struct vmqs_config {
  int32_t device;       /* HIP device ordinal (required)                   */
  uint32_t local_node;  /* node id that plays node()                       */
} vmqs_config;

typedef struct vmqs_ctx vmqs_ctx;

vmqs_ctx* vmqs_create(const vmqs_config* cfg, int* err);
void vmqs_destroy(vmqs_ctx* ctx);

/* Sets the queue state of n subscriber ids (stream-ordered before later
 * selections; the table grows to the largest id). */
int vmqs_set_states(vmqs_ctx* ctx, const uint32_t* subscribers, const uint8_t* states, size_t n);

/* Host-buffer dispatch of npub publishes' emissions (offsets[0..npub] as
 * vmqg_match_batch wrote them, emits[offsets[0] .. offsets[npub])).
 * chosen[r] for every record r in that range; failed[i] (may be NULL) = the
 * groups of publish i that reached nobody.  Synchronous. */
int vmqs_select_batch(vmqs_ctx* ctx, const vmqg_emit* emits, const uint64_t* offsets, size_t npub,
                      uint32_t policy, uint64_t seed, uint64_t pub_seq, uint8_t* chosen, uint32_t* failed);

/* Device-buffer form: every pointer on the context's device, work on
 * `stream` (NULL = the legacy default stream, see vmqg_match_device), no
 * synchronisation.  d_failed may
 * be NULL.  A publish whose groups exceed the device tables or whose segment
 * exceeds VMQS_MAX_SEGMENT latches VMQG_E_LIMIT for vmqs_select_status. */
int vmqs_select_device(vmqs_ctx* ctx, const vmqg_emit* d_emits, const uint64_t* d_offsets, uint32_t npub,
                       uint32_t policy, uint64_t seed, uint64_t pub_seq, uint8_t* d_chosen, uint32_t* d_failed,
                       void* stream);
int vmqs_select_status(vmqs_ctx* ctx, void* stream);

/* Streams: device calls take the caller's stream (NULL = the legacy default
 * stream).  The context orders its work across streams by recording an event
 * on the stream it last queued on when the next call comes on another one;
 * so a stream passed to any entry point must stay alive until the next call
 * on the context, or be released first with vmqs_release_stream (records that
 * event now; no-op if the context's last work is not on it). */
int vmqs_release_stream(vmqs_ctx* ctx, void* stream);

/* The element key of the record at position p of publish number q (the
 * batch's pub_seq + its index): the 40 high bits of a splitmix64-style mix
 * of (seed, q, p), then p in the low 24 bits, so keys order by (random, p). */
uint64_t vmqs_key(uint64_t seed, uint64_t q, uint32_t p);

/* Average duration (ns) of the select kernels over the timed calls, and the
 * publishes the last checked call sent to the workgroup tier. */
int vmqs_set_timing(vmqs_ctx* ctx, int enable);
int vmqs_kernel_times(vmqs_ctx* ctx, double* select_ns, uint64_t* launches, uint64_t* deferred);

#ifdef __cplusplus
}
#endif
#endif /* VMQS_H */
