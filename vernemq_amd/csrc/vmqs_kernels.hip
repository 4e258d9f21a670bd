// HIP kernels for gfx950: vmq_shared_subscriptions:publish/3 over a match
// batch's emission records (apps/vmq_server/src/vmq_shared_subscriptions.erl
// :18-106, fed by vmq_reg.erl:257-261, 341-346, 373-378).
//
// Per publish, every kind-B record {Node, Group, SubscriberId, SubInfo} is
// an element of its Group's list (add_to_subscriber_group: the map is keyed
// by the group name alone, so one group reached through two filters is one
// list).  Per group:
//   1. filter_subscribers/2 (:90-106): random keeps all; local_only keeps
//      Node == node(); prefer_local keeps the local ones if there is one.
//   2. one random order (:27-28): element key sel_key(seed, q, position).
//   3. publish_online (:46-63): the first element in key order whose queue
//      is online takes the message -> the minimum key among ONLINE elements.
//   4. else publish_any (:65-73) over the offline/draining elements in
//      REVERSE encounter order -> the maximum key among them.
//   5. else {error, no_subscribers}: counted in failed[i].
// Elements with no queue (NOT_FOUND) are skipped in both passes (:54-60).
// The fold fun's no_local clause for kind B (vmq_reg.erl:341-343) matches a
// bare map, which a stored SubInfo ({QoS, Map} or QoS) never is, so it never
// drops a shared member; nothing to do here.
//
// Layout of the work: keys order by (40 random bits, position), so "minimum
// key" and "maximum key" are single 64-bit LDS atomicMin / atomicMax per
// element; a group's slot holds {group, flags, min online key, max offline
// key}.  Tier 1: one wave per publish, 64-slot table and a 4096-bit bitmap
// of winners in LDS, so every chosen[] byte is written exactly once, in
// order.  Tier 2 (long segments, many groups): one workgroup per publish.
// Integer work only, no MFMA; HBM-bound on the 16-B record reads.
#include <hip/hip_runtime.h>

#include "vmqs_engine.h"

namespace vmqs {

using vmqg::kEmpty;
using vmqg::Record;

constexpr uint32_t kFOn = 1u, kFOff = 2u, kFLocal = 4u;

struct alignas(8) GSlot { uint32_t group, flags; unsigned long long on, off; };
static_assert(sizeof(GSlot) == 24, "");

__device__ __forceinline__ uint32_t kind_of(const Record& r) { return r.kind_node >> 24; }
__device__ __forceinline__ uint32_t node_of(const Record& r) { return r.kind_node & 0xFFFFFFu; }
__device__ __forceinline__ uint32_t gslot_home(uint32_t g, uint32_t mask) { return (uint32_t)vmqg::mix64(g) & mask; }

// Find or claim the slot of group g (open addressing, linear probing).
// Returns kEmpty when the table is full.
__device__ __forceinline__ uint32_t gslot_claim(GSlot* t, uint32_t mask, uint32_t g) {
  uint32_t h = gslot_home(g, mask);
  for (uint32_t n = 0; n <= mask; n++, h = (h + 1) & mask) {
    const uint32_t cur = atomicCAS(&t[h].group, kEmpty, g);
    if (cur == kEmpty || cur == g) return h;
  }
  return kEmpty;
}
__device__ __forceinline__ uint32_t gslot_find(const GSlot* t, uint32_t mask, uint32_t g) {
  uint32_t h = gslot_home(g, mask);
  while (t[h].group != g) h = (h + 1) & mask;   // present: claimed in pass 1
  return h;
}

__device__ __forceinline__ uint32_t state_of(const SArgs& a, uint32_t sub) {
  return sub < a.n_states ? a.states[sub] : (uint32_t)VMQS_ONLINE;
}

// Pass 2 body: one kind-B element at position p.
__device__ __forceinline__ void offer(const SArgs& a, GSlot* t, uint32_t mask, const Record& r, uint64_t q,
                                      uint32_t p) {
  const uint32_t h = gslot_find(t, mask, r.group);
  const bool local = node_of(r) == a.local_node;
  const bool elig = a.policy == VMQS_POLICY_RANDOM ? true
                    : a.policy == VMQS_POLICY_LOCAL_ONLY ? local
                                                          : (local || !(t[h].flags & kFLocal));
  if (!elig) return;
  const uint32_t s = state_of(a, r.subscriber);
  if (s == VMQS_NOT_FOUND) return;
  const unsigned long long k = sel_key(a.seed, q, p);
  if (s == VMQS_ONLINE) {
    atomicMin(&t[h].on, k);
    atomicOr(&t[h].flags, kFOn);
  } else {
    atomicMax(&t[h].off, k);
    atomicOr(&t[h].flags, kFOff);
  }
}

__device__ __forceinline__ void lds_fence() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup"); }

// ---- tier 1: one wavefront per publish --------------------------------------
constexpr uint32_t kWaves = 4;
constexpr uint32_t kBitWords = kWaveMax / 32;

__global__ __launch_bounds__(256) void k_select_wave(SArgs a) {
  __shared__ GSlot tab[kWaves][kWaveGroups];
  __shared__ uint32_t win[kWaves][kBitWords];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t i = blockIdx.x * kWaves + w;
  if (i >= a.npub) return;
  const uint64_t s0 = a.offsets[i];
  const uint32_t n = (uint32_t)min<uint64_t>(a.offsets[i + 1] - s0, 0xFFFFFFFFull);
  if (n > kWaveMax) {
    if (lane == 0) a.defer[atomicAdd(&a.status[0], 1u)] = i;
    return;
  }
  GSlot* t = tab[w];
  const uint32_t mask = kWaveGroups - 1;
  const Record* rec = a.emits + s0;
  uint8_t* ch = a.chosen + s0;
  for (uint32_t k = lane; k < kWaveGroups; k += 64) t[k] = GSlot{kEmpty, 0u, ~0ull, 0ull};
  lds_fence();
  __builtin_amdgcn_wave_barrier();
  // pass 1: the groups of the segment and whether each has a local member
  bool any = false, ovf = false;
  for (uint32_t p = lane; p < n; p += 64) {
    const Record r = rec[p];
    if (kind_of(r) != VMQG_EMIT_GROUP) continue;
    any = true;
    const uint32_t h = gslot_claim(t, mask, r.group);
    if (h == kEmpty) { ovf = true; continue; }
    if (node_of(r) == a.local_node) atomicOr(&t[h].flags, kFLocal);
  }
  if (__ballot(ovf)) {
    if (lane == 0) a.defer[atomicAdd(&a.status[0], 1u)] = i;
    return;
  }
  if (!__ballot(any)) {   // no shared member: nothing chosen
    for (uint32_t p = lane; p < n; p += 64) ch[p] = 0;
    if (lane == 0 && a.failed) a.failed[i] = 0;
    return;
  }
  for (uint32_t k = lane; k < kBitWords; k += 64) win[w][k] = 0;
  lds_fence();
  __builtin_amdgcn_wave_barrier();
  // pass 2: filter, key, offer
  const uint64_t q = a.pub_seq + i;
  for (uint32_t p = lane; p < n; p += 64) {
    const Record r = rec[p];
    if (kind_of(r) == VMQG_EMIT_GROUP) offer(a, t, mask, r, q, p);
  }
  lds_fence();
  __builtin_amdgcn_wave_barrier();
  // pass 3: one winner per group (online first, else publish_any's pick)
  uint32_t nf = 0;
  for (uint32_t k = lane; k < kWaveGroups; k += 64) {
    const GSlot s = t[k];
    if (s.group == kEmpty) continue;
    if (s.flags & (kFOn | kFOff)) {
      const uint32_t p = (uint32_t)((s.flags & kFOn ? s.on : s.off) & 0xFFFFFFu);
      atomicOr(&win[w][p >> 5], 1u << (p & 31));
    } else {
      nf++;
    }
  }
  lds_fence();
  __builtin_amdgcn_wave_barrier();
  // pass 4: every chosen byte once
  for (uint32_t p = lane; p < n; p += 64) ch[p] = (win[w][p >> 5] >> (p & 31)) & 1u;
  for (int o = 32; o > 0; o >>= 1) nf += __shfl_xor(nf, o);
  if (lane == 0 && a.failed) a.failed[i] = nf;
}

// ---- tier 2: one workgroup per deferred publish --------------------------------
__global__ __launch_bounds__(256) void k_select_block(SArgs a) {
  __shared__ GSlot t[kBlockGroups];
  __shared__ uint32_t s_ovf, s_nf;
  const uint32_t mask = kBlockGroups - 1;
  const uint32_t count = *(volatile uint32_t*)&a.status[0];
  for (uint32_t j = blockIdx.x; j < count; j += gridDim.x) {   // every block exits after the list
    const uint32_t i = a.defer[j];
    const uint64_t s0 = a.offsets[i], n = a.offsets[i + 1] - s0;
    const Record* rec = a.emits + s0;
    uint8_t* ch = a.chosen + s0;
    __syncthreads();   // the previous publish's table reads are done
    for (uint32_t k = threadIdx.x; k < kBlockGroups; k += blockDim.x) t[k] = GSlot{kEmpty, 0u, ~0ull, 0ull};
    if (threadIdx.x == 0) { s_ovf = n > VMQS_MAX_SEGMENT ? 1u : 0u; s_nf = 0; }
    __syncthreads();
    for (uint64_t p = threadIdx.x; p < n; p += blockDim.x) {
      const Record r = rec[p];
      ch[p] = 0;
      if (kind_of(r) != VMQG_EMIT_GROUP) continue;
      const uint32_t h = gslot_claim(t, mask, r.group);
      if (h == kEmpty) { s_ovf = 1u; continue; }
      if (node_of(r) == a.local_node) atomicOr(&t[h].flags, kFLocal);
    }
    __threadfence();   // the zero bytes are visible before any winner byte
    __syncthreads();
    if (s_ovf) {
      if (threadIdx.x == 0) {
        atomicOr(&a.status[1], kErrLimit);
        if (a.failed) a.failed[i] = 0;
      }
      continue;
    }
    const uint64_t q = a.pub_seq + i;
    for (uint64_t p = threadIdx.x; p < n; p += blockDim.x) {
      const Record r = rec[p];
      if (kind_of(r) == VMQG_EMIT_GROUP) offer(a, t, mask, r, q, (uint32_t)p);
    }
    __syncthreads();
    uint32_t nf = 0;
    for (uint32_t k = threadIdx.x; k < kBlockGroups; k += blockDim.x) {
      const GSlot s = t[k];
      if (s.group == kEmpty) continue;
      if (s.flags & (kFOn | kFOff)) ch[(s.flags & kFOn ? s.on : s.off) & 0xFFFFFFu] = 1;
      else nf++;
    }
    if (nf) atomicAdd(&s_nf, nf);
    __syncthreads();
    if (threadIdx.x == 0 && a.failed) a.failed[i] = s_nf;
  }
}

hipError_t launch_select(const SArgs& a, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  if (e0) hipEventRecord(e0, st);
  if (a.npub) {
    k_select_wave<<<(a.npub + kWaves - 1) / kWaves, 256, 0, st>>>(a);
    k_select_block<<<kBlockGrid, 256, 0, st>>>(a);
  }
  if (e1) hipEventRecord(e1, st);
  return hipGetLastError();
}

}  // namespace vmqs
