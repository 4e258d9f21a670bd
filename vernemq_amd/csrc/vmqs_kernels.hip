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
// key} (tier 1 keeps local / all pairs, see below).  Tier 1: one wave per publish, 64-slot table and a 4096-bit bitmap
// of winners in LDS, so every chosen[] byte is written exactly once, in
// order.  Tier 2 (long segments, many groups): one workgroup per publish.
// Integer work only, no MFMA.  The byte bound is one read of the 16-B
// records (8.27 GB of HBM traffic per launch for 8.05 GB algorithmic on the
// SS workload), but the kernel runs at ~36 % of the HBM peak: it is
// latency-bound per wave (load -> LDS claim -> reduction -> bitmap ->
// write), see DESIGN.md "Shared-subscription dispatch".
#include <hip/hip_ext.h>
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

// ---- tier 1: one wavefront per publish, one read of the segment ----------------
// prefer_local's eligible set depends on whether the group has a local member,
// which is only known after the whole segment was seen; rather than reading the
// records twice, each slot keeps the extremes over the local members and over
// all members, and pass 3 picks the pair the policy selects.
constexpr uint32_t kWaves = 4;
constexpr uint32_t kBitWords = kWaveMax / 32;
#ifndef VMQS_UNROLL
#define VMQS_UNROLL 4
#endif
constexpr uint32_t kUnroll = VMQS_UNROLL;   // records in flight per lane (A/B: tools/build_variants.py)
#ifndef VMQS_KIND_SCAN
#define VMQS_KIND_SCAN 0   // A/B: 1 = a kind-word pre-pass (SS 2,075 vs 1,848 us: off)
#endif
constexpr uint32_t kKindScan = 16;          // kind words in flight per lane in the pre-pass
constexpr uint32_t kFOnL = 8u, kFOffL = 16u;

struct alignas(8) WSlot { uint32_t group, flags; unsigned long long on_l, on_a, off_l, off_a; };
static_assert(sizeof(WSlot) == 40, "");

__device__ __forceinline__ uint32_t wslot_claim(WSlot* t, uint32_t mask, uint32_t g) {
  uint32_t h = gslot_home(g, mask);
  for (uint32_t n = 0; n <= mask; n++, h = (h + 1) & mask) {
    const uint32_t cur = atomicCAS(&t[h].group, kEmpty, g);
    if (cur == kEmpty || cur == g) return h;
  }
  return kEmpty;
}

// One kind-B element at position p: claim its group's slot and offer its key.
// Returns false when the slot table is full.
__device__ __forceinline__ bool offer1(const SArgs& a, WSlot* t, uint32_t mask, const Record& r, uint32_t s,
                                       uint64_t q, uint32_t p) {
  const uint32_t h = wslot_claim(t, mask, r.group);
  if (h == kEmpty) return false;
  const bool local = node_of(r) == a.local_node;
  if (local) atomicOr(&t[h].flags, kFLocal);
  if (s == VMQS_NOT_FOUND) return true;
  const unsigned long long k = sel_key(a.seed, q, p);
  if (s == VMQS_ONLINE) {
    atomicMin(&t[h].on_a, k);
    if (local) atomicMin(&t[h].on_l, k);
    atomicOr(&t[h].flags, local ? (kFOn | kFOnL) : kFOn);
  } else {
    atomicMax(&t[h].off_a, k);
    if (local) atomicMax(&t[h].off_l, k);
    atomicOr(&t[h].flags, local ? (kFOff | kFOffL) : kFOff);
  }
  return true;
}

#ifndef VMQS_WIDE_CHOSEN
#define VMQS_WIDE_CHOSEN 1
#endif

// Writes chosen[0..n) of one segment: bit p of `win` (all zero when win is
// null).  Wide form: byte head up to 4-B alignment, then one dword of four
// chosen bytes per lane, then the byte tail.
__device__ __forceinline__ void write_chosen(uint8_t* ch, uint32_t n, const uint32_t* win, uint32_t lane) {
#define VMQS_BIT(p) (win ? (win[(p) >> 5] >> ((p) & 31)) & 1u : 0u)
#if VMQS_WIDE_CHOSEN
  const uint32_t head = min(n, (uint32_t)((4u - ((uint32_t)(uintptr_t)ch & 3u)) & 3u));
  if (lane < head) ch[lane] = (uint8_t)VMQS_BIT(lane);
  const uint32_t nw = (n - head) >> 2;
  uint32_t* cw = reinterpret_cast<uint32_t*>(ch + head);
  for (uint32_t k = lane; k < nw; k += 64) {
    const uint32_t p = head + 4 * k;
    cw[k] = VMQS_BIT(p) | VMQS_BIT(p + 1) << 8 | VMQS_BIT(p + 2) << 16 | VMQS_BIT(p + 3) << 24;
  }
  for (uint32_t p = head + 4 * nw + lane; p < n; p += 64) ch[p] = (uint8_t)VMQS_BIT(p);
#else
  for (uint32_t p = lane; p < n; p += 64) ch[p] = (uint8_t)VMQS_BIT(p);
#endif
#undef VMQS_BIT
}

#ifndef VMQS_WAVES_PER_EU
#define VMQS_WAVES_PER_EU 8
#endif
// 8 waves per SIMD: the kernel is latency-bound, so residency (bytes in
// flight) matters more than the registers the unrolled loop would take.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VMQS_WAVES_PER_EU, 8)))
void k_select_wave(SArgs a) {
  __shared__ WSlot tab[kWaves][kWaveGroups];
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
  WSlot* t = tab[w];
  const uint32_t mask = kWaveGroups - 1;
  const Record* rec = a.emits + s0;
  uint8_t* ch = a.chosen + s0;
#if VMQS_KIND_SCAN
  // pass 0: is there a shared member at all?  Only each record's kind word,
  // kKindScan records per lane in flight (a 1,000-record segment in one
  // round); most segments (exact and plain wildcard subscribers) have none
  // and need neither the group table nor a second look at their records.
  {
    bool anyb = false;
    for (uint32_t base = 0; base < n; base += 64 * kKindScan) {
      uint32_t kw[kKindScan];
#pragma unroll
      for (uint32_t j = 0; j < kKindScan; j++) {
        const uint32_t p = base + j * 64 + lane;
        kw[j] = p < n ? rec[p].kind_node : 0u;
      }
#pragma unroll
      for (uint32_t j = 0; j < kKindScan; j++) anyb |= (kw[j] >> 24) == VMQG_EMIT_GROUP;
      if (__ballot(anyb)) break;
    }
    if (!__ballot(anyb)) {
      write_chosen(ch, n, nullptr, lane);
      if (lane == 0 && a.failed) a.failed[i] = 0;
      return;
    }
  }
#endif
  for (uint32_t k = lane; k < kWaveGroups; k += 64) t[k] = WSlot{kEmpty, 0u, ~0ull, ~0ull, 0ull, 0ull};
  for (uint32_t k = lane; k < kBitWords; k += 64) win[w][k] = 0;
  lds_fence();
  __builtin_amdgcn_wave_barrier();
  // pass 1: groups, local flags and keys in one read of the segment.
  // Members of a group are emitted contiguously, so most record instructions
  // hold one group: each lane keeps running extremes for the wave's current
  // group, and the wave reduces them and updates the group's slot only when
  // the group changes (or at the end) — not per instruction.
  const uint64_t q = a.pub_seq + i;
  bool any = false, ovf = false;
  uint32_t cg = kEmpty, cfl = 0;   // the current uniform group; this lane's flags for it
  unsigned long long c_on_a = ~0ull, c_on_l = ~0ull, c_off_a = 0ull, c_off_l = 0ull;
  auto flush = [&]() {
    if (cg == kEmpty) return;
    for (int o = 32; o > 0; o >>= 1) {
      c_on_a = min(c_on_a, __shfl_xor(c_on_a, o));
      c_on_l = min(c_on_l, __shfl_xor(c_on_l, o));
      c_off_a = max(c_off_a, __shfl_xor(c_off_a, o));
      c_off_l = max(c_off_l, __shfl_xor(c_off_l, o));
    }
    uint32_t fl = 0;
    for (uint32_t b = 1; b <= kFOffL; b <<= 1) fl |= __ballot(cfl & b) ? b : 0u;
    if (lane == 0) {
      const uint32_t h = wslot_claim(t, mask, cg);
      if (h == kEmpty) {
        ovf = true;
      } else {
        if (fl) atomicOr(&t[h].flags, fl);
        if (fl & kFOn) atomicMin(&t[h].on_a, c_on_a);
        if (fl & kFOnL) atomicMin(&t[h].on_l, c_on_l);
        if (fl & kFOff) atomicMax(&t[h].off_a, c_off_a);
        if (fl & kFOffL) atomicMax(&t[h].off_l, c_off_l);
      }
    }
    cg = kEmpty; cfl = 0;
    c_on_a = ~0ull; c_on_l = ~0ull; c_off_a = 0ull; c_off_l = 0ull;
  };
  for (uint32_t base = 0; base < n; base += 64 * kUnroll) {
    Record r[kUnroll];
#pragma unroll
    for (uint32_t j = 0; j < kUnroll; j++) {
      const uint32_t p = base + j * 64 + lane;
      if (p < n) r[j] = rec[p];
      else r[j].kind_node = 0;
    }
    // queue states of the members, all loads in flight before any is used
    uint32_t sv[kUnroll];
#pragma unroll
    for (uint32_t j = 0; j < kUnroll; j++)
      sv[j] = kind_of(r[j]) == VMQG_EMIT_GROUP ? state_of(a, r[j].subscriber) : (uint32_t)VMQS_NOT_FOUND;
#pragma unroll
    for (uint32_t j = 0; j < kUnroll; j++) {
      const bool isb = kind_of(r[j]) == VMQG_EMIT_GROUP;
      const uint64_t mb = __ballot(isb);
      if (!mb) continue;
      any = true;
      const uint32_t g0 = __builtin_amdgcn_readfirstlane(__shfl(r[j].group, (uint32_t)__builtin_ctzll(mb)));
      const bool mixed = __ballot(isb && r[j].group != g0) != 0;
      if (mixed || g0 != cg) flush();
      if (mixed) {   // mixed groups: per-lane atomics
        if (isb && !offer1(a, t, mask, r[j], sv[j], q, base + j * 64 + lane)) ovf = true;
        continue;
      }
      cg = g0;
      if (!isb) continue;
      const bool local = node_of(r[j]) == a.local_node;
      const uint32_t st = sv[j];
      const unsigned long long k = sel_key(a.seed, q, base + j * 64 + lane);
      const bool on = st == VMQS_ONLINE, off = st == VMQS_OFFLINE || st == VMQS_DRAINING;
      cfl |= (local ? kFLocal : 0u) | (on ? kFOn : 0u) | (on && local ? kFOnL : 0u) | (off ? kFOff : 0u) |
             (off && local ? kFOffL : 0u);
      if (on) { c_on_a = min(c_on_a, k); if (local) c_on_l = min(c_on_l, k); }
      if (off) { c_off_a = max(c_off_a, k); if (local) c_off_l = max(c_off_l, k); }
    }
  }
  flush();
  if (__ballot(ovf)) {
    if (lane == 0) a.defer[atomicAdd(&a.status[0], 1u)] = i;
    return;
  }
  if (!__ballot(any)) {   // no shared member: nothing chosen
    write_chosen(ch, n, nullptr, lane);
    if (lane == 0 && a.failed) a.failed[i] = 0;
    return;
  }
  lds_fence();
  __builtin_amdgcn_wave_barrier();
  // pass 3: one winner per group (online first, else publish_any's pick)
  uint32_t nf = 0;
  for (uint32_t k = lane; k < kWaveGroups; k += 64) {
    const WSlot s = t[k];
    if (s.group == kEmpty) continue;
    const bool loc = a.policy == VMQS_POLICY_LOCAL_ONLY ||
                     (a.policy == VMQS_POLICY_PREFER_LOCAL && (s.flags & kFLocal));
    const bool on = s.flags & (loc ? kFOnL : kFOn), off = s.flags & (loc ? kFOffL : kFOff);
    if (on || off) {
      const uint32_t p = (uint32_t)((on ? (loc ? s.on_l : s.on_a) : (loc ? s.off_l : s.off_a)) & 0xFFFFFFu);
      atomicOr(&win[w][p >> 5], 1u << (p & 31));
    } else {
      nf++;
    }
  }
  lds_fence();
  __builtin_amdgcn_wave_barrier();
  // pass 4: every chosen byte once
  write_chosen(ch, n, win[w], lane);
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

// e0 / e1: start of the wave tier, end of the block tier, recorded by the
// dispatches themselves (no marker packets between launches)
hipError_t launch_select(const SArgs& a, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  const uint32_t g = (a.npub + kWaves - 1) / kWaves;
  if (!a.npub) {
    if (e0) { hipEventRecord(e0, st); hipEventRecord(e1, st); }
  } else if (e0) {
    hipExtLaunchKernelGGL(k_select_wave, dim3(g), dim3(256), 0, st, e0, (hipEvent_t) nullptr, 0, a);
    hipExtLaunchKernelGGL(k_select_block, dim3(kBlockGrid), dim3(256), 0, st, (hipEvent_t) nullptr, e1, 0, a);
  } else {
    k_select_wave<<<g, 256, 0, st>>>(a);
    k_select_block<<<kBlockGrid, 256, 0, st>>>(a);
  }
  return hipGetLastError();
}

}  // namespace vmqs
