// Decoupled look-back shared by the one-launch offset scan (vmqg_kernels.hip) and by the retained-store kernels
// (vmqr_kernels.hip).  Each tile / chunk owns one 8-B granule
// {tag:20, flag:2, value:42}; the granule is its own flag, written and read
// with agent-scope relaxed atomics (cdna_hip_programming.md Guideline 16,
// R2), so no fence is needed.  `tag` distinguishes calls: granules of an
// earlier call read as "not posted yet"; the host clears the array before
// a tag is reused.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vmqg {

constexpr uint64_t kLbValueMask = (1ull << 42) - 1;
constexpr uint64_t kLbAgg = 1, kLbIncl = 2;
constexpr uint32_t kErrLookback = 16u;
constexpr uint32_t kSpinLimit = 1u << 26;

__device__ __forceinline__ uint64_t lb_pack(uint32_t tag, uint64_t flag, uint64_t v) {
  return ((uint64_t)tag << 44) | (flag << 42) | (v & kLbValueMask);
}
__device__ __forceinline__ void lb_store(uint64_t* p, uint64_t x) {
  __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t lb_load(uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive output base of `chunk`, computed by one whole wave.  Posts the
// chunk's aggregate first so successors can pass over it, then looks back
// over 64 x kLbDepth predecessors per round (lane i loads chunk - 1 - i - 64 k
// for k < kLbDepth, all loads in flight together): the nearest predecessor
// with an inclusive prefix ends the walk, the aggregates of the ones in
// between are summed.  A round is retried while a granule it needs is not
// yet posted (tag of an earlier call).
#ifndef VMQG_LB_DEPTH
#define VMQG_LB_DEPTH 4
#endif
constexpr int kLbDepth = VMQG_LB_DEPTH;

// kSleep: s_sleep between rounds that found a granule not yet posted —
// longer for callers with many waves spinning at once (their loads slow the
// waves still working).
// `err`: the caller's error word (kErrLookback is OR-ed in when a round spins
// past kSpinLimit).
template <int kSleep = 1>
__device__ inline uint64_t lookback(uint64_t* lb, uint32_t tag, uint32_t* err, uint32_t chunk, uint64_t agg) {
  const uint32_t lane = __lane_id();
  if (chunk == 0) {
    if (lane == 0) lb_store(lb, lb_pack(tag, kLbIncl, agg));
    return 0;
  }
  if (lane == 0) lb_store(lb + chunk, lb_pack(tag, kLbAgg, agg));
  uint64_t excl = 0;
  int64_t top = (int64_t)chunk - 1;
  for (uint32_t spins = 0;;) {
    uint64_t x[kLbDepth];
#pragma unroll
    for (int k = 0; k < kLbDepth; k++) {
      const int64_t j = top - (int64_t)lane - 64 * k;
      x[k] = j >= 0 ? lb_load(lb + j) : 0;
    }
    uint64_t sum = 0;
    bool done = false, retry = false;
#pragma unroll
    for (int k = 0; k < kLbDepth; k++) {
      if (done || retry) continue;
      const int64_t j = top - (int64_t)lane - 64 * k;
      const bool ready = j >= 0 && (uint32_t)(x[k] >> 44) == tag;
      const uint64_t incl = __ballot(ready && ((x[k] >> 42) & 3) == kLbIncl);
      const uint64_t waiting = __ballot(j >= 0 && !ready);
      const uint32_t stop = incl ? (uint32_t)__builtin_ctzll(incl) : 64u;   // nearest inclusive predecessor
      const uint64_t need = stop >= 63 ? ~0ull : ((2ull << stop) - 1);       // lanes 0..stop
      if (waiting & need) { retry = true; continue; }
      uint64_t v = (lane <= stop && j >= 0) ? (x[k] & kLbValueMask) : 0;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t lo = __shfl_xor((uint32_t)v, o, 64), hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
        v += ((uint64_t)hi << 32) | lo;
      }
      sum += v;
      if (stop < 64 || top - 64 * k - 63 <= 0) done = true;
    }
    if (retry) {
      if (++spins > kSpinLimit) { if (lane == 0) atomicOr(err, kErrLookback); break; }
      __builtin_amdgcn_s_sleep(kSleep);
      continue;   // the whole round again (its granules may have moved on)
    }
    excl += sum;
    if (done) break;
    top -= 64 * kLbDepth;
  }
  if (lane == 0) lb_store(lb + chunk, lb_pack(tag, kLbIncl, excl + agg));
  return excl;
}


}  // namespace vmqg
