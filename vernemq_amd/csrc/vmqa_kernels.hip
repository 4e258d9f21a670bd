// HIP kernel for gfx950: vmq_acl:check/4 for a batch of requests
// (apps/vmq_acl/src/vmq_acl.erl:179-204).
//
// One lane per request (64 requests per wave).  A request walks, in the
// reference's order, the `all` list of its type (check_all_acl :190-192),
// its user's list (check_user_acl :194-197: an open-addressed probe for
// {user, type}) and the pattern list (check_pattern_acl :199-204, with
// subst/5's %u / %c / %m replaced by the request's user, client id and
// mountpoint while comparing, :206-217), each rule tested with
// vmq_topic:match/2 (vmq_topic.erl:53-65) until one holds
// (iterate_until_true).  The wave steps through the lists together: lanes
// of one type read the same rule: the `all` and pattern rules are staged in
// LDS once per block (up to 48 KiB; else read from the L2-resident table),
// the first 4 topic words sit in registers; a lane that has its verdict
// idles until the wave's last lane has one.  Integer compares only, no MFMA; bound by the rule
// and topic word loads (L2-resident tables).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "vmqa_engine.h"

namespace vmqa {

using vmqg::kEmpty;
using vmqg::kHash;
using vmqg::kPlus;

constexpr uint32_t kErrReq = 1u;   // status[1]: a request without a topic word, or of no known type

// vmq_topic:match(TIn, Rule), clause order kept (vmq_topic.erl:53-65):
// [H|T1],[H|T2] ; [_|T1],['+'|T2] ; (_, ['#']) ; otherwise false.  With
// `subst`, rule words %u / %c / %m are read as the request's user, client
// id and mountpoint (an undefined user's VMQA_NO_USER equals no word).  The
// first kPre topic words come from registers (constant indices, results
// by value), the rest from memory.
constexpr uint32_t kPre = 4;

struct Subst { bool on; uint32_t user, client, mp; };

__device__ __forceinline__ uint32_t subst_word(uint32_t fi, const Subst& s) {
  if (!s.on) return fi;
  return fi == VMQA_WORD_USER ? s.user : fi == VMQA_WORD_CLIENT ? s.client : fi == VMQA_WORD_MOUNTPOINT ? s.mp : fi;
}

template <class FP>
__device__ __forceinline__ bool acl_match(const uint32_t (&tw)[kPre], const uint32_t* t, uint32_t nt, FP f,
                                          uint32_t nf, const Subst& s) {
  bool done = false, res = false;
#pragma unroll
  for (uint32_t k = 0; k < kPre; k++) {
    const uint32_t fk = k < nf ? subst_word(f[k], s) : 0u;
    const bool end = k == nt && k == nf;
    const bool step = k < nt && k < nf && (tw[k] == fk || fk == kPlus);
    if (!done && !step) res = end || (k + 1 == nf && fk == kHash);
    done = done || !step;
  }
  if (done) return res;
  for (uint32_t i = kPre;; i++) {
    if (i == nt && i == nf) return true;
    if (i >= nf) return false;
    const uint32_t fi = subst_word(f[i], s);
    if (i < nt && (t[i] == fi || fi == kPlus)) continue;
    return i + 1 == nf && fi == kHash;
  }
}

// kLds: the fixed lists (all / pattern, both types) staged in LDS
template <bool kLds>
__global__ __launch_bounds__(256) void k_acl_check(AArgs a) {
  extern __shared__ uint32_t s_fixed[];
  if (kLds) {
    for (uint32_t i = threadIdx.x; i < a.fixed_words; i += blockDim.x) s_fixed[i] = a.fixed[i];
    __syncthreads();
  }
  const uint32_t* fx = kLds ? s_fixed : a.fixed;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = r < a.n;
  vmqa_req q{};
  if (live) q = a.reqs[r];
  const bool ok = live && q.nwords > 0 && (q.type == VMQA_READ || q.type == VMQA_WRITE);
  if (live && !ok) atomicOr(&a.status[1], kErrReq);
  const uint32_t ty = q.type == VMQA_WRITE ? 1u : 0u;
  const uint32_t* t = a.words + q.word_off;
  uint32_t tw[kPre];
#pragma unroll
  for (uint32_t k = 0; k < kPre; k++) tw[k] = ok && k < q.nwords ? t[k] : 0u;
  bool allowed = false;
  // the three lists of this lane, in check/4's order: all, its user's, pattern
  AList lst[3] = {{0, 0}, {0, 0}, {0, 0}};
  if (ok) {
    lst[0] = a.heads[ty];
    lst[2] = a.heads[2 + ty];
    if (q.user != VMQA_NO_USER) {
      for (uint64_t i = user_hash(q.user, ty) & a.users_mask, n = 0; n <= a.users_mask; i = (i + 1) & a.users_mask, n++) {
        const USlot s = a.users[i];
        if (s.user == kEmpty) break;
        if (s.user == q.user && s.type == ty) { lst[1] = AList{s.off, s.count}; break; }
      }
    }
  }
  const Subst none{false, 0, 0, 0}, pat{true, q.user, q.client, q.mountpoint};
#pragma unroll
  for (int k = 0; k < 3; k++) {
    for (uint32_t i = 0;; i++) {
      const bool act = ok && !allowed && i < lst[k].count;
      if (!__ballot(act)) break;   // every lane of the wave has its verdict, or this list is done
      if (act) {
        if (k == 1) {   // the user's rows: global
          const ARule rule = a.rules[a.lists[lst[k].off + i]];
          allowed = acl_match(tw, t, q.nwords, a.rwords + rule.words_off, rule.nwords, none);
        } else {        // all / pattern rows: the fixed lists
          const uint32_t j = lst[k].off + i;
          allowed = acl_match(tw, t, q.nwords, fx + fx[2 * j + 1], fx[2 * j], k == 2 ? pat : none);
        }
      }
    }
  }
  if (live) a.out[r] = allowed ? 1 : 0;
}

// e0 / e1 (both or neither): recorded by the dispatch itself
hipError_t launch_acl_check(const AArgs& a, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  const uint32_t g = (a.n + 255) / 256;
  if (a.fixed_words <= kFixedLdsWords)
    hipExtLaunchKernelGGL(k_acl_check<true>, dim3(g), dim3(256), (uint32_t)a.fixed_words * 4, st, e0, e1, 0, a);
  else
    hipExtLaunchKernelGGL(k_acl_check<false>, dim3(g), dim3(256), 0, st, e0, e1, 0, a);
  return hipGetLastError();
}

}  // namespace vmqa
