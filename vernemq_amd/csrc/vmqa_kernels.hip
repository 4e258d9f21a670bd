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
// of one type read the same rule, so the `all` and pattern rules are
// broadcast loads; a lane that has its verdict idles until the wave's
// last lane has one.  Integer compares only, no MFMA; bound by the rule
// and topic word loads (L2-resident tables).
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
// id and mountpoint (an undefined user's VMQA_NO_USER equals no word).
__device__ __forceinline__ bool acl_match(const uint32_t* t, uint32_t nt, const uint32_t* f, uint32_t nf, bool subst,
                                          uint32_t user, uint32_t client, uint32_t mp) {
  for (uint32_t i = 0;; i++) {
    if (i == nt && i == nf) return true;
    if (i >= nf) return false;
    uint32_t fi = f[i];
    if (subst) fi = fi == VMQA_WORD_USER ? user : fi == VMQA_WORD_CLIENT ? client : fi == VMQA_WORD_MOUNTPOINT ? mp : fi;
    if (i < nt && (t[i] == fi || fi == kPlus)) continue;
    return i + 1 == nf && fi == kHash;
  }
}

__global__ __launch_bounds__(256) void k_acl_check(AArgs a) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = r < a.n;
  vmqa_req q{};
  if (live) q = a.reqs[r];
  const bool ok = live && q.nwords > 0 && (q.type == VMQA_READ || q.type == VMQA_WRITE);
  if (live && !ok) atomicOr(&a.status[1], kErrReq);
  const uint32_t ty = q.type == VMQA_WRITE ? 1u : 0u;
  const uint32_t* t = a.words + q.word_off;
  bool allowed = false;
  // the three lists of this lane: all, its user's, pattern
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
#pragma unroll
  for (int k = 0; k < 3; k++) {
    for (uint32_t i = 0;; i++) {
      const bool act = ok && !allowed && i < lst[k].count;
      if (!__ballot(act)) break;   // every lane of the wave has its verdict, or this list is done
      if (act) {
        const ARule rule = a.rules[a.lists[lst[k].off + i]];
        allowed = acl_match(t, q.nwords, a.rwords + rule.words_off, rule.nwords, k == 2, q.user, q.client,
                            q.mountpoint);
      }
    }
  }
  if (live) a.out[r] = allowed ? 1 : 0;
}

hipError_t launch_acl_check(const AArgs& a, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  if (e0) hipEventRecord(e0, st);
  k_acl_check<<<(a.n + 255) / 256, 256, 0, st>>>(a);
  if (e1) hipEventRecord(e1, st);
  return hipGetLastError();
}

}  // namespace vmqa
