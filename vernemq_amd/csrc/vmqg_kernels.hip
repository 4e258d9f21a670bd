// HIP kernels for gfx950 (MI355X): the publish -> matched-subscriber path of
// vmq_reg_trie:fold/4 (apps/vmq_server/src/vmq_reg_trie.erl:59-98).
//
// Fast tier — work unit: a GROUP of G lanes owns one publish.  COUNT runs
// one lane per publish (fast_g 1, the default: 64 publishes per wave in
// flight), EMIT two lanes per publish over the same 64-publish chunks
// (fast_g 2 and 4 keep G lanes in both passes).  A group walks the trie from
// an LDS frontier stack — per frontier node the word and '+' edge probes are
// issued as independent 64-B bucket loads before either is resolved (the
// ets:lookup calls of trie_match/4 and 'trie_match_#'/2, :358-383), the '#'
// child read from its alias record — so many frontier nodes and many
// publishes share each memory round trip.  '#' children and end-of-topic
// nodes are compacted (ballot + mbcnt) into an LDS candidate list; their
// node records (match/4, :283-303) give the subscriber-list keys.  The
// exact-topic probe (the `{Topic, node()}` candidate and
// get_remote_subscribers/2, :62, :514-520) is a fingerprint lookup.  Remote
// nodes < 64 are OR-ed into a 64-bit mask: exactly the `Remotes` dedupe of
// fold_/5 (:78-84).  The group lists are interleaved across the block's
// groups with an XOR swizzle, so groups at the same depth hit distinct banks.
//
// Keys per publish: <= 2 go to a 32-B key cache, 3..8 to spill slots; a
// WIDE publish (more keys than that — a $share group hosted on many nodes,
// Q2) keeps only its totals and its candidate paths, marked in its chunk's
// 64-bit mask; the EMIT tail launch expands it again with the whole wave
// (emit_many).  A publish whose (MP, topic) another publish of the batch
// already walks is not walked again (batch-wide dedupe, k_match_fast and
// dedupe_fixup): it takes the representative's key cache and count.
//
// Deferral tiers — a publish whose lists overflow the fast tier's, or that
// meets a remote node >= 64, is retried four lanes per publish (lists 4x
// larger) by the COUNT wave-tier launch; what overflows even those is walked
// by one whole wave with bounded LDS buffers (flushing candidates into keys
// and keys into output as they fill: only the frontier stack needs room,
// bounded by the trie depth; tier 2 puts it in global memory).  The EMIT
// tail launch walks those again and writes them (records and range mode
// alike).  Remote nodes >= 64 go to a 4,096-bit set.  No publish is refused.
//
// Launches per batch: COUNT, COUNT's wave tier (deferred publishes and the
// dedupe fixup; reads its list lengths on the device: empty = ~4 us), the
// one-launch chunk-total scan (decoupled look-back), EMIT, the EMIT tail
// (whole-wave walks, huge publishes, output groups, wide publishes; empty =
// ~4 us).  Every hand-off of payload between workgroups crosses one of these
// launch boundaries.  Output is either the 16-B records (lookup_subs +
// fold__, :87-98) or, in range mode, one 8-B {record off, count} per
// non-empty subscriber-list key plus {node, 0} per remote node.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "vmqg_common.h"
#include "vmqg_kernels.h"
#include "vmqg_lookback.h"

namespace vmqg {

constexpr int kWaves = 4;          // waves per 256-thread block
#ifndef VMQG_EXACT_FILTER
#define VMQG_EXACT_FILTER 1        // A/B: 0 = always probe the exact table
#endif
#ifndef VMQG_EMIT_U
#define VMQG_EMIT_U 8              // records in flight per lane in the fast EMIT copy (A/B: 2, 4, 8)
#endif
// fast-tier LDS lists per group, sized so a block stays near 28 KiB
template <int G> struct FastCaps { static constexpr uint32_t S = 8 * G, C = 4 * G, K = 4 * G; };
#ifndef VMQG_SPILL_KEYS
#define VMQG_SPILL_KEYS 8                   // A/B: 2 = no spill (every publish with > 2 keys is re-walked)
#endif
constexpr uint32_t kSpillKeys = 8;          // spill slots per publish (more keys: re-walk)
constexpr uint32_t kDeferred = 0xFFFFFFFEu; // key cache: the wave tier owns the publish
constexpr uint32_t kMany = 0xFFFFFFFDu;     // key cache: more keys than the lists hold; EMIT expands the
                                            // candidates COUNT left in the spill slots, wave-wide

// Per-call status counters (a.status; two sets used by alternate calls: each
// call's first kernel zeroes the set of the call after it, so no reset
// launch is needed) and the sticky error word (a.err, cleared only by
// vmqg_match_status).
// Publish lists (a.deferred, kLists x npub entries): [0, npub) publishes the
// fast pass could not hold (retried four lanes per publish by the COUNT
// wave-tier launch), [npub, 2 npub) publishes walked by a whole wave,
// [2 npub, 3 npub) duplicates of a batch-wide dedupe representative,
// [3 npub, 4 npub) their dedupe-table slots and [4 npub, 5 npub) the huge
// publishes (records mode, >= kHugeRecords records: copied by every wave of
// the EMIT tail, a segment each).
constexpr uint32_t kLists = 5;
#ifndef VMQG_HUGE_RECORDS
#define VMQG_HUGE_RECORDS 65536
#endif
constexpr uint32_t kHugeRecords = VMQG_HUGE_RECORDS;
constexpr uint32_t kHugeFlag = 0x40000000u;  // key cache word 1 (nk <= 8): a huge publish, the tail copies it
#ifndef VMQG_WALK_U
#define VMQG_WALK_U 4   // records in flight per lane in a whole-wave walk's copy (8: the tail at 151 VGPRs, 3 waves/SIMD; 4: 128, 4)
#endif
#ifndef VMQG_DD_ON_PCT
#define VMQG_DD_ON_PCT 50   // dedupe auto mode: on while more than this % of the sampled publishes repeat
#endif
#ifndef VMQG_TAIL_U
#define VMQG_TAIL_U 8   // records in flight per lane in the tail's copies (wide, grouped, huge)
#endif
constexpr uint32_t kHugeSeg = 64 * 8 * 4;     // records per tail wave and segment
// Output groups (records mode): publishes of >= kGroupMin records with <= 2
// keys or wide are grouped by a signature of what they emit (key cache, or
// candidates + exact key + remote nodes + the '$' flag) into slots of
// kGroupCap; the EMIT tail writes a slot's members back to back from one
// wave, so their source lists are read from HBM once per slot and from that
// CU's L1 / L2 for the rest (config D: every site/s/x/alarm/z publish copies
// site s's 1,000-record list, every jobs/q/x publish queue q's 40 keys).
#ifndef VMQG_GROUP_MIN
#define VMQG_GROUP_MIN 128
#endif
constexpr uint32_t kGroupMin = VMQG_GROUP_MIN;
constexpr uint32_t kGroupCap = 60;
constexpr uint32_t kGroupFlag = 0x20000000u;  // key cache word 1 (nk <= 2): a grouped publish, the tail writes it
// Heavy publishes (records mode, a.heavy_min > 0): >= heavy_min records from
// <= 2 keys.  Their sources are lists many publishes share (config D: site
// s's 1,000 alarm records for every site/s/x/alarm/z publish); copied by the
// fast EMIT, each is fetched into whichever XCD's L2 the chunk lands on, so
// every XCD pulls every list (3.4 GB fetched for 4.2 GB written per batch).
// COUNT buckets them by their first key (kXcds buckets, one per XCD: a byte
// per publish, 1 + bucket, 0 for the others) and the EMIT tail's blocks
// b ≡ x (mod 8) — which run on XCD x (profiles/xcd_probe_r04.txt) — copy
// bucket x: each list is read into one L2.
constexpr uint32_t kHeavyFlag = 0x10000000u;  // key cache word 1 (nk <= 2): a heavy publish, the tail copies it
constexpr uint32_t kXcds = 8;
__device__ __forceinline__ uint32_t heavy_bucket(uint32_t off0) { return (off0 * 0x9E3779B1u) >> 29; }   // top 3 bits
struct alignas(16) GroupSlot {
  unsigned long long word;   // {call tag: 24, signature: 32, members: 8}
  uint32_t pad[2];
  uint32_t m[kGroupCap];     // member publishes
};
static_assert(sizeof(GroupSlot) == 256, "");
// progress words of the calling wave (VMQG_DEBUG_SYNC diagnosis; a.dbg null otherwise)
#define DBGW(slot, v)                                                                                        \
  do {                                                                                                       \
    if (a.dbg)                                                                                               \
      __hip_atomic_store(a.dbg + ((uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6)) * 8 + (slot), (uint32_t)(v), \
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);                                       \
  } while (0)
enum : uint32_t { kStDeferred = 0, kStTier2 = 1, kStTicket = 2, kStWalked = 3, kStMany = 4, kStWalkOvf = 5,
                  kStWaveEnt = 6 /* u64: entries written by the EMIT wave tier (whole-wave walks) */,
                  kStWideEnt = 24 /* u64: entries written for wide publishes by the EMIT tail */,
                  kStDup = 8 /* duplicates listed for the fixup */, kStDupTried = 9 /* publishes probed */,
                  kStDupWalked = 10 /* duplicates walked after all (representative deferred / words differ) */,
                  kStHuge = 11 /* huge publishes listed for the tail */,
                  kStGrouped = 12 /* publishes in output groups */,
                  kStReps = 13 /* dedupe on: publishes COUNT walks (list 2) */,
                  kStHeavy = 17 /* heavy publishes the EMIT tail copies by XCD */,
                  kStWords = 32 };
#ifndef VMQG_WIDE_RECORDS
#define VMQG_WIDE_RECORDS 0x7fffffff   // A/B: a publish with at least this many records is wide too (256: config D 2,724 vs 2,526 us per batch, off)
#endif
enum : uint32_t { kErrFrontier = 2u, kErrOverflow = 4u, kErrMismatch = 8u };   // kErrLookback = 16 (lookback.h)

__device__ __forceinline__ uint32_t prefix_bits(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// G consecutive lanes of a wavefront acting as one unit.
template <int G>
struct Group {
  uint32_t lane, gidx;
  uint64_t mask;
  __device__ Group() {
    const uint32_t l = __lane_id();
    lane = l % G;
    gidx = l / G;
    mask = G == 64 ? ~0ull : (((1ull << G) - 1) << (gidx * G));
  }
  __device__ uint64_t ballot(bool p) const { return __ballot(p) & mask; }
  __device__ uint32_t incl_scan(uint32_t v) const {
#pragma unroll
    for (int o = 1; o < G; o <<= 1) {
      const uint32_t t = __shfl_up(v, o, G);
      if (lane >= (uint32_t)o) v += t;
    }
    return v;
  }
  __device__ uint32_t last(uint32_t v) const { return __shfl(v, G - 1, G); }
  __device__ uint32_t bcast(uint32_t v, uint32_t src) const { return __shfl(v, (int)src, G); }
  __device__ uint64_t or64(uint64_t v) const {
#pragma unroll
    for (int o = G / 2; o >= 1; o >>= 1) {
      const uint32_t lo = __shfl_xor((uint32_t)v, o, G), hi = __shfl_xor((uint32_t)(v >> 32), o, G);
      v |= ((uint64_t)hi << 32) | lo;
    }
    return v;
  }
  __device__ uint64_t sum64(uint64_t v) const {
#pragma unroll
    for (int o = G / 2; o >= 1; o >>= 1) {
      const uint32_t lo = __shfl_xor((uint32_t)v, o, G), hi = __shfl_xor((uint32_t)(v >> 32), o, G);
      v += ((uint64_t)hi << 32) | lo;
    }
    return v;
  }
  __device__ uint32_t max32(uint32_t v) const {
#pragma unroll
    for (int o = G / 2; o >= 1; o >>= 1) { const uint32_t t = __shfl_xor(v, o, G); v = t > v ? t : v; }
    return v;
  }
};

__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

// Wave-uniform values as the compiler sees them (scalar registers): loops
// and branches on them are scalar branches, so no lane can leave a ticket
// loop on its own.  (A ticket loop whose exit the compiler took for
// divergent hung the wide phase: lane 0, the one taking the tickets, left
// it while the other lanes kept reading ticket 0.)
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}
// One ticket per wave, taken by its first active lane.
__device__ __forceinline__ uint32_t wave_ticket(uint32_t* ctr) {
  uint32_t t = 0;
  if (__lane_id() == uni(__lane_id())) t = atomicAdd(ctr, 1u);
  return uni(t);
}

__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t v) {
  const uint32_t lane = __lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o, 64);
    if (lane >= (uint32_t)o) v += t;
  }
  return v;
}

__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v) {
  const uint32_t lane = __lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t t = __shfl_up(v, o, 64);
    if (lane >= (uint32_t)o) v += t;
  }
  return v;
}

// ---------------------------------------------------------------- probes
struct Bucket { uint4 s0, s1, s2, s3; };

__device__ __forceinline__ Bucket load_bucket(const EdgeSlot* t, uint64_t b) {
  const uint4* p = reinterpret_cast<const uint4*>(t + b * kEdgeSlotsPerBucket);
  return Bucket{p[0], p[1], p[2], p[3]};
}

// 1 = found (child + the child's edge flags set), 0 = absent (an empty slot
// ends the chain), 2 = go on with the next bucket
__device__ __forceinline__ int scan_bucket(const Bucket& B, uint32_t parent, uint32_t word, uint32_t& child,
                                           uint32_t& cflags) {
  if (B.s0.x == parent && B.s0.y == word) { child = B.s0.z; cflags = B.s0.w; return 1; }
  if (B.s1.x == parent && B.s1.y == word) { child = B.s1.z; cflags = B.s1.w; return 1; }
  if (B.s2.x == parent && B.s2.y == word) { child = B.s2.z; cflags = B.s2.w; return 1; }
  if (B.s3.x == parent && B.s3.y == word) { child = B.s3.z; cflags = B.s3.w; return 1; }
  if (B.s0.x == kEmpty || B.s1.x == kEmpty || B.s2.x == kEmpty || B.s3.x == kEmpty) return 0;
  return 2;
}

// Continue a probe chain from bucket b+1 (rare: the first bucket was full).
__device__ __noinline__ uint2 probe_rest(const EdgeSlot* t, uint64_t mask, uint64_t b, uint32_t parent,
                                         uint32_t word) {
  for (uint64_t i = 0; i < mask; i++) {
    b = (b + 1) & mask;
    uint32_t c = kNone, f = 0;
    const int r = scan_bucket(load_bucket(t, b), parent, word, c, f);
    if (r == 1) return make_uint2(c, f);
    if (r == 0) break;
  }
  return make_uint2(kNone, 0u);
}

__device__ __forceinline__ void probe(const EdgeSlot* t, uint64_t mask, uint64_t b, const Bucket& B,
                                      uint32_t parent, uint32_t word, uint32_t& child, uint32_t& cflags) {
  if (scan_bucket(B, parent, word, child, cflags) == 2) {
    const uint2 r = probe_rest(t, mask, b, parent, word);
    child = r.x;
    cflags = r.y;
  }
}

constexpr uint32_t kDepthMask = 0x0FFFFFFFu;   // frontier entry: {path, depth | child flags << 28}
constexpr uint32_t kUnresolved = 0xFFFFFFFFu;  // key list entry still holds a key id

// One step of trie_match/4 + 'trie_match_#'/2 (vmq_reg_trie.erl:358-383) for
// up to G frontier entries, one per lane: the word and '+' edge probes,
// issued before either is resolved; the '#' child is its aliased record.  The node's cached edge flags (`fl`) skip '#' / '+'
// / literal probes that must miss.
struct StepOut { uint32_t hc, wc, pc, wf, pf; bool at_end; };

template <int G>
__device__ __forceinline__ StepOut probe_step(const MatchArgs& a, const Group<G>& g, bool act, uint32_t node,
                                              uint32_t d, uint32_t fl, uint32_t L, const uint32_t* w,
                                              uint32_t wreg) {
  const bool at_end = act && d == L;
  const uint32_t wsh = g.bcast(wreg, d % G);   // all group lanes take part
  uint32_t wd = kUnknownWord;
  if (act && !at_end) wd = d < (uint32_t)G ? wsh : w[d];
  const bool do_h = act && (fl & kHasHash);
  // the W probe of [W, <<"+">>] (:366-375) for any word the dictionary has:
  // a publish word equal to '+' (or '#') probes that edge literally — so a
  // '+' word follows the '+' edge twice, as the reference's foldl does (a
  // plugin publish's Topic reaches fold/4 unvalidated, vmq_reg.erl:572-594)
  const uint32_t wneed = wd == kPlus ? kHasPlus : wd == kHash ? kHasHash : kHasWord;
  const bool do_w = act && !at_end && (fl & wneed) && wd != kUnknownWord;
  const bool do_p = act && !at_end && (fl & kHasPlus);
  const uint64_t bw = edge_hash(node, wd) & a.edge_mask;
  const uint64_t bp = edge_hash(node, kPlus) & a.edge_mask;
  Bucket Bw{}, Bp{};
  if (do_w) Bw = load_bucket(a.edges, bw);
  if (do_p) Bp = load_bucket(a.edges, bp);
#ifndef VMQG_HASH_ALIAS
#define VMQG_HASH_ALIAS 1   // A/B: 0 = probe the '#' edge and read the child's own record
#endif
#if VMQG_HASH_ALIAS
  // the '#' child: no probe, its record is aliased at node_cap + node
  StepOut o{do_h ? (uint32_t)(a.node_cap + node) : kNone, kNone, kNone, 0, 0, at_end};
#else
  const uint64_t bh = edge_hash(node, kHash) & a.edge_mask;
  Bucket Bh{};
  if (do_h) Bh = load_bucket(a.edges, bh);
  StepOut o{kNone, kNone, kNone, 0, 0, at_end};
  uint32_t hf = 0;
  if (do_h) probe(a.edges, a.edge_mask, bh, Bh, node, kHash, o.hc, hf);
#endif
  if (do_w) probe(a.edges, a.edge_mask, bw, Bw, node, wd, o.wc, o.wf);
  if (do_p) probe(a.edges, a.edge_mask, bp, Bp, node, kPlus, o.pc, o.pf);
  return o;
}

// The child flags of a mountpoint's root (its own record caches them: a
// root has no incoming edge slot); a trie-less mountpoint (R1: exact
// subscriptions only) then walks nothing.
__device__ __forceinline__ uint32_t root_flags(const MatchArgs& a, uint32_t mp) {
  if (!(a.opts & kOptRootFlags)) return kHasAll;
  return (a.nodes[mp].meta >> kRootFlagShift) & kHasAll;
}

// Exact-topic fingerprint of the publish, computed by the G lanes of a group;
// `wild`: the publish holds a '+' / '#' word (only a wildcard topic, which
// has no filter bit, can equal it).
template <int G>
__device__ __forceinline__ uint64_t publish_fp(const vmqg_pub& pub, const uint32_t* w, uint32_t wreg,
                                               const Group<G>& g, bool& wild) {
  const uint32_t L = pub.nwords;
  uint64_t part = 0;
  bool wl = false;
  for (uint32_t i = g.lane; i < L; i += G) {
    const uint32_t x = i < (uint32_t)G ? wreg : w[i];
    part += fp_word(x, i);
    wl |= x == kPlus || x == kHash;
  }
  wild = g.ballot(wl) != 0;
  return fp_final(g.sum64(part), pub.mountpoint, L);
}

// The exact slot of (MP, Topic), or null: fingerprint probe, then the MP and
// words compared group-parallel — the slot holds the first 7 words (one
// 128-B line verifies a topic of <= 7 words), exwords the rest.  `xst`
// (COUNT's fast pass counts it): 1 looked up, 2 the table probed, 4 found.
// The exbits filter (a.exfilter) saves the table's line for a publish with
// no exact topic but costs its own line for one with; the COUNT wave tier
// turns it off while most lookups pass it and on while most miss (exmode).
template <int G>
__device__ const ExactSlot* find_exact(const MatchArgs& a, const vmqg_pub& pub, const uint32_t* w, uint32_t wreg,
                                       const Group<G>& g, uint32_t& xst, bool use_filter) {
  const uint32_t L = pub.nwords;
  bool wild;
  const uint64_t fp = publish_fp<G>(pub, w, wreg, g, wild);
  xst = wild ? 0u : 1u;
#if VMQG_EXACT_FILTER
  // the filter's bit (an L2-resident word) before the table's random line
#ifndef VMQG_EXFILTER_RUNTIME
#define VMQG_EXFILTER_RUNTIME 1   // A/B: 0 = the filter always on (no runtime switch)
#endif
  if ((!VMQG_EXFILTER_RUNTIME || use_filter) && !wild) {
    const uint64_t xb = exbit_of(fp, a.exbits_mask + 1);
    if (!((a.exbits[xb >> 5] >> (xb & 31)) & 1u)) return nullptr;
  }
#endif
  xst |= 2u;
  uint64_t b = fp & a.exact_mask;
  for (uint64_t iter = 0; iter <= a.exact_mask; iter++) {
    const ExactSlot* bk = a.exact + b * kExactSlotsPerBucket;
    bool seen_empty = false;
    // one slot at a time: each 64-B slot is a memory request of its own, so
    // the second is read only when the first is not the topic
#pragma unroll 1
    for (uint32_t j = 0; j < kExactSlotsPerBucket; j++) {
      const ExactSlot& e = bk[j];
      const uint4 h = *reinterpret_cast<const uint4*>(&e);   // {fp lo, fp hi, nwords, words_off}
      const uint32_t nw = h.z;
      if (nw == kEmpty) { seen_empty = true; break; }
      if ((((uint64_t)h.y << 32) | h.x) != fp || (nw & ~kExactFlags) != L || e.mp != pub.mountpoint) continue;
      // inline words, then the rest (two loops: one loop selecting between
      // the two loads costs the one-lane COUNT 16 B of scratch spills)
      bool diff = false;
      const uint32_t Li = L < kExactInline ? L : kExactInline;
      for (uint32_t i = g.lane; i < Li; i += G) diff |= e.w[i] != (i < (uint32_t)G ? wreg : w[i]);
      uint32_t i1 = g.lane;
      if (i1 < kExactInline) i1 += (kExactInline - i1 + G - 1) / G * G;
      for (uint32_t i = i1; i < L; i += G) diff |= a.exwords[e.words_off + (i - kExactInline)] != (i < (uint32_t)G ? wreg : w[i]);
      if (g.ballot(diff) == 0) { xst |= 4u; return &e; }
    }
    if (seen_empty) break;
    b = (b + 1) & a.exact_mask;
  }
  return nullptr;
}
template <int G>
__device__ __forceinline__ const ExactSlot* find_exact(const MatchArgs& a, const vmqg_pub& pub, const uint32_t* w,
                                                       uint32_t wreg, const Group<G>& g, uint32_t& xst) {
  return find_exact<G>(a, pub, w, wreg, g, xst, a.exfilter != 0);
}

// ============================================================== fast tier
// A group's three lists live in LDS interleaved over the block's SLOTS
// groups: entry i of group `slot` sits at i * SLOTS + (slot ^ swz(i)), the
// XOR moving the G consecutive entries a group touches at once onto
// different banks, so neither the G lanes of a group nor groups at the same
// depth conflict (SLOTS is a multiple of 32).
// SLOTS_ = GPW: one wave's groups only (the fused scan's per-wave slices).
template <int G, uint32_t SLOTS_ = kWaves * (64 / G)>
struct FastScratch {
  static constexpr uint32_t GPW = 64 / G, SLOTS = SLOTS_;
  // 32 / G = 1 << SH, or SLOTS / G when the lists hold one wave's groups
  static constexpr uint32_t SH0 = G == 1 ? 5 : G == 2 ? 4 : G == 4 ? 3 : 2;
  static constexpr uint32_t SH = (32u / G) <= SLOTS / G ? SH0 : (SLOTS / G == 4 ? 2 : SLOTS / G == 2 ? 1 : 0);
  static constexpr uint32_t SC = FastCaps<G>::S, CC = FastCaps<G>::C, KC = FastCaps<G>::K;
  uint2* stack; uint32_t* cand; uint2* keys;
  uint32_t slot;
  __device__ uint32_t at(uint32_t i) const { return i * SLOTS + (slot ^ ((i & (G - 1)) << SH)); }
  __device__ uint2& st(uint32_t i) const { return stack[at(i)]; }
  __device__ uint32_t& cd(uint32_t i) const { return cand[at(i)]; }
  __device__ uint2& ky(uint32_t i) const { return keys[at(i)]; }
};

// Per-publish result of the walk: keys[0..nk) hold {record off, cum start}.
struct Matched {
  uint32_t nk, nkr, ksum, total_rec;   // keys, non-empty keys, records, record-mode total
  uint64_t rmask;
  bool overflow;                        // the lists overflowed or a node >= 64: the wave tier takes it
  bool walk_ovf;                        // ... because the frontier or candidate list overflowed
  bool many;                            // more keys than the key list holds: totals only (nk, keys unset);
  uint32_t nc, ex_off, ex_cnt;          // the candidates stay in the LDS list, the exact key is {ex_off, ex_cnt}
};

// Records and non-empty keys of one multi-key candidate (its keylist ids ->
// keydesc counts), for the many-key totals.
__device__ __forceinline__ void sum_keys(const MatchArgs& a, uint32_t key, uint32_t n, uint32_t& sum, uint32_t& nkr) {
#if VMQG_SUM_UNROLL
#pragma unroll 4
#else
#pragma unroll 1
#endif
  for (uint32_t j = 0; j < n; j++) {
    const uint32_t kid = a.keylist[key + j];
    const uint32_t c = kid < a.key_cap ? a.keydesc[kid].count : 0u;
    sum += c;
    nkr += c != 0;
  }
}

template <int G, uint32_t SL>
__device__ Matched walk_publish(const MatchArgs& a, const vmqg_pub& pub, const FastScratch<G, SL>& s,
                                const Group<G>& g) {
  const uint32_t L = pub.nwords;
  const uint32_t* w = a.words + pub.word_off;
  const bool dollar = (pub.flags & VMQG_PUB_DOLLAR) != 0;
  const bool mp_ok = pub.mountpoint < a.max_mp;   // L == 0: the root alone (trie_match/4 :361-363)
  // lane i of the group keeps word i (i < G); deeper words come from memory
  const uint32_t wreg = g.lane < L ? w[g.lane] : kUnknownWord;
  Matched m{0, 0, 0, 0, 0, false, false, false, 0, 0, 0};
  uint32_t nc = 0, sp = 0;
  if (mp_ok) {
    if (g.lane == 0) s.st(0) = make_uint2(pub.mountpoint, root_flags(a, pub.mountpoint) << 28);   // {MP, root}
    sp = 1;
  }
  wave_sync();

  // ---- trie_match/4 + 'trie_match_#'/2  (vmq_reg_trie.erl:358-383)
  while (sp > 0) {
    const uint32_t k = sp < (uint32_t)G ? sp : (uint32_t)G;
    const uint32_t base = sp - k;
    const bool act = g.lane < k;
    uint32_t node = 0, d = 0, fl = 0;
    if (act) { const uint2 e = s.st(base + g.lane); node = e.x; d = e.y & kDepthMask; fl = e.y >> 28; }
    sp = base;
    wave_sync();
    const StepOut o = probe_step<G>(a, g, act, node, d, fl, L, w, wreg);
    // candidates: the '#' child (:377-383) and, with no words left, the node itself (:361-363)
    const uint64_t m_hc = g.ballot(o.hc != kNone), m_end = g.ballot(o.at_end);
    const uint32_t n_hc = (uint32_t)__popcll(m_hc), n_new_c = n_hc + (uint32_t)__popcll(m_end);
    // frontier: the W and '+' children (:364-375)
    const uint64_t m_wc = g.ballot(o.wc != kNone), m_pc = g.ballot(o.pc != kNone);
    const uint32_t n_pc = (uint32_t)__popcll(m_pc), n_new_s = n_pc + (uint32_t)__popcll(m_wc);
    if (nc + n_new_c > s.CC || sp + n_new_s > s.SC) { m.overflow = m.walk_ovf = true; break; }
    if (o.hc != kNone) s.cd(nc + prefix_bits(m_hc)) = o.hc;
    if (o.at_end) s.cd(nc + n_hc + prefix_bits(m_end)) = node;
    nc += n_new_c;
    if (o.pc != kNone) s.st(sp + prefix_bits(m_pc)) = make_uint2(o.pc, (d + 1) | (o.pf << 28));
    if (o.wc != kNone) s.st(sp + n_pc + prefix_bits(m_wc)) = make_uint2(o.wc, (d + 1) | (o.wf << 28));
    sp += n_new_s;
    wave_sync();
  }

  // ---- candidates -> subscriber-list keys: match/4, match_/3 (:283-303)
  // Keys go to the LDS key list; a publish with more keys than it holds
  // (a $share filter hosted on many nodes: one key per {Node, Group} entry,
  // :68-72) switches to many-key mode: only its totals are kept here, and
  // EMIT expands the candidates again, wave-wide.
  uint64_t rmask = 0;
  uint32_t nk = 0;
  uint32_t msum = 0, mnkr = 0;   // many-key mode: this lane's records / non-empty keys
  // into many-key mode: the keys listed so far become totals
  auto to_many = [&]() {
    m.many = true;
    for (uint32_t i = g.lane; i < nk; i += G) {
      const uint2 e = s.ky(i);
      uint32_t c = e.y;
      if (e.y == kUnresolved) c = e.x < a.key_cap ? a.keydesc[e.x].count : 0u;
      msum += c;
      mnkr += c != 0;
    }
  };
  if (!m.overflow) {
    for (uint32_t c0 = 0; c0 < nc; c0 += G) {
      const uint32_t ci = c0 + g.lane;
      uint32_t nkeys = 0, key = kNone, off0 = 0, cnt0 = 0;
      bool high = false;
      if (ci < nc) {
        const uint32_t path = s.cd(ci);
        if (path < 2 * a.node_cap) {   // own records, then '#' aliases
          const uint4 r = *reinterpret_cast<const uint4*>(a.nodes + path);
          const uint2 r2 = *reinterpret_cast<const uint2*>(&a.nodes[path].off0);
          const bool valid = (r.x & kNodeEmits) == kNodeEmits &&
                             !(dollar && (r.x & kNodeDollarSkip));   // MQTT-4.7.2-1 (:285-288)
          if (valid) {
            nkeys = (r.x >> 8) & 0xFFFFFFu;
            key = r.y;
            off0 = r2.x;
            cnt0 = r2.y;
            rmask |= ((uint64_t)r.w << 32) | r.z;
            high = (r.x & kNodeHigh) != 0;
          }
        }
      }
      const uint32_t incl = g.incl_scan(nkeys);
      const uint32_t tot = g.last(incl);
      if (g.ballot(high) != 0) { m.overflow = true; break; }
      if (!m.many && nk + tot > s.KC) to_many();
      if (!m.many) {
        const uint32_t at = nk + incl - nkeys;
        if (nkeys == 1) s.ky(at) = make_uint2(off0, cnt0);   // resolved inline
        else for (uint32_t j = 0; j < nkeys; j++) s.ky(at + j) = make_uint2(a.keylist[key + j], kUnresolved);
      } else if (nkeys == 1) {
        msum += cnt0;
        mnkr += cnt0 != 0;
      } else if (nkeys > 1) {
        sum_keys(a, key, nkeys, msum, mnkr);
      }
      nk += tot;
      wave_sync();
    }
  }
  wave_sync();

  // ---- the exact candidate {Topic, node()} and remote exact subscribers (:62, :514-520)
  if (!m.overflow && mp_ok) {
    uint32_t xst;
    const ExactSlot* e = find_exact<G>(a, pub, w, wreg, g, xst);
    if (e) {
      const uint4 q = *reinterpret_cast<const uint4*>(&e->off);   // {off, count, rmask lo, hi}
      rmask |= ((uint64_t)q.w << 32) | q.z;
      if (e->nwords & kExactHigh) m.overflow = true;
      else if (q.y != 0) {
        if (!m.many && nk + 1 > s.KC) to_many();
        m.ex_off = q.x;
        m.ex_cnt = q.y;
        if (m.many) {
          if (g.lane == 0) { msum += q.y; mnkr += 1; }
        } else if (g.lane == 0) {
          s.ky(nk) = make_uint2(q.x, q.y);
        }
        nk += 1;
      }
    }
  }
  wave_sync();
  m.rmask = g.or64(rmask);
  if (a.local_node < kLowNodes) m.rmask &= ~(1ull << a.local_node);
  if (m.overflow) return m;
  if (m.many) {   // totals only; the candidates stay in the LDS list for COUNT to spill
    m.nc = nc;
    m.nk = nk;
    m.ksum = (uint32_t)g.sum64(msum);
    m.nkr = (uint32_t)g.sum64(mnkr);
    m.total_rec = m.ksum + (uint32_t)__popcll(m.rmask);
    return m;
  }

  m.nc = nc;
  // ---- record ranges per key: lookup_subs/1 (:87-94)
  uint32_t ksum = 0, nkr = 0;
  for (uint32_t k0 = 0; k0 < nk; k0 += G) {
    const uint32_t ki = k0 + g.lane;
    uint32_t cnt = 0, off = 0;
    if (ki < nk) {
      const uint2 e = s.ky(ki);
      if (e.y != kUnresolved) { off = e.x; cnt = e.y; }
      else if (e.x < a.key_cap) { const uint2 kd = *reinterpret_cast<const uint2*>(a.keydesc + e.x); off = kd.x; cnt = kd.y; }
    }
    const uint32_t incl = g.incl_scan(cnt);
    nkr += (uint32_t)__popcll(g.ballot(cnt != 0));
    wave_sync();
    if (ki < nk) s.ky(ki) = make_uint2(off, ksum + incl - cnt);
    ksum += g.last(incl);
  }
  wave_sync();
  m.nk = nk;
  m.nkr = nkr;
  m.ksum = ksum;
  m.total_rec = ksum + (uint32_t)__popcll(m.rmask);
  return m;
}

// Output entries of a publish: records (OUT 0) or ranges (OUT 1).
template <int OUT>
__device__ __forceinline__ uint32_t out_total(const Matched& m) {
  return OUT ? m.nkr + (uint32_t)__popcll(m.rmask) : m.total_rec;
}

// j-th set bit of m (j < popcount(m))
__device__ __forceinline__ uint32_t select_bit(uint64_t m, uint32_t j) {
  for (; j > 0; j--) m &= m - 1;
  return (uint32_t)__builtin_ctzll(m);
}

// r-th emission of a publish whose keys are {off, cum start} in `ks`.
template <class Keys>
__device__ __forceinline__ uint4 emission(const MatchArgs& a, const Keys& ks, uint32_t nk, uint32_t ksum,
                                          uint64_t rmask, uint32_t r) {
  if (r < ksum) {
    uint32_t lo = 0, hi = nk;   // last key whose cumulative start <= r
    while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (ks(mid).y <= r) lo = mid; else hi = mid; }
    const uint2 kk = ks(lo);
    return *reinterpret_cast<const uint4*>(a.records + kk.x + (r - kk.y));
  }
  // j-th remote node of the mask, in node order (fold_/5 :78-84)
  return make_uint4((VMQG_EMIT_REMOTE << 24) | select_bit(rmask, r - ksum), kNone, kNone, kNone);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void store_rec(Record* out, uint64_t i, uint4 v) {
  if (NT) {
    u32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(out + i));
  } else {
    *reinterpret_cast<uint4*>(out + i) = v;
  }
}

__device__ __forceinline__ void store_range(vmqg_range* out, uint64_t i, uint32_t off, uint32_t count) {
  *reinterpret_cast<uint2*>(out + i) = make_uint2(off, count);
}

// ------------------------------------------------------------ COUNT pass
// Returns the publish's count on the group's lane 0 (0 when deferred: a
// later tier adds it to the chunk total), 0 on the other lanes; `fl` (lane
// 0) says how it was served: 0 fast tier, 1 many-key mode, 2 deferred by a
// walk overflow, 3 deferred otherwise (remote nodes >= 64).  Deferred
// publishes go to list RETRY ? 2 (whole-wave walks) : 0 (the 4-lane retry).
__device__ __forceinline__ unsigned long long dd_key_of(const MatchArgs& a, uint64_t fp) {
  return ((unsigned long long)a.dd_tag << 40) | (fp >> 24);
}

// Output-group signatures: what a publish emits.  <= 2 keys: its key-cache
// word {off0, c0, off1, c1} and remote mask; wide: its candidates, exact
// key, remote mask and '$' flag (the order-relevant inputs of emit_many).
__device__ __forceinline__ uint64_t group_sig_keys(uint4 w1, uint64_t rmask) {
  return mix64(mix64(((uint64_t)w1.x << 32) | w1.y) ^ (((uint64_t)w1.z << 32) | w1.w)) ^ rmask;
}
template <class CandFn>
__device__ __forceinline__ uint64_t group_sig_many(uint32_t ex_off, uint32_t ex_cnt, bool dollar, uint64_t rmask,
                                                   uint32_t nc, CandFn cand) {
  uint64_t sig = mix64(((uint64_t)ex_off << 32) ^ ex_cnt ^ ((uint64_t)dollar << 63));
  sig = mix64(sig ^ rmask) ^ nc;
  for (uint32_t i = 0; i < nc; i++) sig = mix64(sig + cand(i));
  return sig;
}

// Joins publish p to the output group of signature `sig` (a slot with room,
// or a new one claimed by CAS; full slots chain to the next).  One lane.
__device__ bool group_insert(const MatchArgs& a, uint64_t sig64, uint32_t p) {
  GroupSlot* gs = reinterpret_cast<GroupSlot*>(a.groups);
  const unsigned long long T = (unsigned long long)a.dd_tag << 40;
  const uint32_t sig = (uint32_t)(sig64 >> 32);
  uint64_t i = sig64 & a.gs_mask;
  for (uint32_t probe = 0; probe < 32; probe++, i = (i + 1) & a.gs_mask) {
    unsigned long long* wp = &gs[i].word;
    unsigned long long w = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      if ((w >> 40) != a.dd_tag) {   // a slot of an older call: claim it as member 0
        const unsigned long long prev = atomicCAS(wp, w, T | ((unsigned long long)sig << 8) | 1ull);
        if (prev == w) { gs[i].m[0] = p; return true; }
        w = prev;
        continue;
      }
      if ((uint32_t)(w >> 8) != sig) break;                 // another signature
      const uint32_t n = (uint32_t)(w & 0xFF);
      if (n >= kGroupCap) break;                            // full: the chain goes on in the next slot
      const unsigned long long prev = atomicCAS(wp, w, w + 1);
      if (prev == w) { gs[i].m[n] = p; return true; }
      w = prev;
    }
  }
  return false;   // no room: EMIT writes it as usual
}

// Block-level aggregation of COUNT's fast pass (one global atomic per block
// and counter, not per wave or per publish: 16,384 waves adding to ONE word
// take 200 us serialised on MI355X, spread over 64 words 9 us —
// tools/atomic_probe.hip, profiles/atomic_probe_r04.jsonl).  The deferred
// publishes are buffered in LDS and appended to list 0 with one atomic per
// block at the end (a full buffer falls back to the global counter).
constexpr uint32_t kDefBuf = 509;
struct CountAgg {
  uint32_t many, walkovf, grouped, pad0;    // per-block sums of the status counters
  uint32_t ndef, base;                      // buffered deferred publishes; their list-0 base
  uint32_t pad1, pad2;
  uint32_t heavy;                           // heavy publishes marked for the EMIT tail
  uint32_t def[kDefBuf];
};

// FEAT: batch dedupe and output groups compiled in (the COUNT variant the
// host picks when either is on: their code costs the lean variant scratch
// spills, 79 -> 90 us on config C)
template <int G, int OUT, bool RETRY = false, uint32_t SL = kWaves * (64 / G), bool FEAT = true>
__device__ uint32_t count_publish(const MatchArgs& a, uint32_t p, const FastScratch<G, SL>& s, const Group<G>& g,
                                  uint32_t& fl, CountAgg* agg = nullptr) {
  const vmqg_pub pub = a.pubs[p];
  const Matched m = walk_publish<G, SL>(a, pub, s, g);
  fl = 0;
  // wide publishes — more keys than the spill slots hold — are written by a
  // whole wave in the EMIT tail launch, expanded again from their candidates
  const bool many = !m.overflow && (m.many || m.nk > VMQG_SPILL_KEYS || m.ksum >= VMQG_WIDE_RECORDS);
  // 3..8 keys: the group copies its key list to the publish's spill slots
  const bool spill = !m.overflow && !many && m.nk > 2;
  if (spill)
    for (uint32_t i = g.lane; i < m.nk; i += G) a.keyspill[(uint64_t)p * kSpillKeys + i] = s.ky(i);
  // many keys: the candidate paths (<= FastCaps::C <= 16 words) instead
  if (many)
    for (uint32_t i = g.lane; i < m.nc; i += G)
      reinterpret_cast<uint32_t*>(a.keyspill)[(uint64_t)p * 2 * kSpillKeys + i] = s.cd(i);
  if (g.lane != 0) return 0;
  uint4* kc = reinterpret_cast<uint4*>(a.keycache) + (uint64_t)p * 2;
  if (m.overflow) {   // a later tier counts it (and writes offsets[p])
    a.heavybyte[p] = 0;
    const uint32_t k = !RETRY && agg ? atomicAdd(&agg->ndef, 1u) : kDefBuf;   // LDS
    if (k < kDefBuf) {
      agg->def[k] = p;
    } else {
      const uint32_t idx = atomicAdd(&a.status[RETRY ? kStWalked : kStDeferred], 1u);
      a.deferred[(RETRY ? (uint64_t)a.npub : 0ull) + idx] = p;   // each list holds npub entries
    }
    a.offsets[p] = 0;
    kc[0] = make_uint4(0, kDeferred, 0, 0);
    fl = m.walk_ovf ? 2 : 3;
    return 0;
  }
  const uint32_t total = out_total<OUT>(m);
  a.offsets[p] = total;
  uint32_t hb = 0;   // 1 + bucket for a heavy publish (heavybyte), else 0
  // key cache: total, nk, remote mask, up to two {record off, count}
  // (3..8 keys: the keys in the spill slots, kc[1].y = their record total;
  // many keys: kc[1] = {candidates, record total, the exact key's off, count})
  if (many) {
    kc[0] = make_uint4(total, kMany, (uint32_t)m.rmask, (uint32_t)(m.rmask >> 32));
    kc[1] = make_uint4(m.nc, m.ksum, m.ex_off, m.ex_cnt);
    fl = 1;
    if (FEAT && OUT == 0 && total >= kGroupMin && a.groups) {   // an output group instead of the chunk mask: fl 5
      const uint64_t sig = group_sig_many(m.ex_off, m.ex_cnt, (pub.flags & VMQG_PUB_DOLLAR) != 0, m.rmask, m.nc,
                                          [&](uint32_t i) { return s.cd(i); });
      if (group_insert(a, sig, p)) fl = 5;
    }
  } else {
    // a huge records-mode publish (R2's one topic of 4M subscribers): every
    // wave of the EMIT tail copies a segment of it (one wave would take ms)
    const bool huge = OUT == 0 && total >= kHugeRecords;
    uint32_t hf = huge ? kHugeFlag : 0u;
    if (huge) a.deferred[4ull * a.npub + atomicAdd(&a.status[kStHuge], 1u)] = p;
    if (m.nk <= 2) {
      const uint2 k0 = m.nk > 0 ? s.ky(0) : make_uint2(0, 0);
      const uint2 k1 = m.nk > 1 ? s.ky(1) : make_uint2(0, m.ksum);
      const uint32_t c0 = m.nk > 1 ? k1.y : m.ksum;
      const uint4 w1 = make_uint4(k0.x, c0, k1.x, m.ksum - c0);
      if (FEAT && OUT == 0 && !huge && total >= kGroupMin && a.groups &&
          group_insert(a, group_sig_keys(w1, m.rmask), p)) {
        hf = kGroupFlag;   // the EMIT tail writes it with its output group: fl 6
        fl = 6;
      } else if (OUT == 0 && !huge && a.heavy_min && total >= a.heavy_min) {
        hf = kHeavyFlag;   // the EMIT tail copies it on its first key's XCD: fl 8
        fl = 8;
      }
      hb = hf == kHeavyFlag ? 1 + heavy_bucket(k0.x) : 0u;
      kc[0] = make_uint4(total, m.nk | hf, (uint32_t)m.rmask, (uint32_t)(m.rmask >> 32));
      kc[1] = w1;
    } else {
      kc[0] = make_uint4(total, m.nk | hf, (uint32_t)m.rmask, (uint32_t)(m.rmask >> 32));
      kc[1] = make_uint4(0, m.ksum, 0, 0);
    }
  }
  a.heavybyte[p] = (uint8_t)hb;
  return total;
}

// Marks the wide publishes among a wave's groups (fl == 1 on a group's lane
// 0) in their chunk's 64-bit mask (bit = publish % gpw), which the EMIT tail
// launch walks: the fast pass stores its chunk's whole mask (no atomics),
// the retry and the dedupe fixup OR single bits into masks the fast pass
// already stored.
template <int G>
__device__ __forceinline__ uint64_t group_bits_to_publish_bits(uint64_t m) {
  uint64_t wm = 0;
  for (; m; m &= m - 1) wm |= 1ull << ((uint32_t)__builtin_ctzll(m) / G);
  return wm;
}

template <int G, bool RETRY>
__device__ __forceinline__ void mark_wide(const MatchArgs& a, const Group<G>& g, uint32_t fl, uint32_t p,
                                          uint32_t* many = nullptr) {
  const bool w = g.lane == 0 && fl == 1;
  const uint64_t m_all = __ballot(w);
  const uint32_t c = p / a.gpw;
  if (RETRY) {
    if (w) atomicOr(reinterpret_cast<unsigned long long*>(a.widemask + c), 1ull << (p % a.gpw));
  } else if (__lane_id() == 0) {   // p: the wave's first publish; the chunk's mask stored whole
    a.widemask[c] = group_bits_to_publish_bits<G>(m_all);
  }
  if (m_all && __lane_id() == 0) atomicAdd(many ? many : &a.status[kStMany], (uint32_t)__popcll(m_all));
}

// ------------------------------------------------------------- EMIT pass
// Per-group result of the resolve step, staged in LDS for the wave copy.
struct GroupMeta {
  uint32_t rel, span, nk, ksum;      // output start relative to the wave's first publish, length
  uint32_t rm_lo, rm_hi, crel, c0;   // crel: start among the wave's copied records
  uint32_t off0, off1, pad0, pad1;   // nk <= 2 (key cache): key 0 = [off0, +c0), key 1 = [off1, +ksum-c0)
  uint4 pre0, pre1;                  // a one-record key's record, loaded during the resolve
};

// Resolve publish first + gidx of a wave from the key cache (<= 2 keys) or
// the spill slots (3..8 keys).  Leaves the keys {off, cum start} in the
// group's LDS key list; [obase, oend) is the publish's output range.  Returns kResOk,
// kResMany (many-key mode: written wave-wide by emit_many) or kResSkip (the
// wave tier writes it, or an error is latched).
enum : int { kResSkip = 0, kResOk = 1, kResMany = 2 };

template <int G, int OUT>
__device__ int resolve(const MatchArgs& a, uint32_t p, const FastScratch<G>& s, const Group<G>& g,
                       uint32_t& nk, uint32_t& ksum, uint64_t& rmask, uint64_t obase, uint64_t oend) {
  const uint4* kc = reinterpret_cast<const uint4*>(a.keycache) + (uint64_t)p * 2;
  const uint4 h = kc[0];
  uint32_t total;
  if (h.y == kDeferred) return kResSkip;   // written by the wave tier
  const bool many = h.y == kMany;
  if (!many && (h.y & (kHugeFlag | kGroupFlag | kHeavyFlag))) return kResSkip;   // the EMIT tail writes it
  if (many) {
    total = h.x;
  } else {
    total = h.x; nk = h.y; rmask = ((uint64_t)h.w << 32) | h.z;
    const uint4 k = kc[1];
    ksum = k.y + k.w;
    if (nk > 2) {   // spilled by COUNT: {off, cum start} as the walk left them
      for (uint32_t i = g.lane; i < nk; i += G) s.ky(i) = a.keyspill[(uint64_t)p * kSpillKeys + i];
    } else if (g.lane == 0) {
      s.ky(0) = make_uint2(k.x, 0u);
      s.ky(1) = make_uint2(k.z, k.y);
    }
    wave_sync();
  }
  const uint64_t cap = OUT ? a.rng_cap : a.out_cap;
  if (oend > cap) { if (g.lane == 0) atomicOr(a.err, kErrOverflow); return kResSkip; }
  if (oend - obase != total) { if (g.lane == 0) atomicOr(a.err, kErrMismatch); return kResSkip; }
  return many ? kResMany : kResOk;
}

// Wide publish p (key cache kMany), written by a group of SW lanes (two
// publishes per wave at SW = 32, so one's chain of dependent metadata loads
// overlaps the other's copy) into [ob, oe): its candidates' node records
// (match/4, match_/3 :283-303) give the keys, SW at a time (lookup_subs/1
// :87-94), then the exact key, then the remote nodes in node order (fold_/5
// :78-84) — the order and totals COUNT used.  Records mode copies each batch
// of keys' records with SW lanes x U in flight (the key of each record from
// a per-lane cursor over `kb`, the group's SW-entry LDS buffer of {record
// off, cum start}).  `act` false: the group has no publish (it still takes
// part in nothing but the group-local shuffles).  Candidates <= 16 < SW.
template <int OUT, bool NT, int U, int SW>
__device__ void emit_many(const MatchArgs& a, const Group<SW>& g, bool act, uint32_t p, uint64_t ob, uint64_t oe,
                          uint2* kb) {
  static_assert(SW >= 32, "a lane per candidate (<= 16) plus one for the exact key");
  const uint32_t lane = g.lane;
  uint32_t nkeys = 0, key = 0, off0 = 0, cnt0 = 0, nc = 0;
  uint64_t rmask = 0;
  if (act) {
    const uint4* kc = reinterpret_cast<const uint4*>(a.keycache) + (uint64_t)p * 2;
    const uint4 h = kc[0], k1 = kc[1];
    nc = k1.x;
    rmask = ((uint64_t)h.w << 32) | h.z;
    const bool dollar = (a.pubs[p].flags & VMQG_PUB_DOLLAR) != 0;
    // lane c < nc: candidate c; lane nc: the exact key
    if (lane < nc) {
      const uint32_t path = reinterpret_cast<const uint32_t*>(a.keyspill)[(uint64_t)p * 2 * kSpillKeys + lane];
      if (path < 2 * a.node_cap) {
        const NodeRec r = a.nodes[path];
        if ((r.meta & kNodeEmits) == kNodeEmits && !(dollar && (r.meta & kNodeDollarSkip))) {
          nkeys = (r.meta >> 8) & 0xFFFFFFu;
          key = r.key; off0 = r.off0; cnt0 = r.cnt0;
        }
      }
    } else if (lane == nc && k1.w != 0) {
      nkeys = 1; off0 = k1.z; cnt0 = k1.w;
    }
  }
  const uint32_t kincl = g.incl_scan(nkeys);
  const uint32_t K = g.last(kincl);
  const uint32_t kstart = kincl - nkeys;
  uint64_t run = 0;
  DBGW(6, K);
  DBGW(7, nc);
  for (uint32_t k0 = 0; k0 < K; k0 += SW) {
    const uint32_t ki = k0 + lane;
    // the candidate owning key ki: the last c whose keys start at or before it
    uint32_t c = 0;
    for (uint32_t q = 1; q <= nc; q++) if (g.bcast(kstart, q) <= ki) c = q;
    const uint32_t c_n = g.bcast(nkeys, c), c_key = g.bcast(key, c), c_ks = g.bcast(kstart, c);
    const uint32_t c_off0 = g.bcast(off0, c), c_cnt0 = g.bcast(cnt0, c);
    uint32_t off = 0, cnt = 0;
    if (ki < K) {
      if (c_n == 1) { off = c_off0; cnt = c_cnt0; }
      else {
        const uint32_t kid = a.keylist[c_key + (ki - c_ks)];
        if (kid < a.key_cap) { const KeyDesc kd = a.keydesc[kid]; off = kd.off; cnt = kd.count; }
      }
    }
    if (OUT == 1) {
      const uint64_t mb = g.ballot(cnt != 0);
      if (cnt != 0 && ob + run + prefix_bits(mb) < oe) store_range(a.out_rng, ob + run + prefix_bits(mb), off, cnt);
      run += (uint32_t)__popcll(mb);
      continue;
    }
    const uint32_t incl = g.incl_scan(cnt);
    const uint32_t tot = g.last(incl);
    const uint32_t nb = K - k0 < (uint32_t)SW ? K - k0 : (uint32_t)SW;
    kb[lane] = make_uint2(off, incl - cnt);
    wave_sync();
    uint32_t j = 0;
    for (uint32_t r0 = lane; r0 < tot; r0 += SW * U) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t r = r0 + SW * u;
        if (r < tot) {
          while (j + 1 < nb && kb[j + 1].y <= r) j++;
          const uint2 kk = kb[j];
          v[u] = *reinterpret_cast<const uint4*>(a.records + kk.x + (r - kk.y));
        }
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t r = r0 + SW * u;
        if (r < tot && ob + run + r < oe) store_rec<NT>(a.out, ob + run + r, v[u]);
      }
    }
    run += tot;
    wave_sync();
  }
  // remote nodes < 64 (COUNT already dropped the local node)
  const uint32_t nrem = (uint32_t)__popcll(rmask);
  for (uint32_t j = lane; j < nrem; j += SW) {
    const uint32_t node = select_bit(rmask, j);
    if (ob + run + j >= oe) break;
    if (OUT == 0) store_rec<NT>(a.out, ob + run + j, make_uint4((VMQG_EMIT_REMOTE << 24) | node, kNone, kNone, kNone));
    else store_range(a.out_rng, ob + run + j, node, 0u);
  }
  run += nrem;
  if (act && lane == 0 && run != oe - ob) atomicOr(a.err, kErrMismatch);
}

// A grouped publish of <= 2 keys (key cache {off0, c0, off1, c1}) written
// by the whole wave into [ob, oe): key 0's records, key 1's, then the
// remote nodes in node order (fold_/5, vmq_reg_trie.erl:78-84).
template <bool NT>
__device__ void emit_keys2(const MatchArgs& a, uint4 h, uint4 k1, uint64_t ob, uint64_t oe) {
  const uint32_t lane = __lane_id();
  const uint32_t c0 = k1.y, ks = k1.y + k1.w;
  const uint64_t rm = ((uint64_t)h.w << 32) | h.z;
  const uint32_t tot = (uint32_t)(oe - ob);
  constexpr int U = VMQG_TAIL_U;
  for (uint32_t r0 = lane; r0 < tot; r0 += 64 * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t r = r0 + 64 * u;
      if (r < tot) {
        if (r < c0) v[u] = *reinterpret_cast<const uint4*>(a.records + k1.x + r);
        else if (r < ks) v[u] = *reinterpret_cast<const uint4*>(a.records + k1.z + (r - c0));
        else v[u] = make_uint4((VMQG_EMIT_REMOTE << 24) | select_bit(rm, r - ks), kNone, kNone, kNone);
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t r = r0 + 64 * u;
      if (r < tot) store_rec<NT>(a.out, ob + r, v[u]);
    }
  }
  if (lane == 0 && tot != h.x) atomicOr(a.err, kErrMismatch);
}

// Output ranges of the GPW publishes [first, first + n) of one chunk: the
// chunk's base (the scanned chunk totals) plus the exclusive prefix of the
// counts COUNT left in offsets[]; each group's lane 0 writes its publish's
// final offset.  Returns the chunk base.
template <int G, int GPW>
__device__ __forceinline__ uint64_t chunk_offsets(const MatchArgs& a, uint32_t first, uint32_t n, const Group<G>& g,
                                                  uint64_t& obase, uint64_t& oend) {
  const uint32_t p = first + g.gidx;
  const bool valid = g.gidx < n;
  const uint64_t wbase = a.chunk[first / GPW];
  const uint64_t cnt = valid ? a.offsets[p] : 0;
  const uint64_t incl = wave_incl_scan64(g.lane == 0 ? cnt : 0);
  const uint64_t excl = __shfl(incl - (g.lane == 0 ? cnt : 0), __lane_id() & ~(uint32_t)(G - 1), 64);
  obase = wbase + excl;
  oend = obase + cnt;
  if (valid && g.lane == 0) a.offsets[p] = obase;
  return wbase;
}

// Records mode: EMIT for the GPW consecutive publishes [first, first + n)
// of one wave.  Resolve is per group; the copy is wave-wide over the wave's
// output range minus the ranges of publishes the wave tier writes, so every
// store instruction writes up to 64 x 16 B = 1 KiB contiguous.
template <int G, int GPW, bool NT, int U, bool PRE = false>
__device__ void emit_wave(const MatchArgs& a, uint32_t first, uint32_t n, const FastScratch<G>& s,
                          const Group<G>& g, GroupMeta* gm, uint32_t slot0, uint64_t pre_obase = 0,
                          uint64_t pre_oend = 0, uint64_t pre_wbase = 0) {
  const uint32_t p = first + g.gidx;
  const bool valid = g.gidx < n;
  uint64_t obase = pre_obase, oend = pre_oend;
  // PRE: the positions come from the caller (a chunk of two waves' worth of
  // publishes, chunk_positions64)
  const uint64_t wbase = PRE ? pre_wbase : chunk_offsets<G, GPW>(a, first, n, g, obase, oend);
  uint32_t nk = 0, ksum = 0;
  uint64_t rmask = 0;
  int res = kResSkip;
  if (valid) res = resolve<G, 0>(a, p, s, g, nk, ksum, rmask, obase, oend);
  const bool ok = res == kResOk;   // many-key publishes: the EMIT wave-tier launch writes them
  // key-cache groups (<= 2 keys) copy from {off0, c0, off1} directly; the
  // record of a one-record key (a publish's own exact subscriber, say) is
  // loaded now, by every group at once, instead of as a lone HBM miss in
  // the middle of the copy (key 0's by lane 0, key 1's by lane 1, or by
  // lane 0 too when a group is one lane)
  constexpr uint32_t kPre1Lane = G > 1 ? 1u : 0u;
  uint32_t off0 = 0, off1 = 0, c0 = 0;
  uint4 pre0 = make_uint4(0, 0, 0, 0), pre1 = make_uint4(0, 0, 0, 0);
  if (ok && nk <= 2) {
    const uint2 k0 = s.ky(0), k1 = s.ky(1);
    off0 = k0.x;
    off1 = k1.x;
    c0 = nk >= 2 ? k1.y : ksum;
    if (g.lane == 0 && nk >= 1 && c0 == 1) pre0 = *reinterpret_cast<const uint4*>(a.records + off0);
    if (g.lane == kPre1Lane && nk == 2 && ksum - c0 == 1) pre1 = *reinterpret_cast<const uint4*>(a.records + off1);
  }
  if (g.lane == 0)
    gm[g.gidx] = GroupMeta{valid ? (uint32_t)(obase - wbase) : 0u, ok ? (uint32_t)(oend - obase) : 0u,
                           nk == 0 ? 1 : nk, ksum, (uint32_t)rmask, (uint32_t)(rmask >> 32), 0u, c0,
                           off0, off1, 0u, 0u, pre0, make_uint4(0, 0, 0, 0)};
  wave_sync();
  if (g.lane == kPre1Lane) gm[g.gidx].pre1 = pre1;
  // compact the copied ranges: crel = exclusive scan of the ok spans
  const uint32_t lane = __lane_id();
  const uint32_t sp = lane < (uint32_t)GPW ? gm[lane].span : 0u;
  const uint32_t incl = wave_incl_scan32(sp);
  if (lane < (uint32_t)GPW) gm[lane].crel = incl - sp;
  const uint32_t Tok = __shfl(incl, GPW - 1, 64);
  wave_sync();
  // U records per lane in flight: all loads issued before the stores
  uint32_t j = 0;
  for (uint32_t r0 = lane; r0 < Tok; r0 += 64 * U) {
    uint4 v[U];
    uint64_t dst[U];
    bool w[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t r = r0 + 64 * u;
      w[u] = r < Tok;
      if (w[u]) {
        while (j + 1 < (uint32_t)GPW && gm[j + 1].crel <= r) j++;
        const GroupMeta& m = gm[j];
        const uint32_t q = r - m.crel;
        const uint32_t mk = m.nk, ks = m.ksum, mc0 = m.c0;
        const uint64_t rm = ((uint64_t)m.rm_hi << 32) | m.rm_lo;
        if (mk <= 2) {
          if (q < mc0) v[u] = mc0 == 1 ? m.pre0 : *reinterpret_cast<const uint4*>(a.records + m.off0 + q);
          else if (q < ks) v[u] = ks - mc0 == 1 ? m.pre1 : *reinterpret_cast<const uint4*>(a.records + m.off1 + (q - mc0));
          else v[u] = make_uint4((VMQG_EMIT_REMOTE << 24) | select_bit(rm, q - ks), kNone, kNone, kNone);
        } else {   // re-walked: keys {off, cum start} in the group's LDS list
          FastScratch<G> sj = s;
          sj.slot = slot0 + j;
          v[u] = emission(a, [&](uint32_t i) -> uint2 { return sj.ky(i); }, mk, ks, rm, q);
        }
        dst[u] = wbase + m.rel + q;
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (w[u]) store_rec<NT>(a.out, dst[u], v[u]);
  }
  wave_sync();
}

// Range mode: each group writes its publish's non-empty keys as
// {record off, count}, then its remote nodes as {node, 0}.
template <int G>
__device__ int emit_ranges_group(const MatchArgs& a, uint32_t p, const FastScratch<G>& s, const Group<G>& g,
                                 uint64_t obase, uint64_t oend) {
  uint32_t nk = 0, ksum = 0;
  uint64_t rmask = 0;
  const int res = resolve<G, 1>(a, p, s, g, nk, ksum, rmask, obase, oend);
  if (res != kResOk) return res;   // many-key publishes: the EMIT wave-tier launch
  uint32_t pos = 0;
  for (uint32_t k0 = 0; k0 < nk; k0 += G) {
    const uint32_t ki = k0 + g.lane;
    uint32_t off = 0, cnt = 0;
    if (ki < nk) {
      const uint2 e = s.ky(ki);
      const uint32_t next = ki + 1 < nk ? s.ky(ki + 1).y : ksum;
      off = e.x;
      cnt = next - e.y;
    }
    const uint64_t mb = g.ballot(cnt != 0);
    if (cnt != 0) store_range(a.out_rng, obase + pos + prefix_bits(mb), off, cnt);   // mb: this group's lanes only
    pos += (uint32_t)__popcll(mb);
  }
  const uint32_t nrem = (uint32_t)__popcll(rmask);
  for (uint32_t j = g.lane; j < nrem; j += G) store_range(a.out_rng, obase + pos + j, select_bit(rmask, j), 0u);
  return res;
}

// ============================================================== wave tier
constexpr uint32_t kWStack = 256, kWCand = 256, kWKeys = 256, kHiWords = kMaxNodes / 32;
#ifndef VMQG_WIDE_LANES
#define VMQG_WIDE_LANES 64   // lanes per wide publish in the EMIT tail (A/B, config D: 64 -> 2,606 us, 32 -> 3,056)
#endif
constexpr int kWideLanes = VMQG_WIDE_LANES;
struct WaveLds {
  uint2 stack[kWStack];   // tier 1's frontier stack
  uint32_t cand[kWCand];  // candidate paths awaiting resolution
  uint2 keys[kWKeys];     // {record off, count}, then {record off, cum start}
  uint32_t hb[kHiWords];  // remote-node set (4,096 bits)
};

template <int MODE, int OUT, bool NT>
struct WaveWalk {
  const MatchArgs& a;
  WaveLds& W;
  uint2* stack;
  uint32_t scap;
  uint64_t obase;       // output position of the publish (MODE 1)
  uint64_t oend;        // ... and its end: no store at or past it, whatever the walk finds
  uint64_t run = 0;     // entries counted / written so far (wave-uniform)
  uint32_t nc = 0, nk = 0;
  uint64_t rm = 0;      // lane-partial remote mask (nodes < 64)
  bool dollar = false;

  __device__ WaveWalk(const MatchArgs& a_, WaveLds& W_, uint2* st, uint32_t cap, uint64_t ob, uint64_t oe)
      : a(a_), W(W_), stack(st), scap(cap), obase(ob), oend(oe) {}

  __device__ void add_high(uint32_t off, uint32_t cnt) {   // remote nodes >= 64 into the set
    for (uint32_t j = 0; j < cnt; j++) {
      const uint32_t n = a.keylist[off + j];
      if (n < kMaxNodes) atomicOr(&W.hb[n >> 5], 1u << (n & 31));
    }
  }

  // the buffered keys -> count / records / ranges
  __device__ void flush_keys() {
    const uint32_t lane = __lane_id();
    if (nk == 0) return;
    if (MODE == 0 && OUT == 1) { run += nk; nk = 0; return; }
    if (MODE == 1 && OUT == 1) {
      for (uint32_t k = lane; k < nk; k += 64)
        if (obase + run + k < oend) store_range(a.out_rng, obase + run + k, W.keys[k].x, W.keys[k].y);
      run += nk;
      nk = 0;
      wave_sync();
      return;
    }
    // records: cumulative starts
    uint32_t tot = 0;
    for (uint32_t k0 = 0; k0 < nk; k0 += 64) {
      const uint32_t k = k0 + lane;
      const uint32_t c = k < nk ? W.keys[k].y : 0u;
      const uint32_t incl = wave_incl_scan32(c);
      wave_sync();
      if (MODE == 1 && k < nk) W.keys[k].y = tot + incl - c;
      tot += __shfl(incl, 63, 64);
    }
    wave_sync();
    if (MODE == 1) {
      constexpr int U = VMQG_WALK_U;
      const uint32_t n = nk;
      auto ks = [&](uint32_t i) -> uint2 { return W.keys[i]; };
      for (uint32_t r0 = lane; r0 < tot; r0 += 64 * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint32_t r = r0 + 64 * u;
          if (r < tot) v[u] = emission(a, ks, n, tot, 0, r);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint32_t r = r0 + 64 * u;
          if (r < tot && obase + run + r < oend) store_rec<NT>(a.out, obase + run + r, v[u]);
        }
      }
      wave_sync();
    }
    run += tot;
    nk = 0;
  }

  // the buffered candidates -> keys (match/4, match_/3 :283-303)
  __device__ void flush_cands() {
    const uint32_t lane = __lane_id();
    for (uint32_t c0 = 0; c0 < nc; c0 += 64) {
      const uint32_t ci = c0 + lane;
      uint32_t nkeys = 0, key = kNone, off0 = 0, cnt0 = 0;
      if (ci < nc) {
        const uint32_t path = W.cand[ci];
        if (path < 2 * a.node_cap) {   // own records, then '#' aliases
          const NodeRec r = a.nodes[path];
          const bool valid = (r.meta & kNodeEmits) == kNodeEmits && !(dollar && (r.meta & kNodeDollarSkip));
          if (valid) {
            nkeys = (r.meta >> 8) & 0xFFFFFFu;
            key = r.key; off0 = r.off0; cnt0 = r.cnt0;
            rm |= ((uint64_t)r.rmask_hi << 32) | r.rmask_lo;
            if (r.meta & kNodeHigh) add_high(r.hi_off, r.hi_cnt);
          }
        }
      }
      const Group<64> g;
      const uint32_t maxk = g.max32(nkeys);
      for (uint32_t j = 0; j < maxk; j++) {
        uint32_t off = 0, cnt = 0;
        if (j < nkeys) {
          if (nkeys == 1) { off = off0; cnt = cnt0; }
          else {
            const uint32_t kid = a.keylist[key + j];
            if (kid < a.key_cap) { const KeyDesc kd = a.keydesc[kid]; off = kd.off; cnt = kd.count; }
          }
        }
        const uint64_t mb = __ballot(cnt != 0);
        const uint32_t nn = (uint32_t)__popcll(mb);
        if (nk + nn > kWKeys) flush_keys();
        if (cnt != 0) W.keys[nk + prefix_bits(mb)] = make_uint2(off, cnt);
        nk += nn;
        wave_sync();
      }
    }
    nc = 0;
    wave_sync();
  }

  // returns false when the frontier stack overflowed (tier 2 retries)
  __device__ bool run_publish(uint32_t p) {
    const Group<64> g;
    const uint32_t lane = __lane_id();
    const vmqg_pub pub = a.pubs[p];
    const uint32_t L = pub.nwords;
    const uint32_t* w = a.words + pub.word_off;
    dollar = (pub.flags & VMQG_PUB_DOLLAR) != 0;
    // an empty Topic list walks the root alone: trie_match(MP, root, [], _) (:361-363)
    const bool mp_ok = pub.mountpoint < a.max_mp;
    const uint32_t wreg = lane < L ? w[lane] : kUnknownWord;
    for (uint32_t i = lane; i < kHiWords; i += 64) W.hb[i] = 0;
    uint32_t sp = 0;
    if (mp_ok) { if (lane == 0) stack[0] = make_uint2(pub.mountpoint, root_flags(a, pub.mountpoint) << 28); sp = 1; }
    wave_sync();
    while (sp > 0) {
      const uint32_t k = sp < 64u ? sp : 64u;
      const uint32_t base = sp - k;
      const bool act = lane < k;
      uint32_t node = 0, d = 0, fl = 0;
      if (act) { const uint2 e = stack[base + lane]; node = e.x; d = e.y & kDepthMask; fl = e.y >> 28; }
      sp = base;
      wave_sync();
      const StepOut o = probe_step<64>(a, g, act, node, d, fl, L, w, wreg);
      const uint64_t m_hc = __ballot(o.hc != kNone), m_end = __ballot(o.at_end);
      const uint32_t n_hc = (uint32_t)__popcll(m_hc), n_new_c = n_hc + (uint32_t)__popcll(m_end);
      const uint64_t m_wc = __ballot(o.wc != kNone), m_pc = __ballot(o.pc != kNone);
      const uint32_t n_pc = (uint32_t)__popcll(m_pc), n_new_s = n_pc + (uint32_t)__popcll(m_wc);
      if (sp + n_new_s > scap) return false;
      if (nc + n_new_c > kWCand) flush_cands();   // n_new_c <= 128 < kWCand
      if (o.hc != kNone) W.cand[nc + prefix_bits(m_hc)] = o.hc;
      if (o.at_end) W.cand[nc + n_hc + prefix_bits(m_end)] = node;
      nc += n_new_c;
      if (o.pc != kNone) stack[sp + prefix_bits(m_pc)] = make_uint2(o.pc, (d + 1) | (o.pf << 28));
      if (o.wc != kNone) stack[sp + n_pc + prefix_bits(m_wc)] = make_uint2(o.wc, (d + 1) | (o.wf << 28));
      sp += n_new_s;
      wave_sync();
    }
    flush_cands();
    if (mp_ok) {
      uint32_t xst;
      const ExactSlot* e = find_exact<64>(a, pub, w, wreg, g, xst);
      if (e) {
        const uint32_t nw = e->nwords;
        rm |= e->rmask;
        if (e->count != 0) {
          if (nk + 1 > kWKeys) flush_keys();
          if (lane == 0) W.keys[nk] = make_uint2(e->off, e->count);
          nk += 1;
        }
        if (nw & kExactHigh) {   // {count, ids} after the words beyond the inline ones
          const uint32_t* hl = a.exwords + e->words_off + exact_tail_words(L);
          const uint32_t cnt = hl[0];
          for (uint32_t j = lane; j < cnt; j += 64) {
            const uint32_t n = hl[1 + j];
            if (n < kMaxNodes) atomicOr(&W.hb[n >> 5], 1u << (n & 31));
          }
        }
      }
    }
    wave_sync();
    flush_keys();
    // remote nodes in node order (fold_/5 :78-84): lane l owns nodes [64 l, 64 l + 64)
    const uint64_t low = g.or64(rm);
    wave_sync();
    uint64_t word = ((uint64_t)W.hb[2 * lane + 1] << 32) | W.hb[2 * lane];
    if (lane == 0) word |= low;
    if (lane == (a.local_node >> 6)) word &= ~(1ull << (a.local_node & 63));
    const uint32_t c = (uint32_t)__popcll(word);
    const uint32_t incl = wave_incl_scan32(c);
    if (MODE == 1) {
      uint64_t pos = obase + run + incl - c;
      while (word) {
        const uint32_t b = (uint32_t)__builtin_ctzll(word);
        word &= word - 1;
        const uint32_t node = lane * 64 + b;
        if (pos >= oend) break;
        if (OUT == 0) store_rec<NT>(a.out, pos, make_uint4((VMQG_EMIT_REMOTE << 24) | node, kNone, kNone, kNone));
        else store_range(a.out_rng, pos, node, 0u);
        pos++;
      }
    }
    run += __shfl(incl, 63, 64);
    wave_sync();
    return true;
  }
};

// One publish walked by the whole wave: the frontier stack in LDS, and if it
// outgrows it, walked again with the wave's stack in global scratch (o_cap
// entries, sized from the trie depth so it cannot overflow).  COUNT writes
// offsets[p] and adds to the chunk total; EMIT re-walks in the same order,
// writes [ob, oe) and checks the count.
//
// The fused phases (gstack null) borrow one of the o_waves global stacks for
// the second walk: claimed from the bitmap a.o_slots, released after.  A
// wave that finds every stack taken waits for one; a holder is in the middle
// of a walk, which never waits on anything, so it always comes back.
//
// A stack's bytes pass from holder to holder inside one launch, across XCDs
// whose L2s are not coherent: a holder's dirty stack lines left in its XCD's
// L2 could be written back to HBM AFTER the next holder (another XCD) wrote
// the same addresses, and the next holder's re-read after an eviction would
// see the old entries (test_more_global_stack_walks_than_stacks: 3,072
// concurrent records-mode walks, 45 count mismatches without this).  So the
// holder releases at agent scope (L2 write-back) before it clears its bit,
// and the claimer acquires at agent scope (this CU's L1 invalidated) after
// it set it (MI355X_MICROARCH.md, inter-workgroup visibility).
#ifndef VMQG_STACK_FENCES
#define VMQG_STACK_FENCES 1   // A/B only: 0 = the round-3 hand-off without fences (wrong under contention)
#endif
__device__ __forceinline__ void release_ostack(const MatchArgs& a, uint32_t slot) {
  if (VMQG_STACK_FENCES) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  atomicAnd(a.o_slots + slot / 32, ~(1u << (slot % 32)));
}
__device__ uint32_t claim_ostack(const MatchArgs& a) {
  const uint32_t lane = __lane_id(), nw = (a.o_waves + 31) / 32;
  uint32_t slot = kNone;
  if (lane == 0) {
    for (uint32_t spins = 0; slot == kNone; spins++) {
      for (uint32_t i = 0; i < nw && slot == kNone; i++) {
        const uint32_t valid = i + 1 < nw || a.o_waves % 32 == 0 ? ~0u : (1u << (a.o_waves % 32)) - 1;
        uint32_t cur = __hip_atomic_load(a.o_slots + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (slot == kNone && (~cur & valid)) {
          const uint32_t b = (uint32_t)__builtin_ctz(~cur & valid);
          const uint32_t old = atomicOr(a.o_slots + i, 1u << b);
          if (!(old & (1u << b))) slot = i * 32 + b;
          cur = old | (1u << b);
        }
      }
      if (slot == kNone) {
        if (spins > (1u << 20)) break;   // none came back (never expected): the walk is refused loudly
        __builtin_amdgcn_s_sleep(8);
      }
    }
    if (VMQG_STACK_FENCES && slot != kNone) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  return __shfl(slot, 0, 64);
}

#ifndef VMQG_WALK_CALL
#define VMQG_WALK_CALL 0   // A/B: 1 = the walk as a call (a kernel with a call sets up scratch: +4 us per empty launch)
#endif
template <int MODE, int OUT, bool NT>
__device__ __attribute__((noinline)) void wave_publish_call(const MatchArgs& a, WaveLds& W, uint2* gstack, uint32_t p,
                                                          uint64_t ob, uint64_t oe);
template <int MODE, int OUT, bool NT>
__device__ __forceinline__ void wave_publish_body(const MatchArgs& a, WaveLds& W, uint2* gstack, uint32_t p,
                                                  uint64_t ob, uint64_t oe) {
  const uint32_t lane = __lane_id();
  WaveWalk<MODE, OUT, NT> w1(a, W, W.stack, kWStack, ob, oe);
  bool ok = w1.run_publish(p);
  uint64_t total = w1.run;
  if (!ok) {
    if (MODE == 0 && lane == 0) atomicAdd(&a.status[kStTier2], 1u);
    const uint32_t slot = gstack ? kNone : claim_ostack(a);
    if (gstack || slot != kNone) {
      WaveWalk<MODE, OUT, NT> w2(a, W, gstack ? gstack : a.o_stack + (uint64_t)slot * a.o_cap, a.o_cap, ob, oe);
      ok = w2.run_publish(p);
      total = w2.run;
    }
    wave_sync();   // every lane's stack stores issued before the release
    if (slot != kNone && lane == 0) release_ostack(a, slot);
    if (!ok && lane == 0) atomicOr(a.err, kErrFrontier);
  }
  if (ok && lane == 0) {
    if (MODE == 0) {
      a.offsets[p] = total;
      // its count in the key cache too: EMIT's many-key phase reads every count from there
      reinterpret_cast<uint4*>(a.keycache)[(uint64_t)p * 2] = make_uint4((uint32_t)total, kDeferred, 0, 0);
      atomicAdd(reinterpret_cast<unsigned long long*>(a.chunk + p / a.gpw), (unsigned long long)total);
    } else if (total != oe - ob) {
      atomicOr(a.err, kErrMismatch);
    } else {
      atomicAdd(reinterpret_cast<unsigned long long*>(a.status + kStWaveEnt), (unsigned long long)total);
    }
  }
  wave_sync();
}
template <int MODE, int OUT, bool NT>
__device__ __attribute__((noinline)) void wave_publish_call(const MatchArgs& a, WaveLds& W, uint2* gstack, uint32_t p,
                                                          uint64_t ob, uint64_t oe) {
  wave_publish_body<MODE, OUT, NT>(a, W, gstack, p, ob, oe);
}
template <int MODE, int OUT, bool NT>
__device__ __forceinline__ void wave_publish(const MatchArgs& a, WaveLds& W, uint2* gstack, uint32_t p, uint64_t ob,
                                             uint64_t oe) {
  if (VMQG_WALK_CALL) wave_publish_call<MODE, OUT, NT>(a, W, gstack, p, ob, oe);
  else wave_publish_body<MODE, OUT, NT>(a, W, gstack, p, ob, oe);
}

// A deferred publish per group of four lanes (sixteen per wave, `valid`):
// retried four lanes per publish (a publish served there gets its key cache
// as in the fast pass and its count added to its chunk's total); what
// overflows even those lists (or all, at fast_g 4, whose fast pass already
// had them) is walked by the whole wave and listed for EMIT (list 1).
template <int OUT, bool NT, uint32_t SL>
__device__ void count_deferred_group(const MatchArgs& a, const FastScratch<4, SL>& s, const Group<4>& g, WaveLds& W,
                                     uint2* gstack, bool valid, uint32_t p) {
  const uint32_t lane = __lane_id();
  const bool retry = a.fast_g != 4;
  if (!valid) p = 0;
  uint32_t fl = 2, c = 0;
  if (retry && valid) {
    c = count_publish<4, OUT, true, SL>(a, p, s, g, fl);
    if (g.lane == 0 && (fl <= 1 || fl >= 5))
      atomicAdd(reinterpret_cast<unsigned long long*>(a.chunk + p / a.gpw), (unsigned long long)c);
  }
  wave_sync();
  if (retry) {
    mark_wide<4, true>(a, g, fl, p);
    const uint32_t n_heavy = (uint32_t)__popcll(__ballot(valid && g.lane == 0 && fl == 8));
    if (lane == 0 && n_heavy) atomicAdd(&a.status[kStHeavy], n_heavy);
    const uint32_t n_grp = (uint32_t)__popcll(__ballot(valid && g.lane == 0 && (fl == 5 || fl == 6)));
    if (lane == 0 && n_grp) atomicAdd(&a.status[kStGrouped], n_grp);
  }
  // what the retry could not hold (or all, at fast_g 4): one whole-wave walk each
  uint64_t ov = __ballot(valid && g.lane == 0 && (fl == 2 || fl == 3));
  if (!retry && ov) {   // list 1 for EMIT (the retry's count_publish listed its own)
    uint32_t at = 0;
    if (lane == 0) at = atomicAdd(&a.status[kStWalked], (uint32_t)__popcll(ov));
    at = __shfl(at, 0, 64);
    if (valid && g.lane == 0) a.deferred[(uint64_t)a.npub + at + prefix_bits(ov)] = p;
  }
  while (ov) {
    const uint32_t l = (uint32_t)__builtin_ctzll(ov);
    ov &= ov - 1;
    wave_publish<0, OUT, NT>(a, W, gstack, __shfl(p, l, 64), 0, 0);
  }
}


// --------------------------------------------------------------- kernels
// Positions of the publishes of a 64-publish chunk (the chunks of a one-lane
// COUNT, fast_g 1): lane l reads publish first + l's count, the wave scans
// them from the chunk's base and writes the final offsets; returns lane l's
// position and count for the halves to pick up.
__device__ __forceinline__ void chunk_positions64(const MatchArgs& a, uint32_t first, uint32_t nch, uint64_t& pos,
                                                  uint64_t& cnt) {
  const uint32_t lane = __lane_id();
  const bool valid = lane < nch;
  cnt = valid ? a.offsets[first + lane] : 0;
  const uint64_t incl = wave_incl_scan64(cnt);
  pos = a.chunk[first / 64] + incl - cnt;
  if (valid) a.offsets[first + lane] = pos;
}

template <int MODE, int OUT, int G, bool NT, int CH = 64 / G, bool FEAT = false>
#ifndef VMQG_COUNT_WPE
#define VMQG_COUNT_WPE 4    // COUNT waves per SIMD the register budget must allow, 2+ lanes per publish (A/B: 4, 5)
#endif
#ifndef VMQG_COUNT_WPE1
#define VMQG_COUNT_WPE1 5   // ... one lane per publish (96 VGPRs, no spills)
#endif
__global__ __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(MODE == 0 ? (G == 1 ? VMQG_COUNT_WPE1 : VMQG_COUNT_WPE) : 4)))
void k_match_fast(MatchArgs a) {
  using FS = FastScratch<G>;
  constexpr int GPW = FS::GPW;
  if (MODE == 0 && blockIdx.x == 0 && threadIdx.x < kStWords) a.status_next[threadIdx.x] = 0;
  __shared__ uint2 st[MODE == 0 ? FS::SC * FS::SLOTS : 1];
  __shared__ uint32_t cd[MODE == 0 ? FS::CC * FS::SLOTS : 1];
  __shared__ uint2 ky[FS::KC * FS::SLOTS];
  __shared__ GroupMeta gm[kWaves][MODE == 1 && OUT == 0 ? GPW : 1];
  const Group<G> g;
  const uint32_t wv = threadIdx.x >> 6;
  const FS s{st, cd, ky, wv * GPW + g.gidx};
  // EMIT writes every publish resolve can serve; the wide ones (kResMany)
  // and the whole-wave walks (kDeferred) are the EMIT tail launch's
  if constexpr (MODE == 1 && CH != GPW) {
    // EMIT over the 64-publish chunks of a one-lane COUNT, as two halves of
    // GPW = 32 publishes with two lanes per publish
    static_assert(CH == 2 * GPW, "");
    const uint32_t stride = gridDim.x * kWaves * CH;
    for (uint32_t base = (blockIdx.x * kWaves + wv) * CH; base < a.npub; base += stride) {
      const uint32_t nch = a.npub - base < (uint32_t)CH ? a.npub - base : (uint32_t)CH;
      uint64_t pos, cnt;
      chunk_positions64(a, base, nch, pos, cnt);
      for (uint32_t h = 0; h < 2; h++) {
        const uint32_t first = base + h * GPW;
        if (nch <= h * GPW) break;
        const uint32_t n = nch - h * GPW < (uint32_t)GPW ? nch - h * GPW : (uint32_t)GPW;
        const uint32_t q = h * GPW + g.gidx;
        const uint64_t ob = __shfl(pos, q, 64), oe = ob + __shfl(cnt, q, 64);
        const uint64_t wb = __shfl(pos, h * GPW, 64);
        if (OUT == 0) {
          emit_wave<G, GPW, NT, VMQG_EMIT_U, true>(a, first, n, s, g, gm[wv], wv * GPW, ob, oe, wb);
        } else if (g.gidx < n) {
          emit_ranges_group<G>(a, first + g.gidx, s, g, ob, oe);
        }
        wave_sync();
      }
    }
    return;
  }
  __shared__ uint32_t agg_raw[MODE == 0 ? sizeof(CountAgg) / 4 : 1];
  CountAgg* agg = MODE == 0 ? reinterpret_cast<CountAgg*>(agg_raw) : nullptr;
  if (MODE == 0) {
    if (threadIdx.x < 9) (&agg->many)[threadIdx.x] = 0;
    __syncthreads();
  }
  const uint32_t stride = gridDim.x * kWaves * GPW;
  if constexpr (MODE == 0 && FEAT) {
    if (a.dd_claimed) {
      // batch dedupe on: only the representatives k_dd_classify listed (list
      // 2), GPW per wave, dense; their chunks' totals, masks and fast-pass
      // bits were zeroed by k_dd_claim and are accumulated here (atomics on
      // one word per chunk, not one word for the launch)
      const uint32_t nr = uni(a.status[kStReps]);
      const uint32_t* R = a.deferred + 2ull * a.npub;
      for (uint32_t base = (blockIdx.x * kWaves + wv) * GPW; base < nr; base += stride) {
        const uint32_t n = nr - base < (uint32_t)GPW ? nr - base : (uint32_t)GPW;
        uint32_t fl = 2, p = 0;
        uint64_t c = 0;
        if (g.gidx < n) {
          p = R[base + g.gidx];
          c = count_publish<G, OUT, false, kWaves * (64 / G), FEAT>(a, p, s, g, fl, agg);
        }
        if (g.gidx < n && g.lane == 0) {
          const uint32_t ch = p / a.gpw;
          if (c) atomicAdd(reinterpret_cast<unsigned long long*>(a.chunk + ch), (unsigned long long)c);
          if (fl <= 1 || fl >= 5) atomicOr(a.fastdone + p / 32, 1u << (p % 32));
          if (fl == 1) atomicOr(reinterpret_cast<unsigned long long*>(a.widemask + ch), 1ull << (p % a.gpw));
        }
        const uint32_t n_heavy = (uint32_t)__popcll(__ballot(g.gidx < n && g.lane == 0 && fl == 8));
        if (__lane_id() == 0 && n_heavy) atomicAdd(&agg->heavy, n_heavy);
        const uint32_t n_many = (uint32_t)__popcll(__ballot(g.gidx < n && g.lane == 0 && fl == 1));
        const uint32_t n_wovf = (uint32_t)__popcll(__ballot(g.gidx < n && g.lane == 0 && fl == 2));
        const uint32_t n_grp = (uint32_t)__popcll(__ballot(g.gidx < n && g.lane == 0 && (fl == 5 || fl == 6)));
        if (__lane_id() == 0) {
          if (n_many) atomicAdd(&agg->many, n_many);
          if (n_wovf) atomicAdd(&agg->walkovf, n_wovf);
          if (n_grp) atomicAdd(&agg->grouped, n_grp);
        }
        wave_sync();
      }
    }
  }
  for (uint32_t base = (blockIdx.x * kWaves + wv) * GPW; base < a.npub; base += stride) {
    const uint32_t n = a.npub - base < (uint32_t)GPW ? a.npub - base : (uint32_t)GPW;
    if (MODE == 0) {
      if (FEAT && a.dd_claimed) break;   // the representatives' loop above did the work
      uint64_t c = 0;
      uint32_t fl = 0;
      if (g.gidx < n) c = count_publish<G, OUT, false, kWaves * (64 / G), FEAT>(a, base + g.gidx, s, g, fl, agg);
      // the chunk's total (publishes the wave tier takes add theirs later)
      const uint64_t tot = __shfl(wave_incl_scan64(c), 63, 64);
      if (__lane_id() == 0) a.chunk[base / GPW] = tot;
      // wide publishes: the chunk's mask for the EMIT tail launch
      mark_wide<G, false>(a, g, fl, base, &agg->many);
      const uint32_t n_heavy = (uint32_t)__popcll(__ballot(g.gidx < n && g.lane == 0 && fl == 8));
      if (__lane_id() == 0 && n_heavy) atomicAdd(&agg->heavy, n_heavy);
      const uint32_t n_wovf = (uint32_t)__popcll(__ballot(g.lane == 0 && fl == 2));
      if (__lane_id() == 0 && n_wovf) atomicAdd(&agg->walkovf, n_wovf);
      const uint32_t n_grp = (uint32_t)__popcll(__ballot(g.gidx < n && g.lane == 0 && (fl == 5 || fl == 6)));
      if (__lane_id() == 0 && n_grp) atomicAdd(&agg->grouped, n_grp);
    } else if (OUT == 0) {
      emit_wave<G, GPW, NT, VMQG_EMIT_U>(a, base, n, s, g, gm[wv], wv * GPW);
    } else {
      uint64_t ob, oe;
      chunk_offsets<G, GPW>(a, base, n, g, ob, oe);
      if (g.gidx < n) emit_ranges_group<G>(a, base + g.gidx, s, g, ob, oe);
    }
    wave_sync();
  }
  if (MODE == 0) {   // the block's counters and deferred publishes, one global atomic each
    __syncthreads();
    const uint32_t nd = agg->ndef < kDefBuf ? agg->ndef : kDefBuf;
    if (threadIdx.x == 0) agg->base = nd ? atomicAdd(&a.status[kStDeferred], nd) : 0u;
    if (threadIdx.x == 64 && agg->many) atomicAdd(&a.status[kStMany], agg->many);
    if (threadIdx.x == 128 && agg->walkovf) atomicAdd(&a.status[kStWalkOvf], agg->walkovf);
    if (threadIdx.x == 192 && agg->grouped) atomicAdd(&a.status[kStGrouped], agg->grouped);
    if (threadIdx.x == 96 && agg->heavy) atomicAdd(&a.status[kStHeavy], agg->heavy);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nd; i += blockDim.x) a.deferred[agg->base + i] = agg->def[i];
  }
}

// Wave tiers, one launch after each fast pass (each reads its list lengths
// on the device and exits at once when they are empty).
//
// COUNT: the publishes the fast pass deferred (list 0) are retried four
// lanes per publish (16 per wave, lists 4x the one-lane pass's: a deep
// multi-wildcard walk fits); a publish served there gets its key cache as in
// the fast pass and its count added to its chunk's total.  What overflows
// even those lists is walked by the whole wave at once (and listed for
// EMIT: list 1).  With fast_g 4 the fast pass already had these lists: its
// deferrals go straight to the whole-wave walk.
//
// EMIT tail: the whole-wave walks again (list 1), then the huge publishes
// (every wave a segment of each), the output groups (a slot's members back
// to back) and the wide publishes of the chunk masks (one per wave).
#ifndef VMQG_TAIL_WPE
#define VMQG_TAIL_WPE 8   // EMIT tail: asks for 8 waves per SIMD; gfx950 build (round 4): 128 VGPRs, 4 waves (groups, huge, wide, walks in one kernel)
#endif
template <int MODE, int OUT, bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MODE == 1 ? VMQG_TAIL_WPE : 1)))
void k_match_wave(MatchArgs a) {
  __shared__ WaveLds lds[kWaves];
  __shared__ unsigned long long s_wsum;   // EMIT tail: the block's wide / grouped entries
  __shared__ uint32_t s_wdone;            // the block's waves done (its last wave flushes the sums)
  if (threadIdx.x == 0) { s_wsum = 0; s_wdone = 0; }
  __syncthreads();
  const uint32_t wv = threadIdx.x >> 6, lane = __lane_id();
  const uint64_t gw = (uint64_t)blockIdx.x * kWaves + wv;
  const uint32_t nwaves = gridDim.x * kWaves;
  uint2* gstack = a.o_stack + gw * a.o_cap;
  if constexpr (MODE == 0) {
    using FS = FastScratch<4>;
    constexpr uint32_t GPW = FS::GPW;
    __shared__ uint2 st[FS::SC * FS::SLOTS];
    __shared__ uint32_t cd[FS::CC * FS::SLOTS];
    __shared__ uint2 ky[FS::KC * FS::SLOTS];
    const Group<4> g;
    const FS s{st, cd, ky, wv * GPW + g.gidx};
    // block 0 sets the next call's dedupe mode from this call's counts:
    // on while more than half the sampled publishes repeat another
    if (gw == 0 && lane == 0 && a.dd_claimed) {
      const uint32_t tried = a.status[kStDupTried], dups = a.status[kStDup];
      if (tried >= 256) {
        const uint32_t mode = (uint64_t)dups * 100u > (uint64_t)tried * VMQG_DD_ON_PCT ? 1u : 0u;
        *a.dd_mode = mode;
        if (a.dd_host) *a.dd_host = mode;   // host-mapped: the host reads it before its next calls
      }
    }
    // COUNT's deferred publishes (list 0), sixteen per wave, then the
    // duplicates the fixup could not serve, sixteen at a time (one call
    // site of the retry: the walk is inlined once)
    // (with dedupe on, k_dd_fixup appended the duplicates it could not
    // serve to list 0: they are walked here like COUNT's own deferrals)
    // A short list (no more publishes than waves) is mostly heavy
    // publishes — what overflowed four lanes already (dedupe on) or a few
    // wide frontiers: one per wave, so their whole-wave walks run side by
    // side instead of one after another in the first few waves.
    const uint32_t nd = uni(a.status[kStDeferred]);
    const uint32_t per = nd <= nwaves ? 1u : GPW;
    for (uint32_t d0 = (uint32_t)gw * per; d0 < nd; d0 += nwaves * per) {
      const bool valid = g.gidx < per && d0 + g.gidx < nd;
      const uint32_t p = a.deferred[valid ? d0 + g.gidx : d0];
      count_deferred_group<OUT, NT>(a, s, g, lds[wv], gstack, valid, p);
      wave_sync();
    }
    return;
  } else {
    // the whole-wave walks (list 1); a walk that outgrows its LDS stack
    // borrows a global one (this grid has more waves than there are stacks)
    const uint64_t cap = OUT ? a.rng_cap : a.out_cap;
#ifndef VMQG_TAIL_NOWALK
#define VMQG_TAIL_NOWALK 0   // A/B only (wrong with walked publishes): the tail without its walker
#endif
    const uint32_t n = VMQG_TAIL_NOWALK ? 0u : uni(a.status[kStWalked]);
    for (uint32_t d = (uint32_t)gw; d < n; d += nwaves) {
      const uint32_t p = uni(a.deferred[(uint64_t)a.npub + d]);
      const uint64_t ob = uni64(a.offsets[p]), oe = uni64(a.offsets[p + 1]);
      if (oe > cap || ob > oe) {
        if (lane == 0) atomicOr(a.err, kErrOverflow);
        continue;
      }
      if (!VMQG_TAIL_NOWALK) wave_publish<1, OUT, NT>(a, lds[wv], nullptr, p, ob, oe);
    }
    // the huge publishes, every wave a segment of each (records mode)
    if (OUT == 0) {
      const uint32_t nh = uni(a.status[kStHuge]);
      for (uint32_t hi = 0; hi < nh; hi++) {
        const uint32_t p = uni(a.deferred[4ull * a.npub + hi]);
        const uint64_t ob = uni64(a.offsets[p]), oe = uni64(a.offsets[p + 1]);
        if (oe > cap || ob > oe) {
          if (gw == 0 && lane == 0) atomicOr(a.err, kErrOverflow);
          continue;
        }
        const uint4* kc = reinterpret_cast<const uint4*>(a.keycache) + (uint64_t)p * 2;
        const uint4 h = kc[0], k1 = kc[1];
        const uint32_t nk = h.y & ~kHugeFlag, ksum = k1.y + k1.w;
        const uint64_t rmask = ((uint64_t)h.w << 32) | h.z;
        if (gw == 0 && lane == 0 && oe - ob != h.x) atomicOr(a.err, kErrMismatch);
        // keys {off, cum start}: the key cache's two, or the spill slots
        const uint2* sp = a.keyspill + (uint64_t)p * kSpillKeys;
        auto ks = [&](uint32_t i) -> uint2 {
          if (nk > 2) return sp[i];
          return i == 0 ? make_uint2(k1.x, 0u) : make_uint2(k1.z, k1.y);
        };
        const uint64_t total = oe - ob;
        const uint64_t nseg = (total + kHugeSeg - 1) / kHugeSeg;
        for (uint64_t sg = gw; sg < nseg; sg += nwaves) {
          const uint64_t r0 = sg * kHugeSeg;
          const uint32_t n = (uint32_t)(total - r0 < kHugeSeg ? total - r0 : kHugeSeg);
          constexpr int U = VMQG_TAIL_U;
          for (uint32_t j = lane; j < n; j += 64 * U) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
              const uint32_t r = j + 64 * u;
              if (r < n) v[u] = emission(a, ks, nk == 0 ? 1u : nk, ksum, rmask, (uint32_t)(r0 + r));
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
              const uint32_t r = j + 64 * u;
              if (r < n) store_rec<NT>(a.out, ob + r0 + r, v[u]);
            }
          }
        }
      }
    }
    // then, one publish at a time per wave (one call site of each writer,
    // so the walk and copy code is inlined once): the output groups — a
    // slot's members back to back, their sources staying in this CU's L1 /
    // L2 after the first member — and then the wide publishes of the chunk
    // masks COUNT left, at the positions EMIT wrote into offsets[]
    bool groups_on = OUT == 0 && uni(a.status[kStGrouped]) != 0;
    bool heavy_on = OUT == 0 && uni(a.status[kStHeavy]) != 0;
    bool wide_on = uni(a.status[kStMany]) != 0;
    uint64_t written = 0;
    if (OUT == 0 && heavy_on) {
      // heavy publishes: the blocks b = x (mod kXcds) — on XCD x — take the
      // bucket-x publishes, their waves striding over 64-publish blocks; one
      // publish ahead: the next one's offsets and key cache load while this
      // one copies (a heavy list copies in about the time those two dependent
      // loads take)
      const uint32_t nblk = (a.npub + 63) / 64;
      const uint32_t hx = blockIdx.x & (kXcds - 1);
      const uint32_t hstride = (gridDim.x - hx + kXcds - 1) / kXcds * kWaves;
      uint32_t hc = (blockIdx.x / kXcds) * kWaves + wv, hcc = 0;
      uint64_t hm = 0;
      auto next_heavy = [&](uint32_t& q) -> bool {
        while (hm == 0 && hc < nblk) {   // 64 publishes' bucket bytes per step, one per lane
          const uint32_t x = hc * 64 + lane;
          hm = __ballot(x < a.npub && a.heavybyte[x] == 1 + hx);
          hcc = hc;
          hc += hstride;
        }
        if (!hm) return false;
        q = hcc * 64 + (uint32_t)__builtin_ctzll(hm);
        hm &= hm - 1;
        return true;
      };
      uint32_t p = 0;
      bool have = next_heavy(p);
      uint64_t ob_n = 0, oe_n = 0;   // loaded per lane (uniform values): made scalar only when used
      uint4 h_n{0, 0, 0, 0}, k_n{0, 0, 0, 0};
      if (have && p < a.npub) {
        ob_n = a.offsets[p]; oe_n = a.offsets[p + 1];
        h_n = reinterpret_cast<const uint4*>(a.keycache)[(uint64_t)p * 2];
        k_n = reinterpret_cast<const uint4*>(a.keycache)[(uint64_t)p * 2 + 1];
      }
      while (have) {
        const uint32_t pc = p;
        const uint64_t obv = ob_n, oev = oe_n;
        const uint4 hv = h_n, kv = k_n;
        have = next_heavy(p);
        if (have && p < a.npub) {
          ob_n = a.offsets[p]; oe_n = a.offsets[p + 1];
          h_n = reinterpret_cast<const uint4*>(a.keycache)[(uint64_t)p * 2];
          k_n = reinterpret_cast<const uint4*>(a.keycache)[(uint64_t)p * 2 + 1];
        }
        if (pc >= a.npub) { if (lane == 0) atomicOr(a.err, kErrMismatch); continue; }
        const uint64_t ob = uni64(obv), oe = uni64(oev);
        if (oe > cap || ob > oe) {
          if (lane == 0) atomicOr(a.err, kErrOverflow);
          continue;
        }
        emit_keys2<NT>(a, hv, kv, ob, oe);
        written += oe - ob;
        wave_sync();
      }
      heavy_on = false;
    }
    if (groups_on || wide_on) {
      const GroupSlot* gs = reinterpret_cast<const GroupSlot*>(a.groups);
      const uint32_t nchunks = (a.npub + a.gpw - 1) / a.gpw;
      uint64_t si = gw, cur = 0, m = 0;
      uint32_t j = 0, gn = 0, c = (uint32_t)gw, cc = 0;
      for (;;) {
        uint32_t p = 0;
        bool have = false;
        if (groups_on) {
          while (j >= gn && si <= a.gs_mask) {
            const unsigned long long w = uni64(gs[si].word);
            gn = (w >> 40) == a.dd_tag ? (uint32_t)(w & 0xFF) : 0u;
            j = 0;
            cur = si;
            si += nwaves;
          }
          if (j < gn) { p = uni(gs[cur].m[j]); j++; have = true; }
          else groups_on = false;
        }
        if (!have && wide_on) {
          while (m == 0 && c < nchunks) { m = uni64(a.widemask[c]); cc = c; c += nwaves; }
          if (m) {
            p = cc * a.gpw + (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            have = true;
          } else {
            wide_on = false;
          }
        }
        if (!have) break;
        if (p >= a.npub) { if (lane == 0) atomicOr(a.err, kErrMismatch); continue; }
        const uint64_t ob = uni64(a.offsets[p]), oe = uni64(a.offsets[p + 1]);
        if (oe > cap || ob > oe) {
          if (lane == 0) atomicOr(a.err, kErrOverflow);
          continue;
        }
        const uint4* kc = reinterpret_cast<const uint4*>(a.keycache) + (uint64_t)p * 2;
        const uint4 h = kc[0], k1 = kc[1];
        if (uni(h.y) == kMany) emit_many<OUT, NT, VMQG_TAIL_U, 64>(a, Group<64>(), true, p, ob, oe, lds[wv].keys);
        else if (OUT == 0) emit_keys2<NT>(a, h, k1, ob, oe);
        written += oe - ob;
        wave_sync();
      }
    }
    // the block's entries in one global atomic (its last wave adds them)
    if (lane == 0) {
      if (written) __hip_atomic_fetch_add(&s_wsum, (unsigned long long)written, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (__hip_atomic_fetch_add(&s_wdone, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) == kWaves - 1) {
        const unsigned long long tot = __hip_atomic_load(&s_wsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (tot) atomicAdd(reinterpret_cast<unsigned long long*>(a.status + kStWideEnt), tot);
      }
    }
  }
}

// ------------------------------------------------------------------ scan
// Exclusive scan of the per-chunk totals COUNT wrote (one chunk = the GPW
// publishes one wave takes) into chunk bases, in ONE launch: tiles taken by
// ticket, chained by a decoupled look-back; writes offsets[npub] = the batch
// total.  EMIT turns a chunk base and its publishes' counts into their
// offsets, so the per-publish counts are read and written once, by EMIT,
// instead of by a scan pass of their own.
#ifndef VMQG_SCAN_ITEMS
#define VMQG_SCAN_ITEMS 16   // counts per thread (A/B: 4, 8, 16)
#endif
constexpr uint32_t kScanItems = VMQG_SCAN_ITEMS, kScanBlock = 256, kScanTile = kScanItems * kScanBlock;

__global__ __launch_bounds__(256) void k_scan_offsets(MatchArgs a) {
  __shared__ uint64_t part[kScanBlock];
  __shared__ uint32_t s_tile;
  __shared__ uint64_t s_base;
  const uint32_t nchunks = (a.npub + a.gpw - 1) / a.gpw;
  const uint64_t n = (uint64_t)nchunks + 1;
  const uint32_t ntiles = (uint32_t)((n + kScanTile - 1) / kScanTile);
  uint64_t* v = a.chunk;
  for (;;) {
    if (threadIdx.x == 0) s_tile = atomicAdd(&a.status[kStTicket], 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    if (tile >= ntiles) break;
    const uint64_t base = (uint64_t)tile * kScanTile + (uint64_t)threadIdx.x * kScanItems;
    uint64_t x[kScanItems];
    uint64_t acc = 0;
#pragma unroll
    for (uint32_t i = 0; i < kScanItems; i++) { x[i] = base + i < nchunks ? v[base + i] : 0; acc += x[i]; }
    part[threadIdx.x] = acc;
    __syncthreads();
    for (uint32_t o = 1; o < kScanBlock; o <<= 1) {
      const uint64_t t = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
      __syncthreads();
      part[threadIdx.x] += t;
      __syncthreads();
    }
    if (threadIdx.x < 64) {
      const uint64_t b = lookback(a.lookback, a.lb_tag, a.err, tile, part[kScanBlock - 1]);
      if (threadIdx.x == 0) s_base = b;
    }
    __syncthreads();
    uint64_t run = s_base + part[threadIdx.x] - acc;
#pragma unroll
    for (uint32_t i = 0; i < kScanItems; i++) {
      if (base + i < n) v[base + i] = run;
      if (base + i == nchunks) a.offsets[a.npub] = run;   // the batch total
      run += x[i];
    }
    __syncthreads();
  }
}

uint32_t scan_tiles(uint64_t nchunks) { return (uint32_t)((nchunks + 1 + kScanTile - 1) / kScanTile); }

// ---------------------------------------------------------------- patches
__global__ __launch_bounds__(256) void k_apply_patches(uint8_t* arena, const uint32_t* patches, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t* pr = patches + i * 6;
    const uint64_t off = (uint64_t)pr[0] | ((uint64_t)pr[1] << 32);
    *reinterpret_cast<uint4*>(arena + off) = make_uint4(pr[2], pr[3], pr[4], pr[5]);
  }
}

// One lane's fingerprint of its publish (claim / classify): the word loads
// are issued four at a time, not one dependent round trip per level.
__device__ __forceinline__ uint64_t lane_pub_fp(const MatchArgs& a, const vmqg_pub& pub) {
  const uint32_t* w = a.words + pub.word_off;
  const uint32_t n = pub.nwords;
  uint64_t part = 0;
  uint32_t i = 0;
  for (; i + 4 <= n; i += 4) {
    const uint32_t x0 = w[i], x1 = w[i + 1], x2 = w[i + 2], x3 = w[i + 3];
    part += fp_word(x0, i) + fp_word(x1, i + 1) + fp_word(x2, i + 2) + fp_word(x3, i + 3);
  }
  for (; i < n; i++) part += fp_word(w[i], i);
  return fp_final(part, pub.mountpoint, n);
}

// Two publishes' word ids equal (four loads in flight per step).
__device__ __forceinline__ bool lane_words_equal(const uint32_t* x, const uint32_t* y, uint32_t n) {
  bool eq = true;
  uint32_t k = 0;
  for (; eq && k + 4 <= n; k += 4)
    eq = ((x[k] ^ y[k]) | (x[k + 1] ^ y[k + 1]) | (x[k + 2] ^ y[k + 2]) | (x[k + 3] ^ y[k + 3])) == 0;
  for (; eq && k < n; k++) eq = x[k] == y[k];
  return eq;
}

// ------------------------------------------------ exact-filter sampling
// The exbits filter is worth its (L2-resident) word per lookup only while
// most exact lookups would miss the table: C's publishes never have an exact
// topic (filter on), R1's always do (filter off: it is then one more line per
// publish).  With option "exfilter" 2 (auto) the host launches this sampler
// before COUNT on the first call and every 64th: 4,096 publishes spread over
// the batch test their filter bit; the launch's last block turns the counts
// into the mode of the next calls (host-mapped dd_host[1]: 2 off, 3 on) —
// on while fewer than half of the lookups pass the filter.  COUNT itself
// counts nothing: per-publish counters cost the one-lane COUNT 13-25 us of
// 80 on config C (profiles/ab_r05_excount/).
constexpr uint32_t kExSamples = 4096;
__global__ __launch_bounds__(256) void k_ex_sample(MatchArgs a) {
  __shared__ uint32_t s_t, s_q;
  if (threadIdx.x == 0) { s_t = 0; s_q = 0; }
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  bool looked = false, pass = false;
  if (i < kExSamples && a.npub) {
    const uint32_t p = (uint32_t)((uint64_t)i * a.npub / kExSamples);
    const vmqg_pub pub = a.pubs[p];
    if (pub.mountpoint < a.max_mp && pub.nwords > 0) {
      const uint32_t* w = a.words + pub.word_off;
      bool wild;
      const uint64_t fp = publish_fp<1>(pub, w, w[0], Group<1>(), wild);
      if (!wild) {
        looked = true;
        const uint64_t xb = exbit_of(fp, a.exbits_mask + 1);
        pass = ((a.exbits[xb >> 5] >> (xb & 31)) & 1u) != 0;
      }
    }
  }
  const uint32_t nt = (uint32_t)__popcll(__ballot(looked)), nq = (uint32_t)__popcll(__ballot(pass));
  if (__lane_id() == 0 && nt) { atomicAdd(&s_t, nt); atomicAdd(&s_q, nq); }   // LDS
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint32_t* acc = a.dd_mode + 4;   // persistent words: looked up, passed, blocks done
  if (s_t) { atomicAdd(&acc[0], s_t); atomicAdd(&acc[1], s_q); }
  __threadfence();
  if (atomicAdd(&acc[2], 1u) != gridDim.x - 1) return;
  // the last block: every block's counts are in (each fenced before its ticket)
  const uint32_t t = atomicExch(&acc[0], 0u), q = atomicExch(&acc[1], 0u);
  atomicExch(&acc[2], 0u);
  if (t >= 256 && a.dd_host) a.dd_host[1] = (q * 2u < t ? 1u : 0u) + 2u;
}

hipError_t launch_ex_sample(const MatchArgs& a, hipStream_t st) {
  k_ex_sample<<<kExSamples / 256, 256, 0, st>>>(a);
  return hipGetLastError();
}

// ------------------------------------------------------------ dedupe claim
// Batch dedupe with the mode on: every publish stores its key and its id
// into its table slot with plain stores; within the launch the last writer
// wins (per XCD L2, then at write-back), and COUNT — one launch later, so
// every L2 sees the final table — reads the slot with plain loads: the last
// writer represents its topic, a publish of another topic in the slot just
// walks.  No atomics: a hot topic's slot is one line every publish of it
// would otherwise CAS (tools/atomic_probe.hip: 16 hot slots, 1.2 ms per
// 2^20 CAS; plain stores 7 us).
__global__ __launch_bounds__(256) void k_dd_claim(MatchArgs a) {
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < a.npub; p += gridDim.x * blockDim.x) {
    // COUNT accumulates the representatives' chunk totals, masks and bits
    if (p % a.gpw == 0) {
      const uint32_t c = p / a.gpw;
      a.chunk[c] = 0;
      a.widemask[c] = 0;
      a.ddmask[c] = 0;
    }
    if (p % 32 == 0) a.fastdone[p / 32] = 0;
    a.heavybyte[p] = 0;   // COUNT walks only the representatives
    const vmqg_pub pub = a.pubs[p];
    if (pub.nwords == 0 || pub.mountpoint >= a.max_mp) continue;
    const uint64_t fp = lane_pub_fp(a, pub);
    const uint32_t i = (uint32_t)(fp & a.dd_mask);
    a.dd_key[i] = dd_key_of(a, fp);
    a.dd_rep[i] = p;
  }
}

// After the claim: each publish reads its slot (plain loads: a hot topic's
// slot stays in L2).  The slot's last writer, or a publish whose slot holds
// another topic, walks: it joins the representatives' list (list 2, dense,
// buffered in LDS, one atomic per block); a publish whose words equal its
// slot's writer's is a duplicate (a bit in its chunk's mask, the
// representative at list 3 [publish]).  Each block takes one contiguous
// range of publishes.
constexpr uint32_t kClsBuf = 4096;
__global__ __launch_bounds__(256) void k_dd_classify(MatchArgs a) {
  __shared__ uint32_t buf[kClsBuf];
  __shared__ uint32_t nbuf, dups, base;
  if (threadIdx.x == 0) { nbuf = 0; dups = 0; }
  if (blockIdx.x == 0 && threadIdx.x == 0) a.status[kStDupTried] = a.npub;
  __syncthreads();
  const uint32_t per = (uint32_t)(((uint64_t)a.npub + gridDim.x - 1) / gridDim.x + 255) & ~255u;
  const uint32_t lo = blockIdx.x * per, hi = lo + per < a.npub ? lo + per : a.npub;
  for (uint32_t b0 = lo; b0 < hi; b0 += 256) {
    const uint32_t p = b0 + threadIdx.x;
    bool walk = false, dup = false;
    uint32_t rep = kNone;
    if (p < hi) {
      const vmqg_pub pub = a.pubs[p];
      walk = true;
      if (pub.nwords > 0 && pub.mountpoint < a.max_mp) {
        const uint64_t fp = lane_pub_fp(a, pub);
        const uint32_t i = (uint32_t)(fp & a.dd_mask);
        if (a.dd_key[i] == dd_key_of(a, fp)) {
          rep = a.dd_rep[i];
          if (rep != p && rep < a.npub) {
            // same MP, flags and word ids: the same answer (a word no filter
            // has is one id, and only the '$' flag, which the ids do not
            // carry, changes what the same ids match)
            const vmqg_pub R = a.pubs[rep];
            const bool eq = R.mountpoint == pub.mountpoint && R.nwords == pub.nwords && R.flags == pub.flags &&
                            lane_words_equal(a.words + R.word_off, a.words + pub.word_off, pub.nwords);
            dup = eq;
            walk = !eq;
          }
        }
      }
    }
    // A wave holds 64 consecutive publishes from a multiple of 64 (ranges
    // start at multiples of 256), so each of its chunks' duplicate masks is a
    // slice of one ballot, stored whole by the chunk's first lane: no atomics
    // on the mask words, and one LDS atomic per wave for each count.
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t m_dup = __ballot(dup), m_walk = __ballot(walk);
    if (dup) a.deferred[3ull * a.npub + p] = rep;
    if (p < hi && p % a.gpw == 0)
      a.ddmask[p / a.gpw] = (m_dup >> lane) & (a.gpw == 64 ? ~0ull : (1ull << a.gpw) - 1);
    uint32_t k0 = 0;
    if (lane == 0) {
      if (m_dup) atomicAdd(&dups, (uint32_t)__popcll(m_dup));   // LDS
      if (m_walk) k0 = atomicAdd(&nbuf, (uint32_t)__popcll(m_walk));   // LDS
    }
    k0 = uni(k0);
    if (walk) buf[k0 + prefix_bits(m_walk)] = p;
    __syncthreads();
    if (nbuf + 256 > kClsBuf || b0 + 256 >= hi) {   // flush: one global atomic for the block
      if (threadIdx.x == 0) base = nbuf ? atomicAdd(&a.status[kStReps], nbuf) : 0u;
      __syncthreads();
      for (uint32_t k = threadIdx.x; k < nbuf; k += blockDim.x) a.deferred[2ull * a.npub + base + k] = buf[k];
      __syncthreads();
      if (threadIdx.x == 0) nbuf = 0;
      __syncthreads();
    }
  }
  if (threadIdx.x == 0 && dups) atomicAdd(&a.status[kStDup], dups);
}

// After COUNT: every duplicate whose representative COUNT's fast pass
// served takes its key cache, spill slots and count (one lane per publish,
// one wave per 64 publishes, so the loads of many duplicates are in flight
// at once); the others — their representative was deferred — join list 0,
// which the COUNT wave tier walks like COUNT's own deferrals.
template <int OUT>
__global__ __launch_bounds__(256) void k_dd_fixup(MatchArgs a) {
  __shared__ uint32_t buf[kDefBuf];
  __shared__ uint32_t nbuf, base, n_many, n_walk, n_grp;
  if (threadIdx.x == 0) { nbuf = 0; n_many = 0; n_walk = 0; n_grp = 0; }
  __syncthreads();
  const uint32_t lane = __lane_id(), wv = threadIdx.x >> 6;
  const uint32_t stride = gridDim.x * kWaves * 64;
  for (uint32_t b0 = (blockIdx.x * kWaves + wv) * 64; b0 < a.npub; b0 += stride) {
    const uint32_t p = b0 + lane;
    const bool valid = p < a.npub && ((a.ddmask[p / a.gpw] >> (p % a.gpw)) & 1);
    bool ok = false, grouped = false, walk = false, heavy = false;
    uint64_t add = 0;
    if (valid) {
      const uint32_t rep = a.deferred[3ull * a.npub + p];
      ok = rep < a.npub && rep != p && ((a.fastdone[rep / 32] >> (rep % 32)) & 1u);
      walk = !ok;
      if (ok) {
        const uint4* rk = reinterpret_cast<const uint4*>(a.keycache) + (uint64_t)rep * 2;
        uint4* pk = reinterpret_cast<uint4*>(a.keycache) + (uint64_t)p * 2;
        uint4 h = rk[0];
        const uint4 k1 = rk[1];
        const uint64_t rmask = ((uint64_t)h.w << 32) | h.z;
        if (h.y != kMany && (h.y & kGroupFlag)) {   // the representative's output group (groups on only)
          grouped = OUT == 0 && a.groups && group_insert(a, group_sig_keys(k1, rmask), p);
          if (!grouped) h.y &= ~kGroupFlag;
        }
        pk[0] = h;
        pk[1] = k1;
        const uint32_t nkf = h.y == kMany ? 0u : h.y & ~(kHugeFlag | kGroupFlag | kHeavyFlag);
        if (h.y == kMany || (nkf > 2 && nkf <= kSpillKeys)) {   // spilled keys or candidate paths: 64 B
          const uint4* rs = reinterpret_cast<const uint4*>(a.keyspill + (uint64_t)rep * kSpillKeys);
          uint4* ps = reinterpret_cast<uint4*>(a.keyspill + (uint64_t)p * kSpillKeys);
#pragma unroll
          for (int q = 0; q < 4; q++) ps[q] = rs[q];
        }
        a.offsets[p] = h.x;
        add = h.x;
        if (h.y == kMany) {
          if (OUT == 0 && a.groups && h.x >= kGroupMin) {
            const uint32_t* cands = reinterpret_cast<const uint32_t*>(a.keyspill) + (uint64_t)p * 2 * kSpillKeys;
            grouped = group_insert(a, group_sig_many(k1.z, k1.w, (a.pubs[p].flags & VMQG_PUB_DOLLAR) != 0, rmask,
                                                     k1.x, [&](uint32_t c) { return cands[c]; }), p);
          }
          if (!grouped) atomicOr(reinterpret_cast<unsigned long long*>(a.widemask + p / a.gpw), 1ull << (p % a.gpw));
        } else if (h.y & kHugeFlag) {
          a.deferred[4ull * a.npub + atomicAdd(&a.status[kStHuge], 1u)] = p;
        } else if (h.y & kHeavyFlag) {   // the representative's bucket: the same first key
          a.heavybyte[p] = (uint8_t)(1 + heavy_bucket(k1.x));
          heavy = true;   // counted per wave below (one global atomic, not one per duplicate)
        }
      } else {
        a.offsets[p] = 0;
        reinterpret_cast<uint4*>(a.keycache)[(uint64_t)p * 2] = make_uint4(0, kDeferred, 0, 0);
      }
    }
    // the chunk totals: one atomic per chunk the wave covers
    if (a.gpw == 64) {
      const uint64_t tot = __shfl(wave_incl_scan64(add), 63, 64);
      if (lane == 0 && tot) atomicAdd(reinterpret_cast<unsigned long long*>(a.chunk + b0 / 64), (unsigned long long)tot);
    } else if (add) {
      atomicAdd(reinterpret_cast<unsigned long long*>(a.chunk + p / a.gpw), (unsigned long long)add);
    }
    const uint32_t nm = (uint32_t)__popcll(__ballot(ok && !grouped && reinterpret_cast<const uint4*>(a.keycache)[(uint64_t)p * 2].y == kMany));
    const uint32_t ng = (uint32_t)__popcll(__ballot(grouped));
    const uint32_t nhv = (uint32_t)__popcll(__ballot(heavy));
    if (lane == 0 && nhv) atomicAdd(&a.status[kStHeavy], nhv);
    const uint64_t wm = __ballot(walk);
    if (lane == 0) {
      if (nm) atomicAdd(&n_many, nm);
      if (ng) atomicAdd(&n_grp, ng);
      if (wm) atomicAdd(&n_walk, (uint32_t)__popcll(wm));
    }
    if (walk) {   // to list 0 (LDS buffer; a full buffer goes straight to the global list)
      const uint32_t k = atomicAdd(&nbuf, 1u);
      if (k < kDefBuf) buf[k] = p;
      else a.deferred[atomicAdd(&a.status[kStDeferred], 1u)] = p;
    }
  }
  __syncthreads();
  const uint32_t nd = nbuf < kDefBuf ? nbuf : kDefBuf;
  if (threadIdx.x == 0) base = nd ? atomicAdd(&a.status[kStDeferred], nd) : 0u;
  if (threadIdx.x == 64 && n_many) atomicAdd(&a.status[kStMany], n_many);
  if (threadIdx.x == 128 && n_walk) atomicAdd(&a.status[kStDupWalked], n_walk);
  if (threadIdx.x == 192 && n_grp) atomicAdd(&a.status[kStGrouped], n_grp);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nd; i += blockDim.x) a.deferred[base + i] = buf[i];
}

// ---------------------------------------------------------------- launch
static inline uint32_t div_up(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

hipError_t launch_dd_fixup(const MatchArgs& a, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
  uint32_t g = div_up(a.npub, kWaves * 64);
  if (g > (uint32_t)a.cus * 8) g = (uint32_t)a.cus * 8;
  if (g < 1) g = 1;
  if (a.out_rng) {
    if (t0) hipExtLaunchKernelGGL(k_dd_fixup<1>, dim3(g), dim3(256), 0, st, t0, t1, 0, a);
    else k_dd_fixup<1><<<g, 256, 0, st>>>(a);
  } else {
    if (t0) hipExtLaunchKernelGGL(k_dd_fixup<0>, dim3(g), dim3(256), 0, st, t0, t1, 0, a);
    else k_dd_fixup<0><<<g, 256, 0, st>>>(a);
  }
  return hipGetLastError();
}

hipError_t launch_dd_classify(const MatchArgs& a, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
  uint32_t g = a.cus * 8;   // one contiguous range of publishes per block: 8 blocks per CU
  if (g > div_up(a.npub, 256)) g = div_up(a.npub, 256);
  if (g < 1) g = 1;
  if (t0) hipExtLaunchKernelGGL(k_dd_classify, dim3(g), dim3(256), 0, st, t0, t1, 0, a);
  else k_dd_classify<<<g, 256, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_dd_claim(const MatchArgs& a, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
  uint32_t g = div_up(a.npub, 256);
  if (g > a.cus * 8) g = a.cus * 8;
  if (g < 1) g = 1;
  if (t0) hipExtLaunchKernelGGL(k_dd_claim, dim3(g), dim3(256), 0, st, t0, t1, 0, a);
  else k_dd_claim<<<g, 256, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_scan(const MatchArgs& a, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
  uint32_t g = scan_tiles((a.npub + a.gpw - 1) / a.gpw);
  if (g > 2048) g = 2048;
  if (t0) hipExtLaunchKernelGGL(k_scan_offsets, dim3(g), dim3(kScanBlock), 0, st, t0, t1, 0, a);
  else k_scan_offsets<<<g, kScanBlock, 0, st>>>(a);
  return hipGetLastError();
}

// ============================================ COUNT over trie-less tables
// When the device tables hold no trie edge (every subscription exact: the
// reference's bench_single_lookups, R1; one hot topic, R2), a publish's
// only candidates are its exact topic's local key and remote subscribers
// (vmq_reg_trie.erl:62, 73-84, 514-520): COUNT is one exact-table probe.
// The walk's machinery (LDS stacks, per-step ballots) is skipped, and each
// lane takes K publishes of K chunks at once — their publish, word and
// bucket loads issued together — so K random lines per lane are in flight
// instead of one dependent chain after another (the one-lane COUNT waits
// 83 % of its cycles on memory on R1: SQ_WAIT_ANY / SQ_WAVE_CYCLES).
// Writes exactly what the fast COUNT writes for such a publish: offsets,
// the key cache (<= 1 key), heavy bytes, chunk totals, chunk wide masks (0);
// a publish with remote nodes >= 64 goes to list 0 for the wave tier, a huge
// one to the tail's list.
constexpr uint32_t kExK = 4;
template <int OUT>
__global__ __launch_bounds__(256) void k_count_exact(MatchArgs a) {
  if (blockIdx.x == 0 && threadIdx.x < kStWords) a.status_next[threadIdx.x] = 0;
  const uint32_t lane = __lane_id(), wv = threadIdx.x >> 6;
  const uint32_t nchunks = (a.npub + 63) / 64;
  const uint32_t step = gridDim.x * kWaves * kExK;
  for (uint32_t c0 = (blockIdx.x * kWaves + wv) * kExK; c0 < nchunks; c0 += step) {
    vmqg_pub pub[kExK];
    bool look[kExK];
    uint64_t fp[kExK];
#pragma unroll
    for (uint32_t k = 0; k < kExK; k++) {
      const uint32_t p = (c0 + k) * 64 + lane;
      pub[k] = p < a.npub ? a.pubs[p] : vmqg_pub{0xFFFFFFFFu, 0, 0, 0};
    }
    // fingerprints: every publish's words in flight together
#pragma unroll
    for (uint32_t k = 0; k < kExK; k++) {
      const uint32_t L = pub[k].nwords;
      const uint32_t* w = a.words + pub[k].word_off;
      look[k] = pub[k].mountpoint < a.max_mp && L > 0;
      uint64_t part = 0;
      bool wild = false;
      for (uint32_t i = 0; look[k] && i < L; i++) {
        const uint32_t x = w[i];
        part += fp_word(x, i);
        wild |= x == kPlus || x == kHash;
      }
      fp[k] = fp_final(part, pub[k].mountpoint, L);
      // a '+' / '#' word equals only a wildcard topic, which has no filter bit
      if (look[k] && !wild && a.exfilter) {
        const uint64_t xb = exbit_of(fp[k], a.exbits_mask + 1);
        look[k] = ((a.exbits[xb >> 5] >> (xb & 31)) & 1u) != 0;
      }
    }
    // the buckets' first slots, all in flight (the second slot is a 64-B
    // memory request of its own: read only when the first does not match)
    uint4 h0[kExK];
#pragma unroll
    for (uint32_t k = 0; k < kExK; k++) {
      if (look[k]) {
        const ExactSlot* bk = a.exact + (fp[k] & a.exact_mask) * kExactSlotsPerBucket;
        h0[k] = *reinterpret_cast<const uint4*>(&bk[0]);   // {fp lo, fp hi, nwords, words_off}
      }
    }
#pragma unroll
    for (uint32_t k = 0; k < kExK; k++) {
      const uint32_t p = (c0 + k) * 64 + lane;
      const bool valid = p < a.npub;
      const uint32_t L = pub[k].nwords;
      const uint32_t* w = a.words + pub[k].word_off;
      // the slot is read as whole 16-B quarters ({fp, nwords, words_off},
      // {off, count, rmask}, {mp, w0..w2}, {w3..w6}): each load instruction is
      // one L2 request per lane, so a field-by-field read costs the probe
      // several requests to the same line
      bool found = false, deferred = false;
      uint4 hit{0, 0, 0, 0};
      if (look[k]) {
        uint64_t b = fp[k] & a.exact_mask;
        uint4 s0 = h0[k];
        for (uint64_t iter = 0; iter <= a.exact_mask && !found; iter++) {
          const ExactSlot* bk = a.exact + b * kExactSlotsPerBucket;
          bool empty = false;
#pragma unroll
          for (uint32_t j = 0; j < kExactSlotsPerBucket; j++) {
            if (found || empty) continue;
            const uint4 sj = j == 0 ? s0 : *reinterpret_cast<const uint4*>(&bk[j]);
            if (sj.z == kEmpty) { empty = true; continue; }
            const uint64_t f = ((uint64_t)sj.y << 32) | sj.x;
            if (f != fp[k] || (sj.z & ~kExactFlags) != L) continue;
            const uint4* q = reinterpret_cast<const uint4*>(&bk[j]);
            const uint4 q2 = q[2];   // {mp, w0, w1, w2}
            bool diff = q2.x != pub[k].mountpoint;
            diff |= (L > 0 && q2.y != w[0]) || (L > 1 && q2.z != w[1]) || (L > 2 && q2.w != w[2]);
            if (!diff && L > 3) {
              const uint4 q3 = q[3];   // {w3, w4, w5, w6}
              diff |= q3.x != w[3] || (L > 4 && q3.y != w[4]) || (L > 5 && q3.z != w[5]) || (L > 6 && q3.w != w[6]);
            }
            for (uint32_t i = kExactInline; !diff && i < L; i++) diff |= a.exwords[sj.w + (i - kExactInline)] != w[i];
            if (!diff) {
              found = true;
              hit = q[1];   // {off, count, rmask lo, hi}
              deferred = (sj.z & kExactHigh) != 0;   // remote nodes >= 64: the wave tier
            }
          }
          if (found || empty) break;
          b = (b + 1) & a.exact_mask;   // the bucket is full: the next one
          s0 = *reinterpret_cast<const uint4*>(&a.exact[b * kExactSlotsPerBucket]);
        }
      }
      // the fold of fold_/5 and lookup_subs/1 for the one candidate
      const uint32_t off = hit.x, cnt = hit.y;
      uint64_t rmask = ((uint64_t)hit.w << 32) | hit.z;
      if (a.local_node < kLowNodes) rmask &= ~(1ull << a.local_node);
      const uint32_t nk = cnt ? 1u : 0u;
      const uint32_t total = OUT ? nk + (uint32_t)__popcll(rmask) : cnt + (uint32_t)__popcll(rmask);
      uint32_t hb = 0, cnt_out = 0;
      bool heavy = false;
      if (valid) {
        uint4* kc = reinterpret_cast<uint4*>(a.keycache) + (uint64_t)p * 2;
        if (deferred) {
          const uint32_t idx = atomicAdd(&a.status[kStDeferred], 1u);
          a.deferred[idx] = p;
          a.offsets[p] = 0;
          kc[0] = make_uint4(0, kDeferred, 0, 0);
        } else {
          cnt_out = total;
          a.offsets[p] = total;
          const bool huge = OUT == 0 && total >= kHugeRecords;
          uint32_t hf = huge ? kHugeFlag : 0u;
          if (huge) a.deferred[4ull * a.npub + atomicAdd(&a.status[kStHuge], 1u)] = p;
          else if (OUT == 0 && a.heavy_min && total >= a.heavy_min) {
            hf = kHeavyFlag;
            heavy = true;
            hb = 1 + heavy_bucket(nk ? off : 0u);
          }
          kc[0] = make_uint4(total, nk | hf, (uint32_t)rmask, (uint32_t)(rmask >> 32));
          kc[1] = make_uint4(nk ? off : 0u, cnt, 0u, 0u);
        }
        a.heavybyte[p] = (uint8_t)hb;
      }
      // the totals and (empty) wide masks of the gpw-publish chunks these 64
      // publishes make up: what the fast pass stores
      const uint64_t incl = wave_incl_scan64(cnt_out);
      const uint32_t gpw = a.gpw;
      const uint32_t first = lane & ~(gpw - 1), last = first + gpw - 1;
      const uint64_t hi = __shfl(incl, (int)last, 64);
      const uint64_t lo = __shfl(incl, first ? (int)first - 1 : 0, 64);
      const uint32_t nh = (uint32_t)__popcll(__ballot(heavy));
      if (lane == first && p < a.npub) {
        a.chunk[p / gpw] = hi - (first ? lo : 0ull);
        a.widemask[p / gpw] = 0;
      }
      if (lane == 0 && nh) atomicAdd(&a.status[kStHeavy], nh);
    }
  }
}

template <int OUT>
static void launch_count_exact(const MatchArgs& a, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
  const uint32_t nchunks = (a.npub + 63) / 64;
  uint32_t g = div_up(nchunks, kWaves * kExK);
  const uint32_t cap = (uint32_t)a.cus * 8u;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  if (t0) hipExtLaunchKernelGGL(k_count_exact<OUT>, dim3(g), dim3(256), 0, st, t0, t1, 0, a);
  else k_count_exact<OUT><<<g, 256, 0, st>>>(a);
}

#ifndef VMQG_EMIT_EXACT
#define VMQG_EMIT_EXACT 1   // A/B: 0 = trie-less batches take the general EMIT
#endif
#ifndef VMQG_EMIT_EXK
#define VMQG_EMIT_EXK 2   // 64-publish blocks per wave in flight in k_emit_exact (A/B on R1: 1 / 2 / 4 / 8)
#endif
constexpr uint32_t kExE = VMQG_EMIT_EXK;
#ifndef VMQG_EMIT_EXACT_WPE
#define VMQG_EMIT_EXACT_WPE 1   // waves per SIMD the register budget must allow (1: no bound)
#endif
// ============================================= EMIT over trie-less tables
// The EMIT of a k_count_exact COUNT: a publish has at most its exact
// topic's key (its records) and remote nodes, so nothing needs resolving —
// one lane per publish, kExK 64-publish blocks per wave with their offset,
// key-cache and chunk-base loads in flight together (the general EMIT takes
// a 64-publish chunk at a time, two lanes per publish, through the key-cache
// resolve and LDS GroupMeta: R1 spends 190 us there for one record a
// publish).  Writes what the general EMIT writes: every publish's final
// offset, and the records (or ranges) of the publishes it serves; deferred
// (kDeferred), wide (kMany), huge and heavy publishes are left to the wave
// tier / EMIT tail as there.  Records mode: a block whose publishes emit at
// most one record each is written lane by lane (consecutive positions: the
// stores coalesce); any other block is copied by the whole wave over the
// concatenated record spans, U records per lane in flight.
struct ExEmitLds {
  uint4 h[64], k[64];   // key-cache words of the block's publishes
  uint64_t ob[64];      // their output positions
  uint32_t crel[65];    // exclusive scan of the served spans
};

__device__ __forceinline__ uint4 exact_emission(const MatchArgs& a, uint32_t p, uint4 h, uint4 k, uint32_t r) {
  const uint32_t nk = h.y, c0 = k.y, ks = k.y + k.w;
  const uint64_t rm = ((uint64_t)h.w << 32) | h.z;
  if (nk > 2) {   // spilled keys (not produced by a trie-less COUNT; kept general)
    const uint2* sp = a.keyspill + (uint64_t)p * kSpillKeys;
    return emission(a, [&](uint32_t i) -> uint2 { return sp[i]; }, nk, ks, rm, r);
  }
  if (r < c0) return *reinterpret_cast<const uint4*>(a.records + k.x + r);
  if (r < ks) return *reinterpret_cast<const uint4*>(a.records + k.z + (r - c0));
  return make_uint4((VMQG_EMIT_REMOTE << 24) | select_bit(rm, r - ks), kNone, kNone, kNone);
}

template <int OUT, bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VMQG_EMIT_EXACT_WPE)))
void k_emit_exact(MatchArgs a) {
  __shared__ ExEmitLds lds[kWaves];
  const uint32_t lane = __lane_id(), wv = threadIdx.x >> 6;
  ExEmitLds& L = lds[wv];
  const uint32_t nblk = (a.npub + 63) / 64;
  const uint32_t step = gridDim.x * kWaves * kExE;
  const uint64_t cap = OUT ? a.rng_cap : a.out_cap;
  const uint32_t gpw = a.gpw;
  const uint32_t seg = lane & ~(gpw - 1);   // first lane of this lane's gpw-publish chunk
  for (uint32_t b0 = (blockIdx.x * kWaves + wv) * kExE; b0 < nblk; b0 += step) {
    uint64_t cnt[kExE], cb[kExE];
    uint4 h[kExE], k[kExE];
#pragma unroll
    for (uint32_t j = 0; j < kExE; j++) {
      const uint32_t p = (b0 + j) * 64 + lane;
      const bool valid = p < a.npub;
      cnt[j] = valid ? a.offsets[p] : 0ull;
      cb[j] = valid ? a.chunk[p / gpw] : 0ull;
      const uint4* kc = reinterpret_cast<const uint4*>(a.keycache) + (uint64_t)p * 2;
      h[j] = valid ? kc[0] : make_uint4(0, kDeferred, 0, 0);
      k[j] = valid ? kc[1] : make_uint4(0, 0, 0, 0);
    }
    // positions: the chunk's base plus the exclusive prefix within the chunk
    uint64_t ob[kExE];
    bool ok[kExE];
    uint32_t single = 0;   // bit j: block j's served publishes emit <= 1 entry each
#pragma unroll
    for (uint32_t j = 0; j < kExE; j++) {
      const uint32_t p = (b0 + j) * 64 + lane;
      const bool valid = p < a.npub;
      const uint64_t incl = wave_incl_scan64(cnt[j]);
      const uint64_t lo = __shfl(incl, seg ? (int)seg - 1 : 0, 64);
      ob[j] = cb[j] + incl - cnt[j] - (seg ? lo : 0ull);
      if (valid) a.offsets[p] = ob[j];
      const uint32_t hy = h[j].y;
      ok[j] = valid && hy != kDeferred && hy != kMany && !(hy & (kHugeFlag | kGroupFlag | kHeavyFlag));
      if (ok[j] && ob[j] + cnt[j] > cap) { atomicOr(a.err, kErrOverflow); ok[j] = false; }
      if (ok[j] && cnt[j] != h[j].x) { atomicOr(a.err, kErrMismatch); ok[j] = false; }
      if (__ballot(ok[j] && (cnt[j] > 1 || hy > 2)) == 0) single |= 1u << j;
    }
    if constexpr (OUT == 1) {
      // ranges: {record off, count} per non-empty key, then {node, 0} per
      // remote node (emit_ranges_group's order)
#pragma unroll
      for (uint32_t j = 0; j < kExE; j++) {
        if (!ok[j]) continue;
        const uint32_t p = (b0 + j) * 64 + lane;
        const uint32_t nk = h[j].y;
        const uint64_t rm = ((uint64_t)h[j].w << 32) | h[j].z;
        uint64_t o = ob[j];
        if (nk > 2) {
          const uint2* sp = a.keyspill + (uint64_t)p * kSpillKeys;
          const uint32_t ks = k[j].y + k[j].w;
          for (uint32_t i = 0; i < nk; i++) {
            const uint2 e = sp[i];
            const uint32_t c = (i + 1 < nk ? sp[i + 1].y : ks) - e.y;
            if (c) store_range(a.out_rng, o++, e.x, c);
          }
        } else {
          if (k[j].y) store_range(a.out_rng, o++, k[j].x, k[j].y);
          if (k[j].w) store_range(a.out_rng, o++, k[j].z, k[j].w);
        }
        for (uint64_t m = rm; m; m &= m - 1) store_range(a.out_rng, o++, (uint32_t)__builtin_ctzll(m), 0u);
      }
    } else {
      // blocks of <= 1 record per publish: every lane's record loaded, then stored
      uint4 v[kExE];
#pragma unroll
      for (uint32_t j = 0; j < kExE; j++)
        if ((single >> j) & 1u && ok[j] && cnt[j] == 1) {   // key 0's record, key 1's, or the one remote node
          const uint64_t rm = ((uint64_t)h[j].w << 32) | h[j].z;
          v[j] = k[j].y ? *reinterpret_cast<const uint4*>(a.records + k[j].x)
                 : k[j].w ? *reinterpret_cast<const uint4*>(a.records + k[j].z)
                          : make_uint4((VMQG_EMIT_REMOTE << 24) | (uint32_t)__builtin_ctzll(rm), kNone, kNone, kNone);
        }
#pragma unroll
      for (uint32_t j = 0; j < kExE; j++)
        if ((single >> j) & 1u && ok[j] && cnt[j] == 1) store_rec<NT>(a.out, ob[j], v[j]);
      // the other blocks: the whole wave over the block's served spans (the
      // key cache and the positions just written re-read, L2 hits, rather
      // than held in registers across the blocks: 88 VGPRs instead of 132)
      uint32_t okm = 0;
#pragma unroll
      for (uint32_t j = 0; j < kExE; j++) okm |= ok[j] ? 1u << j : 0u;
#pragma unroll 1
      for (uint32_t j = 0; j < kExE; j++) {
        if ((single >> j) & 1u) continue;
        const uint32_t p = (b0 + j) * 64 + lane;
        const bool okj = (okm >> j) & 1u;
        const uint4* kc = reinterpret_cast<const uint4*>(a.keycache) + (uint64_t)p * 2;
        const uint4 hj = okj ? kc[0] : make_uint4(0, 0, 0, 0), kj = okj ? kc[1] : make_uint4(0, 0, 0, 0);
        const uint32_t sp = okj ? hj.x : 0u;   // == its count (checked above)
        const uint32_t incl = wave_incl_scan32(sp);
        L.h[lane] = hj;
        L.k[lane] = kj;
        L.ob[lane] = okj ? a.offsets[p] : 0ull;
        L.crel[lane] = incl - sp;
        if (lane == 63) L.crel[64] = incl;
        wave_sync();
        const uint32_t T = L.crel[64];
        constexpr int U = 4;
        uint32_t q = 0;   // the publish of record r: a cursor moving forward with r
        for (uint32_t r0 = lane; r0 < T; r0 += 64 * U) {
          uint4 v2[U];
          uint64_t dst[U];
#pragma unroll
          for (int u = 0; u < U; u++) {
            const uint32_t r = r0 + 64 * u;
            if (r < T) {
              while (q + 1 < 64 && L.crel[q + 1] <= r) q++;
              const uint32_t rr = r - L.crel[q];
              v2[u] = exact_emission(a, (b0 + j) * 64 + q, L.h[q], L.k[q], rr);
              dst[u] = L.ob[q] + rr;
            }
          }
#pragma unroll
          for (int u = 0; u < U; u++)
            if (r0 + 64 * u < T) store_rec<NT>(a.out, dst[u], v2[u]);
        }
        wave_sync();
      }
    }
  }
}

template <int OUT>
static void launch_emit_exact(const MatchArgs& a, bool nt, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
  const uint32_t nblk = (a.npub + 63) / 64;
  uint32_t g = div_up(nblk, kWaves * kExE);
  const uint32_t cap = (uint32_t)a.cus * 8u;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  if (nt) {
    if (t0) hipExtLaunchKernelGGL(k_emit_exact<OUT, true>, dim3(g), dim3(256), 0, st, t0, t1, 0, a);
    else k_emit_exact<OUT, true><<<g, 256, 0, st>>>(a);
  } else {
    if (t0) hipExtLaunchKernelGGL(k_emit_exact<OUT, false>, dim3(g), dim3(256), 0, st, t0, t1, 0, a);
    else k_emit_exact<OUT, false><<<g, 256, 0, st>>>(a);
  }
}

// ================ COUNT, scan and EMIT in one launch over trie-less tables
// (option "fused", on by default).  The trie-less COUNT above hands EMIT a
// 32-B key cache, a heavy byte and an offset per publish through HBM and
// EMIT reads them back behind a scan launch; here one kernel probes, counts,
// scans and writes: tiles of kFxTile publishes taken by ticket, each wave
// kFxK 64-publish chunks with all their probes in flight (as
// k_count_exact), the tile's base from a decoupled look-back, then every
// publish's offset and entries.  Nothing is handed over except a huge
// records-mode publish (>= kHugeRecords records): its key cache and the
// tail's list, as k_count_exact leaves them.  Remote nodes >= 64 (the exact
// slot's high list) are emitted here too, from exwords.
#ifndef VMQG_FX_K
#define VMQG_FX_K 2   // 64-publish chunks per wave per tile (A/B on R1: 1, 2, 3, 4, 6, 8)
#endif
#ifndef VMQG_FX_PREFETCH
#define VMQG_FX_PREFETCH 0   // 1: a one-record publish's record loaded before the look-back (A/B: more VGPRs)
#endif
#ifndef VMQG_FX_U
#define VMQG_FX_U 4   // entries per lane in flight in the whole-wave copy
#endif
#ifndef VMQG_FX_BPC
#define VMQG_FX_BPC 4   // fused blocks per CU
#endif
#ifndef VMQG_FX_DEFER
#define VMQG_FX_DEFER 1   // a tile's look-back and entries one iteration after its probes (0: at once)
#endif
constexpr uint32_t kFxK = VMQG_FX_K;
constexpr uint32_t kFxTile = kWaves * kFxK * 64;
struct FxWave {
  uint32_t off[64], cnt[64], hoff[64], nh[64];
  uint64_t rm[64], ob[64];
  uint32_t crel[65];
};
// one tile's per-publish results, held from its probes to its entries (the
// tile's look-back is resolved one iteration later: VMQG_FX_DEFER)
struct FxState {
  uint32_t off[kFxK][64], cnt[kFxK][64], hoff[kFxK][64], tot[kFxK][64];
  uint64_t rm[kFxK][64];
  uint4 one[kFxK][64];
  uint32_t onem[64];
};
struct FxLds {
  uint64_t wtot[kWaves], wprev[kWaves];
  uint64_t base, agg, agg_prev;
  uint32_t tile;
  FxWave w[kWaves];
#if VMQG_FX_DEFER
  FxState t[kWaves];
#endif
};

// the r-th entry of a publish: its key's records, then its remote nodes
// (< 64 from the mask, then the high list), as fold_/5 (vmq_reg_trie.erl:68-84)
__device__ __forceinline__ uint4 fx_emission(const MatchArgs& a, uint32_t off, uint32_t cnt, uint64_t rm, uint32_t hoff,
                                             uint32_t r) {
  if (r < cnt) return *reinterpret_cast<const uint4*>(a.records + off + r);
  const uint32_t nr = (uint32_t)__popcll(rm);
  const uint32_t node = r - cnt < nr ? select_bit(rm, r - cnt) : a.exwords[hoff + 1 + (r - cnt - nr)];
  return make_uint4((VMQG_EMIT_REMOTE << 24) | node, kNone, kNone, kNone);
}

// One 64-publish chunk's offsets and entries (lane = publish p at output
// offset ob): ranges; records — a huge publish left for the EMIT tail, a
// one-entry publish by its own lane, the rest by the whole wave over their
// concatenated entries, U per lane in flight.
template <int OUT, bool NT>
__device__ __forceinline__ void fx_emit_chunk(const MatchArgs& a, FxWave& W, uint32_t p, uint64_t ob, uint64_t cap,
                                              uint32_t off, uint32_t cnt, uint32_t hoff, uint32_t tot, uint64_t rm,
                                              bool has_one, uint4 one) {
  const uint32_t lane = __lane_id();
  const bool valid = p < a.npub;
  const uint32_t nh = hoff != kNone ? a.exwords[hoff] : 0u;   // remote nodes >= 64 (rare: re-read)
  if (valid) a.offsets[p] = ob;
  bool ok = valid && tot > 0;
  if (ok && ob + tot > cap) { atomicOr(a.err, kErrOverflow); ok = false; }
  if constexpr (OUT == 1) {
    if (ok) {
      uint64_t o = ob;
      if (cnt) store_range(a.out_rng, o++, off, cnt);
      for (uint64_t m = rm; m; m &= m - 1) store_range(a.out_rng, o++, (uint32_t)__builtin_ctzll(m), 0u);
      for (uint32_t i = 0; i < nh; i++) store_range(a.out_rng, o++, a.exwords[hoff + 1 + i], 0u);
    }
  } else {
    // a huge publish: the EMIT tail copies it with every wave (its key cache and list, as k_count_exact)
    const bool huge = ok && tot >= kHugeRecords && nh == 0;
    if (huge) {
      uint4* kc = reinterpret_cast<uint4*>(a.keycache) + (uint64_t)p * 2;
      const uint32_t nk = cnt ? 1u : 0u;
      kc[0] = make_uint4(tot, nk | kHugeFlag, (uint32_t)rm, (uint32_t)(rm >> 32));
      kc[1] = make_uint4(nk ? off : 0u, cnt, 0u, 0u);
      a.deferred[4ull * a.npub + atomicAdd(&a.status[kStHuge], 1u)] = p;
      ok = false;
    }
    if (ok && tot == 1) {   // one entry: this lane writes it (the chunk's stores coalesce)
      store_rec<NT>(a.out, ob, has_one ? one : fx_emission(a, off, cnt, rm, hoff, 0));
      ok = false;
    }
    if (__ballot(ok)) {
      const uint32_t sp = ok ? tot : 0u;
      const uint32_t in32 = wave_incl_scan32(sp);
      W.off[lane] = off; W.cnt[lane] = cnt; W.rm[lane] = rm; W.hoff[lane] = hoff;
      W.ob[lane] = ob;
      W.crel[lane] = in32 - sp;
      if (lane == 63) W.crel[64] = in32;
      wave_sync();
      const uint32_t T = W.crel[64];
      constexpr int U = VMQG_FX_U;
      uint32_t q = 0;
      for (uint32_t r0 = lane; r0 < T; r0 += 64 * U) {
        uint4 v[U];
        uint64_t dst[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint32_t r = r0 + 64 * u;
          if (r < T) {
            while (q + 1 < 64 && W.crel[q + 1] <= r) q++;
            const uint32_t rr = r - W.crel[q];
            v[u] = fx_emission(a, W.off[q], W.cnt[q], W.rm[q], W.hoff[q], rr);
            dst[u] = W.ob[q] + rr;
          }
        }
#pragma unroll
        for (int u = 0; u < U; u++)
          if (r0 + 64 * u < T) store_rec<NT>(a.out, dst[u], v[u]);
      }
      wave_sync();
    }
  }
}

template <int OUT, bool NT>
__global__ __launch_bounds__(256) void k_match_exact_fused(MatchArgs a) {
  __shared__ FxLds S;
  if (blockIdx.x == 0 && threadIdx.x < kStWords) a.status_next[threadIdx.x] = 0;
  const uint32_t lane = __lane_id(), wv = threadIdx.x >> 6;
  FxWave& W = S.w[wv];
  const uint32_t ntiles = (a.npub + kFxTile - 1) / kFxTile;
  const uint64_t cap = OUT ? a.rng_cap : a.out_cap;
#if VMQG_FX_DEFER
  FxState& T = S.t[wv];
  uint32_t prev = kNone;   // the tile probed in the previous iteration, entries not yet written (block-uniform)
#endif
  for (;;) {
#if VMQG_FX_DEFER
    // the block that holds the last tile knows no later ticket is a tile
    if (threadIdx.x == 0)
      S.tile = prev != kNone && prev + 1 >= ntiles ? ntiles : atomicAdd(&a.status[kStTicket], 1u);
#else
    if (threadIdx.x == 0) S.tile = atomicAdd(&a.status[kStTicket], 1u);
#endif
    __syncthreads();
    const uint32_t tile = S.tile;
#if VMQG_FX_DEFER
    const bool have = tile < ntiles;
    if (!have && prev == kNone) break;
    const bool probe_on = have;   // a block past the last tile still writes its previous tile's entries
    const uint32_t p0 = (have ? tile : 0u) * kFxTile + wv * (kFxK * 64);
#else
    if (tile >= ntiles) break;
    constexpr bool probe_on = true;
    const uint32_t p0 = tile * kFxTile + wv * (kFxK * 64);
#endif
    // ---- probes (k_count_exact's, kFxK chunks in flight)
    vmqg_pub pub[kFxK];
    bool look[kFxK];
    uint64_t fp[kFxK];
#pragma unroll
    for (uint32_t k = 0; k < kFxK; k++) {
      const uint32_t p = p0 + k * 64 + lane;
      pub[k] = probe_on && p < a.npub ? a.pubs[p] : vmqg_pub{0xFFFFFFFFu, 0, 0, 0};
    }
#pragma unroll
    for (uint32_t k = 0; k < kFxK; k++) {
      const uint32_t L = pub[k].nwords;
      const uint32_t* w = a.words + pub[k].word_off;
      look[k] = pub[k].mountpoint < a.max_mp && L > 0;
      uint64_t part = 0;
      bool wild = false;
      for (uint32_t i = 0; look[k] && i < L; i++) {
        const uint32_t x = w[i];
        part += fp_word(x, i);
        wild |= x == kPlus || x == kHash;
      }
      fp[k] = fp_final(part, pub[k].mountpoint, L);
      if (look[k] && !wild && a.exfilter) {
        const uint64_t xb = exbit_of(fp[k], a.exbits_mask + 1);
        look[k] = ((a.exbits[xb >> 5] >> (xb & 31)) & 1u) != 0;
      }
    }
    uint4 h0[kFxK];
#pragma unroll
    for (uint32_t k = 0; k < kFxK; k++)
      if (look[k]) h0[k] = *reinterpret_cast<const uint4*>(&a.exact[(fp[k] & a.exact_mask) * kExactSlotsPerBucket]);
    uint32_t off[kFxK], cnt[kFxK], hoff[kFxK], tot[kFxK];   // held across the look-back: kept lean
    uint64_t rm[kFxK];
    uint4 one[kFxK];   // a one-record publish's record, from its slot (or loaded while the tile is scanned)
    uint32_t onem = 0;
#pragma unroll
    for (uint32_t k = 0; k < kFxK; k++) {
      const uint32_t L = pub[k].nwords;
      const uint32_t* w = a.words + pub[k].word_off;
      bool found = false, has_one = false;
      uint4 hit{0, 0, 0, 0};
      uint32_t hi_at = kNone;
      if (look[k]) {
        uint64_t b = fp[k] & a.exact_mask;
        uint4 s0 = h0[k];
        for (uint64_t iter = 0; iter <= a.exact_mask && !found; iter++) {
          const ExactSlot* bk = a.exact + b * kExactSlotsPerBucket;
          bool empty = false;
#pragma unroll
          for (uint32_t j = 0; j < kExactSlotsPerBucket; j++) {
            if (found || empty) continue;
            const uint4 sj = j == 0 ? s0 : *reinterpret_cast<const uint4*>(&bk[j]);
            if (sj.z == kEmpty) { empty = true; continue; }
            const uint64_t f = ((uint64_t)sj.y << 32) | sj.x;
            if (f != fp[k] || (sj.z & ~kExactFlags) != L) continue;
            const uint4* q = reinterpret_cast<const uint4*>(&bk[j]);
            // the rest of the slot's line at once: its words, records and,
            // for a short topic with one record, that record (kExactOne)
            const bool inl = OUT == 0 && (sj.z & kExactOne) != 0;
            const uint4 q1 = q[1], q2 = q[2];
            const uint4 q3 = (L > 3 || inl) ? q[3] : make_uint4(0, 0, 0, 0);
            bool diff = q2.x != pub[k].mountpoint;
            diff |= (L > 0 && q2.y != w[0]) || (L > 1 && q2.z != w[1]) || (L > 2 && q2.w != w[2]);
            if (L > 3)
              diff |= q3.x != w[3] || (L > 4 && q3.y != w[4]) || (L > 5 && q3.z != w[5]) || (L > 6 && q3.w != w[6]);
            for (uint32_t i = kExactInline; !diff && i < L; i++) diff |= a.exwords[sj.w + (i - kExactInline)] != w[i];
            if (!diff) {
              found = true;
              hit = q1;
              if (inl) { one[k] = q3; has_one = true; }
              if (sj.z & kExactHigh) hi_at = sj.w + exact_tail_words(L);   // {count, node ids} of nodes >= 64
            }
          }
          if (found || empty) break;
          b = (b + 1) & a.exact_mask;
          s0 = *reinterpret_cast<const uint4*>(&a.exact[b * kExactSlotsPerBucket]);
        }
      }
      off[k] = hit.x;
      cnt[k] = hit.y;
#if VMQG_FX_PREFETCH
      if (OUT == 0 && hit.y == 1 && !has_one) { one[k] = *reinterpret_cast<const uint4*>(a.records + hit.x); has_one = true; }
#endif
      onem |= has_one ? 1u << k : 0u;
      rm[k] = ((uint64_t)hit.w << 32) | hit.z;
      if (a.local_node < kLowNodes) rm[k] &= ~(1ull << a.local_node);
      hoff[k] = hi_at;
      const uint32_t nr = (uint32_t)__popcll(rm[k]) + (hi_at != kNone ? a.exwords[hi_at] : 0u);
      tot[k] = OUT ? (cnt[k] ? 1u : 0u) + nr : cnt[k] + nr;
    }
    // ---- offsets: lane, chunk and wave prefixes; the tile's aggregate
    uint64_t excl[kFxK], wsum = 0;   // each publish's offset within its wave's entries
#pragma unroll
    for (uint32_t k = 0; k < kFxK; k++) {
      const uint64_t incl = wave_incl_scan64(tot[k]);
      excl[k] = wsum + incl - tot[k];
      wsum += __shfl(incl, 63, 64);
    }
    if (lane == 0) S.wtot[wv] = wsum;
    __syncthreads();
#if VMQG_FX_DEFER
    // post this tile's aggregate now (successors can look past it at once),
    // then resolve the previous tile: its predecessors have long posted, so
    // its look-back does not wait; then write the previous tile's entries
    // from LDS while this tile's results stay in registers
    if (have && threadIdx.x == 0) {
      uint64_t agg = 0;
      for (uint32_t x = 0; x < kWaves; x++) agg += S.wtot[x];
      S.agg = agg;
      lb_store(a.lookback + tile, lb_pack(a.lb_tag, tile == 0 ? kLbIncl : kLbAgg, agg));
    }
    if (prev != kNone) {
      if (wv == 0) {
        const uint64_t b = lookback(a.lookback, a.lb_tag, a.err, prev, S.agg_prev);
        if (lane == 0) {
          S.base = b;
          if (prev == ntiles - 1) a.offsets[a.npub] = b + S.agg_prev;   // the batch total
        }
      }
      __syncthreads();
      uint64_t wb = S.base;
      for (uint32_t x = 0; x < wv; x++) wb += S.wprev[x];
      const uint32_t q0 = prev * kFxTile + wv * (kFxK * 64);
      const uint32_t om = T.onem[lane];
      uint64_t run = 0;
#pragma unroll 1
      for (uint32_t k = 0; k < kFxK; k++) {
        const uint32_t t = T.tot[k][lane];
        const uint64_t incl = wave_incl_scan64(t);
        fx_emit_chunk<OUT, NT>(a, W, q0 + k * 64 + lane, wb + run + incl - t, cap, T.off[k][lane], T.cnt[k][lane],
                               T.hoff[k][lane], t, T.rm[k][lane], (om >> k) & 1u, T.one[k][lane]);
        run += __shfl(incl, 63, 64);
      }
    }
    __syncthreads();   // the previous tile's state and sums are consumed
    if (!have) break;
#pragma unroll
    for (uint32_t k = 0; k < kFxK; k++) {
      T.off[k][lane] = off[k]; T.cnt[k][lane] = cnt[k]; T.hoff[k][lane] = hoff[k]; T.tot[k][lane] = tot[k];
      T.rm[k][lane] = rm[k];
      if ((onem >> k) & 1u) T.one[k][lane] = one[k];
    }
    T.onem[lane] = onem;
    if (lane == 0) S.wprev[wv] = S.wtot[wv];
    if (threadIdx.x == 0) S.agg_prev = S.agg;
    prev = tile;
    (void)excl;
#else
    if (wv == 0) {
      uint64_t agg = 0;
#pragma unroll
      for (uint32_t x = 0; x < kWaves; x++) agg += S.wtot[x];
      const uint64_t b = lookback(a.lookback, a.lb_tag, a.err, tile, agg);
      if (lane == 0) {
        S.base = b;
        if (tile == ntiles - 1) a.offsets[a.npub] = b + agg;   // the batch total
      }
    }
    __syncthreads();
    uint64_t wbase = S.base;
    for (uint32_t x = 0; x < wv; x++) wbase += S.wtot[x];
    // ---- entries
#pragma unroll
    for (uint32_t k = 0; k < kFxK; k++)
      fx_emit_chunk<OUT, NT>(a, W, p0 + k * 64 + lane, wbase + excl[k], cap, off[k], cnt[k], hoff[k], tot[k], rm[k],
                             (onem >> k) & 1u, one[k]);
    __syncthreads();   // the next tile reuses S
#endif
  }
}

hipError_t launch_exact_fused(const MatchArgs& a, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
  uint32_t g = (a.npub + kFxTile - 1) / kFxTile;
  const uint32_t cap = (uint32_t)a.cus * VMQG_FX_BPC;   // only started blocks take tickets: no look-back waits on an unstarted tile
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  const bool nt = (a.opts & kOptNtStores) != 0;
  auto go = [&](auto kern) {
    if (t0) hipExtLaunchKernelGGL(kern, dim3(g), dim3(256), 0, st, t0, t1, 0, a);
    else kern<<<g, 256, 0, st>>>(a);
  };
  if (a.out_rng) go(k_match_exact_fused<1, false>);
  else if (nt) go(k_match_exact_fused<0, true>);
  else go(k_match_exact_fused<0, false>);
  return hipGetLastError();
}

uint32_t exact_fused_tiles(uint64_t npub) { return (uint32_t)((npub + kFxTile - 1) / kFxTile); }

template <int MODE, int OUT, int G, bool NT, int CH = 64 / G>
static void launch_fast_k(const MatchArgs& a, uint32_t g, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
  // COUNT with dedupe or output groups on: the FEAT variant
  if constexpr (MODE == 0) {
    if (a.dd_force != 0 || a.groups != nullptr) {
      if (t0) hipExtLaunchKernelGGL(k_match_fast<MODE, OUT, G, NT, CH, true>, dim3(g), dim3(256), 0, st, t0, t1, 0, a);
      else k_match_fast<MODE, OUT, G, NT, CH, true><<<g, 256, 0, st>>>(a);
      return;
    }
  }
  if (t0) hipExtLaunchKernelGGL(k_match_fast<MODE, OUT, G, NT, CH>, dim3(g), dim3(256), 0, st, t0, t1, 0, a);
  else k_match_fast<MODE, OUT, G, NT, CH><<<g, 256, 0, st>>>(a);
}

template <int MODE, int OUT>
static void launch_fast(const MatchArgs& a, uint32_t g, bool nt, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
  // trie-less tables (every subscription exact): COUNT is one exact probe per publish
  if (a.trieless && !a.dd_claimed && a.groups == nullptr) {
    if (MODE == 0) launch_count_exact<OUT>(a, st, t0, t1);
    else if (VMQG_EMIT_EXACT) launch_emit_exact<OUT>(a, nt, st, t0, t1);
    if (MODE == 0 || VMQG_EMIT_EXACT) return;
  }
  if (MODE == 0 && a.dd_claimed && a.dd_g == 4 && a.fast_g != 4) {
    // dedupe on: the representatives are few, so COUNT gives each four lanes
    // (more waves to hide each walk's dependent steps; lists 4x larger)
    g = (uint32_t)((a.npub + kWaves * 16 - 1) / (kWaves * 16));
    const uint32_t cap = (uint32_t)a.cus * (a.count_bpc ? a.count_bpc : 8u);
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    if (nt) launch_fast_k<0, OUT, 4, true>(a, g, st, t0, t1);
    else launch_fast_k<0, OUT, 4, false>(a, g, st, t0, t1);
    return;
  }
  if (a.fast_g == 4) {
    if (nt) launch_fast_k<MODE, OUT, 4, true>(a, g, st, t0, t1);
    else launch_fast_k<MODE, OUT, 4, false>(a, g, st, t0, t1);
  } else if (a.fast_g == 1) {   // one-lane COUNT; EMIT two lanes per publish over its 64-publish chunks
    if (MODE == 0) {
      if (nt) launch_fast_k<0, OUT, 1, true>(a, g, st, t0, t1);
      else launch_fast_k<0, OUT, 1, false>(a, g, st, t0, t1);
    } else {
      if (nt) launch_fast_k<1, OUT, 2, true, 64>(a, g, st, t0, t1);
      else launch_fast_k<1, OUT, 2, false, 64>(a, g, st, t0, t1);
    }
  } else {
    if (nt) launch_fast_k<MODE, OUT, 2, true>(a, g, st, t0, t1);
    else launch_fast_k<MODE, OUT, 2, false>(a, g, st, t0, t1);
  }
}

template <int MODE, int OUT, bool NT>
static void launch_wave_k(const MatchArgs& a, uint32_t g, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
  if (t0) hipExtLaunchKernelGGL(k_match_wave<MODE, OUT, NT>, dim3(g), dim3(256), 0, st, t0, t1, 0, a);
  else k_match_wave<MODE, OUT, NT><<<g, 256, 0, st>>>(a);
}

template <int MODE, int OUT>
static void launch_wave(const MatchArgs& a, uint32_t g, bool nt, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
  if (nt) launch_wave_k<MODE, OUT, true>(a, g, st, t0, t1);
  else launch_wave_k<MODE, OUT, false>(a, g, st, t0, t1);
}

hipError_t launch_match(const MatchArgs& a, int mode, int tier, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
  const bool nt = (a.opts & kOptNtStores) != 0;
  const int out = a.out_rng ? 1 : 0;
  if (tier == 0) {
    // publishes per wave: 64 / lanes per publish (fast_g 1: 64 for both passes)
    const uint32_t G = a.fast_g == 4 ? 4 : a.fast_g == 1 ? 1 : 2;
    uint32_t g = div_up(a.npub, kWaves * (64 / G));
    // grid-stride beyond bpc blocks per CU (option count_bpc / emit_bpc; 8 default)
    const uint32_t bpc = mode == 0 ? a.count_bpc : a.emit_bpc;
    const uint32_t cap = (uint32_t)a.cus * (bpc ? bpc : 8u);
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    if (mode == 0) { if (out) launch_fast<0, 1>(a, g, nt, st, t0, t1); else launch_fast<0, 0>(a, g, nt, st, t0, t1); }
    else if (out) launch_fast<1, 1>(a, g, nt, st, t0, t1);
    else launch_fast<1, 0>(a, g, nt, st, t0, t1);
  } else {
    // reads its list lengths on the device (exits at once when empty).
    // COUNT's: one wave per deferred publish, each wave with its own global
    // stack; EMIT's tail: eight blocks per CU, global stacks borrowed
#ifndef VMQG_TAIL_BPC
#define VMQG_TAIL_BPC 8   // EMIT tail blocks per CU (A/B, config D tail: 8 -> 2,269 us, 3 -> 2,418, 2 -> 2,605; C's empty tail 4.4 vs 4.1 us)
#endif
    const uint32_t g = mode == 0 ? a.o_waves / kWaves : (uint32_t)a.cus * VMQG_TAIL_BPC;
    if (mode == 0) { if (out) launch_wave<0, 1>(a, g, nt, st, t0, t1); else launch_wave<0, 0>(a, g, nt, st, t0, t1); }
    else { if (out) launch_wave<1, 1>(a, g, nt, st, t0, t1); else launch_wave<1, 0>(a, g, nt, st, t0, t1); }
  }
  return hipGetLastError();
}


hipError_t launch_patches(uint8_t* arena, const void* d_patches, uint64_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  uint32_t g = div_up(n, 256);
  if (g > 4096) g = 4096;
  k_apply_patches<<<g, 256, 0, st>>>(arena, reinterpret_cast<const uint32_t*>(d_patches), n);
  return hipGetLastError();
}

}  // namespace vmqg
