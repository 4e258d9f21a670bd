// HIP kernels for gfx950 (MI355X): the publish -> matched-subscriber path of
// vmq_reg_trie:fold/4 (apps/vmq_server/src/vmq_reg_trie.erl:59-98).
//
// Work unit: a GROUP of G lanes owns one publish (G = 8 on the fast path, so
// a 64-lane wavefront keeps 8 publishes in flight; G = 64 on the slow path).
// The group walks the trie in chunks: up to G frontier entries {path, depth}
// are popped from the group's LDS stack, one per lane, and each active lane
// issues its three edge probes ('#', the publish word, '+') as independent
// 64-B bucket loads before resolving any of them — the ets:lookup calls of
// trie_match/4 and 'trie_match_#'/2 (:358-383), many frontier nodes and many
// publishes per memory round trip.  '#' children and end-of-topic nodes are
// compacted (ballot + mbcnt) into an LDS candidate list; their node records
// (match/4, :283-303) give the subscriber-list keys, compacted into an LDS
// key list.  The exact-topic probe (the `{Topic, node()}` candidate and
// get_remote_subscribers/2, :62, :514-520) is a fingerprint lookup computed
// group-parallel.  Remote nodes are OR-ed into a 64-bit mask: exactly the
// `Remotes` dedupe of fold_/5 (:78-84).
//
// Passes per batch: COUNT (walk; per-publish emission count, plus a 32-B key
// cache {total, nk, remote mask, <=2 x (record off, count)}), a device scan
// (counts -> offsets), EMIT (records from the key cache; re-walk only for
// publishes with > 2 keys), writing the 16-B records (lookup_subs + fold__,
// :87-98) group-contiguously.  Publishes that overflow the LDS lists go to
// the SLOW instantiation (G = 64, scratch in global memory).
#include <hip/hip_runtime.h>

#include "vmqg_common.h"
#include "vmqg_kernels.h"
#include "vmqg_lookback.h"

namespace vmqg {

constexpr int kWaves = 4;          // waves per 256-thread block
#ifndef VMQG_EMIT_U
#define VMQG_EMIT_U 8              // records in flight per lane in the tier-0 EMIT copy (A/B: 2, 4, 8)
#endif
// fast-tier LDS lists per group, sized so a block stays near 28 KiB
template <int G> struct FastCaps { static constexpr uint32_t S = 8 * G, C = 4 * G, K = 4 * G; };
constexpr uint32_t kRewalk = 0xFFFFFFFFu;   // key cache: EMIT must re-walk

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
};

__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

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

struct Scratch {
  uint2* stack;    // {path, depth}
  uint32_t* cand;  // path ids
  uint2* keys;     // key id, then {record off, cumulative start}
  uint32_t scap, ccap, kcap;
};

enum : uint32_t { kErrDeferFull = 1u, kErrFrontier = 2u, kErrOverflow = 4u, kErrMismatch = 8u };

// Per-publish result of the walk: keys[0..nk) hold {record off, cum start}.
struct Matched {
  uint32_t nk, ksum, total;
  uint64_t rmask;
  bool overflow;
};

// ----------------------------------------------------- walk + resolution
template <int G>
__device__ Matched walk_publish(const MatchArgs& a, const vmqg_pub& pub, const Scratch& s, const Group<G>& g) {
  const uint32_t L = pub.nwords;
  const uint32_t* w = a.words + pub.word_off;
  const bool dollar = (pub.flags & VMQG_PUB_DOLLAR) != 0;
  const bool mp_ok = pub.mountpoint < a.max_mp && L > 0;
  // lane i of the group keeps word i (i < G); deeper words come from memory
  const uint32_t wreg = g.lane < L ? w[g.lane] : kUnknownWord;
  Matched m{0, 0, 0, 0, false};
  uint32_t nc = 0, sp = 0;
  if (mp_ok) {
    if (g.lane == 0) s.stack[0] = make_uint2(pub.mountpoint, kHasAll << 28);   // {MP, root}: probe all
    sp = 1;
  }
  wave_sync();

  // ---- trie_match/4 + 'trie_match_#'/2  (vmq_reg_trie.erl:358-383)
  while (sp > 0) {
    const uint32_t k = sp < (uint32_t)G ? sp : (uint32_t)G;
    const uint32_t base = sp - k;
    const bool act = g.lane < k;
    uint32_t node = 0, d = 0, fl = 0;
    if (act) { const uint2 e = s.stack[base + g.lane]; node = e.x; d = e.y & kDepthMask; fl = e.y >> 28; }
    sp = base;
    wave_sync();
    const bool at_end = act && d == L;
    const uint32_t wsh = g.bcast(wreg, d % G);   // all group lanes take part
    uint32_t wd = kUnknownWord;
    if (act && !at_end) wd = d < (uint32_t)G ? wsh : w[d];
    // the node's cached edge flags skip '#' / '+' probes that must miss
    const bool do_h = act && (fl & kHasHash);
    const bool do_w = act && !at_end && (fl & kHasWord) && wd != kPlus && wd != kHash && wd != kUnknownWord;
    const bool do_p = act && !at_end && (fl & kHasPlus);
    const uint64_t bh = edge_hash(node, kHash) & a.edge_mask;
    const uint64_t bw = edge_hash(node, wd) & a.edge_mask;
    const uint64_t bp = edge_hash(node, kPlus) & a.edge_mask;
    Bucket Bh{}, Bw{}, Bp{};
    if (do_h) Bh = load_bucket(a.edges, bh);
    if (do_w) Bw = load_bucket(a.edges, bw);
    if (do_p) Bp = load_bucket(a.edges, bp);
    uint32_t hc = kNone, wc = kNone, pc = kNone, hf = 0, wf = 0, pf = 0;
    if (do_h) probe(a.edges, a.edge_mask, bh, Bh, node, kHash, hc, hf);
    if (do_w) probe(a.edges, a.edge_mask, bw, Bw, node, wd, wc, wf);
    if (do_p) probe(a.edges, a.edge_mask, bp, Bp, node, kPlus, pc, pf);

    // candidates: the '#' child (:377-383) and, with no words left, the node itself (:361-363)
    const uint64_t m_hc = g.ballot(hc != kNone), m_end = g.ballot(at_end);
    const uint32_t n_hc = (uint32_t)__popcll(m_hc), n_new_c = n_hc + (uint32_t)__popcll(m_end);
    // frontier: the W and '+' children (:364-375)
    const uint64_t m_wc = g.ballot(wc != kNone), m_pc = g.ballot(pc != kNone);
    const uint32_t n_pc = (uint32_t)__popcll(m_pc), n_new_s = n_pc + (uint32_t)__popcll(m_wc);
    if (nc + n_new_c > s.ccap || sp + n_new_s > s.scap) { m.overflow = true; break; }
    if (hc != kNone) s.cand[nc + prefix_bits(m_hc)] = hc;
    if (at_end) s.cand[nc + n_hc + prefix_bits(m_end)] = node;
    nc += n_new_c;
    if (pc != kNone) s.stack[sp + prefix_bits(m_pc)] = make_uint2(pc, (d + 1) | (pf << 28));
    if (wc != kNone) s.stack[sp + n_pc + prefix_bits(m_wc)] = make_uint2(wc, (d + 1) | (wf << 28));
    sp += n_new_s;
    wave_sync();
  }

  // ---- candidates -> subscriber-list keys: match/4, match_/3 (:283-303)
  uint64_t rmask = 0;
  uint32_t nk = 0;
  if (!m.overflow) {
    for (uint32_t c0 = 0; c0 < nc; c0 += G) {
      const uint32_t ci = c0 + g.lane;
      uint32_t nkeys = 0, key = kNone, off0 = 0, cnt0 = 0;
      if (ci < nc) {
        const uint32_t path = s.cand[ci];
        if (path < a.node_cap) {
          const uint4 r = *reinterpret_cast<const uint4*>(a.nodes + path);
          const uint2 r2 = *reinterpret_cast<const uint2*>(&a.nodes[path].off0);
          const bool valid = (r.x & kNodeEmits) == kNodeEmits &&
                             !(dollar && (r.x & kNodeDollarSkip));   // MQTT-4.7.2-1 (:285-288)
          if (valid) {
            nkeys = r.x >> 8;
            key = r.y;
            off0 = r2.x;
            cnt0 = r2.y;
            rmask |= ((uint64_t)r.w << 32) | r.z;
          }
        }
      }
      const uint32_t incl = g.incl_scan(nkeys);
      const uint32_t tot = g.last(incl);
      if (nk + tot > s.kcap) { m.overflow = true; break; }
      const uint32_t at = nk + incl - nkeys;
      if (nkeys == 1) s.keys[at] = make_uint2(off0, cnt0);   // resolved inline
      else for (uint32_t j = 0; j < nkeys; j++) s.keys[at + j] = make_uint2(a.keylist[key + j], kUnresolved);
      nk += tot;
    }
  }
  wave_sync();

  // ---- the exact candidate {Topic, node()} and remote exact subscribers (:62, :514-520)
  if (!m.overflow && mp_ok) {
    uint64_t part = 0;
    for (uint32_t i = g.lane; i < L; i += G) part += fp_word(i < (uint32_t)G ? wreg : w[i], i);
    const uint64_t fp = fp_final(g.sum64(part), pub.mountpoint, L);
    uint64_t b = fp & a.exact_mask;
    for (uint64_t iter = 0; iter <= a.exact_mask; iter++) {
      const ExactSlot* bk = a.exact + b * kExactSlotsPerBucket;
      bool seen_empty = false, found = false;
      for (uint32_t j = 0; j < kExactSlotsPerBucket && !found; j++) {
        const ExactSlot e = bk[j];
        if (e.nwords == kEmpty) { seen_empty = true; break; }
        if (e.fp != fp || e.nwords != L) continue;
        // exactness: the stored MP and words, compared group-parallel
        const uint32_t* xw = a.exwords + e.words_off;
        bool diff = g.lane == 0 && xw[0] != pub.mountpoint;
        for (uint32_t i = g.lane; i < L; i += G) diff |= xw[1 + i] != (i < (uint32_t)G ? wreg : w[i]);
        if (g.ballot(diff) != 0) continue;
        found = true;
        rmask |= e.rmask;
        if (e.count != 0) {
          if (nk + 1 > s.kcap) m.overflow = true;
          else { if (g.lane == 0) s.keys[nk] = make_uint2(e.off, e.count); nk += 1; }
        }
      }
      if (found || seen_empty) break;
      b = (b + 1) & a.exact_mask;
    }
  }
  wave_sync();
  m.rmask = g.or64(rmask) & ~(1ull << a.local_node);
  if (m.overflow) return m;

  // ---- record ranges per key: lookup_subs/1 (:87-94)
  uint32_t ksum = 0;
  for (uint32_t k0 = 0; k0 < nk; k0 += G) {
    const uint32_t ki = k0 + g.lane;
    uint32_t cnt = 0, off = 0;
    if (ki < nk) {
      const uint2 e = s.keys[ki];
      if (e.y != kUnresolved) { off = e.x; cnt = e.y; }
      else if (e.x < a.key_cap) { const uint2 kd = *reinterpret_cast<const uint2*>(a.keydesc + e.x); off = kd.x; cnt = kd.y; }
    }
    const uint32_t incl = g.incl_scan(cnt);
    wave_sync();
    if (ki < nk) s.keys[ki] = make_uint2(off, ksum + incl - cnt);
    ksum += g.last(incl);
  }
  wave_sync();
  m.nk = nk;
  m.ksum = ksum;
  m.total = ksum + (uint32_t)__popcll(m.rmask);
  return m;
}

// r-th emission of a publish whose keys are {off, cum start} in `keys`.
__device__ __forceinline__ uint4 emission(const MatchArgs& a, const uint2* keys, uint32_t nk, uint32_t ksum,
                                          uint64_t rmask, uint32_t r) {
  if (r < ksum) {
    uint32_t lo = 0, hi = nk;   // last key whose cumulative start <= r
    while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (keys[mid].y <= r) lo = mid; else hi = mid; }
    const uint2 kk = keys[lo];
    return *reinterpret_cast<const uint4*>(a.records + kk.x + (r - kk.y));
  }
  // j-th remote node of the mask, in node order (fold_/5 :78-84)
  uint64_t m = rmask;
  for (uint32_t j = r - ksum; j > 0; j--) m &= m - 1;
  return make_uint4((VMQG_EMIT_REMOTE << 24) | (uint32_t)__builtin_ctzll(m), kNone, kNone, kNone);
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

// Tiers: 0 = fast (G = fast_g lanes per publish, small LDS lists); 1 = wave
// (G = 64, one publish per wave, publishes deferred by tier 0): 256-entry LDS
// lists first, the wave's global scratch (o_cap entries) when those overflow.
template <int TIER>
__device__ __forceinline__ void defer_or_fail(const MatchArgs& a, uint32_t p) {
  if (TIER == 0) {
    const uint32_t idx = atomicAdd(&a.status[0], 1u);
    if (idx < a.deferred_cap) a.deferred[idx] = p;
    else atomicOr(&a.status[1], kErrDeferFull);
  } else {
    atomicOr(&a.status[1], kErrFrontier);
  }
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

// ------------------------------------------------------------ COUNT pass
// Returns false when the walk overflowed `s`.  Tier 0 defers the publish;
// tier 1 returns to its caller, which retries with global scratch (tier 2
// role: an overflow there is a frontier error).
template <int G, int TIER>
__device__ bool count_publish(const MatchArgs& a, uint32_t p, const Scratch& s, const Group<G>& g) {
  const vmqg_pub pub = a.pubs[p];
  const Matched m = walk_publish<G>(a, pub, s, g);
  if (m.overflow && TIER == 1) return false;
  if (g.lane != 0) return !m.overflow;
  uint4* kc = reinterpret_cast<uint4*>(a.keycache) + (uint64_t)p * 2;
  if (m.overflow) {
    defer_or_fail<TIER>(a, p);
    a.offsets[p] = 0;
    kc[0] = make_uint4(0, kRewalk, 0, 0);
    return false;
  }
  a.offsets[p] = m.total;
  // key cache: total, nk, remote mask, up to two {record off, count}
  if (m.nk <= 2) {
    const uint2 k0 = m.nk > 0 ? s.keys[0] : make_uint2(0, 0);
    const uint2 k1 = m.nk > 1 ? s.keys[1] : make_uint2(0, m.ksum);
    const uint32_t c0 = m.nk > 1 ? k1.y : m.ksum;
    kc[0] = make_uint4(m.total, m.nk, (uint32_t)m.rmask, (uint32_t)(m.rmask >> 32));
    kc[1] = make_uint4(k0.x, c0, k1.x, m.ksum - c0);
  } else {
    kc[0] = make_uint4(m.total, kRewalk, 0, 0);
  }
  return true;
}

// ------------------------------------------------------------- EMIT pass
// Per-group result of the resolve step, staged in LDS for the wave copy.
struct GroupMeta {
  uint32_t rel, span, nk, ksum;   // output start relative to the wave's first publish, length
  uint32_t rm_lo, rm_hi, ok, crel;   // crel: start among the wave's copied (ok) records
};

// EMIT for the GPW consecutive publishes [first, first + n) of one wave.
// Resolve (key cache or re-walk) is per group; the copy is wave-wide over
// the wave's output range minus the ranges of publishes a later tier
// writes, so every store instruction writes up to 64 x 16 B = 1 KiB
// contiguous.  `s2` (tier 1): global scratch for a re-walk that overflows `s`.
template <int G, int GPW, bool NT, int U>
__device__ void emit_wave(const MatchArgs& a, uint32_t first, uint32_t n, const Scratch& s, const Scratch* s2,
                          const Group<G>& g, GroupMeta* gm, const uint2* keys_wave, uint32_t kstride) {
  const uint32_t p = first + g.gidx;
  const bool valid = g.gidx < n;
  uint32_t total = 0, nk = 0, ksum = 0;
  uint64_t rmask = 0, obase = 0, oend = 0;
  bool ok = valid;
  if (valid) {
    const uint4* kc = reinterpret_cast<const uint4*>(a.keycache) + (uint64_t)p * 2;
    const uint4 h = kc[0];
    obase = a.offsets[p];
    oend = a.offsets[p + 1];
    if (h.y == kRewalk) {
      Matched m = walk_publish<G>(a, a.pubs[p], s, g);
      if (m.overflow && s2) {
        m = walk_publish<G>(a, a.pubs[p], *s2, g);
        keys_wave = s2->keys;   // G == 64: one publish per wave
      }
      if (m.overflow) ok = false;   // written by the next tier (or a latched frontier error)
      else { total = m.total; nk = m.nk; ksum = m.ksum; rmask = m.rmask; }
    } else {
      total = h.x; nk = h.y < 2 ? h.y : 2; rmask = ((uint64_t)h.w << 32) | h.z;
      const uint4 k = kc[1];
      ksum = k.y + k.w;
      if (g.lane == 0) {
        s.keys[0] = make_uint2(k.x, 0u);
        s.keys[1] = make_uint2(k.z, k.y);
      }
    }
    if (ok && oend > a.out_cap) { if (g.lane == 0) atomicOr(&a.status[1], kErrOverflow); ok = false; }
    if (ok && oend - obase != total) { if (g.lane == 0) atomicOr(&a.status[1], kErrMismatch); ok = false; }
  }
  const uint64_t wbase = a.offsets[first];
  if (g.lane == 0)
    gm[g.gidx] = GroupMeta{valid ? (uint32_t)(obase - wbase) : 0u, ok ? (uint32_t)(oend - obase) : 0u,
                           nk == 0 ? 1 : nk, ksum, (uint32_t)rmask, (uint32_t)(rmask >> 32), ok ? 1u : 0u, 0u};
  wave_sync();
  // compact the copied ranges: crel = exclusive scan of the ok spans
  const uint32_t lane = __lane_id();
  uint32_t Tok;
  if (GPW == 1) {
    Tok = gm[0].span;
  } else {
    const uint32_t sp = lane < (uint32_t)GPW ? gm[lane].span : 0u;
    const uint32_t incl = wave_incl_scan32(sp);
    if (lane < (uint32_t)GPW) gm[lane].crel = incl - sp;
    Tok = __shfl(incl, GPW - 1, 64);
    wave_sync();
  }
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
        const GroupMeta m = gm[j];
        const uint64_t rm = ((uint64_t)m.rm_hi << 32) | m.rm_lo;
        v[u] = emission(a, keys_wave + (uint64_t)j * kstride, m.nk, m.ksum, rm, r - m.crel);
        dst[u] = wbase + m.rel + (r - m.crel);
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (w[u]) store_rec<NT>(a.out, dst[u], v[u]);
  }
  wave_sync();
}

// --------------------------------------------------------------- kernels
template <int MODE, int G, bool NT>
__global__ __launch_bounds__(256) void k_match_fast(MatchArgs a) {
  constexpr int GPW = 64 / G;   // groups (publishes) per wave
  constexpr uint32_t SC = FastCaps<G>::S, CC = FastCaps<G>::C, KC = FastCaps<G>::K;
  __shared__ uint2 st[kWaves * GPW][SC];
  __shared__ uint32_t cd[kWaves * GPW][CC];
  __shared__ uint2 ky[kWaves * GPW][KC];
  __shared__ GroupMeta gm[kWaves][GPW];
  const Group<G> g;
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t slot = wv * GPW + g.gidx;
  const Scratch s{st[slot], cd[slot], ky[slot], SC, CC, KC};
  const uint32_t stride = gridDim.x * kWaves * GPW;
  for (uint32_t base = (blockIdx.x * kWaves + wv) * GPW; base < a.npub; base += stride) {
    const uint32_t n = a.npub - base < (uint32_t)GPW ? a.npub - base : (uint32_t)GPW;
    if (MODE == 0) {
      if (g.gidx < n) count_publish<G, 0>(a, base + g.gidx, s, g);
    } else {
      emit_wave<G, GPW, NT, VMQG_EMIT_U>(a, base, n, s, nullptr, g, gm[wv], ky[wv * GPW], KC);
    }
    wave_sync();
  }
}

// Tier 1: one publish per wave from the deferred list; LDS lists, then the
// wave's global scratch.
template <int MODE, bool NT>
__global__ __launch_bounds__(256) void k_match_wave(MatchArgs a) {
  constexpr uint32_t kMidCap = 256;
  __shared__ uint2 st[kWaves][kMidCap];
  __shared__ uint32_t cd[kWaves][kMidCap];
  __shared__ uint2 ky[kWaves][kMidCap];
  __shared__ GroupMeta gm[kWaves][1];
  const Group<64> g;
  const uint32_t wv = threadIdx.x >> 6;
  const uint64_t gw = (uint64_t)blockIdx.x * kWaves + wv;
  const Scratch s{st[wv], cd[wv], ky[wv], kMidCap, kMidCap, kMidCap};
  const Scratch so{a.o_stack + gw * a.o_cap, a.o_cand + gw * a.o_cap, a.o_keys + gw * a.o_cap,
                   a.o_cap, a.o_cap, a.o_cap};
  uint32_t n = a.status[0];
  if (n > a.deferred_cap) n = a.deferred_cap;
  const uint32_t nwaves = gridDim.x * kWaves;
  for (uint32_t d = (uint32_t)gw; d < n; d += nwaves) {
    const uint32_t p = a.deferred[d];
    if (MODE == 0) {
      if (!count_publish<64, 1>(a, p, s, g)) {
        if (__lane_id() == 0) atomicAdd(&a.status[2], 1u);
        count_publish<64, 2>(a, p, so, g);
      }
    } else {
      emit_wave<64, 1, NT, 8>(a, p, 1, s, &so, g, gm[wv], s.keys, 0);
    }
    wave_sync();
  }
}

// ------------------------------------------------------ fused single pass
// k_match_fused: one launch does what COUNT + scan + EMIT do above.  A block
// takes chunks of CH = 4 * (64 / G) consecutive publishes by ticket (so a
// chunk's predecessors are always owned by running blocks) and for each:
//   1. walks every publish with G lanes (fast LDS lists, as COUNT);
//   2. publishes that overflow the fast lists are walked again by a whole
//      wave with global scratch (o_stack / o_cand / o_keys) — their count;
//   3. scans the chunk's counts (per wave, then across the 4 waves);
//   4. gets the chunk's output base by decoupled look-back over the
//      predecessors' 8-B {tag, flag, value} granules (agent-scope relaxed
//      atomics: the granule is its own flag, cdna_hip_programming.md G16 R2);
//   5. writes offsets[] for its publishes;
//   6. copies the fast publishes' records wave-wide (contiguous, NT stores),
//      skipping the ranges of the wave-path publishes;
//   7. re-walks each wave-path publish with a whole wave and copies its
//      records.
// The walk of one chunk overlaps the record stores of the other blocks on
// the CU, which a COUNT -> EMIT kernel boundary forbids.
struct FusedMeta {               // per publish of the chunk
  uint32_t rel, span, crel, ok;  // output start / length relative to the wave; start among ok records
  uint32_t nk, ksum, rm_lo, rm_hi;
};

// Wave path (G = 64, global scratch) of the fused kernel: a publish whose
// frontier / candidate / key lists overflow the fast LDS lists.  Kept out of
// line so the fast walk's register budget is not the sum of both paths.
__device__ __noinline__ uint32_t wave_path_count(const MatchArgs& a, uint32_t p, const Scratch& so) {
  const Group<64> g64;
  const Matched mo = walk_publish<64>(a, a.pubs[p], so, g64);
  return mo.overflow ? kNone : mo.total;
}

template <bool NT, int U>
__device__ __noinline__ void wave_path_emit(const MatchArgs& a, uint32_t p, const Scratch& so, uint64_t ob,
                                            uint32_t want) {
  const Group<64> g64;
  const uint32_t lane = __lane_id();
  const Matched mo = walk_publish<64>(a, a.pubs[p], so, g64);
  if (mo.overflow) return;   // latched by the count
  if (mo.total != want) { if (lane == 0) atomicOr(&a.status[1], kErrMismatch); return; }
  uint32_t kk = 0;
  for (uint32_t r0 = lane; r0 < mo.total; r0 += 64 * U) {
    uint4 v[U];
    bool w[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t r = r0 + 64 * u;
      w[u] = r < mo.total;
      if (w[u]) {
        if (r < mo.ksum) {
          while (kk + 1 < mo.nk && so.keys[kk + 1].y <= r) kk++;
          const uint2 kd = so.keys[kk];
          v[u] = *reinterpret_cast<const uint4*>(a.records + kd.x + (r - kd.y));
        } else {
          v[u] = emission(a, so.keys, 1, mo.ksum, mo.rmask, r);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (w[u]) store_rec<NT>(a.out, ob + r0 + 64 * u, v[u]);
  }
}

template <int G, bool NT, int U>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_match_fused(MatchArgs a) {
  constexpr int GPW = 64 / G;                 // publishes per wave
  constexpr uint32_t CH = kWaves * GPW;       // publishes per chunk
  constexpr uint32_t SC = FastCaps<G>::S, CC = FastCaps<G>::C, KC = FastCaps<G>::K;
  __shared__ uint2 st[CH][SC];
  __shared__ uint32_t cd[CH][CC];
  __shared__ uint2 ky[CH][KC];
  __shared__ FusedMeta fm[CH];
  __shared__ uint32_t tot[CH], ovl[CH];
  __shared__ uint64_t wtot[kWaves];
  __shared__ uint32_t s_chunk, s_novf;
  __shared__ uint64_t s_base;
  const Group<G> g;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = __lane_id();
  const uint32_t slot = wv * GPW + g.gidx;
  const Scratch s{st[slot], cd[slot], ky[slot], SC, CC, KC};
  const uint64_t gw = (uint64_t)blockIdx.x * kWaves + wv;
  const Scratch so{a.o_stack + gw * a.o_cap, a.o_cand + gw * a.o_cap, a.o_keys + gw * a.o_cap,
                   a.o_cap, a.o_cap, a.o_cap};
  for (;;) {
    if (threadIdx.x == 0) { s_chunk = atomicAdd(&a.status[3], 1u); s_novf = 0; }
    __syncthreads();
    const uint32_t chunk = s_chunk;
    if (chunk >= a.nchunks) break;
    const uint32_t base = chunk * CH;

    // 1. fast walks (trie_match/4 + match/4 + lookup_subs/1 of every publish)
    const uint32_t p = base + slot;
    const bool have = p < a.npub;
    Matched m{0, 0, 0, 0, false};
    if (have) m = walk_publish<G>(a, a.pubs[p], s, g);
    if (g.lane == 0) {
      const bool ok = have && !m.overflow;
      tot[slot] = ok ? m.total : 0;
      fm[slot] = FusedMeta{0, 0, 0, ok ? 1u : 0u, m.nk == 0 ? 1u : m.nk, m.ksum, (uint32_t)m.rmask,
                           (uint32_t)(m.rmask >> 32)};
      if (have && m.overflow) ovl[atomicAdd(&s_novf, 1u)] = slot;
    }
    __syncthreads();

    // 2. publishes that overflowed the fast lists: counted by whole waves
    const uint32_t novf = s_novf;
    for (uint32_t k = wv; k < novf; k += kWaves) {
      const uint32_t j = ovl[k];
      const uint32_t t = wave_path_count(a, base + j, so);
      if (lane == 0) {
        if (t == kNone) atomicOr(&a.status[1], kErrFrontier);
        else tot[j] = t;
      }
    }
    if (threadIdx.x == 0 && novf) atomicAdd(&a.status[0], novf);
    __syncthreads();

    // 3. offsets inside the chunk: per-wave scans of the counts and of the
    //    fast publishes' counts, then the waves' totals
    const uint32_t me = wv * GPW + lane;
    const uint32_t cnt = lane < (uint32_t)GPW ? tot[me] : 0u;
    const uint32_t cnt_ok = lane < (uint32_t)GPW && fm[me].ok ? cnt : 0u;
    const uint32_t incl = wave_incl_scan32(cnt);
    const uint32_t incl_ok = wave_incl_scan32(cnt_ok);
    const uint32_t wsum = __shfl(incl, 63, 64), wsum_ok = __shfl(incl_ok, 63, 64);
    if (lane < (uint32_t)GPW) { fm[me].rel = incl - cnt; fm[me].span = cnt; fm[me].crel = incl_ok - cnt_ok; }
    if (lane == 0) wtot[wv] = wsum;
    __syncthreads();
    uint64_t wrel = 0, agg = 0;
#pragma unroll
    for (uint32_t w = 0; w < (uint32_t)kWaves; w++) { if (w < wv) wrel += wtot[w]; agg += wtot[w]; }

    // 4. chunk base: decoupled look-back
    if (wv == 0) {
      const uint64_t b = lookback(a.lookback, a.lb_tag, a.status, chunk, agg);
      if (lane == 0) s_base = b;
    }
    __syncthreads();
    const uint64_t cbase = s_base;
    const bool fits = cbase + agg <= a.out_cap;
    if (threadIdx.x == 0 && !fits) atomicOr(&a.status[1], kErrOverflow);

    // 5. offsets (exclusive prefix; the batch's last publish also writes the total)
    if (lane < (uint32_t)GPW) {
      const uint32_t pp = base + me;
      if (pp < a.npub) a.offsets[pp] = cbase + wrel + (incl - cnt);
      if (pp + 1 == a.npub) a.offsets[a.npub] = cbase + agg;
    }

    // 6. fast publishes: one contiguous copy per wave, U records per lane in flight
    if (fits) {
      const uint64_t wbase = cbase + wrel;
      const FusedMeta* wm = fm + wv * GPW;
      uint32_t j = 0;
      for (uint32_t r0 = lane; r0 < wsum_ok; r0 += 64 * U) {
        uint4 v[U];
        uint64_t dst[U];
        bool w[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint32_t r = r0 + 64 * u;
          w[u] = r < wsum_ok;
          if (w[u]) {
            while (j + 1 < (uint32_t)GPW && wm[j + 1].crel <= r) j++;
            const FusedMeta mm = wm[j];
            const uint64_t rm = ((uint64_t)mm.rm_hi << 32) | mm.rm_lo;
            v[u] = emission(a, ky[wv * GPW + j], mm.nk, mm.ksum, rm, r - mm.crel);
            dst[u] = wbase + mm.rel + (r - mm.crel);
          }
        }
#pragma unroll
        for (int u = 0; u < U; u++)
          if (w[u]) store_rec<NT>(a.out, dst[u], v[u]);
      }
    }

    // 7. wave-path publishes: re-walk, then a 64-lane copy in key order
    for (uint32_t k = wv; fits && k < novf; k += kWaves) {
      const uint32_t j = ovl[k];
      uint64_t ob = cbase + fm[j].rel;   // + the totals of the waves before publish j's
      for (uint32_t w = 0; w < j / GPW; w++) ob += wtot[w];
      wave_path_emit<NT, U>(a, base + j, so, ob, tot[j]);
    }
    __syncthreads();   // LDS is reused by the next chunk
  }
}

uint32_t fused_chunk(uint32_t fast_g) { return kWaves * (64 / fast_g); }

template <int GG, int U>
static hipError_t launch_fused_g(const MatchArgs& a, uint32_t grid, bool nt, hipStream_t st) {
  if (nt) k_match_fused<GG, true, U><<<grid, 256, 0, st>>>(a);
  else k_match_fused<GG, false, U><<<grid, 256, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_fused(const MatchArgs& a, uint32_t grid, uint32_t unroll, hipStream_t st) {
  const bool nt = (a.opts & kOptNtStores) != 0;
  if (grid < 1) grid = 1;
  if (a.fast_g == 2) return unroll == 8 ? launch_fused_g<2, 8>(a, grid, nt, st) : launch_fused_g<2, 4>(a, grid, nt, st);
  if (a.fast_g == 8) return unroll == 8 ? launch_fused_g<8, 8>(a, grid, nt, st) : launch_fused_g<8, 4>(a, grid, nt, st);
  return unroll == 8 ? launch_fused_g<4, 8>(a, grid, nt, st) : launch_fused_g<4, 4>(a, grid, nt, st);
}

int fused_blocks_per_cu(uint32_t fast_g, uint32_t unroll) {
  int n = 0;
  const void* f;
  if (fast_g == 2) f = unroll == 8 ? (const void*)k_match_fused<2, true, 8> : (const void*)k_match_fused<2, true, 4>;
  else if (fast_g == 8) f = unroll == 8 ? (const void*)k_match_fused<8, true, 8> : (const void*)k_match_fused<8, true, 4>;
  else f = unroll == 8 ? (const void*)k_match_fused<4, true, 8> : (const void*)k_match_fused<4, true, 4>;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, 256, 0) != hipSuccess) return 0;
  return n;
}

// ------------------------------------------------------------------ scan
// Exclusive scan of the per-publish counts in offsets[0, npub) into
// offsets[0, npub] (offsets[npub] = total) in ONE launch: tiles of 4,096
// taken by ticket, chained by the same decoupled look-back as the fused
// kernel.  Slot npub is never read (no memset before the COUNT pass).
constexpr uint32_t kScanItems = 16, kScanBlock = 256, kScanTile = kScanItems * kScanBlock;

__global__ __launch_bounds__(256) void k_scan_offsets(MatchArgs a) {
  __shared__ uint64_t part[kScanBlock];
  __shared__ uint32_t s_tile;
  __shared__ uint64_t s_base;
  const uint64_t n = (uint64_t)a.npub + 1;
  const uint32_t ntiles = (uint32_t)((n + kScanTile - 1) / kScanTile);
  uint64_t* v = a.offsets;
  for (;;) {
    if (threadIdx.x == 0) s_tile = atomicAdd(&a.status[3], 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    if (tile >= ntiles) break;
    const uint64_t base = (uint64_t)tile * kScanTile + (uint64_t)threadIdx.x * kScanItems;
    uint64_t x[kScanItems];
    uint64_t acc = 0;
#pragma unroll
    for (uint32_t i = 0; i < kScanItems; i++) { x[i] = base + i < a.npub ? v[base + i] : 0; acc += x[i]; }
    part[threadIdx.x] = acc;
    __syncthreads();
    for (uint32_t o = 1; o < kScanBlock; o <<= 1) {
      const uint64_t t = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
      __syncthreads();
      part[threadIdx.x] += t;
      __syncthreads();
    }
    if (threadIdx.x < 64) {
      const uint64_t b = lookback(a.lookback, a.lb_tag, a.status, tile, part[kScanBlock - 1]);
      if (threadIdx.x == 0) s_base = b;
    }
    __syncthreads();
    uint64_t run = s_base + part[threadIdx.x] - acc;
#pragma unroll
    for (uint32_t i = 0; i < kScanItems; i++) {
      if (base + i < n) v[base + i] = run;
      run += x[i];
    }
    __syncthreads();
  }
}

uint32_t scan_tiles(uint64_t npub) { return (uint32_t)((npub + 1 + kScanTile - 1) / kScanTile); }

// ---------------------------------------------------------------- patches
__global__ __launch_bounds__(256) void k_apply_patches(uint8_t* arena, const uint32_t* patches, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t* pr = patches + i * 6;
    const uint64_t off = (uint64_t)pr[0] | ((uint64_t)pr[1] << 32);
    *reinterpret_cast<uint4*>(arena + off) = make_uint4(pr[2], pr[3], pr[4], pr[5]);
  }
}

// ---------------------------------------------------------------- launch
static inline uint32_t div_up(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

hipError_t launch_scan(const MatchArgs& a, hipStream_t st) {
  uint32_t g = scan_tiles(a.npub);
  if (g > 2048) g = 2048;
  k_scan_offsets<<<g, kScanBlock, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_match(const MatchArgs& a, int mode, int tier, hipStream_t st) {
  const bool nt = (a.opts & kOptNtStores) != 0;
  if (tier == 0) {
    const uint32_t G = (a.fast_g == 2 || a.fast_g == 8) ? a.fast_g : 4;
    uint32_t g = div_up(a.npub, kWaves * (64 / G));
    const uint32_t cap = 256u * 8u;   // grid-stride beyond 8 blocks per CU
    if (g > cap) g = cap;
    if (g < 1) g = 1;
#define VMQG_FAST(GG)                                                       \
    if (mode == 0) k_match_fast<0, GG, false><<<g, 256, 0, st>>>(a);        \
    else if (nt) k_match_fast<1, GG, true><<<g, 256, 0, st>>>(a);           \
    else k_match_fast<1, GG, false><<<g, 256, 0, st>>>(a);
    if (G == 2) { VMQG_FAST(2) }
    else if (G == 4) { VMQG_FAST(4) }
    else { VMQG_FAST(8) }
#undef VMQG_FAST
  } else {
    // reads its list length on the device (exits at once when empty); one
    // wave per deferred publish, as many waves as have global scratch
    const uint32_t g = a.o_waves / kWaves;
    if (mode == 0) k_match_wave<0, false><<<g, 256, 0, st>>>(a);
    else if (nt) k_match_wave<1, true><<<g, 256, 0, st>>>(a);
    else k_match_wave<1, false><<<g, 256, 0, st>>>(a);
  }
  return hipGetLastError();
}

int wave_blocks_per_cu() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)k_match_wave<1, true>, 256, 0) != hipSuccess) return 0;
  return n;
}

hipError_t launch_patches(uint8_t* arena, const void* d_patches, uint64_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  uint32_t g = div_up(n, 256);
  if (g > 4096) g = 4096;
  k_apply_patches<<<g, 256, 0, st>>>(arena, reinterpret_cast<const uint32_t*>(d_patches), n);
  return hipGetLastError();
}

}  // namespace vmqg
