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

namespace vmqg {

constexpr int kWaves = 4;          // waves per 256-thread block
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
    const bool do_w = act && !at_end && wd != kPlus && wd != kHash && wd != kUnknownWord;
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

// Tiers: 0 = fast (G = kFastG lanes per publish, small LDS lists),
// 1 = mid (G = 64, one publish per wave, large LDS lists, publishes deferred
// by tier 0), 2 = slow (G = 64, global-memory lists, deferred by tier 1).
template <int TIER>
__device__ __forceinline__ void defer_or_fail(const MatchArgs& a, uint32_t p) {
  if (TIER == 0) {
    const uint32_t idx = atomicAdd(&a.status[0], 1u);
    if (idx < a.deferred_cap) a.deferred[idx] = p;
    else atomicOr(&a.status[1], kErrDeferFull);
  } else if (TIER == 1) {
    const uint32_t idx = atomicAdd(&a.status[2], 1u);
    if (idx < a.deferred_cap) a.deferred2[idx] = p;
    else atomicOr(&a.status[1], kErrDeferFull);
  } else {
    atomicOr(&a.status[1], kErrFrontier);
  }
}

// ------------------------------------------------------------ COUNT pass
template <int G, int TIER>
__device__ void count_publish(const MatchArgs& a, uint32_t p, const Scratch& s, const Group<G>& g) {
  const vmqg_pub pub = a.pubs[p];
  const Matched m = walk_publish<G>(a, pub, s, g);
  if (g.lane != 0) return;
  uint4* kc = reinterpret_cast<uint4*>(a.keycache) + (uint64_t)p * 2;
  if (m.overflow) {
    defer_or_fail<TIER>(a, p);
    a.offsets[p] = 0;
    kc[0] = make_uint4(0, kRewalk, 0, 0);
    return;
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
}

// ------------------------------------------------------------- EMIT pass
// Per-group result of the resolve step, staged in LDS for the wave copy.
struct GroupMeta {
  uint32_t rel, span, nk, ksum;   // output start relative to the wave's first publish, length
  uint32_t rm_lo, rm_hi, ok, pad;
};

// EMIT for the GPW consecutive publishes [first, first + n) of one wave.
// Resolve (key cache or re-walk) is per group; the copy is wave-wide over
// the wave's contiguous output range, so every store instruction writes
// 64 x 16 B = 1 KiB contiguous.
template <int G, int GPW, bool NT>
__device__ void emit_wave(const MatchArgs& a, uint32_t first, uint32_t n, const Scratch& s, const Group<G>& g,
                          GroupMeta* gm, const uint2* keys_wave, uint32_t kstride) {
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
      const Matched m = walk_publish<G>(a, a.pubs[p], s, g);
      if (m.overflow) ok = false;   // written by the next tier
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
  const uint64_t wend = a.offsets[first + n];
  const uint32_t T = wend > a.out_cap ? 0 : (uint32_t)(wend - wbase);
  if (g.lane == 0)
    gm[g.gidx] = GroupMeta{valid ? (uint32_t)(obase - wbase) : T, (uint32_t)(oend - obase), nk == 0 ? 1 : nk,
                           ksum, (uint32_t)rmask, (uint32_t)(rmask >> 32), ok ? 1u : 0u, 0u};
  wave_sync();
  // 4 records per lane in flight: all loads issued before the stores
  uint32_t j = 0;
  for (uint32_t r0 = __lane_id(); r0 < T; r0 += 256) {
    uint4 v[4];
    bool w[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t r = r0 + 64 * u;
      w[u] = false;
      if (r < T) {
        while (j + 1 < (uint32_t)GPW && gm[j + 1].rel <= r) j++;
        const GroupMeta m = gm[j];
        if (m.ok) {
          const uint64_t rm = ((uint64_t)m.rm_hi << 32) | m.rm_lo;
          v[u] = emission(a, keys_wave + (uint64_t)j * kstride, m.nk, m.ksum, rm, r - m.rel);
          w[u] = true;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; u++)
      if (w[u]) store_rec<NT>(a.out, wbase + r0 + 64 * u, v[u]);
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
      emit_wave<G, GPW, NT>(a, base, n, s, g, gm[wv], ky[wv * GPW], KC);
    }
    wave_sync();
  }
}

// Tiers 1 and 2: one publish per wave from the deferred lists.
template <int MODE, int TIER>
__global__ __launch_bounds__(256) void k_match_deferred(MatchArgs a) {
  constexpr uint32_t kMidCap = 256;
  __shared__ uint2 st[TIER == 1 ? kWaves : 1][TIER == 1 ? kMidCap : 1];
  __shared__ uint32_t cd[TIER == 1 ? kWaves : 1][TIER == 1 ? kMidCap : 1];
  __shared__ uint2 ky[TIER == 1 ? kWaves : 1][TIER == 1 ? kMidCap : 1];
  __shared__ GroupMeta gm[kWaves][1];
  const Group<64> g;
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t gw = blockIdx.x * kWaves + wv;
  Scratch s;
  if (TIER == 1) {
    s = Scratch{st[wv], cd[wv], ky[wv], kMidCap, kMidCap, kMidCap};
  } else {
    s = Scratch{a.g_stack + (uint64_t)gw * a.g_scap, a.g_cand + (uint64_t)gw * a.g_ccap,
                a.g_keys + (uint64_t)gw * a.g_kcap, a.g_scap, a.g_ccap, a.g_kcap};
  }
  const uint32_t* list = TIER == 1 ? a.deferred : a.deferred2;
  uint32_t n = TIER == 1 ? a.status[0] : a.status[2];
  if (n > a.deferred_cap) n = a.deferred_cap;
  const uint32_t nwaves = gridDim.x * kWaves;
  for (uint32_t d = gw; d < n; d += nwaves) {
    const uint32_t p = list[d];
    if (MODE == 0) count_publish<64, TIER>(a, p, s, g);
    else emit_wave<64, 1, false>(a, p, 1, s, g, gm[wv], s.keys, 0);
    wave_sync();
  }
}

// ------------------------------------------------------------------ scan
// In-place exclusive scan of n u64 values (n-1 counts followed by a 0 slot
// gives offsets[n-1] = total).  Block = 256 threads x 8 items.
constexpr uint32_t kScanItems = 8, kScanBlock = 256, kScanTile = kScanItems * kScanBlock;

__global__ __launch_bounds__(256) void k_scan_tiles(uint64_t* v, uint64_t n, uint64_t* tile_sums) {
  __shared__ uint64_t part[kScanBlock];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
  uint64_t x[kScanItems];
  uint64_t acc = 0;
#pragma unroll
  for (uint32_t i = 0; i < kScanItems; i++) { x[i] = base + i < n ? v[base + i] : 0; acc += x[i]; }
  part[threadIdx.x] = acc;
  __syncthreads();
  for (uint32_t o = 1; o < kScanBlock; o <<= 1) {
    const uint64_t t = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
    __syncthreads();
    part[threadIdx.x] += t;
    __syncthreads();
  }
  uint64_t run = part[threadIdx.x] - acc;
#pragma unroll
  for (uint32_t i = 0; i < kScanItems; i++) {
    if (base + i < n) v[base + i] = run;
    run += x[i];
  }
  if (threadIdx.x == kScanBlock - 1 && tile_sums) tile_sums[blockIdx.x] = part[kScanBlock - 1];
}

__global__ __launch_bounds__(256) void k_scan_add(uint64_t* v, uint64_t n, const uint64_t* tile_offs) {
  const uint64_t add = tile_offs[blockIdx.x];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  for (uint32_t i = threadIdx.x; i < kScanTile; i += kScanBlock)
    if (base + i < n) v[base + i] += add;
}

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

hipError_t launch_scan(uint64_t* v, uint64_t n, uint64_t* tmp, hipStream_t st) {
  // tmp must hold scan_tmp_elems(n) u64
  const uint64_t tiles = (n + kScanTile - 1) / kScanTile;
  if (tiles <= 1) {
    k_scan_tiles<<<1, kScanBlock, 0, st>>>(v, n, nullptr);
    return hipGetLastError();
  }
  k_scan_tiles<<<(uint32_t)tiles, kScanBlock, 0, st>>>(v, n, tmp);
  const hipError_t e = launch_scan(tmp, tiles, tmp + tiles, st);
  if (e != hipSuccess) return e;
  k_scan_add<<<(uint32_t)tiles, kScanBlock, 0, st>>>(v, n, tmp);
  return hipGetLastError();
}

uint64_t scan_tmp_elems(uint64_t n) {
  uint64_t tot = 0;
  for (uint64_t t = (n + kScanTile - 1) / kScanTile; t > 1; t = (t + kScanTile - 1) / kScanTile) tot += t;
  return tot + 1;
}

hipError_t launch_match(const MatchArgs& a, int mode, int tier, hipStream_t st) {
  if (tier == 0) {
    const uint32_t G = (a.fast_g == 2 || a.fast_g == 8) ? a.fast_g : 4;
    const bool nt = (a.opts & kOptNtStores) != 0;
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
  } else if (tier == 1) {
    const uint32_t g = 256;   // reads its list length on the device; exits at once when empty
    if (mode == 0) k_match_deferred<0, 1><<<g, 256, 0, st>>>(a);
    else k_match_deferred<1, 1><<<g, 256, 0, st>>>(a);
  } else {
    const uint32_t g = a.g_waves / kWaves;
    if (mode == 0) k_match_deferred<0, 2><<<g, 256, 0, st>>>(a);
    else k_match_deferred<1, 2><<<g, 256, 0, st>>>(a);
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
