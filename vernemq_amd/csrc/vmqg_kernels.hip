// HIP kernels for gfx950 (MI355X): the publish -> matched-subscriber path of
// vmq_reg_trie:fold/4 (apps/vmq_server/src/vmq_reg_trie.erl:59-98).
//
// One wavefront (64 lanes) owns one publish at a time (grid-stride over the
// batch).  The wave walks the trie breadth-in-chunks: up to 64 frontier
// entries {path, depth} are popped from an LDS stack, one per lane, and each
// active lane issues its three edge probes ('#', the publish word, '+') as
// independent 64-B bucket loads before resolving any of them — the
// lookups of trie_match/4 and 'trie_match_#'/2 (:358-383) for 64 frontier
// nodes in one memory round trip.  '#' children and end-of-topic nodes are
// compacted (ballot + mbcnt) into an LDS candidate list; the candidates'
// node records (match/4, :283-303) are then loaded 64 at a time and their
// subscriber-list keys compacted into an LDS key list.  The exact-topic probe
// (the `{Topic, node()}` candidate and get_remote_subscribers/2, :62, :514-520)
// runs wave-uniformly.  Remote nodes are OR-ed into a 64-bit mask, which is
// exactly the `Remotes` dedupe of fold_/5 (:78-84).
//
// Two passes per batch: COUNT writes each publish's emission count, a
// device scan turns counts into offsets, EMIT re-walks and writes the 16-B
// records (lookup_subs + fold__, :87-98) with coalesced 1-KiB wave stores.
// A publish whose frontier / candidate / key lists overflow LDS is deferred
// to the SLOW instantiation (same code, scratch in global memory).
#include <hip/hip_runtime.h>

#include "vmqg_common.h"
#include "vmqg_kernels.h"

namespace vmqg {

constexpr int kWaves = 4;         // waves per 256-thread block
constexpr uint32_t kSCap = 256;   // LDS frontier stack entries per wave
constexpr uint32_t kCCap = 256;   // LDS candidate entries per wave
constexpr uint32_t kKCap = 256;   // LDS key entries per wave

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t prefix_bits(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const uint32_t l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = __shfl_up(v, o, 64);
    if (l >= (uint32_t)o) v += t;
  }
  return v;
}

__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    uint32_t lo = __shfl_xor((uint32_t)v, o, 64), hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
    v |= ((uint64_t)hi << 32) | lo;
  }
  return v;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    uint32_t lo = __shfl_xor((uint32_t)v, o, 64), hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}

__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

// ---------------------------------------------------------------- probes
struct Bucket { uint4 s0, s1, s2, s3; };

__device__ __forceinline__ Bucket load_bucket(const EdgeSlot* t, uint64_t b) {
  const uint4* p = reinterpret_cast<const uint4*>(t + b * kEdgeSlotsPerBucket);
  return Bucket{p[0], p[1], p[2], p[3]};
}

// 1 = found (child set), 0 = absent (an empty slot ends the chain), 2 = go on
__device__ __forceinline__ int scan_bucket(const Bucket& B, uint32_t parent, uint32_t word, uint32_t& child) {
  if (B.s0.x == parent && B.s0.y == word) { child = B.s0.z; return 1; }
  if (B.s1.x == parent && B.s1.y == word) { child = B.s1.z; return 1; }
  if (B.s2.x == parent && B.s2.y == word) { child = B.s2.z; return 1; }
  if (B.s3.x == parent && B.s3.y == word) { child = B.s3.z; return 1; }
  if (B.s0.x == kEmpty || B.s1.x == kEmpty || B.s2.x == kEmpty || B.s3.x == kEmpty) return 0;
  return 2;
}

// Continue a probe chain from bucket b+1 (rare: the first bucket was full).
__device__ __noinline__ uint32_t probe_rest(const EdgeSlot* t, uint64_t mask, uint64_t b, uint32_t parent,
                                            uint32_t word) {
  for (uint64_t i = 0; i < mask; i++) {
    b = (b + 1) & mask;
    uint32_t c = kNone;
    int r = scan_bucket(load_bucket(t, b), parent, word, c);
    if (r == 1) return c;
    if (r == 0) return kNone;
  }
  return kNone;
}

// ------------------------------------------------------------- scratch
template <bool SLOW>
struct Scratch {
  uint2* stack;   // {path, depth}
  uint32_t* cand; // path ids
  uint2* keys;    // key id, then {record off, cumulative start}
  uint32_t scap, ccap, kcap;
};

enum : uint32_t { kErrDeferFull = 1u, kErrFrontier = 2u, kErrOverflow = 4u, kErrMismatch = 8u };

// ------------------------------------------------------------- one publish
template <int MODE, bool SLOW>
__device__ void match_publish(const MatchArgs& a, uint32_t p, const Scratch<SLOW>& s) {
  const uint32_t lane = lane_id();
  const vmqg_pub pub = a.pubs[p];
  const uint32_t L = pub.nwords;
  const uint32_t* w = a.words + pub.word_off;
  const bool dollar = (pub.flags & VMQG_PUB_DOLLAR) != 0;
  // lane i keeps word i (i < 64) in a register; deeper words come from memory
  const uint32_t wreg = lane < L ? w[lane] : kUnknownWord;

  bool overflow = false;
  uint32_t nc = 0;   // candidates
  uint32_t sp = 0;   // stack depth

  if (pub.mountpoint < a.max_mp && L > 0) {
    if (lane == 0) s.stack[0] = make_uint2(pub.mountpoint, 0u);  // {MP, root}
    sp = 1;
  }
  wave_sync();

  // ---- trie walk: trie_match/4 + 'trie_match_#'/2  (vmq_reg_trie.erl:358-383)
  while (sp > 0) {
    const uint32_t k = sp < 64u ? sp : 64u;
    const uint32_t base = sp - k;
    const bool act = lane < k;
    uint32_t node = 0, d = 0;
    if (act) { const uint2 e = s.stack[base + lane]; node = e.x; d = e.y; }
    sp = base;
    wave_sync();
    const bool at_end = act && d == L;
    // every lane takes part in the shuffle (the source lane may be inactive)
    const uint32_t wsh = __shfl(wreg, (int)(d & 63u), 64);
    uint32_t wd = kUnknownWord;
    if (act && !at_end) wd = d < 64u ? wsh : w[d];
    const bool do_w = act && !at_end && wd != kPlus && wd != kHash && wd != kUnknownWord;
    const bool do_p = act && !at_end;
    // issue the three bucket loads before resolving any of them
    const uint64_t bh = edge_hash(node, kHash) & a.edge_mask;
    const uint64_t bw = edge_hash(node, wd) & a.edge_mask;
    const uint64_t bp = edge_hash(node, kPlus) & a.edge_mask;
    Bucket Bh{}, Bw{}, Bp{};
    if (act) Bh = load_bucket(a.edges, bh);
    if (do_w) Bw = load_bucket(a.edges, bw);
    if (do_p) Bp = load_bucket(a.edges, bp);
    uint32_t hc = kNone, wc = kNone, pc = kNone;
    if (act) { int r = scan_bucket(Bh, node, kHash, hc); if (r == 2) hc = probe_rest(a.edges, a.edge_mask, bh, node, kHash); }
    if (do_w) { int r = scan_bucket(Bw, node, wd, wc); if (r == 2) wc = probe_rest(a.edges, a.edge_mask, bw, node, wd); }
    if (do_p) { int r = scan_bucket(Bp, node, kPlus, pc); if (r == 2) pc = probe_rest(a.edges, a.edge_mask, bp, node, kPlus); }

    // candidates: the '#' child (:377-383) and, with no words left, the node itself (:361-363)
    const uint64_t m_hc = __ballot(hc != kNone), m_end = __ballot(at_end);
    const uint32_t n_new_c = (uint32_t)(__popcll(m_hc) + __popcll(m_end));
    // frontier pushes: the W and '+' children (:364-375)
    const uint64_t m_wc = __ballot(wc != kNone), m_pc = __ballot(pc != kNone);
    const uint32_t n_new_s = (uint32_t)(__popcll(m_wc) + __popcll(m_pc));
    if (nc + n_new_c > s.ccap || sp + n_new_s > s.scap) { overflow = true; break; }
    if (hc != kNone) s.cand[nc + prefix_bits(m_hc)] = hc;
    if (at_end) s.cand[nc + __popcll(m_hc) + prefix_bits(m_end)] = node;
    nc += n_new_c;
    // push '+' children first so that the W branch is popped first (any order is valid)
    if (pc != kNone) s.stack[sp + prefix_bits(m_pc)] = make_uint2(pc, d + 1);
    if (wc != kNone) s.stack[sp + __popcll(m_pc) + prefix_bits(m_wc)] = make_uint2(wc, d + 1);
    sp += n_new_s;
    wave_sync();
  }

  // ---- candidates -> subscriber-list keys: match/4, match_/3 (:283-303)
  uint64_t rmask = 0;
  uint32_t nk = 0;
  if (!overflow) {
    for (uint32_t c0 = 0; c0 < nc; c0 += 64) {
      const uint32_t ci = c0 + lane;
      uint32_t nkeys = 0, key = kNone, meta = 0;
      uint64_t rm = 0;
      if (ci < nc) {
        const uint32_t path = s.cand[ci];
        if (path < a.node_cap) {
          const uint4 r = *reinterpret_cast<const uint4*>(a.nodes + path);
          meta = r.x;
          const bool valid = (meta & kNodeEmits) == kNodeEmits &&
                             !(dollar && (meta & kNodeDollarSkip));  // MQTT-4.7.2-1 (:285-288)
          if (valid) {
            nkeys = meta >> 8;
            key = r.y;
            rm = ((uint64_t)r.w << 32) | r.z;
          }
        }
      }
      rmask |= rm;
      const uint32_t incl = wave_incl_scan(nkeys);
      const uint32_t tot = __shfl(incl, 63, 64);
      if (nk + tot > s.kcap) { overflow = true; break; }
      const uint32_t at = nk + incl - nkeys;
      if (nkeys == 1) s.keys[at] = make_uint2(key, 0u);
      else for (uint32_t j = 0; j < nkeys; j++) s.keys[at + j] = make_uint2(a.keylist[key + j], 0u);
      nk += tot;
    }
  }
  wave_sync();

  // ---- the exact candidate {Topic, node()} and remote exact subscribers (:62, :514-520)
  if (!overflow && pub.mountpoint < a.max_mp) {
    uint64_t part = 0;
    for (uint32_t i = lane; i < L; i += 64) part += fp_word(i < 64 ? wreg : w[i], i);
    const uint64_t fp = fp_final(wave_sum64(part), pub.mountpoint, L);
    uint64_t b = fp & a.exact_mask;
    for (uint64_t iter = 0; iter <= a.exact_mask; iter++) {
      const ExactSlot* bk = a.exact + b * kExactSlotsPerBucket;
      bool seen_empty = false, found = false;
      for (uint32_t j = 0; j < kExactSlotsPerBucket && !found; j++) {
        const ExactSlot e = bk[j];
        if (e.nwords == kEmpty) { seen_empty = true; break; }
        if (e.fp != fp || e.mp != pub.mountpoint || e.nwords != L) continue;
        // exactness: compare the stored words lane-parallel
        bool diff = false;
        for (uint32_t i = lane; i < L; i += 64) diff |= a.exwords[e.words_off + i] != (i < 64 ? wreg : w[i]);
        if (__ballot(diff) != 0) continue;
        found = true;
        rmask |= e.rmask;
        if (e.key != kNone) {
          if (nk + 1 > s.kcap) overflow = true;
          else { if (lane == 0) s.keys[nk] = make_uint2(e.key, 0u); nk += 1; }
        }
      }
      if (found || seen_empty) break;
      b = (b + 1) & a.exact_mask;
    }
  }
  wave_sync();
  rmask = wave_or64(rmask) & ~(1ull << a.local_node);

  if (overflow) {
    if (MODE == 0) {
      if (lane == 0) {
        if (SLOW) {
          atomicOr(&a.status[1], kErrFrontier);
          a.offsets[p] = 0;
        } else {
          const uint32_t idx = atomicAdd(&a.status[0], 1u);
          if (idx < a.deferred_cap) a.deferred[idx] = p;
          else atomicOr(&a.status[1], kErrDeferFull);
          a.offsets[p] = 0;
        }
      }
    }
    return;
  }

  // ---- record counts per key: lookup_subs/1 (:87-94)
  uint32_t ksum = 0;
  for (uint32_t k0 = 0; k0 < nk; k0 += 64) {
    const uint32_t ki = k0 + lane;
    uint32_t cnt = 0, off = 0;
    if (ki < nk) {
      const uint32_t key = s.keys[ki].x;
      if (key < a.key_cap) { const uint2 kd = *reinterpret_cast<const uint2*>(a.keydesc + key); off = kd.x; cnt = kd.y; }
    }
    const uint32_t incl = wave_incl_scan(cnt);
    wave_sync();
    if (ki < nk) s.keys[ki] = make_uint2(off, ksum + incl - cnt);
    ksum += __shfl(incl, 63, 64);
  }
  const uint32_t nrem = (uint32_t)__popcll(rmask);
  const uint32_t total = ksum + nrem;

  if (MODE == 0) {
    if (lane == 0) a.offsets[p] = total;
    return;
  }

  // ---- EMIT: fold__/4 (:96-98) — one FoldFun argument per record
  const uint64_t obase = a.offsets[p], oend = a.offsets[p + 1];
  if (oend > a.out_cap) { if (lane == 0) atomicOr(&a.status[1], kErrOverflow); return; }
  if (oend - obase != total) { if (lane == 0) atomicOr(&a.status[1], kErrMismatch); return; }
  wave_sync();
  for (uint32_t r = lane; r < total; r += 64) {
    uint4 v;
    if (r < ksum) {
      uint32_t lo = 0, hi = nk;  // last key with cum_start <= r
      while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (s.keys[mid].y <= r) lo = mid; else hi = mid; }
      const uint2 kk = s.keys[lo];
      v = *reinterpret_cast<const uint4*>(a.records + kk.x + (r - kk.y));
    } else {
      // j-th remote node of the mask, in node order (fold_/5 :78-84)
      uint64_t m = rmask;
      for (uint32_t j = r - ksum; j > 0; j--) m &= m - 1;
      const uint32_t node = (uint32_t)__builtin_ctzll(m);
      v = make_uint4((VMQG_EMIT_REMOTE << 24) | node, kNone, kNone, kNone);
    }
    *reinterpret_cast<uint4*>(a.out + obase + r) = v;
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void k_match_fast(MatchArgs a) {
  __shared__ uint2 st[kWaves][kSCap];
  __shared__ uint32_t cd[kWaves][kCCap];
  __shared__ uint2 ky[kWaves][kKCap];
  const uint32_t wv = threadIdx.x >> 6;
  Scratch<false> s{st[wv], cd[wv], ky[wv], kSCap, kCCap, kKCap};
  const uint32_t nwaves = gridDim.x * kWaves;
  for (uint32_t p = blockIdx.x * kWaves + wv; p < a.npub; p += nwaves) {
    match_publish<MODE, false>(a, p, s);
    wave_sync();
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void k_match_slow(MatchArgs a) {
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t gw = blockIdx.x * kWaves + wv;
  Scratch<true> s{a.g_stack + (uint64_t)gw * a.g_scap, a.g_cand + (uint64_t)gw * a.g_ccap,
                  a.g_keys + (uint64_t)gw * a.g_kcap, a.g_scap, a.g_ccap, a.g_kcap};
  uint32_t n = a.status[0];
  if (n > a.deferred_cap) n = a.deferred_cap;
  const uint32_t nwaves = gridDim.x * kWaves;
  for (uint32_t d = gw; d < n; d += nwaves) {
    match_publish<MODE, true>(a, a.deferred[d], s);
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
    uint64_t t = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
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
  hipError_t e = launch_scan(tmp, tiles, tmp + tiles, st);
  if (e != hipSuccess) return e;
  k_scan_add<<<(uint32_t)tiles, kScanBlock, 0, st>>>(v, n, tmp);
  return hipGetLastError();
}

uint64_t scan_tmp_elems(uint64_t n) {
  uint64_t tot = 0;
  for (uint64_t t = (n + kScanTile - 1) / kScanTile; t > 1; t = (t + kScanTile - 1) / kScanTile) tot += t;
  return tot + 1;
}

uint32_t fast_grid(uint32_t npub) {
  const uint32_t want = div_up(npub, kWaves);
  const uint32_t cap = 256u * 16u;  // grid-stride beyond 16 blocks per CU
  return want < 1 ? 1 : (want < cap ? want : cap);
}

hipError_t launch_match(const MatchArgs& a, int mode, bool slow, hipStream_t st) {
  if (!slow) {
    const uint32_t g = fast_grid(a.npub);
    if (mode == 0) k_match_fast<0><<<g, 256, 0, st>>>(a);
    else k_match_fast<1><<<g, 256, 0, st>>>(a);
  } else {
    const uint32_t g = a.g_waves / kWaves;
    if (mode == 0) k_match_slow<0><<<g, 256, 0, st>>>(a);
    else k_match_slow<1><<<g, 256, 0, st>>>(a);
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
