// HIP kernels for gfx950: vmq_retain_srv:match_fold/4 for a batch of
// subscription filters (apps/vmq_server/src/vmq_retain_srv.erl:75-99).
//
// The reference answers a wildcard filter with a full ets:foldl over the
// retained table, testing every entry with vmq_topic:match/2.  Here the same
// test runs on the rows of ONE list: the filter's partition {MP, w0, w1}
// when its first two words are literal, {MP, w0} when only the first is,
// else (first word '+', or exactly '#') the MP's list — every other row of
// the table fails the test anyway (other MP, or different leading words,
// vmq_topic.erl:55-65).  Lists are cut into
// chunks of `chunk_rows` rows so that one huge list spreads over the chip:
//   k_rt_plan   one thread per filter: has_wildcard/1 (:239-242); the exact
//               ets:lookup (:93-98) as a fingerprint probe + word compare;
//               else the list, its length and its chunk count;
//   scan        chunk counts -> first chunk of each filter (one launch);
//   k_rt_count  one wave per chunk: 64 rows per step, one row per lane,
//               vmq_topic:match/2 against the filter words staged in LDS;
//               matches per chunk;
//   scan        chunk matches -> output offsets (one launch, device-side n);
//   k_rt_emit   the same walk writing the matching rows' message ids,
//               ballot + mbcnt compacted, contiguous per chunk; and the
//               per-filter offsets.
// Bound: HBM / L2 reads of 16-B rows and their words; no MFMA (integer
// compares only).
#include <hip/hip_runtime.h>

#include "vmqr_engine.h"
#include "vmqg_lookback.h"

namespace vmqr {

using vmqg::kEmpty;
using vmqg::kHash;
using vmqg::kNone;
using vmqg::kPlus;

constexpr int kW = 4;                 // waves per 256-thread block
constexpr uint32_t kFW = 64;          // filter words staged in LDS per wave
constexpr uint64_t kKindExact = 1ull << 62, kKindList = 2ull << 62, kCountMask = (1ull << 62) - 1;
constexpr uint32_t kErrChunks = 32u;  // status[1]: the batch needs more chunk slots than allocated
constexpr uint32_t kErrOut = 4u;      // status[1]: output overflow (VMQG_E_OVERFLOW)

__host__ __device__ inline uint64_t fp_of(uint32_t mp, const uint32_t* w, uint32_t L) {
  uint64_t s = 0;
  for (uint32_t i = 0; i < L; i++) s += vmqg::fp_word(w[i], i);
  return vmqg::fp_final(s, mp, L);
}
uint64_t retain_fp(uint32_t mp, const uint32_t* w, uint32_t L) { return fp_of(mp, w, L); }

// vmq_topic:match(T, F), vmq_topic.erl:53-65, clause order kept:
// [H|T1],[H|T2] ; [_|T1],['+'|T2] ; (_, ['#']) ; otherwise false.
__device__ __forceinline__ bool topic_match(const uint32_t* t, uint32_t nt, const uint32_t* f, uint32_t nf) {
  uint32_t i = 0;
  for (;;) {
    if (i == nt && i == nf) return true;
    if (i < nt && i < nf) {
      const uint32_t fw = f[i];
      if (t[i] == fw || fw == kPlus) { i++; continue; }
    }
    return i + 1 == nf && f[i] == kHash;
  }
}

// ------------------------------------------------------------------ plan
__global__ __launch_bounds__(256) void k_rt_plan(RArgs a) {
  for (uint32_t f = blockIdx.x * blockDim.x + threadIdx.x; f < a.nf; f += gridDim.x * blockDim.x) {
    const vmqg_pub F = a.filters[f];
    const uint32_t* w = a.words + F.word_off;
    const uint32_t L = F.nwords;
    uint64_t off = 0, cnt = 0, kind = kKindList, chunks = 0;
    if (L > 0 && F.mountpoint < a.max_mp) {
      bool wild = w[L - 1] == kHash;   // has_wildcard/1: '#' as the last word ...
      for (uint32_t i = 0; i < L && !wild; i++) wild = w[i] == kPlus;   // ... or '+' anywhere
      if (!wild) {
        // ets:lookup(?RETAIN_CACHE, {MP, Topic})
        kind = kKindExact;
        const uint64_t fp = fp_of(F.mountpoint, w, L);
        for (uint64_t i = fp & a.exact_mask, n = 0; n <= a.exact_mask; i = (i + 1) & a.exact_mask, n++) {
          const XSlot x = a.exact[i];
          if (x.state == 0) break;
          if (x.state != kXLive || x.fp != fp) continue;
          const RRow r = a.rows[x.row];
          bool eq = r.mp == F.mountpoint && r.nwords == L;
          for (uint32_t k = 0; eq && k < L; k++) eq = a.rwords[r.words_off + k] == w[k];
          if (eq) { off = x.row; cnt = 1; break; }
        }
        chunks = cnt;
      } else {
        bool unknown = false;   // a literal word no retained topic holds: nothing can match (:55-57)
        for (uint32_t i = 0; i < L && !unknown; i++) unknown = w[i] == vmqg::kUnknownWord;
        if (unknown) {
          cnt = 0;
        } else if (w[0] == kPlus || (L == 1 && w[0] == kHash)) {
          const MpList m = a.mpl[F.mountpoint];
          off = m.off; cnt = m.count;
        } else {
          // literal prefix of one or two words: the rows whose first words
          // are those (a literal filter word must equal the topic's,
          // vmq_topic.erl:55-57; '#' after two literals still needs them)
          const uint32_t w1 = L >= 2 && w[1] != kPlus && w[1] != kHash ? w[1] : kNone;
          for (uint64_t b = part_hash(F.mountpoint, w[0], w1) & a.ptab_mask, n = 0; n <= a.ptab_mask;
               b = (b + 1) & a.ptab_mask, n++) {
            bool done = false;
            for (uint32_t j = 0; j < kPSlotsPerBucket; j++) {
              const PSlot s = a.ptab[b * kPSlotsPerBucket + j];
              if (s.mp == kEmpty) { done = true; break; }
              if (s.mp == F.mountpoint && s.w0 == w[0] && s.w1 == w1) { off = s.off; cnt = s.count; done = true; break; }
            }
            if (done) break;
          }
        }
        chunks = (cnt + a.chunk_rows - 1) / a.chunk_rows;
      }
    }
    a.plan[2 * (uint64_t)f] = off;
    a.plan[2 * (uint64_t)f + 1] = cnt | kind;
    a.fchunks[f] = chunks;
  }
}

// ------------------------------------------------------------------ scans
// In-place exclusive scan of v[0, n) into v[0, n] (v[n] = total, v[n] never
// read), one launch, tiles by ticket + decoupled look-back.  n = n_host, or
// min(*n_dev, n_host) when n_dev is set (the chunk count is only known on
// the device; n_host is then the array's capacity).
constexpr uint32_t kSI = 16, kSB = 256, kST = kSI * kSB;

__global__ __launch_bounds__(256) void k_rt_scan(uint64_t* v, uint64_t n_host, const uint64_t* n_dev, uint32_t* ticket,
                                                 uint64_t* lb, uint32_t tag, uint32_t* status) {
  __shared__ uint64_t part[kSB];
  __shared__ uint32_t s_tile;
  __shared__ uint64_t s_base;
  const uint64_t n = n_dev ? (*n_dev < n_host ? *n_dev : n_host) : n_host;
  const uint32_t ntiles = (uint32_t)((n + 1 + kST - 1) / kST);
  for (;;) {
    if (threadIdx.x == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    if (tile >= ntiles) break;
    const uint64_t base = (uint64_t)tile * kST + (uint64_t)threadIdx.x * kSI;
    uint64_t x[kSI];
    uint64_t acc = 0;
#pragma unroll
    for (uint32_t i = 0; i < kSI; i++) { x[i] = base + i < n ? v[base + i] : 0; acc += x[i]; }
    part[threadIdx.x] = acc;
    __syncthreads();
    for (uint32_t o = 1; o < kSB; o <<= 1) {
      const uint64_t t = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
      __syncthreads();
      part[threadIdx.x] += t;
      __syncthreads();
    }
    if (threadIdx.x < 64) {
      const uint64_t b = vmqg::lookback(lb, tag, status, tile, part[kSB - 1]);
      if (threadIdx.x == 0) s_base = b;
    }
    __syncthreads();
    uint64_t run = s_base + part[threadIdx.x] - acc;
#pragma unroll
    for (uint32_t i = 0; i < kSI; i++) {
      if (base + i <= n) v[base + i] = run;
      run += x[i];
    }
    __syncthreads();
  }
}

// ------------------------------------------------------ count / emit pass
// Chunk c of the batch -> its filter (last f with fchunks[f] <= c) and its
// row range; the filter's words staged in the wave's LDS slice.
struct ChunkWork {
  uint32_t f, L, mp;
  uint64_t kind, off, lo, hi;
  const uint32_t* fw;   // filter words (LDS, or global for > kFW words)
};

__device__ __forceinline__ ChunkWork chunk_work(const RArgs& a, uint64_t c, uint32_t* lds_fw) {
  uint32_t lo = 0, hi = a.nf;   // fchunks[lo] <= c < fchunks[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a.fchunks[mid] <= c) lo = mid; else hi = mid;
  }
  ChunkWork k;
  k.f = lo;
  const vmqg_pub F = a.filters[lo];
  k.L = F.nwords;
  k.mp = F.mountpoint;
  const uint64_t pc = a.plan[2 * (uint64_t)lo + 1];
  k.kind = pc & ~kCountMask;
  k.off = a.plan[2 * (uint64_t)lo];
  const uint64_t cnt = pc & kCountMask;
  const uint64_t kth = c - a.fchunks[lo];
  k.lo = kth * a.chunk_rows;
  k.hi = k.lo + a.chunk_rows < cnt ? k.lo + a.chunk_rows : cnt;
  const uint32_t* w = a.words + F.word_off;
  const uint32_t lane = __lane_id();
  if (k.L <= kFW) {
    if (lane < k.L) lds_fw[lane] = w[lane];
    __builtin_amdgcn_wave_barrier();
    k.fw = lds_fw;
  } else {
    k.fw = w;
  }
  return k;
}

// Row i of the chunk matches?  Exact chunks hold the looked-up row (already
// verified by the plan); list chunks test vmq_topic:match/2 on the row.
__device__ __forceinline__ bool row_hits(const RArgs& a, const ChunkWork& k, uint64_t i, uint32_t& msg) {
  const uint32_t id = k.kind == kKindExact ? (uint32_t)k.off : a.lists[k.off + i];
  const RRow r = a.rows[id];
  msg = r.msg;
  if (k.kind == kKindExact) return true;
  return r.mp == k.mp && topic_match(a.rwords + r.words_off, r.nwords, k.fw, k.L);
}

template <int MODE>
__global__ __launch_bounds__(256) void k_rt_walk(RArgs a) {
  __shared__ uint32_t fw[kW][kFW];
  const uint32_t wv = threadIdx.x >> 6, lane = __lane_id();
  const uint64_t total = a.fchunks[a.nf];
  if (MODE == 0 && blockIdx.x == 0 && threadIdx.x == 0 && total > a.chunk_cap) atomicOr(&a.status[1], kErrChunks);
  const uint64_t ntot = total < a.chunk_cap ? total : a.chunk_cap;
  if (MODE == 1) {
    // per-filter offsets: first output of the filter's first chunk
    const uint64_t grand = a.ccount[ntot];
    if (grand > a.out_cap && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&a.status[1], kErrOut);
    for (uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; f <= a.nf; f += (uint64_t)gridDim.x * blockDim.x) {
      const uint64_t fc = a.fchunks[f];
      a.offsets[f] = a.ccount[fc < ntot ? fc : ntot];
    }
    if (grand > a.out_cap || total > a.chunk_cap) return;
  }
  for (uint64_t c = (uint64_t)blockIdx.x * kW + wv; c < ntot; c += (uint64_t)gridDim.x * kW) {
    const ChunkWork k = chunk_work(a, c, fw[wv]);
    uint64_t run = MODE == 1 ? a.ccount[c] : 0;
    for (uint64_t i0 = k.lo; i0 < k.hi; i0 += 64) {
      const uint64_t i = i0 + lane;
      uint32_t msg = 0;
      const bool hit = i < k.hi && row_hits(a, k, i, msg);
      const uint64_t m = __ballot(hit);
      if (MODE == 1 && hit) a.out[run + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = msg;
      run += (uint64_t)__popcll(m);
    }
    if (MODE == 0 && lane == 0) a.ccount[c] = run;
    __builtin_amdgcn_wave_barrier();
  }
}

// ---------------------------------------------------------------- launch
hipError_t launch_retain_match(const RArgs& a, uint32_t grid, hipStream_t st, hipEvent_t ec0, hipEvent_t ec1,
                               hipEvent_t ee0, hipEvent_t ee1) {
  const uint32_t gp = (a.nf + 255) / 256;
  k_rt_plan<<<gp < 2048 ? gp : 2048, 256, 0, st>>>(a);
  uint32_t gs = (uint32_t)((a.nf + 1 + kST) / kST);
  k_rt_scan<<<gs < 2048 ? gs : 2048, kSB, 0, st>>>(a.fchunks, a.nf, nullptr, a.status + 3, a.lookback, a.lb_tag,
                                                   a.status);
  if (ec0) hipEventRecord(ec0, st);
  k_rt_walk<0><<<grid, 256, 0, st>>>(a);
  if (ec1) hipEventRecord(ec1, st);
  // chunk totals: the count is device-side (fchunks[nf]); the ticket loop
  // stops at the real tile count, the grid only bounds the parallelism
  gs = (uint32_t)((a.chunk_cap + 1 + kST) / kST);
  k_rt_scan<<<gs < 1024 ? gs : 1024, kSB, 0, st>>>(a.ccount, a.chunk_cap, a.fchunks + a.nf, a.status + 4, a.lookback,
                                                   a.lb_tag + 1, a.status);
  if (ee0) hipEventRecord(ee0, st);
  k_rt_walk<1><<<grid, 256, 0, st>>>(a);
  if (ee1) hipEventRecord(ee1, st);
  return hipGetLastError();
}

}  // namespace vmqr
