// HIP kernels for gfx950: vmq_retain_srv:match_fold/4 for a batch of
// subscription filters (apps/vmq_server/src/vmq_retain_srv.erl:75-99).
//
// The reference answers a wildcard filter with a full ets:foldl over the
// retained table, testing every entry with vmq_topic:match/2.  Here the same
// test runs on the rows of ONE list: the shortest of the lists the filter's
// literal words select — {MP, w0, w1} for two literal leading words, or
// {MP, w_k, k} for a literal word at position k — else the MP's list (a
// filter of '+' and '#' only).  Every other row fails the test anyway (other
// MP, or a different word where the filter has a literal,
// vmq_topic.erl:55-65).  The rows of all filters' lists form one flat,
// filter-major row space (filter f owns rows [rpfx[f], rpfx[f+1])):
//   k_rt_plan   one thread per filter: has_wildcard/1 (:239-242); the exact
//               ets:lookup (:93-98) as a fingerprint probe + word compare;
//               else the shortest selecting list and its length;
//   scan        rows per filter -> rpfx (one launch, decoupled look-back);
//   k_rt_walk   one wave per 1,024-row tile, tiles taken in ticket order:
//               64 rows per step, one row per lane, each lane's filter found
//               in an LDS window of rpfx; vmq_topic:match/2 of the row's
//               topic (its 32-B list entry carries the first words) against
//               the filter; hits (message ids) compacted in
//               LDS with ballot + mbcnt; the tile's output base from a
//               decoupled look-back over the tiles before it; then one
//               contiguous store of the tile's hits and the offsets of the
//               filters whose rows start in the tile.  One pass: no count
//               pass, no second scan.
// Bound: HBM / L2 reads of 16-B rows, their words and the 4-B list entries;
// no MFMA (integer compares only).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "vmqr_engine.h"
#include "vmqg_lookback.h"

namespace vmqr {

using vmqg::kEmpty;
using vmqg::kHash;
using vmqg::kNone;
using vmqg::kPlus;

constexpr int kW = 4;                 // waves per 256-thread block
constexpr uint64_t kShortList = 64;   // plan: a list this short ends the search for a shorter one
constexpr uint64_t kKindExact = 1ull << 62, kKindList = 2ull << 62, kCountMask = (1ull << 62) - 1;
constexpr uint32_t kErrChunks = 32u;  // status[1]: the batch walks more tiles than look-back granules
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
  // this call's status words and walk tickets start at zero (read only by
  // the kernels after this one on the stream)
  if (blockIdx.x == 0 && threadIdx.x < 8) {
    a.status[threadIdx.x] = 0;
    a.tickets[threadIdx.x * kTicketStride] = 0;
  }
  for (uint32_t f = blockIdx.x * blockDim.x + threadIdx.x; f < a.nf; f += gridDim.x * blockDim.x) {
    const vmqg_pub F = a.filters[f];
    const uint32_t* w = a.words + F.word_off;
    const uint32_t L = F.nwords;
    uint64_t off = 0, cnt = 0, kind = kKindList;
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
      } else {
        bool unknown = false;   // a literal word no retained topic holds: nothing can match (:55-57)
        for (uint32_t i = 0; i < L && !unknown; i++) unknown = w[i] == vmqg::kUnknownWord;
        if (unknown) {
          cnt = 0;
        } else {
          // the shortest list a literal word selects: {MP, w0, w1}, or
          // {MP, w_k, k} for a literal at position k; else the MP list
          // (first word '+' and no other literal, or exactly '#')
          const MpList m = a.mpl[F.mountpoint];
          off = m.off; cnt = m.count;
          const uint32_t np = L < kMaxPos ? L : kMaxPos;
          for (uint32_t k = 0; k <= np; k++) {
            uint32_t ka, kb, kk;
            if (k == 0) {   // the pair list
              if (L < 2 || w[0] == kPlus || w[0] == kHash || w[1] == kPlus || w[1] == kHash) continue;
              ka = w[0]; kb = w[1]; kk = kPair;
            } else {
              ka = w[k - 1]; kb = k - 1; kk = kPos;
              if (ka == kPlus || ka == kHash) continue;
            }
            uint64_t o = 0, c = 0;   // a missing list: no retained topic has that word there
            for (uint64_t b = part_hash(F.mountpoint, ka, kb, kk) & a.ptab_mask, n = 0; n <= a.ptab_mask;
                 b = (b + 1) & a.ptab_mask, n++) {
              bool done = false;
              for (uint32_t j = 0; j < kPSlotsPerBucket; j++) {
                const PSlot s = a.ptab[b * kPSlotsPerBucket + j];
                if (s.mp == kEmpty) { done = true; break; }
                if (s.mp == F.mountpoint && s.a == ka && s.b == kb && s.kind == kk) { o = s.off; c = s.count; done = true; break; }
              }
              if (done) break;
            }
            if (c < cnt) { off = o; cnt = c; }
            if (cnt <= kShortList) break;   // one walk step: no further probe can pay for itself
          }
        }
      }
    }
    a.plan[2 * (uint64_t)f] = off;
    a.plan[2 * (uint64_t)f + 1] = cnt | kind;
    a.rpfx[f] = cnt;   // rows the walk visits for this filter
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
      const uint64_t b = vmqg::lookback(lb, tag, status + 1, tile, part[kSB - 1]);
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

// ------------------------------------------------------------- walk pass
constexpr uint32_t kGroups = kTileRows / 64;    // 64-row steps per tile
constexpr uint32_t kWin = 64;                   // rpfx window (filters) per step
#ifndef VMQR_U
#define VMQR_U 4
#endif
constexpr uint32_t kU = VMQR_U;                 // 64-row steps in flight per lane
constexpr uint32_t kClasses = 8;                // ticket counters (block classes)
constexpr uint32_t kPre = kLWords;              // topic / filter words in registers per row
static_assert(kGroups % kU == 0, "");

// vmq_topic:match/2 as topic_match, with the first kPre words of both
// already in registers (the rest read from memory).
__device__ __forceinline__ bool topic_match_pre(const uint32_t (&tw)[kPre], const uint32_t (&fw)[kPre],
                                                const uint32_t* t, uint32_t nt, const uint32_t* f, uint32_t nf) {
  bool done = false, res = false;
#pragma unroll
  for (uint32_t k = 0; k < kPre; k++) {   // constant indices, results by value: the words stay in registers
    const uint32_t tk = tw[k], fk = fw[k];
    const bool end = k == nt && k == nf;
    const bool step = k < nt && k < nf && (tk == fk || fk == kPlus);
    if (!done && !step) res = end || (k + 1 == nf && fk == kHash);
    done = done || !step;
  }
  if (done) return res;
  for (uint32_t i = kPre;;) {
    if (i == nt && i == nf) return true;
    const uint32_t fi = i < nf ? f[i] : 0u;
    if (i < nt && i < nf && (t[i] == fi || fi == kPlus)) { i++; continue; }
    return i + 1 == nf && fi == kHash;
  }
}

// Last filter f in [lo, hi) with rpfx[f] <= x (rpfx[lo] <= x < rpfx[hi]),
// 64-ary search by the whole wave: each round probes 64 evenly spaced
// entries with one load per lane.
__device__ __forceinline__ uint32_t wave_search(const uint64_t* rpfx, uint32_t lo, uint32_t hi, uint64_t x) {
  const uint32_t lane = __lane_id();
  while (hi - lo > 1) {
    const uint32_t step = (hi - lo + 63) / 64;
    const uint32_t p = lo + lane * step;
    const bool le = p < hi && rpfx[p] <= x;
    const uint64_t m = __ballot(le);                      // lanes 0..k* (monotone)
    const uint32_t k = 63 - __builtin_clzll(m);           // lane 0 always qualifies
    lo = lo + k * step;
    hi = lo + step < hi ? lo + step : hi;
  }
  return lo;
}

__global__ __launch_bounds__(256) void k_rt_walk(RArgs a) {
  __shared__ uint32_t s_hits[kW][kTileRows];     // message ids of the tile's hits, in row order
  __shared__ uint64_t s_mask[kW][kGroups];       // hit mask per 64-row step
  __shared__ uint64_t s_win[kW][kWin + 1];       // rpfx[f0 .. f0 + 64]
  __shared__ uint32_t s_round;
  const uint32_t wv = threadIdx.x >> 6, lane = __lane_id();
  const uint64_t R = a.rpfx[a.nf];                // rows of the batch
  const uint64_t ntiles = (R + kTileRows - 1) / kTileRows;
  if (ntiles > a.tile_cap) {                      // granules exhausted: the host grows them and reruns
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&a.status[1], kErrChunks);
    return;
  }
  if (ntiles == 0) {                              // no filter has a row: every offset is 0
    for (uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; f <= a.nf; f += (uint64_t)gridDim.x * blockDim.x)
      a.offsets[f] = 0;
    return;
  }
  uint32_t* hits = s_hits[wv];
  uint64_t* mask = s_mask[wv];
  uint64_t* win = s_win[wv];
  // Tiles by ticket, one atomic per block and round: class c = blockIdx % 8
  // (one XCD each under round-robin dispatch) owns tiles c, c + 8, ...;
  // round r of a class-c block gives its wave w tile (4r + w) * 8 + c.
  // Look-back waits only on lower tiles, and the lowest tile in progress
  // never waits on an untaken one: its class's blocks hold lower rounds.
  const uint32_t cls = blockIdx.x % kClasses;
  for (;;) {
    if (threadIdx.x == 0) s_round = atomicAdd(a.tickets + cls * kTicketStride, 1u);
    __syncthreads();
    const uint32_t round = s_round;
    if (((uint64_t)round * kW) * kClasses + cls >= ntiles) break;   // uniform in the block
    const uint64_t tile64 = ((uint64_t)round * kW + wv) * kClasses + cls;
    if (tile64 < ntiles) {
    const uint32_t tile = (uint32_t)tile64;
    const uint64_t base = (uint64_t)tile * kTileRows;
    const uint64_t end = base + kTileRows < R ? base + kTileRows : R;
    uint32_t f0 = wave_search(a.rpfx, 0, a.nf, base);   // filter of the tile's first row
    uint32_t nh = 0;                                     // hits so far in the tile
    // kU steps of 64 rows at a time: each lane has kU rows in flight, every
    // load of one row independent of the others'
    for (uint32_t g = 0; g < kGroups; g += kU) {
      const uint64_t g0 = base + (uint64_t)g * 64;
      if (g0 >= end) {
        if (lane == 0) for (uint32_t h = g; h < kGroups; h++) mask[h] = 0;
        break;
      }
      // window of filter starts around these rows
      const uint32_t wf = f0 + lane;
      win[lane] = wf <= a.nf ? a.rpfx[wf] : ~0ull;
      if (lane == 0) win[kWin] = f0 + kWin <= a.nf ? a.rpfx[f0 + kWin] : ~0ull;
      __builtin_amdgcn_wave_barrier();
      uint32_t f[kU];
      uint64_t pc[kU], off[kU];
      bool ok[kU];
#pragma clang loop unroll(full)
      for (uint32_t u = 0; u < kU; u++) {
        const uint64_t gi = g0 + u * 64 + lane;
        ok[u] = gi < end;
        f[u] = f0;
        if (!ok[u]) continue;
        uint64_t start;
        if (win[kWin] <= gi) {
          // more than 64 filter starts before this row (runs of empty
          // filters): search the rest of rpfx
          uint32_t lo = f0 + kWin, hi = a.nf;
          while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (a.rpfx[mid] <= gi) lo = mid; else hi = mid;
          }
          f[u] = lo;
          start = a.rpfx[lo];
        } else {
          uint32_t lo = 0, hi = kWin;   // win[lo] <= gi < win[hi]
          while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (win[mid] <= gi) lo = mid; else hi = mid;
          }
          f[u] = f0 + lo;
          start = win[lo];
        }
        pc[u] = a.plan[2 * (uint64_t)f[u] + 1];
        off[u] = a.plan[2 * (uint64_t)f[u]] + (gi - start);   // list slot (exact: the row)
      }
      // one 32-B list entry per candidate (exact filters: the looked-up row)
      LEnt e[kU];
      vmqg_pub F[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; u++) {
        if (!ok[u]) continue;
        if ((pc[u] & ~kCountMask) == kKindExact) {
          e[u].msg = a.rows[(uint32_t)off[u]].msg;
        } else {
          e[u] = a.lists[off[u]];
          F[u] = a.filters[f[u]];
        }
      }
      // the filter's first kPre words in registers (the topic's are in the entry)
      uint32_t fw[kU][kPre];
#pragma unroll
      for (uint32_t u = 0; u < kU; u++) {
        const bool list = ok[u] && (pc[u] & ~kCountMask) != kKindExact;
#pragma unroll
        for (uint32_t k = 0; k < kPre; k++) fw[u][k] = list && k < F[u].nwords ? a.words[F[u].word_off + k] : 0u;
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; u++) {
        bool hit = false;
        if (ok[u]) {
          // the plan already verified an exact filter's key; list rows all
          // belong to the filter's MP
          hit = (pc[u] & ~kCountMask) == kKindExact ||
                topic_match_pre(e[u].w, fw[u], a.rwords + e[u].words_off, e[u].nwords, a.words + F[u].word_off,
                                F[u].nwords);
        }
        const uint64_t m = __ballot(hit);
        if (hit)
          hits[nh + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
              e[u].msg;
        if (lane == 0) mask[g + u] = m;
        nh += (uint32_t)__popcll(m);
      }
      // the next rows start at the filter of the last row (lanes past the
      // end kept f0, and the loop ends with them)
      f0 = __builtin_amdgcn_readlane(f[kU - 1], 63);
      __builtin_amdgcn_wave_barrier();
    }
    __builtin_amdgcn_wave_barrier();
#ifdef VMQR_DIAG_SKIP_LOOKBACK   // A/B diagnostics only (tools/rt_ab.sh): wrong offsets
    const uint64_t pre = 0;
#else
    const uint64_t pre = vmqg::lookback<32>(a.lookback, a.lb_tag + 1, a.status + 1, tile, nh);
#endif
    const uint64_t total = pre + nh;
    if (total > a.out_cap) {
      if (lane == 0) atomicOr(&a.status[1], kErrOut);
    } else {
      for (uint32_t i = lane; i < nh; i += 64) a.out[pre + i] = hits[i];
    }
    // offsets of the filters whose rows start in this tile (the last tile
    // also takes the ones starting at R: trailing empty filters and [nf])
    const bool last = tile + 1 == ntiles;
    // first candidate: the filter holding row base - 1 (its start is < base)
    for (uint32_t fb = base ? wave_search(a.rpfx, 0, a.nf, base - 1) : 0;; fb += 64) {
      const uint32_t ff = fb + lane;
      const uint64_t p = ff <= a.nf ? a.rpfx[ff] : ~0ull;
      const bool mine = p >= base && (p < base + kTileRows || (last && p == R)) && ff <= a.nf;
      if (mine) {
        const uint64_t rel = p - base;
        const uint32_t gq = (uint32_t)(rel >> 6);
        uint64_t c = 0;
        for (uint32_t h = 0; h < gq && h < kGroups; h++) c += (uint64_t)__popcll(mask[h]);
        if (gq < kGroups) c += (uint64_t)__popcll(mask[gq] & ((1ull << (rel & 63)) - 1));
        a.offsets[ff] = pre + c;
      }
      const uint64_t beyond = __ballot(ff > a.nf || (p >= base + kTileRows && !(last && p == R)));
      if (beyond) break;   // rpfx is monotone: the tile's filters are done
    }
    }
    __syncthreads();   // s_round is rewritten next round
  }
}

// ---------------------------------------------------------------- launch
int walk_blocks_per_cu() {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_rt_walk, 256, 0) != hipSuccess || nb < 1) nb = 1;
  return nb;
}

// t[0..6) (all or none): {start, stop} of the plan, the scan and the walk,
// recorded by the dispatches themselves (hipExtLaunchKernel) rather than by
// marker packets between the launches
hipError_t launch_retain_match(const RArgs& a, uint32_t grid, hipStream_t st, const hipEvent_t* t) {
  const uint32_t gp = (a.nf + 255) / 256;
  const uint32_t gs = (uint32_t)((a.nf + 1 + kST) / kST);
  if (t) {
    hipExtLaunchKernelGGL(k_rt_plan, dim3(gp < 2048 ? gp : 2048), dim3(256), 0, st, t[0], t[1], 0, a);
    hipExtLaunchKernelGGL(k_rt_scan, dim3(gs < 2048 ? gs : 2048), dim3(kSB), 0, st, t[2], t[3], 0, a.rpfx,
                          (uint64_t)a.nf, (const uint64_t*)nullptr, a.status + 3, a.lookback, a.lb_tag, a.status);
    hipExtLaunchKernelGGL(k_rt_walk, dim3(grid), dim3(256), 0, st, t[4], t[5], 0, a);
  } else {
    k_rt_plan<<<gp < 2048 ? gp : 2048, 256, 0, st>>>(a);
    k_rt_scan<<<gs < 2048 ? gs : 2048, kSB, 0, st>>>(a.rpfx, a.nf, nullptr, a.status + 3, a.lookback, a.lb_tag,
                                                     a.status);
    k_rt_walk<<<grid, 256, 0, st>>>(a);
  }
  return hipGetLastError();
}

}  // namespace vmqr
