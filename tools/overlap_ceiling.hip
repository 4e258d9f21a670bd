// Does COUNT's work overlap EMIT's on MI355X?  COUNT is bound by the rate of
// random 64-B line reads (3 dependent bucket probes per publish into a 270 MB
// table), EMIT by 16-B streaming stores (1.1 GB per 2^20 publishes).  If the
// two limits are different resources, one launch that runs both kinds of work
// side by side on every CU finishes sooner than the two launches back to back.
//
//   probe  : 2^20 chains x 3 dependent random bucket reads (2 lanes a chain)
//   store  : 1.1 GB of wave-contiguous 16-B non-temporal stores, 8 per lane
//   mixed  : one launch, waves grid-stride over tickets; ticket t is a probe
//            chunk (32 chains per wave) or a store tile (8 KiB per wave)
//            interleaved in proportion, so every CU runs both all the time
//            (a first version drew tickets from one atomic counter: 7x
//            slower, the counter serialised every wave)
//
// Prints one JSON line per variant: probe alone, store alone, their sum, mixed;
// then both kernels launched together on two streams.
//
// build: hipcc --offload-arch=gfx950 -O3 -o overlap_ceiling tools/overlap_ceiling.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(err_)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

constexpr int U = 8;                     // records per lane per store tile
constexpr uint64_t kTile = 64ull * U;    // records per store tile (8 KiB)
constexpr uint32_t kChainsPerWave = 32;  // 2 lanes per chain

__device__ __forceinline__ void probe_chunk(const uint4* tab, uint32_t nb, uint32_t c0, uint32_t nchains, uint32_t salt,
                                            uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63, sub = lane & 1;
  const uint32_t c = c0 + lane / 2;
  if (c >= nchains) return;
  uint32_t b = mix(c ^ salt) % nb, acc = 0;
#pragma unroll
  for (int d = 0; d < 3; d++) {
    const uint4 v0 = tab[(uint64_t)b * 4 + sub * 2], v1 = tab[(uint64_t)b * 4 + sub * 2 + 1];
    uint32_t h = v0.x ^ v0.y ^ v0.z ^ v0.w ^ v1.x ^ v1.y ^ v1.z ^ v1.w;
    h ^= __shfl_xor(h, 1, 64);
    acc += h;
    b = mix(h + d) % nb;
  }
  if (sub == 0) out[c] = acc;
}

__device__ __forceinline__ void store_tile(uint4* out, uint64_t n, uint64_t base, const uint4* src) {
  const uint32_t lane = threadIdx.x & 63;
  uint4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++) v[u] = src[(base + u * 64 + lane) & 63];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint64_t i = base + u * 64 + lane;
    if (i < n) {
      u32x4 x = {v[u].x, v[u].y, v[u].z, v[u].w};
      __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(out + i));
    }
  }
}

__global__ __launch_bounds__(256) void k_probe(const uint4* tab, uint32_t nb, uint32_t nchains, uint32_t salt, uint32_t* out) {
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
  for (uint32_t c0 = wave * kChainsPerWave; c0 < nchains; c0 += nw * kChainsPerWave)
    probe_chunk(tab, nb, c0, nchains, salt, out);
}

__global__ __launch_bounds__(256) void k_store(uint4* out, uint64_t n, const uint4* src) {
  const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * (uint64_t)blockDim.x) >> 6;
  for (uint64_t base = wave * kTile; base < n; base += nw * kTile) store_tile(out, n, base, src);
}

// tickets: P probe chunks and S store tiles, dealt so that ticket t is a probe
// chunk iff floor((t+1) P / (P+S)) > floor(t P / (P+S))
__global__ __launch_bounds__(256) void k_mixed(const uint4* tab, uint32_t nb, uint32_t nchains, uint32_t salt, uint32_t* pout,
                                               uint4* out, uint64_t n, const uint4* src) {
  const uint64_t P = (nchains + kChainsPerWave - 1) / kChainsPerWave, S = (n + kTile - 1) / kTile, T = P + S;
  const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * (uint64_t)blockDim.x) >> 6;
  for (uint64_t t = wave; t < T; t += nw) {
    const uint64_t pa = (uint64_t)t * P / T, pb = (uint64_t)(t + 1) * P / T;
    if (pb > pa) probe_chunk(tab, nb, (uint32_t)pa * kChainsPerWave, nchains, salt, pout);
    else store_tile(out, n, (t - pa) * kTile, src);
  }
}

int main() {
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t n = 67947762;   // config C's records per 2^20 publishes
  const uint32_t nchains = 1u << 20;
  const uint64_t tbytes = 270ull << 20;
  uint4 *out, *src, *tab;
  uint32_t* pout;
  CK(hipMalloc(&out, n * 16 + 4096));
  CK(hipMalloc(&src, 64 * 16));
  CK(hipMemset(src, 1, 64 * 16));
  CK(hipMalloc(&tab, tbytes));
  CK(hipMalloc(&pout, 4ull * nchains));
  {
    uint32_t* h = (uint32_t*)malloc(tbytes);
    uint64_t s = 0x1234567;
    for (uint64_t i = 0; i < tbytes / 4; i++) { s = s * 6364136223846793005ull + 1442695040888963407ull; h[i] = (uint32_t)(s >> 33); }
    CK(hipMemcpy(tab, h, tbytes, hipMemcpyHostToDevice));
    free(h);
  }
  const uint32_t nb = (uint32_t)(tbytes / 64);
  hipEvent_t ev[4];
  for (auto& x : ev) CK(hipEventCreate(&x));
  for (int bpc : {4, 8, 16}) {
    const int blocks = bpc * cus, reps = 10;
    double tp = 0, ts = 0, tm = 0;
    for (int r = 0; r < reps + 2; r++) {
      CK(hipEventRecord(ev[0]));
      k_probe<<<blocks, 256>>>(tab, nb, nchains, 11u * r + 3u, pout);
      CK(hipEventRecord(ev[1]));
      k_store<<<blocks, 256>>>(out, n, src);
      CK(hipEventRecord(ev[2]));
      k_mixed<<<blocks, 256>>>(tab, nb, nchains, 11u * r + 5u, pout, out, n, src);
      CK(hipEventRecord(ev[3]));
      CK(hipEventSynchronize(ev[3]));
      float a, b, c;
      CK(hipEventElapsedTime(&a, ev[0], ev[1]));
      CK(hipEventElapsedTime(&b, ev[1], ev[2]));
      CK(hipEventElapsedTime(&c, ev[2], ev[3]));
      if (r >= 2) { tp += a; ts += b; tm += c; }
    }
    tp *= 1e3 / reps; ts *= 1e3 / reps; tm *= 1e3 / reps;
    printf("{\"blocks_per_cu\": %d, \"probe_us\": %.1f, \"store_us\": %.1f, \"sum_us\": %.1f, \"mixed_us\": %.1f, "
           "\"mixed_over_sum\": %.3f}\n", bpc, tp, ts, tp + ts, tm, tm / (tp + ts));
    fflush(stdout);
  }
  // the same two kernels on two streams (concurrent dispatch from two HW
  // queues), grids of pb / sb blocks per CU: the probe work split in slices,
  // each slice's probe launched after the previous slice's store on the other
  // stream, as a COUNT(i+1) || EMIT(i) pipeline would
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  hipEvent_t e0, e1, ea, eb;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventCreateWithFlags(&ea, hipEventDisableTiming)); CK(hipEventCreateWithFlags(&eb, hipEventDisableTiming));
  const int pairs[][2] = {{2, 2}, {4, 4}, {2, 4}, {4, 8}, {1, 3}};
  for (auto& pr : pairs) {
    const int reps = 10;
    double tt = 0;
    for (int r = 0; r < reps + 2; r++) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, sa));
      k_probe<<<pr[0] * cus, 256, 0, sa>>>(tab, nb, nchains, 13u * r + 1u, pout);
      k_store<<<pr[1] * cus, 256, 0, sb>>>(out, n, src);
      CK(hipEventRecord(eb, sb));
      CK(hipStreamWaitEvent(sa, eb, 0));
      CK(hipEventRecord(e1, sa));
      CK(hipEventSynchronize(e1));
      float a;
      CK(hipEventElapsedTime(&a, e0, e1));
      if (r >= 2) tt += a;
    }
    tt *= 1e3 / reps;
    printf("{\"two_streams\": true, \"probe_blocks_per_cu\": %d, \"store_blocks_per_cu\": %d, \"both_us\": %.1f}\n",
           pr[0], pr[1], tt);
    fflush(stdout);
  }
  CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1)); CK(hipEventDestroy(ea)); CK(hipEventDestroy(eb));
  CK(hipStreamDestroy(sa)); CK(hipStreamDestroy(sb));
  for (auto& x : ev) CK(hipEventDestroy(x));
  CK(hipFree(out)); CK(hipFree(src)); CK(hipFree(tab)); CK(hipFree(pout));
  return 0;
}
