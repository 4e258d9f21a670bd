// Store-bandwidth ceiling for the EMIT pass's output pattern on MI355X:
// 16-B records written wave-contiguously (64 lanes x 16 B = 1 KiB per store
// instruction), U records in flight per lane, 1.1 GB per launch (config C's
// EMIT output), from (a) registers only, (b) a 64-record L2-resident source
// list (EMIT copies one 64-record fan-out list per publish), under each store
// cache policy of gfx950 (plain, nt, sc1, sc0 sc1, sc1 nt), grid-strided or
// with each block owning one contiguous slice.
//
// Second question per variant: what does the 1.1 GB stream do to a 270 MB
// table (config C's arena) that the next pass (COUNT) reads at random?  After
// each store launch a probe launch reads 2^20 random 64-B buckets of the
// table; its time, next to the store's, is the cost the policy puts on COUNT.
// Prints one JSON line per variant.
//
// build: hipcc --offload-arch=gfx950 -O3 -o store_ceiling tools/store_ceiling.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// P: 0 plain, 1 nt (__builtin_nontemporal_store), 2 sc1, 3 sc0 sc1, 4 sc1 nt
template <int P>
__device__ __forceinline__ void store16(uint4* p, uint4 v) {
  u32x4 x = {v.x, v.y, v.z, v.w};
  if (P == 0) *p = v;
  else if (P == 1) __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
  else if (P == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
  else if (P == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(x) : "memory");
  else asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(x) : "memory");
}

// SLICE = false: grid-stride over 64*U-record wave tiles; true: block b owns
// records [b*n/B, (b+1)*n/B), its waves interleaving 64*U-record tiles.
template <int P, bool SRC, int U, bool SLICE>
__global__ __launch_bounds__(256) void k_store(uint4* out, uint64_t n, const uint4* src) {
  const uint64_t lane = threadIdx.x & 63;
  uint64_t lo = 0, hi = n, wave, nwaves;
  if (SLICE) {
    lo = n * blockIdx.x / gridDim.x;
    hi = n * (blockIdx.x + 1) / gridDim.x;
    wave = threadIdx.x >> 6;
    nwaves = blockDim.x >> 6;
  } else {
    wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    nwaves = (gridDim.x * (uint64_t)blockDim.x) >> 6;
  }
  for (uint64_t base = lo + wave * 64 * U; base < hi; base += nwaves * 64 * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t i = base + u * 64 + lane;
      v[u] = SRC ? src[i & 63] : make_uint4((uint32_t)i, (uint32_t)(i >> 32), 7u, 9u);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t i = base + u * 64 + lane;
      if (i < hi) store16<P>(out + i, v[u]);
    }
  }
}

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// 2^20 chains of 3 dependent random 64-B bucket reads (COUNT's shape), 2
// lanes per chain; a different start set every launch (salt).
__global__ __launch_bounds__(256) void k_probe(const uint4* tab, uint32_t nb, uint32_t nchains, uint32_t salt,
                                               uint32_t* out) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t sub = threadIdx.x & 1, grp = tid / 2, ngrp = gridDim.x * blockDim.x / 2;
  for (uint32_t c = grp; c < nchains; c += ngrp) {
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
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

struct Ctx {
  uint4* out; uint64_t n; const uint4* src;
  const uint4* tab; uint32_t nb; uint32_t* pout;
  int cus;
};

template <int P, bool SRC, int U, bool SLICE>
static void run(const char* name, const Ctx& c, int bpc, int reps) {
  const int blocks = bpc * c.cus;
  hipEvent_t ev[3];
  for (auto& x : ev) CK(hipEventCreate(&x));
  for (int w = 0; w < 2; w++) {
    k_store<P, SRC, U, SLICE><<<blocks, 256>>>(c.out, c.n, c.src);
    k_probe<<<8 * c.cus, 256>>>(c.tab, c.nb, 1u << 20, 99u + w, c.pout);
  }
  double st = 0, pr = 0;
  for (int r = 0; r < reps; r++) {
    CK(hipEventRecord(ev[0]));
    k_store<P, SRC, U, SLICE><<<blocks, 256>>>(c.out, c.n, c.src);
    CK(hipEventRecord(ev[1]));
    k_probe<<<8 * c.cus, 256>>>(c.tab, c.nb, 1u << 20, 7u * r + 1u, c.pout);
    CK(hipEventRecord(ev[2]));
    CK(hipEventSynchronize(ev[2]));
    float a = 0, b = 0;
    CK(hipEventElapsedTime(&a, ev[0], ev[1]));
    CK(hipEventElapsedTime(&b, ev[1], ev[2]));
    st += a; pr += b;
  }
  const double us = st * 1e3 / reps, pus = pr * 1e3 / reps;
  printf("{\"variant\": \"%s\", \"blocks_per_cu\": %d, \"bytes\": %llu, \"us_per_launch\": %.1f, \"TBps\": %.3f, "
         "\"probe_after_us\": %.1f}\n",
         name, bpc, (unsigned long long)(c.n * 16), us, c.n * 16.0 / (us * 1e-6) / 1e12, pus);
  fflush(stdout);
  for (auto& x : ev) CK(hipEventDestroy(x));
}

int main() {
  Ctx c;
  c.n = 67947762;   // config C: records per 2^20-publish batch
  uint4* src;
  CK(hipMalloc(&c.out, c.n * 16 + 4096));
  CK(hipMalloc(&src, 64 * 16));
  CK(hipMemset(src, 1, 64 * 16));
  c.src = src;
  const uint64_t tbytes = 270ull << 20;   // config C's arena
  uint4* tab;
  CK(hipMalloc(&tab, tbytes));
  {
    uint32_t* h = (uint32_t*)malloc(tbytes);
    uint64_t s = 0x1234567;
    for (uint64_t i = 0; i < tbytes / 4; i++) { s = s * 6364136223846793005ull + 1442695040888963407ull; h[i] = (uint32_t)(s >> 33); }
    CK(hipMemcpy(tab, h, tbytes, hipMemcpyHostToDevice));
    free(h);
  }
  c.tab = tab;
  c.nb = (uint32_t)(tbytes / 64);
  CK(hipMalloc(&c.pout, 4u << 20));
  c.cus = 256;
  CK(hipDeviceGetAttribute(&c.cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int reps = 10;
  for (int bpc : {8, 16}) {
    run<0, true, 8, false>("plain_l2src_u8", c, bpc, reps);
    run<1, true, 8, false>("nt_l2src_u8", c, bpc, reps);
    run<2, true, 8, false>("sc1_l2src_u8", c, bpc, reps);
    run<3, true, 8, false>("sc0sc1_l2src_u8", c, bpc, reps);
    run<4, true, 8, false>("sc1nt_l2src_u8", c, bpc, reps);
    run<0, false, 8, false>("plain_regs_u8", c, bpc, reps);
    run<2, false, 8, false>("sc1_regs_u8", c, bpc, reps);
    run<0, true, 8, true>("plain_l2src_u8_slice", c, bpc, reps);
    run<1, true, 8, true>("nt_l2src_u8_slice", c, bpc, reps);
    run<2, true, 8, true>("sc1_l2src_u8_slice", c, bpc, reps);
    run<2, true, 16, false>("sc1_l2src_u16", c, bpc, reps);
  }
  CK(hipFree(c.out));
  CK(hipFree(src));
  CK(hipFree(tab));
  CK(hipFree(c.pout));
  return 0;
}
