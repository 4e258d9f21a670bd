// Store-bandwidth ceiling for the EMIT pass's output pattern on MI355X:
// 16-B records written wave-contiguously (64 lanes x 16 B = 1 KiB per store
// instruction), U records in flight per lane, 1.1 GB per launch (config C's
// EMIT output), from (a) registers only, (b) a 64-record L2-resident source
// list (EMIT copies one 64-record fan-out list per publish), with plain and
// non-temporal stores.  Prints one JSON line per variant.
//
// build: hipcc --offload-arch=gfx950 -O3 -o store_ceiling tools/store_ceiling.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT, bool SRC, int U>
__global__ __launch_bounds__(256) void k_store(uint4* out, uint64_t n, const uint4* src) {
  const uint64_t lane = threadIdx.x & 63;
  const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = (gridDim.x * (uint64_t)blockDim.x) >> 6;
  for (uint64_t base = wave * 64 * U; base < n; base += nwaves * 64 * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t i = base + u * 64 + lane;
      v[u] = SRC ? src[i & 63] : make_uint4((uint32_t)i, (uint32_t)(i >> 32), 7u, 9u);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t i = base + u * 64 + lane;
      if (i < n) {
        if (NT) {
          u32x4 x = {v[u].x, v[u].y, v[u].z, v[u].w};
          __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(out + i));
        } else {
          out[i] = v[u];
        }
      }
    }
  }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <bool NT, bool SRC, int U>
static void run(const char* name, uint4* out, uint64_t n, const uint4* src, int blocks, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; w++) k_store<NT, SRC, U><<<blocks, 256>>>(out, n, src);
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; r++) k_store<NT, SRC, U><<<blocks, 256>>>(out, n, src);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / reps;
  printf("{\"variant\": \"%s\", \"blocks\": %d, \"bytes\": %llu, \"us_per_launch\": %.1f, \"TBps\": %.3f}\n", name, blocks,
         (unsigned long long)(n * 16), us, n * 16.0 / (us * 1e-6) / 1e12);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main() {
  const uint64_t n = 67947762;   // config C: records per 2^20-publish batch
  uint4 *out, *src;
  CK(hipMalloc(&out, n * 16 + 4096));
  CK(hipMalloc(&src, 64 * 16));
  CK(hipMemset(src, 1, 64 * 16));
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int reps = 20;
  for (int bpc : {4, 8, 16}) {
    const int blocks = bpc * cus;
    run<true, false, 8>("nt_regs_u8", out, n, src, blocks, reps);
    run<false, false, 8>("plain_regs_u8", out, n, src, blocks, reps);
    run<true, true, 8>("nt_l2src_u8", out, n, src, blocks, reps);
    run<true, false, 4>("nt_regs_u4", out, n, src, blocks, reps);
  }
  CK(hipFree(out));
  CK(hipFree(src));
  return 0;
}
