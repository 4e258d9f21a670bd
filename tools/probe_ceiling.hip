// Random-probe ceiling for the COUNT pass's access pattern on MI355X:
// 2^20 chains (one per publish) of D dependent 64-B bucket reads from a
// table of T bytes (config C's arena 270 MB, config D's 2.35 GB), a group of
// G lanes per chain reading the bucket together (16 B per lane for G = 4,
// 32 B for G = 2), C chains interleaved per group (C publishes per group in
// flight).  The next bucket index is a hash of the bucket's contents, so the
// reads are truly dependent.  Prints one JSON line per variant: the time, the
// buckets per second and the 64-B lines' bandwidth.
//
// build: hipcc --offload-arch=gfx950 -O3 -o probe_ceiling tools/probe_ceiling.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

template <int G, int C, int D>
__global__ __launch_bounds__(256) void k_probe(const uint4* tab, uint32_t nb, uint32_t nchains, uint32_t* out) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t sub = threadIdx.x & (G - 1);
  const uint32_t grp = tid / G, ngrp = gridDim.x * blockDim.x / G;
  for (uint32_t c0 = grp * C; c0 < nchains; c0 += ngrp * C) {
    uint32_t b[C], acc[C];
#pragma unroll
    for (int c = 0; c < C; c++) { b[c] = mix(c0 + c) % nb; acc[c] = 0; }
#pragma unroll
    for (int d = 0; d < D; d++) {
      uint4 v[C][4 / G];
#pragma unroll
      for (int c = 0; c < C; c++)
#pragma unroll
        for (int k = 0; k < 4 / G; k++) v[c][k] = tab[(uint64_t)b[c] * 4 + sub * (4 / G) + k];
#pragma unroll
      for (int c = 0; c < C; c++) {
        uint32_t h = 0;
#pragma unroll
        for (int k = 0; k < 4 / G; k++) h ^= v[c][k].x ^ v[c][k].y ^ v[c][k].z ^ v[c][k].w;
        // every lane of the group needs the same next bucket: combine the group's parts
#pragma unroll
        for (int s = 1; s < G; s <<= 1) h ^= __shfl_xor(h, s, 64);
        acc[c] += h;
        b[c] = mix(h + d) % nb;
      }
    }
#pragma unroll
    for (int c = 0; c < C; c++)
      if (sub == 0 && c0 + c < nchains) out[c0 + c] = acc[c];
  }
}

// Probes of 64-B buckets on 128-B lines, each followed (F = 1) by a dependent
// 16-B read of the line's other half (an edge slot's side payload): is the
// follow-up an L2 hit or a second random access?
template <int G, int F, int D>
__global__ __launch_bounds__(256) void k_probe_line(const uint4* tab, uint32_t nl, uint32_t nchains, uint32_t* out) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t sub = threadIdx.x & (G - 1);
  const uint32_t grp = tid / G, ngrp = gridDim.x * blockDim.x / G;
  for (uint32_t c = grp; c < nchains; c += ngrp) {
    uint32_t b = mix(c) % nl, acc = 0;
#pragma unroll
    for (int d = 0; d < D; d++) {
      uint4 v[4 / G];
#pragma unroll
      for (int k = 0; k < 4 / G; k++) v[k] = tab[(uint64_t)b * 8 + sub * (4 / G) + k];
      uint32_t h = 0;
#pragma unroll
      for (int k = 0; k < 4 / G; k++) h ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
#pragma unroll
      for (int s = 1; s < G; s <<= 1) h ^= __shfl_xor(h, s, 64);
      if (F) {
        const uint4 q = tab[(uint64_t)b * 8 + 4 + (h & 3)];
        h += q.x ^ q.w;
      }
      acc += h;
      b = mix(h + d) % nl;
    }
    if (sub == 0) out[c] = acc;
  }
}

template <int G, int F, int D>
static void run_line(const char* table, const uint4* tab, uint32_t nl, uint32_t nchains, uint32_t* out, int bpc, int cus) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int blocks = bpc * cus, reps = 20;
  for (int w = 0; w < 3; w++) k_probe_line<G, F, D><<<blocks, 256>>>(tab, nl, nchains, out);
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; r++) k_probe_line<G, F, D><<<blocks, 256>>>(tab, nl, nchains, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / reps, probes = (double)nchains * D;
  printf("{\"table\": \"%s\", \"kind\": \"64B of a 128B line%s\", \"G\": %d, \"depth\": %d, \"blocks_per_cu\": %d, "
         "\"us_per_launch\": %.1f, \"Gprobes_per_s\": %.2f}\n",
         table, F ? " + dependent 16B of its other half" : "", G, D, bpc, us, probes / (us * 1e-6) / 1e9);
  fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}


template <int G, int C, int D>
static void run(const char* table, const uint4* tab, uint32_t nb, uint32_t nchains, uint32_t* out, int bpc, int cus) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int blocks = bpc * cus, reps = 20;
  for (int w = 0; w < 3; w++) k_probe<G, C, D><<<blocks, 256>>>(tab, nb, nchains, out);
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; r++) k_probe<G, C, D><<<blocks, 256>>>(tab, nb, nchains, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / reps, probes = (double)nchains * D;
  printf("{\"table\": \"%s\", \"G\": %d, \"chains_per_group\": %d, \"depth\": %d, \"blocks_per_cu\": %d, "
         "\"us_per_launch\": %.1f, \"Gprobes_per_s\": %.2f, \"TBps_64B\": %.3f}\n",
         table, G, C, D, bpc, us, probes / (us * 1e-6) / 1e9, probes * 64 / (us * 1e-6) / 1e12);
  fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main() {
  const uint32_t nchains = 1u << 20;
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t* out;
  CK(hipMalloc(&out, 4ull * nchains * sizeof(uint32_t)));   // the independent-probe variant runs 4x the chains
  struct { const char* name; uint64_t bytes; } tables[2] = {{"270MB", 270ull << 20}, {"2350MB", 2350ull << 20}};
  for (auto& t : tables) {
    uint4* tab;
    CK(hipMalloc(&tab, t.bytes));
    uint32_t* h = (uint32_t*)malloc(t.bytes);
    uint64_t s = 0x1234567;
    for (uint64_t i = 0; i < t.bytes / 4; i++) { s = s * 6364136223846793005ull + 1442695040888963407ull; h[i] = (uint32_t)(s >> 33); }
    CK(hipMemcpy(tab, h, t.bytes, hipMemcpyHostToDevice));
    free(h);
    const uint32_t nb = (uint32_t)(t.bytes / 64);
    for (int bpc : {4, 8}) {
      run<2, 1, 4>(t.name, tab, nb, nchains, out, bpc, cus);
      run<2, 2, 4>(t.name, tab, nb, nchains, out, bpc, cus);
      run<4, 1, 4>(t.name, tab, nb, nchains, out, bpc, cus);
      run<4, 2, 4>(t.name, tab, nb, nchains, out, bpc, cus);
      run<1, 1, 4>(t.name, tab, nb, nchains, out, bpc, cus);
      run<2, 1, 1>(t.name, tab, nb, nchains * 4, out, bpc, cus);   // independent probes, same count
      const uint32_t nl = (uint32_t)(t.bytes / 128);
      run_line<2, 0, 4>(t.name, tab, nl, nchains, out, bpc, cus);
      run_line<2, 1, 4>(t.name, tab, nl, nchains, out, bpc, cus);
      run_line<2, 0, 8>(t.name, tab, nl, nchains, out, bpc, cus);
    }
    CK(hipFree(tab));
  }
  CK(hipFree(out));
  return 0;
}
