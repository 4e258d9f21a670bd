// Cost of the global atomics and hint loads a batch-wide table needs, on one
// MI355X (tools/Makefile -> tools/bin/atomic_probe; prints JSON lines):
//   counter      every wave of a 2^20-lane grid adds 1 to ONE word (agent scope)
//   counter64    ... to one of 64 words 64 B apart (wave id % 64)
//   cas_random   every lane CASes a random slot of a 2^21-slot table (8 B)
//   cas_hot16    every lane CASes one of 16 slots (a hot-topic batch)
//   aload_hot16  every lane atomic-loads (relaxed, agent) one of 16 slots
//   load_hot16   every lane plain-loads one of 16 slots
//   store_hot16  every lane plain-stores to one of 16 slots (last writer wins)
//   store_random every lane plain-stores to a random slot of the table
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x;
}

template <int KIND>
__global__ __launch_bounds__(256) void k_probe(unsigned long long* tbl, unsigned long long* ctr, uint64_t mask, uint32_t salt,
                                               unsigned long long* sink) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t h = mix(t * 0x9E3779B97F4A7C15ull + salt);
  unsigned long long acc = 0;
  if (KIND == 0) {
    if ((threadIdx.x & 63) == 0) atomicAdd(ctr, 1ull);
  } else if (KIND == 1) {
    if ((threadIdx.x & 63) == 0) atomicAdd(ctr + ((t >> 6) % 64) * 8, 1ull);
  } else if (KIND == 2) {
    acc = atomicCAS(tbl + (h & mask), 0ull, (unsigned long long)h | 1);
  } else if (KIND == 3) {
    acc = atomicCAS(tbl + (h & 15) * 8, 0ull, (unsigned long long)salt | 1);
  } else if (KIND == 4) {
    acc = __hip_atomic_load(tbl + (h & 15) * 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (KIND == 5) {
    acc = tbl[(h & 15) * 8];
  } else if (KIND == 6) {
    tbl[(h & 15) * 8] = (unsigned long long)t;
  } else if (KIND == 7) {
    tbl[h & mask] = (unsigned long long)t;
  }
  if (acc == 0x123456789ull) sink[0] = acc;   // keeps the loads
}

template <int KIND>
static float run(unsigned long long* tbl, unsigned long long* ctr, uint64_t mask, unsigned long long* sink, uint32_t n) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  float best = 1e30f;
  for (int rep = 0; rep < 5; rep++) {
    hipMemset(tbl, 0, (mask + 1) * 8);
    hipMemset(ctr, 0, 64 * 64 * 8);
    hipDeviceSynchronize();
    hipEventRecord(a);
    k_probe<KIND><<<n / 256, 256>>>(tbl, ctr, mask, rep * 7919u + 1, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  return best * 1e3f;
}

int main() {
  const uint64_t slots = 1ull << 21;
  const uint32_t n = 1u << 20;
  unsigned long long *tbl, *ctr, *sink;
  hipMalloc(&tbl, slots * 8);
  hipMalloc(&ctr, 64 * 64 * 8);
  hipMalloc(&sink, 64);
  const char* names[] = {"counter", "counter64", "cas_random", "cas_hot16", "aload_hot16", "load_hot16", "store_hot16",
                         "store_random"};
  float us[8];
  us[0] = run<0>(tbl, ctr, slots - 1, sink, n);
  us[1] = run<1>(tbl, ctr, slots - 1, sink, n);
  us[2] = run<2>(tbl, ctr, slots - 1, sink, n);
  us[3] = run<3>(tbl, ctr, slots - 1, sink, n);
  us[4] = run<4>(tbl, ctr, slots - 1, sink, n);
  us[5] = run<5>(tbl, ctr, slots - 1, sink, n);
  us[6] = run<6>(tbl, ctr, slots - 1, sink, n);
  us[7] = run<7>(tbl, ctr, slots - 1, sink, n);
  for (int k = 0; k < 8; k++)
    printf("{\"probe\": \"%s\", \"lanes\": %u, \"waves\": %u, \"us\": %.2f}\n", names[k], n, n / 64, us[k]);
  return 0;
}
