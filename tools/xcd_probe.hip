// xcd_probe: which XCD (XCC) and CU each workgroup of a launch runs on, from
// the hardware registers HW_REG_XCC_ID / HW_REG_HW_ID read by its first
// lane.  Checks the dispatch assumption behind any XCD-aware blockIdx
// mapping (workgroup i on XCD i mod 8); round 3's "XCD label" tail variant
// relied on it.  Prints one JSON line: blocks per XCD, how many blocks sit
// on XCD blockIdx % 8, and the first 32 (block, xcc, se, cu) tuples.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/bin/xcd_probe tools/xcd_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_probe(uint32_t* out, uint32_t spin) {
  if (threadIdx.x == 0) {
    uint32_t xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
  // keep the block resident a little, so later blocks are placed by the
  // dispatcher while earlier ones still run (a steady-state grid)
  for (uint32_t i = 0; i < spin; i++) __builtin_amdgcn_s_sleep(1);
}

int main(int argc, char** argv) {
  const uint32_t blocks = argc > 1 ? (uint32_t)atoi(argv[1]) : 2048;
  const uint32_t threads = argc > 2 ? (uint32_t)atoi(argv[2]) : 256;
  uint32_t* d = nullptr;
  if (hipMalloc(&d, blocks * 8) != hipSuccess) return 1;
  (void)hipMemset(d, 0xff, blocks * 8);
  k_probe<<<blocks, threads>>>(d, 200);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::vector<uint32_t> h(2 * blocks);
  (void)hipMemcpy(h.data(), d, blocks * 8, hipMemcpyDeviceToHost);
  uint32_t per[16] = {0}, match = 0;
  for (uint32_t b = 0; b < blocks; b++) {
    const uint32_t x = h[2 * b] & 0xF;
    per[x]++;
    match += x == b % 8;
  }
  printf("{\"blocks\": %u, \"threads\": %u, \"per_xcc\": [", blocks, threads);
  for (int i = 0; i < 8; i++) printf("%s%u", i ? ", " : "", per[i]);
  printf("], \"xcc_is_block_mod_8\": %u, \"first\": [", match);
  for (uint32_t b = 0; b < 32 && b < blocks; b++) {
    const uint32_t hw = h[2 * b + 1];
    printf("%s[%u, %u, %u, %u]", b ? ", " : "", b, h[2 * b] & 0xF, (hw >> 13) & 7, (hw >> 8) & 0xF);
  }
  printf("]}\n");
  (void)hipFree(d);
  return 0;
}
