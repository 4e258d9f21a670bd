// Launch interface between the host engine and the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/vmqg.h"
#include "vmqg_common.h"

namespace vmqg {

struct MatchArgs {
  const EdgeSlot* edges; uint64_t edge_mask;      // bucket mask
  const NodeRec* nodes; uint64_t node_cap;
  const KeyDesc* keydesc; uint64_t key_cap;
  const uint32_t* keylist;
  const Record* records;
  const ExactSlot* exact; uint64_t exact_mask;    // bucket mask
  const uint32_t* exwords;
  uint32_t max_mp, local_node;
  const vmqg_pub* pubs; const uint32_t* words; uint32_t npub, pad0;
  uint64_t* offsets;                              // npub + 1
  void* keycache;                                 // npub x 32 B (COUNT -> EMIT)
  Record* out; uint64_t out_cap;
  uint32_t* status;                               // [0] tier-1 list count, [1] error bits,
                                                  // [2] tier-1 publishes that needed global scratch,
                                                  // [3] next tile / chunk ticket (scan, fused kernel)
  uint32_t* deferred; uint32_t deferred_cap, pad1;
  uint32_t fast_g, opts;                          // tuning: lanes per publish (4|8), kOpt* bits
  // decoupled look-back (scan tiles, fused chunks)
  uint64_t* lookback;                             // per tile / chunk: {tag, flag, value} granule
  uint32_t lb_tag, nchunks;                       // this call's granule tag (never 0); fused chunks
  uint2* o_stack; uint32_t* o_cand; uint2* o_keys;  // global scratch of the wave path, o_cap entries per wave
  uint32_t o_cap, o_waves;
};

constexpr uint32_t kOptNtStores = 1u;   // non-temporal stores for the emitted records

// mode 0 = COUNT, 1 = EMIT; tier 0 = fast groups, 1 = wave path (grid a.o_waves / 4)
hipError_t launch_match(const MatchArgs& a, int mode, int tier, hipStream_t st);
// counts in offsets[0, npub) -> exclusive offsets[0, npub] (one launch, look-back)
hipError_t launch_scan(const MatchArgs& a, hipStream_t st);
uint32_t scan_tiles(uint64_t npub);
int wave_blocks_per_cu();
// One-pass match: walk + count + chunk offsets (decoupled look-back) + emit.
// `grid` blocks (<= a.o_waves / 4); publishes per chunk = fused_chunk(a.fast_g).
hipError_t launch_fused(const MatchArgs& a, uint32_t grid, uint32_t unroll, hipStream_t st);
uint32_t fused_chunk(uint32_t fast_g);
// resident blocks of the fused kernel per CU (occupancy query)
int fused_blocks_per_cu(uint32_t fast_g, uint32_t unroll);
hipError_t launch_patches(uint8_t* arena, const void* d_patches, uint64_t n, hipStream_t st);

}  // namespace vmqg
