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
  uint32_t* status;                               // [0] tier-1 list count, [1] error bits, [2] tier-2 count
  uint32_t* deferred; uint32_t deferred_cap, g_waves;
  uint32_t* deferred2;
  uint2* g_stack; uint32_t* g_cand; uint2* g_keys;  // slow-path scratch, per wave
  uint32_t g_scap, g_ccap, g_kcap, pad1;
  uint32_t fast_g, opts;                          // tuning: lanes per publish (4|8), kOpt* bits
};

constexpr uint32_t kOptNtStores = 1u;   // non-temporal stores for the emitted records

hipError_t launch_match(const MatchArgs& a, int mode, int tier, hipStream_t st);
hipError_t launch_scan(uint64_t* v, uint64_t n, uint64_t* tmp, hipStream_t st);
uint64_t scan_tmp_elems(uint64_t n);
hipError_t launch_patches(uint8_t* arena, const void* d_patches, uint64_t n, hipStream_t st);

}  // namespace vmqg
