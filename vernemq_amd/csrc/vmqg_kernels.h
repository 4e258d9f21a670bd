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
  const uint32_t* keylist;                        // key ids of multi-key filters; remote nodes >= 64
  const Record* records;
  const ExactSlot* exact; uint64_t exact_mask;    // bucket mask
  const uint32_t* exwords;
  const uint32_t* exbits; uint64_t exbits_mask;   // exact-topic filter (bits - 1)
  uint32_t max_mp, local_node;
  const vmqg_pub* pubs; const uint32_t* words; uint32_t npub;
  uint32_t exfilter;                              // 1: test the exbits filter before the exact table (auto, see exmode)
  uint64_t* offsets;                              // npub + 1
  void* keycache;                                 // npub x 32 B (COUNT -> EMIT)
  uint64_t* chunk;                                // per chunk of gpw publishes: COUNT's total, then its output base
  uint32_t gpw;                                   // publishes per chunk (64 / fast-tier lanes per publish)
  uint2* keyspill;                                // npub x kSpillKeys {record off, cum start}: 3..8-key publishes
  Record* out; uint64_t out_cap;                  // records mode
  vmqg_range* out_rng; uint64_t rng_cap;          // range mode (out_rng != null)
  uint32_t* status;                               // this call's counters: [0] deferred publishes,
                                                  // [1] of those, walked with a global stack, [2] scan ticket,
                                                  // [3] publishes EMIT hands to the wave tier (none today)
  uint32_t* status_next;                          // the next call's counters (zeroed by this call)
  uint32_t* err;                                  // error bits, sticky until vmqg_match_status
  uint32_t* deferred;                             // kLists x npub: retry, whole-wave walks, duplicates + slots
  uint32_t fast_g, opts;                          // tuning: lanes per publish (2|4), kOpt* bits
  uint32_t count_bpc, emit_bpc;                   // tuning: fast-tier grid cap in blocks per CU (0 = 8)
  uint32_t cus, pad2;                             // compute units of the device
  uint64_t* lookback;                             // per scan tile: {tag, flag, value} granule
  uint32_t lb_tag, pad1;                          // this call's granule tag (never 0)
  uint2* o_stack;                                 // wave tier: global frontier stacks, o_cap entries per wave
  uint32_t o_cap, o_waves;
  uint32_t* dbg;                                  // VMQG_DEBUG_SYNC only: per-wave progress words in host memory
  uint32_t* o_slots;                              // o_waves bits: stacks borrowed by the EMIT tail's walks
  uint64_t* widemask;                             // per chunk of gpw publishes: its wide publishes (COUNT -> EMIT tail)
  // batch-wide dedupe (COUNT -> the COUNT wave tier's fixup)
  uint64_t* dd_key;                               // dd_mask + 1 slots: {call tag: 24, fingerprint bits: 40}
  uint32_t* dd_rep;                               // ... the publish that claimed the slot
  uint64_t dd_mask;
  uint32_t dd_tag, dd_force;                      // this call's tag (never 0); 0 off, 1 on, 2 auto (dd_mode)
  uint32_t* dd_mode;                              // persistent: the mode the last call's fixup chose
  uint32_t* fastdone;                             // bit per publish: served by COUNT's fast pass
  void* groups; uint64_t gs_mask;                 // output groups (records mode): 256-B slots, tagged by dd_tag
  uint64_t* ddmask;                               // per chunk: its duplicates (COUNT -> the fix-up)
  uint32_t dd_claimed, dd_g;                      // dedupe on this call; lanes per representative in COUNT (1|2|4)
  uint8_t* heavybyte;                             // per publish: 1 + its first key's bucket if heavy, else 0
  uint32_t heavy_min;                             // records mode: heavy publishes have >= this many records (0 off)
  uint32_t trieless;                              // the device tables have no trie edge: only exact topics match
  uint32_t* dd_host;                              // host-mapped words: [0] the dedupe mode, [1] the exbits-filter
                                                  // mode for the next calls (k_ex_sample)
};

constexpr uint32_t kOptNtStores = 1u;   // non-temporal stores for the emitted records
constexpr uint32_t kOptRootFlags = 2u;  // a walk starts from its root's cached child flags (else probes all three)

// mode 0 = COUNT, 1 = EMIT; tier 0 = fast groups, 1 = wave tier (grid a.o_waves / 4).
// t0 / t1 (both or neither): timing events recorded by the kernel's own
// dispatch (hipExtLaunchKernel), not by marker packets between launches.
hipError_t launch_match(const MatchArgs& a, int mode, int tier, hipStream_t st, hipEvent_t t0 = nullptr,
                        hipEvent_t t1 = nullptr);
// counts in offsets[0, npub) -> exclusive offsets[0, npub] (one launch, look-back)
hipError_t launch_scan(const MatchArgs& a, hipStream_t st, hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
uint32_t scan_tiles(uint64_t nchunks);   // look-back tiles of the chunk-total scan
hipError_t launch_patches(uint8_t* arena, const void* d_patches, uint64_t n, hipStream_t st);
// batch dedupe, mode on: every publish stores {tag | fingerprint, publish}
// into its table slot (plain stores, the last writer wins) before COUNT
hipError_t launch_dd_claim(const MatchArgs& a, hipStream_t st, hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
// ... then sorts the publishes into representatives (list 2, COUNT walks
// them) and duplicates (chunk masks; their representative at list 3)
hipError_t launch_dd_classify(const MatchArgs& a, hipStream_t st, hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
// after COUNT: duplicates take their representative's results, or join list 0
hipError_t launch_dd_fixup(const MatchArgs& a, hipStream_t st, hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
// exact-filter auto mode: samples 4,096 publishes' filter bits, the last
// block writes the next calls' filter mode to dd_host[1]
hipError_t launch_ex_sample(const MatchArgs& a, hipStream_t st);
// trie-less tables: COUNT, scan and EMIT (records or ranges) in one launch,
// tiles chained by look-back (a.lookback >= exact_fused_tiles granules);
// huge records-mode publishes are left to the EMIT tail
hipError_t launch_exact_fused(const MatchArgs& a, hipStream_t st, hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
uint32_t exact_fused_tiles(uint64_t npub);

}  // namespace vmqg
