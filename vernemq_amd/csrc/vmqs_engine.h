// Shared-subscription dispatcher of libvmqgpu (include/vmqs.h): what
// vmq_shared_subscriptions:publish/3 does with the $share members a fold
// collected, run on the match batch's emission records in HBM.
//
// Device state: one byte of queue state per SubscriberId id (grown on
// demand; new ids read VMQS_ONLINE), a status block and the tier-2 list.
//
// Kernels (vmqs_kernels.hip), both integer-only and bound by reading the
// 16-B records once and writing one byte per record:
//   k_select_wave  one wavefront per publish, its groups in a 64-slot LDS
//                  table; segments over kWaveMax records or with more than
//                  kWaveGroups distinct groups go to
//   k_select_block one 256-thread workgroup per deferred publish, a
//                  kBlockGroups-slot LDS table (more groups: VMQG_E_LIMIT).
#pragma once
#include <hip/hip_runtime.h>

#include <utility>
#include <vector>

#include "../../include/vmqs.h"
#include "vmqg_chain.h"
#include "vmqg_common.h"

namespace vmqs {

constexpr uint32_t kWaveGroups = 64;      // LDS group slots per wave (tier 1)
constexpr uint32_t kWaveMax = 4096;       // records per publish in tier 1
constexpr uint32_t kBlockGroups = 2048;   // LDS group slots per workgroup (tier 2)
constexpr uint32_t kBlockGrid = 512;      // tier-2 workgroups (they loop over the deferred list)
constexpr uint32_t kErrLimit = 1u;        // status[1]: a publish exceeded the tier-2 table / VMQS_MAX_SEGMENT

// The element key of vmqs.h: 40 random bits over the position.
VMQG_HD uint64_t sel_key(uint64_t seed, uint64_t q, uint32_t p) {
  const uint64_t h = vmqg::mix64(vmqg::mix64(seed ^ (q * 0x9E3779B97F4A7C15ull)) + (uint64_t)p * 0xD1B54A32D192ED03ull);
  return (h & ~0xFFFFFFull) | (p & 0xFFFFFFu);
}

// Launch interface.
struct SArgs {
  const vmqg::Record* emits; const uint64_t* offsets;
  uint32_t npub, policy, local_node, n_states;
  uint64_t seed, pub_seq;
  const uint8_t* states;
  uint8_t* chosen; uint32_t* failed;
  uint32_t* defer;     // tier-2 publish list
  uint32_t* status;    // [0] tier-2 count (per call) [1] error bits (latched)
};
hipError_t launch_select(const SArgs& a, hipStream_t st, hipEvent_t e0, hipEvent_t e1);

struct SelEngine {
  vmqs_config cfg{};
  int device = -1;
  hipStream_t stream = nullptr;
  uint8_t* d_states = nullptr; uint64_t n_states = 0, states_cap = 0;
  std::vector<uint8_t> h_states;   // host copy of the state table
  uint32_t* d_status = nullptr;
  hipEvent_t ev_sel = nullptr;     // state-table updates and selects chain across streams (vmqg_chain.h)
  hipStream_t sel_stream = vmqg::no_stream();
  uint32_t* d_defer = nullptr; uint64_t defer_cap = 0;
  void* d_e = nullptr; uint64_t d_e_cap = 0;   // host-buffer staging
  void* d_o = nullptr; uint64_t d_o_cap = 0;
  void* d_c = nullptr; uint64_t d_c_cap = 0;
  void* d_f = nullptr; uint64_t d_f_cap = 0;
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> t_sel;
  double sum_ns = 0; uint64_t n_timed = 0, last_deferred = 0;

  ~SelEngine();
  int init(const vmqs_config& c);
  int set_states(const uint32_t* subs, const uint8_t* states, size_t n);
  int select_device(const vmqg_emit* d_emits, const uint64_t* d_offsets, uint32_t npub, uint32_t policy,
                    uint64_t seed, uint64_t pub_seq, uint8_t* d_chosen, uint32_t* d_failed, hipStream_t st);
  int select_status(hipStream_t st);
  void collect_times();
};

}  // namespace vmqs
