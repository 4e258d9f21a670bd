// ACL checker of libvmqgpu (include/vmqa.h): the six tables of
// apps/vmq_acl/src/vmq_acl.erl as a device image, rebuilt and uploaded on
// every vmqa_load (ACL reloads are rare; checks are per publish).
//
// Device arena (one allocation, regions 256-B aligned):
//   rules  : ARule {nwords, words_off} per table row
//   rwords : u32 pool of the rows' topic words
//   lists  : u32 row ids: all-read, all-write, pattern-read, pattern-write,
//            then one list per {user, type}
//   fixed  : the all / pattern rules of both types packed for LDS staging:
//            per rule {nwords, word index into `fixed`}, then their words
//   heads  : 4 x AList {off, count} (rule indexes into `fixed`) for the
//            all-read, all-write, pattern-read, pattern-write lists
//   users  : open-addressed {user, type} -> AList (16-B slots), for
//            check_user_acl's ets:match on {{User, '$1'}, '_'} (:194-197)
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/vmqa.h"
#include "vmqg_chain.h"
#include "vmqg_common.h"

namespace vmqa {

struct alignas(8) ARule { uint32_t nwords, words_off; };
struct alignas(8) AList { uint32_t off, count; };
struct alignas(16) USlot { uint32_t user, type, off, count; };   // user == kEmpty: free
static_assert(sizeof(ARule) == 8 && sizeof(AList) == 8 && sizeof(USlot) == 16, "");

VMQG_HD uint64_t user_hash(uint32_t user, uint32_t type) {
  return vmqg::mix64(((uint64_t)user << 2) | type);
}

// Launch interface (vmqa_kernels.hip).
struct AArgs {
  const ARule* rules; const uint32_t* rwords; const uint32_t* lists;
  const AList* heads;                  // [0] all-read [1] all-write [2] pattern-read [3] pattern-write
  const uint32_t* fixed; uint32_t fixed_words, pad1;   // the lists heads[] index (see above)
  const USlot* users; uint64_t users_mask;
  const vmqa_req* reqs; const uint32_t* words; uint32_t n, pad0;
  uint8_t* out;
  uint32_t* status;                    // [1] error bits
};
constexpr uint32_t kFixedLdsWords = 12288;   // 48 KiB: the fixed lists are staged in LDS up to this size
hipError_t launch_acl_check(const AArgs& a, hipStream_t st, hipEvent_t e0, hipEvent_t e1);

struct AclEngine {
  vmqa_config cfg{};
  bool has_device = false;
  int device = -1;
  std::unordered_map<std::string, uint32_t> word_index;
  std::vector<std::string> word_text;
  // the image (host copy) and its layout
  std::vector<uint8_t> image;
  uint64_t rules_off = 0, rwords_off = 0, lists_off = 0, heads_off = 0, users_off = 0, users_slots = 0;
  uint64_t fixed_off = 0, fixed_words = 0;
  uint64_t n_rules = 0, n_users = 0, loads = 0;
  // device
  hipStream_t stream = nullptr;
  hipEvent_t ev_done = nullptr;        // uploads and checks chain across streams (vmqg_chain.h)
  hipStream_t chk_stream = vmqg::no_stream();
  uint8_t* d_arena = nullptr; uint64_t d_arena_bytes = 0;
  uint32_t* d_status = nullptr;
  void* d_r = nullptr; uint64_t d_r_cap = 0;   // host-buffer staging
  void* d_w = nullptr; uint64_t d_w_cap = 0;
  void* d_o = nullptr; uint64_t d_o_cap = 0;
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> t_check;
  double sum_ns = 0; uint64_t n_timed = 0;

  ~AclEngine();
  int init(const vmqa_config& c);
  uint32_t intern(const uint8_t* b, size_t n, bool create);
  int load(const vmqa_rule* rules, size_t n, const uint32_t* words, size_t nwords);
  int check_device(const vmqa_req* d_reqs, uint32_t n, const uint32_t* d_words, uint8_t* d_out, hipStream_t st);
  int check_status(hipStream_t st);
  void collect_times();

 private:
  int upload();
};

}  // namespace vmqa
