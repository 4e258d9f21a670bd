// Retained-message store of libvmqgpu (include/vmqr.h): host engine with the
// semantics of vmq_retain_srv's ets set (apps/vmq_server/src/vmq_retain_srv.erl)
// plus a byte-exact host mirror of the device arena the match kernels read
// (vmqr_kernels.hip).  Same delta discipline as the subscription engine:
// every mutation marks 16-B chunks dirty and an apply ships them as patches;
// growth re-lays the arena out and ships the whole image.
//
// Device arena (one allocation, regions 256-B aligned):
//   rows   : RRow per retained key {msg, nwords, words_off, mp}
//   rwords : u32 pool of the keys' topic words
//   lists  : pool of 32-B entries (row id, msg, the topic's first words):
//            per MP (all its rows); per {MP, k, w}
//            (position list: rows whose word k is w, k < kMaxPos) and per
//            {MP, w0, w1} (pair list: rows whose first two words are those).
//            A wildcard filter scans the shortest list one of its literal
//            words selects: a row outside it fails vmq_topic:match/2 anyway
//            (a literal filter word must equal the topic's, vmq_topic.erl:55-57)
//   ptab   : open-addressed {MP, kind, a, b} -> list, 2 slots per 64-B bucket
//   mpl    : per MP its list {off, count}
//   exact  : open-addressed fingerprint of (MP, words) -> row, for filters
//            without a wildcard (ets:lookup, :93-98)
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/vmqr.h"
#include "vmqg_chain.h"
#include "vmqg_common.h"
#include "vmqg_engine.h"

namespace vmqr {

using vmqg::FlatIndex;
using vmqg::Patch;

struct alignas(16) RRow { uint32_t msg, nwords, words_off, mp; };
// list entry: a copy of the row the walk tests, so that one coalesced 32-B
// load per candidate suffices whatever the list order (words past the
// first kLWords are read from rwords)
constexpr uint32_t kLWords = 4;
struct alignas(16) LEnt { uint32_t row, msg, nwords, words_off, w[kLWords]; };
// list slot: kind kPair {MP, w0, w1} or kPos {MP, word, position}; mp == kEmpty: free
struct alignas(32) PSlot { uint32_t mp, a, b, kind, off, count, pad[2]; };
constexpr uint32_t kPair = 1, kPos = 2;
constexpr uint32_t kMaxPos = 16;   // word positions with a position list
struct alignas(16) XSlot { uint64_t fp; uint32_t row, state; };    // state 0 free, 1 live, 2 deleted
struct alignas(8) MpList { uint32_t off, count; };
static_assert(sizeof(LEnt) == 32, "");
static_assert(sizeof(RRow) == 16 && sizeof(PSlot) == 32 && sizeof(XSlot) == 16 && sizeof(MpList) == 8, "");
constexpr uint32_t kPSlotsPerBucket = 2;
VMQG_HD uint64_t part_hash(uint32_t mp, uint32_t a, uint32_t b, uint32_t kind) {
  return vmqg::mix64(vmqg::mix64(((uint64_t)mp << 32) | a) ^ (((uint64_t)kind << 32) | b));
}
constexpr uint32_t kXLive = 1, kXTomb = 2;

struct RLayout {
  uint64_t magic, total_bytes;
  uint64_t rows_off, rwords_off, lists_off, ptab_off, mpl_off, exact_off;
  uint64_t rows_cap, rwords_cap, lists_cap, ptab_buckets, max_mp, exact_slots;
  uint64_t pad[18];
};
static_assert(sizeof(RLayout) == 256, "");
constexpr uint64_t kRLayoutMagic = 0x31726D7176ull;   // "vmqr1"

// Launch interface (vmqr_kernels.hip).
#ifndef VMQR_TILE_ROWS
#define VMQR_TILE_ROWS 1024
#endif
constexpr uint32_t kTileRows = VMQR_TILE_ROWS;   // rows of the flattened walk per look-back tile
struct RArgs {
  const RRow* rows; const uint32_t* rwords; const LEnt* lists;
  const PSlot* ptab; uint64_t ptab_mask;          // bucket mask
  const MpList* mpl; uint32_t max_mp, pad0;
  const XSlot* exact; uint64_t exact_mask;        // slot mask
  const vmqg_pub* filters; const uint32_t* words; uint32_t nf, pad1;
  uint64_t* plan;        // nf x 2: {list off | row, count | kind << 62}
  uint64_t* rpfx;        // nf + 1: rows per filter -> exclusive prefix (scan); [nf] = rows of the batch
  uint32_t* out; uint64_t out_cap;
  uint64_t* offsets;     // nf + 1
  uint32_t* status;      // [1] error bits, [3] scan ticket, [4] walk ticket
  uint64_t* lookback; uint32_t lb_tag, pad2;
  uint64_t tile_cap;     // look-back granules: the walk's tiles must fit
  uint32_t* tickets;     // walk tickets: kClasses counters, kTicketStride apart (zeroed per call)
};
constexpr uint32_t kTicketStride = 64;   // u32: 256 B between the counters
int walk_blocks_per_cu();   // resident blocks of the walk kernel per CU (the walk grid)
// t: null, or {start, stop} events of the plan, the scan and the walk (6)
hipError_t launch_retain_match(const RArgs& a, uint32_t grid, hipStream_t st, const hipEvent_t* t);

uint64_t retain_fp(uint32_t mp, const uint32_t* w, uint32_t L);

struct RRowInfo {
  uint32_t mp = 0, msg = 0;
  std::vector<uint32_t> words;
  std::vector<uint32_t> part;        // its lists besides the MP list (pair, then positions)
  std::vector<uint32_t> ppos;        // its position in each (kNone while not live)
  uint32_t mpos = vmqg::kNone;       // position in the MP list
  uint64_t xslot = ~0ull;
  uint32_t words_off = vmqg::kNone;
  bool live = false;
};

struct RList {
  uint64_t off = 0, cap = 0;
  std::vector<uint32_t> rows;
};

struct RetainEngine {
  vmqr_config cfg{};
  bool has_device = false;
  int device = -1;
  // dictionary (VMQG_WORD_PLUS / _HASH / _SHARE reserved as in vmqg)
  std::unordered_map<std::string, uint32_t> word_index;
  std::vector<std::string> word_text;
  // ?RETAIN_CACHE: one row per distinct key ever inserted (live or not)
  std::vector<RRowInfo> rows;
  FlatIndex key_index;                 // hash(mp, words) -> row (verified)
  uint64_t n_live = 0;
  // pair and position lists
  FlatIndex part_index;                // part_hash -> list (verified)
  std::vector<RList> parts;
  std::vector<uint32_t> part_mp, part_a, part_b, part_kind;
  std::vector<uint64_t> part_slot;
  std::vector<RList> mplists;          // per MP
  // mirror
  RLayout lay{};
  std::vector<uint64_t> mirror;
  std::vector<uint64_t> dirty_bits, dirty_chunks;
  bool full_image = false;
  uint64_t rwords_top = 0, lists_top = 0, lists_garbage = 0, exact_used = 0;
  uint64_t epoch = 0, rebuilds = 0;
  // device
  hipStream_t stream = nullptr;
  hipEvent_t ev_match_done = nullptr;   // recorded by order_on when the stream changes
  hipStream_t ev_stream = vmqg::no_stream();      // the stream patches / matches were last queued on
  uint8_t* d_arena = nullptr; uint64_t d_arena_bytes = 0;
  Patch* h_patch = nullptr; uint64_t h_patch_cap = 0;
  Patch* d_patch = nullptr; uint64_t d_patch_cap = 0;
  uint32_t* d_status = nullptr;
  uint32_t* d_tickets = nullptr;
  int walk_grid = 0;
  uint64_t* d_plan = nullptr; uint64_t plan_cap = 0;       // filters
  uint64_t walk_rows_hint = 1ull << 26;   // rows the first look-back allocation covers (option)
  uint32_t last_nf = 0;                    // filters of the last match_device call
  uint64_t* d_lookback = nullptr; uint64_t lookback_cap = 0; uint32_t lb_tag = 0;
  void* d_f = nullptr; uint64_t d_f_cap = 0;   // host-buffer staging
  void* d_w = nullptr; uint64_t d_w_cap = 0;
  void* d_o = nullptr; uint64_t d_o_cap = 0;
  void* d_offs = nullptr; uint64_t d_offs_cap = 0;
  int cu_count = 256;
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> t_count, t_scan, t_emit;   // plan, scan, walk
  double sum_count_ns = 0, sum_emit_ns = 0; uint64_t n_timed = 0;
  std::string dump_text;

  ~RetainEngine();
  int init(const vmqr_config& c);
  uint32_t intern(const uint8_t* b, size_t n, bool create);
  int apply(const vmqr_op* ops, size_t n, const uint32_t* words, size_t nwords);
  int match_device(const vmqg_pub* d_filters, uint32_t nf, const uint32_t* d_words, uint32_t* d_out,
                   uint64_t out_cap, uint64_t* d_offsets, hipStream_t st);
  int match_status(hipStream_t st);
  int grow_tiles(uint64_t rows, hipStream_t st);   // look-back granules for a walk over `rows`
  void collect_times();
  int order_on(hipStream_t st);
  std::string dump();

 private:
  void insert(uint32_t mp, const uint32_t* w, uint32_t L, uint32_t msg);
  void erase(uint32_t mp, const uint32_t* w, uint32_t L);
  uint32_t find_row(uint32_t mp, const uint32_t* w, uint32_t L) const;
  uint32_t part_of(uint32_t mp, uint32_t a, uint32_t b, uint32_t kind);
  template <class T> T* region(uint64_t off) { return reinterpret_cast<T*>(reinterpret_cast<uint8_t*>(mirror.data()) + off); }
  void touch(uint64_t off, uint64_t bytes);
  // which = -1: the row's MP list; else its list R.part[which]
  bool list_push(uint32_t row, int which);
  void list_remove(uint32_t row, int which);
  bool write_list_head(bool part, uint32_t id);
  bool write_row(uint32_t r);
  LEnt entry_of(uint32_t r) const;
  void put_entry(uint64_t slot, uint32_t r);
  bool place_exact(uint32_t r);
  bool place_part(uint32_t p);
  RLayout plan_layout(uint32_t scale) const;
  void rebuild();
  int upload();
};

}  // namespace vmqr
