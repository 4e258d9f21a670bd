// Shared host/device definitions of the device image ("arena") that the host
// engine (vmqg_engine.cpp) maintains and the HIP kernels (vmqg_kernels.hip)
// read.  Every table lives in ONE device allocation so that a delta batch is
// a list of 16-byte patches (offset, bytes) and a replica is a plain copy.
//
// Layout of the arena (all regions 256-B aligned):
//   edges   : open-addressed hash (parent path, word) -> child path.
//             Buckets of 4 x 16-B slots (one 64-B line per probe).  The
//             slot's 4th word caches the CHILD's edge flags (has a '#' /
//             '+' edge), so the walk never issues a probe that must miss.
//             This is vmq_trie (vmq_reg_trie.erl:41,43,138).
//   nodes   : indexed by path id, 32 B.  Folds vmq_trie_node (:42,139), the
//             vmq_trie_topic entry of the same path (:140) and the resolved
//             subscriber-list keys of that entry (the first one inline as
//             {record off, count}) into one record, so that a trie hit needs
//             one load to know what it emits.
//   keydesc : indexed by key id, 8 B {record offset, count} — one
//             vmq_trie_subs key ({MP,Topic} or {MP,Group,Topic}) (:141-142).
//   keylist : u32 pool of key ids for filters with >= 2 node entries.
//   records : 16-B emission records (vmqg_emit) grouped per key.
//   exact   : open-addressed hash of (MP, Topic) -> {local key's record off +
//             count, remote-node mask}: the `{Topic, node()}` candidate of
//             fold/4 (:62) plus vmq_trie_remote_subs (:143, :514-520), for
//             every topic with a local key or remote entries — wildcard
//             filters too: fold/4 takes the Topic word list as given, so a
//             publish whose words are literally "a", "+" finds the local key
//             of the filter a/+ (add_subscriber keys every local
//             subscription, :257-260, :498-501).  64-B slots holding the MP
//             and the first 7 words, two per 128-B bucket: one line verifies
//             a topic of <= 7 words.
//   exwords : u32 pool: per exact topic its words beyond the 7th, then
//             {count, remote nodes >= 64} (only when it has some).
//   exbits  : one bit per fingerprint class of the non-wildcard exact topics
//             (one per exact slot, so it stays L2-resident): a publish whose
//             bit is clear skips the exact-table probe (a publish holding a
//             '+' / '#' word always probes).
#pragma once
#include <stddef.h>
#include <stdint.h>

// The host's page-safe 16-B over-reads of short words are still over-reads
// to a sanitizer: sanitized builds read byte-exact.
#if defined(__SANITIZE_ADDRESS__) || defined(__SANITIZE_THREAD__)
#define VMQG_NO_OVERREAD 1
#elif defined(__has_feature)
#if __has_feature(address_sanitizer) || __has_feature(thread_sanitizer)
#define VMQG_NO_OVERREAD 1
#endif
#endif

#if defined(__HIPCC__) || defined(__HIP__)
#define VMQG_HD __host__ __device__ __forceinline__
#else
#define VMQG_HD inline
#endif

namespace vmqg {

constexpr uint32_t kEmpty = 0xFFFFFFFFu;   // slot never used
constexpr uint32_t kTomb = 0xFFFFFFFEu;    // slot deleted (probe continues)
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kPlus = 0u, kHash = 1u, kShare = 2u, kUnknownWord = 0xFFFFFFFFu;

// node record flags (low 8 bits of NodeRec.meta; nkeys in the high 24 bits)
constexpr uint32_t kNodeRec = 1u;       // vmq_trie_node record exists
constexpr uint32_t kNodeTopic = 2u;     // ... and its `topic` field is set
constexpr uint32_t kNodeFilter = 4u;    // vmq_trie_topic entry exists for the path
constexpr uint32_t kNodeDollarSkip = 8u;  // path is [#] or starts with + (:285-288)
constexpr uint32_t kNodeHigh = 16u;       // remote nodes >= 64 listed at {hi_off, hi_cnt} (keylist pool)
// a root (path id < max_mountpoints) has no incoming edge slot to cache its
// child flags: its own record carries them, kHas* << kRootFlagShift
constexpr uint32_t kRootFlagShift = 5;
constexpr uint32_t kNodeEmits = kNodeRec | kNodeTopic | kNodeFilter;

// child flags cached in EdgeSlot.flags
constexpr uint32_t kHasHash = 1u;   // the child has a '#' edge
constexpr uint32_t kHasPlus = 2u;   // the child has a '+' edge
constexpr uint32_t kHasWord = 4u;   // the child has an edge of a literal word
constexpr uint32_t kHasAll = kHasHash | kHasPlus | kHasWord;

struct alignas(16) EdgeSlot { uint32_t parent, word, child, flags; };
// meta = flags | nkeys << 8; nkeys == 1: {off0, cnt0} inline; nkeys >= 2: key = keylist offset.
// rmask: remote nodes < 64; nodes >= 64 (kNodeHigh) are listed in the keylist pool at hi_off.
// The node region holds 2 x node_cap records: [p] is path p's own, [node_cap + p]
// a copy of the record of p's '#' child while the edge (p, '#') exists (else
// empty), so a '#' candidate costs one record read and no edge probe.
struct alignas(16) NodeRec { uint32_t meta, key, rmask_lo, rmask_hi, off0, cnt0, hi_off, hi_cnt; };
struct alignas(8) KeyDesc { uint32_t off, count; };
struct alignas(16) Record { uint32_t kind_node, group, subscriber, subinfo; };
// ExactSlot.nwords bit: remote nodes >= 64 follow in exwords ({count, node
// ids}, after the words beyond the inline ones); the slot's rmask holds the
// nodes < 64.
constexpr uint32_t kExactHigh = 0x40000000u;
// ExactSlot.nwords bit: a topic of <= 3 words whose local key holds one
// record keeps that record in w[3..6] (the slot's last 16 B), so the
// trie-less match writes it without a second random read
constexpr uint32_t kExactOne = 0x20000000u;
constexpr uint32_t kExactFlags = kExactHigh | kExactOne;
constexpr uint32_t kExactInline = 7;   // words held in the slot itself
constexpr uint32_t kExactOneMaxWords = 3;
struct alignas(64) ExactSlot {
  uint64_t fp;
  uint32_t nwords, words_off;   // nwords == kEmpty / kTomb marks free slots; exwords[words_off..]: words [7, L),
                                // then the high-node list (kNone when there is neither)
  uint32_t off, count;          // the local {MP,Topic} key's records (count 0: none)
  uint64_t rmask;               // remote nodes with exact subscriptions
  uint32_t mp;
  uint32_t w[kExactInline];     // words [0, min(L, 7)); the rest 0
};
static_assert(sizeof(EdgeSlot) == 16 && sizeof(NodeRec) == 32 && sizeof(Record) == 16, "");
static_assert(sizeof(ExactSlot) == 64 && sizeof(KeyDesc) == 8, "");
// the exact-only COUNT reads a slot as four 16-B quarters
static_assert(offsetof(ExactSlot, nwords) == 8 && offsetof(ExactSlot, off) == 16 && offsetof(ExactSlot, rmask) == 24 &&
              offsetof(ExactSlot, mp) == 32 && offsetof(ExactSlot, w) == 36, "ExactSlot quarters");
// exwords entries before a slot's high-node list
VMQG_HD uint32_t exact_tail_words(uint32_t L) { return L > kExactInline ? L - kExactInline : 0u; }

constexpr uint32_t kEdgeSlotsPerBucket = 4;
constexpr uint32_t kMaxNodes = 4096;        // VMQG_MAX_NODES: one 64-bit bitset word per lane
constexpr uint32_t kLowNodes = 64;          // nodes held in the inline 64-bit masks
constexpr uint32_t kMaxMountpoints = 1u << 24;   // mountpoint ids (roots grow on demand up to this)
constexpr uint32_t kExactSlotsPerBucket = 2;   // 128-B buckets: one L2 line per probe

// Arena layout.  Fixed-size POD: it is what a replica needs to read an image
// (VMQG_LAYOUT_BYTES in vmqg.h bounds it).
struct Layout {
  uint64_t magic;
  uint64_t total_bytes;
  uint64_t edge_off, node_off, keydesc_off, keylist_off, rec_off, exact_off, exwords_off;
  uint64_t edge_buckets;     // power of two
  uint64_t node_cap;         // path ids (the node region holds 2 x node_cap records)
  uint64_t key_cap;          // key ids
  uint64_t keylist_cap;      // u32 entries
  uint64_t rec_cap;          // records
  uint64_t exact_buckets;    // power of two
  uint64_t exwords_cap;      // u32 entries
  uint64_t max_mountpoints;
  uint64_t local_node;
  uint64_t max_depth;        // deepest trie path (sizes the wave tier's global stack)
  uint64_t exbits_off;       // exact-topic filter: one bit per fingerprint class, set for every
  uint64_t exbits_words;     // ... non-wildcard exact topic placed since the last re-layout (u32 words, power of two)
  uint64_t pad[11];
};
static_assert(sizeof(Layout) == 256, "layout must be 256 bytes");
constexpr uint64_t kLayoutMagic = 0x34676D7176ull;  // "vmqg4" (64-B exact slots with inline words; exbits one per slot; root child flags)

// 24-byte patch record: write 16 bytes at arena offset `off` (16-B aligned).
struct Patch { uint64_t off; uint32_t data[4]; };
static_assert(sizeof(Patch) == 24, "");

VMQG_HD uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}
VMQG_HD uint64_t edge_hash(uint32_t parent, uint32_t word) {
  return mix64(((uint64_t)parent << 32) | word);
}
// Exact-topic fingerprint: an order-sensitive sum of per-position mixes, so
// a wave can compute it lane-parallel.  Equal fingerprints are verified
// word by word (exwords), so collisions cost a compare, never a wrong match.
VMQG_HD uint64_t fp_word(uint32_t word, uint32_t pos) {
  return mix64(((uint64_t)word << 32) ^ (uint64_t)(pos * 0x9E3779B9u + 1u));
}
VMQG_HD uint64_t fp_final(uint64_t sum, uint32_t mp, uint32_t nwords) {
  return mix64(sum + mix64(((uint64_t)mp << 32) | nwords));
}
// The exact-topic filter's bit for a fingerprint (bits: a power of two): a
// clear bit means no exact topic has that fingerprint, so the exact table
// (a random HBM line) need not be probed.  Bits are never cleared between
// re-layouts: a deleted topic's bit only costs a probe that misses.
VMQG_HD uint64_t exbit_of(uint64_t fp, uint64_t bits) { return (fp >> 24) & (bits - 1); }

}  // namespace vmqg
