// Host engine of libvmqgpu: owns the authoritative subscription state with
// the semantics of vmq_reg_trie's event handlers and keeps a byte-exact host
// mirror of the device arena.  Every table mutation is written to the mirror
// and recorded as a dirty 16-B chunk; vmqg_apply_ops ships the dirty chunks
// as patches (or, after a re-layout, the whole image) to the device.
#pragma once
#include <hip/hip_runtime.h>

#include <sys/mman.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstring>
#include <cstdlib>
#include <memory>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "vmqg_chain.h"
#include "vmqg_common.h"
#include "vmqg_kernels.h"

namespace vmqg {

// Allocator for the engine's big tables (the arena mirror, the indexes, the
// path / key / topic arrays): blocks of >= 4 MiB are 2-MiB aligned and
// advised to transparent huge pages, so the random lookups of a delta batch
// do not pay a page walk each.
template <class T>
struct HugeAlloc {
  using value_type = T;
  HugeAlloc() = default;
  template <class U> HugeAlloc(const HugeAlloc<U>&) {}
  T* allocate(size_t n) {
    const size_t bytes = n * sizeof(T);
    if (bytes < (4u << 20)) {
      void* p = ::operator new(bytes);
      return static_cast<T*>(p);
    }
    const size_t huge = 2u << 20, rounded = (bytes + huge - 1) & ~(huge - 1);
    void* p = std::aligned_alloc(huge, rounded);
    if (!p) throw std::bad_alloc();
    madvise(p, rounded, MADV_HUGEPAGE);
    return static_cast<T*>(p);
  }
  void deallocate(T* p, size_t n) {
    if (n * sizeof(T) < (4u << 20)) ::operator delete(p);
    else std::free(p);
  }
  template <class U> bool operator==(const HugeAlloc<U>&) const { return true; }
  template <class U> bool operator!=(const HugeAlloc<U>&) const { return false; }
};
template <class T> using HugeVec = std::vector<T, HugeAlloc<T>>;

// NodeOrGroup of a vmq_trie_topic node list: Node | {Node, Group}
struct Nog {
  uint32_t node, group;  // group == kNone for a plain node
  bool operator==(const Nog& o) const { return node == o.node && group == o.group; }
};

// Open-addressed uint64 -> uint32 index (linear probing, load <= 1/2
// counting tombstones).  Several values may share a key (topic_index keys by
// a 64-bit hash of MP + words): find() takes a predicate that verifies the
// stored value.  Paths, topics and keys are erased when vmq_reg_trie would
// no longer hold them (Engine::reclaim), so the index follows the live set.
class FlatIndex {
 public:
  static constexpr uint32_t kVoid = 0xFFFFFFFFu;
  static constexpr uint32_t kGone = 0xFFFFFFFEu;   // erased: probes continue past it
  void reserve(uint64_t n) { if (n * 2 > slots_.size()) regrow(n * 2); }
  // first value stored under `key` for which ok(value) holds, else kVoid
  template <class Ok>
  uint32_t find(uint64_t key, Ok ok) const {
    if (slots_.empty()) return kVoid;
    const uint64_t m = slots_.size() - 1;
    for (uint64_t i = mix64(key) & m;; i = (i + 1) & m) {
      const Slot& s = slots_[i];
      if (s.val == kVoid) return kVoid;
      if (s.val != kGone && s.key == key && ok(s.val)) return s.val;
    }
  }
  uint32_t find(uint64_t key) const { return find(key, [](uint32_t) { return true; }); }
  // software prefetch of the slot `key` hashes to
  void prefetch(uint64_t key) const {
    if (!slots_.empty()) __builtin_prefetch(&slots_[mix64(key) & (slots_.size() - 1)]);
  }
  // (key, val) must not be stored already; an erased slot on the probe path
  // is taken before an empty one, so erase + insert churn leaves no trail of
  // tombstones (a table full of them would be rehashed: a stall of the stage)
  void insert(uint64_t key, uint32_t val) {
    if ((n_ + gone_ + 1) * 2 > slots_.size())   // mostly tombstones: rehash at the same size
      regrow(std::max<uint64_t>(1024, (n_ + 1) * 4 > slots_.size() ? slots_.size() * 2 : slots_.size()));
    const uint64_t m = slots_.size() - 1;
    uint64_t i = mix64(key) & m, reuse = ~0ull;
    for (; slots_[i].val != kVoid; i = (i + 1) & m)
      if (slots_[i].val == kGone && reuse == ~0ull) reuse = i;
    if (reuse != ~0ull) { i = reuse; gone_--; }
    slots_[i] = Slot{key, val};
    n_++;
  }
  // erases the entry (key, val); false if absent
  bool erase(uint64_t key, uint32_t val) {
    if (slots_.empty()) return false;
    const uint64_t m = slots_.size() - 1;
    for (uint64_t i = mix64(key) & m;; i = (i + 1) & m) {
      Slot& s = slots_[i];
      if (s.val == kVoid) return false;
      if (s.val == val && s.key == key) { s.val = kGone; n_--; gone_++; return true; }
    }
  }
  uint64_t size() const { return n_; }
  uint64_t bytes() const { return slots_.size() * sizeof(Slot); }

 private:
  struct Slot { uint64_t key; uint32_t val; };
  void put(uint64_t key, uint32_t val) {
    const uint64_t m = slots_.size() - 1;
    uint64_t i = mix64(key) & m;
    while (slots_[i].val != kVoid) i = (i + 1) & m;
    slots_[i] = Slot{key, val};
  }
  void regrow(uint64_t want) {
    uint64_t cap = 1;
    while (cap < want) cap <<= 1;
    HugeVec<Slot> old;
    old.swap(slots_);
    slots_.assign(cap, Slot{0, kVoid});
    for (const Slot& s : old) if (s.val != kVoid && s.val != kGone) put(s.key, s.val);
    gone_ = 0;
  }
  HugeVec<Slot> slots_;
  uint64_t n_ = 0, gone_ = 0;
};

// Word dictionary: topic words -> dense ids (vmq_topic words; the interning
// contract of SURVEY §7).  Open addressing over 32-B slots holding the word's
// 64-bit hash, id, length and first 16 bytes, so looking up a word of at most
// 16 bytes touches one cache line — the publish hot path (vmqg_prepare_publish*)
// is one such lookup per word, and the batched form prefetches a block of
// topics' slots before resolving any.
//
// One writer, any number of readers, no lock (vmq_reg_trie's tables are
// read_concurrency ETS, vmq_reg_trie.erl:136-137): lookups never write and
// never wait.  A slot is filled before its id is published (release; readers
// load the id with acquire, then the rest); a table that grows is rebuilt
// aside and swapped in whole, the old one kept until the dictionary dies
// (readers may still be probing it; all retired tables together are smaller
// than the live one); word texts live in fixed chunks that never move.  A
// reader that started before an insert may miss that word: the batch layer's
// generation check (vmqgb_batch_recheck) prepares such publishes again.
class WordDict {
 public:
  static constexpr uint32_t kVoid = 0xFFFFFFFFu;
  WordDict() : dir_(new std::atomic<std::string*>[kChunks]) {
    for (uint32_t i = 0; i < kChunks; i++) dir_[i].store(nullptr, std::memory_order_relaxed);
  }
  ~WordDict() {
    for (uint32_t i = 0; i < kChunks; i++) delete[] dir_[i].load(std::memory_order_relaxed);
  }
  WordDict(const WordDict&) = delete;
  WordDict& operator=(const WordDict&) = delete;
  // a word as the lookup sees it: hash and its first 16 bytes, zero padded
  struct Key { uint64_t h, k0, k1; const uint8_t* p; size_t n; };
  static Key key(const uint8_t* p, size_t n) {
    Key k{0, 0, 0, p, n};
#if defined(VMQG_NO_OVERREAD)
    constexpr bool kWide = false;   // the page-safe over-read below is still an over-read to ASan
#else
    constexpr bool kWide = true;
#endif
    if (n >= 16 || (kWide && ((uintptr_t)p & 4095) <= 4096 - 16)) {
      // 16 bytes readable (the word's own, or without crossing a page): two
      // loads, the bytes past the word masked off (the same zero padding as below)
      memcpy(&k.k0, p, 8);
      memcpy(&k.k1, p + 8, 8);
      if (n < 8) { k.k0 &= n ? ~0ull >> (64 - 8 * n) : 0ull; k.k1 = 0; }
      else if (n < 16) k.k1 &= n > 8 ? ~0ull >> (64 - 8 * (n - 8)) : 0ull;
    } else {
      uint8_t buf[16] = {0};
      memcpy(buf, p, n < 16 ? n : 16);
      memcpy(&k.k0, buf, 8);
      memcpy(&k.k1, buf + 8, 8);
    }
    uint64_t h = mix64(k.k0 ^ (0x9E3779B97F4A7C15ull * (n + 1))) ^ k.k1;
    for (size_t i = 16; i < n; i += 8) {
      uint64_t v = 0;
      memcpy(&v, p + i, n - i < 8 ? n - i : 8);
      h = mix64(h ^ v) + i;
    }
    k.h = mix64(h);
    return k;
  }
  void prefetch(const Key& k) const {
    const Table* t = tab_.load(std::memory_order_acquire);
    if (t) __builtin_prefetch(&t->slots[k.h & t->mask]);
  }
  uint32_t find(const Key& k) const {
    const Table* t = tab_.load(std::memory_order_acquire);
    return t ? find_in(*t, k) : kVoid;
  }
  // id of the word, added when absent (the writer only): a released id
  // (remove) first, else the next dense one
  uint32_t intern(const Key& k) {
    const uint32_t f = find(k);
    if (f != kVoid) return f;
    const uint64_t n = count_.load(std::memory_order_relaxed);
    if (free_.empty() && n >= 0xFFFFFF00ull) throw std::bad_alloc();   // ids above are reserved (kUnknownWord, ...)
    const Table* t = tab_.load(std::memory_order_relaxed);
    if (!t || (live_ + gone_ + 1) * 2 > t->mask + 1)   // full, or full of erased slots: rebuilt aside
      t = regrow(std::max<uint64_t>(1024, t && (live_ + 1) * 4 <= t->mask + 1 ? t->mask + 1 : (t ? (t->mask + 1) * 2 : 0)));
    uint32_t id;
    if (!free_.empty()) { id = free_.back(); free_.pop_back(); }
    else id = (uint32_t)n;
    std::string* chunk = dir_[id >> kChunkBits].load(std::memory_order_relaxed);
    if (!chunk) {
      chunk = new std::string[kChunkWords];
      dir_[id >> kChunkBits].store(chunk, std::memory_order_release);
    }
    chunk[id & (kChunkWords - 1)].assign(reinterpret_cast<const char*>(k.p), k.n);
    if (put(*t, Slot{k.h, id, (uint32_t)k.n, k.k0, k.k1})) gone_--;
    live_++;
    gen_.fetch_add(1, std::memory_order_release);
    if (id == n) count_.store(n + 1, std::memory_order_release);
    return id;
  }
  // Takes a word out of the table (the writer only): later lookups miss it
  // (its slot is marked erased, probes continue past it); its id stays
  // reserved and its text readable for the readers that found it before.
  void erase(uint32_t id) {
    const std::string& w = text(id);
    const Key k = key(reinterpret_cast<const uint8_t*>(w.data()), w.size());
    const Table* t = tab_.load(std::memory_order_relaxed);
    Slot* sl = const_cast<Slot*>(t->slots.data());
    for (uint64_t i = k.h & t->mask;; i = (i + 1) & t->mask) {
      const uint32_t v = sl[i].id;
      if (v == kVoid) return;   // not in the table
      if (v == id) { __atomic_store_n(&sl[i].id, kGone, __ATOMIC_RELEASE); gone_++; live_--; return; }
    }
  }
  // An erased word put back under its id (an op that names it after all).
  void revive(uint32_t id) {
    const std::string& w = text(id);
    const Key k = key(reinterpret_cast<const uint8_t*>(w.data()), w.size());
    if (find(k) != kVoid) return;
    const Table* t = tab_.load(std::memory_order_relaxed);
    if ((live_ + gone_ + 1) * 2 > t->mask + 1) t = regrow((t->mask + 1) * 2);
    if (put(*t, Slot{k.h, id, (uint32_t)k.n, k.k0, k.k1})) gone_--;
    live_++;
  }
  // Frees an erased word's text and makes its id reusable (the writer only,
  // once no reader that could hold the id is running: vmqg_dict_release).
  void release(uint32_t id) {
    std::string().swap(dir_[id >> kChunkBits].load(std::memory_order_relaxed)[id & (kChunkWords - 1)]);
    free_.push_back(id);
  }
  const std::string& text(uint32_t id) const {
    return dir_[id >> kChunkBits].load(std::memory_order_acquire)[id & (kChunkWords - 1)];
  }
  // ids handed out so far are < id_bound(); words in the table = size()
  uint64_t id_bound() const { return count_.load(std::memory_order_acquire); }
  size_t size() const { return live_; }
  // words interned so far, reused ids included (the batch layer's staleness
  // check of prepared publishes that held unknown words)
  uint64_t generation() const { return gen_.load(std::memory_order_acquire); }
  // tables replaced by a rebuild, kept for readers still probing them until
  // a grace period ends (free_tables_before)
  void free_tables_before(uint64_t token) {
    size_t k = 0;
    for (size_t i = 0; i < retired_.size(); i++) {
      if (retired_[i].second < token) retired_[i].first.reset();
      else retired_[k++] = std::move(retired_[i]);
    }
    retired_.resize(k);
  }
  uint64_t retire_token = 0;   // the writer's grace token now (vmqg_dict_grace_token)
  uint64_t bytes() const {
    const Table* t = tab_.load(std::memory_order_relaxed);
    uint64_t b = t ? (t->mask + 1) * sizeof(Slot) : 0;
    for (auto& r : retired_) b += (r.first->mask + 1) * sizeof(Slot);
    return b + (count_.load(std::memory_order_relaxed) + kChunkWords - 1) / kChunkWords * kChunkWords * sizeof(std::string);
  }

 private:
  static constexpr uint32_t kChunkBits = 16, kChunkWords = 1u << kChunkBits, kChunks = 1u << 16;
  struct alignas(32) Slot { uint64_t h; uint32_t id, len; uint64_t k0, k1; };
  struct Table {
    HugeVec<Slot> slots;
    uint64_t mask;
  };
  static constexpr uint32_t kGone = 0xFFFFFFFEu;   // an erased slot: probes continue
  static uint32_t load_id(const Slot& s) { return __atomic_load_n(&s.id, __ATOMIC_ACQUIRE); }
  uint32_t find_in(const Table& t, const Key& k) const {
    for (uint64_t i = k.h & t.mask;; i = (i + 1) & t.mask) {
      const Slot& s = t.slots[i];
      const uint32_t id = load_id(s);
      if (id == kVoid) return kVoid;
      if (id == kGone) continue;
      if (s.h == k.h && s.len == k.n && s.k0 == k.k0 && s.k1 == k.k1 &&
          (k.n <= 16 || memcmp(text(id).data() + 16, k.p + 16, k.n - 16) == 0))
        return id;
    }
  }
  // The id is stored last: a reader that sees it sees the slot's other
  // fields.  An erased slot on the probe path is taken before an empty one
  // (churn leaves no trail of tombstones to rehash); a reader that loaded the
  // erased word's id before compares the new fields with its key: no match
  // unless it is the same word, interned again — then it returns the old id,
  // which its grace period keeps from being reused (a lookup from before the
  // new subscription).  Returns whether an erased slot was taken.
  static bool put(const Table& t, const Slot& s) {
    Slot* sl = const_cast<Slot*>(t.slots.data());
    for (uint64_t i = s.h & t.mask;; i = (i + 1) & t.mask) {
      const uint32_t v = sl[i].id;
      if (v == kVoid || v == kGone) {
        sl[i].h = s.h; sl[i].len = s.len; sl[i].k0 = s.k0; sl[i].k1 = s.k1;
        __atomic_store_n(&sl[i].id, s.id, __ATOMIC_RELEASE);
        return v == kGone;
      }
    }
  }
  const Table* regrow(uint64_t want) {
    uint64_t cap = 1;
    while (cap < want) cap <<= 1;
    auto nt = std::make_unique<Table>();
    nt->slots.assign(cap, Slot{0, kVoid, 0, 0, 0});
    nt->mask = cap - 1;
    if (const Table* old = tab_.load(std::memory_order_relaxed))
      for (const Slot& s : old->slots) if (s.id != kVoid && s.id != kGone) put(*nt, s);
    gone_ = 0;
    const Table* t = nt.get();
    // the old table stays until a grace period taken after now ends: readers may be probing it
    if (cur_) retired_.emplace_back(std::move(cur_), retire_token);
    cur_ = std::move(nt);
    tab_.store(t, std::memory_order_release);
    return t;
  }
  std::atomic<const Table*> tab_{nullptr};
  std::unique_ptr<Table> cur_;
  std::vector<std::pair<std::unique_ptr<Table>, uint64_t>> retired_;   // {table, token when retired}
  std::unique_ptr<std::atomic<std::string*>[]> dir_;   // word texts, kChunkWords per chunk
  std::atomic<uint64_t> count_{0};   // id bound
  std::atomic<uint64_t> gen_{0};     // interns, reused ids included
  uint64_t live_ = 0, gone_ = 0;     // live words, erased slots of the current table
  std::vector<uint32_t> free_;       // released ids
};

struct PathInfo {
  uint32_t parent, word, mp, depth;
  uint64_t in_slot = ~0ull;         // edge-table slot of the edge (parent, word) -> this path, if present
  uint8_t eflags = 0;               // this path's own '#' / '+' / literal edges present (kHas*)
  uint32_t nlit = 0;                // its live literal-word edges (kHasWord while > 0)
  uint32_t nchild = 0;              // interned child paths (a path with any is not reclaimed)
  uint32_t topic_id = kNone;        // (MP, path words) term, once known
  uint32_t kl_off = 0, kl_cap = 0;  // keylist range owned by this path
  uint32_t hn_off = 0, hn_cap = 0;  // keylist range of its remote nodes >= 64
  uint8_t rec = 0, topic_set = 0;   // vmq_trie_node record / its topic field
  uint8_t filter = 0;               // vmq_trie_topic entry exists
  uint8_t dollar_skip = 0, first_plus = 0, dirty = 0;
  int64_t ec = 0;                   // edge_count
  int64_t total = 0;                // vmq_trie_topic TotalCnt
  std::vector<std::pair<Nog, int64_t>> nodes;   // vmq_trie_topic node list
};

struct RecordHash {
  size_t operator()(const Record& r) const {
    return (size_t)mix64(((uint64_t)r.kind_node << 32 | r.group) ^ mix64((uint64_t)r.subscriber << 32 | r.subinfo));
  }
};
struct RecordEq {
  bool operator()(const Record& a, const Record& b) const {
    return a.kind_node == b.kind_node && a.group == b.group && a.subscriber == b.subscriber && a.subinfo == b.subinfo;
  }
};

// One vmq_trie_subs key ({MP,Topic} or {MP,Group,Topic}) with its values.
struct KeyInfo {
  uint32_t topic_id = kNone, group = kNone;   // group != kNone: a $share group key
  uint8_t dirty = 0;
  std::vector<Record> vals;
  std::unique_ptr<std::unordered_map<Record, uint32_t, RecordHash, RecordEq>> idx;
  uint64_t off = 0, cap = 0;                  // record range in the arena
  std::vector<uint32_t> dirty_pos;            // record slots changed since the last flush
};

// One (MP, Topic) term: the local key, the vmq_trie_remote_subs entry and
// the exact-table slot that serves both to publishes.
struct TopicInfo {
  uint32_t mp;
  std::vector<uint32_t> words;
  uint32_t local_key = kNone;
  uint32_t path = kNone;            // trie path of the same (MP, Topic), once created
  uint8_t dirty = 0, wild = 0;      // wild: a '+' / '#' word (no exbits filter bit: only such a publish equals it)
  std::vector<std::pair<uint32_t, int64_t>> remote;
  uint64_t slot = ~0ull;
  uint32_t ngroup = 0;              // $share group keys {MP, Group, Topic} of this topic
  uint32_t words_off = kNone;
  uint32_t xw_len = 0;              // exwords entries owned: words beyond the inline ones, [count, remote nodes >= 64]
};

struct Engine {
  vmqg_config cfg{};
  bool replica = false;
  bool has_device = false;

  // ---- dictionary
  WordDict dict;
  // Word reclamation: a word is held by the trie paths, exact/filter topics
  // and $share group keys that name it; one nothing holds any more is
  // retired at the end of the stage, and dropped (its id reusable) by
  // vmqg_dict_release once the caller's readers have passed a grace period
  // (vmq_reg_trie's tables hold no word that no row uses).
  HugeVec<uint32_t> word_refs;
  HugeVec<uint64_t> word_tag;        // the grace token when it last became unreferenced
  std::vector<uint8_t> word_state;   // 0 in use or fresh, 1 retired (pending), 2 released
  std::vector<uint32_t> word_zero;   // unreferenced (or freshly interned) during this stage
  std::vector<uint32_t> word_retired;
  uint64_t words_released = 0;
  void word_ref(uint32_t w) { if (w >= 3) word_refs[w]++; }
  void word_unref(uint32_t w) { if (w >= 3 && --word_refs[w] == 0) word_zero.push_back(w); }
  void retire_words();
  void release_words(uint64_t token);
  // The caller's SubscriberId / SubInfo ids held by records (vmq_trie_subs
  // values): ids the last stage's ops named, or whose last record it
  // removed, that no record holds now are reported (vmqg_released_ids) so the
  // caller can drop their terms.
  HugeVec<uint32_t> term_refs[2];          // [0] subscriber ids, [1] subinfo ids
  std::vector<uint32_t> term_cand[2], term_released[2];
  std::vector<uint8_t> term_mark[2];
  void term_ref(int kind, uint32_t id) {
    if (id >= term_refs[kind].size()) term_refs[kind].resize(std::max<size_t>(1024, (size_t)id * 2), 0);
    term_refs[kind][id]++;
  }
  void term_unref(int kind, uint32_t id) { if (--term_refs[kind][id] == 0) term_cand[kind].push_back(id); }
  void record_in(const Record& r) { term_ref(0, r.subscriber); term_ref(1, r.subinfo); }
  void record_out(const Record& r) { term_unref(0, r.subscriber); term_unref(1, r.subinfo); }
  void collect_released_terms();
  uint64_t host_bytes() const {
    uint64_t b = mirror.capacity() * 8 + dirty_bits.capacity() * 8 + paths.capacity() * sizeof(PathInfo) +
                 keys.capacity() * sizeof(KeyInfo) + topics.capacity() * sizeof(TopicInfo) + path_index.bytes() +
                 topic_index.bytes() + group_key_index.bytes() + dict.bytes() +
                 word_refs.capacity() * 4 + word_tag.capacity() * 8 + word_state.capacity() +
                 term_refs[0].capacity() * 4 + term_refs[1].capacity() * 4;
    for (const RecBuf& r : rb) b += r.recs.capacity() * sizeof(Record);
    return b;
  }

  // ---- logical state
  HugeVec<PathInfo> paths;                              // ids [0, max_mp) are roots
  FlatIndex path_index;                                     // parent<<32|word -> path
  HugeVec<KeyInfo> keys;
  FlatIndex group_key_index;                                // topic<<32|group -> key
  HugeVec<TopicInfo> topics;
  FlatIndex topic_index;                                    // hash(mp, words) -> topic (verified)
  // ids of reclaimed paths / keys / topics, reused before new ones (Engine::reclaim)
  std::vector<uint32_t> free_paths, free_keys, free_topics;
  std::vector<uint32_t> reclaim_paths, reclaim_topics;   // this stage's candidates (reclaim)
  uint32_t opt_reclaim = 1;                                // vmqg_set_option "reclaim": 0 keeps dropped rows
  uint64_t reclaimed_paths = 0, reclaimed_keys = 0, reclaimed_topics = 0;
  uint64_t n_trie_nodes = 0, n_trie_topics = 0, n_subs_objects = 0, n_fanout = 0, n_remote_keys = 0;

  // ---- mirror of the device arena
  Layout lay{};                     // the host mirror's layout (the writer's)
  Layout dlay{};                    // the device arena's: what match calls read (set by commit)
  HugeVec<uint64_t> mirror;         // lay.total_bytes / 8 words
  HugeVec<uint64_t> dirty_bits;     // one bit per 16-B chunk
  std::vector<uint64_t> dirty_chunks;
  std::vector<uint32_t> dirty_paths, dirty_keys, dirty_topics;
  uint64_t edge_live = 0, edge_tomb = 0, exact_live = 0, exact_tomb = 0;
  uint64_t rec_top = 0, rec_garbage = 0, kl_top = 0, kl_garbage = 0, xw_top = 0, xw_garbage = 0;
  bool full_image = false;          // the pending upload is a whole image
  // epoch: the tables the device holds (matches queued now see them); an
  // apply is staged on the host (staged_epoch = epoch + 1) while matches
  // run, then committed: shipped to the device, epoch = staged_epoch
  // (atomic: vmqg_epoch is a reader call, made beside the writer's commit)
  std::atomic<uint64_t> epoch{0};
  uint64_t rebuilds = 0;
  uint64_t staged_epoch = 0;
  bool staged = false, patches_ready = false;
  // a commit whose upload failed: the stage stays pending (epoch unchanged,
  // matches keep answering from the device's tables), the next commit ships
  // the whole image, and a stage may be added on top of it meanwhile
  bool commit_failed = false;
  uint32_t fault_commits = 0;       // vmqg_set_option "fail_commits": test hook, the next n uploads fail
  uint32_t max_depth = 0;           // deepest path interned (sizes the wave tier's stack)
  std::vector<Patch> last_patches;
  bool last_full = false;
  // apply accounting (vmqg_stats): host work only, separate from device waits
  uint64_t ops_applied = 0, apply_host_ns = 0, apply_upload_ns = 0, apply_wait_ns = 0, patch_bytes = 0,
           image_bytes = 0;

  // ---- device
  int device = -1;
  hipStream_t stream = nullptr;
  uint8_t* d_arena = nullptr; uint64_t d_arena_bytes = 0;
  // patch staging ring: pinned host + device buffers, each reusable once its
  // event (recorded after the patch kernel) has fired, so vmqg_apply_ops
  // never waits for matches still queued on the stream
  static constexpr int kStage = 4;
  struct Stage { Patch* h = nullptr; Patch* d = nullptr; uint64_t cap = 0; hipEvent_t ev = nullptr; bool used = false; };
  Stage stage[kStage];
  int stage_next = 0;
  uint32_t* d_status = nullptr;
  uint32_t* d_deferred = nullptr; uint64_t deferred_cap = 0;   // publishes
  uint64_t call_seq = 0; uint32_t last_set = 0;                // status set of the next / last match call
  void* d_keycache = nullptr; uint64_t keycache_cap = 0;   // publishes
  void* d_dd = nullptr; uint64_t dd_slots = 0; uint32_t dd_tag = 0;   // batch-wide dedupe table
  uint32_t opt_dedupe = 2;                                 // vmqg_set_option "dedupe": 0 off, 1 on, 2 auto (default)
  void* d_groups = nullptr; uint64_t gs_slots = 0;         // output groups (records mode)
  uint32_t opt_dd_g = 4;                                   // vmqg_set_option "dd_g": lanes per representative (1|4)
  uint32_t opt_groups = 0;                                 // vmqg_set_option "groups": 0 off (default: A/B, DESIGN), 1 on
  uint32_t opt_exfilter = 2;                               // vmqg_set_option "exfilter": 0 off, 1 on, 2 auto (default)
  uint64_t ex_next = 0;                                    // auto: the sampler runs on calls after this one (k_ex_sample)
  uint32_t opt_trieless = 1;                               // vmqg_set_option "trieless": the exact-only COUNT when no edge exists
  uint32_t opt_exact_one = 1;                              // vmqg_set_option "exact_one": a short topic's one record inline in its exact slot
  uint32_t opt_fused = 1;                                  // vmqg_set_option "fused": trie-less COUNT + scan + EMIT in one launch
  bool d_trieless = false;                                 // the device tables have no trie edge (set by commit)
  uint32_t opt_heavy_min = 0;                              // vmqg_set_option "heavy_min": records mode, EMIT tail by XCD (0 off)
  // host-buffer match staging
  void* d_pubs = nullptr; uint64_t d_pubs_cap = 0;
  void* d_words = nullptr; uint64_t d_words_cap = 0;
  void* d_offs = nullptr; uint64_t d_offs_cap = 0;
  void* d_out = nullptr; uint64_t d_out_cap = 0;
  hipEvent_t ev_match_done = nullptr;   // recorded by order_on when the stream changes
  hipStream_t ev_stream = vmqg::no_stream();      // the stream table changes / matches were last queued on
  bool timing = false;
  uint32_t opt_fast_g = 0, opt_flags = kOptNtStores | kOptRootFlags;   // vmqg_set_option (defaults: A/B-tuned on MI355X)
  static constexpr uint32_t kFastG1Min = 262144;       // fast_g auto: one lane per publish from this many publishes
  uint32_t opt_count_bpc = 5, opt_emit_bpc = 16;       // fast-tier grid caps, blocks per CU (A/B-tuned)
  // look-back granules (tagged per call), global stack of the tier-2 wave path
  uint64_t* d_lookback = nullptr; uint64_t lookback_cap = 0; uint32_t lb_tag = 0;
  uint2* d_ostack = nullptr; uint64_t ostack_bytes = 0;
  uint32_t* o_slots = nullptr;      // after the stacks: one bit per stack borrowed by an EMIT tail walk
  uint32_t o_cap = 0, o_waves = 0;
  uint64_t o_cap_floor = 0;         // raised by vmqg_match_batch if a tier-2 stack ever overflowed
  int cu_count = 0;
  uint32_t last_deferred[2] = {0, 0};   // whole-wave walks (LDS / global stack) of the last checked batch
  uint32_t last_many = 0, last_retried = 0;    // ... many-key publishes / retried four lanes per publish
  uint64_t last_wave_entries = 0;              // ... entries (records or ranges) the EMIT wave tier wrote
  uint64_t last_wide_entries = 0;              // ... entries the EMIT tail wrote for wide publishes
  uint64_t last_dedup = 0, last_dedup_walked = 0;  // ... duplicates served from a representative / walked anyway
  uint32_t* h_ddmode = nullptr;      // host-mapped dedupe mode word (written by the device)
  mutable uint64_t dd_next = 0, dd_gap = 64;   // auto dedupe: the next probe call, the gap after it
  uint32_t* d_ddmode_host = nullptr; // ... its device address
  uint32_t last_err_bits = 0;   // error bits the last match_status collected
  // epoch of the last apply that rewrote a record slot (or re-laid out the
  // arena): range results of an older epoch index records that may have
  // changed (vmqg_records_at refuses them)
  uint64_t rec_epoch = 0;
  // Readers' copies of the record table (vmqg_records_pin, option
  // "reader_records"): two buffers, left-right.  Readers pin the buffer whose
  // epochs cover their round's and never wait; the writer brings the other
  // one up to date (the records its last two applies changed) once the
  // readers still on it have left, then directs new readers to it.
  struct RecBuf {
    HugeVec<Record> recs;
    uint64_t epoch = 0, rec_epoch = 0;   // content = the tables of every epoch in [rec_epoch, epoch]
    std::atomic<uint32_t> readers{0};
    std::atomic<uint32_t> closed{1};     // the writer is updating it: no new readers
  };
  RecBuf rb[2];
  std::atomic<uint32_t> rb_active{0};
  bool rb_on = false;
  bool rb_full_next = true;             // the inactive buffer needs a whole copy (re-layout)
  std::vector<uint64_t> rb_prev, rb_changed;   // record slots the last / this apply changed
  uint64_t rb_waits = 0, rb_wait_ns = 0;       // the writer waited for readers to leave a buffer
  // device status: two per-call counter sets of kStatusSet words, then the sticky error word
  static constexpr uint32_t kStatusSet = 32, kStatusBytes = 512;
  static constexpr uint32_t kStatusDdMode = 100;   // persistent word: the dedupe mode the last call chose
                                                   // (words 104-106: k_ex_sample's counts and ticket)
  // per-launch timing: COUNT fast tier, COUNT wave tier, scan, EMIT fast tier, EMIT wave tier
  static constexpr int kTimedStages = 5, kTimedEvents = 8;   // + the dedupe claim / classify / fix-up passes (into COUNT)
  std::vector<std::array<hipEvent_t, 2 * kTimedEvents>> t_ev;
  double sum_stage_ns[kTimedStages] = {0, 0, 0, 0, 0}; uint64_t n_timed = 0;

  std::string dump_text;

  ~Engine();
  int init(const vmqg_config& c);

  // dictionary
  uint32_t intern(const uint8_t* b, size_t n, bool create);
  const std::string& word_text(uint32_t id) const { return dict.text(id); }

  // state machine (vmq_reg_trie.erl:253-539)
  int apply_ops(const vmqg_op* ops, size_t n, const uint32_t* words, size_t nwords);   // stage + commit
  int stage_ops(const vmqg_op* ops, size_t n, const uint32_t* words, size_t nwords);   // host half
  int commit();                                                                         // device half
  void stage_patches();
  void publish_records();
  int records_pin(uint64_t ep, const Record** recs, uint64_t* n, uint32_t* pin);
  void records_unpin(uint32_t pin) { rb[pin & 1].readers.fetch_sub(1, std::memory_order_release); }
  void enable_reader_records();
  void handle_add(const vmqg_op& op, const uint32_t* w);
  void handle_delete(const vmqg_op& op, const uint32_t* w);
  void add_complex_topic(uint32_t mp, const uint32_t* w, uint32_t L, Nog nog, bool wildcard);
  void del_complex_topic(uint32_t mp, const uint32_t* w, uint32_t L, Nog nog, bool wildcard);
  void trie_add_path(uint32_t parent, uint32_t word, uint32_t child);
  void trie_delete(uint32_t p, const std::vector<uint32_t>& chain, const uint32_t* w, uint32_t L);
  void insert_trie_subs(uint32_t key, const Record& v);
  void del_trie_subs(uint32_t key, const Record& v);

  uint32_t path_child(uint32_t parent, uint32_t word, bool create);
  bool path_chain(uint32_t mp, const uint32_t* w, uint32_t L, bool create, std::vector<uint32_t>& chain);
  uint32_t topic_id(uint32_t mp, const uint32_t* w, uint32_t L, bool create);
  void prefetch_op(const vmqg_op& op, const uint32_t* w, int stage);   // apply_ops software pipeline
  std::vector<uint32_t> scratch_u32;                                 // write_path / write_topic lists
  uint32_t local_key(uint32_t tid, bool create);
  uint32_t group_key(uint32_t tid, uint32_t group, bool create);
  void mark_path(uint32_t p) { if (!paths[p].dirty) { paths[p].dirty = 1; dirty_paths.push_back(p); } }
  void mark_key(uint32_t k) { if (!keys[k].dirty) { keys[k].dirty = 1; dirty_keys.push_back(k); } }
  void mark_topic(uint32_t t) { if (!topics[t].dirty) { topics[t].dirty = 1; dirty_topics.push_back(t); } }

  // mirror
  template <class T> T* region(uint64_t off) { return reinterpret_cast<T*>(reinterpret_cast<uint8_t*>(mirror.data()) + off); }
  void touch(uint64_t off, uint64_t bytes);
  void edge_insert(uint32_t parent, uint32_t word, uint32_t child);
  void edge_erase(uint32_t parent, uint32_t word, uint32_t child);
  void refresh_incoming_flags(uint32_t node);
  bool write_high_list(uint32_t& off, uint32_t& cap, const std::vector<uint32_t>& nodes);
  Layout plan_layout(uint64_t extra_edges, uint32_t scale, bool compact) const;
  void rebuild(uint64_t extra_edges, bool compact = false);
  void grow_mountpoints(uint32_t need);
  void free_key(uint32_t k);
  void reclaim();
  bool flush_incremental();
  bool write_key(uint32_t k);
  bool write_path(uint32_t p);
  void write_hash_alias(uint32_t parent);
  bool write_topic(uint32_t t);
  uint64_t exact_fp(const TopicInfo& t) const;

  // device
  int upload();
  int ship_patches(const std::vector<Patch>& pl);
  bool follow_ok = false;           // replica: its tables are a committed epoch of its primary's
  int follow(const Engine& primary);
  int arena_digest(uint64_t* out);
  int order_on(hipStream_t st);
  int ensure_match_scratch(uint64_t npub, hipStream_t st);
  int ensure_lookback(uint64_t granules, hipStream_t st);
  int ensure_wave_scratch(hipStream_t st);
  MatchArgs args_for(const vmqg_pub* pubs, uint32_t npub, const uint32_t* words, uint64_t* offs) const;
  // out_rng == null: records mode into out; else range mode into out_rng
  int match_device(const vmqg_pub* d_pubs, uint32_t npub, const uint32_t* d_words, Record* d_out,
                   uint64_t out_cap, vmqg_range* d_rng, uint64_t rng_cap, uint64_t* d_offsets, hipStream_t st);
  uint32_t stack_depth() const { return dlay.max_depth; }   // the device tables' deepest path
  int match_status(hipStream_t st);
  void collect_times();

  std::string dump();
};

}  // namespace vmqg
