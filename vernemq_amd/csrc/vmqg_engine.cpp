// Host engine: interned restatement of vmq_reg_trie's delta handling over
// the device-image mirror.  See vmqg_engine.h for the data model; every
// state-machine function cites the Erlang clause it reproduces
// (apps/vmq_server/src/vmq_reg_trie.erl unless noted).
#include "vmqg_chain.h"
#include "vmqg_engine.h"

#ifndef VMQG_EXACT_SLOTS_PER_TOPIC
#define VMQG_EXACT_SLOTS_PER_TOPIC 4   // exact-table slots per topic (A/B: 2)
#endif

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <unistd.h>
#include <cstring>

namespace vmqg {

static uint64_t next_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}
static uint64_t align256(uint64_t v) { return (v + 255) & ~255ull; }

Engine::~Engine() {
  if (has_device) {
    hipSetDevice(device);
    if (stream) hipStreamSynchronize(stream);
    for (auto& ev : t_ev) for (auto e : ev) hipEventDestroy(e);
    if (ev_match_done) hipEventDestroy(ev_match_done);
    for (Stage& sg : stage) {
      if (sg.ev) hipEventDestroy(sg.ev);
      if (sg.h) hipHostFree(sg.h);
      hipFree(sg.d);
    }
    hipFree(d_arena); hipFree(d_status); hipFree(d_deferred);
    hipFree(d_keycache); hipFree(d_dd); hipFree(d_groups);
    if (h_ddmode) hipHostFree(h_ddmode);
    hipFree(d_lookback); hipFree(d_ostack);
    hipFree(d_pubs); hipFree(d_words); hipFree(d_offs); hipFree(d_out);
    if (stream) hipStreamDestroy(stream);
  }
}

int Engine::init(const vmqg_config& c) {
  cfg = c;
  if (cfg.max_nodes == 0) cfg.max_nodes = VMQG_MAX_NODES;
  if (cfg.max_mountpoints == 0) cfg.max_mountpoints = 1024;
  if (cfg.max_nodes > VMQG_MAX_NODES || cfg.local_node >= cfg.max_nodes) return VMQG_E_LIMIT;
  static_assert(VMQG_MAX_NODES == kMaxNodes, "the wave tier's node set is kMaxNodes bits");
  if (cfg.max_mountpoints > kMaxMountpoints) return VMQG_E_LIMIT;
  replica = (cfg.flags & VMQG_CFG_REPLICA) != 0;
  // reserved words
  for (const char* s : {"+", "#", "$share"}) intern(reinterpret_cast<const uint8_t*>(s), strlen(s), true);
  if (!replica) {
    paths.resize(cfg.max_mountpoints);
    for (uint32_t m = 0; m < cfg.max_mountpoints; m++) {
      paths[m].parent = kNone; paths[m].word = kNone; paths[m].mp = m; paths[m].depth = 0;
    }
    rebuild(0);
  }
  if (cfg.device >= 0) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || cfg.device >= n) return VMQG_E_DEVICE;
    device = cfg.device;
    if (hipSetDevice(device) != hipSuccess) return VMQG_E_DEVICE;
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return VMQG_E_DEVICE;
    if (hipEventCreateWithFlags(&ev_match_done, hipEventDisableTiming) != hipSuccess) return VMQG_E_DEVICE;
    has_device = true;
    if (hipMalloc(&d_status, kStatusBytes) != hipSuccess) return VMQG_E_NOMEM;
    if (hipMemset(d_status, 0, kStatusBytes) != hipSuccess) return VMQG_E_DEVICE;
    // the dedupe mode word the COUNT wave tier writes and the host reads
    // before each call (whether to launch the claim pass)
    if (hipHostMalloc((void**)&h_ddmode, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return VMQG_E_NOMEM;
    h_ddmode[0] = 0;
    h_ddmode[1] = 0;
    if (hipHostGetDevicePointer((void**)&d_ddmode_host, h_ddmode, 0) != hipSuccess) return VMQG_E_DEVICE;
    for (Stage& sg : stage)
      if (hipEventCreateWithFlags(&sg.ev, hipEventDisableTiming) != hipSuccess) return VMQG_E_DEVICE;
    if (hipDeviceGetAttribute(&cu_count, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cu_count < 1)
      cu_count = 256;
    if (!replica) {
      int rc = upload();
      if (rc) return rc;
    }
  }
  return VMQG_OK;
}

// ------------------------------------------------------------ dictionary
uint32_t Engine::intern(const uint8_t* b, size_t n, bool create) {
  const WordDict::Key k = WordDict::key(b, n);
  if (!create) {
    const uint32_t id = dict.find(k);
    return id == WordDict::kVoid ? kUnknownWord : id;
  }
  const uint32_t id = dict.intern(k);
  if (id >= word_refs.size()) {
    const size_t m = std::max<size_t>(1024, (size_t)id * 2);
    word_refs.resize(m, 0);
    word_tag.resize(m, 0);
    word_state.resize(m, 0);
  }
  if (word_state[id] == 2) word_state[id] = 0;   // a released id taken by a new word
  if (word_refs[id] == 0 && id >= 3) word_zero.push_back(id);   // retired at the stage end unless used
  return id;
}

// Stage end: words nothing holds any more are retired: taken out of the
// dictionary at once (a lookup from now on misses them, as a word no filter
// ever had), their ids reserved until a grace period taken after now ends
// (vmqg_dict_release): readers that found them before still hold the ids.
void Engine::retire_words() {
  for (uint32_t w : word_zero) {
    if (word_refs[w] != 0 || word_state[w] != 0) continue;
    dict.erase(w);
    word_tag[w] = dict.retire_token;
    word_state[w] = 1;
    word_retired.push_back(w);
  }
  word_zero.clear();
}

void Engine::collect_released_terms() {
  for (int k = 0; k < 2; k++) {
    term_released[k].clear();
    if (term_mark[k].size() < term_refs[k].size()) term_mark[k].resize(term_refs[k].size(), 0);
    for (uint32_t id : term_cand[k]) {
      if (id < term_refs[k].size() && term_refs[k][id]) continue;
      if (id >= term_mark[k].size()) term_mark[k].resize(std::max<size_t>(1024, (size_t)id * 2), 0);
      if (term_mark[k][id]) continue;
      term_mark[k][id] = 1;
      term_released[k].push_back(id);
    }
    for (uint32_t id : term_released[k]) term_mark[k][id] = 0;
    term_cand[k].clear();
  }
}

// vmqg_dict_release: the ids of words retired before `token` was taken are
// reusable (their texts freed); dictionary tables replaced before it are
// freed.  A retired word an op named again was revived (stage_ops).
void Engine::release_words(uint64_t token) {
  size_t k = 0;
  for (uint32_t w : word_retired) {
    if (word_state[w] != 1) continue;   // revived
    if (word_tag[w] < token) { dict.release(w); word_state[w] = 2; words_released++; continue; }
    word_retired[k++] = w;
  }
  word_retired.resize(k);
  dict.free_tables_before(token);
}

// ------------------------------------------------------------- paths/keys
uint32_t Engine::path_child(uint32_t parent, uint32_t word, bool create) {
  const uint64_t k = ((uint64_t)parent << 32) | word;
  const uint32_t found = path_index.find(k);
  if (found != FlatIndex::kVoid) return found;
  if (!create) return kNone;
  PathInfo pi;
  pi.parent = parent; pi.word = word; pi.mp = paths[parent].mp; pi.depth = paths[parent].depth + 1;
  // MQTT-4.7.2-1 filters: exactly [#], or starting with + (vmq_reg_trie.erl:285-288)
  pi.first_plus = pi.depth == 1 ? (word == kPlus) : paths[parent].first_plus;
  pi.dollar_skip = pi.first_plus || (pi.depth == 1 && word == kHash);
  if (pi.depth > max_depth) max_depth = pi.depth;
  uint32_t id;
  if (!free_paths.empty()) { id = free_paths.back(); free_paths.pop_back(); paths[id] = std::move(pi); }
  else { id = (uint32_t)paths.size(); paths.push_back(std::move(pi)); }
  paths[parent].nchild++;
  word_ref(word);
  path_index.insert(k, id);
  return id;
}

bool Engine::path_chain(uint32_t mp, const uint32_t* w, uint32_t L, bool create, std::vector<uint32_t>& chain) {
  chain.resize(L + 1);
  chain[0] = mp;
  for (uint32_t i = 0; i < L; i++) {
    chain[i + 1] = path_child(chain[i], w[i], create);
    if (chain[i + 1] == kNone) return false;
  }
  return true;
}

static uint64_t topic_hash(uint32_t mp, const uint32_t* w, uint32_t L) {
  uint64_t h = mix64(((uint64_t)mp << 32) | L);
  for (uint32_t i = 0; i < L; i++) h = mix64(h ^ ((uint64_t)w[i] * 0x9E3779B97F4A7C15ull + i));
  return h;
}

// The (MP, Topic) term of an op: the $share prefix is not part of it.
static inline void op_topic(const vmqg_op& op, const uint32_t*& w, uint32_t& L) {
  L = op.nwords;
  if (L >= 3 && w[0] == kShare) { w += 2; L -= 2; }
}

// apply_ops keeps the lookups of later ops in flight while it handles the
// current one: stage 0 (8 ops ahead) prefetches the topic's index slot,
// stage 1 (4 ahead) the topic record it names, stage 2 (2 ahead) the
// topic's words and its local key.  The handlers then find them in cache.
void Engine::prefetch_op(const vmqg_op& op, const uint32_t* w, int stage) {
  uint32_t L;
  op_topic(op, w, L);
  const uint64_t h = topic_hash(op.mountpoint, w, L);
  if (stage == 0) { topic_index.prefetch(h); return; }
  const uint32_t t = topic_index.find(h);   // unverified: a prefetch hint only
  if (t == FlatIndex::kVoid || t >= topics.size()) return;
  const TopicInfo& T = topics[t];
  if (stage == 1) { __builtin_prefetch(&T); return; }
  __builtin_prefetch(T.words.data());
  if (T.local_key != kNone) {
    __builtin_prefetch(&keys[T.local_key]);
    if (!keys[T.local_key].vals.empty()) __builtin_prefetch(keys[T.local_key].vals.data());
  }
}

uint32_t Engine::topic_id(uint32_t mp, const uint32_t* w, uint32_t L, bool create) {
  const uint64_t h = topic_hash(mp, w, L);
  const uint32_t found = topic_index.find(h, [&](uint32_t id) {
    const TopicInfo& t = topics[id];
    return t.mp == mp && t.words.size() == L && std::equal(t.words.begin(), t.words.end(), w);
  });
  if (found != FlatIndex::kVoid) return found;
  if (!create) return kNone;
  TopicInfo t;
  t.mp = mp;
  t.words.assign(w, w + L);
  for (uint32_t i = 0; i < L; i++) if (w[i] == kPlus || w[i] == kHash) t.wild = 1;
  uint32_t id;
  if (!free_topics.empty()) { id = free_topics.back(); free_topics.pop_back(); topics[id] = std::move(t); }
  else { id = (uint32_t)topics.size(); topics.push_back(std::move(t)); }
  for (uint32_t i = 0; i < L; i++) word_ref(w[i]);
  topic_index.insert(h, id);
  return id;
}

static uint32_t new_key(HugeVec<KeyInfo>& keys, std::vector<uint32_t>& free_keys) {
  if (!free_keys.empty()) {
    const uint32_t k = free_keys.back();
    free_keys.pop_back();
    keys[k] = KeyInfo();
    return k;
  }
  keys.emplace_back();
  return (uint32_t)keys.size() - 1;
}

uint32_t Engine::local_key(uint32_t tid, bool create) {
  if (topics[tid].local_key != kNone || !create) return topics[tid].local_key;
  const uint32_t k = new_key(keys, free_keys);
  keys[k].topic_id = tid;
  topics[tid].local_key = k;
  mark_key(k);
  return k;
}

uint32_t Engine::group_key(uint32_t tid, uint32_t group, bool create) {
  const uint64_t gk = ((uint64_t)tid << 32) | group;
  const uint32_t found = group_key_index.find(gk);
  if (found != FlatIndex::kVoid) return found;
  if (!create) return kNone;
  const uint32_t k = new_key(keys, free_keys);
  keys[k].topic_id = tid;
  keys[k].group = group;
  topics[tid].ngroup++;
  word_ref(group);
  group_key_index.insert(gk, k);
  mark_key(k);
  return k;
}

// ------------------------------------------------------------------ mirror
void Engine::touch(uint64_t off, uint64_t bytes) {
  if (full_image) return;
  for (uint64_t c = off >> 4, e = (off + bytes + 15) >> 4; c < e; c++) {
    uint64_t& w = dirty_bits[c >> 6];
    const uint64_t bit = 1ull << (c & 63);
    if (!(w & bit)) { w |= bit; dirty_chunks.push_back(c); }
  }
}

// `node` gained or lost a '#' / '+' edge or its first / last literal edge:
// refresh the child flags cached in its incoming slot (they let the walk
// skip probes that must miss).
void Engine::refresh_incoming_flags(uint32_t node) {
  const PathInfo& P = paths[node];
  if (P.parent == kNone) { mark_path(node); return; }   // a root: its own record carries them (write_path)
  if (P.in_slot == ~0ull) return;
  EdgeSlot& s = region<EdgeSlot>(lay.edge_off)[P.in_slot];
  if (s.flags != P.eflags) {
    s.flags = P.eflags;
    touch(lay.edge_off + P.in_slot * sizeof(EdgeSlot), sizeof(EdgeSlot));
  }
}

// (parent, word) -> child.  Path ids are interned by (parent, word), so the
// edge exists iff the child's in_slot is set (ets:insert of an identical
// #trie{} is a no-op).
void Engine::edge_insert(uint32_t parent, uint32_t word, uint32_t child) {
  if (paths[child].in_slot != ~0ull) return;
  EdgeSlot* t = region<EdgeSlot>(lay.edge_off);
  const uint64_t mask = lay.edge_buckets - 1;
  uint64_t b = edge_hash(parent, word) & mask;
  for (uint64_t i = 0; i < lay.edge_buckets; i++, b = (b + 1) & mask) {
    for (uint32_t j = 0; j < kEdgeSlotsPerBucket; j++) {
      const uint64_t si = b * kEdgeSlotsPerBucket + j;
      EdgeSlot& s = t[si];
      if (s.parent == kEmpty || s.parent == kTomb) {
        if (s.parent == kTomb) edge_tomb--;
        s = EdgeSlot{parent, word, child, paths[child].eflags};
        edge_live++;
        paths[child].in_slot = si;
        touch(lay.edge_off + si * sizeof(EdgeSlot), sizeof(EdgeSlot));
        if (word == kHash || word == kPlus) {
          paths[parent].eflags |= word == kHash ? kHasHash : kHasPlus;
          refresh_incoming_flags(parent);
          if (word == kHash) write_hash_alias(parent);
        } else if (paths[parent].nlit++ == 0) {
          paths[parent].eflags |= kHasWord;
          refresh_incoming_flags(parent);
        }
        return;
      }
    }
  }
}

void Engine::edge_erase(uint32_t parent, uint32_t word, uint32_t child) {
  const uint64_t si = paths[child].in_slot;
  if (si == ~0ull) return;
  EdgeSlot* t = region<EdgeSlot>(lay.edge_off);
  t[si] = EdgeSlot{kTomb, kTomb, kTomb, 0};
  paths[child].in_slot = ~0ull;
  edge_live--; edge_tomb++;
  touch(lay.edge_off + si * sizeof(EdgeSlot), sizeof(EdgeSlot));
  if (word == kHash || word == kPlus) {
    paths[parent].eflags &= ~(word == kHash ? kHasHash : kHasPlus);
    refresh_incoming_flags(parent);
    if (word == kHash) write_hash_alias(parent);
  } else if (--paths[parent].nlit == 0) {
    paths[parent].eflags &= ~kHasWord;
    refresh_incoming_flags(parent);
  }
}

Layout Engine::plan_layout(uint64_t extra_edges, uint32_t scale, bool compact) const {
  Layout L{};
  L.magic = kLayoutMagic;
  L.max_mountpoints = cfg.max_mountpoints;
  L.local_node = cfg.local_node;
  L.max_depth = max_depth;
  uint64_t recs = 0, kl = 0, xw = 0, ex = 0;
  for (auto& k : keys) recs += next_pow2(k.vals.size() ? k.vals.size() : 1);
  for (auto& p : paths) {
    if (!p.filter) continue;
    if (p.nodes.size() >= 2) kl += next_pow2(p.nodes.size());
    uint64_t nh = 0;
    for (auto& e : p.nodes) nh += e.first.group == kNone && e.first.node >= kLowNodes;
    if (nh) kl += next_pow2(nh);
  }
  for (auto& t : topics) {
    const bool has = (t.local_key != kNone && !keys[t.local_key].vals.empty()) || !t.remote.empty();
    if (!has) continue;
    ex++;
    uint64_t nh = 0;
    for (auto& r : t.remote) nh += r.first >= kLowNodes;
    xw += exact_tail_words((uint32_t)t.words.size()) + (nh ? nh + 1 : 0);
  }
  const uint64_t edges_need = edge_live + extra_edges;
  const uint64_t edge_slots = next_pow2(std::max<uint64_t>(4096, std::max<uint64_t>(edges_need * 2, cfg.hint_edges * 2)));
  L.edge_buckets = edge_slots / kEdgeSlotsPerBucket;
  L.node_cap = std::max<uint64_t>({4096, paths.size() + paths.size() / 2, cfg.hint_paths + cfg.max_mountpoints});
  L.key_cap = std::max<uint64_t>({4096, keys.size() + keys.size() / 2, cfg.hint_keys});
  // keylists (multi-key filters, remote nodes >= 64) and exact-topic words:
  // sized from the hints too, so a bulk load does not re-lay the arena out
  L.keylist_cap = std::max<uint64_t>({4096, kl * 2, cfg.hint_keys / 16});
  L.rec_cap = std::max<uint64_t>({16384, recs * 2, cfg.hint_records * 2});
  // exact slots per topic (load <= 0.25): a lookup that misses its bucket's
  // first slot reads a second 64-B slot (or the next bucket) — one more
  // memory request in a probe that is one request otherwise.  R1's COUNT at
  // load 0.49 / 0.24 / 0.12: 336 / 285 / 273 us; D's +10 us (its 8M topics'
  // table 1 -> 2 GB), E's -8 us, A's -2 us (profiles/ab_r05_exact_load/)
  const uint64_t spt = VMQG_EXACT_SLOTS_PER_TOPIC;
  const uint64_t exact_slots = next_pow2(std::max<uint64_t>(4096, std::max<uint64_t>(ex * spt + 1024, cfg.hint_exact * spt)));
  L.exact_buckets = exact_slots / kExactSlotsPerBucket;
  L.exwords_cap = std::max<uint64_t>({16384, xw * 2, cfg.hint_exact});
  // one filter bit per exact slot (8 KiB at least): 2 MB for R1's 16M slots,
  // small enough to stay in L2 next to the walk's lines
  L.exbits_words = std::max<uint64_t>(2048, exact_slots / 32);
  uint64_t o = 0;
  if (!compact && lay.total_bytes) {   // a growth re-layout never shrinks a region
    L.edge_buckets = std::max<uint64_t>(L.edge_buckets, lay.edge_buckets);
    L.node_cap = std::max<uint64_t>(L.node_cap, lay.node_cap);
    L.key_cap = std::max<uint64_t>(L.key_cap, lay.key_cap);
    L.keylist_cap = std::max<uint64_t>(L.keylist_cap, lay.keylist_cap);
    L.rec_cap = std::max<uint64_t>(L.rec_cap, lay.rec_cap);
    L.exact_buckets = std::max<uint64_t>(L.exact_buckets, lay.exact_buckets);
    L.exwords_cap = std::max<uint64_t>(L.exwords_cap, lay.exwords_cap);
    L.exbits_words = std::max<uint64_t>(L.exbits_words, lay.exbits_words);
  }
  L.edge_buckets *= scale; L.node_cap *= scale; L.key_cap *= scale; L.keylist_cap *= scale;
  L.rec_cap *= scale; L.exact_buckets *= scale; L.exwords_cap *= scale; L.exbits_words *= scale;
  L.edge_off = o;    o = align256(o + L.edge_buckets * kEdgeSlotsPerBucket * sizeof(EdgeSlot));
  L.node_off = o;    o = align256(o + 2 * L.node_cap * sizeof(NodeRec));   // records, then '#'-child aliases
  L.keydesc_off = o; o = align256(o + L.key_cap * sizeof(KeyDesc));
  L.keylist_off = o; o = align256(o + L.keylist_cap * sizeof(uint32_t));
  L.rec_off = o;     o = align256(o + L.rec_cap * sizeof(Record));
  L.exact_off = o;   o = align256(o + L.exact_buckets * kExactSlotsPerBucket * sizeof(ExactSlot));
  L.exwords_off = o; o = align256(o + L.exwords_cap * sizeof(uint32_t));
  L.exbits_off = o;  o = align256(o + L.exbits_words * sizeof(uint32_t));
  L.total_bytes = o;
  return L;
}

// Re-lay the arena out from the logical state (tables rehashed without
// tombstones, record/keylist/exword pools compacted).  The next upload
// ships the whole image.
void Engine::rebuild(uint64_t extra_edges, bool compact) {
  std::vector<EdgeSlot> live;
  if (!mirror.empty()) {
    const EdgeSlot* t = region<EdgeSlot>(lay.edge_off);
    for (uint64_t i = 0; i < lay.edge_buckets * kEdgeSlotsPerBucket; i++)
      if (t[i].parent != kEmpty && t[i].parent != kTomb) live.push_back(t[i]);
  }
  for (uint32_t scale = 1;; scale *= 2) {
    edge_live = edge_tomb = 0;
    lay = plan_layout(std::max<uint64_t>(extra_edges, live.size()), scale, compact);
    mirror.assign(lay.total_bytes / 8, 0);
    memset(region<uint8_t>(lay.edge_off), 0xFF, lay.edge_buckets * kEdgeSlotsPerBucket * sizeof(EdgeSlot));
    memset(region<uint8_t>(lay.exact_off), 0xFF, lay.exact_buckets * kExactSlotsPerBucket * sizeof(ExactSlot));
    dirty_bits.assign((lay.total_bytes / 16 + 63) / 64, 0);
    dirty_chunks.clear();
    full_image = true;
    exact_live = exact_tomb = 0;
    rec_top = rec_garbage = kl_top = kl_garbage = xw_top = xw_garbage = 0;
    for (auto& p : paths) { p.in_slot = ~0ull; p.nlit = 0; p.eflags &= ~kHasWord; }   // re-counted below
    for (auto& e : live) edge_insert(e.parent, e.word, e.child);
    for (auto& k : keys) { k.off = 0; k.cap = 0; k.dirty_pos.clear(); }
    for (auto& t : topics) { t.slot = ~0ull; t.words_off = kNone; t.xw_len = 0; }
    for (auto& p : paths) { p.kl_off = 0; p.kl_cap = 0; p.hn_off = 0; p.hn_cap = 0; }
    bool ok = true;
    for (uint32_t k = 0; ok && k < keys.size(); k++) ok = write_key(k);
    for (uint32_t p = 0; ok && p < paths.size(); p++) ok = write_path(p);
    for (uint32_t t = 0; ok && t < topics.size(); t++) ok = write_topic(t);
    if (ok) break;
  }
  for (auto& k : keys) k.dirty = 0;
  for (auto& p : paths) p.dirty = 0;
  for (auto& t : topics) t.dirty = 0;
  dirty_keys.clear(); dirty_paths.clear(); dirty_topics.clear();
  rebuilds++;
}

// An empty subscriber-list key is dropped: vmq_reg_trie deletes the
// vmq_trie_subs row of its last value (vmq_reg_trie.erl:472-496), and a later
// subscription makes a new key.  The paths and the exact slot that named it
// are rewritten in the same flush (marked here), so no device record keeps
// the id, which the next key may take.
void Engine::free_key(uint32_t k) {
  KeyInfo& K = keys[k];
  const uint32_t tid = K.topic_id;
  TopicInfo& t = topics[tid];
  if (K.group != kNone) {
    group_key_index.erase(((uint64_t)tid << 32) | K.group, k);
    t.ngroup--;
    word_unref(K.group);
  } else if (t.local_key == k) {
    t.local_key = kNone;
  }
  rec_garbage += K.cap;
  K.vals = std::vector<Record>();
  K.idx.reset();
  K.dirty_pos = std::vector<uint32_t>();
  K.off = K.cap = 0;
  K.topic_id = kNone;
  K.group = kNone;
  KeyDesc* kd = region<KeyDesc>(lay.keydesc_off) + k;
  if (k < lay.key_cap && (kd->off | kd->count)) {
    kd->off = 0; kd->count = 0;
    touch(lay.keydesc_off + (uint64_t)k * sizeof(KeyDesc), sizeof(KeyDesc));
  }
  free_keys.push_back(k);
  reclaimed_keys++;
  if (t.path != kNone) mark_path(t.path);
  mark_topic(tid);
}

// After the flush: paths and topics nothing holds any more are dropped
// (their ids reused), so the host tables and the arena follow the live set
// as vmq_reg_trie's ETS tables do (trie_delete_path / del_trie_subs /
// del_remote_subscriber delete rows, vmq_reg_trie.erl:417-441, 472-539).
//   a path: not a root, no vmq_trie_node record, no incoming edge, no child
//     path, no vmq_trie_topic entry — its parent may follow;
//   a topic: no local key, no group key, no remote refcounts, no trie path,
//     no exact slot.
// A dropped path's device record is cleared (no edge leads to it: no walk
// reads it; the clear keeps the image exact for a reused id).
void Engine::reclaim() {
  // the stage's dirty paths and topics (as flush_incremental found them),
  // plus the paths and topics free_key marked (already in those lists)
  std::vector<uint32_t> work, tw;
  work.swap(reclaim_paths);
  tw.swap(reclaim_topics);
  for (uint32_t p : dirty_paths) work.push_back(p);   // a flush without re-layout leaves them listed
  for (uint32_t t : dirty_topics) tw.push_back(t);
  const NodeRec empty{0, kNone, 0, 0, 0, 0, 0, 0};
  while (!work.empty()) {
    const uint32_t p = work.back();
    work.pop_back();
    PathInfo& P = paths[p];
    if (p < cfg.max_mountpoints || P.parent == kNone || P.rec || P.filter || P.in_slot != ~0ull || P.nchild ||
        !P.nodes.empty())
      continue;
    path_index.erase(((uint64_t)P.parent << 32) | P.word, p);
    const uint32_t parent = P.parent;
    paths[parent].nchild--;
    work.push_back(parent);
    if (P.topic_id != kNone) {
      topics[P.topic_id].path = kNone;
      tw.push_back(P.topic_id);
    }
    kl_garbage += P.kl_cap + P.hn_cap;
    word_unref(P.word);
    if (p < lay.node_cap) {
      NodeRec* nr = region<NodeRec>(lay.node_off);
      if (memcmp(&nr[p], &empty, sizeof empty)) { nr[p] = empty; touch(lay.node_off + (uint64_t)p * sizeof(NodeRec), sizeof(NodeRec)); }
      if (memcmp(&nr[lay.node_cap + p], &empty, sizeof empty)) {
        nr[lay.node_cap + p] = empty;
        touch(lay.node_off + (lay.node_cap + p) * sizeof(NodeRec), sizeof(NodeRec));
      }
    }
    const uint8_t was_dirty = P.dirty;
    P = PathInfo();
    P.parent = kNone; P.word = kNone; P.mp = kNone; P.depth = 0;
    P.dirty = was_dirty;   // still listed in dirty_paths: the stage clears the flag
    free_paths.push_back(p);
    reclaimed_paths++;
  }
  for (uint32_t t : tw) {
    TopicInfo& T = topics[t];
    if (T.words.empty() && T.mp == kNone) continue;   // dropped already (listed twice)
    if (T.local_key != kNone || T.ngroup || !T.remote.empty() || T.path != kNone || T.slot != ~0ull) continue;
    topic_index.erase(topic_hash(T.mp, T.words.data(), (uint32_t)T.words.size()), t);
    for (uint32_t w : T.words) word_unref(w);
    xw_garbage += T.xw_len;
    const uint8_t was_dirty = T.dirty;
    T = TopicInfo();
    T.mp = kNone;
    T.dirty = was_dirty;
    free_topics.push_back(t);
    reclaimed_topics++;
  }
}

// Mountpoint m's root is path m (a walk starts at path pub.mountpoint), so
// the roots are the first cfg.max_mountpoints path ids.  In vmq_reg_trie a
// mountpoint is only part of every key (vmq_reg_trie.erl:60, 279-281, 320):
// there is no limit.  A change on a mountpoint past the root range grows it
// (doubling): every other path id moves up by the growth, the edges in the
// mirror are renumbered, and the arena is re-laid out (a full image: the
// next commit ships it, replicas reload it).  Called at the start of a stage,
// before any handler has marked anything dirty.
void Engine::grow_mountpoints(uint32_t need) {
  const uint32_t old = cfg.max_mountpoints;
  uint64_t m = old ? old : 1;
  while (m < need) m *= 2;
  m = std::min<uint64_t>(m, kMaxMountpoints);
  const uint32_t shift = (uint32_t)m - old;
  if (!shift) return;
  auto mv = [old, shift](uint32_t p) { return p == kNone || p < old ? p : p + shift; };
  // the live edges, renumbered where rebuild() collects them
  if (!mirror.empty()) {
    EdgeSlot* t = region<EdgeSlot>(lay.edge_off);
    for (uint64_t i = 0; i < lay.edge_buckets * kEdgeSlotsPerBucket; i++)
      if (t[i].parent != kEmpty && t[i].parent != kTomb) { t[i].parent = mv(t[i].parent); t[i].child = mv(t[i].child); }
  }
  paths.insert(paths.begin() + old, shift, PathInfo{});
  for (uint32_t r = old; r < (uint32_t)m; r++) {
    paths[r].parent = kNone; paths[r].word = kNone; paths[r].mp = r; paths[r].depth = 0;
  }
  FlatIndex idx;
  idx.reserve(paths.size());
  for (uint64_t p = m; p < paths.size(); p++) {
    if (paths[p].parent == kNone) continue;   // a reclaimed id (free_paths)
    paths[p].parent = mv(paths[p].parent);
    idx.insert(((uint64_t)paths[p].parent << 32) | paths[p].word, (uint32_t)p);
  }
  path_index = std::move(idx);
  for (auto& t : topics) t.path = mv(t.path);
  for (auto& p : dirty_paths) p = mv(p);
  for (auto& p : free_paths) p = mv(p);
  cfg.max_mountpoints = (uint32_t)m;
  rebuild(0);
}

bool Engine::write_key(uint32_t k) {
  KeyInfo& K = keys[k];
  if (k >= lay.key_cap) return false;
  const uint64_t n = K.vals.size();
  Record* recs = region<Record>(lay.rec_off);
  if (n > K.cap) {   // relocate: the whole list is written at its new range
    const uint64_t cap = next_pow2(n);
    if (rec_top + cap > lay.rec_cap) return false;
    rec_garbage += K.cap;
    K.off = rec_top; K.cap = cap; rec_top += cap;
    memcpy(recs + K.off, K.vals.data(), n * sizeof(Record));
    touch(lay.rec_off + K.off * sizeof(Record), n * sizeof(Record));
  } else {           // in place: only the slots insert / swap-remove changed
    for (uint32_t pos : K.dirty_pos) {
      if (pos >= n) continue;
      recs[K.off + pos] = K.vals[pos];
      touch(lay.rec_off + (K.off + pos) * sizeof(Record), sizeof(Record));
    }
  }
  K.dirty_pos.clear();
  KeyDesc* kd = region<KeyDesc>(lay.keydesc_off) + k;
  kd->off = (uint32_t)K.off; kd->count = (uint32_t)n;
  touch(lay.keydesc_off + (uint64_t)k * sizeof(KeyDesc), sizeof(KeyDesc));
  return true;
}

bool Engine::write_path(uint32_t p) {
  if (p >= lay.node_cap) return false;
  PathInfo& P = paths[p];
  NodeRec r{0, kNone, 0, 0, 0, 0, 0, 0};
  uint32_t flags = 0;
  if (P.rec) flags |= kNodeRec;
  if (P.rec && P.topic_set) flags |= kNodeTopic;
  if (P.filter) flags |= kNodeFilter;
  if (P.dollar_skip) flags |= kNodeDollarSkip;
  if (P.parent == kNone) flags |= (uint32_t)(P.eflags & kHasAll) << kRootFlagShift;
  std::vector<uint32_t> ks;
  std::vector<uint32_t>& high = scratch_u32;
  high.clear();
  uint64_t rmask = 0;
  if (P.filter) {
    // match_/3 (:301-303): one candidate per node-list entry; a key that does
    // not exist in vmq_trie_subs contributes nothing (lookup_subs -> [])
    for (auto& e : P.nodes) {
      if (e.first.group != kNone) {                                                   // :68-72
        const uint32_t k = group_key(P.topic_id, e.first.group, false);
        if (k != kNone) ks.push_back(k);
      } else if (e.first.node == cfg.local_node) {                                     // :73-77
        const uint32_t k = local_key(P.topic_id, false);
        if (k != kNone) ks.push_back(k);
      } else if (e.first.node < kLowNodes) {
        rmask |= 1ull << e.first.node;                                                 // :78-84
      } else {
        high.push_back(e.first.node);
      }
    }
  }
  if (!high.empty()) {
    std::sort(high.begin(), high.end());
    if (!write_high_list(P.hn_off, P.hn_cap, high)) return false;
    flags |= kNodeHigh;
    r.hi_off = P.hn_off;
    r.hi_cnt = (uint32_t)high.size();
  }
  if (ks.size() == 1) {
    r.key = ks[0];
    r.off0 = (uint32_t)keys[ks[0]].off;
    r.cnt0 = (uint32_t)keys[ks[0]].vals.size();
  } else if (ks.size() >= 2) {
    if (ks.size() > P.kl_cap) {   // grow: a new range; the old one becomes garbage
      const uint64_t cap = next_pow2(ks.size());
      if (kl_top + cap > lay.keylist_cap) return false;
      kl_garbage += P.kl_cap;
      P.kl_off = (uint32_t)kl_top;
      P.kl_cap = (uint32_t)cap;
      kl_top += cap;
    }
    r.key = P.kl_off;
    uint32_t* kl = region<uint32_t>(lay.keylist_off) + P.kl_off;
    for (size_t i = 0; i < ks.size(); i++) {
      if (kl[i] != ks[i]) { kl[i] = ks[i]; touch(lay.keylist_off + (P.kl_off + i) * 4, 4); }
    }
  }
  r.meta = flags | ((uint32_t)std::min<size_t>(ks.size(), 0xFFFFFF) << 8);
  r.rmask_lo = (uint32_t)rmask; r.rmask_hi = (uint32_t)(rmask >> 32);
  *(region<NodeRec>(lay.node_off) + p) = r;
  touch(lay.node_off + (uint64_t)p * sizeof(NodeRec), sizeof(NodeRec));
  if (P.word == kHash && P.parent != kNone) write_hash_alias(P.parent);
  return true;
}

// Record slot node_cap + parent holds a copy of the record of parent's '#'
// child while the edge (parent, '#') exists, else an empty record: the walk
// reads it for a node whose cached flags say it has a '#' edge (and for the
// roots, always) instead of probing the edge table first (a '#' path is a
// leaf, so its record is all the walk needs of it).
void Engine::write_hash_alias(uint32_t parent) {
  if (parent >= lay.node_cap) return;
  const uint32_t c = path_child(parent, kHash, false);
  NodeRec r{0, kNone, 0, 0, 0, 0, 0, 0};
  if (c != kNone && c < lay.node_cap && paths[c].in_slot != ~0ull) r = region<NodeRec>(lay.node_off)[c];
  NodeRec* dst = region<NodeRec>(lay.node_off) + lay.node_cap + parent;
  if (memcmp(dst, &r, sizeof(r)) != 0) {
    *dst = r;
    touch(lay.node_off + (lay.node_cap + parent) * sizeof(NodeRec), sizeof(NodeRec));
  }
}

uint64_t Engine::exact_fp(const TopicInfo& t) const {
  uint64_t s = 0;
  for (uint32_t i = 0; i < t.words.size(); i++) s += fp_word(t.words[i], i);
  return fp_final(s, t.mp, (uint32_t)t.words.size());
}

// A remote-node list (nodes >= 64, sorted) in the keylist pool, in place
// when its range has room, else at a fresh range (the old one is garbage).
bool Engine::write_high_list(uint32_t& off, uint32_t& cap, const std::vector<uint32_t>& nodes) {
  if (nodes.size() > cap) {
    const uint64_t c = next_pow2(nodes.size());
    if (kl_top + c > lay.keylist_cap) return false;
    kl_garbage += cap;
    off = (uint32_t)kl_top;
    cap = (uint32_t)c;
    kl_top += c;
  }
  uint32_t* kl = region<uint32_t>(lay.keylist_off) + off;
  for (size_t i = 0; i < nodes.size(); i++) {
    if (kl[i] != nodes[i]) { kl[i] = nodes[i]; touch(lay.keylist_off + (uint64_t)(off + i) * 4, 4); }
  }
  return true;
}

// The exact-table slot of one (MP, Topic): the `{Topic, node()}` candidate
// (its local key's records) and vmq_trie_remote_subs (remote nodes: < 64 in
// the slot's mask, the others listed in exwords).  Wildcard topics get one
// too (fold/4 looks the Topic word list up as given, :62, :514-520), without
// a filter bit: only a publish holding a '+' / '#' word can equal them.
bool Engine::write_topic(uint32_t ti) {
  TopicInfo& t = topics[ti];
  const bool local = t.local_key != kNone && !keys[t.local_key].vals.empty();
  const bool has = local || !t.remote.empty();
  ExactSlot* tab = region<ExactSlot>(lay.exact_off);
  if (!has) {
    if (t.slot != ~0ull) {
      ExactSlot& s = tab[t.slot];
      s.nwords = kTomb;
      touch(lay.exact_off + t.slot * sizeof(ExactSlot), 16);
      t.slot = ~0ull;
      xw_garbage += t.xw_len;
      t.words_off = kNone;
      t.xw_len = 0;
      exact_live--; exact_tomb++;
    }
    return true;
  }
  uint64_t rmask = 0;
  std::vector<uint32_t>& high = scratch_u32;
  high.clear();
  for (auto& r : t.remote) {
    if (r.first < kLowNodes) rmask |= 1ull << r.first;
    else high.push_back(r.first);
  }
  if (high.size() > 1) std::sort(high.begin(), high.end());
  const uint32_t L = (uint32_t)t.words.size();
  const uint32_t tail = exact_tail_words(L);
  const uint32_t need = tail + (high.empty() ? 0 : 1 + (uint32_t)high.size());
  const bool fresh = t.slot == ~0ull;
  if (fresh && (exact_live + exact_tomb + 1) * 10 > lay.exact_buckets * kExactSlotsPerBucket * 7) return false;
  if (need > t.xw_len) {   // (re)place the words beyond the inline ones [+ the high list]
    if (xw_top + need > lay.exwords_cap) return false;
    xw_garbage += t.xw_len;
    t.words_off = (uint32_t)xw_top;
    t.xw_len = need;
    uint32_t* xw = region<uint32_t>(lay.exwords_off) + xw_top;
    if (tail) {
      memcpy(xw, t.words.data() + kExactInline, tail * 4);
      touch(lay.exwords_off + xw_top * 4, (uint64_t)tail * 4);
    }
    xw_top += need;
  }
  if (!high.empty()) {
    uint32_t* hl = region<uint32_t>(lay.exwords_off) + t.words_off + tail;
    hl[0] = (uint32_t)high.size();
    memcpy(hl + 1, high.data(), high.size() * 4);
    touch(lay.exwords_off + ((uint64_t)t.words_off + tail) * 4, (1 + high.size()) * 4);
  }
  const uint64_t fp = exact_fp(t);
  if (fresh) {
    const uint64_t mask = lay.exact_buckets - 1;
    uint64_t b = fp & mask;
    for (;;) {
      uint64_t found = ~0ull;
      for (uint32_t j = 0; j < kExactSlotsPerBucket; j++) {
        ExactSlot& s = tab[b * kExactSlotsPerBucket + j];
        if (s.nwords == kEmpty || s.nwords == kTomb) { found = b * kExactSlotsPerBucket + j; break; }
      }
      if (found != ~0ull) {
        if (tab[found].nwords == kTomb) exact_tomb--;
        exact_live++;
        t.slot = found;
        if (!t.wild) {
          const uint64_t bit = exbit_of(fp, lay.exbits_words * 32);
          uint32_t* xb = region<uint32_t>(lay.exbits_off) + (bit >> 5);
          if (!(*xb & (1u << (bit & 31)))) {
            *xb |= 1u << (bit & 31);
            touch(lay.exbits_off + (bit >> 5) * 4, 4);
          }
        }
        break;
      }
      b = (b + 1) & mask;
    }
  }
  ExactSlot s{};
  s.fp = fp;
  s.nwords = L | (high.empty() ? 0u : kExactHigh);
  s.words_off = need ? t.words_off : kNone;
  s.off = local ? (uint32_t)keys[t.local_key].off : 0;
  s.count = local ? (uint32_t)keys[t.local_key].vals.size() : 0;
  s.rmask = rmask;
  s.mp = t.mp;
  for (uint32_t i = 0; i < L && i < kExactInline; i++) s.w[i] = t.words[i];
  if (opt_exact_one && L <= kExactOneMaxWords && s.count == 1) {   // the one record inline (keys are written first)
    s.nwords |= kExactOne;
    memcpy(&s.w[kExactOneMaxWords], &keys[t.local_key].vals[0], sizeof(Record));
  }
  ExactSlot& d = tab[t.slot];
  // an update changes the first half (records, remote nodes) and, for a
  // short topic, the inline record
  const size_t upd = L <= kExactOneMaxWords ? sizeof(ExactSlot) : 32;
  if (fresh) {
    d = s;
    touch(lay.exact_off + t.slot * sizeof(ExactSlot), sizeof(ExactSlot));
  } else if (memcmp(&d, &s, upd) != 0) {
    memcpy(&d, &s, upd);
    touch(lay.exact_off + t.slot * sizeof(ExactSlot), upd);
  }
  return true;
}

bool Engine::flush_incremental() {
  // keys first (record ranges), then the paths and exact slots that inline them
  for (size_t i = 0; i < dirty_keys.size(); i++) {
    if (i + 4 < dirty_keys.size()) __builtin_prefetch(&keys[dirty_keys[i + 4]]);
    if (i + 2 < dirty_keys.size()) {
      const KeyInfo& K = keys[dirty_keys[i + 2]];
      if (K.topic_id != kNone) __builtin_prefetch(&topics[K.topic_id]);
      __builtin_prefetch(region<KeyDesc>(lay.keydesc_off) + dirty_keys[i + 2]);
    }
    const uint32_t k = dirty_keys[i];
    if (keys[k].topic_id == kNone) continue;   // dropped (free_key): its rows were cleared there
    if (!write_key(k)) return false;
    const TopicInfo& t = topics[keys[k].topic_id];
    if (t.path != kNone) mark_path(t.path);
    if (keys[k].group == kNone) mark_topic(keys[k].topic_id);
  }
  for (size_t i = 0; i < dirty_paths.size(); i++) if (!write_path(dirty_paths[i])) return false;
  const ExactSlot* tab = region<ExactSlot>(lay.exact_off);
  for (size_t i = 0; i < dirty_topics.size(); i++) {
    if (i + 4 < dirty_topics.size()) __builtin_prefetch(&topics[dirty_topics[i + 4]]);
    if (i + 2 < dirty_topics.size()) {
      const TopicInfo& T = topics[dirty_topics[i + 2]];
      if (T.slot != ~0ull) __builtin_prefetch(&tab[T.slot]);
      if (T.local_key != kNone) __builtin_prefetch(&keys[T.local_key]);
    }
    if (!write_topic(dirty_topics[i])) return false;
  }
  return true;
}

// ------------------------------------------------------- state machine
// add_and_inc/2 (:409-415) and rem_and_dec/2 (:399-407)
template <class K>
static void add_and_inc(std::vector<std::pair<K, int64_t>>& v, const K& n) {
  for (auto& e : v) if (e.first == n) { e.second++; return; }
  v.insert(v.begin(), {n, 1});
}
template <class K>
static void rem_and_dec(std::vector<std::pair<K, int64_t>>& v, const K& n) {
  for (size_t i = 0; i < v.size(); i++)
    if (v[i].first == n) { if (v[i].second == 1) v.erase(v.begin() + i); else v[i].second--; return; }
}

static bool contains_wildcard(const uint32_t* w, uint32_t L) {   // vmq_topic.erl:91-95
  for (uint32_t i = 0; i < L; i++) if (w[i] == kPlus) return true;
  return L > 0 && w[L - 1] == kHash;
}

// trie_add_path/2 (:340-356)
void Engine::trie_add_path(uint32_t parent, uint32_t word, uint32_t child) {
  PathInfo& P = paths[parent];
  if (P.rec) {
    if (paths[child].in_slot == ~0ull) {
      P.ec++;
      mark_path(parent);
      edge_insert(parent, word, child);
    }
  } else {
    P.rec = 1; P.ec = 1; P.topic_set = 0;
    n_trie_nodes++;
    mark_path(parent);
    edge_insert(parent, word, child);
  }
}

// add_complex_topic/4 (:318-337)
void Engine::add_complex_topic(uint32_t mp, const uint32_t* w, uint32_t L, Nog nog, bool wildcard) {
  if (!wildcard) return;
  std::vector<uint32_t> chain;
  path_chain(mp, w, L, true, chain);
  const uint32_t p = chain[L];
  if (paths[p].topic_id == kNone) {
    paths[p].topic_id = topic_id(mp, w, L, true);
    topics[paths[p].topic_id].path = p;
  }
  PathInfo& P = paths[p];
  if (!P.filter) { P.filter = 1; P.total = 1; P.nodes.assign(1, {nog, 1}); n_trie_topics++; }  // :321-323
  else { add_and_inc(P.nodes, nog); P.total++; }                                                  // :324-326
  mark_path(p);
  if (P.rec && P.topic_set) return;                                                                // :330-331
  for (uint32_t i = 0; i < L; i++) trie_add_path(chain[i], w[i], chain[i + 1]);                  // :334
  PathInfo& Q = paths[p];
  if (!Q.rec) n_trie_nodes++;
  Q.rec = 1; Q.ec = 0; Q.topic_set = 1;   // :336 — fresh record, edge_count 0 (Q1)
  mark_path(p);
}

// trie_delete/2 (:417-425) + trie_delete_path/2 (:427-441)
void Engine::trie_delete(uint32_t p, const std::vector<uint32_t>& chain, const uint32_t* w, uint32_t L) {
  PathInfo& P = paths[p];
  if (!(P.rec && P.ec == 0)) return;
  P.rec = 0; P.topic_set = 0;
  n_trie_nodes--;
  mark_path(p);
  for (int64_t i = (int64_t)L - 1; i >= 0; i--) {
    const uint32_t parent = chain[i];
    edge_erase(parent, w[i], chain[i + 1]);
    PathInfo& Q = paths[parent];
    if (!Q.rec) return;                                  // :439-440
    if (Q.ec == 1 && !Q.topic_set) {                     // :434-436
      Q.rec = 0; n_trie_nodes--; mark_path(parent);
      continue;
    }
    Q.ec--; mark_path(parent);                           // :437-438
    return;
  }
}

// del_complex_topic/4 (:385-397)
void Engine::del_complex_topic(uint32_t mp, const uint32_t* w, uint32_t L, Nog nog, bool wildcard) {
  if (!wildcard) return;
  std::vector<uint32_t> chain;
  if (!path_chain(mp, w, L, false, chain)) return;
  const uint32_t p = chain[L];
  PathInfo& P = paths[p];
  if (!P.filter) return;
  if (P.total > 1) { rem_and_dec(P.nodes, nog); P.total--; mark_path(p); }           // :389-391
  else if (P.total == 1) {                                                            // :392-394
    P.filter = 0; P.total = 0; P.nodes.clear(); n_trie_topics--; mark_path(p);
    trie_delete(p, chain, w, L);
  }
}

// insert_trie_subs/2 (:448-464)
void Engine::insert_trie_subs(uint32_t key, const Record& v) {
  KeyInfo& K = keys[key];
  const size_t n = K.vals.size();
  RecordEq eq;
  if (n == 1 && eq(K.vals[0], v)) return;                     // :453-455 duplicate
  if (n >= 2) {
    if (K.idx) { if (K.idx->count(v)) return; }
    else for (auto& x : K.vals) if (eq(x, v)) return;         // fanout set: no duplicates
  }
  if (n == 0) n_subs_objects++;                               // :451-452
  if (n == 1) n_fanout += 2;                                  // :458-463 promote both
  else if (n >= 2) n_fanout++;                                // :456-457
  K.vals.push_back(v);
  record_in(v);
  K.dirty_pos.push_back((uint32_t)K.vals.size() - 1);
  if (!K.idx && K.vals.size() > 32) {
    K.idx.reset(new std::unordered_map<Record, uint32_t, RecordHash, RecordEq>());
    for (uint32_t i = 0; i < K.vals.size(); i++) (*K.idx)[K.vals[i]] = i;
  } else if (K.idx) {
    (*K.idx)[v] = (uint32_t)K.vals.size() - 1;
  }
  mark_key(key);
}

// del_trie_subs/2 (:472-496)
void Engine::del_trie_subs(uint32_t key, const Record& v) {
  KeyInfo& K = keys[key];
  const size_t n = K.vals.size();
  if (n == 0) return;                                         // :474-476
  if (n == 1) {                                               // :494-495 value-blind (Q3)
    record_out(K.vals[0]);
    K.vals.clear();
    n_subs_objects--;
    mark_key(key);
    return;
  }
  // :477-493 fanout: delete the object, fold back when one remains
  size_t pos = ~(size_t)0;
  if (K.idx) { auto it = K.idx->find(v); if (it != K.idx->end()) pos = it->second; }
  else { RecordEq eq; for (size_t i = 0; i < n; i++) if (eq(K.vals[i], v)) { pos = i; break; } }
  if (pos == ~(size_t)0) return;
  record_out(K.vals[pos]);
  if (K.idx) {
    K.idx->erase(v);
    if (pos != n - 1) { K.vals[pos] = K.vals[n - 1]; (*K.idx)[K.vals[pos]] = (uint32_t)pos; }
  } else if (pos != n - 1) {
    K.vals[pos] = K.vals[n - 1];
  }
  if (pos != n - 1) K.dirty_pos.push_back((uint32_t)pos);
  K.vals.pop_back();
  if (n - 1 == 1) n_fanout -= 2; else n_fanout -= 1;
  mark_key(key);
}

// handle_add_event/2 (:253-264)
void Engine::handle_add(const vmqg_op& op, const uint32_t* w) {
  const uint32_t L = op.nwords, mp = op.mountpoint;
  if (L >= 2 && w[0] == kShare) {                                  // :253-256
    const uint32_t G = w[1];
    add_complex_topic(mp, w + 2, L - 2, Nog{op.node, G}, true);
    const uint32_t tid = topic_id(mp, w + 2, L - 2, true);
    const uint32_t k = group_key(tid, G, true);                    // add_subscriber_group :443-446
    insert_trie_subs(k, Record{(VMQG_EMIT_GROUP << 24) | op.node, G, op.subscriber, op.subinfo});
    return;
  }
  const bool wc = contains_wildcard(w, L);
  add_complex_topic(mp, w, L, Nog{op.node, kNone}, wc);
  const uint32_t tid = topic_id(mp, w, L, true);
  if (op.node == cfg.local_node) {                                 // :257-260
    const uint32_t k = local_key(tid, true);                       // add_subscriber :498-501
    insert_trie_subs(k, Record{(VMQG_EMIT_LOCAL << 24) | op.node, kNone, op.subscriber, op.subinfo});
    mark_topic(tid);
  } else {                                                         // :261-264, add_remote_subscriber :503-512
    TopicInfo& t = topics[tid];
    if (t.remote.empty()) n_remote_keys++;
    add_and_inc(t.remote, op.node);
    mark_topic(tid);
  }
}

// handle_delete_event/2 (:266-277)
void Engine::handle_delete(const vmqg_op& op, const uint32_t* w) {
  const uint32_t L = op.nwords, mp = op.mountpoint;
  if (L >= 2 && w[0] == kShare) {
    const uint32_t G = w[1];
    del_complex_topic(mp, w + 2, L - 2, Nog{op.node, G}, true);
    const uint32_t tid = topic_id(mp, w + 2, L - 2, false);
    if (tid == kNone) return;
    const uint32_t k = group_key(tid, G, false);                   // del_subscriber_group :467-470
    if (k != kNone) del_trie_subs(k, Record{(VMQG_EMIT_GROUP << 24) | op.node, G, op.subscriber, op.subinfo});
    return;
  }
  del_complex_topic(mp, w, L, Nog{op.node, kNone}, contains_wildcard(w, L));
  const uint32_t tid = topic_id(mp, w, L, false);
  if (tid == kNone) return;
  if (op.node == cfg.local_node) {
    const uint32_t k = local_key(tid, false);                      // del_subscriber :522-525
    if (k != kNone) del_trie_subs(k, Record{(VMQG_EMIT_LOCAL << 24) | op.node, kNone, op.subscriber, op.subinfo});
    mark_topic(tid);
  } else {                                                         // del_remote_subscriber :527-539
    TopicInfo& t = topics[tid];
    if (t.remote.empty()) return;
    rem_and_dec(t.remote, op.node);
    if (t.remote.empty()) n_remote_keys--;
    mark_topic(tid);
  }
}

int Engine::apply_ops(const vmqg_op* ops, size_t n, const uint32_t* words, size_t nwords) {
  const int rc = stage_ops(ops, n, words, nwords);
  if (rc && !staged) return rc;   // rejected before any change
  const int rc2 = commit();
  return rc ? rc : rc2;
}

// The host half of an apply: the state machine, the mirror, the patch list,
// the readers' record buffer.  Runs while match calls are queued and
// running (they read only the device side: dlay, the arena, scratch).
int Engine::stage_ops(const vmqg_op* ops, size_t n, const uint32_t* words, size_t nwords) {
  if (replica) return VMQG_E_STATE;
  // the previous stage is not committed yet (unless its commit failed: this
  // one adds to it, and the next commit ships both as one image)
  if (staged && !commit_failed) return VMQG_E_STATE;
  const auto t0 = std::chrono::steady_clock::now();
  // validate the whole batch before touching state
  uint64_t add_words = 0;
  uint32_t top_mp = 0;
  for (size_t i = 0; i < n; i++) {
    const vmqg_op& o = ops[i];
    if (o.kind != VMQG_OP_ADD && o.kind != VMQG_OP_DEL) return VMQG_E_INVAL;
    if (o.mountpoint >= kMaxMountpoints || o.node >= cfg.max_nodes) return VMQG_E_LIMIT;
    if (o.mountpoint >= top_mp) top_mp = o.mountpoint + 1;
    if (o.nwords == 0 || (uint64_t)o.word_off + o.nwords > nwords) return VMQG_E_INVAL;
    const uint32_t* w = words + o.word_off;
    for (uint32_t j = 0; j < o.nwords; j++)   // ids the dictionary handed out and has not released
      if (w[j] >= dict.id_bound() || (w[j] < word_state.size() && word_state[w[j]] == 2)) return VMQG_E_INVAL;
    // [<<"$share">>, Group] has no topic: triples([]) has no clause (vmq_topic.erl:71)
    if (o.nwords == 2 && w[0] == kShare) return VMQG_E_INVAL;
    // only wildcard and $share topics enter the trie (add_complex_topic/4 :318-319)
    if (o.kind == VMQG_OP_ADD && ((o.nwords >= 3 && w[0] == kShare) || contains_wildcard(w, o.nwords)))
      add_words += o.nwords;
  }
  const bool on_top = staged;
  staged = true;
  staged_epoch = epoch + 1;
  if (on_top) full_image = true;   // the failed commit's changes and this stage's: one image
  // a word retired at an earlier stage end that an op names (interned before
  // it retired, applied after) is put back under its id
  for (size_t i = 0; i < n; i++)
    for (uint32_t j = 0; j < ops[i].nwords; j++) {
      const uint32_t w = words[ops[i].word_off + j];
      if (w < word_state.size() && word_state[w] == 1) { dict.revive(w); word_state[w] = 0; word_zero.push_back(w); }
    }
  if (top_mp > cfg.max_mountpoints) grow_mountpoints(top_mp);   // a new mountpoint past the roots
  // the edge table must absorb every edge this batch could add
  if ((edge_live + edge_tomb + add_words) * 10 > lay.edge_buckets * kEdgeSlotsPerBucket * 7) rebuild(add_words);
  for (size_t i = 0; i < n; i++) {
    if (i + 8 < n) prefetch_op(ops[i + 8], words + ops[i + 8].word_off, 0);
    if (i + 4 < n) prefetch_op(ops[i + 4], words + ops[i + 4].word_off, 1);
    if (i + 2 < n) prefetch_op(ops[i + 2], words + ops[i + 2].word_off, 2);
    const uint32_t* w = words + ops[i].word_off;
    if (ops[i].kind == VMQG_OP_ADD) handle_add(ops[i], w);
    else handle_delete(ops[i], w);
  }
  // subscriber-list keys left empty go before the flush writes the paths and
  // exact slots that name them (vmq_reg_trie deletes such rows,
  // vmq_reg_trie.erl:472-496)
  if (opt_reclaim)
    for (size_t i = 0; i < dirty_keys.size(); i++)
      if (keys[dirty_keys[i]].vals.empty() && keys[dirty_keys[i]].topic_id != kNone) free_key(dirty_keys[i]);
  const bool garbage_heavy = rec_garbage > lay.rec_cap / 2 || kl_garbage > lay.keylist_cap / 2 ||
                             xw_garbage > lay.exwords_cap / 2 ||
                             exact_tomb * 4 > lay.exact_buckets * kExactSlotsPerBucket;
  // the candidates of reclaim(): a re-layout below clears the dirty lists
  if (opt_reclaim) {
    reclaim_paths.assign(dirty_paths.begin(), dirty_paths.end());
    reclaim_topics.assign(dirty_topics.begin(), dirty_topics.end());
  }
  if (garbage_heavy) rebuild(0, true);                // compaction
  else if (!flush_incremental()) rebuild(0);         // growth (writes every dirty item too)
  if (opt_reclaim) {
    reclaim();   // paths and topics nothing holds any more (after their last writes)
    retire_words();
  }
  for (size_t i = 0; i < n; i++) {   // the ops' terms: reported if no record holds them
    term_cand[0].push_back(ops[i].subscriber);
    term_cand[1].push_back(ops[i].subinfo);
  }
  collect_released_terms();
  for (uint32_t k : dirty_keys) keys[k].dirty = 0;
  for (uint32_t p : dirty_paths) paths[p].dirty = 0;
  for (uint32_t t : dirty_topics) topics[t].dirty = 0;
  dirty_keys.clear(); dirty_paths.clear(); dirty_topics.clear();
  lay.max_depth = max_depth;   // replicas size their stacks from the layout
  ops_applied += n;
  stage_patches();
  if (rb_on) publish_records();
  patches_ready = true;
  apply_host_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                       std::chrono::steady_clock::now() - t0).count();
  return VMQG_OK;
}

// The device half: ships what the stage left (serialised with match calls
// by the caller), after which matches see the new tables.
int Engine::commit() {
  if (!staged) return VMQG_OK;
  if (!patches_ready) {   // a stage that ended early (out of memory): ship what it changed
    stage_patches();
    if (rb_on) publish_records();
  }
  const auto t1 = std::chrono::steady_clock::now();
  int rc;
  if (fault_commits) { fault_commits--; rc = VMQG_E_DEVICE; }
  else rc = upload();
  if (rc) {
    // The device tables are those of `epoch` (or, after a device fault, in
    // doubt): the stage stays pending, matches keep answering from `epoch`,
    // and the next commit re-uploads the whole mirror (authoritative).
    commit_failed = true;
    full_image = true;
    apply_upload_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                           std::chrono::steady_clock::now() - t1).count();
    return rc;
  }
  commit_failed = false;
  staged = false;
  patches_ready = false;
  epoch = staged_epoch;
  apply_upload_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                         std::chrono::steady_clock::now() - t1).count();
  return rc;
}

// The pending changes as a patch list (the 16-B dirty chunks) or, after a
// re-layout, the whole image; the record slots among them (rec_epoch, the
// readers' buffers).
void Engine::stage_patches() {
  last_patches.clear();
  rb_changed.clear();
  if (!full_image && dirty_chunks.size() * sizeof(Patch) > lay.total_bytes / 2) {
    // patches would outweigh the image (bulk loads): ship the image instead
    full_image = true;
    std::fill(dirty_bits.begin(), dirty_bits.end(), 0);
    dirty_chunks.clear();
  }
  last_full = full_image;
  if (!full_image) {
    last_patches.reserve(dirty_chunks.size());
    const uint8_t* base = reinterpret_cast<const uint8_t*>(mirror.data());
    static_assert(sizeof(Record) == 16, "a record is one 16-B chunk");
    const uint64_t rec_lo = lay.rec_off >> 4, rec_hi = (lay.rec_off + lay.rec_cap * sizeof(Record)) >> 4;
    for (uint64_t c : dirty_chunks) {
      if (c >= rec_lo && c < rec_hi) {   // a record slot rewritten: older ranges are stale
        rec_epoch = staged_epoch;
        if (rb_on) rb_changed.push_back(c - rec_lo);
      }
      Patch p;
      p.off = c * 16;
      memcpy(p.data, base + p.off, 16);
      last_patches.push_back(p);
      dirty_bits[c >> 6] = 0;
    }
    dirty_chunks.clear();
    patch_bytes += last_patches.size() * sizeof(Patch);
  } else {
    image_bytes += lay.total_bytes;
    rec_epoch = staged_epoch;   // re-laid out: every record may have moved
  }
}

// Left-right update of the readers' record buffers: close the inactive one,
// wait for the readers still on it (rounds more than one apply old: rare),
// bring it to this stage's records, open it and send new readers there.
void Engine::publish_records() {
  const uint32_t cur = rb_active.load(std::memory_order_relaxed);
  RecBuf& b = rb[cur ^ 1];
  b.closed.store(1, std::memory_order_seq_cst);
  if (b.readers.load(std::memory_order_seq_cst) != 0) {
    const auto w0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0; b.readers.load(std::memory_order_seq_cst) != 0; spin++)
      if (spin > 256) sched_yield();
    rb_waits++;
    rb_wait_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                      std::chrono::steady_clock::now() - w0).count();
  }
  const Record* src = region<Record>(lay.rec_off);
  if (last_full || rb_full_next || b.recs.size() != lay.rec_cap) {
    b.recs.assign(src, src + lay.rec_cap);
  } else {
    for (uint64_t i : rb_prev) b.recs[i] = src[i];
    for (uint64_t i : rb_changed) b.recs[i] = src[i];
  }
  b.epoch = staged_epoch;
  b.rec_epoch = rec_epoch;
  b.closed.store(0, std::memory_order_seq_cst);
  rb_active.store(cur ^ 1, std::memory_order_release);
  rb_full_next = last_full;
  rb_prev.swap(rb_changed);
}

// Both buffers from the committed state (the writer's side, before any reader).
void Engine::enable_reader_records() {
  if (rb_on) return;
  const Record* src = region<Record>(lay.rec_off);
  // both copies made before either is committed: an allocation failure
  // (bad_alloc, VMQG_E_NOMEM at the ABI) leaves the option off and nothing changed
  HugeVec<Record> c0(src, src + lay.rec_cap), c1(src, src + lay.rec_cap);
  rb[0].recs.swap(c0);
  rb[1].recs.swap(c1);
  for (RecBuf& b : rb) {
    b.epoch = epoch;
    b.rec_epoch = rec_epoch;
    b.closed.store(0, std::memory_order_seq_cst);
  }
  rb_prev.clear();
  rb_full_next = false;
  rb_on = true;
}

// A reader's pin on a buffer holding the records of epoch `ep` (its round's):
// the active one, else the other while it is still open.  Never waits.
int Engine::records_pin(uint64_t ep, const Record** recs, uint64_t* n, uint32_t* pin) {
  if (!rb_on) return VMQG_E_STATE;
  const uint32_t first = rb_active.load(std::memory_order_acquire);
  for (uint32_t k = 0; k < 2; k++) {
    RecBuf& b = rb[first ^ k];
    b.readers.fetch_add(1, std::memory_order_seq_cst);
    if (!b.closed.load(std::memory_order_seq_cst) && b.rec_epoch <= ep && ep <= b.epoch) {
      *recs = b.recs.data();
      *n = b.recs.size();
      *pin = first ^ k;
      return VMQG_OK;
    }
    b.readers.fetch_sub(1, std::memory_order_release);
  }
  return VMQG_E_STATE;
}

// --------------------------------------------------------------- device
// Ships the staged changes: a patch batch or the whole image.  Patches are
// staged in a ring of pinned buffers and applied by k_apply_patches on the
// context stream after everything queued before (matches included); the
// call does not wait for them.  A full image is copied synchronously
// (re-layouts are rare and the arena may be reallocated).
int Engine::upload() {
  dlay = lay;
  d_trieless = edge_live == 0;   // every subscription exact: COUNT is one exact probe per publish
  if (!has_device) { full_image = false; return VMQG_OK; }
  hipSetDevice(device);
  // tables must not change under a match still reading them (queued on any
  // stream: order_on chains them)
  if (order_on(stream) != VMQG_OK) return VMQG_E_DEVICE;
  if (full_image) {
    last_full = true;   // replicas reload the image too (a retried commit's patches were not shipped)
    if (hipStreamSynchronize(stream) != hipSuccess) return VMQG_E_DEVICE;
    if (d_arena_bytes < lay.total_bytes) {
      if (d_arena) hipFree(d_arena);
      d_arena = nullptr; d_arena_bytes = 0;
      if (hipMalloc(&d_arena, lay.total_bytes) != hipSuccess) return VMQG_E_NOMEM;
      d_arena_bytes = lay.total_bytes;
    }
    if (hipMemcpy(d_arena, mirror.data(), lay.total_bytes, hipMemcpyHostToDevice) != hipSuccess)
      return VMQG_E_DEVICE;
    full_image = false;
    std::fill(dirty_bits.begin(), dirty_bits.end(), 0);
    return VMQG_OK;
  }
  return ship_patches(last_patches);
}

// A patch list through the staging ring onto the context stream (after
// everything queued before it): the primary's own applies, and a replica
// following its primary (vmqg_replica_follow).
int Engine::ship_patches(const std::vector<Patch>& pl) {
  const uint64_t np = pl.size();
  if (np == 0) return VMQG_OK;
  Stage& sg = stage[stage_next];
  stage_next = (stage_next + 1) % kStage;
  if (sg.used) {   // its batch has landed: waits only when the host runs kStage batches ahead of the GPU
    const auto w0 = std::chrono::steady_clock::now();
    if (hipEventSynchronize(sg.ev) != hipSuccess) return VMQG_E_DEVICE;
    apply_wait_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                         std::chrono::steady_clock::now() - w0).count();
  }
  if (sg.cap < np) {
    if (sg.h) hipHostFree(sg.h);
    hipFree(sg.d);
    sg.h = nullptr; sg.d = nullptr; sg.cap = 0;
    const uint64_t cap = next_pow2(np);
    if (hipHostMalloc(&sg.h, cap * sizeof(Patch)) != hipSuccess) return VMQG_E_NOMEM;
    if (hipMalloc(&sg.d, cap * sizeof(Patch)) != hipSuccess) return VMQG_E_NOMEM;
    sg.cap = cap;
  }
  memcpy(sg.h, pl.data(), np * sizeof(Patch));
  if (hipMemcpyAsync(sg.d, sg.h, np * sizeof(Patch), hipMemcpyHostToDevice, stream) != hipSuccess)
    return VMQG_E_DEVICE;
  if (launch_patches(d_arena, sg.d, np, stream) != hipSuccess) return VMQG_E_DEVICE;
  if (hipEventRecord(sg.ev, stream) != hipSuccess) return VMQG_E_DEVICE;
  sg.used = true;
  return VMQG_OK;
}

// A replica context brought to its primary's committed tables (include/vmqg.h
// vmqg_replica_follow): the primary's last patch list when the replica holds
// the epoch just before and that apply shipped patches, else the whole image
// from the primary's host mirror (byte-identical to the primary's device
// arena while no stage is pending).  Runs on the replica's stream after the
// matches already queued there; the replica then answers at the primary's
// epoch, so range results index the primary's record table of that epoch.
int Engine::follow(const Engine& p) {
  if (!replica || p.replica) return VMQG_E_STATE;
  if (!has_device) return VMQG_E_DEVICE;
  const uint64_t pe = p.epoch;
  if (follow_ok && epoch == pe) return VMQG_OK;
  hipSetDevice(device);
  Layout a = p.dlay, b = dlay;
  a.max_depth = b.max_depth = 0;
  const bool same_regions = memcmp(&a, &b, sizeof(a)) == 0;
  const bool patches = follow_ok && epoch + 1 == pe && !p.last_full && same_regions && d_arena;
  follow_ok = false;   // until this call has shipped everything
  if (order_on(stream) != VMQG_OK) return VMQG_E_DEVICE;
  if (patches) {
    const int rc = ship_patches(p.last_patches);
    if (rc) return rc;
  } else {
    // the mirror is ahead of the primary's device tables while its stage is
    // pending (a failed commit): the replica stays at its epoch until then
    if (p.staged) return VMQG_E_STATE;
    const uint64_t bytes = p.dlay.total_bytes;
    if (hipStreamSynchronize(stream) != hipSuccess) return VMQG_E_DEVICE;
    if (d_arena_bytes < bytes) {
      if (d_arena) hipFree(d_arena);
      d_arena = nullptr; d_arena_bytes = 0;
      if (hipMalloc(&d_arena, bytes) != hipSuccess) return VMQG_E_NOMEM;
      d_arena_bytes = bytes;
    }
    if (hipMemcpy(d_arena, p.mirror.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return VMQG_E_DEVICE;
  }
  lay = dlay = p.dlay;
  d_trieless = p.d_trieless;
  epoch = pe;
  follow_ok = true;
  return VMQG_OK;
}

// FNV-style digest of the device arena's first dlay.total_bytes (tests:
// a replica's tables are the primary's byte for byte).
int Engine::arena_digest(uint64_t* out) {
  if (!has_device || !d_arena) return VMQG_E_DEVICE;
  hipSetDevice(device);
  std::vector<uint64_t> h(dlay.total_bytes / 8);
  if (hipStreamSynchronize(stream) != hipSuccess) return VMQG_E_DEVICE;
  if (hipMemcpy(h.data(), d_arena, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return VMQG_E_DEVICE;
  uint64_t d = 0xcbf29ce484222325ull;
  for (uint64_t w : h) d = (d ^ w) * 0x100000001b3ull;
  *out = d ^ dlay.total_bytes;
  return VMQG_OK;
}

// Table changes and matches form one chain across streams (vmqg_chain.h).
int Engine::order_on(hipStream_t st) { return chain_order(ev_match_done, ev_stream, st); }

int Engine::ensure_match_scratch(uint64_t npub, hipStream_t st) {
  if (npub > keycache_cap || npub > deferred_cap) {
    if (hipStreamSynchronize(st) != hipSuccess) return VMQG_E_DEVICE;
    hipFree(d_keycache);
    hipFree(d_deferred);
    d_keycache = nullptr; d_deferred = nullptr;
    keycache_cap = deferred_cap = 0;
    const uint64_t cap = next_pow2(std::max<uint64_t>(npub, 1024));
    // 32-B key cache + kSpillKeys x 8-B spilled keys per publish, then the
    // chunk totals (one per 16, 32 or 64 publishes, + 1), per chunk a 64-bit
    // wide-publish mask, then one fast-pass bit per publish
    // ... then a heavy-publish bucket byte per publish
    if (hipMalloc(&d_keycache, cap * (32 + 8 * 8) + 3 * (cap / 16 + 2) * 8 + (cap / 32 + 2) * 4 + cap + 64) != hipSuccess)
      return VMQG_E_NOMEM;
    // publish lists: retry, whole-wave walks, duplicates, their slots, huge (vmqg_kernels.hip kLists)
    if (hipMalloc(&d_deferred, 5 * cap * sizeof(uint32_t)) != hipSuccess) return VMQG_E_NOMEM;
    keycache_cap = cap;
    deferred_cap = cap;
  }
  // the dedupe table: 2 slots per publish, older calls' slots free by their tag
  const uint64_t slots = next_pow2(std::max<uint64_t>(2 * npub, 4096));
  if (slots > dd_slots) {
    if (hipStreamSynchronize(st) != hipSuccess) return VMQG_E_DEVICE;
    hipFree(d_dd);
    d_dd = nullptr;
    dd_slots = 0;
    if (hipMalloc(&d_dd, slots * 12) != hipSuccess) return VMQG_E_NOMEM;
    if (hipMemsetAsync(d_dd, 0, slots * 12, st) != hipSuccess) return VMQG_E_DEVICE;
    dd_slots = slots;
    dd_tag = 0;
    // the tags restart: output-group slots of older calls must not carry one
    if (d_groups && hipMemsetAsync(d_groups, 0, gs_slots * 256, st) != hipSuccess) return VMQG_E_DEVICE;
  }
  // output groups: 256-B slots, a 16th of the publishes (slots of older calls free by the same tag)
  const uint64_t gslots = next_pow2(std::max<uint64_t>(npub / 16, 1024));
  if (gslots > gs_slots) {
    if (hipStreamSynchronize(st) != hipSuccess) return VMQG_E_DEVICE;
    hipFree(d_groups);
    d_groups = nullptr;
    gs_slots = 0;
    if (hipMalloc(&d_groups, gslots * 256) != hipSuccess) return VMQG_E_NOMEM;
    if (hipMemsetAsync(d_groups, 0, gslots * 256, st) != hipSuccess) return VMQG_E_DEVICE;
    gs_slots = gslots;
  }
  if (++dd_tag >= (1u << 24)) {   // tags are 24 bits: clear before reuse
    if (hipMemsetAsync(d_dd, 0, dd_slots * 12, st) != hipSuccess) return VMQG_E_DEVICE;
    if (hipMemsetAsync(d_groups, 0, gs_slots * 256, st) != hipSuccess) return VMQG_E_DEVICE;
    dd_tag = 1;
  }
  return VMQG_OK;
}

// Look-back granules for `granules` scan tiles; advances the call's tag.
int Engine::ensure_lookback(uint64_t granules, hipStream_t st) {
  if (granules > lookback_cap) {
    if (d_lookback) { hipStreamSynchronize(st); hipFree(d_lookback); }
    d_lookback = nullptr;
    lookback_cap = next_pow2(std::max<uint64_t>(granules, 1024));
    if (hipMalloc(&d_lookback, lookback_cap * 8) != hipSuccess) { lookback_cap = 0; return VMQG_E_NOMEM; }
    if (hipMemsetAsync(d_lookback, 0, lookback_cap * 8, st) != hipSuccess) return VMQG_E_DEVICE;
    lb_tag = 0;
  }
  if (++lb_tag >= (1u << 20)) {   // granule tags are 20 bits: clear before reuse
    if (hipMemsetAsync(d_lookback, 0, lookback_cap * 8, st) != hipSuccess) return VMQG_E_DEVICE;
    lb_tag = 1;
  }
  return VMQG_OK;
}

// Wave tier: each wave has an LDS stack and a global one of o_cap entries.
// A wave pops <= 64 entries and pushes <= 2 per entry, one depth further, so
// its stack holds < 64 entries per trie level plus one step's pushes:
// 64 (depth + 4) entries cannot overflow.
int Engine::ensure_wave_scratch(hipStream_t st) {
  const uint64_t need = std::max<uint64_t>({1024, 64ull * (stack_depth() + 4), o_cap_floor});
  if (need > (1ull << 31)) return VMQG_E_LIMIT;
  if (o_cap >= need && d_ostack) return VMQG_OK;
  // two 256-thread blocks per CU (8 waves) when the stacks fit 256 MiB, at
  // least 64 waves for deep tries
  uint64_t waves = (256ull << 20) / (need * sizeof(uint2));
  waves = std::max<uint64_t>(64, std::min<uint64_t>(8ull * (uint64_t)cu_count, waves)) & ~3ull;
  if (d_ostack) { hipStreamSynchronize(st); hipFree(d_ostack); }
  d_ostack = nullptr; o_waves = 0; o_cap = 0;
  // the stacks, then one bit per stack: borrowed by the fused phases (held
  // only during one walk, so the bitmap is all zero between calls)
  const uint64_t stack_bytes = waves * need * sizeof(uint2);
  if (hipMalloc(&d_ostack, stack_bytes + (waves + 31) / 32 * 4) != hipSuccess) return VMQG_E_NOMEM;
  o_slots = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(d_ostack) + stack_bytes);
  if (hipMemsetAsync(o_slots, 0, (waves + 31) / 32 * 4, st) != hipSuccess) return VMQG_E_DEVICE;
  o_cap = (uint32_t)need;
  o_waves = (uint32_t)waves;
  return VMQG_OK;
}

// The device tables as the last commit left them (dlay): a stage running
// beside this call may be re-laying the host mirror out (lay).
MatchArgs Engine::args_for(const vmqg_pub* pubs, uint32_t npub, const uint32_t* words, uint64_t* offs) const {
  MatchArgs a{};
  a.edges = reinterpret_cast<const EdgeSlot*>(d_arena + dlay.edge_off);
  a.edge_mask = dlay.edge_buckets - 1;
  a.nodes = reinterpret_cast<const NodeRec*>(d_arena + dlay.node_off);
  a.node_cap = dlay.node_cap;
  a.keydesc = reinterpret_cast<const KeyDesc*>(d_arena + dlay.keydesc_off);
  a.key_cap = dlay.key_cap;
  a.keylist = reinterpret_cast<const uint32_t*>(d_arena + dlay.keylist_off);
  a.records = reinterpret_cast<const Record*>(d_arena + dlay.rec_off);
  a.exact = reinterpret_cast<const ExactSlot*>(d_arena + dlay.exact_off);
  a.exact_mask = dlay.exact_buckets - 1;
  a.exwords = reinterpret_cast<const uint32_t*>(d_arena + dlay.exwords_off);
  a.exbits = reinterpret_cast<const uint32_t*>(d_arena + dlay.exbits_off);
  a.exbits_mask = dlay.exbits_words * 32 - 1;
  a.max_mp = (uint32_t)dlay.max_mountpoints;
  a.local_node = (uint32_t)dlay.local_node;
  a.pubs = pubs; a.words = words; a.npub = npub;
  a.offsets = offs;
  a.keycache = d_keycache;
  a.keyspill = reinterpret_cast<uint2*>(static_cast<char*>(d_keycache) + keycache_cap * 32);
  a.chunk = reinterpret_cast<uint64_t*>(static_cast<char*>(d_keycache) + keycache_cap * (32 + 8 * 8));
  a.widemask = a.chunk + (keycache_cap / 16 + 2);
  a.ddmask = a.widemask + (keycache_cap / 16 + 2);
  a.fastdone = reinterpret_cast<uint32_t*>(a.ddmask + (keycache_cap / 16 + 2));
  a.heavybyte = reinterpret_cast<uint8_t*>(a.fastdone + (keycache_cap / 32 + 2));
  a.heavy_min = opt_heavy_min;
  a.trieless = opt_trieless && d_trieless ? 1u : 0u;   // replicas: as their primary's (follow)
  a.dd_key = static_cast<uint64_t*>(d_dd);
  a.dd_rep = reinterpret_cast<uint32_t*>(static_cast<char*>(d_dd) + dd_slots * 8);
  a.dd_mask = dd_slots - 1;
  a.dd_tag = dd_tag;
  // dedupe: 1 on (claim + classify passes, COUNT walks the representatives
  // only), 2 auto: on while the last decision the device wrote to the
  // host-mapped word says so
  // (auto: while off, a probe call runs deduped anyway to measure the
  // repetition — the first call, then after 64, 128, ... up to 8,192 calls
  // while the probes keep finding distinct topics)
  bool claimed = opt_dedupe == 1;
  // auto: a call of fewer than 256 publishes is never deduped nor probed (the
  // device judges only calls of >= 256; a small call would keep a large
  // call's verdict and pay the claim passes for nothing)
  if (opt_dedupe == 2 && npub >= 256) {
    if (*reinterpret_cast<volatile uint32_t*>(h_ddmode)) {
      claimed = true;
      dd_gap = 64;
      dd_next = call_seq + 64;
    } else if (call_seq >= dd_next) {
      claimed = true;
      dd_next = call_seq + dd_gap;
      dd_gap = std::min<uint64_t>(dd_gap * 2, 8192);
    }
  }
  // the exbits filter: on until the device's counters say most lookups pass it
  const uint32_t xm = reinterpret_cast<volatile uint32_t*>(h_ddmode)[1];
  a.exfilter = opt_exfilter == 2 ? (xm == 2u ? 0u : 1u) : opt_exfilter;
  a.dd_force = claimed ? 1u : 0u;
  a.dd_claimed = claimed;
  a.dd_g = opt_dd_g;
  a.dd_host = d_ddmode_host;
  a.dd_mode = d_status + kStatusDdMode;
  a.groups = opt_groups ? d_groups : nullptr;
  a.gs_mask = gs_slots - 1;
  // lanes per publish: auto (0) gives a call of fewer than 262,144 publishes
  // two lanes (twice the waves: a small batch fills the chip; config A 184 ->
  // 172 us per call), a larger one one lane in COUNT (config C, A/B-tuned)
  const uint32_t fg = opt_fast_g ? opt_fast_g : (npub >= kFastG1Min ? 1u : 2u);
  a.gpw = 64 / (fg == 4 ? 4 : fg == 1 ? 1 : 2);   // publishes per chunk
  a.status = d_status + kStatusSet * (call_seq & 1);
  a.status_next = d_status + kStatusSet * ((call_seq + 1) & 1);
  a.err = d_status + 2 * kStatusSet;
  a.deferred = d_deferred;
  a.fast_g = fg; a.opts = opt_flags;
  a.count_bpc = opt_count_bpc; a.emit_bpc = opt_emit_bpc;
  a.cus = (uint32_t)cu_count;
  a.lookback = d_lookback; a.lb_tag = lb_tag;
  a.o_stack = d_ostack; a.o_cap = o_cap; a.o_waves = o_waves; a.o_slots = o_slots;
  return a;
}

// VMQG_DEBUG_SYNC=<seconds>: wait for each launch of a match call and name
// the one still running after that many seconds, then end the process (a
// diagnosis aid for a launch that does not finish; off by default).
static double debug_limit() {
  static const double lim = [] { const char* e = getenv("VMQG_DEBUG_SYNC"); return e ? atof(e) : 0.0; }();
  return lim;
}
static uint32_t* debug_words() {   // 8 progress words per wave, host memory the kernels write directly
  static uint32_t* w = [] {
    void* p = nullptr;
    if (debug_limit() > 0 && hipHostMalloc(&p, (size_t)8 * 4 * 65536, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) p = nullptr;
    return static_cast<uint32_t*>(p);
  }();
  return w;
}
static void debug_sync(hipStream_t st, const char* what) {
  const double lim = debug_limit();
  if (lim <= 0) return;
  const auto t0 = std::chrono::steady_clock::now();
  while (hipStreamQuery(st) == hipErrorNotReady) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > lim) {
      fprintf(stderr, "vmqg debug: %s still running after %.0f s\n", what, lim);
      if (uint32_t* w = debug_words()) {
        uint32_t hist[16] = {0};
        int shown = 0;
        for (uint32_t i = 0; i < 65536; i++) {
          const volatile uint32_t* q = w + (size_t)i * 8;
          hist[q[0] & 15]++;
          if (q[0] != 0 && q[0] != 9 && shown < 40) {
            shown++;
            fprintf(stderr, "  wave %u: phase %u base %u ticket %u/%u p %u k0 %u K %u nc %u\n", i, q[0], q[1],
                    q[2] & 15, q[2] >> 4, q[3], q[5], q[6], q[7]);
          }
        }
        fprintf(stderr, "  phases: 0:%u 1:%u 2:%u 9:%u\n", hist[0], hist[1], hist[2], hist[9]);
      }
      fflush(stderr);
      _exit(3);
    }
  }
  fprintf(stderr, "vmqg debug: %s done\n", what);
}

int Engine::match_device(const vmqg_pub* d_pubs_, uint32_t npub, const uint32_t* d_words_, Record* d_out_,
                         uint64_t out_cap, vmqg_range* d_rng, uint64_t rng_cap, uint64_t* d_offsets,
                         hipStream_t st) {
  if (!has_device) return VMQG_E_DEVICE;
  // the tables the device holds, as their layout says (a layout larger than
  // the arena would send every read past it)
  if (!d_arena || d_arena_bytes < dlay.total_bytes || dlay.magic != kLayoutMagic) return VMQG_E_STATE;
  hipSetDevice(device);
  // table changes (patches, images) land before this match: the primary's on
  // the context stream, a replica's on whatever stream the caller gave
  if (order_on(st) != VMQG_OK) return VMQG_E_DEVICE;
  if (npub == 0) return hipMemsetAsync(d_offsets, 0, 8, st) == hipSuccess ? VMQG_OK : VMQG_E_DEVICE;
  int rc;
  if ((rc = ensure_match_scratch(npub, st)) ||
      (rc = ensure_lookback(std::max<uint64_t>(scan_tiles((npub + 15) / 16), exact_fused_tiles(npub)), st)) ||
      (rc = ensure_wave_scratch(st)))
    return rc;
  MatchArgs a = args_for(d_pubs_, npub, d_words_, d_offsets);
  if ((a.dbg = debug_words())) memset(a.dbg, 0, (size_t)8 * 4 * 65536);
  a.out = d_out_; a.out_cap = out_cap;
  a.out_rng = d_rng; a.rng_cap = rng_cap;
  last_set = call_seq & 1;
  call_seq++;
  // kernel timing (vmqg_set_timing): events written by each dispatch itself
  // (hipExtLaunchKernel), so timing adds no marker packets between launches
  std::array<hipEvent_t, 2 * kTimedEvents> ev{};
  if (timing) {
    for (int k = 0; k < 2 * kTimedStages; k++) hipEventCreate(&ev[k]);
    if (a.dd_claimed) for (int k = 10; k < 16; k++) hipEventCreate(&ev[k]);
    t_ev.push_back(ev);
  }
  // exact-filter auto mode: the sampler on the first call and every 64th
  if (opt_exfilter == 2 && npub >= 1024 && call_seq > ex_next) {
    ex_next = call_seq + 63;
    if (launch_ex_sample(a, st) != hipSuccess) return VMQG_E_DEVICE;
  }
  // dedupe on: the claim and classify passes (timed with COUNT)
  if (a.dd_claimed && (launch_dd_claim(a, st, ev[10], ev[11]) != hipSuccess ||
                       launch_dd_classify(a, st, ev[12], ev[13]) != hipSuccess))
    return VMQG_E_DEVICE;
  // trie-less tables: COUNT, scan and EMIT in one launch, then the EMIT tail
  // (huge publishes); the stages it replaces record no time
  if (opt_fused && a.trieless && !a.dd_claimed && a.groups == nullptr && a.heavy_min == 0) {
    if (timing)
      for (int k = 2; k < 8; k++) { hipEventDestroy(ev[k]); ev[k] = nullptr; t_ev.back()[k] = nullptr; }
    if (launch_exact_fused(a, st, ev[0], ev[1]) != hipSuccess) return VMQG_E_DEVICE;
    debug_sync(st, "fused COUNT/EMIT");
    if (launch_match(a, 1, 1, st, ev[8], ev[9]) != hipSuccess) return VMQG_E_DEVICE;
    debug_sync(st, "EMIT tail");
    return VMQG_OK;
  }
  // COUNT: fast groups (with dedupe on, the representatives, then the
  // duplicates' fix-up), then the wave tier for what they deferred
  if (launch_match(a, 0, 0, st, ev[0], ev[1]) != hipSuccess) return VMQG_E_DEVICE;
  if (a.dd_claimed && launch_dd_fixup(a, st, ev[14], ev[15]) != hipSuccess) return VMQG_E_DEVICE;
  debug_sync(st, "COUNT");
  if (launch_match(a, 0, 1, st, ev[2], ev[3]) != hipSuccess) return VMQG_E_DEVICE;
  debug_sync(st, "COUNT wave tier");
  if (launch_scan(a, st, ev[4], ev[5]) != hipSuccess) return VMQG_E_DEVICE;
  debug_sync(st, "scan");
  // EMIT: the fast tier, then the tail (whole-wave walks, wide publishes)
  if (launch_match(a, 1, 0, st, ev[6], ev[7]) != hipSuccess) return VMQG_E_DEVICE;
  debug_sync(st, "EMIT");
  if (launch_match(a, 1, 1, st, ev[8], ev[9]) != hipSuccess) return VMQG_E_DEVICE;
  debug_sync(st, "EMIT tail");
  return VMQG_OK;
}

// Status words: two sets of per-call counters (kStatusSet words each: [0]
// publishes the fast pass deferred to the 4-lane retry, [1] whole-wave walks
// with a global stack, [2] scan ticket, [3] whole-wave walks, [4] wide
// publishes, [5] fast-pass deferrals by a walk overflow, [6..7] entries the
// EMIT tail wrote for whole-wave walks, [24..25] ... for wide publishes)
// used by alternate calls, then the error bits latched since the previous
// vmqg_match_status.
int Engine::match_status(hipStream_t st) {
  if (!has_device) return VMQG_E_DEVICE;
  hipSetDevice(device);
  if (order_on(st) != VMQG_OK) return VMQG_E_DEVICE;   // the matches queued on any stream
  uint32_t h[2 * kStatusSet + 1] = {0};
  if (hipMemcpyAsync(h, d_status, sizeof(h), hipMemcpyDeviceToHost, st) != hipSuccess) return VMQG_E_DEVICE;
  if (hipStreamSynchronize(st) != hipSuccess) return VMQG_E_DEVICE;
  if (hipMemsetAsync(d_status + 2 * kStatusSet, 0, 4, st) != hipSuccess) return VMQG_E_DEVICE;
  if (hipStreamSynchronize(st) != hipSuccess) return VMQG_E_DEVICE;
  const uint32_t* c = h + kStatusSet * last_set;
  last_deferred[0] = c[3];
  last_deferred[1] = c[1];
  last_retried = c[0];
  last_many = c[4];
  last_wave_entries = (uint64_t)c[6] | ((uint64_t)c[7] << 32);
  last_wide_entries = (uint64_t)c[24] | ((uint64_t)c[25] << 32);
  last_dedup = c[8];
  last_dedup_walked = c[10];
  const uint32_t err = h[2 * kStatusSet];
  last_err_bits = err;
  if (err && debug_limit() > 0) fprintf(stderr, "vmqg debug: match status error bits 0x%x\n", err);
  if (err & 2u) return VMQG_E_FRONTIER;
  if (err & 4u) return VMQG_E_OVERFLOW;
  if (err & (8u | 16u)) return VMQG_E_DEVICE;   // count mismatch, look-back timeout
  return VMQG_OK;
}

void Engine::collect_times() {
  if (!has_device) return;
  hipSetDevice(device);
  for (auto& ev : t_ev) {
    hipEventSynchronize(ev[2 * kTimedStages - 1] ? ev[2 * kTimedStages - 1] : ev[2 * kTimedStages - 3]);
    for (int k = 0; k < kTimedEvents; k++) {
      float ms = 0;
      if (ev[2 * k]) hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]);   // null: the stage made no launch
      sum_stage_ns[k < kTimedStages ? k : 0] += ms * 1e6;   // the dedupe claim pass counts as COUNT
    }
    n_timed++;
    for (auto e : ev) if (e) hipEventDestroy(e);
  }
  t_ev.clear();
}

// ------------------------------------------------------------------ dump
static std::string esc(const std::string& s) {
  static const char* hx = "0123456789abcdef";
  std::string o = "\"";
  for (unsigned char c : s) {
    if (c >= 0x20 && c < 0x7f && c != '"' && c != '\\') o += (char)c;
    else { o += "\\x"; o += hx[c >> 4]; o += hx[c & 15]; }
  }
  return o + "\"";
}

std::string Engine::dump() {
  std::vector<std::string> lines;
  auto path_words = [&](uint32_t p) {
    std::vector<uint32_t> w;
    while (paths[p].parent != kNone) { w.push_back(paths[p].word); p = paths[p].parent; }
    std::reverse(w.begin(), w.end());
    return w;
  };
  auto show_words = [&](const std::vector<uint32_t>& w) {
    std::string o = "[";
    for (size_t i = 0; i < w.size(); i++) { if (i) o += ","; o += esc(word_text(w[i])); }
    return o + "]";
  };
  auto nid = [&](uint32_t p) {
    return "mp#" + std::to_string(paths[p].mp) + "|" +
           (paths[p].parent == kNone ? std::string("root") : show_words(path_words(p)));
  };
  const EdgeSlot* et = region<EdgeSlot>(lay.edge_off);
  for (uint64_t i = 0; i < lay.edge_buckets * kEdgeSlotsPerBucket; i++) {
    const EdgeSlot& e = et[i];
    if (e.parent == kEmpty || e.parent == kTomb) continue;
    lines.push_back("trie " + nid(e.parent) + " " + esc(word_text(e.word)) + " -> " + show_words(path_words(e.child)));
  }
  auto show_nog = [&](const Nog& n) {
    return n.group == kNone ? "node#" + std::to_string(n.node)
                            : "{node#" + std::to_string(n.node) + "," + esc(word_text(n.group)) + "}";
  };
  for (uint32_t p = 0; p < paths.size(); p++) {
    const PathInfo& P = paths[p];
    if (P.rec)
      lines.push_back("node " + nid(p) + " ec=" + std::to_string(P.ec) + " topic=" +
                      (P.topic_set ? show_words(path_words(p)) : std::string("undefined")));
    if (P.filter) {
      std::string l = "topic mp#" + std::to_string(P.mp) + "|" + show_words(path_words(p)) +
                      " total=" + std::to_string(P.total) + " [";
      for (size_t i = 0; i < P.nodes.size(); i++) {
        if (i) l += ",";
        l += show_nog(P.nodes[i].first) + ":" + std::to_string(P.nodes[i].second);
      }
      lines.push_back(l + "]");
    }
  }
  auto show_key = [&](const KeyInfo& K) {
    const TopicInfo& t = topics[K.topic_id];
    if (K.group != kNone)
      return "{mp#" + std::to_string(t.mp) + "," + esc(word_text(K.group)) + "," + show_words(t.words) + "}";
    return "{mp#" + std::to_string(t.mp) + "," + show_words(t.words) + "}";
  };
  auto show_val = [&](const Record& r) {
    const uint32_t kind = r.kind_node >> 24, node = r.kind_node & 0xFFFFFF;
    const std::string sid = "sub#" + std::to_string(r.subscriber), si = "info#" + std::to_string(r.subinfo);
    if (kind == VMQG_EMIT_GROUP)
      return "{node#" + std::to_string(node) + "," + esc(word_text(r.group)) + "," + sid + "," + si + "}";
    return "{" + sid + "," + si + "}";
  };
  for (const KeyInfo& K : keys) {
    if (K.vals.empty()) continue;
    if (K.vals.size() == 1) { lines.push_back("subs " + show_key(K) + " " + show_val(K.vals[0])); continue; }
    lines.push_back("subs " + show_key(K) + " fanout");
    for (auto& v : K.vals) lines.push_back("fanout " + show_key(K) + " " + show_val(v));
  }
  for (const TopicInfo& t : topics) {
    if (t.remote.empty()) continue;
    std::string l = "remote mp#" + std::to_string(t.mp) + "|" + show_words(t.words) + " [";
    for (size_t i = 0; i < t.remote.size(); i++) {
      if (i) l += ",";
      l += "node#" + std::to_string(t.remote[i].first) + ":" + std::to_string(t.remote[i].second);
    }
    lines.push_back(l + "]");
  }
  std::sort(lines.begin(), lines.end());
  std::string out;
  for (auto& l : lines) { out += l; out += '\n'; }
  return out;
}

}  // namespace vmqg
