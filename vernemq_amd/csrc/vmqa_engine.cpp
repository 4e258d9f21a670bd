// ACL checker host engine (see vmqa_engine.h).  Citations are to
// apps/vmq_acl/src/vmq_acl.erl unless noted.
#include "vmqa_engine.h"
#include "vmqg_chain.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <set>
#include <tuple>

namespace vmqa {

using vmqg::kEmpty;

static uint64_t next_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}
static uint64_t align256(uint64_t v) { return (v + 255) & ~255ull; }

AclEngine::~AclEngine() {
  if (!has_device) return;
  hipSetDevice(device);
  if (stream) hipStreamSynchronize(stream);
  for (auto& e : t_check) { hipEventDestroy(e.first); hipEventDestroy(e.second); }
  if (ev_done) hipEventDestroy(ev_done);
  hipFree(d_arena); hipFree(d_status); hipFree(d_r); hipFree(d_w); hipFree(d_o);
  if (stream) hipStreamDestroy(stream);
}

int AclEngine::init(const vmqa_config& c) {
  cfg = c;
  for (const char* s : {"+", "#", "$share", "%u", "%c", "%m"}) intern(reinterpret_cast<const uint8_t*>(s), strlen(s), true);
  if (cfg.device >= 0) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || cfg.device >= n) return VMQG_E_DEVICE;
    device = cfg.device;
    if (hipSetDevice(device) != hipSuccess) return VMQG_E_DEVICE;
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return VMQG_E_DEVICE;
    if (hipEventCreateWithFlags(&ev_done, hipEventDisableTiming) != hipSuccess) return VMQG_E_DEVICE;
    has_device = true;
    if (hipMalloc(&d_status, 64) != hipSuccess) return VMQG_E_NOMEM;
  }
  return load(nullptr, 0, nullptr, 0);   // the empty tables of init/0 (:105-112)
}

uint32_t AclEngine::intern(const uint8_t* b, size_t n, bool create) {
  std::string s(reinterpret_cast<const char*>(b), n);
  auto it = word_index.find(s);
  if (it != word_index.end()) return it->second;
  if (!create) return vmqg::kUnknownWord;
  const uint32_t id = (uint32_t)word_text.size();
  if (id >= VMQA_EPHEMERAL) return vmqg::kUnknownWord;
  word_text.push_back(s);
  word_index.emplace(std::move(s), id);
  return id;
}

// The six ets sets as one image: rows deduplicated (a set absorbs a
// repeated key, t/3 :233-238), grouped into the lists check/4 walks.
int AclEngine::load(const vmqa_rule* rules, size_t n, const uint32_t* words, size_t nwords) {
  for (size_t i = 0; i < n; i++) {   // validate the whole batch first
    const vmqa_rule& r = rules[i];
    if ((r.type != VMQA_READ && r.type != VMQA_WRITE) || r.table > VMQA_TABLE_PATTERN) return VMQG_E_INVAL;
    if (r.nwords == 0 || (uint64_t)r.word_off + r.nwords > nwords) return VMQG_E_INVAL;
    if (r.table == VMQA_TABLE_USER && r.user >= word_text.size()) return VMQG_E_INVAL;
    for (uint32_t j = 0; j < r.nwords; j++) if (words[r.word_off + j] >= word_text.size()) return VMQG_E_INVAL;
  }
  // key: {type, table, user, words}
  using Key = std::tuple<uint32_t, uint32_t, uint32_t, std::vector<uint32_t>>;
  std::set<Key> keys;
  for (size_t i = 0; i < n; i++) {
    const vmqa_rule& r = rules[i];
    keys.emplace(r.type - 1, r.table, r.table == VMQA_TABLE_USER ? r.user : 0,
                 std::vector<uint32_t>(words + r.word_off, words + r.word_off + r.nwords));
  }
  std::vector<std::vector<uint32_t>> fixed(4);                 // all-r, all-w, pattern-r, pattern-w
  std::map<std::pair<uint32_t, uint32_t>, std::vector<uint32_t>> per_user;   // {user, type} -> row ids
  std::vector<ARule> rl;
  std::vector<uint32_t> rw;
  for (const Key& k : keys) {
    const uint32_t id = (uint32_t)rl.size();
    const auto& w = std::get<3>(k);
    rl.push_back(ARule{(uint32_t)w.size(), (uint32_t)rw.size()});
    rw.insert(rw.end(), w.begin(), w.end());
    const uint32_t type = std::get<0>(k), table = std::get<1>(k);
    if (table == VMQA_TABLE_ALL) fixed[type].push_back(id);
    else if (table == VMQA_TABLE_PATTERN) fixed[2 + type].push_back(id);
    else per_user[{std::get<2>(k), type}].push_back(id);
  }
  // the fixed lists, packed: per rule {nwords, word index}, then the words
  std::vector<uint32_t> fx;
  uint32_t nfixed = 0;
  for (auto& f : fixed) nfixed += (uint32_t)f.size();
  fx.resize(2 * (size_t)nfixed);
  uint32_t ri = 0;
  std::vector<AList> fheads(4);
  for (int h = 0; h < 4; h++) {
    fheads[h] = AList{ri, (uint32_t)fixed[h].size()};
    for (uint32_t id : fixed[h]) {
      fx[2 * ri] = rl[id].nwords;
      fx[2 * ri + 1] = (uint32_t)fx.size();
      fx.insert(fx.end(), rw.begin() + rl[id].words_off, rw.begin() + rl[id].words_off + rl[id].nwords);
      ri++;
    }
  }
  uint64_t nlist = 0;
  for (auto& u : per_user) nlist += u.second.size();
  users_slots = next_pow2(std::max<uint64_t>(64, per_user.size() * 4));   // load <= 1/4
  uint64_t o = 0;
  rules_off = o;  o = align256(o + std::max<size_t>(1, rl.size()) * sizeof(ARule));
  rwords_off = o; o = align256(o + std::max<size_t>(1, rw.size()) * 4);
  lists_off = o;  o = align256(o + std::max<uint64_t>(1, nlist) * 4);
  fixed_off = o;  o = align256(o + std::max<size_t>(1, fx.size()) * 4);
  heads_off = o;  o = align256(o + 4 * sizeof(AList));
  users_off = o;  o = align256(o + users_slots * sizeof(USlot));
  fixed_words = fx.size();
  image.assign(o, 0);
  memcpy(image.data() + rules_off, rl.data(), rl.size() * sizeof(ARule));
  memcpy(image.data() + rwords_off, rw.data(), rw.size() * 4);
  memcpy(image.data() + fixed_off, fx.data(), fx.size() * 4);
  memcpy(image.data() + heads_off, fheads.data(), 4 * sizeof(AList));
  uint32_t* lists = reinterpret_cast<uint32_t*>(image.data() + lists_off);
  USlot* slots = reinterpret_cast<USlot*>(image.data() + users_off);
  for (uint64_t i = 0; i < users_slots; i++) slots[i] = USlot{kEmpty, 0, 0, 0};
  uint32_t top = 0;
  std::set<uint32_t> users;
  for (auto& u : per_user) {
    const uint64_t mask = users_slots - 1;
    uint64_t i = user_hash(u.first.first, u.first.second) & mask;
    while (slots[i].user != kEmpty) i = (i + 1) & mask;
    slots[i] = USlot{u.first.first, u.first.second, top, (uint32_t)u.second.size()};
    for (uint32_t id : u.second) lists[top++] = id;
    users.insert(u.first.first);
  }
  n_rules = rl.size();
  n_users = users.size();
  loads++;
  return upload();
}

int AclEngine::upload() {
  if (!has_device) return VMQG_OK;
  hipSetDevice(device);
  // tables must not change under a check still reading them
  if (vmqg::chain_order(ev_done, chk_stream, stream) != VMQG_OK) return VMQG_E_DEVICE;
  if (hipStreamSynchronize(stream) != hipSuccess) return VMQG_E_DEVICE;
  if (d_arena_bytes < image.size()) {
    if (d_arena) hipFree(d_arena);
    d_arena = nullptr; d_arena_bytes = 0;
    if (hipMalloc(&d_arena, image.size()) != hipSuccess) return VMQG_E_NOMEM;
    d_arena_bytes = image.size();
  }
  if (hipMemcpyAsync(d_arena, image.data(), image.size(), hipMemcpyHostToDevice, stream) != hipSuccess)
    return VMQG_E_DEVICE;
  if (hipStreamSynchronize(stream) != hipSuccess) return VMQG_E_DEVICE;
  return VMQG_OK;
}

int AclEngine::check_device(const vmqa_req* d_reqs, uint32_t n, const uint32_t* d_words, uint8_t* d_out,
                            hipStream_t st) {
  if (!has_device) return VMQG_E_DEVICE;
  hipSetDevice(device);
  if (vmqg::chain_order(ev_done, chk_stream, st) != VMQG_OK) return VMQG_E_DEVICE;
  if (hipMemsetAsync(d_status, 0, 32, st) != hipSuccess) return VMQG_E_DEVICE;
  if (n == 0) return VMQG_OK;
  AArgs a{};
  a.rules = reinterpret_cast<const ARule*>(d_arena + rules_off);
  a.rwords = reinterpret_cast<const uint32_t*>(d_arena + rwords_off);
  a.lists = reinterpret_cast<const uint32_t*>(d_arena + lists_off);
  a.heads = reinterpret_cast<const AList*>(d_arena + heads_off);
  a.fixed = reinterpret_cast<const uint32_t*>(d_arena + fixed_off);
  a.fixed_words = (uint32_t)fixed_words;
  a.users = reinterpret_cast<const USlot*>(d_arena + users_off);
  a.users_mask = users_slots - 1;
  a.reqs = d_reqs; a.words = d_words; a.n = n; a.out = d_out; a.status = d_status;
  hipEvent_t e[2] = {nullptr, nullptr};
  if (timing) for (auto& x : e) hipEventCreate(&x);
  if (launch_acl_check(a, st, e[0], e[1]) != hipSuccess) return VMQG_E_DEVICE;
  if (timing) t_check.push_back({e[0], e[1]});
  return VMQG_OK;
}

int AclEngine::check_status(hipStream_t st) {
  if (!has_device) return VMQG_E_DEVICE;
  hipSetDevice(device);
  if (vmqg::chain_order(ev_done, chk_stream, st) != VMQG_OK) return VMQG_E_DEVICE;
  uint32_t h[8] = {0};
  if (hipMemcpyAsync(h, d_status, 32, hipMemcpyDeviceToHost, st) != hipSuccess) return VMQG_E_DEVICE;
  if (hipStreamSynchronize(st) != hipSuccess) return VMQG_E_DEVICE;
  if (hipMemsetAsync(d_status, 0, 32, st) != hipSuccess) return VMQG_E_DEVICE;
  if (h[1]) return VMQG_E_INVAL;   // a request without a topic word or of no known type
  return VMQG_OK;
}

void AclEngine::collect_times() {
  if (!has_device) return;
  for (auto& e : t_check) {
    float ms = 0;
    hipEventSynchronize(e.second);
    hipEventElapsedTime(&ms, e.first, e.second);
    sum_ns += ms * 1e6; n_timed++;
    hipEventDestroy(e.first); hipEventDestroy(e.second);
  }
  t_check.clear();
}

}  // namespace vmqa
