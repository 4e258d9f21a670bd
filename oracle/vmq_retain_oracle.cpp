// TEST INFRASTRUCTURE ONLY — CPU restatement of VerneMQ's retained-message
// store, apps/vmq_server/src/vmq_retain_srv.erl (reference checkout at
// /root/reference).  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it, and only as the checker / the timed CPU
// baseline; the product (libvmqgpu's vmqr_* path) never links it.
//
// What it restates, lookup for lookup:
//   ?RETAIN_CACHE  ets set keyed {MP, RoutingKey}            :52-61
//   delete/2       ets:delete                                :63-66
//   insert/3       ets:insert (a set: a new value replaces)  :68-71
//   match_fold/4   has_wildcard(Topic) -> ets:foldl over the WHOLE table,
//                  FoldFun({T, Payload}) for every {{M, T}, _} with M == MP
//                  and vmq_topic:match(T, Topic); otherwise ets:lookup of
//                  {MP, Topic}                               :75-99
//   has_wildcard/1                                           :239-242
//   vmq_topic:match/2   apps/vmq_commons/src/vmq_topic.erl:53-65
//   stats/0 (entry count)                                    :101-113
// Payloads are opaque u32 ids (the #retain_msg{} lives with the caller).
// ets:foldl visits a set in an unspecified order: results are compared as
// multisets.
//
// Encoding (little endian): str = u32 len + bytes; words = u32 n + n strs;
// a key = str MP + words Topic.
#include <chrono>
#include <cstdint>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

using Words = std::vector<std::string>;

struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  bool bad = false;
  uint32_t u32() {
    if (e - p < 4) { bad = true; return 0; }
    uint32_t v;
    memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  std::string str() {
    const uint32_t n = u32();
    if (bad || (size_t)(e - p) < n) { bad = true; return {}; }
    std::string s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
  Words words() {
    const uint32_t n = u32();
    Words w;
    for (uint32_t i = 0; i < n && !bad; i++) w.push_back(str());
    return w;
  }
};

std::string key_of(const std::string& mp, const Words& t) {
  std::string k;
  auto put = [&](const std::string& s) {
    const uint32_t n = (uint32_t)s.size();
    k.append(reinterpret_cast<const char*>(&n), 4);
    k += s;
  };
  put(mp);
  for (auto& w : t) put(w);
  return k;
}

// vmq_retain_srv.erl:239-242
bool has_wildcard(const Words& t) {
  for (size_t i = 0; i < t.size(); i++) {
    if (t[i] == "+") return true;                        // [<<"+">>|_]
    if (t[i] == "#" && i + 1 == t.size()) return true;   // [<<"#">>]
  }
  return false;                                          // []
}

// vmq_topic:match/2, vmq_topic.erl:53-65, clause by clause in order
bool topic_match(const Words& t, const Words& f) {
  size_t i = 0;
  for (;;) {
    if (i == t.size() && i == f.size()) return true;                  // match([], [])
    if (i < t.size() && i < f.size() && t[i] == f[i]) { i++; continue; }   // [H|T1], [H|T2]
    if (i < t.size() && i < f.size() && f[i] == "+") { i++; continue; }    // [_|T1], [+|T2]
    if (i + 1 == f.size() && f[i] == "#") return true;                // match(_, [#])
    return false;                                                     // the three false clauses
  }
}

struct Entry {
  std::string mp;
  Words topic;
  uint32_t payload;
};

struct RetainOracle {
  std::unordered_map<std::string, Entry> cache;   // ?RETAIN_CACHE
  std::vector<uint32_t> out;

  void insert(const std::string& mp, const Words& t, uint32_t payload) {   // :68-71
    cache[key_of(mp, t)] = Entry{mp, t, payload};
  }
  void erase(const std::string& mp, const Words& t) { cache.erase(key_of(mp, t)); }   // :63-66

  // match_fold/4 with FoldFun = append the payload (:75-99)
  void match_fold(const std::string& mp, const Words& f) {
    if (has_wildcard(f)) {
      for (auto& kv : cache) {   // ets:foldl: full table scan
        const Entry& e = kv.second;
        if (e.mp == mp && topic_match(e.topic, f)) out.push_back(e.payload);
      }
    } else {
      auto it = cache.find(key_of(mp, f));
      if (it != cache.end()) out.push_back(it->second.payload);
    }
  }
};

}  // namespace

extern "C" {

RetainOracle* retain_oracle_new() { return new RetainOracle(); }
void retain_oracle_free(RetainOracle* o) { delete o; }
uint64_t retain_oracle_size(RetainOracle* o) { return o->cache.size(); }

// buf: u32 n_ops, then per op u8 kind (1 insert, 2 delete), key, u32 payload
int retain_oracle_apply(RetainOracle* o, const uint8_t* buf, size_t n) {
  Reader r{buf, buf + n};
  const uint32_t nops = r.u32();
  for (uint32_t i = 0; i < nops && !r.bad; i++) {
    if (r.p >= r.e) { r.bad = true; break; }
    const uint8_t kind = *r.p++;
    const std::string mp = r.str();
    const Words t = r.words();
    const uint32_t payload = r.u32();
    if (r.bad) break;
    if (kind == 1) o->insert(mp, t, payload);
    else if (kind == 2) o->erase(mp, t);
    else return -1;
  }
  return r.bad ? -1 : 0;
}

// buf: u32 n_filters, then per filter a key.  Writes, for each filter, the
// payload ids match_fold folds over; *offs (n + 1 entries) delimits them.
long retain_oracle_match(RetainOracle* o, const uint8_t* buf, size_t n, uint64_t* offs, uint64_t cap) {
  Reader r{buf, buf + n};
  const uint32_t nf = r.u32();
  o->out.clear();
  for (uint32_t i = 0; i < nf && !r.bad; i++) {
    if (i < cap) offs[i] = o->out.size();
    const std::string mp = r.str();
    const Words f = r.words();
    if (!r.bad) o->match_fold(mp, f);
  }
  if (nf < cap) offs[nf] = o->out.size();
  return r.bad ? -1 : (long)o->out.size();
}

const uint32_t* retain_oracle_out(RetainOracle* o, size_t* n) {
  *n = o->out.size();
  return o->out.data();
}

// CPU baseline: `reps` passes of match_fold over a filter batch, one thread;
// returns ns, *matches = payloads folded per pass.
long long retain_oracle_match_timed(RetainOracle* o, const uint8_t* buf, size_t n, int reps,
                                    unsigned long long* matches) {
  Reader r{buf, buf + n};
  const uint32_t nf = r.u32();
  std::vector<std::pair<std::string, Words>> fs;
  for (uint32_t i = 0; i < nf && !r.bad; i++) {
    std::string mp = r.str();
    Words f = r.words();
    fs.emplace_back(std::move(mp), std::move(f));
  }
  if (r.bad) return -1;
  const auto t0 = std::chrono::steady_clock::now();
  unsigned long long m = 0;
  for (int k = 0; k < reps; k++) {
    for (auto& f : fs) {
      o->out.clear();
      o->match_fold(f.first, f.second);
      m += o->out.size();
    }
  }
  const auto t1 = std::chrono::steady_clock::now();
  if (matches) *matches = reps ? m / (unsigned long long)reps : 0;
  return (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
}

int retain_oracle_topic_match(const uint8_t* buf, size_t n) {   // vmq_topic:match(T, F)
  Reader r{buf, buf + n};
  const Words t = r.words(), f = r.words();
  return r.bad ? -1 : (topic_match(t, f) ? 1 : 0);
}

int retain_oracle_has_wildcard(const uint8_t* buf, size_t n) {
  Reader r{buf, buf + n};
  const Words f = r.words();
  return r.bad ? -1 : (has_wildcard(f) ? 1 : 0);
}

}  // extern "C"
