// TEST INFRASTRUCTURE ONLY — CPU restatement of VerneMQ's file-based ACL
// plugin, apps/vmq_acl/src/vmq_acl.erl (reference checkout at
// /root/reference).  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it, and only as the checker / the timed CPU
// baseline; the product (libvmqgpu's vmqa_* path) never links it.
//
// What it restates, clause for clause:
//   the six ets sets  vmq_acl_{read,write}_{all,user,pattern}      :38-45
//   load_from_list/1  age_entries, parse, del_aged_entries          :128-144, :268-276
//   parse_acl_line/2  the clause order of :146-177 ("#" comment, "topic
//                     read ", "topic write ", "topic ", "user ", "pattern
//                     read ", "pattern write ", "pattern ", "\n", eof); a
//                     line no clause takes crashes the load (function_clause)
//                     with the tables as far as they got
//   in/3              strip the last byte, validate_topic(subscribe), insert
//                     into t/3's table                              :219-238
//   check/4           all -> user -> pattern, iterate_until_true    :179-204
//   topic/3, subst/5  %u %c %m word substitution                    :206-217
//   vmq_topic:match/2 (vmq_topic.erl:53-65) via vmq_topic_oracle.h
// A user is a binary or the atom `undefined` (anonymous clients).
//
// Encoding (little endian): str = u32 len + bytes; words = u32 n + n strs.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "vmq_topic_oracle.h"

namespace {

using vmq_topic_oracle::Words;
using vmq_topic_oracle::erl_match;

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

enum Type { READ = 0, WRITE = 1 };

// A parse-time user: the atom `all` (before any "user" line) or a binary.
struct PUser { bool all; std::string name; };

struct Acl {
  // ets sets: key -> value (1 fresh, 2 aged)
  std::map<Words, int> all[2], pattern[2];
  std::map<std::pair<std::string, Words>, int> user[2];
  std::string out;

  // age_entries/0 (:268-271): every key's value becomes 2
  void age() {
    for (int t = 0; t < 2; t++) {
      for (auto& kv : all[t]) kv.second = 2;
      for (auto& kv : pattern[t]) kv.second = 2;
      for (auto& kv : user[t]) kv.second = 2;
    }
  }
  // del_aged_entries/0 (:273-276): ets:match_delete(T, {'_', 2})
  void del_aged() {
    for (int t = 0; t < 2; t++) {
      for (auto it = all[t].begin(); it != all[t].end();) it = it->second == 2 ? all[t].erase(it) : std::next(it);
      for (auto it = pattern[t].begin(); it != pattern[t].end();)
        it = it->second == 2 ? pattern[t].erase(it) : std::next(it);
      for (auto it = user[t].begin(); it != user[t].end();) it = it->second == 2 ? user[t].erase(it) : std::next(it);
    }
  }
  // in/3 (:219-231) + t/3 (:233-238).  Returns false on the crash of an
  // empty topic (TopicLen = -1: badmatch).
  bool in(Type ty, const PUser& u, bool is_pattern, const std::string& topic) {
    if (topic.empty()) return false;
    const std::string st = topic.substr(0, topic.size() - 1);   // the last byte is dropped, newline or not
    Words w;
    if (vmq_topic_oracle::validate_topic(1, st, w) != vmq_topic_oracle::V_OK) return true;   // warning, skipped
    if (is_pattern) pattern[ty][w] = 1;
    else if (u.all) all[ty][w] = 1;
    else user[ty][{u.name, w}] = 1;
    return true;
  }
  static bool prefix(const std::string& line, const char* p, std::string& rest) {
    const size_t n = strlen(p);
    if (line.compare(0, n, p) != 0 || line.size() < n) return false;
    rest = line.substr(n);
    return true;
  }
  // load_from_list/1 (:128-144): 0 ok, -1 the parse crashed at a line (the
  // tables keep what was done until then: aged entries included)
  int load(const std::vector<std::string>& lines) {
    age();
    PUser u{true, ""};
    for (const std::string& line : lines) {
      std::string rest;
      if (!line.empty() && line[0] == '#') continue;                                   // :146-148
      if (prefix(line, "topic read ", rest)) { if (!in(READ, u, false, rest)) return -1; continue; }     // :149-151
      if (prefix(line, "topic write ", rest)) { if (!in(WRITE, u, false, rest)) return -1; continue; }   // :152-154
      if (prefix(line, "topic ", rest)) {                                                // :155-158
        if (!in(READ, u, false, rest) || !in(WRITE, u, false, rest)) return -1;
        continue;
      }
      if (prefix(line, "user ", rest)) {                                                 // :159-162
        if (rest.empty()) return -1;   // UserLen = -1: badmatch
        u = PUser{false, rest.substr(0, rest.size() - 1)};
        continue;
      }
      if (prefix(line, "pattern read ", rest)) { if (!in(READ, u, true, rest)) return -1; continue; }    // :163-165
      if (prefix(line, "pattern write ", rest)) { if (!in(WRITE, u, true, rest)) return -1; continue; }  // :166-168
      if (prefix(line, "pattern ", rest)) {                                              // :169-172
        if (!in(READ, u, true, rest) || !in(WRITE, u, true, rest)) return -1;
        continue;
      }
      if (line == "\n") continue;                                                        // :173-174
      return -1;                                                                         // function_clause
    }
    del_aged();                                                                          // eof (:175-177)
    return 0;
  }
  // check/4 (:179-188) with the user a binary (has_user) or undefined.
  // Returns -1 for the function_clause of a topic without a first word.
  int check(Type ty, const Words& tin, bool has_user, const std::string& usr, const std::string& mp,
            const std::string& client) const {
    if (tin.empty()) return -1;
    for (auto& kv : all[ty]) if (erl_match(tin, kv.first)) return 1;                 // check_all_acl :190-192
    if (has_user) {                                                                     // check_user_acl :194-197
      for (auto it = user[ty].lower_bound({usr, Words{}}); it != user[ty].end() && it->first.first == usr; ++it)
        if (erl_match(tin, it->first.second)) return 1;
    }
    for (auto& kv : pattern[ty]) {                                                      // check_pattern_acl :199-204
      // topic/3 + subst/5 (:206-217): %u -> User, %c -> ClientId, %m -> MP.
      // An undefined user puts the atom into the word list: no topic word
      // equals it and it is neither '+' nor '#', so match/2 cannot pass it —
      // and no clause ends a match before the filter's last word.
      Words t;
      bool atom = false;
      for (const std::string& w : kv.first) {
        if (w == "%u") {
          if (!has_user) atom = true;
          t.push_back(usr);
        } else if (w == "%c") {
          t.push_back(client);
        } else if (w == "%m") {
          t.push_back(mp);
        } else {
          t.push_back(w);
        }
      }
      if (!atom && erl_match(tin, t)) return 1;
    }
    return 0;
  }
  // canonical listing of the six tables
  std::string dump() const {
    std::vector<std::string> lines;
    auto show = [](const Words& w) {
      std::string s = "[";
      for (size_t i = 0; i < w.size(); i++) s += (i ? "," : "") + w[i];
      return s + "]";
    };
    const char* tn[2] = {"read", "write"};
    for (int t = 0; t < 2; t++) {
      for (auto& kv : all[t]) lines.push_back(std::string(tn[t]) + " all " + show(kv.first));
      for (auto& kv : pattern[t]) lines.push_back(std::string(tn[t]) + " pattern " + show(kv.first));
      for (auto& kv : user[t]) lines.push_back(std::string(tn[t]) + " user " + kv.first.first + " " + show(kv.first.second));
    }
    std::sort(lines.begin(), lines.end());
    std::string s;
    for (auto& l : lines) s += l + "\n";
    return s;
  }
};

struct Req { Type ty; Words tin; bool has_user; std::string usr, mp, client; };

bool read_reqs(Reader& r, std::vector<Req>& out) {
  const uint32_t n = r.u32();
  for (uint32_t i = 0; i < n && !r.bad; i++) {
    Req q;
    q.ty = r.u32() == 2 ? WRITE : READ;
    q.tin = r.words();
    q.has_user = r.u32() != 0;
    q.usr = r.str();
    q.mp = r.str();
    q.client = r.str();
    out.push_back(std::move(q));
  }
  return !r.bad;
}

}  // namespace

extern "C" {

Acl* acl_oracle_new() { return new Acl(); }
void acl_oracle_free(Acl* a) { delete a; }

// buf: u32 n lines, then str per line (as file:read_line returns them)
int acl_oracle_load(Acl* a, const uint8_t* buf, size_t n) {
  Reader r{buf, buf + n};
  const uint32_t nl = r.u32();
  std::vector<std::string> lines;
  for (uint32_t i = 0; i < nl && !r.bad; i++) lines.push_back(r.str());
  if (r.bad) return -2;
  return a->load(lines);
}

// buf: u32 n, per request u32 type (1 read, 2 write), words topic, u32
// has_user, str user, str mp, str client.  out[i] = 1 allowed, 0 not, -1 crash.
int acl_oracle_check(Acl* a, const uint8_t* buf, size_t n, int8_t* out, size_t cap) {
  Reader r{buf, buf + n};
  std::vector<Req> reqs;
  if (!read_reqs(r, reqs) || reqs.size() > cap) return -2;
  for (size_t i = 0; i < reqs.size(); i++) {
    const Req& q = reqs[i];
    out[i] = (int8_t)a->check(q.ty, q.tin, q.has_user, q.usr, q.mp, q.client);
  }
  return (int)reqs.size();
}

// CPU baseline: `reps` passes over a request batch, one thread; returns ns,
// *allowed = allowed requests per pass.
long long acl_oracle_check_timed(Acl* a, const uint8_t* buf, size_t n, int reps, unsigned long long* allowed) {
  Reader r{buf, buf + n};
  std::vector<Req> reqs;
  if (!read_reqs(r, reqs)) return -1;
  const auto t0 = std::chrono::steady_clock::now();
  unsigned long long m = 0;
  for (int k = 0; k < reps; k++)
    for (const Req& q : reqs) m += a->check(q.ty, q.tin, q.has_user, q.usr, q.mp, q.client) == 1;
  const auto t1 = std::chrono::steady_clock::now();
  if (allowed) *allowed = reps ? m / (unsigned long long)reps : 0;
  return (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
}

const char* acl_oracle_dump(Acl* a, size_t* n) {
  a->out = a->dump();
  *n = a->out.size();
  return a->out.data();
}

}  // extern "C"
