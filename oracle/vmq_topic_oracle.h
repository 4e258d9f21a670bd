// TEST INFRASTRUCTURE ONLY — CPU restatement of the parts of
// apps/vmq_commons/src/vmq_topic.erl the oracles share: topic splitting and
// validation (validate_topic/2, :82-133) and match/2 (:53-65).  Included by
// vmq_trie_oracle.cpp and vmq_acl_oracle.cpp; never by the product.
#pragma once
#include <string>
#include <vector>

namespace vmq_topic_oracle {

using Words = std::vector<std::string>;

// validate_topic/2  vmq_topic.erl:82-133.  Error codes mirror the atoms.
enum { V_OK = 0, V_EMPTY = 1, V_TOO_LONG = 2, V_PLUS_PUB = 3, V_HASH_PUB = 4,
       V_PLUS_WORD = 5, V_HASH_WORD = 6, V_BAD_SHARED = 7 };

inline int validate_publish(const std::string& topic, Words& out) {
  // validate_publish_topic/3  vmq_topic.erl:97-112
  size_t seg = 0;
  out.clear();
  for (;;) {
    std::string rest = topic.substr(seg);
    if (rest.compare(0, 2, "+/") == 0 || rest == "+") return V_PLUS_PUB;  // :97-98
    if (rest == "#") return V_HASH_PUB;                                     // :99
    size_t L = 0;
    for (;;) {                                                              // :100-111
      if (L < rest.size() && rest[L] == '/') { out.push_back(rest.substr(0, L)); seg += L + 1; break; }
      if (L == rest.size()) { out.push_back(rest); return V_OK; }
      if (rest[L] == '+') return V_PLUS_WORD;
      if (rest[L] == '#') return V_HASH_WORD;
      L++;
    }
  }
}

inline int validate_shared(const Words& t) {
  // validate_shared_subscription/1  vmq_topic.erl:131-133
  if (!t.empty() && t[0] == "$share") return t.size() >= 3 ? V_OK : V_BAD_SHARED;
  return V_OK;
}

inline int validate_subscribe(const std::string& topic, Words& out) {
  // validate_subscribe_topic/3  vmq_topic.erl:114-129
  size_t seg = 0;
  out.clear();
  for (;;) {
    std::string rest = topic.substr(seg);
    if (rest.compare(0, 2, "+/") == 0) { out.push_back("+"); seg += 2; continue; }  // :114
    if (rest == "+" || rest == "#") { out.push_back(rest); return validate_shared(out); }  // :115-116
    size_t L = 0;
    bool next = false;
    for (;;) {
      if (L < rest.size() && rest[L] == '/') { out.push_back(rest.substr(0, L)); seg += L + 1; next = true; break; }
      if (L == rest.size()) { out.push_back(rest); return validate_shared(out); }
      if (rest[L] == '+') return V_PLUS_WORD;
      if (rest[L] == '#') return V_HASH_WORD;
      L++;
    }
    if (!next) break;
  }
  return V_OK;
}

inline int validate_topic(int type, const std::string& topic, Words& out) {
  if (topic.empty()) return V_EMPTY;                 // vmq_topic.erl:82-83
  if (topic.size() > 65536) return V_TOO_LONG;       // :84-85 (MAX_LEN :45)
  return type == 0 ? validate_publish(topic, out) : validate_subscribe(topic, out);
}

// vmq_topic:match/2, vmq_topic.erl:53-65, clause by clause in order.  The
// first argument may itself hold '+' / '#' words (vmq_acl checks subscribe
// filters with it): they only meet the clauses by equality.
inline bool erl_match(const Words& t, const Words& f) {
  size_t i = 0;
  for (;;) {
    if (i == t.size() && i == f.size()) return true;                       // match([], [])
    if (i < t.size() && i < f.size() && t[i] == f[i]) { i++; continue; }   // [H|T1], [H|T2]
    if (i < t.size() && i < f.size() && f[i] == "+") { i++; continue; }    // [_|T1], [+|T2]
    if (i + 1 == f.size() && f[i] == "#") return true;                     // match(_, [#])
    return false;                                                          // the three false clauses
  }
}

}  // namespace vmq_topic_oracle
