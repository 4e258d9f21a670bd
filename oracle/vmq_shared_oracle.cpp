// TEST INFRASTRUCTURE ONLY — CPU restatement of VerneMQ's shared-subscription
// dispatch, the checker for libvmqgpu's include/vmqs.h.  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may call it.
//
// Follows, clause by clause:
//   apps/vmq_server/src/vmq_reg.erl:344-346, 373-378  the fold fun puts each
//       kind-B entry {Node, Group, SubscriberId, SubInfo} at the HEAD of
//       SubscriberGroups[Group] (add_to_subscriber_group)
//   apps/vmq_server/src/vmq_shared_subscriptions.erl
//       :18-36  publish/3: per group, filter_subscribers, then
//               [S || {_, S} <- lists:sort([{rand:uniform(), N} || N <- Subscribers])]
//       :38-44  publish_to_group: publish_online, else publish_any of the rest
//       :46-63  publish_online: foldl in random order; ok -> throw(done);
//               offline/draining -> prepended to Acc; anything else dropped
//       :65-73  publish_any: first member whose publish_ succeeds
//       :75-88  publish_: local queue lookup / remote enqueue
//       :90-106 filter_subscribers: random | prefer_local | local_only
// rand:uniform() is replaced by the counter-based key of include/vmqs.h
// (element at position p of the publish's emission segment), so results
// are deterministic; the element's list position plays N's role in the
// tie-break.  The reference's entries carry their fold position only
// implicitly, so this restatement keys each collected entry by the position
// of the record it came from.
//
// Queue states: 0 not_found (publish_ -> {error, not_found}), 1 online
// (ok), 2 offline, 3 draining ({error, offline|draining} online, ok for
// `any`).
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <map>
#include <thread>
#include <vector>

namespace {

uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

uint64_t sel_key(uint64_t seed, uint64_t q, uint32_t p) {
  const uint64_t h = mix64(mix64(seed ^ (q * 0x9E3779B97F4A7C15ull)) + (uint64_t)p * 0xD1B54A32D192ED03ull);
  return (h & ~0xFFFFFFull) | (p & 0xFFFFFFu);
}

struct Rec { uint32_t kind_node, group, subscriber, subinfo; };
struct Member { uint32_t node, subscriber, pos; };   // {Node, SubscriberId, QoS} + its fold position

enum { kNotFound = 0, kOnline = 1, kOffline = 2, kDraining = 3 };
enum { kRandom = 0, kPreferLocal = 1, kLocalOnly = 2 };

struct Ctx {
  const uint8_t* states; uint64_t n_states; uint32_t local;
  uint32_t state(uint32_t sub) const { return sub < n_states ? states[sub] : (uint32_t)kOnline; }
};

// filter_subscribers/2 (:90-106)
std::vector<Member> filter_subscribers(const std::vector<Member>& subs, uint32_t policy, uint32_t local) {
  if (policy == kRandom) return subs;
  std::vector<Member> loc;
  for (const Member& m : subs) if (m.node == local) loc.push_back(m);
  if (policy == kPreferLocal && loc.empty()) return subs;
  return loc;
}

// publish_/3 with QState online (true) or any (false): ok?
bool publish_(const Ctx& c, const Member& m, bool online, uint32_t* err_state) {
  const uint32_t s = c.state(m.subscriber);
  *err_state = s;
  if (s == kNotFound) return false;
  if (!online) return true;
  return s == kOnline;
}

// publish_to_group/2 (:38-44) -> chosen position or -1
int64_t publish_to_group(const Ctx& c, const std::vector<Member>& ordered) {
  std::vector<Member> not_online;   // publish_online's Acc (prepended)
  for (const Member& m : ordered) {
    uint32_t s;
    if (publish_(c, m, true, &s)) return m.pos;   // throw(done)
    if (s == kOffline || s == kDraining) not_online.insert(not_online.begin(), m);
  }
  for (const Member& m : not_online) {            // publish_any/2 (:65-73)
    uint32_t s;
    if (publish_(c, m, false, &s)) return m.pos;
  }
  return -1;                                        // {error, no_subscribers}
}

// vmq_reg:publish/5 tail for one publish: collect groups, then publish/3.
uint32_t dispatch_one(const Ctx& c, const Rec* r, uint64_t n, uint32_t policy, uint64_t seed, uint64_t q,
                      uint8_t* chosen) {
  std::map<uint32_t, std::vector<Member>> groups;   // SubscriberGroups (a map: order irrelevant)
  for (uint64_t p = 0; p < n; p++) {
    chosen[p] = 0;
    if ((r[p].kind_node >> 24) != 2u) continue;
    auto& g = groups[r[p].group];
    g.insert(g.begin(), Member{r[p].kind_node & 0xFFFFFFu, r[p].subscriber, (uint32_t)p});
  }
  uint32_t failed = 0;
  for (auto& kv : groups) {
    std::vector<Member> subs = filter_subscribers(kv.second, policy, c.local);
    // lists:sort([{rand:uniform(), N} || N <- Subscribers])
    std::vector<std::pair<uint64_t, Member>> keyed;
    for (const Member& m : subs) keyed.push_back({sel_key(seed, q, m.pos), m});
    std::sort(keyed.begin(), keyed.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    std::vector<Member> ordered;
    for (auto& k : keyed) ordered.push_back(k.second);
    const int64_t pos = publish_to_group(c, ordered);
    if (pos < 0) failed++;
    else chosen[pos] = 1;
  }
  return failed;
}

}  // namespace

extern "C" {

uint64_t shared_oracle_key(uint64_t seed, uint64_t q, uint32_t p) { return sel_key(seed, q, p); }

// emits: 16-B records; offsets[0..npub] absolute into emits / chosen.
void shared_oracle_select(const void* emits, const uint64_t* offsets, uint64_t npub, uint32_t policy,
                          uint64_t seed, uint64_t pub_seq, const uint8_t* states, uint64_t n_states,
                          uint32_t local_node, uint8_t* chosen, uint32_t* failed) {
  const Rec* r = static_cast<const Rec*>(emits);
  const Ctx c{states, n_states, local_node};
  for (uint64_t i = 0; i < npub; i++) {
    const uint32_t f = dispatch_one(c, r + offsets[i], offsets[i + 1] - offsets[i], policy, seed, pub_seq + i,
                                    chosen + offsets[i]);
    if (failed) failed[i] = f;
  }
}

// CPU baseline: `reps` passes over the batch on `threads` threads
// (publishes partitioned).  Returns elapsed ns.
long long shared_oracle_select_timed(const void* emits, const uint64_t* offsets, uint64_t npub, uint32_t policy,
                                     uint64_t seed, const uint8_t* states, uint64_t n_states, uint32_t local_node,
                                     uint8_t* chosen, int reps, int threads) {
  const auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < reps; k++) {
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; t++) {
      const uint64_t lo = npub * t / threads, hi = npub * (t + 1) / threads;
      ts.emplace_back([=] {
        shared_oracle_select(emits, offsets + lo, hi - lo, policy, seed, lo, states, n_states, local_node, chosen,
                             nullptr);
      });
    }
    for (auto& t : ts) t.join();
  }
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

}  // extern "C"
