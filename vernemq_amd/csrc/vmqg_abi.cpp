// extern "C" boundary of libvmqgpu (include/vmqg.h).  No C++ exception and
// no torch type crosses it; every entry point maps onto the Engine.
#include <sched.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <new>

#include "vmqg_chain.h"
#include "vmqg_nullorder.h"
#include "vmqg_engine.h"

using vmqg::Engine;

struct vmqg_ctx {
  Engine e;
};

#define GUARD_BEGIN try {
#define GUARD_END                               \
  }                                             \
  catch (const std::bad_alloc&) {               \
    return VMQG_E_NOMEM;                        \
  }                                             \
  catch (...) {                                 \
    return VMQG_E_INVAL;                        \
  }

extern "C" {

int vmqg_abi_version(void) { return VMQG_ABI_VERSION; }

#ifndef VMQG_BUILD_ID
#define VMQG_BUILD_ID "vmqg-build:unknown"
#endif
const char* vmqg_build_id(void) { return VMQG_BUILD_ID; }

vmqg_ctx* vmqg_create(const vmqg_config* cfg, int* err) {
  int rc = VMQG_OK;
  vmqg_ctx* c = nullptr;
  try {
    if (!cfg) { rc = VMQG_E_INVAL; }
    else {
      c = new vmqg_ctx();
      rc = c->e.init(*cfg);
      if (rc != VMQG_OK) { delete c; c = nullptr; }
    }
  } catch (const std::bad_alloc&) {
    delete c; c = nullptr; rc = VMQG_E_NOMEM;
  } catch (...) {
    delete c; c = nullptr; rc = VMQG_E_INVAL;
  }
  if (err) *err = rc;
  return c;
}

void vmqg_destroy(vmqg_ctx* ctx) { delete ctx; }

int vmqg_intern_words(vmqg_ctx* ctx, const uint8_t* bytes, const uint64_t* offs, uint32_t n, int create,
                      uint32_t* ids_out) {
  if (!ctx || (n && (!bytes || !offs || !ids_out))) return VMQG_E_INVAL;
  GUARD_BEGIN
  for (uint32_t i = 0; i < n; i++) {
    if (offs[i + 1] < offs[i]) return VMQG_E_INVAL;
    ids_out[i] = ctx->e.intern(bytes + offs[i], offs[i + 1] - offs[i], create != 0);
  }
  return VMQG_OK;
  GUARD_END
}

// The words of a publish topic, 8 bytes at a time: on_word(start, len) per
// '/'-separated word (empty words kept), false as soon as a '+' or '#'
// appears (vmq_topic:validate_topic(publish, T), vmq_topic.erl:82-112).
// Loads never cross into the next page past the topic's end.
}  // extern "C"
template <class F>
static inline bool split_publish_topic(const uint8_t* p, size_t len, F&& on_word) {
  constexpr uint64_t kOnes = 0x0101010101010101ull, kHigh = 0x8080808080808080ull;
  size_t start = 0;
  for (size_t i = 0; i < len; i += 8) {
    const size_t m = len - i < 8 ? len - i : 8;
    uint64_t x = 0;
#if defined(VMQG_NO_OVERREAD)
    constexpr bool kWide = false;   // a page-safe over-read is still one to ASan
#else
    constexpr bool kWide = true;
#endif
    if (m == 8 || (kWide && ((uintptr_t)(p + i) & 4095) <= 4096 - 8)) memcpy(&x, p + i, 8);
    else memcpy(&x, p + i, m);
    const uint64_t valid = m == 8 ? ~0ull : ~0ull >> (64 - 8 * m);
    auto eq = [x, valid](uint8_t c) {
      const uint64_t y = x ^ (kOnes * c);
      return (y - kOnes) & ~y & kHigh & valid;   // exact per byte below the first match, enough for "any"
    };
    if (eq('+') | eq('#')) return false;
    for (uint64_t sl = eq('/'); sl; sl &= sl - 1) {
      // the zero-byte trick can flag a false byte only above a true one:
      // confirm each candidate separator
      const size_t j = i + ((size_t)__builtin_ctzll(sl) >> 3);
      if (p[j] != '/') continue;
      on_word(start, j - start);
      start = j + 1;
    }
  }
  on_word(start, len - start);
  return true;
}
extern "C" {

// vmq_topic:validate_topic(publish, Topic)  (vmq_topic.erl:82-112): split on
// '/', keep empty words, reject '+' / '#' anywhere, size 0 or > 65,536.
int vmqg_prepare_publish(vmqg_ctx* ctx, uint32_t mountpoint, const uint8_t* topic, size_t len,
                         uint32_t* words_out, uint32_t cap, vmqg_pub* pub) {
  if (!ctx || !pub || (len && !topic)) return VMQG_E_INVAL;
  if (len == 0 || len > 65536) return VMQG_E_INVAL;
  GUARD_BEGIN
  uint32_t n = 0, unknown = 0;
  bool over = false;
  const bool ok = split_publish_topic(topic, len, [&](size_t start, size_t wl) {
    if (n >= cap) { over = true; return; }
    const uint32_t id = ctx->e.intern(topic + start, wl, false);
    unknown |= id == vmqg::kUnknownWord;
    words_out[n++] = id;
  });
  if (!ok) return VMQG_E_INVAL;
  if (over) return VMQG_E_OVERFLOW;
  pub->mountpoint = mountpoint;
  pub->word_off = 0;
  pub->nwords = n;
  pub->flags = (topic[0] == '$' ? VMQG_PUB_DOLLAR : 0u) | (unknown ? VMQG_PUB_UNKNOWN : 0u);
  return VMQG_OK;
  GUARD_END
}

// The batched form: topics are split block by block; every word of a block is
// hashed and its dictionary slot prefetched, then the block's words are
// resolved — the probes of ~kBlock topics overlap instead of each costing a
// full memory round trip (a 1M-word dictionary is 64 MB of slots).
int vmqg_prepare_publishes(vmqg_ctx* ctx, size_t n, const uint32_t* mountpoints, const uint8_t* const* topics,
                           const size_t* lens, vmqg_pub* pubs_out, int32_t* rc_out, uint32_t* words_out,
                           size_t wcap, size_t* nwords_out) {
  if (!ctx || (n && (!mountpoints || !topics || !lens || !pubs_out || !rc_out || !words_out))) return VMQG_E_INVAL;
  GUARD_BEGIN
  const vmqg::WordDict& d = ctx->e.dict;
  constexpr size_t kBlock = 64;
  static thread_local std::vector<vmqg::WordDict::Key> keys;
  size_t nw = 0;
  for (size_t lo = 0; lo < n; lo += kBlock) {
    const size_t hi = std::min(n, lo + kBlock);
    keys.clear();
    // split + validate (vmq_topic:validate_topic(publish, T), vmq_topic.erl:82-112),
    // hash and prefetch; words_out holds the key index until resolved
    for (size_t t = lo; t < hi; t++) {
      const uint8_t* tp = topics[t];
      const size_t len = lens[t];
      vmqg_pub& pub = pubs_out[t];
      pub = vmqg_pub{mountpoints[t], (uint32_t)nw, 0, 0};
      rc_out[t] = VMQG_OK;
      if (len == 0 || len > 65536 || !tp) { rc_out[t] = VMQG_E_INVAL; pub.mountpoint = 0; continue; }
      if (nw + len + 1 > wcap) {
        // a topic of len bytes has <= len + 1 words: count them before giving up
        size_t words = 1;
        for (size_t i = 0; i < len; i++) words += tp[i] == '/';
        if (nw + words > wcap) return VMQG_E_OVERFLOW;
      }
      const size_t k0 = keys.size();
      const bool bad = !split_publish_topic(tp, len, [&](size_t start, size_t wl) {
        keys.push_back(vmqg::WordDict::key(tp + start, wl));
        d.prefetch(keys.back());
        words_out[nw + pub.nwords++] = (uint32_t)(keys.size() - 1);
      });
      if (bad) {
        keys.resize(k0);
        rc_out[t] = VMQG_E_INVAL;
        pub = vmqg_pub{0, (uint32_t)nw, 0, 0};
        continue;
      }
      if (tp[0] == '$') pub.flags |= VMQG_PUB_DOLLAR;
      nw += pub.nwords;
    }
    // resolve the block's words (their slots are on their way)
    for (size_t t = lo; t < hi; t++) {
      vmqg_pub& pub = pubs_out[t];
      if (rc_out[t]) continue;
      uint32_t unknown = 0;
      for (uint32_t j = 0; j < pub.nwords; j++) {
        uint32_t& w = words_out[pub.word_off + j];
        const uint32_t f = d.find(keys[w]);
        w = f == vmqg::WordDict::kVoid ? vmqg::kUnknownWord : f;
        unknown |= w == vmqg::kUnknownWord;
      }
      if (unknown) pub.flags |= VMQG_PUB_UNKNOWN;
    }
  }
  if (nwords_out) *nwords_out = nw;
  return VMQG_OK;
  GUARD_END
}

// fold/4 takes the Topic word list as given (vmq_reg_trie.erl:59-66): each
// word looked up as one dictionary key, nothing split or validated.  Blocks
// of publishes are hashed and prefetched before they are resolved, as above.
int vmqg_prepare_word_lists(vmqg_ctx* ctx, size_t n, const uint32_t* mountpoints, const uint32_t* counts,
                            const uint8_t* const* words, const size_t* lens, vmqg_pub* pubs_out,
                            uint32_t* words_out, size_t wcap, size_t* nwords_out) {
  if (!ctx || (n && (!mountpoints || !counts || !pubs_out))) return VMQG_E_INVAL;
  GUARD_BEGIN
  const vmqg::WordDict& d = ctx->e.dict;
  constexpr size_t kBlock = 64;
  static thread_local std::vector<vmqg::WordDict::Key> keys;
  size_t nw = 0;
  for (size_t lo = 0; lo < n; lo += kBlock) {
    const size_t hi = std::min(n, lo + kBlock);
    keys.clear();
    const size_t nw0 = nw;
    for (size_t t = lo; t < hi; t++) {
      const uint32_t c = counts[t];
      if (nw + c > wcap) return VMQG_E_OVERFLOW;
      if (c && (!words || !lens || !words_out)) return VMQG_E_INVAL;
      vmqg_pub& pub = pubs_out[t];
      pub = vmqg_pub{mountpoints[t], (uint32_t)nw, c, 0};
      for (uint32_t j = 0; j < c; j++) {
        const uint8_t* p = words[nw + j];
        const size_t l = lens[nw + j];
        if (l && !p) return VMQG_E_INVAL;
        static const uint8_t kNoBytes[16] = {0};   // an empty binary may come without a pointer
        keys.push_back(vmqg::WordDict::key(l ? p : kNoBytes, l));
        d.prefetch(keys.back());
      }
      // MQTT-4.7.2-1 is decided on the first word's first byte (vmq_reg_trie.erl:285-288)
      if (c && lens[nw] && words[nw][0] == '$') pub.flags |= VMQG_PUB_DOLLAR;
      nw += c;
    }
    for (size_t k = 0; k < nw - nw0; k++) {
      const uint32_t f = d.find(keys[k]);
      words_out[nw0 + k] = f == vmqg::WordDict::kVoid ? vmqg::kUnknownWord : f;
    }
    for (size_t t = lo; t < hi; t++) {
      vmqg_pub& pub = pubs_out[t];
      for (uint32_t j = 0; j < pub.nwords; j++)
        if (words_out[pub.word_off + j] == vmqg::kUnknownWord) { pub.flags |= VMQG_PUB_UNKNOWN; break; }
    }
  }
  if (nwords_out) *nwords_out = nw;
  return VMQG_OK;
  GUARD_END
}

uint64_t vmqg_dict_generation(vmqg_ctx* ctx) { return ctx ? ctx->e.dict.generation() : 0; }

int vmqg_released_ids(vmqg_ctx* ctx, uint32_t kind, const uint32_t** ids, size_t* n) {
  if (!ctx || kind > 1 || !ids || !n) return VMQG_E_INVAL;
  *ids = ctx->e.term_released[kind].data();
  *n = ctx->e.term_released[kind].size();
  return VMQG_OK;
}

uint64_t vmqg_dict_grace_token(vmqg_ctx* ctx) { return ctx ? ++ctx->e.dict.retire_token : 0; }

int vmqg_dict_release(vmqg_ctx* ctx, uint64_t token) {
  if (!ctx) return VMQG_E_INVAL;
  if (ctx->e.replica) return VMQG_E_STATE;
  GUARD_BEGIN
  ctx->e.release_words(token);
  return VMQG_OK;
  GUARD_END
}

int vmqg_apply_stage(vmqg_ctx* ctx, const vmqg_op* ops, size_t n, const uint32_t* words, size_t nwords) {
  if (!ctx || (n && !ops) || (nwords && !words)) return VMQG_E_INVAL;
  GUARD_BEGIN
  return ctx->e.stage_ops(ops, n, words, nwords);
  GUARD_END
}

int vmqg_apply_commit(vmqg_ctx* ctx, uint64_t* epoch_out) {
  if (!ctx) return VMQG_E_INVAL;
  GUARD_BEGIN
  const int rc = ctx->e.commit();
  if (epoch_out) *epoch_out = ctx->e.epoch;
  return rc;
  GUARD_END
}

int vmqg_apply_ops(vmqg_ctx* ctx, const vmqg_op* ops, size_t n, const uint32_t* words, size_t nwords,
                   uint64_t* epoch_out) {
  const int rc = vmqg_apply_stage(ctx, ops, n, words, nwords);
  if (rc && (!ctx || !ctx->e.staged)) return rc;   // rejected before any change
  const int rc2 = vmqg_apply_commit(ctx, epoch_out);
  return rc ? rc : rc2;
}

static int grow(void** p, uint64_t* cap, uint64_t need) {
  if (*cap >= need) return VMQG_OK;
  if (*p) hipFree(*p);
  *p = nullptr;
  uint64_t c = 1;
  while (c < need) c <<= 1;
  if (hipMalloc(p, c) != hipSuccess) { *cap = 0; return VMQG_E_NOMEM; }
  *cap = c;
  return VMQG_OK;
}

// Host-buffer match in records (esz 16) or range (esz 8) mode: stage the
// batch, match on the context stream, copy offsets (and, when they fit, the
// entries) back.  A tier-2 stack overflow (never expected: the stack is
// sized from the trie depth) is retried with a 4x larger stack, so a
// publish the reference answers is never refused.
static int match_host(Engine& e, const vmqg_pub* pubs, size_t npub, const uint32_t* words, size_t nwords,
                      void* out, size_t esz, size_t out_cap, size_t* out_n, uint64_t* offsets) {
  if (!e.has_device) return VMQG_E_DEVICE;
  for (size_t i = 0; i < npub; i++)
    if ((uint64_t)pubs[i].word_off + pubs[i].nwords > nwords) return VMQG_E_INVAL;   // 0 words: fold(MP, [])
  hipSetDevice(e.device);
  int rc;
  if ((rc = grow(&e.d_pubs, &e.d_pubs_cap, (npub + 1) * sizeof(vmqg_pub)))) return rc;
  if ((rc = grow(&e.d_words, &e.d_words_cap, (nwords + 1) * sizeof(uint32_t)))) return rc;
  if ((rc = grow(&e.d_offs, &e.d_offs_cap, (npub + 1) * sizeof(uint64_t)))) return rc;
  if ((rc = grow(&e.d_out, &e.d_out_cap, (out_cap + 1) * esz))) return rc;
  hipStream_t st = e.stream;
  if (npub && hipMemcpyAsync(e.d_pubs, pubs, npub * sizeof(vmqg_pub), hipMemcpyHostToDevice, st) != hipSuccess)
    return VMQG_E_DEVICE;
  if (nwords && hipMemcpyAsync(e.d_words, words, nwords * 4, hipMemcpyHostToDevice, st) != hipSuccess)
    return VMQG_E_DEVICE;
  for (int attempt = 0;; attempt++) {
    vmqg::Record* rec = esz == sizeof(vmqg_emit) ? static_cast<vmqg::Record*>(e.d_out) : nullptr;
    vmqg_range* rng = esz == sizeof(vmqg_range) ? static_cast<vmqg_range*>(e.d_out) : nullptr;
    rc = e.match_device(static_cast<const vmqg_pub*>(e.d_pubs), (uint32_t)npub, static_cast<const uint32_t*>(e.d_words),
                        rec, rec ? out_cap : 0, rng, rng ? out_cap : 0, static_cast<uint64_t*>(e.d_offs), st);
    if (rc) return rc;
    if (hipMemcpyAsync(offsets, e.d_offs, (npub + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, st) != hipSuccess)
      return VMQG_E_DEVICE;
    rc = e.match_status(st);
    if (rc != VMQG_E_FRONTIER || attempt >= 6) break;
    e.o_cap_floor = std::max<uint64_t>(e.o_cap_floor, (uint64_t)e.o_cap * 4);
  }
  const uint64_t total = offsets[npub];
  if (out_n) *out_n = total;
  if (rc == VMQG_E_OVERFLOW || total > out_cap) return VMQG_E_OVERFLOW;
  if (rc) return rc;
  if (total && hipMemcpy(out, e.d_out, total * esz, hipMemcpyDeviceToHost) != hipSuccess) return VMQG_E_DEVICE;
  return VMQG_OK;
}

int vmqg_match_batch(vmqg_ctx* ctx, const vmqg_pub* pubs, size_t npub, const uint32_t* words, size_t nwords,
                     vmqg_emit* out, size_t out_cap, size_t* out_n, uint64_t* offsets) {
  if (!ctx || !offsets || (npub && !pubs) || (nwords && !words) || (out_cap && !out)) return VMQG_E_INVAL;
  if (npub > 0xFFFFFFF0u) return VMQG_E_LIMIT;
  GUARD_BEGIN
  return match_host(ctx->e, pubs, npub, words, nwords, out, sizeof(vmqg_emit), out_cap, out_n, offsets);
  GUARD_END
}

int vmqg_match_ranges(vmqg_ctx* ctx, const vmqg_pub* pubs, size_t npub, const uint32_t* words, size_t nwords,
                      vmqg_range* out, size_t out_cap, size_t* out_n, uint64_t* offsets) {
  if (!ctx || !offsets || (npub && !pubs) || (nwords && !words) || (out_cap && !out)) return VMQG_E_INVAL;
  if (npub > 0xFFFFFFF0u) return VMQG_E_LIMIT;
  GUARD_BEGIN
  return match_host(ctx->e, pubs, npub, words, nwords, out, sizeof(vmqg_range), out_cap, out_n, offsets);
  GUARD_END
}

// ---- pipelined host-buffer matching (vmqg_hbatch_*) --------------------
struct vmqg_hbatch {
  int device = -1;
  hipStream_t cs = nullptr;                     // copy stream: H2D of the inputs, D2H of the entries
  hipEvent_t ev_in = nullptr, ev_k = nullptr, ev_out = nullptr;
  vmqg_pub* h_pubs = nullptr; uint32_t* h_words = nullptr; uint64_t* h_offs = nullptr;
  void* h_out = nullptr; uint32_t* h_err = nullptr;
  uint64_t h_pubs_cap = 0, h_words_cap = 0, h_offs_cap = 0, h_out_cap = 0;   // bytes
  void* d_pubs = nullptr; void* d_words = nullptr; void* d_offs = nullptr; void* d_out = nullptr;
  uint64_t d_pubs_cap = 0, d_words_cap = 0, d_offs_cap = 0, d_out_cap = 0;   // bytes
  uint64_t want_entries = 0;   // output capacity (entries) of the next submit
  uint64_t out_entries = 0;    // ... of the submitted one
  uint64_t spec_entries = 0;   // entries already copied back with the offsets (speculative D2H)
  double per_pub = 2.0;        // entries per publish seen so far (sizes the speculative copy)
  size_t npub = 0, esz = 16;
  uint64_t epoch = 0, total = 0;
  bool frontier = false;
  int state = 0;               // 0 idle, 1 submitted, 2 offsets read
};

// Waits for a round's event by polling (with yields) for up to ~2 ms, then
// blocking: an interrupt-driven wake-up costs tens of microseconds per round,
// a poll of the completion signal under one; the poller yields its core to
// the batchers that are preparing or folding.
static hipError_t wait_event(hipEvent_t ev) {
  for (int i = 0; i < 20000; i++) {
    const hipError_t q = hipEventQuery(ev);
    if (q != hipErrorNotReady) return q;
    sched_yield();
  }
  return hipEventSynchronize(ev);
}

static int grow_pinned(void** p, uint64_t* cap, uint64_t need) {
  if (*cap >= need) return VMQG_OK;
  if (*p) hipHostFree(*p);
  *p = nullptr;
  uint64_t c = 4096;
  while (c < need) c <<= 1;
  if (hipHostMalloc(p, c, hipHostMallocDefault) != hipSuccess) { *cap = 0; return VMQG_E_NOMEM; }
  *cap = c;
  return VMQG_OK;
}

vmqg_hbatch* vmqg_hbatch_new(vmqg_ctx* ctx) {
  if (!ctx || !ctx->e.has_device) return nullptr;
  vmqg_hbatch* hb = new (std::nothrow) vmqg_hbatch();
  if (!hb) return nullptr;
  hb->device = ctx->e.device;
  hipSetDevice(hb->device);
  const unsigned evf = hipEventDisableTiming | hipEventBlockingSync;   // waiters sleep: batchers need the cores
  if (hipStreamCreateWithFlags(&hb->cs, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&hb->ev_in, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&hb->ev_k, evf) != hipSuccess || hipEventCreateWithFlags(&hb->ev_out, evf) != hipSuccess ||
      hipHostMalloc((void**)&hb->h_err, 64, hipHostMallocDefault) != hipSuccess) {
    vmqg_hbatch_free(hb);
    return nullptr;
  }
  return hb;
}

void vmqg_hbatch_free(vmqg_hbatch* hb) {
  if (!hb) return;
  hipSetDevice(hb->device);
  if (hb->cs) hipStreamSynchronize(hb->cs);
  if (hb->state == 1 && hb->ev_k) hipEventSynchronize(hb->ev_k);
  for (hipEvent_t e : {hb->ev_in, hb->ev_k, hb->ev_out}) if (e) hipEventDestroy(e);
  for (void* p : {(void*)hb->h_pubs, (void*)hb->h_words, (void*)hb->h_offs, hb->h_out, (void*)hb->h_err})
    if (p) hipHostFree(p);
  for (void* p : {hb->d_pubs, hb->d_words, hb->d_offs, hb->d_out}) if (p) hipFree(p);
  if (hb->cs) hipStreamDestroy(hb->cs);
  delete hb;
}

int vmqg_hbatch_inputs(vmqg_hbatch* hb, size_t npub, size_t nwords, vmqg_pub** pubs, uint32_t** words) {
  if (!hb || !pubs || !words || hb->state == 1) return VMQG_E_INVAL;
  int rc;
  if ((rc = grow_pinned((void**)&hb->h_pubs, &hb->h_pubs_cap, (npub + 1) * sizeof(vmqg_pub))) ||
      (rc = grow_pinned((void**)&hb->h_words, &hb->h_words_cap, (nwords + 1) * sizeof(uint32_t))))
    return rc;
  *pubs = hb->h_pubs;
  *words = hb->h_words;
  return VMQG_OK;
}

int vmqg_hbatch_submit(vmqg_ctx* ctx, vmqg_hbatch* hb, size_t npub, size_t nwords, int ranges) {
  if (!ctx || !hb || hb->state == 1 || npub > 0xFFFFFFF0u) return VMQG_E_INVAL;
  if (npub && (hb->h_pubs_cap < npub * sizeof(vmqg_pub) || hb->h_words_cap < nwords * sizeof(uint32_t)))
    return VMQG_E_INVAL;
  GUARD_BEGIN
  Engine& e = ctx->e;
  if (!e.has_device || e.device != hb->device) return VMQG_E_DEVICE;
  for (size_t i = 0; i < npub; i++)
    if ((uint64_t)hb->h_pubs[i].word_off + hb->h_pubs[i].nwords > nwords)
      return VMQG_E_INVAL;
  hipSetDevice(e.device);
  const size_t esz = ranges ? sizeof(vmqg_range) : sizeof(vmqg_emit);
  if (hb->esz != esz) hb->want_entries = 0;   // a mode change restarts the output sizing
  hb->esz = esz;
  hb->want_entries = std::max<uint64_t>(hb->want_entries, (uint64_t)npub * (ranges ? 4 : 8) + 1024);
  int rc;
  if ((rc = grow(&hb->d_pubs, &hb->d_pubs_cap, (npub + 1) * sizeof(vmqg_pub))) ||
      (rc = grow(&hb->d_words, &hb->d_words_cap, (nwords + 1) * sizeof(uint32_t))) ||
      (rc = grow(&hb->d_offs, &hb->d_offs_cap, (npub + 1) * sizeof(uint64_t))) ||
      (rc = grow(&hb->d_out, &hb->d_out_cap, hb->want_entries * esz)) ||
      (rc = grow_pinned((void**)&hb->h_offs, &hb->h_offs_cap, (npub + 1) * sizeof(uint64_t))))
    return rc;
  hb->out_entries = hb->d_out_cap / esz;
  if (hb->frontier) {   // the last match overflowed a tier-2 stack: a larger one (as match_host)
    e.o_cap_floor = std::max<uint64_t>(e.o_cap_floor, (uint64_t)e.o_cap * 4);
    hb->frontier = false;
  }
  // inputs on the copy stream, so they overlap the kernels already queued
  if (npub) {
    if (hipMemcpyAsync(hb->d_pubs, hb->h_pubs, npub * sizeof(vmqg_pub), hipMemcpyHostToDevice, hb->cs) != hipSuccess ||
        (nwords && hipMemcpyAsync(hb->d_words, hb->h_words, nwords * 4, hipMemcpyHostToDevice, hb->cs) != hipSuccess) ||
        hipEventRecord(hb->ev_in, hb->cs) != hipSuccess || hipStreamWaitEvent(e.stream, hb->ev_in, 0) != hipSuccess)
      return VMQG_E_DEVICE;
  }
  vmqg::Record* rec = ranges ? nullptr : static_cast<vmqg::Record*>(hb->d_out);
  vmqg_range* rng = ranges ? static_cast<vmqg_range*>(hb->d_out) : nullptr;
  rc = e.match_device(static_cast<const vmqg_pub*>(hb->d_pubs), (uint32_t)npub, static_cast<const uint32_t*>(hb->d_words),
                      rec, rec ? hb->out_entries : 0, rng, rng ? hb->out_entries : 0, static_cast<uint64_t*>(hb->d_offs),
                      e.stream);
  if (rc) return rc;
  // this match's offsets and error bits back, and the bits cleared for the
  // next call; with them, speculatively, as many entries as this hbatch's
  // batches have had per publish (+ 25 %): when they all fit, the entries
  // need no second round trip (one wait per round instead of two)
  uint32_t* d_err = e.d_status + 2 * Engine::kStatusSet;
  hb->spec_entries = std::min<uint64_t>(hb->out_entries, (uint64_t)(hb->per_pub * 1.25 * (double)npub) + 256);
  if ((rc = grow_pinned(&hb->h_out, &hb->h_out_cap, hb->spec_entries * esz + 16))) return rc;
  if (hipMemcpyAsync(hb->h_offs, hb->d_offs, (npub + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, e.stream) != hipSuccess ||
      hipMemcpyAsync(hb->h_err, d_err, 4, hipMemcpyDeviceToHost, e.stream) != hipSuccess ||
      hipMemsetAsync(d_err, 0, 4, e.stream) != hipSuccess ||
      (hb->spec_entries &&
       hipMemcpyAsync(hb->h_out, hb->d_out, hb->spec_entries * esz, hipMemcpyDeviceToHost, e.stream) != hipSuccess) ||
      hipEventRecord(hb->ev_k, e.stream) != hipSuccess)
    return VMQG_E_DEVICE;
  hb->npub = npub;
  hb->epoch = e.epoch;
  hb->state = 1;
  return VMQG_OK;
  GUARD_END
}

int vmqg_hbatch_offsets(vmqg_hbatch* hb, const uint64_t** offsets, uint64_t* total, uint64_t* epoch) {
  if (!hb || hb->state == 0) return VMQG_E_INVAL;
  hipSetDevice(hb->device);
  if (hb->state == 1) {
    if (wait_event(hb->ev_k) != hipSuccess) { hb->state = 0; return VMQG_E_DEVICE; }
    hb->state = 2;
  }
  hb->total = hb->h_offs[hb->npub];
  if (hb->npub) hb->per_pub = 0.75 * hb->per_pub + 0.25 * ((double)hb->total / (double)hb->npub);
  if (offsets) *offsets = hb->h_offs;
  if (total) *total = hb->total;
  if (epoch) *epoch = hb->epoch;
  const uint32_t err = *hb->h_err;
  if (err & 2u) { hb->frontier = true; hb->state = 0; return VMQG_E_FRONTIER; }
  if ((err & 4u) || hb->total > hb->out_entries) {
    hb->want_entries = hb->total + hb->total / 4 + 1024;
    hb->state = 0;
    return VMQG_E_OVERFLOW;
  }
  if (err & (8u | 16u)) { hb->state = 0; return VMQG_E_DEVICE; }
  return VMQG_OK;
}

int vmqg_hbatch_entries(vmqg_hbatch* hb, const void** entries) {
  if (!hb || hb->state != 2) return VMQG_E_INVAL;
  hipSetDevice(hb->device);
  hb->state = 0;
  if (hb->total > hb->spec_entries) {   // the rest, behind the speculative part already here
    const uint64_t have = hb->spec_entries;
    if (hb->h_out_cap < hb->total * hb->esz + 16) {   // a larger pinned buffer: keep what arrived
      void* nb = nullptr;
      uint64_t ncap = 0;
      int rc;
      if ((rc = grow_pinned(&nb, &ncap, hb->total * hb->esz + 16))) return rc;
      memcpy(nb, hb->h_out, have * hb->esz);
      hipHostFree(hb->h_out);
      hb->h_out = nb;
      hb->h_out_cap = ncap;
    }
    char* dst = static_cast<char*>(hb->h_out) + have * hb->esz;
    const char* src = static_cast<const char*>(hb->d_out) + have * hb->esz;
    if (hipMemcpyAsync(dst, src, (hb->total - have) * hb->esz, hipMemcpyDeviceToHost, hb->cs) != hipSuccess ||
        hipEventRecord(hb->ev_out, hb->cs) != hipSuccess || wait_event(hb->ev_out) != hipSuccess)
      return VMQG_E_DEVICE;
  }
  if (entries) *entries = hb->h_out;
  return VMQG_OK;
}

int vmqg_match_device(vmqg_ctx* ctx, const vmqg_pub* d_pubs, uint32_t npub, const uint32_t* d_words,
                      vmqg_emit* d_out, uint64_t out_cap, uint64_t* d_offsets, void* stream) {
  if (!ctx || !d_offsets || (npub && (!d_pubs || !d_words))) return VMQG_E_INVAL;
  GUARD_BEGIN
  hipSetDevice(ctx->e.device);
  return ctx->e.match_device(d_pubs, npub, d_words, reinterpret_cast<vmqg::Record*>(d_out), out_cap, nullptr, 0,
                             d_offsets, vmqg::caller_stream(stream));
  GUARD_END
}

int vmqg_match_ranges_device(vmqg_ctx* ctx, const vmqg_pub* d_pubs, uint32_t npub, const uint32_t* d_words,
                             vmqg_range* d_out, uint64_t out_cap, uint64_t* d_offsets, void* stream) {
  if (!ctx || !d_offsets || (npub && (!d_pubs || !d_words)) || (out_cap && !d_out)) return VMQG_E_INVAL;
  GUARD_BEGIN
  // a non-null range buffer selects range mode even at out_cap 0
  static vmqg_range dummy;
  hipSetDevice(ctx->e.device);
  return ctx->e.match_device(d_pubs, npub, d_words, nullptr, 0, d_out ? d_out : &dummy, out_cap, d_offsets,
                             vmqg::caller_stream(stream));
  GUARD_END
}

int vmqg_records(vmqg_ctx* ctx, const vmqg_emit** recs, uint64_t* n) {
  if (!ctx || !recs || !n) return VMQG_E_INVAL;
  Engine& e = ctx->e;
  if (e.replica) return VMQG_E_STATE;
  *recs = reinterpret_cast<const vmqg_emit*>(e.region<uint8_t>(e.lay.rec_off));
  *n = e.lay.rec_cap;
  return VMQG_OK;
}

int vmqg_epoch(vmqg_ctx* ctx, uint64_t* epoch) {
  if (!ctx || !epoch) return VMQG_E_INVAL;
  *epoch = ctx->e.epoch;
  return VMQG_OK;
}

int vmqg_records_at(vmqg_ctx* ctx, uint64_t epoch, const vmqg_emit** recs, uint64_t* n) {
  if (!ctx || !recs || !n) return VMQG_E_INVAL;
  Engine& e = ctx->e;
  if (e.replica) return VMQG_E_STATE;
  if (epoch > e.epoch || e.rec_epoch > epoch) return VMQG_E_STATE;   // a later apply rewrote record slots
  return vmqg_records(ctx, recs, n);
}

int vmqg_records_pin(vmqg_ctx* ctx, uint64_t epoch, const vmqg_emit** recs, uint64_t* n, uint32_t* pin) {
  if (!ctx || !recs || !n || !pin) return VMQG_E_INVAL;
  const vmqg::Record* r = nullptr;
  const int rc = ctx->e.records_pin(epoch, &r, n, pin);
  *recs = reinterpret_cast<const vmqg_emit*>(r);
  return rc;
}

void vmqg_records_unpin(vmqg_ctx* ctx, uint32_t pin) {
  if (ctx) ctx->e.records_unpin(pin);
}

int vmqg_release_stream(vmqg_ctx* ctx, void* stream) {
  if (!ctx) return VMQG_E_INVAL;
  if (!ctx->e.has_device) return VMQG_OK;
  hipSetDevice(ctx->e.device);
  return vmqg::chain_release(ctx->e.ev_match_done, ctx->e.ev_stream, vmqg::caller_stream(stream));
}

int vmqg_match_status(vmqg_ctx* ctx, void* stream) {
  if (!ctx) return VMQG_E_INVAL;
  GUARD_BEGIN
  return ctx->e.match_status(vmqg::caller_stream(stream));
  GUARD_END
}

int vmqg_stats(vmqg_ctx* ctx, vmqg_stats_t* out) {
  if (!ctx || !out) return VMQG_E_INVAL;
  const Engine& e = ctx->e;
  out->subs = e.n_subs_objects + e.n_remote_keys;
  out->device_bytes = e.has_device ? e.d_arena_bytes : e.lay.total_bytes;
  out->trie_edges = e.edge_live;
  out->trie_nodes = e.n_trie_nodes;
  out->trie_topics = e.n_trie_topics;
  out->subs_objects = e.n_subs_objects;
  out->fanout_objects = e.n_fanout;
  out->remote_keys = e.n_remote_keys;
  out->epoch = e.epoch;
  out->rebuilds = e.rebuilds;
  out->paths = e.paths.size() - e.free_paths.size();
  out->words = e.dict.size();
  out->keys = e.keys.size() - e.free_keys.size();
  out->topics = e.topics.size() - e.free_topics.size();
  out->words_retired = e.word_retired.size();
  out->words_released = e.words_released;
  out->host_bytes = e.host_bytes();
  out->deferred_tier1 = e.last_deferred[0];
  out->deferred_tier2 = e.last_deferred[1];
  out->ops_applied = e.ops_applied;
  out->apply_host_ns = e.apply_host_ns;
  out->apply_upload_ns = e.apply_upload_ns;
  out->apply_wait_ns = e.apply_wait_ns;
  out->patch_bytes = e.patch_bytes;
  out->image_bytes = e.image_bytes;
  out->max_depth = e.stack_depth();
  out->many_key = e.last_many;
  out->retried = e.last_retried;
  out->wave_entries = e.last_wave_entries;
  out->wide_entries = e.last_wide_entries;
  out->dedup = e.last_dedup;
  out->dedup_walked = e.last_dedup_walked;
  out->error_bits = e.last_err_bits;
  out->reader_waits = e.rb_waits;
  out->reader_wait_ns = e.rb_wait_ns;
  return VMQG_OK;
}

int vmqg_dump(vmqg_ctx* ctx, const char** text, size_t* len) {
  if (!ctx || !text || !len) return VMQG_E_INVAL;
  if (ctx->e.replica) return VMQG_E_STATE;
  GUARD_BEGIN
  ctx->e.dump_text = ctx->e.dump();
  *text = ctx->e.dump_text.data();
  *len = ctx->e.dump_text.size();
  return VMQG_OK;
  GUARD_END
}

int vmqg_set_option(vmqg_ctx* ctx, const char* name, int64_t value) {
  if (!ctx || !name) return VMQG_E_INVAL;
  GUARD_BEGIN   // "reader_records" copies the record table twice: bad_alloc -> VMQG_E_NOMEM
  Engine& e = ctx->e;
  const std::string n(name);
  if (n == "fast_g") {
    if (value != 0 && value != 1 && value != 2 && value != 4) return VMQG_E_INVAL;
    e.opt_fast_g = (uint32_t)value;
  } else if (n == "trieless") {
    if (value < 0 || value > 1) return VMQG_E_INVAL;
    e.opt_trieless = (uint32_t)value;
  } else if (n == "fused") {
    if (value < 0 || value > 1) return VMQG_E_INVAL;
    e.opt_fused = (uint32_t)value;
  } else if (n == "exact_one") {   // slots written from now on; either kind is matched alike
    if (value < 0 || value > 1) return VMQG_E_INVAL;
    e.opt_exact_one = (uint32_t)value;
  } else if (n == "root_flags") {
    e.opt_flags = value ? (e.opt_flags | vmqg::kOptRootFlags) : (e.opt_flags & ~vmqg::kOptRootFlags);
  } else if (n == "nt_stores") {
    e.opt_flags = value ? (e.opt_flags | vmqg::kOptNtStores) : (e.opt_flags & ~vmqg::kOptNtStores);
  } else if (n == "dedupe") {
    if (value < 0 || value > 2) return VMQG_E_INVAL;
    e.opt_dedupe = (uint32_t)value;
  } else if (n == "groups") {
    if (value < 0 || value > 1) return VMQG_E_INVAL;
    e.opt_groups = (uint32_t)value;
  } else if (n == "heavy_min") {
    if (value < 0 || value > (1 << 30)) return VMQG_E_INVAL;
    e.opt_heavy_min = (uint32_t)value;
  } else if (n == "reader_records") {   // the readers' record buffers (vmqg_records_pin): on only
    if (value != 1 || e.replica) return VMQG_E_INVAL;
    e.enable_reader_records();
  } else if (n == "exfilter") {
    if (value < 0 || value > 2) return VMQG_E_INVAL;
    e.opt_exfilter = (uint32_t)value;
  } else if (n == "dd_g") {
    if (value != 1 && value != 4) return VMQG_E_INVAL;
    e.opt_dd_g = (uint32_t)value;
  } else if (n == "count_bpc" || n == "emit_bpc") {
    if (value < 0 || value > 32) return VMQG_E_INVAL;
    (n == "count_bpc" ? e.opt_count_bpc : e.opt_emit_bpc) = (uint32_t)value;
  } else if (n == "reclaim") {   // 0: dropped paths / keys / topics / words are kept (memory for speed)
    if (value < 0 || value > 1 || e.replica) return VMQG_E_INVAL;
    e.opt_reclaim = (uint32_t)value;
  } else if (n == "fail_commits") {   // test hook: the next `value` commits fail as a device error would
    if (value < 0 || value > 1000 || e.replica) return VMQG_E_INVAL;
    e.fault_commits = (uint32_t)value;
  } else {
    return VMQG_E_INVAL;
  }
  return VMQG_OK;
  GUARD_END
}

int vmqg_set_timing(vmqg_ctx* ctx, int enable) {
  if (!ctx) return VMQG_E_INVAL;
  ctx->e.collect_times();
  ctx->e.timing = enable != 0;
  for (double& x : ctx->e.sum_stage_ns) x = 0;
  ctx->e.n_timed = 0;
  return VMQG_OK;
}

int vmqg_kernel_times(vmqg_ctx* ctx, double* count_ns, double* emit_ns, uint64_t* launches) {
  if (!ctx) return VMQG_E_INVAL;
  GUARD_BEGIN
  Engine& e = ctx->e;
  e.collect_times();
  if (count_ns) *count_ns = e.n_timed ? e.sum_stage_ns[0] / e.n_timed : 0;
  if (emit_ns) *emit_ns = e.n_timed ? e.sum_stage_ns[3] / e.n_timed : 0;
  if (launches) *launches = e.n_timed;
  return VMQG_OK;
  GUARD_END
}

int vmqg_kernel_times_ex(vmqg_ctx* ctx, double* stage_ns, uint64_t* launches) {
  if (!ctx) return VMQG_E_INVAL;
  GUARD_BEGIN
  Engine& e = ctx->e;
  e.collect_times();
  for (int k = 0; k < Engine::kTimedStages; k++)
    if (stage_ns) stage_ns[k] = e.n_timed ? e.sum_stage_ns[k] / e.n_timed : 0;
  if (launches) *launches = e.n_timed;
  return VMQG_OK;
  GUARD_END
}

int vmqg_arena(vmqg_ctx* ctx, void** d_ptr, uint64_t* bytes, uint8_t* layout_out) {
  if (!ctx) return VMQG_E_INVAL;
  if (d_ptr) *d_ptr = ctx->e.d_arena;
  if (bytes) *bytes = ctx->e.dlay.total_bytes;
  if (layout_out) memcpy(layout_out, &ctx->e.dlay, sizeof(vmqg::Layout));
  return VMQG_OK;
}

int vmqg_export_image(vmqg_ctx* ctx, void* dst, uint64_t cap) {
  if (!ctx || !dst) return VMQG_E_INVAL;
  Engine& e = ctx->e;
  if (e.replica) return VMQG_E_STATE;
  if (cap < e.lay.total_bytes) return VMQG_E_OVERFLOW;
  memcpy(dst, e.mirror.data(), e.lay.total_bytes);
  return VMQG_OK;
}

int vmqg_replica_load(vmqg_ctx* ctx, const uint8_t* layout, const void* d_src, void* stream) {
  if (!ctx || !layout || !d_src) return VMQG_E_INVAL;
  Engine& e = ctx->e;
  if (!e.replica) return VMQG_E_STATE;
  if (!e.has_device) return VMQG_E_DEVICE;
  vmqg::Layout L;
  memcpy(&L, layout, sizeof(L));
  if (L.magic != vmqg::kLayoutMagic) return VMQG_E_INVAL;
  // every match reads the exact-topic filter bits: a layout whose filter is
  // missing or outside the image would send find_exact out of bounds
  if (L.exbits_words == 0 || (L.exbits_words & (L.exbits_words - 1)) != 0 || L.exbits_off % 4 != 0 ||
      L.exbits_off > L.total_bytes || L.exbits_words * 4 > L.total_bytes - L.exbits_off)
    return VMQG_E_INVAL;
  hipSetDevice(e.device);
  hipStream_t st = vmqg::caller_stream(stream);
  if (e.d_arena_bytes < L.total_bytes) {
    if (hipDeviceSynchronize() != hipSuccess) return VMQG_E_DEVICE;
    if (e.d_arena) hipFree(e.d_arena);
    e.d_arena = nullptr; e.d_arena_bytes = 0;
    if (hipMalloc(&e.d_arena, L.total_bytes) != hipSuccess) return VMQG_E_NOMEM;
    e.d_arena_bytes = L.total_bytes;
  }
  e.lay = L;
  e.dlay = L;
  // after the matches already queued, before the ones queued later
  if (e.order_on(st) != VMQG_OK) return VMQG_E_DEVICE;
  if (hipMemcpyAsync(e.d_arena, d_src, L.total_bytes, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return VMQG_E_DEVICE;
  e.epoch++;
  return VMQG_OK;
}

int vmqg_last_patches(vmqg_ctx* ctx, const void** host_ptr, uint64_t* bytes, int* full_image) {
  if (!ctx || !host_ptr || !bytes) return VMQG_E_INVAL;
  *host_ptr = ctx->e.last_patches.data();
  *bytes = ctx->e.last_patches.size() * sizeof(vmqg::Patch);
  if (full_image) *full_image = ctx->e.last_full ? 1 : 0;
  return VMQG_OK;
}

int vmqg_replica_sync_layout(vmqg_ctx* ctx, const uint8_t* layout) {
  if (!ctx || !layout) return VMQG_E_INVAL;
  Engine& e = ctx->e;
  if (!e.replica) return VMQG_E_STATE;
  vmqg::Layout L;
  memcpy(&L, layout, sizeof(L));
  if (L.magic != vmqg::kLayoutMagic) return VMQG_E_INVAL;
  // every region must be where the replica's image has it
  vmqg::Layout a = L, b = e.lay;
  a.max_depth = b.max_depth = 0;
  if (memcmp(&a, &b, sizeof(a)) != 0) return VMQG_E_STATE;
  e.lay.max_depth = L.max_depth;
  e.dlay.max_depth = L.max_depth;
  return VMQG_OK;
}

int vmqg_replica_follow(vmqg_ctx* replica, vmqg_ctx* primary) {
  if (!replica || !primary) return VMQG_E_INVAL;
  GUARD_BEGIN
  return replica->e.follow(primary->e);
  GUARD_END
}

int vmqg_arena_digest(vmqg_ctx* ctx, uint64_t* digest) {
  if (!ctx || !digest) return VMQG_E_INVAL;
  GUARD_BEGIN
  return ctx->e.arena_digest(digest);
  GUARD_END
}

int vmqg_apply_patches_device(vmqg_ctx* ctx, const void* d_patches, uint64_t bytes, void* stream) {
  if (!ctx || (bytes && !d_patches) || bytes % sizeof(vmqg::Patch)) return VMQG_E_INVAL;
  Engine& e = ctx->e;
  if (!e.has_device || !e.d_arena) return VMQG_E_DEVICE;
  hipSetDevice(e.device);
  hipStream_t st = vmqg::caller_stream(stream);
  // tables change only after the matches queued before, and matches queued
  // later (on any stream) see the patches
  if (e.order_on(st) != VMQG_OK) return VMQG_E_DEVICE;
  if (vmqg::launch_patches(e.d_arena, d_patches, bytes / sizeof(vmqg::Patch), st) != hipSuccess)
    return VMQG_E_DEVICE;
  e.epoch++;
  return VMQG_OK;
}

}  // extern "C"
