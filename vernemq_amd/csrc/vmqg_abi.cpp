// extern "C" boundary of libvmqgpu (include/vmqg.h).  No C++ exception and
// no torch type crosses it; every entry point maps onto the Engine.
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

// vmq_topic:validate_topic(publish, Topic)  (vmq_topic.erl:82-112): split on
// '/', keep empty words, reject '+' / '#' anywhere, size 0 or > 65,536.
int vmqg_prepare_publish(vmqg_ctx* ctx, uint32_t mountpoint, const uint8_t* topic, size_t len,
                         uint32_t* words_out, uint32_t cap, vmqg_pub* pub) {
  if (!ctx || !pub || (len && !topic)) return VMQG_E_INVAL;
  if (len == 0 || len > 65536) return VMQG_E_INVAL;
  GUARD_BEGIN
  uint32_t n = 0;
  size_t start = 0;
  for (size_t i = 0; i <= len; i++) {
    if (i < len && (topic[i] == '+' || topic[i] == '#')) return VMQG_E_INVAL;
    if (i == len || topic[i] == '/') {
      if (n >= cap) return VMQG_E_OVERFLOW;
      words_out[n++] = ctx->e.intern(topic + start, i - start, false);
      start = i + 1;
    }
  }
  pub->mountpoint = mountpoint;
  pub->word_off = 0;
  pub->nwords = n;
  pub->flags = topic[0] == '$' ? VMQG_PUB_DOLLAR : 0u;
  return VMQG_OK;
  GUARD_END
}

int vmqg_apply_ops(vmqg_ctx* ctx, const vmqg_op* ops, size_t n, const uint32_t* words, size_t nwords,
                   uint64_t* epoch_out) {
  if (!ctx || (n && !ops) || (nwords && !words)) return VMQG_E_INVAL;
  GUARD_BEGIN
  int rc = ctx->e.apply_ops(ops, n, words, nwords);
  if (epoch_out) *epoch_out = ctx->e.epoch;
  return rc;
  GUARD_END
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
    if (pubs[i].nwords == 0 || (uint64_t)pubs[i].word_off + pubs[i].nwords > nwords) return VMQG_E_INVAL;
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
  out->paths = e.paths.size();
  out->words = e.word_text.size();
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
  Engine& e = ctx->e;
  const std::string n(name);
  if (n == "fast_g") {
    if (value != 1 && value != 2 && value != 4) return VMQG_E_INVAL;
    e.opt_fast_g = (uint32_t)value;
  } else if (n == "nt_stores") {
    e.opt_flags = value ? (e.opt_flags | vmqg::kOptNtStores) : (e.opt_flags & ~vmqg::kOptNtStores);
  } else if (n == "count_bpc" || n == "emit_bpc") {
    if (value < 0 || value > 32) return VMQG_E_INVAL;
    (n == "count_bpc" ? e.opt_count_bpc : e.opt_emit_bpc) = (uint32_t)value;
  } else {
    return VMQG_E_INVAL;
  }
  return VMQG_OK;
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
  if (bytes) *bytes = ctx->e.lay.total_bytes;
  if (layout_out) memcpy(layout_out, &ctx->e.lay, sizeof(vmqg::Layout));
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
  return VMQG_OK;
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
