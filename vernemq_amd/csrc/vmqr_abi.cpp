// extern "C" boundary of the retained-message matcher (include/vmqr.h).
#include <cstring>
#include <new>
#include <string>

#include "vmqr_engine.h"
#include "vmqg_chain.h"
#include "vmqg_nullorder.h"

using vmqr::RetainEngine;

struct vmqr_ctx {
  RetainEngine e;
};

#define GUARD_BEGIN try {
#define GUARD_END                   \
  }                                 \
  catch (const std::bad_alloc&) {   \
    return VMQG_E_NOMEM;            \
  }                                 \
  catch (...) {                     \
    return VMQG_E_INVAL;            \
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

extern "C" {

vmqr_ctx* vmqr_create(const vmqr_config* cfg, int* err) {
  int rc = VMQG_OK;
  vmqr_ctx* c = nullptr;
  try {
    if (!cfg) rc = VMQG_E_INVAL;
    else {
      c = new vmqr_ctx();
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

void vmqr_destroy(vmqr_ctx* ctx) { delete ctx; }

int vmqr_intern_words(vmqr_ctx* ctx, const uint8_t* bytes, const uint64_t* offs, uint32_t n, int create,
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

int vmqr_apply(vmqr_ctx* ctx, const vmqr_op* ops, size_t n, const uint32_t* words, size_t nwords) {
  if (!ctx || (n && !ops) || (nwords && !words)) return VMQG_E_INVAL;
  GUARD_BEGIN
  return ctx->e.apply(ops, n, words, nwords);
  GUARD_END
}

int vmqr_match_device(vmqr_ctx* ctx, const vmqg_pub* d_filters, uint32_t n, const uint32_t* d_words,
                      uint32_t* d_out, uint64_t out_cap, uint64_t* d_offsets, void* stream) {
  if (!ctx || !d_offsets || (n && (!d_filters || !d_words))) return VMQG_E_INVAL;
  GUARD_BEGIN
  hipSetDevice(ctx->e.device);
  return ctx->e.match_device(d_filters, n, d_words, d_out, out_cap, d_offsets, vmqg::caller_stream(stream));
  GUARD_END
}

int vmqr_release_stream(vmqr_ctx* ctx, void* stream) {
  if (!ctx) return VMQG_E_INVAL;
  if (!ctx->e.ev_match_done) return VMQG_OK;
  hipSetDevice(ctx->e.device);
  return vmqg::chain_release(ctx->e.ev_match_done, ctx->e.ev_stream, vmqg::caller_stream(stream));
}

int vmqr_match_status(vmqr_ctx* ctx, void* stream) {
  if (!ctx) return VMQG_E_INVAL;
  GUARD_BEGIN
  return ctx->e.match_status(vmqg::caller_stream(stream));
  GUARD_END
}

// Host buffers: copy in, match, copy out; the look-back tiles grow and the
// batch reruns when a batch walks more rows than they cover.
int vmqr_match_batch(vmqr_ctx* ctx, const vmqg_pub* filters, size_t n, const uint32_t* words, size_t nwords,
                     uint32_t* out, size_t out_cap, size_t* out_n, uint64_t* offsets) {
  if (!ctx || !offsets || (n && !filters) || (nwords && !words) || (out_cap && !out)) return VMQG_E_INVAL;
  if (n > 0xFFFFFFF0u) return VMQG_E_LIMIT;
  GUARD_BEGIN
  RetainEngine& e = ctx->e;
  if (!e.has_device) return VMQG_E_DEVICE;
  for (size_t i = 0; i < n; i++)
    if (filters[i].nwords == 0 || (uint64_t)filters[i].word_off + filters[i].nwords > nwords) return VMQG_E_INVAL;
  hipSetDevice(e.device);
  int rc;
  if ((rc = grow(&e.d_f, &e.d_f_cap, (n + 1) * sizeof(vmqg_pub)))) return rc;
  if ((rc = grow(&e.d_w, &e.d_w_cap, (nwords + 1) * 4))) return rc;
  if ((rc = grow(&e.d_offs, &e.d_offs_cap, (n + 1) * 8))) return rc;
  if ((rc = grow(&e.d_o, &e.d_o_cap, (out_cap + 1) * 4))) return rc;
  hipStream_t st = e.stream;
  if (n && hipMemcpyAsync(e.d_f, filters, n * sizeof(vmqg_pub), hipMemcpyHostToDevice, st) != hipSuccess)
    return VMQG_E_DEVICE;
  if (nwords && hipMemcpyAsync(e.d_w, words, nwords * 4, hipMemcpyHostToDevice, st) != hipSuccess)
    return VMQG_E_DEVICE;
  for (int attempt = 0;; attempt++) {
    rc = e.match_device(static_cast<const vmqg_pub*>(e.d_f), (uint32_t)n, static_cast<const uint32_t*>(e.d_w),
                        static_cast<uint32_t*>(e.d_o), out_cap, static_cast<uint64_t*>(e.d_offs), st);
    if (rc) return rc;
    rc = e.match_status(st);
    if (rc != VMQG_E_FRONTIER || attempt > 0) break;
    // match_status grew the look-back tiles for this batch: run it again
  }
  if (hipMemcpyAsync(offsets, e.d_offs, (n + 1) * 8, hipMemcpyDeviceToHost, st) != hipSuccess) return VMQG_E_DEVICE;
  if (hipStreamSynchronize(st) != hipSuccess) return VMQG_E_DEVICE;
  const uint64_t total = offsets[n];
  if (out_n) *out_n = total;
  if (rc == VMQG_E_OVERFLOW || total > out_cap) return VMQG_E_OVERFLOW;
  if (rc) return rc;
  if (total && hipMemcpy(out, e.d_o, total * 4, hipMemcpyDeviceToHost) != hipSuccess) return VMQG_E_DEVICE;
  return VMQG_OK;
  GUARD_END
}

int vmqr_stats(vmqr_ctx* ctx, vmqr_stats_t* out) {
  if (!ctx || !out) return VMQG_E_INVAL;
  const RetainEngine& e = ctx->e;
  out->retained = e.n_live;
  out->device_bytes = e.has_device ? e.d_arena_bytes : e.lay.total_bytes;
  out->partitions = e.parts.size();
  out->epoch = e.epoch;
  out->rebuilds = e.rebuilds;
  out->words = e.word_text.size();
  return VMQG_OK;
}

int vmqr_dump(vmqr_ctx* ctx, const char** text, size_t* len) {
  if (!ctx || !text || !len) return VMQG_E_INVAL;
  GUARD_BEGIN
  ctx->e.dump_text = ctx->e.dump();
  *text = ctx->e.dump_text.data();
  *len = ctx->e.dump_text.size();
  return VMQG_OK;
  GUARD_END
}

int vmqr_set_option(vmqr_ctx* ctx, const char* name, int64_t value) {
  if (!ctx || !name) return VMQG_E_INVAL;
  if (!strcmp(name, "walk_rows_hint") && value >= 1) {
    ctx->e.walk_rows_hint = (uint64_t)value;
    return VMQG_OK;
  }
  return VMQG_E_INVAL;
}

int vmqr_set_timing(vmqr_ctx* ctx, int enable) {
  if (!ctx) return VMQG_E_INVAL;
  ctx->e.collect_times();
  ctx->e.timing = enable != 0;
  ctx->e.sum_count_ns = ctx->e.sum_emit_ns = 0;
  ctx->e.n_timed = 0;
  return VMQG_OK;
}

int vmqr_kernel_times(vmqr_ctx* ctx, double* count_ns, double* emit_ns, uint64_t* launches) {
  if (!ctx) return VMQG_E_INVAL;
  GUARD_BEGIN
  RetainEngine& e = ctx->e;
  e.collect_times();
  if (count_ns) *count_ns = e.n_timed ? e.sum_count_ns / e.n_timed : 0;
  if (emit_ns) *emit_ns = e.n_timed ? e.sum_emit_ns / e.n_timed : 0;
  if (launches) *launches = e.n_timed;
  return VMQG_OK;
  GUARD_END
}

}  // extern "C"
