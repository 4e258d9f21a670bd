// extern "C" boundary of the ACL checker (include/vmqa.h).
#include <new>

#include "vmqa_engine.h"
#include "vmqg_chain.h"
#include "vmqg_nullorder.h"

using vmqa::AclEngine;

struct vmqa_ctx {
  AclEngine e;
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

vmqa_ctx* vmqa_create(const vmqa_config* cfg, int* err) {
  int rc = VMQG_OK;
  vmqa_ctx* c = nullptr;
  try {
    if (!cfg) rc = VMQG_E_INVAL;
    else {
      c = new vmqa_ctx();
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

void vmqa_destroy(vmqa_ctx* ctx) { delete ctx; }

int vmqa_intern_words(vmqa_ctx* ctx, const uint8_t* bytes, const uint64_t* offs, uint32_t n, int create,
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

int vmqa_load(vmqa_ctx* ctx, const vmqa_rule* rules, size_t n, const uint32_t* words, size_t nwords) {
  if (!ctx || (n && !rules) || (nwords && !words)) return VMQG_E_INVAL;
  GUARD_BEGIN
  return ctx->e.load(rules, n, words, nwords);
  GUARD_END
}

int vmqa_check_device(vmqa_ctx* ctx, const vmqa_req* d_reqs, uint32_t n, const uint32_t* d_words,
                      uint8_t* d_allowed, void* stream) {
  if (!ctx || (n && (!d_reqs || !d_words || !d_allowed))) return VMQG_E_INVAL;
  GUARD_BEGIN
  hipSetDevice(ctx->e.device);
  return ctx->e.check_device(d_reqs, n, d_words, d_allowed, vmqg::caller_stream(stream));
  GUARD_END
}

int vmqa_release_stream(vmqa_ctx* ctx, void* stream) {
  if (!ctx) return VMQG_E_INVAL;
  if (!ctx->e.ev_done) return VMQG_OK;
  hipSetDevice(ctx->e.device);
  return vmqg::chain_release(ctx->e.ev_done, ctx->e.chk_stream, vmqg::caller_stream(stream));
}

int vmqa_check_status(vmqa_ctx* ctx, void* stream) {
  if (!ctx) return VMQG_E_INVAL;
  GUARD_BEGIN
  return ctx->e.check_status(vmqg::caller_stream(stream));
  GUARD_END
}

// Host buffers: validate, copy in, check, copy out.
int vmqa_check_batch(vmqa_ctx* ctx, const vmqa_req* reqs, size_t n, const uint32_t* words, size_t nwords,
                     uint8_t* allowed) {
  if (!ctx || (n && (!reqs || !allowed)) || (nwords && !words)) return VMQG_E_INVAL;
  if (n > 0xFFFFFFF0u) return VMQG_E_LIMIT;
  GUARD_BEGIN
  AclEngine& e = ctx->e;
  if (!e.has_device) return VMQG_E_DEVICE;
  for (size_t i = 0; i < n; i++) {
    const vmqa_req& q = reqs[i];
    if (q.nwords == 0 || (uint64_t)q.word_off + q.nwords > nwords) return VMQG_E_INVAL;
    if (q.type != VMQA_READ && q.type != VMQA_WRITE) return VMQG_E_INVAL;
  }
  if (n == 0) return VMQG_OK;
  hipSetDevice(e.device);
  int rc;
  if ((rc = grow(&e.d_r, &e.d_r_cap, n * sizeof(vmqa_req)))) return rc;
  if ((rc = grow(&e.d_w, &e.d_w_cap, (nwords + 1) * 4))) return rc;
  if ((rc = grow(&e.d_o, &e.d_o_cap, n + 1))) return rc;
  hipStream_t st = e.stream;
  if (hipMemcpyAsync(e.d_r, reqs, n * sizeof(vmqa_req), hipMemcpyHostToDevice, st) != hipSuccess) return VMQG_E_DEVICE;
  if (nwords && hipMemcpyAsync(e.d_w, words, nwords * 4, hipMemcpyHostToDevice, st) != hipSuccess)
    return VMQG_E_DEVICE;
  if ((rc = e.check_device(static_cast<const vmqa_req*>(e.d_r), (uint32_t)n, static_cast<const uint32_t*>(e.d_w),
                           static_cast<uint8_t*>(e.d_o), st)))
    return rc;
  if ((rc = e.check_status(st))) return rc;
  if (hipMemcpy(allowed, e.d_o, n, hipMemcpyDeviceToHost) != hipSuccess) return VMQG_E_DEVICE;
  return VMQG_OK;
  GUARD_END
}

int vmqa_stats(vmqa_ctx* ctx, vmqa_stats_t* out) {
  if (!ctx || !out) return VMQG_E_INVAL;
  const AclEngine& e = ctx->e;
  out->rules = e.n_rules;
  out->users = e.n_users;
  out->device_bytes = e.has_device ? e.d_arena_bytes : e.image.size();
  out->loads = e.loads;
  out->words = e.word_text.size();
  return VMQG_OK;
}

int vmqa_set_timing(vmqa_ctx* ctx, int enable) {
  if (!ctx) return VMQG_E_INVAL;
  ctx->e.collect_times();
  ctx->e.timing = enable != 0;
  ctx->e.sum_ns = 0;
  ctx->e.n_timed = 0;
  return VMQG_OK;
}

int vmqa_kernel_times(vmqa_ctx* ctx, double* check_ns, uint64_t* launches) {
  if (!ctx) return VMQG_E_INVAL;
  GUARD_BEGIN
  AclEngine& e = ctx->e;
  e.collect_times();
  if (check_ns) *check_ns = e.n_timed ? e.sum_ns / e.n_timed : 0;
  if (launches) *launches = e.n_timed;
  return VMQG_OK;
  GUARD_END
}

}  // extern "C"
