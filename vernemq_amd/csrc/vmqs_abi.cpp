// Shared-subscription dispatcher: host engine and the extern "C" boundary of
// include/vmqs.h.  Citations are to
// apps/vmq_server/src/vmq_shared_subscriptions.erl unless noted.
#include <cstring>
#include <new>

#include "vmqs_engine.h"
#include "vmqg_chain.h"
#include "vmqg_nullorder.h"

namespace vmqs {

SelEngine::~SelEngine() {
  if (device < 0) return;
  hipSetDevice(device);
  if (stream) hipStreamSynchronize(stream);
  for (auto& e : t_sel) { hipEventDestroy(e.first); hipEventDestroy(e.second); }
  if (ev_sel) hipEventDestroy(ev_sel);
  hipFree(d_states); hipFree(d_status); hipFree(d_defer);
  hipFree(d_e); hipFree(d_o); hipFree(d_c); hipFree(d_f);
  if (stream) hipStreamDestroy(stream);
}

int SelEngine::init(const vmqs_config& c) {
  cfg = c;
  int n = 0;
  if (c.device < 0 || hipGetDeviceCount(&n) != hipSuccess || c.device >= n) return VMQG_E_DEVICE;
  device = c.device;
  if (hipSetDevice(device) != hipSuccess) return VMQG_E_DEVICE;
  if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return VMQG_E_DEVICE;
  if (hipMalloc(&d_status, 64) != hipSuccess) return VMQG_E_NOMEM;
  if (hipEventCreateWithFlags(&ev_sel, hipEventDisableTiming) != hipSuccess) return VMQG_E_DEVICE;
  if (hipMemsetAsync(d_status, 0, 64, stream) != hipSuccess) return VMQG_E_DEVICE;
  return hipStreamSynchronize(stream) == hipSuccess ? VMQG_OK : VMQG_E_DEVICE;
}

// The host's view of each member's queue (vmq_reg:get_queue_pid and the
// queue's online/offline/drain state that enqueue_many checks, :75-88).
int SelEngine::set_states(const uint32_t* subs, const uint8_t* st, size_t n) {
  uint64_t top = n_states;
  for (size_t i = 0; i < n; i++) {
    if (st[i] > VMQS_DRAINING) return VMQG_E_INVAL;
    if ((uint64_t)subs[i] + 1 > top) top = (uint64_t)subs[i] + 1;
  }
  if (top > h_states.size()) h_states.resize(top, (uint8_t)VMQS_ONLINE);
  for (size_t i = 0; i < n; i++) h_states[subs[i]] = st[i];
  hipSetDevice(device);
  // selects still running on any stream read the old table: the copy (and a
  // free of the old buffer) waits for them
  if (vmqg::chain_order(ev_sel, sel_stream, stream) != VMQG_OK) return VMQG_E_DEVICE;
  if (top > states_cap) {
    uint64_t c = 4096;
    while (c < top) c <<= 1;
    uint8_t* d = nullptr;
    if (hipMalloc(&d, c) != hipSuccess) return VMQG_E_NOMEM;
    if (hipStreamSynchronize(stream) != hipSuccess) { hipFree(d); return VMQG_E_DEVICE; }
    hipFree(d_states);
    d_states = d;
    states_cap = c;
  }
  n_states = top;
  // the whole table: the host copy is the truth; uploads are rare (state changes batch)
  if (top && hipMemcpyAsync(d_states, h_states.data(), top, hipMemcpyHostToDevice, stream) != hipSuccess)
    return VMQG_E_DEVICE;
  return hipStreamSynchronize(stream) == hipSuccess ? VMQG_OK : VMQG_E_DEVICE;
}

int SelEngine::select_device(const vmqg_emit* d_emits, const uint64_t* d_offsets, uint32_t npub, uint32_t policy,
                             uint64_t seed, uint64_t pub_seq, uint8_t* d_chosen, uint32_t* d_failed,
                             hipStream_t st) {
  if (policy > VMQS_POLICY_LOCAL_ONLY) return VMQG_E_INVAL;
  hipSetDevice(device);
  if (vmqg::chain_order(ev_sel, sel_stream, st) != VMQG_OK) return VMQG_E_DEVICE;
  if (npub > defer_cap) {
    uint64_t c = 1024;
    while (c < npub) c <<= 1;
    if (hipStreamSynchronize(st) != hipSuccess) return VMQG_E_DEVICE;
    hipFree(d_defer);
    d_defer = nullptr;
    if (hipMalloc(&d_defer, c * 4) != hipSuccess) { defer_cap = 0; return VMQG_E_NOMEM; }
    defer_cap = c;
  }
  if (hipMemsetAsync(d_status, 0, 4, st) != hipSuccess) return VMQG_E_DEVICE;   // tier-2 count
  SArgs a{};
  a.emits = reinterpret_cast<const vmqg::Record*>(d_emits);
  a.offsets = d_offsets;
  a.npub = npub; a.policy = policy; a.local_node = cfg.local_node; a.n_states = (uint32_t)n_states;
  a.seed = seed; a.pub_seq = pub_seq;
  a.states = d_states; a.chosen = d_chosen; a.failed = d_failed;
  a.defer = d_defer; a.status = d_status;
  hipEvent_t e[2] = {nullptr, nullptr};
  if (timing) for (auto& x : e) hipEventCreate(&x);
  if (launch_select(a, st, e[0], e[1]) != hipSuccess) return VMQG_E_DEVICE;
  if (timing) t_sel.push_back({e[0], e[1]});
  return VMQG_OK;
}

int SelEngine::select_status(hipStream_t st) {
  hipSetDevice(device);
  if (vmqg::chain_order(ev_sel, sel_stream, st) != VMQG_OK) return VMQG_E_DEVICE;
  uint32_t h[2] = {0, 0};
  if (hipMemcpyAsync(h, d_status, 8, hipMemcpyDeviceToHost, st) != hipSuccess) return VMQG_E_DEVICE;
  if (hipStreamSynchronize(st) != hipSuccess) return VMQG_E_DEVICE;
  last_deferred = h[0];
  if (h[1]) {
    if (hipMemsetAsync(d_status + 1, 0, 4, st) != hipSuccess) return VMQG_E_DEVICE;
    if (hipStreamSynchronize(st) != hipSuccess) return VMQG_E_DEVICE;
    return VMQG_E_LIMIT;
  }
  return VMQG_OK;
}

void SelEngine::collect_times() {
  for (auto& e : t_sel) {
    float ms = 0;
    hipEventSynchronize(e.second);
    hipEventElapsedTime(&ms, e.first, e.second);
    sum_ns += ms * 1e6; n_timed++;
    hipEventDestroy(e.first); hipEventDestroy(e.second);
  }
  t_sel.clear();
}

}  // namespace vmqs

using vmqs::SelEngine;

struct vmqs_ctx {
  SelEngine e;
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

vmqs_ctx* vmqs_create(const vmqs_config* cfg, int* err) {
  int rc = VMQG_OK;
  vmqs_ctx* c = nullptr;
  try {
    if (!cfg) rc = VMQG_E_INVAL;
    else {
      c = new vmqs_ctx();
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

void vmqs_destroy(vmqs_ctx* ctx) { delete ctx; }

uint64_t vmqs_key(uint64_t seed, uint64_t q, uint32_t p) { return vmqs::sel_key(seed, q, p); }

int vmqs_set_states(vmqs_ctx* ctx, const uint32_t* subscribers, const uint8_t* states, size_t n) {
  if (!ctx || (n && (!subscribers || !states))) return VMQG_E_INVAL;
  GUARD_BEGIN
  return ctx->e.set_states(subscribers, states, n);
  GUARD_END
}

int vmqs_select_device(vmqs_ctx* ctx, const vmqg_emit* d_emits, const uint64_t* d_offsets, uint32_t npub,
                       uint32_t policy, uint64_t seed, uint64_t pub_seq, uint8_t* d_chosen, uint32_t* d_failed,
                       void* stream) {
  if (!ctx || (npub && (!d_emits || !d_offsets || !d_chosen))) return VMQG_E_INVAL;
  GUARD_BEGIN
  hipSetDevice(ctx->e.device);
  return ctx->e.select_device(d_emits, d_offsets, npub, policy, seed, pub_seq, d_chosen, d_failed,
                              vmqg::caller_stream(stream));
  GUARD_END
}

int vmqs_release_stream(vmqs_ctx* ctx, void* stream) {
  if (!ctx) return VMQG_E_INVAL;
  if (!ctx->e.ev_sel) return VMQG_OK;
  hipSetDevice(ctx->e.device);
  return vmqg::chain_release(ctx->e.ev_sel, ctx->e.sel_stream, vmqg::caller_stream(stream));
}

int vmqs_select_status(vmqs_ctx* ctx, void* stream) {
  if (!ctx) return VMQG_E_INVAL;
  GUARD_BEGIN
  return ctx->e.select_status(vmqg::caller_stream(stream));
  GUARD_END
}

// Host buffers: validate, copy the batch's records and rebased offsets in,
// select, copy chosen / failed out.
int vmqs_select_batch(vmqs_ctx* ctx, const vmqg_emit* emits, const uint64_t* offsets, size_t npub,
                      uint32_t policy, uint64_t seed, uint64_t pub_seq, uint8_t* chosen, uint32_t* failed) {
  if (!ctx || !offsets || policy > VMQS_POLICY_LOCAL_ONLY) return VMQG_E_INVAL;
  if (npub > 0xFFFFFFF0u) return VMQG_E_LIMIT;
  GUARD_BEGIN
  SelEngine& e = ctx->e;
  for (size_t i = 0; i < npub; i++) {
    if (offsets[i + 1] < offsets[i]) return VMQG_E_INVAL;
    if (offsets[i + 1] - offsets[i] > VMQS_MAX_SEGMENT) return VMQG_E_LIMIT;
  }
  if (npub == 0) return VMQG_OK;
  const uint64_t base = offsets[0], total = offsets[npub] - base;
  if (total && (!emits || !chosen)) return VMQG_E_INVAL;
  hipSetDevice(e.device);
  int rc;
  if ((rc = grow(&e.d_e, &e.d_e_cap, (total + 1) * sizeof(vmqg_emit)))) return rc;
  if ((rc = grow(&e.d_o, &e.d_o_cap, (npub + 1) * 8))) return rc;
  if ((rc = grow(&e.d_c, &e.d_c_cap, total + 1))) return rc;
  if ((rc = grow(&e.d_f, &e.d_f_cap, npub * 4))) return rc;
  std::vector<uint64_t> rb(npub + 1);
  for (size_t i = 0; i <= npub; i++) rb[i] = offsets[i] - base;
  hipStream_t st = e.stream;
  if (total && hipMemcpyAsync(e.d_e, emits + base, total * sizeof(vmqg_emit), hipMemcpyHostToDevice, st) != hipSuccess)
    return VMQG_E_DEVICE;
  if (hipMemcpyAsync(e.d_o, rb.data(), (npub + 1) * 8, hipMemcpyHostToDevice, st) != hipSuccess) return VMQG_E_DEVICE;
  if ((rc = e.select_device(static_cast<const vmqg_emit*>(e.d_e), static_cast<const uint64_t*>(e.d_o),
                            (uint32_t)npub, policy, seed, pub_seq, static_cast<uint8_t*>(e.d_c),
                            static_cast<uint32_t*>(e.d_f), st)))
    return rc;
  if ((rc = e.select_status(st))) return rc;
  if (total && hipMemcpy(chosen + base, e.d_c, total, hipMemcpyDeviceToHost) != hipSuccess) return VMQG_E_DEVICE;
  if (failed && hipMemcpy(failed, e.d_f, npub * 4, hipMemcpyDeviceToHost) != hipSuccess) return VMQG_E_DEVICE;
  return VMQG_OK;
  GUARD_END
}

int vmqs_set_timing(vmqs_ctx* ctx, int enable) {
  if (!ctx) return VMQG_E_INVAL;
  ctx->e.collect_times();
  ctx->e.timing = enable != 0;
  ctx->e.sum_ns = 0;
  ctx->e.n_timed = 0;
  return VMQG_OK;
}

int vmqs_kernel_times(vmqs_ctx* ctx, double* select_ns, uint64_t* launches, uint64_t* deferred) {
  if (!ctx) return VMQG_E_INVAL;
  GUARD_BEGIN
  SelEngine& e = ctx->e;
  e.collect_times();
  if (select_ns) *select_ns = e.n_timed ? e.sum_ns / e.n_timed : 0;
  if (launches) *launches = e.n_timed;
  if (deferred) *deferred = e.last_deferred;
  return VMQG_OK;
  GUARD_END
}

}  // extern "C"
