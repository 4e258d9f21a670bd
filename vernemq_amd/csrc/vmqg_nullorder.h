// Ordering for device entry points called with stream = NULL.
//
// The ABI reads a NULL `stream` as "the context's own stream" (include/*.h).
// That stream is non-blocking, so by itself it would neither wait for work
// the caller queued on the legacy default stream — whose handle is also NULL,
// e.g. torch's default stream filling the inputs — nor make later default-
// stream work (reading the outputs back) wait for it.  NullOrder, held for
// the duration of such a call, orders the context stream after the default
// stream on entry and the default stream after the context stream on exit,
// so a NULL call behaves like default-stream work.  Calls with an explicit
// stream are ordered by that stream alone.
#pragma once
#include <hip/hip_runtime.h>

namespace vmqg {

struct NullOrder {
  hipStream_t ctx;
  hipEvent_t ev;
  bool on;
  NullOrder(void* caller_stream, hipStream_t ctx_stream, hipEvent_t& ev_slot)
      : ctx(ctx_stream), ev(nullptr), on(caller_stream == nullptr && ctx_stream != nullptr) {
    if (!on) return;
    if (!ev_slot && hipEventCreateWithFlags(&ev_slot, hipEventDisableTiming) != hipSuccess) ev_slot = nullptr;
    ev = ev_slot;
    if (!ev) { on = false; return; }
    hipEventRecord(ev, nullptr);
    hipStreamWaitEvent(ctx, ev, 0);
  }
  ~NullOrder() {
    if (!on) return;
    hipEventRecord(ev, ctx);
    hipStreamWaitEvent(nullptr, ev, 0);
  }
  NullOrder(const NullOrder&) = delete;
  NullOrder& operator=(const NullOrder&) = delete;
};

}  // namespace vmqg
