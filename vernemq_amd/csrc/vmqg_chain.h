// One ordering chain across the streams a context's work is queued on.
//
// Table changes and matches (or selects, checks) must not overtake each
// other, whichever caller streams they are queued on.  Instead of recording
// an event after every call (a marker between two calls on one stream costs
// the GPU ~27 us of idle time per call on MI355X,
// profiles/step_overhead_r02_*), the context remembers the stream it queued
// on last; work about to be queued on another stream first records `ev` on
// that one and waits for it.  So an event is recorded only when the stream
// changes, and the chain property holds: each piece of work is ordered
// after everything queued before it on any stream.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/vmqg.h"

namespace vmqg {

// "no work queued yet" (NULL is a real stream: the legacy default stream)
inline hipStream_t no_stream() { return reinterpret_cast<hipStream_t>(~uintptr_t(0)); }
// "`ev` already marks the end of everything queued so far" (the stream it
// was recorded on may be gone: chain_release)
inline hipStream_t ev_recorded() { return reinterpret_cast<hipStream_t>(~uintptr_t(1)); }

inline int chain_order(hipEvent_t ev, hipStream_t& last, hipStream_t st) {
  if (last == ev_recorded()) {
    if (hipStreamWaitEvent(st, ev, 0) != hipSuccess) return VMQG_E_DEVICE;
  } else if (last != no_stream() && st != last) {
    if (hipEventRecord(ev, last) != hipSuccess) return VMQG_E_DEVICE;
    if (hipStreamWaitEvent(st, ev, 0) != hipSuccess) return VMQG_E_DEVICE;
  }
  last = st;
  return VMQG_OK;
}

// The caller is about to destroy `st`: if the chain's last work is on it,
// record `ev` there now, while the stream is alive, so the next call waits
// for that event instead of recording on a destroyed stream.
inline int chain_release(hipEvent_t ev, hipStream_t& last, hipStream_t st) {
  if (last != st || last == no_stream() || last == ev_recorded()) return VMQG_OK;
  if (hipEventRecord(ev, st) != hipSuccess) return VMQG_E_DEVICE;
  last = ev_recorded();
  return VMQG_OK;
}

}  // namespace vmqg
