// The stream a device entry point runs on.
//
// The ABI reads a NULL `stream` as the legacy default stream (torch's default
// stream handle is NULL too): the call's work is queued on that stream
// itself (handle NULL), so it is ordered after the default-stream work
// the caller queued before (e.g. the copies filling its inputs) and before
// the default-stream work it queues after (reading the outputs back), with
// no cross-stream handshake.  An earlier version ran NULL calls on the
// context's own stream and tied it to the default stream with an event pair
// per call: ~28 us of GPU idle time per call on MI355X
// (profiles/gap_r02_context_stream.json vs gap_r02_legacy_stream.json).  Calls with an explicit stream run on it.
#pragma once
#include <hip/hip_runtime.h>

namespace vmqg {

// (Engines therefore never read a NULL stream as their own: internal work
// names the context stream explicitly.  The hipStreamLegacy sentinel is not
// used: hipEventRecord on it crashed the runtime.)
inline hipStream_t caller_stream(const void* s) { return static_cast<hipStream_t>(const_cast<void*>(s)); }

}  // namespace vmqg
