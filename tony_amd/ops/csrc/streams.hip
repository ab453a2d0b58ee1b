// Cross-stream dependencies for the eager step's stream forks and joins (ops/streams.py, the
// Inception branch streams, the weight-gradient side stream, the gradient buckets' communication
// stream): ~150 per Inception-v3 step.  Through torch's Python API a fork is an Event.record +
// Stream.wait_event pair, ~7.6 us of host time on an MI355X host (tools/host_micro.py); here it is
// one fast-call into hipEventRecord + hipStreamWaitEvent on a pooled timing-free event.  Inside a
// HIP-graph capture the pair becomes a graph edge exactly as torch's would.
#include "common.h"

// n timing-disabled events (the fork ring); handles written to out[0..n)
TONY_API int tony_event_pool(int n, uint64_t* out) {
  if (n <= 0 || out == nullptr) return -1;
  for (int i = 0; i < n; ++i) {
    hipEvent_t e;
    const hipError_t err = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (err != hipSuccess) return static_cast<int>(err);
    out[i] = reinterpret_cast<uint64_t>(e);
  }
  return 0;
}

// `to` waits for everything enqueued on `from` so far (a recorded event may be recorded again
// once the wait on it is enqueued: the wait captures the state at enqueue time)
TONY_API int tony_fork(void* event, hipStream_t from, hipStream_t to) {
  hipError_t e = hipEventRecord(static_cast<hipEvent_t>(event), from);
  if (e != hipSuccess) return static_cast<int>(e);
  return static_cast<int>(hipStreamWaitEvent(to, static_cast<hipEvent_t>(event), 0));
}
