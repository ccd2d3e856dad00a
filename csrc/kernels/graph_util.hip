// ddpx — host helpers for captured training steps.
//
// hipGraphUpload: a freshly instantiated graph executable is uploaded to the device on its first launch unless
// it is uploaded beforehand; the captured multi-step training graphs (ddpx.runtime.graphs.CapturedStep) are
// uploaded right after capture, so their first replay costs what every later replay costs.
#include "ddpx_common.h"

#include <thread>

// exec: the hipGraphExec_t of a captured graph (torch.cuda.CUDAGraph.raw_cuda_graph_exec()).
DDPX_API int ddpx_graph_upload(void* exec, hipStream_t s) {
  if (!exec) return -1;
  return (int)hipGraphUpload(reinterpret_cast<hipGraphExec_t>(exec), s);
}

// Capture bookkeeping for ddpx.runtime.graphs.capture_step (profiles/r5_capture/NOTES.md): the capture status
// of ANY stream (torch only answers for the current one) and a hard end of a capture that torch's capture_end
// could not end.  On ROCm 7 an unjoined capture (a forked side stream not joined back) makes
// hipStreamEndCapture fail while BOTH streams stay "active", and a stream whose capture was invalidated keeps
// reporting "invalidated" afterwards: every later synchronous copy on it fails (torch's memcpy_and_sync
// requires the status "none").
// status: 0 none, 1 active, 2 invalidated; id: the capture's id (0 when none).
DDPX_API int ddpx_stream_capture_info(hipStream_t s, int* status, unsigned long long* id) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long cid = 0;
  hipError_t e = hipStreamGetCaptureInfo(s, &st, &cid);
  *status = (int)st;
  *id = st == hipStreamCaptureStatusNone ? 0 : cid;
  return (int)e;
}

// End the capture running on `s` (from the thread that began it) and destroy whatever graph it produced.
// Returns the hipStreamEndCapture code (the capture is over either way unless the code is a wrong-thread /
// unmatched error).
DDPX_API int ddpx_stream_end_capture_discard(hipStream_t s) {
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(s, &g);
  // an unjoined end hands back the graph while the capture stays active (it still owns it): only a clean end
  // transfers it
  if (g && e == hipSuccess) (void)hipGraphDestroy(g);
  (void)hipGetLastError();  // do not leave the code behind for torch's next launch check
  return (int)e;
}

static hipStreamCaptureStatus capture_status(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  (void)hipStreamGetCaptureInfo(s, &st, nullptr);
  return st;
}

static void end_and_drop(hipStream_t s) {
  hipGraph_t g = nullptr;
  // only a clean end hands over the graph: after an unmatched / unjoined end it may still belong to the origin
  if (hipStreamEndCapture(s, &g) == hipSuccess && g) (void)hipGraphDestroy(g);
}

// Bring a stream that a failed capture left behind back to the capture status "none" (measured on ROCm 7,
// benchmarks/capture_probe.hip): a side stream still "active" after its origin's capture ended is ended on its
// own (hipErrorStreamCaptureUnmatched, after which it reads "invalidated"); an "invalidated" stream returns to
// "none" after one empty capture.  An origin stream whose unjoined end failed refuses a second end on its own
// thread (hipErrorStreamCaptureWrongThread); that end is retried from a helper thread.  Returns the final status.
DDPX_API int ddpx_stream_force_reset(hipStream_t s) {
  if (capture_status(s) == hipStreamCaptureStatusActive) {
    end_and_drop(s);
    if (capture_status(s) == hipStreamCaptureStatusActive) {
      std::thread t([s] { end_and_drop(s); });
      t.join();
    }
  }
  if (capture_status(s) == hipStreamCaptureStatusInvalidated) {
    if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) == hipSuccess) end_and_drop(s);
  }
  (void)hipGetLastError();
  return (int)capture_status(s);
}
