// ddpx — host helpers for captured training steps.
//
// hipGraphUpload: a freshly instantiated graph executable is uploaded to the device on its first launch unless
// it is uploaded beforehand; the captured multi-step training graphs (ddpx.runtime.graphs.CapturedStep) are
// uploaded right after capture, so their first replay costs what every later replay costs.
#include "ddpx_common.h"

// exec: the hipGraphExec_t of a captured graph (torch.cuda.CUDAGraph.raw_cuda_graph_exec()).
DDPX_API int ddpx_graph_upload(void* exec, hipStream_t s) {
  if (!exec) return -1;
  return (int)hipGraphUpload(reinterpret_cast<hipGraphExec_t>(exec), s);
}
