// ddpx — pipelined bf16 MFMA GEMM, A M-contig, B K-contig: every tile config of the pipe core for this
// operand-layout class (csrc/include/ddpx_pipe.h; entry points in ddpx_gemm_dispatch.h, used by gemm_pipe.hip).
#include "ddpx_gemm_dispatch.h"

namespace ddpx {
namespace pipe {

hipError_t dispatch_mk(const Params& p, int cfg, int splits, hipStream_t s) {
  return dispatch<false, true, MODE_PLAIN, MODE_PLAIN>(p, cfg, splits, s);
}

}  // namespace pipe
}  // namespace ddpx
