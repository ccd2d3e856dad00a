// ddpx — pipelined bf16 MFMA GEMM, forward-shaped products (A K-contig, B K-contig: Y = X W^T): every tile config of the pipe core for this
// operand-layout class (csrc/include/ddpx_pipe.h; entry points in ddpx_gemm_dispatch.h, used by gemm_pipe.hip).
#include "ddpx_gemm_dispatch.h"

namespace ddpx {
namespace pipe {

hipError_t dispatch_kk(const Params& p, int cfg, int splits, hipStream_t s) {
  return dispatch<true, true, MODE_PLAIN, MODE_PLAIN>(p, cfg, splits, s);
}

}  // namespace pipe
}  // namespace ddpx
