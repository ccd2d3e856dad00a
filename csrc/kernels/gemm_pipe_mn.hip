// ddpx — pipelined bf16 MFMA GEMM, weight-gradient-shaped products (A M-contig, B N-contig: dW = dY^T X) and their fused-SGD prefetch tiles: every tile config of the pipe core for this
// operand-layout class (csrc/include/ddpx_pipe.h; entry points in ddpx_gemm_dispatch.h, used by gemm_pipe.hip).
#include "ddpx_gemm_dispatch.h"

namespace ddpx {
namespace pipe {

hipError_t dispatch_mn(const Params& p, int cfg, int splits, hipStream_t s) {
  return dispatch<false, false, MODE_PLAIN, MODE_PLAIN>(p, cfg, splits, s);
}

hipError_t dispatch_sgd_prefetch_mn(const Params& p, int cfg, hipStream_t s) {
  return dispatch_sgd_prefetch<false, false>(p, cfg, s);
}

}  // namespace pipe
}  // namespace ddpx
