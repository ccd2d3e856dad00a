// ddpx — pipelined bf16 MFMA GEMM, in-launch split-K tiles (A K-contig): every tile config of the pipe core for this
// operand-layout class (csrc/include/ddpx_pipe.h; entry points in ddpx_gemm_dispatch.h, used by gemm_pipe.hip).
#include "ddpx_gemm_dispatch.h"

namespace ddpx {
namespace pipe {

hipError_t dispatch_sk_kk(const Params& p, int cfg, int splits, hipStream_t s) {
  return dispatch_sk<true, true>(p, cfg, splits, s);
}

hipError_t dispatch_sk_kn(const Params& p, int cfg, int splits, hipStream_t s) {
  return dispatch_sk<true, false>(p, cfg, splits, s);
}

}  // namespace pipe
}  // namespace ddpx
