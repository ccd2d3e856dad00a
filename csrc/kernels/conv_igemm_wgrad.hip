// ddpx — implicit-GEMM 3x3 convolution, weight gradient (dy^T x im2col of x, split-K partials): every tile config of the pipe core with im2col
// addressing (csrc/include/ddpx_pipe.h; entry point in ddpx_gemm_dispatch.h, used by conv_igemm.hip).
#include "ddpx_gemm_dispatch.h"

namespace ddpx {
namespace pipe {

hipError_t dispatch_conv_wgrad(const Params& p, int cfg, int splits, hipStream_t s) {
  return dispatch<false, false, MODE_PLAIN, MODE_IM2COL_COL>(p, cfg, splits, s);
}

}  // namespace pipe
}  // namespace ddpx
