// ddpx — implicit-GEMM 3x3 convolution, forward (im2col A x weights: y = conv(x, W)): every tile config of the pipe core with im2col
// addressing (csrc/include/ddpx_pipe.h; entry point in ddpx_gemm_dispatch.h, used by conv_igemm.hip).
#include "ddpx_gemm_dispatch.h"

namespace ddpx {
namespace pipe {

hipError_t dispatch_conv_fwd(const Params& p, int cfg, hipStream_t s) {
  return dispatch<true, true, MODE_IM2COL_FWD, MODE_PLAIN>(p, cfg, 1, s);
}

}  // namespace pipe
}  // namespace ddpx
