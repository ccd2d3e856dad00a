// ddpx — per-layout dispatch entry points of the pipelined GEMM (csrc/include/ddpx_pipe.h).
//
// Each operand-layout class instantiates every tile config of the pipe core; they live in separate
// translation units (csrc/kernels/gemm_pipe_{kk,kn,mk,mn,sk}.hip, conv_igemm_{fwd,dgrad,wgrad}.hip) so an in-tree build compiles them in
// parallel instead of one multi-minute file.
#pragma once

#include "ddpx_pipe.h"

namespace ddpx {
namespace pipe {

// A K-contig / M-contig  x  B K-contig / N-contig, plain (non-im2col) operands.
hipError_t dispatch_kk(const Params& p, int cfg, int splits, hipStream_t s);
hipError_t dispatch_kn(const Params& p, int cfg, int splits, hipStream_t s);
hipError_t dispatch_mk(const Params& p, int cfg, int splits, hipStream_t s);
hipError_t dispatch_mn(const Params& p, int cfg, int splits, hipStream_t s);
// in-launch split-K (A K-contig) and the fused-SGD prefetch tiles (plain wgrad layout)
hipError_t dispatch_sk_kk(const Params& p, int cfg, int splits, hipStream_t s);
hipError_t dispatch_sk_kn(const Params& p, int cfg, int splits, hipStream_t s);
hipError_t dispatch_sgd_prefetch_mn(const Params& p, int cfg, hipStream_t s);
// implicit-GEMM 3x3 convolutions (csrc/kernels/conv_igemm_{fwd,dgrad,wgrad}.hip)
hipError_t dispatch_conv_fwd(const Params& p, int cfg, hipStream_t s);
hipError_t dispatch_conv_dgrad(const Params& p, int cfg, hipStream_t s);
hipError_t dispatch_conv_wgrad(const Params& p, int cfg, int splits, hipStream_t s);

}  // namespace pipe
}  // namespace ddpx
