"""Host wrappers: 3x3 implicit-GEMM convolutions, BatchNorm/ReLU/MaxPool, average pool (NHWC bf16).

Kernels: ``csrc/kernels/conv_igemm.hip`` and ``csrc/kernels/bn_pool.hip``.  Every wrapper checks shapes,
dtypes and contiguity on the host before launching.
"""
from __future__ import annotations

import torch

from ..runtime import native


def _req(c, msg):
    if not c:
        raise ValueError(msg)


def _nhwc(x, name, C=None):
    _req(x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous(), f"{name} must be contiguous bf16 on GPU")
    _req(x.data_ptr() % 16 == 0, f"{name} must be 16-B aligned")
    if C is not None:
        _req(x.shape[-1] == C, f"{name}: expected {C} channels, got {tuple(x.shape)}")


def padded_channels(c: int) -> int:
    return max(8, (c + 7) // 8 * 8)


def weight_prep(w: torch.Tensor, wf: torch.Tensor, wd: torch.Tensor):
    """fp32 torch weight [Co,Ci,3,3] -> wf [Co,9,Cp] and wd [9,Co,Cp] (bf16, zero-padded channels)."""
    Co, Ci = w.shape[0], w.shape[1]
    Cp = padded_channels(Ci)
    _req(tuple(w.shape) == (Co, Ci, 3, 3) and w.dtype == torch.float32 and w.is_contiguous(), "bad conv weight")
    _req(wf.numel() == Co * 9 * Cp and wd.numel() == Co * 9 * Cp, "bad prepared-weight buffers")
    native.check(native.kernels().ddpx_conv_weight_prep(w.data_ptr(), Co, Ci, Cp, wf.data_ptr(), wd.data_ptr(),
                                                        native.stream_handle()), "ddpx_conv_weight_prep")


def conv_fwd(x, wf, Co, stats=True, tile=-1):
    """y [N*H*W, Co] bf16 (+ per-tile BN statistics [T,2,Co] fp32 and tile rows)."""
    N, H, W, C = x.shape
    _nhwc(x, "x")
    _req(C % 8 == 0 and wf.numel() == Co * 9 * C, "conv_fwd: weight/input channel mismatch")
    lib = native.kernels()
    P = N * H * W
    y = torch.empty((P, Co), dtype=torch.bfloat16, device=x.device)
    st, T, BM = None, 0, 0
    if stats:
        T = lib.ddpx_conv_fwd_tiles_m(P, C, Co, tile)
        BM = lib.ddpx_conv_fwd_tile_rows(P, C, Co, tile)
        st = torch.empty((T, 2, Co), dtype=torch.float32, device=x.device)
    native.check(lib.ddpx_conv_fwd(x.data_ptr(), wf.data_ptr(), y.data_ptr(), native.ptr(st), N, H, W, C, Co, tile,
                                   native.stream_handle()), "ddpx_conv_fwd")
    return y, st, T, BM


def conv_fwd_act(x, wf, Co, bias, tile=-1):
    """act [N*H*W, Co] bf16 = relu(conv(x) + bias), bias + ReLU in the GEMM epilogue (DeepNN's conv blocks)."""
    N, H, W, C = x.shape
    _nhwc(x, "x")
    _req(C % 8 == 0 and wf.numel() == Co * 9 * C, "conv_fwd_act: weight/input channel mismatch")
    _req(bias.dtype == torch.float32 and bias.numel() == Co and bias.is_contiguous(), "conv_fwd_act: bias fp32 [Co]")
    act = torch.empty((N * H * W, Co), dtype=torch.bfloat16, device=x.device)
    native.check(native.kernels().ddpx_conv_fwd_act(x.data_ptr(), wf.data_ptr(), act.data_ptr(), bias.data_ptr(),
                                                    N, H, W, C, Co, tile, native.stream_handle()), "ddpx_conv_fwd_act")
    return act


def conv_dgrad_act(dy, wd, N, H, W, C, Co, act, tile=-1):
    """(dz [N*H*W, C] bf16, (part [T, C] fp32, T)): the data gradient masked by the ReLU of the block below
    (``act`` = its relu(conv + bias) output, [N*H*W, C]) in the GEMM epilogue, with per-row-tile column sums of
    dz (that block's bias gradient, finished by :func:`colsum_finish`)."""
    _nhwc(dy, "dy", Co)
    _nhwc(act, "act", C)
    _req(act.numel() == N * H * W * C, "conv_dgrad_act: act must be [N*H*W, C]")
    _req(wd.numel() == 9 * Co * C, "conv_dgrad_act: bad weight buffer")
    lib = native.kernels()
    T = lib.ddpx_conv_dgrad_tiles_m(N, H, W, C, Co, tile)
    part = torch.empty((T, C), dtype=torch.float32, device=dy.device)
    dz = torch.empty((N * H * W, C), dtype=torch.bfloat16, device=dy.device)
    native.check(lib.ddpx_conv_dgrad_act(dy.data_ptr(), wd.data_ptr(), dz.data_ptr(), N, H, W, C, Co, tile,
                                         act.data_ptr(), part.data_ptr(), native.stream_handle()), "ddpx_conv_dgrad_act")
    return dz, (part, T)


def colsum_finish(part, T, C, out=None, accumulate=False, sgd=None):
    """out (=|+=) Σ_t part[t] in row-tile order, or applied as ``sgd``'s update (fused optimizer)."""
    _req(out is not None or sgd is not None, "colsum_finish: out or sgd")
    if out is not None:
        _req(out.numel() == C and out.is_contiguous() and out.dtype in (torch.float32, torch.bfloat16),
             "colsum_finish: bad out")
    lib = native.kernels()
    ws = torch.empty(lib.ddpx_colsum_ws_floats(T, C), dtype=torch.float32, device=part.device)
    native.check(lib.ddpx_colsum_finish(part.data_ptr(), T, C, ws.data_ptr(), native.ptr(out),
                                                     int(out is not None and out.dtype == torch.bfloat16),
                                                     int(accumulate), *native.sgd_args(sgd), native.stream_handle()),
                 "ddpx_colsum_finish")


def conv_dgrad(dy, wd, N, H, W, C, Co, tile=-1):
    """dx [N,H,W,C] bf16 = dgrad(dy [N*H*W, Co], wd [9,Co,C])."""
    _nhwc(dy, "dy", Co)
    _req(wd.numel() == 9 * Co * C, "conv_dgrad: bad weight buffer")
    dx = torch.empty((N, H, W, C), dtype=torch.bfloat16, device=dy.device)
    native.check(native.kernels().ddpx_conv_dgrad(dy.data_ptr(), wd.data_ptr(), dx.data_ptr(), N, H, W, C, Co, tile,
                                                  native.stream_handle()), "ddpx_conv_dgrad")
    return dx


def conv_dgrad_bn(dy, wd, N, H, W, C, Co, bn_y, a, b, mean, rstd, pool, tile=-1):
    """(dx, (part, B)): the data gradient of the conv, with the BatchNorm backward pass-1 sums of the block below
    (its pre-BN activation ``bn_y`` [N, H', W', C], H' = 2H when a 2x2 max-pool sits between) from the GEMM
    epilogue: ``bn_backward(..., part=(part, B))`` then skips its own reduce over dx and bn_y.  (dx, None) for
    the layers whose data-gradient tile has no fused variant (measured slower there, profiles/r5_vgg)."""
    _nhwc(dy, "dy", Co)
    _req(wd.numel() == 9 * Co * C, "conv_dgrad_bn: bad weight buffer")
    lib = native.kernels()
    B = lib.ddpx_conv_dgrad_parts(N, H, W, C, Co, tile)
    if B == 0:  # no fused variant for this layer's tile: plain data gradient, bn_backward reduces itself
        return conv_dgrad(dy, wd, N, H, W, C, Co, tile), None
    part = torch.empty((B, 2, C), dtype=torch.float32, device=dy.device)
    dx = torch.empty((N, H, W, C), dtype=torch.bfloat16, device=dy.device)
    native.check(lib.ddpx_conv_dgrad_bn(dy.data_ptr(), wd.data_ptr(), dx.data_ptr(), N, H, W, C, Co, tile,
                                        bn_y.data_ptr(), a.data_ptr(), b.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                        int(pool), part.data_ptr(), native.stream_handle()), "ddpx_conv_dgrad_bn")
    return dx, (part, B)


def conv_wgrad(dy, x, Co, Cr, out=None, accumulate=False, sgd=None, tile=-1, prepared=None):
    """Weight gradient in torch layout [Co,Cr,3,3] (written to ``out`` or applied through ``sgd``).
    ``prepared`` = (wf, wd) with ``sgd``: the update also rewrites the bf16 GEMM layouts ``weight_prep`` makes
    (whose zero channel padding it keeps), so the next forward needs no weight_prep pass."""
    N, H, W, C = x.shape
    _nhwc(x, "x")
    _nhwc(dy, "dy", Co)
    lib = native.kernels()
    P = N * H * W
    S = lib.ddpx_conv_wgrad_splits(P, C, Co, tile)
    part = torch.empty((S, Co, 9 * C), dtype=torch.float32, device=x.device)
    s = native.stream_handle()
    native.check(lib.ddpx_conv_wgrad(dy.data_ptr(), x.data_ptr(), part.data_ptr(), S, N, H, W, C, Co, tile, s),
                 "ddpx_conv_wgrad")
    if sgd is None:
        _req(out is not None and out.numel() == Co * Cr * 9 and out.is_contiguous(), "conv_wgrad: bad out")
        _req(prepared is None, "conv_wgrad: prepared layouts are written by the fused SGD only")
    wf, wd = prepared if prepared is not None else (None, None)
    if prepared is not None:
        _req(wf.numel() == Co * 9 * C and wd.numel() == Co * 9 * C and wf.dtype == wd.dtype == torch.bfloat16,
             "conv_wgrad: bad prepared-weight buffers")
    native.check(lib.ddpx_conv_wgrad_reduce(part.data_ptr(), S, Co, Cr, C, native.ptr(out),
                                            int(out is not None and out.dtype == torch.bfloat16), int(accumulate),
                                            *native.sgd_args(sgd), native.ptr(wf), native.ptr(wd), s),
                 "ddpx_conv_wgrad_reduce")


def bn_finalize(stats, T, BM, M, bn_mod, training, a, b, mean, rstd):
    C = bn_mod.num_features
    lib = native.kernels()
    nbt = bn_mod.num_batches_tracked if (training and bn_mod.num_batches_tracked is not None) else None
    native.check(lib.ddpx_bn_finalize(native.ptr(stats), T, BM, M, C, bn_mod.weight.data_ptr(),
                                      bn_mod.bias.data_ptr(), bn_mod.running_mean.data_ptr(),
                                      bn_mod.running_var.data_ptr(), native.ptr(nbt), float(bn_mod.momentum),
                                      float(bn_mod.eps), int(training), a.data_ptr(), b.data_ptr(), mean.data_ptr(),
                                      rstd.data_ptr(), native.stream_handle()), "ddpx_bn_finalize")


def bn_finalize_sync(stats, T, BM, M, bn_mod, a, b, mean, rstd, comm):
    """SyncBatchNorm forward statistics (training): this rank's (mean, M2) from the tile statistics, one
    all-gather of [2][C] per rank on the current stream (RCCL: graph-capturable), then the rank-ordered
    Chan merge + running-stat update + affine coefficients in ``ddpx_bn_finalize``.  Every rank must hold
    the same number of rows M (equal DistributedSampler shards)."""
    C = bn_mod.num_features
    lib = native.kernels()
    dev = a.device
    local = torch.empty(2 * C, dtype=torch.float32, device=dev)
    native.check(lib.ddpx_bn_local_stats(stats.data_ptr(), T, BM, M, C, local.data_ptr(), native.stream_handle()),
                 "ddpx_bn_local_stats")
    ws = comm.world_size
    gathered = torch.empty(ws * 2 * C, dtype=torch.float32, device=dev)
    comm.allgather(gathered, local)
    bn_finalize(gathered, ws, M, ws * M, bn_mod, True, a, b, mean, rstd)


def bn_backward_sync(gout, y, a, b, mean, rstd, N, H, W, C, pool, comm, dgamma=None, dbeta=None,
                     accumulate=False, part=None):
    """SyncBatchNorm backward: local (sum dy, sum dy*xhat) -> all-reduce -> dy with the global means;
    dgamma / dbeta stay local (DDP averages them, as torch's SyncBatchNorm).  ``part``: the local pass-1
    partials from the data gradient's epilogue (``conv_dgrad_bn``), as in ``bn_backward``."""
    _nhwc(gout, "gout", C)
    _nhwc(y, "y", C)
    lib = native.kernels()
    dev = y.device
    sums = torch.empty(2 * C, dtype=torch.float32, device=dev)
    gdt = dgamma.dtype if dgamma is not None else torch.float32
    s = native.stream_handle()
    if part is not None:
        pt, B = part
        native.check(lib.ddpx_bn_bwd_sums_from_part(pt.data_ptr(), B, C, sums.data_ptr(), native.ptr(dgamma),
                                                    native.ptr(dbeta), int(gdt == torch.bfloat16), int(accumulate),
                                                    s), "ddpx_bn_bwd_sums_from_part")
    else:
        B = lib.ddpx_bn_bwd_blocks(N, H, W, C)
        pt = torch.empty((B, 2, C), dtype=torch.float32, device=dev)
        native.check(lib.ddpx_bn_bwd_sums(gout.data_ptr(), y.data_ptr(), a.data_ptr(), b.data_ptr(), mean.data_ptr(),
                                          rstd.data_ptr(), N, H, W, C, int(pool), 1, pt.data_ptr(), sums.data_ptr(),
                                          native.ptr(dgamma), native.ptr(dbeta), int(gdt == torch.bfloat16),
                                          int(accumulate), s), "ddpx_bn_bwd_sums")
    comm.allreduce_(sums, op="sum")
    native.check(lib.ddpx_scale_f32(sums.data_ptr(), 2 * C, 1.0 / (comm.world_size * N * H * W), s), "ddpx_scale_f32")
    dy = torch.empty((N * H * W, C), dtype=torch.bfloat16, device=dev)
    native.check(lib.ddpx_bn_bwd_apply(gout.data_ptr(), y.data_ptr(), a.data_ptr(), b.data_ptr(), mean.data_ptr(),
                                       rstd.data_ptr(), sums.data_ptr(), sums[C:].data_ptr(), N, H, W, C, int(pool),
                                       1, dy.data_ptr(), s), "ddpx_bn_bwd_apply")
    return dy


def bn_apply(y, a, b, N, H, W, C, relu=True, pool=False):
    _nhwc(y, "y", C)
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    out = torch.empty((N, Ho, Wo, C), dtype=torch.bfloat16, device=y.device)
    native.check(native.kernels().ddpx_bn_apply(y.data_ptr(), a.data_ptr(), b.data_ptr(), N, H, W, C, int(relu),
                                                int(pool), out.data_ptr(), native.stream_handle()), "ddpx_bn_apply")
    return out


def bn_backward(gout, y, a, b, mean, rstd, N, H, W, C, pool, dgamma=None, dbeta=None, accumulate=False,
                sgd_gamma=None, sgd_beta=None, part=None):
    """dy [N*H*W, C] bf16; dgamma/dbeta stored (fp32/bf16) or applied through sgd_gamma / sgd_beta.  ``part`` =
    (partials [B, 2, C], B): the pass-1 sums already made by the data gradient that produced ``gout``
    (``conv_dgrad_bn``)."""
    _nhwc(gout, "gout", C)
    _nhwc(y, "y", C)
    lib = native.kernels()
    dev = y.device
    if part is not None:
        pt, B = part
        c1 = torch.empty(C, dtype=torch.float32, device=dev)
        c2 = torch.empty(C, dtype=torch.float32, device=dev)
        dy = torch.empty((N * H * W, C), dtype=torch.bfloat16, device=dev)
        gdt = dgamma.dtype if dgamma is not None else torch.float32
        sg, sb = native.sgd_args(sgd_gamma), native.sgd_args(sgd_beta)
        lr = sg[3] if sgd_gamma is not None else None
        mom, wd = (sg[4], sg[5]) if sgd_gamma is not None else (0.0, 0.0)
        native.check(lib.ddpx_bn_bwd_tail(gout.data_ptr(), y.data_ptr(), a.data_ptr(), b.data_ptr(), mean.data_ptr(),
                                          rstd.data_ptr(), N, H, W, C, int(pool), 1, pt.data_ptr(), B, c1.data_ptr(),
                                          c2.data_ptr(), native.ptr(dgamma), native.ptr(dbeta),
                                          int(gdt == torch.bfloat16), int(accumulate), dy.data_ptr(), sg[0], sg[1],
                                          sb[0], sb[1], lr, mom, wd, native.stream_handle()), "ddpx_bn_bwd_tail")
        return dy
    B = lib.ddpx_bn_bwd_blocks(N, H, W, C)
    part = torch.empty((B, 2, C), dtype=torch.float32, device=dev)
    c1 = torch.empty(C, dtype=torch.float32, device=dev)
    c2 = torch.empty(C, dtype=torch.float32, device=dev)
    dy = torch.empty((N * H * W, C), dtype=torch.bfloat16, device=dev)
    gdt = dgamma.dtype if dgamma is not None else torch.float32
    sg, sb = native.sgd_args(sgd_gamma), native.sgd_args(sgd_beta)
    lr = sg[3] if sgd_gamma is not None else None
    mom, wd = (sg[4], sg[5]) if sgd_gamma is not None else (0.0, 0.0)
    native.check(lib.ddpx_bn_bwd(gout.data_ptr(), y.data_ptr(), a.data_ptr(), b.data_ptr(), mean.data_ptr(),
                                 rstd.data_ptr(), N, H, W, C, int(pool), 1, part.data_ptr(), c1.data_ptr(),
                                 c2.data_ptr(), native.ptr(dgamma), native.ptr(dbeta), int(gdt == torch.bfloat16),
                                 int(accumulate), dy.data_ptr(), sg[0], sg[1], sb[0], sb[1], lr, mom, wd,
                                 native.stream_handle()), "ddpx_bn_bwd")
    return dy


def avgpool(x):
    N, H, W, C = x.shape
    _nhwc(x, "x")
    out = torch.empty((N, C), dtype=torch.bfloat16, device=x.device)
    native.check(native.kernels().ddpx_avgpool(x.data_ptr(), N, H * W, C, out.data_ptr(), native.stream_handle()),
                 "ddpx_avgpool")
    return out


def avgpool_backward(g, N, H, W, C):
    _nhwc(g, "g", C)
    gx = torch.empty((N, H, W, C), dtype=torch.bfloat16, device=g.device)
    native.check(native.kernels().ddpx_avgpool_bwd(g.data_ptr(), N, H * W, C, gx.data_ptr(), native.stream_handle()),
                 "ddpx_avgpool_bwd")
    return gx
