"""Host wrappers for the memory-bound native kernels (casts, column sums, SGD).

CPU tensors take an equivalent torch path (the CPU is a supported device for
the reference-shaped workloads, BASELINE config 1); GPU tensors always take the
native HIP path.
"""
from __future__ import annotations

import torch

from ..runtime import native


def cast_bf16_(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """dst (bf16) <- src (fp32), both contiguous with equal numel."""
    if src.numel() != dst.numel():
        raise ValueError("cast: numel mismatch")
    if not src.is_cuda:
        dst.copy_(src.to(torch.bfloat16))
        return dst
    if src.dtype != torch.float32 or dst.dtype != torch.bfloat16:
        raise ValueError("cast: expected fp32 -> bf16")
    if not (src.is_contiguous() and dst.is_contiguous()):
        raise ValueError("cast: tensors must be contiguous")
    lib = native.kernels()
    native.check(lib.ddpx_cast_f32_bf16(src.data_ptr(), dst.data_ptr(), src.numel(), native.stream_handle()),
                 "ddpx_cast_f32_bf16")
    return dst


def colsum_bf16(x: torch.Tensor, out: torch.Tensor, scale: float = 1.0, accumulate: bool = False):
    """out[n] (=|+=) scale * sum_m x[m, n]   (bias gradient of a Linear)."""
    if x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("colsum: x must be a row-contiguous 2-D tensor")
    M, N = x.shape
    if out.numel() != N or out.dtype != torch.float32:
        raise ValueError("colsum: out must be fp32 [N]")
    if not x.is_cuda:
        s = x.float().sum(0) * scale
        if accumulate:
            out.add_(s.view_as(out))
        else:
            out.copy_(s.view_as(out))
        return out
    if x.dtype != torch.bfloat16:
        raise ValueError("colsum: x must be bf16 on GPU")
    lib = native.kernels()
    native.check(lib.ddpx_colsum_bf16(x.data_ptr(), out.data_ptr(), M, N, x.stride(0), float(scale),
                                      int(accumulate), native.stream_handle()), "ddpx_colsum_bf16")
    return out


def sgd_flat_(param: torch.Tensor, momentum_buf: torch.Tensor, grad: torch.Tensor, shadow: torch.Tensor | None,
              lr: float | torch.Tensor, momentum: float, weight_decay: float, grad_scale: float = 1.0,
              nesterov: bool = False, first: bool = False, mx8=None):
    """One fused SGD step over flat contiguous buffers (torch.optim.SGD semantics, dampening=0).

    ``lr`` may be a Python float or a 0-d fp32 device tensor (graph-capturable path).
    ``mx8`` = (codes uint8 [n], E8M0 scales uint8 [n / 32]), n % 32 == 0: also write the updated parameters as
    MX-FP8 e4m3 blocks of 32 consecutive elements (the fp8 forward's weight operand; GPU only).
    """
    n = param.numel()
    if momentum_buf.numel() != n or grad.numel() != n or (shadow is not None and shadow.numel() != n):
        raise ValueError("sgd_flat: buffers must have equal numel")
    if not param.is_cuda:
        lr_v = float(lr) if not torch.is_tensor(lr) else float(lr.item())
        # one cache-blocked sweep: each 256K-element block goes through every pass while it is still in
        # L2 (whole-buffer passes with full-size temporaries cost ~3.7x on the 29M-parameter MLP); the
        # per-element arithmetic and its rounding order are torch.optim.SGD's
        blk = 1 << 18
        tmp = torch.empty(min(n, blk), dtype=torch.float32)
        pf, bf, gf = param.view(-1), momentum_buf.view(-1), grad.view(-1)
        sf = shadow.view(-1) if shadow is not None else None
        for s in range(0, n, blk):
            e = min(n, s + blk)
            p, g = pf[s:e], gf[s:e]
            d = tmp[:e - s]
            d.copy_(g)
            if grad_scale != 1.0:
                d.mul_(grad_scale)
            if weight_decay:
                d.add_(p, alpha=weight_decay)
            if momentum:
                b = bf[s:e]
                if first:
                    b.copy_(d)
                else:
                    b.mul_(momentum).add_(d)
                if nesterov:
                    d.add_(b, alpha=momentum)
                else:
                    d = b
            p.add_(d, alpha=-lr_v)
            if sf is not None:
                sf[s:e].copy_(p)
        return param
    lib = native.kernels()
    lr_dev = lr.data_ptr() if torch.is_tensor(lr) else None
    lr_host = 0.0 if torch.is_tensor(lr) else float(lr)
    rc = lib.ddpx_sgd_flat(param.data_ptr(), momentum_buf.data_ptr(), grad.data_ptr(),
                           int(grad.dtype == torch.bfloat16), native.ptr(shadow), n, lr_dev, lr_host,
                           float(momentum), float(weight_decay), float(grad_scale), int(nesterov), int(first),
                           native.ptr(mx8[0] if mx8 else None), native.ptr(mx8[1] if mx8 else None),
                           native.stream_handle())
    native.check(rc, "ddpx_sgd_flat")
    return param


def scale_(x: torch.Tensor, s: float):
    if not x.is_cuda or x.dtype != torch.float32:
        return x.mul_(s)
    lib = native.kernels()
    native.check(lib.ddpx_scale_f32(x.data_ptr(), x.numel(), float(s), native.stream_handle()), "ddpx_scale_f32")
    return x
