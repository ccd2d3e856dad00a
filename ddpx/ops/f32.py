"""The reference's fp32 recipe on native MI355X kernels (``--dtype fp32``).

``/root/reference/singlegpu.py:134`` builds the VGG in fp32 and ``:248-249`` reports "fp32 model has
accuracy"; this module runs that precision end to end on ``csrc/kernels/f32_train.hip`` instead of
torch/MIOpen: exact-f32 MFMA (``v_mfma_f32_16x16x4_f32``) GEMMs for Linear and the 3x3 convolutions
(implicit GEMM over NHWC, weight gradients split over N*H*W and reduced in fixed order), BatchNorm2d
statistics / apply+ReLU+MaxPool / backward, global average pool and the 10-class head + cross-entropy.

The fp32 masters in the flat parameter store are read directly (no compute shadow); gradients land in
``main_grad`` (DDP bucket storage) through the ``FlatParams`` grad protocol, so DDP, the flat SGD and
the checkpoint format are the same as on the bf16 path.
"""
from __future__ import annotations

import torch

from ..runtime import native

DENSE_KC, DENSE_OC, IM2COL_KC, IM2COL_OC = 0, 1, 2, 3
F_RELU, F_ACCUM = 1, 2

_P, _I, _I64, _F = native.c_void_p, native.c_int, native.c_int64, native.c_float
for _sig in (
        ("ddpx_f32_gemm", _I, _I, _P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _I, _I64, _P, _P, _I, _I,
         _P),
        ("ddpx_f32_splitk_reduce", _I, _P, _I, _I64, _P, _I, _P),
        ("ddpx_f32_conv_wprep", _I, _P, _I, _I, _I, _P, _P, _P),
        ("ddpx_f32_conv_wgrad_reduce", _I, _P, _I, _I, _I, _I, _P, _I, _P),
        ("ddpx_f32_bn_stats", _I, _P, _I, _I, _I, _P, _P),
        ("ddpx_f32_bn_finalize", _I, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _F, _F, _I, _P, _P, _P, _P, _P, _P),
        ("ddpx_f32_bn_apply", _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P),
        ("ddpx_f32_bn_bwd_sums", _I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P),
        ("ddpx_f32_bias_act_bwd_sums", _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P),
        ("ddpx_f32_bn_bwd_finalize", _I, _P, _I, _I, _I, _P, _P, _P, _P, _I, _P, _P),
        ("ddpx_f32_bn_bwd_apply", _I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P),
        ("ddpx_f32_avgpool", _I, _P, _I, _I, _I, _P, _I, _P),
        ("ddpx_f32_head_fwd", _I, _P, _P, _P, _P, _I, _I, _I, _P, _P, _P, _P),
        ("ddpx_f32_head_bwd", _I, _P, _P, _P, _P, _I, _I, _I, _P, _P, _I, _P, _I, _F, _P),
        ("ddpx_f32_nchw_flatten", _I, _P, _I, _I, _I, _I, _P, _P),
        ("ddpx_f32_set_staging", _I, _I),
        ("ddpx_f32_set_block", _I, _I),
        ("ddpx_f32_conv_fwd_stats", _I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P),
        ("ddpx_dropout_fwd_f32", _I, _P, _P, _I64, _F, _P, _P, _P),
        ("ddpx_f32_colsum", _I, _P, _I, _I, _P, _I, _P),
        ("ddpx_f32_wgrad_sgd", _I, _P, _I, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _F, _F, _P),
        ("ddpx_f32_splitk_epi", _I, _P, _I, _I, _I, _P, _P, _P, _I, _P),
        ("ddpx_f32_wino_ok", _I, _I, _I, _I, _I),
        ("ddpx_f32_wino_conv_mask", _I, _P, _P, _P, _P, _P, _I, _P, _I, _I, _I, _I, _I, _P),
        ("ddpx_f32_colsum_part", _I, _P, _I, _I, _I, _P, _P),
        ("ddpx_f32_wino_wprep", _I, _P, _I, _I, _I, _P, _P, _P),
        ("ddpx_f32_wino_conv", _I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P),
        ("ddpx_f32_wino_wgrad_ok", _I, _I, _I, _I, _I),
        ("ddpx_f32_wino_wgrad_splits", _I, _I, _I, _I, _I, _I),
        ("ddpx_f32_wino_wgrad", _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _I, _P),
):
    native.register_kernel_sig(*_sig)



def bn_chunk_rows(P: int, C: int) -> int:
    """Pixel rows per BatchNorm statistics chunk: ~16K elements, so a layer splits into enough workgroups
    to fill the chip (2048 at 64 channels x 32x32 x 512 images) with short per-thread row loops."""
    return max(8, min(P, 16384 // C))


def _req(c, msg):
    if not c:
        raise ValueError(msg)


def _f32(t, name):
    _req(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous(), f"{name} must be contiguous fp32 on GPU")
    _req(t.data_ptr() % 16 == 0, f"{name} must be 16-B aligned")


def set_staging(dma: bool) -> bool:
    """GEMM operand staging of the f32 core: LDS-DMA ring (True, the default) or register-staged (False;
    DDPX_F32_STAGING=reg).  Returns the previous setting."""
    return bool(native.kernels().ddpx_f32_set_staging(int(bool(dma))))


def set_block(kb: int) -> int:
    """Summation block of the LDS-DMA core's blocked mode in 16-k K-steps (1, 2 or 4 = default); 1 reproduces the
    register-staged kernel bitwise.  Returns the previous setting."""
    return int(native.kernels().ddpx_f32_set_block(int(kb)))


def _call(name, *args):
    native.check(getattr(native.kernels(), name)(*args, native.stream_handle()), name)


def gemm(amode, a, lda, bmode, b, ldb, M, N, K, out, ldc=None, bias=None, mask=None, relu=False, accumulate=False,
         geom=(0, 0, 0, 1), splits=1, split_stride=0, tile=-1):
    """out (+)= A B on the f32 MFMA core (operand modes: see f32_train.hip)."""
    flags = (F_RELU if relu else 0) | (F_ACCUM if accumulate else 0)
    _call("ddpx_f32_gemm", amode, a.data_ptr(), lda, bmode, b.data_ptr(), ldb, M, N, K, *geom, splits,
          out.data_ptr(), N if ldc is None else ldc, split_stride, native.ptr(bias), native.ptr(mask), flags, tile)


# ---------------------------------------------------------------------------------------------- Linear
# DDPX_F32_SPLITK (default 2): the batch-row (M <= 1024) Linear forward / data gradient as 2 in-grid K splits on
# 64x64 tiles (1024 workgroups instead of 512: 4 per CU) and one finishing pass with the epilogue
# (profiles/r5_mlp32: fc0 / fc1 152 / 178 -> 129 / 153 us + 7 us); 1 = one pass.  The split changes the summation
# into two half-length chains added at the end (closer to fp64, not bitwise the one-pass result).
import os as _os_lin  # noqa: E402

_F32_SPLITK = int(_os_lin.environ.get("DDPX_F32_SPLITK", "2"))


def _splitk_linear(amode, a, lda, bmode, b, ldb, M, N, K, bias=None, mask=None, relu=False):
    S = _F32_SPLITK
    if S < 2 or M > 1024 or N % 4 or K < 1024 or (M * N) < (1 << 20):
        return None
    part = torch.empty((S, M, N), dtype=torch.float32, device=a.device)
    gemm(amode, a, lda, bmode, b, ldb, M, N, K, part, tile=2, splits=S, split_stride=M * N)
    out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    _call("ddpx_f32_splitk_epi", part.data_ptr(), S, M, N, out.data_ptr(), native.ptr(bias), native.ptr(mask),
          int(relu))
    return out


def linear_fwd(x, w, bias=None, relu=False):
    """y = x W^T + b [relu] — x [M,K], W [N,K] (torch layout)."""
    M, K = x.shape
    N = w.shape[0]
    _f32(x, "x")
    _f32(w, "w")
    _req(w.shape[1] == K, "linear_fwd: shape mismatch")
    y = _splitk_linear(DENSE_KC, x, K, DENSE_KC, w, K, M, N, K, bias=bias, relu=relu)
    if y is not None:
        return y
    y = torch.empty((M, N), dtype=torch.float32, device=x.device)
    gemm(DENSE_KC, x, K, DENSE_KC, w, K, M, N, K, y, bias=bias, relu=relu)
    return y


def linear_dgrad(dy, w, mask=None):
    """dx = dy W [* (mask > 0)] — dy [M,N], W [N,K]."""
    M, N = dy.shape
    K = w.shape[1]
    _f32(dy, "dy")
    dx = _splitk_linear(DENSE_KC, dy, N, DENSE_OC, w, K, M, K, N, mask=mask)
    if dx is not None:
        return dx
    dx = torch.empty((M, K), dtype=torch.float32, device=dy.device)
    gemm(DENSE_KC, dy, N, DENSE_OC, w, K, M, K, N, dx, mask=mask)
    return dx


def linear_wgrad(dy, x, out, accumulate=False):
    """dW (+)= dy^T x — dy [M,N], x [M,K], dW [N,K]."""
    M, N = dy.shape
    K = x.shape[1]
    _req(out.shape == (N, K) and out.is_contiguous(), "linear_wgrad: bad output")
    gemm(DENSE_OC, dy, N, DENSE_OC, x, K, N, K, M, out, accumulate=accumulate)


def linear_wgrad_sgd(dy, x, sgd):
    """W -= SGD(dy^T x) in the weight-gradient GEMM's epilogue (fused optimizer, single process); ``sgd`` =
    FlatParams.fused_spec(W).  False when the core cannot (register-staged core): the caller stores the
    gradient instead."""
    M, N = dy.shape
    K = x.shape[1]
    p, buf, sh, lr, mom, wd = sgd
    _req(p.numel() == N * K, "linear_wgrad_sgd: parameter size")
    r = native.kernels().ddpx_f32_wgrad_sgd(dy.data_ptr(), N, x.data_ptr(), K, M, N, K, -1, p.data_ptr(),
                                             native.ptr(buf), native.ptr(sh), lr.data_ptr(), float(mom), float(wd),
                                             native.stream_handle())
    if r == -6:
        return False
    native.check(r, "ddpx_f32_wgrad_sgd")
    return True


def colsum(x, out, accumulate=False):
    M, N = x.shape
    _call("ddpx_f32_colsum", x.data_ptr(), M, N, out.data_ptr(), int(accumulate))


def head_forward(h, w, b, targets=None):
    """(loss [scalar] or None, logits [M,NC], dlogits [M,NC] or None) of the fp32 classifier head."""
    M, K = h.shape
    NC = w.shape[0]
    _f32(h, "h")
    logits = torch.empty((M, NC), dtype=torch.float32, device=h.device)
    loss = dl = None
    if targets is not None:
        _req(targets.dtype == torch.int64 and targets.numel() == M, "targets must be int64 [M]")
        loss = torch.empty((), dtype=torch.float32, device=h.device)
        dl = torch.empty_like(logits)
    _call("ddpx_f32_head_fwd", h.data_ptr(), w.data_ptr(), b.data_ptr(), native.ptr(targets), M, K, NC,
          logits.data_ptr(), native.ptr(loss), native.ptr(dl))
    return loss, logits, dl


def head_backward(dl, grad_out, h, w, dW, db, accumulate=False, relu_mask=False, want_dh=True, dh_scale=1.0):
    M, K = h.shape
    NC = w.shape[0]
    go = grad_out.float().contiguous() if grad_out is not None else None
    dh = torch.empty_like(h) if want_dh else None
    _call("ddpx_f32_head_bwd", dl.data_ptr(), native.ptr(go), h.data_ptr(), w.data_ptr(), M, K, NC, native.ptr(dW),
          native.ptr(db), int(accumulate), native.ptr(dh), int(relu_mask), float(dh_scale))
    return dh


def nchw_flatten(x):
    """torch.flatten(x, 1) of the NCHW tensor an NHWC fp32 activation [N,H,W,C] stands for: [N, C*H*W]."""
    N, H, W, C = x.shape
    _f32(x, "x")
    out = torch.empty((N, C * H * W), dtype=torch.float32, device=x.device)
    _call("ddpx_f32_nchw_flatten", x.data_ptr(), N, H * W, C, 0, out.data_ptr())
    return out


def nchw_unflatten(g, N, H, W, C):
    """Gradient of nchw_flatten: [N, C*H*W] -> NHWC [N,H,W,C]."""
    _f32(g, "g")
    out = torch.empty((N, H, W, C), dtype=torch.float32, device=g.device)
    _call("ddpx_f32_nchw_flatten", g.data_ptr(), N, H * W, C, 1, out.data_ptr())
    return out


def dropout_(x, p, rng, rng_done):
    """Inverted Dropout(p) of an fp32 tensor; generator state (seed, offset) device-resident in ``rng``."""
    _f32(x, "x")
    _req(x.numel() % 4 == 0, "dropout: numel % 4 != 0")
    out = torch.empty_like(x)
    _call("ddpx_dropout_fwd_f32", x.data_ptr(), out.data_ptr(), x.numel(), float(p), rng.data_ptr(),
          rng_done.data_ptr())
    return out


# ---------------------------------------------------------------------------------------------- conv / BN
def conv_channels(ci: int) -> int:
    """Input channels as stored (NHWC, 16-B pixels: the 3-channel image is zero-padded to 4)."""
    return max(4, (ci + 3) // 4 * 4)


def conv_wprep(w, wf, wd):
    Co, Ci = w.shape[:2]
    Cp = conv_channels(Ci)
    _req(wf.numel() == 9 * Cp * Co and (wd is None or wd.numel() == 9 * Co * Ci), "conv_wprep: bad buffers")
    _call("ddpx_f32_conv_wprep", w.data_ptr(), Co, Ci, Cp, wf.data_ptr(), native.ptr(wd))


def conv_fwd(x, wf, Co):
    """y [N*H*W, Co] = conv3x3(x [N,H,W,Cp], pad 1)."""
    N, H, W, C = x.shape
    _f32(x, "x")
    P = N * H * W
    y = torch.empty((P, Co), dtype=torch.float32, device=x.device)
    gemm(IM2COL_KC, x, 0, DENSE_OC, wf, Co, P, Co, 9 * C, y, geom=(C, H, W, 1))
    return y


def conv_fwd_stats(x, wf, Co):
    """(y, (stats, T, R)) — the forward convolution with the BatchNorm tile statistics (mean, M2 of every R-row
    output tile) emitted by the GEMM epilogue (LDS-DMA core), or (y, None) when that path does not apply."""
    N, H, W, C = x.shape
    _f32(x, "x")
    P = N * H * W
    y = torch.empty((P, Co), dtype=torch.float32, device=x.device)
    T = (P + 63) // 64  # enough rows of statistics for the smaller tile
    stats = torch.empty((T, 2, Co), dtype=torch.float32, device=x.device)
    r = native.kernels().ddpx_f32_conv_fwd_stats(x.data_ptr(), wf.data_ptr(), y.data_ptr(), N, H, W, C, Co,
                                                 stats.data_ptr(), native.stream_handle())
    if r < 0:
        if r == -10:  # register-staged core selected: plain forward, statistics by their own pass
            gemm(IM2COL_KC, x, 0, DENSE_OC, wf, Co, P, Co, 9 * C, y, geom=(C, H, W, 1))
            return y, None
        native.check(r, "ddpx_f32_conv_fwd_stats")
    return y, (stats, (P + r - 1) // r, r)


def conv_dgrad(dy, wd, N, H, W, C, Co):
    """dx [N,H,W,C] = transposed conv of dy [N*H*W, Co] with wd [(r,s,co), ci]."""
    _f32(dy, "dy")
    dx = torch.empty((N, H, W, C), dtype=torch.float32, device=dy.device)
    gemm(IM2COL_KC, dy, 0, DENSE_OC, wd, C, N * H * W, C, 9 * Co, dx, geom=(Co, H, W, -1))
    return dx


# ------------------------------------------------------------------ Winograd F(2x2, 3x3) (csrc/kernels/f32_wino.hip)
# The forward and data-gradient 3x3 convolutions with >= DDPX_F32_WINO_MIN_C input channels (default 16: every
# layer but the 3-channel image one) run as fp32 Winograd F(2,3), MIOpen's algorithm for the
# stock fp32 recipe, with 2.25x fewer multiplies than the exact implicit GEMM.  DDPX_F32_WINO=0: the direct
# implicit GEMM everywhere (the weight gradient always is).
import os as _os  # noqa: E402

_WINO = _os.environ.get("DDPX_F32_WINO", "1") != "0"
_WINO_MIN_C = int(_os.environ.get("DDPX_F32_WINO_MIN_C", "16"))


def wino_applies(H, W, C, K) -> bool:
    return _WINO and C >= _WINO_MIN_C and bool(native.kernels().ddpx_f32_wino_ok(H, W, C, K))


def wino_wprep(w, uf, ud):
    """uf [16][Cp][Co] (forward) and ud [16][Co][Ci] (data gradient, flipped kernel) = G g G^T of w [Co,Ci,3,3]."""
    Co, Ci = w.shape[:2]
    Cp = conv_channels(Ci)
    _req(uf is None or uf.numel() == 16 * Cp * Co, "wino_wprep: bad forward buffer")
    _req(ud is None or ud.numel() == 16 * Co * Ci, "wino_wprep: bad data-gradient buffer")
    _call("ddpx_f32_wino_wprep", w.data_ptr(), Co, Ci, Cp, native.ptr(uf), native.ptr(ud))


def wino_conv(x, u, K, stats=False, bias=None, relu=False, mask=None):
    """y [N*H*W, K] = [relu](conv3x3(x [N,H,W,C]) [+ bias]) through F(2,3) with u [16][C][K]; with ``stats``:
    (y, (part, T, 256)), the BatchNorm chunk statistics of every 256-pixel output chunk from the epilogue.
    ``mask`` [N*H*W, K] (a data gradient through the ReLU of the block below): y = 0 where mask <= 0."""
    N, H, W, C = x.shape
    _f32(x, "x")
    if mask is not None:
        _f32(mask, "mask")
        _req(mask.numel() == N * H * W * K, "wino_conv: bad mask")
    y = torch.empty((N * H * W, K), dtype=torch.float32, device=x.device)
    T = (N * (H // 2) * (W // 2) + 63) // 64
    st = torch.empty((T, 2, K), dtype=torch.float32, device=x.device) if stats else None
    r = native.kernels().ddpx_f32_wino_conv_mask(x.data_ptr(), u.data_ptr(), y.data_ptr(), native.ptr(st),
                                                  native.ptr(bias), int(relu), native.ptr(mask), N, H, W, C, K,
                                                  native.stream_handle())
    native.check(r if r < 0 else 0, "ddpx_f32_wino_conv")
    return (y, (st, T, r)) if stats else y


def wgrad_splits(Co, Ncols, P):
    tiles = ((Co + 127) // 128) * ((Ncols + 127) // 128)
    s = max(1, min(P // 1024, (2048 + tiles - 1) // tiles))
    return s


# Weight gradient through F(2,3) too (csrc/kernels/f32_wino.hip wino_wgrad_kernel: dW = G^T (sum over tiles of
# (A dY A^T) (.) (B^T x B)) G, 4/9 of the direct product's multiplies); DDPX_F32_WINO_WGRAD=0: the direct split-K
# implicit GEMM.  Applies at Cp % 32 == 0, Co % 64 == 0, even H and W.
_WINO_WGRAD = _os.environ.get("DDPX_F32_WINO_WGRAD", "1") != "0"
# DDPX_F32_WINO_WGRAD_PAD=0: 32-output-channel layers keep the direct weight gradient (A/B)
_WINO_WGRAD_PAD = _os.environ.get("DDPX_F32_WINO_WGRAD_PAD", "1") != "0"


def wino_wgrad_applies(H, W, Cp, Co) -> bool:
    return _WINO and _WINO_WGRAD and bool(native.kernels().ddpx_f32_wino_wgrad_ok(H, W, Cp, Co))


def wino_wgrad(dy, x, Co, Ci, out, accumulate=False):
    """out [Co,Ci,3,3] (+)= the Winograd F(2,3) weight gradient from dy [P, Co] and x [N,H,W,Cp]."""
    N, H, W, Cp = x.shape
    _f32(x, "x")
    _req(dy.dtype == torch.float32 and dy.is_contiguous() and dy.numel() == N * H * W * Co, "wino_wgrad: bad dy")
    _req(out.dtype == torch.float32 and out.is_contiguous() and out.numel() == Co * Ci * 9, "wino_wgrad: bad out")
    lib = native.kernels()
    S = lib.ddpx_f32_wino_wgrad_splits(N, H, W, Cp, Co)
    part = torch.empty((S, 16, Co, Cp), dtype=torch.float32, device=dy.device)
    du = torch.empty((16, Co, Cp), dtype=torch.float32, device=dy.device)
    _call("ddpx_f32_wino_wgrad", x.data_ptr(), dy.data_ptr(), part.data_ptr(), du.data_ptr(), N, H, W, Cp, Co, Ci, S,
          out.data_ptr(), int(accumulate))


def conv_wgrad(dy, x, Co, Ci, out, accumulate=False):
    """out [Co,Ci,3,3] (+)= weight gradient from dy [P, Co] and x [N,H,W,Cp]."""
    N, H, W, Cp = x.shape
    if wino_wgrad_applies(H, W, Cp, Co):
        return wino_wgrad(dy, x, Co, Ci, out, accumulate)
    if _WINO_WGRAD_PAD and Co == 32 and dy.is_cuda and wino_wgrad_applies(H, W, Cp, 64):
        # 32 output channels (DeepNN's 64 -> 32 layer): the Winograd weight gradient over dy zero-padded to 64
        # channels (its 4/9 multiplies beat the direct GEMM's tile padded from 32 to 64 rows: 121 us there)
        dyp = torch.nn.functional.pad(dy.view(-1, Co), (0, 64 - Co))
        tmp = torch.empty(64 * Ci * 9, dtype=torch.float32, device=dy.device)
        wino_wgrad(dyp, x, 64, Ci, tmp)
        o = out.view(-1)
        if accumulate:
            o.add_(tmp[:Co * Ci * 9])
        else:
            o.copy_(tmp[:Co * Ci * 9])
        return None
    return direct_wgrad(dy, x, Co, Ci, out, accumulate)


def direct_wgrad(dy, x, Co, Ci, out, accumulate=False):
    """conv_wgrad on the exact implicit GEMM (split over N*H*W, reduced in fixed order)."""
    N, H, W, Cp = x.shape
    P = N * H * W
    ncol = 9 * Cp
    S = wgrad_splits(Co, ncol, P)
    part = torch.empty((S, Co, ncol), dtype=torch.float32, device=dy.device)
    gemm(DENSE_OC, dy, Co, IM2COL_OC, x, 0, Co, ncol, P, part, geom=(Cp, H, W, 1), splits=S,
         split_stride=Co * ncol)
    _call("ddpx_f32_conv_wgrad_reduce", part.data_ptr(), S, Co, Ci, Cp, out.data_ptr(), int(accumulate))


def bn_forward(y, N, H, W, C, bn, training, pool, stats=None, comm=None):
    """(x_next, a, b, mean, rstd): statistics + running-stat update + [pool](relu(a*(y-mean)+b)), a = gamma*rstd,
    b = beta.  ``stats`` = (part, T, R): chunk statistics already made (the conv GEMM epilogue).

    ``comm`` (SyncBatchNorm, ``--sync_bn`` under DDP; /root/reference/multigpu.py:127): this rank's (mean, M2) is
    merged from its chunk statistics (``ddpx_bn_local_stats``), all-gathered ([world][2][C], one collective on the
    current stream: graph-capturable on RCCL), and the finalize merges the ranks in rank order as equal chunks
    of P rows each, so the batch statistics and the running-stat update (unbiased with the global count, as
    torch's SyncBatchNorm) are the global ones.  Every rank holds the same P (equal DistributedSampler shards)."""
    dev = y.device
    P = N * H * W
    a = torch.empty(C, dtype=torch.float32, device=dev)
    b, mean, rstd = torch.empty_like(a), torch.empty_like(a), torch.empty_like(a)
    if training and stats is not None:
        part, T, R = stats
    else:
        R = bn_chunk_rows(P, C)
        T = (P + R - 1) // R
        part = torch.empty((T, 2, C), dtype=torch.float32, device=dev) if training else a
        if training:
            _call("ddpx_f32_bn_stats", y.data_ptr(), P, C, R, part.data_ptr())
    Ptot = P
    if training and comm is not None:
        local = torch.empty(2 * C, dtype=torch.float32, device=dev)
        native.check(native.kernels().ddpx_bn_local_stats(part.data_ptr(), T, R, P, C, local.data_ptr(),
                                                          native.stream_handle()), "ddpx_bn_local_stats")
        ws = comm.world_size
        part = torch.empty(ws * 2 * C, dtype=torch.float32, device=dev)
        comm.allgather(part, local)
        T, R, Ptot = ws, P, ws * P
    nbt = bn.num_batches_tracked if (training and bn.num_batches_tracked is not None) else None
    _call("ddpx_f32_bn_finalize", part.data_ptr(), T, R, Ptot, C, bn.weight.data_ptr(), bn.bias.data_ptr(),
          bn.running_mean.data_ptr(), bn.running_var.data_ptr(), native.ptr(nbt), float(bn.momentum),
          float(bn.eps), int(training), a.data_ptr(), b.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
          native.ptr(_fin_ws(T, C, dev)))
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    out = torch.empty((N, Ho, Wo, C), dtype=torch.float32, device=dev)
    _call("ddpx_f32_bn_apply", y.data_ptr(), a.data_ptr(), b.data_ptr(), mean.data_ptr(), N, H, W, C, 1, int(pool),
          out.data_ptr())
    return out, a, b, mean, rstd


_FIN_SPLIT_MAX, _FIN_SPLIT_MAX_C = 32, 1024  # f32_train.hip kFinSplitMax / kFinSplitMaxC


def _fin_ws(T, C, dev):
    """fp64 workspace [2][32][C] of the split BatchNorm merges (f32_train.hip bn_fin_*), from the caching allocator
    on the current stream, or None where the merge does not split (the kernels then take the one-pass merge)."""
    if T < 1024 or C > _FIN_SPLIT_MAX_C:
        return None
    return torch.empty(2 * _FIN_SPLIT_MAX * C, dtype=torch.float64, device=dev)


def bn_backward(g, y, a, b, mean, rstd, N, H, W, C, pool, dgamma, dbeta, accumulate=False, comm=None):
    """dy [P, C] of BatchNorm+ReLU(+MaxPool) given the block output gradient g; dgamma/dbeta (+)= ...

    ``comm`` (SyncBatchNorm): the per-channel means c1 = mean(dy), c2 = mean(dy * xhat) are summed over the ranks
    (one all-reduce of [2][C]) and divided by the world size — the global means, every rank holding P rows — before
    the apply; dgamma / dbeta stay this rank's sums (DDP averages them), as in torch's SyncBatchNorm."""
    _f32(g, "g")
    P = N * H * W
    R = bn_chunk_rows(P, C)
    T = (P + R - 1) // R
    part = torch.empty((T, 2, C), dtype=torch.float32, device=y.device)
    _call("ddpx_f32_bn_bwd_sums", g.data_ptr(), y.data_ptr(), a.data_ptr(), b.data_ptr(), mean.data_ptr(),
          rstd.data_ptr(), N, H, W, C, int(pool), R, part.data_ptr())
    cc = torch.empty(2 * C, dtype=torch.float32, device=y.device)
    c1, c2 = cc[:C], cc[C:]
    _call("ddpx_f32_bn_bwd_finalize", part.data_ptr(), T, P, C, c1.data_ptr(), c2.data_ptr(), native.ptr(dgamma),
          native.ptr(dbeta), int(accumulate), native.ptr(_fin_ws(T, C, y.device)))
    if comm is not None:
        comm.allreduce_(cc, op="sum")
        native.check(native.kernels().ddpx_scale_f32(cc.data_ptr(), 2 * C, 1.0 / comm.world_size,
                                                     native.stream_handle()), "ddpx_scale_f32")
    dy = torch.empty((P, C), dtype=torch.float32, device=y.device)
    _call("ddpx_f32_bn_bwd_apply", g.data_ptr(), y.data_ptr(), a.data_ptr(), b.data_ptr(), mean.data_ptr(),
          rstd.data_ptr(), c1.data_ptr(), c2.data_ptr(), N, H, W, C, int(pool), dy.data_ptr())
    return dy


def avgpool(x):
    N, H, W, C = x.shape
    out = torch.empty((N, C), dtype=torch.float32, device=x.device)
    _call("ddpx_f32_avgpool", x.data_ptr(), N, H * W, C, out.data_ptr(), 0)
    return out


def avgpool_backward(g, N, H, W, C):
    dx = torch.empty((N, H, W, C), dtype=torch.float32, device=g.device)
    _call("ddpx_f32_avgpool", g.data_ptr(), N, H * W, C, dx.data_ptr(), 1)
    return dx


# ---------------------------------------------------------------------------------------------- grads
def _grad_write(flat, p, fn):
    """Run fn(out, accumulate) into p's gradient slot (DDP bucket storage) and announce it."""
    g, acc = flat.grad_target(p)
    fn(g, acc)
    flat.grad_done(p)


# ---------------------------------------------------------------------------------------------- VGG
class _VGGPlan:
    def __init__(self, model):
        self.blocks = _blocks_of(model)
        dev = model.classifier.weight.device
        self.wf, self.wd, self.uf, self.ud = [], [], [], []
        H = 32  # CIFAR-10: the pools halve it after blocks 1, 3, 5, 7
        for bi, (conv, _, pool) in enumerate(self.blocks):
            Co, Ci = conv.weight.shape[:2]
            Cp = conv_channels(Ci)
            # Winograd for the forward (and, below the first block, the data gradient) where it applies; the
            # direct layouts only where it does not
            wino = dev.type == "cuda" and wino_applies(H, H, Cp, Co)
            dwino = wino and bi > 0 and wino_applies(H, H, Co, Ci)  # the data gradient: Co -> Ci channels
            self.uf.append(torch.empty(16 * Cp * Co, dtype=torch.float32, device=dev) if wino else None)
            self.ud.append(torch.empty(16 * Co * Ci, dtype=torch.float32, device=dev) if dwino else None)
            direct = not wino or (bi > 0 and not dwino)
            self.wf.append(torch.empty(9 * Cp * Co, dtype=torch.float32, device=dev) if direct else None)
            self.wd.append(torch.empty(9 * Co * Ci, dtype=torch.float32, device=dev)
                           if (direct and Ci % 4 == 0) else None)
            if pool:
                H //= 2


def _blocks_of(model):
    from torch import nn
    mods = list(model.backbone.children())
    blocks, i = [], 0
    while i < len(mods):
        conv, bn = mods[i], mods[i + 1]
        assert isinstance(conv, nn.Conv2d) and isinstance(bn, nn.BatchNorm2d)
        i += 3
        pool = i < len(mods) and isinstance(mods[i], nn.MaxPool2d)
        if pool:
            i += 1
        blocks.append((conv, bn, pool))
    return blocks


def _vgg_plan(model):
    p = getattr(model, "_ddpx_plan_f32", None)
    if p is None:
        p = _VGGPlan(model)
        model._ddpx_plan_f32 = p
    return p


def prep_vgg_input(x):
    """NHWC fp32 with 4 channels (the loader's ``nhwc4_f32`` layout), or NCHW fp32 from a reference loader."""
    if x.dim() == 4 and x.shape[-1] == 4 and x.dtype == torch.float32:
        return x.contiguous()
    if x.dim() == 4 and x.shape[1] == 3:
        x = x.float().permute(0, 2, 3, 1)
        return torch.nn.functional.pad(x, (0, 1)).contiguous()
    raise ValueError(f"unsupported VGG input {tuple(x.shape)} {x.dtype}")


def _sync_comm(model, training):
    """SyncBatchNorm communicator (``--sync_bn`` under DDP at world size > 1), else None."""
    comm = getattr(model, "sync_bn_comm", None)
    return comm if (training and comm is not None and comm.world_size > 1) else None


def _vgg_forward(model, x, targets, training):
    plan = _vgg_plan(model)
    saved = []
    comm = _sync_comm(model, training)
    N, H, W, C = x.shape
    for bi, (conv, bn, pool) in enumerate(plan.blocks):
        Co = conv.weight.shape[0]
        wino = plan.uf[bi] is not None and H == W and wino_applies(H, W, C, Co)
        if wino:
            wino_wprep(conv.weight, plan.uf[bi], plan.ud[bi])
            if plan.wd[bi] is not None:  # data gradient on the direct GEMM
                conv_wprep(conv.weight, plan.wf[bi], plan.wd[bi])
            if training:
                y, st = wino_conv(x, plan.uf[bi], Co, stats=True)
            else:
                y, st = wino_conv(x, plan.uf[bi], Co), None
        else:
            if plan.wf[bi] is None:  # planned for Winograd at another input size: direct layouts on demand
                plan.wf[bi] = torch.empty(9 * C * Co, dtype=torch.float32, device=x.device)
                plan.wd[bi] = torch.empty(9 * Co * conv.weight.shape[1], dtype=torch.float32, device=x.device)
                plan.ud[bi] = None
            conv_wprep(conv.weight, plan.wf[bi], plan.wd[bi])
            if training:
                y, st = conv_fwd_stats(x, plan.wf[bi], Co)
            else:
                y, st = conv_fwd(x, plan.wf[bi], Co), None
        xn, a, b, mean, rstd = bn_forward(y, N, H, W, Co, bn, training, pool, stats=st, comm=comm)
        saved.append((x, y, a, b, mean, rstd, (N, H, W, C, Co), wino))
        x = xn
        H, W, C = xn.shape[1], xn.shape[2], Co
    feat = avgpool(x)
    cls = model.classifier
    loss, logits, dl = head_forward(feat, cls.weight, cls.bias, targets)
    return saved, (x.shape, feat), loss, logits, dl


def _vgg_backward(model, saved, last, dl, grad_out):
    plan = _vgg_plan(model)
    flat = model.classifier.weight._ddpx_flat
    cls = model.classifier
    xshape, feat = last
    dW, acc = flat.grad_target(cls.weight)
    db, _ = flat.grad_target(cls.bias)
    dfeat = head_backward(dl, grad_out, feat, cls.weight, dW, db, accumulate=acc)
    flat.grad_done(cls.weight)
    flat.grad_done(cls.bias)
    g = avgpool_backward(dfeat, *xshape)
    comm = _sync_comm(model, True)
    for bi in range(len(plan.blocks) - 1, -1, -1):
        conv, bn, pool = plan.blocks[bi]
        x, y, a, b, mean, rstd, (N, H, W, C, Co), wino = saved[bi]
        dgam, accg = flat.grad_target(bn.weight)
        dbet, _ = flat.grad_target(bn.bias)
        dy = bn_backward(g, y, a, b, mean, rstd, N, H, W, Co, pool, dgam, dbet, accumulate=accg, comm=comm)
        flat.grad_done(bn.weight)
        flat.grad_done(bn.bias)
        _grad_write(flat, conv.weight, lambda o, ac: conv_wgrad(dy, x, Co, conv.weight.shape[1], o, ac))
        if bi > 0:
            if wino and plan.ud[bi] is not None:  # made by this step's forward (Winograd data gradient planned)
                g = wino_conv(dy.view(N, H, W, Co), plan.ud[bi], C).view(N, H, W, C)
            else:
                g = conv_dgrad(dy, plan.wd[bi], N, H, W, C, Co)


class _VGGLossF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, targets, model, *params):
        saved, last, loss, _, dl = _vgg_forward(model, x, targets, model.training)
        ctx.model, ctx.saved, ctx.last, ctx.dl, ctx.n = model, saved, last, dl, len(params)
        return loss

    @staticmethod
    def backward(ctx, grad_loss):
        _vgg_backward(ctx.model, ctx.saved, ctx.last, ctx.dl, grad_loss)
        ctx.saved = ctx.last = ctx.dl = None
        return (None, None, None) + (None,) * ctx.n


def vgg_loss(model, x, targets):
    return _VGGLossF32.apply(prep_vgg_input(x), targets, model, *model.parameters())


def vgg_logits(model, x):
    """Inference logits (no autograd through the native fp32 path)."""
    with torch.no_grad():
        _, _, _, logits, _ = _vgg_forward(model, prep_vgg_input(x), None, model.training)
    return logits


# ---------------------------------------------------------------------------------------------- DeepNN
# /root/reference/singlegpu.py:18-44 at the reference's precision: [conv3x3+bias -> ReLU] x2 -> MaxPool2 ->
# [conv3x3+bias -> ReLU] x2 -> MaxPool2 -> flatten (C,H,W) -> Linear(2048,512) -> ReLU -> Dropout(0.1) ->
# Linear(512,10).  Conv bias + ReLU in the GEMM epilogue; the pool (and the backward's ReLU mask + first-max
# routing + bias gradient) through the BatchNorm kernels with the identity affine (a = 1, b = 0, mean = 0,
# rstd = 1, and c1 = c2 = 0 in the apply: dy = routed, masked gradient).
class _DeepNNPlan:
    def __init__(self, model):
        mods = list(model.features.children())
        self.blocks, i = [], 0
        while i < len(mods):
            conv = mods[i]
            i += 2  # conv, relu
            pool = i < len(mods) and isinstance(mods[i], torch.nn.MaxPool2d)
            if pool:
                i += 1
            self.blocks.append((conv, pool))
        cls = list(model.classifier.children())
        self.lin0, self.drop, self.lin1 = cls[0], cls[2], cls[3]
        dev = self.lin0.weight.device
        self.wf, self.wd, self.uf, self.ud = [], [], [], []
        H = 32
        for bi, (conv, pool) in enumerate(self.blocks):
            Co, Ci = conv.weight.shape[:2]
            Cp = conv_channels(Ci)
            # Winograd F(2,3) forward (+ bias + ReLU epilogue) and data gradient where it applies (the 128 -> 64,
            # 64 -> 64 and 64 -> 32 layers), the direct implicit GEMM elsewhere
            wino = dev.type == "cuda" and wino_applies(H, H, Cp, Co)
            dwino = wino and bi > 0 and wino_applies(H, H, Co, Ci)  # the data gradient: Co -> Ci channels
            self.uf.append(torch.empty(16 * Cp * Co, dtype=torch.float32, device=dev) if wino else None)
            self.ud.append(torch.empty(16 * Co * Ci, dtype=torch.float32, device=dev) if dwino else None)
            self.wf.append(torch.empty(9 * Cp * Co, dtype=torch.float32, device=dev))
            self.wd.append(torch.empty(9 * Co * Ci, dtype=torch.float32, device=dev) if Ci % 4 == 0 else None)
            if pool:
                H //= 2
        cmax = max(c.weight.shape[0] for c, _ in self.blocks)
        self.ones = torch.ones(cmax, dtype=torch.float32, device=dev)
        self.zeros = torch.zeros(cmax, dtype=torch.float32, device=dev)
        self.scratch = torch.empty(2 * cmax, dtype=torch.float32, device=dev)
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self.rng = torch.tensor([seed, 0], dtype=torch.int64, device=dev)
        self.rng_done = torch.zeros(1, dtype=torch.int32, device=dev)


def _deepnn_plan(model):
    p = getattr(model, "_ddpx_plan_f32", None)
    if p is None:
        p = _DeepNNPlan(model)
        model._ddpx_plan_f32 = p
    return p


def bias_act_backward(g, y, N, H, W, C, pool, plan, dbias, accumulate=False):
    """dy [P, C] and dbias (+)= sum dy of out = [maxpool2](y), y = relu(conv + bias) (the ReLU mask and the pool's
    first-max routing recomputed from y)."""
    _f32(g, "g")
    P = N * H * W
    R = bn_chunk_rows(P, C)
    T = (P + R - 1) // R
    one, zero = plan.ones[:C], plan.zeros[:C]
    part = torch.empty((T, 2, C), dtype=torch.float32, device=y.device)
    dy = torch.empty((P, C), dtype=torch.float32, device=y.device)
    # the sums pass writes dy = gz too where the 4-channel path applies (no sums needed for it: no normalisation)
    wrote = native.kernels().ddpx_f32_bias_act_bwd_sums(g.data_ptr(), y.data_ptr(), one.data_ptr(), zero.data_ptr(),
                                                        N, H, W, C, int(pool), R, part.data_ptr(), dy.data_ptr(),
                                                        native.stream_handle())
    if wrote < 0:
        native.check(wrote, "ddpx_f32_bias_act_bwd_sums")
    c1, c2 = plan.scratch[:C], plan.scratch[C:2 * C]
    _call("ddpx_f32_bn_bwd_finalize", part.data_ptr(), T, P, C, c1.data_ptr(), c2.data_ptr(), None, dbias.data_ptr(),
          int(accumulate), native.ptr(_fin_ws(T, C, y.device)))
    if wrote != 1:
        _call("ddpx_f32_bn_bwd_apply", g.data_ptr(), y.data_ptr(), one.data_ptr(), zero.data_ptr(), zero.data_ptr(),
              one.data_ptr(), zero.data_ptr(), zero.data_ptr(), N, H, W, C, int(pool), dy.data_ptr())
    return dy


# DDPX_F32_DGRAD_MASK=1: the Winograd data gradient into a non-pooled conv + ReLU block applies that block's ReLU
# mask in its epilogue, and the block only sums the bias gradient (colsum_bias) instead of the one-pass
# bias_act_backward (default 0).  Measured even (profiles/r6_f32epi): the first conv's backward pass drops
# 156 -> 49 us, but the mask read in the 128 -> 64 layer's dgrad epilogue adds 126 us (377 -> 503).
_DGRAD_MASK = _os.environ.get("DDPX_F32_DGRAD_MASK", "0") != "0"


def colsum_bias(dy, P, C, plan, dbias, accumulate=False):
    """dbias (+)= sum over the P rows of dy [P, C] (fixed-order chunk sums merged by bn_bwd_finalize)."""
    R = bn_chunk_rows(P, C)
    T = (P + R - 1) // R
    part = torch.empty((T, 2, C), dtype=torch.float32, device=dy.device)
    _call("ddpx_f32_colsum_part", dy.data_ptr(), P, C, R, part.data_ptr())
    c1, c2 = plan.scratch[:C], plan.scratch[C:2 * C]
    _call("ddpx_f32_bn_bwd_finalize", part.data_ptr(), T, P, C, c1.data_ptr(), c2.data_ptr(), None, dbias.data_ptr(),
          int(accumulate), native.ptr(_fin_ws(T, C, dy.device)))


def _deepnn_forward(model, x, targets, training):
    plan = _deepnn_plan(model)
    saved = []
    N, H, W, C = x.shape
    for bi, (conv, pool) in enumerate(plan.blocks):
        Co = conv.weight.shape[0]
        P = N * H * W
        # the data-gradient algorithm follows THIS forward's branch (saved below); the plan is never changed, so
        # one forward at another input size (an eval) does not demote later 32x32 steps to the direct dgrad
        wino = plan.uf[bi] is not None and H == W and wino_applies(H, W, C, Co)
        if wino:
            wino_wprep(conv.weight, plan.uf[bi], plan.ud[bi])
            if bi > 0 and plan.ud[bi] is None:  # data gradient on the direct GEMM
                conv_wprep(conv.weight, plan.wf[bi], plan.wd[bi])
            y = wino_conv(x, plan.uf[bi], Co, bias=conv.bias, relu=True)
        else:
            conv_wprep(conv.weight, plan.wf[bi], plan.wd[bi])  # this input size: direct forward and data gradient
            y = torch.empty((P, Co), dtype=torch.float32, device=x.device)
            gemm(IM2COL_KC, x, 0, DENSE_OC, plan.wf[bi], Co, P, Co, 9 * C, y, geom=(C, H, W, 1), bias=conv.bias,
                 relu=True)
        if pool:
            xn = torch.empty((N, H // 2, W // 2, Co), dtype=torch.float32, device=x.device)
            _call("ddpx_f32_bn_apply", y.data_ptr(), plan.ones.data_ptr(), plan.zeros.data_ptr(),
                  plan.zeros.data_ptr(), N, H, W, Co, 1, 1, xn.data_ptr())
        else:
            xn = y.view(N, H, W, Co)
        saved.append((x, y, (N, H, W, C, Co), pool, wino))
        x = xn
        H, W, C = xn.shape[1], xn.shape[2], Co
    feat = nchw_flatten(x)
    l0, l1 = plan.lin0, plan.lin1
    a0 = linear_fwd(feat, l0.weight, l0.bias, relu=True)
    p = float(plan.drop.p)
    drop = training and p > 0.0
    d0 = dropout_(a0, p, plan.rng, plan.rng_done) if drop else a0
    loss, logits, dl = head_forward(d0, l1.weight, l1.bias, targets)
    scale = 1.0 / (1.0 - p) if drop else 1.0
    return saved, (x.shape, feat, d0, scale), loss, logits, dl


def _deepnn_backward(model, saved, last, dl, grad_out):
    plan = _deepnn_plan(model)
    l0, l1 = plan.lin0, plan.lin1
    flat = l0.weight._ddpx_flat
    xshape, feat, d0, scale = last
    dW1, acc = flat.grad_target(l1.weight)
    db1, _ = flat.grad_target(l1.bias)
    # Dropout + ReLU backward folded into the head's dh: mask d0 > 0 (kept and positive), scale 1/(1-p)
    dd0 = head_backward(dl, grad_out, d0, l1.weight, dW1, db1, accumulate=acc, relu_mask=True, dh_scale=scale)
    flat.grad_done(l1.weight)
    flat.grad_done(l1.bias)
    _grad_write(flat, l0.bias, lambda o, ac: colsum(dd0, o, ac))
    _grad_write(flat, l0.weight, lambda o, ac: linear_wgrad(dd0, feat, o, ac))
    g = nchw_unflatten(linear_dgrad(dd0, l0.weight), *xshape)
    g_masked = False  # g already through the block's ReLU (the producing dgrad's epilogue applied the mask)
    for bi in range(len(plan.blocks) - 1, -1, -1):
        conv, pool = plan.blocks[bi]
        x, y, (N, H, W, C, Co), _, wino = saved[bi]
        dy = None

        def bias_grad(o, ac):
            nonlocal dy
            if g_masked:
                dy = g.reshape(N * H * W, Co)
                colsum_bias(dy, N * H * W, Co, plan, o, ac)
            else:
                dy = bias_act_backward(g, y, N, H, W, Co, pool, plan, o, ac)
        _grad_write(flat, conv.bias, bias_grad)
        _grad_write(flat, conv.weight, lambda o, ac: conv_wgrad(dy, x, Co, conv.weight.shape[1], o, ac))
        if bi > 0:
            if wino and plan.ud[bi] is not None:  # made by this step's forward (Winograd data gradient planned)
                below_pool = plan.blocks[bi - 1][1]
                mask = saved[bi - 1][1] if _DGRAD_MASK and not below_pool else None
                g = wino_conv(dy.view(N, H, W, Co), plan.ud[bi], C, mask=mask).view(N, H, W, C)
                g_masked = mask is not None
            else:
                g = conv_dgrad(dy, plan.wd[bi], N, H, W, C, Co)
                g_masked = False


class _DeepNNLossF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, targets, model, *params):
        saved, last, loss, _, dl = _deepnn_forward(model, x, targets, model.training)
        ctx.model, ctx.saved, ctx.last, ctx.dl, ctx.n = model, saved, last, dl, len(params)
        return loss

    @staticmethod
    def backward(ctx, grad_loss):
        _deepnn_backward(ctx.model, ctx.saved, ctx.last, ctx.dl, grad_loss)
        ctx.saved = ctx.last = ctx.dl = None
        return (None, None, None) + (None,) * ctx.n


def deepnn_loss(model, x, targets):
    return _DeepNNLossF32.apply(prep_vgg_input(x), targets, model, *model.parameters())


def deepnn_logits(model, x):
    with torch.no_grad():
        _, _, _, logits, _ = _deepnn_forward(model, prep_vgg_input(x), None, model.training)
    return logits


# ---------------------------------------------------------------------------------------------- MLP
def _mlp_forward(model, x, targets):
    lins = model.linears()
    hs = [x]
    for lin in lins[:-1]:
        hs.append(linear_fwd(hs[-1], lin.weight, lin.bias, relu=True))
    last = lins[-1]
    loss, logits, dl = head_forward(hs[-1], last.weight, last.bias, targets)
    return hs, loss, logits, dl


def _mlp_backward(model, hs, dl, grad_out):
    lins = model.linears()
    flat = lins[0].weight._ddpx_flat
    last = lins[-1]
    dW, acc = flat.grad_target(last.weight)
    db, _ = flat.grad_target(last.bias)
    dz = head_backward(dl, grad_out, hs[-1], last.weight, dW, db, accumulate=acc, relu_mask=True)
    flat.grad_done(last.weight)
    flat.grad_done(last.bias)
    for i in range(len(lins) - 2, -1, -1):
        lin = lins[i]
        sw = flat.fused_spec(lin.weight)
        if sw is not None:
            # single process, SGD(fused_backward): the data gradient reads W_i first, then the weight-gradient
            # GEMM updates W_i in its epilogue (no gradient stored, no separate optimizer pass over W_i)
            dz_next = linear_dgrad(dz, lin.weight, mask=hs[i]) if i > 0 else None
            if linear_wgrad_sgd(dz, hs[i], sw):
                flat.mark_updated(lin.weight)
            else:
                _grad_write(flat, lin.weight, lambda o, ac: linear_wgrad(dz, hs[i], o, ac))
            _grad_write(flat, lin.bias, lambda o, ac: colsum(dz, o, ac))
            if i > 0:
                flat.release(lin.weight)
                dz = dz_next
            continue
        _grad_write(flat, lin.weight, lambda o, ac: linear_wgrad(dz, hs[i], o, ac))
        _grad_write(flat, lin.bias, lambda o, ac: colsum(dz, o, ac))
        if i > 0:
            dz = linear_dgrad(dz, lin.weight, mask=hs[i])
            flat.release(lin.weight)  # last read of W_i in this backward


class _MLPLossF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, targets, model, *params):
        hs, loss, _, dl = _mlp_forward(model, x, targets)
        ctx.model, ctx.hs, ctx.dl, ctx.n = model, hs, dl, len(params)
        return loss

    @staticmethod
    def backward(ctx, grad_loss):
        _mlp_backward(ctx.model, ctx.hs, ctx.dl, grad_loss)
        ctx.hs = ctx.dl = None
        return (None, None, None) + (None,) * ctx.n


def mlp_loss(model, x, targets):
    x = x.reshape(x.shape[0], -1).float().contiguous()
    return _MLPLossF32.apply(x, targets, model, *model.parameters())


def mlp_logits(model, x):
    with torch.no_grad():
        _, _, logits, _ = _mlp_forward(model, x.reshape(x.shape[0], -1).float().contiguous(), None)
    return logits
