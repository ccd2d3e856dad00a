"""Host wrappers for the gfx950 bf16 MFMA GEMM (``csrc/kernels/gemm_pipe.hip`` on ``csrc/include/ddpx_pipe.h``).

Every wrapper validates shapes, dtypes, contiguity and alignment on the host
before launching: the kernel's grid and loaders assume exactly these layouts.
The three Linear products map onto one kernel with per-operand layouts, so no
transpose is ever materialised:

=========  ============================  ===========  ===========
product    math                          A layout     B layout
=========  ============================  ===========  ===========
forward    Y[M,N]  = X[M,K] · W[N,K]ᵀ    K-contig     K-contig
dgrad      dX[M,K] = dY[M,N] · W[N,K]    K-contig     N-contig
wgrad      dW[N,K] = dY[M,N]ᵀ · X[M,K]   M-contig     N-contig
=========  ============================  ===========  ===========
"""
from __future__ import annotations

import os

import torch

from ..runtime import native

# In-launch split-K for the M=512-row products (forward / dgrad): 128x128 tiles, K split over 2-4
# workgroups whose fp32 partials are combined by the last split of each tile inside the same launch
# (``csrc/include/ddpx_pipe.h``).  Planned by the native side; DDPX_SPLITK=0 turns it off there.

EPI_F32 = 0
EPI_BF16 = 1
EPI_BIAS_BF16 = 2
EPI_BIAS_RELU_BF16 = 3
EPI_BIAS_F32 = 4
EPI_RELUMASK_BF16 = 5
EPI_SGD = 6  # fused optimizer: the product is a gradient applied to (master, momentum, shadow) in place

_OUT_DTYPE = {
    EPI_F32: torch.float32,
    EPI_BF16: torch.bfloat16,
    EPI_BIAS_BF16: torch.bfloat16,
    EPI_BIAS_RELU_BF16: torch.bfloat16,
    EPI_BIAS_F32: torch.float32,
    EPI_RELUMASK_BF16: torch.bfloat16,
}


def _req(cond, msg):
    if not cond:
        raise ValueError(msg)


def _check_bf16_2d(t, name):
    _req(t.is_cuda, f"{name} must be a GPU tensor")
    _req(t.dtype == torch.bfloat16, f"{name} must be bf16, got {t.dtype}")
    _req(t.dim() == 2, f"{name} must be 2-D, got shape {tuple(t.shape)}")
    _req(t.stride(1) == 1, f"{name} must be row-contiguous")
    _req(t.stride(0) % 8 == 0, f"{name} leading dimension must be a multiple of 8")
    _req(t.data_ptr() % 16 == 0, f"{name} must be 16-byte aligned")


def plan(M, N, K, a_kcontig, b_kcontig, epi):
    """(splits, cfg, slab_floats, tickets) of the default launch; splits > 1 = in-launch split-K."""
    cfg = native.c_int(0)
    sf = native.c_int64(0)
    nt = native.c_int(0)
    s = native.kernels().ddpx_gemm_pipe_plan(M, N, K, int(a_kcontig), int(b_kcontig), int(epi),
                                             native.ctypes.byref(cfg), native.ctypes.byref(sf), native.ctypes.byref(nt))
    return s, cfg.value, sf.value, nt.value


_TICKETS: dict = {}
_CS_TICKETS: dict = {}
# superseded ticket buffers stay allocated: a HIP graph captured earlier keeps their addresses and its
# replays still take tickets there (freeing them would hand those replays recycled, non-zero memory)
_RETIRED: list = []


def _tickets(dev, n, pool=None):
    """Per-device tile tickets of the in-launch combines (zero between launches: each last arriver resets
    its own).  GEMMs on one device run in stream order, so one buffer per kind serves every launch."""
    pool = _TICKETS if pool is None else pool
    t = pool.get(dev)
    if t is None or t.numel() < n:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("GEMM tickets: first launch of this size must happen outside graph capture")
        if t is not None:
            _RETIRED.append(t)
        t = pool[dev] = torch.zeros((max(n, 4096),), dtype=torch.int32, device=dev)
    return t


def tile_dims(cfg):
    bm, bn = native.c_int(0), native.c_int(0)
    native.kernels().ddpx_gemm_tile_dims(int(cfg), native.ctypes.byref(bm), native.ctypes.byref(bn))
    return bm.value, bn.value


def gemm_raw(a, b, c, *, M, N, K, lda, ldb, ldc, a_kcontig, b_kcontig, epi, bias=None, aux=None, ldaux=0,
             accumulate=False, alpha=1.0, tile=-1, colsum=None, stream=None, sgd=None, splits=None,
             cs_out=None, cs_accumulate=False, cs_sgd=None):
    """``splits`` (with an explicit ``tile``): force the in-launch split-K on that tile config.

    ``colsum`` ([tiles_m, N] fp32 scratch) with ``cs_out`` (fp32 / bf16 [N]) or ``cs_sgd``: the column
    sums of the stored output are finished inside the launch (the last row tile of each column tile adds
    the partials in order) and stored / accumulated into ``cs_out`` or applied as an SGD update."""
    lib = native.kernels()
    s = native.stream_handle(stream)
    slab, sf, tk = None, 0, None
    nt = 0
    if splits is not None and splits > 1:
        _req(tile >= 0 and sgd is None, "forced split-K needs an explicit tile and no fused optimizer")
        bm, bn = tile_dims(tile)
        nt = ((M + bm - 1) // bm) * ((N + bn - 1) // bn)
        sf = splits * nt * bm * bn
    else:
        splits = 1
        if tile < 0 and sgd is None:
            splits, cfg, sf, nt = plan(M, N, K, a_kcontig, b_kcontig, epi)
            if splits > 1:
                tile = cfg
    if splits > 1:
        slab = torch.empty(sf, dtype=torch.float32, device=a.device)
        tk = _tickets(a.device, nt)
    cs_t, cs_flags = None, 0
    if cs_out is not None or cs_sgd is not None:
        _req(colsum is not None and sgd is None, "in-launch column sums need the colsum scratch, no EPI_SGD")
        cs_t = _tickets(a.device, N, pool=_CS_TICKETS)
        cs_flags = int(cs_out is not None and cs_out.dtype == torch.bfloat16) | (2 if cs_accumulate else 0)
        sgd = cs_sgd  # the bias SGD rides on the (otherwise unused) optimizer arguments
    rc = lib.ddpx_gemm_pipe(a.data_ptr(), b.data_ptr(), c.data_ptr(), native.ptr(bias), native.ptr(aux),
                            native.ptr(colsum), M, N, K, lda, ldb, ldc, ldaux, int(a_kcontig), int(b_kcontig), epi,
                            int(accumulate), float(alpha), tile, *native.sgd_args(sgd), splits, native.ptr(slab), sf,
                            native.ptr(tk), native.ptr(cs_out), cs_flags, native.ptr(cs_t), s)
    native.check(rc, f"ddpx_gemm_pipe(M={M},N={N},K={K},epi={epi})")
    return c


def tiles_m(M, N, K, a_kcontig, b_kcontig, tile=-1):
    """Rows of per-tile column-sum partials the kernel chosen for this shape writes."""
    return native.kernels().ddpx_gemm_pipe_tiles_m(M, N, K, int(a_kcontig), int(b_kcontig), tile)


def linear_fwd(x, w, bias=None, relu=False, out=None, out_dtype=torch.bfloat16, tile=-1, splits=None):
    """Y = act(X Wᵀ + b).  X [M,K] bf16, W [N,K] bf16, b [N] fp32."""
    _check_bf16_2d(x, "x")
    _check_bf16_2d(w, "w")
    M, K = x.shape
    N, K2 = w.shape
    _req(K == K2, f"inner dims differ: x {tuple(x.shape)} vs w {tuple(w.shape)}")
    if bias is not None:
        _req(bias.dtype == torch.float32 and bias.numel() == N and bias.is_contiguous(), "bias must be fp32 [N]")
    if out_dtype == torch.bfloat16:
        epi = EPI_BIAS_RELU_BF16 if relu else (EPI_BIAS_BF16 if bias is not None else EPI_BF16)
        _req(not (relu and bias is None), "relu epilogue requires a bias")
    else:
        _req(not relu, "fp32 output epilogue has no relu")
        epi = EPI_BIAS_F32 if bias is not None else EPI_F32
    if out is None:
        out = torch.empty((M, N), dtype=_OUT_DTYPE[epi], device=x.device)
    # out may be a column slice of a wider activation (row-chunked weights): row-contiguous is enough
    _req(tuple(out.shape) == (M, N) and out.stride(1) == 1 and out.stride(0) % 8 == 0
         and out.data_ptr() % 16 == 0 and out.dtype == _OUT_DTYPE[epi], "bad out tensor")
    return gemm_raw(x, w, out, M=M, N=N, K=K, lda=x.stride(0), ldb=w.stride(0), ldc=out.stride(0), a_kcontig=True,
                    b_kcontig=True, epi=epi, bias=bias, tile=tile, splits=splits)


def linear_dgrad(dy, w, relu_mask_of=None, out=None, tile=-1, bias_grad=None, bias_grad_accumulate=False,
                 bias_sgd=None, splits=None):
    """dX = dY W (bf16), optionally times (relu_mask_of > 0) — the ReLU backward of the layer below.

    ``bias_grad`` ([K] fp32 or bf16): also produce Σ_m dX[m, :] — the bias gradient of the layer that
    produced ``relu_mask_of`` — from per-tile column sums in the GEMM epilogue, summed in row-tile order
    by the last row tile of each column tile in the same launch (``bias_sgd``: applied as an SGD update).
    """
    _check_bf16_2d(dy, "dy")
    _check_bf16_2d(w, "w")
    M, N = dy.shape
    N2, K = w.shape
    _req(N == N2, f"dy {tuple(dy.shape)} incompatible with w {tuple(w.shape)}")
    epi = EPI_BF16
    if relu_mask_of is not None:
        _check_bf16_2d(relu_mask_of, "relu_mask_of")
        _req(tuple(relu_mask_of.shape) == (M, K), "mask shape must equal dX shape")
        epi = EPI_RELUMASK_BF16
    if out is None:
        out = torch.empty((M, K), dtype=torch.bfloat16, device=dy.device)
    _req(out.shape == (M, K) and out.is_contiguous() and out.dtype == torch.bfloat16, "bad out tensor")
    part = None
    if bias_grad is not None or bias_sgd is not None:
        _req(bias_grad is None or (bias_grad.numel() == K and bias_grad.is_contiguous()),
             "bias_grad must be contiguous [K]")
        _req(bias_sgd is None or bias_sgd[0].numel() == K, "bias_sgd target must have K elements")
        T = tiles_m(M, K, N, True, False, tile)
        part = torch.empty((T, K), dtype=torch.float32, device=dy.device)
    # the in-launch column-sum finish is built for the 4-wave tiles; an explicitly chosen 8-wave tile
    # (tests / probes) leaves the partials to a torch reduction
    in_launch = tile not in _EIGHT_WAVE_TILES
    _req(in_launch or bias_sgd is None, "fused bias SGD needs a 4-wave dgrad tile")
    gemm_raw(dy, w, out, M=M, N=K, K=N, lda=dy.stride(0), ldb=w.stride(0), ldc=K, a_kcontig=True,
             b_kcontig=False, epi=epi, aux=relu_mask_of,
             ldaux=(relu_mask_of.stride(0) if relu_mask_of is not None else 0), tile=tile, colsum=part,
             splits=splits,
             cs_out=bias_grad if in_launch else None, cs_accumulate=bias_grad_accumulate,
             cs_sgd=bias_sgd if in_launch else None)
    if part is not None and not in_launch and bias_grad is not None:
        s = part.sum(0).to(bias_grad.dtype)
        bias_grad.add_(s) if bias_grad_accumulate else bias_grad.copy_(s)
    return out


_EIGHT_WAVE_TILES = (8, 13, 14, 15, 22, 25)  # ddpx_pipe.h eight_wave()


def linear_wgrad(dy, x, out, accumulate=False, tile=-1, sgd=None):
    """dW[N,K] (=|+=) dYᵀ X in fp32/bf16 (written straight into the gradient bucket).

    ``sgd=(master, momentum, shadow, lr, mom, wd)``: fused optimizer — the [N,K] product is applied as
    the gradient of that parameter (SGD in the epilogue); ``out`` is ignored and may be None.
    """
    if sgd is not None:
        _check_bf16_2d(dy, "dy")
        _check_bf16_2d(x, "x")
        M, N = dy.shape
        _, K = x.shape
        _req(sgd[0].numel() == N * K, "sgd target size mismatch")
        return gemm_raw(dy, x, sgd[0], M=N, N=K, K=M, lda=dy.stride(0), ldb=x.stride(0), ldc=K, a_kcontig=False,
                        b_kcontig=False, epi=EPI_SGD, tile=tile, sgd=sgd)
    _check_bf16_2d(dy, "dy")
    _check_bf16_2d(x, "x")
    M, N = dy.shape
    M2, K = x.shape
    _req(M == M2, f"batch dims differ: dy {tuple(dy.shape)} vs x {tuple(x.shape)}")
    _req(out.dtype in (torch.float32, torch.bfloat16), "dW must be fp32 or bf16")
    _req(tuple(out.shape) == (N, K) and out.is_contiguous(), f"dW must be contiguous [{N},{K}]")
    epi = EPI_F32 if out.dtype == torch.float32 else EPI_BF16
    return gemm_raw(dy, x, out, M=N, N=K, K=M, lda=dy.stride(0), ldb=x.stride(0), ldc=K, a_kcontig=False,
                    b_kcontig=False, epi=epi, accumulate=accumulate, tile=tile)


def matmul(a, b, a_kcontig=True, b_kcontig=True, out_dtype=torch.float32, tile=-1):
    """General C = A·B for tests: A given as [M,K] (K-contig) or [K,M]; B as [N,K] or [K,N]."""
    _check_bf16_2d(a, "a")
    _check_bf16_2d(b, "b")
    M, K = a.shape if a_kcontig else (a.shape[1], a.shape[0])
    N, K2 = b.shape if b_kcontig else (b.shape[1], b.shape[0])
    _req(K == K2, "inner dims differ")
    epi = EPI_F32 if out_dtype == torch.float32 else EPI_BF16
    out = torch.empty((M, N), dtype=out_dtype, device=a.device)
    return gemm_raw(a, b, out, M=M, N=N, K=K, lda=a.stride(0), ldb=b.stride(0), ldc=N, a_kcontig=a_kcontig,
                    b_kcontig=b_kcontig, epi=epi, tile=tile)


native.register_kernel_sig("ddpx_wgrad_sgd_pair", native.c_int, *([native.c_void_p, native.c_void_p] + [native.c_int] * 5
                                                                  + [native.c_void_p] * 5) * 2,
                           native.c_int, native.c_void_p, native.c_float, native.c_float, native.c_void_p)


native.register_kernel_sig("ddpx_wgrad_sgd_pair_t", native.c_int, *([native.c_void_p, native.c_void_p] + [native.c_int] * 5
                                                                    + [native.c_void_p] * 7) * 2,
                           native.c_int, native.c_void_p, native.c_float, native.c_float, native.c_void_p)


native.register_kernel_sig("ddpx_wsgd_set_xwg_scratch", None, native.c_void_p, native.c_void_p, native.c_int)
_XWG = {}
# DDPX_WSGD_XWG=1: the two-workgroup pair (measurement variant, measured slower: profiles/r6_pair/NOTES.md)
_XWG_ON = os.environ.get("DDPX_WSGD_XWG", "0") == "1"


def _xwg_scratch(dev):
    """Persistent scratch of the two-workgroup pair (csrc/include/ddpx_wgrad_sgd_xwg.h), made once per device and
    handed to the library: gradient tile slots [CUs][2][64x128] fp32 + counters [2 CUs + 1] int32 (zero; every
    launch leaves them zero; the last word counts poll timeouts)."""
    if dev.index in _XWG:
        return _XWG[dev.index]
    cap = torch.cuda.get_device_properties(dev).multi_processor_count
    T = torch.empty(cap * 2 * 64 * 128, dtype=torch.float32, device=dev)
    cnt = torch.zeros(2 * cap + 1, dtype=torch.int32, device=dev)
    native.kernels().ddpx_wsgd_set_xwg_scratch(T.data_ptr(), cnt.data_ptr(), cap)
    _XWG[dev.index] = (T, cnt, cap)
    return _XWG[dev.index]


def xwg_poll_timeouts(dev) -> int:
    """Poll timeouts of the two-workgroup pair on ``dev`` since its scratch was made (0 = every hand-off healthy)."""
    if dev.index not in _XWG:
        return 0
    _, cnt, cap = _XWG[dev.index]
    return int(cnt[2 * cap].item())


def wgrad_sgd_pair(dy0, x0, sgd0, dy1, x1, sgd1, mx0=None, mx1=None, mxt0=None, mxt1=None) -> bool:
    """Both fused weight-gradient + SGD updates (dW_i = dy_iᵀ x_i applied to sgd_i's parameter) in ONE
    warp-specialised launch.  False (nothing launched) when the pair is not eligible; the caller then
    issues them one by one with :func:`linear_wgrad`.  ``mx_i`` = (codes uint8 [M_i, N_i], E8M0 scales uint8
    [M_i, N_i / 32]): the stream waves also write the updated W_i as MX-FP8 e4m3 (the next forward's
    operand, ``ddpx.ops.fp8``), bitwise what ``fp8.quant`` of the bf16 copy would give.  ``mxt_i`` (with
    both ``mx``; either may be None) = (codes uint8 [N_i, M_i], scales uint8 [N_i, M_i / 32]): W_iᵀ with
    blocks along M_i too (the data gradient's operand), bitwise ``fp8.quant(bf16 copy, rows=False, cols=True)``."""
    for t, n in ((dy0, "dy0"), (x0, "x0"), (dy1, "dy1"), (x1, "x1")):
        _check_bf16_2d(t, n)
    if dy0.shape[0] != dy1.shape[0] or x0.shape[0] != dy0.shape[0] or x1.shape[0] != dy1.shape[0]:
        return False
    if sgd0[3] is not sgd1[3] or sgd0[4] != sgd1[4] or sgd0[5] != sgd1[5]:
        return False  # lr tensor, momentum, weight decay must be shared
    K = dy0.shape[0]
    transposed = mxt0 is not None or mxt1 is not None
    if transposed and (mx0 is None or mx1 is None):
        return False
    args = []
    for dy, x, sg, mx, mxt in ((dy0, x0, sgd0, mx0, mxt0), (dy1, x1, sgd1, mx1, mxt1)):
        M, N = dy.shape[1], x.shape[1]
        _req(sg[0].numel() == M * N, "sgd target size mismatch")
        if mx is not None:
            _req(mx[0].dtype == torch.uint8 and mx[0].numel() == M * N and mx[0].is_contiguous()
                 and mx[1].dtype == torch.uint8 and mx[1].numel() == M * N // 32 and N % 32 == 0,
                 "fp8 copy must be uint8 [M, N] codes + [M, N/32] scales")
        if mxt is not None:
            _req(mxt[0].dtype == torch.uint8 and tuple(mxt[0].shape) == (N, M) and mxt[0].is_contiguous()
                 and mxt[1].dtype == torch.uint8 and tuple(mxt[1].shape) == (N, M // 32) and mxt[1].is_contiguous()
                 and M % 64 == 0, "transposed fp8 copy must be uint8 [N, M] codes + [N, M/32] scales, M % 64 == 0")
        args += [dy.data_ptr(), x.data_ptr(), M, N, dy.stride(0), x.stride(0), N, sg[0].data_ptr(),
                 native.ptr(sg[1]), native.ptr(sg[2]), native.ptr(mx[0] if mx else None),
                 native.ptr(mx[1] if mx else None)]
        if transposed:
            args += [native.ptr(mxt[0] if mxt else None), native.ptr(mxt[1] if mxt else None)]
    lr = sg[3]
    if _XWG_ON:
        _xwg_scratch(dy0.device)
    fn = native.kernels().ddpx_wgrad_sgd_pair_t if transposed else native.kernels().ddpx_wgrad_sgd_pair
    rc = fn(*args, K, lr.data_ptr(), float(sgd0[4]), float(sgd0[5]), native.stream_handle())
    if rc == -20:
        return False
    native.check(rc, "ddpx_wgrad_sgd_pair")
    return True


native.register_kernel_sig("ddpx_wgrad_sgd_dgrad", native.c_int,
                           *([native.c_void_p] * 2 + [native.c_int] * 4 + [native.c_void_p] * 5   # fc1 wgrad + SGD
                             + [native.c_void_p, native.c_int]                                  # W1 (read copy)
                             + [native.c_void_p, native.c_void_p, native.c_int]                 # dX, mask
                             + [native.c_void_p, native.c_int, native.c_int] + [native.c_void_p] * 5  # fc0
                             + [native.c_void_p] * 3                                            # bias SGD
                             + [native.c_void_p, native.c_void_p, native.c_int, native.c_void_p,  # scratch, K, lr
                                native.c_float, native.c_float, native.c_void_p]))
native.register_kernel_sig("ddpx_wgrad_sgd_dgrad_words", native.c_int, native.c_int)

_DG_SCRATCH: dict = {}


def _dg_scratch(dev, rows, n):
    """(colsum [rows, n] fp32, words int32) of the fused data-gradient launch, one pair per device and shape.
    Kept for the process lifetime: captured graphs hold their addresses (the words are re-zeroed by every
    launch's memset node)."""
    key = (dev, rows, n)
    t = _DG_SCRATCH.get(key)
    if t is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("fused data-gradient scratch: first launch of this shape must happen outside capture")
        nw = native.kernels().ddpx_wgrad_sgd_dgrad_words(n)
        t = _DG_SCRATCH[key] = (torch.empty((rows, n), dtype=torch.float32, device=dev),
                                torch.zeros((nw,), dtype=torch.int32, device=dev))
    return t


_CUS: dict = {}


def wgrad_sgd_dgrad_eligible(K, M1, N1, N0, dev) -> bool:
    """Shape check of :func:`wgrad_sgd_dgrad` (mirrors wsgdd::eligible): batch K = 512, 64 x 128 tiles, and
    the fc1 weight-gradient and data-gradient tiles divide evenly over the CUs."""
    if K != 512 or M1 % 64 or N1 % 128 or N0 % 128:
        return False
    cus = _CUS.get(dev)
    if cus is None:
        cus = _CUS[dev] = torch.cuda.get_device_properties(dev).multi_processor_count
    nt1, nd = (M1 // 64) * (N1 // 128), (K // 64) * (N1 // 128)
    return nt1 % cus == 0 and nd % cus == 0 and (nt1 // cus) * (K // 64) == (nd // cus) * (M1 // 64)


def wgrad_sgd_dgrad(dy1, x1, sgd1, w1, relu_mask_of, x0, sgd0, bias_sgd, mx1=None, mx0=None, out=None):
    """fc1's data gradient folded into the fc1 + fc0 weight-gradient + SGD launch (ddpx_wsgd_dgrad.h):

        dX = (dy1 @ w1) * (relu_mask_of > 0)     [batch, in1]    (bias_sgd: SGD of the layer below's bias by
                                                                   the column sums of dX)
        W1 -= sgd(dy1^T x1)  -> sgd1, whose bf16 copy target must NOT alias ``w1`` (the copy read here)
        W0 -= sgd(dX^T x0)   -> sgd0

    Returns dX, or None when the shapes are not eligible (nothing launched)."""
    for t, n in ((dy1, "dy1"), (x1, "x1"), (w1, "w1"), (relu_mask_of, "relu_mask_of"), (x0, "x0")):
        _check_bf16_2d(t, n)
    K, M1 = dy1.shape
    K2, N1 = x1.shape
    K3, N0 = x0.shape
    if K != K2 or K != K3 or tuple(w1.shape) != (M1, N1) or tuple(relu_mask_of.shape) != (K, N1):
        return None
    if sgd1[3] is not sgd0[3] or sgd1[3] is not bias_sgd[3] or sgd1[4] != sgd0[4] or sgd1[5] != sgd0[5]:
        return None
    if sgd1[2] is None or sgd1[2].data_ptr() == w1.data_ptr():
        return None  # the weight's new bf16 copy must go to the other ping-pong buffer
    _req(sgd1[0].numel() == M1 * N1 and sgd0[0].numel() == N1 * N0 and bias_sgd[0].numel() == N1,
         "sgd target size mismatch")
    if (mx1 is None) != (mx0 is None):
        mx1 = mx0 = None
    colsum, words = _dg_scratch(dy1.device, K // 64, N1)
    if out is None:
        out = torch.empty((K, N1), dtype=torch.bfloat16, device=dy1.device)
    lr = sgd1[3]
    args = [dy1.data_ptr(), x1.data_ptr(), M1, N1, dy1.stride(0), x1.stride(0), sgd1[0].data_ptr(), native.ptr(sgd1[1]),
            native.ptr(sgd1[2]), native.ptr(mx1[0] if mx1 else None), native.ptr(mx1[1] if mx1 else None),
            w1.data_ptr(), w1.stride(0), out.data_ptr(), relu_mask_of.data_ptr(), relu_mask_of.stride(0),
            x0.data_ptr(), N0, x0.stride(0), sgd0[0].data_ptr(), native.ptr(sgd0[1]), native.ptr(sgd0[2]),
            native.ptr(mx0[0] if mx0 else None), native.ptr(mx0[1] if mx0 else None),
            bias_sgd[0].data_ptr(), native.ptr(bias_sgd[1]), native.ptr(bias_sgd[2]),
            colsum.data_ptr(), words.data_ptr(), K, lr.data_ptr(), float(sgd1[4]), float(sgd1[5]),
            native.stream_handle()]
    rc = native.kernels().ddpx_wgrad_sgd_dgrad(*args)
    if rc == -20:
        return None
    native.check(rc, "ddpx_wgrad_sgd_dgrad")
    return out


def wgrad_sgd_dgrad_state(dev, n1):
    """(tiles published, spin give-up flag) of the last fused data-gradient launch on ``dev`` for fc1 width
    ``n1`` (words = [n1 / 128 column tickets][done][err]); synchronises."""
    for (d, _, n), (_, words) in _DG_SCRATCH.items():
        if d == dev and n == n1:
            nb = n1 // 128
            w = words.cpu()
            return int(w[nb]), int(w[nb + 1])
    return None
