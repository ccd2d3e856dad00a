"""MX-FP8 (OCP e4m3 / e5m2, E8M0 block-32 scales) quantisation and GEMM on gfx950.

``csrc/kernels/gemm_mx8.hip``.  Used by the wide MLP's fp8 path (BASELINE.json config 5,
SURVEY §7.2 4(g)); fp32 master weights and the SGD update are unchanged.

An MX tensor is ``(q, s)``: ``q`` uint8 [R, C] holding fp8 codes, ``s`` uint8 [R, C/32] holding
E8M0 exponents (value = 2^(s-127)) of each run of 32 consecutive elements of a row.  All GEMM
operands are K-contiguous: ``C = A · Bᵀ`` with A [M, K] and B [N, K].
"""
from __future__ import annotations

import torch

from ..runtime import native
from .gemm import EPI_BF16, EPI_BIAS_BF16, EPI_BIAS_RELU_BF16, EPI_F32, EPI_RELUMASK_BF16, EPI_SGD, _OUT_DTYPE, _req

E4M3 = 0
E5M2 = 1
_TORCH_FP8 = {E4M3: torch.float8_e4m3fn, E5M2: torch.float8_e5m2}
_MAXV = {E4M3: 448.0, E5M2: 57344.0}


class MX:
    """An MX-fp8 operand: codes [R, C] uint8 + E8M0 scales [R, C/32] uint8 + format."""

    __slots__ = ("q", "s", "fmt")

    def __init__(self, q, s, fmt):
        self.q, self.s, self.fmt = q, s, fmt

    @property
    def shape(self):
        return tuple(self.q.shape)

    def dequant(self) -> torch.Tensor:
        """fp32 values (for tests / references)."""
        v = self.q.view(_TORCH_FP8[self.fmt]).float()
        e = self.s.float() - 127.0
        return v * torch.exp2(e).repeat_interleave(32, dim=1)


def quant(x: torch.Tensor, fmt: int = E4M3, rows: bool = True, cols: bool = False, out=None, out_t=None):
    """MX-quantise bf16 ``x`` [R, C]: row blocks (for x as a K-contig operand, K = C) and/or the
    transposed operand xᵀ [C, R] with blocks along R.  Returns MX, or (MX, MX_T) if both.
    ``out`` = (codes uint8 [R, C], scales uint8 [R, C / 32]) contiguous: write the row quantisation there;
    ``out_t`` = (codes uint8 [C, R], scales uint8 [C, R / 32]): the transposed one."""
    _req(x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2 and x.stride(1) == 1, "x must be 2-D bf16 (GPU)")
    R, C = x.shape
    _req(x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0, "x must be 16-B aligned with ld % 8 == 0")
    q = s = qt = st = None
    if rows:
        _req(C % 32 == 0, "row quantisation needs C % 32 == 0")
        if out is not None:
            q, s = out
            _req(q.dtype == torch.uint8 and q.shape == (R, C) and q.is_contiguous() and s.dtype == torch.uint8
                 and s.shape == (R, C // 32) and s.is_contiguous(), "quant out: uint8 [R, C] + [R, C/32]")
        else:
            q = torch.empty((R, C), dtype=torch.uint8, device=x.device)
            s = torch.empty((R, C // 32), dtype=torch.uint8, device=x.device)
    if cols:
        _req(R % 32 == 0 and R % 16 == 0, "transposed quantisation needs R % 32 == 0")
        if out_t is not None:
            qt, st = out_t
            _req(qt.dtype == torch.uint8 and qt.shape == (C, R) and qt.is_contiguous() and st.dtype == torch.uint8
                 and st.shape == (C, R // 32) and st.is_contiguous(), "quant out_t: uint8 [C, R] + [C, R/32]")
        else:
            qt = torch.empty((C, R), dtype=torch.uint8, device=x.device)
            st = torch.empty((C, R // 32), dtype=torch.uint8, device=x.device)
    rc = native.kernels().ddpx_mx8_quant(x.data_ptr(), R, C, x.stride(0), native.ptr(q), C, native.ptr(s),
                                         native.ptr(qt), R, native.ptr(st), int(fmt == E5M2), native.stream_handle())
    native.check(rc, f"ddpx_mx8_quant(R={R},C={C})")
    a = MX(q, s, fmt) if rows else None
    b = MX(qt, st, fmt) if cols else None
    if rows and cols:
        return a, b
    return a if rows else b


def quant_reference(x: torch.Tensor, fmt: int = E4M3) -> MX:
    """Host (torch) reference of the row quantiser: same exponent rule, torch's fp8 rounding."""
    xf = x.float()
    R, C = xf.shape
    blocks = xf.view(R, C // 32, 32)
    amax = blocks.abs().amax(dim=2)
    m, ex = torch.frexp(amax / _MAXV[fmt])
    ex = torch.where(amax > 0, ex, torch.full_like(ex, -127)).clamp(-127, 127)
    scaled = (blocks * torch.exp2(-ex.float()).unsqueeze(2)).clamp(-_MAXV[fmt], _MAXV[fmt])
    q = scaled.reshape(R, C).to(_TORCH_FP8[fmt]).view(torch.uint8)
    return MX(q, (ex + 127).to(torch.uint8), fmt)


def gemm(a: MX, b: MX, out: torch.Tensor | None = None, epi: int = EPI_BF16, bias=None, aux=None,
         accumulate: bool = False, sgd=None, out_dtype=None):
    """``epi(A · Bᵀ)`` with A [M, K] (e4m3 or e5m2) and B [N, K] (e4m3) MX operands."""
    _req(b.fmt == E4M3, "B operand must be e4m3")
    M, K = a.shape
    N, K2 = b.shape
    _req(K == K2, f"inner dims differ: {a.shape} vs {b.shape}")
    _req(K % 128 == 0, "MX-fp8 GEMM needs K % 128 == 0")
    for t in (a.q, b.q):
        _req(t.is_contiguous() and t.data_ptr() % 16 == 0, "fp8 operands must be contiguous, 16-B aligned")
    if bias is not None:
        _req(bias.dtype == torch.float32 and bias.numel() == N, "bias must be fp32 [N]")
    if epi == EPI_SGD:
        _req(sgd is not None and sgd[0].numel() == M * N, "sgd target size mismatch")
        out_t = sgd[0]
        ldc = N
    else:
        if out is None:
            out = torch.empty((M, N), dtype=out_dtype or _OUT_DTYPE[epi], device=a.q.device)
        _req(out.shape == (M, N) and out.is_contiguous() and out.dtype == _OUT_DTYPE[epi], "bad out tensor")
        out_t = out
        ldc = N
    ldaux = aux.stride(0) if aux is not None else 0
    rc = native.kernels().ddpx_gemm_mx8(a.q.data_ptr(), a.s.data_ptr(), b.q.data_ptr(), b.s.data_ptr(),
                                        out_t.data_ptr(), native.ptr(bias), native.ptr(aux), M, N, K, a.q.stride(0),
                                        b.q.stride(0), ldc, ldaux, int(a.fmt == E5M2), epi, int(accumulate), 1.0,
                                        *native.sgd_args(sgd), native.stream_handle())
    native.check(rc, f"ddpx_gemm_mx8(M={M},N={N},K={K},epi={epi})")
    return out


def probe(A8, B8, sa, sb, fa=E4M3):
    """Single-MFMA probe (tests): A8/B8 uint8 [16,128], sa/sb uint8 [16,4] -> fp32 [16,16]."""
    C = torch.empty((16, 16), dtype=torch.float32, device=A8.device)
    rc = native.kernels().ddpx_mx8_probe(A8.data_ptr(), B8.data_ptr(), sa.data_ptr(), sb.data_ptr(), C.data_ptr(),
                                         fa, 0, native.stream_handle())
    native.check(rc, "ddpx_mx8_probe")
    return C


__all__ = ["MX", "E4M3", "E5M2", "quant", "quant_reference", "gemm", "probe", "EPI_F32", "EPI_BF16",
           "EPI_BIAS_BF16", "EPI_BIAS_RELU_BF16", "EPI_RELUMASK_BF16", "EPI_SGD"]
