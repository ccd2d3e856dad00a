"""Model zoo: the reference's VGG and DeepNN, and the BASELINE MLPs."""
from __future__ import annotations

import torch

from .deepnn import DeepNN
from .mlp import MLP
from .vgg import VGG

__all__ = ["VGG", "DeepNN", "MLP", "build_model", "native_kernels_for"]


def native_kernels_for(name: str, dtype: str, kernels: str = "auto") -> bool:
    """Whether ``build_model`` puts ``name`` on the hand-written kernels for ``kernels`` = auto|native|torch.

    auto = native everywhere (measured faster than the stock libraries on every model and precision, including the
    reference's fp32 recipe: VGG 18.79 vs MIOpen 19.46 ms, DeepNN 3.83 vs 4.29 ms per step, profiles/r4_f32);
    ``--kernels torch`` runs the torch/MIOpen ops under the ddpx engine (flat store, fused flat SGD, native DDP)."""
    if kernels == "torch":
        return False
    if kernels == "native":
        return True
    # measured (profiles/r4_f32): at fp32 the native kernels beat MIOpen on both CNNs (VGG 18.79 vs 19.46 ms,
    # DeepNN 3.83 vs 4.29 ms per step, same boxes), so auto is native everywhere
    return True


def build_model(name: str, hidden=None, layers: int = 3, dtype: str = "auto", device=None, kernels: str = "auto",
                fp8: bool = False):
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dtype == "auto":
        dtype = "bf16" if dev.type == "cuda" else "fp32"
    cdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    native = native_kernels_for(name, dtype, kernels)
    if name == "vgg":
        m = VGG()
        # native NHWC kernels on the GPU: bf16 MFMA, or the exact-f32 MFMA path for the reference's fp32
        m.use_native = native and dev.type == "cuda"
        m.native_dtype = "fp32" if dtype == "fp32" else "bf16"
    elif name == "deepnn":
        m = DeepNN()
        m.use_native = native and dev.type == "cuda"
        m.native_dtype = "fp32" if dtype == "fp32" else "bf16"
    elif name in ("mlp", "mlp_wide"):
        h = hidden or (16384 if name == "mlp_wide" else 4096)
        m = MLP(hidden=h, layers=layers, compute_dtype=cdt)
        m.use_native = native
        m.fp8 = bool(fp8)  # MX-FP8 forward / weight-gradient GEMMs on the native path
    else:
        raise ValueError(f"unknown model {name!r}")
    return m
