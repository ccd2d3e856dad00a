"""DeepNN — the smaller CNN defined (but never instantiated) by the reference.

Same layers, order and ``state_dict`` keys as ``/root/reference/singlegpu.py:18-44``:
``features`` = Conv(3→128)-ReLU-Conv(128→64)-ReLU-MaxPool2 → Conv(64→64)-ReLU-
Conv(64→32)-ReLU-MaxPool2; ``classifier`` = Linear(2048→512)-ReLU-Dropout(0.1)-
Linear(512→num_classes).  1,186,986 parameters.

Execution: torch ops on CPU (or with ``use_native`` off); on MI355X with ``use_native`` the whole
network runs through ``ddpx.ops.deepnn_native`` (NHWC bf16 implicit-GEMM convolutions with fused
bias+ReLU+pool passes, MFMA Linear, Philox dropout, fused classifier + cross-entropy), or at fp32
(``native_dtype = "fp32"``, the reference's precision) through ``ddpx.ops.f32`` (exact-f32 MFMA kernels).
"""
from __future__ import annotations

import torch
from torch import nn


class DeepNN(nn.Module):
    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, 128, kernel_size=3, padding=1),
            nn.ReLU(),
            nn.Conv2d(128, 64, kernel_size=3, padding=1),
            nn.ReLU(),
            nn.MaxPool2d(kernel_size=2, stride=2),
            nn.Conv2d(64, 64, kernel_size=3, padding=1),
            nn.ReLU(),
            nn.Conv2d(64, 32, kernel_size=3, padding=1),
            nn.ReLU(),
            nn.MaxPool2d(kernel_size=2, stride=2),
        )
        self.classifier = nn.Sequential(
            nn.Linear(2048, 512),
            nn.ReLU(),
            nn.Dropout(0.1),
            nn.Linear(512, num_classes),
        )
        self.use_native = False
        # native precision: "bf16" (NHWC bf16 MFMA kernels, fp32 masters) or "fp32" (the reference's default
        # precision, on the exact-f32 MFMA kernels of ddpx.ops.f32)
        self.native_dtype = "bf16"

    # ---- ddpx engine protocol (same as VGG) -------------------------------------
    def native_active(self, device) -> bool:
        return torch.device(device).type == "cuda" and self.use_native

    def ddpx_spec(self, device):
        if self.native_active(device):
            from ..runtime import native
            native.kernels()  # fail loudly if the extension is missing on a GPU
            if self.native_dtype == "fp32":
                return {"native_params": list(self.parameters())}
            return {"shadow_dtype": torch.bfloat16, "native_params": list(self.parameters())}
        return {}

    def input_layout(self, device) -> str:
        if not self.native_active(device):
            return "nchw_f32"
        return "nhwc4_f32" if self.native_dtype == "fp32" else "nhwc8_bf16"

    def _native_ok(self, x):
        lin = self.classifier[0]
        if not (self.use_native and x.is_cuda and not x.requires_grad):
            return False
        if self.native_dtype == "fp32":
            return getattr(lin.weight, "_ddpx_flat", None) is not None
        return getattr(lin.weight, "_ddpx_shadow", None) is not None

    def forward_loss(self, x: torch.Tensor, targets: torch.Tensor):
        if self._native_ok(x):
            if self.native_dtype == "fp32":
                from ..ops import f32
                return f32.deepnn_loss(self, x, targets), None
            from ..ops import deepnn_native
            return deepnn_native.deepnn_loss(self, x, targets), None
        logits = self.forward(x)
        return torch.nn.functional.cross_entropy(logits, targets), logits

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self._native_ok(x) and self.native_dtype == "fp32":
            if not torch.is_grad_enabled():  # logits with autograd go through torch ops below
                from ..ops import f32
                return f32.deepnn_logits(self, x)
            from ..ops.f32 import prep_vgg_input
            x = prep_vgg_input(x)[..., :3].permute(0, 3, 1, 2)
        elif self._native_ok(x):
            from ..ops import deepnn_native
            return deepnn_native.deepnn_forward(self, x)
        x = self.features(x)
        x = torch.flatten(x, 1)
        return self.classifier(x)
