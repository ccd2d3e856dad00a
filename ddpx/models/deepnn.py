"""DeepNN — the smaller CNN defined (but never instantiated) by the reference.

Same layers, order and ``state_dict`` keys as ``/root/reference/singlegpu.py:18-44``:
``features`` = Conv(3→128)-ReLU-Conv(128→64)-ReLU-MaxPool2 → Conv(64→64)-ReLU-
Conv(64→32)-ReLU-MaxPool2; ``classifier`` = Linear(2048→512)-ReLU-Dropout(0.1)-
Linear(512→num_classes).  1,186,986 parameters.

Execution: torch ops on CPU (or with ``use_native`` off); on MI355X with ``use_native`` the whole
network runs through ``ddpx.ops.deepnn_native`` (NHWC bf16 implicit-GEMM convolutions with fused
bias+ReLU+pool passes, MFMA Linear, Philox dropout, fused classifier + cross-entropy).
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

    # ---- ddpx engine protocol (same as VGG) -------------------------------------
    def native_active(self, device) -> bool:
        return torch.device(device).type == "cuda" and self.use_native

    def ddpx_spec(self, device):
        if self.native_active(device):
            from ..runtime import native
            native.kernels()  # fail loudly if the extension is missing on a GPU
            return {"shadow_dtype": torch.bfloat16, "native_params": list(self.parameters())}
        return {}

    def input_layout(self, device) -> str:
        return "nhwc8_bf16" if self.native_active(device) else "nchw_f32"

    def _native_ok(self, x):
        lin = self.classifier[0]
        return (self.use_native and x.is_cuda and not x.requires_grad
                and getattr(lin.weight, "_ddpx_shadow", None) is not None)

    def forward_loss(self, x: torch.Tensor, targets: torch.Tensor):
        if self._native_ok(x):
            from ..ops import deepnn_native
            return deepnn_native.deepnn_loss(self, x, targets), None
        logits = self.forward(x)
        return torch.nn.functional.cross_entropy(logits, targets), logits

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self._native_ok(x):
            from ..ops import deepnn_native
            return deepnn_native.deepnn_forward(self, x)
        x = self.features(x)
        x = torch.flatten(x, 1)
        return self.classifier(x)
