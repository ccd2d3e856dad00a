"""VGG-11-style CIFAR-10 network — the model the reference trains.

Architecture and parameter/buffer names are identical to
``/root/reference/singlegpu.py:47-82`` (and its copy ``multigpu.py:36-71``):
``ARCH = [64, 128, 'M', 256, 256, 'M', 512, 512, 'M', 512, 512, 'M']``; each int
adds ``conv{i}`` (3x3, pad 1, no bias) → ``bn{i}`` → ``relu{i}``; each 'M' adds
``pool{j}`` (2x2 max).  ``backbone`` is an ``nn.Sequential`` over an
``OrderedDict`` so ``state_dict`` keys match the reference checkpoint format
byte-for-byte in key / dtype / shape (SURVEY §2.1 "Checkpoint format").

Execution: with fp32 torch ops on CPU (or when native kernels are disabled);
on MI355X the forward/backward of the conv/BN/ReLU/pool blocks run through
``ddpx.ops.conv`` (NHWC bf16 implicit-GEMM on MFMA with fused BN-statistics)
when ``use_native`` is set and the extension provides them.
"""
from __future__ import annotations

from collections import OrderedDict, defaultdict

import torch
from torch import nn


class VGG(nn.Module):
    ARCH = [64, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"]

    def __init__(self, num_classes: int = 10) -> None:
        super().__init__()
        layers = []
        counts = defaultdict(int)

        def add(kind: str, layer: nn.Module) -> None:
            layers.append((f"{kind}{counts[kind]}", layer))
            counts[kind] += 1

        cin = 3
        for x in self.ARCH:
            if x == "M":
                add("pool", nn.MaxPool2d(2))
            else:
                add("conv", nn.Conv2d(cin, x, 3, padding=1, bias=False))
                add("bn", nn.BatchNorm2d(x))
                add("relu", nn.ReLU(True))
                cin = x
        self.backbone = nn.Sequential(OrderedDict(layers))
        self.classifier = nn.Linear(512, num_classes)
        self.use_native = False
        # native precision: "bf16" (NHWC bf16 MFMA kernels, fp32 masters) or "fp32" (the reference's
        # recipe, /root/reference/singlegpu.py:134, on the exact-f32 MFMA kernels of ddpx.ops.f32)
        self.native_dtype = "bf16"

    # ---- ddpx engine protocol -------------------------------------------------
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
        if not (self.use_native and x.is_cuda and not x.requires_grad):
            return False
        if self.native_dtype == "fp32":
            return getattr(self.classifier.weight, "_ddpx_flat", None) is not None
        return getattr(self.classifier.weight, "_ddpx_shadow", None) is not None

    def forward_loss(self, x: torch.Tensor, targets: torch.Tensor):
        """Fused forward + mean cross-entropy on the native path (torch ops otherwise)."""
        if self._native_ok(x):
            if self.native_dtype == "fp32":
                from ..ops import f32
                return f32.vgg_loss(self, x, targets), None
            from ..ops import vgg_native
            return vgg_native.vgg_loss(self, x, targets), None
        logits = self.forward(x)
        return torch.nn.functional.cross_entropy(logits, targets), logits

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self._native_ok(x) and self.native_dtype == "fp32":
            if not torch.is_grad_enabled():  # logits with autograd go through torch ops below
                from ..ops import f32
                return f32.vgg_logits(self, x)
            from ..ops.f32 import prep_vgg_input
            x = prep_vgg_input(x)[..., :3].permute(0, 3, 1, 2)
        elif self._native_ok(x):
            from ..ops import vgg_native
            return vgg_native.vgg_forward(self, x)
        # backbone: [N, 3, 32, 32] => [N, 512, 2, 2]
        x = self.backbone(x)
        # avgpool: [N, 512, 2, 2] => [N, 512]
        x = x.mean([2, 3])
        # classifier: [N, 512] => [N, 10]
        return self.classifier(x)
