"""Toy / wide MLP — the workload BASELINE.json's headline benchmark names.

The reference defines no MLP; SURVEY §7.3 fixes the design: inputs are the
CIFAR-shaped images flattened to 3072 features, then ``layers-1`` hidden
``Linear → ReLU`` blocks and a ``Linear(hidden → 10)`` classifier:

    toy  : 3072 → 4096 → 4096 → 10     (29.4 M params)
    wide : 3072 → 16384 → 16384 → 10   (318.9 M params)

Parameters are plain ``nn.Linear`` modules named ``fc{i}`` so a checkpoint loads
into a vanilla torch MLP with the same names.

On MI355X the whole network runs as ONE autograd node (``ddpx.ops.mlp``): bf16
MFMA GEMMs with bias+ReLU fused in the epilogue, the classifier fused with
softmax-cross-entropy, and a backward that writes fp32 weight gradients
straight into the DDP bucket storage in grad-ready order.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn


class MLP(nn.Module):
    def __init__(self, in_features: int = 3072, hidden: int = 4096, layers: int = 3, num_classes: int = 10,
                 compute_dtype: torch.dtype = torch.bfloat16):
        super().__init__()
        if layers < 2:
            raise ValueError("MLP needs at least 2 layers (1 hidden + classifier)")
        dims = [in_features] + [hidden] * (layers - 1) + [num_classes]
        for i in range(layers):
            lin = nn.Linear(dims[i], dims[i + 1])
            self.add_module(f"fc{i}", lin)
        self.in_features = in_features
        self.hidden = hidden
        self.num_layers = layers
        self.num_classes = num_classes
        self.compute_dtype = compute_dtype
        self.use_native = True
        self.fp8 = False  # MX-FP8 hidden-layer GEMMs (ddpx.ops.mlp), wide-MLP config

    def linears(self):
        return [getattr(self, f"fc{i}") for i in range(self.num_layers)]

    def _native_f32_ok(self, x):
        """The reference's fp32 precision on the exact-f32 MFMA kernels (``ddpx.ops.f32``)."""
        return (self.use_native and x.is_cuda and self.compute_dtype == torch.float32 and not x.requires_grad
                and getattr(self.fc0.weight, "_ddpx_flat", None) is not None)

    def _native_ok(self, x):
        if not (self.use_native and x.is_cuda and self.compute_dtype == torch.bfloat16):
            return False
        fc0 = self.fc0
        return getattr(fc0.weight, "_ddpx_shadow", None) is not None and not x.requires_grad

    def _cpu_fused_ok(self, x):
        """CPU training step on a FlatParams store: one autograd node writing the flat gradients (ops/mlp_cpu)."""
        if not self.use_native or x.is_cuda:
            return False
        from ..ops import mlp_cpu
        return mlp_cpu.eligible(self, x)

    def _flatten(self, x):
        return x.reshape(x.shape[0], -1)

    def _torch_forward(self, x):
        x = self._flatten(x)
        lins = self.linears()
        if x.is_cuda and self.compute_dtype == torch.bfloat16:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                for lin in lins[:-1]:
                    x = F.relu(lin(x))
                return lins[-1](x).float()
        x = x.to(self.fc0.weight.dtype) if self.fc0.weight.dtype == torch.float64 else x.float()
        for lin in lins[:-1]:
            x = F.relu(lin(x))
        return lins[-1](x)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self._native_f32_ok(x) and not torch.is_grad_enabled():
            from ..ops import f32
            return f32.mlp_logits(self, x)
        if self._native_ok(x):
            from ..ops import mlp as mlp_ops
            return mlp_ops.mlp_logits(self, self._flatten(x))
        if self._cpu_fused_ok(x):
            from ..ops import mlp_cpu
            return mlp_cpu.mlp_logits(self, self._flatten(x).float())
        return self._torch_forward(x)

    def forward_loss(self, x: torch.Tensor, targets: torch.Tensor):
        """Fused forward + mean cross-entropy.  Returns (loss, logits-or-None)."""
        if self._native_f32_ok(x):
            from ..ops import f32
            return f32.mlp_loss(self, x, targets), None
        if self._native_ok(x):
            from ..ops import mlp as mlp_ops
            return mlp_ops.mlp_loss(self, self._flatten(x), targets), None
        logits = self.forward(x)
        return F.cross_entropy(logits, targets), logits

    # ---- ddpx engine protocol -------------------------------------------------
    def native_active(self, device) -> bool:
        return (torch.device(device).type == "cuda" and self.use_native
                and self.compute_dtype == torch.bfloat16)

    def ddpx_spec(self, device):
        """Flat-store layout request: bf16 compute shadow + all params written by native kernels."""
        # hidden weights W_l (l >= 1) are read by the data-gradient GEMM after their gradient is produced: a
        # side-stream optimizer may update them only after the model's flat.release (ddpx.parallel.ddp)
        late = [lin.weight for lin in self.linears()[1:-1]]
        if torch.device(device).type == "cuda" and self.use_native and self.compute_dtype == torch.float32:
            from ..runtime import native
            native.kernels()
            # fp32: kernels read the masters
            return {"native_params": list(self.parameters()), "late_read_params": late}
        if self.native_active(device):
            from ..runtime import native
            native.kernels()  # fail loudly if the extension is missing on a GPU
            # weights are read by the kernels only through the bf16 shadow; biases in fp32
            # fp8: 128-element offsets, so every weight's MX copy (codes at the element offset, E8M0 scales at
            # offset / 32) is 16-B / 4-B aligned for the MX GEMM's operand loads
            return {"shadow_dtype": torch.bfloat16, "native_params": list(self.parameters()),
                    "shadow_only_params": [m.weight for m in self.modules() if isinstance(m, nn.Linear)],
                    "align": 128 if getattr(self, "fp8", False) else 64, "late_read_params": late}
        return {}

    def input_layout(self, device) -> str:
        if self.native_active(device):
            return "flat_bf16"
        return "flat_f32" if torch.device(device).type == "cuda" and self.use_native else "nchw_f32"

    @property
    def ddpx_lazy_gather(self) -> bool:
        """The native forward (``ddpx.ops.mlp``) announces every weight read (``FlatParams.before_read``),
        so DDP may defer ZeRO all-gathers into it; the torch path reads parameters directly."""
        return self.use_native and self.compute_dtype == torch.bfloat16 and self.fc0.weight.is_cuda
