"""Placing a model onto the ddpx engine (device + flat parameter store)."""
from __future__ import annotations

import torch
from torch import nn

from .flat_params import FlatParams, flat_of


def prepare_model(model: nn.Module, device, grad_dtype=torch.float32) -> FlatParams:
    """Move ``model`` to ``device`` and flatten its parameters (idempotent)."""
    device = torch.device(device)
    model.to(device)
    f = flat_of(model)
    if f is not None:
        return f
    spec = model.ddpx_spec(device) if hasattr(model, "ddpx_spec") else {}
    f = FlatParams(model, grad_dtype=grad_dtype, shadow_dtype=spec.get("shadow_dtype"),
                   native_params=spec.get("native_params", ()), align=spec.get("align", 64))
    f.shadow_only = {id(p) for p in spec.get("shadow_only_params", ())}
    # None = unknown backward read pattern: a side-stream optimizer then waits for the end of backward
    f.late_read = {id(p) for p in spec["late_read_params"]} if "late_read_params" in spec else None
    return f
