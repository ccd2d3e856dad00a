"""Checkpointing: the reference's format by default, full resumable state opt-in.

Default (``/root/reference/singlegpu.py:118-122``, ``multigpu.py:109-113``):
``torch.save(model_state_dict, "checkpoint.pt")`` — a plain ``OrderedDict``
with the module's own keys (no ``module.`` prefix: multigpu saves
``self.model.module.state_dict()``), each tensor its own storage on the model's
device, overwritten at every save.

Opt-in (absent in the reference): ``checkpoint_full.pt`` with
model, optimizer (momentum), scheduler, epoch, sampler epoch and RNG state,
written atomically (tmp file + ``os.replace``) so a crash never leaves a torn
file, and restored by :func:`load_full_checkpoint` for ``--resume``.
"""
from __future__ import annotations

import os
from collections import OrderedDict

import torch
from torch import nn

CKPT_PATH = "checkpoint.pt"
FULL_CKPT_PATH = "checkpoint_full.pt"


def unwrap(model: nn.Module) -> nn.Module:
    return model.module if hasattr(model, "module") and isinstance(model.module, nn.Module) else model


def model_state_dict(model: nn.Module) -> "OrderedDict[str, torch.Tensor]":
    """state_dict of the unwrapped module with every tensor in its own storage."""
    sd = unwrap(model).state_dict()
    return OrderedDict((k, v.detach().clone()) for k, v in sd.items())


def _atomic_save(obj, path):
    tmp = f"{path}.tmp.{os.getpid()}"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_checkpoint(model: nn.Module, path: str = CKPT_PATH, atomic: bool = True):
    sd = model_state_dict(model)
    if atomic:
        _atomic_save(sd, path)
    else:
        torch.save(sd, path)
    return path


def save_full_checkpoint(path, model, optimizer, scheduler, epoch, extra=None):
    state = {
        "model": model_state_dict(model),
        "optimizer": optimizer.state_dict() if optimizer is not None else None,
        "scheduler": scheduler.state_dict() if scheduler is not None else None,
        "epoch": int(epoch),
        "torch_rng": torch.get_rng_state(),
        "extra": extra or {},
    }
    _atomic_save(state, path)
    return path


def load_full_checkpoint(path, model, optimizer=None, scheduler=None, map_location=None):
    """Restore a full checkpoint written by :func:`save_full_checkpoint`; returns the next epoch."""
    state = torch.load(path, map_location=map_location, weights_only=True)
    m = unwrap(model)
    m.load_state_dict(state["model"])
    flat = getattr(next(m.parameters()), "_ddpx_flat", None)
    if flat is not None:
        flat.refresh_shadow()
    if optimizer is not None and state.get("optimizer") is not None:
        optimizer.load_state_dict(state["optimizer"])
    if scheduler is not None and state.get("scheduler") is not None:
        scheduler.load_state_dict(state["scheduler"])
    if state.get("torch_rng") is not None:
        torch.set_rng_state(state["torch_rng"])
    return int(state["epoch"]) + 1
