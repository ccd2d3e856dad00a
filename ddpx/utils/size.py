"""Model-size reporting, as the reference prints it.

``get_model_size`` and the bit-valued unit constants are the reference's
``/root/reference/singlegpu.py:212-225``: Byte/KiB/MiB/GiB are counts of *bits*,
so ``get_model_size(model) / MiB`` is the size in MiB at ``data_width`` bits
per element.  VGG → 35.20 MiB at fp32.
"""
from __future__ import annotations

from torch import nn

Byte = 8
KiB = 1024 * Byte
MiB = 1024 * KiB
GiB = 1024 * MiB


def get_model_size(model: nn.Module, data_width: int = 32) -> int:
    """Model size in bits: (number of parameter elements) x data_width."""
    num_elements = 0
    for param in model.parameters():
        num_elements += param.numel()
    return num_elements * data_width


def count_params(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())
