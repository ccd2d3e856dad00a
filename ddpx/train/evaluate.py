"""Evaluation: top-1 accuracy in percent, as the reference computes it.

``/root/reference/singlegpu.py:184-209``: ``@torch.inference_mode``,
``model.eval()``, iterate the test loader (tqdm "eval" bar), ``argmax(dim=1)``,
accumulate the correct count on the device, one ``.item()`` at the end.  Each
rank evaluates the full, unsharded test set on the unwrapped module
(``multigpu.py:247``).  Here the argmax/compare/count is one native kernel per
batch accumulating into a device int32 (a single D2H sync at the end).
"""
from __future__ import annotations

import torch
from torch import nn

from ..ops.head import accuracy_count

try:
    from tqdm.auto import tqdm
except ImportError:  # pragma: no cover
    def tqdm(x, **_):
        return x


@torch.inference_mode()
def evaluate(model: nn.Module, dataflow, progress: bool = True) -> float:
    model.eval()
    num_samples = 0
    dev = None
    num_correct = None
    it = tqdm(dataflow, desc="eval", leave=False) if progress else dataflow
    for inputs, targets in it:
        if dev is None:
            dev = inputs.device
            num_correct = torch.zeros((), dtype=torch.int32, device=dev)
        outputs = model(inputs)
        accuracy_count(outputs, targets, num_correct)
        num_samples += targets.size(0)
    model.train()
    if num_samples == 0:
        return 0.0
    return (num_correct.double() / num_samples * 100).item()
