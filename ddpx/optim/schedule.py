"""The reference's triangular one-cycle LR schedule.

``/root/reference/singlegpu.py:142-149`` (and ``multigpu.py:136-143``)::

    lr_lambda = lambda step: np.interp([step / steps_per_epoch],
                                       [0, num_epochs * 0.3, num_epochs], [0, 1, 0])[0]
    scheduler = LambdaLR(optimizer, lr_lambda)      # stepped once per batch

with ``num_epochs = 20`` hard-coded and ``steps_per_epoch`` hard-coded to 98
(single) / 49 (multi).  λ(0) = 0, so the very first step runs with lr = 0, the
peak (λ = 1) is at epoch 6 and λ clamps to 0 after epoch 20.  ``compat`` mode
reproduces the hard-coded constants; ``auto`` uses the real loader length.
"""
from __future__ import annotations

import numpy as np
from torch.optim.lr_scheduler import LambdaLR

REF_NUM_EPOCHS = 20
REF_STEPS_SINGLE = 98
REF_STEPS_MULTI = 49


class OneCycleLambda:
    """Picklable λ(step) = interp(step/steps_per_epoch, [0, 0.3·E, E], [0, 1, 0])."""

    def __init__(self, steps_per_epoch: int, num_epochs: int = REF_NUM_EPOCHS):
        if steps_per_epoch <= 0:
            raise ValueError("steps_per_epoch must be positive")
        self.steps_per_epoch = steps_per_epoch
        self.num_epochs = num_epochs

    def __call__(self, step: int) -> float:
        return float(np.interp([step / self.steps_per_epoch], [0, self.num_epochs * 0.3, self.num_epochs],
                               [0, 1, 0])[0])


def resolve_steps_per_epoch(mode: str, loader_len: int, distributed: bool) -> int:
    if mode == "compat":
        return REF_STEPS_MULTI if distributed else REF_STEPS_SINGLE
    if mode == "auto":
        return max(1, loader_len)
    return int(mode)


def one_cycle(optimizer, steps_per_epoch: int, num_epochs: int = REF_NUM_EPOCHS) -> LambdaLR:
    return LambdaLR(optimizer, OneCycleLambda(steps_per_epoch, num_epochs))
