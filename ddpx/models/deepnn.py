"""DeepNN — the smaller CNN defined (but never instantiated) by the reference.

Same layers, order and ``state_dict`` keys as ``/root/reference/singlegpu.py:18-44``:
``features`` = Conv(3→128)-ReLU-Conv(128→64)-ReLU-MaxPool2 → Conv(64→64)-ReLU-
Conv(64→32)-ReLU-MaxPool2; ``classifier`` = Linear(2048→512)-ReLU-Dropout(0.1)-
Linear(512→num_classes).  1,186,986 parameters.
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

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.features(x)
        x = torch.flatten(x, 1)
        return self.classifier(x)
