"""Bench-size synthetic MLP (BASELINE config #2: "1x MI355X single-process bf16 synthetic MLP").

Reference: ``SimpleNet`` (``train.py:26-36``), widened and deepened.

The reference trains Linear(20,64)-ReLU-Linear(64,1); that workload is launch/latency bound, so
it cannot exercise the matrix cores.  This is the same architecture family scaled up:
``depth`` x [Linear(width, width) + ReLU] followed by Linear(width, 1) + BCE-with-logits, on
synthetic data with the reference's labelling rule (y = 1[sum of the first half of x > 0]).
"""
from __future__ import annotations

import torch
import torch.nn as nn


class SyntheticMLP(nn.Module):
    def __init__(self, width: int = 4096, depth: int = 4, in_features: int | None = None):
        super().__init__()
        self.width = width
        self.depth = depth
        self.in_features = in_features or width
        dims = [self.in_features] + [width] * depth
        self.layers = nn.ModuleList(nn.Linear(dims[i], dims[i + 1]) for i in range(depth))
        self.head = nn.Linear(width, 1)

    def forward(self, x):
        for lin in self.layers:
            x = torch.relu(lin(x))
        return self.head(x)

    def flops_per_sample(self) -> int:
        """Training FLOPs per sample: forward + dgrad + wgrad GEMMs (2 FLOP per MAC each)."""
        macs = sum(l.in_features * l.out_features for l in self.layers) + self.width
        return 6 * macs


def synthetic_batch_data(n: int, features: int, seed: int):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, features, generator=g)
    y = (x[:, : features // 2].sum(1) > 0).float()
    return x, y
