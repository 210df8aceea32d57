"""The reference model: ``Linear(F, H) -> ReLU -> Linear(H, 1)`` (``train.py:26-36``).

Parameter names and order match the reference's ``nn.Sequential``
(``net.0.weight, net.0.bias, net.2.weight, net.2.bias``), so checkpoints are
interchangeable and the random init consumes the global RNG identically.

``flat_layout`` describes how the four tensors are packed into one flat fp32
buffer, which is the layout the fused HIP kernels (``csrc/tiny_mlp.hip``)
and the engine's flat parameter store both use.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch
import torch.nn as nn


class SimpleNet(nn.Module):
    def __init__(self, n_features: int = 20, hidden: int = 64):
        super().__init__()
        self.n_features = n_features
        self.hidden = hidden
        self.net = nn.Sequential(
            nn.Linear(n_features, hidden),
            nn.ReLU(),
            nn.Linear(hidden, 1),
        )

    def forward(self, x):
        return self.net(x)


def simple_net_layout(n_features: int, hidden: int) -> List[Tuple[str, Tuple[int, ...], int]]:
    """(name, shape, offset) of each parameter inside the dense flat buffer."""
    shapes = [("net.0.weight", (hidden, n_features)), ("net.0.bias", (hidden,)),
              ("net.2.weight", (1, hidden)), ("net.2.bias", (1,))]
    out, off = [], 0
    for name, shp in shapes:
        out.append((name, shp, off))
        n = 1
        for d in shp:
            n *= d
        off += n
    return out


def simple_net_numel(n_features: int, hidden: int) -> int:
    return hidden * n_features + 2 * hidden + 1


def pack_simple_net(model: SimpleNet) -> torch.Tensor:
    return torch.cat([p.detach().reshape(-1).float() for p in model.parameters()])


def unpack_simple_net(flat: torch.Tensor, n_features: int, hidden: int) -> Dict[str, torch.Tensor]:
    return {name: flat[off:off + int(torch.tensor(shp).prod())].view(shp).clone()
            for name, shp, off in simple_net_layout(n_features, hidden)}
