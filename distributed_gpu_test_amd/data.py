"""Synthetic data and data-parallel sampling.

Reference behaviour being reproduced (``train.py``):

* ``make_synthetic_data`` (``train.py:19-24``) re-seeds the *global* RNG and
  draws ``x ~ N(0,1)^{N x F}``; the label is ``1[sum(x[:, :F/2]) > 0]``.  The
  model is built *after* the data, so its init depends on this RNG
  consumption.  ``make_synthetic_data`` below consumes the RNG in
  exactly the same order.
* ``DistributedSampler(ds, shuffle=True)`` (``train.py:69``) shuffles with
  seed ``0 + epoch`` (NOT ``--seed``), pads by wrap-around to a
  multiple of the world size and takes a strided shard.  ``shard_indices``
  reimplements that algorithm bit-exactly so the per-rank index plan can be
  built once and uploaded to the GPU (no per-step H2D copies).
  The reference crashes at world_size 1 (``sampler.set_epoch`` on ``None``,
  SURVEY Q1); here world_size 1 uses the same sampler algorithm with
  ``num_replicas=1``, which is what the survey's oracle row for ws=1 uses.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Iterator, List, Optional, Tuple

import torch


def make_synthetic_data(n_samples: int = 200, n_features: int = 20, seed: int = 42):
    torch.manual_seed(seed)
    x = torch.randn(n_samples, n_features)
    linear_sep = x[:, : n_features // 2].sum(dim=1)
    y = (linear_sep > 0).float().unsqueeze(1)
    return x, y


def get_dataloader(x: torch.Tensor, y: torch.Tensor, batch_size: int = 32, shuffle: bool = True):
    """Plain host-side ``DataLoader`` over ``(x, y)``.  The reference defines this helper but never
    calls it (``train.py:38-40``); it is kept for API parity.  The training paths use the
    device-resident dataset and sampler plans below instead."""
    from torch.utils.data import DataLoader, TensorDataset
    return DataLoader(TensorDataset(x, y), batch_size=batch_size, shuffle=shuffle)


def shard_indices(n: int, world_size: int, rank: int, epoch: int, seed: int = 0,
                  shuffle: bool = True, drop_last: bool = False) -> List[int]:
    """Indices rank ``rank`` sees in ``epoch`` — ``torch.utils.data.DistributedSampler``'s algorithm."""
    if not 0 <= rank < world_size:
        raise ValueError(f"rank {rank} out of range for world_size {world_size}")
    if drop_last and n % world_size != 0:
        num_samples = math.ceil((n - world_size) / world_size)
    else:
        num_samples = math.ceil(n / world_size)
    total_size = num_samples * world_size
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        indices = torch.randperm(n, generator=g).tolist()
    else:
        indices = list(range(n))
    if not drop_last:
        padding = total_size - len(indices)
        if padding <= len(indices):
            indices += indices[:padding]
        else:
            indices += (indices * math.ceil(padding / len(indices)))[:padding]
    else:
        indices = indices[:total_size]
    return indices[rank:total_size:world_size]


def batch_plan(indices: List[int], batch_size: int, drop_last: bool = False) -> torch.Tensor:
    """[steps, batch_size] int32 index plan; the short tail batch is padded with -1."""
    steps = len(indices) // batch_size if drop_last else math.ceil(len(indices) / batch_size)
    plan = torch.full((steps, batch_size), -1, dtype=torch.int32)
    for s in range(steps):
        chunk = indices[s * batch_size:(s + 1) * batch_size]
        plan[s, :len(chunk)] = torch.tensor(chunk, dtype=torch.int32)
    return plan


def steps_per_epoch(n: int, world_size: int, batch_size: int) -> int:
    return math.ceil(math.ceil(n / world_size) / batch_size)


def gather_batch(rows: torch.Tensor, *tensors: torch.Tensor) -> Tuple[torch.Tensor, ...]:
    """The minibatch ``t[rows]`` of every dataset tensor (x, y, ...).  On the GPU: one HIP launch for
    all of them (``csrc/data.hip``), fresh contiguous outputs, instead of one ``index_select`` per
    tensor -- the generic engine's step is host-bound and each launch is ~4-5 us of it.  Indices must
    lie in ``[0, rows)`` (an out-of-range index yields a zero row, as no check may sync the step)."""
    if rows.is_cuda and 0 < len(tensors) <= 4 and rows.dtype == torch.long and rows.dim() == 1:
        for t in tensors:  # (a plain loop: this runs every step of a host-bound loop)
            if not (t.is_cuda and t.dim() >= 1 and t.is_contiguous() and (t.stride(0) * t.element_size()) % 4 == 0):
                break
        else:
            global _HOT
            if _HOT is None:
                from .ops import _ext
                _HOT = _ext.hot()
            return tuple(_HOT.gather_rows(rows.contiguous(), list(tensors)))  # (checks the devices)
    return tuple(t.index_select(0, rows) for t in tensors)


_HOT = None  # ops._ext.hot(), looked up on the first GPU gather


@dataclass
class SyntheticDataset:
    """Device-resident dataset + per-rank sampler.  Iteration yields device tensors."""
    x: torch.Tensor
    y: torch.Tensor
    batch_size: int
    world_size: int = 1
    rank: int = 0
    sampler_seed: int = 0
    epoch: int = 0

    def to(self, device) -> "SyntheticDataset":
        self.x = self.x.to(device)
        self.y = self.y.to(device)
        return self

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    @property
    def n(self) -> int:
        return self.x.shape[0]

    def plan(self, epoch: Optional[int] = None) -> torch.Tensor:
        e = self.epoch if epoch is None else epoch
        return batch_plan(shard_indices(self.n, self.world_size, self.rank, e, self.sampler_seed),
                          self.batch_size)

    def __len__(self) -> int:
        return steps_per_epoch(self.n, self.world_size, self.batch_size)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        idx = shard_indices(self.n, self.world_size, self.rank, self.epoch, self.sampler_seed)
        dev_idx = torch.tensor(idx, dtype=torch.long, device=self.x.device)
        for s in range(0, len(idx), self.batch_size):
            yield gather_batch(dev_idx[s:s + self.batch_size], self.x, self.y)
