"""Device abstraction: the role of ``deepspeed.accelerator.get_accelerator()``.

The reference calls ``get_accelerator().set_device(local_rank)`` (``train.py:61``).  Two
implementations: ``hip`` (AMD Instinct via PyTorch-ROCm, whose device namespace is ``torch.cuda``;
collectives go to RCCL through the ``nccl`` backend name) and ``cpu`` (gloo).  ``DGT_ACCELERATOR``
forces one.
"""
from __future__ import annotations

import os
from typing import Optional

import torch


class HipAccelerator:
    name = "hip"

    def is_available(self) -> bool:
        return torch.cuda.is_available()

    def device_count(self) -> int:
        return torch.cuda.device_count()

    def current_device(self) -> int:
        return torch.cuda.current_device()

    def set_device(self, index: int) -> None:
        torch.cuda.set_device(index)

    def device(self, index: Optional[int] = None) -> torch.device:
        return torch.device("cuda", self.current_device() if index is None else index)

    def device_name(self, index: Optional[int] = None) -> str:
        return f"cuda:{self.current_device() if index is None else index}"

    def device_properties(self, index: Optional[int] = None):
        return torch.cuda.get_device_properties(self.current_device() if index is None else index)

    def arch(self, index: Optional[int] = None) -> str:
        return getattr(self.device_properties(index), "gcnArchName", "unknown")

    def communication_backend_name(self) -> str:
        return "nccl"  # ProcessGroupNCCL is backed by RCCL on ROCm

    def synchronize(self) -> None:
        torch.cuda.synchronize()

    def Stream(self, **kw):
        return torch.cuda.Stream(**kw)

    def Event(self, **kw):
        return torch.cuda.Event(**kw)

    def stream(self, s):
        return torch.cuda.stream(s)

    def current_stream(self):
        return torch.cuda.current_stream()

    def memory_allocated(self) -> int:
        return torch.cuda.memory_allocated()

    def max_memory_allocated(self) -> int:
        return torch.cuda.max_memory_allocated()

    def total_memory(self, index: Optional[int] = None) -> int:
        return self.device_properties(index).total_memory

    def manual_seed(self, seed: int) -> None:
        torch.cuda.manual_seed(seed)

    def graph(self, g, **kw):
        return torch.cuda.graph(g, **kw)


class CpuAccelerator:
    name = "cpu"

    def is_available(self) -> bool:
        return True

    def device_count(self) -> int:
        return 1

    def current_device(self) -> int:
        return 0

    def set_device(self, index: int) -> None:
        pass

    def device(self, index: Optional[int] = None) -> torch.device:
        return torch.device("cpu")

    def device_name(self, index: Optional[int] = None) -> str:
        return "cpu"

    def arch(self, index: Optional[int] = None) -> str:
        return "cpu"

    def communication_backend_name(self) -> str:
        return "gloo"

    def synchronize(self) -> None:
        pass

    def memory_allocated(self) -> int:
        return 0

    def max_memory_allocated(self) -> int:
        return 0

    def manual_seed(self, seed: int) -> None:
        torch.manual_seed(seed)


_ACCEL = None


def get_accelerator():
    global _ACCEL
    if _ACCEL is None:
        forced = os.environ.get("DGT_ACCELERATOR")
        if forced == "cpu" or (forced is None and not torch.cuda.is_available()):
            _ACCEL = CpuAccelerator()
        else:
            _ACCEL = HipAccelerator()
    return _ACCEL
