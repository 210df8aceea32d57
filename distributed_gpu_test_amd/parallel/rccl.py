"""Native RCCL communicator (``csrc/rccl_comm.cpp``) for stream-ordered, graph-capturable collectives.

Reference: the NCCL communicator behind ``deepspeed.init_distributed()`` (``train.py:59``) and ``train.py:113``.

``ProcessGroupNCCL`` (the ``nccl`` backend = RCCL on ROCm) is the general path.  This thin native
communicator exists for the places where a collective must sit INSIDE a captured HIP graph next to
the kernels that produce and consume its buffer (``TinyMLPTrainer(impl="graph")``): the collective
is enqueued on the caller's current stream with no Python, watchdog or event bookkeeping.

Bootstrap: rank 0 draws an ``ncclUniqueId``; it is shared through the existing process group.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..ops._ext import require
from . import comm

SUM, PROD, MAX, MIN, AVG = 0, 1, 2, 3, 4


class RcclComm:
    def __init__(self, device: Optional[torch.device] = None):
        self.ops = require()
        self.rank, self.world_size = comm.get_rank(), comm.get_world_size()
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        uid = bytes(self.ops.rccl_unique_id().numpy().tobytes()) if self.rank == 0 else None
        uid = comm.all_gather_object(uid)[0]
        t = torch.frombuffer(bytearray(uid), dtype=torch.uint8)
        self.handle = self.ops.rccl_comm_init(t, self.rank, self.world_size, self.device.index)
        # first collective outside any graph: RCCL connects its channels lazily
        warm = torch.zeros(16, device=self.device)
        self.all_reduce(warm)
        torch.cuda.synchronize(self.device)

    @staticmethod
    def version() -> int:
        return int(require().rccl_version())

    def all_reduce(self, t: torch.Tensor, op: int = SUM) -> torch.Tensor:
        self.ops.rccl_all_reduce(self.handle, t, op)
        return t

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: int = SUM) -> torch.Tensor:
        self.ops.rccl_reduce_scatter(self.handle, out, inp, op)
        return out

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        self.ops.rccl_all_gather(self.handle, out, inp)
        return out

    def broadcast(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        self.ops.rccl_broadcast(self.handle, t, root)
        return t

    def close(self) -> None:
        if self.handle:
            try:
                self.ops.rccl_comm_destroy(self.handle)
            except Exception:
                pass
            self.handle = 0
