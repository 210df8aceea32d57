"""IPC mailboxes for the one-shot xGMI exchange (``csrc/comm.hip``, ``csrc/tiny_mlp.hip``).

Reference: the per-step 5.6 KB gradient all-reduce of ``train.py:113``.

Each rank allocates ONE uncached device buffer (``hipExtMallocWithFlags(hipDeviceMallocUncached)``:
peers' writes land in HBM and are read without stale cache lines), exports it with
``hipIpcGetMemHandle``, and every rank maps every peer's buffer (``hipIpcOpenMemHandle``).  The
handles travel over the already-initialised process group (``all_gather_object``), so no extra
rendezvous is needed.

Buffer layout: LL lines ``[2 parity][8 src ranks][stride / 2]`` of 16 bytes; a line carries two
``{payload float, tag}`` pairs (``csrc/dgt_common.h``), so ``stride`` payload floats take
``8 * stride`` bytes per slot.  (The fused trainer's kernel fills the same slots with LL3 lines,
three payload floats and one tag per 16 bytes, ``csrc/dgt_common.h`` ``ll3_put``.)  A channel carries a monotonically increasing sequence number per
exchange and the tag of exchange ``seq`` is ``seq + 1``; a reader polls its own mailbox until
every line carries the expected tag.  No flags and no fences: the tag travels with the data.

Before the channel is trusted, ``selftest`` runs a one-shot all-reduce with a bounded spin and
compares it against the process group's own all-reduce (RCCL).  Any mismatch or timeout on any
rank disables the channel everywhere and callers fall back to RCCL.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from ..launch import hostname
from ..ops._ext import require
from . import comm

MAX_RANKS = 8
TICKS_PER_SECOND = 100_000_000  # s_memrealtime runs at 100 MHz
MEM_KINDS = {"coarse": 0, "uncached": 1, "fine": 2}


def mem_kind() -> str:
    """Mailbox memory: ``uncached`` (default: correct by construction across GPUs, no cache ever
    holds a mailbox line) or ``fine`` (``DGT_IPC_MEM=fine``: cacheable fine-grained memory)."""
    k = os.environ.get("DGT_IPC_MEM", "uncached")
    if k not in MEM_KINDS:
        raise ValueError(f"DGT_IPC_MEM must be one of {sorted(MEM_KINDS)}")
    return k


class IpcChannel:
    def __init__(self, stride_floats: int, device: Optional[torch.device] = None, timeout_s: float = 30.0,
                 group=None):
        if not torch.cuda.is_available():
            raise RuntimeError("IpcChannel needs a GPU")
        self.ops = require()
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.rank = comm.get_rank()
        self.world_size = comm.get_world_size()
        if self.world_size > MAX_RANKS:
            raise ValueError(f"one-shot exchange supports up to {MAX_RANKS} ranks (one xGMI hop)")
        self.stride = (int(stride_floats) + 255) // 256 * 256
        self.nbytes = 2 * MAX_RANKS * self.stride * 8
        self.timeout_ticks = int(timeout_s * TICKS_PER_SECOND)
        self.seq = 0
        self.local_ptr = 0
        self.base_ptrs: List[int] = []
        self._opened: List[int] = []
        self.error: Optional[BaseException] = None
        self._bar: Optional[torch.Tensor] = None
        self._bar_out: Optional[torch.Tensor] = None
        self.status = torch.zeros(1, dtype=torch.int32, device=self.device)
        handle = b""
        # IPC handles only name memory on THIS node: a job that spans nodes never opens them
        # (callers fall back to RCCL, which bridges nodes over the network)
        hosts = comm.all_gather_object(hostname())
        if len(set(hosts)) > 1:
            self.error = RuntimeError(f"ranks span {len(set(hosts))} hosts: no cross-node IPC mailboxes")
        else:
            try:
                self.local_ptr = self.ops.ipc_alloc(self.nbytes, MEM_KINDS[mem_kind()], self.device.index)
                handle = bytes(self.ops.ipc_handle(self.local_ptr).numpy().tobytes())
            except Exception as e:  # IPC not supported here: every rank must learn it below
                self.error = e
        handles = comm.all_gather_object(handle)
        if self.error is None:
            try:
                for r, h in enumerate(handles):
                    if r == self.rank:
                        self.base_ptrs.append(self.local_ptr)
                    elif not h:
                        raise RuntimeError(f"rank {r} could not export its mailbox")
                    else:
                        t = torch.frombuffer(bytearray(h), dtype=torch.uint8)
                        p = self.ops.ipc_open(t, self.device.index)
                        self._opened.append(p)
                        self.base_ptrs.append(p)
            except Exception as e:
                self.error = e
        # every rank agrees on usability before anybody launches a kernel that waits on peers
        self.healthy = comm.all_reduce_max(0.0 if self.error is None else 1.0) == 0.0
        self.data_ptrs = list(self.base_ptrs) if self.healthy else []

    # ------------------------------------------------------------------ one-shot all-reduce
    def next_seq(self, n: int = 1) -> int:
        s = self.seq
        self.seq += n
        return s

    def allreduce(self, inp: torch.Tensor, out: Optional[torch.Tensor] = None, scale: float = 1.0,
                  reps: int = 1) -> torch.Tensor:
        """out = scale * sum over ranks of inp.  ``reps > 1`` repeats the all-reduce back to back
        inside one launch (latency measurement; needs ``out`` distinct from ``inp``)."""
        out = inp if out is None else out
        if reps > 1 and out.data_ptr() == inp.data_ptr():
            raise ValueError("repeated one-shot all-reduce needs out != inp")
        self.ops.oneshot_allreduce(inp, out, float(scale), self.data_ptrs, self.rank, self.world_size,
                                   self.stride, self.next_seq(reps), self.timeout_ticks, self.status, int(reps))
        return out

    def barrier(self) -> None:
        """Device-side barrier through the mailboxes: a one-shot all-reduce of one 16-byte line,
        queued on the current stream.  A rank's kernel ends only after every peer's kernel has
        written to it, and a peer launches its kernel only once its host reached the barrier, so
        after the caller's stream sync every rank has arrived.  A few microseconds on xGMI against
        tens for a process-group barrier; a timeout sets ``status`` (see ``check_status``)."""
        if self._bar is None:
            self._bar = torch.zeros(4, device=self.device)
            self._bar_out = torch.empty_like(self._bar)
        self.allreduce(self._bar, self._bar_out)

    def check_status(self) -> int:
        return int(self.status.item())

    def selftest(self, n: int = 4096, timeout_s: float = 10.0) -> bool:
        """Compare one-shot results with the process group's all-reduce; agree across ranks."""
        if not self.healthy:
            return False
        ok = True
        saved = self.timeout_ticks
        self.timeout_ticks = int(timeout_s * TICKS_PER_SECOND)
        n = min(n, self.stride) // 4 * 4
        g = torch.Generator(device="cpu").manual_seed(1234 + self.rank)
        x = torch.randn(n, generator=g).to(self.device)
        ref = comm.all_reduce_(x.clone())  # unconditional: every rank issues the same collectives
        try:
            got = torch.empty_like(x)
            for _ in range(3):  # both parities + a wrap of the first
                self.allreduce(x, got, 1.0)
            torch.cuda.synchronize(self.device)
            if self.check_status() != 0:
                ok = False
            if ok and not torch.allclose(got, ref, rtol=1e-5, atol=1e-5):
                ok = False
        except Exception:
            ok = False
        finally:
            self.timeout_ticks = saved
        self.healthy = comm.all_reduce_max(0.0 if ok else 1.0) == 0.0
        self.status.zero_()
        return self.healthy

    def close(self) -> None:
        for p in self._opened:
            try:
                self.ops.ipc_close(p)
            except Exception:
                pass
        self._opened = []
        if self.local_ptr:
            try:
                self.ops.ipc_free(self.local_ptr)
            except Exception:
                pass
            self.local_ptr = 0


def ipc_disabled_by_env() -> bool:
    return os.environ.get("DGT_DISABLE_IPC", "0") not in ("", "0", "false", "False")
