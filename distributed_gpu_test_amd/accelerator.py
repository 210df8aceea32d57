"""Device abstraction: the role of ``deepspeed.accelerator.get_accelerator()``.

The reference calls ``get_accelerator().set_device(local_rank)`` (``train.py:12,61``).  Here the
accelerator is the ONE place that decides where a run computes and which collective backend it
uses: ``comm.init_distributed`` binds the rank's device and picks the backend through it, and the
engine, the trainers, ``train.py`` and ``bench.py`` take their default device from it.

Two implementations: ``hip`` (AMD Instinct through PyTorch-ROCm, whose device namespace is
``torch.cuda``; collectives go to RCCL through the ``nccl`` backend name) and ``cpu`` (gloo).
``DGT_ACCELERATOR=cpu|hip`` forces one; by default ``hip`` when a GPU is visible.
"""
from __future__ import annotations

import os
import threading
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

    def set_device(self, local_rank: int) -> None:
        """Bind ``local_rank``'s GPU.  A local rank beyond the visible devices (a wrong
        ``HIP_VISIBLE_DEVICES`` or ``GPUS_PER_NODE``) is an error: silently wrapping it onto a card
        another rank uses would oversubscribe the node.  ``DGT_ALLOW_OVERSUBSCRIBE=1`` wraps on
        purpose (the one-card multi-rank rehearsals); train.py and bench.py report it as
        ``oversubscribed``."""
        n = max(torch.cuda.device_count(), 1)
        if local_rank >= n and not allow_oversubscribe():
            raise RuntimeError(f"local rank {local_rank} has no GPU of its own: {n} visible device(s) "
                               f"(HIP_VISIBLE_DEVICES={os.environ.get('HIP_VISIBLE_DEVICES', '<unset>')}); "
                               "fix --nproc-per-node / GPUS_PER_NODE, or set DGT_ALLOW_OVERSUBSCRIBE=1 to share cards")
        torch.cuda.set_device(local_rank % n)
        set_wait_mode(os.environ.get("DGT_HIP_WAIT", ""))

    def device(self, index: Optional[int] = None) -> torch.device:
        return torch.device("cuda", self.current_device() if index is None else index)

    def communication_backend_name(self) -> str:
        return "nccl"  # ProcessGroupNCCL is backed by RCCL on ROCm

    def synchronize(self) -> None:
        torch.cuda.synchronize()


class CpuAccelerator:
    name = "cpu"

    def is_available(self) -> bool:
        return True

    def device_count(self) -> int:
        return 1

    def current_device(self) -> int:
        return 0

    def set_device(self, local_rank: int) -> None:
        pass

    def device(self, index: Optional[int] = None) -> torch.device:
        return torch.device("cpu")

    def communication_backend_name(self) -> str:
        return "gloo"

    def synchronize(self) -> None:
        pass


def allow_oversubscribe() -> bool:
    return os.environ.get("DGT_ALLOW_OVERSUBSCRIBE", "0") not in ("", "0", "false", "False")


def device_identity(device) -> str:
    """Host + PCI address of ``device``: ranks sharing one card report the same string (a CPU rank
    is its own device: there is no card to share)."""
    import socket
    if device.type != "cuda":
        import torch.distributed as dist
        return f"{socket.gethostname()}/cpu-rank{dist.get_rank() if dist.is_initialized() else 0}"
    p = torch.cuda.get_device_properties(device)
    return f"{socket.gethostname()}/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"


# hipSetDeviceFlags schedule bits: how a host thread waits for the device (synchronize, events)
_WAIT_FLAGS = {"auto": 0, "spin": 1, "yield": 2, "blocking": 4}


def set_wait_mode(mode: str) -> bool:
    """``DGT_HIP_WAIT=spin|yield|blocking|auto``: the current device's host wait mode.  ``spin`` keeps
    the waiting thread polling the completion signal instead of sleeping on an interrupt once the
    runtime's short active-wait window has passed, which shortens the launch -> completion -> wake-up
    round trip of a short kernel.  Empty: leave the runtime default.  Returns True if applied."""
    if not mode:
        return False
    if mode not in _WAIT_FLAGS:
        raise ValueError(f"DGT_HIP_WAIT must be one of {sorted(_WAIT_FLAGS)}, got {mode!r}")
    import ctypes
    rc = ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(ctypes.c_uint(_WAIT_FLAGS[mode]))
    if rc != 0:
        raise RuntimeError(f"hipSetDeviceFlags({mode}) failed with HIP error {rc}")
    return True


def _current_cpu() -> "int | None":
    """The CPU this thread last ran on (/proc/self/task/<tid>/stat field 39), or None."""
    try:
        tid = threading.get_native_id()
        with open(f"/proc/self/task/{tid}/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        return int(fields[36])  # (fields after the comm: state is field 3, processor is field 39)
    except (OSError, ValueError, IndexError):
        return None


def pin_host_thread(local_rank: int = 0, local_world_size: int = 1) -> "int | None":
    """Pin the calling thread to ONE CPU of its allowed set (``"amd": {"pin_host_thread": true}`` /
    ``DGT_PIN_HOST_THREAD=1``).  A host-bound engine step (a whole-step graph: ~18 us of host enqueue
    per ~19.5 us of device time) runs 19.4-25.7 us/step from process to process unpinned -- the
    thread's slow steps are scheduler hiccups (host enqueue p90 36-50 us against 18-20) -- and
    19.5-19.7 pinned (profiles/r6_engine_graph_variance.txt).  One rank: the CPU it runs on now (the
    scheduler's NUMA placement kept); N ranks per node: spread evenly over the allowed set so no two
    ranks share a core.  Only this thread is pinned (``sched_setaffinity`` of its own tid): threads
    that already exist (the HIP runtime's, RCCL's) keep their set, but threads and processes this
    thread starts LATER inherit the one CPU -- create a multi-worker DataLoader first, or leave the
    option off.  Returns the CPU, or None if nothing was pinned."""
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return None
    if not allowed:
        return None
    if local_world_size > 1:
        cpu = allowed[(local_rank * len(allowed)) // local_world_size]
    else:
        cpu = _current_cpu()
        if cpu not in allowed:
            cpu = allowed[0]
    try:
        os.sched_setaffinity(threading.get_native_id(), {cpu})
    except OSError:
        return None
    return cpu


_CONCURRENT: dict = {}


def concurrent_stream(device, tries: int = 8, slot: int = 0):
    """A stream of torch's pool that runs BESIDE the device's current stream: (stream, probed_ok).
    ``slot``: independent users (the engine's reducer 0, the MLP trainer's comm 1 / optimizer 2
    streams) get streams of their own.

    HIP maps a process's streams onto at most GPU_MAX_HW_QUEUES (4 here) hardware queues, round
    robin; two streams on one queue run strictly in turn, so a side stream that happens to share the
    compute stream's queue overlaps nothing (profiles/r6_engine_overlap_trace_v3.txt: every kernel of
    both streams on queue 1).  A stream of its own queue class -- another priority, or a CU mask --
    does get a queue of its own, but a fifth queue oversubscribes the hardware scheduler, which then
    time-slices: every kernel of the process ran ~2.5x longer (profiles/r6_reducer_launch_ab.txt).
    There is no API that names a stream's queue, so this MEASURES it: the current stream is held by
    a ~8 ms spin kernel and an event is recorded on a candidate stream; a candidate whose event
    completes while the spin still runs sits on another queue.  The first such candidate is kept
    (per device and slot, once per process); if none is found, the last candidate comes back with False."""
    import torch
    idx = torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device()
    key = (idx, slot)
    hit = _CONCURRENT.get(key)
    if hit is not None:
        return hit
    import time
    dev = torch.device("cuda", idx)
    cur = torch.cuda.current_stream(dev)
    cand = None
    found = False
    for _ in range(tries):
        cand = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize(dev)
        spin_done = torch.cuda.Event()
        mark = torch.cuda.Event()
        with torch.cuda.stream(cur):
            torch.cuda._sleep(16_000_000)  # ~8 ms at ~2 GHz
            spin_done.record(cur)
        mark.record(cand)
        t0 = time.perf_counter()
        while not mark.query() and time.perf_counter() - t0 < 0.005:
            pass
        found = mark.query() and not spin_done.query()
        torch.cuda.synchronize(dev)
        if found:
            break
    _CONCURRENT[key] = (cand, found)
    return cand, found


_ACCEL = None


def get_accelerator():
    global _ACCEL
    if _ACCEL is None:
        forced = os.environ.get("DGT_ACCELERATOR")
        if forced not in (None, "", "cpu", "hip"):
            raise ValueError(f"DGT_ACCELERATOR must be 'cpu' or 'hip', got {forced!r}")
        if forced == "hip" and not torch.cuda.is_available():
            raise RuntimeError("DGT_ACCELERATOR=hip but no GPU is visible")
        if forced == "cpu" or (not forced and not torch.cuda.is_available()):
            _ACCEL = CpuAccelerator()
        else:
            _ACCEL = HipAccelerator()
    return _ACCEL


def reset_accelerator() -> None:
    """Forget the cached choice (tests that change ``DGT_ACCELERATOR``)."""
    global _ACCEL
    _ACCEL = None
