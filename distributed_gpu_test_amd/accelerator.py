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
