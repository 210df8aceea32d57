"""Tracing: roctx ranges and an optional torch.profiler session.

Reference: the training loop ``train.py:98-117`` (no tracing there).

The reference has no profiling.  Here every engine phase is wrapped in a named range (roctx on
ROCm through ``torch.cuda.nvtx``, visible in ``rocprofv3 --marker-trace`` timelines), and
``train.py --profile DIR`` records a kineto trace of the first steps (Chrome-trace JSON per rank).
Kernel-level numbers come from ``rocprofv3 --kernel-trace --stats`` (see profiles/).
"""
from __future__ import annotations

import contextlib
import os

import torch

_ENABLED = os.environ.get("DGT_ROCTX", "0") not in ("", "0")


class _Range:
    __slots__ = ("name",)

    def __init__(self, name: str):
        self.name = name

    def __enter__(self):
        torch.cuda.nvtx.range_push(self.name)

    def __exit__(self, *exc):
        torch.cuda.nvtx.range_pop()
        return False


_NULL = contextlib.nullcontext()


def range(name: str):  # noqa: A001 - mirrors nvtx.range
    """A roctx range when tracing is on; otherwise one shared no-op context (the engine's host-bound
    eager step enters several per step: no generator object per call)."""
    if _ENABLED and torch.cuda.is_available():
        return _Range(name)
    return _NULL


def enable(flag: bool = True) -> None:
    global _ENABLED
    _ENABLED = flag


class Profiler:
    """``with Profiler(dir, rank, steps):`` ... ``prof.step()`` per training step.  The fused path
    calls ``step()`` once per epoch (one kernel launch runs the epoch) with ``wait=warmup=0``."""

    def __init__(self, out_dir: str | None, rank: int = 0, active_steps: int = 20, wait: int = 1, warmup: int = 2):
        self.out_dir = out_dir
        self.rank = rank
        self.prof = None
        if out_dir:
            os.makedirs(out_dir, exist_ok=True)
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self.prof = torch.profiler.profile(
                activities=acts, schedule=torch.profiler.schedule(wait=wait, warmup=warmup, active=active_steps, repeat=1),
                on_trace_ready=self._save, record_shapes=False)

    def _save(self, p):
        path = os.path.join(self.out_dir, f"trace_rank{self.rank}.json")
        p.export_chrome_trace(path)

    def __enter__(self):
        if self.prof is not None:
            self.prof.__enter__()
        return self

    def __exit__(self, *exc):
        if self.prof is not None:
            self.prof.__exit__(*exc)
        return False

    def step(self):
        if self.prof is not None:
            self.prof.step()
