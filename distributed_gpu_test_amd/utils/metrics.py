"""Structured metrics: a JSONL sink and a throughput timer.

Reference: ``train.py:119-121`` (epoch loss print) and DeepSpeed's ``steps_per_print`` progress lines.

DeepSpeed's ``ThroughputTimer`` derives samples/sec from ``train_batch_size`` (which the reference
hard-codes to 64 while the real global batch is 4 x world_size), so it over-reports.
``ThroughputTimer`` here counts the samples actually processed.  ``MetricsSink`` writes one JSON
object per optimizer step when ``DGT_METRICS_JSONL`` names a file (``{rank}`` is substituted).
``health_event`` appends run-time health events (e.g. an exchange fallback) to ``DGT_HEALTH_LOG``,
the job's health log next to the pre-flight report (``slurm_train.sbatch``).
"""
from __future__ import annotations

import json
import os
import time
from typing import Any, Dict, Optional


class ThroughputTimer:
    def __init__(self, samples_per_step: int, window: int = 10):
        self.samples_per_step = samples_per_step
        self.window = max(1, window)
        self._t_start: Optional[float] = None
        self._window_t0: Optional[float] = None
        self._window_steps = 0
        self._last_sps: Optional[float] = None
        self.total_steps = 0
        self.total_time = 0.0

    def start(self) -> None:
        if self._t_start is None:
            self._t_start = time.perf_counter()
        if self._window_t0 is None:
            self._window_t0 = time.perf_counter()

    def stop(self, global_step: int) -> None:
        self._window_steps += 1
        self.total_steps += 1
        if self._window_steps >= self.window and self._window_t0 is not None:
            dt = time.perf_counter() - self._window_t0
            if dt > 0:
                self._last_sps = self._window_steps * self.samples_per_step / dt
                self.total_time += dt
            self._window_t0 = time.perf_counter()
            self._window_steps = 0

    def samples_per_sec(self) -> Optional[float]:
        return self._last_sps


class MetricsSink:
    def __init__(self, path: Optional[str]):
        self.path = path
        self._fh = open(path, "a") if path else None

    @classmethod
    def from_env(cls, rank: int) -> "MetricsSink":
        p = os.environ.get("DGT_METRICS_JSONL")
        if not p:
            return cls(None)
        p = p.replace("{rank}", str(rank))
        if "{rank}" not in os.environ.get("DGT_METRICS_JSONL", "") and rank != 0:
            return cls(None)  # one shared file: rank 0 only
        d = os.path.dirname(p)
        if d:
            os.makedirs(d, exist_ok=True)
        return cls(p)

    @property
    def enabled(self) -> bool:
        return self._fh is not None

    def log(self, record: Dict[str, Any]) -> None:
        if self._fh is None:
            return
        rec = {"ts": time.time(), **{k: v for k, v in record.items() if v is not None}}
        self._fh.write(json.dumps(rec) + "\n")
        self._fh.flush()

    def close(self) -> None:
        if self._fh is not None:
            self._fh.close()
            self._fh = None


def health_event(record: Dict[str, Any]) -> None:
    """Append one JSON line to ``DGT_HEALTH_LOG`` (``{rank}`` substituted; a shared file is
    appended to by every rank: one short line per event, written with a single write call)."""
    p = os.environ.get("DGT_HEALTH_LOG")
    if not p:
        return
    p = p.replace("{rank}", str(record.get("rank", 0)))
    d = os.path.dirname(p)
    if d:
        os.makedirs(d, exist_ok=True)
    line = json.dumps({"ts": time.time(), **{k: v for k, v in record.items() if v is not None}}) + "\n"
    with open(p, "a") as fh:
        fh.write(line)
