"""Fault injection.

The reference's only failure hook is a commented-out ``sys.exit(1)`` after training
(``train.py:129``); uncommenting it exercises the CI failure path.  Here the same is a flag:

    --fail-at RANK:STEP[:MODE]     or     DGT_FAIL_AT=RANK:STEP[:MODE]

RANK may be ``*`` (every rank).  STEP is the global optimizer step after which the fault fires
(``end`` = after training, the reference's location).  MODE:

* ``exit``  (default) — ``sys.exit(1)``: a clean non-zero exit, propagated by torchrun/srun to
  ``job_status.txt`` = fail;
* ``abort`` — ``os.abort()``: a crash (signal), like a segfaulting worker;
* ``hang``  — sleep forever: exercises the process-group / CI timeouts;
* ``nan``   — poison the loss with NaN from that step on (the training must notice / skip);
* ``corrupt`` — the fused kernel's in-kernel xGMI gradient exchange sends rank RANK+1 one wrong
  payload at step STEP (``csrc/tiny_mlp.hip``): a silent data corruption that only the per-epoch
  replica check (``TinyMLPTrainer.verify_replicas``) can catch.  No effect on the RCCL paths.

``DGT_FAIL_ONCE=<path>`` makes the fault fire only while ``<path>`` does not exist (it is created
just before firing): a restarted job (torchrun ``--max-restarts``) then runs through, which is how
elastic recovery + ``--resume`` is exercised.
"""
from __future__ import annotations

import os
import sys
import time
from dataclasses import dataclass
from typing import Optional

import torch

MODES = ("exit", "abort", "hang", "nan", "corrupt")
PASSIVE = ("nan", "corrupt")  # modes that alter data instead of ending the process


@dataclass
class FaultSpec:
    rank: Optional[int]  # None = every rank
    step: Optional[int]  # None = end of training
    mode: str = "exit"


def parse_fault(spec: Optional[str]) -> Optional[FaultSpec]:
    if not spec:
        return None
    parts = spec.split(":")
    if len(parts) < 2 or len(parts) > 3:
        raise ValueError(f"bad fault spec {spec!r}: expected RANK:STEP[:MODE]")
    rank = None if parts[0] in ("*", "all") else int(parts[0])
    step = None if parts[1] in ("end", "") else int(parts[1])
    mode = parts[2] if len(parts) == 3 else "exit"
    if mode not in MODES:
        raise ValueError(f"bad fault mode {mode!r}: expected one of {MODES}")
    return FaultSpec(rank, step, mode)


class FaultInjector:
    def __init__(self, spec: Optional[FaultSpec], rank: int):
        self.spec = spec
        self.rank = rank

    @classmethod
    def from_env(cls, rank: int, spec: Optional[str] = None) -> "FaultInjector":
        return cls(parse_fault(spec if spec is not None else os.environ.get("DGT_FAIL_AT")), rank)

    def _mine(self) -> bool:
        return self.spec is not None and (self.spec.rank is None or self.spec.rank == self.rank)

    def fire(self) -> None:
        once = os.environ.get("DGT_FAIL_ONCE")
        if once:
            if os.path.exists(once):
                return
            with open(once, "w") as fh:
                fh.write(f"rank {self.rank}\n")
        mode = self.spec.mode
        print(f"[dgt] fault injection on rank {self.rank}: {mode}", file=sys.stderr, flush=True)
        if mode == "exit":
            sys.exit(1)
        if mode == "abort":
            os.abort()
        if mode == "hang":
            while True:
                time.sleep(3600)

    def maybe_fire(self, step: int) -> None:
        if self._mine() and self.spec.step is not None and self.spec.mode not in PASSIVE and step >= self.spec.step:
            self.fire()

    def maybe_fire_end(self) -> None:
        if self._mine() and self.spec.step is None and self.spec.mode not in PASSIVE:
            self.fire()

    def maybe_corrupt_loss(self, loss: torch.Tensor, step: int) -> torch.Tensor:
        if (self._mine() and self.spec.mode == "nan" and (self.spec.step is None or step >= self.spec.step)):
            return loss * float("nan")
        return loss

    def corrupt_step(self) -> int:
        """1-based optimizer step at which this rank corrupts an exchange payload (-1 = never)."""
        if self._mine() and self.spec.mode == "corrupt" and self.spec.step is not None:
            return int(self.spec.step)
        return -1
