"""DeepSpeed-compatible LR schedules (``scheduler.type`` in the JSON config) and the fp16 loss scaler.

Reference: the DeepSpeed JSON dict of ``train.py:78-83`` (``fp16`` key) and the DS ``scheduler`` schema it accepts.
"""
from __future__ import annotations

import math
from typing import Any, Dict


class WarmupLR:
    """lr = min + (max - min) * gamma; gamma: log or linear warmup over ``warmup_num_steps``, then 1."""

    def __init__(self, warmup_min_lr: float = 0.0, warmup_max_lr: float = 0.001, warmup_num_steps: int = 1000,
                 warmup_type: str = "log", last_batch_iteration: int = -1, **_):
        self.min_lr = float(warmup_min_lr)
        self.max_lr = float(warmup_max_lr)
        self.warmup_num_steps = max(2, int(warmup_num_steps))
        self.warmup_type = warmup_type
        self.inverse_log_warm_up = 1.0 / math.log(self.warmup_num_steps)
        self.last_batch_iteration = last_batch_iteration

    def _gamma(self) -> float:
        it = self.last_batch_iteration
        if it < self.warmup_num_steps:
            if self.warmup_type == "log":
                return self.inverse_log_warm_up * math.log(it + 1)
            return it / self.warmup_num_steps
        return 1.0

    def get_lr(self) -> float:
        if self.last_batch_iteration < 0:
            return self.min_lr
        return self.min_lr + (self.max_lr - self.min_lr) * self._gamma()

    def step(self, last_batch_iteration: int | None = None) -> float:
        self.last_batch_iteration = (self.last_batch_iteration + 1 if last_batch_iteration is None
                                     else last_batch_iteration)
        return self.get_lr()

    def state_dict(self) -> Dict[str, Any]:
        return {"last_batch_iteration": self.last_batch_iteration}

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        self.last_batch_iteration = int(sd["last_batch_iteration"])


class WarmupDecayLR(WarmupLR):
    """WarmupLR followed by linear decay to 0 at ``total_num_steps``."""

    def __init__(self, total_num_steps: int, warmup_min_lr: float = 0.0, warmup_max_lr: float = 0.001,
                 warmup_num_steps: int = 1000, warmup_type: str = "log", last_batch_iteration: int = -1, **_):
        super().__init__(warmup_min_lr, warmup_max_lr, warmup_num_steps, warmup_type, last_batch_iteration)
        self.total_num_steps = int(total_num_steps)

    def _gamma(self) -> float:
        it = self.last_batch_iteration
        if it < self.warmup_num_steps:
            return super()._gamma()
        return max(0.0, float(self.total_num_steps - it) /
                   float(max(1.0, self.total_num_steps - self.warmup_num_steps)))


def build_scheduler(kind: str | None, params: Dict[str, Any]):
    if kind is None:
        return None
    if kind == "WarmupLR":
        return WarmupLR(**params)
    if kind == "WarmupDecayLR":
        return WarmupDecayLR(**params)
    raise ValueError(f"unknown scheduler {kind}")


class LossScaler:
    """fp16 loss scaling: static (``loss_scale > 0``) or dynamic with hysteresis (DeepSpeed defaults)."""

    def __init__(self, loss_scale: float = 0.0, initial_scale_power: int = 16, scale_window: int = 1000,
                 min_scale: float = 1.0, hysteresis: int = 2):
        self.dynamic = loss_scale == 0.0
        self.scale = float(2 ** initial_scale_power) if self.dynamic else float(loss_scale)
        self.scale_window = scale_window
        self.min_scale = min_scale
        self.hysteresis = hysteresis
        self._hyst = hysteresis
        self._good = 0

    def update(self, overflow: bool) -> None:
        if not self.dynamic:
            return
        if overflow:
            if self._hyst <= 1:
                self.scale = max(self.scale / 2.0, self.min_scale)
                self._hyst = self.hysteresis
            else:
                self._hyst -= 1
            self._good = 0
        else:
            self._good += 1
            if self._good % self.scale_window == 0:
                self.scale *= 2.0
                self._hyst = self.hysteresis

    def state_dict(self) -> Dict[str, Any]:
        return {"scale": self.scale, "good": self._good, "hyst": self._hyst}

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        self.scale, self._good, self._hyst = float(sd["scale"]), int(sd["good"]), int(sd["hyst"])
