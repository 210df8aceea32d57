"""Conversion between flat Adam buffers and ``torch.optim.Adam.state_dict()`` format.

Reference: the optimizer state DeepSpeed writes with ``save_checkpoint`` (``train.py:125``).

Checkpoints store optimizer state in torch's own per-parameter format so a checkpoint written by
the fused HIP path can be loaded into a plain ``torch.optim.Adam`` (and vice versa).
"""
from __future__ import annotations

from typing import Any, Dict, List, Sequence, Tuple

import torch

Segment = Tuple[int, Tuple[int, ...]]  # (offset into the flat buffer, shape)


def _numel(shape: Sequence[int]) -> int:
    n = 1
    for d in shape:
        n *= int(d)
    return n


def flat_to_adam_state(exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, segments: List[Segment], step: int,
                       lr: float, betas, eps: float, weight_decay: float, adamw: bool = False) -> Dict[str, Any]:
    state = {}
    if step > 0:
        for i, (off, shape) in enumerate(segments):
            n = _numel(shape)
            state[i] = {
                "step": torch.tensor(float(step)),
                "exp_avg": exp_avg[off:off + n].detach().view(shape).cpu().clone(),
                "exp_avg_sq": exp_avg_sq[off:off + n].detach().view(shape).cpu().clone(),
            }
    group = {"lr": float(lr), "betas": (float(betas[0]), float(betas[1])), "eps": float(eps),
             "weight_decay": float(weight_decay), "amsgrad": False, "maximize": False, "foreach": None,
             "capturable": False, "differentiable": False, "fused": None,
             "params": list(range(len(segments)))}
    if adamw:
        group["decoupled_weight_decay"] = True
    return {"state": state, "param_groups": [group]}


def adam_state_to_flat(sd: Dict[str, Any], exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor,
                       segments: List[Segment]) -> int:
    """Fill flat moment buffers from a torch Adam state_dict; returns the step count."""
    exp_avg.zero_()
    exp_avg_sq.zero_()
    step = 0
    for i, (off, shape) in enumerate(segments):
        st = sd["state"].get(i, sd["state"].get(str(i)))
        if not st:
            continue
        n = _numel(shape)
        exp_avg[off:off + n].copy_(st["exp_avg"].reshape(-1).to(exp_avg))
        exp_avg_sq[off:off + n].copy_(st["exp_avg_sq"].reshape(-1).to(exp_avg_sq))
        step = int(float(st["step"]))
    return step


def adam_hparams(optimizer) -> Dict[str, Any]:
    """Hyper-parameters of a client ``torch.optim.Adam``/``AdamW`` (one param group)."""
    if len(optimizer.param_groups) != 1:
        raise ValueError("the fused engine supports a single parameter group")
    g = optimizer.param_groups[0]
    name = type(optimizer).__name__.lower()
    if g.get("amsgrad", False):
        raise ValueError("amsgrad is not supported by the fused Adam kernel")
    return {"lr": float(g["lr"]), "betas": tuple(float(b) for b in g["betas"]), "eps": float(g["eps"]),
            "weight_decay": float(g.get("weight_decay", 0.0)),
            "adamw": name == "adamw" or bool(g.get("decoupled_weight_decay", False))}
