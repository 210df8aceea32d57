"""``autograd.Function.apply`` without its Python prologue.

``Function.apply`` (torch/autograd/function.py) checks for functorch transforms and rebuilds the
argument tuple through ``unwrap_dead_wrappers`` before it reaches the C++ ``_FunctionBase.apply``:
~2.5 us of host time per call on the MI355X box's CPU, paid by every fused node on the engine's
hot path (a graphed forward plus the fused loss is two calls per step, a host-bound ~50 us step).
The wrapper below calls the C++ entry directly when no functorch transform is active and falls back
to ``Function.apply`` otherwise, so vmap / grad over the framework's ops keep working.  Only for
Functions without ``setup_context`` (their apply binds no default arguments).
"""
from __future__ import annotations

import torch


def fast_apply(cls):
    if cls.setup_context is not torch.autograd.function._SingleLevelFunction.setup_context:
        return cls.apply
    base = getattr(torch._C, "_FunctionBase", None)
    active = getattr(torch._C, "_are_functorch_transforms_active", None)
    if base is None or "apply" not in base.__dict__ or active is None:
        return cls.apply  # (a torch without these internals: the public entry; compat.py reports it)
    raw = base.__dict__["apply"].__get__(None, cls)
    slow = cls.apply

    def apply(*args):
        if active():
            return slow(*args)
        return raw(*args)

    apply.__doc__ = f"{cls.__name__}.apply (C++ entry, no Python prologue)"
    return apply
