"""The PyTorch this framework was validated on, and the torch internals its fast paths use.

Reference: the acceptance job runs the image (``slurm_train.sbatch:34-35``), so the image's torch is
the one that matters; the reference's own image pip-installs an unpinned torch (``Dockerfile:10-12``).

The engine's host fast paths reach below torch's public API:

* HIP graphs kept after instantiation: ``torch.cuda.CUDAGraph(keep_graph=True)``, ``.instantiate()``,
  ``.raw_cuda_graph()`` (``runtime/graph_module.py``, ``runtime/graph_step.py``: the direct launcher
  reads the captured kernel nodes);
* the saved state of torch's BCE-with-logits backward node (``_saved_self``, ``_saved_target``,
  ``_saved_reduction``, ...): the engine forms d loss / d logits of the reference's criterion with its
  own loss kernel (``engine._direct_backward``, ``engine._tail_runner``);
* ``torch._C._autograd._get_current_graph_task_keep_graph`` (``ops/loss.py`` keep_graph) and the C++
  ``_FunctionBase.apply`` (``utils/fnapply.py``);
* ``Tensor.register_post_accumulate_grad_hook`` (the bucket reducer's trigger).

``features()`` probes each one once (no GPU needed).  A missing one turns its path off LOUDLY: one
``[dgt] graph paths off: <reason>`` line on stderr (rank 0) and a ``{"event": "fallback"}`` record in
the metrics sink -- never a silent eager run.  ``MIN_TORCH`` is the oldest torch the whole test suite
has run on; the Dockerfile pins a base at or above it (``tests/test_compat.py`` parses it) and the
image build runs ``python3 -m distributed_gpu_test_amd.compat --strict``.
"""
from __future__ import annotations

import inspect
import sys
from typing import Dict, Optional, Tuple

import torch

MIN_TORCH: Tuple[int, int] = (2, 10)

_FEATURES: Optional[Dict[str, str]] = None
_REPORTED: set = set()


def torch_version(v: Optional[str] = None) -> Tuple[int, int]:
    """(major, minor) of a torch version string ("2.10.0+rocm7.0" -> (2, 10))."""
    s = (v or torch.__version__).split("+")[0]
    parts = [p for p in s.split(".")[:2]]
    out = []
    for p in parts:
        digits = "".join(ch for ch in p if ch.isdigit())
        out.append(int(digits or 0))
    while len(out) < 2:
        out.append(0)
    return out[0], out[1]


def _probe_graph() -> str:
    g = getattr(torch.cuda, "CUDAGraph", None)
    if g is None:
        return "torch.cuda.CUDAGraph is missing"
    params = {}
    for ctor in (g.__new__, g.__init__):  # (torch 2.10: the Python __new__ carries it)
        try:
            params.update(inspect.signature(ctor).parameters)
        except (TypeError, ValueError):
            pass
    if "keep_graph" not in params:
        return "torch.cuda.CUDAGraph has no keep_graph argument"
    for name in ("instantiate", "raw_cuda_graph", "capture_begin", "capture_end", "replay"):
        if not hasattr(g, name):
            return f"torch.cuda.CUDAGraph has no {name}()"
    if not hasattr(torch.cuda, "graph_pool_handle"):
        return "torch.cuda.graph_pool_handle is missing"
    return ""


def _probe_bce_node() -> str:
    z = torch.zeros(2, requires_grad=True)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(z, torch.ones(2))
    node = loss.grad_fn
    if type(node).__name__ != "BinaryCrossEntropyWithLogitsBackward0":
        return f"torch's BCE-with-logits backward node is {type(node).__name__}"
    for attr in ("_saved_self", "_saved_target", "_saved_reduction", "_saved_weight", "_saved_pos_weight"):
        try:
            getattr(node, attr)
        except AttributeError:
            return f"BinaryCrossEntropyWithLogitsBackward0 has no {attr}"
    if node._saved_reduction != 1:
        return "BinaryCrossEntropyWithLogitsBackward0._saved_reduction does not encode mean as 1"
    return ""


def _probe_keep_graph() -> str:
    ag = getattr(torch._C, "_autograd", None)
    if ag is None or not hasattr(ag, "_get_current_graph_task_keep_graph"):
        return "torch._C._autograd._get_current_graph_task_keep_graph is missing"
    return ""


def _probe_fn_apply() -> str:
    base = getattr(torch._C, "_FunctionBase", None)
    if base is None or "apply" not in base.__dict__:
        return "torch._C._FunctionBase.apply is missing"
    if not hasattr(torch._C, "_are_functorch_transforms_active"):
        return "torch._C._are_functorch_transforms_active is missing"
    return ""


def _probe_post_hook() -> str:
    if not hasattr(torch.Tensor, "register_post_accumulate_grad_hook"):
        return "Tensor.register_post_accumulate_grad_hook is missing"
    return ""


def features() -> Dict[str, str]:
    """feature -> "" (available) or the reason it is not; probed once."""
    global _FEATURES
    if _FEATURES is None:
        f = {}
        for name, probe in (("hip_graph", _probe_graph), ("torch_bce_node", _probe_bce_node),
                            ("keep_graph", _probe_keep_graph), ("fn_apply", _probe_fn_apply),
                            ("post_accumulate_hook", _probe_post_hook)):
            try:
                f[name] = probe()
            except Exception as e:  # noqa: BLE001 -- a probe that breaks is a missing feature
                f[name] = f"probe failed: {type(e).__name__}: {e}"
        if torch_version() < MIN_TORCH:
            f["torch_version"] = (f"torch {torch.__version__} is older than MIN_TORCH "
                                  f"{MIN_TORCH[0]}.{MIN_TORCH[1]} (the validated stack)")
        else:
            f["torch_version"] = ""
        _FEATURES = f
    return _FEATURES


def has(name: str) -> bool:
    return not features().get(name, "")


def report_fallback(what: str, reason: str, metrics=None) -> None:
    """One loud line per (what, reason) on rank 0, plus a metrics record: ``[dgt] graph paths off: ...``."""
    key = (what, reason)
    if key not in _REPORTED:
        _REPORTED.add(key)
        import torch.distributed as dist
        rank0 = not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0
        if rank0:
            print(f"[dgt] {what} off: {reason}", file=sys.stderr, flush=True)
    if metrics is not None and getattr(metrics, "enabled", False):
        metrics.log({"event": "fallback", "what": what, "reason": reason})


def check(strict: bool = False) -> Dict[str, str]:
    """Every feature's status; ``strict`` raises if any is missing (the image build's gate)."""
    f = features()
    bad = {k: v for k, v in f.items() if v}
    if strict and bad:
        raise RuntimeError("dgt: this torch lacks what the validated fast paths use: " +
                           "; ".join(f"{k}: {v}" for k, v in bad.items()))
    return f


if __name__ == "__main__":
    status = check(strict="--strict" in sys.argv)
    print(f"torch {torch.__version__} (MIN_TORCH {MIN_TORCH[0]}.{MIN_TORCH[1]}):")
    for k, v in status.items():
        print(f"  {k:22s} {'ok' if not v else v}")
