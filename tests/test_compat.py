"""The torch the framework's fast paths need (``distributed_gpu_test_amd/compat.py``) and the image's
pin of it (reference: the acceptance job runs the image, ``slurm_train.sbatch:34-35``)."""
import os
import re

import pytest
import torch

from distributed_gpu_test_amd import compat

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_version_parse():
    assert compat.torch_version("2.10.0+rocm7.0") == (2, 10)
    assert compat.torch_version("2.7.1") == (2, 7)
    assert compat.torch_version("2.11.0a0+git123") == (2, 11)
    assert compat.torch_version("3") == (3, 0)


def test_this_torch_has_every_feature():
    """The suite's own torch: every probe passes (what the GPU tests then exercise)."""
    f = compat.check(strict=True)
    assert set(f) == {"hip_graph", "torch_bce_node", "keep_graph", "fn_apply", "post_accumulate_hook",
                      "torch_version"}
    assert compat.torch_version() >= compat.MIN_TORCH


def test_dockerfile_base_torch_at_least_min():
    df = open(os.path.join(ROOT, "Dockerfile")).read()
    base = re.search(r"^ARG BASE_IMAGE=(\S+)$", df, re.M).group(1)
    rel = re.search(r"pytorch_release_([0-9.]+)", base).group(1)
    assert compat.torch_version(rel) >= compat.MIN_TORCH, base
    # the build gate: the image fails to build rather than ship fast paths that would fall back
    assert "python3 -m distributed_gpu_test_amd.compat --strict" in df
    gate = df.index("RUN cd /opt/dgt && python3 -m distributed_gpu_test_amd.compat --strict")
    assert df.index("FROM ${BASE_IMAGE}") < gate < df.index("python3 tools/build_ext.py")
    ci = open(os.path.join(ROOT, ".github", "workflows", "distributed-gpu-test-ci.yaml")).read()
    tags = re.findall(r"rocm/pytorch:\S*pytorch_release_([0-9.]+)", ci)
    assert tags and all(compat.torch_version(t) >= compat.MIN_TORCH for t in tags), tags
    assert "compat --strict" in ci


class _Sink:
    enabled = True

    def __init__(self):
        self.records = []

    def log(self, r):
        self.records.append(r)


def test_missing_feature_is_loud(monkeypatch, capsys):
    """A torch without the graph internals: the fallback says so (one stderr line + a metrics record)."""
    reason = "torch.cuda.CUDAGraph has no keep_graph argument"
    monkeypatch.setattr(compat, "_FEATURES", dict(compat.features(), hip_graph=reason))
    monkeypatch.setattr(compat, "_REPORTED", set())
    sink = _Sink()
    compat.report_fallback("graph paths", reason, sink)
    compat.report_fallback("graph paths", reason, sink)  # one line, two records
    err = capsys.readouterr().err
    assert err.count(f"[dgt] graph paths off: {reason}") == 1
    assert sink.records[0] == {"event": "fallback", "what": "graph paths", "reason": reason}
    assert not compat.has("hip_graph")
    with pytest.raises(RuntimeError, match="hip_graph"):
        compat.check(strict=True)


def test_engine_graph_config_without_graph_internals(monkeypatch, capsys):
    """An engine asked for graph_module on a torch without the graph internals turns it off loudly."""
    import distributed_gpu_test_amd as dgt
    from distributed_gpu_test_amd.engine import Engine
    from distributed_gpu_test_amd.config import parse_config
    monkeypatch.setattr(compat, "_FEATURES", dict(compat.features(), hip_graph="no raw_cuda_graph"))
    monkeypatch.setattr(compat, "_REPORTED", set())
    dgt.init_distributed()
    m = torch.nn.Sequential(torch.nn.Linear(4, 8), torch.nn.ReLU(), torch.nn.Linear(8, 1))
    cfg = parse_config({"train_batch_size": 4, "amd": {"graph_module": True}}, 1)
    e = Engine(m, cfg, device=torch.device("cpu"))
    # (on the CPU graph_module is off anyway; the report comes from the config asking for it)
    assert not e.graph_module
    e.close()
    step = Engine(m, parse_config({"train_batch_size": 4, "amd": {"hip_graph": True}}, 1),
                  device=torch.device("cpu"))
    step.graph_step(lambda x: x.sum())
    assert step.graphed is None and step.graph_fallback_reason
    step.close()
    assert "[dgt] graph paths off" in capsys.readouterr().err


def test_engine_without_bce_internals_uses_autograd(monkeypatch):
    """Without the BCE node's saved state the engine never reads it (the autograd path instead)."""
    from distributed_gpu_test_amd import engine
    z = torch.zeros(3, requires_grad=True)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(z, torch.ones(3))
    monkeypatch.setattr(compat, "_FEATURES", dict(compat.features(), torch_bce_node="missing"))
    assert not engine._torch_mean_bce(loss.grad_fn)
    monkeypatch.setattr(compat, "_FEATURES", dict(compat.features(), torch_bce_node=""))
    assert engine._torch_mean_bce(loss.grad_fn)
