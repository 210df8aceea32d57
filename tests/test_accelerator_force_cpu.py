"""The accelerator is the single CPU/HIP selection point (reference ``get_accelerator()``,
``train.py:12,61``), and ``DGT_FORCE_COLLECTIVES`` makes a 1-rank run issue its collectives (CPU/gloo
half of tests/test_gpu_force_collectives.py)."""
import os
import subprocess
import sys

import pytest
import torch

from distributed_gpu_test_amd import accelerator

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_forced_cpu_accelerator(monkeypatch):
    monkeypatch.setenv("DGT_ACCELERATOR", "cpu")
    accelerator.reset_accelerator()
    try:
        acc = accelerator.get_accelerator()
        assert acc.name == "cpu" and acc.communication_backend_name() == "gloo"
        assert acc.device() == torch.device("cpu")
        from distributed_gpu_test_amd.parallel import comm
        monkeypatch.delenv("DGT_BACKEND", raising=False)
        assert comm.default_backend() == "gloo"
    finally:
        accelerator.reset_accelerator()


def test_bad_accelerator_name(monkeypatch):
    monkeypatch.setenv("DGT_ACCELERATOR", "cuda")
    accelerator.reset_accelerator()
    try:
        import pytest
        with pytest.raises(ValueError):
            accelerator.get_accelerator()
    finally:
        accelerator.reset_accelerator()


def test_train_py_on_forced_cpu_accelerator(tmp_path):
    """DGT_ACCELERATOR=cpu: train.py picks gloo and the CPU engine, and prints the ws=1 oracle."""
    env = dict(os.environ, DGT_ACCELERATOR="cpu", DGT_QUIET="1")
    env.pop("DGT_BACKEND", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "train.py"), "--epochs", "2", "--no-save"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "backend=gloo" in r.stderr, r.stderr[-2000:]
    assert "Epoch  1 finished. Avg loss: 0.4301" in r.stdout and "Epoch  2 finished. Avg loss: 0.1461" in r.stdout


def test_forced_collectives_engine_cpu():
    """Engine ZeRO-0 and ZeRO-1 at world size 1 on gloo: forced collectives run and change no bit."""
    code = r'''
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, %r)
import distributed_gpu_test_amd as dgt
from distributed_gpu_test_amd.parallel import comm
comm.init_distributed(backend="gloo")
calls = {"n": 0}
for name in ("all_reduce", "reduce_scatter_tensor", "all_gather_into_tensor", "broadcast"):
    f = getattr(dist, name)
    def w(*a, _f=f, **k):
        calls["n"] += 1
        return _f(*a, **k)
    setattr(dist, name, w)
out = {}
for stage in (0, 1):
    res = []
    for flag in ("0", "1"):
        os.environ["DGT_FORCE_COLLECTIVES"] = flag
        calls["n"] = 0
        torch.manual_seed(4)
        m = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 1))
        e, _, _, _ = dgt.initialize(model=m, config={"train_batch_size": 8,
                                                      "zero_optimization": {"stage": stage, "reduce_bucket_size": 1024}})
        g = torch.Generator().manual_seed(1)
        for _ in range(4):
            x, y = torch.randn(8, 16, generator=g), (torch.rand(8, 1, generator=g) > 0.5).float()
            e.backward(torch.nn.functional.binary_cross_entropy_with_logits(e(x), y))
            e.step()
        res.append((e.store.param_buf.clone(), calls["n"]))
    assert torch.equal(res[0][0], res[1][0]), stage
    assert res[1][1] > res[0][1] == 0, (stage, res[0][1], res[1][1])
print("FORCED_OK")
comm.destroy()
''' % ROOT
    env = dict(os.environ, DGT_QUIET="1", DGT_ACCELERATOR="cpu")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "FORCED_OK" in r.stdout, r.stderr[-3000:]


def test_wait_mode_validation():
    """DGT_HIP_WAIT: empty leaves the runtime default; unknown modes are rejected before any HIP call."""
    from distributed_gpu_test_amd.accelerator import set_wait_mode
    assert set_wait_mode("") is False
    with pytest.raises(ValueError):
        set_wait_mode("busy")


def test_hip_set_device_refuses_silent_oversubscription(monkeypatch):
    """a local rank beyond the visible GPUs is an error (a wrong HIP_VISIBLE_DEVICES or
    GPUS_PER_NODE), unless DGT_ALLOW_OVERSUBSCRIBE=1 asks for the one-card rehearsal's wrap."""
    import pytest
    import torch
    from distributed_gpu_test_amd.accelerator import HipAccelerator
    bound = []
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 2)
    monkeypatch.setattr(torch.cuda, "set_device", lambda i: bound.append(i))
    monkeypatch.delenv("DGT_HIP_WAIT", raising=False)
    monkeypatch.delenv("DGT_ALLOW_OVERSUBSCRIBE", raising=False)
    acc = HipAccelerator()
    acc.set_device(1)
    with pytest.raises(RuntimeError, match="no GPU of its own"):
        acc.set_device(3)
    monkeypatch.setenv("DGT_ALLOW_OVERSUBSCRIBE", "1")
    acc.set_device(3)
    assert bound == [1, 1]
