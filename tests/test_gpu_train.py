"""End to end on one MI355X: the reference CLI (`train.py`, single process, no launcher) on the
fused kernel and on the generic engine, checkpoint + resume, the engine's less common DeepSpeed
options on the GPU against the same engine on the CPU, and the health report."""
import json
import os
import re
import subprocess
import sys

import pytest
import torch

os.environ.setdefault("DGT_QUIET", "1")
import distributed_gpu_test_amd as dgt  # noqa: E402

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_WS1 = [0.4301, 0.1461, 0.0865, 0.0637, 0.0516]  # SURVEY §6.2, rank-0 "Avg loss" per epoch


def _train(*args, timeout=240):
    env = dict(os.environ, DGT_QUIET="1", MASTER_ADDR="127.0.0.1")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "train.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _losses(stdout):
    return [float(m) for m in re.findall(r"Epoch\s+\d+ finished\. Avg loss: ([0-9.]+)", stdout)]


def test_train_py_fused_reproduces_oracle_and_saves(tmp_path):
    r = _train("--save-dir", str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "impl=fused" in r.stderr
    assert _losses(r.stdout) == ORACLE_WS1
    assert r.stdout.count("Training completed.") == 1
    for e in range(1, 6):  # 2000 samples / batch 4 = 500 steps per epoch
        d = tmp_path / f"epoch{e}"
        assert (d / "latest").read_text() == f"global_step{500 * e}"
        assert (d / f"global_step{500 * e}" / "mp_rank_00_model_states.pt").exists()


def test_train_py_fused_resume_continues_identically(tmp_path):
    part = _train("--epochs", "2", "--save-dir", str(tmp_path))
    assert part.returncode == 0, part.stderr[-3000:]
    res = _train("--epochs", "4", "--resume", "--save-dir", str(tmp_path))
    assert res.returncode == 0, res.stderr[-3000:]
    assert _losses(part.stdout) == ORACLE_WS1[:2]
    assert _losses(res.stdout) == ORACLE_WS1[2:4]


def test_train_py_zero1_config_runs_on_fused_kernel(tmp_path):
    """BASELINE config #5's DeepSpeed ZeRO-1 JSON on one GPU: train.py picks the fused kernel (a
    one-rank ZeRO-1 has nothing to shard), prints the oracle and writes a zero_pp_rank_0 shard that
    zero_to_fp32 consolidates to the module weights; --resume continues from it."""
    from distributed_gpu_test_amd.utils.zero_to_fp32 import consolidate
    cfg = os.path.join(ROOT, "configs", "ds_zero1.json")
    r = _train("--epochs", "2", "--save-dir", str(tmp_path), "--deepspeed_config", cfg)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "impl=fused" in r.stderr and "zero_stage=1" in r.stderr, r.stderr[-2000:]
    assert _losses(r.stdout) == ORACLE_WS1[:2]
    tag = tmp_path / "epoch2" / "global_step1000"
    assert (tag / "zero_pp_rank_0_mp_rank_00_optim_states.pt").exists()
    full = consolidate(str(tmp_path / "epoch2"))
    mod = torch.load(tag / "mp_rank_00_model_states.pt", weights_only=True)["module"]
    for k, v in mod.items():
        assert torch.equal(full[k], v.float()), k
    res = _train("--epochs", "3", "--resume", "--save-dir", str(tmp_path), "--deepspeed_config", cfg)
    assert res.returncode == 0, res.stderr[-3000:]
    assert _losses(res.stdout) == ORACLE_WS1[2:3]


def test_bench_zero1_driver_shape():
    """bench.py --zero-stage 1 at the driver's shape on one GPU: the CLI's ZeRO-1 selection reaches
    the fused kernel and keeps >= 300k it/s.  At one rank nothing is sharded (the owner shard is the
    whole vector), so this pins the plumbing only; the sharded exchange itself is covered by the
    multi-rank rehearsals in tests/test_gpu_multiproc.py.  The launcher variables are scrubbed: the
    child must resolve as a bare single process whatever this pytest process carries."""
    env = dict(os.environ, DGT_QUIET="1")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT", "GROUP_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "20", "--warmup", "5",
                        "--zero-stage", "1"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["config"]["zero_stage"] == 1 and out["config"]["impl"] == "fused"
    assert out["value"] >= 300_000, out["value"]
    print(out["value"])


def test_train_py_engine_on_gpu_reproduces_oracle(tmp_path):
    r = _train("--impl", "engine", "--epochs", "2", "--no-save")
    assert r.returncode == 0, r.stderr[-3000:]
    assert _losses(r.stdout) == ORACLE_WS1[:2]


ENGINE_CFGS = {
    "gas2-clip": {"train_batch_size": 32, "gradient_accumulation_steps": 2, "gradient_clipping": 0.5},
    "zero2-clip": {"train_batch_size": 16, "zero_optimization": {"stage": 2}, "gradient_clipping": 1.0},
    "adamw": {"train_batch_size": 16, "optimizer": {"type": "AdamW", "params": {"lr": 3e-3, "weight_decay": 0.05}}},
    "warmuplr": {"train_batch_size": 16, "optimizer": {"type": "Adam", "params": {"lr": 2e-3}},
                 "scheduler": {"type": "WarmupLR", "params": {"warmup_num_steps": 4, "warmup_max_lr": 2e-3}}},
}


def test_engine_options_gpu_match_cpu(tmp_path):
    """The HIP path (fused Adam, device-side clip coefficient, flat buckets) vs the same engine on
    the CPU (plain PyTorch ops; a subprocess with the GPU hidden), fp32."""
    names = list(ENGINE_CFGS)
    cfgs = [dict(ENGINE_CFGS[n]) for n in names]
    for c in cfgs:
        c.setdefault("optimizer", {"type": "Adam", "params": {"lr": 2e-3}})
    (tmp_path / "cfgs.json").write_text(json.dumps(cfgs))
    worker = os.path.join(ROOT, "tests", "engine_cfg_worker.py")
    outs = {}
    for side, hide in (("gpu", False), ("cpu", True)):
        env = dict(os.environ, DGT_QUIET="1", MASTER_ADDR="127.0.0.1")
        for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
            env.pop(k, None)
        if hide:
            env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
        r = subprocess.run([sys.executable, worker, str(tmp_path / "cfgs.json"), str(tmp_path / f"{side}.pt")],
                           cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        outs[side] = torch.load(tmp_path / f"{side}.pt", weights_only=True)
    assert outs["gpu"]["device"] == ["cuda"] * len(names) and outs["cpu"]["device"] == ["cpu"] * len(names)
    for n, got, want in zip(names, outs["gpu"]["params"], outs["cpu"]["params"]):
        torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-5, msg=lambda m: f"{n}: {m}")


def _mlp(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(32, 128), torch.nn.ReLU(), torch.nn.Linear(128, 1))


def test_engine_fp16_loss_scaling_gpu():
    m = _mlp(1)
    cfg = {"train_batch_size": 16, "fp16": {"enabled": True, "initial_scale_power": 8},
           "optimizer": {"type": "Adam", "params": {"lr": 2e-3}}}
    engine, _, _, _ = dgt.initialize(model=m.cuda(), config=cfg)
    crit = torch.nn.BCEWithLogitsLoss()
    g = torch.Generator().manual_seed(7)
    losses = []
    for _ in range(40):
        x = torch.randn(16, 32, generator=g).cuda()
        y = (x[:, :16].sum(1, keepdim=True) > 0).float()
        loss = crit(engine(x).float(), y)
        engine.backward(loss)
        engine.step()
        losses.append(float(loss.detach()))
    assert all(torch.isfinite(torch.tensor(losses)))
    assert sum(losses[-5:]) < sum(losses[:5])
    assert engine.loss_scaler is not None and engine.loss_scaler.scale > 0
    engine.close()


def test_health_report_on_gpu(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "health.py"), "--out-dir", str(tmp_path),
                        "--tag", "test", "--no-bw", "--strict"], cwd=ROOT, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    files = list(tmp_path.glob("*.json"))
    assert files, r.stdout[-2000:]
    rep = json.loads(files[0].read_text())
    assert int(rep["gpu"]["gpu_count"]) >= 1


def test_train_py_fused_profile_trace(tmp_path):
    """--profile on the default (fused) path: one profiler step per epoch launch; the kineto trace
    holds the fused kernel and, with DGT_ROCTX=1, the per-epoch roctx ranges."""
    os.environ["DGT_ROCTX"] = "1"
    try:
        r = _train("--epochs", "2", "--no-save", "--profile", str(tmp_path / "prof"))
    finally:
        os.environ.pop("DGT_ROCTX", None)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "impl=fused" in r.stderr
    text = (tmp_path / "prof" / "trace_rank0.json").read_text()
    assert "tiny_mlp_train_kernel" in text


@pytest.mark.parametrize("impl", ["auto", "engine"])
def test_train_py_model_mlp_saves_and_resumes_on_gpu(tmp_path, impl):
    """BASELINE config #2 as a train.py job on the GPU: MLPTrainer (auto) or the
    engine's MFMA chain saves DeepSpeed-layout checkpoints every epoch and --resume continues to the
    uninterrupted run's epoch loss."""
    common = ["--model", "mlp", "--width", "512", "--depth", "2", "--mlp-batches", "4", "--impl", impl]
    cfg = tmp_path / "mlp.json"
    cfg.write_text(json.dumps({"train_micro_batch_size_per_gpu": 256, "bf16": {"enabled": True},
                               "communication_data_type": "fp32", "zero_optimization": {"stage": 0},
                               "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}}))
    full = _train(*common, "--epochs", "3", "--deepspeed_config", str(cfg), "--save-dir", str(tmp_path / "a"))
    assert full.returncode == 0, full.stderr[-3000:]
    lf = _losses(full.stdout)
    assert len(lf) == 3 and lf[2] < lf[0]
    part = _train(*common, "--epochs", "2", "--deepspeed_config", str(cfg), "--save-dir", str(tmp_path / "b"))
    assert part.returncode == 0, part.stderr[-3000:]
    res = _train(*common, "--epochs", "3", "--resume", "--deepspeed_config", str(cfg), "--save-dir",
                 str(tmp_path / "b"))
    assert res.returncode == 0, res.stderr[-3000:]
    assert _losses(res.stdout) == lf[2:], (res.stdout, lf)
