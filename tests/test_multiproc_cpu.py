"""T2: end-to-end train.py under torchrun with the gloo backend (SURVEY §4 tier T2)."""
import json
import os
import re
import subprocess
import sys

import pytest

from distributed_gpu_test_amd.launch import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = {  # SURVEY §6.2 / BASELINE.md: rank-0 "Avg loss" per epoch
    1: [0.4301, 0.1461, 0.0865, 0.0637, 0.0516],
    2: [0.5126, 0.2219, 0.1250, 0.0857, 0.0741],
    4: [0.5857, 0.3375, 0.1943, 0.1321, 0.0969],
}
pytestmark = pytest.mark.slow


def run(nproc, *args, env=None, timeout=300, script="train.py"):
    e = dict(os.environ)
    e.update({"DGT_QUIET": "1", "OMP_NUM_THREADS": "1", "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""})
    e.update(env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, script), *args]
    return subprocess.run(cmd, cwd=ROOT, env=e, capture_output=True, text=True, timeout=timeout)


def epoch_losses(stdout):
    return [float(m) for m in re.findall(r"Epoch\s+\d+ finished\. Avg loss: ([0-9.]+)", stdout)]


@pytest.mark.parametrize("ws", [2, 4])
def test_train_py_matches_oracle(ws, tmp_path):
    r = run(ws, "--save-dir", str(tmp_path), "--deepspeed", "--distributed-backend", "nccl")
    assert r.returncode == 0, r.stderr[-3000:]
    assert epoch_losses(r.stdout) == ORACLE[ws]
    assert r.stdout.count("Training completed.") == 1  # printed by local_rank 0 only
    steps = {2: 250, 4: 125}[ws]
    for e in range(1, 6):
        d = tmp_path / f"epoch{e}"
        assert (d / "latest").read_text() == f"global_step{steps * e}"
        assert (d / f"global_step{steps * e}" / "mp_rank_00_model_states.pt").exists()


def test_tiny_trainer_torch_impl_matches_oracle(tmp_path):
    r = run(2, "--impl", "torch", "--epochs", "3", "--save-dir", str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert epoch_losses(r.stdout) == ORACLE[2][:3]


def test_zero1_equals_zero0_and_writes_shards(tmp_path):
    r = run(2, "--deepspeed_config", os.path.join(ROOT, "configs", "ds_zero1.json"), "--epochs", "2",
            "--save-dir", str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert epoch_losses(r.stdout) == ORACLE[2][:2]
    tag = tmp_path / "epoch2" / "global_step500"
    assert (tag / "mp_rank_00_model_states.pt").exists()
    assert (tag / "zero_pp_rank_0_mp_rank_00_optim_states.pt").exists()
    assert (tag / "zero_pp_rank_1_mp_rank_00_optim_states.pt").exists()
    # the consolidation script reproduces the module weights from the shards
    out = tmp_path / "fp32.pt"
    c = subprocess.run([sys.executable, str(tmp_path / "epoch2" / "zero_to_fp32.py"), str(tmp_path / "epoch2"),
                        str(out)], capture_output=True, text=True, timeout=120)
    assert c.returncode == 0, c.stderr
    import torch
    full = torch.load(out, weights_only=True)
    mod = torch.load(tag / "mp_rank_00_model_states.pt", weights_only=True)["module"]
    for k, v in mod.items():
        torch.testing.assert_close(full[k], v.float())


def test_resume_continues_identically(tmp_path):
    full = run(2, "--epochs", "3", "--save-dir", str(tmp_path / "a"))
    assert full.returncode == 0, full.stderr[-2000:]
    part = run(2, "--epochs", "2", "--save-dir", str(tmp_path / "b"))
    assert part.returncode == 0
    res = run(2, "--epochs", "3", "--resume", "--save-dir", str(tmp_path / "b"))
    assert res.returncode == 0, res.stderr[-2000:]
    assert epoch_losses(res.stdout) == epoch_losses(full.stdout)[2:]


def test_elastic_restart_resumes_from_checkpoint(tmp_path):
    clean = run(2, "--epochs", "3", "--save-dir", str(tmp_path / "clean"))
    assert clean.returncode == 0
    e = dict(os.environ)
    cmd_env = {"DGT_FAIL_ONCE": str(tmp_path / "fired")}
    # elastic restarts need the c10d rendezvous (static rendezvous keeps stale peer addresses)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--max-restarts=1", "--rdzv-backend=c10d", f"--rdzv-endpoint=127.0.0.1:{free_port()}",
                        "--rdzv-id=elastic-test",
                        os.path.join(ROOT, "train.py"), "--epochs", "3", "--resume", "--fail-at", "0:300",
                        "--save-dir", str(tmp_path / "elastic")],
                       cwd=ROOT, env={**e, "DGT_QUIET": "1", "OMP_NUM_THREADS": "1", "CUDA_VISIBLE_DEVICES": "",
                                      "HIP_VISIBLE_DEVICES": "", **cmd_env},
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert (tmp_path / "fired").exists()
    # first attempt printed epoch 1 and died in epoch 2; the restart resumed at epoch 2
    assert epoch_losses(r.stdout) == epoch_losses(clean.stdout)[:1] + epoch_losses(clean.stdout)[1:]


@pytest.mark.parametrize("spec", ["1:end", "0:3:exit", "*:2:abort"])
def test_fault_injection_fails_the_job(spec, tmp_path):
    r = run(2, "--epochs", "1", "--fail-at", spec, "--no-save", timeout=180)
    assert r.returncode != 0


def test_world_size_3_fails_batch_assertion():
    r = run(3, "--epochs", "1", "--no-save")
    assert r.returncode != 0
    assert "train_batch_size" in r.stderr


def test_mlp_trainer_zero1_matches_zero0():
    """bf16 MLP trainer: reduce-scatter + sharded Adam + all-gather == all-reduce + full Adam."""
    r = run(2, script=os.path.join("tests", "mlp_zero_worker.py"))
    assert r.returncode == 0, r.stderr[-3000:]
    m = re.search(r"RESULT diff=(\S+) rank_diff=(\S+) shard=(\d+) full=(\d+) exchange=(\S+)", r.stdout)
    assert m, r.stdout[-2000:]
    assert float(m.group(1)) == 0.0 and float(m.group(2)) == 0.0
    assert int(m.group(3)) * 2 == int(m.group(4))
    assert "reducescatter+allgather" in m.group(5)
    # --bucket-mb: other bucket cuts of the same all-reduce are bit-identical
    b = re.search(r"bucket_diff=(\S+) small_buckets=(\d+)", r.stdout)
    assert b and float(b.group(1)) == 0.0 and int(b.group(2)) > 2, r.stdout[-2000:]


def test_mpirun_style_launch_matches_oracle(tmp_path):
    """Ranks started the way mpirun starts them (only OMPI_COMM_WORLD_* + MASTER_* set)."""
    port = free_port()
    procs = []
    for r in range(2):
        e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
        e.update({"DGT_QUIET": "1", "OMPI_COMM_WORLD_RANK": str(r), "OMPI_COMM_WORLD_SIZE": "2",
                  "OMPI_COMM_WORLD_LOCAL_RANK": str(r), "OMPI_COMM_WORLD_LOCAL_SIZE": "2",
                  "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "OMP_NUM_THREADS": "1",
                  "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""})
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "train.py"), "--epochs", "2", "--no-save"],
                                      cwd=ROOT, env=e, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    assert all(p.returncode == 0 for p in procs), outs[0][1][-2000:] + outs[1][1][-2000:]
    assert epoch_losses(outs[0][0]) == ORACLE[2][:2]


def test_bf16_gradient_wire_error_eight_ranks():
    """bound the error an 8-rank bf16 gradient sum adds over an fp32 wire.
    Measured (gloo, CPU; RCCL's ring order emulated): fp32 wire 6e-10, bf16 wire 3.7e-3 relative
    RMS, against 1.7e-3 for rounding one fp32 gradient to bf16 at all: the bf16 wire roughly
    doubles the gradient's own bf16 error.  MLPTrainer keeps bf16 as the default wire (half the
    collective and Adam bytes, as DeepSpeed's bf16 mode does) and communication_data_type=fp32
    (fp32 gradients straight out of the wgrad epilogue) removes the accumulation error."""
    r = run(8, script="tests/bf16_wire_worker.py", timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("RESULT ")][-1][len("RESULT "):])
    print(res)
    assert res["fp32_wire_rel_rms"] < 1e-6
    # bf16 unit roundoff is 2^-9 = 1.95e-3; 7 rounded additions stay within a few of it
    assert res["bf16_wire_rel_rms"] < 8e-3 and res["bf16_ring_rel_rms"] < 8e-3
    assert res["bf16_ring_max_over_l1"] < 7 * 2.0 ** -8  # <= (ws - 1) unit roundoffs of the magnitudes
    assert 5e-4 < res["bf16_input_quant_rel_rms"] < 2e-3


def test_profile_trace_on_default_trainer_path(tmp_path):
    """--profile wraps the TinyMLPTrainer path too (the default on a GPU: one profiler step per
    fused epoch launch), not only the engine loop."""
    r = run(1, "--impl", "torch", "--epochs", "2", "--no-save", "--profile", str(tmp_path / "prof"))
    assert r.returncode == 0, r.stderr[-3000:]
    trace = tmp_path / "prof" / "trace_rank0.json"
    assert trace.exists() and trace.stat().st_size > 1000


def test_exchange_fallback_reruns_epoch_cpu(tmp_path):
    """The run-time fallback's mechanics on the CPU (the torch path emulates the fused kernel's
    ``corrupt`` fault: rank 1 receives a gradient sum off by 1.0 at step 37).  The epoch-end replica
    check sees the divergence on both ranks; both restore the epoch-start snapshot, re-run the epoch
    and the job prints the uninterrupted oracle, exits 0, and logs exchange_fallback to stderr, the
    metrics JSONL and the health log."""
    health = tmp_path / "health.jsonl"
    r = run(2, "--impl", "torch", "--epochs", "2", "--no-save", "--fail-at", "0:37:corrupt",
            env={"DGT_HEALTH_LOG": str(health), "DGT_METRICS_JSONL": str(tmp_path / "m.jsonl")})
    assert r.returncode == 0, r.stderr[-3000:]
    assert epoch_losses(r.stdout) == ORACLE[2][:2]
    assert "oversubscribed=False" in r.stderr  # CPU ranks are their own devices
    assert "exchange_fallback at epoch 1" in r.stderr and "replicas diverged" in r.stderr, r.stderr[-2000:]
    ev = [json.loads(l) for l in health.read_text().splitlines()]
    assert sorted(e["rank"] for e in ev) == [0, 1] and all(e["event"] == "exchange_fallback" for e in ev)
    assert any(json.loads(l).get("event") == "exchange_fallback" for l in (tmp_path / "m.jsonl").read_text().splitlines())


def test_exchange_fallback_strict_fails_cpu():
    r = run(2, "--impl", "torch", "--epochs", "1", "--no-save", "--fail-at", "0:37:corrupt", "--strict-exchange")
    assert r.returncode != 0, r.stderr[-2000:]  # the workers exit 2; torchrun reports the failure
    assert "[dgt] FATAL" in r.stderr and "replicas diverged" in r.stderr and "exitcode  : 2" in r.stderr
    assert "Training completed." not in r.stdout


def _mlp_cfg(tmp_path, stage):
    p = tmp_path / f"mlp_z{stage}.json"
    p.write_text(json.dumps({"train_micro_batch_size_per_gpu": 64, "gradient_accumulation_steps": 1,
                             "bf16": {"enabled": True}, "communication_data_type": "fp32",
                             "zero_optimization": {"stage": stage},
                             "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}}))
    return str(p)


def test_train_py_model_mlp_zero1_checkpoint_resume_consolidate(tmp_path):
    """BASELINE config #2 as a train.py job: --model mlp runs MLPTrainer with the
    DeepSpeed JSON's micro-batch / ZeRO stage, saves DeepSpeed-layout checkpoints every epoch and
    resumes from them bit-exactly; the ZeRO-1 shards consolidate (zero_to_fp32) to exactly the
    ZeRO-0 run's fp32 masters."""
    import torch
    from distributed_gpu_test_amd.utils.zero_to_fp32 import consolidate
    common = ["--model", "mlp", "--width", "128", "--depth", "2", "--mlp-batches", "4"]
    full = {}
    for stage in (0, 1):
        r = run(2, *common, "--epochs", "3", "--deepspeed_config", _mlp_cfg(tmp_path, stage),
                "--save-dir", str(tmp_path / f"full{stage}"))
        assert r.returncode == 0, r.stderr[-3000:]
        full[stage] = epoch_losses(r.stdout)
        assert len(full[stage]) == 3 and full[stage][2] < full[stage][0]
    assert full[0] == full[1]
    z0 = torch.load(tmp_path / "full0" / "epoch3" / "global_step12" / "mp_rank_00_model_states.pt",
                    weights_only=True)["module"]
    tag1 = tmp_path / "full1" / "epoch3" / "global_step12"
    assert (tag1 / "zero_pp_rank_1_mp_rank_00_optim_states.pt").exists()
    cons = consolidate(str(tmp_path / "full1" / "epoch3"))
    for k, v in z0.items():
        assert torch.equal(cons[k], v), k
    part = run(2, *common, "--epochs", "2", "--deepspeed_config", _mlp_cfg(tmp_path, 1),
               "--save-dir", str(tmp_path / "part"))
    assert part.returncode == 0, part.stderr[-3000:]
    res = run(2, *common, "--epochs", "3", "--resume", "--deepspeed_config", _mlp_cfg(tmp_path, 1),
              "--save-dir", str(tmp_path / "part"))
    assert res.returncode == 0, res.stderr[-3000:]
    assert epoch_losses(res.stdout) == full[1][2:]


def test_train_py_model_mlp_engine_path(tmp_path):
    """--model mlp --impl engine: the same model through initialize / backward / step."""
    r = run(1, "--model", "mlp", "--width", "128", "--depth", "2", "--mlp-batches", "4", "--epochs", "2",
            "--impl", "engine", "--deepspeed_config", _mlp_cfg(tmp_path, 0), "--save-dir", str(tmp_path / "e"))
    assert r.returncode == 0, r.stderr[-3000:]
    l = epoch_losses(r.stdout)
    assert len(l) == 2 and l[1] < l[0]
    assert (tmp_path / "e" / "epoch2" / "global_step8" / "mp_rank_00_model_states.pt").exists()


def test_reducer_launcher_thread_matches_inline():
    """The gradient reducer's launcher thread (parallel/reducer.py) issues every bucket's collective
    from one side thread in notification order: the reduced gradients are bit-identical to launching
    on the backward thread, at stage 0 and 1, with and without a wire-dtype cast; buckets follow the
    layers (a layer's weight and bias share one)."""
    r = run(2, script="tests/reducer_thread_worker.py")
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("RESULT ")][-1][7:])
    assert len(res) == 4
    for k, v in res.items():
        assert v["equal"], (k, v)
        assert v["thread_launches"] == 3 * v["buckets"] and v["inline_thread_launches"] == 0, (k, v)
        assert all(sorted(p) in ([0, 1], [2, 3], [4, 5], [6, 7], [4, 5, 6, 7], [2, 3, 4, 5, 6, 7])
                   for p in v["bucket_params"]), v["bucket_params"]
