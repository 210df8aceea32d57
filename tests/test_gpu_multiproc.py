"""GPU multi-rank rehearsal on ONE MI355X: 2 ranks share the card over gloo, exercising the IPC
mailboxes (hipIpcGetMemHandle / hipIpcOpenMemHandle across processes) and the in-kernel one- and
two-shot gradient exchanges of the fused trainer.  The 8-GPU xGMI run happens only in the driver's scaling
bench; these tests pin the protocol (LL tags, parities, rank-order sums) on real hardware."""
import os
import re
import subprocess
import sys

import pytest

from distributed_gpu_test_amd.launch import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE2 = [0.5126, 0.2219, 0.1250, 0.0857, 0.0741]
ORACLE = {4: [0.5857, 0.3375, 0.1943, 0.1321, 0.0969], 8: [0.6378, 0.4770, 0.3251, 0.2162, 0.1515]}
pytestmark = pytest.mark.gpu


def run(nproc, script, *args, env=None, timeout=300):
    e = dict(os.environ)
    e.update({"DGT_QUIET": "1", "DGT_BACKEND": "gloo", "OMP_NUM_THREADS": "1", "DGT_EXCHANGE_TIMEOUT_S": "20"})
    e.update(env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, script), *args]
    return subprocess.run(cmd, cwd=ROOT, env=e, capture_output=True, text=True, timeout=timeout)


def losses(out):
    return [float(m) for m in re.findall(r"Avg loss: ([0-9.]+)", out)]


def test_fused_ipc_exchange_two_ranks_one_gpu(tmp_path):
    r = run(2, "train.py", "--impl", "fused", "--epochs", "3", "--save-dir", str(tmp_path))
    assert r.returncode == 0, r.stderr[-4000:]
    assert "exchange=ipc-oneshot-xgmi" in r.stderr, r.stderr[-2000:]
    assert losses(r.stdout) == ORACLE2[:3]


def test_stepwise_two_ranks_one_gpu(tmp_path):
    r = run(2, "train.py", "--impl", "stepwise", "--epochs", "2", "--no-save")
    assert r.returncode == 0, r.stderr[-4000:]
    assert losses(r.stdout) == ORACLE2[:2]


def test_engine_oneshot_two_ranks_one_gpu(tmp_path):
    r = run(2, "train.py", "--impl", "engine", "--epochs", "2", "--no-save")
    assert r.returncode == 0, r.stderr[-4000:]
    assert "oneshot=yes" in r.stderr, r.stderr[-2000:]
    assert losses(r.stdout) == ORACLE2[:2]


def test_engine_fused_linear_two_ranks_one_gpu(tmp_path):
    """Kernel injection with in-place gradient accumulation: the bucket hooks still fire (one-shot
    all-reduce per bucket) and the run prints the ws=2 oracle."""
    import json
    cfg = tmp_path / "ds.json"
    cfg.write_text(json.dumps({"train_batch_size": 64, "gradient_accumulation_steps": 1,
                               "zero_optimization": {"stage": 0}, "amd": {"fused_linear": True}}))
    r = run(2, "train.py", "--impl", "engine", "--epochs", "2", "--no-save", "--deepspeed_config", str(cfg))
    assert r.returncode == 0, r.stderr[-4000:]
    assert losses(r.stdout) == ORACLE2[:2]


def test_engine_graph_module_two_ranks_one_gpu(tmp_path):
    """amd.graph_module under two ranks: the graphed backward still fires the bucket hooks, the
    gradients are averaged across ranks and the run prints the ws=2 oracle."""
    r = run(2, "train.py", "--impl", "engine", "--epochs", "2", "--no-save",
            "--deepspeed_config", os.path.join(ROOT, "configs", "ds_graph_module.json"))
    assert r.returncode == 0, r.stderr[-4000:]
    assert losses(r.stdout) == ORACLE2[:2]


def test_bench_two_ranks_one_gpu():
    r = run(2, "bench.py", "--gpus", "2", "--steps", "3000", "--warmup", "300", "--no-sweep")
    assert r.returncode == 0, r.stderr[-4000:]
    import json
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    # two processes on one card: n_gpus counts physical devices, ranks counts processes
    assert out["n_gpus"] == 1 and out["ranks"] == 2 and out["oversubscribed"] is True
    assert out["params_consistent_across_ranks"] is True
    assert out["config"]["exchange"] == "ipc-oneshot-xgmi"
    assert out["config"]["closing_barrier"] == "ipc-device"
    print(line)


def test_bench_driver_shape_two_ranks_device_barrier():
    """The driver's --steps 20 --warmup 5 shape at 2 ranks: the device barrier brackets the timed
    region, and a process-group-barrier run agrees on the trained parameters' consistency."""
    import json
    for env, kind in (({}, "ipc-device"), ({"DGT_BENCH_PG_BARRIER": "1"}, "process-group")):
        r = run(2, "bench.py", "--gpus", "2", "--steps", "20", "--warmup", "5", "--no-sweep", env=env)
        assert r.returncode == 0, r.stderr[-4000:]
        out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
        assert out["config"]["closing_barrier"] == kind and out["params_consistent_across_ranks"] is True
        assert out["steps"] == 20 and out["warmup"] == 5


def test_corrupted_exchange_fails_train_py(tmp_path):
    """--fail-at 0:37:corrupt makes rank 0's fused kernel send rank 1 one wrong gradient payload at
    step 37: training itself runs through, and the end-of-epoch replica check must fail the job."""
    r = run(2, "train.py", "--impl", "fused", "--epochs", "2", "--no-save", "--fail-at", "0:37:corrupt")
    assert r.returncode != 0, r.stdout[-2000:]
    assert "replicas diverged" in r.stderr, r.stderr[-3000:]
    assert "exchange=ipc-oneshot-xgmi" in r.stderr
    assert "Training completed." not in r.stdout


def test_corrupted_exchange_falls_back_in_bench():
    """A replica divergence after the IPC-exchange run is detected on every rank; bench.py then
    re-runs the timed region on the RCCL path (the corrupt fault does not touch it), says so on
    stderr and in the JSON, and reports the consistent RCCL-path number."""
    import json
    r = run(2, "bench.py", "--gpus", "2", "--steps", "200", "--warmup", "20", "--no-sweep",
            env={"DGT_FAIL_AT": "1:100:corrupt"})
    assert r.returncode == 0, r.stderr[-4000:]
    assert "re-running on the RCCL path" in r.stderr
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert "parameters differ across ranks" in out["ipc_fallback_reason"]
    assert out["params_consistent_across_ranks"] is True
    assert not out["config"]["exchange"].startswith("ipc")


def test_oneshot_sweep_two_ranks_one_gpu():
    """The standalone LL one-shot all-reduce at every sweep size (64 B .. 1 MiB) gives exact sums."""
    r = run(2, "bench.py", "--gpus", "2", "--steps", "200", "--warmup", "20")
    assert r.returncode == 0, r.stderr[-4000:]
    import json
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    sweep = out["oneshot_xgmi_sweep"]
    assert sweep and sweep[-1]["bytes"] == 1024 * 1024
    assert all(row["correct"] for row in sweep), sweep
    print(json.dumps(sweep))


def test_engine_zero1_two_ranks_one_gpu(tmp_path):
    """ZeRO-1 on HIP tensors: reduce-scatter into the shard, fused Adam on the shard, all-gather."""
    r = run(2, "train.py", "--impl", "engine", "--deepspeed_config", os.path.join(ROOT, "configs", "ds_zero1.json"),
            "--epochs", "2", "--save-dir", str(tmp_path))
    assert r.returncode == 0, r.stderr[-4000:]
    assert losses(r.stdout) == ORACLE2[:2]
    tag = tmp_path / "epoch2" / "global_step500"
    assert (tag / "zero_pp_rank_1_mp_rank_00_optim_states.pt").exists()


def test_bench_mlp_zero1_two_ranks_one_gpu():
    """bf16 MLP with ZeRO-1 (reduce-scatter, shard Adam, all-gather) on HIP tensors: ranks agree."""
    r = run(2, "bench.py", "--gpus", "2", "--model", "mlp", "--width", "512", "--depth", "2", "--batch", "256",
            "--zero-stage", "1", "--steps", "20", "--warmup", "2", "--no-sweep")
    assert r.returncode == 0, r.stderr[-4000:]
    import json
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["params_consistent_across_ranks"] is True
    assert "reducescatter+allgather" in out["config"]["exchange"]


@pytest.mark.parametrize("mode", ["twoshot", "oneshot"])
@pytest.mark.parametrize("ws", [4, 8])
def test_fused_ipc_exchange_many_ranks_one_gpu(tmp_path, ws, mode):
    """The 4- and 8-rank exchanges (every mailbox slot) on one card, both protocols: the code path
    the 8 x MI355X scaling run takes (one-shot by default), checked against the survey's oracle.
    Both sum in rank order, so both print the same oracle digits."""
    r = run(ws, "train.py", "--impl", "fused", "--epochs", "2", "--no-save", timeout=600, env={"DGT_XCH": mode})
    assert r.returncode == 0, r.stderr[-4000:]
    assert f"exchange=ipc-{mode}-xgmi" in r.stderr, r.stderr[-2000:]
    assert losses(r.stdout) == ORACLE[ws][:2]


def test_twoshot_matches_oneshot_bitwise_four_ranks(tmp_path):
    """The two-shot's owners sum every rank in rank order, as the one-shot does: parameters after
    an epoch are bit-identical between the protocols."""
    import torch
    out = {}
    for mode in ("oneshot", "twoshot"):
        d = tmp_path / mode
        r = run(4, "train.py", "--impl", "fused", "--epochs", "1", "--save-dir", str(d), env={"DGT_XCH": mode})
        assert r.returncode == 0, r.stderr[-4000:]
        ck = [p for p in d.rglob("*.pt")]
        assert ck, list(d.rglob("*"))
        out[mode] = {p.relative_to(d).as_posix(): torch.load(p, map_location="cpu", weights_only=True) for p in ck}
    assert out["oneshot"].keys() == out["twoshot"].keys()
    a, b = _flat_tensors(out["oneshot"]), _flat_tensors(out["twoshot"])
    assert a.keys() == b.keys() and any("module" in k for k in a), sorted(a)[:8]
    for k in a:
        assert torch.equal(a[k], b[k]), k


def _flat_tensors(obj, prefix=""):
    """Every tensor inside nested dicts / lists, keyed by its path."""
    import torch
    if torch.is_tensor(obj):
        return {prefix: obj}
    out = {}
    items = obj.items() if isinstance(obj, dict) else enumerate(obj) if isinstance(obj, (list, tuple)) else ()
    for k, v in items:
        out.update(_flat_tensors(v, f"{prefix}/{k}"))
    return out


def test_corrupted_twoshot_exchange_fails_train_py():
    """Two-shot at 4 ranks: rank 0 all-gathers one wrong sum to rank 1 only; the replica check
    must fail the job."""
    r = run(4, "train.py", "--impl", "fused", "--epochs", "1", "--no-save", "--fail-at", "0:37:corrupt",
            env={"DGT_XCH": "twoshot"})
    assert r.returncode != 0, r.stdout[-2000:]
    assert "exchange=ipc-twoshot-xgmi" in r.stderr
    assert "replicas diverged" in r.stderr, r.stderr[-3000:]


def test_bench_eight_ranks_one_gpu():
    r = run(8, "bench.py", "--gpus", "8", "--steps", "2000", "--warmup", "200", "--no-sweep", timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    import json
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 1 and out["ranks"] == 8 and out["oversubscribed"] is True
    assert out["params_consistent_across_ranks"] is True
    assert out["config"]["exchange"] == "ipc-oneshot-xgmi"
    print(json.dumps(out))


@pytest.mark.parametrize("ws", [2, 3, 4])
def test_fused_exchange_every_shape(ws):
    """Every compiled (features, hidden) shape, dense (F = 20, 32, 8) and wide (H = 128) payload
    layouts, through the in-kernel exchange: matches the stepwise trainer to fp32 rounding and the
    ranks stay bit-identical."""
    import json
    r = run(ws, "tests/xch_shapes_worker.py", timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("RESULT ")][-1][7:])
    assert len(res) == 4, res
    for shape, row in res.items():
        assert row["exchange"] == "ipc-oneshot-xgmi", (shape, row)
        assert row["consistent"], (shape, row)
        assert row["max_abs_diff"] < 1e-5, (shape, row)
    print(json.dumps(res))
