"""GPU multi-rank rehearsal on ONE MI355X: 2-8 ranks share the card over gloo, exercising the IPC
mailboxes (hipIpcGetMemHandle / hipIpcOpenMemHandle across processes), the in-kernel one-shot and
ZeRO-1 exchanges of the fused trainer in both line formats (LL3 / LL2), the start-up stress test
and the run-time fallback to the RCCL path.  The 8-GPU xGMI run happens only in the driver's scaling
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
    e.update({"DGT_QUIET": "1", "DGT_BACKEND": "gloo", "OMP_NUM_THREADS": "1", "DGT_EXCHANGE_TIMEOUT_S": "20",
              "DGT_ALLOW_OVERSUBSCRIBE": "1"})
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
    assert out["config"]["exchange"].startswith("ipc-oneshot-xgmi")
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


@pytest.mark.parametrize("ws", [2, 8])
def test_corrupted_exchange_falls_back_train_py(tmp_path, ws):
    """--fail-at 0:37:corrupt makes rank 0's fused kernel send rank 1 one wrong gradient payload at
    step 37.  The end-of-epoch replica check sees the divergence on every rank; the job restores
    the epoch-start snapshot, re-runs the epoch on the RCCL path, prints the oracle to 4 dp, exits
    0 and logs exchange_fallback to stderr, the metrics JSONL and the health log."""
    import json
    metrics, health = tmp_path / "m_{rank}.jsonl", tmp_path / "health.jsonl"
    r = run(ws, "train.py", "--impl", "fused", "--epochs", "2", "--no-save", "--fail-at", "0:37:corrupt",
            env={"DGT_METRICS_JSONL": str(metrics), "DGT_HEALTH_LOG": str(health)}, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "exchange=ipc-oneshot-xgmi" in r.stderr
    assert "exchange_fallback at epoch 1" in r.stderr and "replicas diverged" in r.stderr, r.stderr[-3000:]
    want = ORACLE2 if ws == 2 else ORACLE[ws]
    assert losses(r.stdout) == want[:2]
    assert "Training completed." in r.stdout
    events = [json.loads(l) for l in health.read_text().splitlines()]
    assert len(events) == ws and all(e["event"] == "exchange_fallback" and e["epoch"] == 1 for e in events)
    assert all(e["to"].startswith(("graph", "stepwise")) for e in events), events
    m0 = [json.loads(l) for l in (tmp_path / "m_0.jsonl").read_text().splitlines()]
    assert any(e.get("event") == "exchange_fallback" for e in m0)


def test_corrupted_exchange_strict_fails_train_py():
    """--strict-exchange keeps the old contract: the divergence fails the job (rc 2) on every rank."""
    r = run(2, "train.py", "--impl", "fused", "--epochs", "2", "--no-save", "--fail-at", "0:37:corrupt",
            "--strict-exchange")
    assert r.returncode != 0, r.stdout[-2000:]
    assert "replicas diverged" in r.stderr, r.stderr[-3000:]
    assert "exchange_fallback" not in r.stderr
    assert "Training completed." not in r.stdout


def test_stress_selftest_reported_and_ll2_selectable(tmp_path):
    """Start-up: the exchange stress test (>= 1000 exchanges, torn-line-revealing payloads) runs
    and passes; DGT_XCH_LINE=ll2 selects the 8-byte-pair line format, which trains to the same
    oracle."""
    for line in ("auto", "ll2"):
        r = run(2, "train.py", "--impl", "fused", "--epochs", "1", "--no-save",
                env={"DGT_XCH_LINE": line, "DGT_XCH_STRESS_STEPS": "5000"})
        assert r.returncode == 0, r.stderr[-4000:]
        want = "ll2" if line == "ll2" else "ll3"
        assert f"exchange=ipc-oneshot-xgmi/{want}" in r.stderr, r.stderr[-2000:]
        assert '"test": "stress"' in r.stderr and '"steps": 5000' in r.stderr and '"max_bad_words": 0' in r.stderr
        assert losses(r.stdout) == ORACLE2[:1]


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


@pytest.mark.parametrize("zero", [0, 1])
@pytest.mark.parametrize("ws", [4, 8])
def test_fused_ipc_exchange_many_ranks_one_gpu(tmp_path, ws, zero):
    """The 4- and 8-rank exchanges (every mailbox slot) on one card, ZeRO-0 (one-shot) and ZeRO-1
    (reduce-scatter to owners, owner Adam, parameter all-gather): the code paths the 8 x MI355X
    scaling run takes, checked against the survey's oracle.  Both sum in rank order, so both print
    the same oracle digits."""
    cfg = os.path.join(ROOT, "configs", "ds_zero1.json" if zero else "ds_zero0.json")
    r = run(ws, "train.py", "--impl", "fused", "--epochs", "2", "--no-save", "--deepspeed_config", cfg, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert f"exchange=ipc-{'zero1' if zero else 'oneshot'}-xgmi" in r.stderr, r.stderr[-2000:]
    assert losses(r.stdout) == ORACLE[ws][:2]


def test_zero1_matches_zero0_bitwise_and_consolidates(tmp_path):
    """Fused ZeRO-1 at 4 ranks: parameters after an epoch are bit-identical to the one-shot
    ZeRO-0 run (owners sum every rank in rank order and apply the same Adam); each rank writes a
    zero_pp_rank shard of the elements it owns, zero_to_fp32 consolidates them to the module's
    weights, and the run resumes from the shards (epoch 2 prints the uninterrupted oracle)."""
    import torch
    from distributed_gpu_test_amd.utils.zero_to_fp32 import consolidate
    out = {}
    for zero in (0, 1):
        d = tmp_path / f"z{zero}"
        cfg = os.path.join(ROOT, "configs", "ds_zero1.json" if zero else "ds_zero0.json")
        r = run(4, "train.py", "--impl", "fused", "--epochs", "1", "--save-dir", str(d), "--deepspeed_config", cfg)
        assert r.returncode == 0, r.stderr[-4000:]
        ck = d / "epoch1"
        out[zero] = torch.load(ck / "global_step125" / "mp_rank_00_model_states.pt", map_location="cpu",
                               weights_only=True)["module"]
    for k in out[0]:
        assert torch.equal(out[0][k], out[1][k]), k
    ck = tmp_path / "z1" / "epoch1"
    for rr in range(4):
        assert (ck / "global_step125" / f"zero_pp_rank_{rr}_mp_rank_00_optim_states.pt").exists()
    full = consolidate(str(ck))
    for k, v in out[1].items():
        assert torch.equal(full[k], v.float()), k
    r = run(4, "train.py", "--impl", "fused", "--epochs", "2", "--resume", "--save-dir", str(tmp_path / "z1"),
            "--deepspeed_config", os.path.join(ROOT, "configs", "ds_zero1.json"))
    assert r.returncode == 0, r.stderr[-4000:]
    assert losses(r.stdout) == ORACLE[4][1:2]


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


def test_corrupted_zero1_exchange_falls_back():
    """ZeRO-1 at 4 ranks: rank 0 all-gathers one wrong parameter to rank 1 only; the replica check
    catches it, the moments are gathered from their owners and the epoch re-runs on RCCL."""
    r = run(4, "train.py", "--impl", "fused", "--epochs", "2", "--no-save", "--fail-at", "0:37:corrupt",
            "--deepspeed_config", os.path.join(ROOT, "configs", "ds_zero1.json"))
    assert r.returncode == 0, r.stderr[-4000:]
    assert "exchange=ipc-zero1-xgmi" in r.stderr
    assert "exchange_fallback at epoch 1" in r.stderr, r.stderr[-3000:]
    assert losses(r.stdout) == ORACLE[4][:2]


def test_bench_eight_ranks_one_gpu():
    r = run(8, "bench.py", "--gpus", "8", "--steps", "2000", "--warmup", "200", "--no-sweep", timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    import json
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 1 and out["ranks"] == 8 and out["oversubscribed"] is True
    assert out["params_consistent_across_ranks"] is True
    assert out["config"]["exchange"].startswith("ipc-oneshot-xgmi")
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
        assert row["exchange"] == "ipc-oneshot-xgmi/ll3", (shape, row)
        assert row["consistent"], (shape, row)
        assert row["max_abs_diff"] < 1e-5, (shape, row)
        # LL2 and ZeRO-1 move the same gradients: bit-identical parameters
        assert row["ll2_equal"] and row["zero1_equal"] and row["zero1_ll2_equal"], (shape, row)
    print(json.dumps(res))


def test_bench_secondary_blocks_two_ranks_one_gpu():
    """The N > 1 secondary blocks (bf16 MLP config #2, the fp32 engine MLP, ZeRO-1 config #5) run
    their multi-rank code paths before the first 8-GPU run does: two ranks on the card (gloo,
    --force-secondary, a few steps each); every block reports steps and no error."""
    import json
    r = run(2, "bench.py", "--gpus", "2", "--steps", "20", "--warmup", "5", "--no-sweep", "--force-secondary",
            "--secondary-steps", "3", "--secondary-warmup", "1", timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    for key in ("bf16_mlp", "fp32_engine_mlp", "bf16_mlp_zero1"):
        assert key in out and out[key].get("error") is None, (key, out.get(key))
        assert out[key]["steps"] == 3 and out[key]["iters_per_s"] > 0, out[key]
