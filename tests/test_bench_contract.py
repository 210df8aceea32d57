"""bench.py's driver contract on the CPU (gloo): one JSON line from rank 0 with the required keys,
exactly K timed steps after W warmup steps, whole-job aggregate value, the BASELINE metric."""
import json
import os
import subprocess
import sys

from distributed_gpu_test_amd.launch import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def _json_lines(out):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def _check(d, n, steps, warmup):
    assert REQUIRED <= set(d), REQUIRED - set(d)
    baseline = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == baseline["metric"]
    assert d["n_gpus"] == n and d["steps"] == steps and d["warmup"] == warmup
    assert d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # whole-job aggregate: iterations summed over ranks
    assert abs(d["value"] - n * 1e3 / d["ms_per_step"]) / d["value"] < 0.02
    cfg = d["config"]
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(cfg)
    assert cfg["parallelism"] == f"dp{n}" and cfg["global_batch"] == 4 * n
    assert d["params_consistent_across_ranks"] is True


def test_bench_single_process_cpu():
    env = dict(os.environ, DGT_QUIET="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "40", "--warmup", "5"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    _check(lines[0], 1, 40, 5)
    assert lines[0]["config"]["closing_barrier"] == "none (1 rank)"


def test_bench_same_run_baseline_cpu():
    """The headline's same-run baseline (the reference loop on torch) fills ``vs_baseline``."""
    env = dict(os.environ, DGT_QUIET="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "40", "--warmup", "5",
                        "--force-baselines", "--baseline-steps", "30"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_lines(r.stdout)[-1]
    _check(d, 1, 40, 5)
    b = d["baseline"]
    assert b["impl"] == "engine" and b["steps"] == 30 and b["warmup"] == 20 and b["iters_per_s"] > 0
    # two windows, the fastest is the baseline's rate
    assert len(b["windows_iters_per_s"]) == 2 and b["iters_per_s"] == max(b["windows_iters_per_s"])
    assert abs(d["vs_baseline"] - d["global_steps_per_sec"] / b["iters_per_s"]) < 0.02 * d["vs_baseline"] + 0.01
    assert d["baselines"] == {}  # no secondary block on the CPU, so no secondary baseline either


def test_attach_baselines_keys():
    import bench
    sec = {"bf16_mlp": {"iters_per_s": 1500.0}, "fp32_engine_mlp": {"error": "x"}}
    bench.attach_baselines(sec, {"headline": {"iters_per_s": 2.0, "impl": "engine"},
                                 "bf16_mlp": {"iters_per_s": 750.0, "impl": "torch-autocast-bf16"},
                                 "fp32_engine_mlp": {"iters_per_s": 10.0, "impl": "torch-fp32"}})
    assert sec["bf16_mlp"]["torch_baseline_iters_per_s"] == 750.0 and sec["bf16_mlp"]["speedup"] == 2.0
    assert sec["bf16_mlp"]["torch_baseline_impl"] == "torch-autocast-bf16"
    assert "speedup" not in sec["fp32_engine_mlp"]


def test_bench_two_ranks_gloo_cpu():
    env = dict(os.environ, DGT_QUIET="1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
           f"--master-port={free_port()}", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "30",
           "--warmup", "3", "--force-baselines", "--baseline-steps", "20"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    _check(lines[0], 2, 30, 3)
    # no IPC mailboxes on the CPU: the process group's barrier brackets the timed region
    assert lines[0]["config"]["closing_barrier"] == "process-group"
    # the same-run baseline at N = 2 (its all-reduce on the process group), two windows, max over ranks
    b = lines[0]["baseline"]
    assert b["steps"] == 20 and len(b["windows_iters_per_s"]) == 2 and lines[0]["vs_baseline"] > 0, b


def test_bench_self_launches_n_ranks_cpu():
    """``python bench.py --gpus 2`` with no launcher env starts its own 2 ranks (a torchrun child
    process) and relays rank 0's single JSON line; the exit code is the child's."""
    env = dict(os.environ, DGT_QUIET="1", OMP_NUM_THREADS="1")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "30",
                        "--warmup", "3"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    _check(lines[0], 2, 30, 3)
    assert lines[0]["ranks"] == 2 and lines[0]["config"]["parallelism"] == "dp2"
    assert "starting 2 ranks under torchrun" in r.stderr


def test_exchange_line_selection(monkeypatch):
    import pytest
    from distributed_gpu_test_amd.runtime.tiny_trainer import line_candidates
    monkeypatch.delenv("DGT_XCH_LINE", raising=False)
    assert line_candidates() == [3, 2]  # auto: LL3 if its stress test passes, else LL2
    monkeypatch.setenv("DGT_XCH_LINE", "ll2")
    assert line_candidates() == [2]
    monkeypatch.setenv("DGT_XCH_LINE", "ll4")
    with pytest.raises(ValueError):
        line_candidates()


def test_zero1_owner_map_partitions_every_element():
    """The fused kernel's ZeRO-1 lane ownership covers every parameter exactly once, spreads the
    elements evenly over the ranks and puts b2 on rank 0 (lane 0 writes it back)."""
    import torch
    from distributed_gpu_test_amd.models.simple_net import simple_net_numel
    from distributed_gpu_test_amd.runtime.tiny_trainer import zero1_owner_map
    for f, h in ((20, 64), (32, 64), (20, 128), (8, 16)):
        for ws in (1, 2, 3, 4, 8):
            own = zero1_owner_map(f, h, ws)
            assert own.numel() == simple_net_numel(f, h) and int(own.min()) == 0 and int(own.max()) == ws - 1
            counts = torch.bincount(own, minlength=ws)
            assert int(counts.max() - counts.min()) <= (simple_net_numel(f, h) // ws) // 2 + 16, counts
            assert int(own[-1]) == 0


def test_zero1_checksum_mismatch_detects_altered_transfers():
    """The ZeRO-1 kernel's transfer checksums: a clean epoch passes; an all-gathered parameter or a
    reduce-scattered gradient that arrived altered is named (csrc/dgt_common.h Exchange::xsum)."""
    import torch
    from distributed_gpu_test_amd.runtime.tiny_trainer import XSUM_WORDS, zero1_checksum_mismatch
    ws = 3
    g = torch.Generator().manual_seed(0)
    words = torch.randint(-2**31, 2**31 - 1, (ws, XSUM_WORDS // 2), generator=g, dtype=torch.int64)
    xs = [torch.zeros(XSUM_WORDS, dtype=torch.int32) for _ in range(ws)]
    for t in range(XSUM_WORDS // 2):
        o = (t % 64) % ws
        ag = int(words[0, t]) & 0x7fffffff
        acc = 0
        for p in range(ws):
            xs[p][2 * t] = ag  # every rank received what the owner sent
            if p != o:
                s = int(words[p, t]) & 0x7fffffff
                xs[p][2 * t + 1] = s
                acc ^= s
        xs[o][2 * t + 1] = acc
    assert zero1_checksum_mismatch(xs, ws) is None
    bad = [x.clone() for x in xs]
    bad[2][2 * 5 + 1] ^= 1  # thread 5's lane is owned by rank 2 (5 % 3): its received gradients differ
    assert "reduce-scattered to rank 2" in zero1_checksum_mismatch(bad, ws)
    bad = [x.clone() for x in xs]
    bad[1][2 * 6] ^= 1 << 20  # thread 6 owned by rank 0: rank 1 received an altered parameter
    assert "arrived altered on rank 1" in zero1_checksum_mismatch(bad, ws)


def test_sweep_error_keeps_the_headline(monkeypatch, capsys):
    """An RCCL error in the middle of the all-reduce sweep (here: dist.all_reduce raising from the
    128 KiB size on) is recorded in ``allreduce_sweep_error``; the run still exits 0 with one headline
    line that carries the sizes measured before the error."""
    import torch.distributed as dist
    import bench
    real = dist.all_reduce

    def flaky(t, *a, **k):
        if t.numel() >= 16384:
            raise RuntimeError("injected RCCL failure")
        return real(t, *a, **k)

    monkeypatch.setattr(dist, "all_reduce", flaky)
    monkeypatch.setenv("DGT_FORCE_COLLECTIVES", "1")
    monkeypatch.setenv("DGT_QUIET", "1")
    rc = bench.main(["--steps", "20", "--warmup", "3", "--force-sweep", "--sweep-max-mb", "1"])
    assert rc == 0
    lines = _json_lines(capsys.readouterr().out)
    assert len(lines) == 1
    d = lines[0]
    assert "injected RCCL failure" in d["allreduce_sweep_error"] and d["hung"] is None
    assert [r["bytes"] for r in d["allreduce_sweep"]] == [8, 32, 128, 512, 2048, 8192, 32768]
    assert d["value"] > 0 and d["steps"] == 20


def test_run_bounded_error_and_deadline():
    import time
    import bench
    assert bench.run_bounded(lambda: 7, 5.0) == (7, None, False)
    r, err, hung = bench.run_bounded(lambda: 1 / 0, 5.0)
    assert r is None and "ZeroDivisionError" in err and not hung
    t0 = time.perf_counter()
    r, err, hung = bench.run_bounded(lambda: time.sleep(30), 0.5)
    assert hung and "timeout" in err and time.perf_counter() - t0 < 5


def test_sweep_budget_stops_growing(monkeypatch):
    """The sweep stops growing the message size once its wall-clock budget is spent."""
    import torch
    import torch.distributed as dist
    import bench
    from distributed_gpu_test_amd.parallel import comm
    monkeypatch.setenv("DGT_FORCE_COLLECTIVES", "1")
    comm.init_distributed(backend="gloo")
    try:
        out = bench.allreduce_sweep(torch.device("cpu"), 1024, 1, budget_s=0.0)
        assert len(out) == 1 and out[0]["bytes"] == 8 and out[0]["busbw_GBps"] == 0.0
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_secondary_block_cpu():
    """A secondary block (here a small MLPTrainer on the CPU) reports its own timing keys."""
    import argparse
    import torch
    import bench
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    from distributed_gpu_test_amd.runtime.mlp_trainer import MLPTrainer
    args = argparse.Namespace(secondary_steps=3, secondary_warmup=1)
    dev = torch.device("cpu")
    blk = bench.run_secondary("bf16_mlp", "small", lambda: MLPTrainer(SyntheticMLP(128, 2), batch_size=128,
                                                                      device=dev, bucket_mb=0.01), args, dev, 1)
    assert blk["steps"] == 3 and blk["ms_per_step"] > 0 and blk["iters_per_s"] > 0
    assert blk["model_tflops"] >= 0 and blk["bucket_mb"] == 0.01 and blk["mean_loss"] > 0


def test_engine_config_knobs():
    import argparse
    import bench
    a = argparse.Namespace(ds_config=None, bucket_mb=8.0, oneshot_max_bytes=4096)
    cfg = bench.engine_config(a, os.path.join(ROOT, "configs", "ds_bench_mlp_fp32.json"))
    assert cfg["zero_optimization"]["reduce_bucket_size"] == 2 * 1024 * 1024
    assert cfg["amd"]["oneshot_max_bytes"] == 4096 and cfg["amd"]["fused_linear"] is True
    cfg = bench.engine_config(argparse.Namespace(ds_config=None, bucket_mb=None, oneshot_max_bytes=None), None)
    assert cfg["train_batch_size"] == 64  # the reference's in-code dict


def test_bench_sweep_hang_still_prints_headline():
    """A hung collective in the sweep (rank 1 wedged) ends every rank at the sweep's deadline; rank 0
    prints the headline line with ``hung`` set and the job exits 0 -- the scaling point survives."""
    import time
    env = dict(os.environ, DGT_QUIET="1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
           f"--master-port={free_port()}", os.path.join(ROOT, "tests", "bench_hang_worker.py"), "--gpus", "2",
           "--steps", "20", "--warmup", "3", "--force-sweep", "--sweep-max-mb", "1", "--sweep-deadline-s", "8"]
    t0 = time.perf_counter()
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["hung"] == "allreduce_sweep" and "timeout" in d["allreduce_sweep_error"]
    assert d["value"] > 0 and d["ranks"] == 2
    assert time.perf_counter() - t0 < 120
