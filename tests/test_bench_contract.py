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


def test_bench_two_ranks_gloo_cpu():
    env = dict(os.environ, DGT_QUIET="1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
           f"--master-port={free_port()}", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "30",
           "--warmup", "3"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    _check(lines[0], 2, 30, 3)
    # no IPC mailboxes on the CPU: the process group's barrier brackets the timed region
    assert lines[0]["config"]["closing_barrier"] == "process-group"


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
