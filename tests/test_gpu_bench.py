"""bench.py on the GPU as the driver runs it: the headline line plus the post-headline blocks of
BASELINE config #2 (``bf16_mlp``) and the fp32 engine MLP, and the RCCL all-reduce sweep executed
on hardware at one rank (``DGT_FORCE_COLLECTIVES=1``: a 1-rank RCCL communicator, algbw only) so the
sweep code has run before a scaling box runs it.

Reference: the headline is the loop of ``train.py:98-117``; config #2 is its model at bench scale
(SURVEY 6.4); the sweep is the per-step all-reduce of ``train.py:113`` measured rccl-tests style."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _bench(*argv, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
              "DGT_FORCE_COLLECTIVES", "DGT_BACKEND"):
        env.pop(k, None)
    env.update(env_extra or {})
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    wall = time.perf_counter() - t0
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return lines[0], wall, r.stderr


def test_driver_shape_with_secondary_blocks():
    d, wall, err = _bench("--steps", "20", "--warmup", "5")
    assert d["value"] > 100_000 and d["hung"] is None, d
    for key in ("bf16_mlp", "fp32_engine_mlp"):
        blk = d[key]
        assert "error" not in blk, (key, blk, err[-2000:])
        assert blk["iters_per_s"] > 0 and blk["model_tflops"] > 0 and blk["steps"] == 200
        assert blk["block_wall_s"] < 30, (key, blk)
    assert d["bf16_mlp"]["dtype"] == "bf16" and d["fp32_engine_mlp"]["dtype"] == "fp32"
    print(json.dumps({"wall_s": round(wall, 1), "value": d["value"],
                      **{k: {kk: d[k][kk] for kk in ("iters_per_s", "model_tflops", "block_wall_s")}
                         for k in ("bf16_mlp", "fp32_engine_mlp")}}))


def test_rccl_sweep_runs_on_one_gpu_forced():
    d, wall, err = _bench("--steps", "20", "--warmup", "5", "--no-secondary", "--sweep-max-mb", "64",
                          env_extra={"DGT_FORCE_COLLECTIVES": "1"})
    sw = d["allreduce_sweep"]
    assert d["allreduce_sweep_error"] is None and d["hung"] is None, err[-2000:]
    assert [r["bytes"] for r in sw][:3] == [8, 32, 128] and sw[-1]["bytes"] == 32 * 1024 * 1024  # sizes 8 B x 4^k up to 64 MiB
    assert all(r["algbw_GBps"] > 0 and r["busbw_GBps"] == 0.0 for r in sw)  # 1 rank: busbw 0 by convention
    print(json.dumps({"wall_s": round(wall, 1), "sweep": sw}))
