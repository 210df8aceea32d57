"""Whole-step fuzz diagnosis: check after every step, print where the engine leaves torch's trajectory."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_engine_fuzz as f  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "whole_step"
for seed in (0, 1, 2):
    try:
        f._fuzz(seed, mode, steps=80, check_every=1)
        print("seed", seed, "ok", flush=True)
    except AssertionError as e:
        print("seed", seed, "FAIL", e, flush=True)
