"""Runs the engine on a small MLP for each DeepSpeed config in a JSON list and saves the final
parameters (one process: with the GPU hidden it is the CPU reference for tests/test_gpu_train.py)."""
import json
import os
import sys

import torch

os.environ.setdefault("DGT_QUIET", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_gpu_test_amd as dgt  # noqa: E402


def mlp(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(32, 128), torch.nn.ReLU(), torch.nn.Linear(128, 1))


def run_engine(cfg, n=12, seed=5):
    g = torch.Generator().manual_seed(seed)
    engine, _, _, _ = dgt.initialize(model=mlp(), config=cfg)
    dev = engine.device
    crit = torch.nn.BCEWithLogitsLoss()
    for _ in range(n):
        x = torch.randn(16, 32, generator=g).to(dev)
        y = (torch.rand(16, 1, generator=g) > 0.5).float().to(dev)
        engine.backward(crit(engine(x).float(), y))
        engine.step()
    out = torch.nn.utils.parameters_to_vector(engine.module.parameters()).detach().float().cpu()
    engine.close()
    return out, dev.type


if __name__ == "__main__":
    cfgs = json.loads(open(sys.argv[1]).read())
    res = [run_engine(c) for c in cfgs]
    torch.save({"params": [r[0] for r in res], "device": [r[1] for r in res]}, sys.argv[2])
