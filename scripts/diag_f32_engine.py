#!/usr/bin/env python3
"""fp32 engine SyntheticMLP(1024, 4) gradients vs plain PyTorch after one step, per parameter
(relative L2 and worst element relative to the gradient's scale), under: the default path, the
wgrad's fused row sums replaced by the column-sum pass, and the autograd backward instead of the
engine's direct one.  Set DGT_F32_SMALL_KGROUPS in the environment for the k-group arm."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd import initialize  # noqa: E402
from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP, synthetic_batch_data  # noqa: E402
from distributed_gpu_test_amd.ops import linear as lin  # noqa: E402


def run(tag, rowsum=True, direct=True):
    lin._FUSED_ROWSUM = rowsum
    torch.manual_seed(0)
    model = SyntheticMLP(1024, 4)
    ref = copy.deepcopy(model).cuda()
    cfg = {"train_micro_batch_size_per_gpu": 1024, "gradient_accumulation_steps": 1,
           "zero_optimization": {"stage": 0}, "optimizer": {"type": "Adam", "params": {"lr": 1e-4}},
           "amd": {"fused_linear": True, "direct_backward": direct}}
    engine, _, _, _ = initialize(model=model, config=cfg)
    x, y = synthetic_batch_data(1024, 1024, 7)
    x, y = x.cuda(), y.cuda()
    crit = torch.nn.BCEWithLogitsLoss()
    loss = crit(engine(x).view(-1), y)
    engine.backward(loss)
    rl = crit(ref(x).view(-1), y)
    rl.backward()
    torch.cuda.synchronize()
    out = []
    for (name, p), q in zip(model.named_parameters(), ref.parameters()):
        rel = float((p.grad - q.grad).norm() / q.grad.norm().clamp_min(1e-30))
        worst = float((p.grad - q.grad).abs().max() / q.grad.abs().max().clamp_min(1e-30))
        out.append(f"{name} {rel:.2e}/{worst:.2e}")
    print(tag, f"kg={os.environ.get('DGT_F32_SMALL_KGROUPS', 'auto')}", f"direct={engine.direct_backwards}",
          " ".join(out), flush=True)
    engine.close()


run("default")
run("colsum", rowsum=False)
run("autograd", direct=False)
