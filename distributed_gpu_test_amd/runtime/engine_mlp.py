"""The bench-size SyntheticMLP through the DeepSpeed-style API, with the trainer surface that
``train.py --model mlp`` and ``bench.py --model mlp --impl dgt-engine`` drive.

Reference: the loop of ``train.py:98-117`` -- ``engine(x)``, the user's BCE-with-logits loss,
``engine.backward(loss)``, ``engine.step()`` -- on BASELINE config #2's model.  With a bf16 config
the engine runs the model on the hand-written MFMA GEMM chain (``ops/mfma_linear.py``), its Adam
on the flat fp32 masters (``ops.adam_flat_``) and its collectives on RCCL buckets.
"""
from __future__ import annotations

import torch

from .. import initialize
from ..models.synthetic_mlp import SyntheticMLP, synthetic_batch_data
from ..ops import BCEWithLogitsLoss
from ..parallel import comm


class EngineMLPTrainer:
    def __init__(self, model: SyntheticMLP, batch_size: int, n_batches: int, ds_config, seed: int = 1234):
        self.engine, _, _, _ = initialize(model=model, config=ds_config)
        self.model = model
        self.device = self.engine.device
        self.B, self.n_batches = batch_size, n_batches
        x, y = synthetic_batch_data(batch_size * n_batches, model.in_features, seed + comm.get_rank())
        # the dataset held in the compute dtype (as MLPTrainer holds it): no per-step input cast
        self.X, self.Y = x.to(self.device, self.engine.dtype), y.to(self.device)
        self.loss_acc = torch.zeros(1, dtype=torch.float64, device=self.device)
        # the framework's drop-in for nn.BCEWithLogitsLoss (one HIP kernel: loss + d loss / d logits),
        # as train.py uses on the engine path; it reads the bf16 logits as they are and adds the loss
        # into the fp64 loss log in the same kernel (sum_into)
        self.crit = BCEWithLogitsLoss(sum_into=self.loss_acc)
        world = comm.get_world_size()
        self.exchange = "none" if world == 1 else f"{comm.backend_name()}-bucketed"
        self.impl = f"dgt-engine+mfma{self.engine.fused_linear_layers}+zero{self.engine.stage}"
        self.dtype_name = {torch.float32: "fp32", torch.bfloat16: "bf16", torch.float16: "fp16"}[self.engine.dtype]
        self.zero_stage = self.engine.stage
        self.global_steps = 0

    def flops_per_step(self) -> int:
        return self.model.flops_per_sample() * self.B

    def epoch_plan(self, epoch: int):
        plan = torch.arange(self.n_batches, dtype=torch.int32).view(-1, 1)
        return plan, torch.ones(self.n_batches, dtype=torch.int32)

    def run_plan(self, plan, counts) -> None:
        for _ in range(int(plan.shape[0])):
            j = self.global_steps % self.n_batches
            x, y = self.X[j * self.B:(j + 1) * self.B], self.Y[j * self.B:(j + 1) * self.B]
            loss = self.crit(self.engine(x).view(-1), y)
            self.engine.backward(loss)
            self.engine.step()
            self.global_steps += 1

    @property
    def params(self) -> torch.Tensor:
        return self.engine.store.param_buf.detach()

    def check(self) -> None:
        pass

    def save_checkpoint(self, save_dir: str, ds_config=None) -> str:
        return self.engine.save_checkpoint(save_dir)

    def load_checkpoint(self, load_dir: str):
        out = self.engine.load_checkpoint(load_dir)
        self.global_steps = self.engine.global_steps
        return out

    def close(self) -> None:
        self.engine.close()
