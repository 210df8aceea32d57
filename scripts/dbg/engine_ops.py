"""Which aten ops launch the engine bf16 MLP step's large elementwise kernels (shapes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import json  # noqa: E402

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP  # noqa: E402
from distributed_gpu_test_amd.runtime.engine_mlp import EngineMLPTrainer  # noqa: E402

cfg = json.load(open("configs/ds_bench_mlp_bf16.json"))
torch.manual_seed(0)
tr = EngineMLPTrainer(SyntheticMLP(4096, 4), 1024, 4, cfg)
for _ in range(3):
    tr.run_plan(*[t[:1] for t in tr.epoch_plan(1)])
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    tr.run_plan(*[t[:1] for t in tr.epoch_plan(1)])
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=30, max_name_column_width=40,
                                                         max_shapes_column_width=90))
