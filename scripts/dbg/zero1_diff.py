"""Debug: where do the fused one-shot and ZeRO-1 runs differ (ws = 3, 20x64)?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("DGT_QUIET", "1")
import torch  # noqa: E402

from distributed_gpu_test_amd.data import make_synthetic_data  # noqa: E402
from distributed_gpu_test_amd.models import SimpleNet  # noqa: E402
from distributed_gpu_test_amd.parallel import comm  # noqa: E402
from distributed_gpu_test_amd.runtime.tiny_trainer import TinyMLPTrainer  # noqa: E402


def train(zero, steps, n=512):
    x, y = make_synthetic_data(n, 20, 7)
    torch.manual_seed(11)
    tr = TinyMLPTrainer(SimpleNet(20, 64), x, y, 4, impl="fused", device=torch.device("cuda", 0), zero_stage=zero)
    plan, counts = tr.epoch_plan(1)
    tr.run_plan(plan[:steps], counts[:steps])
    torch.cuda.synchronize()
    p = tr.params[: tr.numel].detach().clone().cpu()
    tr.close()
    return p, counts[:steps].tolist()


comm.init_distributed(backend="gloo")
for steps in (1, 2, 10, 42, 43):
    p0, c = train(0, steps)
    p1, _ = train(1, steps)
    d = (p0 - p1).abs()
    idx = torch.nonzero(d).view(-1)[:12].tolist()
    if comm.get_rank() == 0:
        print(f"steps={steps} counts_tail={c[-2:]} ndiff={int((d > 0).sum())} max={float(d.max()):.3g} idx={idx}",
              flush=True)
comm.destroy()
