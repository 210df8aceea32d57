"""torchrun worker for test_multiproc_cpu: the bf16 MLP trainer with zero_stage 0 and 1 on the
same data; prints both parameter vectors' checksums and their max difference (rank 0)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP  # noqa: E402
from distributed_gpu_test_amd.parallel import comm  # noqa: E402
from distributed_gpu_test_amd.runtime.mlp_trainer import MLPTrainer  # noqa: E402


def run(stage, device, bucket_mb=None):
    torch.manual_seed(3)
    tr = MLPTrainer(SyntheticMLP(width=128, depth=2), batch_size=64, n_batches=2, lr=1e-3, device=device,
                    zero_stage=stage, bucket_mb=bucket_mb)
    for s in range(4):
        tr.step(s)
    return tr.params.clone(), tr


def main():
    comm.init_distributed()
    device = torch.device("cpu")
    p0, _ = run(0, device)
    p1, t1 = run(1, device)
    ref = p1.clone()
    torch.distributed.broadcast(ref, 0)
    diff = (p0 - p1).abs().max().item()
    rank_diff = (ref - p1).abs().max().item()
    # gradient buckets of other sizes: a layer split over several collectives (0.01 MiB) and both
    # layers in one (1 MiB) give the per-layer result bit for bit
    bdiff = max((p0 - run(0, device, mb)[0]).abs().max().item() for mb in (0.01, 1.0))
    nb = len(run(0, device, 0.01)[1].buckets)
    if comm.get_rank() == 0:
        print(f"RESULT diff={diff:.3e} rank_diff={rank_diff:.3e} shard={t1.master_w.numel()} "
              f"full={t1.total_w} exchange={t1.exchange} bucket_diff={bdiff:.3e} small_buckets={nb}", flush=True)
    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
