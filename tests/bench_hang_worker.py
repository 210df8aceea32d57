"""torchrun worker for test_bench_contract: rank 1's RCCL sweep hangs (it never returns), as a
wedged collective would.  Every rank must still end, and rank 0 must still print its headline line
with ``hung`` set -- the sweep runs in a worker thread under a hard deadline."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

_real = bench.allreduce_sweep


def _sweep(device, max_mb, world, budget_s=60.0, out=None):
    import torch.distributed as dist
    if dist.get_rank() == 1:
        time.sleep(3600)  # wedged: never reaches the collectives rank 0 is waiting in
    return _real(device, max_mb, world, budget_s, out)


bench.allreduce_sweep = _sweep
sys.exit(bench.main())
