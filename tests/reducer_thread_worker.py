"""2-rank gloo worker (tests/test_multiproc_cpu.py): the reducer's launcher thread issues the same
collectives, with the same results, as launching on the backward thread -- stage 0 (all-reduce) and
stage 1 (reduce-scatter), buckets aligned to layers (FlatLayout units), a wire dtype cast."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from distributed_gpu_test_amd.parallel import comm  # noqa: E402
from distributed_gpu_test_amd.parallel.reducer import GradReducer  # noqa: E402
from distributed_gpu_test_amd.runtime.flat import FlatLayout  # noqa: E402


def run(stage, thread, dtype):
    rank, ws = comm.get_rank(), comm.get_world_size()
    shapes = [(64, 32), (64,), (48, 64), (48,), (16, 48), (16,), (1, 16), (1,)]
    units = [[0, 1], [2, 3], [4, 5], [6, 7]]
    layout = FlatLayout(shapes, 1024, ws, shard=stage >= 1, units=units)
    g = torch.Generator().manual_seed(11 + rank)
    grad = torch.randn(layout.total, generator=g).to(dtype)
    red = GradReducer(grad, layout, stage, ws, rank, comm_dtype=torch.float32, launch_thread=thread)
    outs = []
    for step in range(3):
        grad.mul_(1.5)
        red.arm(True)
        for i in reversed(range(len(shapes))):  # backward order: last layer first
            red.on_grad_ready(i)
        red.finish()
        outs.append(red.reduced.clone())
    red.close()
    return torch.stack(outs), layout, red.thread_launches


def main():
    comm.init_distributed(backend="gloo")
    res = {}
    for stage in (0, 1):
        for dtype in (torch.float32, torch.bfloat16):
            a, layout, n_thread = run(stage, True, dtype)
            b, _, n_inline = run(stage, False, dtype)
            res[f"stage{stage}_{str(dtype)[6:]}"] = {
                "equal": bool(torch.equal(a, b)), "thread_launches": n_thread, "inline_thread_launches": n_inline,
                "buckets": len(layout.buckets), "bucket_params": [b_.params for b_ in layout.buckets]}
    if comm.get_rank() == 0:
        print("RESULT " + json.dumps(res), flush=True)
    dist.barrier()
    comm.destroy()


if __name__ == "__main__":
    main()
