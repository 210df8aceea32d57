"""torchrun worker (gloo, CPU): how much error a bf16 gradient collective adds over an fp32 one.

Every rank holds a bf16 gradient (what the MLP trainer's wgrad epilogue writes by default) shaped
like a real one: a per-rank N(0, 1) tensor scaled per 4096-element row by a log-uniform factor
(gradient rows span orders of magnitude).  The same tensors are summed three ways:
  * fp32 wire   : all_reduce of the fp32 upcast (what communication_data_type=fp32 sends);
  * bf16 wire   : all_reduce in bf16 through the process group;
  * bf16 ring   : RCCL's ring order emulated on rank 0 (chunk c accumulates ranks c+1, c+2, ...
                  with a bf16 rounding after every hop), the worst realistic accumulation order.
Errors are relative to the exact (fp64) sum, RMS over elements and normalised per row.
Rank 0 prints ``RESULT {json}``."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.parallel import comm  # noqa: E402


def grads(rank, rows=64, cols=4096):
    g = torch.Generator().manual_seed(1000 + rank)
    scale = torch.exp(torch.empty(rows, 1).uniform_(-6, 0, generator=torch.Generator().manual_seed(7)))
    return (torch.randn(rows, cols, generator=g) * scale).bfloat16()


def rel_rms(err, ref):
    # per-row RMS error over per-row RMS magnitude, then RMS over rows
    return float(((err.pow(2).mean(1) / ref.pow(2).mean(1).clamp_min(1e-30)).mean()).sqrt())


def main():
    comm.init_distributed(backend="gloo")
    ws, rank = comm.get_world_size(), comm.get_rank()
    g = grads(rank)
    exact = g.double()
    dist.all_reduce(exact)
    f32 = g.float()
    dist.all_reduce(f32)
    b16 = g.clone()
    dist.all_reduce(b16)
    everyone = [torch.empty_like(g) for _ in range(ws)]
    dist.all_gather(everyone, g)
    if rank == 0:
        flat = [t.reshape(-1) for t in everyone]
        n = flat[0].numel()
        chunk = (n + ws - 1) // ws
        ring = torch.empty(n, dtype=torch.bfloat16)
        for c in range(ws):  # chunk c: reduce-scatter starts at rank c+1 and ends at rank c
            sl = slice(c * chunk, min(n, (c + 1) * chunk))
            acc = flat[(c + 1) % ws][sl].clone()
            for k in range(2, ws + 1):
                acc = (acc.float() + flat[(c + k) % ws][sl].float()).bfloat16()
            ring[sl] = acc
        ring = ring.view_as(g)
        l1 = torch.stack([t.double().abs() for t in everyone]).sum(0)
        raw = torch.randn(64, 4096, generator=torch.Generator().manual_seed(5)).double()
        res = {
            "world_size": ws,
            "fp32_wire_rel_rms": rel_rms(f32.double() - exact, exact),
            "bf16_wire_rel_rms": rel_rms(b16.double() - exact, exact),
            "bf16_ring_rel_rms": rel_rms(ring.double() - exact, exact),
            # worst element against the sum of the magnitudes it accumulated (cancellation-proof)
            "bf16_ring_max_over_l1": float(((ring.double() - exact).abs() / l1.clamp_min(1e-30)).max()),
            # reference point: rounding ONE fp32 gradient to bf16 (what the bf16 wgrad epilogue does)
            "bf16_input_quant_rel_rms": rel_rms(raw.float().bfloat16().double() - raw, raw),
        }
        print("RESULT " + json.dumps(res), flush=True)
    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
