"""Multi-rank worker for tests/test_gpu_multiproc.py::test_fused_exchange_every_shape: every
compiled (features, hidden) shape of the fused kernel trains through the in-kernel IPC exchange
(dense and padded LL3 payload layouts alike) and must match the stepwise trainer (per-step
kernels + a host all-reduce over the control-plane backend) and keep the ranks bit-identical.

Every shape also trains with the LL2 line format and with the ZeRO-1 exchange (both line formats):
they move the same gradients in the same rank order, so their parameters must be bit-identical to
the one-shot LL3 run.

Prints one ``RESULT {json}`` line on rank 0: "F,H" -> {"exchange", "max_abs_diff", "consistent",
"ll2_equal", "zero1_equal", "zero1_ll2_equal"}.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DGT_QUIET", "1")

import torch  # noqa: E402

from distributed_gpu_test_amd.data import make_synthetic_data  # noqa: E402
from distributed_gpu_test_amd.models import SimpleNet  # noqa: E402
from distributed_gpu_test_amd.parallel import comm  # noqa: E402
from distributed_gpu_test_amd.runtime.tiny_trainer import ReplicaDivergence, TinyMLPTrainer  # noqa: E402

SHAPES = [(20, 64), (32, 64), (20, 128), (8, 16)]


def train(f, h, impl, dev, steps=60, line="ll3", zero=0):
    os.environ["DGT_XCH_LINE"] = line
    x, y = make_synthetic_data(512, f, 7)
    torch.manual_seed(11)
    tr = TinyMLPTrainer(SimpleNet(f, h), x, y, 4, impl=impl, device=dev, zero_stage=zero)
    plan, counts = tr.epoch_plan(1)
    tr.run_plan(plan[:steps], counts[:steps])
    torch.cuda.synchronize(dev)
    try:
        tr.verify_replicas()
        consistent = True
    except ReplicaDivergence:
        consistent = False
    out = tr.params[: tr.numel].detach().clone(), tr.exchange, consistent
    tr.close()
    return out


def main():
    comm.init_distributed(backend="gloo")
    dev = torch.device("cuda", 0)
    res = {}
    for f, h in SHAPES:
        pf, xch, ok = train(f, h, "fused", dev)
        ps, _, ok_s = train(f, h, "stepwise", dev)
        p2, x2, ok2 = train(f, h, "fused", dev, line="ll2")
        pz, xz, okz = train(f, h, "fused", dev, zero=1)
        pz2, xz2, okz2 = train(f, h, "fused", dev, line="ll2", zero=1)
        res[f"{f},{h}"] = {"exchange": xch, "max_abs_diff": float((pf - ps).abs().max()),
                           "consistent": bool(ok and ok_s and ok2 and okz and okz2),
                           "ll2_equal": bool(torch.equal(pf, p2)) and x2.endswith("ll2"),
                           "zero1_equal": bool(torch.equal(pf, pz)) and xz.startswith("ipc-zero1"),
                           "zero1_ll2_equal": bool(torch.equal(pf, pz2)) and xz2 == "ipc-zero1-xgmi/ll2"}
    if comm.get_rank() == 0:
        print("RESULT " + json.dumps(res), flush=True)
    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
