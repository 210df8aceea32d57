"""One-GPU worker for tests/test_gpu_force_collectives.py (and its rocprofv3 trace).

Every N > 1 code path that talks to RCCL runs here at world size 1 with ``DGT_FORCE_COLLECTIVES=1``
on the ``nccl`` backend (ProcessGroupNCCL of size 1 plus the native communicator), so the async
work handles, side streams, events and in-graph collectives execute on real hardware before an
8-GPU run does.  Each case runs twice — collectives off, then forced on — and must give bit-identical
parameters (a 1-rank sum is the identity).  The number of collective calls of each forced run is
counted through wrappers, so a case that silently skipped its collectives fails too.

Prints one ``RESULT {json}`` line: case -> {"equal": bool, "calls": int}.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DGT_QUIET", "1")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from distributed_gpu_test_amd.parallel import comm  # noqa: E402
from distributed_gpu_test_amd.parallel import rccl as rccl_mod  # noqa: E402

CALLS = {"n": 0}


def _count(fn):
    def wrapped(*a, **k):
        CALLS["n"] += 1
        return fn(*a, **k)
    return wrapped


for _name in ("all_reduce", "reduce_scatter_tensor", "all_gather_into_tensor", "broadcast"):
    setattr(dist, _name, _count(getattr(dist, _name)))
for _name in ("all_reduce", "reduce_scatter", "all_gather"):
    setattr(rccl_mod.RcclComm, _name, _count(getattr(rccl_mod.RcclComm, _name)))


def forced(flag: bool):
    os.environ["DGT_FORCE_COLLECTIVES"] = "1" if flag else "0"


def run_pair(fn):
    out, extra = [], {}
    for flag in (False, True):
        forced(flag)
        CALLS["n"] = 0
        p = fn()
        if isinstance(p, tuple):  # (params, {key: value}) -- the forced run's extras are reported
            p, ex = p
            extra = {f"{k}_{'forced' if flag else 'off'}": v for k, v in ex.items()} | extra
        torch.cuda.synchronize()
        out.append((p.detach().clone(), CALLS["n"]))
    forced(False)
    return {"equal": bool(torch.equal(out[0][0], out[1][0])), "calls": out[1][1], "calls_off": out[0][1], **extra}


def engine_case(stage, graph):
    import distributed_gpu_test_amd as dgt

    def fn():
        torch.manual_seed(4)
        m = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.ReLU(), torch.nn.Linear(256, 1))
        cfg = {"train_batch_size": 32, "zero_optimization": {"stage": stage, "reduce_bucket_size": 4096},
               "amd": {"hip_graph": graph}}
        engine, _, _, _ = dgt.initialize(model=m, optimizer=torch.optim.Adam(m.parameters(), lr=1e-3), config=cfg)
        crit = torch.nn.BCEWithLogitsLoss()
        g = torch.Generator().manual_seed(5)
        batches = [(torch.randn(32, 64, generator=g).cuda(), (torch.rand(32, 1, generator=g) > 0.5).float().cuda())
                   for _ in range(8)]
        if graph:
            step = engine.graph_step(lambda bx, by: crit(engine(bx).float(), by))
            assert engine.graphed is not None, engine.graph_fallback_reason
            for x, y in batches:
                step(x, y)
        else:
            for x, y in batches:
                engine.backward(crit(engine(x).float(), y))
                engine.step()
        p = engine.store.param_buf.detach().clone()
        engine.close()
        return p
    return fn


def engine_mlp_case(dtype, stage):
    """The SyntheticMLP through the engine on the fused chains (bf16: the MFMA GEMM chain; fp32: the
    exact-fp32 GEMM chain), one bucket per layer: every layer's collective is launched from inside
    the chain's backward (ops.linear.grad_ready), counted as ``layer_notifications``."""
    import distributed_gpu_test_amd as dgt
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP

    def fn():
        torch.manual_seed(6)
        m = SyntheticMLP(width=256, depth=3)
        cfg = {"train_micro_batch_size_per_gpu": 128, "gradient_accumulation_steps": 1,
               "zero_optimization": {"stage": stage, "reduce_bucket_size": 4096},
               "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}}
        if dtype == "bf16":
            cfg.update({"bf16": {"enabled": True}, "communication_data_type": "fp32"})
        engine, _, _, _ = dgt.initialize(model=m, config=cfg)
        from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
        crit = BCEWithLogitsLoss()
        g = torch.Generator().manual_seed(7)
        for _ in range(6):
            x = torch.randn(128, 256, generator=g).cuda().to(engine.dtype)
            y = (torch.rand(128, generator=g) > 0.5).float().cuda()
            engine.backward(crit(engine(x).view(-1), y))
            engine.step()
        p = engine.store.param_buf.detach().float().clone()
        extra = {"layer_notifications": engine.layer_notifications, "buckets": len(engine.layout.buckets),
                 "fused_layers": engine.fused_linear_layers, "thread_launches": engine.reducer.thread_launches + engine.reducer.native_launches,
                 "native": engine.reducer.native is not None}
        engine.close()
        return p, extra
    return fn


def engine_fuzz_case(dtype, stage, gas, seed, steps=24, width=256):
    """The engine MLP (fused chains, one bucket per layer) through seeded random transitions --
    batch 128 / 256, the fused or torch's BCE, a no-grad forward in between, a retained graph taken
    backward twice, lr changes, extra zero_grad calls -- so that the reducer's per-layer launches,
    its launcher thread and the accumulation across backwards are exercised in orders no listed case
    has; the forced run must still give the collective-free run's bits."""
    import random

    import distributed_gpu_test_amd as dgt
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss

    def fn():
        torch.manual_seed(100 + seed)
        rnd = random.Random(seed)
        m = SyntheticMLP(width=width, depth=3)
        cfg = {"train_micro_batch_size_per_gpu": 128, "gradient_accumulation_steps": gas,
               "zero_optimization": {"stage": stage, "reduce_bucket_size": 4096},
               "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}}
        if dtype == "bf16":
            cfg.update({"bf16": {"enabled": True}, "communication_data_type": "fp32"})
        engine, opt, _, _ = dgt.initialize(model=m, config=cfg)
        fused, tbce = BCEWithLogitsLoss(), torch.nn.BCEWithLogitsLoss()
        g = torch.Generator().manual_seed(1000 + seed)
        counts = {"eval": 0, "retain": 0, "torch_bce": 0, "lr": 0, "zero_grad": 0, "b256": 0}
        for _ in range(steps * gas):
            b = rnd.choice([128, 256])
            counts["b256"] += b == 256
            x = torch.randn(b, width, generator=g).cuda().to(engine.dtype)
            y = (torch.rand(b, generator=g) > 0.5).float().cuda()
            if rnd.random() < 0.15:
                counts["eval"] += 1
                with torch.no_grad():
                    engine(x)
            out = engine(x).view(-1)
            if rnd.random() < 0.5:
                counts["torch_bce"] += 1
                loss = tbce(out.float(), y)
            else:
                loss = fused(out, y)
            if rnd.random() < 0.2:
                counts["retain"] += 1
                engine.backward(loss, retain_graph=True)
                engine.backward(loss)
            else:
                engine.backward(loss)
            engine.step()
            if rnd.random() < 0.1:
                counts["zero_grad"] += 1
                engine.zero_grad()
            if rnd.random() < 0.15:
                counts["lr"] += 1
                opt.param_groups[0]["lr"] = rnd.choice([5e-4, 1e-3, 2e-3])
        p = engine.store.param_buf.detach().float().clone()
        extra = {"layer_notifications": engine.layer_notifications,
                 "launches": engine.reducer.thread_launches + engine.reducer.native_launches, **counts}
        engine.close()
        return p, extra
    return fn


def fuzz_cases(names):
    """fuzz_<bf16|fp32>_zero<stage>_gas<gas>_s<seed>[_w<width>] -> the case (requested by name only;
    width 1024 puts the bf16 chain's products on the GEMM's small-grid split-K mode)."""
    out = {}
    for n in names:
        if n.startswith("fuzz_"):
            parts = n.split("_")
            _, dtype, z, ga, sd = parts[:5]
            width = int(parts[5][1:]) if len(parts) > 5 else 256
            out[n] = engine_fuzz_case(dtype, int(z[4:]), int(ga[3:]), int(sd[1:]), width=width)
    return out


def mlp_case(schedule, stage):
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    from distributed_gpu_test_amd.runtime.mlp_trainer import MLPTrainer

    def fn():
        torch.manual_seed(3)
        # fuse_adam=False: the single-rank fused wgrad+Adam exists only WITHOUT collectives, so both
        # runs of the pair must take the gradient-buffer path the N > 1 schedules use
        tr = MLPTrainer(SyntheticMLP(width=256, depth=3), batch_size=128, n_batches=2, lr=1e-3,
                        device=torch.device("cuda", 0), zero_stage=stage, schedule=schedule, fuse_adam=False)
        for s in range(5):
            tr.step(s)
        tr.join()
        return tr.params.clone()
    return fn


def tiny_case(impl):
    from distributed_gpu_test_amd.data import make_synthetic_data
    from distributed_gpu_test_amd.models import SimpleNet
    from distributed_gpu_test_amd.runtime.tiny_trainer import TinyMLPTrainer

    def fn():
        torch.manual_seed(42)
        x, y = make_synthetic_data(2000, 20, 42)
        tr = TinyMLPTrainer(SimpleNet(20, 64), x, y, 4, impl=impl, device=torch.device("cuda", 0))
        plan, counts = tr.epoch_plan(1)
        tr.run_plan(plan[:120], counts[:120])
        p = tr.params.clone()
        tr.close()
        return p
    return fn


def main():
    comm.init_distributed(backend="nccl")
    assert comm.backend_name() == "nccl" and comm.get_world_size() == 1
    only = set(sys.argv[1:])
    cases = {}
    for stage in (0, 1):
        for graph in (False, True):
            cases[f"engine_zero{stage}_{'graph' if graph else 'eager'}"] = engine_case(stage, graph)
    for dtype in ("bf16", "fp32"):
        for stage in (0, 1):
            cases[f"engine_mlp_{dtype}_zero{stage}"] = engine_mlp_case(dtype, stage)
    for schedule in ("overlap", "serial", "flat"):
        for stage in (0, 1):
            cases[f"mlp_{schedule}_zero{stage}"] = mlp_case(schedule, stage)
    for impl in ("graph", "stepwise"):
        cases[f"tiny_{impl}"] = tiny_case(impl)
    cases.update(fuzz_cases(only))
    res = {}
    for name, fn in cases.items():
        if only and name not in only:
            continue
        res[name] = run_pair(fn)
        print(f"[force] {name}: {res[name]}", file=sys.stderr, flush=True)
    print("RESULT " + json.dumps(res), flush=True)
    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
