#!/usr/bin/env python3
"""Headline benchmark: training iterations/s of the reference's synthetic MLP (+ all-reduce bus GB/s).

Metric (BASELINE.json): "iters/sec + allreduce bus GB/s, synthetic MLP at 1/2/4/8 MI355X".
Config: the reference workload exactly — SimpleNet Linear(20,64)-ReLU-Linear(64,1), fp32,
micro-batch 4 per rank, BCE-with-logits, Adam(lr=1e-3), DistributedSampler over the 2000x20
synthetic dataset (seed 42), data-parallel over N ranks with a gradient all-reduce every step
(weak scaling: per-rank work is fixed).  Every timed step does the full forward, loss, backward,
cross-rank gradient reduction and optimizer update; nothing is cached or skipped.

    python bench.py                                  # 1 GPU
    torchrun --nproc-per-node N bench.py --gpus N    # N GPUs, one rank per GPU (RCCL/xGMI)

The timed region of the fused path holds exactly one kernel launch that runs all K optimizer
steps, including every step's Adam bias corrections (formed in double by the kernel's prologue).
Before it, untimed: the W warmup steps, the sampler's index plan of the K steps (the DataLoader's
work, uploaded once, as the trainer does once per epoch) and the sizing of the kernel's workspace.

The timed region is bracketed on both sides by a barrier and a device synchronisation, and the
time is the maximum over ranks.  With N > 1 and IPC mailboxes the barrier is device-side: a 16-byte
one-shot all-reduce over the same mailboxes (opening: after the process group's barrier; closing:
queued behind the last step, then one sync), ``config.closing_barrier`` says which was used.

``n_gpus`` counts distinct physical devices (host + PCI address gathered over ranks); ``ranks`` is
the process count and ``oversubscribed`` is true when ranks share a device.  A run whose ranks end
with different parameters exits non-zero and prints no headline line.

``value`` is the whole-job aggregate the driver contract asks for ("total tokens/s, not per-GPU";
here: rank-iterations/s = N x global DP steps/s, i.e. samples/s / 4).  Under weak scaling it grows
with N when the global step rate holds, so the driver's efficiency value_N / (N x value_1) is exactly
global_steps_per_sec_N / global_steps_per_sec_1.  The reference's own iteration -- one synchronised DP
step (``train.py:104-117``) -- is reported beside it as ``global_steps_per_sec``.

``allreduce_busbw_GBps`` is the peak RCCL all-reduce bus bandwidth of a size sweep (8 B - 1 GiB) run
after the timed region (rccl-tests convention, busbw = algbw x 2(n-1)/n).  The sweep runs in a
worker thread under a wall-clock budget (``--sweep-budget-s``; it stops growing the size once the
budget is spent) and a hard deadline: an RCCL error is recorded in ``allreduce_sweep_error`` and a
hang ends the job after the headline line is printed, so neither can cost the headline.

After everything else, the same guarded runner times the same-run PyTorch baselines ("match or beat",
SURVEY 6.4(a)): the reference's own loop on the reference model (``baseline``: nn.Module eager,
autograd, RCCL all-reduce at N > 1, torch.optim.Adam, a per-step ``loss.item()``) -- ``vs_baseline``
is the headline over it -- and plain PyTorch-ROCm on each secondary block's model (``baselines``;
each block gets ``torch_baseline_iters_per_s`` and ``speedup``).  Each baseline is timed in two
back-to-back windows and its rate is the faster one (``windows_iters_per_s`` lists both): a host
hiccup cannot make the baseline look slow.  ``--no-baselines`` turns them off.

After the headline's timed region, and outside it, the same guarded runner times BASELINE config #2
(``bf16_mlp``: SyntheticMLP(4096, 4), batch 1024 per GPU, bf16 MFMA GEMMs, MLPTrainer), the fp32
engine MLP (``fp32_engine_mlp``: SyntheticMLP(1024, 4) through the DeepSpeed-style engine on the
exact-fp32 MFMA GEMM) and, at N > 1, the ZeRO-1 variant of config #2 (``bf16_mlp_zero1``, config #5)
-- each a short warmup + timed block with its own ms_per_step / iters_per_s / model_tflops
(``--no-secondary`` turns them off; a failure is recorded as ``error`` in its block).
"""
from __future__ import annotations

import argparse
import functools
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "iters/sec + allreduce bus GB/s, synthetic MLP at 1/2/4/8 MI355X"


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20000, help="timed optimizer steps")
    ap.add_argument("--warmup", type=int, default=2000, help="untimed warmup steps")
    ap.add_argument("--impl", default="fused", choices=["fused", "graph", "stepwise", "engine", "dgt-engine"],
                    help="fused: one-launch HIP training kernel (IPC exchange over xGMI); graph: per-step HIP "
                         "kernels + native RCCL captured in a HIP graph; stepwise: the same launched eagerly with "
                         "ProcessGroupNCCL; engine: PyTorch eager + RCCL (the reference-equivalent stack); "
                         "dgt-engine: this framework's DeepSpeed-style engine on the nn.Module "
                         "(--deepspeed-config, e.g. configs/ds_graph.json for whole-step HIP graphs)")
    ap.add_argument("--deepspeed-config", "--deepspeed_config", dest="ds_config", default=None,
                    help="dgt-engine: DeepSpeed JSON config (default: the reference's in-code dict)")
    ap.add_argument("--model", default="simple", choices=["simple", "mlp"],
                    help="simple: the reference SimpleNet (headline); mlp: bench-size bf16 synthetic MLP on the "
                         "HIP MFMA GEMMs (BASELINE config #2)")
    ap.add_argument("--width", type=int, default=4096)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--batch", type=int, default=1024, help="mlp: per-GPU micro-batch")
    ap.add_argument("--torch-dtype", default="bf16", choices=["bf16", "fp32"],
                    help="--model mlp --impl engine: the PyTorch stack's compute dtype (bf16 autocast, or plain fp32 on "
                         "hipBLASLt's exact-fp32 GEMMs: the baseline for the fp32 engine MLP)")
    ap.add_argument("--zero-stage", type=int, default=0, choices=[0, 1],
                    help="0 = all-reduce the gradients; 1 = ZeRO-1: reduce-scatter them, shard Adam, all-gather "
                         "the parameters (simple: inside the fused kernel's exchange; mlp: per-layer RCCL)")
    ap.add_argument("--comm-dtype", default=None, choices=["bf16", "fp32"],
                    help="mlp: gradient wire dtype (DeepSpeed communication_data_type; default bf16)")
    ap.add_argument("--no-sweep", action="store_true", help="skip the all-reduce bus bandwidth sweep")
    ap.add_argument("--sweep-max-mb", type=int, default=1024)  # rccl-tests range: 8 B .. 1 GiB
    ap.add_argument("--force-sweep", action="store_true",
                    help="run the all-reduce sweep on any backend/device (gloo on the CPU: tests)")
    ap.add_argument("--sweep-budget-s", type=float, default=60.0,
                    help="stop growing the sweep's message size once this much wall time is spent")
    ap.add_argument("--sweep-deadline-s", type=float, default=None,
                    help="hard deadline of the sweep thread (default: the budget + 120 s)")
    ap.add_argument("--pg-timeout-s", type=float, default=180.0,
                    help="process-group timeout (a hung collective becomes an error after this long)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the post-headline bf16 MLP / fp32 engine MLP blocks")
    # (200 timed steps: 0.06 s of the fp32 block, 0.14 s of the bf16 one -- past the first-steps ramp)
    ap.add_argument("--force-secondary", action="store_true",
                    help="run the secondary blocks also when ranks share a card (a rehearsal of the N > 1 blocks)")
    ap.add_argument("--no-baselines", action="store_true",
                    help="skip the same-run PyTorch baselines (the reference-equivalent stack for the headline "
                         "and for each secondary block)")
    ap.add_argument("--baseline-steps", type=int, default=200, help="timed steps of the headline's torch baseline")
    ap.add_argument("--force-baselines", action="store_true",
                    help="run the baselines on any device (the CPU tests: the headline's, as no secondary block runs)")
    ap.add_argument("--secondary-steps", type=int, default=200)
    ap.add_argument("--secondary-warmup", type=int, default=20)
    ap.add_argument("--secondary-budget-s", type=float, default=90.0,
                    help="hard deadline for each secondary block (setup + warmup + timed steps)")
    # N > 1 knobs, echoed in the JSON config so a scaling run is self-describing
    ap.add_argument("--schedule", default=None, choices=["auto", "overlap", "serial", "flat"],
                    help="mlp: optimizer schedule (MLPTrainer; auto = flat at N=1, overlap at N>1)")
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="gradient bucket size in MiB: mlp = MLPTrainer's all-reduce buckets (default one per "
                         "layer); dgt-engine = zero_optimization.reduce_bucket_size")
    ap.add_argument("--oneshot-max-bytes", type=int, default=None,
                    help="dgt-engine: amd.oneshot_max_bytes (buckets at or below go over the IPC one-shot "
                         "all-reduce instead of RCCL)")
    return ap.parse_known_args(argv)[0]


def build_plan(trainer, n_steps: int):
    plans, counts, e = [], [], 1
    total = 0
    while total < n_steps:
        p, c = trainer.epoch_plan(e)
        plans.append(p)
        counts.append(c)
        total += p.shape[0]
        e += 1
    return torch.cat(plans)[:n_steps].contiguous(), torch.cat(counts)[:n_steps].contiguous()


def oneshot_sweep(device, world: int, max_bytes: int = 1024 * 1024):
    """The IPC one-shot all-reduce over xGMI (csrc/comm.hip) on the small sizes where latency rules."""
    from distributed_gpu_test_amd.parallel.comm import all_reduce_max as comm_max
    from distributed_gpu_test_amd.parallel.ipc import IpcChannel
    if world < 2:
        return []
    ch = IpcChannel(max_bytes // 4, device, timeout_s=10.0)
    try:
        if not ch.selftest():
            return []
        out = []
        size = 64
        reps = 200
        while size <= max_bytes:
            n = size // 4
            t = torch.ones(n, dtype=torch.float32, device=device)
            o = torch.empty_like(t)
            iters = 20
            for _ in range(3):
                ch.allreduce(t, o)
            torch.cuda.synchronize()
            # a timed-out exchange (status word) ends the sweep on every rank: each further launch
            # would spin until its own timeout
            if comm_max(float(ch.check_status() != 0)) > 0:
                print(f"[bench] one-shot sweep stopped at {size} B: exchange timeout", file=sys.stderr)
                break
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                ch.allreduce(t, o)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / iters
            # device latency: `reps` back-to-back all-reduces inside one launch (no host gaps)
            dist.barrier()
            t0 = time.perf_counter()
            ch.allreduce(t, o, reps=reps)
            torch.cuda.synchronize()
            dt_dev = (time.perf_counter() - t0) / reps
            ok = ch.check_status() == 0 and bool(torch.all(o == float(world)).item())
            algbw = n * 4 / dt_dev / 1e9
            out.append({"bytes": n * 4, "us": dt_dev * 1e6, "us_per_launch": dt * 1e6, "algbw_GBps": algbw,
                        "busbw_GBps": algbw * 2 * (world - 1) / world, "correct": ok})
            if comm_max(0.0 if ok else 1.0) > 0:
                break
            size *= 4
        return out
    finally:
        ch.close()


def allreduce_sweep(device, max_mb: int, world: int, budget_s: float = 60.0, out: "list | None" = None):
    """RCCL all-reduce bus bandwidth over message sizes (rccl-tests all_reduce_perf columns).

    Runs at N > 1, or at N = 1 under ``DGT_FORCE_COLLECTIVES=1`` (a 1-rank RCCL communicator: algbw
    only, busbw is 0 by the 2(n-1)/n convention), so the code has run on hardware before a scaling
    box runs it.  Once ``budget_s`` of wall time is spent the size stops growing; the decision is
    all-reduced (MAX) so every rank leaves the loop at the same size.  Results are appended to
    ``out`` as they come, so a caller that gave up waiting still has the finished sizes."""
    from distributed_gpu_test_amd.parallel import comm
    results = [] if out is None else out
    if world < 2 and not comm.force_collectives():
        return results
    sync = torch.cuda.synchronize if device.type == "cuda" else (lambda: None)
    start = time.perf_counter()
    size = 8
    while size <= max_mb * 1024 * 1024:
        n = max(1, size // 4)
        t = torch.ones(n, dtype=torch.float32, device=device)
        iters = 20 if size <= (1 << 22) else 5
        for _ in range(3):
            dist.all_reduce(t)
        sync()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(t)
        sync()
        dt = (time.perf_counter() - t0) / iters
        dt = comm.all_reduce_max(dt)  # the slowest rank's time, as rccl-tests reports
        algbw = n * 4 / dt / 1e9
        results.append({"bytes": n * 4, "us": dt * 1e6, "algbw_GBps": algbw,
                        "busbw_GBps": algbw * 2 * (world - 1) / world})
        del t
        if comm.all_reduce_max(float(time.perf_counter() - start > budget_s)) > 0:
            break
        size *= 4
    return results


def run_bounded(fn, deadline_s: float, device=None):
    """Run ``fn()`` in a daemon thread with a hard deadline: returns (result, error, hung).

    The informational parts of the bench (collective sweeps, secondary workloads) go through here so
    that neither an exception nor a hung collective costs the headline line: an exception comes back
    as ``error``; a call still running at the deadline comes back as ``hung`` -- the caller then
    issues no further collective (they would queue behind the stuck one), prints its line and ends
    the process with ``os._exit``."""
    import threading
    box = {}

    def target():
        try:
            if device is not None and device.type == "cuda":
                torch.cuda.set_device(device)  # the current device is per thread
            box["r"] = fn()
        except BaseException as e:  # noqa: BLE001 -- recorded, never raised into the headline path
            box["e"] = f"{type(e).__name__}: {e}"[:500]

    th = threading.Thread(target=target, daemon=True, name="dgt-bench-bounded")
    th.start()
    th.join(deadline_s)
    if th.is_alive():
        return None, f"timeout: still running after {deadline_s:.0f} s", True
    return box.get("r"), box.get("e"), False


def timed_block(trainer, steps: int, warmup: int, device) -> float:
    """W untimed steps, then K steps between barrier + sync on both sides; max over ranks (s)."""
    from distributed_gpu_test_amd.parallel import comm
    sync = torch.cuda.synchronize if device.type == "cuda" else (lambda: None)
    plan, counts = build_plan(trainer, warmup + steps)
    if warmup:
        trainer.run_plan(plan[:warmup], counts[:warmup])
    sync()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    trainer.run_plan(plan[warmup:], counts[warmup:])
    sync()
    comm.barrier()
    sync()
    return comm.all_reduce_max(time.perf_counter() - t0)


def secondary_specs(args, device, world: int):
    """The post-headline blocks: (key, description, factory) -- BASELINE config #2 (bf16 MLP on the
    MFMA GEMMs), the fp32 engine MLP, and at N > 1 config #5 (ZeRO-1 of config #2)."""
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP

    def bf16_mlp(zero_stage):
        def make():
            from distributed_gpu_test_amd.runtime.mlp_trainer import MLPTrainer
            torch.manual_seed(1234)
            model = SyntheticMLP(4096, 4)
            return MLPTrainer(model, batch_size=1024, lr=1e-4, device=device, zero_stage=zero_stage,
                              schedule=args.schedule, bucket_mb=args.bucket_mb if zero_stage == 0 else None)
        return make

    def fp32_engine_mlp():
        from distributed_gpu_test_amd.runtime.engine_mlp import EngineMLPTrainer
        torch.manual_seed(1234)
        cfg = json.load(open(os.path.join(ROOT, "configs", "ds_bench_mlp_fp32.json")))
        cfg = dict(cfg, train_micro_batch_size_per_gpu=1024)
        cfg.pop("train_batch_size", None)
        return EngineMLPTrainer(SyntheticMLP(1024, 4), 1024, 8, cfg)

    specs = [("bf16_mlp", "SyntheticMLP 4x[Linear(4096,4096)+ReLU] + Linear(4096,1), batch 1024/GPU, bf16 MFMA, "
              "MLPTrainer, ZeRO-0 (BASELINE config #2)", bf16_mlp(0)),
             ("fp32_engine_mlp", "SyntheticMLP 4x[Linear(1024,1024)+ReLU] + Linear(1024,1), batch 1024/GPU, fp32 "
              "(exact-fp32 MFMA GEMM), DeepSpeed-style engine, configs/ds_bench_mlp_fp32.json", fp32_engine_mlp)]
    if world > 1:
        specs.append(("bf16_mlp_zero1", "as bf16_mlp with ZeRO-1: reduce-scatter + sharded Adam + all-gather "
                      "(BASELINE config #5)", bf16_mlp(1)))
    return specs


def baseline_specs(args, device, world: int):
    """The same-run PyTorch baselines ("match or beat": SURVEY 6.4(a)), each (key, description, factory,
    steps, warmup): the headline's is the reference's own loop (``train.py:104-117``: nn.Module eager,
    autograd, RCCL all-reduce of the gradients at N > 1, torch.optim.Adam, a per-step ``loss.item()``
    host sync) on the reference model and micro-batch; the secondary blocks' are the same model and
    batch in plain PyTorch-ROCm (hipBLASLt GEMMs, torch's fused Adam, DDP at N > 1): bf16 autocast
    for ``bf16_mlp``, fp32 for ``fp32_engine_mlp``."""
    from distributed_gpu_test_amd.data import make_synthetic_data
    from distributed_gpu_test_amd.models import SimpleNet
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP

    def headline():
        torch.manual_seed(42)
        x, y = make_synthetic_data(2000, 20, 42)
        return EngineBench(SimpleNet(20, 64), x, y, 4, device)

    def mlp(width, autocast):
        def make():
            torch.manual_seed(1234)
            return TorchMLPBench(SyntheticMLP(width, 4), 1024, device, autocast=autocast)
        return make

    return [("headline", "reference loop: PyTorch eager SimpleNet + torch.optim.Adam + RCCL all-reduce + per-step "
             "loss.item() (train.py:104-117), fp32, micro-batch 4", headline, args.baseline_steps, 20),
            ("bf16_mlp", "PyTorch-ROCm: SyntheticMLP(4096, 4) bf16 autocast (hipBLASLt) + fused torch Adam"
             + (" + DDP" if world > 1 else ""), mlp(4096, True), 100, 20),
            ("fp32_engine_mlp", "PyTorch-ROCm: SyntheticMLP(1024, 4) fp32 (hipBLASLt) + fused torch Adam"
             + (" + DDP" if world > 1 else ""), mlp(1024, False), 200, 20)]


def attach_baselines(secondary: dict, baselines: dict) -> None:
    """Each secondary block gets its same-run torch baseline's rate and the speedup over it."""
    for key, b in baselines.items():
        if key in secondary and "iters_per_s" in b and "iters_per_s" in secondary[key]:
            secondary[key]["torch_baseline_iters_per_s"] = b["iters_per_s"]
            secondary[key]["torch_baseline_impl"] = b["impl"]
            secondary[key]["speedup"] = round(secondary[key]["iters_per_s"] / b["iters_per_s"], 3)


def run_baseline(desc: str, make, steps: int, warmup: int, device, windows: int = 2) -> dict:
    """The torch baseline, timed in ``windows`` back-to-back windows of ``steps`` steps; the FASTEST
    window is its rate (an eager, host-bound loop: one host hiccup in a single window made the
    baseline 2.5x slower in one of three fresh processes, and so the ratio against it 2x better)."""
    tr = make()
    try:
        elapsed = [timed_block(tr, steps, warmup if w == 0 else 0, device) for w in range(windows)]
        best = min(elapsed)
        return {"model": desc, "impl": tr.impl, "steps": steps, "warmup": warmup,
                "ms_per_step": round(best / steps * 1e3, 6), "iters_per_s": round(steps / best, 2),
                "windows_iters_per_s": [round(steps / e, 2) for e in elapsed]}
    finally:
        tr.close()
        del tr
        if device.type == "cuda":
            torch.cuda.synchronize()
            torch.cuda.empty_cache()


def run_secondary(key: str, desc: str, make, args, device, world: int) -> dict:
    """One secondary block (setup + warmup + timed steps); raises on failure (run_bounded catches)."""
    tr = make()
    try:
        elapsed = timed_block(tr, args.secondary_steps, args.secondary_warmup, device)
        gsps = args.secondary_steps / elapsed
        flops = tr.flops_per_step()
        return {"model": desc, "steps": args.secondary_steps, "warmup": args.secondary_warmup,
                "ms_per_step": round(elapsed / args.secondary_steps * 1e3, 6),
                "iters_per_s": round(gsps, 2),  # global DP steps/s
                "iters_per_s_sum_over_ranks": round(gsps * world, 2),
                "model_tflops": round(flops * world * gsps / 1e12, 2),
                "dtype": getattr(tr, "dtype_name", "bf16"), "impl": tr.impl, "exchange": tr.exchange,
                "zero_stage": getattr(tr, "zero_stage", 0), "schedule": getattr(tr, "schedule", None),
                "bucket_mb": getattr(tr, "bucket_mb", None),
                "mean_loss": round(float(tr.loss_acc.item()) / max(1, args.secondary_steps + args.secondary_warmup), 6)}
    finally:
        tr.close()
        del tr
        if device.type == "cuda":
            torch.cuda.synchronize()
            torch.cuda.empty_cache()


def timed_run(trainer, plan, counts, args, device, comm):
    """W untimed warmup steps, then exactly K timed steps between barrier + device syncs.
    Returns (max elapsed over ranks, mean loss over the timed steps).  Raises on every rank if the
    fused kernel failed on any rank."""
    if hasattr(trainer, "reserve"):  # workspace sizing (allocation only) before anything is timed
        trainer.reserve(max(args.warmup, args.steps))
    # the last warmup step is held back and launched right before the opening sync (below), so the
    # host launch path is as hot for the timed launch as in a steady-state loop
    warm_last = args.warmup > 0 and os.environ.get("DGT_BENCH_WARM_LAST", "1") == "1"
    # the launch's host-side preparation (plan checks, stream lookup, argument packing) is done
    # outside the bracket; the bracket holds the launch call itself and all K steps
    bind = getattr(trainer, "bind_launch", None) or (lambda p, c: functools.partial(trainer.run_plan, p, c))
    if args.warmup:
        # the last few warmup steps run as single-step launches through the same bound-launch path
        # the timed region uses: that path (HIP runtime, ctypes, Python) is then as warm for the
        # timed launch as in steady state, not on its first or second call
        tail = min(args.warmup, 4)
        head = args.warmup - tail
        if head:
            trainer.run_plan(plan[:head], counts[:head])
        for s in range(head, args.warmup - (1 if warm_last else 0)):
            bind(plan[s:s + 1], counts[s:s + 1])()
    timed_plan, timed_counts = plan[args.warmup:], counts[args.warmup:]  # views; the upload happened in build_plan
    last_plan, last_counts = plan[args.warmup - 1:args.warmup], counts[args.warmup - 1:args.warmup]
    trainer.loss_acc.zero_()  # queued behind the warmup: the bracket's opening sync has nothing left to wait on
    if device.type == "cuda":
        torch.cuda.synchronize()
    failed = _failed(trainer)
    if comm.all_reduce_max(float(failed)) > 0:
        raise RuntimeError("warmup failed on some rank")
    barrier = comm.barrier if comm.collectives_on() else (lambda: None)  # a 1-rank barrier is a no-op
    gpu = device.type == "cuda"
    # The ranks' kernels wait for each other from their first exchange, so start skew between the
    # ranks lands inside the slowest rank's timed region.  Opening barrier: the process-group
    # barrier, then (with IPC mailboxes) a device-side barrier whose kernels end within a
    # microsecond of each other on every rank, so the hosts leave their syncs nearly together.
    use_dev = comm.collectives_on() and not os.environ.get("DGT_BENCH_PG_BARRIER")
    multi = comm.collectives_on()  # decided outside the timed region: the lookup costs microseconds
    launch = bind(timed_plan, timed_counts)
    barrier()
    warm_loss = None
    if warm_last:  # the held-back warmup step; its loss is taken back out of the timed mean below
        bind(last_plan, last_counts)()
        warm_loss = trainer.loss_acc.clone()
    if use_dev:
        getattr(trainer, "device_barrier", lambda: False)()
    if gpu:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    launch()
    t1 = time.perf_counter()
    # closing barrier: with IPC mailboxes a device-side barrier queued behind the last step (one
    # tiny one-shot all-reduce, done when every rank's steps are), then ONE sync; otherwise sync +
    # the process group's barrier + sync.  One rank: the sync alone (its barrier is a no-op, so a
    # second sync would only time an idle round trip)
    device_barrier = use_dev and getattr(trainer, "device_barrier", lambda: False)()
    if gpu:
        torch.cuda.synchronize()
    t2 = time.perf_counter()
    if not device_barrier and multi:
        barrier()
        if gpu:
            torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if os.environ.get("DGT_BENCH_BREAKDOWN"):
        print(f"[bench] timed region: host launch {1e6 * (t1 - t0):.1f} us, device wait {1e6 * (t2 - t1):.1f} us, "
              f"closing barrier+sync {1e6 * (elapsed - (t2 - t0)):.1f} us "
              f"({'device barrier inside the wait' if device_barrier else 'process-group barrier'})",
              file=sys.stderr, flush=True)
    if comm.all_reduce_max(float(_failed(trainer))) > 0:
        raise RuntimeError("timed run failed on some rank")
    total = trainer.loss_acc - warm_loss if warm_loss is not None else trainer.loss_acc
    mean_loss = float(total.item()) / max(1, args.steps)
    return comm.all_reduce_max(elapsed), mean_loss


def closing_barrier_kind(trainer, world: int) -> str:
    """Which barrier closed the timed region (see timed_run)."""
    from distributed_gpu_test_amd.parallel import comm
    if not comm.collectives_on():
        return "none (1 rank)"
    ch = getattr(trainer, "channel", None)
    ipc = ch is not None and ch.healthy and not os.environ.get("DGT_BENCH_PG_BARRIER")
    return "ipc-device" if ipc else "process-group"


def _failed(trainer) -> bool:
    try:
        trainer.check()
        return False
    except RuntimeError as e:
        print(f"[bench] rank failure: {e}", file=sys.stderr, flush=True)
        return True


def device_identity(device) -> str:
    from distributed_gpu_test_amd.accelerator import device_identity as ident
    return ident(device)


def params_consistent(params, world: int) -> bool:
    """Every rank must hold bit-identical parameters after data-parallel training."""
    if world == 1:
        return True
    p = params.detach().clone()
    ref = p.clone()
    dist.broadcast(ref, 0)
    flag = torch.tensor([0.0 if torch.equal(p, ref) else 1.0], device=p.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    return flag.item() == 0.0


def self_launch(args, argv) -> "int | None":
    """``python bench.py --gpus N`` (N > 1) with no launcher around it: start the N ranks the way the
    reference's job does (``slurm_train.sbatch:18-23,36`` spawns ``nproc_per_node`` workers) -- one
    torchrun CHILD process (never an exec: nothing here has touched the GPU yet, and nothing will in
    this process), static rendezvous on 127.0.0.1, the same argv.  Rank 0's JSON line reaches our
    stdout unchanged (inherited stdio); the return value is the child's exit code.  Returns None when
    this process already is a rank (torchrun / SLURM / mpirun variables present) or N == 1."""
    from distributed_gpu_test_amd.launch import free_port, resolve_rank_info
    if args.gpus <= 1 or resolve_rank_info().source != "bare":
        return None
    import subprocess
    argv = list(sys.argv[1:] if argv is None else argv)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__), *argv]
    print(f"[bench] --gpus {args.gpus} without a launcher: starting {args.gpus} ranks under torchrun",
          file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def main(argv=None):
    args = parse_args(argv)
    rc = self_launch(args, argv)
    if rc is not None:
        return rc
    os.environ.setdefault("DGT_QUIET", "1")  # the engine's steps_per_print lines would be timed too
    from distributed_gpu_test_amd.data import make_synthetic_data
    from distributed_gpu_test_amd.models import SimpleNet
    from distributed_gpu_test_amd.parallel import comm
    from distributed_gpu_test_amd.runtime.tiny_trainer import TinyMLPTrainer

    # a short process-group timeout: one hung collective becomes an error within minutes, well
    # inside any driver limit, instead of after torch's default 30 minutes
    info = comm.init_distributed(timeout_s=args.pg_timeout_s)
    world, rank = comm.get_world_size(), comm.get_rank()
    if args.gpus != world:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}", file=sys.stderr)
    from distributed_gpu_test_amd.accelerator import get_accelerator
    device = get_accelerator().device()

    torch.manual_seed(42)
    x, y = make_synthetic_data(2000, 20, 42)
    model = SimpleNet(20, 64)
    B = 4
    if args.model == "mlp":
        from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
        from distributed_gpu_test_amd.runtime.mlp_trainer import MLPTrainer
        model = SyntheticMLP(args.width, args.depth)
        B = args.batch
        if args.impl == "engine":
            trainer = TorchMLPBench(model, B, device, autocast=args.torch_dtype == "bf16")
        elif args.impl == "dgt-engine":
            from distributed_gpu_test_amd.runtime.engine_mlp import EngineMLPTrainer
            cfg = engine_config(args, os.path.join(ROOT, "configs", "ds_bench_mlp_bf16.json"))
            cfg = dict(cfg, train_micro_batch_size_per_gpu=B)
            cfg.pop("train_batch_size", None)
            trainer = EngineMLPTrainer(model, B, 8, cfg)
        else:
            cdt = {None: None, "bf16": torch.bfloat16, "fp32": torch.float32}[args.comm_dtype]
            trainer = MLPTrainer(model, batch_size=B, lr=1e-4, device=device, zero_stage=args.zero_stage,
                                 comm_dtype=cdt, schedule=args.schedule, bucket_mb=args.bucket_mb)
    elif args.impl == "engine":
        trainer = EngineBench(model, x, y, B, device)
    elif args.impl == "dgt-engine":
        trainer = DgtEngineBench(model, x, y, B, device, engine_config(args, None))
    else:
        trainer = TinyMLPTrainer(model, x, y, B, lr=1e-3, impl=args.impl if device.type == "cuda" else "torch",
                                 device=device, zero_stage=args.zero_stage)
    plan, counts = build_plan(trainer, args.warmup + args.steps)
    selftest = list(getattr(trainer, "xch_report", []))  # the IPC trainer's, kept across a fallback
    fallback_reason = None
    try:
        elapsed_max, mean_loss = timed_run(trainer, plan, counts, args, device, comm)
        # every rank must hold identical parameters after DP training
        consistent = params_consistent(trainer.params, world)
        if not consistent and getattr(trainer, "channel", None) is not None:
            raise RuntimeError("parameters differ across ranks after the IPC-exchange run")
    except RuntimeError as e:
        # the fused kernel reports a cross-GPU exchange timeout through its status word, and a
        # replica divergence is seen by every rank through the check above; either way the whole
        # job re-runs on the RCCL path (loudly, and recorded in the JSON) instead of dying
        if getattr(trainer, "impl", "") != "fused":
            raise
        fallback_reason = str(e)
        print(f"[bench] WARNING: fused IPC path failed ({e}); re-running on the RCCL path",
              file=sys.stderr, flush=True)
        trainer.close()
        # use_ipc=False: the trainer's own automatic fallback (HIP graph with the native RCCL
        # communicator, or plain ProcessGroupNCCL if that cannot be set up on every rank)
        trainer = TinyMLPTrainer(model, x, y, B, lr=1e-3, impl="fused", device=device, use_ipc=False,
                                 zero_stage=args.zero_stage)
        plan, counts = build_plan(trainer, args.warmup + args.steps)
        elapsed_max, mean_loss = timed_run(trainer, plan, counts, args, device, comm)
        consistent = params_consistent(trainer.params, world)

    # a divergent run (after any fallback) has no headline
    if not consistent:
        if rank == 0:
            print(json.dumps({"metric": METRIC, "error": "parameters differ across ranks after training",
                              "impl": trainer.impl, "exchange": trainer.exchange}), file=sys.stderr, flush=True)
        trainer.close()
        comm.destroy()
        return 3
    devices = comm.all_gather_object(device_identity(device))
    n_devices = len(set(devices))

    # ---- informational parts, after the headline's timed region: every one runs through
    # run_bounded, so an error is recorded and a hang ends the job only after the line is printed
    hung = None
    collectives = world > 1 or comm.force_collectives()
    sweep, sweep_error = [], None
    if not args.no_sweep and collectives and (args.force_sweep or (device.type == "cuda" and
                                                                   comm.backend_name() == "nccl")):
        _, sweep_error, h = run_bounded(
            functools.partial(allreduce_sweep, device, args.sweep_max_mb, world, args.sweep_budget_s, sweep),
            args.sweep_deadline_s if args.sweep_deadline_s is not None else args.sweep_budget_s + 120.0, device)
        if sweep_error:
            print(f"[bench] RCCL all-reduce sweep stopped: {sweep_error}", file=sys.stderr, flush=True)
        hung = "allreduce_sweep" if h else None
    oneshot = []
    if not hung and not args.no_sweep and device.type == "cuda" and world > 1 and fallback_reason is None:
        # (after an IPC failure the mailboxes are not retried)
        res, err, h = run_bounded(functools.partial(oneshot_sweep, device, world), 120.0, device)
        oneshot = res or []
        if err:
            print(f"[bench] one-shot sweep skipped: {err}", file=sys.stderr)
        hung = "oneshot_sweep" if h else None
    secondary = {}
    # (the driver runs the default: the fused headline; other --impl / --model runs skip the blocks)
    # (ranks sharing a card -- a rehearsal on gloo -- would time host-staged collectives: skipped)
    if (not hung and not args.no_secondary and args.model == "simple" and args.impl == "fused" and device.type == "cuda"
            and (n_devices == world or args.force_secondary)):
        for key, desc, make in secondary_specs(args, device, world):
            t_block = time.perf_counter()
            res, err, h = run_bounded(functools.partial(run_secondary, key, desc, make, args, device, world),
                                      args.secondary_budget_s, device)
            block = res if res is not None else {"model": desc, "error": err}
            block["block_wall_s"] = round(time.perf_counter() - t_block, 2)
            secondary[key] = block
            if err:
                print(f"[bench] secondary block {key} failed: {err}", file=sys.stderr, flush=True)
            if h:
                hung = key
                break
            # a block that failed on one rank may have left the others mid-collective: stop there.
            # (The agreement is itself a collective: bounded too, a wedged peer must not keep this
            # rank from printing)
            bad, _, h = run_bounded(functools.partial(comm.all_reduce_max, float(err is not None)), 60.0, device)
            if h:
                hung = f"{key}:agreement"
                break
            if bad is None or bad > 0:
                break
    # ---- the same-run PyTorch baselines (after everything above, outside every timed region)
    baselines = {}
    if (not hung and not args.no_baselines and args.model == "simple" and args.impl == "fused"
            and ((device.type == "cuda" and (n_devices == world or args.force_secondary)) or args.force_baselines)):
        for key, desc, make, steps, warm in baseline_specs(args, device, world):
            if key != "headline" and key not in secondary:
                continue
            res, err, h = run_bounded(functools.partial(run_baseline, desc, make, steps, warm, device),
                                      args.secondary_budget_s, device)
            baselines[key] = res if res is not None else {"model": desc, "error": err}
            if err:
                print(f"[bench] baseline {key} failed: {err}", file=sys.stderr, flush=True)
            if h:
                hung = f"baseline_{key}"
                break
            bad, _, h = run_bounded(functools.partial(comm.all_reduce_max, float(err is not None)), 60.0, device)
            if h:
                hung = f"baseline_{key}:agreement"
                break
            if bad is None or bad > 0:
                break
    attach_baselines(secondary, baselines)
    small_os = min(oneshot, key=lambda r: abs(r["bytes"] - 5632)) if oneshot else None
    peak_busbw = max((r["busbw_GBps"] for r in sweep), default=None)
    small = min(sweep, key=lambda r: abs(r["bytes"] - 5632)) if sweep else None

    ms = elapsed_max / args.steps * 1e3
    global_steps_per_s = args.steps / elapsed_max
    if args.model == "mlp":
        tflops = trainer.flops_per_step() * world * global_steps_per_s / 1e12
        dtype = getattr(trainer, "dtype_name", "bf16")
        model_desc = (f"SyntheticMLP {args.depth}x[Linear({args.width},{args.width})+ReLU] + Linear({args.width},1) "
                      f"+ BCEWithLogits + Adam, {dtype} MFMA")
    else:
        tflops = None
        model_desc = "SimpleNet Linear(20,64)-ReLU-Linear(64,1) + BCEWithLogits + Adam(1e-3)"
        dtype = "fp32"
    out = {
        "metric": METRIC,
        "value": round(world * global_steps_per_s, 2),
        "unit": "iters/s, whole job (N ranks x global DP steps/s)",
        "n_gpus": n_devices,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 6),
        "higher_is_better": True,
        "scaling": "weak",
        # value / the same run's reference-equivalent stack (torch eager + RCCL + torch Adam + per-step
        # loss.item(), in the same rank-iterations/s unit); null when that baseline did not run
        "vs_baseline": (round(global_steps_per_s / baselines["headline"]["iters_per_s"], 2)
                        if "iters_per_s" in baselines.get("headline", {}) else None),
        "dtype": dtype,
        "data": ("synthetic (2000x20 N(0,1), seed 42; random-init SimpleNet)" if args.model == "simple" else
                 "synthetic N(0,1) batches, random-init weights"),
        "config": {"model": model_desc,
                   "global_batch": B * world, "seq_len": 1, "parallelism": f"dp{world}",
                   "micro_batch_per_gpu": B, "impl": trainer.impl, "exchange": trainer.exchange,
                   "zero_stage": args.zero_stage, "closing_barrier": closing_barrier_kind(trainer, world),
                   "schedule": getattr(trainer, "schedule", None), "bucket_mb": args.bucket_mb,
                   "oneshot_max_bytes": args.oneshot_max_bytes, "pg_timeout_s": args.pg_timeout_s},
        "global_steps_per_sec": round(global_steps_per_s, 2),
        "samples_per_sec": round(global_steps_per_s * B * world, 2),
        "mean_loss": round(mean_loss, 6),
        "model_tflops": None if tflops is None else round(tflops, 2),
        "ranks": world,
        "oversubscribed": n_devices < world,
        "params_consistent_across_ranks": consistent,
        "ipc_fallback_reason": fallback_reason,
        "exchange_selftest": selftest,
        "allreduce_busbw_GBps": None if peak_busbw is None else round(peak_busbw, 2),
        "allreduce_5KB_us": None if small is None else round(small["us"], 2),
        "oneshot_xgmi_5KB_us": None if small_os is None else round(small_os["us"], 2),
        "allreduce_sweep": [{k: round(v, 3) for k, v in r.items()} for r in sweep],
        "oneshot_xgmi_sweep": [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}
                               for r in oneshot],
        "allreduce_sweep_error": sweep_error,
        "hung": hung,
    }
    if baselines:
        out["baseline"] = baselines.get("headline")
        out["baselines"] = {k: v for k, v in baselines.items() if k != "headline"}
    if getattr(trainer, "graph_stats", None) is not None:
        out["engine_graph_replays"] = trainer.graph_stats
    out.update(secondary)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if hung:
        # a collective is stuck in a worker thread: a barrier or destroy would queue behind it.  The
        # line is out; end this rank now (every rank reaches its own deadline the same way)
        print(f"[bench] {hung} hung; exiting without process-group teardown", file=sys.stderr, flush=True)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
    trainer.close()
    comm.destroy()
    return 0


def engine_config(args, default_path):
    """The dgt-engine DeepSpeed config (``--deepspeed-config``, else ``default_path``, else the
    reference's in-code dict) with the bench's N > 1 knobs applied."""
    from distributed_gpu_test_amd.config import REFERENCE_DS_CONFIG
    path = args.ds_config or default_path
    cfg = json.load(open(path)) if path else json.loads(json.dumps(REFERENCE_DS_CONFIG))
    if args.bucket_mb is not None:
        z = dict(cfg.get("zero_optimization", {}))
        z["reduce_bucket_size"] = z["allgather_bucket_size"] = max(1, int(args.bucket_mb * (1 << 20) / 4))
        cfg["zero_optimization"] = z
    if args.oneshot_max_bytes is not None:
        a = dict(cfg.get("amd", {}))
        a["oneshot_max_bytes"] = int(args.oneshot_max_bytes)
        cfg["amd"] = a
    return cfg


class EngineBench:
    """The reference-equivalent stack: nn.Module eager + autograd + RCCL all-reduce + torch Adam."""

    impl = "engine"

    def __init__(self, model, x, y, B, device):
        from distributed_gpu_test_amd import data as dgt_data
        from distributed_gpu_test_amd.parallel import comm
        self.model = model.to(device)
        self.device = device
        self.x, self.y = x.to(device), y.to(device).reshape(-1, 1)
        self.B = B
        self.world = comm.get_world_size()
        self.rank = comm.get_rank()
        self._data = dgt_data
        if self.world > 1:
            for p in self.model.parameters():
                dist.broadcast(p.data, 0)
        self.opt = torch.optim.Adam(self.model.parameters(), lr=1e-3)
        self.crit = torch.nn.BCEWithLogitsLoss()
        self.loss_acc = torch.zeros(1, dtype=torch.float64, device=device)
        self.params = torch.nn.utils.parameters_to_vector(self.model.parameters())
        self.exchange = f"{comm.backend_name()}-allreduce" if self.world > 1 else "none"

    def epoch_plan(self, epoch):
        idx = self._data.shard_indices(self.x.shape[0], self.world, self.rank, epoch)
        plan = self._data.batch_plan(idx, self.B)
        return plan, (plan >= 0).sum(1).to(torch.int32)

    def run_plan(self, plan, counts):
        plan_d = plan.to(self.device).long()
        for s in range(plan.shape[0]):
            rows = plan_d[s, : int(counts[s])]
            loss = self.crit(self.model(self.x[rows]), self.y[rows])
            self.opt.zero_grad(set_to_none=True)
            loss.backward()
            if self.world > 1:
                flat = torch.cat([p.grad.reshape(-1) for p in self.model.parameters()])
                dist.all_reduce(flat)
                flat.div_(self.world)
                torch.nn.utils.vector_to_parameters(flat, [p.grad for p in self.model.parameters()])
            self.opt.step()
            self.loss_acc += loss.item()  # the reference's per-step host sync (train.py:115)
        self.params = torch.nn.utils.parameters_to_vector(self.model.parameters()).detach()

    def check(self):
        pass

    def close(self):
        pass


class TorchMLPBench:
    """The reference-equivalent stack for the bench-size MLP (BASELINE config #2): nn.Module with
    fp32 parameters, bf16 autocast (hipBLASLt GEMMs), autograd, bucketed DDP-style all-reduce
    (torch's own Reducer via DistributedDataParallel when N > 1) and torch's fused Adam."""

    impl = "torch-autocast-bf16"

    def __init__(self, model, B, device, n_batches=8, seed=1234, autocast=True):
        from distributed_gpu_test_amd.models.synthetic_mlp import synthetic_batch_data
        from distributed_gpu_test_amd.parallel import comm
        self.world, self.rank = comm.get_world_size(), comm.get_rank()
        self.device, self.B, self.n_batches = device, B, n_batches
        self.model = model.to(device)
        if self.world > 1:
            self.model = torch.nn.parallel.DistributedDataParallel(self.model, device_ids=[device.index])
        self.opt = torch.optim.Adam(self.model.parameters(), lr=1e-4, fused=device.type == "cuda")
        x, y = synthetic_batch_data(B * n_batches, model.in_features, seed + self.rank)
        self.X, self.Y = x.to(device), y.to(device)
        self.loss_acc = torch.zeros(1, dtype=torch.float64, device=device)
        self.global_steps = 0
        self.exchange = f"{comm.backend_name()}-ddp" if self.world > 1 else "none"
        self._flops = model.flops_per_sample() * B
        self.autocast = autocast
        if not autocast:  # plain fp32: hipBLASLt's exact-fp32 GEMMs (TF32 is off by default in torch)
            self.impl, self.dtype_name = "torch-fp32", "fp32"

    def flops_per_step(self):
        return self._flops

    def epoch_plan(self, epoch):
        plan = torch.arange(self.n_batches, dtype=torch.int32).view(-1, 1)
        return plan, torch.ones(self.n_batches, dtype=torch.int32)

    def run_plan(self, plan, counts):
        crit = torch.nn.BCEWithLogitsLoss()
        for _ in range(int(plan.shape[0])):
            j = self.global_steps % self.n_batches
            x, y = self.X[j * self.B:(j + 1) * self.B], self.Y[j * self.B:(j + 1) * self.B]
            with torch.autocast(device_type=self.device.type, dtype=torch.bfloat16, enabled=self.autocast):
                loss = crit(self.model(x).view(-1).float(), y)
            self.opt.zero_grad(set_to_none=True)
            loss.backward()
            self.opt.step()
            self.loss_acc += loss.detach().double()
            self.global_steps += 1

    @property
    def params(self):
        return torch.nn.utils.parameters_to_vector(self.model.parameters()).detach()

    def check(self):
        pass

    def close(self):
        pass


class DgtEngineBench(EngineBench):
    """This framework's engine (``initialize`` + DeepSpeed JSON) on the reference nn.Module: flat
    bucketed gradients, fused HIP Adam, ZeRO-0/1, and with ``"amd": {"hip_graph": true}`` the whole
    step (forward, backward, RCCL collective, Adam) replayed from a HIP graph."""

    impl = "dgt-engine"

    def __init__(self, model, x, y, B, device, cfg=None):
        from distributed_gpu_test_amd.config import REFERENCE_DS_CONFIG
        from distributed_gpu_test_amd.engine import initialize
        from distributed_gpu_test_amd.parallel import comm
        from distributed_gpu_test_amd import data as dgt_data
        if cfg is None:
            cfg = dict(REFERENCE_DS_CONFIG)
        elif isinstance(cfg, str):
            cfg = json.load(open(cfg))
        self._data = dgt_data
        self.device = device
        self.world, self.rank = comm.get_world_size(), comm.get_rank()
        self.x, self.y = x.to(device), y.to(device).reshape(-1, 1)
        self.B = B
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)
        self.engine, _, _, _ = initialize(model=model, optimizer=opt, model_parameters=model.parameters(), config=cfg)
        from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
        self.loss_acc = torch.zeros(1, dtype=torch.float64, device=device)
        # fused HIP loss + gradient kernel, which also adds the loss into the device-side loss log
        # (the reference's loss.item() sum, train.py:115) -- no launch of its own
        crit = BCEWithLogitsLoss(sum_into=self.loss_acc)

        gather = dgt_data.gather_batch

        def loss_fn(rows):
            # the batch gather and the loss log are part of the step, so a HIP graph captures them
            # with it; the gather is the data loader's (data.gather_batch: x and y rows in one launch)
            xb, yb = gather(rows, self.x, self.y)
            return crit(self.engine(xb).float(), yb)

        if self.engine.config.amd.hip_graph:
            self.step = self.engine.graph_step(loss_fn)
        else:
            def step(rows):
                loss = loss_fn(rows)
                self.engine.backward(loss)
                self.engine.step()
            self.step = step
        graphed = self.engine.graphed is not None
        self.exchange = ("none" if self.world == 1 else
                         ("rccl-native-in-hipgraph" if graphed else f"{comm.backend_name()}-bucketed"))
        self._impl = ("dgt-engine" + ("+hipgraph" if graphed else "") + ("+fusedlinear" if self.engine.fused_linear_layers else "")
                      + ("+graphmodule" if self.engine.graph_module else ""))

    @property
    def impl(self) -> str:
        """Named after the paths the steps actually took (the graphed tail is chosen per step)."""
        tail = "+graphtail" if getattr(self.engine, "tail_steps", 0) else ""
        return f"{self._impl}{tail}+zero{self.engine.stage}"

    @impl.setter
    def impl(self, value):
        pass

    def run_plan(self, plan, counts):
        plan_d = plan.to(self.device).long()
        # the per-step row views, sliced before the loop (the DataLoader's batches of the reference)
        batches = [plan_d[s, :c] for s, c in enumerate(counts.tolist())]
        for rows in batches:
            self.step(rows)

    @property
    def graph_stats(self):
        """graph_module: forward replays of the copying graphs and of the graphs bound to the
        batch's recurring addresses (engine.py _bound_runner)."""
        fns = list(self.engine._graphed_fwd.values())
        if not fns:
            return None
        return {"copying": sum(f.replays for f in fns),
                "bound": sum(b.replays for f in fns for b in f.bound.values()),
                "bound_graphs": sum(len(f.bound) for f in fns), "evictions": sum(f.evictions for f in fns)}

    @property
    def params(self):
        return self.engine.store.param_buf.detach()

    @params.setter
    def params(self, value):
        pass

    def close(self):
        self.engine.close()


if __name__ == "__main__":
    sys.exit(main())
