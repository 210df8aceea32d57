#!/usr/bin/env python3
"""train.py — the distributed acceptance-test training job, MI355X-native.

Same CLI, stdout and checkpoint layout as the reference ``train.py`` (dashabalashova/
distributed-gpu-test): a 2-layer MLP trained data-parallel on 2000 synthetic samples for
``--epochs`` epochs, printing ``Epoch  e finished. Avg loss: x.xxxx`` per epoch and
``Training completed.`` at the end, and saving ``<save-dir>/epoch{e}/global_step{N}/...``
after every epoch (``train.py:42-129``).  Unknown flags (``--deepspeed``,
``--distributed-backend nccl``, ``--local-rank=N``) are ignored, as in the reference.

Differences by design:
* world_size 1 works (the reference crashes in ``sampler.set_epoch``);
* on a GPU the default ``--impl auto`` runs the fused HIP training kernel (one launch per epoch,
  gradient exchange over xGMI inside the kernel); ``--impl engine`` runs the generic
  DeepSpeed-style engine (PyTorch modules + bucketed RCCL all-reduce + fused Adam);
* extra flags: ``--deepspeed_config``, ``--impl``, ``--backend``, ``--fail-at``, ``--resume``,
  ``--no-save``, ``--dist-timeout``, ``--strict-exchange``;
* the fused path survives a failing in-kernel exchange: a timeout or replica divergence at an
  epoch's end restores the epoch-start state on every rank and re-runs the epoch on the RCCL path
  (``exchange_fallback`` on stderr, in ``DGT_METRICS_JSONL`` and ``DGT_HEALTH_LOG``; rc stays 0),
  unless ``--strict-exchange`` keeps it fatal (rc 2), as the reference's job succeeds whenever
  NCCL works (``slurm_train.sbatch:34-44``).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import sys

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import distributed_gpu_test_amd as dgt  # noqa: E402
from distributed_gpu_test_amd.accelerator import get_accelerator  # noqa: E402
from distributed_gpu_test_amd.config import REFERENCE_DS_CONFIG, parse_config  # noqa: E402
from distributed_gpu_test_amd.data import SyntheticDataset, make_synthetic_data  # noqa: E402
from distributed_gpu_test_amd.models import SimpleNet  # noqa: E402
from distributed_gpu_test_amd.ops import BCEWithLogitsLoss  # noqa: E402
from distributed_gpu_test_amd.parallel import comm  # noqa: E402
from distributed_gpu_test_amd.utils.fault import FaultInjector  # noqa: E402

N_SAMPLES, N_FEATURES, HIDDEN, MICRO_BATCH = 2000, 20, 64, 4


def parse_args(argv=None):
    p = argparse.ArgumentParser(allow_abbrev=False)  # "--deepspeed" must not match --deepspeed_config
    p.add_argument("--train-batch-size", type=int, default=64)  # parsed, unused (reference Q2)
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--save-dir", type=str, default="ds_checkpoints")
    # additions
    p.add_argument("--deepspeed_config", "--deepspeed-config", dest="deepspeed_config", default=None)
    p.add_argument("--impl", default="auto", choices=["auto", "fused", "graph", "stepwise", "engine", "torch"])
    p.add_argument("--backend", default=None, choices=["nccl", "gloo"])
    p.add_argument("--fail-at", default=None, help="RANK:STEP[:exit|abort|hang|nan] (STEP 'end' = after training)")
    p.add_argument("--resume", action="store_true", help="continue from the newest checkpoint in --save-dir")
    p.add_argument("--no-save", action="store_true")
    p.add_argument("--dist-timeout", type=float, default=1800.0)
    p.add_argument("--profile", default=None, help="write a torch.profiler (kineto) trace per rank to this dir "
                   "(every path; roctx ranges with DGT_ROCTX=1 name the phases / fused epoch launches)")
    p.add_argument("--model", default="simple", choices=["simple", "mlp"],
                   help="simple: the reference SimpleNet (default); mlp: the bench-size bf16 SyntheticMLP on the "
                        "hand-written MFMA GEMMs (BASELINE config #2; default config configs/ds_bench_mlp_bf16.json)")
    p.add_argument("--width", type=int, default=4096, help="mlp: hidden width")
    p.add_argument("--depth", type=int, default=4, help="mlp: hidden layers")
    p.add_argument("--mlp-batches", type=int, default=8, help="mlp: optimizer steps per epoch (per-rank batches)")
    p.add_argument("--strict-exchange", action="store_true",
                   help="fail the job (rc 2) on an in-kernel exchange timeout / replica divergence instead of "
                        "re-running the epoch on the RCCL path")
    p.add_argument("--debug-sync", action="store_true",
                   help="serialize kernels (AMD_SERIALIZE_KERNEL=3) and sync comm/compute streams: race hunting")
    return p.parse_known_args(argv)[0]


def run_mlp(args, cfg, ds_config, world: int, local_rank: int) -> None:
    """BASELINE config #2 as a train.py / SLURM job: the bench-size bf16 SyntheticMLP, per-rank
    synthetic batches (weak scaling, as bench.py --model mlp), the DeepSpeed JSON's micro-batch,
    Adam hyper-parameters, ZeRO stage and communication dtype, epoch loss lines and per-epoch
    checkpoints in the reference's layout.  ``--impl auto`` runs MLPTrainer (hand-written MFMA
    GEMMs with fused bias / ReLU / mask / transposed-copy epilogues, one flat fused Adam over the
    fp32 masters after backward, per-layer RCCL buckets); ``--impl engine`` runs the same model through
    ``initialize`` (the engine's bf16 MFMA Linear chain)."""
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    from distributed_gpu_test_amd.runtime.mlp_trainer import MLPTrainer
    from distributed_gpu_test_amd.utils.tracing import Profiler
    model = SyntheticMLP(args.width, args.depth)
    B = cfg.train_micro_batch_size_per_gpu
    o = cfg.optimizer
    lr, betas, eps = (o.lr, tuple(o.betas), o.eps) if o is not None else (args.lr, (0.9, 0.999), 1e-8)
    cdt = {"fp32": torch.float32, "float32": torch.float32, "bf16": torch.bfloat16, "bfloat16": torch.bfloat16,
           None: None}[cfg.communication_data_type]
    if args.impl == "engine":
        from distributed_gpu_test_amd.runtime.engine_mlp import EngineMLPTrainer
        trainer = EngineMLPTrainer(model, B, args.mlp_batches, ds_config)
    else:
        trainer = MLPTrainer(model, batch_size=B, n_batches=args.mlp_batches, lr=lr, betas=betas, eps=eps,
                             zero_stage=cfg.zero_stage if cfg.zero_stage in (0, 1) else 0, comm_dtype=cdt)
    over = oversubscribed(trainer.device)
    if comm.get_rank() == 0:
        print(f"[dgt] model=mlp impl={trainer.impl} width={args.width} depth={args.depth} micro_batch={B} "
              f"zero_stage={getattr(trainer, 'zero_stage', cfg.zero_stage)} exchange={trainer.exchange} "
              f"world_size={world} oversubscribed={over}", file=sys.stderr, flush=True)
    start_epoch = 1
    if args.resume:
        found = newest_checkpoint(args.save_dir)
        if found:
            trainer.load_checkpoint(found[1])
            start_epoch = found[0] + 1
    plan, counts = trainer.epoch_plan(1)
    prof = Profiler(args.profile, comm.get_rank())
    with prof:
        for epoch in range(start_epoch, args.epochs + 1):
            trainer.loss_acc.zero_()
            trainer.run_plan(plan, counts)
            prof.step()
            avg_loss = float(trainer.loss_acc.item()) / max(1, int(plan.shape[0]))
            if local_rank == 0:
                print(f"Epoch {epoch:2d} finished. Avg loss: {avg_loss:.4f}", flush=True)
            if not args.no_save:
                save_dir = os.path.join(args.save_dir, f"epoch{epoch}")
                os.makedirs(save_dir, exist_ok=True)
                trainer.save_checkpoint(save_dir, ds_config=cfg.to_dict())
    trainer.close()


def oversubscribed(device) -> bool:
    """True when ranks share a physical device (host + PCI address gathered over ranks), as
    bench.py reports it; a job that wraps ranks onto fewer cards says so instead of silently
    oversubscribing them (accelerator.set_device refuses unless DGT_ALLOW_OVERSUBSCRIBE=1)."""
    from distributed_gpu_test_amd.accelerator import device_identity
    ids = comm.all_gather_object(device_identity(device))
    return len(set(ids)) < len(ids)


def newest_checkpoint(save_dir: str):
    best = None
    for d in glob.glob(os.path.join(save_dir, "epoch*")):
        m = re.fullmatch(r"epoch(\d+)", os.path.basename(d))
        if m and os.path.exists(os.path.join(d, "latest")):
            e = int(m.group(1))
            if best is None or e > best[0]:
                best = (e, d)
    return best


def main(argv=None) -> int:
    args = parse_args(argv)
    if args.debug_sync:  # serialize to bisect ordering bugs between streams
        os.environ.setdefault("AMD_SERIALIZE_KERNEL", "3")
        os.environ.setdefault("AMD_SERIALIZE_COPY", "3")
    torch.manual_seed(args.seed)
    info = comm.init_distributed(backend=args.backend, timeout_s=args.dist_timeout)
    local_rank, world = info.local_rank, comm.get_world_size()
    faults = FaultInjector.from_env(comm.get_rank(), args.fail_at)
    if args.fail_at:
        os.environ["DGT_FAIL_AT"] = args.fail_at

    if args.model == "mlp" and args.deepspeed_config is None:
        args.deepspeed_config = os.path.join(ROOT, "configs", "ds_bench_mlp_bf16.json")
    ds_config = REFERENCE_DS_CONFIG if args.deepspeed_config is None else json.load(open(args.deepspeed_config))
    if args.debug_sync:
        ds_config = dict(ds_config, amd=dict(ds_config.get("amd", {}), debug_sync_streams=True))
    cfg = parse_config(ds_config, world)  # DeepSpeed's batch assertion on every path

    if args.model == "mlp":
        run_mlp(args, cfg, ds_config, world, local_rank)
        if local_rank == 0:
            print("Training completed.", flush=True)
        faults.maybe_fire_end()
        return 0

    x, y = make_synthetic_data(n_samples=N_SAMPLES, n_features=N_FEATURES, seed=args.seed)
    model = SimpleNet(n_features=x.shape[1], hidden=HIDDEN)
    optimizer = torch.optim.Adam(model.parameters(), lr=args.lr)

    gpu = get_accelerator().name == "hip"
    impl = args.impl
    if impl == "auto":
        from distributed_gpu_test_amd.runtime.tiny_trainer import fused_supported
        # ZeRO-0 and ZeRO-1 (sharded in-kernel exchange) both run on the fused kernel
        fused_ok = gpu and cfg.zero_stage in (0, 1) and cfg.gradient_accumulation_steps == 1 and \
            cfg.compute_dtype == "fp32" and fused_supported(N_FEATURES, HIDDEN, MICRO_BATCH)
        impl = "fused" if fused_ok else "engine"

    start_epoch = 1
    if impl in ("fused", "graph", "stepwise", "torch"):
        from distributed_gpu_test_amd.runtime.tiny_trainer import TinyMLPTrainer
        trainer = TinyMLPTrainer(model, x, y, MICRO_BATCH, lr=args.lr, impl=impl, ds_config=cfg.to_dict(),
                                 device=None if impl != "torch" else torch.device("cpu"),
                                 zero_stage=cfg.zero_stage if cfg.zero_stage in (0, 1) else 0,
                                 strict_exchange=args.strict_exchange or None)
        over = oversubscribed(trainer.device)
        if comm.get_rank() == 0:
            print(f"[dgt] impl={trainer.impl} exchange={trainer.exchange} zero_stage={trainer.zero_stage} "
                  f"world_size={world} oversubscribed={over}", file=sys.stderr, flush=True)
            for rep in trainer.xch_report:
                print(f"[dgt] exchange self-test: {json.dumps(rep)}", file=sys.stderr, flush=True)
        if args.resume:
            found = newest_checkpoint(args.save_dir)
            if found:
                trainer.load_checkpoint(found[1])
                start_epoch = found[0] + 1
        from distributed_gpu_test_amd.utils.tracing import Profiler
        # one profiler step per epoch: the fused path runs a whole epoch in one kernel launch
        prof = Profiler(args.profile, comm.get_rank(), active_steps=max(1, args.epochs - start_epoch + 1), wait=0,
                        warmup=0)
        with prof:
            for epoch in range(start_epoch, args.epochs + 1):
                avg_loss = trainer.run_epoch(epoch)
                prof.step()
                if local_rank == 0:
                    print(f"Epoch {epoch:2d} finished. Avg loss: {avg_loss:.4f}", flush=True)
                if not args.no_save:
                    save_dir = os.path.join(args.save_dir, f"epoch{epoch}")
                    os.makedirs(save_dir, exist_ok=True)
                    trainer.save_checkpoint(save_dir)
        if trainer.fallbacks and comm.get_rank() == 0:
            print(f"[dgt] finished on {trainer.impl}/{trainer.exchange} after {len(trainer.fallbacks)} "
                  f"exchange_fallback(s)", file=sys.stderr, flush=True)
        trainer.close()
    else:
        engine, optimizer, _, _ = dgt.initialize(args=ds_config, model=model, optimizer=optimizer,
                                                 model_parameters=model.parameters(), config=ds_config)
        device = engine.device
        over = oversubscribed(device)
        if comm.get_rank() == 0:
            print(f"[dgt] impl=engine zero_stage={cfg.zero_stage} dtype={cfg.compute_dtype} "
                  f"oneshot={'yes' if engine.oneshot is not None else 'no'} backend={comm.backend_name()} "
                  f"world_size={world} oversubscribed={over}", file=sys.stderr, flush=True)
        data = SyntheticDataset(x, y, MICRO_BATCH, world, comm.get_rank()).to(device)
        # fused HIP loss + gradient kernel on GPU (torch's own loss on CPU)
        criterion = BCEWithLogitsLoss()
        if args.resume:
            found = newest_checkpoint(args.save_dir)
            if found:
                engine.load_checkpoint(found[1])
                start_epoch = found[0] + 1
        train_step = None
        if cfg.amd.hip_graph:
            train_step = engine.graph_step(lambda bx, by: criterion(engine(bx).float(), by))
            if comm.get_rank() == 0:
                why = engine.graph_fallback_reason
                print(f"[dgt] hip_graph={'on' if engine.graphed is not None else 'off (' + why + ')'}",
                      file=sys.stderr, flush=True)
        from distributed_gpu_test_amd.utils.tracing import Profiler
        prof = Profiler(args.profile, comm.get_rank())
        with prof:
            for epoch in range(start_epoch, args.epochs + 1):
                engine.train()
                data.set_epoch(epoch)
                loss_acc = torch.zeros((), dtype=torch.float64, device=device)
                steps = 0
                for batch_x, batch_y in data:
                    if train_step is not None:  # whole step replayed from a HIP graph
                        loss = train_step(batch_x, batch_y)
                    else:
                        logits = engine(batch_x)
                        loss = criterion(logits.float(), batch_y)
                        engine.backward(loss)
                        engine.step()
                    prof.step()
                    loss_acc += loss.detach().double()  # on device: no per-step host sync
                    steps += 1
                avg_loss = float(loss_acc.item()) / max(1, steps)
                if local_rank == 0:
                    print(f"Epoch {epoch:2d} finished. Avg loss: {avg_loss:.4f}", flush=True)
                if not args.no_save:
                    save_dir = os.path.join(args.save_dir, f"epoch{epoch}")
                    os.makedirs(save_dir, exist_ok=True)
                    engine.save_checkpoint(save_dir)
        engine.close()

    if local_rank == 0:
        print("Training completed.", flush=True)
    faults.maybe_fire_end()  # the reference's commented-out sys.exit(1) (train.py:129), as a flag
    return 0


if __name__ == "__main__":
    from distributed_gpu_test_amd.runtime.tiny_trainer import ExchangeFailure, ReplicaDivergence
    try:
        rc = main()
    except (ReplicaDivergence, ExchangeFailure) as e:  # --strict-exchange: every rank raises it, rc 2
        print(f"[dgt] FATAL: {e}", file=sys.stderr, flush=True)
        rc = 2
    comm.destroy()
    sys.exit(rc)
