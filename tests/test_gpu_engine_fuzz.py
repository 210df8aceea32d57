"""Differential fuzz of the engine's host fast paths against plain PyTorch.

Reference: ``engine(x)`` / ``engine.backward(loss)`` / ``engine.step()`` (``train.py:107,113-114``).

The engine's eager step has grown fast paths that keep state across steps: the graphed module
(forward / backward replays, bound-address graphs with an LRU of 4, the graphed tail that runs Adam
inside ``backward``), the whole-step HIP graph, the direct backward without autograd, deferred
zeroing of the gradient bucket, the persistent unit seed.  Each test below drives the reference
model (SimpleNet 20-64-1, fp32) through ``SEEDS`` x ``STEPS`` random transitions and compares the
parameters with ``torch.optim.Adam`` + autograd fed the same batches:

* eager <-> ``graph_module`` (replays, bound graphs, the tail) <-> whole-step graph (``graph_step``);
* batch sizes beyond the 4 graphed signatures (eager steps in a graphed engine) and more than 4
  batch addresses per shape (bound-graph eviction);
* ``retain_graph=True``, a user-set ``.grad``, learning-rate changes, ``gradient_accumulation_steps=2``;
* torch's ``nn.BCEWithLogitsLoss`` vs the framework's fused loss.

``test_fuzz_catches_defer_bug`` re-introduces the ADVICE r4 bug (deferred zeroing under
graph_module: a graphed backward adding onto a stale bucket) and checks that the fuzz fails on it.
"""
import copy
import os
import random

import pytest
import torch

os.environ.setdefault("DGT_QUIET", "1")
import distributed_gpu_test_amd as dgt  # noqa: E402

pytestmark = pytest.mark.gpu

# DGT_FUZZ_SEEDS=N widens the sweep to seeds 0 .. N-1 (a long run; the suite's default is 3)
SEEDS = tuple(range(int(os.environ.get("DGT_FUZZ_SEEDS", "3") or 3)))
STEPS = 200
RTOL, ATOL = 1e-4, 1e-6


def _pool(X, Y, sizes, per_size, rnd):
    """Per batch size, ``per_size`` batches at distinct addresses (all alive): > 4 addresses per
    shape, so bound graphs are created, reused and evicted."""
    pool = {}
    for b in sizes:
        pool[b] = []
        for _ in range(per_size):
            rows = torch.tensor([rnd.randrange(X.shape[0]) for _ in range(b)], device=X.device)
            pool[b].append((X[rows].contiguous(), Y[rows].contiguous()))
    return pool


def _fuzz(seed: int, mode: str, steps: int = STEPS, mutate=None, check_every: int = 50):
    """Returns the list of (step, max abs diff, allowed) at each checkpoint; raises on mismatch."""
    from distributed_gpu_test_amd.models import SimpleNet
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
    rnd = random.Random(1000 + seed)
    torch.manual_seed(seed)
    model = SimpleNet(20, 64)
    ref = copy.deepcopy(model).cuda()
    gas = 2 if mode == "gas2" else 1
    amd = {"graph_module": mode == "graph_module"}
    cfg = {"train_micro_batch_size_per_gpu": 4, "gradient_accumulation_steps": gas, "amd": amd}
    lr = 1e-3
    client = torch.optim.Adam(model.parameters(), lr=lr)
    engine, _, _, _ = dgt.initialize(model=model, optimizer=client, config=cfg)
    if mutate is not None:
        mutate(engine)
    ref_opt = torch.optim.Adam(ref.parameters(), lr=lr)
    X = torch.randn(512, 20, device="cuda")
    Y = (X[:, :10].sum(1, keepdim=True) > 0).float()
    # 6 shapes: 2 of them beyond the graphed engine's 4 signatures run eagerly
    sizes = (4, 8, 2, 3, 5, 6)
    pool = _pool(X, Y, sizes, 6, rnd)
    fw_crit, t_crit = BCEWithLogitsLoss(), torch.nn.BCEWithLogitsLoss()
    whole = None
    if mode == "whole_step":
        whole = engine.graph_step(lambda bx, by: fw_crit(engine(bx), by))
        assert engine.graphed is not None, engine.graph_fallback_reason
    ref_params = list(ref.parameters())
    micro = 0
    checks = []
    counts = {"whole": 0, "retain": 0, "user_grad": 0, "lr": 0, "torch_bce": 0}
    hist = []  # (step, what it did): the failure message carries the last few
    for s in range(steps):
        window_start = micro % gas == 0
        if window_start and rnd.random() < 0.05:  # lr change (the client optimizer's, read each step)
            lr = rnd.choice([1e-3, 5e-4, 2e-3])
            client.param_groups[0]["lr"] = lr
            for g in ref_opt.param_groups:
                g["lr"] = lr
            counts["lr"] += 1
        b = rnd.choice(sizes)
        x, y = rnd.choice(pool[b])
        if whole is not None and rnd.random() < 0.5:
            whole(x, y)  # forward + backward + Adam as one replay
            counts["whole"] += 1
            hist.append((s, f"whole B={b}"))
            ref_loss = torch.nn.functional.binary_cross_entropy_with_logits(ref(x), y)
            ref_opt.zero_grad(set_to_none=True)
            ref_loss.backward()
            ref_opt.step()
            ref_opt.zero_grad(set_to_none=True)
            micro += 1
        else:
            user_grad = window_start and rnd.random() < 0.06
            if user_grad:  # a user-set .grad at the start of a window: backward accumulates onto it
                k = rnd.randrange(len(ref_params))
                c = torch.full_like(ref_params[k], rnd.choice([1e-3, -2e-3]))
                list(model.parameters())[k].grad = c.clone()
                ref_params[k].grad = c.clone()
                counts["user_grad"] += 1
            use_torch = rnd.random() < 0.4
            counts["torch_bce"] += int(use_torch)
            loss = (t_crit if use_torch else fw_crit)(engine(x), y)
            retain = rnd.random() < 0.1
            counts["retain"] += int(retain)
            engine.backward(loss, retain_graph=retain)
            engine.step()
            hist.append((s, f"eager B={b} torch_bce={use_torch} retain={retain} user_grad={user_grad} lr={lr}"))
            ref_loss = torch.nn.functional.binary_cross_entropy_with_logits(ref(x), y)
            (ref_loss / gas).backward(retain_graph=retain)
            micro += 1
            if micro % gas == 0:
                ref_opt.step()
                ref_opt.zero_grad(set_to_none=True)
            del loss
        if (s + 1) % check_every == 0 or s + 1 == steps:
            torch.cuda.synchronize()
            got = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
            want = torch.cat([p.detach().reshape(-1) for p in ref_params])
            diff = (got - want).abs()
            allowed = ATOL + RTOL * want.abs()
            checks.append((s + 1, float(diff.max()), bool((diff <= allowed).all())))
            if not checks[-1][2]:
                engine.close()
                raise AssertionError(f"seed {seed} mode {mode}: parameters left torch's trajectory by step {s + 1} "
                                     f"(max |diff| {checks[-1][1]:.3g}); transitions {counts}; last ops {hist[-6:]}")
    stats = {"counts": counts, "tail_steps": engine.tail_steps, "direct_backwards": engine.direct_backwards,
             "graph_module": engine.graph_module, "evictions": sum(f.evictions for f in engine._graphed_fwd.values()),
             "bound": sum(len(f.bound) for f in engine._graphed_fwd.values()),
             "whole_replays": engine.graphed.replays if engine.graphed is not None else 0}
    engine.close()
    return checks, stats


@pytest.mark.parametrize("seed", SEEDS)
@pytest.mark.parametrize("mode", ["graph_module", "whole_step", "gas2"])
def test_engine_fuzz_matches_torch(mode, seed):
    checks, st = _fuzz(seed, mode)
    assert all(ok for _, _, ok in checks), checks
    c = st["counts"]
    assert c["retain"] > 0 and c["torch_bce"] > 0 and c["user_grad"] > 0
    if mode == "graph_module":
        # the fast paths really ran: the graphed tail, and bound graphs past the LRU
        assert st["graph_module"] and st["tail_steps"] > 0, st
        assert st["evictions"] > 0 or st["bound"] > 0, st
    elif mode == "whole_step":
        assert st["whole_replays"] > 0 and st["direct_backwards"] > 0, st
    # (gas2: the 1/gas-scaled loss takes autograd's path, not the direct backward)


def test_fuzz_catches_defer_bug():
    """deferred zeroing let a graphed backward add onto the last eager step's gradients.
    Re-enabling it under graph_module must make the fuzz fail."""
    def reintroduce(engine):
        engine._defer_capable = True

    failed = 0
    for seed in SEEDS:
        try:
            _fuzz(seed, "graph_module", mutate=reintroduce)
        except AssertionError:
            failed += 1
    assert failed > 0, "the fuzz did not notice deferred zeroing under graph_module"


def test_fuzz_catches_whole_step_counter_bug(monkeypatch):
    """Round 6: the whole-step graph's device step counter was never re-synced after eager steps of
    the same engine (Adam's bias correction then used a stale step).  With the re-sync disabled the
    fuzz must fail."""
    from distributed_gpu_test_amd.runtime import graph_step
    orig = graph_step.GraphedStep._sync

    def stale(self):
        self._step_host = self.e.global_steps - self.e.skipped_steps  # "in sync": never re-filled
        return orig(self)

    monkeypatch.setattr(graph_step.GraphedStep, "_sync", stale)
    failed = 0
    for seed in SEEDS:
        try:
            _fuzz(seed, "whole_step")
        except AssertionError:
            failed += 1
    assert failed > 0, "the fuzz did not notice a stale whole-step step counter"
