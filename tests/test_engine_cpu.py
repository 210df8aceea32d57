"""T1: the engine (DeepSpeed replacement) vs plain PyTorch fp32 references, single process (gloo)."""
import copy
import os

import pytest
import torch

os.environ.setdefault("DGT_QUIET", "1")

import distributed_gpu_test_amd as dgt  # noqa: E402
from distributed_gpu_test_amd.data import make_synthetic_data  # noqa: E402
from distributed_gpu_test_amd.models import SimpleNet  # noqa: E402
from distributed_gpu_test_amd.runtime.flat import FlatLayout  # noqa: E402
from distributed_gpu_test_amd.runtime.schedules import LossScaler, WarmupDecayLR, WarmupLR  # noqa: E402


def _mlp(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(12, 32), torch.nn.ReLU(), torch.nn.Linear(32, 16), torch.nn.Tanh(),
                               torch.nn.Linear(16, 1))


def _batches(n, seed=1, bs=8):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(bs, 12, generator=g), (torch.rand(bs, 1, generator=g) > 0.5).float()) for _ in range(n)]


def _reference_run(model, batches, lr=1e-3, gas=1, clip=0.0, wd=0.0, adamw=False, betas=(0.9, 0.999)):
    opt = (torch.optim.AdamW if adamw else torch.optim.Adam)(model.parameters(), lr=lr, weight_decay=wd, betas=betas)
    crit = torch.nn.BCEWithLogitsLoss()
    for i, (x, y) in enumerate(batches):
        loss = crit(model(x), y) / gas
        loss.backward()
        if (i + 1) % gas == 0:
            if clip > 0:
                torch.nn.utils.clip_grad_norm_(model.parameters(), clip)
            opt.step()
            opt.zero_grad()
    return torch.nn.utils.parameters_to_vector(model.parameters()).detach()


def _engine_run(model, batches, config, optimizer=None):
    engine, _, _, _ = dgt.initialize(model=model, optimizer=optimizer, config=config)
    crit = torch.nn.BCEWithLogitsLoss()
    for x, y in batches:
        loss = crit(engine(x).float(), y)
        engine.backward(loss)
        engine.step()
    out = torch.nn.utils.parameters_to_vector(engine.module.parameters()).detach().float()
    return engine, out


@pytest.mark.parametrize("bucket", [64, 10_000_000])
def test_stage0_matches_torch_adam(bucket):
    m = _mlp()
    ref = _reference_run(copy.deepcopy(m), _batches(12))
    cfg = {"train_batch_size": 8, "zero_optimization": {"stage": 0, "reduce_bucket_size": bucket}}
    engine, got = _engine_run(m, _batches(12), cfg, torch.optim.Adam(m.parameters(), lr=1e-3))
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    assert engine.global_steps == 12
    engine.close()


def test_gradient_accumulation_and_clipping_and_adamw():
    m = _mlp(3)
    ref = _reference_run(copy.deepcopy(m), _batches(12, 5), lr=5e-3, gas=3, clip=0.05, wd=0.1, adamw=True)
    cfg = {"train_micro_batch_size_per_gpu": 8, "gradient_accumulation_steps": 3, "gradient_clipping": 0.05,
           "optimizer": {"type": "AdamW", "params": {"lr": 5e-3, "weight_decay": 0.1}}}
    engine, got = _engine_run(m, _batches(12, 5), cfg)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    assert engine.global_steps == 4
    engine.close()


def test_stage1_single_rank_matches_stage0():
    m = _mlp(4)
    cfg0 = {"train_batch_size": 8, "zero_optimization": {"stage": 0}}
    cfg1 = {"train_batch_size": 8, "zero_optimization": {"stage": 1, "reduce_bucket_size": 100}}
    e0, p0 = _engine_run(copy.deepcopy(m), _batches(6), cfg0)
    e1, p1 = _engine_run(copy.deepcopy(m), _batches(6), cfg1)
    torch.testing.assert_close(p0, p1, rtol=1e-6, atol=1e-7)
    e0.close()
    e1.close()


def test_bf16_engine_runs_with_fp32_master():
    m = _mlp(5)
    cfg = {"train_batch_size": 8, "bf16": {"enabled": True}}
    engine, got = _engine_run(m, _batches(4), cfg)
    assert next(engine.module.parameters()).dtype == torch.bfloat16
    assert engine.master.dtype == torch.float32
    torch.testing.assert_close(engine.master.to(torch.bfloat16), engine.store.param_buf)
    engine.close()


def test_checkpoint_round_trip(tmp_path):
    cfg = {"train_batch_size": 8, "scheduler": {"type": "WarmupLR", "params": {"warmup_num_steps": 5,
                                                                               "warmup_max_lr": 0.01}}}
    m = _mlp(6)
    engine, _ = _engine_run(copy.deepcopy(m), _batches(4), cfg)
    path = engine.save_checkpoint(str(tmp_path), client_state={"epoch": 3})
    assert os.path.exists(os.path.join(tmp_path, "latest"))
    assert open(os.path.join(tmp_path, "latest")).read() == "global_step4"
    assert os.path.exists(os.path.join(path, "mp_rank_00_model_states.pt"))
    crit = torch.nn.BCEWithLogitsLoss()
    for x, y in _batches(3, 9):
        engine.backward(crit(engine(x), y))
        engine.step()
    a = torch.nn.utils.parameters_to_vector(engine.module.parameters()).detach().clone()
    engine.close()

    e2, _, _, _ = dgt.initialize(model=_mlp(99), config=cfg)
    _, client = e2.load_checkpoint(str(tmp_path))
    assert client == {"epoch": 3} and e2.global_steps == 4
    for x, y in _batches(3, 9):
        e2.backward(crit(e2(x), y))
        e2.step()
    b = torch.nn.utils.parameters_to_vector(e2.module.parameters()).detach()
    torch.testing.assert_close(a, b)
    # the optimizer state is torch.optim.Adam's format
    sd = torch.load(os.path.join(path, "mp_rank_00_model_states.pt"), weights_only=True)
    opt = torch.optim.Adam(_mlp().parameters())
    opt.load_state_dict(sd["optimizer"])
    assert sd["global_steps"] == 4 and sd["dp_world_size"] == 1
    e2.close()


def test_bf16_stage0_checkpoint_keeps_fp32_masters(tmp_path):
    """bf16 run: the module holds bf16 weights, so the fp32 masters ride in the optimizer state and a
    resumed run continues bit for bit (the GPU twin: test_train_py_model_mlp_saves_and_resumes_on_gpu)."""
    cfg = {"train_batch_size": 8, "bf16": {"enabled": True}, "zero_optimization": {"stage": 0}}
    crit = torch.nn.BCEWithLogitsLoss()
    engine, _ = _engine_run(_mlp(6), _batches(4), cfg)
    engine.save_checkpoint(str(tmp_path))
    m4 = engine.master.clone()
    for x, y in _batches(3, 9):
        engine.backward(crit(engine(x).float(), y))
        engine.step()
    a, ma = engine.master.clone(), torch.nn.utils.parameters_to_vector(engine.module.parameters()).detach()
    engine.close()
    e2, _, _, _ = dgt.initialize(model=_mlp(99), config=cfg)
    e2.load_checkpoint(str(tmp_path))
    for x, y in _batches(3, 9):
        e2.backward(crit(e2(x).float(), y))
        e2.step()
    assert torch.equal(e2.master, a)
    assert torch.equal(torch.nn.utils.parameters_to_vector(e2.module.parameters()).detach(), ma)
    sd = torch.load(os.path.join(tmp_path, "global_step4", "mp_rank_00_model_states.pt"), weights_only=True)
    assert sd["optimizer"]["single_partition_of_fp32_groups"][0].dtype == torch.float32
    torch.optim.Adam(_mlp().parameters()).load_state_dict(sd["optimizer"])  # still torch Adam's format
    # zero_to_fp32 returns the exact fp32 masters of a bf16 stage-0 run, not the rounded module copy
    from distributed_gpu_test_amd.utils.zero_to_fp32 import consolidate
    full = consolidate(str(tmp_path))
    opt = sd["optimizer"]
    assert opt["fp32_param_names"] == [n for n, _ in _mlp().named_parameters()]
    for name, (off, shape) in zip(opt["fp32_param_names"], opt["fp32_param_segments"]):
        assert full[name].shape == shape
        assert torch.equal(full[name].reshape(-1), m4[off:off + full[name].numel()]), name
    assert any(not torch.equal(full[n], full[n].bfloat16().float()) for n in opt["fp32_param_names"])
    e2.close()


def test_flat_layout_buckets_and_shards():
    shapes = [(64, 20), (64,), (1, 64), (1,)]
    lay = FlatLayout(shapes, bucket_elems=100, world_size=4, shard=True)
    assert all(o % 16 == 0 for o in lay.offsets)
    assert all(b.numel % (16 * 4) == 0 for b in lay.buckets)
    assert lay.buckets[-1].params == [3] or 3 in lay.buckets[-1].params  # last layer reduced first
    covered = sorted(i for b in lay.buckets for i in b.params)
    assert covered == [0, 1, 2, 3]
    assert sum(n for _, n in lay.shard_ranges(2)) == lay.shard_numel()


def test_flat_layout_units_keep_layers_whole():
    """Round 6: a layer's weight and bias never straddle buckets; a layer bigger than the bucket size is
    a bucket of its own (bias included) -- one collective per layer, launched when the layer is done."""
    import pytest
    shapes = [(4096, 4096), (4096,)] * 4 + [(1, 4096), (1,)]
    units = [[0, 1], [2, 3], [4, 5], [6, 7], [8, 9]]
    lay = FlatLayout(shapes, bucket_elems=8 << 20, units=units)
    assert [b.params for b in lay.buckets] == [[0, 1], [2, 3], [4, 5], [6, 7], [8, 9]]
    per_param = FlatLayout(shapes, bucket_elems=8 << 20)  # (the old per-parameter grouping)
    assert len(per_param.buckets) > len(lay.buckets)  # biases were singleton buckets
    # small layers still share a bucket, in backward order
    small = FlatLayout([(8, 4), (8,), (8, 8), (8,), (1, 8), (1,)], bucket_elems=1 << 20, units=[[0, 1], [2, 3], [4, 5]])
    assert [b.params for b in small.buckets] == [[0, 1, 2, 3, 4, 5]]
    with pytest.raises(ValueError):
        FlatLayout(shapes, 1 << 20, units=[[0, 1], [2, 3]])  # units must cover every parameter


def test_engine_layer_units_follow_modules():
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    from distributed_gpu_test_amd.engine import Engine
    from distributed_gpu_test_amd.config import parse_config
    m = SyntheticMLP(64, 3)
    e = Engine(m, parse_config({"train_batch_size": 4, "zero_optimization": {"reduce_bucket_size": 1024}}, 1),
               device=torch.device("cpu"))
    names = dict(enumerate(e.param_names))
    for b in e.layout.buckets:
        owners = {names[i].rsplit(".", 1)[0] for i in b.params}
        for o in owners:  # every bucket holds whole modules: weight and bias together
            assert all(names[i].rsplit(".", 1)[0] != o or i in b.params for i in names)
    e.close()


def test_schedules_and_loss_scaler():
    s = WarmupLR(warmup_min_lr=0.0, warmup_max_lr=1.0, warmup_num_steps=10, warmup_type="linear")
    vals = [s.step() for _ in range(12)]
    assert vals[0] == 0.0 and abs(vals[5] - 0.5) < 1e-9 and vals[11] == 1.0
    d = WarmupDecayLR(total_num_steps=20, warmup_min_lr=0.0, warmup_max_lr=1.0, warmup_num_steps=10,
                      warmup_type="linear")
    vals = [d.step() for _ in range(21)]
    assert vals[10] == 1.0 and abs(vals[15] - 0.5) < 1e-9 and vals[20] == 0.0
    ls = LossScaler(0.0, initial_scale_power=4, scale_window=2, hysteresis=1)
    ls.update(True)
    assert ls.scale == 8.0
    ls.update(False)
    ls.update(False)
    assert ls.scale == 16.0


def test_simplenet_engine_reproduces_reference_epoch_loss():
    torch.manual_seed(42)
    x, y = make_synthetic_data(2000, 20, 42)
    model = SimpleNet(20, 64)
    from distributed_gpu_test_amd.config import REFERENCE_DS_CONFIG
    from distributed_gpu_test_amd.data import SyntheticDataset
    engine, _, _, _ = dgt.initialize(model=model, optimizer=torch.optim.Adam(model.parameters(), lr=1e-3),
                                     config=REFERENCE_DS_CONFIG)
    data = SyntheticDataset(x, y, 4)
    data.set_epoch(1)
    crit = torch.nn.BCEWithLogitsLoss()
    tot = 0.0
    for bx, by in data:
        loss = crit(engine(bx), by)
        engine.backward(loss)
        engine.step()
        tot += loss.item()
    assert round(tot / len(data), 4) == 0.4301  # SURVEY §6.2 oracle, ws=1 epoch 1
    engine.close()


def test_hip_graph_config_falls_back_to_eager_on_cpu():
    import distributed_gpu_test_amd as dgt
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 1))
    engine, _, _, _ = dgt.initialize(model=m, config={"train_batch_size": 4, "amd": {"hip_graph": True}})
    crit = torch.nn.BCEWithLogitsLoss()
    step = engine.graph_step(lambda bx, by: crit(engine(bx), by))
    assert engine.graphed is None and "GPU" in engine.graph_fallback_reason
    x, y = torch.randn(4, 8), (torch.rand(4, 1) > 0.5).float()
    l0 = float(step(x, y))
    for _ in range(20):
        loss = float(step(x, y))
    assert loss < l0 and engine.global_steps == 21
    engine.close()


def test_graph_module_config_parses_and_stays_eager_on_cpu():
    from distributed_gpu_test_amd.config import parse_config
    assert parse_config({"train_batch_size": 4, "amd": {"graph_module": True}}).amd.graph_module
    assert parse_config({"train_batch_size": 4}).amd.fused_linear is None  # auto
    assert parse_config({"train_batch_size": 4, "amd": {"fused_linear": False}}).amd.fused_linear is False
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 1))
    engine, _, _, _ = dgt.initialize(model=m, config={"train_batch_size": 4, "amd": {"graph_module": True}})
    assert engine.graph_module is False  # HIP graphs only: the CPU engine runs the module eagerly
    crit = torch.nn.BCEWithLogitsLoss()
    x, y = torch.randn(4, 8), (torch.rand(4, 1) > 0.5).float()
    engine.backward(crit(engine(x), y))
    engine.step()
    assert engine.global_steps == 1 and not engine._graphed_fwd
    engine.close()


def test_fused_bce_falls_back_to_torch_on_cpu():
    import torch
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
    z = torch.randn(8, 1, requires_grad=True)
    y = (torch.rand(8, 1) > 0.5).float()
    ref_z = z.detach().clone().requires_grad_(True)
    loss = BCEWithLogitsLoss()(z, y)
    ref = torch.nn.BCEWithLogitsLoss()(ref_z, y)
    loss.backward()
    ref.backward()
    assert torch.equal(loss, ref) and torch.equal(z.grad, ref_z.grad)
    acc = torch.zeros(1, dtype=torch.float64)
    BCEWithLogitsLoss(sum_into=acc)(z.detach(), y)
    BCEWithLogitsLoss(sum_into=acc)(z.detach(), y)
    assert torch.equal(acc, torch.zeros(1, dtype=torch.float64).add_(ref.detach()).add_(ref.detach()))
    import pytest
    with pytest.raises(ValueError):
        BCEWithLogitsLoss(sum_into=torch.zeros(1))(z, y)  # fp64 only


def test_inject_fused_linear_keeps_parameters_and_falls_back_on_cpu():
    """Kernel injection swaps Linear(+ReLU) in place: same Parameter objects, same state_dict keys,
    ReLU folded; on CPU the forward falls back to F.linear and matches the original module."""
    from distributed_gpu_test_amd.ops.linear import FusedChain, FusedLinear, inject_fused_linear
    m = _mlp(3)
    ref = copy.deepcopy(m)
    params = [id(p) for p in m.parameters()]
    keys = list(m.state_dict().keys())
    assert inject_fused_linear(m) == 3
    assert [id(p) for p in m.parameters()] == params and list(m.state_dict().keys()) == keys
    assert isinstance(m[0], FusedLinear) and m[0].relu and isinstance(m[1], torch.nn.Identity)
    assert isinstance(m[2], FusedLinear) and not m[2].relu and isinstance(m[3], torch.nn.Tanh)
    nested = SimpleNet()
    nested_ref = copy.deepcopy(nested)
    nested_keys = list(nested.state_dict().keys())
    assert inject_fused_linear(nested) == 2 and nested.net[0].relu
    # a Sequential left holding only fused layers becomes one FusedChain (same object and keys);
    # one with another layer type (the Tanh above) stays a plain Sequential
    assert type(nested.net) is FusedChain and list(nested.state_dict().keys()) == nested_keys
    assert type(m) is torch.nn.Sequential
    x = torch.randn(5, 12)
    torch.testing.assert_close(m(x), ref(x))
    x20 = torch.randn(4, 20)
    torch.testing.assert_close(nested(x20), nested_ref(x20))


def test_inject_fused_linear_fuses_synthetic_mlp_relus():
    """SyntheticMLP applies its ReLUs with torch.relu in forward (no ReLU modules to fold): the fp32
    injection swaps in FusedSyntheticMLP, whose layers carry relu=True and whose head does not -- the
    same Parameter objects and state_dict keys, still a SyntheticMLP, the same outputs and gradients
    on the CPU fallback, and a second injection changes nothing."""
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    from distributed_gpu_test_amd.ops.linear import FusedLinear, FusedSyntheticMLP, inject_fused_linear
    torch.manual_seed(0)
    m = SyntheticMLP(32, 3)
    ref = copy.deepcopy(m)
    params, keys = [id(p) for p in m.parameters()], list(m.state_dict().keys())
    assert inject_fused_linear(m) == 4
    assert type(m) is FusedSyntheticMLP and isinstance(m, SyntheticMLP)
    assert [id(p) for p in m.parameters()] == params and list(m.state_dict().keys()) == keys
    assert all(isinstance(l, FusedLinear) and l.relu for l in m.layers)
    assert isinstance(m.head, FusedLinear) and not m.head.relu
    x = torch.randn(6, 32)
    out, want = m(x), ref(x)
    torch.testing.assert_close(out, want)
    out.sum().backward()
    want.sum().backward()
    for p, q in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, q.grad)
    assert inject_fused_linear(m) == 0 and type(m) is FusedSyntheticMLP


class _ScaleGradInPlace(torch.autograd.Function):
    """A user Function whose backward edits grad_output IN PLACE (legal autograd code)."""

    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return g.mul_(3.0)


@pytest.mark.parametrize("gas", [1, 2])
def test_backward_seed_survives_in_place_grad_output(gas):
    """a loss whose grad_fn edits its incoming gradient in place must not corrupt later
    steps through a shared backward seed: the engine's trajectory equals plain torch's."""
    m = _mlp(21)
    ref = copy.deepcopy(m)
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    crit = torch.nn.BCEWithLogitsLoss()
    batches = _batches(6, 22)
    for i, (x, y) in enumerate(batches):
        (_ScaleGradInPlace.apply(crit(ref(x), y)) / gas).backward()
        if (i + 1) % gas == 0:
            opt.step()
            opt.zero_grad()
    engine, _, _, _ = dgt.initialize(model=m, optimizer=torch.optim.Adam(m.parameters(), lr=1e-3),
                                     config={"train_micro_batch_size_per_gpu": 8, "gradient_accumulation_steps": gas})
    for x, y in batches:
        engine.backward(_ScaleGradInPlace.apply(crit(engine(x), y)))
        engine.step()
    got = torch.nn.utils.parameters_to_vector(engine.module.parameters()).detach()
    want = torch.nn.utils.parameters_to_vector(ref.parameters()).detach()
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-6)
    engine.close()


def test_allgather_bucket_size_groups_buckets():
    """ZeRO's all-gather is grouped by allgather_bucket_size (one coalesced RCCL
    launch per group on GPUs): a small size splits the reduce buckets into several groups, the
    default (8M elements = 32 MiB fp32) keeps them in one; numerics are unchanged."""
    torch.manual_seed(23)
    m = torch.nn.Sequential(torch.nn.Linear(12, 256), torch.nn.ReLU(), torch.nn.Linear(256, 64), torch.nn.Tanh(),
                            torch.nn.Linear(64, 1))
    base = {"train_batch_size": 8}
    cap = 5000
    e_small, p_small = _engine_run(copy.deepcopy(m), _batches(4, 24), dict(base, zero_optimization={
        "stage": 1, "reduce_bucket_size": 1024, "allgather_bucket_size": cap}))
    e_def, p_def = _engine_run(copy.deepcopy(m), _batches(4, 24), dict(base, zero_optimization={
        "stage": 1, "reduce_bucket_size": 1024}))
    assert e_small.config.zero.allgather_bucket_size == cap
    assert e_def.config.zero.allgather_bucket_size == 8 * 1024 * 1024
    g_small, g_def = e_small._allgather_group_plan(), e_def._allgather_group_plan()
    nb = len(e_small.layout.buckets)
    assert nb > 2 and len(g_def) == 1 and 1 < len(g_small) <= nb
    assert sorted(i for g in g_small for i in g) == list(range(nb))
    for g in g_small:  # every group fits the cap unless it is a single oversized bucket
        assert len(g) == 1 or sum(e_small.layout.buckets[i].numel for i in g) <= cap
    torch.testing.assert_close(p_small, p_def, rtol=0, atol=0)
    e_small.close()
    e_def.close()


def test_zero_to_fp32_rejects_duplicated_index_shards(tmp_path):
    """Element-wise ZeRO shards must cover every element exactly once: an index listed twice (and
    so another one missing) is an error, not a silent overwrite."""
    from distributed_gpu_test_amd.utils.zero_to_fp32 import consolidate
    tag = tmp_path / "global_step1"
    tag.mkdir()
    (tmp_path / "latest").write_text("global_step1")
    torch.save({"module": {"w": torch.zeros(4)}}, tag / "mp_rank_00_model_states.pt")
    meta = {"partition_world_size": 2, "total": 4, "names": ["w"], "offsets": [0], "shapes": [(4,)]}

    def shards(i0, i1):
        for r, idx in enumerate((i0, i1)):
            st = dict(meta, index=torch.tensor(idx), fp32_flat=torch.tensor([float(v + 1) for v in idx]))
            torch.save({"optimizer_state_dict": st}, tag / f"zero_pp_rank_{r}_mp_rank_00_optim_states.pt")

    shards([0, 2], [1, 3])
    assert torch.equal(consolidate(str(tmp_path))["w"], torch.tensor([1.0, 2.0, 3.0, 4.0]))
    shards([0, 0], [1, 3])  # element 0 twice, element 2 never
    with pytest.raises(RuntimeError, match="exactly once"):
        consolidate(str(tmp_path))
    shards([0, 2], [2, 3])  # element 2 from both ranks
    with pytest.raises(RuntimeError, match="exactly once"):
        consolidate(str(tmp_path))


def test_mlp_trainer_bucket_plan_cpu():
    """MLPTrainer's gradient buckets (bench.py --bucket-mb): contiguous pieces from the top of the
    weight region, each a multiple of ALIGN x world_size elements, issued after the wgrad of the
    lowest layer they touch; every layer's update waits for the last bucket covering it."""
    import torch
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    from distributed_gpu_test_amd.runtime.mlp_trainer import ALIGN, MLPTrainer
    torch.manual_seed(0)
    model = SyntheticMLP(width=128, depth=3)
    per_layer = MLPTrainer(model, batch_size=64, n_batches=1, device=torch.device("cpu"))
    L, n = 3, 128 * 128
    assert per_layer.buckets == [(per_layer.w_off[i], per_layer.w_off[i] + per_layer.w_len[i]) for i in (2, 1, 0)]
    assert per_layer.update_after == [0, 1, 2] and per_layer.bucket_mb is None
    # 0.01 MiB of bf16 = 5,242 elements -> 5,184 (a multiple of 64): each layer in 4 pieces, the
    # cuts not aligned with the layer boundaries
    t = MLPTrainer(model, batch_size=64, n_batches=1, device=torch.device("cpu"), bucket_mb=0.01)
    spans = t.buckets
    assert spans[0][1] == t.total_w and spans[-1][0] == 0
    assert all(a[0] == b[1] for a, b in zip(spans, spans[1:]))  # contiguous, descending
    assert all((hi - lo) % ALIGN == 0 and hi - lo <= 5184 for lo, hi in spans)
    assert sorted(b for bs in t.bucket_ready for b in bs) == list(range(len(spans)))
    for i in range(L):
        lo_layer = t.w_off[i]
        last = next(lo for lo, hi in spans if lo <= lo_layer < hi)
        assert t.update_after[i] == max(j for j in range(L) if t.w_off[j] <= last) <= i
    # one bucket for everything: issued after layer 0's wgrad, every update after it
    big = MLPTrainer(model, batch_size=64, n_batches=1, device=torch.device("cpu"), bucket_mb=64)
    assert big.buckets == [(0, big.total_w)] and big.update_after == [0, 0, 0] and big.bucket_ready[0] == [0]
    assert n * L <= big.total_w


def test_adam_flat_step_ticket_cpu_advances_counter():
    """adam_flat_ on CPU with step_dev + step_ticket: the update is step_dev + 1 and step_dev advances,
    as the HIP kernel does (tests/test_gpu_tiny_mlp.py)."""
    import torch
    from distributed_gpu_test_amd.ops import adam_flat_
    p = torch.randn(8)
    m, v = torch.zeros(8), torch.zeros(8)
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    step_dev = torch.full((), 2, dtype=torch.int64)
    gr = torch.randn(8)
    adam_flat_(p, gr, m, v, 1, 1e-3, step_dev=step_dev, step_ticket=torch.zeros((), dtype=torch.int32))
    adam_flat_(p2, gr, m2, v2, 3, 1e-3)
    assert int(step_dev) == 3 and torch.equal(p, p2)


def test_fast_apply_matches_function_apply_and_functorch():
    """utils/fnapply.fast_apply: the C++ Function.apply entry gives the same outputs and gradients as
    Function.apply, and under a functorch transform it defers to Function.apply."""
    import torch
    from distributed_gpu_test_amd.utils.fnapply import fast_apply

    class Sq(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, k):
            ctx.save_for_backward(x)
            ctx.k = k
            return x * x * k

        @staticmethod
        def backward(ctx, g):
            (x,) = ctx.saved_tensors
            return 2 * x * ctx.k * g, None

        @staticmethod
        def setup_context(ctx, inputs, output):  # makes the class functorch-capable
            x, k = inputs
            ctx.save_for_backward(x)
            ctx.k = k

    class Plain(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, k):
            ctx.save_for_backward(x)
            ctx.k = k
            return x * x * k

        @staticmethod
        def backward(ctx, g):
            (x,) = ctx.saved_tensors
            return 2 * x * ctx.k * g, None

    fast = fast_apply(Plain)
    x1 = torch.randn(5, requires_grad=True)
    x2 = x1.detach().clone().requires_grad_(True)
    fast(x1, 3.0).sum().backward()
    Plain.apply(x2, 3.0).sum().backward()
    assert torch.equal(x1.grad, x2.grad)
    # a class with setup_context keeps Function.apply (it binds default arguments)
    assert fast_apply(Sq) == Sq.apply
    # under a functorch transform the wrapper defers to Function.apply (which raises for a class
    # without setup_context, exactly as calling Function.apply directly would)
    import pytest
    with pytest.raises(RuntimeError):
        torch.func.grad(lambda t: fast(t, 3.0).sum())(torch.randn(5))


def test_bound_runner_policy_lru_budget_and_churn(monkeypatch):
    """Engine._bound_runner (graph_module's in-place input graphs), the host policy alone (a stand-in
    for GraphedModule, no GPU): an address is bound once seen twice in the last 8 calls; at most
    MAX_BOUND_ADDRESSES pairs; a pair unused for 16 calls makes room for a new address; a churning
    pattern stops binding after 16 evictions; the memory budget caps the pairs."""
    import types
    from distributed_gpu_test_amd import engine as eng_mod
    from distributed_gpu_test_amd.runtime import graph_module as gm

    made = []

    class FakeRunner:
        def __init__(self, module, params, args, warmup=2, tail=None, bind_inputs=False):
            assert bind_inputs and warmup == 0
            self.pending = False
            made.append(args[0].data_ptr())

    monkeypatch.setattr(gm, "GraphedModule", FakeRunner)

    class FakeTensor:
        def __init__(self, p):
            self.p = p
            self.requires_grad = False

        def data_ptr(self):
            return self.p

        def is_contiguous(self):
            return True

    def fresh_fn(footprint=0):
        return types.SimpleNamespace(bound={}, recent=(), bind_failed=None, calls=0, evictions=0,
                                     footprint=footprint)

    eng = types.SimpleNamespace(MAX_BOUND_ADDRESSES=eng_mod.Engine.MAX_BOUND_ADDRESSES,
                                BIND_BUDGET_BYTES=eng_mod.Engine.BIND_BUDGET_BYTES, _runners=[],
                                module=None, params=[], store=types.SimpleNamespace(rebind_grads=lambda: False),
                                _tail_callable=lambda: None)
    call = lambda fn, p: eng_mod.Engine._bound_runner(eng, fn, FakeTensor(p))  # noqa: E731

    fn = fresh_fn()
    # a period-3 address cycle: each address is bound on its third appearance, then reused
    seq = [0, 512, 1024] * 6
    got = [call(fn, p) is not None for p in seq]
    assert made == [0, 512, 1024] and sum(got) == len(seq) - 6
    # a new phase of addresses: the old pairs go stale (unused for > 16 calls) and make room
    made.clear()
    for p in [4096, 8192] * 12:
        call(fn, p)
    assert made == [4096, 8192] and len(fn.bound) <= eng.MAX_BOUND_ADDRESSES and fn.evictions >= 1
    # churn: every address new twice in a row -> evictions run out, binding stops
    fn2 = fresh_fn()
    for k in range(40):
        for _ in range(3):  # a new address, bound on its third call
            call(fn2, (1 << 20) + k * 64)
        for _ in range(17):  # ... then aged past the 16-call window by another (bound) address
            call(fn2, 7)
    assert fn2.bind_failed == "input addresses keep changing" and fn2.evictions == 16
    # budget: a pair the size of the budget leaves no room for a second one
    fn3 = fresh_fn(footprint=eng.BIND_BUDGET_BYTES)
    for q in [1, 1, 1, 2, 2, 2]:
        call(fn3, q)
    assert list(fn3.bound) == [1]


def test_bce_module_call_keeps_hooks():
    """ops.BCEWithLogitsLoss skips nn.Module's call path only when no hook could observe the call:
    with a forward hook registered the hook fires, and the value is torch's either way."""
    import torch
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
    z, y = torch.randn(6, 1), (torch.rand(6, 1) > 0.5).float()
    crit = BCEWithLogitsLoss()
    want = torch.nn.functional.binary_cross_entropy_with_logits(z, y)
    assert torch.allclose(crit(z, y), want)
    seen = []
    h = crit.register_forward_hook(lambda m, args, out: seen.append(float(out)))
    assert torch.allclose(crit(z, y), want) and len(seen) == 1
    h.remove()
    crit(z, y)
    assert len(seen) == 1
