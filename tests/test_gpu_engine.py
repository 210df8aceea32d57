"""The generic engine on the GPU (fused HIP Adam over flat buffers) vs plain PyTorch fp32."""
import copy
import json
import os

import pytest
import torch

os.environ.setdefault("DGT_QUIET", "1")
import distributed_gpu_test_amd as dgt  # noqa: E402

pytestmark = pytest.mark.gpu


def _mlp(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.ReLU(), torch.nn.Linear(256, 1))


def _batches(n, seed=1, bs=32):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(bs, 64, generator=g).cuda(), (torch.rand(bs, 1, generator=g) > 0.5).float().cuda())
            for _ in range(n)]


def test_engine_gpu_fp32_matches_torch():
    m = _mlp()
    ref = copy.deepcopy(m).cuda()
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    crit = torch.nn.BCEWithLogitsLoss()
    for x, y in _batches(10):
        opt.zero_grad()
        crit(ref(x), y).backward()
        opt.step()
    engine, _, _, _ = dgt.initialize(model=m, optimizer=torch.optim.Adam(m.parameters(), lr=1e-3),
                                     config={"train_batch_size": 32, "gradient_clipping": 0.0})
    assert engine.device.type == "cuda"
    for x, y in _batches(10):
        engine.backward(crit(engine(x), y))
        engine.step()
    got = torch.nn.utils.parameters_to_vector(engine.module.parameters())
    want = torch.nn.utils.parameters_to_vector(ref.parameters())
    torch.testing.assert_close(got, want, rtol=2e-4, atol=2e-5)
    engine.close()


def test_engine_gpu_bf16():
    m = _mlp(2)
    engine, _, _, _ = dgt.initialize(model=m, config={"train_batch_size": 32, "bf16": {"enabled": True},
                                                      "communication_data_type": "fp32"})
    crit = torch.nn.BCEWithLogitsLoss()
    first = None
    for x, y in _batches(30, 3):
        loss = crit(engine(x).float(), y)
        first = first if first is not None else float(loss)
        engine.backward(loss)
        engine.step()
    assert float(loss) < first
    torch.testing.assert_close(engine.master.to(torch.bfloat16), engine.store.param_buf)
    engine.close()


def _run_engine(cfg, batches, seed=4, graph=False, crit=None):
    m = _mlp(seed)
    engine, _, _, _ = dgt.initialize(model=m, optimizer=torch.optim.Adam(m.parameters(), lr=1e-3), config=cfg)
    crit = crit or torch.nn.BCEWithLogitsLoss()
    losses = []
    if graph:
        step = engine.graph_step(lambda bx, by: crit(engine(bx).float(), by))
        assert engine.graphed is not None, engine.graph_fallback_reason
        for x, y in batches:
            losses.append(float(step(x, y)))  # the static loss must be read before the next replay
    else:
        for x, y in batches:
            loss = crit(engine(x).float(), y)
            engine.backward(loss)
            engine.step()
            losses.append(float(loss))
    params = engine.store.param_buf.detach().clone()
    return engine, losses, params


@pytest.mark.parametrize("extra", [{}, {"gradient_clipping": 0.5}, {"zero_optimization": {"stage": 1}}])
def test_engine_hip_graph_matches_eager(extra):
    """Whole-step HIP-graph replay (forward + backward + Adam from a device step counter) gives the
    eager engine's trajectory, including a second captured shape (a short batch)."""
    batches = _batches(12, 5) + _batches(1, 6, bs=8) + _batches(12, 7) + _batches(4, 8, bs=8)
    cfg = {"train_batch_size": 32, **extra}
    e1, l1, p1 = _run_engine(dict(cfg), batches)
    e2, l2, p2 = _run_engine(dict(cfg, amd={"hip_graph": True}), batches, graph=True)
    assert e2.graphed.replays >= 20 and not e2.graphed.failed, (e2.graphed.replays, e2.graphed.failed)
    assert len(e2.graphed.graphs) == 2  # one per input shape
    assert e2.global_steps == len(batches)
    torch.testing.assert_close(torch.tensor(l2), torch.tensor(l1), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(p2, p1, rtol=1e-5, atol=1e-6)
    e1.close()
    e2.close()


@pytest.mark.parametrize("extra", [{}, {"gradient_clipping": 0.5}, {"zero_optimization": {"stage": 1}},
                                   {"gradient_accumulation_steps": 2, "train_batch_size": 64},
                                   {"bf16": {"enabled": True}}])
def test_engine_graph_module_matches_eager(extra):
    """amd.graph_module: the module's forward and backward replay HIP graphs under the ordinary
    engine(x) / backward / step calls.  Same kernels, same accumulation order: the trajectory
    matches the eager engine, across a second input shape (a short batch)."""
    batches = _batches(10, 5) + _batches(1, 6, bs=8) + _batches(10, 7) + _batches(3, 8, bs=8)
    cfg = {"train_batch_size": 32, **extra}
    e1, l1, p1 = _run_engine(dict(cfg), batches)
    e2, l2, p2 = _run_engine(dict(cfg, amd={"graph_module": True}), batches)
    assert e2.graph_module, e2.graph_module_reason
    assert len(e2._graphed_fwd) == 2  # one graph pair per input shape
    torch.testing.assert_close(torch.tensor(l2), torch.tensor(l1), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(p2, p1, rtol=1e-5, atol=1e-6)
    e1.close()
    e2.close()


@pytest.mark.parametrize("extra", [{}, {"gradient_clipping": 0.5}, {"zero_optimization": {"stage": 1}},
                                   {"bf16": {"enabled": True}}, {"gradient_accumulation_steps": 2,
                                                                 "train_batch_size": 64}])
def test_engine_graph_tail_matches_eager(extra):
    """amd.graph_module with the framework's fused BCE: engine.backward replays backward + collective +
    clip + Adam as one graph (engine.step() only counts), across two input shapes; the trajectory
    matches the eager engine.  gas = 2 needs a host decision per micro-step: no tail, same results."""
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
    batches = _batches(10, 5) + _batches(1, 6, bs=8) + _batches(10, 7) + _batches(3, 8, bs=8)
    cfg = {"train_batch_size": 32, **extra}
    e1, l1, p1 = _run_engine(dict(cfg), batches, crit=BCEWithLogitsLoss())
    e2, l2, p2 = _run_engine(dict(cfg, amd={"graph_module": True}), batches, crit=BCEWithLogitsLoss())
    assert e2.graph_module, e2.graph_module_reason
    if "gradient_accumulation_steps" in extra:
        assert e2.tail_steps == 0 and "gradient_accumulation" in e2.tail_reason
    else:
        assert e2.tail_steps == len(batches), (e2.tail_steps, e2.tail_reason)
    assert e1.global_steps == e2.global_steps
    tol = dict(rtol=2e-2, atol=2e-3) if "bf16" in extra else dict(rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(torch.tensor(l2), torch.tensor(l1), **tol)
    torch.testing.assert_close(p2.float(), p1.float(), **tol)
    # after the tail the gradient bucket is zero, as after an eager step
    assert not e2.store.grad_buf.any()
    e1.close()
    e2.close()


def test_engine_graph_tail_falls_back_for_other_losses_and_lr_changes():
    """A loss the engine cannot differentiate itself (here torch's BCE summed instead of averaged)
    takes the autograd path; a changed lr disables the captured tail (its lr is baked in)."""
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
    m = _mlp(3)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    e, _, _, _ = dgt.initialize(model=m, optimizer=opt, config={"train_batch_size": 32, "amd": {"graph_module": True}})
    fused, torch_bce = BCEWithLogitsLoss(), torch.nn.BCEWithLogitsLoss(reduction="sum")
    for i, (x, y) in enumerate(_batches(6, 9)):
        loss = (fused if i % 2 == 0 else torch_bce)(e(x), y)
        e.backward(loss)
        e.step()
    assert e.tail_steps == 3
    opt.param_groups[0]["lr"] = 5e-4
    x, y = _batches(1, 10)[0]
    e.backward(fused(e(x), y))
    e.step()
    assert e.tail_steps == 3 and "lr" in e.tail_reason
    e.close()


def test_engine_graph_module_shape_cap_and_eval():
    """Beyond MAX_GRAPHED_SHAPES input shapes, and in eval mode, the module runs eagerly."""
    m = _mlp(9)
    engine, _, _, _ = dgt.initialize(model=m, config={"train_batch_size": 32, "amd": {"graph_module": True}})
    crit = torch.nn.BCEWithLogitsLoss()
    for bs in (4, 8, 12, 16, 20, 24):
        x, y = _batches(1, bs, bs=bs)[0]
        engine.backward(crit(engine(x), y))
        engine.step()
    assert len(engine._graphed_fwd) == engine.MAX_GRAPHED_SHAPES and engine.graph_module
    engine.eval()
    with torch.no_grad():
        out = engine(_batches(1, 3, bs=5)[0][0])
    assert out.shape == (5, 1)
    engine.close()


@pytest.mark.parametrize("bf16", [False, True])
def test_engine_graph_module_after_eager_step_keeps_gradients(bf16):
    """graph_module + the injected kernels, an eager step (a 5th input shape, past
    MAX_GRAPHED_SHAPES) followed by graphed steps whose loss is torch's BCE (no graphed tail): the
    graphed backward must not add onto the eager step's gradients, nor lose its own.  The whole
    trajectory matches the engine without graph_module."""
    sizes = [32, 8, 12, 16, 20, 32, 8, 20, 32, 32, 12, 20, 16]
    g = torch.Generator().manual_seed(11)
    batches = [(torch.randn(bs, 64, generator=g).cuda(), (torch.rand(bs, 1, generator=g) > 0.5).float().cuda())
               for bs in sizes]
    cfg = {"train_batch_size": 32, **({"bf16": {"enabled": True}} if bf16 else {})}
    e1, l1, p1 = _run_engine(dict(cfg), batches)
    e2, l2, p2 = _run_engine(dict(cfg, amd={"graph_module": True}), batches)
    assert e2.graph_module and len(e2._graphed_fwd) == e2.MAX_GRAPHED_SHAPES
    assert not e2._defer_capable and (bf16 or e2.fused_linear_layers > 0)
    tol = dict(rtol=2e-2, atol=2e-3) if bf16 else dict(rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(torch.tensor(l2), torch.tensor(l1), **tol)
    torch.testing.assert_close(p2.float(), p1.float(), **tol)
    e1.close()
    e2.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,dtype", [(4, torch.float32), (1000, torch.float32), (5000, torch.bfloat16)])
def test_fused_bce_matches_torch(n, dtype):
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
    g = torch.Generator().manual_seed(n)
    z0 = (torch.randn(n, 1, generator=g) * 4).to(dtype)
    y = (torch.rand(n, 1, generator=g) > 0.5).float()
    z = z0.cuda().requires_grad_(True)
    loss = BCEWithLogitsLoss()(z, y.cuda())
    loss.backward()
    zr = z0.float().requires_grad_(True)
    ref = torch.nn.BCEWithLogitsLoss()(zr, y)
    ref.backward()
    torch.testing.assert_close(loss.cpu(), ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(z.grad.float().cpu(), zr.grad, rtol=1e-2 if dtype == torch.bfloat16 else 1e-5,
                               atol=1e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fused_bce_sum_into_is_the_loss_log(dtype):
    """``sum_into``: the loss kernel adds the fp32 loss into an fp64 running sum, bit for bit what
    ``acc.add_(loss.detach())`` gives, and leaves loss and gradient unchanged."""
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
    g = torch.Generator().manual_seed(9)
    acc, ref = torch.zeros(1, dtype=torch.float64, device="cuda"), torch.zeros(1, dtype=torch.float64, device="cuda")
    for _ in range(5):
        z0 = (torch.randn(1000, 1, generator=g) * 3).to(dtype).cuda()
        y = (torch.rand(1000, 1, generator=g) > 0.5).float().cuda()
        za, zb = z0.clone().requires_grad_(True), z0.clone().requires_grad_(True)
        la = BCEWithLogitsLoss(sum_into=acc)(za, y)
        lb = BCEWithLogitsLoss()(zb, y)
        ref.add_(lb.detach())
        la.backward()
        lb.backward()
        assert torch.equal(la, lb) and torch.equal(za.grad, zb.grad)
    assert torch.equal(acc, ref), (acc, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fused_bce_unit_seed_is_bitwise_plain_seed(dtype):
    """The engine's persistent unit seed returns the saved gradient (bf16: the kernel's once-rounded
    copy) -- bit for bit autograd's dz * ones cast to the logits' dtype, and the seed stays 1."""
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
    from distributed_gpu_test_amd.ops.loss import unit_seed
    g = torch.Generator().manual_seed(7)
    z0 = (torch.randn(3000, 1, generator=g) * 4).to(dtype).cuda()
    y = (torch.rand(3000, 1, generator=g) > 0.5).float().cuda()
    grads = []
    for seed in (torch.ones((), device="cuda"), unit_seed(torch.device("cuda", 0))):
        z = z0.clone().requires_grad_(True)
        BCEWithLogitsLoss()(z, y).backward(seed)
        assert z.grad.dtype == dtype
        grads.append(z.grad)
    assert torch.equal(grads[0], grads[1])
    assert unit_seed(torch.device("cuda", 0)).item() == 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,relu,bias,need_dx", [(4, 64, 20, True, True, False), (4, 1, 64, False, True, True),
                                                     (7, 33, 19, True, False, True), (256, 128, 96, True, True, True)])
def test_fused_linear_matches_torch(M, N, K, relu, bias, need_dx):
    """csrc/linear.hip forward + one-launch backward vs plain PyTorch fp32 (ReLU mask, dx, dW, db)."""
    from distributed_gpu_test_amd.ops.linear import _FusedLinearFn
    g = torch.Generator().manual_seed(M * 1000 + N)
    x0, w0 = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.3
    b0 = torch.randn(N, generator=g) if bias else None
    dy0 = torch.randn(M, N, generator=g)
    xs = [x0.clone().requires_grad_(need_dx), x0.cuda().requires_grad_(need_dx)]
    ws = [w0.clone().requires_grad_(True), w0.cuda().requires_grad_(True)]
    bs = [None, None] if b0 is None else [b0.clone().requires_grad_(True), b0.cuda().requires_grad_(True)]
    ref = torch.nn.functional.linear(xs[0], ws[0], bs[0])
    ref = torch.relu(ref) if relu else ref
    ref.backward(dy0)
    got = _FusedLinearFn.apply(xs[1], ws[1], bs[1], relu)
    got.backward(dy0.cuda())
    torch.testing.assert_close(got.detach().cpu(), ref.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ws[1].grad.cpu(), ws[0].grad, rtol=1e-5, atol=1e-5)
    if bias:
        torch.testing.assert_close(bs[1].grad.cpu(), bs[0].grad, rtol=1e-5, atol=1e-5)
    if need_dx:
        torch.testing.assert_close(xs[1].grad.cpu(), xs[0].grad, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_engine_fused_linear_matches_plain(graph):
    """Kernel injection ("amd": {"fused_linear": true}) keeps the eager engine's trajectory, eager
    and under whole-step HIP-graph replay."""
    batches = _batches(10, 11) + _batches(2, 12, bs=8)
    base = {"train_batch_size": 32}
    e1, l1, p1 = _run_engine(dict(base, amd={"fused_linear": False}), batches)
    assert e1.fused_linear_layers == 0
    amd = {"fused_linear": True, "hip_graph": graph}
    e2, l2, p2 = _run_engine(dict(base, amd=amd), batches, graph=graph)
    assert e2.fused_linear_layers == 2
    torch.testing.assert_close(torch.tensor(l2), torch.tensor(l1), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(p2, p1, rtol=1e-4, atol=1e-5)
    e1.close()
    e2.close()


@pytest.mark.gpu
def test_fused_linear_grad_in_place_accumulates_and_fires_hooks():
    """grad_in_place backward adds into the existing .grad tensors (two backwards accumulate) and
    fires each parameter's post-accumulate hook once per backward, as AccumulateGrad does."""
    from distributed_gpu_test_amd.ops.linear import inject_fused_linear
    torch.manual_seed(9)
    ref = torch.nn.Sequential(torch.nn.Linear(20, 64), torch.nn.ReLU(), torch.nn.Linear(64, 1)).cuda()
    m = copy.deepcopy(ref)
    assert inject_fused_linear(m, grad_in_place=True) == 2
    fired = []
    for i, p in enumerate(m.parameters()):
        p.grad = torch.zeros_like(p)
        p.register_post_accumulate_grad_hook(lambda _p, i=i: fired.append(i))
    from distributed_gpu_test_amd.ops.linear import engine_backward
    x = torch.randn(4, 20, device="cuda")
    for _ in range(2):
        with engine_backward():  # in place only inside the engine's backward
            m(x).square().sum().backward()
        ref(x).square().sum().backward()
    assert sorted(fired) == [0, 0, 1, 1, 2, 2, 3, 3]
    for p, q in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_engine_fused_linear_auto_default():
    """fused_linear unset = auto: an fp32 GPU engine injects the fused Linear kernels, a bf16 one
    and a graph_module one do not."""
    cases = [({}, 2), ({"amd": {"graph_module": True}}, 2), ({"bf16": {"enabled": True}}, 0),
             ({"amd": {"fused_linear": False}}, 0)]
    for extra, want in cases:
        m = _mlp(4)
        e, _, _, _ = dgt.initialize(model=m, config=dict({"train_batch_size": 32}, **extra))
        assert e.fused_linear_layers == want, extra
        e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("in_place", [False, True])
def test_fused_chain_is_bitwise_per_layer(in_place):
    """A Sequential of fused layers runs as one autograd node (FusedChain): same kernels in the same
    order as layer by layer, so outputs, input gradients and parameter gradients are bit-identical,
    and with grad_in_place every parameter's post-accumulate hook fires once per backward."""
    from distributed_gpu_test_amd.ops.linear import FusedChain, inject_fused_linear
    torch.manual_seed(21)
    base = torch.nn.Sequential(torch.nn.Linear(20, 64), torch.nn.ReLU(), torch.nn.Linear(64, 32),
                               torch.nn.ReLU(), torch.nn.Linear(32, 1)).cuda()
    chain, layered = copy.deepcopy(base), copy.deepcopy(base)
    assert inject_fused_linear(chain, grad_in_place=in_place) == 3 and type(chain) is FusedChain
    inject_fused_linear(layered, grad_in_place=in_place)
    fired = []
    for net in (chain, layered):
        for i, p in enumerate(net.parameters()):
            if in_place:
                p.grad = torch.zeros_like(p)
                p.register_post_accumulate_grad_hook(lambda _p, i=i, net=net: fired.append((id(net), i)))
    from distributed_gpu_test_amd.ops.linear import engine_backward
    x0 = torch.randn(4, 20, device="cuda")
    outs, dxs = [], []
    for net in (chain, layered):
        x = x0.clone().requires_grad_(True)
        for _ in range(2):
            y = net(x) if net is chain else _layer_by_layer(net, x)
            with engine_backward():
                y.square().sum().backward()
        outs.append(y.detach())
        dxs.append(x.grad)
    assert torch.equal(outs[0], outs[1]) and torch.equal(dxs[0], dxs[1])
    for p, q in zip(chain.parameters(), layered.parameters()):
        assert torch.equal(p.grad, q.grad)
    if in_place:
        assert sorted(i for n, i in fired if n == id(chain)) == sorted(list(range(6)) * 2)


def _layer_by_layer(net, x):
    for m in net:
        x = m(x)
    return x


@pytest.mark.gpu
def test_autograd_grad_on_injected_engine_returns_grads():
    """with the default fused-Linear injection (in-place gradients), a plain
    torch.autograd.grad on the engine's parameters returns the right tensors and leaves the flat
    gradient buckets untouched: the kernels accumulate in place only inside engine.backward."""
    m = _mlp(13)
    ref = copy.deepcopy(m).cuda()
    e, _, _, _ = dgt.initialize(model=m, config={"train_batch_size": 32})
    assert e.fused_linear_layers == 2
    x, y = _batches(1, 14)[0]
    crit = torch.nn.BCEWithLogitsLoss()
    gs = torch.autograd.grad(crit(e(x), y), list(e.module.parameters()))
    want = torch.autograd.grad(crit(ref(x), y), list(ref.parameters()))
    assert all(g is not None for g in gs)
    for g, w in zip(gs, want):
        torch.testing.assert_close(g, w, rtol=1e-5, atol=1e-6)
    assert float(e.store.grad_buf.abs().max()) == 0.0
    e.backward(crit(e(x), y))  # the engine's own backward still accumulates in place
    assert float(e.store.grad_buf.abs().max()) > 0.0
    e.close()


@pytest.mark.gpu
def test_fused_chain_frozen_layer_stays_frozen():
    """a layer frozen after injection gets no gradient from the chain's backward, so the
    flat Adam leaves it unchanged; the trainable layers still learn."""
    torch.manual_seed(31)
    m = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.ReLU(), torch.nn.Linear(128, 64), torch.nn.ReLU(),
                            torch.nn.Linear(64, 1))
    e, _, _, _ = dgt.initialize(model=m, config={"train_batch_size": 32})
    assert e.fused_linear_layers == 3
    frozen = e.module[2].weight
    frozen.requires_grad_(False)
    before = frozen.detach().clone()
    head = e.module[4].weight.detach().clone()
    crit = torch.nn.BCEWithLogitsLoss()
    for x, y in _batches(3, 15):
        e.backward(crit(e(x), y))
        e.step()
    assert torch.equal(frozen.detach(), before)
    assert not torch.equal(e.module[4].weight.detach(), head)
    e.close()


@pytest.mark.gpu
def test_graph_module_keeps_buffers_and_rng_and_guards_double_forward():
    """graph_module's capture warmup leaves BatchNorm running stats as they were, and a
    second forward of one signature before the first one's backward runs eagerly (the pending
    backward keeps its activations): both calls' gradients reach the buckets, as in the eager engine.
    Both runs use F.linear (fused_linear off); the captured GEMMs may still pick other hipBLASLt
    algorithms than eager ones (other stream, other workspace), so the first step's gradients are
    compared at fp32-reassociation tolerance and the Adam trajectory at a loose one -- a lost or
    doubled contribution of either call would be off by tens of percent."""
    def net(seed):
        torch.manual_seed(seed)
        return torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.BatchNorm1d(128), torch.nn.ReLU(),
                                   torch.nn.Linear(128, 1))
    crit = torch.nn.BCEWithLogitsLoss()
    res = []
    for amd in ({"graph_module": False, "fused_linear": False}, {"graph_module": True, "fused_linear": False}):
        e, _, _, _ = dgt.initialize(model=net(17), config={"train_batch_size": 32, "amd": amd})
        torch.manual_seed(5)
        losses, first_grad = [], None
        for x, y in _batches(6, 18):
            out1 = e(x)
            out2 = e(x * 0.5)  # same signature, before out1's backward
            loss = crit(out1, y) + crit(out2, y)
            e.backward(loss)
            if first_grad is None:
                first_grad = torch.cat([p.grad.detach().reshape(-1).clone() for p in e.module.parameters()])
            e.step()
            losses.append(float(loss))
        res.append((losses, first_grad, e.store.param_buf.detach().clone(),
                    [b.detach().clone() for b in e.module.buffers()]))
        e.close()
    (l1, g1, p1, b1), (l2, g2, p2, b2) = res
    torch.testing.assert_close(g2, g1, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(torch.tensor(l2), torch.tensor(l1), rtol=2e-2, atol=1e-4)
    torch.testing.assert_close(p2, p1, rtol=0, atol=2e-2)
    for u, v in zip(b1, b2):  # running stats: 12 updates in both runs, none from the capture warmup
        torch.testing.assert_close(u.float(), v.float(), rtol=2e-2, atol=1e-3)


def _bf16_mlp_engine(fused, seed=41, width=512, depth=3, B=256, steps=4, extra=None):
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    from distributed_gpu_test_amd.runtime.engine_mlp import EngineMLPTrainer
    torch.manual_seed(seed)
    cfg = {"train_micro_batch_size_per_gpu": B, "bf16": {"enabled": True},
           "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}, "amd": {"fused_linear": fused}, **(extra or {})}
    tr = EngineMLPTrainer(SyntheticMLP(width, depth), B, 4, cfg)
    losses = []
    for _ in range(steps):
        tr.loss_acc.zero_()
        tr.run_plan(*[t[:1] for t in tr.epoch_plan(1)])
        losses.append(float(tr.loss_acc.item()))
    return tr, losses


@pytest.mark.gpu
def test_engine_bf16_mfma_chain_matches_autograd_engine():
    """a bf16 engine injects the MFMA Linear chain (every Linear incl. the head) and
    follows the trajectory of the same engine on autograd + F.linear within bf16 tolerance."""
    a, la = _bf16_mlp_engine(True)
    b, lb = _bf16_mlp_engine(False)
    assert a.engine.fused_linear_layers == 4 and b.engine.fused_linear_layers == 0
    torch.testing.assert_close(torch.tensor(la), torch.tensor(lb), rtol=2e-2, atol=2e-3)
    torch.testing.assert_close(a.engine.master, b.engine.master, rtol=0, atol=2e-3)
    assert not a.engine.linear_fallbacks or all("MFMA" not in k for k in a.engine.linear_fallbacks)
    a.close()
    b.close()


@pytest.mark.gpu
def test_engine_bf16_gradient_accumulation_uses_accumulating_epilogue():
    """gas = 2: the second micro-step's wgrad / bias row sums accumulate into the bf16 bucket; the
    trajectory still follows the autograd engine."""
    extra = {"gradient_accumulation_steps": 2}
    a, la = _bf16_mlp_engine(True, steps=4, extra=extra)
    b, lb = _bf16_mlp_engine(False, steps=4, extra=extra)
    assert a.engine.global_steps == 2
    torch.testing.assert_close(torch.tensor(la), torch.tensor(lb), rtol=2e-2, atol=2e-3)
    torch.testing.assert_close(a.engine.master, b.engine.master, rtol=0, atol=2e-3)
    a.close()
    b.close()


@pytest.mark.gpu
def test_engine_bf16_chain_called_twice_before_backward():
    """Two forwards of the MFMA chain before one backward, right after zero_grad: each weight
    gradient is written twice in that backward -- stored the first time (the bucket was zero), added
    the second -- and matches the autograd engine's gradient of the same two-call loss."""
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    grads = []
    for fused in (True, False):
        torch.manual_seed(7)
        cfg = {"train_micro_batch_size_per_gpu": 256, "bf16": {"enabled": True},
               "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}, "amd": {"fused_linear": fused}}
        e, _, _, _ = dgt.initialize(model=SyntheticMLP(256, 2), config=cfg)
        g = torch.Generator().manual_seed(3)
        x = torch.randn(256, 256, generator=g).to(torch.bfloat16).cuda()
        y = (torch.rand(256, generator=g) > 0.5).float().cuda()
        crit = torch.nn.BCEWithLogitsLoss()
        loss = crit(e(x).view(-1).float(), y) + crit(e(x * 0.5).view(-1).float(), y)
        e.backward(loss)
        grads.append(torch.cat([p.grad.float().reshape(-1) for p in e.module.parameters()]))
        e.close()
    torch.testing.assert_close(grads[0], grads[1], rtol=3e-2, atol=2e-4)


@pytest.mark.gpu
def test_engine_bf16_deferred_zero_grad_matches_autograd_engine():
    """After a backward that stored every gradient view, the step skips the bucket's zero fill; in
    a step that falls back to F.linear (batch 192: not a multiple of 128) autograd's accumulation
    into the stale views is preceded by a zero of each view (tensor hook), the next step fills the
    bucket again, and every step's gradients match the autograd engine's."""
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    engines = []
    for fused in (True, False):
        torch.manual_seed(11)
        cfg = {"train_micro_batch_size_per_gpu": 256, "bf16": {"enabled": True},
               "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}, "amd": {"fused_linear": fused}}
        engines.append(dgt.initialize(model=SyntheticMLP(256, 2), config=cfg)[0])
    crit = torch.nn.BCEWithLogitsLoss()
    g = torch.Generator().manual_seed(4)
    deferred = []
    for k, B in enumerate((256, 256, 256, 192, 256, 256)):
        x = torch.randn(B, 256, generator=g).to(torch.bfloat16).cuda()
        y = (torch.rand(B, generator=g) > 0.5).float().cuda()
        grads = []
        for e in engines:
            deferred.append(e._zero_deferred)
            if k == 2:  # a user-set gradient on a deferred step folds into a zeroed buffer
                p0 = next(e.module.parameters())
                p0.grad = torch.full_like(p0, 0.01)
            e.backward(crit(e(x).view(-1).float(), y))
            grads.append(torch.cat([p.grad.float().reshape(-1) for p in e.module.parameters()]))
            e.step()
        torch.testing.assert_close(grads[0], grads[1], rtol=3e-2, atol=3e-4)
    assert deferred[0::2] == [False, True, True, True, False, True]  # the fallback step: a real fill after it
    assert not any(deferred[1::2])  # autograd's F.linear path adds: never deferred
    for e in engines:
        e.close()


@pytest.mark.gpu
def test_engine_bf16_step_runs_no_vendor_gemm():
    """The bf16 engine step launches this framework's GEMM / head / Adam kernels and no hipBLASLt
    (Cijk_*) or rocBLAS kernel (torch profiler kernel names of two steps)."""
    from torch.profiler import ProfilerActivity, profile
    tr, _ = _bf16_mlp_engine(True, steps=1)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        tr.run_plan(*tr.epoch_plan(1))
        torch.cuda.synchronize()
    names = [e.key for e in prof.key_averages()]
    assert any("gemm_nt_kernel" in n for n in names), names
    assert any("skinny" in n for n in names) and any("adam_flat" in n for n in names), names
    vendor = [n for n in names if n.startswith("Cijk") or "rocblas" in n.lower() or "gemv" in n.lower()]
    assert not vendor, vendor
    tr.close()


@pytest.mark.gpu
def test_engine_bf16_matches_mlp_trainer():
    """The DeepSpeed-API path and the bench trainer (MLPTrainer) on the same model, data and Adam:
    same trajectory within bf16 tolerance (the engine keeps bf16 biases, MLPTrainer fp32 ones)."""
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    from distributed_gpu_test_amd.runtime.mlp_trainer import MLPTrainer
    eng, le = _bf16_mlp_engine(True, seed=43, steps=3)
    torch.manual_seed(43)
    mt = MLPTrainer(SyntheticMLP(512, 3), batch_size=256, n_batches=4, lr=1e-3, device=torch.device("cuda"))
    lm = []
    for _ in range(3):
        mt.loss_acc.zero_()
        mt.run_plan(*[t[:1] for t in mt.epoch_plan(1)])
        lm.append(float(mt.loss_acc.item()))
    torch.testing.assert_close(torch.tensor(le), torch.tensor(lm), rtol=2e-2, atol=2e-3)
    for i in range(3):
        w_eng = eng.engine.module.layers[i].weight.detach().float()
        w_mt = mt.W[i].float()
        d = (w_eng - w_mt).abs()
        # three Adam steps of lr 1e-3 move a weight by at most ~3e-3: an element whose tiny gradient
        # has opposite signs in the two paths' roundings may differ by up to twice that; the bulk of
        # the weights must agree to within bf16 rounding of the updates
        assert float(d.max()) <= 7e-3, float(d.max())
        # (Adam's first step moves every weight by lr * sign(g): a sign that differs between the two
        # paths' roundings -- a gradient that nearly cancels -- is a 2e-3 gap from step 1 on)
        assert float((d > 2e-3).float().mean()) < 2e-2 and float(d.mean()) < 3e-4, (float(d.mean()), i)
    eng.close()


@pytest.mark.gpu
def test_engine_bf16_mfma_chain_bias_free_linears():
    """a bf16 chain whose Linears have no bias runs the MFMA chain (zero-bias epilogue)
    and follows the autograd engine."""
    import torch.nn as nn

    def run(fused):
        from distributed_gpu_test_amd import initialize
        torch.manual_seed(5)
        model = nn.Sequential(nn.Linear(256, 256, bias=False), nn.ReLU(), nn.Linear(256, 256, bias=False),
                              nn.ReLU(), nn.Linear(256, 1))
        cfg = {"train_micro_batch_size_per_gpu": 128, "bf16": {"enabled": True},
               "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}, "amd": {"fused_linear": fused}}
        eng, _, _, _ = initialize(model=model, config=cfg)
        g = torch.Generator().manual_seed(0)
        x = torch.randn(128, 256, generator=g).cuda()
        y = (torch.randn(128, generator=g) > 0).float().cuda()
        losses = []
        for _ in range(3):
            loss = torch.nn.functional.binary_cross_entropy_with_logits(eng(x).view(-1).float(), y)
            eng.backward(loss)
            eng.step()
            losses.append(float(loss))
        return eng, losses

    a, la = run(True)
    b, lb = run(False)
    assert a.fused_linear_layers == 3
    torch.testing.assert_close(torch.tensor(la), torch.tensor(lb), rtol=2e-2, atol=2e-3)
    torch.testing.assert_close(a.master, b.master, rtol=0, atol=2e-3)
    a.close()
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [{}, {"gradient_clipping": 0.5}, {"zero_optimization": {"stage": 1}}])
def test_engine_direct_backward_matches_autograd(extra):
    """Eager engine + fused BCE of an injected Linear chain: engine.backward calls the two backward
    functions itself (no autograd engine) and fires the bucket hooks; bit-identical to autograd."""
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
    batches = _batches(8, 11) + _batches(2, 12, bs=8)
    cfg = {"train_batch_size": 32, **extra}
    e1, l1, p1 = _run_engine(dict(cfg, amd={"direct_backward": False}), batches, crit=BCEWithLogitsLoss())
    e2, l2, p2 = _run_engine(dict(cfg), batches, crit=BCEWithLogitsLoss())
    assert e1.direct_backwards == 0 and e2.direct_backwards == len(batches)
    assert l1 == l2
    assert torch.equal(p1, p2)
    # torch's own mean BCE takes the direct backward too (d loss / d logits from the fused loss
    # kernel; test_eager_direct_backward_with_torch_bce compares that trajectory with plain torch)
    e3, l3, p3 = _run_engine(dict(cfg), batches)
    assert e3.direct_backwards == len(batches) and all(v == v for v in l3)
    for e in (e1, e2, e3):
        e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("B,F", [(64, 64), (512, 256)])  # the small-batch kernels; the tiled fp32 GEMM
def test_engine_fp32_deferred_zero_grad_direct_backward(B, F):
    """fp32 fused Linear kernels STORE a gradient view on its first write of a backward, so the
    engine defers the bucket's zero fill as for bf16; the direct backward still runs (it calls the
    engine's own tensor hook), a user-set gradient folds into a zeroed buffer, and every step's
    gradients match the autograd engine's on F.linear."""
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
    engines = []
    for fused in (True, False):
        torch.manual_seed(12)
        cfg = {"train_micro_batch_size_per_gpu": B,
               "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}, "amd": {"fused_linear": fused}}
        engines.append(dgt.initialize(model=SyntheticMLP(F, 2), config=cfg)[0])
    crit = BCEWithLogitsLoss()
    g = torch.Generator().manual_seed(5)
    deferred = []
    for k in range(5):
        x = torch.randn(B, F, generator=g).cuda()
        y = (torch.rand(B, generator=g) > 0.5).float().cuda()
        grads = []
        for e in engines:
            deferred.append(e._zero_deferred)
            if k == 2:
                p0 = next(e.module.parameters())
                p0.grad = torch.full_like(p0, 0.01)
            e.backward(crit(e(x).view(-1), y))
            grads.append(torch.cat([p.grad.reshape(-1) for p in e.module.parameters()]))
            e.step()
        torch.testing.assert_close(grads[0], grads[1], rtol=1e-4, atol=1e-6)
    assert deferred[0::2] == [False, True, True, True, True]
    assert not any(deferred[1::2])
    assert engines[0].direct_backwards == 5
    for e in engines:
        e.close()


@pytest.mark.gpu
def test_engine_direct_backward_frees_activations_and_refuses_second_backward():
    """the direct backward frees the chain's activations and d loss / d logits
    at once, as autograd's backward does (not when the caller drops ``loss``), and a second
    backward through the same graph raises instead of adding the gradients again.  With
    retain_graph the autograd path keeps them (and hands out a copy of the unit-seed gradient)."""
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
    torch.manual_seed(13)
    B, F = 8192, 256
    engine = dgt.initialize(model=SyntheticMLP(F, 3), config={
        "train_micro_batch_size_per_gpu": B, "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}})[0]
    crit = BCEWithLogitsLoss()
    g = torch.Generator().manual_seed(6)
    x = torch.randn(B, F, generator=g).cuda()
    y = (torch.rand(B, generator=g) > 0.5).float().cuda()
    engine.backward(crit(engine(x).view(-1), y))  # warm: buffers, kernels
    engine.step()
    torch.cuda.synchronize()
    loss = crit(engine(x).view(-1), y)
    before = torch.cuda.memory_allocated()
    engine.backward(loss)
    torch.cuda.synchronize()
    after = torch.cuda.memory_allocated()
    assert engine.direct_backwards == 2
    # 2 hidden activations of B x F fp32 (+ d loss / d logits) no longer held by the graph
    assert before - after >= 2 * B * F * 4, (before, after)
    with pytest.raises(RuntimeError, match="second time"):
        loss.backward()
    engine.step()
    # retain_graph: the autograd path, the graph stays usable
    loss = crit(engine(x).view(-1), y)
    engine.backward(loss, retain_graph=True)
    node = loss.grad_fn
    assert node.dz is not None and not node.freed
    engine.step()
    engine.close()


@pytest.mark.gpu
@pytest.mark.parametrize("bf16", [False, True])
def test_graph_module_fused_bce_writes_gradient_in_place(bf16):
    """graph_module + the framework's fused BCE: the loss kernel writes d loss / d logits straight into
    the backward graph's static input (no copy before the replay), only for the first loss on a fresh
    forward replay; a second loss on the same output gets its own buffer.  Trajectory as eager."""
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
    crit = BCEWithLogitsLoss()
    cfg = {"train_batch_size": 32, **({"bf16": {"enabled": True}} if bf16 else {})}
    batches = _batches(6, 21)
    e1, l1, p1 = _run_engine(dict(cfg), batches, crit=crit)
    m = _mlp(4)
    e2 = dgt.initialize(model=m, optimizer=torch.optim.Adam(m.parameters(), lr=1e-3),
                        config=dict(cfg, amd={"graph_module": True}))[0]
    losses = []
    for i, (x, y) in enumerate(batches):
        out = e2(x)
        loss = crit(out.float() if not bf16 else out, y)
        # the graph pair this forward replayed (bf16: the engine's cast of x recurs at one address,
        # so a bound pair takes over)
        runner = next((r for r in e2._runners if r.pending), None)
        if i > 0:  # (the first forward of a signature captures; its output is not a replay)
            buf = loss.grad_fn.lp if bf16 else loss.grad_fn.dz
            assert buf.data_ptr() == runner.static_gout[0].data_ptr()
            extra = crit(out.float() if not bf16 else out, y)  # a second loss: its own buffer
            eb = extra.grad_fn.lp if bf16 else extra.grad_fn.dz
            assert eb.data_ptr() != runner.static_gout[0].data_ptr()
            del extra
        e2.backward(loss)
        e2.step()
        losses.append(float(loss))
    tol = dict(rtol=2e-2, atol=2e-3) if bf16 else dict(rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(torch.tensor(losses), torch.tensor(l1), **tol)
    torch.testing.assert_close(e2.store.param_buf.float(), p1.float(), **tol)
    e1.close()
    e2.close()


@pytest.mark.gpu
@pytest.mark.parametrize("in_place", [False, True])
@pytest.mark.parametrize("B,F,H,O,relu_out", [(4, 20, 64, 1, False), (16, 32, 128, 8, True), (3, 17, 40, 5, False)])
def test_fused_chain2_one_launch_is_bitwise_per_layer(B, F, H, O, relu_out, in_place):
    """A two-layer chain (the reference SimpleNet's shape among others) runs forward and backward as
    ONE launch each (csrc/linear.hip linear2_*): outputs, input gradients and parameter gradients
    bit-identical to the layer-by-layer kernels, in place into .grad views or returned."""
    from distributed_gpu_test_amd.ops.linear import FusedChain, engine_backward, inject_fused_linear
    torch.manual_seed(B + F)
    layers = [torch.nn.Linear(F, H), torch.nn.ReLU(), torch.nn.Linear(H, O)] + ([torch.nn.ReLU()] if relu_out else [])
    base = torch.nn.Sequential(*layers).cuda()
    chain, layered = copy.deepcopy(base), copy.deepcopy(base)
    assert inject_fused_linear(chain, grad_in_place=in_place) == 2 and type(chain) is FusedChain
    inject_fused_linear(layered, grad_in_place=in_place)
    for net in (chain, layered):
        for p in net.parameters():
            if in_place:
                p.grad = torch.zeros_like(p)
    x0 = torch.randn(B, F, device="cuda")
    outs, dxs = [], []
    for net in (chain, layered):
        x = x0.clone().requires_grad_(True)
        for _ in range(2):  # the second backward accumulates
            y = net(x) if net is chain else _layer_by_layer(net, x)
            with engine_backward():
                (y * torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y)).sum().backward()
        outs.append(y.detach())
        dxs.append(x.grad)
    assert torch.equal(outs[0], outs[1]) and torch.equal(dxs[0], dxs[1])
    for p, q in zip(chain.parameters(), layered.parameters()):
        assert torch.equal(p.grad, q.grad)


@pytest.mark.gpu
@pytest.mark.parametrize("shape,dtype", [((50, 20), torch.float32), ((50, 1), torch.float32), ((40, 8, 4), torch.float32),
                                         ((33, 6), torch.bfloat16), ((33, 3), torch.bfloat16), ((20, 5), torch.int32)])
def test_gather_batch_matches_index_select(shape, dtype):
    """data.gather_batch: the rows of every dataset tensor in one launch (csrc/data.hip), equal to
    index_select, for 16-byte and 4-byte row words and for rows it cannot take (6-byte bf16 rows:
    index_select itself)."""
    from distributed_gpu_test_amd.data import gather_batch
    g = torch.Generator().manual_seed(shape[0])
    x = (torch.randn(shape, generator=g) * 100).to(dtype).cuda()
    y = torch.randn(shape[0], 1, generator=g).cuda()
    rows = torch.randint(0, shape[0], (17,), generator=g).cuda()
    gx, gy = gather_batch(rows, x, y)
    assert torch.equal(gx, x.index_select(0, rows)) and torch.equal(gy, y.index_select(0, rows))
    assert gx.is_contiguous() and gx.data_ptr() != x.data_ptr()
    e, = gather_batch(rows[:0], x)
    assert e.shape == (0,) + tuple(shape[1:])


@pytest.mark.gpu
def test_gather_batch_out_of_range_is_a_zero_row():
    from distributed_gpu_test_amd.data import gather_batch
    x = torch.arange(1, 41, dtype=torch.float32, device="cuda").view(10, 4)
    got, = gather_batch(torch.tensor([3, 10, -1, 0], device="cuda"), x)
    assert torch.equal(got[0], x[3]) and torch.equal(got[3], x[0]) and not got[1:3].any()


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [{}, {"zero_optimization": {"stage": 1}}, {"bf16": {"enabled": True}}])
def test_graph_module_binds_recurring_input_addresses(extra):
    """graph_module: a loader's fresh batch lands at the same address step after step (the caching
    allocator recycles its block), so the engine captures graphs that read the input in place (no
    copy into a static input) and replays them while the input is there; a batch elsewhere takes the
    copying graph.  The trajectory matches the eager engine, with and without the graphed tail."""
    from distributed_gpu_test_amd.data import gather_batch
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
    g = torch.Generator().manual_seed(31)
    X = torch.randn(400, 64, generator=g).cuda()
    Y = (torch.rand(400, 1, generator=g) > 0.5).float().cuda()
    plan = torch.randint(0, 400, (24, 32), generator=g).cuda()
    cfg = {"train_batch_size": 32, **extra}
    tol = dict(rtol=2e-2, atol=2e-3) if "bf16" in extra else dict(rtol=1e-5, atol=1e-6)
    for crit in (BCEWithLogitsLoss(), torch.nn.BCEWithLogitsLoss()):
        runs = []
        for amd in ({}, {"graph_module": True}):
            m = _mlp(12)
            e = dgt.initialize(model=m, optimizer=torch.optim.Adam(m.parameters(), lr=1e-3),
                               config=dict(cfg, amd=amd))[0]
            losses, keep = [], []
            for s in range(plan.shape[0]):
                xb, yb = gather_batch(plan[s], X, Y)
                if s in (20, 21):
                    keep.append(xb)  # held across steps: the next batches land elsewhere
                loss = crit(e(xb).float(), yb)
                e.backward(loss)
                e.step()
                losses.append(float(loss))
            runs.append((e, losses, e.store.param_buf.detach().float().clone()))
        (e1, l1, p1), (e2, l2, p2) = runs
        fn = next(iter(e2._graphed_fwd.values()))
        assert fn.bound and fn.bind_failed is None, fn.bind_failed
        bound_replays = sum(b.replays for b in fn.bound.values())
        # (how many of the 24 steps land on a bound address depends on the caching allocator's state)
        assert bound_replays >= 8 and fn.replays >= 1, (bound_replays, fn.replays)
        assert all(b.held is None and not b.pending for b in fn.bound.values())
        torch.testing.assert_close(torch.tensor(l2), torch.tensor(l1), **tol)
        torch.testing.assert_close(p2, p1, **tol)
        e1.close()
        e2.close()


@pytest.mark.gpu
def test_graph_module_bound_graph_guards_double_forward_and_off_switch():
    """A second forward of a bound input before its backward runs eagerly (its activations are
    pending); amd.graph_bind_inputs=false never binds."""
    from distributed_gpu_test_amd.data import gather_batch
    X = torch.randn(64, 64, device="cuda")
    Y = (torch.rand(64, 1, device="cuda") > 0.5).float()
    rows = torch.arange(32, device="cuda")
    for bind in (True, False):
        m = _mlp(13)
        e = dgt.initialize(model=m, config={"train_batch_size": 32,
                                            "amd": {"graph_module": True, "graph_bind_inputs": bind}})[0]
        crit = torch.nn.BCEWithLogitsLoss()
        for _ in range(16):  # (an address binds on its third visit; a few addresses may take turns)
            xb, yb = gather_batch(rows, X, Y)
            e.backward(crit(e(xb), yb))
            e.step()
        fn = next(iter(e._graphed_fwd.values()))
        assert bool(fn.bound) == bind
        if bind:
            spare = []
            xb, yb = gather_batch(rows, X, Y)
            while xb.data_ptr() not in fn.bound and len(spare) < 8:  # a batch at a bound address
                spare.append((xb, yb))
                xb, yb = gather_batch(rows, X, Y)
            b = fn.bound[xb.data_ptr()]
            out1 = e(xb)
            assert b.pending and b.held is not None
            out2 = e(xb)  # eager: must not overwrite out1's activations
            assert out2.data_ptr() != out1.data_ptr()
            e.backward(crit(out1, yb) + crit(out2, yb))
            e.step()
            assert not b.pending and b.held is None
        e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [{}, {"zero_optimization": {"stage": 1}}, {"gradient_clipping": 0.5}])
def test_hip_graph_step_with_fused_bce_drops_seed_and_zero_fill(extra):
    """Whole-step HIP graph with the framework's fused BCE: the backward seed is the persistent unit
    (the BCE backward launches nothing) and, since the injected kernels store every gradient view,
    the captured step has no zero fill of the bucket.  Same trajectory as the eager engine; the
    short batch signature as well."""
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
    batches = _batches(10, 41) + _batches(1, 42, bs=8) + _batches(10, 43) + _batches(3, 44, bs=8)
    cfg = {"train_batch_size": 32, **extra}
    e1, l1, p1 = _run_engine(dict(cfg), batches, crit=BCEWithLogitsLoss())
    e2, l2, p2 = _run_engine(dict(cfg, amd={"hip_graph": True}), batches, graph=True, crit=BCEWithLogitsLoss())
    assert e2.graphed.replays >= 15 and not e2.graphed.failed, e2.graphed.failed
    assert e2.graphed.all_stored and all(e2.graphed.all_stored.values()), e2.graphed.all_stored
    torch.testing.assert_close(torch.tensor(l2), torch.tensor(l1), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(p2, p1, rtol=1e-5, atol=1e-6)
    e1.close()
    e2.close()


@pytest.mark.gpu
def test_graph_direct_launch_matches_replay():
    """A graph that captured a short chain of kernels runs as those kernels re-launched directly
    (runtime/graph_module.direct_launcher, csrc/bindings.cpp direct_plan): same outputs bit for bit
    as replaying the graph, on the current stream, reading the captured addresses' current
    contents; a graph holding a copy node gets no plan."""
    from distributed_gpu_test_amd.runtime.graph_module import direct_launcher
    from distributed_gpu_test_amd.ops import _ext
    dev = torch.device("cuda", 0)
    x = torch.randn(64, 32, device=dev)
    w = torch.randn(16, 32, device=dev)
    out = torch.empty(64, 16, device=dev)
    g = torch.cuda.CUDAGraph(keep_graph=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g.capture_begin()
        out.copy_(torch.nn.functional.gelu(x @ w.t()))  # several kernels: no plan (over the limit)
        g.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    g.instantiate()
    d = direct_launcher(g)
    if d is not None:  # a chain of plain kernels: the launches reproduce the replay
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        ref = out.clone()
        out.zero_()
        d()
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
    # a graph holding a copy node gets no plan
    dst, src0 = torch.empty(1 << 20, device=dev), torch.randn(1 << 20, device=dev)
    gc_ = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.stream(s):
        s.wait_stream(torch.cuda.current_stream())
        gc_.capture_begin()
        dst.copy_(src0)
        gc_.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    gc_.instantiate()
    plan = _ext.fast().graph_direct_plan(int(gc_.raw_cuda_graph()), 0)
    assert plan is None or plan.kernels == 1  # (a copy captured as a kernel is a kernel)
    # one kernel: a plan, and its launches write exactly what the replays write
    y = torch.zeros(1 << 16, device=dev)
    src = torch.randn(1 << 16, device=dev)
    g1 = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.stream(s):
        s.wait_stream(torch.cuda.current_stream())
        g1.capture_begin()
        torch.add(src, 1.5, out=y)
        g1.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    g1.instantiate()
    d = direct_launcher(g1)
    assert d is not None and d.kernels == 1
    y.zero_()
    g1.replay()
    torch.cuda.synchronize()
    ref = y.clone()
    y.zero_()
    src.mul_(1.0)  # (same values)
    d()
    torch.cuda.synchronize()
    assert torch.equal(y, ref) and torch.equal(ref, src + 1.5)
    src.add_(1.0)  # the launcher reads the captured addresses' CURRENT contents, as a replay does
    d()
    torch.cuda.synchronize()
    assert torch.equal(y, src + 1.5)


@pytest.mark.gpu
def test_graph_module_forward_uses_direct_launch():
    """The reference model's graphed forward (one fused-chain kernel) and graphed tail (backward,
    Adam, zero fill) are launched directly, and the trajectory is bit-identical to replaying every
    graph (DGT_GRAPH_DIRECT=0)."""
    import subprocess
    import sys
    code = r"""
import json, torch
import distributed_gpu_test_amd as dgt
from distributed_gpu_test_amd.models import SimpleNet
from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
from distributed_gpu_test_amd.data import gather_batch
torch.manual_seed(0)
m = SimpleNet(20, 64)
cfg = {"train_batch_size": 4, "amd": {"graph_module": True}}
e, _, _, _ = dgt.initialize(model=m, model_parameters=m.parameters(), config=cfg)
X = torch.randn(256, 20, device="cuda"); Y = (torch.rand(256, 1, device="cuda") > 0.5).float()
crit = BCEWithLogitsLoss()
for s in range(40):
    rows = torch.arange(4 * (s % 8), 4 * (s % 8) + 4, device="cuda")
    xb, yb = gather_batch(rows, X, Y)
    loss = crit(e(xb), yb); e.backward(loss); e.step()
torch.cuda.synchronize()
runners = list(e._runners)
print(json.dumps({"direct": [r.fwd_direct is not None and getattr(r, "tail_direct", None) is not None
                             for r in runners],
                  "params": [p.detach().cpu().double().sum().item() for p in m.parameters()],
                  "bits": [p.detach().cpu().view(torch.int32).sum().item() for p in m.parameters()]}))
"""
    outs = {}
    for flag in ("1", "0"):
        env = dict(os.environ, DGT_GRAPH_DIRECT=flag, DGT_QUIET="1")
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240,
                           cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        assert r.returncode == 0, r.stderr[-3000:]
        outs[flag] = json.loads(r.stdout.strip().splitlines()[-1])
    assert outs["1"]["direct"] and all(outs["1"]["direct"])
    assert not any(outs["0"]["direct"])
    assert outs["1"]["bits"] == outs["0"]["bits"]


@pytest.mark.gpu
def test_graph_tail_with_torch_bce():
    """The reference's own criterion (torch.nn.BCEWithLogitsLoss, mean, reference train.py:96) takes the
    graphed tail too: dL/dz comes from the framework's loss kernel straight into the backward graph's
    input, and the trajectory matches the eager engine's autograd backward.  A weighted BCE (not the
    kernel's gradient) keeps the autograd path."""
    batches = _batches(10, 5) + _batches(3, 8, bs=8)
    cfg = {"train_batch_size": 32}
    e1, l1, p1 = _run_engine(dict(cfg), batches)
    e2, l2, p2 = _run_engine(dict(cfg, amd={"graph_module": True}), batches)
    assert e2.tail_steps == len(batches), (e2.tail_steps, e2.tail_reason)
    torch.testing.assert_close(torch.tensor(l2), torch.tensor(l1), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(p2, p1, rtol=1e-5, atol=1e-6)
    crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([2.0], device="cuda"))
    e3, l3, p3 = _run_engine(dict(cfg, amd={"graph_module": True}), batches, crit=crit)
    e4, l4, p4 = _run_engine(dict(cfg), batches, crit=crit)
    assert e3.tail_steps == 0
    torch.testing.assert_close(p3, p4, rtol=1e-5, atol=1e-6)
    for e in (e1, e2, e3, e4):
        e.close()


@pytest.mark.gpu
def test_eager_direct_backward_with_torch_bce():
    """The eager engine runs torch's own mean BCEWithLogitsLoss (the reference's criterion) through its
    direct backward too (d loss / d logits from the framework's loss kernel, no autograd engine): the
    trajectory matches plain torch; a second backward of the same loss raises, as autograd would."""
    m = _mlp(6)
    ref = copy.deepcopy(m).cuda()
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    crit = torch.nn.BCEWithLogitsLoss()
    for x, y in _batches(8, 12):
        opt.zero_grad()
        crit(ref(x), y).backward()
        opt.step()
    engine, _, _, _ = dgt.initialize(model=m, optimizer=torch.optim.Adam(m.parameters(), lr=1e-3),
                                     config={"train_batch_size": 32})
    for x, y in _batches(8, 12):
        loss = crit(engine(x), y)
        engine.backward(loss)
        engine.step()
    assert engine.direct_backwards == 8
    got = torch.nn.utils.parameters_to_vector(engine.module.parameters())
    want = torch.nn.utils.parameters_to_vector(ref.parameters())
    torch.testing.assert_close(got, want, rtol=2e-4, atol=2e-5)
    x, y = _batches(1, 13)[0]
    loss = crit(engine(x), y)
    engine.backward(loss)
    with pytest.raises(RuntimeError, match="second time"):
        engine.backward(loss)
    engine.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ds_graph.json", "ds_graph_fused.json", "ds_zero1_graph.json", "ds_graph_module.json",
                                  "ds_zero0.json", "ds_fused_linear.json"])
def test_shipped_configs_take_their_fast_paths(name):
    """Each shipped config on the reference loop (bench.py's DgtEngineBench: gather, forward, the
    framework's BCE, backward, step) engages the path it is for -- a silent eager fallback (e.g. on a
    torch without the graph internals, compat.py) fails here: whole-step graph replays for
    ``hip_graph``, graphed-tail steps for ``graph_module``, direct backwards for the eager configs."""
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    from distributed_gpu_test_amd.data import make_synthetic_data
    from distributed_gpu_test_amd.models import SimpleNet
    cfg = json.load(open(os.path.join(root, "configs", name)))
    torch.manual_seed(42)
    x, y = make_synthetic_data(2000, 20, 42)
    mask = os.sched_getaffinity(0)
    try:
        tr = bench.DgtEngineBench(SimpleNet(20, 64), x, y, 4, torch.device("cuda", 0), cfg)
        plan, counts = tr.epoch_plan(1)
        tr.run_plan(plan[:30], counts[:30])
        torch.cuda.synchronize()
    finally:
        os.sched_setaffinity(0, mask)  # (the graph configs pin the host thread: not the rest of the suite)
    e = tr.engine
    amd = cfg.get("amd", {})
    assert (e.host_cpu is not None) == bool(amd.get("pin_host_thread")), e.host_cpu
    if amd.get("hip_graph"):
        assert e.graphed is not None and e.graphed.replays > 0 and not e.graphed.failed, \
            (e.graph_fallback_reason, getattr(e.graphed, "failed", None))
    elif amd.get("graph_module"):
        assert e.graph_module and e.tail_steps > 0, (e.graph_module_reason, e.tail_reason)
    else:
        assert e.direct_backwards == 30, e.direct_backwards
    assert float(tr.loss_acc.item()) > 0
    tr.close()


@pytest.mark.gpu
def test_graph_module_dropout_draws_fresh_masks():
    """a graph that consumes RNG (dropout) is replayed, not re-launched with its captured
    arguments: every step draws a new mask and the generator advances (graph_module.rng_checked)."""
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.Dropout(0.5), torch.nn.Linear(64, 1))
    e, _, _, _ = dgt.initialize(model=m, config={"train_batch_size": 8, "amd": {"graph_module": True},
                                                 "optimizer": {"type": "Adam", "params": {"lr": 0.0}}})
    x = torch.randn(8, 16, device="cuda")
    y = torch.ones(8, 1, device="cuda")
    crit = torch.nn.BCEWithLogitsLoss()
    outs = []
    for _ in range(6):
        s0 = torch.cuda.get_rng_state()
        out = e(x)
        outs.append(out.detach().clone())
        e.backward(crit(out, y))
        e.step()
        assert not torch.equal(s0, torch.cuda.get_rng_state())  # the generator moved
    assert e._graphed_fwd, e.graph_module_reason
    # lr 0: same weights every step, so any change of the output is a new dropout mask
    assert len({tuple(o.view(-1).tolist()) for o in outs[2:]}) == len(outs[2:])
    e.close()


@pytest.mark.gpu
def test_fused_linear_refuses_inplace_modified_input():
    """the fused Linear nodes hold their input and weights as attributes; an in-place
    change between forward and backward raises, as autograd's saved-tensor check would."""
    m = _mlp(3)
    e, _, _, _ = dgt.initialize(model=m, config={"train_batch_size": 32})
    assert e.fused_linear_layers == 2
    x, y = _batches(1)[0]
    out = e(x)
    x.mul_(2.0)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        e.backward(torch.nn.functional.binary_cross_entropy_with_logits(out, y))
    e.close()


@pytest.mark.gpu
def test_concurrent_stream_runs_beside_the_current_stream():
    """accelerator.concurrent_stream: a pool stream measured to sit on a hardware queue other than the
    current stream's -- an event recorded on it completes while a spin kernel holds the current stream."""
    import time
    from distributed_gpu_test_amd.accelerator import concurrent_stream
    s, ok = concurrent_stream(torch.device("cuda", 0))
    assert ok and s is not None
    assert concurrent_stream(torch.device("cuda", 0))[0] is s  # cached per device
    torch.cuda.synchronize()
    spin, mark = torch.cuda.Event(), torch.cuda.Event()
    torch.cuda._sleep(16_000_000)
    spin.record()
    mark.record(s)
    t0 = time.perf_counter()
    while not mark.query() and time.perf_counter() - t0 < 0.005:
        pass
    assert mark.query() and not spin.query()
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_graph_module_retained_fused_bce_backward_twice():
    """with graph_module the fused BCE writes d loss / d logits into the backward graph's
    static input; a scaled (gas = 2) backward under retain_graph copies dz * g over it.  A second
    backward through the retained graph must still read the unscaled dz (the BCE keeps a private copy)."""
    from distributed_gpu_test_amd.models import SimpleNet
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss
    torch.manual_seed(3)
    m = SimpleNet(20, 64)
    ref = copy.deepcopy(m).cuda()
    e, _, _, _ = dgt.initialize(model=m, optimizer=torch.optim.Adam(m.parameters(), lr=1e-3),
                                config={"train_micro_batch_size_per_gpu": 8, "gradient_accumulation_steps": 2,
                                        "amd": {"graph_module": True}})
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    x = torch.randn(8, 20, device="cuda")
    y = (torch.rand(8, 1, device="cuda") > 0.5).float()
    crit = BCEWithLogitsLoss()
    for _ in range(3):  # (the first forwards capture; later ones replay and claim the gout buffer)
        loss = crit(e(x), y)
        e.backward(loss, retain_graph=True)
        e.step()
        e.backward(loss)
        e.step()
        rl = torch.nn.functional.binary_cross_entropy_with_logits(ref(x), y)
        (rl / 2).backward(retain_graph=True)
        (rl / 2).backward()
        ropt.step()
        ropt.zero_grad(set_to_none=True)
    assert e._graphed_fwd, e.graph_module_reason
    got = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    want = torch.cat([p.detach().reshape(-1) for p in ref.parameters()])
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-6)
    e.close()
