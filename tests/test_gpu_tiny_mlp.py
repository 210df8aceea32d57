"""GPU numerics of the fused tiny-MLP kernels vs plain-PyTorch fp32 references."""
import pytest
import torch

from distributed_gpu_test_amd.data import make_synthetic_data
from distributed_gpu_test_amd.models import SimpleNet
from distributed_gpu_test_amd.ops import _ext, adam_flat_, adam_flat_reference_, tiny_mlp_step_reference
from distributed_gpu_test_amd.runtime.tiny_trainer import TinyMLPTrainer

pytestmark = pytest.mark.gpu

ORACLE_WS1 = [0.4301, 0.1461, 0.0865, 0.0637, 0.0516]


def _setup(F=20, H=64, n=2000, seed=42):
    torch.manual_seed(seed)
    x, y = make_synthetic_data(n, F, seed)
    return x, y, SimpleNet(F, H)


def test_extension_loaded_on_gpu():
    assert _ext.available(), "native extension must load on a GPU box"
    assert torch.ops.dgt.tiny_mlp_supported(20, 64)


@pytest.mark.parametrize("F,H,B", [(20, 64, 4), (20, 64, 3), (32, 64, 16), (8, 16, 1), (20, 128, 7)])
def test_grad_kernel_matches_reference(F, H, B):
    dev = torch.device("cuda")
    x, y, m = _setup(F, H, 64)
    tr = TinyMLPTrainer(m, x, y, batch_size=B, impl="stepwise")
    plan, counts = tr.epoch_plan(1)
    ops = _ext.require()
    g = torch.zeros_like(tr.params)
    loss_acc = torch.zeros(1, dtype=torch.float64, device=dev)
    ops.tiny_mlp_grad(tr.x, tr.y, plan, counts, 0, tr.params, g, loss_acc, F, H)
    rows = plan[0, : int(counts[0])].long()
    ref_loss, ref_g = tiny_mlp_step_reference(tr.params.double(), tr.x[rows].double(), tr.y[rows].double(), F, H)
    torch.cuda.synchronize()
    assert abs(loss_acc.item() - ref_loss) < 1e-5
    torch.testing.assert_close(g.double(), ref_g, rtol=1e-4, atol=1e-6)


def test_fused_epoch_matches_torch_reference():
    x, y, m = _setup()
    _, _, m_ref = _setup()  # same seed -> identical init
    ref = TinyMLPTrainer(m_ref, x, y, 4, impl="torch", device=torch.device("cuda"))
    fused = TinyMLPTrainer(m, x, y, 4, impl="fused")
    torch.testing.assert_close(fused.params, ref.params)
    l_ref = ref.run_epoch(1)
    l_fused = fused.run_epoch(1)
    assert abs(l_ref - l_fused) < 1e-5
    torch.testing.assert_close(fused.params, ref.params, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(fused.exp_avg_sq, ref.exp_avg_sq, rtol=1e-3, atol=1e-9)


def test_fused_reproduces_reference_oracle_ws1():
    x, y, m = _setup()
    tr = TinyMLPTrainer(m, x, y, 4, impl="fused")
    losses = [round(tr.run_epoch(e), 4) for e in range(1, 6)]
    assert losses == ORACLE_WS1


@pytest.mark.parametrize("prepared", [True, False])
def test_bound_launch_is_bitwise_run_plan(prepared):
    """bench.py's bound launch (``bind_launch``: the argument block prepared once, launched through
    hipModuleLaunchKernel, or the per-argument entry point) trains exactly as ``run_plan``: same
    parameters, moments, loss and step count, bit for bit, over several launches of one plan and a
    launch of another."""
    x, y, m1 = _setup()
    _, _, m2 = _setup()
    a = TinyMLPTrainer(m1, x, y, 4, impl="fused")
    b = TinyMLPTrainer(m2, x, y, 4, impl="fused")
    plan, counts = a.epoch_plan(1)
    p20, c20 = plan[:20], counts[:20]
    a.reserve(20)
    b.reserve(20)
    launch = b.bind_launch(p20, c20, prepared=prepared)
    other = b.bind_launch(plan[20:23], counts[20:23], prepared=prepared)
    for _ in range(3):
        a.run_plan(p20, c20)
        launch()
    a.run_plan(plan[20:23], counts[20:23])
    other()
    torch.cuda.synchronize()
    assert a.global_steps == b.global_steps == 63
    for ta, tb in ((a.params, b.params), (a.exp_avg, b.exp_avg), (a.exp_avg_sq, b.exp_avg_sq),
                   (a.loss_acc, b.loss_acc)):
        assert torch.equal(ta, tb)
    a.check()
    b.check()


def test_stepwise_matches_fused():
    x, y, m1 = _setup()
    _, _, m2 = _setup()
    a = TinyMLPTrainer(m1, x, y, 4, impl="fused")
    b = TinyMLPTrainer(m2, x, y, 4, impl="stepwise")
    for e in (1, 2):
        la, lb = a.run_epoch(e), b.run_epoch(e)
        assert abs(la - lb) < 1e-5
    torch.testing.assert_close(a.params, b.params, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("gdt,lpdt", [(torch.float32, None), (torch.bfloat16, torch.bfloat16),
                                       (torch.float16, torch.float16), (torch.float32, torch.bfloat16)])
@pytest.mark.parametrize("wd,adamw", [(0.0, False), (0.01, False), (0.01, True)])
def test_adam_flat_matches_reference(gdt, lpdt, wd, adamw):
    n = 4096 * 3 + 8
    g = torch.Generator().manual_seed(0)
    p = torch.randn(n, generator=g).cuda()
    grads = [torch.randn(n, generator=g).cuda().to(gdt) for _ in range(3)]
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    lp = torch.empty(n, device="cuda", dtype=lpdt) if lpdt else None
    scale = torch.tensor([0.5], device="cuda")
    for step, gr in enumerate(grads, 1):
        adam_flat_(p, gr, m, v, step, 1e-3, 0.9, 0.999, 1e-8, wd, adamw, grad_scale=0.25, grad_scale_dev=scale,
                   param_lp=lp)
        adam_flat_reference_(p2, gr, m2, v2, step, 1e-3, 0.9, 0.999, 1e-8, wd, adamw, grad_scale=0.25,
                             grad_scale_dev=scale)
    torch.testing.assert_close(p, p2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m, m2, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(v, v2, rtol=1e-5, atol=1e-9)
    if lp is not None:
        torch.testing.assert_close(lp, p2.to(lpdt))


@pytest.mark.parametrize("n", [4096 * 3 + 4, 4])
@pytest.mark.parametrize("gdt,lpdt", [(torch.float32, torch.bfloat16), (torch.bfloat16, torch.bfloat16),
                                       (torch.float16, torch.float16)])
def test_adam_flat_unaligned_16bit_slices(n, gdt, lpdt):
    """16-bit gradient / low-precision slices that start 8 bytes (not 16) into their buffer give the
    same bits as aligned ones (the kernel moves 8-byte groups of 16-bit elements)."""
    g = torch.Generator().manual_seed(1)
    p0 = torch.randn(n + 4, generator=g).cuda()
    gr0 = torch.randn(n + 4, generator=g).cuda().to(gdt)
    outs = []
    for off in (0, 4):
        p, m, v = p0[4:4 + n].clone(), torch.full((n,), 0.1, device="cuda"), torch.full((n,), 0.2, device="cuda")
        gbuf = torch.zeros(n + 4, device="cuda", dtype=gdt)
        gbuf[off:off + n] = gr0[:n]
        gr = gbuf[off:off + n]
        lpbuf = torch.empty(n + 4, device="cuda", dtype=lpdt)
        lp = lpbuf[off:off + n]
        adam_flat_(p, gr, m, v, 3, 1e-3, 0.9, 0.999, 1e-8, 0.01, True, param_lp=lp)
        outs.append((p, m, v, lp.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_adam_rejects_misaligned_slices():
    p = torch.zeros(16, device="cuda")
    g = torch.zeros(16, device="cuda")
    with pytest.raises(RuntimeError):
        adam_flat_(p[2:14], g[2:14], torch.zeros(12, device="cuda"), torch.zeros(12, device="cuda"), 1, 1e-3, 0.9,
                   0.999, 1e-8, 0.0, False)


def test_graph_impl_matches_oracle_and_stepwise():
    x, y, m1 = _setup()
    _, _, m2 = _setup()
    g = TinyMLPTrainer(m1, x, y, 4, impl="graph")
    s = TinyMLPTrainer(m2, x, y, 4, impl="stepwise")
    losses = [round(g.run_epoch(e), 4) for e in range(1, 4)]
    assert losses == ORACLE_WS1[:3]
    for e in range(1, 4):
        s.run_epoch(e)
    torch.testing.assert_close(g.params, s.params, rtol=1e-5, atol=1e-7)
    assert int(g.step_dev.item()) == g.global_steps == 1500
    # a plan that is not a multiple of the captured epoch: graph replays + eager tail
    plan, counts = g.epoch_plan(4)
    g.run_plan(plan[:300], counts[:300])
    s.run_plan(plan[:300], counts[:300])
    torch.testing.assert_close(g.params, s.params, rtol=1e-5, atol=1e-7)


def test_native_rccl_comm_single_rank():
    from distributed_gpu_test_amd.parallel import comm
    from distributed_gpu_test_amd.parallel.rccl import RcclComm
    comm.init_distributed()
    c = RcclComm()
    t = torch.arange(1024, dtype=torch.float32, device="cuda")
    c.all_reduce(t)
    torch.testing.assert_close(t, torch.arange(1024, dtype=torch.float32, device="cuda"))
    out = torch.empty(1024, device="cuda")
    c.all_gather(out, t)
    torch.testing.assert_close(out, t)
    assert RcclComm.version() >= 22000
    c.close()


def test_in_kernel_bias_corrections_are_launch_split_invariant():
    """The fused kernel forms Adam's bias corrections itself (an LDS ring refilled every T = 256
    steps), so how the steps are split into launches must not change a single bit: one launch of
    700 steps (crossing two ring refills) against launches of 1, 37, 255, 257 and 150 steps."""
    dev = torch.device("cuda", 0)
    outs = []
    for cuts in ((700,), (1, 37, 255, 257, 150)):
        x, y, m = _setup()
        tr = TinyMLPTrainer(m, x, y, 4, impl="fused", device=dev)
        p1, c1 = tr.epoch_plan(1)
        p2, c2 = tr.epoch_plan(2)
        plan, counts = torch.cat([p1, p2]), torch.cat([c1, c2])
        s = 0
        for n in cuts:
            tr.run_plan(plan[s:s + n], counts[s:s + n])
            s += n
        torch.cuda.synchronize()
        tr.check()
        outs.append((tr.params.clone(), tr.exp_avg.clone(), tr.exp_avg_sq.clone(), float(tr.loss_acc.item())))
    for a, b in zip(outs[0][:3], outs[1][:3]):
        assert torch.equal(a, b)
    # the loss log folds 4-step groups in fp32 (deferred ring, aligned to the launch start) into a
    # double: only the grouping depends on the split
    assert abs(outs[0][3] - outs[1][3]) <= 1e-6 * abs(outs[0][3])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1412, 1 << 20])
def test_adam_flat_advances_device_step_itself(n):
    """adam_flat_ with step_ticket: the launch uses step_dev + 1 and stores it back from its last
    block (a graph-replayed step needs no increment node); bitwise the host-step update, over one
    block and over 1,024 blocks; the ticket returns to zero after every launch."""
    g = torch.Generator(device="cuda").manual_seed(n)
    p = torch.randn(n, device="cuda", generator=g)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    step_dev = torch.full((), 4, dtype=torch.int64, device="cuda")
    ticket = torch.zeros((), dtype=torch.int32, device="cuda")
    for t in range(5, 9):
        gr = torch.randn(n, device="cuda", generator=g)
        adam_flat_(p, gr, m, v, 1, 1e-3, 0.9, 0.999, 1e-8, 0.0, False, step_dev=step_dev, step_ticket=ticket)
        adam_flat_(p2, gr, m2, v2, t, 1e-3, 0.9, 0.999, 1e-8, 0.0, False)
        assert int(step_dev) == t and int(ticket) == 0
    assert torch.equal(p, p2) and torch.equal(m, m2) and torch.equal(v, v2)
