"""Exact-fp32 MFMA GEMM (csrc/gemm_f32.hip) against fp32/fp64 PyTorch references of the same ops.

Every layout pair the Linear layers use (forward MK.NK, dgrad MK.KN, wgrad KM.KN; plus KM.NK),
aligned and ragged shapes (the 16-byte load path and the scalar one), every tile configuration the
planner picks (128x64 and 64x64 wave tiles, the in-workgroup K splits), K tails that are not a
multiple of the chunk, and the epilogues (bias, ReLU, accumulate, ReLU mask on A).  Then the engine-facing ops:
FusedLinear / FusedChain at shapes beyond the small-batch kernels, with autograd gradients compared
to nn.Linear in fp32."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from distributed_gpu_test_amd.ops import _ext
    return _ext.require()


def _operands(M, N, K, la, lb, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    a = torch.randn(M, K, device="cuda", generator=g)   # logical A[m][k]
    b = torch.randn(N, K, device="cuda", generator=g)   # logical B[n][k]
    A = a if la == 0 else a.t().contiguous()
    B = b if lb == 0 else b.t().contiguous()
    return a, b, A, B


def _ref(a, b, bias=None, relu=False, mask=None):
    a64 = a.double() if mask is None else (a * (mask > 0)).double()
    out = a64 @ b.double().t()
    if bias is not None:
        out = out + bias.double()
    if relu:
        out = out.clamp_min(0)
    return out


def _close(got, ref, a, b):
    # fp32 fma chain vs fp64: error bounded by ~K * 2^-24 * sum|a b|; rtol 1e-5 on that scale
    scale = (a.abs().double() @ b.abs().double().t()).clamp_min(1.0)
    err = ((got.double() - ref).abs() / scale).max().item()
    assert err <= 1e-5, err


SHAPES = [
    (256, 256, 256),      # aligned, 64x64 tiles
    (1024, 1024, 1024),   # aligned, 64x64 tiles (64 x 128^2 tiles < 256)
    (2048, 2048, 512),    # aligned, 64x64 wave tiles in 2 x 2 (128x128 workgroup tiles)
    (4096, 2048, 256),    # aligned, 128x64 wave tiles (256x128 workgroup tiles)
    (1000, 999, 1004),    # ragged M / N, K % 4 == 0 (16-byte staging with zero fill)
    (77, 130, 67),        # everything ragged, K odd (scalar staging)
    (64, 64, 8192),       # tiny grid, long K: the in-workgroup K split
    (3, 5, 7),            # degenerate
]


@pytest.mark.parametrize("lb", [0, 1])
@pytest.mark.parametrize("M,N,K", [(1024, 1024, 1024), (2048, 2048, 512), (1000, 999, 1004), (77, 130, 67),
                                   (64, 64, 8192), (4096, 1024, 256), (1000, 1000, 1000)])
def test_gemm_f32_output_mask(M, N, K, lb):
    """``maskC``: the product stored as C * 1[maskC > 0] (a dgrad writing the ReLU-masked gradient of
    the layer below), in every epilogue form (per-column and float4 stores, the in-workgroup K-split
    reduce), equal bit for bit to the plain product masked afterwards."""
    ops = _ops()
    a, b, A, B = _operands(M, N, K, 0, lb, seed=K)
    mk = torch.randn(M, N, device="cuda")
    C = torch.empty(M, N, device="cuda")
    ops.gemm_f32(A, B, None, None, C, 0, lb, False, False, None, mk)
    plain = torch.empty(M, N, device="cuda")
    ops.gemm_f32(A, B, None, None, plain, 0, lb, False, False)
    assert torch.equal(C, torch.where(mk > 0, plain, torch.zeros_like(plain)))


@pytest.mark.parametrize("la", [0, 1])
@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (1024, 1024, 1024), (2048, 2048, 512), (1000, 999, 1004),
                                   (77, 130, 67), (64, 64, 8192), (4096, 1, 1024)])
def test_gemm_f32_fused_rowsum(M, N, K, la, masked, accumulate):
    """``rowsum[m] (+)= sum_k A'(m, k)`` formed while the GEMM stages A (A' = A after the ReLU mask):
    the wgrad's bias gradient without a separate column-sum pass.  Every tile size, the in-workgroup K-split
    path (slice partials summed by the reduce kernel), the scalar and 16-byte staging, both A
    layouts; the product itself is unchanged."""
    ops = _ops()
    a, b, A, B = _operands(M, N, K, la, 0, seed=M + K)
    mask = None
    if masked:
        m = (torch.randn(M, K, device="cuda") > 0).float()
        mask = m if la == 0 else m.t().contiguous()
    C = torch.randn(M, N, device="cuda") if accumulate else torch.empty(M, N, device="cuda")
    rs = torch.randn(M, device="cuda") if accumulate else torch.full((M,), float("nan"), device="cuda")
    C0, rs0 = C.clone(), rs.clone()
    ops.gemm_f32(A, B, mask, None, C, la, 0, False, accumulate, rs)
    ref = _ref(a, b, mask=m if masked else None)
    want_rs = (a * (m > 0) if masked else a).double().sum(1)
    if accumulate:
        ref, want_rs = ref + C0.double(), want_rs + rs0.double()
    _close(C, ref, a, b)
    scale = (a.abs().double().sum(1)).clamp_min(1.0)
    err = ((rs.double() - want_rs).abs() / scale).max().item()
    assert err <= 1e-5, err


@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1), (1, 1), (1, 0)])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_f32_layouts(M, N, K, la, lb):
    ops = _ops()
    a, b, A, B = _operands(M, N, K, la, lb)
    C = torch.empty(M, N, device="cuda")
    ops.gemm_f32(A, B, None, None, C, la, lb, False, False)
    _close(C, _ref(a, b), a, b)


@pytest.mark.parametrize("M,N,K", [(512, 384, 256), (1000, 999, 1004), (64, 64, 8192), (77, 130, 67),
                                   (4096, 2048, 128)])
def test_gemm_f32_epilogues(M, N, K):
    ops = _ops()
    a, b, A, B = _operands(M, N, K, 0, 0, seed=1)
    bias = torch.randn(N, device="cuda")
    C = torch.empty(M, N, device="cuda")
    ops.gemm_f32(A, B, None, bias, C, 0, 0, True, False)
    _close(C, _ref(a, b, bias, relu=True), a, b)
    assert (C >= 0).all()
    # accumulate into an existing C (gradient accumulation into .grad views)
    C0 = torch.randn(M, N, device="cuda")
    C = C0.clone()
    ops.gemm_f32(A, B, None, None, C, 0, 0, False, True)
    _close(C, C0.double() + _ref(a, b), a, b)
    # ReLU mask on A (the backward's g = dy * 1[y > 0]), in both A layouts
    mask = torch.randn(M, K, device="cuda")
    for la in (0, 1):
        Aa = a if la == 0 else a.t().contiguous()
        Ma = mask if la == 0 else mask.t().contiguous()
        C = torch.empty(M, N, device="cuda")
        ops.gemm_f32(Aa, B, Ma, None, C, la, 0, False, False)
        _close(C, _ref(a, b, mask=mask), a, b)


def test_gemm_f32_asymmetric_identity():
    """A = I with an asymmetric B catches a row/column swap of the epilogue (guide §3)."""
    ops = _ops()
    n = 192
    A = torch.eye(n, device="cuda")
    B = torch.arange(n * n, device="cuda", dtype=torch.float32).view(n, n) * 1e-3  # B[n][k]
    C = torch.empty(n, n, device="cuda")
    ops.gemm_f32(A, B, None, None, C, 0, 0, False, False)
    assert torch.equal(C, B.t())


@pytest.mark.parametrize("M,N", [(1024, 1024), (4096, 64), (1000, 999), (33, 7), (5000, 1)])
def test_colsum_f32(M, N):
    ops = _ops()
    dy = torch.randn(M, N, device="cuda")
    y = torch.randn(M, N, device="cuda")
    db = torch.empty(N, device="cuda")
    ops.colsum_f32(dy, None, db, False)
    torch.testing.assert_close(db.double(), dy.double().sum(0), rtol=1e-5, atol=1e-4)
    ops.colsum_f32(dy, y, db, True)
    want = dy.double().sum(0) + (dy * (y > 0)).double().sum(0)
    torch.testing.assert_close(db.double(), want, rtol=1e-5, atol=2e-4)


@pytest.mark.parametrize("M,K,N,relu", [(1024, 1024, 1024, True), (512, 300, 700, False), (1000, 2048, 1, False),
                                        (1024, 1024, 1, False), (512, 256, 3, True)])  # the last two: skinny
def test_fused_linear_tiled_matches_nn_linear(M, K, N, relu):
    """FusedLinear beyond the small-batch kernels: forward, dx, dW, db vs nn.Linear in fp32."""
    from distributed_gpu_test_amd.ops import linear as L
    torch.manual_seed(0)
    lin = torch.nn.Linear(K, N).cuda()
    fl = L.FusedLinear.from_linear(lin, relu=relu)
    x = torch.randn(M, K, device="cuda", requires_grad=True)
    x2 = x.detach().clone().requires_grad_(True)
    before = dict(L.FALLBACKS)
    y = fl(x)
    ref = lin(x2)
    ref = torch.relu(ref) if relu else ref
    # against fp64 on the fp32 error scale (as _close): forward, then dx = g W, dW = g^T x, db
    w64, b64 = lin.weight.detach().double(), lin.bias.detach().double()
    x64 = x.detach().double()
    z64 = x64 @ w64.t() + b64
    y64 = z64.clamp_min(0) if relu else z64
    _close(y, y64, x.detach(), lin.weight.detach())
    torch.testing.assert_close(y, ref, rtol=1e-4, atol=5e-5)  # and hipBLASLt's fp32 within rounding
    gy = torch.randn_like(y)
    gx, gw, gb = torch.autograd.grad(y, (x, lin.weight, lin.bias), gy)
    rx, rw, rb = torch.autograd.grad(ref, (x2, lin.weight, lin.bias), gy)
    # the ReLU mask from the fp32 forward itself (a z within rounding of 0 may differ in fp64)
    g64 = gy.double() * (y.detach() > 0) if relu else gy.double()
    _close(gx, g64 @ w64, g64.float(), lin.weight.detach().t())
    _close(gw, g64.t() @ x64, g64.float().t(), x.detach().t())
    torch.testing.assert_close(gb.double(), g64.sum(0), rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(gx, rx, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(gw, rw, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(gb, rb, rtol=1e-4, atol=1e-3)
    assert dict(L.FALLBACKS) == before, L.FALLBACKS


@pytest.mark.parametrize("N", [1, 2, 4])
@pytest.mark.parametrize("M,K", [(1024, 1024), (192, 96)])  # 4 tiles per block; 1 (K % 128 != 0)
@pytest.mark.parametrize("mask,ymask,accumulate,with_dx", [(False, False, False, True), (True, False, False, True),
                                                          (True, True, True, True), (False, True, False, False)])
def test_skinny_f32_matches_fp64(N, M, K, mask, ymask, accumulate, with_dx):
    """The fp32 head kernels (csrc/head.hip skinny_f32): z = relu?(a W^T + b); backward with the
    head's own ReLU (y), the layer below's mask on dx, store or accumulate into dW / db."""
    ops = _ops()
    g = torch.Generator(device="cuda").manual_seed(N * 7 + M)
    a = torch.randn(M, K, device="cuda", generator=g).clamp_min(0) if mask else torch.randn(M, K, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g)
    b = torch.randn(N, device="cuda", generator=g)
    z = torch.empty(M, N, device="cuda")
    ops.skinny_f32_fwd(a, W, b, z, ymask)
    z64 = a.double() @ W.double().t() + b.double()
    if ymask:
        z64 = z64.clamp_min(0)
    _close(z, z64, a, W)
    dz = torch.randn(M, N, device="cuda", generator=g)
    dW0, db0 = torch.randn(N, K, device="cuda", generator=g), torch.randn(N, device="cuda", generator=g)
    dW, db = dW0.clone(), db0.clone()
    dx = torch.full((M, K), float("nan"), device="cuda") if with_dx else None
    ops.skinny_f32_bwd(dz, z if ymask else None, a, W, mask, dx, dW, db, accumulate)
    g64 = dz.double() * (z > 0) if ymask else dz.double()
    if with_dx:
        dx64 = g64 @ W.double()
        if mask:
            dx64 = dx64 * (a > 0)
        _close(dx, dx64, g64.float(), W.t())
    dW64 = g64.t() @ a.double() + (dW0.double() if accumulate else 0)
    db64 = g64.sum(0) + (db0.double() if accumulate else 0)
    torch.testing.assert_close(dW.double(), dW64, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(db.double(), db64, rtol=1e-5, atol=1e-4)


def test_engine_fp32_mlp_runs_no_vendor_gemm():
    """The DeepSpeed-style engine on a fp32 SyntheticMLP(1024, 4) at batch 1024 with kernel
    injection: the model runs as ONE fused chain node (ReLUs in the GEMM epilogues and the dgrad
    masks, not torch's clamp / threshold kernels), every Linear on a hand-written kernel (no
    F.linear fallback), and the first steps match the same model trained by plain PyTorch fp32 +
    torch Adam."""
    import copy
    from distributed_gpu_test_amd import initialize
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP, synthetic_batch_data
    torch.manual_seed(0)
    model = SyntheticMLP(1024, 4)
    ref = copy.deepcopy(model).cuda()
    cfg = {"train_micro_batch_size_per_gpu": 1024, "gradient_accumulation_steps": 1,
           "zero_optimization": {"stage": 0}, "optimizer": {"type": "Adam", "params": {"lr": 1e-4}},
           "amd": {"fused_linear": True}}
    from distributed_gpu_test_amd.ops.linear import FALLBACKS
    before = dict(FALLBACKS)
    engine, _, _, _ = initialize(model=model, config=cfg)
    assert engine.fused_linear_layers == 5
    opt = torch.optim.Adam(ref.parameters(), lr=1e-4)
    x, y = synthetic_batch_data(1024, 1024, 7)
    x, y = x.cuda(), y.cuda()
    crit = torch.nn.BCEWithLogitsLoss()
    for step in range(3):
        out = engine(x)
        assert type(out.grad_fn).__name__ == "_FusedChainFnBackward", type(out.grad_fn).__name__
        loss = crit(out.view(-1), y)
        engine.backward(loss)
        rl = crit(ref(x).view(-1), y)
        opt.zero_grad()
        rl.backward()
        torch.testing.assert_close(loss, rl, rtol=1e-4, atol=1e-5)
        if step == 0:  # the gradients themselves (Adam's first step is ~lr * sign(g): compare before it)
            # two fp32 summation orders put a few activations near 0 on different sides of the ReLU, so
            # a handful of mask bits (and the |dy x| terms they gate) differ: compare in norm and
            # relative to the gradient's scale, not element by element at 1e-6 (the kernels' own
            # exactness against fp64 is pinned above at 1e-5 normalised)
            for (name, p), q in zip(model.named_parameters(), ref.parameters()):
                rel = float((p.grad - q.grad).norm() / q.grad.norm().clamp_min(1e-30))
                worst = float((p.grad - q.grad).abs().max() / q.grad.abs().max().clamp_min(1e-30))
                assert rel < 1e-4 and worst < 2e-3, f"{name}: relative L2 {rel:.2e}, worst {worst:.2e}"
        engine.step()
        opt.step()
    assert engine.linear_fallbacks == before, engine.linear_fallbacks
    got = torch.nn.utils.parameters_to_vector(model.parameters())
    want = torch.nn.utils.parameters_to_vector(ref.parameters())
    # Adam's first steps move each weight by ~lr * sign(g): a near-zero gradient component whose sign
    # differs between two fp32 summation orders moves apart by up to 2 lr per step
    torch.testing.assert_close(got, want, rtol=0, atol=1e-3)
    engine.close()


# Small grids that the 64x64 K-split-4 tile still leaves under-filled (tiles < 256): the GEMM splits
# K across workgroups too (gemm_f32_split) and the last workgroup of a tile to arrive sums the
# partials in slice order.  Aligned, ragged M / N, a K tail that is not a whole 16-deep chunk.
SPLIT_SHAPES = [(256, 1024, 1024), (128, 512, 4096), (192, 320, 2004), (100, 200, 3000), (64, 64, 8192)]


@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1), (1, 1), (1, 0)])
@pytest.mark.parametrize("M,N,K", SPLIT_SHAPES)
def test_gemm_f32_split_k_layouts(M, N, K, la, lb):
    ops = _ops()
    a, b, A, B = _operands(M, N, K, la, lb, seed=N)
    C = torch.empty(M, N, device="cuda")
    ops.gemm_f32(A, B, None, None, C, la, lb, False, False)
    _close(C, _ref(a, b), a, b)


@pytest.mark.parametrize("M,N,K", SPLIT_SHAPES)
def test_gemm_f32_split_k_epilogues(M, N, K):
    """Bias + ReLU, accumulate, the ReLU mask on A and the output mask run once per tile, by the
    workgroup that sums the partials."""
    ops = _ops()
    a, b, A, B = _operands(M, N, K, 0, 0, seed=7)
    bias = torch.randn(N, device="cuda")
    C = torch.empty(M, N, device="cuda")
    ops.gemm_f32(A, B, None, bias, C, 0, 0, True, False)
    _close(C, _ref(a, b, bias, relu=True), a, b)
    C0 = torch.randn(M, N, device="cuda")
    C = C0.clone()
    ops.gemm_f32(A, B, None, None, C, 0, 0, False, True)
    _close(C, C0.double() + _ref(a, b), a, b)
    mask = torch.randn(M, K, device="cuda")
    mk = torch.randn(M, N, device="cuda")
    Bt = b.t().contiguous()
    C = torch.empty(M, N, device="cuda")
    ops.gemm_f32(A, Bt, mask, None, C, 0, 1, False, False, None, mk)  # the dgrad form
    _close(C, torch.where(mk > 0, _ref(a, b, mask=mask), torch.zeros((), dtype=torch.float64, device="cuda")), a, b)


@pytest.mark.parametrize("M,N,K", [(256, 1024, 1024), (192, 320, 2004)])
def test_gemm_f32_split_k_deterministic_and_rearmed(M, N, K):
    """The slice-order sum gives the same bits on every call whichever workgroup arrives last, and
    each launch leaves the tile counters at zero (a stale counter would skip the epilogue: C keeps
    its NaN fill); also across a second stream (its own workspace)."""
    ops = _ops()
    a, b, A, B = _operands(M, N, K, 0, 0, seed=3)
    first = None
    side = torch.cuda.Stream()
    for i in range(6):
        C = torch.full((M, N), float("nan"), device="cuda")
        if i % 2:
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                ops.gemm_f32(A, B, None, None, C, 0, 0, False, False)
            torch.cuda.current_stream().wait_stream(side)
        else:
            ops.gemm_f32(A, B, None, None, C, 0, 0, False, False)
        assert not C.isnan().any()
        if first is None:
            first = C
            _close(C, _ref(a, b), a, b)
        else:
            assert torch.equal(C, first)


def test_gemm_f32_split_k_knob_off_matches_reference(tmp_path):
    """DGT_F32_SPLIT=1 turns the cross-workgroup split off (read once per process): a subprocess
    computes the same product without it; both agree with the fp64 reference and differ only by
    summation order."""
    import os
    import subprocess
    import sys
    M, N, K = 256, 1024, 1024
    ops = _ops()
    a, b, A, B = _operands(M, N, K, 0, 0, seed=11)
    C = torch.empty(M, N, device="cuda")
    ops.gemm_f32(A, B, None, None, C, 0, 0, False, False)
    src = (
        "import torch\n"
        "from distributed_gpu_test_amd.ops import _ext\n"
        "ops = _ext.require()\n"
        f"g = torch.Generator(device='cuda').manual_seed(11)\n"
        f"a = torch.randn({M}, {K}, device='cuda', generator=g); b = torch.randn({N}, {K}, device='cuda', generator=g)\n"
        f"C = torch.empty({M}, {N}, device='cuda')\n"
        "ops.gemm_f32(a, b, None, None, C, 0, 0, False, False)\n"
        f"torch.save(C.cpu(), {str(tmp_path / 'c.pt')!r})\n")
    env = dict(os.environ, DGT_F32_SPLIT="1")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", src], env=env, cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    off = torch.load(tmp_path / "c.pt", weights_only=True).cuda()
    _close(off, _ref(a, b), a, b)
    _close(C, _ref(a, b), a, b)
    assert not torch.equal(off, C)  # a different summation order: the split path did run
