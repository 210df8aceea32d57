"""The 256x128 split-K bf16 GEMM (``csrc/gemm.hip`` gemm_nt_sk_kernel, variant 9) against a plain
PyTorch fp32 reference of the same product + epilogue, its determinism (the two K halves meet
through a per-tile ticket: the result must not depend on which half finished first, and every
launch must leave the ticket words re-armed), its per-stream workspace, and its agreement with the
unsplit 128x128 kernels it replaces on the MLP's M = 1024 products."""
import pytest
import torch

from distributed_gpu_test_amd.ops.gemm import gemm_nt, gemm_nt_reference

pytestmark = pytest.mark.gpu

# (M, N, K): the tile count (M / 256) * (N / 128) must be a multiple of 8
SHAPES = [(256, 1024, 256), (512, 512, 512), (256, 1024, 2048), (1024, 4096, 4096)]
EPIS = ["plain", "bias_relu_T", "bias_relu", "bias_T", "bias", "mask_T",
        "kn_plain", "kn_T", "kn_mask_T", "kn_mask_T_colsum"]


def _operands(M, N, K, seed):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16).cuda()
    B = torch.randn(N, K, generator=g).to(torch.bfloat16).cuda()
    Bkn = torch.randn(K, N, generator=g).to(torch.bfloat16).cuda()
    bias = torch.randn(N, generator=g).cuda()
    mask = (torch.randn(M, N, generator=g) > 0).to(torch.bfloat16).cuda()
    return A, B, Bkn, bias, mask


def _run(epi, A, B, Bkn, bias, mask, variant):
    M, N = A.shape[0], B.shape[0]
    kn = epi.startswith("kn_")
    kw = {}
    if "bias" in epi:
        kw["bias"] = bias
    if "relu" in epi:
        kw["relu"] = True
    if "mask" in epi:
        kw["mask"] = mask
    C = torch.full((M, N), float("nan"), device="cuda").to(torch.bfloat16)
    CT = torch.full((N, M), float("nan"), device="cuda").to(torch.bfloat16) if "_T" in epi else None
    cs = torch.full((M // 128, N), float("nan"), device="cuda") if epi.endswith("colsum") else None
    gemm_nt(A, Bkn if kn else B, C=C, CT=CT, b_kn=kn, variant=variant, colsum=cs, **kw)
    return C, CT, cs, kw


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("epi", EPIS)
def test_gemm_sk_matches_fp32_reference(M, N, K, epi):
    A, B, Bkn, bias, mask = _operands(M, N, K, M + N + K)
    C, CT, cs, kw = _run(epi, A, B, Bkn, bias, mask, 9)
    kn = epi.startswith("kn_")
    ref = gemm_nt_reference(A, Bkn if kn else B, b_kn=kn, **kw)  # fp32 on the GPU
    tol = dict(rtol=2e-2, atol=2e-2 * K ** 0.5)
    torch.testing.assert_close(C.float(), ref.to(torch.bfloat16).float(), **tol)
    if CT is not None:
        assert torch.equal(CT, C.t()), "C^T must hold the same bf16 values as C"
    if cs is not None:
        want = C.float().view(M // 128, 128, N).sum(1)  # the kernel sums its own bf16 outputs
        torch.testing.assert_close(cs, want, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("epi", ["bias_relu_T", "kn_mask_T_colsum"])
def test_gemm_sk_deterministic_and_rearmed(epi):
    """Ten launches on one workspace give the same bits: which half comes first differs from launch
    to launch, fp32 a + b == b + a, and a ticket left un-armed would make a later launch read a
    stale partial (or wait on a flag that never rises)."""
    A, B, Bkn, bias, mask = _operands(1024, 4096, 4096, 7)
    first = _run(epi, A, B, Bkn, bias, mask, 9)
    for _ in range(9):
        again = _run(epi, A, B, Bkn, bias, mask, 9)
        for x, y in zip(first[:3], again[:3]):
            if x is not None:
                assert torch.equal(x, y)


@pytest.mark.parametrize("epi", ["bias_relu_T", "bias_relu", "kn_mask_T_colsum"])
def test_gemm_sk_agrees_with_unsplit_kernels(epi):
    """On the MLP's M = 1024 products the split-K sum (two fp32 half-K partials, added once) differs
    from the 128x128 kernels' single K loop only by fp32 summation order: the bf16 outputs agree to
    one rounding step."""
    A, B, Bkn, bias, mask = _operands(1024, 4096, 4096, 11)
    C9 = _run(epi, A, B, Bkn, bias, mask, 9)[0].float()
    C5 = _run(epi, A, B, Bkn, bias, mask, 5 if epi.startswith("kn_") else 3)[0].float()
    diff = (C9 - C5).abs()
    assert float((diff > 0).float().mean()) < 0.05
    assert float((diff / C5.abs().clamp_min(1.0)).max()) <= 2 ** -7


def test_gemm_sk_two_streams_use_separate_workspaces():
    """Two split-K products in flight on two streams at once must not share tickets or partials."""
    A, B, Bkn, bias, mask = _operands(1024, 4096, 4096, 3)
    A2 = torch.flip(A, dims=[0]).contiguous()
    want1 = _run("bias_relu_T", A, B, Bkn, bias, mask, 9)[0]
    want2 = _run("bias_relu_T", A2, B, Bkn, bias, mask, 9)[0]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs = []
    for _ in range(4):
        with torch.cuda.stream(s1):
            o1 = _run("bias_relu_T", A, B, Bkn, bias, mask, 9)[0]
        with torch.cuda.stream(s2):
            o2 = _run("bias_relu_T", A2, B, Bkn, bias, mask, 9)[0]
        outs.append((o1, o2))
    torch.cuda.synchronize()
    for o1, o2 in outs:
        assert torch.equal(o1, want1) and torch.equal(o2, want2)


def test_gemm_sk_rejects_unfit_shapes_and_epilogues():
    A = torch.randn(256, 256, device="cuda").bfloat16()
    B = torch.randn(512, 256, device="cuda").bfloat16()  # 1 x 4 = 4 tiles: not a multiple of 8
    with pytest.raises(RuntimeError, match="split-K"):
        gemm_nt(A, B, C=torch.empty(256, 512, device="cuda").bfloat16(), variant=9)
    B = torch.randn(1024, 256, device="cuda").bfloat16()
    with pytest.raises(RuntimeError, match="split-K"):  # fp32 output: not a staged bf16 epilogue
        gemm_nt(A, B, C=torch.empty(256, 1024, device="cuda"), out_f32=True, variant=9)


def test_gemm_shape_rule_keeps_the_unsplit_kernels_by_default():
    """The split-K kernel is opt-in (DGT_GEMM_SK=1): on the MLP's M = 1024 products it measured
    slower than the 128x128 kernels (profiles/r6_gemm_m1024_splitk.jsonl), so variant 0 gives the
    unsplit kernels' bits -- and variant 9's under DGT_GEMM_SK=1."""
    import os
    if os.environ.get("DGT_GEMM_VARIANT"):
        pytest.skip("variant forced by the environment")
    A, B, Bkn, bias, mask = _operands(1024, 4096, 4096, 5)
    sk = os.environ.get("DGT_GEMM_SK", "0") not in ("", "0")
    for epi, unsplit in [("bias_relu_T", 3), ("kn_mask_T_colsum", 5)]:
        want = _run(epi, A, B, Bkn, bias, mask, 9 if sk else unsplit)[0]
        assert torch.equal(_run(epi, A, B, Bkn, bias, mask, 0)[0], want)


_HANDOVER = r"""
import sys, torch
sys.path.insert(0, {root!r})
from tests.test_gemm_sk import _operands, _run
A, B, Bkn, bias, mask = _operands(1024, 4096, 4096, 13)
outs = {{}}
for epi in ("bias_relu_T", "kn_mask_T_colsum"):
    for rep in range(3):
        C, CT, cs, _ = _run(epi, A, B, Bkn, bias, mask, 9)
        outs[f"{{epi}}_{{rep}}"] = [t.cpu() for t in (C, CT, cs) if t is not None]
torch.save(outs, {path!r})
"""


def test_gemm_sk_handover_paths_give_the_same_bits(tmp_path):
    """DGT_GEMM_SK_XS=9 (bit 3: a finisher never waits for its partner's publish) drives the
    hand-over paths -- the finisher gives its row half up and the publisher finishes it, or the
    publish lands first and the give-up loses the compare-and-swap -- which a normal launch takes
    only when a partner is late by ~20 us.  Every launch must still give the normal launch's bits."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = str(tmp_path / "handover.pt")
    env = dict(os.environ, DGT_GEMM_SK_XS="9")
    r = subprocess.run([sys.executable, "-c", _HANDOVER.format(root=root, path=path)], cwd=root, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    got = torch.load(path, weights_only=True)
    A, B, Bkn, bias, mask = _operands(1024, 4096, 4096, 13)
    for epi in ("bias_relu_T", "kn_mask_T_colsum"):
        want = [t.cpu() for t in _run(epi, A, B, Bkn, bias, mask, 9)[:3] if t is not None]
        for rep in range(3):
            for x, y in zip(got[f"{epi}_{rep}"], want):
                assert torch.equal(x, y), (epi, rep)


# ---- the 128x128 kernel's split-K mode (variant 10): small grids, K split 2 / 4 / 8 ways
SKN_SHAPES = [(128, 4096, 4096), (256, 4096, 4096), (512, 4096, 4096), (128, 512, 1024), (256, 1024, 2048)]


@pytest.mark.parametrize("M,N,K", SKN_SHAPES)
@pytest.mark.parametrize("epi", EPIS)
def test_gemm_skn_matches_fp32_reference(M, N, K, epi):
    A, B, Bkn, bias, mask = _operands(M, N, K, 3 * M + N + K)
    C, CT, cs, kw = _run(epi, A, B, Bkn, bias, mask, 10)
    kn = epi.startswith("kn_")
    ref = gemm_nt_reference(A, Bkn if kn else B, b_kn=kn, **kw)
    torch.testing.assert_close(C.float(), ref.to(torch.bfloat16).float(), rtol=2e-2, atol=2e-2 * K ** 0.5)
    if CT is not None:
        assert torch.equal(CT, C.t())
    if cs is not None:
        torch.testing.assert_close(cs, C.float().view(M // 128, 128, N).sum(1), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("epi", ["bias_relu_T", "kn_mask_T_colsum"])
@pytest.mark.parametrize("M", [128, 256, 512])
def test_gemm_skn_deterministic_close_to_unsplit_and_picked_by_the_shape_rule(epi, M):
    """The slices are summed in slice order by whichever block arrives last: ten launches give the
    same bits; against the unsplit kernel only fp32 summation order differs (one bf16 rounding step
    at most); variant 0 runs this mode for grids of at most 128 tiles (DGT_GEMM_SKN=1, default)."""
    import os
    A, B, Bkn, bias, mask = _operands(M, 4096, 4096, 17 + M)
    first = _run(epi, A, B, Bkn, bias, mask, 10)
    for _ in range(9):
        again = _run(epi, A, B, Bkn, bias, mask, 10)
        for x, y in zip(first[:3], again[:3]):
            if x is not None:
                assert torch.equal(x, y)
    C10 = first[0].float()
    C3 = _run(epi, A, B, Bkn, bias, mask, 3)[0].float()
    d = (C10 - C3).abs()
    assert float((d > 0).float().mean()) < 0.05
    assert float((d / C3.abs().clamp_min(1.0)).max()) <= 2 ** -7
    if os.environ.get("DGT_GEMM_SKN", "1") != "0" and not os.environ.get("DGT_GEMM_VARIANT"):
        assert torch.equal(_run(epi, A, B, Bkn, bias, mask, 0)[0], first[0])


def test_gemm_skn_rejects_grids_it_does_not_fit():
    A = torch.randn(1024, 4096, device="cuda").bfloat16()
    B = torch.randn(4096, 4096, device="cuda").bfloat16()  # 256 tiles: the grid already fills the chip
    with pytest.raises(RuntimeError, match="split-K mode"):
        gemm_nt(A, B, C=torch.empty(1024, 4096, device="cuda").bfloat16(), variant=10)


@pytest.mark.parametrize("mode", ["graph_module", "hip_graph"])
def test_engine_bf16_small_batch_split_k_under_graph_capture(mode):
    """The engine's bf16 chain at batch 128 on 1024-wide layers runs its products on the split-K
    mode (8 tiles -> split 2); under graph_module / the whole-step graph its per-stream workspace is
    first allocated inside a capture.  Both graphed trajectories follow the eager engine's."""
    import distributed_gpu_test_amd as dgt
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    from distributed_gpu_test_amd.ops import BCEWithLogitsLoss

    def run(amd):
        torch.manual_seed(9)
        m = SyntheticMLP(width=1024, depth=2)
        cfg = {"train_micro_batch_size_per_gpu": 128, "bf16": {"enabled": True},
               "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}, "amd": amd}
        engine, _, _, _ = dgt.initialize(model=m, config=cfg)
        crit = BCEWithLogitsLoss()
        g = torch.Generator().manual_seed(10)
        batches = [(torch.randn(128, 1024, generator=g).cuda().bfloat16(), (torch.rand(128, generator=g) > 0.5).float().cuda())
                   for _ in range(8)]
        losses = []
        if amd.get("hip_graph"):
            step = engine.graph_step(lambda bx, by: crit(engine(bx).view(-1), by))
            assert engine.graphed is not None, engine.graph_fallback_reason
            for x, y in batches:
                losses.append(float(step(x, y)))
        else:
            for x, y in batches:
                loss = crit(engine(x).view(-1), y)
                engine.backward(loss)
                engine.step()
                losses.append(float(loss))
        return engine, losses, engine.store.param_buf.detach().float().clone()

    e1, l1, p1 = run({})
    e2, l2, p2 = run({mode: True})
    if mode == "graph_module":
        assert e2.graph_module, e2.graph_module_reason
    else:
        assert e2.graphed.replays >= 6 and not e2.graphed.failed, (e2.graphed.replays, e2.graphed.failed)
    torch.testing.assert_close(torch.tensor(l2), torch.tensor(l1), rtol=2e-2, atol=2e-3)
    torch.testing.assert_close(p2, p1, rtol=2e-2, atol=2e-3)
    e1.close()
    e2.close()


# ---- the 256x256 kernel's split-K 2 mode (variant 11): 100-128 tiles of 256x256 (M = 1024 x N = 8192)
SPK256_EPIS = ["plain", "bias_relu_T", "bias_relu", "bias_T", "bias", "mask_T"]


@pytest.mark.parametrize("M,N,K", [(512, 1024, 1024), (1024, 8192, 2048), (2048, 4096, 4096)])
@pytest.mark.parametrize("epi", SPK256_EPIS)
def test_gemm_spk256_matches_fp32_reference(M, N, K, epi):
    A, B, Bkn, bias, mask = _operands(M, N, K, 5 * M + N + K)
    C, CT, _, kw = _run(epi, A, B, Bkn, bias, mask, 11)
    ref = gemm_nt_reference(A, B, **kw)
    torch.testing.assert_close(C.float(), ref.to(torch.bfloat16).float(), rtol=2e-2, atol=2e-2 * K ** 0.5)
    if CT is not None:
        assert torch.equal(CT, C.t())


def test_gemm_spk256_deterministic_close_to_unsplit_and_picked_by_the_shape_rule():
    import os
    A, B, Bkn, bias, mask = _operands(1024, 8192, 4096, 23)
    first = _run("bias_relu_T", A, B, Bkn, bias, mask, 11)
    for _ in range(5):
        again = _run("bias_relu_T", A, B, Bkn, bias, mask, 11)
        assert torch.equal(first[0], again[0]) and torch.equal(first[1], again[1])
    C8 = _run("bias_relu_T", A, B, Bkn, bias, mask, 8)[0].float()
    d = (first[0].float() - C8).abs()
    assert float((d > 0).float().mean()) < 0.05
    assert float((d / C8.abs().clamp_min(1.0)).max()) <= 2 ** -7
    if os.environ.get("DGT_GEMM_SKN", "1") != "0" and not os.environ.get("DGT_GEMM_VARIANT"):
        assert torch.equal(_run("bias_relu_T", A, B, Bkn, bias, mask, 0)[0], first[0])


def test_gemm_spk256_rejects_a_kn_operand():
    A = torch.randn(1024, 2048, device="cuda").bfloat16()
    Bkn = torch.randn(2048, 8192, device="cuda").bfloat16()
    with pytest.raises(RuntimeError):
        gemm_nt(A, Bkn, C=torch.empty(1024, 8192, device="cuda").bfloat16(), b_kn=True, variant=11)


# ---- a [K, N] operand on a 256x256-sized grid: transposed once, then the NT 256x256 kernel
@pytest.mark.parametrize("M,N,K", [(4096, 4096, 1024), (2048, 8192, 512)])
@pytest.mark.parametrize("epi", ["kn_plain", "kn_T", "kn_mask_T", "kn_mask_T_colsum"])
def test_gemm_kn_large_grid_runs_transposed_and_matches_reference(M, N, K, epi):
    import os
    A, B, Bkn, bias, mask = _operands(M, N, K, 7 * M + N + K)
    C, CT, cs, kw = _run(epi, A, B, Bkn, bias, mask, 0)
    ref = gemm_nt_reference(A, Bkn, b_kn=True, **kw)
    torch.testing.assert_close(C.float(), ref.to(torch.bfloat16).float(), rtol=2e-2, atol=2e-2 * K ** 0.5)
    if CT is not None:
        assert torch.equal(CT, C.t())
    if cs is not None:
        torch.testing.assert_close(cs, C.float().view(M // 128, 128, N).sum(1), rtol=1e-5, atol=1e-3)
    if cs is None and os.environ.get("DGT_GEMM_KN_T", "1") != "0" and not os.environ.get("DGT_GEMM_VARIANT"):
        # the same bits as the NT product on an explicit B^T (the 256x256 kernel)
        C2 = torch.empty_like(C)
        CT2 = torch.empty_like(CT) if CT is not None else None
        gemm_nt(A, Bkn.t().contiguous(), C=C2, CT=CT2, variant=8, **kw)
        assert torch.equal(C, C2)


@pytest.mark.parametrize("path", ["skn", "spk256", "kn_large"])
def test_gemm_split_paths_read_strided_operands(path):
    """Row-strided operands (column blocks of a wider matrix) on every split / transposed path: the
    K-slice offsets and the staging use the row strides, and a strided [K, N] operand keeps the
    [K, N] kernels (the transposition needs a contiguous one)."""
    g = torch.Generator().manual_seed(31)
    if path == "skn":
        M, N, K = 256, 4096, 4096
    elif path == "spk256":
        M, N, K = 1024, 8192, 2048
    else:
        M, N, K = 4096, 4096, 1024
    Aw = torch.randn(M, K + 256, generator=g).to(torch.bfloat16).cuda()
    A = Aw[:, 128:128 + K]
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    if path == "kn_large":
        Bw = torch.randn(K, N + 256, generator=g).to(torch.bfloat16).cuda()
        B = Bw[:, 64:64 + N]
        gemm_nt(A, B, C=C, b_kn=True)
        ref = A.float() @ B.float()
    else:
        Bw = torch.randn(N, K + 128, generator=g).to(torch.bfloat16).cuda()
        B = Bw[:, 64:64 + K]
        gemm_nt(A, B, C=C)
        ref = A.float() @ B.float().t()
    torch.testing.assert_close(C.float(), ref.to(torch.bfloat16).float(), rtol=2e-2, atol=2e-2 * K ** 0.5)
