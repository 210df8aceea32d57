"""bf16 MFMA GEMM + synthetic-MLP trainer vs plain PyTorch fp32 references.

CPU runs check the trainer's math through the reference ops; GPU runs (marker ``gpu``) check the
HIP kernels against the same references."""
import copy

import pytest
import torch

from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
from distributed_gpu_test_amd.ops.gemm import gemm_nt, gemm_nt_reference, mlp_head, rowsum_bf16, transpose_bf16
from distributed_gpu_test_amd.runtime.mlp_trainer import MLPTrainer


def _trainer_vs_torch(device, grad_dtype=torch.bfloat16):
    """One step of the trainer vs torch autograd on the same bf16-rounded weights and inputs:
    returns (trainer gradient, reference gradient, trainer loss, reference loss)."""
    torch.manual_seed(0)
    model = SyntheticMLP(width=128, depth=2)
    ref = copy.deepcopy(model)
    tr = MLPTrainer(model, batch_size=128, n_batches=2, lr=1e-3, device=device, grad_dtype=grad_dtype,
                    fuse_adam=False)  # the gradients are inspected
    x = tr.X[:128].float().cpu()
    y = tr.Y[:128].float().cpu()
    with torch.no_grad():
        for name, p in ref.named_parameters():
            if "layers" in name and "weight" in name:
                p.copy_(p.to(torch.bfloat16).float())
    ref_loss = torch.nn.functional.binary_cross_entropy_with_logits(ref(x).view(-1), y)
    ref_loss.backward()
    tr.step(0)
    got = torch.cat([tr.grad_of(n).reshape(-1).float().cpu() for n, _ in ref.named_parameters()])
    want = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])
    return got, want, float(tr.loss_acc.item()), float(ref_loss)


def _check(device, grad_dtype=torch.bfloat16):
    got, want, loss, ref_loss = _trainer_vs_torch(device, grad_dtype)
    assert abs(loss - ref_loss) < 1e-2 * max(1.0, abs(ref_loss))
    scale = want.abs().max()
    torch.testing.assert_close(got / scale, want / scale, rtol=0, atol=3e-2)  # bf16 activations
    cos = torch.nn.functional.cosine_similarity(got, want, dim=0)
    assert cos > 0.999, float(cos)


@pytest.mark.parametrize("grad_dtype", [torch.bfloat16, torch.float32])
def test_trainer_cpu_reference_path(grad_dtype):
    _check(torch.device("cpu"), grad_dtype)


gpu = pytest.mark.gpu


@gpu
@pytest.mark.parametrize("M,N,K,variant", [(128, 128, 64, 1), (256, 384, 128, 1), (512, 256, 1024, 1),
                                           (256, 256, 128, 2), (512, 768, 256, 2), (768, 512, 1152, 2),
                                           (2048, 1024, 4096, 2),
                                           (128, 128, 64, 4), (384, 256, 192, 4), (512, 256, 1024, 4),
                                           (128, 128, 64, 3), (384, 256, 192, 3), (512, 256, 1024, 3),
                                           (128, 128, 128, 5), (384, 256, 256, 5), (512, 256, 1024, 5),
                                           (384, 256, 192, 5),
                                           (256, 128, 128, 0), (1024, 512, 256, 0)])
@pytest.mark.parametrize("epi", ["plain", "bias_relu_T", "bias_T", "bias", "bf16bias_relu_T", "mask_T", "f32", "f32_acc",
                                 "bf16_acc"])
def test_gemm_nt_matches_reference(M, N, K, variant, epi):
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16).cuda()
    B = torch.randn(N, K, generator=g).to(torch.bfloat16).cuda()
    bias = torch.randn(N, generator=g).cuda()
    if epi.startswith("bf16bias"):  # a bf16 module's bias, read as it is
        bias, epi = bias.to(torch.bfloat16), epi[4:]
    mask = (torch.randn(M, N, generator=g) > 0).to(torch.bfloat16).cuda()
    kw = {}
    if epi == "bias_relu_T":
        kw = dict(bias=bias, relu=True)
    elif epi.startswith("bias"):
        kw = dict(bias=bias)
    elif epi == "mask_T":
        kw = dict(mask=mask)
    f32 = epi.startswith("f32")
    acc = epi.endswith("_acc")
    C = (torch.randn(M, N, generator=g) if acc else torch.zeros(M, N)).cuda().to(torch.float32 if f32 else torch.bfloat16)
    C0 = C.clone()
    CT = torch.zeros(N, M, dtype=torch.bfloat16).cuda() if epi.endswith("_T") else None
    gemm_nt(A, B, C=C, CT=CT, out_f32=f32, accumulate=acc, variant=variant, **kw)
    ref = gemm_nt_reference(A.cpu(), B.cpu(), **{k: (v.cpu() if torch.is_tensor(v) else v)
                                                  for k, v in kw.items()}).cuda()
    if acc:
        # bf16: the epilogue rounds the product to bf16, then sums with C in fp32 (rounded once more)
        ref = (ref if f32 else ref.to(torch.bfloat16).float()) + C0.float()
    tol = dict(rtol=2e-2, atol=2e-2 * K ** 0.5) if not f32 else dict(rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(C.float(), ref if f32 else ref.to(torch.bfloat16).float(), **tol)
    if CT is not None:
        torch.testing.assert_close(CT.float(), ref.t().to(torch.bfloat16).float(), rtol=2e-2, atol=2e-2 * K ** 0.5)


@gpu
@pytest.mark.parametrize("n,variant", [(128, 1), (256, 2), (128, 4)])
def test_gemm_identity_with_asymmetric_operand(n, variant):
    # A = I with an asymmetric B catches a transposed C write (cdna_hip_programming.md §3)
    M = N = K = n
    A = torch.eye(M, dtype=torch.bfloat16).cuda()
    B = torch.arange(N * K, dtype=torch.float32).remainder(251).reshape(N, K).to(torch.bfloat16).cuda()
    C = torch.empty(M, N, dtype=torch.float32).cuda()
    gemm_nt(A, B, C=C, out_f32=True, variant=variant)
    torch.testing.assert_close(C, B.float().t())


@gpu
def test_gemm_256_large_k_repeated():
    """The pipelined kernel over many K-tiles and a full wave of blocks, several launches: staging
    races show up as rare wrong tiles, so compare every launch with an fp32 reference."""
    M, N, K = 2048, 4096, 2048
    g = torch.Generator().manual_seed(7)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16).cuda()
    B = torch.randn(N, K, generator=g).to(torch.bfloat16).cuda()
    ref = A.float() @ B.float().t()
    C = torch.empty(M, N, dtype=torch.float32).cuda()
    for v in (2, 8):
        for _ in range(5):
            C.fill_(float("nan"))
            gemm_nt(A, B, C=C, out_f32=True, variant=v)
            torch.testing.assert_close(C, ref, rtol=1e-3, atol=1e-2)


@gpu
@pytest.mark.parametrize("K", [128, 256, 384, 1024])
@pytest.mark.parametrize("epi", ["plain", "bias_relu_t", "f32_acc", "adam"])
def test_gemm_256_cross_phase_prefetch_is_bitwise_variant2(K, epi):
    """Variant 8 (the 256x256 kernel reading phase P + 1's fragments during phase P's MFMAs) runs
    variant 2's MFMAs in the same order per accumulator: every epilogue's output, the fused Adam's
    state included, equals variant 2's bit for bit -- at one loop iteration (K = 128: only the
    drain iteration), two, three and eight."""
    from distributed_gpu_test_amd.ops.gemm import gemm_nt_adam_
    g = torch.Generator().manual_seed(K)
    M, N = 512, 768
    A = torch.randn(M, K, generator=g).to(torch.bfloat16).cuda()
    B = torch.randn(N, K, generator=g).to(torch.bfloat16).cuda()
    bias = torch.randn(N, generator=g).cuda()
    base = torch.randn(M, N, generator=g).cuda()
    outs = []
    for v in (2, 8):
        if epi == "plain":
            C = torch.empty(M, N, dtype=torch.bfloat16).cuda()
            gemm_nt(A, B, C=C, variant=v)
            outs.append([C])
        elif epi == "bias_relu_t":
            C = torch.empty(M, N, dtype=torch.bfloat16).cuda()
            CT = torch.empty(N, M, dtype=torch.bfloat16).cuda()
            gemm_nt(A, B, C=C, CT=CT, bias=bias, relu=True, variant=v)
            outs.append([C, CT])
        elif epi == "f32_acc":
            C = base.clone()
            gemm_nt(A, B, C=C, out_f32=True, accumulate=True, variant=v)
            outs.append([C])
        else:
            p, m, s = base.clone(), torch.zeros(M, N).cuda(), torch.zeros(M, N).cuda()
            pb = torch.empty(M, N, dtype=torch.bfloat16).cuda()
            gemm_nt_adam_(A, B, p, m, s, pb, 3, 1e-3, 0.9, 0.999, 1e-8, variant=v)
            outs.append([p, m, s, pb])
    assert all(torch.equal(x, y) for x, y in zip(*outs))
    if epi == "f32_acc":
        torch.testing.assert_close(outs[1][0], base + A.float() @ B.float().t(), rtol=1e-3, atol=1e-2)


@gpu
def test_gemm_256_asm_staging_high_address():
    """The 256x256 kernel's asm DMAs take their base from SGPRs as two 32-bit halves: operands whose
    address has bit 31 of the low word set (a sign-extension bug there faulted only on such
    addresses) must give the fp32 reference's result."""
    M, N, K = 512, 512, 1024
    nbytes = (M + N) * K * 2
    buf = torch.empty((1 << 32) + nbytes + 4096, dtype=torch.uint8, device="cuda")
    low = buf.data_ptr() & 0xFFFFFFFF
    off = 0 if (low >= 0x80000000 and low + nbytes < (1 << 32)) else ((0x80000000 - low) % (1 << 32))
    off = (off + 255) // 256 * 256
    A = buf[off:off + M * K * 2].view(torch.bfloat16).view(M, K)
    B = buf[off + M * K * 2:off + nbytes].view(torch.bfloat16).view(N, K)
    assert (A.data_ptr() & 0xFFFFFFFF) >= 0x80000000 and (B.data_ptr() & 0xFFFFFFFF) >= 0x80000000
    g = torch.Generator().manual_seed(3)
    A.copy_(torch.randn(M, K, generator=g).bfloat16())
    B.copy_(torch.randn(N, K, generator=g).bfloat16())
    C = torch.empty(M, N, dtype=torch.float32, device="cuda")
    gemm_nt(A, B, C=C, out_f32=True, variant=2)
    torch.testing.assert_close(C, A.float() @ B.float().t(), rtol=1e-3, atol=1e-2)
    del buf


@gpu
def test_gemm_strided_operand():
    A = torch.randn(128, 64).to(torch.bfloat16).cuda()
    wide = torch.randn(128, 256).to(torch.bfloat16).cuda()
    Bv = wide[:, 64:128]  # row stride 256
    C = torch.empty(128, 128, dtype=torch.float32).cuda()
    gemm_nt(A, Bv, C=C, out_f32=True)
    torch.testing.assert_close(C, A.float() @ Bv.float().t(), rtol=1e-4, atol=1e-3)


@gpu
def test_transpose_rowsum_head():
    for shape in [(192, 320), (100, 72), (64, 4096)]:  # full 64 x 64 tiles (register kernel) and ragged
        x = torch.randn(*shape).to(torch.bfloat16).cuda()
        xt = torch.empty(shape[1], shape[0], dtype=torch.bfloat16).cuda()
        transpose_bf16(x, xt)
        assert torch.equal(xt, x.t().contiguous()), shape
    x = torch.randn(192, 320).to(torch.bfloat16).cuda()
    out = torch.empty(192).cuda()
    rowsum_bf16(x, out)
    torch.testing.assert_close(out, x.float().sum(1), rtol=1e-4, atol=1e-3)
    B, D = 128, 256
    a = torch.relu(torch.randn(B, D)).to(torch.bfloat16)
    w, b0, y = torch.randn(D) * 0.1, torch.tensor([0.05]), (torch.rand(B) > 0.5).float()
    bufs = lambda dev: [torch.zeros(B, device=dev), torch.zeros(D, device=dev), torch.zeros(1, device=dev),
                        torch.zeros(1, dtype=torch.float64, device=dev),
                        torch.zeros(B, D, dtype=torch.bfloat16, device=dev),
                        torch.zeros(D, B, dtype=torch.bfloat16, device=dev)]
    ref, got = bufs("cpu"), bufs("cuda")
    mlp_head(a, w, b0, y, *ref)
    mlp_head(a.cuda(), w.cuda(), b0.cuda(), y.cuda(), *got)
    for r, g_ in zip(ref, got):
        torch.testing.assert_close(g_.cpu().float(), r.float(), rtol=2e-2, atol=1e-4)


@gpu
@pytest.mark.parametrize("kn", [False, True])
@pytest.mark.parametrize("fr", [3, 5])
def test_gemm_variant3_is_bitwise_variant4(kn, fr):
    """Front-loaded fragment reads (variant 3) change the schedule only: same MFMAs in the same
    order, so every epilogue output equals variant 4's bit for bit."""
    g = torch.Generator().manual_seed(11 + kn)
    M, N, K = 512, 384, 1024
    A = torch.randn(M, K, generator=g).to(torch.bfloat16).cuda()
    B = torch.randn(*((K, N) if kn else (N, K)), generator=g).to(torch.bfloat16).cuda()
    mask = (torch.randn(M, N, generator=g) > 0).to(torch.bfloat16).cuda()
    bias = torch.randn(N, generator=g).cuda()
    outs = []
    for v in (4, fr):
        C = torch.empty(M, N, dtype=torch.bfloat16).cuda()
        CT = torch.empty(N, M, dtype=torch.bfloat16).cuda()
        if kn:
            gemm_nt(A, B, C=C, CT=CT, mask=mask, b_kn=True, variant=v)
        else:
            gemm_nt(A, B, C=C, CT=CT, bias=bias, relu=True, variant=v)
        outs.append((C, CT))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@gpu
@pytest.mark.parametrize("rp", [6, 7])
@pytest.mark.parametrize("epi", ["bias_relu_t", "bias", "f32"])
def test_gemm_register_prefetch_is_bitwise_variant3(rp, epi):
    """The register-prefetch kernels (6: 2 K-tiles in VGPRs, 7: 4) stage the same LDS image and run
    variant 3's fragment reads and MFMAs: every epilogue output equals variant 3's bit for bit, and
    a [K, N] product (the dgrad, plain and with the mask + C^T + column-sum epilogue) equals the
    unsplit kernels' (variant 5, itself bitwise variant 4; for this small grid the shape rule would
    pick the split-K mode, variant 10)."""
    g = torch.Generator().manual_seed(rp)
    M, N, K = 512, 384, 1024
    A = torch.randn(M, K, generator=g).to(torch.bfloat16).cuda()
    B = torch.randn(N, K, generator=g).to(torch.bfloat16).cuda()
    bias = torch.randn(N, generator=g).cuda()
    outs = []
    for v in (3, rp):
        if epi == "f32":
            C = torch.empty(M, N, dtype=torch.float32).cuda()
            gemm_nt(A, B, C=C, out_f32=True, variant=v)
            outs.append((C, C))
            continue
        C = torch.empty(M, N, dtype=torch.bfloat16).cuda()
        CT = torch.empty(N, M, dtype=torch.bfloat16).cuda()
        if epi == "bias_relu_t":
            gemm_nt(A, B, C=C, CT=CT, bias=bias, relu=True, variant=v)
        else:
            gemm_nt(A, B, C=C, bias=bias, variant=v)
            CT = C
        outs.append((C, CT))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    Bkn = torch.randn(K, N, generator=g).to(torch.bfloat16).cuda()
    C0 = torch.empty(M, N, dtype=torch.bfloat16).cuda()
    C1 = torch.empty(M, N, dtype=torch.bfloat16).cuda()
    gemm_nt(A, Bkn, C=C0, b_kn=True, variant=5)
    gemm_nt(A, Bkn, C=C1, b_kn=True, variant=rp)
    assert torch.equal(C0, C1)
    mask = (torch.randn(M, N, generator=g) > 0).to(torch.bfloat16).cuda()
    outs = []
    for v in (5, rp):
        C = torch.empty(M, N, dtype=torch.bfloat16).cuda()
        CT = torch.empty(N, M, dtype=torch.bfloat16).cuda()
        cs = torch.empty(M // 128, N, dtype=torch.float32).cuda()
        gemm_nt(A, Bkn, C=C, CT=CT, mask=mask, b_kn=True, variant=v, colsum=cs)
        outs.append((C, CT, cs))
    assert all(torch.equal(x, y) for x, y in zip(*outs))


@gpu
@pytest.mark.parametrize("N,mask", [(1, True), (3, False)])
def test_skinny_head_matches_reference_and_is_reproducible(N, mask):
    """skinny_fwd/bwd_bf16 (the engine chain's Linear(K, N <= 4) head) against the fp32 reference;
    the backward's dW is a fixed-order sum of per-tile partials, so two runs agree bit for bit."""
    from distributed_gpu_test_amd.ops.gemm import skinny_bwd_bf16, skinny_fwd_bf16
    M, K = 1024, 512
    g = torch.Generator().manual_seed(N)
    a = torch.relu(torch.randn(M, K, generator=g)).to(torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, generator=g).to(torch.bfloat16)
    dz = (torch.randn(M, N, generator=g) * 1e-2).to(torch.bfloat16)
    z = torch.empty(M, N, dtype=torch.bfloat16).cuda()
    skinny_fwd_bf16(a.cuda(), W.cuda(), b.cuda(), z)
    torch.testing.assert_close(z.cpu().float(), a.float() @ W.float().t() + b.float(), rtol=2e-2, atol=2e-2)
    runs = []
    for _ in range(2):
        out = [torch.empty(M, K, dtype=torch.bfloat16).cuda(), torch.empty(K, M, dtype=torch.bfloat16).cuda(),
               torch.full((N, K), 0.5).cuda(), torch.full((N,), 0.25).cuda()]
        skinny_bwd_bf16(dz.cuda(), a.cuda(), W.cuda(), mask, *out)
        runs.append([t.cpu() for t in out])
    gref = dz.float() @ W.float()
    if mask:
        gref = gref * (a.float() > 0)
    torch.testing.assert_close(runs[0][0].float(), gref, rtol=2e-2, atol=1e-4)
    assert torch.equal(runs[0][1], runs[0][0].t().contiguous())
    torch.testing.assert_close(runs[0][2], 0.5 + dz.float().t() @ a.float(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(runs[0][3], 0.25 + dz.float().sum(0), rtol=1e-4, atol=1e-4)
    for x, y in zip(*runs):
        assert torch.equal(x, y)
    # straight into bf16 gradient views: stored (first write of a backward), then accumulated
    dWh, dbh = torch.full((N, K), 7.0, dtype=torch.bfloat16).cuda(), torch.full((N,), 7.0, dtype=torch.bfloat16).cuda()
    g2, gT2 = torch.empty(M, K, dtype=torch.bfloat16).cuda(), torch.empty(K, M, dtype=torch.bfloat16).cuda()
    skinny_bwd_bf16(dz.cuda(), a.cuda(), W.cuda(), mask, g2, gT2, dWh, dbh, accumulate=False)
    torch.testing.assert_close(dWh.cpu().float(), (dz.float().t() @ a.float()).bfloat16().float(), rtol=1e-2, atol=1e-3)
    torch.testing.assert_close(dbh.cpu().float(), dz.float().sum(0).bfloat16().float(), rtol=1e-2, atol=1e-3)
    skinny_bwd_bf16(dz.cuda(), a.cuda(), W.cuda(), mask, g2, gT2, dWh, dbh, accumulate=True)
    torch.testing.assert_close(dWh.cpu().float(), 2 * (dz.float().t() @ a.float()), rtol=2e-2, atol=2e-3)


@gpu
@pytest.mark.parametrize("grad_dtype", [torch.bfloat16, torch.float32])
def test_trainer_gpu_matches_torch(grad_dtype):
    _check(torch.device("cuda"), grad_dtype)


def _run_schedule(device, schedule, steps=3):
    torch.manual_seed(0)
    model = SyntheticMLP(width=128, depth=3)
    # fuse_adam=False: the schedules are those of the gradient-buffer path (the single-rank fused
    # wgrad+Adam has no schedule; test_mlp_fused_adam_matches_unfused_fp32_grads covers it)
    tr = MLPTrainer(model, batch_size=128, n_batches=2, lr=1e-3, device=device, schedule=schedule, fuse_adam=False)
    for s in range(steps):
        tr.step(s)
    tr.join()
    return tr


def test_trainer_schedules_agree_cpu():
    """serial (per-layer Adam) and flat (one Adam launch) give the same update."""
    a, b = _run_schedule(torch.device("cpu"), "serial"), _run_schedule(torch.device("cpu"), "flat")
    assert torch.equal(a.master_w, b.master_w) and torch.equal(a.m_w, b.m_w) and torch.equal(a.v_w, b.v_w)


@gpu
def test_trainer_overlap_schedule_is_bitwise_serial():
    """Side-stream per-layer updates are a schedule change only: same parameters bit for bit (the
    head's dw is a fixed-order sum of per-tile partials, so the small fp32 region and the loss are
    reproducible too)."""
    dev = torch.device("cuda")
    runs = {s: _run_schedule(dev, s, steps=4) for s in ("overlap", "serial", "flat")}
    base = runs["serial"]
    for name in ("overlap", "flat"):
        r = runs[name]
        assert torch.equal(r.master_w, base.master_w), name
        assert torch.equal(r.params_bf16, base.params_bf16), name
        assert torch.equal(r.master_s, base.master_s), name
        assert torch.equal(r.loss_acc, base.loss_acc), name


@gpu
@pytest.mark.parametrize("M,N,K,variant", [(128, 128, 64, 1), (256, 384, 128, 1), (128, 128, 64, 4),
                                           (384, 256, 192, 4), (512, 256, 1024, 4), (256, 512, 512, 0),
                                           (128, 128, 64, 3), (384, 256, 192, 3), (512, 256, 1024, 3),
                                           (128, 128, 128, 5), (384, 256, 256, 5), (512, 256, 1024, 5)])
@pytest.mark.parametrize("epi", ["plain", "mask_T", "T", "f32"])
def test_gemm_b_kn_matches_reference(M, N, K, variant, epi):
    """B given as [K, N] (the dgrad reading W[out, in] directly through transposed LDS reads)."""
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16).cuda()
    B = torch.randn(K, N, generator=g).to(torch.bfloat16).cuda()
    mask = (torch.randn(M, N, generator=g) > 0).to(torch.bfloat16).cuda()
    f32 = epi == "f32"
    C = torch.zeros(M, N, dtype=torch.float32 if f32 else torch.bfloat16).cuda()
    CT = torch.zeros(N, M, dtype=torch.bfloat16).cuda() if epi.endswith("T") else None
    kw = dict(mask=mask) if epi == "mask_T" else {}
    gemm_nt(A, B, C=C, CT=CT, out_f32=f32, variant=variant, b_kn=True, **kw)
    ref = gemm_nt_reference(A.cpu(), B.cpu(), b_kn=True, **{k: v.cpu() for k, v in kw.items()}).cuda()
    tol = dict(rtol=1e-4, atol=1e-3) if f32 else dict(rtol=2e-2, atol=2e-2 * K ** 0.5)
    torch.testing.assert_close(C.float(), ref if f32 else ref.to(torch.bfloat16).float(), **tol)
    if CT is not None:
        torch.testing.assert_close(CT.float(), ref.t().to(torch.bfloat16).float(), rtol=2e-2, atol=2e-2 * K ** 0.5)


@gpu
@pytest.mark.parametrize("variant", [1, 3, 4, 5])
def test_gemm_b_kn_identity_asymmetric(variant):
    # A = I: C must equal B exactly, catching any transposed / swizzled fragment read
    n = 256
    A = torch.eye(n, dtype=torch.bfloat16).cuda()
    B = torch.arange(n * n, dtype=torch.float32).remainder(251).reshape(n, n).to(torch.bfloat16).cuda()
    C = torch.empty(n, n, dtype=torch.float32).cuda()
    gemm_nt(A, B, C=C, out_f32=True, variant=variant, b_kn=True)
    torch.testing.assert_close(C, B.float())


@pytest.mark.parametrize("comm,want", [(None, torch.bfloat16), (torch.bfloat16, torch.bfloat16),
                                       (torch.float32, torch.float32)])
def test_trainer_comm_dtype_selects_gradient_wire(comm, want):
    """communication_data_type for the MLP trainer: the collectives carry the gradient buffer, so
    an fp32 wire means fp32 gradients from the wgrad epilogue (and the step still trains)."""
    torch.manual_seed(0)
    tr = MLPTrainer(SyntheticMLP(width=64, depth=2), batch_size=32, n_batches=2, lr=1e-3,
                    device=torch.device("cpu"), comm_dtype=comm)
    assert tr.grads_w.dtype == want
    before = tr.params.clone()
    tr.step(0)
    assert not torch.equal(before, tr.params)


@gpu
@pytest.mark.parametrize("M,N,K,variant", [(128, 128, 64, 1), (256, 384, 128, 4), (512, 256, 1024, 4),
                                           (512, 256, 1024, 3), (512, 256, 1024, 5), (256, 256, 128, 2),
                                           (512, 768, 256, 2), (512, 768, 1024, 2),
                                           (1024, 1024, 1024, 0)])
@pytest.mark.parametrize("wd,adamw", [(0.0, False), (0.01, True)])
def test_gemm_nt_adam_matches_reference(M, N, K, variant, wd, adamw):
    """wgrad + Adam in one launch (kEpiAdam epilogue through LDS, both kernels) against an fp32
    gradient GEMM followed by the reference Adam."""
    from distributed_gpu_test_amd.ops.gemm import gemm_nt_adam_
    from distributed_gpu_test_amd.ops.reference import adam_flat_reference_
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A = (torch.randn(M, K, generator=g) * 0.1).to(torch.bfloat16).cuda()
    B = (torch.randn(N, K, generator=g) * 0.1).to(torch.bfloat16).cuda()
    p = torch.randn(M, N, generator=g).cuda()
    m = (torch.randn(M, N, generator=g) * 1e-2).cuda()
    v = (torch.rand(M, N, generator=g) * 1e-3).cuda()
    lp = torch.empty(M, N, dtype=torch.bfloat16).cuda()
    grad = (A.float() @ B.float().t()) * 0.5
    p2, m2, v2 = p.clone().view(-1), m.clone().view(-1), v.clone().view(-1)
    adam_flat_reference_(p2, grad.reshape(-1), m2, v2, 7, 1e-3, 0.9, 0.999, 1e-8, wd, adamw)
    gemm_nt_adam_(A, B, p, m, v, lp, 7, 1e-3, 0.9, 0.999, 1e-8, wd, adamw, grad_scale=0.5, variant=variant)
    torch.testing.assert_close(p.view(-1), p2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m.view(-1), m2, rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(v.view(-1), v2, rtol=1e-4, atol=1e-9)
    assert torch.equal(lp, p.to(torch.bfloat16))


@gpu
def test_mlp_fused_adam_matches_unfused_fp32_grads():
    """The fused single-rank step (dgrad first, then wgrad + Adam in one launch per layer) moves the
    parameters exactly like the unfused step with fp32 gradients: same fp32 gradient values, same
    per-element Adam."""
    outs = []
    for fused in (False, True):
        torch.manual_seed(0)
        tr = MLPTrainer(SyntheticMLP(width=256, depth=3), batch_size=128, n_batches=2, lr=1e-3,
                        device=torch.device("cuda"), grad_dtype=torch.float32, fuse_adam=fused)
        assert tr.fused_adam == fused
        for s in range(4):
            tr.step(s)
        torch.cuda.synchronize()
        outs.append((tr.params.clone(), tr.master_w.clone(), tr.m_w.clone(), tr.v_w.clone(), float(tr.loss_acc.item())))
    for a, b in zip(outs[0][:4], outs[1][:4]):
        assert torch.equal(a, b)
    assert outs[0][4] == outs[1][4]


@gpu
def test_mlp_side_stream_wgrad_adam_is_bitwise_in_line(monkeypatch):
    """DGT_MLP_WGA_SIDE=1 moves each fused wgrad+Adam launch to a side stream beside the dgrads
    (three rotating gradient buffers, the next forward waits per layer): a schedule change only."""
    def run(side):
        monkeypatch.setenv("DGT_MLP_WGA_SIDE", "1" if side else "0")
        torch.manual_seed(0)
        tr = MLPTrainer(SyntheticMLP(width=256, depth=3), batch_size=256, n_batches=2, lr=1e-3,
                        device=torch.device("cuda"))
        for s in range(4):
            tr.step(s)
        tr.join()
        torch.cuda.synchronize()
        return tr
    a, b = run(False), run(True)
    assert b._wga_side and not a._wga_side
    assert torch.equal(a.master_w, b.master_w) and torch.equal(a.params_bf16, b.params_bf16)
    assert torch.equal(a.m_w, b.m_w) and torch.equal(a.loss_acc, b.loss_acc)


@gpu
def test_dgrad_colsum_and_head_partials():
    """The bias-gradient partials: the [K, N] dgrad epilogue's per-128-row-tile column sums of its
    bf16 output (colsum), the head's per-64-row-tile sums of g and of dz a, and their one-launch
    fixed-order reduction (partials_reduce_multi: bitwise the in-order sum)."""
    from distributed_gpu_test_amd.ops.gemm import partials_reduce_multi
    g_ = torch.Generator().manual_seed(5)
    M, N, K = 1024, 512, 256
    A = torch.randn(M, K, generator=g_).bfloat16().cuda()
    W = torch.randn(K, N, generator=g_).bfloat16().cuda()
    mask = (torch.randn(M, N, generator=g_) > 0).bfloat16().cuda()
    C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    CT = torch.empty(N, M, dtype=torch.bfloat16, device="cuda")
    cs = torch.full((M // 128, N), float("nan"), device="cuda")
    gemm_nt(A, W, C=C, CT=CT, mask=mask, b_kn=True, colsum=cs)
    want = C.float().view(M // 128, 128, N).sum(1)  # the kernel's own output, tile by tile
    torch.testing.assert_close(cs, want, rtol=1e-5, atol=1e-4)
    cs2 = torch.empty_like(cs)
    gemm_nt(A, W, C=C, CT=CT, mask=mask, b_kn=True, colsum=cs2)
    assert torch.equal(cs, cs2)  # fixed order
    # head partials
    B, D = 256, 512
    a = torch.relu(torch.randn(B, D, generator=g_)).bfloat16().cuda()
    w, b0 = (torch.randn(D, generator=g_) * 0.1).cuda(), torch.tensor([0.05]).cuda()
    y = (torch.rand(B, generator=g_) > 0.5).float().cuda()
    outs = [torch.zeros(B, device="cuda"), torch.zeros(D, device="cuda"), torch.zeros(1, device="cuda"),
            torch.zeros(1, dtype=torch.float64, device="cuda"), torch.empty(B, D, dtype=torch.bfloat16, device="cuda"),
            torch.empty(D, B, dtype=torch.bfloat16, device="cuda")]
    dwp, bp = torch.empty(B // 64, D, device="cuda"), torch.empty(B // 64, D, device="cuda")
    mlp_head(a, w, b0, y, *outs, dw_part=dwp, bias_part=bp)
    dz, gh = outs[0], outs[4]
    torch.testing.assert_close(bp, gh.float().view(B // 64, 64, D).sum(1), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dwp, (dz.view(B // 64, 64, 1) * a.float().view(B // 64, 64, D)).sum(1),
                               rtol=1e-4, atol=1e-7)
    # one launch, several segments, the tiles added in order
    o1, o2, o3 = torch.empty(N, device="cuda"), torch.empty(D, device="cuda"), torch.empty(D, device="cuda")
    partials_reduce_multi([(cs, o1), (bp, o2), (dwp, o3)])
    for p, o in ((cs, o1), (bp, o2), (dwp, o3)):
        acc = torch.zeros_like(p[0])
        for t in range(p.shape[0]):
            acc += p[t]
        assert torch.equal(o, acc)


@gpu
def test_skinny_bias_part_and_bf16_accumulating_reduce():
    """The engine chain's bias gradients: skinny_bwd's per-64-row-tile column sums of its bf16 g,
    reduced with the dgrad colsum into bf16 gradient views (stored, or added to what is there: the
    sum in fp32, rounded once) -- the CPU reference's bits."""
    from distributed_gpu_test_amd.ops.gemm import partials_reduce_multi, skinny_bwd_bf16
    g_ = torch.Generator().manual_seed(9)
    M, K, N = 512, 384, 2
    dz = torch.randn(M, N, generator=g_).bfloat16()
    a = torch.relu(torch.randn(M, K, generator=g_)).bfloat16()
    w = torch.randn(N, K, generator=g_).bfloat16()
    outs = {}
    for dev in ("cpu", "cuda"):
        g = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
        dw, db = torch.zeros(N, K, device=dev), torch.zeros(N, device=dev)
        bp = torch.full((M // 64, K), float("nan"), device=dev)
        skinny_bwd_bf16(dz.to(dev), a.to(dev), w.to(dev), True, g, None, dw, db, bias_part=bp)
        outs[dev] = (g, bp)
    torch.testing.assert_close(outs["cuda"][0].cpu(), outs["cpu"][0], rtol=1e-2, atol=1e-2)
    gc, bpc = outs["cuda"]
    torch.testing.assert_close(bpc, gc.float().view(M // 64, 64, K).sum(1), rtol=1e-5, atol=1e-5)
    # dW left as per-row-tile partials for the caller (dw itself untouched; db still formed)
    parts = {}
    for dev in ("cpu", "cuda"):
        g = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
        dw, db = torch.full((N, K), 7.0, device=dev), torch.zeros(N, device=dev)
        dwp = torch.empty(M // 64, N * K, device=dev)
        skinny_bwd_bf16(dz.to(dev), a.to(dev), w.to(dev), True, g, None, dw, db, accumulate=False, dw_part=dwp)
        assert bool((dw == 7.0).all())
        parts[dev] = (dwp, db)
    torch.testing.assert_close(parts["cuda"][0].cpu(), parts["cpu"][0], rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(parts["cuda"][1].cpu(), parts["cpu"][1], rtol=1e-4, atol=1e-4)
    # bf16 outs (stored / accumulated), an fp32 accumulate, one launch; every out against the CPU path
    base = torch.randn(K, generator=g_)
    views = {dev: (torch.zeros(K, dtype=torch.bfloat16, device=dev), base.bfloat16().to(dev),
                   base.clone().to(dev)) for dev in ("cpu", "cuda")}
    p = bpc.cpu()
    for dev in ("cpu", "cuda"):
        o1, o2, o3 = views[dev]
        partials_reduce_multi([(p.to(dev), o1), (p.to(dev), o2, True), (p.to(dev), o3, True)])
    for x, y in zip(views["cuda"], views["cpu"]):
        assert torch.equal(x.cpu(), y)


@gpu
def test_partials_reduce_with_adam_is_bitwise_adam_flat():
    """The small region's reduction + Adam in one launch gives adam_flat's bits (and the gradients)."""
    from distributed_gpu_test_amd.ops.adam import adam_flat_
    from distributed_gpu_test_amd.ops.gemm import partials_reduce_multi
    g_ = torch.Generator().manual_seed(9)
    n = 1028  # exactly the three segments: adam_flat over it touches the same elements
    grads = torch.zeros(n, device="cuda")
    parts = [torch.randn(8, 512, generator=g_).cuda() for _ in range(2)]
    master = torch.randn(n, generator=g_).cuda()
    m, v = (torch.randn(n, generator=g_) * 1e-2).cuda(), (torch.rand(n, generator=g_) * 1e-3).cuda()
    grads[1024:1028] = torch.tensor([0.5, 0.0, 0.0, 0.0], device="cuda")  # a one-tile in-place segment
    ref = [t.clone() for t in (grads, master, m, v)]
    pairs = lambda g: [(parts[0], g[0:512]), (parts[1], g[512:1024]), (g[1024:1028].view(1, 4), g[1024:1028])]
    partials_reduce_multi(pairs(grads), adam=(grads, master, m, v, 3, 1e-3, 0.9, 0.999, 1e-8, 0.01, True, 0.5))
    partials_reduce_multi(pairs(ref[0]))
    adam_flat_(ref[1], ref[0], ref[2], ref[3], 3, 1e-3, 0.9, 0.999, 1e-8, 0.01, True, grad_scale=0.5)
    for a, b in zip((grads, master, m, v), ref):
        assert torch.equal(a, b)
