"""The generic engine on the GPU (fused HIP Adam over flat buffers) vs plain PyTorch fp32."""
import copy
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
