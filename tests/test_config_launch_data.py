"""T0 unit tests: config schema + batch assertion, rank discovery, sampler parity."""
import json
import os
import socket

import pytest
import torch
from torch.utils.data import DistributedSampler, TensorDataset

from distributed_gpu_test_amd.config import REFERENCE_DS_CONFIG, ConfigError, parse_config, resolve_batch
from distributed_gpu_test_amd.data import (SyntheticDataset, batch_plan, make_synthetic_data, shard_indices,
                                           steps_per_epoch)
from distributed_gpu_test_amd.launch import expand_nodelist, resolve_rank_info, slurm_master_port


# ------------------------------------------------------------------ config
@pytest.mark.parametrize("ws,micro", [(1, 64), (2, 32), (4, 16), (8, 8), (16, 4)])
def test_reference_config_derives_micro_batch(ws, micro):
    cfg = parse_config(REFERENCE_DS_CONFIG, ws)
    assert cfg.train_batch_size == 64
    assert cfg.train_micro_batch_size_per_gpu == micro
    assert cfg.gradient_accumulation_steps == 1
    assert cfg.zero_stage == 0 and cfg.compute_dtype == "fp32"


@pytest.mark.parametrize("ws", [3, 5, 6, 7])
def test_reference_config_rejects_non_divisor_world_sizes(ws):
    # DeepSpeed's assertion fails for these; the message says why
    with pytest.raises(ConfigError, match="train_batch_size"):
        parse_config(REFERENCE_DS_CONFIG, ws)


def test_batch_derivations():
    assert resolve_batch(None, 4, 2, 8) == (64, 4, 2)
    assert resolve_batch(64, 4, None, 8) == (64, 4, 2)
    assert resolve_batch(64, None, 2, 8) == (64, 4, 2)
    assert resolve_batch(None, 4, None, 3) == (12, 4, 1)
    with pytest.raises(ConfigError):
        resolve_batch(64, 4, 1, 8)
    with pytest.raises(ConfigError):
        resolve_batch(None, None, None, 1)


def test_full_schema(tmp_path):
    raw = {"train_micro_batch_size_per_gpu": 8, "gradient_accumulation_steps": 2, "bf16": {"enabled": True},
           "zero_optimization": {"stage": 1, "reduce_bucket_size": 1000},
           "optimizer": {"type": "AdamW", "params": {"lr": 3e-4, "betas": [0.8, 0.99], "weight_decay": 0.1}},
           "scheduler": {"type": "WarmupLR", "params": {"warmup_num_steps": 10}},
           "gradient_clipping": 1.0, "steps_per_print": 5, "amd": {"allreduce": "rccl"}}
    p = tmp_path / "c.json"
    p.write_text(json.dumps(raw))
    cfg = parse_config(str(p), 4)
    assert cfg.train_batch_size == 64 and cfg.compute_dtype == "bf16" and cfg.zero_stage == 1
    assert cfg.optimizer.adamw and cfg.optimizer.betas == (0.8, 0.99)
    assert cfg.scheduler.type == "WarmupLR" and cfg.gradient_clipping == 1.0 and cfg.amd.allreduce == "rccl"
    with pytest.raises(ConfigError):
        parse_config({"train_batch_size": 8, "fp16": {"enabled": True}, "bf16": {"enabled": True}}, 1)
    with pytest.raises(ConfigError):
        parse_config({"train_batch_size": 8, "zero_optimization": {"stage": 3}}, 1)


def test_shipped_configs_parse():
    import glob
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = glob.glob(os.path.join(root, "configs", "*.json"))
    assert files
    for f in files:
        parse_config(f, 8)


# ------------------------------------------------------------------ launch
def test_expand_nodelist():
    assert expand_nodelist("gpu[01-03,07],login1") == ["gpu01", "gpu02", "gpu03", "gpu07", "login1"]
    assert expand_nodelist("node5") == ["node5"]
    assert expand_nodelist("r[1-2]n[0-1]") == ["r1n0", "r1n1", "r2n0", "r2n1"]
    assert expand_nodelist("a-b[9-11]") == ["a-b9", "a-b10", "a-b11"]


def test_rank_info_torchrun():
    env = {"RANK": "5", "LOCAL_RANK": "1", "WORLD_SIZE": "8", "LOCAL_WORLD_SIZE": "4", "GROUP_RANK": "1",
           "MASTER_ADDR": "10.0.0.1", "MASTER_PORT": "1234"}
    ri = resolve_rank_info(env)
    assert (ri.rank, ri.local_rank, ri.world_size, ri.node_rank, ri.source) == (5, 1, 8, 1, "torchrun")
    assert ri.master_addr == "10.0.0.1" and ri.master_port == 1234


def test_rank_info_slurm():
    env = {"SLURM_PROCID": "9", "SLURM_LOCALID": "1", "SLURM_NTASKS": "16", "SLURM_NTASKS_PER_NODE": "8",
           "SLURM_NODEID": "1", "SLURM_JOB_NODELIST": "mi355x-[003-004]", "SLURM_JOB_ID": "4242"}
    ri = resolve_rank_info(env)
    assert (ri.rank, ri.local_rank, ri.world_size, ri.local_world_size, ri.node_rank) == (9, 1, 16, 8, 1)
    assert ri.master_addr == "mi355x-003" and ri.master_port == slurm_master_port("4242") and ri.source == "slurm"
    assert slurm_master_port("4242") != slurm_master_port("4243")


def test_rank_info_bare():
    ri = resolve_rank_info({})
    assert (ri.rank, ri.world_size, ri.source) == (0, 1, "bare")
    env = ri.export({})
    assert env["WORLD_SIZE"] == "1" and env["RANK"] == "0"


_LAUNCH_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_ADDR",
                "MASTER_PORT", "TORCH_NCCL_ASYNC_ERROR_HANDLING")


def test_init_distributed_leaves_environ_unchanged(monkeypatch):
    """In-process init + destroy writes nothing into os.environ (a later child process must not
    inherit rank variables and believe it is a torchrun rank)."""
    from distributed_gpu_test_amd.parallel import comm
    comm.destroy()
    for k in _LAUNCH_VARS:
        monkeypatch.delenv(k, raising=False)
    before = dict(os.environ)
    info = comm.init_distributed(backend="gloo")
    assert (info.world_size, info.source) == (1, "bare")
    assert dict(os.environ) == before
    assert resolve_rank_info().source == "bare"
    comm.destroy()
    assert dict(os.environ) == before and not comm.is_initialized()


def test_world_size_one_never_opens_a_tcp_port(monkeypatch):
    """RANK=0 WORLD_SIZE=1 with MASTER_PORT pointing at a port another process holds (the
    GPUTEST_r03 EADDRINUSE failure): a 1-rank job rendezvouses on a HashStore and starts anyway."""
    from distributed_gpu_test_amd.parallel import comm
    comm.destroy()
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as busy:
        busy.bind(("127.0.0.1", 0))
        busy.listen(1)
        port = busy.getsockname()[1]
        monkeypatch.setenv("RANK", "0")
        monkeypatch.setenv("WORLD_SIZE", "1")
        monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
        monkeypatch.setenv("MASTER_PORT", str(port))
        info = comm.init_distributed(backend="gloo", timeout_s=20)
        assert (info.world_size, info.source) == (1, "torchrun")
        assert comm.get_world_size() == 1
        comm.destroy()


# ------------------------------------------------------------------ data
def test_synthetic_data_matches_reference_rng_order():
    torch.manual_seed(0)
    x, y = make_synthetic_data(2000, 20, 42)
    torch.manual_seed(42)
    x2 = torch.randn(2000, 20)
    assert torch.equal(x, x2)
    assert torch.equal(y, (x2[:, :10].sum(1) > 0).float().unsqueeze(1))
    # the model is initialised AFTER the data from the re-seeded RNG
    w_after = torch.nn.Linear(20, 64).weight.detach().clone()
    torch.manual_seed(42)
    torch.randn(2000, 20)
    assert torch.equal(torch.nn.Linear(20, 64).weight.detach(), w_after)


@pytest.mark.parametrize("n,ws", [(2000, 1), (2000, 2), (2000, 8), (2000, 16), (10, 3), (7, 16)])
@pytest.mark.parametrize("epoch", [1, 3])
def test_shard_indices_match_distributed_sampler(n, ws, epoch):
    ds = TensorDataset(torch.zeros(n, 1))
    for r in range(ws):
        s = DistributedSampler(ds, num_replicas=ws, rank=r, shuffle=True)
        s.set_epoch(epoch)
        assert shard_indices(n, ws, r, epoch) == list(s)


def test_batch_plan_and_steps():
    idx = shard_indices(2000, 8, 3, 1)
    plan = batch_plan(idx, 4)
    assert plan.shape == (63, 4) and steps_per_epoch(2000, 8, 4) == 63
    assert (plan[-1] >= 0).sum() == 2  # short last batch at ws=8
    assert plan[plan >= 0].tolist() == idx


def test_dataset_iteration():
    x, y = make_synthetic_data(50, 6, 1)
    ds = SyntheticDataset(x, y, batch_size=4, world_size=2, rank=1)
    ds.set_epoch(2)
    batches = list(ds)
    assert len(batches) == len(ds) == 7
    idx = shard_indices(50, 2, 1, 2)
    assert torch.equal(torch.cat([b[0] for b in batches]), x[idx])


def test_get_dataloader_helper():
    from distributed_gpu_test_amd.data import get_dataloader, make_synthetic_data
    x, y = make_synthetic_data(100, 20, 42)
    dl = get_dataloader(x, y, batch_size=32, shuffle=False)
    bx, by = next(iter(dl))
    assert bx.shape == (32, 20) and by.shape == (32, 1)
    assert torch.equal(bx, x[:32])
    assert sum(b[0].shape[0] for b in dl) == 100


def test_rank_info_mpi():
    ompi = {"OMPI_COMM_WORLD_RANK": "5", "OMPI_COMM_WORLD_SIZE": "16", "OMPI_COMM_WORLD_LOCAL_RANK": "5",
            "OMPI_COMM_WORLD_LOCAL_SIZE": "8", "MASTER_ADDR": "10.0.0.1", "MASTER_PORT": "29600"}
    ri = resolve_rank_info(ompi)
    assert (ri.rank, ri.world_size, ri.local_rank, ri.local_world_size, ri.node_rank, ri.source) == \
        (5, 16, 5, 8, 0, "mpi")
    assert (ri.master_addr, ri.master_port) == ("10.0.0.1", 29600)
    pmi = {"PMI_RANK": "9", "PMI_SIZE": "16", "MPI_LOCALRANKID": "1", "MPI_LOCALNRANKS": "8"}
    ri = resolve_rank_info(pmi)
    assert (ri.rank, ri.local_rank, ri.node_rank, ri.master_addr) == (9, 1, 1, "127.0.0.1")
    # torchrun variables win when both are present
    assert resolve_rank_info({**ompi, "RANK": "0", "WORLD_SIZE": "1"}).source == "torchrun"


def test_gather_batch_cpu_is_index_select():
    """data.gather_batch off the GPU: index_select per tensor (the one-launch HIP gather is GPU-only,
    tests/test_gpu_engine.py); SyntheticDataset yields through it."""
    import torch
    from distributed_gpu_test_amd.data import SyntheticDataset, gather_batch
    x, y = torch.randn(30, 5), torch.randn(30, 1)
    rows = torch.tensor([4, 0, 29, 4])
    gx, gy = gather_batch(rows, x, y)
    assert torch.equal(gx, x[rows]) and torch.equal(gy, y[rows])
    ds = SyntheticDataset(x, y, 4, world_size=2, rank=1)
    batches = list(ds)
    assert len(batches) == len(ds) and batches[0][0].shape == (4, 5)
