"""Process-group setup and thin collective helpers.

Replaces ``deepspeed.init_distributed()`` + ``get_accelerator().set_device`` (``train.py:59-61``;
SURVEY X2/X3).  Backend choice: ``nccl`` — which IS RCCL on ROCm, riding xGMI between the GPUs of
a node — whenever a GPU is present, ``gloo`` otherwise (the CPU plumbing config of BASELINE.json).
No MPI discovery: rank info comes from ``launch.resolve_rank_info`` (torchrun env, SLURM env or a
bare single process).
"""
from __future__ import annotations

import datetime
import os
from typing import Any, List, Optional

import torch
import torch.distributed as dist

from ..accelerator import get_accelerator
from ..launch import RankInfo, resolve_rank_info

_RANK_INFO: Optional[RankInfo] = None
_ENV_SET: List[str] = []  # os.environ keys init_distributed added (destroy() removes them)


def default_backend() -> str:
    """``DGT_BACKEND`` overrides; else the accelerator's: nccl (= RCCL) on HIP, gloo on CPU."""
    env = os.environ.get("DGT_BACKEND")
    if env:
        return env
    return get_accelerator().communication_backend_name()


def _oversubscribed(info: RankInfo) -> bool:
    from ..accelerator import allow_oversubscribe
    return (info.world_size > 1 and allow_oversubscribe() and get_accelerator().name == "hip"
            and info.local_world_size > torch.cuda.device_count())


def init_distributed(backend: Optional[str] = None, timeout_s: float = 1800.0,
                     rank_info: Optional[RankInfo] = None, set_device: bool = True) -> RankInfo:
    """Create the default process group (idempotent) and bind this rank's GPU.

    The caller's ``os.environ`` is left alone: the rank variables are never exported (a child
    process that inherited them would believe it was a torchrun rank).  A world-size-1 job, however
    it was started, rendezvouses on an in-memory ``HashStore`` and opens no TCP port; a multi-rank
    job started by SLURM or mpirun gets an explicit ``TCPStore`` built from the resolved rank info,
    so ``env://`` (which reads ``RANK``/``MASTER_*``) is only used when torchrun already set them.
    """
    global _RANK_INFO
    info = rank_info or resolve_rank_info()
    if backend is None:
        backend = default_backend()
        if backend == "nccl" and not os.environ.get("DGT_BACKEND") and _oversubscribed(info):
            # RCCL refuses two ranks on one device ("invalid usage"): a rehearsal that shares cards on
            # purpose (DGT_ALLOW_OVERSUBSCRIBE=1) runs its process group on gloo, host-staged
            backend = "gloo"
            if info.rank == 0:
                import sys
                print(f"[dgt] {info.local_world_size} ranks share {torch.cuda.device_count()} GPU(s): process "
                      "group on gloo (RCCL needs one device per rank)", file=sys.stderr, flush=True)
    accel = get_accelerator()
    if backend == "nccl":
        if accel.name != "hip":
            raise RuntimeError("backend 'nccl' (RCCL) requested but the accelerator is "
                               f"{accel.name!r} (no GPU visible, or DGT_ACCELERATOR=cpu)")
        if set_device:  # the reference's get_accelerator().set_device(local_rank) (train.py:61)
            accel.set_device(info.local_rank)
        # hangs become errors instead of silent stalls; a torch knob read when the
        # process group is created, restored by destroy()
        if "TORCH_NCCL_ASYNC_ERROR_HANDLING" not in os.environ:
            os.environ["TORCH_NCCL_ASYNC_ERROR_HANDLING"] = "1"
            _ENV_SET.append("TORCH_NCCL_ASYNC_ERROR_HANDLING")
    if not dist.is_initialized():
        timeout = datetime.timedelta(seconds=timeout_s)
        restart = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") or 0)
        if info.world_size == 1:
            # a lone process has nobody to rendezvous with: an in-memory store, no TCP port to race
            # for, whatever launcher variables the environment happens to carry
            dist.init_process_group(backend=backend, store=dist.HashStore(), rank=0, world_size=1,
                                    timeout=timeout)
        elif restart > 0:
            # elastic restart (torchrun --max-restarts): the agent's store still holds the previous
            # attempt's keys (dead peers' addresses); rendezvous under a per-attempt prefix instead
            agent_store = os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"
            store = dist.TCPStore(info.master_addr, info.master_port, info.world_size,
                                  is_master=(info.rank == 0 and not agent_store), timeout=timeout)
            store = dist.PrefixStore(f"/dgt/attempt_{restart}", store)
            dist.init_process_group(backend=backend, store=store, rank=info.rank, world_size=info.world_size,
                                    timeout=timeout)
        elif info.source == "torchrun":
            # torchrun exported RANK / MASTER_*; env:// also honours its agent-hosted store
            dist.init_process_group(backend=backend, init_method="env://", rank=info.rank,
                                    world_size=info.world_size, timeout=timeout)
        else:
            # SLURM / mpirun / explicit rank info: the rendezvous store straight from the resolved
            # info (rank 0 hosts it), nothing written into the environment
            store = dist.TCPStore(info.master_addr, info.master_port, info.world_size,
                                  is_master=(info.rank == 0), timeout=timeout)
            dist.init_process_group(backend=backend, store=store, rank=info.rank, world_size=info.world_size,
                                    timeout=timeout)
    _RANK_INFO = info
    return info


def rank_info() -> RankInfo:
    if _RANK_INFO is not None:
        return _RANK_INFO
    return resolve_rank_info()


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def get_rank() -> int:
    return dist.get_rank() if is_initialized() else 0


def get_world_size() -> int:
    return dist.get_world_size() if is_initialized() else 1


def backend_name() -> str:
    return dist.get_backend() if is_initialized() else "none"


def force_collectives() -> bool:
    """``DGT_FORCE_COLLECTIVES=1``: issue every collective of the training paths even at world
    size 1, so a one-GPU run executes the exact async RCCL code (streams, events, work handles,
    in-graph communicator) that an N-GPU run takes.  Numerically a no-op (a 1-rank sum)."""
    return os.environ.get("DGT_FORCE_COLLECTIVES", "0") not in ("", "0", "false", "False")


def collectives_on(world_size: Optional[int] = None) -> bool:
    """Whether the training paths issue their gradient / parameter collectives."""
    ws = get_world_size() if world_size is None else world_size
    return is_initialized() and (ws > 1 or force_collectives())


def barrier() -> None:
    if collectives_on():
        if backend_name() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_gather_object(obj: Any) -> List[Any]:
    if not is_initialized() or get_world_size() == 1:
        return [obj]
    out: List[Any] = [None] * get_world_size()
    dist.all_gather_object(out, obj)
    return out


def needs_host_staging(t: torch.Tensor) -> bool:
    """gloo cannot reduce HIP tensors: stage them through host memory (tests / 1-GPU rehearsals)."""
    return t.is_cuda and backend_name() == "gloo"


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if collectives_on():
        if needs_host_staging(t):
            c = t.detach().cpu()
            dist.broadcast(c, src)
            t.copy_(c)
        else:
            dist.broadcast(t, src)
    return t


def all_reduce_(t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
    if collectives_on():
        if needs_host_staging(t):
            c = t.detach().cpu()
            dist.all_reduce(c, op=op)
            t.copy_(c)
        else:
            dist.all_reduce(t, op=op)
    return t


def all_reduce_max(value: float, device: Optional[torch.device] = None) -> float:
    if not is_initialized() or get_world_size() == 1:
        return float(value)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend_name() == "nccl" else torch.device("cpu")
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def destroy() -> None:
    """Reference teardown (``train.py:131-140``): barrier, destroy, swallow errors of dead peers."""
    try:
        barrier()
    except Exception:
        pass
    try:
        if is_initialized():
            dist.destroy_process_group()
    except Exception:
        pass
    global _RANK_INFO
    _RANK_INFO = None
    while _ENV_SET:
        os.environ.pop(_ENV_SET.pop(), None)
