"""DeepSpeed-layout checkpoints (save AND load).

The reference calls ``model_engine.save_checkpoint(save_dir/epoch{e})`` after every epoch
(``train.py:123-125``) and never resumes.  DeepSpeed's layout is kept so existing
tooling keeps working:

    <save_dir>/latest                                   -> text: the tag
    <save_dir>/<tag>/mp_rank_00_model_states.pt         -> module state_dict, optimizer (stage 0),
                                                           global_steps, global_samples, ds_config ...
    <save_dir>/<tag>/zero_pp_rank_{r}_mp_rank_00_optim_states.pt   (ZeRO-1/2: each rank's shard)
    <save_dir>/zero_to_fp32.py                          -> consolidates ZeRO shards to an fp32 state_dict

Tag defaults to ``global_step{N}``.  Before writing, every rank checks that it saves under the
same tag (DeepSpeed's sha1 MAX/MIN all-reduce validation).  Loading uses
``torch.load(weights_only=True)`` only: checkpoints hold tensors, numbers, strings and lists.
"""
from __future__ import annotations

import hashlib
import os
import shutil
from typing import Any, Dict, Optional, Tuple

import torch
import torch.distributed as dist

from ..parallel import comm

DS_VERSION = "dgt-amd-0.1.0"
MODEL_FILE = "mp_rank_00_model_states.pt"


def zero_shard_file(rank: int) -> str:
    return f"zero_pp_rank_{rank}_mp_rank_00_optim_states.pt"


def validate_tag(tag: str, mode: str = "warn") -> bool:
    """All ranks must save under the same tag (DeepSpeed ``_checkpoint_tag_validation``)."""
    if not comm.is_initialized() or comm.get_world_size() == 1:
        return True
    digest = hashlib.sha1(tag.encode()).digest()
    dev = torch.device("cuda", torch.cuda.current_device()) if comm.backend_name() == "nccl" else torch.device("cpu")
    t = torch.tensor(list(digest), dtype=torch.int32, device=dev)
    mx, mn = t.clone(), t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(mn, op=dist.ReduceOp.MIN)
    ok = bool(torch.equal(mx, mn))
    if not ok:
        msg = f"checkpoint tag {tag!r} differs across ranks"
        if mode == "fail":
            raise RuntimeError(msg)
        if comm.get_rank() == 0:
            print(f"[dgt] WARNING: {msg}", flush=True)
    return ok


def save(save_dir: str, tag: Optional[str], global_steps: int, model_state: Dict[str, Any],
         optimizer_state: Optional[Dict[str, Any]], extra: Dict[str, Any], ds_config: Dict[str, Any],
         zero_shard: Optional[Dict[str, Any]] = None, save_latest: bool = True) -> str:
    tag = tag or f"global_step{global_steps}"
    validate_tag(tag)
    rank = comm.get_rank()
    path = os.path.join(save_dir, tag)
    if rank == 0:
        os.makedirs(path, exist_ok=True)
    comm.barrier()
    os.makedirs(path, exist_ok=True)
    if rank == 0:
        state = {
            "module": model_state,
            "buffer_names": [],
            "optimizer": optimizer_state,
            "param_shapes": [{k: list(v.shape) for k, v in model_state.items()}],
            "lr_scheduler": extra.get("lr_scheduler"),
            "sparse_tensor_module_names": [],
            "skipped_steps": int(extra.get("skipped_steps", 0)),
            "global_steps": int(global_steps),
            "global_samples": int(extra.get("global_samples", 0)),
            "dp_world_size": int(extra.get("dp_world_size", comm.get_world_size())),
            "mp_world_size": 1,
            "ds_config": ds_config,
            "ds_version": DS_VERSION,
            "client_state": extra.get("client_state", {}),
        }
        torch.save(state, os.path.join(path, MODEL_FILE))
    if zero_shard is not None:
        torch.save({"optimizer_state_dict": zero_shard, "ds_config": ds_config, "ds_version": DS_VERSION},
                   os.path.join(path, zero_shard_file(rank)))
    if rank == 0:
        if save_latest:
            with open(os.path.join(save_dir, "latest"), "w") as fh:
                fh.write(tag)
        script = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "utils", "zero_to_fp32.py")
        if os.path.exists(script):
            shutil.copyfile(script, os.path.join(save_dir, "zero_to_fp32.py"))
    comm.barrier()
    return path


def resolve_tag(load_dir: str, tag: Optional[str]) -> Optional[str]:
    if tag is not None:
        return tag
    latest = os.path.join(load_dir, "latest")
    if not os.path.exists(latest):
        return None
    with open(latest) as fh:
        return fh.read().strip()


def load(load_dir: str, tag: Optional[str] = None, rank: Optional[int] = None
         ) -> Tuple[Optional[str], Optional[Dict[str, Any]], Optional[Dict[str, Any]]]:
    """Return (path, model_states, zero_shard_or_None); (None, None, None) if nothing to load."""
    tag = resolve_tag(load_dir, tag)
    if tag is None:
        return None, None, None
    path = os.path.join(load_dir, tag)
    mfile = os.path.join(path, MODEL_FILE)
    if not os.path.exists(mfile):
        return None, None, None
    states = torch.load(mfile, map_location="cpu", weights_only=True)
    r = comm.get_rank() if rank is None else rank
    zfile = os.path.join(path, zero_shard_file(r))
    shard = None
    if os.path.exists(zfile):
        shard = torch.load(zfile, map_location="cpu", weights_only=True)["optimizer_state_dict"]
    return path, states, shard
