#!/usr/bin/env python3
"""Consolidate a ZeRO-1/2 checkpoint into one fp32 state_dict (DeepSpeed's zero_to_fp32.py role).

Reference: the script DeepSpeed copies next to checkpoints written at ``train.py:125``.

    python zero_to_fp32.py <checkpoint_dir> <output.pt> [--tag global_stepN]

<checkpoint_dir> is the directory holding ``latest`` (e.g. ds_checkpoints/epoch5).  Each rank's
``zero_pp_rank_{r}_mp_rank_00_optim_states.pt`` holds its fp32 master shard, either contiguous per
gradient bucket (the engine: for every bucket (start, numel) rank r owns elements
[start + r*numel/W, start + (r+1)*numel/W)) or as an explicit ``index`` of owned flat elements (the
fused kernel's lane ownership, ``runtime/tiny_trainer.py`` ``zero1_owner_map``).
Stage-0 checkpoints (no shards) are converted from the module weights.  Loads use
``torch.load(weights_only=True)`` only.
"""
import argparse
import glob
import os
import re

import torch


def consolidate(ckpt_dir, tag=None):
    if tag is None:
        with open(os.path.join(ckpt_dir, "latest")) as fh:
            tag = fh.read().strip()
    path = os.path.join(ckpt_dir, tag)
    model = torch.load(os.path.join(path, "mp_rank_00_model_states.pt"), map_location="cpu", weights_only=True)
    files = glob.glob(os.path.join(path, "zero_pp_rank_*_mp_rank_00_optim_states.pt"))
    if not files:
        out = {}
        opt = model.get("optimizer") or {}
        fp32 = opt.get("single_partition_of_fp32_groups")
        if fp32 and "fp32_param_names" in opt:
            # stage 0 of a bf16 / fp16 run: the exact fp32 masters, not the module's rounded copy
            flat = fp32[0].float()
            for name, (off, shape) in zip(opt["fp32_param_names"], opt["fp32_param_segments"]):
                if name is None:
                    continue
                numel = 1
                for d in shape:
                    numel *= d
                out[name] = flat[off:off + numel].view(tuple(shape)).clone()
        for k, v in model["module"].items():
            out.setdefault(k, v.float())
        return out
    shards = {}
    for f in files:
        r = int(re.search(r"zero_pp_rank_(\d+)_", os.path.basename(f)).group(1))
        shards[r] = torch.load(f, map_location="cpu", weights_only=True)["optimizer_state_dict"]
    ws = shards[0]["partition_world_size"]
    if sorted(shards) != list(range(ws)):
        raise RuntimeError(f"expected {ws} shards, found ranks {sorted(shards)}")
    meta = shards[0]
    full = torch.zeros(meta["total"], dtype=torch.float32)
    if "index" in meta:  # element-wise ownership: every element exactly once over the ranks
        seen = torch.zeros(meta["total"], dtype=torch.int64)
        for r in range(ws):
            idx = shards[r]["index"].long()
            full[idx] = shards[r]["fp32_flat"].float()
            seen.index_add_(0, idx, torch.ones_like(idx))  # counts repeated indices too
        if not bool((seen == 1).all()):
            raise RuntimeError("index shards do not cover every element exactly once")
    else:
        cursor = [0] * ws
        for start, numel in meta["buckets"]:
            n = numel // ws
            for r in range(ws):
                full[start + r * n:start + (r + 1) * n] = shards[r]["fp32_flat"][cursor[r]:cursor[r] + n]
                cursor[r] += n
    out = {}
    for name, off, shape in zip(meta["names"], meta["offsets"], meta["shapes"]):
        numel = 1
        for d in shape:
            numel *= d
        out[name] = full[off:off + numel].view(shape).clone()
    for k, v in model["module"].items():  # buffers / frozen tensors not in the optimizer
        out.setdefault(k, v.float())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("checkpoint_dir")
    ap.add_argument("output")
    ap.add_argument("--tag", default=None)
    a = ap.parse_args()
    sd = consolidate(a.checkpoint_dir, a.tag)
    torch.save(sd, a.output)
    print(f"wrote {len(sd)} tensors to {a.output}")


if __name__ == "__main__":
    main()
