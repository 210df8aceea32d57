"""Rank / world discovery for every way this framework gets started.

The reference reads ``LOCAL_RANK`` / ``WORLD_SIZE`` from the environment that
``torch.distributed.launch`` sets (``train.py:56-57``), and relies on
DeepSpeed's ``init_distributed`` to find ``RANK`` / ``MASTER_ADDR`` /
``MASTER_PORT``.  Its SLURM script computes ``MASTER_ADDR`` with
``scontrol show hostnames`` and hard-codes ``MASTER_PORT=12345``
(``slurm_train.sbatch:14-15``).

Here one resolver handles four launch modes, in priority order:

1. torchrun / ``torch.distributed.launch`` env (``RANK``, ``WORLD_SIZE`` ...);
2. ``srun`` with one task per GPU (``SLURM_PROCID`` / ``SLURM_NTASKS`` ...);
   ``MASTER_ADDR`` is the first host of ``SLURM_JOB_NODELIST`` (parsed here,
   no ``scontrol`` needed) and the port is derived from ``SLURM_JOB_ID`` so two
   jobs on one head node do not collide;
3. ``mpirun`` (Open MPI ``OMPI_COMM_WORLD_*`` / MPICH ``PMI_*``), DeepSpeed's MPI discovery;
4. bare ``python train.py``: a single rank on 127.0.0.1 (SURVEY Q1/Q9 fixed).
"""
from __future__ import annotations

import os
import re
import socket
from dataclasses import dataclass, asdict
from typing import Dict, List, Mapping, Optional

DEFAULT_PORT = 29500


@dataclass(frozen=True)
class RankInfo:
    rank: int
    local_rank: int
    world_size: int
    local_world_size: int
    node_rank: int
    master_addr: str
    master_port: int
    source: str  # "torchrun" | "slurm" | "mpi" | "bare"

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    def as_dict(self) -> Dict[str, object]:
        return asdict(self)

    def export(self, env: Optional[Dict[str, str]] = None) -> Dict[str, str]:
        """Write the torchrun-style variables (what ``init_process_group('env://')`` reads)."""
        env = os.environ if env is None else env
        env["RANK"] = str(self.rank)
        env["LOCAL_RANK"] = str(self.local_rank)
        env["WORLD_SIZE"] = str(self.world_size)
        env["LOCAL_WORLD_SIZE"] = str(self.local_world_size)
        env["GROUP_RANK"] = str(self.node_rank)
        env["MASTER_ADDR"] = self.master_addr
        env["MASTER_PORT"] = str(self.master_port)
        return env


# --------------------------------------------------------------------------- SLURM helpers
_RANGE = re.compile(r"^(\d+)(?:-(\d+))?$")


def _split_top_level(s: str) -> List[str]:
    """Split a nodelist on commas that are not inside ``[...]``."""
    out, depth, cur = [], 0, []
    for ch in s:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    if cur:
        out.append("".join(cur))
    return [p for p in (x.strip() for x in out) if p]


def expand_nodelist(nodelist: str) -> List[str]:
    """Expand a SLURM hostlist expression like ``scontrol show hostnames`` does.

    ``gpu[01-03,07],login1`` -> ``["gpu01", "gpu02", "gpu03", "gpu07", "login1"]``.
    Zero padding of the range bounds is preserved.  Multiple bracket groups
    (``r[1-2]n[1-2]``) expand as a cartesian product.
    """
    hosts: List[str] = []
    for item in _split_top_level(nodelist):
        parts = re.split(r"(\[[^\]]*\])", item)
        expansions = [""]
        for part in parts:
            if not part:
                continue
            if part.startswith("["):
                choices: List[str] = []
                for rng in part[1:-1].split(","):
                    m = _RANGE.match(rng.strip())
                    if not m:
                        raise ValueError(f"bad range {rng!r} in nodelist {nodelist!r}")
                    lo, hi = m.group(1), m.group(2)
                    if hi is None:
                        choices.append(lo)
                    else:
                        width = len(lo)
                        for v in range(int(lo), int(hi) + 1):
                            choices.append(str(v).zfill(width))
                expansions = [e + c for e in expansions for c in choices]
            else:
                expansions = [e + part for e in expansions]
        hosts.extend(expansions)
    return hosts


def _first_int(s: str) -> int:
    """``SLURM_TASKS_PER_NODE`` looks like ``8(x2),4``: the first count."""
    m = re.match(r"(\d+)", s)
    if not m:
        raise ValueError(f"cannot parse task count {s!r}")
    return int(m.group(1))


def slurm_master_port(job_id: Optional[str], base: int = 20000, span: int = 20000) -> int:
    """Job-unique rendezvous port (the reference hard-codes 12345)."""
    if not job_id:
        return DEFAULT_PORT
    digits = re.sub(r"\D", "", job_id) or "0"
    return base + int(digits) % span


def hostname() -> str:
    """This node's name for same-host decisions (IPC mailboxes only work within one node).
    ``DGT_HOSTNAME`` overrides it: the fake-SLURM multi-node tests run every "node" on one machine."""
    return os.environ.get("DGT_HOSTNAME") or socket.gethostname()


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


# --------------------------------------------------------------------------- resolver
def resolve_rank_info(env: Optional[Mapping[str, str]] = None) -> RankInfo:
    env = os.environ if env is None else env

    if "RANK" in env and "WORLD_SIZE" in env:
        ws = int(env["WORLD_SIZE"])
        rank = int(env["RANK"])
        local_rank = int(env.get("LOCAL_RANK", rank))
        lws = int(env.get("LOCAL_WORLD_SIZE", ws))
        node_rank = int(env.get("GROUP_RANK", env.get("NODE_RANK", rank // max(lws, 1))))
        return RankInfo(rank, local_rank, ws, lws, node_rank,
                        env.get("MASTER_ADDR", "127.0.0.1"),
                        int(env.get("MASTER_PORT", DEFAULT_PORT)), "torchrun")

    if "SLURM_PROCID" in env and "SLURM_NTASKS" in env:
        ws = int(env["SLURM_NTASKS"])
        rank = int(env["SLURM_PROCID"])
        local_rank = int(env.get("SLURM_LOCALID", 0))
        if "SLURM_NTASKS_PER_NODE" in env:
            lws = _first_int(env["SLURM_NTASKS_PER_NODE"])
        elif "SLURM_TASKS_PER_NODE" in env:
            lws = _first_int(env["SLURM_TASKS_PER_NODE"])
        else:
            lws = ws
        node_rank = int(env.get("SLURM_NODEID", rank // max(lws, 1)))
        nodelist = env.get("SLURM_JOB_NODELIST") or env.get("SLURM_NODELIST") or "127.0.0.1"
        master = env.get("MASTER_ADDR") or expand_nodelist(nodelist)[0]
        port = int(env["MASTER_PORT"]) if "MASTER_PORT" in env else slurm_master_port(
            env.get("SLURM_JOB_ID") or env.get("SLURM_JOBID"))
        return RankInfo(rank, local_rank, ws, lws, node_rank, master, port, "slurm")

    # mpirun-launched ranks (DeepSpeed's init_distributed falls back to MPI discovery when the
    # torchrun variables are missing): Open MPI, then MPICH / Intel MPI (PMI).  The
    # rendezvous address comes from MASTER_ADDR / MASTER_PORT (exported to every rank, e.g.
    # `mpirun -x MASTER_ADDR -x MASTER_PORT`); no mpi4py needed.
    mpi = None
    if "OMPI_COMM_WORLD_RANK" in env and "OMPI_COMM_WORLD_SIZE" in env:
        mpi = ("OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK",
               "OMPI_COMM_WORLD_LOCAL_SIZE")
    elif "PMI_RANK" in env and "PMI_SIZE" in env:
        mpi = ("PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID", "MPI_LOCALNRANKS")
    if mpi is not None:
        rank, ws = int(env[mpi[0]]), int(env[mpi[1]])
        local_rank = int(env.get(mpi[2], rank))
        lws = int(env.get(mpi[3], ws))
        return RankInfo(rank, local_rank, ws, lws, rank // max(lws, 1), env.get("MASTER_ADDR", "127.0.0.1"),
                        int(env.get("MASTER_PORT", DEFAULT_PORT)), "mpi")

    return RankInfo(0, int(env.get("LOCAL_RANK", 0)), 1, 1, 0,
                    env.get("MASTER_ADDR", "127.0.0.1"),
                    int(env["MASTER_PORT"]) if "MASTER_PORT" in env else 0, "bare")
