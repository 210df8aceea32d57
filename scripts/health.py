#!/usr/bin/env python3
"""Node health report for the acceptance test.

The reference's acceptance signal is only "the job ran".  This report records what a cluster
operator needs next to that: GPUs and their state (rocm-smi / amd-smi), the xGMI topology, the
ROCm / PyTorch / RCCL versions, and an RCCL bus-bandwidth sweep across the node's GPUs
(``build/bin/rccl_perf``, the rccl-tests equivalent built from ``csrc/tools``).

    python scripts/health.py [--out-dir logs] [--tag job123] [--no-bw] [--strict]

Writes ``<out-dir>/health_<tag>_node<N>.json`` (N = SLURM_PROCID / NODE_RANK / GROUP_RANK / 0) and
prints a short summary.  Missing tools are reported, not fatal; ``--strict`` exits 1 when no GPU is
visible or the bandwidth check reports wrong results.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd, timeout=60):
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
        return {"cmd": " ".join(cmd), "rc": r.returncode, "stdout": r.stdout[-20000:], "stderr": r.stderr[-4000:]}
    except FileNotFoundError:
        return {"cmd": " ".join(cmd), "rc": None, "error": "not found"}
    except subprocess.TimeoutExpired:
        return {"cmd": " ".join(cmd), "rc": None, "error": "timeout"}


def _tool(name):
    p = shutil.which(name) or os.path.join("/opt/rocm/bin", name)
    return p if os.path.exists(p) else None


def gpu_inventory():
    info = {}
    try:
        import torch
        info["torch"] = torch.__version__
        info["hip"] = getattr(torch.version, "hip", None)
        info["gpu_count"] = torch.cuda.device_count()
        if torch.cuda.is_available():
            info["devices"] = []
            for i in range(torch.cuda.device_count()):
                p = torch.cuda.get_device_properties(i)
                info["devices"].append({"index": i, "name": p.name, "arch": getattr(p, "gcnArchName", None),
                                        "total_memory_GB": round(p.total_memory / 2**30, 1),
                                        "multi_processor_count": p.multi_processor_count})
            # GPU-to-GPU access (the fused trainer's IPC mailboxes need it between every pair of
            # a node's GPUs; without it the exchange falls back to RCCL)
            n = torch.cuda.device_count()
            info["peer_access"] = [[i == j or bool(torch.cuda.can_device_access_peer(i, j)) for j in range(n)]
                                   for i in range(n)]
            info["peer_access_all"] = all(all(r) for r in info["peer_access"])
            try:
                info["rccl_version"] = ".".join(str(v) for v in torch.cuda.nccl.version())
            except Exception as e:  # pragma: no cover
                info["rccl_version"] = f"unavailable: {e}"
    except Exception as e:  # pragma: no cover
        info["error"] = str(e)
    return info


def smi_reports():
    out = {}
    smi = _tool("rocm-smi")
    if smi:
        out["rocm_smi"] = _run([smi, "--showuse", "--showmemuse", "--showtemp", "--showpower", "--json"])
        out["rocm_smi_topology"] = _run([smi, "--showtopo"])
    amd = _tool("amd-smi")
    if amd:
        out["amd_smi_metric"] = _run([amd, "metric", "--json"], timeout=120)
        out["amd_smi_xgmi"] = _run([amd, "xgmi"], timeout=60)
    return out


def rccl_perf_path():
    """The rccl-tests equivalent built next to this script (``<DGT_HOME>/build/bin/rccl_perf``)."""
    exe = os.path.join(ROOT, "build", "bin", "rccl_perf")
    return exe if os.access(exe, os.X_OK) else None


def framework_info():
    """Where the framework and its native pieces were found (catches an image whose install was
    hidden by a mount: the SLURM job must run the IMAGE's code, slurm_train.sbatch)."""
    info = {"dgt_home": ROOT, "rccl_perf": rccl_perf_path()}
    try:
        sys.path.insert(0, ROOT)
        import distributed_gpu_test_amd as dgt
        from distributed_gpu_test_amd.ops import _ext
        info["package"] = os.path.dirname(dgt.__file__)
        info["extension"] = _ext.LIB_PATH if _ext.available() else None
    except Exception as e:
        info["package"] = None
        info["error"] = f"{type(e).__name__}: {e}"
    return info


def bandwidth_sweep(ngpus: int):
    exe = rccl_perf_path()
    if exe is None or ngpus < 1:
        return {"skipped": "rccl_perf not built or no GPU"}
    res = {}
    for op in ("all_reduce", "reduce_scatter", "all_gather"):
        r = _run([exe, "-o", op, "-b", "8", "-e", str(1 << 30), "-f", "4", "-g", str(ngpus), "-n", "10",
                  "-w", "3", "-j"], timeout=300)
        rows = []
        for line in (r.get("stdout") or "").splitlines():
            if line.startswith("{"):
                rows.append(json.loads(line))
        res[op] = {"rows": rows, "rc": r.get("rc"),
                   "peak_busbw_GBps": max((x["busbw_GBps"] for x in rows), default=None),
                   "wrong": sum(x["wrong"] for x in rows)}
        if r.get("rc") not in (0, None) and r.get("stderr"):
            res[op]["stderr"] = r["stderr"][-2000:]
    return res


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--out-dir", default="logs")
    ap.add_argument("--tag", default=None)
    ap.add_argument("--no-bw", action="store_true")
    ap.add_argument("--strict", action="store_true")
    a = ap.parse_args(argv)
    node = os.environ.get("SLURM_PROCID") or os.environ.get("NODE_RANK") or os.environ.get("GROUP_RANK") or "0"
    tag = a.tag or time.strftime("%Y%m%d-%H%M%S")
    t0 = time.time()
    rep = {"host": socket.gethostname(), "node": int(node), "time": time.time(), "tag": tag,
           "env": {k: os.environ.get(k) for k in ("SLURM_JOB_ID", "SLURM_JOB_NODELIST", "HIP_VISIBLE_DEVICES",
                                                   "HSA_ENABLE_IPC_MODE_LEGACY", "NCCL_DEBUG")}}
    rep["framework"] = framework_info()
    rep["gpu"] = gpu_inventory()
    rep["smi"] = smi_reports()
    n = int(rep["gpu"].get("gpu_count") or 0)
    rep["rccl_bandwidth"] = {"skipped": "--no-bw"} if a.no_bw else bandwidth_sweep(n)
    rep["elapsed_s"] = round(time.time() - t0, 2)
    os.makedirs(a.out_dir, exist_ok=True)
    path = os.path.join(a.out_dir, f"health_{tag}_node{node}.json")
    with open(path, "w") as fh:
        json.dump(rep, fh, indent=1)
    bw = rep["rccl_bandwidth"]
    peak = bw.get("all_reduce", {}).get("peak_busbw_GBps") if isinstance(bw, dict) else None
    print(f"[health] node{node} {rep['host']}: {n} GPU(s) "
          f"{rep['gpu'].get('devices', [{}])[0].get('name', '') if n else ''} RCCL {rep['gpu'].get('rccl_version')} "
          f"all_reduce peak busbw {peak} GB/s, peer access {rep['gpu'].get('peer_access_all')} -> {path}", flush=True)
    wrong = sum(v.get("wrong", 0) for v in bw.values() if isinstance(v, dict)) if isinstance(bw, dict) else 0
    if a.strict and (n == 0 or wrong or not rep["framework"].get("extension")):
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
