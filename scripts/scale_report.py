#!/usr/bin/env python3
"""Scaling table from the driver's records: BENCH_rNN.json (N = 1) and SCALE_rNN.json (N = 1/2/4/8).

    python scripts/scale_report.py [SCALE_r02.json] [BENCH_r02.json]

Prints, per N: the bench's aggregate value (iters/s summed over ranks), per-GPU value, weak-scaling
efficiency against N = 1 (value_N / (N x value_1)), ms per step, the exchange the run used and the
all-reduce bus bandwidth.  Records the driver marks as skipped or failed are reported as such.
"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _latest(pattern):
    files = sorted(glob.glob(os.path.join(ROOT, pattern)))
    return files[-1] if files else None


def _bench_line(run):
    """The bench's JSON line out of one driver run record (stdout tail)."""
    out = (run or {}).get("stdout_tail", "") if isinstance(run, dict) else ""
    lines = [line for line in out.splitlines() if line.startswith("{") and '"metric"' in line]
    return json.loads(lines[-1]) if lines else None


def rows_from(record):
    """(n, bench dict or None, note) triples from a driver BENCH/SCALE record."""
    if not isinstance(record, dict):
        return []
    if record.get("skipped"):
        return [(None, None, f"skipped: {record.get('reason', '')}")]
    runs = record.get("runs") or record.get("results")
    if isinstance(runs, list):
        out = []
        for r in runs:
            out.append((r.get("n"), _bench_line(r.get("run", r)), r.get("run", r).get("status", "")))
        return out
    if "n" in record:
        return [(record["n"], _bench_line(record.get("run")), record.get("run", {}).get("status", ""))]
    return []


def main(argv):
    scale = argv[1] if len(argv) > 1 else _latest("SCALE_r*.json")
    bench = argv[2] if len(argv) > 2 else _latest("BENCH_r*.json")
    rows = []
    for path in (bench, scale):
        if path and os.path.exists(path):
            rows += [(os.path.basename(path),) + r for r in rows_from(json.load(open(path)))]
    base = next((b["value"] for _, n, b, _ in rows if n == 1 and b), None)
    print(f"{'record':18s} {'N':>2s} {'iters/s':>12s} {'per GPU':>10s} {'eff':>6s} {'ms/step':>9s}  exchange / busbw / note")
    for src, n, b, note in rows:
        if b is None:
            print(f"{src:18s} {str(n or '-'):>2s} {'-':>12s} {'-':>10s} {'-':>6s} {'-':>9s}  {note}")
            continue
        eff = b["value"] / (n * base) if base and n else None
        cfg = b.get("config", {})
        print(f"{src:18s} {n:>2d} {b['value']:>12,.0f} {b['value'] / n:>10,.0f} "
              f"{'' if eff is None else f'{eff:.2f}':>6s} {b['ms_per_step']:>9.5f}  "
              f"{cfg.get('exchange', '')} / {b.get('allreduce_busbw_GBps')} GB/s / n_gpus={b.get('n_gpus')}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
