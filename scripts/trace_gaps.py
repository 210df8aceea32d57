#!/usr/bin/env python3
"""Idle gaps between consecutive kernels in a rocprofv3 --kernel-trace CSV (one queue): how much
of a step's wall time the GPU spends between kernels (launch/dependency bubbles) rather than in
them.  Reports the last N kernels' busy time, wall span and the largest gaps.

    python scripts/trace_gaps.py gpurun_out/prof_mlp/run_kernel_trace.csv [--last 340]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=0, help="only the last N dispatches (steady state)")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    if a.last:
        rows = rows[-a.last:]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
    span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
    gaps = []
    for p, r in zip(rows, rows[1:]):
        gaps.append((int(r["Start_Timestamp"]) - int(p["End_Timestamp"]), p["Kernel_Name"][:50], r["Kernel_Name"][:50]))
    idle = sum(max(g, 0) for g, _, _ in gaps)
    print(f"{len(rows)} kernels: busy {busy / 1e3:.1f} us, span {span / 1e3:.1f} us, idle {idle / 1e3:.1f} us "
          f"({100 * idle / max(span, 1):.1f} %), mean gap {idle / max(len(gaps), 1) / 1e3:.2f} us")
    for g, p, n in sorted(gaps, reverse=True)[:8]:
        print(f"  {g / 1e3:7.2f} us  {p}  ->  {n}")


if __name__ == "__main__":
    main()
