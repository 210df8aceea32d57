#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; KB per dispatch)
joined with the kernel trace's durations: mean MB fetched / written per dispatch, mean us, GB/s.

    python scripts/hbm_summary.py gpurun_out/r6hbm
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    kb = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        for f in glob.glob(os.path.join(root, c, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                kb[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for f in glob.glob(os.path.join(root, c, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for k, v in kb.items():
        fe = sum(v.get("FETCH_SIZE", [0])) / max(1, len(v.get("FETCH_SIZE", [])))
        wr = sum(v.get("WRITE_SIZE", [0])) / max(1, len(v.get("WRITE_SIZE", [])))
        d = sorted(dur.get(k, [0.0]))
        us = d[len(d) // 2]
        rows.append((us * len(v.get("FETCH_SIZE", [])), k, fe / 1024, wr / 1024, us))
    print("# kernel | fetched MB / dispatch | written MB / dispatch | median us (counter runs) | TB/s")
    print("# (FETCH_SIZE as rocprofv3 derives it: on gfx950 it read ~half the flat Adam's expected 0.94 GB")
    print("#  -- treat the fetch column as a lower bound)")
    for _, k, fe, wr, us in sorted(rows, reverse=True)[:14]:
        tbs = (fe + wr) * 1e6 / (us * 1e-6) / 1e12 if us else 0.0
        print(f"{k[:70]:70s} | {fe:9.1f} | {wr:9.1f} | {us:8.1f} | {tbs:6.2f}")


if __name__ == "__main__":
    main()
