#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV outputs: mean counter value per (kernel, counter) over dispatches.

    python scripts/pmc_summary.py gpurun_out/pmcg_0_* [--match SUBSTR]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    vals = defaultdict(list)
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name", "")
                if a.match and a.match not in name:
                    continue
                vals[(name[:70], r["Counter_Name"])].append(float(r["Counter_Value"]))
    kern = sorted({k for k, _ in vals})
    for k in kern:
        print(k)
        for (kk, c), v in sorted(vals.items()):
            if kk == k:
                print(f"  {c:34s} {sum(v) / len(v):16.1f}   (n={len(v)})")


if __name__ == "__main__":
    main()
