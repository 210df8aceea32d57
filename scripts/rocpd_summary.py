#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (``<name>_results.db``) as text for ``profiles/``.

    python scripts/rocpd_summary.py DB [--timeline START:COUNT] [--match SUBSTR]

Prints the per-kernel stats (calls, total / mean us, share), kernel counts per HIP stream, and an
optional excerpt of the dispatch timeline (start offset, duration, stream, name) to show how kernels
of different streams interleave.
"""
import argparse
import sqlite3


def short(name: str, n: int = 90) -> str:
    name = name.replace("void ", "")
    return name if len(name) <= n else name[: n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--timeline", default=None, help="START:COUNT dispatches to list")
    ap.add_argument("--match", default=None, help="start the timeline at the first kernel whose name contains this")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, stream, start, end from kernels order by start"))
    if not rows:
        print("no kernel dispatches")
        return
    t_first = rows[0][2]
    total = sum(r[3] - r[2] for r in rows)
    stats = {}
    for name, _, s, e in rows:
        d = stats.setdefault(name, [0, 0])
        d[0] += 1
        d[1] += e - s
    print(f"{len(rows)} dispatches, {total / 1e3:.1f} us of kernel time, {len(stats)} kernels")
    print(f"{'calls':>6} {'total us':>10} {'mean us':>8} {'share':>6}  kernel")
    for name, (n, t) in sorted(stats.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{n:6d} {t / 1e3:10.1f} {t / n / 1e3:8.2f} {100 * t / total:5.1f}%  {short(name)}")
    print("\nkernels per stream:")
    per = {}
    for name, stream, _, _ in rows:
        per.setdefault(stream, {}).setdefault(short(name, 50), 0)
        per[stream][short(name, 50)] += 1
    for stream, kinds in sorted(per.items()):
        top = sorted(kinds.items(), key=lambda kv: -kv[1])[:4]
        print(f"  {stream:16s} {sum(kinds.values()):6d}  " + ", ".join(f"{k} x{v}" for k, v in top))
    if a.timeline:
        start, count = (int(x) for x in a.timeline.split(":"))
        if a.match:
            hits = [i for i, r in enumerate(rows) if a.match in r[0]]
            start = (hits[0] if hits else 0) + start
        print(f"\ntimeline (dispatches {start}..{start + count - 1}):")
        print(f"{'t0 us':>10} {'dur us':>8}  {'stream':16s} kernel")
        for name, stream, s, e in rows[start:start + count]:
            print(f"{(s - t_first) / 1e3:10.1f} {(e - s) / 1e3:8.2f}  {stream:16s} {short(name, 70)}")


if __name__ == "__main__":
    main()
