"""Host cost per launch in this process: a tiny kernel (x.add_(1)) launched directly, the same op
replayed from a one-node HIP graph, each on the default stream and on a created stream; median
of 5 batches of 2000 launches.  Run it in several fresh processes to see whether the process-to-
process spread of the engine's graph_module loop is in graph launches or in all host work.

    python scripts/graph_launch_probe.py [--cpu N]
"""
import os
import statistics
import sys
import time

if "--cpu" in sys.argv:  # pin before the HIP runtime starts its threads (they inherit the mask)
    os.sched_setaffinity(0, {int(sys.argv[sys.argv.index("--cpu") + 1])})

import torch  # noqa: E402


def per_launch_us(fn, n=2000, batches=5):
    out = []
    for _ in range(batches):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        out.append((time.perf_counter() - t) / n * 1e6)
        torch.cuda.synchronize()
    return statistics.median(out)


def drain_split(fn, n=2000):
    """(host us per launch over the first 32 launches after an idle sync, host us per launch over n,
    wall us per launch over n including the GPU's drain): back-pressure from a full queue shows as
    host cost that tracks the device's time per launch."""
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(32):
        fn()
    first = (time.perf_counter() - t) / 32 * 1e6
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    host = (time.perf_counter() - t) / n * 1e6
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / n * 1e6
    return first, host, wall


def main():
    x = torch.zeros(16, device="cuda")
    res = {}
    for sname, stream in (("default", None), ("side", torch.cuda.Stream())):
        ctx = torch.cuda.stream(stream) if stream is not None else torch.cuda.stream(torch.cuda.current_stream())
        with ctx:
            for _ in range(100):
                x.add_(1)
            res[f"kernel_{sname}"] = per_launch_us(lambda: x.add_(1))
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                x.add_(1)
                g.capture_begin()
                x.add_(1)
                g.capture_end()
            torch.cuda.current_stream().wait_stream(s)
            replay = torch._C._CUDAGraph.replay.__get__(g)
            for _ in range(100):
                replay()
            res[f"graph_{sname}"] = per_launch_us(replay)
            if sname == "default":
                res["graph_first32"], res["graph_host"], res["graph_wall"] = drain_split(replay)
                res["kern_first32"], res["kern_host"], res["kern_wall"] = drain_split(lambda: x.add_(1))
            t = time.perf_counter()
            for _ in range(20000):
                pass
            res["py_loop_20k_us"] = round((time.perf_counter() - t) * 1e6, 1)
    cpus = sorted(os.sched_getaffinity(0))
    res["cpu"] = cpus[0] if len(cpus) == 1 else -1
    print("[launch-probe] " + " ".join(f"{k}={v:.2f}" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
