"""Native tools on the GPU: the rccl-tests-style bus-bandwidth sweep (``csrc/tools/rccl_perf.cpp``,
built by ``tools/build_ext.py`` into ``build/bin``) on every collective, with result checking."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "build", "bin", "rccl_perf")
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("op", ["all_reduce", "reduce_scatter", "all_gather", "broadcast", "alltoall"])
def test_rccl_perf_sweep_checks_results(op):
    if not os.path.exists(TOOL):
        pytest.fail(f"{TOOL} missing: run tools/build_ext.py")
    r = subprocess.run([TOOL, "-o", op, "-g", "1", "-b", "1024", "-e", "1048576", "-f", "4", "-n", "5", "-w", "2",
                        "-c", "1", "-j"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert len(rows) == 6, r.stdout[-2000:]
    for row in rows:
        assert row.get("wrong", 0) == 0, row
