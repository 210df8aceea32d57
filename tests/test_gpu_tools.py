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


ASAN_TOOL = TOOL + "_asan"
ASAN_ENV = {"ASAN_OPTIONS": "detect_leaks=0:verify_asan_link_order=0:halt_on_error=1",
            "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}


@pytest.mark.parametrize("op", ["all_reduce", "reduce_scatter", "all_gather", "broadcast", "alltoall"])
def test_rccl_perf_host_asan_clean(op):
    """The host-AddressSanitizer + UBSan build of the tool (tools/build_ext.py --sanitize: only the
    host compile is instrumented) runs every collective with result checking and reports nothing."""
    if not os.path.exists(ASAN_TOOL):
        pytest.fail(f"{ASAN_TOOL} missing: run tools/build_ext.py --sanitize")
    r = subprocess.run([ASAN_TOOL, "-o", op, "-g", "1", "-b", "1024", "-e", "262144", "-f", "4", "-n", "3", "-w", "1",
                        "-c", "1", "-j"], capture_output=True, text=True, timeout=120, env={**os.environ, **ASAN_ENV})
    assert r.returncode == 0, r.stderr[-3000:]
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    rows = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert len(rows) == 5 and all(row.get("wrong", 0) == 0 for row in rows), r.stdout[-2000:]
