"""Host-side sanitizers on CPU: the standalone native tool built with AddressSanitizer +
UBSan on its host code (``tools/build_ext.py --sanitize``), exercised on its argument-parsing and
error paths, which need no GPU.  The GPU run of the same binary is in tests/test_gpu_tools.py."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = {"ASAN_OPTIONS": "detect_leaks=0:verify_asan_link_order=0:halt_on_error=1",
       "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}


@pytest.fixture(scope="module")
def asan_tool():
    if not (shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc")):
        pytest.skip("hipcc not available")
    sys.path.insert(0, ROOT)
    from tools.build_ext import build_sanitized
    exes = build_sanitized()
    exe = [e for e in exes if os.path.basename(e) == "rccl_perf_asan"]
    assert exe and os.access(exe[0], os.X_OK)
    return exe[0]


@pytest.mark.parametrize("args,needle", [(["-x"], "unknown option"), (["-b"], "missing value")])
def test_asan_tool_error_paths_are_clean(asan_tool, args, needle):
    r = subprocess.run([asan_tool, *args], capture_output=True, text=True, timeout=60, env={**os.environ, **ENV})
    assert r.returncode == 1, (r.returncode, r.stderr[-2000:])
    assert needle in r.stderr
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def test_asan_runtime_is_linked(asan_tool):
    out = subprocess.run(["nm", asan_tool], capture_output=True, text=True).stdout
    assert "__asan_init" in out and "__ubsan_handle" in out
