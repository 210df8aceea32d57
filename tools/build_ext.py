#!/usr/bin/env python3
"""Build the native extension IN-TREE for gfx950 (MI355X).

* ``csrc/*.hip``  -> hipcc --offload-arch=gfx950 -O3 (device + launch code; no torch headers)
* ``csrc/bindings.cpp`` -> hipcc host compile against the installed torch headers
* link -> ``distributed_gpu_test_amd/_C.so`` (loaded with ``torch.ops.load_library``)
* ``csrc/tools/*.cpp`` -> standalone native tools under ``build/bin`` (RCCL bus-bandwidth sweep)

Incremental: an object is rebuilt only when its source or any ``csrc/*.h`` is newer.  hipcc
cross-compiles gfx950 code objects without a GPU, so this runs in the CPU container.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "obj")
BIN = os.path.join(ROOT, "build", "bin")
OUT = os.path.join(ROOT, "distributed_gpu_test_amd", "_C.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
ROCM = os.environ.get("ROCM_HOME", "/opt/rocm")
HIPCC = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")


def _torch_paths():
    import torch
    from torch.utils import cpp_extension
    inc = cpp_extension.include_paths(device_type="cuda")
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


# the fused tiny kernel reads every MFMA result straight back into VALU math: accumulators in
# VGPRs save the v_accvgpr_read round trips (the GEMMs keep the compiler's AGPR choice)
# The exact-fp32 GEMM's loop-carried accumulators: in the default AGPR form the register allocator
# rotates them through v_accvgpr moves at every loop back-edge (96-190 moves per 128-512 MFMAs);
# in VGPR form the loops hold MFMAs, loads and address arithmetic only
_F32_GEMM = ["-mllvm", "-amdgpu-mfma-vgpr-form"]
PER_FILE_FLAGS = {"tiny_mlp.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form", "-mllvm", "-amdgpu-sched-strategy=max-ilp"],
                  **{f"gemm_f32_l{a}{b}.hip": _F32_GEMM for a in "01" for b in "01"}}


def build(verbose: bool = False, force: bool = False, jobs: int = 8, variant: str = "", defines=(),
          file_flags=()) -> str:
    """``variant``: an A/B build of the whole extension with extra ``defines`` (-D) and per-source
    ``file_flags`` ("tiny_mlp.hip=-fno-slp-vectorize") into build/variants/<variant>/_C.so (load it
    with DGT_EXT_LIB=<path>); the default build is untouched."""
    global BUILD, OUT
    if variant:
        BUILD = os.path.join(ROOT, "build", "variants", variant, "obj")
        OUT = os.path.join(ROOT, "build", "variants", variant, "_C.so")
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(BIN, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    common = ["-O3", "-std=c++17", "-fPIC", f"-I{CSRC}", "-Wno-unused-result", *[f"-D{d}" for d in defines]]
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    extra = {}
    for ff in file_flags:
        name, flag = ff.split("=", 1)
        extra.setdefault(name, []).append(flag)
    inc, tlib, abi = _torch_paths()
    jobs_list = []
    objs = []
    for src in hip_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            jobs_list.append([HIPCC, f"--offload-arch={ARCH}", *common, *PER_FILE_FLAGS.get(os.path.basename(src), []),
                              *extra.get(os.path.basename(src), []), "-c", src, "-o", obj])
    # host translation units against the torch headers (op bindings, RCCL communicator)
    for bsrc in sorted(glob.glob(os.path.join(CSRC, "*.cpp"))):
        bobj = os.path.join(BUILD, os.path.basename(bsrc) + ".o")
        objs.append(bobj)
        if force or _newer(bobj, [bsrc] + headers):
            jobs_list.append([HIPCC, *common, f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1",
                              *[f"-I{p}" for p in inc], f"-I{sysconfig.get_paths()['include']}",
                              "-c", bsrc, "-o", bobj])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs_list))
    if force or jobs_list or _newer(OUT, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", OUT,
              f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch", "-ltorch_python", "-lrccl",
              f"-Wl,-rpath,{tlib}"], verbose)

    # standalone native tools (no torch): link straight against ROCm's HIP + RCCL
    for src in sorted(glob.glob(os.path.join(CSRC, "tools", "*.cpp"))):
        exe = os.path.join(BIN, os.path.splitext(os.path.basename(src))[0])
        if force or _newer(exe, [src] + headers):
            _run([HIPCC, f"--offload-arch={ARCH}", *common, src, "-o", exe,
                  f"-L{ROCM}/lib", "-lrccl", f"-Wl,-rpath,{ROCM}/lib"], verbose)
    return OUT


# host-side AddressSanitizer + UBSan builds of the standalone tools.  Only the host
# compile is instrumented: each -fsanitize= directly follows -Xarch_host (GPU ASan needs xnack+
# code objects, which this pool does not run).  Run them with
# ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0 (the HIP runtime keeps its allocations to exit).
SANITIZE = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
            "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-fno-sanitize-recover=undefined"]


def build_sanitized(verbose: bool = False, force: bool = False) -> list:
    os.makedirs(BIN, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    out = []
    for src in sorted(glob.glob(os.path.join(CSRC, "tools", "*.cpp"))):
        exe = os.path.join(BIN, os.path.splitext(os.path.basename(src))[0] + "_asan")
        if force or _newer(exe, [src] + headers):
            _run([HIPCC, f"--offload-arch={ARCH}", "-O1", "-g", "-std=c++17", f"-I{CSRC}", *SANITIZE, src,
                  "-o", exe, f"-L{ROCM}/lib", "-lrccl", f"-Wl,-rpath,{ROCM}/lib"], verbose)
        out.append(exe)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-f", "--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=8)
    ap.add_argument("--sanitize", action="store_true",
                    help="also build host-ASan/UBSan copies of the standalone tools (build/bin/*_asan)")
    ap.add_argument("--variant", default="", help="A/B build into build/variants/<name>/_C.so")
    ap.add_argument("-D", "--define", action="append", default=[], help="extra preprocessor define (variants)")
    ap.add_argument("--file-flag", action="append", default=[], help="FILE=FLAG: extra flag for one source (variants)")
    a = ap.parse_args(argv)
    out = build(verbose=a.verbose, force=a.force, jobs=a.jobs, variant=a.variant, defines=a.define,
                file_flags=a.file_flag)
    print(f"built {out}")
    if a.sanitize:
        for exe in build_sanitized(verbose=a.verbose, force=a.force):
            print(f"built {exe}")


if __name__ == "__main__":
    sys.exit(main())
