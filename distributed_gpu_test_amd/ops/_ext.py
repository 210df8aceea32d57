"""Loader for the in-tree native extension ``distributed_gpu_test_amd/_C.so``.

The extension registers ``torch.ops.dgt.*`` (HIP kernels for gfx950 + the IPC runtime).  It is
built by ``python tools/build_ext.py`` (or ``__graft_entry__.build()``).  On a machine with a GPU a
missing extension is an error, never a silent fallback: ``require()`` raises.
"""
from __future__ import annotations

import os
import threading

import torch

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# DGT_EXT_LIB: an A/B build of the extension (tools/build_ext.py --variant) instead of the in-tree one
LIB_PATH = os.environ.get("DGT_EXT_LIB") or os.path.join(_PKG, "_C.so")
_lock = threading.Lock()
_loaded = False
_error: Exception | None = None


def load() -> bool:
    """Load the extension if it exists; returns whether ``torch.ops.dgt`` is usable."""
    global _loaded, _error
    with _lock:
        if _loaded:
            return True
        if not os.path.exists(LIB_PATH):
            _error = FileNotFoundError(
                f"native extension not built: {LIB_PATH} missing (run `python tools/build_ext.py`)")
            return False
        try:
            torch.ops.load_library(LIB_PATH)
            _loaded = True
        except Exception as e:  # pragma: no cover - only on a broken build
            _error = e
            return False
        return True


def available() -> bool:
    return load()


_OPS = None  # torch.ops.dgt once loaded: require() sits on every eager op call's path


def require():
    """Return ``torch.ops.dgt``; raise if the extension cannot be loaded."""
    global _OPS
    if _OPS is not None:
        return _OPS
    if not load():
        raise RuntimeError(f"distributed_gpu_test_amd native extension unavailable: {_error}")
    _OPS = torch.ops.dgt
    return _OPS


_clib = None


def c_lib():
    """The same library through ctypes, for the dispatcher-free launch entry points
    (``dgt_tiny_launch``: a launch costs hipLaunchKernel, not a boxed op call)."""
    global _clib
    if _clib is None:
        require()
        import ctypes
        lib = ctypes.CDLL(LIB_PATH)
        i64, i32 = ctypes.c_int64, ctypes.c_int
        lib.dgt_tiny_launch.argtypes = [i64, i64, i64, i32, i32, ctypes.c_longlong, ctypes.c_longlong, i64]
        lib.dgt_tiny_launch.restype = i32
        lib.dgt_tiny_prepare.argtypes = [i64, i64, i64, i32, i32, i64, ctypes.POINTER(i32)]
        lib.dgt_tiny_prepare.restype = i64
        lib.dgt_tiny_prepared_free.argtypes = [i64]
        lib.dgt_tiny_prepared_free.restype = None
        lib.dgt_tiny_launch_prepared.argtypes = [i64, ctypes.c_longlong, ctypes.c_longlong]
        lib.dgt_tiny_launch_prepared.restype = i32
        lib.dgt_tiny_launcher_set_stream.argtypes = [i64, i64]
        lib.dgt_tiny_launcher_set_stream.restype = None
        _clib = lib
    return _clib


def gpu_available() -> bool:
    return torch.cuda.is_available()
