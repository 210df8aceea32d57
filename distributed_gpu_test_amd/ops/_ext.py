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


_FAST = None


def fast():
    """The hot eager-path ops (gather_rows, bce_logits, linear_fwd / linear_bwd, linear2_fwd /
    linear2_bwd, adam_flat) as plain pybind11 functions of the same library
    (``csrc/bindings.cpp`` PYBIND11_MODULE): same C++ code and arguments as ``torch.ops.dgt``, without
    the boxed dispatcher's per-call cost.  Positional arguments only."""
    global _FAST
    if _FAST is None:
        require()
        import importlib.util
        spec = importlib.util.spec_from_file_location("distributed_gpu_test_amd._C", LIB_PATH)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _FAST = mod
    return _FAST


class _Hot:
    """``torch.ops.dgt`` with the :func:`fast` functions in place of their dispatcher entries."""

    def __init__(self, fast_mod, ops):
        self._ops = ops
        for name in dir(fast_mod):
            if not name.startswith("_"):
                setattr(self, name, getattr(fast_mod, name))

    def __getattr__(self, name):  # any other op: the dispatcher's, cached on first use
        op = getattr(self._ops, name)
        setattr(self, name, op)
        return op


_HOT = None


def hot():
    """The op namespace of the hot eager paths: :func:`fast` entries where they exist, else
    ``torch.ops.dgt`` (raises like :func:`require` when the extension is missing)."""
    global _HOT
    if _HOT is None:
        _HOT = _Hot(fast(), require())
    return _HOT


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
