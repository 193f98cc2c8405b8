"""ctypes bindings to the in-tree native libraries (``lib/libh2o_hip.so`` and ``lib/libh2o_rt.so``).

GPU ops never fall back silently: if a CUDA(HIP) tensor reaches an op and the HIP library cannot be
loaded, :func:`hip` raises. CPU tensors take the PyTorch reference path of each op (used by the CPU
test-suite and as the numerics oracle for the kernels).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be imported first: shares torch's libamdhip64.so.7)

from .. import build_native

_lock = threading.Lock()
_hip = None
_rt = None

c_int, c_ll, c_ull, c_double, c_void_p = ctypes.c_int, ctypes.c_longlong, ctypes.c_ulonglong, ctypes.c_double, ctypes.c_void_p

_HIP_SIGS = {
    "h2o_tree_sizes": [c_void_p],
    "h2o_tree_plan_size": [],
    "h2o_tree_root": [c_void_p, c_void_p],
    "h2o_tree_level": [c_void_p, c_int, c_int, c_void_p],
    "h2o_tree_find": [c_void_p, c_int, c_void_p],
    "h2o_tree_grow": [c_void_p, c_int, c_int, c_void_p],
    "h2o_hist_pack": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p],
    "h2o_tree_dist": [c_void_p, c_void_p],
    "h2o_rccl_load": [ctypes.c_char_p],
    "h2o_rccl_version": [],
    "h2o_rccl_unique_id": [c_void_p],
    "h2o_rccl_id_bytes": [],
    "h2o_rccl_init": [c_void_p, c_int, c_void_p, c_int],
    "h2o_rccl_destroy": [c_void_p, c_int],
    "h2o_rccl_coll": [c_void_p, c_int, c_void_p, c_void_p, c_ll, c_int, c_void_p],
    "h2o_tree_all": [c_void_p, c_void_p],
    "h2o_tree_leaves": [c_void_p, c_void_p],
    "h2o_hist_build": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p,
                       c_int, c_int, c_void_p, c_void_p, c_int, c_ll, c_int, c_void_p, c_void_p, c_int, c_void_p,
                       c_void_p],
    "h2o_split_find": [c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_double, c_double,
                       c_double, c_double, c_double, c_int, c_int, c_ull, c_int, c_void_p, c_void_p, c_void_p, c_int,
                       c_int, c_int, c_int, c_void_p],
    "h2o_split_reduce": [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_ull, c_int, c_void_p, c_void_p, c_void_p,
                         c_int, c_void_p],
    "h2o_ic_next": [c_void_p] * 6 + [c_int, c_void_p, c_int, c_void_p],
    "h2o_plan": [c_void_p] * 14 + [c_int, c_int, c_double, c_int, c_int, c_void_p],
    "h2o_ranges": [c_void_p] * 6,
    "h2o_zero_hist": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "h2o_route": [c_void_p] * 6 + [c_int] + [c_void_p] * 10 + [c_int, c_ll, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "h2o_leaf_assign": [c_void_p, c_int, c_ll, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                        c_void_p, c_int, c_int, c_void_p],
    "h2o_bin_assign": [c_void_p, c_ll, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                       c_void_p],
    "h2o_amax": [c_void_p, c_ll, c_void_p, c_void_p],
    "h2o_kmeans_mfma_shape": [c_int, c_int, c_void_p],
    "h2o_kmeans_mfma_grid": [c_int, c_int],
    "h2o_kmeans_mfma": [c_void_p, c_ll, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    "h2o_kmeans_update": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "h2o_qscale": [c_void_p, c_void_p, c_void_p, c_ll, c_int, c_void_p],
    "h2o_score_hist": [c_void_p, c_void_p, c_void_p, c_ll, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "h2o_snap_copy": [c_void_p, c_void_p, c_ll, c_void_p],
    "h2o_fine16_build": [c_void_p, c_int, c_ll, c_void_p, c_int, c_void_p, c_void_p],
    "h2o_host_dev_ptr": [c_void_p, c_void_p],
    "h2o_hist_reduce": [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                        c_void_p, c_int, c_int, c_int, c_int, c_void_p],
    "h2o_leaf_values": [c_void_p, c_int, c_int, c_double, c_double, c_double, c_double, c_double, c_void_p, c_void_p],
    "h2o_gbm_step": [c_ll, c_ll, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_float, c_ull,
                     ctypes.c_float, c_void_p, c_void_p, c_int, c_void_p],
    "h2o_add_leaf": [c_ll, c_void_p, c_int, c_void_p, c_void_p, c_void_p],
    "h2o_predict": [c_void_p, c_ll, c_int] + [c_void_p] * 11 + [c_int, c_void_p, c_void_p, c_void_p],
}


# Bumped whenever a C launcher's argument list changes; every native library exports h2o_abi_version()
# (csrc/abi.h) and a library built from older sources is refused instead of being called with shifted
# arguments.
ABI_VERSION = 14


def _check_abi(lib, name: str) -> None:
    fn = getattr(lib, "h2o_abi_version", None)
    got = fn() if fn is not None else -1
    if got != ABI_VERSION:
        raise RuntimeError(f"{name}: native ABI version {got} != expected {ABI_VERSION}; rebuild with "
                           "`python -m llama_github_io_amd.build_native --force`")


def _bind(lib, sigs):
    for name, args in sigs.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = c_int
    return lib


def register_hip_signatures(sigs: dict) -> None:
    """Let other op modules declare their launchers' argtypes."""
    _HIP_SIGS.update(sigs)
    if _hip is not None:
        _bind(_hip, sigs)


def hip():
    """Load (building first if needed) the HIP kernel library. Raises if unavailable."""
    global _hip
    if _hip is None:
        with _lock:
            if _hip is None:
                # build_hip() is a no-op when the library is newer than every source; a stale library
                # (launcher signatures changed since it was built) is rebuilt instead of being loaded
                # H2O_HIP_LIB: an alternative build of the same sources (A/B runs of compile-time kernel variants)
                path = os.environ.get("H2O_HIP_LIB") or build_native.build_hip(
                    force=bool(os.environ.get("H2O_AMD_REBUILD")))
                lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
                _check_abi(lib, "libh2o_hip")
                _hip = _bind(lib, _HIP_SIGS)
    return _hip


def rt():
    """Load (building first if needed) the host runtime library."""
    global _rt
    if _rt is None:
        with _lock:
            if _rt is None:
                path = build_native.build_rt()
                lib = ctypes.CDLL(path)
                _check_abi(lib, "libh2o_rt")
                _rt = lib
    return _rt


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def check(rc: int, name: str) -> None:
    if rc != 0:
        raise RuntimeError(f"HIP launch {name} failed with hipError {rc}")


def call(name: str, *args) -> None:
    rc = getattr(hip(), name)(*args)
    check(rc, name)
