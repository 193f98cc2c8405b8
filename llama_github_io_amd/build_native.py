"""Build the native libraries of the framework IN-TREE.

* ``lib/libh2o_hip.so``  - every ``csrc/*.hip`` (hand-written CDNA4 kernels, gfx950 only) behind a C ABI.
* ``lib/libh2o_rt.so``   - every ``csrc/*.cpp`` (host runtime: CSV tokenizer/type guesser, ...).

The libraries are loaded with ctypes after ``import torch`` so the HIP runtime torch already mapped
(SONAME ``libamdhip64.so.7``) is shared: kernels launch on torch's streams with torch's device pointers.

Usage: ``python -m llama_github_io_amd.build_native [--force]``.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib")
HIP_LIB = os.path.join(LIB, "libh2o_hip.so")
RT_LIB = os.path.join(LIB, "libh2o_rt.so")
ARCH = os.environ.get("H2O_AMD_ARCH", "gfx950")


def _stale(target: str, sources: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    deps = sources + glob.glob(os.path.join(CSRC, "*.h"))
    return any(os.path.getmtime(s) > t for s in deps)


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the MI355X kernels need ROCm's hipcc")


def build_hip(force: bool = False, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    if not force and not _stale(HIP_LIB, srcs):
        return HIP_LIB
    os.makedirs(LIB, exist_ok=True)
    objs = []
    for s in srcs:
        o = os.path.join(LIB, os.path.basename(s) + ".o")
        if force or _stale(o, [s]):
            cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-c", s, "-o", o,
                   "-I", CSRC, "-Wno-unused-result"]
            if verbose:
                print(" ".join(cmd))
            subprocess.run(cmd, check=True)
        objs.append(o)
    tmp = HIP_LIB + ".tmp"
    subprocess.run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + ["-ldl"], check=True)
    os.replace(tmp, HIP_LIB)
    return HIP_LIB


def build_rt(force: bool = False, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.cpp")))
    if not srcs:
        return ""
    if not force and not _stale(RT_LIB, srcs):
        return RT_LIB
    os.makedirs(LIB, exist_ok=True)
    tmp = RT_LIB + ".tmp"
    cmd = ["g++", "-O3", "-march=x86-64-v2", "-shared", "-fPIC", "-std=c++17", "-pthread", "-I", CSRC, "-o", tmp] + srcs + ["-lcrypto"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, RT_LIB)
    return RT_LIB


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_rt(force, verbose)
    build_hip(force, verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv, verbose=True)
    print("built", HIP_LIB, RT_LIB)
