"""Builds the HIP engine (lib/libsdr.so) for gfx950 in-tree with hipcc.

The shared library is the product: a C ABI (include/sdr/sdr.h) over hand-written CDNA4 kernels.
It is built here (cross-compiled, no GPU needed) and travels to the GPU box with the snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "lib", "libsdr.so")
SOURCES = ["sdr_cost.hip", "sdr_paths.hip", "sdr_post.hip", "sdr_engine.hip"]
HEADERS = ["sdr_device.hpp", "sdr_internal.hpp"]
ARCH = os.environ.get("SDR_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build the engine)")


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(ROOT, "include", "sdr", "sdr.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build_native(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-Wno-unused-result",
           "-I", os.path.join(ROOT, "include")]
    cmd += [os.path.join(CSRC, f) for f in SOURCES]
    cmd += ["-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build_native(force=True, verbose=True))
