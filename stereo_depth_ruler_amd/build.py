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
SOURCES = ["sdr_cost.hip", "sdr_cost3.hip", "sdr_cost3k2.hip", "sdr_cost_generic.hip", "sdr_paths.hip", "sdr_post.hip", "sdr_wls.hip", "sdr_rectify.hip",
           "sdr_cloud.hip", "sdr_display.hip", "sdr_engine.hip"]
HEADERS = ["sdr_device.hpp", "sdr_internal.hpp", "sdr_cost_kernel.hpp"]
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


# host-only debug info: device debug info of the unrolled cost kernels takes hipcc tens of minutes
HOST_ASAN = ["-Xarch_host", "-g", "-fno-omit-frame-pointer"] + [x for f in ("-fsanitize=address", "-fsanitize=undefined",
                                                            "-fno-sanitize-recover=undefined")
                                                 for x in ("-Xarch_host", f)]


def build_native(force: bool = False, verbose: bool = False, variant: str = "",
                 defines: tuple = (), extra: tuple = ()) -> str:
    """Compiles each HIP source to an object in parallel (relocatable device code is not needed:
    every kernel is launched from the file that defines it), then links the shared library.
    variant/defines: an experiment build lib/libsdr-<variant>.so with extra -D switches."""
    out = OUT if not variant else os.path.join(os.path.dirname(OUT), f"libsdr-{variant}.so")
    if not variant and not force and not _stale():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    objdir = os.path.join(os.path.dirname(OUT), "obj" + (f"-{variant}" if variant else ""))
    os.makedirs(objdir, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
             "-Wall", "-Wno-unused-function", "-Wno-unused-result",
             "-I", os.path.join(ROOT, "include")] + [f"-D{d}" for d in defines] + list(extra)
    hipcc = _hipcc()
    objs, procs = [], []
    hdr_t = max(os.path.getmtime(d) for d in [os.path.join(CSRC, h) for h in HEADERS] +
                [os.path.join(ROOT, "include", "sdr", "sdr.h")])
    for f in SOURCES:
        obj = os.path.join(objdir, f.replace(".hip", ".o"))
        objs.append(obj)
        # an object newer than its source and every header is reused (same flags: one objdir per variant)
        if not force and os.path.exists(obj) and os.path.getmtime(obj) > max(hdr_t, os.path.getmtime(os.path.join(CSRC, f))):
            continue
        cmd = [hipcc, *flags, "-c", os.path.join(CSRC, f), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((cmd, subprocess.Popen(cmd)))
    failed = [cmd for cmd, p in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    link = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *extra, *objs, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(link))
    subprocess.check_call(link)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    import sys

    # python build.py [variant NAME=V ...]  (-DNAME=V accepted too)
    # python build.py --host-asan  -> lib/libsdr-asan.so, host code under ASan + UBSan (the device
    #                                 code is unchanged: GPU sanitizers are not used on this pool)
    if sys.argv[1:] == ["--host-asan"]:
        print(build_native(force=True, variant="asan", extra=tuple(HOST_ASAN)))
    elif len(sys.argv) > 1:
        defs = tuple(a[2:] if a.startswith("-D") else a for a in sys.argv[2:])
        print(build_native(force=True, variant=sys.argv[1], defines=defs))
    else:
        print(build_native(force=True, verbose=True))
