"""Builds the HIP engine (lib/libsdr.so) for gfx950 in-tree with hipcc.

The shared library is the product: a C ABI (include/sdr/sdr.h) over hand-written CDNA4 kernels.
It is built here (cross-compiled, no GPU needed) and travels to the GPU box with the snapshot.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "lib", "libsdr.so")
SOURCES = ["sdr_cost.hip", "sdr_cost3.hip", "sdr_cost3k2.hip", "sdr_cost_generic.hip", "sdr_paths.hip", "sdr_sweep.hip", "sdr_post.hip", "sdr_wls.hip", "sdr_rectify.hip",
           "sdr_cloud.hip", "sdr_display.hip", "sdr_engine.hip"]
HEADERS = ["sdr_device.hpp", "sdr_internal.hpp", "sdr_cost_kernel.hpp"]
ARCH = os.environ.get("SDR_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build the engine)")


def _deps():
    return [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "sdr", "sdr.h")]


def _hash(paths, extra=()) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.relpath(p, ROOT).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    for x in extra:
        h.update(str(x).encode() + b"\0")
    return h.hexdigest()[:16]


def source_hash() -> str:
    """Hash of every source, header and the ABI header the library is built from, and the target
    arch: the library embeds it (sdr_build_id) and a build is stale exactly when it differs."""
    return _hash(_deps(), (ARCH,))


def built_id(path: str = OUT):
    """The build id embedded in a built library, or None."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(b"SDR_BUILD_ID=")
    return data[i + 13:i + 29].decode(errors="replace") if i >= 0 else None


def _stale() -> bool:
    return built_id() != source_hash()


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
    # the build id is the hash of the sources as they are when the compile starts; if any of them
    # changes before the link is done, the library is not a build of either version: fail
    bid = source_hash()
    objdir = os.path.join(os.path.dirname(OUT), "obj" + (f"-{variant}" if variant else ""))
    os.makedirs(objdir, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
             "-Wall", "-Wno-unused-function", "-Wno-unused-result",
             "-I", os.path.join(ROOT, "include")] + [f"-D{d}" for d in defines] + list(extra)
    hipcc = _hipcc()
    objs, procs = [], []
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "sdr", "sdr.h")]
    for f in SOURCES:
        obj = os.path.join(objdir, f.replace(".hip", ".o"))
        objs.append(obj)
        # an object is reused when its recorded hash (source, headers, flags) still matches
        key = _hash([os.path.join(CSRC, f)] + hdrs, flags)
        stamp = obj + ".hash"
        if not force and os.path.exists(obj) and os.path.exists(stamp):
            with open(stamp) as fh:
                if fh.read() == key:
                    continue
        cmd = [hipcc, *flags, "-c", os.path.join(CSRC, f), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((cmd, subprocess.Popen(cmd), stamp, key))
    failed = [cmd for cmd, p, _, _ in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    for _, _, stamp, key in procs:
        with open(stamp, "w") as fh:
            fh.write(key)
    # the build id: the hash of the sources this library is linked from (sdr_build_id)
    bid_src = os.path.join(objdir, "sdr_build_id.cpp")
    with open(bid_src, "w") as fh:
        fh.write('extern "C" const char* sdr_build_id(void) {\n'
                 f'    static const char id[] = "SDR_BUILD_ID={bid}";\n'
                 '    return id + 13;\n}\n')
    bid_obj = os.path.join(objdir, "sdr_build_id.o")
    subprocess.check_call([hipcc, "-O2", "-fPIC", "-x", "c++", "-c", bid_src, "-o", bid_obj])
    objs.append(bid_obj)
    link = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *extra, *objs, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(link))
    subprocess.check_call(link)
    if source_hash() != bid:
        os.remove(out + ".tmp")
        raise RuntimeError("the engine's sources changed during the build: run it again")
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
