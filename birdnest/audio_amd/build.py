"""Build the in-tree native libraries (hipcc for gfx950, gcc for host-only C).

    libbnflac.so        -- HIP kernels + C ABI (the product)
    libbnflac_synth.so  -- synthetic FLAC workload generator

Outputs go to birdnest/audio_amd/lib/ so they travel with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(PKG))
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib")
INCLUDE = os.path.join(ROOT, "include")

HIP_SOURCES = [os.path.join(CSRC, "bnflac_kernels.hip"), os.path.join(CSRC, "bnflac_sys.hip"),
               os.path.join(CSRC, "bnflac_runtime.cpp"), os.path.join(CSRC, "bnflac_reader.cpp")]
HIP_HEADERS = [os.path.join(CSRC, "bnflac_device.h"), os.path.join(CSRC, "bnflac_md5.h"), os.path.join(INCLUDE, "bnflac.h"),
               os.path.join(INCLUDE, "FLAC_compat.h")]
SYNTH_SOURCES = [os.path.join(CSRC, "synth", "bnflac_synth.c")]
SYNTH_HEADERS = [os.path.join(CSRC, "synth", "bnflac_synth.h")]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


KERNEL_TUS = (0, 1, 2, 3, 4, 5, 7)  # one build of bnflac_kernels.hip per BNF_TU: scan+parse, k_decode<8>, k_decode<32> + k_decode_list, k_decode_st<FLACDECODER>, k_decode_st<others>, k_decode<16>, k_decode_sw (TU 8: bnflac_sys.hip)


HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden"]


def source_hash() -> str:
    """Hash of everything libbnflac.so is built from: every HIP/C++ source and header, the
    kernel TU split and the hipcc flags.  bench.py stamps its line with it, and a committed PMC
    summary (profiles/traffic_*.json) is attached to a bench run only when the stamps match."""
    import hashlib
    h = hashlib.sha256()
    for f in HIP_SOURCES + HIP_HEADERS:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(repr((KERNEL_TUS, HIPCC_FLAGS)).encode())
    return h.hexdigest()[:16]


def build_hip(force=False, verbose=False):
    """Compile the kernel TUs and the runtime in parallel (hipcc -c), then link.

    Development variants (never the product): BNFLAC_VARIANT_DIR=<dir> builds into <dir>
    (objects in <dir>/build) with the extra hipcc flags in BNFLAC_EXTRA_CFLAGS, e.g.
    -DBNFLAC_PHASE_TIMERS; load it with BNFLAC_LIB_DIR=<dir> in the debug tools."""
    vdir = os.environ.get("BNFLAC_VARIANT_DIR")
    libdir = vdir or LIB
    out = os.path.join(libdir, "libbnflac.so")
    if force or _stale(out, HIP_SOURCES + HIP_HEADERS):
        os.makedirs(libdir, exist_ok=True)
        objdir = os.path.join(vdir, "build") if vdir else os.path.join(PKG, "build")
        os.makedirs(objdir, exist_ok=True)
        base = [hipcc()] + HIPCC_FLAGS + ["-I" + INCLUDE]
        if vdir:
            base += os.environ.get("BNFLAC_EXTRA_CFLAGS", "").split()
        jobs, objs = [], []
        # development shortcut: BNFLAC_DEV_TUS="1,3" recompiles only those kernel TUs and
        # reuses the other objects as they are (never set for a real build)
        dev = os.environ.get("BNFLAC_DEV_TUS")
        only = {int(x) for x in dev.split(",")} if dev else None
        for tu in KERNEL_TUS:
            o = os.path.join(objdir, f"bnflac_kernels_tu{tu}.o")
            if only is None or tu in only or not os.path.exists(o):
                jobs.append(base + [f"-DBNF_TU={tu}", "-c", HIP_SOURCES[0], "-o", o])
            objs.append(o)
        for src in HIP_SOURCES[1:]:
            o = os.path.join(objdir, os.path.splitext(os.path.basename(src))[0] + ".o")
            jobs.append(base + ["-c", src, "-o", o])
            objs.append(o)
        procs = []
        for cmd in jobs:
            if verbose:
                print(" ".join(cmd))
            procs.append((cmd, subprocess.Popen(cmd)))
        for cmd, p in procs:
            if p.wait() != 0:
                raise subprocess.CalledProcessError(p.returncode, cmd)
        link = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", out + ".tmp"]
        if verbose:
            print(" ".join(link))
        subprocess.check_call(link)
        os.replace(out + ".tmp", out)
    return out


def build_synth(force=False, verbose=False):
    out = os.path.join(LIB, "libbnflac_synth.so")
    if force or _stale(out, SYNTH_SOURCES + SYNTH_HEADERS):
        os.makedirs(LIB, exist_ok=True)
        cmd = ["gcc", "-O2", "-fPIC", "-shared", "-Wall"] + SYNTH_SOURCES + ["-o", out + ".tmp", "-lm"]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
        os.replace(out + ".tmp", out)
    return out


def build_all(force=False, verbose=False):
    return [build_synth(force, verbose), build_hip(force, verbose)]


if __name__ == "__main__":
    for p in build_all(force="--force" in sys.argv, verbose=True):
        print(p)
