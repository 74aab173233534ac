"""In-tree build: hipcc for gfx950 -> hbbft_amd/libhbx.so; gcc -> oracle C restatement.

Skips a target whose output is newer than all of its sources.  No cmake/ninja."""
from __future__ import annotations

import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


def newer(out, srcs):
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    return all(os.path.getmtime(s) <= t for s in srcs)


def run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=ROOT)


def build_hbx(force=False):
    csrc = os.path.join(ROOT, "hbbft_amd", "csrc")
    srcs = glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp")) + \
        [os.path.join(ROOT, "include", "hbx.h")]
    out = os.path.join(ROOT, "hbbft_amd", "libhbx.so")
    if not force and newer(out, srcs):
        return out
    run([HIPCC, "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-shared", "-fPIC",
         "-o", out, os.path.join(csrc, "hbx_api.hip")])
    return out


def build_cpu_port(force=False):
    """CPU baseline (bench.py cpu_baseline leg only): the reference's per-share algorithm shape."""
    src = os.path.join(ROOT, "tools", "cpu_baseline", "cpu_port.cpp")
    hdrs = glob.glob(os.path.join(ROOT, "hbbft_amd", "csrc", "*.hpp"))
    outdir = os.path.join(ROOT, "oracle", "_build")
    os.makedirs(outdir, exist_ok=True)
    out = os.path.join(outdir, "libcpu_port.so")
    if not force and newer(out, [src] + hdrs):
        return out
    run(["g++", "-O3", "-march=x86-64-v3", "-std=c++17", "-shared", "-fPIC", "-pthread", "-o", out, src])
    return out


if __name__ == "__main__":
    force = "--force" in sys.argv
    build_hbx(force)
    build_cpu_port(force)
