"""Developer tool: a kernel VARIANT of libhbx.so for measurement (tools/build.py's translation units,
some recompiled with extra flags, linked with the main build's other objects) ->
hbbft_amd/libhbx_<name>.so, loaded by hbbft_amd/hbx.py when HBX_LIB_PATH names it (bench.py, tests).

Usage: python tools/build_variant.py <name> <tu,tu,...> [-Dflag ...]
(the main build's objects under build/hbx must exist: python tools/build.py)"""
from __future__ import annotations

import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import build  # noqa: E402
import isa_check  # noqa: E402


def build_variant(name: str, tus, flags):
    csrc = os.path.join(build.ROOT, "hbbft_amd", "csrc")
    build.gen_kdecl(csrc)
    vdir = os.path.join(build.ROOT, "build", f"var_{name}")
    os.makedirs(vdir, exist_ok=True)
    procs = []
    for tu in tus:
        cmd = [build.HIPCC, "-O3", f"--offload-arch={build.ARCH}", "-std=c++17", "-fPIC", f"-DHBX_TU={tu}"] + \
            build.TU_FLAGS.get(tu, []) + list(flags) + ["-c", "-o", os.path.join(vdir, f"tu{tu}.o"),
                                                       os.path.join(csrc, "hbx_api.hip")]
        print("+", " ".join(cmd), flush=True)
        procs.append(subprocess.Popen(cmd, cwd=build.ROOT))
    for p in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, p.args)
    objs = [os.path.join(vdir if tu in tus else os.path.join(build.ROOT, "build", "hbx"), f"tu{tu}.o")
            for tu in range(build.N_TU)]
    out = os.path.join(build.ROOT, "hbbft_amd", f"libhbx_{name}.so")
    build.run([build.HIPCC, f"--offload-arch={build.ARCH}", "-shared", "-fPIC", "-o", out] + objs)
    bad = isa_check.find_hazards(out) + [(n, 0, 0) for n, _ in isa_check.find_dpp_folds(out)]
    if bad:
        os.remove(out)
        raise RuntimeError(f"ISA check failed: {bad[:3]}")
    return out


if __name__ == "__main__":
    name, tus = sys.argv[1], [int(t) for t in sys.argv[2].split(",")]
    print(build_variant(name, tus, sys.argv[3:]))
