"""Developer tool: per-kernel resource usage from gfx950 code objects (AMDGPU metadata notes).

Prints, per kernel: arch VGPRs, AGPRs, spilled VGPRs / SGPRs, private (scratch) bytes per lane and
LDS bytes -- the numbers the step kernels' spill work is judged by.

Usage: python tools/kres.py [-k REGEX] file.o|file.so ...
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_check  # noqa: E402

FIELDS = ((".vgpr_count", "vgpr"), (".agpr_count", "agpr"), (".vgpr_spill_count", "vspill"),
          (".sgpr_spill_count", "sspill"), (".private_segment_fixed_size", "scratch"),
          (".group_segment_fixed_size", "lds"))


def kernel_resources(path: str):
    """{kernel symbol: {field: int}} over every code object inside `path`."""
    res = {}
    with tempfile.TemporaryDirectory() as tmp:
        with open(path, "rb") as fh:
            head = fh.read(20)
        # a device-only compile (--cuda-device-only) is the AMDGPU code object itself (e_machine 224)
        direct = head[:4] == b"\x7fELF" and int.from_bytes(head[18:20], "little") == 224
        if head.startswith(b"__CLANG_OFFLOAD_BUN"):  # a device-only compile without -fno-gpu-rdc bundling
            co = os.path.join(tmp, "co")
            subprocess.check_call([f"{isa_check.LLVM}/clang-offload-bundler", "--type=o",
                                   f"--targets=hipv4-amdgcn-amd-amdhsa--{isa_check.ARCH}", f"--input={path}",
                                   f"--output={co}", "--unbundle"])
            path, direct = co, True
        for co in ([path] if direct else isa_check._code_objects(path, tmp)):
            notes = subprocess.run([f"{isa_check.LLVM}/llvm-readelf", "--notes", co], capture_output=True,
                                   text=True).stdout
            for block in re.split(r"\n\s*- \.agpr_count", notes)[1:]:
                block = ".agpr_count" + block
                m = re.search(r"\.name:\s+(\S+)", block)
                if not m:
                    continue
                d = {}
                for key, short in FIELDS:
                    k = re.search(re.escape(key) + r":\s+(\d+)", block)
                    d[short] = int(k.group(1)) if k else -1
                res[m.group(1)] = d
    return res


if __name__ == "__main__":
    args = sys.argv[1:]
    pat = None
    if args[:1] == ["-k"]:
        pat, args = re.compile(args[1]), args[2:]
    for path in args:
        for name, d in sorted(kernel_resources(path).items()):
            if pat and not pat.search(name):
                continue
            print(f"{name:60s} " + " ".join(f"{k}={v}" for k, v in d.items()))
