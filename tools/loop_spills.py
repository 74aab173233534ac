"""Developer tool: scratch traffic inside loops, per kernel, from a gfx950 code object.

The compiler's "VGPRs Spill" count does not say where the spill code runs: spills in a kernel's
prologue / epilogue cost a few hundred bytes per lane once, spills inside the exponentiation loop
cost that on every iteration.  This lists, per function, the scratch loads/stores inside loop
bodies (instruction ranges closed by a backward branch; nested loops are reported by their
innermost range) and in total.

Usage: python tools/loop_spills.py file.o|file.so|file.co
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_check  # noqa: E402

VERBOSE = "-v" in sys.argv
MIX = "-m" in sys.argv  # instruction mix of every loop body of 300+ instructions
ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")
TARGET = re.compile(r"<[^+>]+\+0x([0-9a-f]+)>")


def _imm(ins: str) -> int:
    v = ins.split(",")[-1].split("//")[0].strip()
    return int(v, 16) if v.startswith("0x") else int(v)


def analyse(disasm: str):
    out = []
    for name, start, body in _funcs(disasm):
        loops = []
        pc_base, lo = None, 0
        for k, (addr, ins) in enumerate(body):
            if ins.startswith(("s_cbranch", "s_branch")):
                m = TARGET.search(ins)
                if m:
                    tgt = start + int(m.group(1), 16)
                    if tgt <= addr:
                        loops.append((tgt, addr))
            # far branches: s_getpc_b64 sX; s_add_u32 lo; s_addc_u32 hi; s_setpc_b64 sX
            if ins.startswith("s_getpc_b64"):
                pc_base = addr + 4
            elif ins.startswith("s_add_u32") and pc_base is not None:
                lo = _imm(ins)
            elif ins.startswith("s_addc_u32") and pc_base is not None:
                hi = _imm(ins)
                off = ((hi & 0xFFFFFFFF) << 32) | (lo & 0xFFFFFFFF)
                if off >= 1 << 63:
                    off -= 1 << 64
                tgt = pc_base + off
                if tgt <= addr:
                    loops.append((tgt, addr))
                pc_base = None
        in_loop = 0
        total = 0
        loop_insts = 0
        inner = {}  # innermost loop (start, end) -> scratch ops in it
        for addr, ins in body:
            sc = ins.startswith("scratch_") or (ins.startswith("buffer_") and "off" in ins)
            inside = [l for l in loops if l[0] <= addr <= l[1]]
            if sc:
                total += 1
                if inside:
                    in_loop += 1
                    l = min(inside, key=lambda l: l[1] - l[0])
                    inner[l] = inner.get(l, 0) + 1
            if inside:
                loop_insts += 1
        if VERBOSE:
            for (a, b), c in sorted(inner.items()):
                n_in = sum(1 for x, _ in body if a <= x <= b)
                print(f"    loop {a:#x}..{b:#x} ({n_in} insts): {c} scratch ops")
        if MIX:
            for a, b in sorted(set(loops)):
                ops = [ins.split()[0] for x, ins in body if a <= x <= b]
                if len(ops) < 300:
                    continue
                mad = sum(o.startswith("v_mad_") for o in ops)
                valu = sum(o.startswith("v_") for o in ops)
                sc = sum(o.startswith(("scratch_", "buffer_")) for o in ops)
                ds = sum(o.startswith("ds_") for o in ops)
                nop = sum(o == "s_nop" for o in ops)
                acc = sum(o.startswith("v_accvgpr") for o in ops)
                top = {}
                for o in ops:
                    if o.startswith("v_") and not o.startswith("v_mad_"):
                        top[o] = top.get(o, 0) + 1
                top = sorted(top.items(), key=lambda kv: -kv[1])[:10]
                print(f"  {name[:40]} loop {a:#x}..{b:#x}: {len(ops)} insts, v_mad {mad}, other VALU {valu - mad} "
                      f"(accvgpr moves {acc}), scratch {sc}, ds {ds}, s_nop {nop}; {top}")
        out.append((name, len(body), total, in_loop, loop_insts, len(loops)))
    return out


def _funcs(disasm: str):
    name, start, body = None, 0, []
    for line in disasm.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            if name:
                yield name, start, body
            name, start, body = m.group(2), int(m.group(1), 16), []
        elif name and line.startswith("\t"):
            a = ADDR.search(line)
            if a:
                body.append((int(a.group(1), 16), line.strip()))
    if name:
        yield name, start, body


def main(path):
    with tempfile.TemporaryDirectory() as tmp:
        cos = [path] if path.endswith(".co") else isa_check._code_objects(path, tmp)
        for co in cos:
            dis = subprocess.run([f"{isa_check.LLVM}/llvm-objdump", "-d", f"--mcpu={isa_check.ARCH}", co],
                                 capture_output=True, text=True, check=True).stdout
            for name, n, total, in_loop, loop_insts, nloops in analyse(dis):
                if total or "fe1" in name or "verify" in name:
                    print(f"{name[:60]:60s} insts {n:7d}  scratch ops {total:5d}  in loops {in_loop:5d}  "
                          f"(loop insts {loop_insts}, loops {nloops})")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        if p not in ("-v", "-m"):
            main(p)
