"""Static check of the gfx950 code objects in libhbx.so (or an object file) for the hazard that hung
three earlier builds (DESIGN.md §4.2 "The hang").

Mechanism, found in the disassembly of the hung coin build (commit 22714e6, cyc_exp_abs_x_d): a
non-kernel function returns with ``s_setpc_b64 s[30:31]`` (the return address of the AMDGPU
calling convention).  When such a function's body is larger than the +-128 KiB reach of
``s_cbranch``/``s_branch``, LLVM's branch relaxation rewrites far branches as
``s_getpc_b64 sX; s_add_u32; s_addc_u32; s_setpc_b64 sX`` -- and in a leaf function it used
s[30:31] for sX without saving it.  The return then jumps to the last far-branch target inside the
function's own loop: the wave never leaves the function (the printf trace of the r03e build
entered the first exp-by-|x| and never returned).  Kernels are not affected (they end in
s_endpgm; nothing lives in s[30:31]).

``find_dpp_folds`` lists every VALU instruction other than a DPP move that carries row_newbcast,
and every reversed-opcode DPP instruction (measured wrong on gfx950; see the comment above it).

``find_hazards`` lists every non-kernel function that performs a far branch through s[30:31]
(an ``s_setpc_b64 s[30:31]`` that is preceded by an ``s_add_u32 s30`` of a relaxation sequence)
and also returns through s[30:31].  tests/test_isa.py asserts the shipped library has none.

Usage: python tools/isa_check.py [path.so|path.o ...]
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ARCH = "gfx950"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _code_objects(path: str, tmp: str):
    """Device code objects (ELF) inside a host .so/.o's .hip_fatbin section."""
    fat = os.path.join(tmp, "fatbin")
    subprocess.check_call([f"{LLVM}/llvm-objcopy", "--dump-section=.hip_fatbin=" + fat, path, os.path.join(tmp, "x")],
                          stderr=subprocess.DEVNULL)
    out = []
    data = open(fat, "rb").read()
    # a linked .so holds one bundle per translation unit: split at the bundle magic
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    for k, s in enumerate(starts):
        e = starts[k + 1] if k + 1 < len(starts) else len(data)
        b = os.path.join(tmp, f"b{k}")
        open(b, "wb").write(data[s:e])
        co = os.path.join(tmp, f"co{k}")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o",
                            f"--targets=hipv4-amdgcn-amd-amdhsa--{ARCH}", f"--input={b}", f"--output={co}",
                            "--unbundle"], stderr=subprocess.DEVNULL)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            out.append(co)
    return out


def _functions(disasm: str):
    """(name, [instruction lines]) per symbol of an llvm-objdump listing."""
    name, body = None, []
    for line in disasm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            if name:
                yield name, body
            name, body = m.group(1), []
        elif name and line.startswith("\t"):
            body.append(line.strip().split("//")[0].strip())
    if name:
        yield name, body


def find_hazards_in_listing(disasm: str):
    bad = []
    for name, body in _functions(disasm):
        if any(i.startswith("s_endpgm") for i in body):
            continue  # a kernel
        returns = any(i == "s_setpc_b64 s[30:31]" for i in body)
        far = 0
        for k, ins in enumerate(body):
            if ins == "s_setpc_b64 s[30:31]" and k >= 1 and body[k - 1].startswith("s_addc_u32 s31"):
                far += 1
        if returns and far:
            bad.append((name, far, len(body)))
    return bad


# A lane move folded into its consumer (DESIGN.md §4.2 "The DPP fold").  The
# engine moves a lane's digit to its 16-lane row with `v_mov_b32_dpp ... row_newbcast:K`; LLVM's DPP
# combiner may fold such a move into the VALU op that consumes it, commuting a subtraction whose
# broadcast operand is the subtrahend into the reversed opcode (`v_sub_u32 d, x, t` ->
# `v_subrev_u32_dpp d, s, x`).  tools/microbench/dppfold.hip (profiles/r06b_dppfold.txt) measured on
# gfx950: folded v_add / v_sub / v_xor are exact (bound_ctrl:1 included), but the REVERSED VOP2
# opcodes (v_subrev_u32_dpp, v_lshlrev_b32_dpp) take the DPP lane selection on the other operand
# (x of lane K minus s of the own lane), with row_newbcast and with quad_perm alike -- the wrong
# sums of round 5.  The moves are pinned (groupd.hpp fqd_from_row), and the build refuses (a) any
# reversed-opcode DPP instruction, whatever its control, and (b) any non-move VALU instruction that
# carries row_newbcast (the broader rule VERDICT r5 asked for).
_DPP_MOVES = ("v_mov_b32_dpp", "v_mov_b64_dpp")


def find_dpp_folds_in_listing(disasm: str):
    """[(function, instruction)] for every DPP-modified VALU op other than a move that uses
    row_newbcast, and every reversed-opcode (…rev…) DPP op."""
    bad = []
    for name, body in _functions(disasm):
        for ins in body:
            op = ins.split(" ", 1)[0]
            if not op.endswith("_dpp") or op in _DPP_MOVES:
                continue
            if "row_newbcast" in ins or "rev_" in op:
                bad.append((name, ins))
    return bad


def _listings(path: str):
    with tempfile.TemporaryDirectory() as tmp:
        for co in _code_objects(path, tmp):
            yield subprocess.run([f"{LLVM}/llvm-objdump", "-d", f"--mcpu={ARCH}", co], capture_output=True,
                                 text=True, check=True).stdout


def find_hazards(path: str):
    bad = []
    for dis in _listings(path):
        bad += find_hazards_in_listing(dis)
    return bad


def find_dpp_folds(path: str):
    bad = []
    for dis in _listings(path):
        bad += find_dpp_folds_in_listing(dis)
    return bad


if __name__ == "__main__":
    paths = sys.argv[1:] or [os.path.join(ROOT, "hbbft_amd", "libhbx.so")]
    rc = 0
    for p in paths:
        hz = find_hazards(p)
        for name, far, n in hz:
            print(f"{p}: {name}: {far} far branch(es) through the return address s[30:31] ({n} instructions)")
            rc = 1
        if not hz:
            print(f"{p}: no far branch through s[30:31] in any returning function")
        folds = find_dpp_folds(p)
        for name, ins in folds[:20]:
            print(f"{p}: {name}: row broadcast folded into a VALU op: {ins}")
        if folds:
            rc = 1
        else:
            print(f"{p}: no row_newbcast outside v_mov_b32_dpp, no reversed-opcode DPP")
    sys.exit(rc)
