"""Generate hbbft_amd/csrc/programs.hpp: the wide-tower "programs" the group executor runs.

Why.  A BLS12-381 pairing check is ~16k Fq multiplications with a long sequential spine; one
lane per check leaves the chip latency-bound.  But each tower operation is a
bilinear map whose Fq products are mostly independent: an Fq12 squaring is 36 independent Fq
products followed by additions.  So a check is run by a GROUP of 16 lanes that share its state in
LDS "slots" (one Fq element = 12 x u32 each); every tower step becomes a short list of STAGES, and
each stage a list of independent INSTRUCTIONS that the 16 lanes split:

    MUL  dst = (sum_i c_i * slot_i) * (sum_j d_j * slot_j)     (one Montgomery product per lane)
    LIN  dst = sum_i c_i * slot_i                              (additions only)
    INV  dst = (sum_i c_i * slot_i)^(p-2)                      (Fermat inversion, one lane)

This script writes each tower algorithm ONCE, symbolically (the same formulas as
hbbft_amd/csrc/field.hpp: Karatsuba Fq2/Fq6, complex Fq12 squaring, mul_by_014 lines, Granger-Scott
cyclotomic squaring, Frobenius), traces it into a DAG of MUL/LIN/INV nodes, schedules the DAG into
dependency stages, materialises operands with too many terms, allocates scratch slots (a slot
freed in stage s is reused only from stage s+1, so lanes of one stage never race), and emits
constant tables.  tests/test_programs.py interprets the emitted tables on random inputs and checks
them against the oracle's Fq12 arithmetic.

Slot classes (runtime bases; see programs.hpp):
  SCR  per-group scratch          X, Y, P, O  per-group operand / output regions
  L    per-block shared (Miller line coefficients)     K  per-block constants (Frobenius gammas)

Run: python tools/gen_programs.py   (rewrites hbbft_amd/csrc/programs.hpp and tools/programs.json)
"""
from __future__ import annotations

import json
import os
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
RQ = 1 << 384

# slot classes
SCR, X, Y, PT, O, L, K = range(7)
CLASS_NAMES = ["SCR", "X", "Y", "P", "O", "L", "K"]
MAX_TERMS = 15     # terms per instruction (16-word encoding: header + 15 terms)
MAX_MUL_TERMS = 4  # terms per MUL operand before the operand is materialised by a LIN
OP_MUL, OP_LIN, OP_INV = 0, 1, 2


# ---------------------------------------------------------------------------------------------
# Symbolic linear forms over Fq
# ---------------------------------------------------------------------------------------------
class Lin:
    __slots__ = ("t",)

    def __init__(self, t=None):
        self.t = {k: v for k, v in (t or {}).items() if v}

    def __add__(self, o):
        r = dict(self.t)
        for k, v in o.t.items():
            r[k] = r.get(k, 0) + v
        return Lin(r)

    def __sub__(self, o):
        return self + o.scale(-1)

    def __neg__(self):
        return self.scale(-1)

    def scale(self, c):
        return Lin({k: v * c for k, v in self.t.items()})

    def weight(self):
        return sum(abs(v) for v in self.t.values())


ZERO = Lin()


class Builder:
    """Traces tower arithmetic into nodes.  Node ids: ('in', cls, idx) for inputs, ('n', k) for
    computed nodes."""

    def __init__(self, name):
        self.name = name
        self.nodes = []      # dict(op, a: Lin, b: Lin|None)
        self.outputs = []    # (cls, idx, Lin)

    def inp(self, cls, idx):
        return Lin({("in", cls, idx): 1})

    def _node(self, op, a, b=None):
        self.nodes.append({"op": op, "a": a, "b": b})
        return Lin({("n", len(self.nodes) - 1): 1})

    def mul(self, a, b):
        return self._node(OP_MUL, a, b)

    def inv(self, a):
        return self._node(OP_INV, a)

    def out(self, cls, idx, lin):
        self.outputs.append((cls, idx, lin))

    def lin(self, lin):
        """Materialise a linear form as its own LIN node (unless it already is a single node)."""
        if len(lin.t) == 1 and list(lin.t.values())[0] == 1:
            return lin
        return self._node(OP_LIN, lin)

    def checkpoint(self, v):
        """Materialise every Fq coefficient of a tower element (nested tuples of Lin)."""
        if isinstance(v, Lin):
            return self.lin(v)
        return tuple(self.checkpoint(x) for x in v)


# ---------------------------------------------------------------------------------------------
# Tower algorithms (mirror hbbft_amd/csrc/field.hpp)
# ---------------------------------------------------------------------------------------------
def f2_add(a, b): return (a[0] + b[0], a[1] + b[1])
def f2_sub(a, b): return (a[0] - b[0], a[1] - b[1])
def f2_neg(a): return (-a[0], -a[1])
def f2_dbl(a): return (a[0].scale(2), a[1].scale(2))
def f2_conj(a): return (a[0], -a[1])
def f2_mul_xi(a): return (a[0] - a[1], a[0] + a[1])


def f2_mul(B, a, b):
    t0 = B.mul(a[0], b[0])
    t1 = B.mul(a[1], b[1])
    t2 = B.mul(a[0] + a[1], b[0] + b[1])
    return (t0 - t1, t2 - t0 - t1)


def f2_sqr(B, a):
    t0 = B.mul(a[0] + a[1], a[0] - a[1])
    t1 = B.mul(a[0], a[1])
    return (t0, t1.scale(2))


def f2_mul_fq(B, a, s):
    return (B.mul(a[0], s), B.mul(a[1], s))


def f6_add(a, b): return tuple(f2_add(x, y) for x, y in zip(a, b))
def f6_sub(a, b): return tuple(f2_sub(x, y) for x, y in zip(a, b))
def f6_neg(a): return tuple(f2_neg(x) for x in a)
def f6_mul_v(a): return (f2_mul_xi(a[2]), a[0], a[1])


def f6_mul(B, a, b):
    t0 = f2_mul(B, a[0], b[0])
    t1 = f2_mul(B, a[1], b[1])
    t2 = f2_mul(B, a[2], b[2])
    c0 = f2_mul(B, f2_add(a[1], a[2]), f2_add(b[1], b[2]))
    c0 = f2_add(t0, f2_mul_xi(f2_sub(f2_sub(c0, t1), t2)))
    c1 = f2_mul(B, f2_add(a[0], a[1]), f2_add(b[0], b[1]))
    c1 = f2_add(f2_sub(f2_sub(c1, t0), t1), f2_mul_xi(t2))
    c2 = f2_mul(B, f2_add(a[0], a[2]), f2_add(b[0], b[2]))
    c2 = f2_add(f2_sub(f2_sub(c2, t0), t2), t1)
    return (c0, c1, c2)


def f6_sqr(B, a):
    s0 = f2_sqr(B, a[0])
    s1 = f2_dbl(f2_mul(B, a[0], a[1]))
    s2 = f2_sqr(B, f2_add(f2_sub(a[0], a[1]), a[2]))
    s3 = f2_dbl(f2_mul(B, a[1], a[2]))
    s4 = f2_sqr(B, a[2])
    c0 = f2_add(s0, f2_mul_xi(s3))
    c1 = f2_add(s1, f2_mul_xi(s4))
    c2 = f2_sub(f2_sub(f2_add(f2_add(s1, s2), s3), s0), s4)
    return (c0, c1, c2)


def f6_mul_by_01(B, a, b0, b1):
    t0 = f2_mul(B, a[0], b0)
    t1 = f2_mul(B, a[1], b1)
    c0 = f2_add(t0, f2_mul_xi(f2_mul(B, a[2], b1)))
    c1 = f2_sub(f2_sub(f2_mul(B, f2_add(a[0], a[1]), f2_add(b0, b1)), t0), t1)
    c2 = f2_add(f2_mul(B, a[2], b0), t1)
    return (c0, c1, c2)


def f6_mul_by_1_fq(B, a, s):
    return (f2_mul_xi(f2_mul_fq(B, a[2], s)), f2_mul_fq(B, a[0], s), f2_mul_fq(B, a[1], s))


def f6_inv(B, a):
    c0 = f2_sub(f2_sqr(B, a[0]), f2_mul_xi(f2_mul(B, a[1], a[2])))
    c1 = f2_sub(f2_mul_xi(f2_sqr(B, a[2])), f2_mul(B, a[0], a[1]))
    c2 = f2_sub(f2_sqr(B, a[1]), f2_mul(B, a[0], a[2]))
    t = f2_add(f2_mul(B, a[0], c0), f2_mul_xi(f2_add(f2_mul(B, a[2], c1), f2_mul(B, a[1], c2))))
    # fq2 inverse: conj(t) / norm(t)
    n = B.mul(t[0], t[0]) + B.mul(t[1], t[1])
    ni = B.inv(n)
    ti = (B.mul(t[0], ni), B.mul(-t[1], ni))
    return (f2_mul(B, c0, ti), f2_mul(B, c1, ti), f2_mul(B, c2, ti))


def f12_mul(B, a, b):
    t0 = f6_mul(B, a[0], b[0])
    t1 = f6_mul(B, a[1], b[1])
    c1 = f6_sub(f6_sub(f6_mul(B, f6_add(a[0], a[1]), f6_add(b[0], b[1])), t0), t1)
    return (f6_add(t0, f6_mul_v(t1)), c1)


def f12_sqr(B, a):
    ab = f6_mul(B, a[0], a[1])
    t = f6_mul(B, f6_add(a[0], a[1]), f6_add(a[0], f6_mul_v(a[1])))
    c0 = f6_sub(f6_sub(t, ab), f6_mul_v(ab))
    return (c0, f6_add(ab, ab))


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_mul_by_014(B, f, c0, c1, c4):
    aa = f6_mul_by_01(B, f[0], c0, c1)
    bb = f6_mul_by_1_fq(B, f[1], c4)
    o = (c1[0] + c4, c1[1])
    s = f6_mul_by_01(B, f6_add(f[1], f[0]), c0, o)
    n1 = f6_sub(f6_sub(s, aa), bb)
    n0 = f6_add(f6_mul_v(bb), aa)
    return (n0, n1)


def f12_inv(B, a):
    t = f6_sub(f6_sqr(B, a[0]), f6_mul_v(f6_sqr(B, a[1])))
    ti = f6_inv(B, t)
    return (f6_mul(B, a[0], ti), f6_neg(f6_mul(B, a[1], ti)))


def f4_sqr(B, a, b):
    t0 = f2_sqr(B, a)
    t1 = f2_sqr(B, b)
    c0 = f2_add(f2_mul_xi(t1), t0)
    c1 = f2_sub(f2_sub(f2_sqr(B, f2_add(a, b)), t0), t1)
    return c0, c1


def f12_cyclotomic_sqr(B, f):
    z0, z4, z3 = f[0]
    z2, z1, z5 = f[1]
    t0, t1 = f4_sqr(B, z0, z1)
    z0 = f2_add(f2_dbl(f2_sub(t0, z0)), t0)
    z1 = f2_add(f2_dbl(f2_add(t1, z1)), t1)
    t0, t1 = f4_sqr(B, z2, z3)
    t2, t3 = f4_sqr(B, z4, z5)
    z4 = f2_add(f2_dbl(f2_sub(t0, z4)), t0)
    z5 = f2_add(f2_dbl(f2_add(t1, z5)), t1)
    t0 = f2_mul_xi(t3)
    z2 = f2_add(f2_dbl(f2_add(t0, z2)), t0)
    z3 = f2_add(f2_dbl(f2_sub(t2, z3)), t2)
    return ((z0, z4, z3), (z2, z1, z5))


# Frobenius constants gamma_{1,i} = xi^(i (p-1)/6) (Fq2) and gamma_{2,i} = gamma_{1,i}^(p+1) (in Fq)
def _f2m(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def _f2pow(a, e):
    r = (1, 0)
    for bit in bin(e)[2:]:
        r = _f2m(r, r)
        if bit == "1":
            r = _f2m(r, a)
    return r


GAMMA1 = [_f2pow((1, 1), i * (P - 1) // 6) for i in range(6)]
GAMMA2 = [_f2m(g, (g[0], (-g[1]) % P))[0] for g in GAMMA1]   # norm(gamma1) lies in Fq
# K-region layout: gamma1[i] for i=1..5 (c0, c1) at 2(i-1), 2(i-1)+1; gamma2[i] for i=1..5 at 10+(i-1)
K_VALUES = []
for i in range(1, 6):
    K_VALUES += [GAMMA1[i][0], GAMMA1[i][1]]
for i in range(1, 6):
    K_VALUES.append(GAMMA2[i])


def kconst(B, idx):
    return B.inp(K, idx)


def f12_frobenius(B, a):
    # order of the w^i coefficients: g0..g5 = c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2
    def coef(g, i):
        gc = f2_conj(g)
        k = (kconst(B, 2 * (i - 1)), kconst(B, 2 * (i - 1) + 1))
        return f2_mul(B, gc, k)
    c0 = (f2_conj(a[0][0]), coef(a[0][1], 2), coef(a[0][2], 4))
    c1 = (coef(a[1][0], 1), coef(a[1][1], 3), coef(a[1][2], 5))
    return (c0, c1)


def f12_frobenius2(B, a):
    def coef(g, i):
        return f2_mul_fq(B, g, kconst(B, 10 + (i - 1)))
    c0 = (a[0][0], coef(a[0][1], 2), coef(a[0][2], 4))
    c1 = (coef(a[1][0], 1), coef(a[1][1], 3), coef(a[1][2], 5))
    return (c0, c1)


# ---------------------------------------------------------------------------------------------
# Fq12 element <-> 12 slots of a region
# ---------------------------------------------------------------------------------------------
def f12_in(B, cls, base=0):
    s = [B.inp(cls, base + k) for k in range(12)]
    return ((s[0:2], s[2:4], s[4:6]), (s[6:8], s[8:10], s[10:12]))


def f12_flat(a):
    out = []
    for c6 in a:
        for c2 in c6:
            out += [c2[0], c2[1]]
    return out


def f12_out(B, cls, a, base=0):
    for k, lin in enumerate(f12_flat(a)):
        B.out(cls, base + k, lin)


def _tup(a):
    return tuple(tuple(tuple(c2) for c2 in c6) for c6 in a)


# ---------------------------------------------------------------------------------------------
# The programs
# ---------------------------------------------------------------------------------------------
def line_eval(B, f, lbase, pbase):
    """f * l(P) for a prepared line (c0, c1 in L[lbase..lbase+3]) at P = (x, y) in P[pbase..]."""
    c0 = (B.inp(L, lbase), B.inp(L, lbase + 1))
    lc1 = (B.inp(L, lbase + 2), B.inp(L, lbase + 3))
    xp, yp = B.inp(PT, pbase), B.inp(PT, pbase + 1)
    c1 = f2_mul_fq(B, lc1, xp)
    return f12_mul_by_014(B, f, c0, c1, yp)


def prog_mstep(sqr: bool):
    """Miller step of a 2-pair loop: O = X^2 (if sqr) * l_A(P_A) * l_B(P_B).
    Lines: A at L[0..3], B at L[4..7]; points: P_A = P[0..1], P_B = P[2..3]."""
    B = Builder("MSTEP_SQR" if sqr else "MSTEP")
    f = f12_in(B, X)
    if sqr:
        f = B.checkpoint(f12_sqr(B, f))
    f = B.checkpoint(line_eval(B, f, 0, 0))
    f = line_eval(B, f, 4, 2)
    f12_out(B, O, f)
    return B


def prog_inv():
    """O = X^-1 (Fq12 inverse through Fq6 and Fq2 down to one Fq inversion)."""
    B = Builder("INV12")
    f12_out(B, O, f12_inv(B, f12_in(B, X)))
    return B


def prog_conj_mul():
    """O = conj(X) * Y  (with Y = X^-1: the first easy-part factor X^(p^6 - 1))."""
    B = Builder("CONJ_MUL")
    f12_out(B, O, f12_mul(B, f12_conj(f12_in(B, X)), f12_in(B, Y)))
    return B


def prog_frob2_mul():
    """O = frob2(X) * X  (the second easy-part factor X^(p^2 + 1))."""
    B = Builder("FROB2_MUL")
    x = f12_in(B, X)
    f12_out(B, O, f12_mul(B, f12_frobenius2(B, x), x))
    return B


def prog_cycsqr():
    B = Builder("CYCSQR")
    f12_out(B, O, f12_cyclotomic_sqr(B, f12_in(B, X)))
    return B


def prog_mul():
    B = Builder("MUL")
    f12_out(B, O, f12_mul(B, f12_in(B, X), f12_in(B, Y)))
    return B


def prog_frob_mul_conj():
    """O = frob(X) * conj(Y)."""
    B = Builder("FROB_MUL_CONJ")
    f12_out(B, O, f12_mul(B, f12_frobenius(B, f12_in(B, X)), f12_conj(f12_in(B, Y))))
    return B


def prog_frob2_mul_conj():
    """O = frob2(X) * conj(X)."""
    B = Builder("FROB2_MUL_CONJ")
    x = f12_in(B, X)
    f12_out(B, O, f12_mul(B, f12_frobenius2(B, x), f12_conj(x)))
    return B


PROGRAMS = [prog_mstep(True), prog_mstep(False), prog_inv(), prog_conj_mul(), prog_frob2_mul(), prog_cycsqr(),
            prog_mul(), prog_frob_mul_conj(), prog_frob2_mul_conj()]


# ---------------------------------------------------------------------------------------------
# Compilation: materialise, schedule, allocate
# ---------------------------------------------------------------------------------------------
GROUP = 16          # lanes per group = instructions per round
BLS_X = 0xD201000000010000
NUM_REGIONS = 4     # Fq12 regions per group (R0..R3)


def pairing_schedule():
    """Program invocations of one 2-pair check e(P_A, Q_A) e(P_B, Q_B) == 1, as data.

    Entries (prog, x_region, y_region, o_region, line): `line` >= 0 means "load prepared line
    `line` of Q_A and Q_B into the L buffer first".  The Miller loop runs over |x| without the
    final conjugation (FE(conj f) = FE(f)^-1, so the ==1 test is unchanged); the final
    exponentiation computes FE(f)^3 (3 is prime to r) with the hard part
    (x-1)^2 (x+p) (x^2+p^2-1) + 3 of hbbft_amd/csrc/pairing.hpp, in 4 regions."""
    names = {B.name: i for i, B in enumerate(PROGRAMS)}
    E = []
    cur, nxt = 0, 1
    k = 0
    for i in range(62, -1, -1):
        E.append((names["MSTEP"] if k == 0 else names["MSTEP_SQR"], cur, 0, nxt, k))
        cur, nxt = nxt, cur
        k += 1
        if (BLS_X >> i) & 1:
            E.append((names["MSTEP"], cur, 0, nxt, k))
            cur, nxt = nxt, cur
            k += 1
    assert k == 68
    free = [r for r in range(NUM_REGIONS) if r != cur]

    def alloc():
        return free.pop(0)

    def release(*rs):
        free.extend(rs)

    def emit(name, x, y=0):
        o = alloc()
        E.append((names[name], x, y, o, -1))
        return o

    def exp_x(g):
        r = emit("CYCSQR", g)
        for i in range(62, -1, -1):
            if i != 62:
                r2 = emit("CYCSQR", r)
                release(r)
                r = r2
            if (BLS_X >> i) & 1:
                r2 = emit("MUL", r, g)
                release(r)
                r = r2
        return r

    inv = emit("INV12", cur)
    t1 = emit("CONJ_MUL", cur, inv)
    release(cur, inv)
    t = emit("FROB2_MUL", t1)
    release(t1)
    s = emit("CYCSQR", t)
    t3 = emit("MUL", s, t)
    release(s)
    e1 = exp_x(t)
    a_conj = emit("MUL", e1, t)          # t^(|x|+1) = conj(t^(x-1))
    release(e1, t)
    e2 = exp_x(a_conj)
    a2 = emit("MUL", e2, a_conj)         # t^((x-1)^2)
    release(e2, a_conj)
    e3 = exp_x(a2)
    b = emit("FROB_MUL_CONJ", a2, e3)    # a2^(x+p)
    release(a2, e3)
    d = emit("FROB2_MUL_CONJ", b)        # b^(p^2-1)
    d2 = emit("MUL", d, t3)
    release(d, t3)
    e4 = exp_x(b)
    release(b)
    e5 = exp_x(e4)                       # b^(x^2)
    release(e4)
    res = emit("MUL", e5, d2)
    return E, res


def compile_program(B: Builder, group: int = GROUP):
    """Trace -> DAG -> list-scheduled rounds of <= `group` instructions -> slot allocation.

    A round is one pass of the group's lanes over its instructions; every lane first loads its
    operands, then multiplies, then stores, so a slot whose last reader runs in round r may be
    the destination of an instruction in round r (reads precede writes within a round)."""
    nodes = []          # dict(op, a: [(ref, coef)], b: [...], dst)
    ids = {}

    def ref(key):
        return ("in", key[1], key[2]) if key[0] == "in" else ("n", ids[key[1]])

    def materialise(lin, limit):
        terms = [(ref(k), c) for k, c in sorted(lin.t.items(), key=lambda kv: str(kv[0]))]
        if len(terms) > limit:
            while len(terms) > MAX_TERMS:
                chunk, terms = terms[:MAX_TERMS], terms[MAX_TERMS:]
                nodes.append({"op": OP_LIN, "a": chunk, "b": [], "dst": None})
                terms.append((("n", len(nodes) - 1), 1))
            if len(terms) > limit:
                nodes.append({"op": OP_LIN, "a": terms, "b": [], "dst": None})
                terms = [(("n", len(nodes) - 1), 1)]
        return terms

    for bi, nd in enumerate(B.nodes):
        if nd["op"] == OP_MUL:
            a = materialise(nd["a"], MAX_MUL_TERMS)
            b = materialise(nd["b"], MAX_MUL_TERMS)
        else:
            a = materialise(nd["a"], MAX_TERMS)
            b = []
        ids[bi] = len(nodes)
        nodes.append({"op": nd["op"], "a": a, "b": b, "dst": None})
    for cls, idx, lin in B.outputs:
        terms = materialise(lin, MAX_TERMS)
        r0 = terms[0][0]
        if len(terms) == 1 and terms[0][1] == 1 and r0[0] == "n" and nodes[r0[1]]["dst"] is None:
            nodes[r0[1]]["dst"] = (cls, idx)
            continue
        nodes.append({"op": OP_LIN, "a": terms, "b": [], "dst": (cls, idx)})
    N = len(nodes)
    deps = [sorted({r[1] for r, _ in n["a"] + n["b"] if r[0] == "n"}) for n in nodes]
    users = [[] for _ in range(N)]
    for k, d in enumerate(deps):
        for j in d:
            users[j].append(k)
    # priority: longest path to a sink (MUL/INV weigh more than LIN)
    w = [1.0 if n["op"] != OP_LIN else 0.35 for n in nodes]
    prio = [0.0] * N
    for k in reversed(range(N)):
        prio[k] = w[k] + max([prio[u] for u in users[k]] + [0.0])
    # list scheduling
    rnd = [None] * N
    done = 0
    r = 0
    while done < N:
        ready = [k for k in range(N) if rnd[k] is None and all(rnd[d] is not None and rnd[d] < r for d in deps[k])]
        ready.sort(key=lambda k: -prio[k])
        for k in ready[:group]:
            rnd[k] = r
        done += min(group, len(ready))
        r += 1
    nrounds = r
    # liveness & scratch allocation
    last = [max([rnd[u] for u in users[k]] + [-1]) for k in range(N)]
    busy = []   # per slot: round after which it is free (its last read round)
    for rr in range(nrounds):
        for k in range(N):
            if rnd[k] != rr or nodes[k]["dst"] is not None:
                continue
            assert last[k] > rr, f"{B.name}: node {k} unused"
            for sl in range(len(busy)):
                if busy[sl] <= rr:
                    busy[sl] = last[k]
                    nodes[k]["dst"] = (SCR, sl)
                    break
            else:
                busy.append(last[k])
                nodes[k]["dst"] = (SCR, len(busy) - 1)
    # emit rounds as stages
    stages, insns = [], []
    for rr in range(nrounds):
        st = [k for k in range(N) if rnd[k] == rr]
        st.sort(key=lambda k: (nodes[k]["op"] == OP_LIN, nodes[k]["op"]))
        stages.append((len(insns), len(st)))
        for k in st:
            n = nodes[k]

            def enc(rf, c):
                loc = (rf[1], rf[2]) if rf[0] == "in" else nodes[rf[1]]["dst"]
                assert -100 < c < 100 and c != 0
                return (loc[0], loc[1], c)
            insns.append({"op": n["op"], "dst": n["dst"], "a": [enc(rf, c) for rf, c in n["a"]],
                          "b": [enc(rf, c) for rf, c in n["b"]]})
    return {"name": B.name, "stages": stages, "insns": insns, "scratch": len(busy),
            "muls": sum(1 for n in nodes if n["op"] == OP_MUL)}


def encode_insn(ins):
    hdr = ins["op"] | (len(ins["a"]) << 4) | (len(ins["b"]) << 8) | (ins["dst"][0] << 12) | (ins["dst"][1] << 16)
    words = [hdr]
    for cls, idx, c in ins["a"] + ins["b"]:
        words.append(idx | (cls << 16) | ((c & 0xFF) << 24))
    words += [0] * (16 - len(words))
    return words


def limbs32(v, n=12):
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def main():
    progs = [compile_program(B) for B in PROGRAMS]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sched, res = pairing_schedule()
    with open(os.path.join(root, "tools", "programs.json"), "w") as f:
        json.dump({"programs": progs, "K": [str(v) for v in K_VALUES], "schedule": sched, "result": res}, f)
    lines = ["// Generated by tools/gen_programs.py -- do not edit by hand.",
             "// Wide-tower programs for the group executor (hbbft_amd/csrc/wide.hpp).", "#pragma once",
             "#include <stdint.h>", "namespace hbx {", "namespace prog {"]
    lines.append(f"constexpr int SCR = {SCR}, X = {X}, Y = {Y}, PT = {PT}, O = {O}, L = {L}, K = {K};")
    all_words, all_stages = [], []
    meta = []
    for pg in progs:
        meta.append((pg["name"], len(all_stages), len(pg["stages"]), pg["scratch"], pg["muls"]))
        for off, cnt in pg["stages"]:
            all_stages.append((len(all_words) // 16 + off, cnt))
        for ins in pg["insns"]:
            all_words += encode_insn(ins)
    max_scr = max(pg["scratch"] for pg in progs)
    lines.append(f"constexpr int MAX_SCRATCH = {max_scr};")
    lines.append(f"constexpr int NUM_K = {len(K_VALUES)};")
    for i, (name, s0, ns, scr, muls) in enumerate(meta):
        lines.append(f"constexpr int {name} = {i};  // stages {ns}, scratch slots {scr}, Fq products {muls}")
    lines.append(f"constexpr int NUM_PROGRAMS = {len(meta)};")
    lines.append("// program -> (first stage, stage count)")
    lines.append("__device__ constexpr uint32_t PROG_STAGES[NUM_PROGRAMS][2] = {" +
                 ", ".join(f"{{{s0}u, {ns}u}}" for _, s0, ns, _, _ in meta) + "};")
    lines.append("// stage -> (first instruction, instruction count)")
    lines.append(f"__device__ constexpr uint32_t STAGES[{len(all_stages)}][2] = {{" +
                 ", ".join(f"{{{a}u, {b}u}}" for a, b in all_stages) + "};")
    lines.append("// instructions, 16 words each: hdr = op | nA<<4 | nB<<8 | dcls<<12 | didx<<16;")
    lines.append("// term = idx | cls<<16 | (int8 coef)<<24")
    lines.append(f"__device__ constexpr uint32_t INSNS[{len(all_words) // 16}][16] = {{")
    for k in range(0, len(all_words), 16):
        lines.append("  {" + ", ".join("0x%08xu" % w for w in all_words[k:k + 16]) + "},")
    lines.append("};")
    lines.append("// K region: Frobenius gammas in Montgomery form (gamma1[1..5] as Fq2, gamma2[1..5] in Fq)")
    lines.append(f"__device__ constexpr uint32_t KCONST[NUM_K][12] = {{")
    for v in K_VALUES:
        lines.append("  {" + ", ".join("0x%08xu" % w for w in limbs32(v * RQ % P)) + "},")
    lines.append("};")
    sched, res = pairing_schedule()
    lines.append("// pairing-check schedule: prog | x<<4 | y<<8 | o<<12 | (line+1)<<16  (line 0 = none)")
    lines.append(f"constexpr int NUM_REGIONS = {NUM_REGIONS};")
    lines.append(f"constexpr int SCHED_LEN = {len(sched)};")
    lines.append(f"constexpr int SCHED_RESULT_REGION = {res};")
    lines.append(f"__device__ constexpr uint32_t SCHED[SCHED_LEN] = {{" +
                 ", ".join("0x%08xu" % (pg | (x << 4) | (y << 8) | (o << 12) | ((ln + 1) << 16))
                           for pg, x, y, o, ln in sched) + "};")
    lines.append("}  // namespace prog")
    lines.append("}  // namespace hbx")
    with open(os.path.join(root, "hbbft_amd", "csrc", "programs.hpp"), "w") as f:
        f.write("\n".join(lines) + "\n")
    for name, s0, ns, scr, muls in meta:
        pg = progs[[m[0] for m in meta].index(name)]
        rounds = sum((cnt + 15) // 16 for _, cnt in pg["stages"])
        print(f"{name:16s} stages {ns:3d}  insns {len(pg['insns']):4d}  muls {muls:4d}  scratch {scr:3d}  rounds@16 {rounds}",
              file=sys.stderr)


if __name__ == "__main__":
    main()
