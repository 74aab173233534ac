"""The wide-tower programs (tools/gen_programs.py -> hbbft_amd/csrc/programs.hpp) interpreted on
the CPU with the executor's semantics (per round: every lane reads, then every lane writes) and
compared with the oracle's Fq12 arithmetic on random inputs."""
import json
import os
import random
import subprocess
import sys

import pytest

from oracle import bls12_381 as bls

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_programs as gp  # noqa: E402

P = bls.P


@pytest.fixture(scope="module")
def progs():
    data = json.load(open(os.path.join(ROOT, "tools", "programs.json")))
    return {pg["name"]: pg for pg in data["programs"]}, [int(v) for v in data["K"]]


def test_tables_in_sync():
    """programs.json / programs.hpp are what the generator produces now."""
    fresh = [gp.compile_program(B) for B in gp.PROGRAMS]
    data = json.load(open(os.path.join(ROOT, "tools", "programs.json")))
    assert json.loads(json.dumps(fresh)) == data["programs"]


def run(pg, K, mem):
    mem = {c: dict(v) for c, v in mem.items()}
    mem.setdefault(gp.SCR, {})
    mem.setdefault(gp.O, {})
    mem[gp.K] = dict(enumerate(K))
    for off, cnt in pg["stages"]:
        assert cnt <= gp.GROUP
        writes = []
        for ins in pg["insns"][off:off + cnt]:
            a = sum(c * mem[cls][idx] for cls, idx, c in ins["a"]) % P
            if ins["op"] == gp.OP_MUL:
                b = sum(c * mem[cls][idx] for cls, idx, c in ins["b"]) % P
                r = a * b % P
            elif ins["op"] == gp.OP_LIN:
                r = a
            else:
                r = pow(a, P - 2, P)
            writes.append((tuple(ins["dst"]), r))
        for (cls, idx), r in writes:
            mem.setdefault(cls, {})[idx] = r
    return mem[gp.O]


def f12_to_slots(a):
    out = []
    for c6 in a:
        for c2 in c6:
            out += [c2[0], c2[1]]
    return dict(enumerate(out))


def slots_to_f12(m):
    v = [m[k] for k in range(12)]
    f2 = [(v[2 * i], v[2 * i + 1]) for i in range(6)]
    return ((f2[0], f2[1], f2[2]), (f2[3], f2[4], f2[5]))


def rand_f12(rnd):
    return slots_to_f12({k: rnd.randrange(P) for k in range(12)})


def cyclotomic(f):
    t = bls.f12_mul(bls.f12_conj(f), bls.f12_inv(f))
    return bls.f12_mul(bls.f12_frobenius_n(t, 2), t)


def line_f12(c0, c1, xp, yp):
    return ((c0, bls.f2_muls(c1, xp), bls.F2_ZERO), (bls.F2_ZERO, (yp, 0), bls.F2_ZERO))


@pytest.mark.parametrize("sqr", [True, False])
def test_mstep(progs, sqr):
    tabs, K = progs
    rnd = random.Random(3 + sqr)
    f = rand_f12(rnd)
    L = {k: rnd.randrange(P) for k in range(8)}
    PT = {k: rnd.randrange(P) for k in range(4)}
    out = run(tabs["MSTEP_SQR" if sqr else "MSTEP"], K, {gp.X: f12_to_slots(f), gp.L: L, gp.PT: PT})
    g = bls.f12_sqr(f) if sqr else f
    g = bls.f12_mul(g, line_f12((L[0], L[1]), (L[2], L[3]), PT[0], PT[1]))
    g = bls.f12_mul(g, line_f12((L[4], L[5]), (L[6], L[7]), PT[2], PT[3]))
    assert slots_to_f12(out) == g


def test_final_exp_pieces(progs):
    tabs, K = progs
    rnd = random.Random(7)
    a, b = rand_f12(rnd), rand_f12(rnd)
    X, Y = f12_to_slots(a), f12_to_slots(b)
    assert slots_to_f12(run(tabs["INV12"], K, {gp.X: X})) == bls.f12_inv(a)
    assert slots_to_f12(run(tabs["CONJ_MUL"], K, {gp.X: X, gp.Y: Y})) == bls.f12_mul(bls.f12_conj(a), b)
    assert slots_to_f12(run(tabs["FROB2_MUL"], K, {gp.X: X})) == bls.f12_mul(bls.f12_frobenius_n(a, 2), a)
    assert slots_to_f12(run(tabs["MUL"], K, {gp.X: X, gp.Y: Y})) == bls.f12_mul(a, b)
    assert slots_to_f12(run(tabs["FROB_MUL_CONJ"], K, {gp.X: X, gp.Y: Y})) == \
        bls.f12_mul(bls.f12_frobenius(a), bls.f12_conj(b))
    assert slots_to_f12(run(tabs["FROB2_MUL_CONJ"], K, {gp.X: X})) == \
        bls.f12_mul(bls.f12_frobenius_n(a, 2), bls.f12_conj(a))
    c = cyclotomic(a)
    assert slots_to_f12(run(tabs["CYCSQR"], K, {gp.X: f12_to_slots(c)})) == bls.f12_sqr(c)


def prepared_lines(Q):
    """68 normalised lines (c0, c1) of Q with l(P) = c0 + c1 x_P v + y_P v w (the layout
    k_prepare_lines writes), from the oracle's affine Miller loop."""
    out = []
    T = Q
    for bit in bin(bls.BLS_X)[3:]:
        xT, yT = T
        lam = bls.f2_mul(bls.f2_muls(bls.f2_sqr(xT), 3), bls.f2_inv(bls.f2_muls(yT, 2)))
        out.append((bls.f2_sub(bls.f2_mul(lam, xT), yT), bls.f2_neg(lam)))
        x3 = bls.f2_sub(bls.f2_sqr(lam), bls.f2_muls(xT, 2))
        T = (x3, bls.f2_sub(bls.f2_mul(lam, bls.f2_sub(xT, x3)), yT))
        if bit == "1":
            xT, yT = T
            lam = bls.f2_mul(bls.f2_sub(yT, Q[1]), bls.f2_inv(bls.f2_sub(xT, Q[0])))
            out.append((bls.f2_sub(bls.f2_mul(lam, xT), yT), bls.f2_neg(lam)))
            x3 = bls.f2_sub(bls.f2_sub(bls.f2_sqr(lam), xT), Q[0])
            T = (x3, bls.f2_sub(bls.f2_mul(lam, bls.f2_sub(xT, x3)), yT))
    assert len(out) == 68
    return out


def run_schedule(progs_by_idx, K, sched, res, PA, QA, PB, QB):
    """Mirror of k_verify_wide's control flow: the schedule table drives everything."""
    la, lb = prepared_lines(QA), prepared_lines(QB)
    R = [dict() for _ in range(gp.NUM_REGIONS)]
    R[0] = {k: (1 if k == 0 else 0) for k in range(12)}
    Pt = {0: PA[0], 1: PA[1], 2: PB[0], 3: PB[1]}
    L = {}
    for prog, x, y, o, line in sched:
        if line >= 0:
            (a0, a1), (b0, b1) = la[line], lb[line]
            L = {0: a0[0], 1: a0[1], 2: a1[0], 3: a1[1], 4: b0[0], 5: b0[1], 6: b1[0], 7: b1[1]}
        out = run(progs_by_idx[prog], K, {gp.X: R[x], gp.Y: R[y], gp.PT: Pt, gp.L: L})
        R[o] = dict(out)
    return all(R[res][k] == (1 if k == 0 else 0) for k in range(12))


def test_pairing_schedule_end_to_end(progs):
    data = json.load(open(os.path.join(ROOT, "tools", "programs.json")))
    tabs, K = progs
    by_idx = [tabs[B.name] for B in gp.PROGRAMS]
    sched, res = data["schedule"], data["result"]
    a = 0xC0FFEE
    P1, Q1 = bls.g1_mul(bls.G1_GEN, a), bls.G2_GEN
    P2, Q2 = bls.g1_neg(bls.G1_GEN), bls.g2_mul(bls.G2_GEN, a)
    assert run_schedule(by_idx, K, sched, res, P1, Q1, P2, Q2)                        # e(aP,Q) e(-P,aQ) = 1
    assert not run_schedule(by_idx, K, sched, res, P1, Q1, P2, bls.g2_mul(bls.G2_GEN, a + 1))
