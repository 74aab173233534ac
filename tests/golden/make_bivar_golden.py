"""Generate the committed SyncKeyGen value-check fixtures with the oracle.

    python tests/golden/make_bivar_golden.py      # bivar_t2.npz (N = 7), bivar_t5.npz (N = 16)

One node's view (our_idx, x = our_idx + 1) of the Part commitments of P proposers and of the Ack
values every sender decrypted for it: SyncKeyGen::handle_ack checks
`part.commit.evaluate(our_idx + 1, sender_idx + 1) == G1Affine::one().mul(val)`
(src/sync_key_gen.rs:449) and handle_part uses `commit.row(our_idx + 1)` (:313).  Commitments are
of random symmetric bivariate polynomials of degree t (oracle/bivar.py, coefficient order
coeff_pos); values are the polynomial's evaluations, with faults: a value off by one ("wrong
value"), a value >= r (not a canonical Fr: the reference cannot deserialise it), and one proposer
whose commitment holds a point off the G1 subgroup (its Part would not deserialise).
Expected per ack: HBX_SHARE_VALID (1) / HBX_SHARE_INVALID (0) / HBX_SHARE_UNDECODABLE (3); per
proposer the compressed row commitment R_j(x), j = 0..t.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bivar  # noqa: E402
from oracle import bls12_381 as bls  # noqa: E402
from oracle import threshold as tc  # noqa: E402
from oracle.chacha_rand04 import ChaChaRng04  # noqa: E402

sys.path.insert(0, HERE)
from make_golden import off_subgroup_g1  # noqa: E402

INVALID, VALID, UNDECODABLE = 0, 1, 3


def make(n: int, p: int, our_idx: int):
    t = (n - 1) // 3
    x = our_idx + 1
    rng = ChaChaRng04([0x68626278, 0x60 + n])
    polys = [bivar.BivarPoly(t, [tc.fr_rand(rng) for _ in range(bivar.n_coeffs(t))]) for _ in range(p)]
    commits = [pl.commitment() for pl in polys]
    bad_commit = p - 1  # one coefficient off the subgroup
    commit_bytes = [[bls.g1_compress(c) for c in cm] for cm in commits]
    commit_bytes[bad_commit][1] = bls.g1_compress(off_subgroup_g1(9090 + n))
    rows = [[bls.g1_compress(r) for r in bivar.row(commits[q], t, x)] for q in range(p)]
    acks_p, acks_y, vals, expect = [], [], [], []
    for q in range(p):
        for s in range(n):
            y = s + 1
            v = polys[q].evaluate(x, y)
            e = VALID
            if (q * n + s) % 5 == 3:
                v = (v + 1) % bls.R
                e = INVALID
            if q == 0 and s == n - 1:
                v = v + bls.R if v + bls.R < (1 << 256) else v  # non-canonical encoding
                e = UNDECODABLE
            if q == bad_commit:
                e = UNDECODABLE
            acks_p.append(q)
            acks_y.append(y)
            vals.append(v.to_bytes(32, "big"))
            expect.append(e)
    # re-check the expected verdicts with the commitment evaluation itself (decodable cases)
    for k in range(0, len(acks_p), 3):
        q, y = acks_p[k], acks_y[k]
        if expect[k] == UNDECODABLE:
            continue
        lhs = bivar.evaluate(commits[q], t, x, y)
        rhs = bls.g1_mul(bls.G1_GEN, int.from_bytes(vals[k], "big"))
        assert (lhs == rhs) == (expect[k] == VALID), k
    M = bivar.n_coeffs(t)
    return dict(n=np.int64(n), t=np.int64(t), x=np.int64(x), p=np.int64(p),
                commits=np.frombuffer(b"".join(b for cm in commit_bytes for b in cm), dtype=np.uint8).reshape(p, M, 48),
                rows=np.frombuffer(b"".join(b for r in rows for b in r), dtype=np.uint8).reshape(p, t + 1, 48),
                commit_status=np.array([UNDECODABLE if q == bad_commit else VALID for q in range(p)], dtype=np.uint8),
                ack_proposer=np.array(acks_p, dtype=np.uint32), ack_y=np.array(acks_y, dtype=np.uint64),
                vals=np.frombuffer(b"".join(vals), dtype=np.uint8).reshape(len(vals), 32),
                expect=np.array(expect, dtype=np.uint8))


def main():
    for name, (n, p, me) in {"bivar_t2": (7, 4, 2), "bivar_t5": (16, 3, 9)}.items():
        d = make(n, p, me)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **d)
        print(name, "acks", len(d["expect"]), "valid", int((d["expect"] == VALID).sum()))


if __name__ == "__main__":
    main()
