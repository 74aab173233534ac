"""CPU restatement (TEST INFRASTRUCTURE ONLY -- the product never imports this) of threshold_crypto's
symmetric bivariate polynomials as SyncKeyGen uses them (reference src/sync_key_gen.rs):

* BivarPoly of degree t over Fr with a_ij = a_ji; its commitment C_ij = g1 * a_ij
  (`our_part.commitment()`, sync_key_gen.rs:291);
* BivarCommitment::row(x) = the univariate commitment R_j = sum_i C_ij x^i
  (`commit.row(idx + 1)`, :313 and :401);
* BivarCommitment::evaluate(x, y) = sum_ij C_ij x^i y^j, compared with g1 * val in handle_ack
  (`part.commit.evaluate(our_idx + 1, sender_idx + 1) != G1Affine::one().mul(val)`, :449).

threshold_crypto (un-vendored, git dependency without a pinned revision, reference Cargo.toml:35)
stores the coefficients of the symmetric matrix once, at coeff_pos(i, j) = j (j + 1) / 2 + i for
i <= j; that index order is what the batch API takes ("parity unpinned" for the order: the crate
source is not available here; the evaluated points do not depend on it).
"""
from __future__ import annotations

from . import bls12_381 as bls


def coeff_pos(i: int, j: int) -> int:
    if i > j:
        i, j = j, i
    return j * (j + 1) // 2 + i


def n_coeffs(t: int) -> int:
    return (t + 1) * (t + 2) // 2


class BivarPoly:
    def __init__(self, t: int, coeff):
        assert len(coeff) == n_coeffs(t)
        self.t = t
        self.coeff = [c % bls.R for c in coeff]

    def a(self, i: int, j: int) -> int:
        return self.coeff[coeff_pos(i, j)]

    def evaluate(self, x: int, y: int) -> int:
        r = 0
        for i in range(self.t + 1):
            for j in range(self.t + 1):
                r += self.a(i, j) * pow(x, i, bls.R) * pow(y, j, bls.R)
        return r % bls.R

    def commitment(self):
        return [bls.g1_mul(bls.G1_GEN, c) for c in self.coeff]


def row(commit, t: int, x: int):
    """R_j = sum_i C_ij x^i, j = 0..t (BivarCommitment::row)."""
    out = []
    for j in range(t + 1):
        acc = None
        for i in range(t, -1, -1):  # Horner in x
            acc = bls.g1_add(bls.g1_mul(acc, x) if acc is not None else None, commit[coeff_pos(i, j)])
        out.append(acc)
    return out


def evaluate(commit, t: int, x: int, y: int):
    """sum_ij C_ij x^i y^j = sum_j R_j(x) y^j (BivarCommitment::evaluate)."""
    acc = None
    for rj in reversed(row(commit, t, x)):
        acc = bls.g1_add(bls.g1_mul(acc, y) if acc is not None else None, rj)
    return acc
