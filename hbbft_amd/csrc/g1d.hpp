// G1 decode and subgroup check in the signed-digit tower (fieldd.hpp) for the decode kernels: every received
// decryption share, U_j and the key shares are checked for membership in G1 at deserialisation
// (pairing 0.14's into_affine).  At N = 256 that is 65,536 checks in the
// epoch's prepare launch, whose share-decode half (3.7 ms) had become slower than its hash chains.
//
// curve.hpp g1_is_torsion_free's criterion and schedule -- phi'(P) == -[x^2] P (eprint 2021/1130
// sec. 6), one double-and-add over the 128-bit x^2 -- with the point arithmetic on 14-digit
// coordinates: carry-free additions and one parallel carry step (fqd_relax) where a digit bound
// needs it.  The double-and-add meets special cases for points outside G1 (a point of small order
// returns to +-P or to the identity), so the addition decides them by exact tests mod p
// (g2d.hpp fqd_is_zero_mod), as g1_add_mixed_i does with fq_is_zero.
#pragma once
#include "g2d.hpp"

namespace hbx {

struct g1jd {
  fqd x, y, z;
};

// 2P, dbl-2009-l (curve.hpp g1_dbl_i); relaxed in and out
HBX_HD g1jd g1d_dbl(const g1jd& p) {
  const fqd A = fqd_sqr(p.x);
  const fqd B = fqd_sqr(p.y);
  const fqd C = fqd_sqr(B);
  const fqd D = fqd_dbl(fqd_relax(fqd_sub(fqd_sub(fqd_sqr(fqd_add(p.x, B)), A), C)));
  const fqd E = fqd_relax(fqd_add(fqd_dbl(A), A));
  const fqd F = fqd_sqr(E);
  const fqd X3 = fqd_relax(fqd_sub(F, fqd_dbl(D)));
  const fqd C8 = fqd_dbl(fqd_dbl(fqd_dbl(C)));
  const fqd Y3 = fqd_relax(fqd_sub(fqd_mul(E, fqd_sub(D, X3)), C8));
  const fqd Z3 = fqd_relax(fqd_dbl(fqd_mul(p.y, p.z)));
  return g1jd{X3, Y3, Z3};
}

// p + (qx, qy) for an affine q, madd-2007-bl (curve.hpp g1_add_mixed_i) with its special cases:
// p = O gives q, p = q doubles, p = -q gives O (exact tests)
HBX_HD g1jd g1d_add_mixed(const g1jd& p, const fqd& qx, const fqd& qy) {
  const fqd one = fqd_const(FQD_ONE);
  if (fqd_is_zero_mod(p.z)) return g1jd{qx, qy, one};
  const fqd Z1Z1 = fqd_sqr(p.z);
  const fqd U2 = fqd_mul(qx, Z1Z1);
  const fqd S2 = fqd_mul(fqd_mul(qy, p.z), Z1Z1);
  const fqd H = fqd_relax(fqd_sub(U2, p.x));
  const fqd rh = fqd_relax(fqd_sub(S2, p.y));  // r / 2
  if (fqd_is_zero_mod(H)) {
    if (fqd_is_zero_mod(rh)) return g1d_dbl(p);
    return g1jd{one, one, fqd_zero()};
  }
  const fqd r = fqd_dbl(rh);
  const fqd HH = fqd_sqr(H);
  const fqd I = fqd_dbl(fqd_dbl(HH));
  const fqd J = fqd_mul(H, I);
  const fqd V = fqd_mul(p.x, I);
  const fqd X3 = fqd_relax(fqd_sub(fqd_sub(fqd_sqr(r), J), fqd_dbl(V)));
  const fqd Y3 = fqd_relax(fqd_sub(fqd_mul(r, fqd_sub(V, X3)), fqd_dbl(fqd_mul(p.y, J))));
  const fqd Z3 = fqd_relax(fqd_sub(fqd_sub(fqd_sqr(fqd_relax(fqd_add(p.z, H))), Z1Z1), HH));
  return g1jd{X3, Y3, Z3};
}

// p + q, add-2007-bl (curve.hpp g1_add_i) without its special cases: for operands that are
// neither the identity nor equal or opposite (the window additions below).  Relaxed in and out.
HBX_HD g1jd g1d_add_nc(const g1jd& p, const g1jd& q) {
  const fqd Z1Z1 = fqd_sqr(p.z);
  const fqd Z2Z2 = fqd_sqr(q.z);
  const fqd U1 = fqd_mul(p.x, Z2Z2);
  const fqd U2 = fqd_mul(q.x, Z1Z1);
  const fqd S1 = fqd_mul(fqd_mul(p.y, q.z), Z2Z2);
  const fqd S2 = fqd_mul(fqd_mul(q.y, p.z), Z1Z1);
  const fqd H = fqd_relax(fqd_sub(U2, U1));
  const fqd I = fqd_sqr(fqd_dbl(H));
  const fqd J = fqd_mul(H, I);
  const fqd r = fqd_dbl(fqd_relax(fqd_sub(S2, S1)));
  const fqd V = fqd_mul(U1, I);
  const fqd X3 = fqd_relax(fqd_sub(fqd_sub(fqd_sqr(r), J), fqd_dbl(V)));
  const fqd Y3 = fqd_relax(fqd_sub(fqd_mul(r, fqd_sub(V, X3)), fqd_dbl(fqd_mul(S1, J))));
  const fqd Z3 = fqd_mul(fqd_relax(fqd_sub(fqd_sub(fqd_sqr(fqd_relax(fqd_add(p.z, q.z))), Z1Z1), Z2Z2)), H);
  return g1jd{X3, Y3, Z3};
}

// curve.hpp g1_mul_u128_w4 (the threshold combine's GLV halves: 4-bit fixed windows, the table
// (1..15) P in per-lane scratch) with the point arithmetic in the digit tower.  P has prime order
// r > 2^128, so a window addition adds m P and n P with 16 <= m, 1 <= n <= 15, m + n < r: never
// equal or opposite points; the accumulator is the identity exactly while the scalar's leading
// windows are zero (a flag, as g2d.hpp g2d_mul_u64_w4_t does).  The same point as the 12-limb
// version (tests/test_hostcheck.py::test_g1_mul_u128_digit_tower).
HBX_HDNI g1j g1d_mul_u128_w4(const g1a& P, const uint32_t* k4) {
  if (P.inf) return g1_identity();
  const fqd px = fqd_from_fq(P.x), py = fqd_from_fq(P.y);
  g1jd tab[16];
  tab[0] = g1jd{fqd_const(FQD_ONE), fqd_const(FQD_ONE), fqd_zero()};
  tab[1] = g1jd{px, py, fqd_const(FQD_ONE)};
#pragma unroll 1
  for (int i = 2; i < 16; i++) tab[i] = g1d_add_mixed(tab[i - 1], px, py);
  const uint32_t top = k4[3] >> 28;
  g1jd acc = tab[top];
  bool ai = top == 0;
#pragma unroll 1
  for (int w = 30; w >= 0; w--) {
    const uint32_t nib = (k4[w >> 3] >> ((w & 7) * 4)) & 0xFu;
    if (!ai) {
#pragma unroll 1
      for (int q = 0; q < 4; q++) acc = g1d_dbl(acc);
    }
    if (nib) {
      acc = ai ? tab[nib] : g1d_add_nc(acc, tab[nib]);
      ai = false;
    }
  }
  if (ai) return g1_identity();
  return g1j{fqd_to_fq(acc.x), fqd_to_fq(acc.y), fqd_to_fq(acc.z)};
}

// P in G1 for an affine point on the curve (curve.hpp g1_is_torsion_free, the same criterion)
HBX_HDNI bool g1_is_torsion_free_d(const g1a& P) {
  if (P.inf) return true;
  const fqd px = fqd_from_fq(P.x), py = fqd_from_fq(P.y);
  g1jd acc{fqd_const(FQD_ONE), fqd_const(FQD_ONE), fqd_zero()};
#pragma unroll 1
  for (int i = 127; i >= 0; i--) {
    acc = g1d_dbl(acc);
    if ((G1_X2[i >> 5] >> (i & 31)) & 1) acc = g1d_add_mixed(acc, px, py);
  }
  if (fqd_is_zero_mod(acc.z)) return false;  // phi'(P) is never O for P != O
  // (beta^2 x_P, y_P) == -(X/Z^2, Y/Z^3)  <=>  X == beta^2 x_P Z^2  and  Y == -y_P Z^3
  const fqd z2 = fqd_sqr(acc.z);
  const fqd z3 = fqd_mul(z2, acc.z);
  const fqd bx = fqd_mul(px, fqd_from_fq(fq_from_const(G1_BETA2)));
  return fqd_is_zero_mod(fqd_sub(acc.x, fqd_mul(bx, z2))) && fqd_is_zero_mod(fqd_add(acc.y, fqd_mul(py, z3)));
}

// curve.hpp g1_decompress with the square root in the digit tower (fieldd.hpp fq_sqrt_d: the same
// root, tests/test_hostcheck.py::test_digit_tower_square_roots)
HBX_HDNI int32_t g1_decompress_d(const uint8_t* b48, g1a& out) {
  return g1_decompress_t(b48, out, [](const fq& a, fq& y) { return fq_sqrt_d(a, y); });
}

}  // namespace hbx
