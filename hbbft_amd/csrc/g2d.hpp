// G2 point arithmetic in the signed-digit tower (fieldd.hpp), for the coin's Lagrange combine
// (k_combine_sigs, common_coin.rs:190 -> PublicKeySet::combine_signatures).
//
// curve.hpp g2_dbl / g2_add / g2_add_mixed / g2_mul_u64_w4 with the same formulas (dbl-2009-l,
// add-2007-bl, madd-2007-bl) and the same Jacobian points out -- only the coordinates' register
// form differs: a doubling is 2M + 5S of fq2d products (one fused column loop each) plus
// carry-free additions, instead of 12-limb products with carry chains (about half the VALU
// instructions; the combine's G2 half is a 64-step doubling chain per lane).
//
// Coordinates are "reduced" (fqd_reduce outputs or product outputs), so any two of them may be
// summed into a product operand.  Special cases (identity operands, equal or opposite points) are
// decided by EXACT tests mod p (fqd_is_zero_mod), as curve.hpp decides them with fq2_eq.
#pragma once
#include "pairingd.hpp"

namespace hbx {

// k p in normalised digit form (digits 0..12 in [0, 2^28), digit 13 signed), k = -2..3
struct fqd_kp_table {
  int32_t d[6][14];
};
constexpr fqd_kp_table make_kp_table() {
  fqd_kp_table t{};
  for (int k = -2; k <= 3; k++) {
    int64_t c = 0;
    for (int i = 0; i < 13; i++) {
      const int64_t v = (int64_t)k * (int64_t)FQ_P28[i] + c;
      const int64_t lo = v & (int64_t)DMASK;
      t.d[k + 2][i] = (int32_t)lo;
      c = (v - lo) / (int64_t)DN;
    }
    t.d[k + 2][13] = (int32_t)((int64_t)k * (int64_t)FQ_P28[13] + c);
  }
  return t;
}
HBX_CONST fqd_kp_table FQD_KP = make_kp_table();

// a == 0 mod p, exactly, for any digit vector with |digits| < 2^31: fqd_reduce brings the value
// into (-1.3 p, 2.3 p) with a unique normalised digit form, which is then compared with that of
// k p for k = -2..3 (a margin of one multiple either side).
HBX_HD bool fqd_is_zero_mod(const fqd& a) {
  const fqd r = fqd_reduce(a);
  bool z = false;
#pragma unroll
  for (int k = 0; k < 6; k++) {
    uint32_t diff = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) diff |= (uint32_t)(r.d[i] ^ FQD_KP.d[k][i]);
    z |= diff == 0;
  }
  return z;
}
HBX_HD bool fq2d_is_zero_mod(const fq2d& a) { return fqd_is_zero_mod(a.c0) && fqd_is_zero_mod(a.c1); }

HBX_HD g2jd g2d_identity() {
  const fq2d one{fqd_const(FQD_ONE), fqd_zero()};
  return g2jd{one, one, fq2d{fqd_zero(), fqd_zero()}};
}

// The point formulas below take their Fq2 products from a policy M (m.mul, m.sqr); g2d_one runs
// every product on the calling lane.  (A lane-pair policy -- each Fq2 product split by output
// component over two lanes, halves swapped by DPP -- was measured in k_combine_sigs and lost: the
// two waves per SIMD it needs leave 256 VGPRs, which spilled.)
struct g2d_one {
  HBX_HD fq2d mul(const fq2d& a, const fq2d& b) const { return fq2d_mul(a, b); }
  HBX_HD fq2d sqr(const fq2d& a) const { return fq2d_sqr(a); }
};

// 2T (curve.hpp g2_dbl; pairingd.hpp line_dbl_step_di without the line)
template <class M>
HBX_HD g2jd g2d_dbl_t(const g2jd& T, const M& m) {
  const fq2d A = m.sqr(T.x);
  const fq2d B = m.sqr(T.y);
  const fq2d C = m.sqr(B);
  const fq2d D = fq2d_reduce(fq2d_dbl(fq2d_sub(fq2d_sub(m.sqr(fq2d_add(T.x, B)), A), C)));
  const fq2d E = fq2d_norm(fq2d_add(fq2d_dbl(A), A));
  const fq2d F = m.sqr(E);
  const fq2d X3 = fq2d_reduce(fq2d_sub(F, fq2d_dbl(D)));
  const fq2d C8 = fq2d_dbl(fq2d_reduce(fq2d_dbl(fq2d_dbl(C))));
  const fq2d Y3 = fq2d_reduce(fq2d_sub(m.mul(E, fq2d_sub(D, X3)), C8));
  const fq2d Z3 = fq2d_reduce(fq2d_dbl(m.mul(T.y, T.z)));
  return g2jd{X3, Y3, Z3};
}

// T + (qx, qy) for an affine point, T != +-Q and T != O (curve.hpp g2_add_mixed's general branch)
template <class M>
HBX_HD g2jd g2d_add_mixed_nc_t(const g2jd& T, const fq2d& qx, const fq2d& qy, const M& m) {
  const fq2d Z1Z1 = m.sqr(T.z);
  const fq2d U2 = m.mul(qx, Z1Z1);
  const fq2d S2 = m.mul(m.mul(qy, T.z), Z1Z1);
  const fq2d H = fq2d_sub(U2, T.x);
  const fq2d HH = m.sqr(H);
  const fq2d I = fq2d_reduce(fq2d_dbl(fq2d_dbl(HH)));
  const fq2d J = m.mul(H, I);
  const fq2d r = fq2d_reduce(fq2d_dbl(fq2d_sub(S2, T.y)));
  const fq2d V = m.mul(T.x, I);
  const fq2d X3 = fq2d_reduce(fq2d_sub(fq2d_sub(m.sqr(r), J), fq2d_dbl(V)));
  const fq2d Y3 = fq2d_reduce(fq2d_sub(m.mul(r, fq2d_sub(V, X3)), fq2d_dbl(m.mul(T.y, J))));
  const fq2d Z3 = fq2d_reduce(fq2d_sub(fq2d_sub(m.sqr(fq2d_norm(fq2d_add(T.z, H))), Z1Z1), HH));
  return g2jd{X3, Y3, Z3};
}

// The general branch of add-2007-bl (curve.hpp g2_add) with its intermediate values; `p + q`
// when H != 0.  U1, S1, S2 and H are returned for the special-case tests.
struct g2d_add_parts {
  fq2d Z1Z1, Z2Z2, U1, S1, S2, H;
};
template <class M>
HBX_HD g2d_add_parts g2d_add_prep(const g2jd& p, const g2jd& q, const M& m) {
  g2d_add_parts s;
  s.Z1Z1 = m.sqr(p.z);
  s.Z2Z2 = m.sqr(q.z);
  s.U1 = m.mul(p.x, s.Z2Z2);
  const fq2d U2 = m.mul(q.x, s.Z1Z1);
  s.S1 = m.mul(m.mul(p.y, q.z), s.Z2Z2);
  s.S2 = m.mul(m.mul(q.y, p.z), s.Z1Z1);
  s.H = fq2d_sub(U2, s.U1);
  return s;
}
template <class M>
HBX_HD g2jd g2d_add_finish(const g2jd& p, const g2jd& q, const g2d_add_parts& s, const M& m) {
  const fq2d I = fq2d_reduce(fq2d_dbl(fq2d_dbl(m.sqr(s.H))));  // (2H)^2
  const fq2d J = m.mul(s.H, I);
  const fq2d r = fq2d_reduce(fq2d_dbl(fq2d_sub(s.S2, s.S1)));
  const fq2d V = m.mul(s.U1, I);
  const fq2d X3 = fq2d_reduce(fq2d_sub(fq2d_sub(m.sqr(r), J), fq2d_dbl(V)));
  const fq2d Y3 = fq2d_reduce(fq2d_sub(m.mul(r, fq2d_sub(V, X3)), fq2d_dbl(m.mul(s.S1, J))));
  const fq2d Zs = fq2d_reduce(fq2d_sub(fq2d_sub(m.sqr(fq2d_norm(fq2d_add(p.z, q.z))), s.Z1Z1), s.Z2Z2));
  const fq2d Z3 = m.mul(Zs, s.H);
  return g2jd{X3, Y3, Z3};
}
// p + q, neither the identity and p != +-q (the window additions of g2d_mul_u64_w4)
template <class M>
HBX_HD g2jd g2d_add_nc_t(const g2jd& p, const g2jd& q, const M& m) {
  return g2d_add_finish(p, q, g2d_add_prep(p, q, m), m);
}

// p + q for any two points (curve.hpp g2_add): identity operands, p = q (doubling) and p = -q
// (identity) by exact tests.
template <class M>
HBX_HD g2jd g2d_add_t(const g2jd& p, const g2jd& q, const M& m) {
  if (fq2d_is_zero_mod(p.z)) return q;
  if (fq2d_is_zero_mod(q.z)) return p;
  const g2d_add_parts s = g2d_add_prep(p, q, m);
  if (fq2d_is_zero_mod(s.H)) {
    if (fq2d_is_zero_mod(fq2d_sub(s.S2, s.S1))) return g2d_dbl_t(p, m);
    return g2d_identity();
  }
  return g2d_add_finish(p, q, s, m);
}

// k P for a 64-bit k and an affine P = (px, py) in G2 (normalised digits), by 4-bit fixed windows
// (curve.hpp g2_mul_u64_w4's schedule): a table (1..15) P in per-lane scratch, then 15 x (4
// doublings + 1 addition).  P has prime order r > 2^64, so every window addition adds m P and
// n P with 16 <= m, 1 <= n <= 15, m + n < r: never equal or opposite points, and the accumulator
// is the identity exactly while the scalar's leading windows are zero -- a flag, not a test.
// inf is set when k = 0.  The doubling and addition are out-of-line calls (DBL, ADD, MADD).
template <class DBL, class ADD, class MADD>
HBX_HD g2jd g2d_mul_u64_w4_t(const fq2d& px, const fq2d& py, uint64_t k, bool& inf, DBL dbl, ADD add, MADD madd) {
  g2jd tab[16];
  tab[0] = g2d_identity();
  tab[1] = g2jd{px, py, fq2d{fqd_const(FQD_ONE), fqd_zero()}};
  tab[2] = dbl(tab[1]);
#pragma unroll 1
  for (int i = 3; i < 16; i++) tab[i] = madd(tab[i - 1], px, py);
  const uint32_t top = (uint32_t)(k >> 60);
  g2jd acc = tab[top];
  bool ai = top == 0;
#pragma unroll 1
  for (int w = 14; w >= 0; w--) {
    const uint32_t nib = (uint32_t)(k >> (4 * w)) & 0xFu;
    if (!ai) {
#pragma unroll 1
      for (int q = 0; q < 4; q++) acc = dbl(acc);
    }
    if (nib) {
      acc = ai ? tab[nib] : add(acc, tab[nib]);
      ai = false;
    }
  }
  inf = ai;
  return acc;
}

// one lane per point operation
HBX_HDNI g2jd g2d_dbl(const g2jd& T) { return g2d_dbl_t(T, g2d_one{}); }
HBX_HDNI g2jd g2d_add_mixed_nc(const g2jd& T, const fq2d& qx, const fq2d& qy) {
  return g2d_add_mixed_nc_t(T, qx, qy, g2d_one{});
}
HBX_HDNI g2jd g2d_add_nc(const g2jd& p, const g2jd& q) { return g2d_add_nc_t(p, q, g2d_one{}); }
HBX_HDNI g2jd g2d_add(const g2jd& p, const g2jd& q) { return g2d_add_t(p, q, g2d_one{}); }
#ifndef HBX_G2D_W4_INLINE_DBL
#define HBX_G2D_W4_INLINE_DBL 1  // 1: the doublings inlined (combine 4.03 -> 3.71 ms), 2: the window additions too (3.70: not worth the code)
#endif
HBX_HDNI g2jd g2d_mul_u64_w4(const fq2d& px, const fq2d& py, uint64_t k, bool& inf) {
  return g2d_mul_u64_w4_t(
      px, py, k, inf,
      [](const g2jd& a) __attribute__((always_inline)) {
#if HBX_G2D_W4_INLINE_DBL
        return g2d_dbl_t(a, g2d_one{});  // the doublings inlined in the window loop: no call frame
#else
        return g2d_dbl(a);
#endif
      },
      [](const g2jd& a, const g2jd& b) __attribute__((always_inline)) {
#if HBX_G2D_W4_INLINE_DBL >= 2
        return g2d_add_nc_t(a, b, g2d_one{});
#else
        return g2d_add_nc(a, b);
#endif
      },
      [](const g2jd& a, const fq2d& x, const fq2d& y) { return g2d_add_mixed_nc(a, x, y); });
}


HBX_HD g2j g2jd_to_g2j(const g2jd& a) { return g2j{fq2d_to_fq2(a.x), fq2d_to_fq2(a.y), fq2d_to_fq2(a.z)}; }

}  // namespace hbx
