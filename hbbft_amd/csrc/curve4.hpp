// G1 point arithmetic on a QUAD of lanes (4 aligned lanes of a wave that hold the same points):
// the Fq products of one doubling / addition issued as rounds of independent products, one per
// lane, exchanged by DPP quad_perm broadcasts (a VALU move per limb, no LDS).
//
// Why.  The Lagrange combine (k_combine: interpolate, honey_badger.rs:340 via threshold_crypto
// PublicKeySet::decrypt) is a latency chain: each lane runs a 128-bit scalar multiplication
// (124 doublings + ~45 additions, ~1,500 dependent Fq products) while most of the chip idles, and
// one wave's product costs its full instruction stream whatever the number of lanes that need it.
// On a quad the doubling (dbl-2009-l) is 3 rounds instead of 7 products and the addition
// (add-2007-bl) 5 rounds instead of 16; the lanes of a wave run 16 quads at once.
//
// Same formulas as curve.hpp g1_dbl_i / g1_add_i, so the coordinates are equal mod p (and, the
// products being fully reduced, equal).  Control flow must be quad-uniform (every lane of a quad
// holds the same values, so data-dependent branches are).
#pragma once
#include "curve.hpp"
#include "dpp.hpp"

namespace hbx {
#if defined(__HIPCC__)

// lane K of the calling lane's quad, to every lane of the quad
template <int K>
__device__ __forceinline__ fq fq_from_quad(const fq& v) {
  static_assert(K >= 0 && K < 4, "quad lane");
  dpp_guard_src<4, K>();
  fq r;
#pragma unroll
  for (int i = 0; i < 12; i++)
    r.l[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.l[i], K | (K << 2) | (K << 4) | (K << 6), 0xf, 0xf, false);
  return r;
}
__device__ __forceinline__ fq fq_sel4(int s, const fq& v0, const fq& v1, const fq& v2, const fq& v3) {
  fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = (s & 2) ? ((s & 1) ? v3.l[i] : v2.l[i]) : ((s & 1) ? v1.l[i] : v0.l[i]);
  return r;
}
// one round: lane s of the quad computes a_s b_s
__device__ __forceinline__ fq q4_round(int s, const fq& a0, const fq& b0, const fq& a1, const fq& b1, const fq& a2,
                                       const fq& b2, const fq& a3, const fq& b3) {
  return fq_mul_inl(fq_sel4(s, a0, a1, a2, a3), fq_sel4(s, b0, b1, b2, b3));
}

// dbl-2009-l: round 1 A = X^2, B = Y^2, Y Z; round 2 C = B^2, (X + B)^2, F = E^2; round 3 E (D - X3)
// (every lane computes it: no exchange)
__device__ __forceinline__ g1j g1_dbl_q4(const g1j& p, int s) {
  fq r = q4_round(s, p.x, p.x, p.y, p.y, p.y, p.z, p.y, p.z);
  const fq A = fq_from_quad<0>(r), B = fq_from_quad<1>(r), YZ = fq_from_quad<2>(r);
  const fq E = fq_add(fq_dbl(A), A);
  const fq XB = fq_add(p.x, B);
  r = q4_round(s, B, B, XB, XB, E, E, E, E);
  const fq C = fq_from_quad<0>(r), T = fq_from_quad<1>(r), F = fq_from_quad<2>(r);
  const fq D = fq_dbl(fq_sub(fq_sub(T, A), C));
  const fq X3 = fq_sub(F, fq_dbl(D));
  const fq C8 = fq_dbl(fq_dbl(fq_dbl(C)));
  const fq Y3 = fq_sub(fq_mul_inl(E, fq_sub(D, X3)), C8);
  return g1j{X3, Y3, fq_dbl(YZ)};
}

// add-2007-bl (complete for identities and P == +-Q, like g1_add_i):
//   round 1 Z1Z1, Z2Z2, Y1 Z2, Y2 Z1;  round 2 U1, U2, S1, S2;  round 3 I = (2H)^2, r^2, (Z1 + Z2)^2;
//   round 4 J = H I, V = U1 I, Z3;  round 5 r (V - X3), S1 J
__device__ __forceinline__ g1j g1_add_q4(const g1j& p, const g1j& q, int s) {
  if (g1j_is_identity(p)) return q;
  if (g1j_is_identity(q)) return p;
  fq r = q4_round(s, p.z, p.z, q.z, q.z, p.y, q.z, q.y, p.z);
  const fq Z1Z1 = fq_from_quad<0>(r), Z2Z2 = fq_from_quad<1>(r), Y1Z2 = fq_from_quad<2>(r), Y2Z1 = fq_from_quad<3>(r);
  r = q4_round(s, p.x, Z2Z2, q.x, Z1Z1, Y1Z2, Z2Z2, Y2Z1, Z1Z1);
  const fq U1 = fq_from_quad<0>(r), U2 = fq_from_quad<1>(r), S1 = fq_from_quad<2>(r), S2 = fq_from_quad<3>(r);
  if (fq_eq(U1, U2)) {
    if (fq_eq(S1, S2)) return g1_dbl_q4(p, s);
    return g1_identity();
  }
  const fq H = fq_sub(U2, U1);
  const fq H2 = fq_dbl(H);
  const fq rr = fq_dbl(fq_sub(S2, S1));
  const fq ZS = fq_add(p.z, q.z);
  r = q4_round(s, H2, H2, rr, rr, ZS, ZS, ZS, ZS);
  const fq I = fq_from_quad<0>(r), RR = fq_from_quad<1>(r), ZZ = fq_from_quad<2>(r);
  const fq Zt = fq_sub(fq_sub(ZZ, Z1Z1), Z2Z2);
  r = q4_round(s, H, I, U1, I, Zt, H, Zt, H);
  const fq J = fq_from_quad<0>(r), V = fq_from_quad<1>(r), Z3 = fq_from_quad<2>(r);
  const fq X3 = fq_sub(fq_sub(RR, J), fq_dbl(V));
  r = q4_round(s, rr, fq_sub(V, X3), S1, J, S1, J, S1, J);
  const fq Y3 = fq_sub(fq_from_quad<0>(r), fq_dbl(fq_from_quad<1>(r)));
  return g1j{X3, Y3, Z3};
}

// g1_mul_u128_w4 (curve.hpp) on a quad: the same 4-bit fixed window, table and digit order
__device__ __noinline__ g1j g1_mul_u128_w4_q4(const g1a& P, const uint32_t* k4, int s) {
  g1j tab[16];
  tab[0] = g1_identity();
  tab[1] = g1_from_affine(P);
#pragma unroll 1
  for (int i = 2; i < 16; i++) tab[i] = g1_add_q4(tab[i - 1], tab[1], s);
  g1j acc = tab[k4[3] >> 28];
  g1j nxt = tab[(k4[3] >> 24) & 0xFu];
#pragma unroll 1
  for (int w = 30; w >= 0; w--) {
    const g1j cur = nxt;
    if (w > 0) nxt = tab[(k4[(w - 1) >> 3] >> (((w - 1) & 7) * 4)) & 0xFu];
#pragma unroll 1
    for (int q = 0; q < 4; q++) acc = g1_dbl_q4(acc, s);
    acc = g1_add_q4(acc, cur, s);
  }
  return acc;
}

#endif  // __HIPCC__
}  // namespace hbx
