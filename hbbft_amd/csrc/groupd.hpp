// G2 arithmetic on a lane GROUP in the signed-digit tower (fieldd.hpp) for the latency-bound
// chains: hash-to-G2's cofactor clearing (hash.hpp hash_g2_group), as hash.hpp's g2_dbl_group /
// g2_add_group rounds with 14-digit operands.
//
// Why (tools/microbench/dblstamp.hip, profiles/r05m_dblstamp.txt): in one 12-limb group doubling
// the three Fq products take 30 % of the time and the modular additions, selects and broadcasts
// between them 70 % -- each 12-limb addition is two dependent carry chains (24 steps) plus a
// select, and a chain runs on one wave, so every dependent step is paid in full.  Here an addition
// is one digit-wise VALU level, and the only normalisation is fqd_relax: ONE parallel carry step
// (digits back under 2^28 + 8, the value kept), three VALU levels instead of fqd_norm's 13-step
// carry chain or fqd_reduce's.  No value reduction is needed: every coordinate of a group operation's
// output is a combination of a few product outputs with small coefficients, so values stay below
// ~32 p, far inside a product's input range (|a b| < p 2^392).  One doubling: 11.4 -> 6.5 us, the
// same points after 4,096 doublings (tools/microbench/dbld.hip, profiles/r05n_dbld.txt).
//
// "Relaxed" below: digits in (-2^28 - 8, 2^28 + 8), value below 2^386.  Product operands are relaxed
// values or sums of two; anything larger is relaxed first.  The special cases of an addition
// (identity operands, equal or opposite points) are decided by exact tests mod p (g2d.hpp
// fqd_is_zero_mod), group-uniformly.
#pragma once
#include "g2d.hpp"
#include "dpp.hpp"

namespace hbx {
#if defined(__HIPCC__)

// lane K of the calling lane's 16-lane row, to every lane of the row (DPP row_newbcast per digit).
// Each moved digit is pinned in a register (HBX_LAUNDER) so the compiler cannot fold the move into
// its consumer as a DPP-modified add / subtract: in the group addition such folded row_newbcast
// operations produced wrong sums on gfx950 (tools/microbench/addcmp.hip: Y1 Z2 differed from the
// same expression outside the function; with the moves pinned both agree and the hash-to-G2
// checksum of profiles/r05o_hashg2.txt is reproduced).
#ifndef HBX_ROW_PIN
#define HBX_ROW_PIN 1  // 0 only in tools/microbench/dppfold.hip's reproduction of the fold
#endif
template <int K>
__device__ __forceinline__ fqd fqd_from_row(const fqd& v) {
  static_assert(K >= 0 && K < 16, "row lane");
  dpp_guard_src<16, K>();
  fqd r;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    r.d[i] = __builtin_amdgcn_update_dpp(0, v.d[i], 0x150 + K, 0xf, 0xf, false);
#if HBX_ROW_PIN
    __asm__("" : "+v"(r.d[i]));  // (not HBX_LAUNDER: pinned in every unit, HBX_NO_LAUNDER ones too)
#endif
  }
  return r;
}
__device__ __forceinline__ fqd fqd_sel8(int s, const fqd& v0, const fqd& v1, const fqd& v2, const fqd& v3, const fqd& v4,
                                        const fqd& v5, const fqd& v6, const fqd& v7) {
  fqd r;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const int32_t lo = (s & 2) ? ((s & 1) ? v3.d[i] : v2.d[i]) : ((s & 1) ? v1.d[i] : v0.d[i]);
    const int32_t hi = (s & 2) ? ((s & 1) ? v7.d[i] : v6.d[i]) : ((s & 1) ? v5.d[i] : v4.d[i]);
    r.d[i] = (s & 4) ? hi : lo;
  }
  return r;
}
// One product round on a 16-lane group from eight two-lane blocks: block b (lanes 2b, 2b + 1) is
// a square of X_b (SQ bit b set: lanes ((a0 + a1)(a0 - a1), a0 a1)) or half of a schoolbook product
// X_b Y_b spanning the 4-aligned blocks 2c, 2c + 1 (lanes a0 b0, a1 b1, a0 b1, a1 b0).  A lane first
// selects its block's X and Y among values that are live anyway (a three-level select tree, like
// the doubling's fqd_sel8), then forms its operands: a 16-entry candidate list per operand -- the
// square sums materialised for every block -- held ~450 registers at once and spilled (~600
// scratch accesses per addition).
__device__ __forceinline__ fq2d fq2d_sel8(int s, const fq2d& v0, const fq2d& v1, const fq2d& v2, const fq2d& v3,
                                          const fq2d& v4, const fq2d& v5, const fq2d& v6, const fq2d& v7) {
  return fq2d{fqd_sel8(s, v0.c0, v1.c0, v2.c0, v3.c0, v4.c0, v5.c0, v6.c0, v7.c0),
              fqd_sel8(s, v0.c1, v1.c1, v2.c1, v3.c1, v4.c1, v5.c1, v6.c1, v7.c1)};
}
template <uint32_t SQ>
__device__ __forceinline__ fqd gd_round(int gl, const fq2d& x0, const fq2d& x1, const fq2d& x2, const fq2d& x3,
                                        const fq2d& x4, const fq2d& x5, const fq2d& x6, const fq2d& x7,
                                        const fq2d& y0, const fq2d& y1, const fq2d& y2, const fq2d& y3,
                                        const fq2d& y4, const fq2d& y5, const fq2d& y6, const fq2d& y7) {
  const int blk = (gl >> 1) & 7, sub = gl & 3;
  const bool sq = ((SQ >> blk) & 1) != 0;
  const fq2d X = fq2d_sel8(blk, x0, x1, x2, x3, x4, x5, x6, x7);
  const fq2d Y = fq2d_sel8(blk, y0, y1, y2, y3, y4, y5, y6, y7);
  fqd a, b;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const int32_t x0d = X.c0.d[i], x1d = X.c1.d[i], y0d = Y.c0.d[i], y1d = Y.c1.d[i];
    // square lanes: (x0 + x1, x0 - x1) | (x0, x1); product lanes: (x0, y0) (x1, y1) (x0, y1) (x1, y0)
    a.d[i] = sq ? ((gl & 1) ? x0d : x0d + x1d) : ((sub & 1) ? x1d : x0d);
    b.d[i] = sq ? ((gl & 1) ? x1d : x0d - x1d) : ((sub == 1 || sub == 2) ? y1d : y0d);
  }
  return fqd_mul(a, b);
}

// Fq2 results of a round: a square from rows (K, K + 1) = ((a0 + a1)(a0 - a1), a0 a1), a product
// from rows (K .. K + 3) = (a0 b0, a1 b1, a0 b1, a1 b0) (schoolbook).  Digits below 2^29.
template <int K>
__device__ __forceinline__ fq2d rows_sqr(const fqd& r) {
  return fq2d{fqd_from_row<K>(r), fqd_dbl(fqd_from_row<K + 1>(r))};
}
template <int K>
__device__ __forceinline__ fq2d rows_mul(const fqd& r) {
  return fq2d{fqd_sub(fqd_from_row<K>(r), fqd_from_row<K + 1>(r)), fqd_add(fqd_from_row<K + 2>(r), fqd_from_row<K + 3>(r))};
}

// 2P on the 8 (or 16) lanes of a group (hash.hpp g2_dbl_group, dbl-2009-l), lane s = gl & 7:
// three rounds, A = X^2, B = Y^2, Y Z; C = B^2, (X + B)^2, E^2; E (D - X3).  Relaxed in and out.
__device__ __forceinline__ g2jd g2d_dbl_group(const g2jd& p, int gl) {
  const int s = gl & 7;
  const fqd x0 = p.x.c0, x1 = p.x.c1, y0 = p.y.c0, y1 = p.y.c1, z0 = p.z.c0, z1 = p.z.c1;
  fqd r = fqd_mul(fqd_sel8(s, fqd_add(x0, x1), x0, fqd_add(y0, y1), y0, y0, y1, y0, y1),
                  fqd_sel8(s, fqd_sub(x0, x1), x1, fqd_sub(y0, y1), y1, z0, z1, z1, z0));
  const fq2d A = rows_sqr<0>(r), B = rows_sqr<2>(r), YZ = rows_mul<4>(r);
  const fq2d S = fq2d_relax(fq2d_add(p.x, B));
  const fq2d E = fq2d_relax(fq2d_add(fq2d_dbl(A), A));
  r = fqd_mul(fqd_sel8(s, fqd_add(B.c0, B.c1), B.c0, fqd_add(S.c0, S.c1), S.c0, fqd_add(E.c0, E.c1), E.c0, E.c0, E.c0),
              fqd_sel8(s, fqd_sub(B.c0, B.c1), B.c1, fqd_sub(S.c0, S.c1), S.c1, fqd_sub(E.c0, E.c1), E.c1, E.c1, E.c1));
  const fq2d C = rows_sqr<0>(r), T = rows_sqr<2>(r), F = rows_sqr<4>(r);
  const fq2d D = fq2d_dbl(fq2d_relax(fq2d_sub(fq2d_sub(T, A), C)));
  const fq2d X3 = fq2d_relax(fq2d_sub(F, fq2d_dbl(D)));
  const fq2d G = fq2d_sub(D, X3);
  r = fqd_mul(fqd_sel8(s, E.c0, E.c1, E.c0, E.c1, E.c0, E.c1, E.c0, E.c1),
              fqd_sel8(s, G.c0, G.c1, G.c1, G.c0, G.c0, G.c1, G.c1, G.c0));
  const fq2d EG = rows_mul<0>(r);
  const fq2d C8 = fq2d_dbl(fq2d_dbl(fq2d_relax(fq2d_dbl(C))));
  return g2jd{X3, fq2d_relax(fq2d_sub(EG, C8)), fq2d_relax(fq2d_dbl(YZ))};
}
__device__ __forceinline__ g2jd g2d_dbl_n_group(g2jd p, int n, int gl) {
  for (int i = 0; i < n; i++) p = g2d_dbl_group(p, gl);
  return p;
}

// P + Q on the 16 lanes of a group (hash.hpp g2_add_group, add-2007-bl) in five rounds, the same
// special cases as g2_add by exact tests.  Relaxed in and out.
__device__ __forceinline__ g2jd g2d_add_group_i(const g2jd& p, const g2jd& q, int gl) {
  if (fq2d_is_zero_mod(p.z)) return q;
  if (fq2d_is_zero_mod(q.z)) return p;
  const fq2d z{fqd_zero(), fqd_zero()};
  // round 1: Z1^2 (0, 1), Z2^2 (2, 3), Y1 Z2 (4..7), Y2 Z1 (8..11), (Z1 + Z2)^2 (12, 13)
  fqd r;
  {
    const fq2d zs = fq2d_relax(fq2d_add(p.z, q.z));
    r = gd_round<0x43>(gl, p.z, q.z, p.y, p.y, q.y, q.y, zs, z, p.z, q.z, q.z, q.z, p.z, p.z, zs, z);
  }
  const fq2d Z1Z1 = rows_sqr<0>(r), Z2Z2 = rows_sqr<2>(r);
  const fq2d Y1Z2 = rows_mul<4>(r), Y2Z1 = rows_mul<8>(r);
  const fq2d ZS = rows_sqr<12>(r);
  // round 2: U1 (0..3), U2 (4..7), S1 (8..11), S2 (12..15)
  r = gd_round<0>(gl, p.x, p.x, q.x, q.x, Y1Z2, Y1Z2, Y2Z1, Y2Z1, Z2Z2, Z2Z2, Z1Z1, Z1Z1, Z2Z2, Z2Z2, Z1Z1, Z1Z1);
  const fq2d U1 = rows_mul<0>(r), S1 = rows_mul<8>(r);
  const fq2d H = fq2d_relax(fq2d_sub(rows_mul<4>(r), U1));
  const fq2d dS = fq2d_relax(fq2d_sub(rows_mul<12>(r), S1));
  if (fq2d_is_zero_mod(H)) {
    if (fq2d_is_zero_mod(dS)) return g2d_dbl_group(p, gl);
    return g2d_identity();
  }
  const fq2d rr = fq2d_dbl(dS);
  // round 3: H^2 (0, 1), dS^2 (2, 3), ((Z1 + Z2)^2 - Z1Z1 - Z2Z2) H (4..7)
  {
    const fq2d zz = fq2d_relax(fq2d_sub(fq2d_sub(ZS, Z1Z1), Z2Z2));
    r = gd_round<0x03>(gl, H, dS, zz, zz, z, z, z, z, H, dS, H, H, z, z, z, z);
  }
  const fq2d I = fq2d_dbl(fq2d_relax(fq2d_dbl(rows_sqr<0>(r))));   // (2H)^2
  const fq2d RR = fq2d_dbl(fq2d_relax(fq2d_dbl(rows_sqr<2>(r))));  // rr^2
  const fq2d Z3 = fq2d_relax(rows_mul<4>(r));
  // round 4: J = H I (0..3), V = U1 I (4..7)
  r = gd_round<0>(gl, H, H, U1, U1, z, z, z, z, I, I, I, I, z, z, z, z);
  const fq2d J = rows_mul<0>(r), V = rows_mul<4>(r);
  const fq2d X3 = fq2d_relax(fq2d_sub(fq2d_relax(fq2d_sub(RR, J)), fq2d_dbl(V)));
  // round 5: rr (V - X3) (0..3), S1 J (4..7)
  {
    const fq2d w = fq2d_sub(V, X3);
    r = gd_round<0>(gl, rr, rr, S1, S1, z, z, z, z, w, w, J, J, z, z, z, z);
  }
  const fq2d Y3 = fq2d_relax(fq2d_sub(rows_mul<0>(r), fq2d_dbl(rows_mul<4>(r))));
  return g2jd{X3, Y3, Z3};
}
// one out-of-line copy for the clearing's few combining additions; the multiplication loop inlines
// its own (a call there saved and restored the caller's live point around every addition)
__device__ __noinline__ g2jd g2d_add_group(const g2jd& p, const g2jd& q, int gl) { return g2d_add_group_i(p, q, gl); }
__device__ __forceinline__ g2jd g2d_neg(const g2jd& p) { return g2jd{p.x, fq2d_neg(p.y), p.z}; }
__device__ __forceinline__ g2jd g2d_sub_group(const g2jd& p, const g2jd& q, int gl) { return g2d_add_group(p, g2d_neg(q), gl); }

// psi(X, Y, Z) = (C1 conj(X), C2 conj(Y), conj(Z)) (curve.hpp g2_psi), products on the calling lane
__device__ __forceinline__ g2jd g2d_psi(const g2jd& p) {
  const fq2d c1 = fq2d_from_fq2(fq2{fq_from_const(PSI_C1_0), fq_from_const(PSI_C1_1)});
  const fq2d c2 = fq2d_from_fq2(fq2{fq_from_const(PSI_C2_0), fq_from_const(PSI_C2_1)});
  return g2jd{fq2d_mul(fq2d_conj(p.x), c1), fq2d_mul(fq2d_conj(p.y), c2), fq2d_relax(fq2d_conj(p.z))};
}

// g2_mul_u64 / g2_mul_gls_d / g2_clear_cofactor (curve.hpp) with the group doubling and addition
__device__ __noinline__ g2jd g2d_mul_u64_group(const g2jd& p, uint64_t k, int gl) {
  g2jd acc = p;
  const int top = 63 - __builtin_clzll(k);
  for (int i = top - 1; i >= 0; i--) {
    acc = g2d_dbl_group(acc, gl);
    if ((k >> i) & 1) acc = g2d_add_group_i(acc, p, gl);
  }
  return acc;
}
__device__ __noinline__ g2jd g2d_mul_gls_d_group(const g2jd& P, int gl) {
  const g2jd P2 = g2d_dbl_group(P, gl);
  const g2jd P4 = g2d_dbl_group(P2, gl);
  g2jd Z = g2d_add_group(P4, P, gl);
  Z = g2d_add_group(g2d_dbl_n_group(Z, 4, gl), Z, gl);
  Z = g2d_add_group(g2d_dbl_n_group(Z, 8, gl), Z, gl);
  const g2jd W = g2d_add_group(g2d_dbl_group(Z, gl), P, gl);
  g2jd acc = g2d_add_group(g2d_dbl_n_group(P2, 3, gl), P, gl);
  acc = g2d_add_group(g2d_dbl_group(acc, gl), P, gl);
  acc = g2d_dbl_n_group(acc, 1 + 8 + 16, gl);
  acc = g2d_add_group(acc, Z, gl);
  acc = g2d_add_group(g2d_dbl_n_group(acc, 16, gl), Z, gl);
  return g2d_add_group(g2d_dbl_n_group(acc, 16, gl), W, gl);
}
// hash.hpp g2_clear_cofactor_group in the digit tower; full = false stops at Q = h_eff P
__device__ __noinline__ g2jd g2d_clear_cofactor_group(const g2jd& P, int gl, bool full) {
  const g2jd t1 = g2d_neg(g2d_mul_u64_group(P, BLS_X, gl));
  g2jd t2 = g2d_psi(P);
  g2jd t3 = g2d_psi(g2d_psi(g2d_dbl_group(P, gl)));
  t3 = g2d_sub_group(t3, t2, gl);
  t2 = g2d_add_group(t1, t2, gl);
  t2 = g2d_neg(g2d_mul_u64_group(t2, BLS_X, gl));
  t3 = g2d_add_group(t3, t2, gl);
  t3 = g2d_sub_group(t3, t1, gl);
  const g2jd Q = g2d_sub_group(t3, P, gl);
  if (!full) return Q;
  const g2jd q1 = g2d_psi(Q);
  const g2jd q2 = g2d_psi(q1);
  const g2jd q3 = g2d_psi(q2);
  const g2jd Rp = g2d_sub_group(g2d_sub_group(g2d_add_group(Q, q1, gl), q2, gl), q3, gl);
  return g2d_mul_gls_d_group(Rp, gl);
}

// ---- Miller-line preparation (k_prepare_lines) ----------------------------------------------
// hbx_kernels.hip line_dbl_step's doubling on the 16 lanes of a group (pairingd.hpp
// line_dbl_step_di's formulas: c0 = 3X^3 - 2Y^2, c1 = -3X^2 Z^2, c2 = 2YZ^3 = Z3 Z^2; T <- 2T) in
// three rounds: A = X^2, B = Y^2, Z^2, Y Z; C = B^2, (X + B)^2, E^2, E X, E Z^2; E (D - X3), Z3 Z^2.
// Relaxed in and out (T and the line's coefficients).
__device__ __forceinline__ void line_dbl_step_groupd(g2jd& T, fq2d& c0, fq2d& c1, fq2d& c2, int gl) {
  const fqd x0 = T.x.c0, x1 = T.x.c1, y0 = T.y.c0, y1 = T.y.c1, z0 = T.z.c0, z1 = T.z.c1;
  const fq2d z{fqd_zero(), fqd_zero()};
  // X^2 (0, 1), Y^2 (2, 3), Z^2 (4, 5), Y Z (8..11)
  fqd r = gd_round<0x07>(gl, T.x, T.y, T.z, z, T.y, T.y, z, z, T.x, T.y, T.z, z, T.z, T.z, z, z);
  const fq2d A = rows_sqr<0>(r), B = rows_sqr<2>(r), ZZ = rows_sqr<4>(r), YZ = rows_mul<8>(r);
  const fq2d E = fq2d_relax(fq2d_add(fq2d_dbl(A), A));
  const fq2d S = fq2d_relax(fq2d_add(T.x, B));
  // B^2 (0, 1), S^2 (2, 3), E^2 (4, 5), E X (8..11), E Z^2 (12..15)
  r = gd_round<0x07>(gl, B, S, E, z, E, E, E, E, B, S, E, z, T.x, T.x, ZZ, ZZ);
  const fq2d C = rows_sqr<0>(r), TT = rows_sqr<2>(r), F = rows_sqr<4>(r), EX = rows_mul<8>(r), EZZ = rows_mul<12>(r);
  c0 = fq2d_relax(fq2d_sub(EX, fq2d_dbl(B)));
  c1 = fq2d_relax(fq2d_neg(EZZ));
  const fq2d D = fq2d_dbl(fq2d_relax(fq2d_sub(fq2d_sub(TT, A), C)));
  const fq2d X3 = fq2d_relax(fq2d_sub(F, fq2d_dbl(D)));
  const fq2d Z3 = fq2d_relax(fq2d_dbl(YZ));
  const fq2d G = fq2d_sub(D, X3);
  r = gd_round<0>(gl, E, E, Z3, Z3, z, z, z, z, G, G, ZZ, ZZ, z, z, z, z);
  const fq2d EG = rows_mul<0>(r);
  c2 = fq2d_relax(rows_mul<4>(r));
  const fq2d C8 = fq2d_dbl(fq2d_dbl(fq2d_relax(fq2d_dbl(C))));
  T = g2jd{X3, fq2d_relax(fq2d_sub(EG, C8)), Z3};
}

// hbx_kernels.hip line_add_step's addition (pairingd.hpp line_add_step_d: num = Y - yQ Z^3,
// den = Z (X - xQ Z^2), c0 = num xQ - yQ den, c1 = -num, c2 = den; T <- T + Q by madd-2007-bl) on
// the 16 lanes of a group in five rounds.  T relaxed in and out; (qx, qy) normalised.
__device__ __forceinline__ void line_add_step_groupd(g2jd& T, const fq2d& qx, const fq2d& qy, fq2d& c0, fq2d& c1,
                                                     fq2d& c2, int gl) {
  const fq2d z{fqd_zero(), fqd_zero()};
  // round 1: Z1Z1 = Z^2 (0, 1), yQ Z (4..7)
  fqd r = gd_round<0x01>(gl, T.z, z, qy, qy, z, z, z, z, T.z, z, T.z, T.z, z, z, z, z);
  const fq2d Z1Z1 = rows_sqr<0>(r), YqZ = rows_mul<4>(r);
  // round 2: U2 = xQ Z1Z1 (0..3), S2 = yQ Z Z1Z1 (4..7)
  r = gd_round<0>(gl, qx, qx, YqZ, YqZ, z, z, z, z, Z1Z1, Z1Z1, Z1Z1, Z1Z1, z, z, z, z);
  const fq2d H = fq2d_relax(fq2d_sub(rows_mul<0>(r), T.x));  // -(X - xQ Z^2)
  const fq2d num = fq2d_relax(fq2d_sub(T.y, rows_mul<4>(r)));
  // round 3: Z H (0..3), H^2 (4, 5), num^2 (6, 7), num xQ (8..11), (Z + H)^2 (12, 13)
  {
    const fq2d zh = fq2d_relax(fq2d_add(T.z, H));
    r = gd_round<0x4C>(gl, T.z, T.z, H, num, num, num, zh, z, H, H, H, num, qx, qx, zh, z);
  }
  c2 = fq2d_relax(fq2d_neg(rows_mul<0>(r)));  // den
  const fq2d HH = rows_sqr<4>(r), NX = rows_mul<8>(r), ZHs = rows_sqr<12>(r);
  const fq2d RR = fq2d_dbl(fq2d_relax(fq2d_dbl(rows_sqr<6>(r))));  // rr^2 = 4 num^2
  const fq2d I = fq2d_dbl(fq2d_relax(fq2d_dbl(HH)));
  c1 = fq2d_relax(fq2d_neg(num));
  // round 4: yQ den (0..3), J = H I (4..7), V = X I (8..11)
  r = gd_round<0>(gl, qy, qy, H, H, T.x, T.x, z, z, c2, c2, I, I, I, I, z, z);
  c0 = fq2d_relax(fq2d_sub(NX, rows_mul<0>(r)));
  const fq2d J = rows_mul<4>(r), V = rows_mul<8>(r);
  const fq2d X3 = fq2d_relax(fq2d_sub(fq2d_relax(fq2d_sub(RR, J)), fq2d_dbl(V)));
  // round 5: rr (V - X3) with rr = 2 (S2 - Y) = -2 num (0..3), Y J (4..7)
  {
    const fq2d rr = fq2d_dbl(c1), w = fq2d_sub(V, X3);
    r = gd_round<0>(gl, rr, rr, T.y, T.y, z, z, z, z, w, w, J, J, z, z, z, z);
  }
  const fq2d Y3 = fq2d_relax(fq2d_sub(rows_mul<0>(r), fq2d_dbl(rows_mul<4>(r))));
  T = g2jd{X3, Y3, fq2d_relax(fq2d_sub(fq2d_sub(ZHs, Z1Z1), HH))};
}

// The 68 raw lines of Q = (qx, qy) (normalised digits) on a lane group: the doubling steps by
// rounds; the five addition steps by rounds too (GADD) or on every lane (pairingd.hpp
// line_add_step_d: fewer registers, for launches that share the chip with full-chip checks).
// Group lane 0 writes (c0, c1) to raw[k] and c2 to c2out[k] (k_normalise_lines converts and
// normalises them).
template <bool GADD>
__device__ void g2d_raw_lines_group(const fq2d& qx, const fq2d& qy, line_pre_d* raw, fq2d* c2out, int gl) {
  g2jd T{qx, qy, fq2d{fqd_const(FQD_ONE), fqd_zero()}};
  int k = 0;
  for (int i = 62; i >= 0; i--) {
    fq2d c0, c1, c2;
    line_dbl_step_groupd(T, c0, c1, c2, gl);
    if (gl == 0) {
      raw[k] = line_pre_d{c0, c1};
      c2out[k] = c2;
    }
    k++;
    if ((BLS_X >> i) & 1) {
      if (GADD) line_add_step_groupd(T, qx, qy, c0, c1, c2, gl);
      else line_add_step_call(T, qx, qy, c0, c1, c2);
      if (gl == 0) {
        raw[k] = line_pre_d{c0, c1};
        c2out[k] = c2;
      }
      k++;
    }
  }
}

#endif  // __HIPCC__
}  // namespace hbx
