// The two-lane share check (k_verify_shares2): one decryption-share check e(S, H') e(-[m]pk, W) == 1
// on a PAIR of lanes, in the signed-digit tower (fieldd.hpp).  Same verdict bits as the one-lane
// check (pairingd.hpp) and as two pairing 0.14 pairings compared (honey_badger.rs:229 via
// threshold_crypto).
//
// Why: one lane per check holds a whole Fq12 (168 registers) plus the Fq6 products' temporaries,
// which spills at one wave per SIMD (95 VGPRs + 9 KB/lane of scratch, 14 GB of scratch traffic per
// N=256 launch).  With f = A0 + A1 w (Fq12 = Fq6[w]/(w^2 - v)), lane 0 of a pair holds A0 and lane
// 1 holds A1 (84 registers each); the other half comes over by a DPP quad permutation (one VALU
// move per dword, no LDS round trip), and every Fq12 operation splits into equal per-lane work:
//   * Miller squaring (Karatsuba): lane 0 computes A0 A1, lane 1 (A0 + A1)(A0 + v A1): one Fq6
//     product each (the one-lane squaring's two), then c0 = t - ab - v ab, c1 = 2 ab;
//   * line product: the line c0 + (c1 x) v + y v w is scaled by 1/y (an Fq factor, which the final
//     exponentiation maps to 1: (p - 1) divides (p^12 - 1)/r), l = (c0/y + (c1 x/y) v) + v w, so
//     lane k computes A_k (c0' + c1' v) (5 Fq2 products) + v^(2-k) A_(1-k) -- the one-lane sparse
//     product's 10 Fq2 products and 3 Fq-by-Fq2 products for the y term are 10 products in all;
//   * general product: lane k computes A_k B_k, and half of the Karatsuba products of
//     (A0 + A1)(B0 + B1) (three Fq2 products each);
//   * cyclotomic squaring (Granger-Scott): each lane produces its own three Fq2 coefficients, each
//     from ONE fused column loop of four digit convolutions and two reductions (lane 0:
//     a^2 + xi b^2, lane 1: 2 a b; operands selected per lane), the one-lane squaring's 9 Fq2
//     squarings split evenly;
//   * Frobenius maps and conjugation are coefficient-wise.
// The per-check scalars: lane 0 holds 1/y of both G1 points, lane 1 x/y (one Fq inversion each).
// Control flow is pair-uniform; every exchange reads the partner lane of the same pair.
#pragma once
#include "pairingd.hpp"

namespace hbx {
#if defined(__HIPCC__)

// quad_perm [1, 0, 3, 2]: each lane reads its pair partner
__device__ __forceinline__ int32_t xchg_i32(int32_t v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true); }

template <class T>
__device__ __forceinline__ T xchg_t(const T& a) {
  static_assert(sizeof(T) % 4 == 0, "dword-sized value");
  T r;
  const int32_t* pa = reinterpret_cast<const int32_t*>(&a);
  int32_t* pr = reinterpret_cast<int32_t*>(&r);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); i++) pr[i] = xchg_i32(pa[i]);
  return r;
}
template <class T>
__device__ __forceinline__ T sel_t(bool c, const T& a, const T& b) {
  T r;
  const int32_t* pa = reinterpret_cast<const int32_t*>(&a);
  const int32_t* pb = reinterpret_cast<const int32_t*>(&b);
  int32_t* pr = reinterpret_cast<int32_t*>(&r);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); i++) pr[i] = c ? pa[i] : pb[i];
  return r;
}

__device__ __forceinline__ fq6d fq6d_one() {
  const fqd z = fqd_zero();
  return fq6d{fq2d{fqd_const(FQD_ONE), z}, fq2d{z, z}, fq2d{z, z}};
}
__device__ __forceinline__ fq6d fq6d_zero() {
  const fqd z = fqd_zero();
  return fq6d{fq2d{z, z}, fq2d{z, z}, fq2d{z, z}};
}
// conj(A0 + A1 w) = A0 - A1 w
__device__ __forceinline__ fq6d conj2d(const fq6d& a, bool l1) { return l1 ? fq6d_neg(a) : a; }

// Miller-loop squaring: (A0 + A1 w)^2 = (t - ab - v ab) + 2 ab w, ab = A0 A1,
// t = (A0 + A1)(A0 + v A1).  Reduced output.
__device__ __forceinline__ fq6d sqr2d(const fq6d& A, bool l1) {
  const fq6d B = xchg_t(A);
  const fq6d X = sel_t(l1, fq6d_norm(fq6d_add(A, B)), A);
  const fq6d Y = sel_t(l1, fq6d_norm(fq6d_add(B, fq6d_mul_v(A))), B);
  const fq6d P = fq6d_mul(X, Y);  // lane 0: ab, lane 1: t
  const fq6d Q = xchg_t(P);
  const fq6d r0 = fq6d_sub(fq6d_sub(Q, P), fq6d_mul_v(P));
  const fq6d r1 = fq6d_add(Q, Q);
  return fq6d_reduce(sel_t(l1, r1, r0));
}

// f * ((c0s + c1s v) + v w): lane 0 A0 L0 + v^2 A1, lane 1 A1 L0 + v A0.  Reduced output.
__device__ __forceinline__ fq6d line2d(const fq6d& A, const fq2d& c0s, const fq2d& c1s, bool l1) {
  const fq6d B = xchg_t(A);
  const fq6d T = fq6d_mul_by_01(A, c0s, c1s);
  const fq6d vB = fq6d_mul_v(B);
  return fq6d_reduce(fq6d_add(T, sel_t(l1, vB, fq6d_mul_v(vB))));
}

// The scaled line's (c0 / y, c1 x / y): lane 0 holds s = 1/y, lane 1 s = x/y.
__device__ __forceinline__ void line_eval2d(const line_pre_d& L, const fqd& s, bool l1, fq2d& c0s, fq2d& c1s) {
  const fq2d mine = fq2d_mul_fq(sel_t(l1, L.c1, L.c0), s);
  const fq2d other = xchg_t(mine);
  c0s = sel_t(l1, other, mine);
  c1s = sel_t(l1, mine, other);
}

// Two Miller loops over prepared lines (pairingd.hpp miller_loop2_d), conjugated for x < 0.
__device__ fq6d miller2d(const line_pre_d* LA, const fqd& sA, bool useA, const line_pre_d* LB, const fqd& sB,
                         bool useB, bool l1) {
  fq6d f = l1 ? fq6d_zero() : fq6d_one();
  int k = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (i != 62) f = sqr2d(f, l1);
    const int steps = ((BLS_X >> i) & 1) ? 4 : 2;  // (A, B) lines of the doubling [+ addition]
#pragma unroll 1
    for (int s = 0; s < steps; s++) {
      const bool b = (s & 1) != 0;
      const line_pre_d L = ld_uniform((b ? LB : LA) + k);
      if (b ? useB : useA) {
        fq2d c0s, c1s;
        line_eval2d(L, b ? sB : sA, l1, c0s, c1s);
        f = line2d(f, c0s, c1s, l1);
      }
      if (b) k++;
    }
  }
  return conj2d(f, l1);
}

// General product (A0 + A1 w)(B0 + B1 w) = (A0 B0 + v A1 B1) + ((A0 + A1)(B0 + B1) - A0 B0 - A1 B1) w.
// Inputs reduced or conjugated reduced; reduced output.
__device__ __noinline__ fq6d mul2d(const fq6d& X, const fq6d& Y, bool l1) {
  const fq6d P = fq6d_mul(X, Y);  // lane 0: X0 Y0, lane 1: X1 Y1
  const fq6d sX = fq6d_norm(fq6d_add(X, xchg_t(X)));
  const fq6d sY = fq6d_norm(fq6d_add(Y, xchg_t(Y)));
  // Karatsuba of sX sY: lane 0 the t_i = sX_i sY_i, lane 1 the u_i (pairs of coefficient sums)
  const fq2d q0 = fq2d_mul(sel_t(l1, fq2d_add(sX.c1, sX.c2), sX.c0), sel_t(l1, fq2d_add(sY.c1, sY.c2), sY.c0));
  const fq2d q1 = fq2d_mul(sel_t(l1, fq2d_add(sX.c0, sX.c1), sX.c1), sel_t(l1, fq2d_add(sY.c0, sY.c1), sY.c1));
  const fq2d q2 = fq2d_mul(sel_t(l1, fq2d_add(sX.c0, sX.c2), sX.c2), sel_t(l1, fq2d_add(sY.c0, sY.c2), sY.c2));
  const fq6d q = fq6d{q0, q1, q2};
  const fq6d qo = xchg_t(q);
  const fq6d t = sel_t(l1, qo, q), u = sel_t(l1, q, qo);
  const fq6d PP = xchg_t(P);
  if (l1) {
    const fq2d s0 = fq2d_add(t.c0, fq2d_mul_xi(fq2d_sub(fq2d_sub(u.c0, t.c1), t.c2)));
    const fq2d s1 = fq2d_add(fq2d_sub(fq2d_sub(u.c1, t.c0), t.c1), fq2d_mul_xi(t.c2));
    const fq2d s2 = fq2d_add(fq2d_sub(fq2d_sub(u.c2, t.c0), t.c2), t.c1);
    return fq6d_reduce(fq6d_sub(fq6d_sub(fq6d{s0, s1, s2}, P), PP));
  }
  return fq6d_reduce(fq6d_add(P, fq6d_mul_v(PP)));
}

// Granger-Scott halves: lane 0 a^2 + xi b^2, lane 1 2 a b, as ONE column loop of four digit
// convolutions re = C1 + C2 - C3, im = C4 + C2 + C3 with
//   lane 0: C1 = (a0 + a1)(a0 - a1), C2 = (b0 + b1)(b0 - b1), C3 = (2 b0) b1,      C4 = (2 a0) a1;
//   lane 1: C1 = (2 a0) b0,          C2 = (a0 - a1) b1,        C3 = (a0 + a1) b1, C4 = (2 a1) b0
// (lane 1: re = 2 a0 b0 - 2 a1 b1, im = 2 a1 b0 + 2 a0 b1).  Inputs reduced (digits 0..12 in
// [0, 2^28)): every operand digit is below 2^29 in magnitude, a column of one convolution below
// 14 x 2^57, re / im below 2^62.4.  Normalised output.
__device__ __forceinline__ fq2d cyc_pair2d(const fq2d& a, const fq2d& b, bool l1) {
  HBX_COUNT_FQMUL(); HBX_COUNT_FQMUL(); HBX_COUNT_FQMUL(); HBX_COUNT_FQMUL();
  int32_t p1[14], q1[14], p2[14], q2[14], p3[14], p4[14], q4[14];
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const int32_t a0 = a.c0.d[i], a1 = a.c1.d[i], b0 = b.c0.d[i], b1 = b.c1.d[i];
    const int32_t as = a0 + a1, ad = a0 - a1;
    p1[i] = l1 ? a0 + a0 : as;
    q1[i] = l1 ? b0 : ad;
    p2[i] = l1 ? ad : b0 + b1;
    q2[i] = l1 ? b1 : b0 - b1;
    p3[i] = l1 ? as : b0 + b0;
    p4[i] = l1 ? a1 + a1 : a0 + a0;
    q4[i] = l1 ? b0 : a1;
  }
  const int32_t* q3 = b.c1.d;
  fq2d r;
  fqd_redc2(
      [&](int k, int jlo, int jhi, int64_t& X, int64_t& Y) {
        int64_t c1 = 0, c2 = 0, c3 = 0, c4 = 0;
#pragma unroll
        for (int j = jlo; j <= jhi; j++) {
          c1 += (int64_t)p1[j] * (int64_t)q1[k - j];
          c2 += (int64_t)p2[j] * (int64_t)q2[k - j];
          c3 += (int64_t)p3[j] * (int64_t)q3[k - j];
          c4 += (int64_t)p4[j] * (int64_t)q4[k - j];
        }
        X = c1 + c2 - c3;
        Y = c4 + c2 + c3;
      },
      r.c0, r.c1);
  return r;
}

// Granger-Scott cyclotomic squaring (fieldd.hpp fq12d_cyclotomic_sqr) on a pair.  With
// c0 = (z0, z4, z3) on lane 0 and c1 = (z2, z1, z5) on lane 1, own slot q becomes
//   lane 0: z0' = 3 (z0^2 + xi z1^2) - 2 z0,  z4' = 3 (z2^2 + xi z3^2) - 2 z4,  z3' = 3 (z4^2 + xi z5^2) - 2 z3;
//   lane 1: z2' = 3 xi (2 z4 z5) + 2 z2,      z1' = 3 (2 z0 z1) + 2 z1,         z5' = 3 (2 z2 z3) + 2 z5.
// Operands (a, b) of slot q: (A.c0 | A.c2, B.c1), (B.c0, A.c2 | A.c1), (A.c1 | A.c0, B.c2)
// (lane 0 | lane 1; B = the partner's half; 2ab is symmetric).
__device__ __forceinline__ fq6d cyc_sqr2d(const fq6d& A, bool l1) {
  const fq6d B = xchg_t(A);
  fq2d T0 = cyc_pair2d(sel_t(l1, A.c2, A.c0), B.c1, l1);
  const fq2d T1 = cyc_pair2d(B.c0, sel_t(l1, A.c1, A.c2), l1);
  const fq2d T2 = cyc_pair2d(sel_t(l1, A.c0, A.c1), B.c2, l1);
  T0 = sel_t(l1, fq2d_mul_xi(T0), T0);
  const fq6d T{T0, T1, T2};
  const fq6d T3 = fq6d_add(fq6d_add(T, T), T);
  const fq6d A2 = fq6d_add(A, A);
  return fq6d_reduce(sel_t(l1, fq6d_add(T3, A2), fq6d_sub(T3, A2)));
}

// Frobenius maps (fieldd.hpp fq12d_frobenius / fq12d_frobenius2): coefficient q of half k is
// multiplied by gamma_{1 or 2, 2q + k} (w-basis index; gamma_0 = 1).
__device__ __forceinline__ fq6d frob2d(const fq6d& A, bool l1) {
  const fq2d k0 = sel_t(l1, fq2d_const(FROBD1_C1_0, FROBD1_C1_1), fq2d{fqd_const(FQD_ONE), fqd_zero()});
  const fq2d k1 = sel_t(l1, fq2d_const(FROBD1_C3_0, FROBD1_C3_1), fq2d_const(FROBD1_C2_0, FROBD1_C2_1));
  const fq2d k2 = sel_t(l1, fq2d_const(FROBD1_C5_0, FROBD1_C5_1), fq2d_const(FROBD1_C4_0, FROBD1_C4_1));
  return fq6d{fq2d_mul(fq2d_conj(A.c0), k0), fq2d_mul(fq2d_conj(A.c1), k1), fq2d_mul(fq2d_conj(A.c2), k2)};
}
__device__ __forceinline__ fq6d frob2_2d(const fq6d& A, bool l1) {
  const fqd k0 = sel_t(l1, fqd_const(FROBD2_C1), fqd_const(FQD_ONE));
  const fqd k1 = sel_t(l1, fqd_const(FROBD2_C3), fqd_const(FROBD2_C2));
  const fqd k2 = sel_t(l1, fqd_const(FROBD2_C5), fqd_const(FROBD2_C4));
  return fq6d{fq2d_mul_fq(A.c0, k0), fq2d_mul_fq(A.c1, k1), fq2d_mul_fq(A.c2, k2)};
}

// f^-1 = (A0 - A1 w) / (A0^2 - v A1^2), the Fq6 inverse through field.hpp's 12-limb one.
__device__ __noinline__ fq6d inv2d(const fq6d& A, bool l1) {
  const fq6d S = fq6d_mul(A, A);  // lane 0: A0^2, lane 1: A1^2
  const fq6d So = xchg_t(S);
  const fq6d N = fq6d_reduce(fq6d_sub(sel_t(l1, So, S), fq6d_mul_v(sel_t(l1, S, So))));
  const fq6d Ni = fq6d_from_fq6(fq6_inv(fq6d_to_fq6(N)));
  return fq6d_reduce(conj2d(fq6d_mul(A, Ni), l1));
}

// g^|x| (g reduced, cyclotomic): squaring runs between the one bits of |x|
__device__ __noinline__ fq6d cyc_exp_abs_x2d(const fq6d& g, bool l1) {
  static_assert(BLS_X == 0xd201000000010000ull, "square-and-multiply runs are specific to |x|");
  fq6d r = g;
#pragma unroll 1
  for (int q = 0; q < 6; q++) {
    const int run = q == 0 ? 1 : q == 1 ? 2 : q == 2 ? 3 : q == 3 ? 9 : q == 4 ? 32 : 16;
#pragma unroll 1
    for (int i = 0; i < run; i++) r = cyc_sqr2d(r, l1);
    if (q < 5) r = mul2d(r, g, l1);
  }
  return r;
}

// f^(3 (p^12 - 1)/r) (pairingd.hpp final_exponentiation_d, the same chain); g^x = conj(g^|x|)
__device__ __noinline__ fq6d final_exp2d(const fq6d& f, bool l1) {
  fq6d t = mul2d(conj2d(f, l1), inv2d(f, l1), l1);
  t = mul2d(frob2_2d(t, l1), t, l1);
  fq6d a = mul2d(conj2d(cyc_exp_abs_x2d(t, l1), l1), conj2d(t, l1), l1);  // t^(x-1)
  a = mul2d(conj2d(cyc_exp_abs_x2d(a, l1), l1), conj2d(a, l1), l1);        // t^((x-1)^2)
  const fq6d b = mul2d(conj2d(cyc_exp_abs_x2d(a, l1), l1), frob2d(a, l1), l1);  // a^(x+p)
  fq6d c = mul2d(cyc_exp_abs_x2d(cyc_exp_abs_x2d(b, l1), l1), frob2_2d(b, l1), l1);
  c = mul2d(c, conj2d(b, l1), l1);                                           // b^(x^2+p^2-1)
  const fq6d t3 = mul2d(cyc_sqr2d(t, l1), t, l1);                            // t^3
  return mul2d(c, t3, l1);
}

// f == 1 for the pair: lane 0 holds (1, 0, 0), lane 1 holds 0
__device__ __forceinline__ bool is_one2d(const fq6d& A, bool l1) {
  const fq6 a = fq6d_to_fq6(A);
  const bool c0ok = l1 ? fq2_is_zero(a.c0) : (fq_eq(a.c0.c0, fq_one()) && fq_is_zero(a.c0.c1));
  const bool mine = c0ok && fq2_is_zero(a.c1) && fq2_is_zero(a.c2);
  return mine && xchg_i32(mine ? 1 : 0) != 0;
}

// The pair's per-check scalars of point P (12-limb affine, not the identity): lane 0 1/y,
// lane 1 x/y.  `neg`: use -P.
__device__ __forceinline__ fqd point_scalar2d(const g1a& P, bool neg, bool l1) {
  const fq y = neg ? fq_neg(P.y) : P.y;
  const fq yi = fq_inv(y);
  return fqd_from_fq(l1 ? fq_mul(P.x, yi) : yi);
}

#endif  // __HIPCC__
}  // namespace hbx
