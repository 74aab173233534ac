// The share check's two-pair Miller loop in the signed-digit tower (fieldd.hpp).
//
// Same loop as pairing.hpp miller_loop2 (same lines, same formulas, the same Fq12 element out):
// 63 squarings of f and the 136 prepared lines of H_j and W_j evaluated at the two G1 points.
// The prepared lines are stored a second time in digit form (line_pre_d, written by
// k_normalise_lines), so the loop reads them without a conversion; the G1 coordinates are
// converted once per check.
#pragma once
#include "fieldd.hpp"
#include "pairing.hpp"

namespace hbx {

struct line_pre_d {
  fq2d c0, c1;
};
HBX_HD line_pre_d line_to_d(const line_pre& l) { return line_pre_d{fq2d_from_fq2(l.c0), fq2d_from_fq2(l.c1)}; }

// f_{|x|,QA}(PA) * f_{|x|,QB}(PB), conjugated for x < 0 (pairing.hpp miller_loop2); (ax, ay) and
// (bx, by) are the affine G1 points in digit form; a pair whose flag is false contributes 1.
HBX_HD fq12d miller_loop2_d(const line_pre_d* LA, const fqd& ax, const fqd& ay, bool useA,
                            const line_pre_d* LB, const fqd& bx, const fqd& by, bool useB) {
  fq12d f = fq12d_one();
  int k = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (i != 62) f = fq12d_sqr(f);
    const int steps = ((BLS_X >> i) & 1) ? 4 : 2;  // (A, B) lines of the doubling [+ addition]
#pragma unroll 1
    for (int s = 0; s < steps; s++) {
      const bool b = (s & 1) != 0;
      const line_pre_d L = ld_uniform((b ? LB : LA) + k);
      if (b ? useB : useA) f = fq12d_mul_by_014(f, L.c0, fq2d_mul_fq(L.c1, b ? bx : ax), b ? by : ay);
      if (b) k++;
    }
  }
  return fq12d_conj(f);
}

// ----------------------------------------------------------------------------------------------
// Lines generated on the fly (a varying G2 point: the coin's signature shares, common_coin.rs:151)
// -- pairing.hpp line_dbl_step / line_add_step / fq12_mul_by_014_f2 / miller_loop_mixed in the
// digit tower.  Values that feed products are reduced (or are sums of two reduced values).  The
// line steps and the Fq2-coefficient line product are out-of-line copies: inlined into the mixed
// loop they made one function too large to compile in reasonable time.
// ----------------------------------------------------------------------------------------------
struct g2jd {
  fq2d x, y, z;
};
// Raw line through the doubling of T, scaled by 2 Y Z^3: c0 = 3X^3 - 2Y^2, c1 = -3X^2 Z^2,
// c2 = 2YZ^3;  T <- 2T.
HBX_HD void line_dbl_step_di(g2jd& T, fq2d& c0, fq2d& c1, fq2d& c2) {
  const fq2d A = fq2d_sqr(T.x);
  const fq2d B = fq2d_sqr(T.y);
  const fq2d C = fq2d_sqr(B);
  const fq2d ZZ = fq2d_sqr(T.z);
  const fq2d E = fq2d_norm(fq2d_add(fq2d_dbl(A), A));
  c0 = fq2d_reduce(fq2d_sub(fq2d_mul(E, T.x), fq2d_dbl(B)));
  c1 = fq2d_neg(fq2d_mul(E, ZZ));
  const fq2d D = fq2d_reduce(fq2d_dbl(fq2d_sub(fq2d_sub(fq2d_sqr(fq2d_add(T.x, B)), A), C)));
  const fq2d F = fq2d_sqr(E);
  const fq2d X3 = fq2d_reduce(fq2d_sub(F, fq2d_dbl(D)));
  const fq2d C8 = fq2d_dbl(fq2d_reduce(fq2d_dbl(fq2d_dbl(C))));
  const fq2d Y3 = fq2d_reduce(fq2d_sub(fq2d_mul(E, fq2d_sub(D, X3)), C8));
  const fq2d Z3 = fq2d_reduce(fq2d_dbl(fq2d_mul(T.y, T.z)));
  c2 = fq2d_mul(Z3, ZZ);
  T = g2jd{X3, Y3, Z3};
}
HBX_HDNI void line_dbl_step_d(g2jd& T, fq2d& c0, fq2d& c1, fq2d& c2) { line_dbl_step_di(T, c0, c1, c2); }
// Raw line through T and the affine base point (qx, qy), scaled by den = Z (X - xQ Z^2):
// c0 = num xQ - yQ den, c1 = -num, c2 = den;  T <- T + Q (madd-2007-bl).
HBX_HD void line_add_step_di(g2jd& T, const fq2d& qx, const fq2d& qy, fq2d& c0, fq2d& c1, fq2d& c2) {
  const fq2d Z1Z1 = fq2d_sqr(T.z);
  const fq2d U2 = fq2d_mul(qx, Z1Z1);
  const fq2d S2 = fq2d_mul(fq2d_mul(qy, T.z), Z1Z1);
  const fq2d H = fq2d_sub(U2, T.x);
  const fq2d num = fq2d_sub(T.y, S2);
  const fq2d den = fq2d_neg(fq2d_mul(T.z, H));
  c0 = fq2d_reduce(fq2d_sub(fq2d_mul(num, qx), fq2d_mul(qy, den)));
  c1 = fq2d_neg(num);
  c2 = den;
  const fq2d HH = fq2d_sqr(H);
  const fq2d I = fq2d_reduce(fq2d_dbl(fq2d_dbl(HH)));
  const fq2d J = fq2d_mul(H, I);
  const fq2d r = fq2d_reduce(fq2d_dbl(fq2d_sub(S2, T.y)));
  const fq2d V = fq2d_mul(T.x, I);
  const fq2d X3 = fq2d_reduce(fq2d_sub(fq2d_sub(fq2d_sqr(r), J), fq2d_dbl(V)));
  const fq2d Y3 = fq2d_reduce(fq2d_sub(fq2d_mul(r, fq2d_sub(V, X3)), fq2d_dbl(fq2d_mul(T.y, J))));
  const fq2d Z3 = fq2d_reduce(fq2d_sub(fq2d_sub(fq2d_sqr(fq2d_norm(fq2d_add(T.z, H))), Z1Z1), HH));
  T = g2jd{X3, Y3, Z3};
}
HBX_HDNI void line_add_step_d(g2jd& T, const fq2d& qx, const fq2d& qy, fq2d& c0, fq2d& c1, fq2d& c2) {
  line_add_step_di(T, qx, qy, c0, c1, c2);
}
// The out-of-line addition step called from a loop that keeps T and the line in registers: through
// copies, so that only the copies' addresses escape into the call.  Passing the loop's own T and
// line by reference kept them in scratch memory across the whole loop -- every doubling step read
// and wrote T there (the coin Miller kernel's 6.6 GB of scratch traffic per launch).
HBX_HD void line_add_step_call(g2jd& T, const fq2d& qx, const fq2d& qy, fq2d& c0, fq2d& c1, fq2d& c2) {
  g2jd t = T;
  fq2d a0, a1, a2;
  line_add_step_d(t, qx, qy, a0, a1, a2);
  T = t;
  c0 = a0;
  c1 = a1;
  c2 = a2;
}
// f * (c0 + c1 v + c4 v w) with c4 in Fq2 (an un-normalised line at a G1 point)
HBX_HD fq12d fq12d_mul_by_014_f2_i(const fq12d& f, const fq2d& c0, const fq2d& c1, const fq2d& c4) {
  const fq6d aa = fq6d_mul_by_01(f.c0, c0, c1);
  const fq6d bb = fq6d{fq2d_mul_xi(fq2d_mul(f.c1.c2, c4)), fq2d_mul(f.c1.c0, c4), fq2d_mul(f.c1.c1, c4)};
  const fq2d o = fq2d_norm(fq2d_add(c1, c4));
  const fq6d s = fq6d_mul_by_01(fq6d_norm(fq6d_add(f.c1, f.c0)), c0, o);
  return fq12d{fq6d_reduce(fq6d_add(fq6d_mul_v(bb), aa)), fq6d_reduce(fq6d_sub(fq6d_sub(s, aa), bb))};
}
HBX_HDNI fq12d fq12d_mul_by_014_f2(const fq12d& f, const fq2d& c0, const fq2d& c1, const fq2d& c4) {
  return fq12d_mul_by_014_f2_i(f, c0, c1, c4);
}
// pairing.hpp miller_loop_mixed: pair A over prepared digit-form lines (plain loads: the lines may
// differ per lane), pair B's lines generated from QB = (qx, qy) and evaluated un-normalised at PB.
// One out-of-line copy (the coin and the PublicKey::verify kernels share it).  With `Tout`, the
// loop's final T = [|x|] QB (Jacobian) is stored there: the coin checks take QB's G2 membership
// from it (g2_torsion_free_from_T) instead of a separate [x] multiplication at decode.
HBX_HDNI fq12d miller_loop_mixed_d(const line_pre_d* LA, const fqd& ax, const fqd& ay, bool useA, const fq2d& qx,
                                 const fq2d& qy, const fqd& bx, const fqd& by, bool useB, g2jd* Tout = nullptr) {
  fq12d f = fq12d_one();
  g2jd T{qx, qy, fq2d{fqd_const(FQD_ONE), fqd_zero()}};
  int k = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (i != 62) f = fq12d_sqr(f);
#pragma unroll 1
    for (int s = 0; s < (((BLS_X >> i) & 1) ? 2 : 1); s++) {
      if (useA) {
        const line_pre_d L = LA[k];
        f = fq12d_mul_by_014(f, L.c0, fq2d_mul_fq(L.c1, ax), ay);
      }
      if (useB) {
        fq2d c0, c1, c2;
        if (s == 0) line_dbl_step_d(T, c0, c1, c2);
        else line_add_step_call(T, qx, qy, c0, c1, c2);
        f = fq12d_mul_by_014_f2(f, c0, fq2d_mul_fq(c1, bx), fq2d_mul_fq(c2, by));
      }
      k++;
    }
  }
  if (Tout) *Tout = T;
  return fq12d_conj(f);
}

// One pair with its lines generated from (qx, qy) and evaluated at (bx, by) -- miller_loop_mixed_d
// with pair A off -- the doubling steps and line products inlined (the two-lane coin check's
// per-lane loop: the out-of-line steps passed the Fq12 accumulator through the call frames, 11.5
// -> 9.3 ms per 1,024-wave launch, tools/microbench/coin_parts.hip).  T = [|x|] Q on return.
HBX_HD fq12d miller_loop_gen_d(const fq2d& qx, const fq2d& qy, const fqd& bx, const fqd& by, g2jd& T) {
  fq12d f = fq12d_one();
  T = g2jd{qx, qy, fq2d{fqd_const(FQD_ONE), fqd_zero()}};
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (i != 62) f = fq12d_sqr(f);
#pragma unroll 1
    for (int s = 0; s < (((BLS_X >> i) & 1) ? 2 : 1); s++) {
      fq2d c0, c1, c2;
      if (s == 0) line_dbl_step_di(T, c0, c1, c2);
      else line_add_step_call(T, qx, qy, c0, c1, c2);
      HBX_SEQ();
      f = fq12d_mul_by_014_f2_i(f, c0, fq2d_mul_fq(c1, bx), fq2d_mul_fq(c2, by));
      HBX_SEQ();
    }
  }
  return fq12d_conj(f);
}

// Q in G2 from the mixed Miller loop's final T = [|x|] Q (eprint 2021/1130 sec. 4: psi(Q) == [x] Q,
// x = -|x|; curve.hpp g2_is_torsion_free computes the same multiplication by itself).  An
// exceptional addition on the way ([k] Q = +-Q, only for Q of small order) leaves T at Z = 0,
// which never equals the finite -psi(Q): rejected, as Q is not in G2.
HBX_HD bool g2_torsion_free_from_T(const g2jd& T, const g2a& Q) {
  if (Q.inf) return true;
  const g2j t{fq2d_to_fq2(T.x), fq2d_to_fq2(T.y), fq2d_to_fq2(T.z)};
  return g2j_eq(g2_neg(t), g2_psi(g2_from_affine(Q)));
}

// Out-of-line copies (one each) for the final exponentiation's cold calls.
HBX_HDNI fq12d fq12d_mul_ni(const fq12d& a, const fq12d& b) { return fq12d_mul(a, b); }
HBX_HDNI fq12d fq12d_frobenius_ni(const fq12d& a) { return fq12d_frobenius(a); }
HBX_HDNI fq12d fq12d_frobenius2_ni(const fq12d& a) { return fq12d_frobenius2(a); }

// r^(2^k) by k cyclotomic squarings (one inlined copy of the squaring)
HBX_HD fq12d cyc_sqr_n_d(fq12d r, int k) {
#pragma unroll 1
  for (int i = 0; i < k; i++) r = fq12d_cyclotomic_sqr(r);
  return r;
}

#if !defined(__HIPCC__)
typedef uint32_t lds_u32;  // host builds (tools/hostcheck): the "LDS slot" is plain memory
constexpr int LDS_FQ12_STRIDE = 1;
#endif
// The Miller loop with the two G1 points parked in this lane's LDS slot (free until the final
// exponentiation overwrites it with the exponentiation base): 4 x 14 dwords, word k at
// park[k * LDS_FQ12_STRIDE], read back at every line.  Holding the 56 coordinate registers across
// the loop was what spilled it (95 VGPRs, most of the kernel's scratch traffic); an LDS read per
// line costs a few cycles.  Same lines, same products, the same Fq12 element out as miller_loop2_d.
HBX_HD void park_put_fqd(lds_u32* park, int which, const fqd& a) {
#pragma unroll
  for (int i = 0; i < 14; i++) park[(which * 14 + i) * LDS_FQ12_STRIDE] = (uint32_t)a.d[i];
}
HBX_HD fqd park_get_fqd(const lds_u32* park, int which) {
  fqd a;
#pragma unroll
  for (int i = 0; i < 14; i++) a.d[i] = (int32_t)park[(which * 14 + i) * LDS_FQ12_STRIDE];
  return a;
}
HBX_HD fq12d miller_loop2_parked_d(const line_pre_d* LA, bool useA, const line_pre_d* LB, bool useB,
                                   const lds_u32* park) {
  fq12d f = fq12d_one();
  int k = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (i != 62) f = fq12d_sqr(f);
    const int steps = ((BLS_X >> i) & 1) ? 4 : 2;  // (A, B) lines of the doubling [+ addition]
#pragma unroll 1
    for (int s = 0; s < steps; s++) {
      const bool b = (s & 1) != 0;
      const line_pre_d L = ld_uniform((b ? LB : LA) + k);
      if (b ? useB : useA) {
        HBX_SEQ();
        const fqd px = park_get_fqd(park, b ? 2 : 0);
        const fqd py = park_get_fqd(park, b ? 3 : 1);
        f = fq12d_mul_by_014(f, L.c0, fq2d_mul_fq(L.c1, px), py);
      }
      if (b) k++;
    }
  }
  return fq12d_conj(f);
}

HBX_HD fq6d fq6d_zero_() {
  const fqd z = fqd_zero();
  return fq6d{fq2d{z, z}, fq2d{z, z}, fq2d{z, z}};
}

// acc += a * y (fieldd.hpp fq6d_mul's Karatsuba), y(q) its Fq2 coefficient q, every Fq2 product
// folded into the accumulator at once, a fence between products (HBX_SEQ); a and y normalised,
// acc normalised (or zero) on entry; carry-normalised on exit.  The digit sums stay below 2^31:
// acc + 7 terms of at most two normalised values each.
// HBX_PIN_OPS: each product's register operand is pinned (an empty asm with the digits as in/out
// VGPR operands) right where the product starts, so the compiler cannot compute the operand's digit
// sums (fq2d_mul's Karatsuba sums) for all six products up front beside the accumulator.
#ifndef HBX_PIN_OPS
#define HBX_PIN_OPS 0
#endif
HBX_HD fq2d fq2d_pin(fq2d a) {
#if HBX_PIN_OPS && defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
  for (int i = 0; i < 14; i++) {
    __asm__ volatile("" : "+v"(a.c0.d[i]));
    __asm__ volatile("" : "+v"(a.c1.d[i]));
  }
#endif
  return a;
}
template <class Y>
HBX_HD void fq6d_mul_acc1(fq6d& acc, const fq6d& a, Y y) {
  {
    const fq2d t0 = fq2d_mul(fq2d_pin(a.c0), y(0));
    acc.c0 = fq2d_add(acc.c0, t0);
    acc.c1 = fq2d_sub(acc.c1, t0);
    acc.c2 = fq2d_sub(acc.c2, t0);
  }
  HBX_SEQ();
  {
    const fq2d t1 = fq2d_mul(fq2d_pin(a.c1), y(1));
    acc.c0 = fq2d_sub(acc.c0, fq2d_mul_xi(t1));
    acc.c1 = fq2d_sub(acc.c1, t1);
    acc.c2 = fq2d_add(acc.c2, t1);
  }
  HBX_SEQ();
  {
    const fq2d t2 = fq2d_mul(fq2d_pin(a.c2), y(2));
    acc.c0 = fq2d_sub(acc.c0, fq2d_mul_xi(t2));
    acc.c1 = fq2d_add(acc.c1, fq2d_mul_xi(t2));
    acc.c2 = fq2d_sub(acc.c2, t2);
  }
  HBX_SEQ();
  acc.c0 = fq2d_add(acc.c0, fq2d_mul_xi(fq2d_mul(fq2d_add(fq2d_pin(a.c1), fq2d_pin(a.c2)), fq2d_add(y(1), y(2)))));
  HBX_SEQ();
  acc.c1 = fq2d_add(acc.c1, fq2d_mul(fq2d_add(fq2d_pin(a.c0), fq2d_pin(a.c1)), fq2d_add(y(0), y(1))));
  HBX_SEQ();
  acc.c2 = fq2d_add(acc.c2, fq2d_mul(fq2d_add(fq2d_pin(a.c0), fq2d_pin(a.c2)), fq2d_add(y(0), y(2))));
  HBX_SEQ();
  acc = fq6d_norm(acc);
}

// Slot words of the scaled Miller loop (word k at park[k * LDS_FQ12_STRIDE]): 0..55 the points'
// scalars (park_scaled_points), 56..139 an Fq6 operand streamed into a product (below).
constexpr int ML_PARK_Y = 56;
HBX_HD void park_put_fq2d(lds_u32* park, int word, const fq2d& a) {
#pragma unroll
  for (int i = 0; i < 14; i++) {
    park[(word + i) * LDS_FQ12_STRIDE] = (uint32_t)a.c0.d[i];
    park[(word + 14 + i) * LDS_FQ12_STRIDE] = (uint32_t)a.c1.d[i];
  }
}
HBX_HD fq2d park_get_fq2d(const lds_u32* park, int word) {
  fq2d a;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    a.c0.d[i] = (int32_t)park[(word + i) * LDS_FQ12_STRIDE];
    a.c1.d[i] = (int32_t)park[(word + 14 + i) * LDS_FQ12_STRIDE];
  }
  return a;
}
// f^2 (fieldd.hpp fq12d_sqr: c0 = (a0 + a1)(a0 + v a1) - ab - v ab, c1 = 2 ab) with the operand
// a0 + v a1 parked in the slot and streamed into its product, one Fq2 coefficient per read: 84
// registers fewer at the squaring's peak, where the loop spilled into AGPRs (~6 % of its
// instructions were accvgpr moves).  The same element.
HBX_HD fq12d fq12d_sqr_parked(const fq12d& a, lds_u32* park) {
  {
    const fq6d y = fq6d_norm(fq6d_add(a.c0, fq6d_mul_v(a.c1)));
    park_put_fq2d(park, ML_PARK_Y, y.c0);
    park_put_fq2d(park, ML_PARK_Y + 28, y.c1);
    park_put_fq2d(park, ML_PARK_Y + 56, y.c2);
  }
  HBX_SEQ();
  fq6d ab = fq6d_zero_();
  fq6d_mul_acc1(ab, a.c0, [&](int q) { return q == 0 ? a.c1.c0 : q == 1 ? a.c1.c1 : a.c1.c2; });
  HBX_SEQ();
  fq6d t = fq6d_zero_();
  fq6d_mul_acc1(t, fq6d_norm(fq6d_add(a.c0, a.c1)), [&](int q) { return park_get_fq2d(park, ML_PARK_Y + 28 * q); });
  return fq12d{fq6d_reduce(fq6d_sub(fq6d_sub(t, ab), fq6d_mul_v(ab))), fq6d_reduce(fq6d_add(ab, ab))};
}

// miller_loop2_parked_d over lines divided by y_P: the slot holds (x_A / y_A, 1 / y_A,
// x_B / y_B, 1 / y_B) (park_scaled_points), each line becomes (c0 / y) + (c1 x / y) v + v w and its
// product costs two Fq-by-Fq2 products for the scaled coefficients instead of one plus the three
// of the c4 = y term (fq12d_mul_by_01v).  The element differs from miller_loop2_parked_d's by a
// product of Fq factors (1 / y per line), which the final exponentiation maps to 1: the same verdict.
HBX_HD fq12d miller_loop2_scaled_d(const line_pre_d* LA, bool useA, const line_pre_d* LB, bool useB,
                                   lds_u32* park) {
  fq12d f = fq12d_one();
  int k = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (i != 62) f = fq12d_sqr_parked(f, park);
    const int steps = ((BLS_X >> i) & 1) ? 4 : 2;  // (A, B) lines of the doubling [+ addition]
#pragma unroll 1
    for (int s = 0; s < steps; s++) {
      const bool b = (s & 1) != 0;
      const line_pre_d L = ld_uniform((b ? LB : LA) + k);
      if (b ? useB : useA) {
        HBX_SEQ();
        const fqd w = park_get_fqd(park, b ? 2 : 0);
        const fqd u = park_get_fqd(park, b ? 3 : 1);
        f = fq12d_mul_by_01v(f, fq2d_mul_fq(L.c0, u), fq2d_mul_fq(L.c1, w));
      }
      if (b) k++;
    }
  }
  return fq12d_conj(f);
}
// (x / y, 1 / y) of the two affine G1 points into the slot (words 0..3), one Fq inversion for both
// (Montgomery's trick); a point at infinity contributes 1 (its pair is not used)
#ifndef HBX_ML_INV
#define HBX_ML_INV 2  // the scalars' inversion: 0 12-limb (inline), 1 digit form inline, 2 digit form out of line
#endif
HBX_HD void park_scaled_points(lds_u32* park, const fq& ax, const fq& ay, bool ainf, const fq& bx, const fq& by,
                               bool binf) {
#if HBX_ML_INV
  // in the digit form throughout (fieldd.hpp fqd_inv; HBX_ML_INV 2: out of line)
  const fqd ya = ainf ? fqd_const(FQD_ONE) : fqd_from_fq(ay), yb = binf ? fqd_const(FQD_ONE) : fqd_from_fq(by);
  bool zero;
#if HBX_ML_INV == 2
  const fqd inv = fqd_inv_ni(fqd_mul(ya, yb), zero);
#else
  const fqd inv = fqd_inv(fqd_mul(ya, yb), zero);
#endif
  const fqd ua = fqd_mul(inv, yb), ub = fqd_mul(inv, ya);
  park_put_fqd(park, 0, fqd_mul(fqd_from_fq(ax), ua));
  park_put_fqd(park, 1, ua);
  park_put_fqd(park, 2, fqd_mul(fqd_from_fq(bx), ub));
  park_put_fqd(park, 3, ub);
#else
  // the 12-limb inversion (round 5).  The digit form inlined raised the Miller kernel 8.31 -> 8.48 ms
  // (profiles/r06k_kernel_stats.txt); out of line (HBX_ML_INV 2, the default) it is neutral to
  // slightly faster (verify 16.96 -> 16.94 ms, coin 13.37 -> 13.33 ms, profiles/r06l_variants.txt)
  const fq ya = ainf ? fq_one() : ay, yb = binf ? fq_one() : by;
  const fq inv = fq_inv_i(fq_mul(ya, yb));
  const fq ua = fq_mul(inv, yb), ub = fq_mul(inv, ya);
  park_put_fqd(park, 0, fqd_from_fq(fq_mul(ax, ua)));
  park_put_fqd(park, 1, fqd_from_fq(ua));
  park_put_fqd(park, 2, fqd_from_fq(fq_mul(bx, ub)));
  park_put_fqd(park, 3, fqd_from_fq(ub));
#endif
}

// miller_loop_gen_d with (qx, qy, bx, by) parked in this lane's LDS slot (free until the final
// exponentiation): 84 registers fewer across the loop; the add steps and every line evaluation
// read them back.  Same element, same T.  (Parking T as well, Q re-read from memory at the add
// steps, spilled more: 748 VGPRs, 18.3 ms per coin round's checks against 367 and 16.3 ms.)
HBX_HD fq12d miller_loop_gen_parked_d(const fq2d& qx, const fq2d& qy, const fqd& bx, const fqd& by, lds_u32* park,
                                      g2jd& T) {
  park_put_fqd(park, 0, qx.c0);
  park_put_fqd(park, 1, qx.c1);
  park_put_fqd(park, 2, qy.c0);
  park_put_fqd(park, 3, qy.c1);
  park_put_fqd(park, 4, bx);
  park_put_fqd(park, 5, by);
  fq12d f = fq12d_one();
  T = g2jd{qx, qy, fq2d{fqd_const(FQD_ONE), fqd_zero()}};
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (i != 62) f = fq12d_sqr(f);
#pragma unroll 1
    for (int s = 0; s < (((BLS_X >> i) & 1) ? 2 : 1); s++) {
      fq2d c0, c1, c2;
      HBX_SEQ();
      if (s == 0) {
        line_dbl_step_di(T, c0, c1, c2);
      } else {
        const fq2d px{park_get_fqd(park, 0), park_get_fqd(park, 1)}, py{park_get_fqd(park, 2), park_get_fqd(park, 3)};
        line_add_step_call(T, px, py, c0, c1, c2);
      }
      HBX_SEQ();
      const fqd ex = park_get_fqd(park, 4), ey = park_get_fqd(park, 5);
      f = fq12d_mul_by_014_f2_i(f, c0, fq2d_mul_fq(c1, ex), fq2d_mul_fq(c2, ey));
      HBX_SEQ();
    }
  }
  return fq12d_conj(f);
}

// The exponentiation base g of g^|x| parked in this lane's LDS slot (pairing.hpp's scheme): 12
// digit-form Fq elements packed as 13 dwords each (digits 0..12 of a reduced value are 28-bit
// fields of bits 0..363, digit 13 a whole dword) -- 156 dwords, lane-interleaved, so four 64-lane
// blocks (one wave per SIMD) fit the 160 KB of a CU.
constexpr int LDS_FQ12D_DWORDS = 156;
HBX_HD void lds_put_fq12d(lds_u32* base, const fq12d& a) {
  const fqd* e = &a.c0.c0.c0;
#pragma unroll
  for (int q = 0; q < 12; q++) {
    uint32_t w[13];
#pragma unroll
    for (int k = 0; k < 12; k++) w[k] = 0;
#pragma unroll
    for (int i = 0; i < 13; i++) {
      const int off = 28 * i, word = off >> 5, sh = off & 31;
      const uint32_t d = (uint32_t)e[q].d[i];
      w[word] |= d << sh;
      if (sh > 4) w[word + 1] |= d >> (32 - sh);
    }
    w[12] = (uint32_t)e[q].d[13];
#pragma unroll
    for (int k = 0; k < 13; k++) base[(q * 13 + k) * LDS_FQ12_STRIDE] = w[k];
  }
}
HBX_HD fq12d lds_get_fq12d(const lds_u32* base) {
  fq12d a;
  fqd* e = &a.c0.c0.c0;
#pragma unroll
  for (int q = 0; q < 12; q++) {
    uint32_t w[13];
#pragma unroll
    for (int k = 0; k < 13; k++) w[k] = base[(q * 13 + k) * LDS_FQ12_STRIDE];
#pragma unroll
    for (int i = 0; i < 13; i++) {
      const int off = 28 * i, word = off >> 5, sh = off & 31;
      uint32_t d = w[word] >> sh;
      if (sh > 4) d |= w[word + 1] << (32 - sh);
      e[q].d[i] = (int32_t)(d & (uint32_t)DMASK);
      HBX_LAUNDER(e[q].d[i]);
    }
    e[q].d[13] = (int32_t)w[12];
  }
  return a;
}
// g^|x| (g reduced, in the cyclotomic subgroup): squaring runs between the one bits of |x|
// (pairing.hpp cyc_exp_abs_x_lds)
HBX_HDNI fq12d cyc_exp_abs_x_d(const fq12d& g_in, lds_u32* gslot) {
  static_assert(BLS_X == 0xd201000000010000ull, "square-and-multiply runs are specific to |x|");
  lds_put_fq12d(gslot, g_in);
  fq12d r = g_in;
#pragma unroll 1
  for (int q = 0; q < 6; q++) {
    const int run = q == 0 ? 1 : q == 1 ? 2 : q == 2 ? 3 : q == 3 ? 9 : q == 4 ? 32 : 16;
    r = cyc_sqr_n_d(r, run);
    if (q < 5) r = fq12d_mul_ni(r, lds_get_fq12d(gslot));
  }
  return r;
}
// f^(3 (p^12 - 1)/r) (pairing.hpp final_exponentiation_lds) in the digit tower; g^x = conj(g^|x|)
// and x^2 = |x|^2
HBX_HDNI fq12d final_exponentiation_d(const fq12d& f, lds_u32* gslot) {
  fq12d t = fq12d_mul_ni(fq12d_conj(f), fq12d_inv(f));
  t = fq12d_mul_ni(fq12d_frobenius2_ni(t), t);
  fq12d a = fq12d_mul_ni(fq12d_conj(cyc_exp_abs_x_d(t, gslot)), fq12d_conj(t));  // t^(x-1)
  a = fq12d_mul_ni(fq12d_conj(cyc_exp_abs_x_d(a, gslot)), fq12d_conj(a));        // t^((x-1)^2)
  const fq12d b = fq12d_mul_ni(fq12d_conj(cyc_exp_abs_x_d(a, gslot)), fq12d_frobenius_ni(a));  // a^(x+p)
  fq12d c = fq12d_mul_ni(cyc_exp_abs_x_d(cyc_exp_abs_x_d(b, gslot), gslot), fq12d_frobenius2_ni(b));
  c = fq12d_mul_ni(c, fq12d_conj(b));                                              // b^(x^2+p^2-1)
  const fq12d t3 = fq12d_mul_ni(cyc_sqr_n_d(t, 1), t);                             // t^3
  return fq12d_mul_ni(c, t3);
}

}  // namespace hbx
