// Optimal-ate pairing pieces for the batched BLS12-381 checks (pairing 0.14.2 `Bls12::pairing`
// = miller_loop + final_exponentiation, reached from threshold_crypto at honey_badger.rs:229,
// :371 and common_coin.rs:151, :196).
//
// MI355X-first restructuring (result bits identical to two independent pairings):
//  * every check e(A, Q1) == e(B, Q2) is evaluated as e(A, Q1) * e(-B, Q2) == 1 with ONE shared
//    Miller loop over both pairs and ONE final exponentiation;
//  * G2 arguments that are per-proposer constants (H_j = hash_g1_g2(U_j, V_j) and W_j) are
//    "prepared" once: the 68 line functions of the loop are stored normalised so that the y_P
//    coefficient is 1, as two Fq2 coefficients (c0, c1):  l(P) = c0 + (c1 x_P) v + y_P v w.
//    All lanes of a workgroup read the same coefficients (wave-uniform loads).
//  * the hard part of the final exponentiation uses 3 Phi_12(p)/r = (x-1)^2 (x+p)(x^2+p^2-1) + 3
//    (computes e^3; e^3 == 1 <=> e == 1 since gcd(3, r) = 1) with Granger-Scott cyclotomic
//    squarings.
#pragma once
#include "curve.hpp"

namespace hbx {

// |x| = 0xd201000000010000: 63 doubling steps after the leading bit, 5 addition steps.
constexpr int MILLER_LINES = 68;

struct line_pre {
  fq2 c0, c1;
};

// Raw line through the doubling of T (Jacobian), scaled by 2 Y Z^3:
//   c0 = 3X^3 - 2Y^2, c1 = -3X^2 Z^2, c2 = 2YZ^3;  T <- 2T.
HBX_HDNI void line_dbl_step(g2j& T, fq2& c0, fq2& c1, fq2& c2) {
  const fq2 A = fq2_sqr(T.x);
  const fq2 B = fq2_sqr(T.y);
  const fq2 C = fq2_sqr(B);
  const fq2 ZZ = fq2_sqr(T.z);
  const fq2 E = fq2_add(fq2_dbl(A), A);
  c0 = fq2_sub(fq2_mul(E, T.x), fq2_dbl(B));
  c1 = fq2_neg(fq2_mul(E, ZZ));
  fq2 D = fq2_sub(fq2_sub(fq2_sqr(fq2_add(T.x, B)), A), C);
  D = fq2_dbl(D);
  const fq2 F = fq2_sqr(E);
  const fq2 X3 = fq2_sub(F, fq2_dbl(D));
  const fq2 C8 = fq2_dbl(fq2_dbl(fq2_dbl(C)));
  const fq2 Y3 = fq2_sub(fq2_mul(E, fq2_sub(D, X3)), C8);
  const fq2 Z3 = fq2_dbl(fq2_mul(T.y, T.z));
  c2 = fq2_mul(Z3, ZZ);
  T = g2j{X3, Y3, Z3};
}

// Raw line through T and the affine base point Q, slope lambda = num/den with
// num = Y - yQ Z^3, den = Z (X - xQ Z^2); scaled by den:
//   c0 = num xQ - yQ den, c1 = -num, c2 = den;  T <- T + Q.
HBX_HDNI void line_add_step(g2j& T, const g2a& Q, fq2& c0, fq2& c1, fq2& c2) {
  const fq2 Z1Z1 = fq2_sqr(T.z);
  const fq2 U2 = fq2_mul(Q.x, Z1Z1);
  const fq2 S2 = fq2_mul(fq2_mul(Q.y, T.z), Z1Z1);
  const fq2 H = fq2_sub(U2, T.x);           // = -(X - xQ Z^2)
  const fq2 num = fq2_sub(T.y, S2);         // Y - yQ Z^3
  const fq2 den = fq2_neg(fq2_mul(T.z, H)); // Z (X - xQ Z^2)
  c0 = fq2_sub(fq2_mul(num, Q.x), fq2_mul(Q.y, den));
  c1 = fq2_neg(num);
  c2 = den;
  // madd-2007-bl
  const fq2 HH = fq2_sqr(H);
  const fq2 I = fq2_dbl(fq2_dbl(HH));
  const fq2 J = fq2_mul(H, I);
  const fq2 r = fq2_dbl(fq2_sub(S2, T.y));
  const fq2 V = fq2_mul(T.x, I);
  const fq2 X3 = fq2_sub(fq2_sub(fq2_sqr(r), J), fq2_dbl(V));
  const fq2 Y3 = fq2_sub(fq2_mul(r, fq2_sub(V, X3)), fq2_dbl(fq2_mul(T.y, J)));
  const fq2 Z3 = fq2_sub(fq2_sub(fq2_sqr(fq2_add(T.z, H)), Z1Z1), HH);
  T = g2j{X3, Y3, Z3};
}

// The 68 raw lines of Q (affine, not infinity): out[k] = (c0, c1) and c2[k] = the y_P
// coefficient, in loop order.  Only the T chain is sequential; normalising (c0, c1) / c2 is 68
// independent inversions (g2_normalise_line), so the device does them one lane per line
// (k_normalise_lines) instead of a batched inversion at the end of this lane's chain.
HBX_HDNI void g2_raw_lines(const g2a& Q, line_pre* out, fq2* c2) {
  g2j T = g2_from_affine(Q);
  int k = 0;
  for (int i = 62; i >= 0; i--) {
    line_dbl_step(T, out[k].c0, out[k].c1, c2[k]);
    k++;
    if ((BLS_X >> i) & 1) {
      line_add_step(T, Q, out[k].c0, out[k].c1, c2[k]);
      k++;
    }
  }
}

// One line scaled so its y_P coefficient is 1.
HBX_HD void g2_normalise_line(line_pre& l, const fq2& c2) {
  const fq2 inv = fq2_inv(c2);
  l.c0 = fq2_mul(l.c0, inv);
  l.c1 = fq2_mul(l.c1, inv);
}

// g2_normalise_line for lines made from (X, Y) of a Jacobian point (X, Y, Z) taken as affine: that
// is the point's image on the isomorphic twist y^2 = x^3 + b' Z^6 under (x, y) -> (Z^2 x, Z^3 y),
// and the doubling / addition steps do not involve b'.  Its lines carry c0' = Z^3 c0, c1' = Z c1,
// c2' = c2, so c0 = c0' / (c2' Z^3) and c1 = c1' Z^2 / (c2' Z^3): the line preparation needs no
// inversion of Z (k_prepare_ct's hash point).
HBX_HD void g2_normalise_line_z(line_pre& l, const fq2& c2, const fq2& z) {
  const fq2 z2 = fq2_sqr(z);
  const fq2 inv = fq2_inv(fq2_mul(c2, fq2_mul(z2, z)));
  l.c0 = fq2_mul(l.c0, inv);
  l.c1 = fq2_mul(fq2_mul(l.c1, z2), inv);
}

// Prepare the 68 normalised lines of Q (affine, not infinity) in one lane (host tools).
// `scratch` holds 2*68 Fq2 of workspace (raw c2 values and their prefix products for one
// batched inversion).
HBX_HDNI void g2_prepare_lines(const g2a& Q, line_pre* out, fq2* scratch) {
  g2_raw_lines(Q, out, scratch);
  fq2 pp = fq2_one();
  for (int k = 0; k < MILLER_LINES; k++) {
    pp = fq2_mul(pp, scratch[k]);
    scratch[MILLER_LINES + k] = pp;
  }
  fq2 inv = fq2_inv(pp);
  for (int j = MILLER_LINES - 1; j >= 0; j--) {
    const fq2 prev = j > 0 ? scratch[MILLER_LINES + j - 1] : fq2_one();
    const fq2 c2inv = fq2_mul(inv, prev);
    inv = fq2_mul(inv, scratch[j]);
    out[j].c0 = fq2_mul(out[j].c0, c2inv);
    out[j].c1 = fq2_mul(out[j].c1, c2inv);
  }
}

// f *= l(P) for a prepared line: l(P) = c0 + (c1 x_P) v + y_P v w.
HBX_HDNI fq12 mul_by_line(const fq12& f, const line_pre& l, const g1a& P) {
  const fq2 c1 = fq2_mul_fq(l.c1, P.x);
  return fq12_mul_by_014(f, l.c0, c1, P.y);
}

// Product of two Miller loops f_{|x|,QA}(PA) * f_{|x|,QB}(PB) over prepared lines, conjugated
// for x < 0.  PA / PB are affine; a pair whose `use` flag is false contributes 1 (a pairing
// with the identity).
// Inlined into its kernel with ONE copy each of the Fq12 squaring and the sparse line product
// (the line loop is not unrolled), Fq products inlined too (FqInl): f stays in registers instead
// of crossing call boundaries through scratch (an out-of-line Fq12 argument/result is a 576-byte
// scratch round trip), and the line addresses stay wave-uniform (kernel argument + block index +
// loop counters).
HBX_HD fq12 miller_loop2(const line_pre* LA, const g1a& PA, bool useA, const line_pre* LB,
                         const g1a& PB, bool useB) {
  fq12 f = fq12_one();
  int k = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (i != 62) f = fq12_sqr_t<FqInl>(f);
    const int steps = ((BLS_X >> i) & 1) ? 4 : 2;  // (A, B) lines of the doubling [+ addition]
#pragma unroll 1
    for (int s = 0; s < steps; s++) {
      const bool b = (s & 1) != 0;
      const line_pre L = ld_uniform((b ? LB : LA) + k);
      if (b ? useB : useA) {
        const fq px = b ? PB.x : PA.x;
        const fq py = b ? PB.y : PA.y;
        f = fq12_mul_by_014_t<FqInl>(f, L.c0, fq2_mul_fq_t<FqInl>(L.c1, px), py);
      }
      if (b) k++;
    }
  }
  return fq12_conj(f);
}

// f * (c0 + c1 v + c4 v w) with c4 in Fq2: an UN-normalised line (l scaled by its Fq2 factor,
// which the final exponentiation removes) evaluated at a G1 point.
HBX_HDNI fq12 fq12_mul_by_014_f2(const fq12& f, const fq2& c0, const fq2& c1, const fq2& c4) {
  const fq6 aa = fq6_mul_by_01(f.c0, c0, c1);
  const fq6 bb = fq6{fq2_mul_xi(fq2_mul(f.c1.c2, c4)), fq2_mul(f.c1.c0, c4), fq2_mul(f.c1.c1, c4)};
  const fq2 o = fq2_add(c1, c4);
  fq6 s = fq6_add(f.c1, f.c0);
  s = fq6_mul_by_01(s, c0, o);
  const fq6 n1 = fq6_sub(fq6_sub(s, aa), bb);
  const fq6 n0 = fq6_add(fq6_mul_v(bb), aa);
  return fq12{n0, n1};
}

// Two-pair Miller loop where pair A uses prepared lines and pair B's G2 point varies per check
// (a signature share, common_coin.rs:151): B's lines are generated on the fly from T = QB and
// evaluated un-normalised at PB.  Returns conj(f) like miller_loop2.
HBX_HDNI fq12 miller_loop_mixed(const line_pre* LA, const g1a& PA, bool useA, const g2a& QB, const g1a& PB,
                                bool useB) {
  fq12 f = fq12_one();
  g2j T = g2_from_affine(QB);
  int k = 0;
  for (int i = 62; i >= 0; i--) {
    if (i != 62) f = fq12_sqr(f);
    if (useA) f = mul_by_line(f, LA[k], PA);
    if (useB) {
      fq2 c0, c1, c2;
      line_dbl_step(T, c0, c1, c2);
      f = fq12_mul_by_014_f2(f, c0, fq2_mul_fq(c1, PB.x), fq2_mul_fq(c2, PB.y));
    }
    k++;
    if ((BLS_X >> i) & 1) {
      if (useA) f = mul_by_line(f, LA[k], PA);
      if (useB) {
        fq2 c0, c1, c2;
        line_add_step(T, QB, c0, c1, c2);
        f = fq12_mul_by_014_f2(f, c0, fq2_mul_fq(c1, PB.x), fq2_mul_fq(c2, PB.y));
      }
      k++;
    }
  }
  return fq12_conj(f);
}

// g^|x| for g in the cyclotomic subgroup.
// One inlined copy of the cyclotomic squaring and of the Fq12 product in a non-unrolled loop:
// r and g stay in registers across the 63 squarings.
HBX_HDNI fq12 cyc_exp_abs_x(const fq12& g_in) {
  const fq12 g = g_in;
  fq12 r = g;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    r = fq12_cyclotomic_sqr_i(r);
    if ((BLS_X >> i) & 1) r = fq12_mul_i(r, g);
  }
  return r;
}
// g^x (x negative) = conj(g^|x|) in the cyclotomic subgroup.
HBX_HD fq12 cyc_exp_x(const fq12& g) { return fq12_conj(cyc_exp_abs_x(g)); }

// f^(3 (p^12 - 1)/r)
HBX_HDNI fq12 final_exponentiation(const fq12& f) {
  // easy part: f^((p^6 - 1)(p^2 + 1))
  fq12 t = fq12_mul(fq12_conj(f), fq12_inv(f));
  t = fq12_mul(fq12_frobenius2(t), t);
  // hard part
  fq12 a = fq12_mul(cyc_exp_x(t), fq12_conj(t));      // t^(x-1)
  a = fq12_mul(cyc_exp_x(a), fq12_conj(a));            // t^((x-1)^2)
  fq12 b = fq12_mul(cyc_exp_x(a), fq12_frobenius(a));  // a^(x+p)
  fq12 c = fq12_mul(cyc_exp_x(cyc_exp_x(b)), fq12_frobenius2(b));
  c = fq12_mul(c, fq12_conj(b));                        // b^(x^2 + p^2 - 1)
  const fq12 t3 = fq12_mul(fq12_cyclotomic_sqr(t), t);  // t^3
  return fq12_mul(c, t3);
}

#if defined(__HIPCC__)
// The same final exponentiation with the exponentiation base parked in LDS.
// Why: in cyc_exp_abs_x the running power r (144 dwords) and the base g (144 dwords) do not both
// fit the 256 VGPRs next to the squaring's temporaries, so the compiler spilled ~60 scratch
// accesses into every cyclotomic squaring and ~560 into every multiplication -- ~300 KB of
// scratch traffic per share check (profiles/r01_s5_pmc_fq28.txt).  g is read only at the 5 one
// bits of |x|, so it lives in this lane's LDS slot instead: 144 dwords, lane-interleaved
// (dword i at base[i * 64]), so a wave's accesses are bank-conflict free.  One slot per lane
// (36 KB per 64-lane block) keeps the single-wave-per-SIMD occupancy.  Each lane touches only its
// own slot: no barrier.
constexpr int LDS_FQ12_STRIDE = 64;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ void lds_put_fq12(lds_u32* base, const fq12& a) {
  const uint32_t* p = reinterpret_cast<const uint32_t*>(&a);
#pragma unroll
  for (int i = 0; i < 144; i++) base[i * LDS_FQ12_STRIDE] = p[i];
}
__device__ __forceinline__ fq12 lds_get_fq12(const lds_u32* base) {
  fq12 a;
  uint32_t* p = reinterpret_cast<uint32_t*>(&a);
#pragma unroll
  for (int i = 0; i < 144; i++) p[i] = base[i * LDS_FQ12_STRIDE];
  return a;
}
// r^(2^k) by k cyclotomic squarings (Fq products inlined): only r is live in the loop
__device__ __forceinline__ fq12 cyc_sqr_n(fq12 r, int k) {
#pragma unroll 1
  for (int i = 0; i < k; i++) r = fq12_cyclotomic_sqr_t<FqInl>(r);
  return r;
}
// g^|x| with |x| = 0xd201000000010000 written out as runs of squarings between its one bits
// (bits 63, 62, 60, 57, 48, 16): no per-bit branch, and g is reloaded from LDS only for the five
// multiplications.
__device__ __noinline__ fq12 cyc_exp_abs_x_lds(const fq12& g_in, lds_u32* gslot) {
  static_assert(BLS_X == 0xd201000000010000ull, "square-and-multiply runs are specific to |x|");
  lds_put_fq12(gslot, g_in);
  // squaring runs before the multiplications at bits 62, 60, 57, 48, 16, then bits 15..0; one
  // copy of the (inlined) squaring loop
  fq12 r = g_in;
#pragma unroll 1
  for (int q = 0; q < 6; q++) {
    const int run = q == 0 ? 1 : q == 1 ? 2 : q == 2 ? 3 : q == 3 ? 9 : q == 4 ? 32 : 16;
    r = cyc_sqr_n(r, run);
    if (q < 5) r = fq12_mul(r, lds_get_fq12(gslot));
  }
  return r;
}
__device__ __forceinline__ fq12 cyc_exp_x_lds(const fq12& g, lds_u32* gslot) {
  return fq12_conj(cyc_exp_abs_x_lds(g, gslot));
}
// f^(3 (p^12 - 1)/r), as final_exponentiation, exponentiations through cyc_exp_x_lds.
__device__ __noinline__ fq12 final_exponentiation_lds(const fq12& f, lds_u32* gslot) {
  fq12 t = fq12_mul(fq12_conj(f), fq12_inv(f));
  t = fq12_mul(fq12_frobenius2(t), t);
  fq12 a = fq12_mul(cyc_exp_x_lds(t, gslot), fq12_conj(t));
  a = fq12_mul(cyc_exp_x_lds(a, gslot), fq12_conj(a));
  fq12 b = fq12_mul(cyc_exp_x_lds(a, gslot), fq12_frobenius(a));
  fq12 c = fq12_mul(cyc_exp_x_lds(cyc_exp_x_lds(b, gslot), gslot), fq12_frobenius2(b));
  c = fq12_mul(c, fq12_conj(b));
  const fq12 t3 = fq12_mul(fq12_cyclotomic_sqr(t), t);
  return fq12_mul(c, t3);
}
#endif

// e(PA, QA) * e(PB, QB) == 1 with prepared lines for QA, QB.
HBX_HD bool pairing_check2(const line_pre* LA, const g1a& PA, const line_pre* LB, const g1a& PB) {
  const fq12 f = miller_loop2(LA, PA, true, LB, PB, true);
  return fq12_is_one(final_exponentiation(f));
}

}  // namespace hbx
