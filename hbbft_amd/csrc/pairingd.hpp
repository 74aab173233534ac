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
