// Developer tool: builds the HIP kernels' __host__ __device__ arithmetic for the CPU so it can be
// unit-tested against the Python oracle in a container without a GPU.  NOT part of the product
// (libhbx.so never contains or calls this); see tests/test_hostcheck.py.
#include <cstring>
#include "../../hbbft_amd/csrc/pairing.hpp"
#include "../../hbbft_amd/csrc/pairingd.hpp"
#include "../../hbbft_amd/csrc/fe1d.hpp"
#include "../../hbbft_amd/csrc/g2d.hpp"
#include "../../hbbft_amd/csrc/g1d.hpp"
#include "../../hbbft_amd/csrc/hash.hpp"
using namespace hbx;
extern "C" {
// canonical big-endian 48-byte operands
void hc_fq_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  fq x = fq_to_mont(fq_from_be(a)), y = fq_to_mont(fq_from_be(b));
  fq_to_be(fq_from_mont(fq_mul(x, y)), out);
}
// raw limbs (little-endian 12 x u32, any value < 2^384): the Montgomery product fq_mul itself,
// so tests can drive lazy-range operands in [0, 2p] and check r = a b 2^-384 mod p, r < 2p
void hc_fq_mul_raw(const uint32_t* a, const uint32_t* b, uint32_t* out) {
  fq x, y;
  for (int i = 0; i < 12; i++) { x.l[i] = a[i]; y.l[i] = b[i]; }
  const fq r = fq_mul(x, y);
  for (int i = 0; i < 12; i++) out[i] = r.l[i];
}
void hc_fq_sqr_raw(const uint32_t* a, uint32_t* out) {
  fq x;
  for (int i = 0; i < 12; i++) x.l[i] = a[i];
  const fq r = fq_sqr(x);
  for (int i = 0; i < 12; i++) out[i] = r.l[i];
}
// subgroup checks on raw affine coordinates (canonical big-endian; G2 as x.c1||x.c0||y.c1||y.c0):
// 1 = in G1/G2, 0 = not, -1 = not on the curve
int hc_g1_torsion_free(const uint8_t* x48, const uint8_t* y48) {
  g1a p;
  p.x = fq_to_mont(fq_from_be(x48));
  p.y = fq_to_mont(fq_from_be(y48));
  p.inf = false;
  const fq rhs = fq_add(fq_mul(fq_sqr(p.x), p.x), fq_from_const(FQ_B1));
  if (!fq_eq(fq_sqr(p.y), rhs)) return -1;
  // the 12-limb check and the digit-tower one (g1d.hpp, the decode kernels'): -2 if they differ
  const bool a = g1_is_torsion_free(p), b = g1_is_torsion_free_d(p);
  return a != b ? -2 : a ? 1 : 0;
}
int hc_g2_torsion_free(const uint8_t* xy192) {
  g2a q;
  q.x = fq2{fq_to_mont(fq_from_be(xy192 + 48)), fq_to_mont(fq_from_be(xy192))};
  q.y = fq2{fq_to_mont(fq_from_be(xy192 + 144)), fq_to_mont(fq_from_be(xy192 + 96))};
  q.inf = false;
  const fq2 rhs = fq2_add(fq2_mul(fq2_sqr(q.x), q.x), g2_b());
  if (!fq2_eq(fq2_sqr(q.y), rhs)) return -1;
  return g2_is_torsion_free(q) ? 1 : 0;
}
void hc_fq_inv(const uint8_t* a, uint8_t* out) {
  fq x = fq_to_mont(fq_from_be(a));
  fq_to_be(fq_from_mont(fq_inv(x)), out);
}
// raw Montgomery limbs (lazy range allowed): fq_inv / fr_inv themselves
void hc_fq_inv_raw(const uint32_t* a, uint32_t* out) {
  fq x;
  for (int i = 0; i < 12; i++) x.l[i] = a[i];
  const fq r = fq_canon(fq_inv(x));
  for (int i = 0; i < 12; i++) out[i] = r.l[i];
}
void hc_fr_inv_raw(const uint32_t* a, uint32_t* out) {
  fr x;
  for (int i = 0; i < 8; i++) x.l[i] = a[i];
  const fr r = fr_csub(fr_inv(x));
  for (int i = 0; i < 8; i++) out[i] = r.l[i];
}
int hc_g1_roundtrip(const uint8_t* in48, uint8_t* out48) {
  g1a p; int st = g1_decompress(in48, p);
  // the decode kernels' digit-tower square root gives the same status and point (-100 if not)
  g1a q; const int sd = g1_decompress_d(in48, q);
  if (sd != st || (st == HBX_PT_OK && !(fq_eq(p.x, q.x) && fq_eq(p.y, q.y)))) return -100;
  if (st != HBX_PT_OK && st != HBX_PT_INFINITY) return st;
  g1_compress(p, out48); return st;
}
int hc_g2_roundtrip(const uint8_t* in96, uint8_t* out96) {
  g2a p; int st = g2_decompress(in96, p);
  if (st != HBX_PT_OK && st != HBX_PT_INFINITY) return st;
  g2_compress(p, out96); return st;
}
// returns 1 if e(PA,QA) e(PB,QB) == 1, 0 if not, negative on decode failure
int hc_pairing_check2(const uint8_t* pa, const uint8_t* qa, const uint8_t* pb, const uint8_t* qb) {
  g1a PA, PB; g2a QA, QB;
  if (g1_decompress(pa, PA) != HBX_PT_OK) return -1;
  if (g1_decompress(pb, PB) != HBX_PT_OK) return -2;
  if (g2_decompress(qa, QA) != HBX_PT_OK) return -3;
  if (g2_decompress(qb, QB) != HBX_PT_OK) return -4;
  static line_pre LA[MILLER_LINES], LB[MILLER_LINES];
  static fq2 scratch[2 * MILLER_LINES];
  g2_prepare_lines(QA, LA, scratch);
  g2_prepare_lines(QB, LB, scratch);
  return pairing_check2(LA, PA, LB, PB) ? 1 : 0;
}
// The share check's digit-form Miller loop (pairingd.hpp) against pairing.hpp's on the same
// prepared lines: 1 = the same Fq12 element, and *check = the pairing check through it.
int hc_miller2_digit_cmp(const uint8_t* pa, const uint8_t* qa, const uint8_t* pb, const uint8_t* qb, int* check) {
  g1a PA, PB; g2a QA, QB;
  if (g1_decompress(pa, PA) != HBX_PT_OK) return -1;
  if (g1_decompress(pb, PB) != HBX_PT_OK) return -2;
  if (g2_decompress(qa, QA) != HBX_PT_OK) return -3;
  if (g2_decompress(qb, QB) != HBX_PT_OK) return -4;
  static line_pre LA[MILLER_LINES], LB[MILLER_LINES];
  static line_pre_d DA[MILLER_LINES], DB[MILLER_LINES];
  static fq2 scratch[2 * MILLER_LINES];
  g2_prepare_lines(QA, LA, scratch);
  g2_prepare_lines(QB, LB, scratch);
  for (int i = 0; i < MILLER_LINES; i++) {
    DA[i] = line_to_d(LA[i]);
    DB[i] = line_to_d(LB[i]);
  }
  const fq12 f = miller_loop2(LA, PA, true, LB, PB, true);
  const fq12 g = fq12d_to_fq12(miller_loop2_d(DA, fqd_from_fq(PA.x), fqd_from_fq(PA.y), true, DB,
                                              fqd_from_fq(PB.x), fqd_from_fq(PB.y), true));
  // the loop with the G1 points parked in the (host: plain) slot gives the same element
  static uint32_t park[LDS_FQ12D_DWORDS];
  park_put_fqd(park, 0, fqd_from_fq(PA.x));
  park_put_fqd(park, 1, fqd_from_fq(PA.y));
  park_put_fqd(park, 2, fqd_from_fq(PB.x));
  park_put_fqd(park, 3, fqd_from_fq(PB.y));
  const fq12 gp = fq12d_to_fq12(miller_loop2_parked_d(DA, true, DB, true, park));
  const fq* a = &f.c0.c0.c0;
  const fq* b = &g.c0.c0.c0;
  const fq* c = &gp.c0.c0.c0;
  int same = 1;
  for (int i = 0; i < 12; i++) same &= (fq_eq(a[i], b[i]) && fq_eq(a[i], c[i])) ? 1 : 0;
  *check = fq12_is_one(final_exponentiation(g)) ? 1 : 0;
  // the digit-form final exponentiation gives the same element as pairing.hpp's
  static uint32_t slot[LDS_FQ12D_DWORDS];
  const fq12 e1 = final_exponentiation(g);
  const fq12 e2 = fq12d_to_fq12(final_exponentiation_d(fq12d_from_fq12(g), slot));
  const fq* x = &e1.c0.c0.c0;
  const fq* y = &e2.c0.c0.c0;
  int same_fe = 1;
  for (int i = 0; i < 12; i++) same_fe &= fq_eq(x[i], y[i]) ? 1 : 0;
  // the loop over lines divided by y_P (miller_loop2_scaled_d, the one-lane Miller kernel): a
  // different element (Fq factors), the same element after the final exponentiation
  park_scaled_points(park, PA.x, PA.y, false, PB.x, PB.y, false);
  const fq12 gs = fq12d_to_fq12(miller_loop2_scaled_d(DA, true, DB, true, park));
  const fq12 e3 = final_exponentiation(gs);
  const fq* z = &e3.c0.c0.c0;
  int same_scaled = 1;
  for (int i = 0; i < 12; i++) same_scaled &= fq_eq(x[i], z[i]) ? 1 : 0;
  return same + 2 * same_fe * same_scaled;
}
// The final exponentiation as k_fe1's five steps (fe1d.hpp) on host slots, against
// final_exponentiation_d on the same Miller output: 1 = the same element, + 2 if the verdicts
// (fq12d_is_one_seq vs fq12_is_one) agree, + 4 if the check holds.
int hc_fe1_chain_cmp(const uint8_t* pa, const uint8_t* qa, const uint8_t* pb, const uint8_t* qb) {
  g1a PA, PB; g2a QA, QB;
  if (g1_decompress(pa, PA) != HBX_PT_OK) return -1;
  if (g1_decompress(pb, PB) != HBX_PT_OK) return -2;
  if (g2_decompress(qa, QA) != HBX_PT_OK) return -3;
  if (g2_decompress(qb, QB) != HBX_PT_OK) return -4;
  static line_pre LA[MILLER_LINES], LB[MILLER_LINES];
  static line_pre_d DA[MILLER_LINES], DB[MILLER_LINES];
  static fq2 scratch[2 * MILLER_LINES];
  g2_prepare_lines(QA, LA, scratch);
  g2_prepare_lines(QB, LB, scratch);
  for (int i = 0; i < MILLER_LINES; i++) {
    DA[i] = line_to_d(LA[i]);
    DB[i] = line_to_d(LB[i]);
  }
  const fq12d fd = miller_loop2_d(DA, fqd_from_fq(PA.x), fqd_from_fq(PA.y), true, DB, fqd_from_fq(PB.x),
                                  fqd_from_fq(PB.y), true);
  static uint32_t slot[LDS_FQ12D_DWORDS];
  const fq12 e1 = fq12d_to_fq12(final_exponentiation_d(fd, slot));
  // the Miller kernel's hand-over: conj(f) stored normalised in slot F
  static uint32_t a[FE1_WORDS], gf[FE1_WORDS], gt[FE1_WORDS], gg[FE1_WORDS];
  s1_put_fq12d<1>(gf, fq12d{fd.c0, fq6d_norm(fd.c1)});
  bool degenerate = false;
  const fq12d e2d = fe1_chain<1, 1>(a, gf, gt, gg, degenerate);
  if (degenerate) return -5;
  const fq12 e2 = fq12d_to_fq12(e2d);
  const fq* x = &e1.c0.c0.c0;
  const fq* y = &e2.c0.c0.c0;
  int same = 1;
  for (int i = 0; i < 12; i++) same &= fq_eq(x[i], y[i]) ? 1 : 0;
  const bool v1 = fq12_is_one(e1), v2 = fq12d_is_one_seq(e2d);
  return same + 2 * (v1 == v2 ? 1 : 0) + 4 * (v2 ? 1 : 0);
}
// k_fe1<0>'s early decision: bit 0 = step 0 found t = 1, bit 1 = the rest of the chain would have met
// a degenerate compressed run (g3 = 0), bit 2 = the chain's verdict is 1
int hc_fe1_step0_one(const uint8_t* pa, const uint8_t* qa, const uint8_t* pb, const uint8_t* qb) {
  g1a PA, PB; g2a QA, QB;
  if (g1_decompress(pa, PA) != HBX_PT_OK || g1_decompress(pb, PB) != HBX_PT_OK) return -1;
  if (g2_decompress(qa, QA) != HBX_PT_OK || g2_decompress(qb, QB) != HBX_PT_OK) return -2;
  static line_pre LA[MILLER_LINES], LB[MILLER_LINES];
  static line_pre_d DA[MILLER_LINES], DB[MILLER_LINES];
  static fq2 scratch[2 * MILLER_LINES];
  g2_prepare_lines(QA, LA, scratch);
  g2_prepare_lines(QB, LB, scratch);
  for (int i = 0; i < MILLER_LINES; i++) {
    DA[i] = line_to_d(LA[i]);
    DB[i] = line_to_d(LB[i]);
  }
  const fq12d fd = miller_loop2_d(DA, fqd_from_fq(PA.x), fqd_from_fq(PA.y), true, DB, fqd_from_fq(PB.x),
                                  fqd_from_fq(PB.y), true);
  static uint32_t a[FE1_WORDS], gf[FE1_WORDS], gt[FE1_WORDS], gg[FE1_WORDS];
  s1_put_fq12d<1>(gf, fq12d{fd.c0, fq6d_norm(fd.c1)});
  const bool one = fe1_step0<1, 1>(a, gf, gt, gg);
  bool degenerate = false;
  fe1_step12<1, 1>(a, gt, gg, degenerate);
  fe1_step34<1, 1>(a, gf, gt, gg, degenerate);
  const bool v = fq12d_is_one_seq(fe1_step56<1, 1>(a, gf, gt, degenerate));
  return (one ? 1 : 0) + (degenerate ? 2 : 0) + (v ? 4 : 0);
}
// digit-form product against the 12-limb one on canonical inputs: out = canonical a b (BE)
void hc_fqd_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  const fqd x = fqd_from_fq(fq_to_mont(fq_from_be(a))), y = fqd_from_fq(fq_to_mont(fq_from_be(b)));
  fq_to_be(fq_from_mont(fqd_to_fq(fqd_mul(x, y))), out);
}
void hc_fq2d_mul(const uint8_t* a, const uint8_t* b, uint8_t* out, int sqr) {
  const fq2d x{fqd_from_fq(fq_to_mont(fq_from_be(a))), fqd_from_fq(fq_to_mont(fq_from_be(a + 48)))};
  const fq2d y{fqd_from_fq(fq_to_mont(fq_from_be(b))), fqd_from_fq(fq_to_mont(fq_from_be(b + 48)))};
  const fq2d r = sqr ? fq2d_sqr(x) : fq2d_mul(x, y);
  fq_to_be(fq_from_mont(fqd_to_fq(r.c0)), out);
  fq_to_be(fq_from_mont(fqd_to_fq(r.c1)), out + 48);
}
// fq4d_sqr_lazy on (a, b) = 4 canonical Fq (BE) each shifted by shift[q] p (-1, 0, 1: the ends of the
// normalised range), against the product itself: out = canonical c0 || c1 (4 x 48 BE)
void hc_fq4d_sqr_lazy(const uint8_t* in, const int* shift, uint8_t* out) {
  fqd v[4];
  for (int q = 0; q < 4; q++) {
    v[q] = fqd_from_fq(fq_to_mont(fq_from_be(in + 48 * q)));
    fqd pd;
    for (int i = 0; i < 14; i++) pd.d[i] = (int32_t)FQ_P28[i] * shift[q];
    v[q] = fqd_norm(fqd_add(v[q], pd));
  }
  fq2d c0, c1;
  fq4d_sqr_lazy(fq2d{v[0], v[1]}, fq2d{v[2], v[3]}, c0, c1);
  const fqd* r[4] = {&c0.c0, &c0.c1, &c1.c0, &c1.c1};
  for (int q = 0; q < 4; q++) fq_to_be(fq_from_mont(fqd_to_fq(*r[q])), out + 48 * q);
}
// e(PA, QA) e(PB, QB) == 1 with QA prepared and QB's lines generated on the fly
int hc_pairing_check_mixed(const uint8_t* pa, const uint8_t* qa, const uint8_t* pb, const uint8_t* qb) {
  g1a PA, PB; g2a QA, QB;
  if (g1_decompress(pa, PA) != HBX_PT_OK) return -1;
  if (g1_decompress(pb, PB) != HBX_PT_OK) return -2;
  if (g2_decompress(qa, QA) != HBX_PT_OK) return -3;
  if (g2_decompress(qb, QB) != HBX_PT_OK) return -4;
  static line_pre LA[MILLER_LINES];
  static fq2 scratch[2 * MILLER_LINES];
  g2_prepare_lines(QA, LA, scratch);
  return fq12_is_one(final_exponentiation(miller_loop_mixed(LA, PA, true, QB, PB, true))) ? 1 : 0;
}
// the coin check in the digit tower (miller_loop_mixed_d + final_exponentiation_d) against
// pairing.hpp's: returns 1 + 2 (Miller output equal) + 4 (final exponentiation equal) when the
// check holds, 0 + 2 + 4 when it does not; -1.. on a bad encoding
int hc_pairing_check_mixed_d(const uint8_t* pa, const uint8_t* qa, const uint8_t* pb, const uint8_t* qb) {
  g1a PA, PB; g2a QA, QB;
  if (g1_decompress(pa, PA) != HBX_PT_OK) return -1;
  if (g1_decompress(pb, PB) != HBX_PT_OK) return -2;
  if (g2_decompress(qa, QA) != HBX_PT_OK) return -3;
  if (g2_decompress(qb, QB) != HBX_PT_OK) return -4;
  static line_pre LA[MILLER_LINES];
  static line_pre_d DA[MILLER_LINES];
  static fq2 scratch[2 * MILLER_LINES];
  g2_prepare_lines(QA, LA, scratch);
  for (int i = 0; i < MILLER_LINES; i++) DA[i] = line_to_d(LA[i]);
  const fq12 f = miller_loop_mixed(LA, PA, true, QB, PB, true);
  const fq12d fd = miller_loop_mixed_d(DA, fqd_from_fq(PA.x), fqd_from_fq(PA.y), true, fq2d_from_fq2(QB.x),
                                       fq2d_from_fq2(QB.y), fqd_from_fq(PB.x), fqd_from_fq(PB.y), true);
  const fq12 g = fq12d_to_fq12(fd);
  static uint32_t slot[LDS_FQ12D_DWORDS];
  const fq12 e1 = final_exponentiation(f);
  const fq12 e2 = fq12d_to_fq12(final_exponentiation_d(fd, slot));
  const fq* a = &f.c0.c0.c0; const fq* b = &g.c0.c0.c0;
  const fq* x = &e1.c0.c0.c0; const fq* y = &e2.c0.c0.c0;
  int same_m = 1, same_e = 1;
  for (int i = 0; i < 12; i++) { same_m &= fq_eq(a[i], b[i]) ? 1 : 0; same_e &= fq_eq(x[i], y[i]) ? 1 : 0; }
  return (fq12_is_one(e2) ? 1 : 0) + 2 * same_m + 4 * same_e;
}
// k * P (P compressed, k 32-byte big-endian canonical scalar) through the GLV split, as k_combine
int hc_g1_mul_glv(const uint8_t* in48, const uint8_t* k32, uint8_t* out48) {
  g1a p; if (g1_decompress(in48, p) != HBX_PT_OK) return -1;
  uint32_t k8[8];
  for (int i = 0; i < 8; i++) {
    const uint8_t* q = k32 + 28 - 4 * i;
    k8[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
  uint32_t k1[4], k2[4];
  g1_glv_split(k8, k1, k2);
  g1a ph = p;
  ph.x = fq_mul(p.x, fq_from_const(G1_BETA));
  g1j r = g1_add(g1_mul_u128_w4(p, k1), g1_mul_u128_w4(ph, k2));  // k_combine's windowed product
  g1_compress(g1_to_affine(r), out48); return 0;
}
// Q = h_eff P (k_prepare_ct's H') and back to h2 P (hbx_get_ct_hashes)
int hc_g2_heff(const uint8_t* in96, uint8_t* q96, uint8_t* h96) {
  g2a p; if (g2_decompress(in96, p) != HBX_PT_OK) return -1;
  const g2j q = g2_heff(g2_from_affine(p));
  g2_compress(g2_to_affine(q), q96);
  g2_compress(g2_to_affine(g2_heff_to_h2(q)), h96);
  return 0;
}
// Lines of Q from (X, Y) of its Jacobian form (x z^2, y z^3, z) taken as affine, corrected by z in
// the normalisation (k_prepare_lines + k_normalise_lines on k_prepare_ct's H'), against the affine
// point's lines: returns the number of differing lines (0 = identical)
int hc_lines_jac_cmp(const uint8_t* in96, const uint8_t* z0_48, const uint8_t* z1_48) {
  g2a q; if (g2_decompress(in96, q) != HBX_PT_OK || q.inf) return -1;
  fq2 z; z.c0 = fq_from_be(z0_48); z.c1 = fq_from_be(z1_48);
  const fq2 zz = fq2_sqr(z);
  g2a qz = q; qz.x = fq2_mul(q.x, zz); qz.y = fq2_mul(q.y, fq2_mul(zz, z));
  static line_pre a[MILLER_LINES], b[MILLER_LINES];
  static fq2 ca[MILLER_LINES], cb[MILLER_LINES];
  g2_raw_lines(q, a, ca);
  g2_raw_lines(qz, b, cb);
  int bad = 0;
  for (int i = 0; i < MILLER_LINES; i++) {
    g2_normalise_line(a[i], ca[i]);
    g2_normalise_line_z(b[i], cb[i], z);
    if (!fq2_eq(a[i].c0, b[i].c0) || !fq2_eq(a[i].c1, b[i].c1)) bad++;
  }
  return bad;
}
// fieldd.hpp fqd_inv on 14 signed digits (any value in (-2p, 3p)): out = the 14 result digits,
// returns the zero flag
int hc_fqd_inv(const int32_t* a14, int32_t* out14) {
  fqd a;
  for (int i = 0; i < 14; i++) a.d[i] = a14[i];
  bool zero = false;
  const fqd r = fqd_inv(a, zero);
  for (int i = 0; i < 14; i++) out14[i] = r.d[i];
  return zero ? 1 : 0;
}
// binv_limbs (batched divsteps) on canonical little-endian limbs: which = 0 mod p (12 limbs),
// 1 mod r (8 limbs)
int hc_binv(const uint32_t* x, int which, uint32_t* out) {
  if (which == 0) binv_limbs<12>(x, FQ_P, out);
  else binv_limbs<8>(x, FR_R, out);
  return 0;
}
int hc_g1_scale_heff_m(const uint8_t* in48, uint8_t* out48) {
  g1a p; if (g1_decompress(in48, p) != HBX_PT_OK) return -1;
  g1_compress(g1_to_affine(g1_mul_scalar(g1_from_affine(p), HEFF_M)), out48); return 0;
}
int hc_g2_clear_cofactor(const uint8_t* in96, uint8_t* out96) {
  g2a p; if (g2_decompress(in96, p) != HBX_PT_OK) return -1;
  g2_compress(g2_to_affine(g2_clear_cofactor(g2_from_affine(p))), out96); return 0;
}
int hc_g2_mul_cofactor(const uint8_t* in96, uint8_t* out96) {
  g2a p; if (g2_decompress(in96, p) != HBX_PT_OK) return -1;
  g2j r = g2_mul_bits(g2_from_affine(p), G2_COFACTOR, G2_COFACTOR_BITS);
  g2_compress(g2_to_affine(r), out96); return 0;
}
}
extern "C" {
void hc_sha256(const uint8_t* m, uint64_t n, uint8_t* out32) { sha256_2(m, n, nullptr, 0, out32); }
void hc_sha3_256(const uint8_t* m, uint64_t n, uint8_t* out32) { sha3_256_2(m, n, nullptr, 0, out32); }
// two-range form (the split point exercises the concatenation path)
void hc_sha3_256_2(const uint8_t* m0, uint64_t n0, const uint8_t* m1, uint64_t n1, uint8_t* out32) {
  sha3_256_2(m0, n0, m1, n1, out32);
}
int hc_hash_g1_g2(const uint8_t* u48, const uint8_t* v, uint64_t vlen, uint8_t* out96) {
  g2j h = hash_g1_g2(u48, v, vlen);
  g2_compress(g2_to_affine(h), out96); return 0;
}
int hc_hash_g1_g2_v(const uint8_t* u48, const uint8_t* v, uint64_t vlen, int variant, uint8_t* out96) {
  g2j h = hash_g1_g2(u48, v, vlen, variant);
  g2_compress(g2_to_affine(h), out96); return 0;
}
int hc_hash_g2_digest(const uint8_t* d32, uint8_t* out96) {
  g2_compress(g2_to_affine(hash_g2_from_digest(d32)), out96); return 0;
}
}
extern "C" {
// G2 membership of a compressed point two ways: bit 0 from the mixed Miller loop's final
// T = [|x|] Q (g2_torsion_free_from_T, the coin checks), bit 1 from g2_is_torsion_free (decode);
// -1 if the bytes do not decode to a curve point.
int hc_g2_membership(const uint8_t* q96) {
  g2a Q;
  const int32_t st = g2_decompress(q96, Q);
  if (st != HBX_PT_OK && st != HBX_PT_INFINITY) return -1;
  const fqd z = fqd_zero();
  const fq gx = fq_from_const(G1_MGEN_X), gy = fq_neg(fq_from_const(G1_MGEN_Y));
  g2jd T;
  (void)miller_loop_mixed_d(nullptr, z, z, false, fq2d_from_fq2(Q.x), fq2d_from_fq2(Q.y), fqd_from_fq(gx), fqd_from_fq(gy),
                            !Q.inf, &T);
  return (g2_torsion_free_from_T(T, Q) ? 1 : 0) | (g2_is_torsion_free(Q) ? 2 : 0);
}
}
extern "C" {
// [k] Q (Q compressed, k 64-bit) by g2_mul_u64_w4 and by g2_mul_u64_naf: 1 if the affine results
// agree, 0 if not, -1 if Q does not decode.
int hc_g2_mul_u64_cmp(const uint8_t* q96, uint64_t k) {
  g2a Q;
  if (g2_decompress(q96, Q) != HBX_PT_OK) return -1;
  const g2a a = g2_to_affine(g2_mul_u64_w4(Q, k)), b = g2_to_affine(g2_mul_u64_naf(Q, k));
  // and the digit-tower multiplication (g2d.hpp, k_combine_sigs)
  bool dinf;
  const g2jd cd = g2d_mul_u64_w4(fq2d_from_fq2(Q.x), fq2d_from_fq2(Q.y), k, dinf);
  const g2a c = dinf ? g2_to_affine(g2_identity()) : g2_to_affine(g2jd_to_g2j(cd));
  if (a.inf || b.inf || c.inf) return a.inf == b.inf && b.inf == c.inf ? 1 : 0;
  return fq2_eq(a.x, b.x) && fq2_eq(a.y, b.y) && fq2_eq(a.x, c.x) && fq2_eq(a.y, c.y) ? 1 : 0;
}
// the threshold combine's 128-bit G1 window multiplication: digit tower (g1d.hpp) against the
// 12-limb curve.hpp g1_mul_u128_w4 (k4: four little-endian words)
int hc_g1_mul_u128_cmp(const uint8_t* p48, const uint32_t* k4) {
  g1a P;
  if (g1_decompress(p48, P) != HBX_PT_OK) return -1;
  const g1a a = g1_to_affine(g1_mul_u128_w4(P, k4)), b = g1_to_affine(g1d_mul_u128_w4(P, k4));
  if (a.inf || b.inf) return a.inf == b.inf ? 1 : 0;
  return fq_eq(a.x, b.x) && fq_eq(a.y, b.y) ? 1 : 0;
}
// g2d_add (digit tower, exact special cases) against g2_add over the cases the combine's lane tree
// can meet: P + Q, P + P, P + (-P), O + P, P + O, O + O, with the operands' Z scaled by z0
// (Jacobian inputs, not only Z = 1).  Returns a bit mask of the cases that agree (63 = all).
int hc_g2d_add_cases(const uint8_t* p96, const uint8_t* q96, uint64_t z0) {
  g2a P, Q;
  if (g2_decompress(p96, P) != HBX_PT_OK || g2_decompress(q96, Q) != HBX_PT_OK) return -1;
  auto small = [](uint64_t v) {
    fq a{};
    a.l[0] = (uint32_t)v;
    a.l[1] = (uint32_t)(v >> 32);
    return fq_to_mont(a);
  };
  const fq2 z{small(z0), small(z0 + 7)};
  auto jac = [&](const g2a& a, bool neg) {
    const fq2 z2 = fq2_sqr(z);
    const fq2 y = neg ? fq2_neg(a.y) : a.y;
    return g2j{fq2_mul(a.x, z2), fq2_mul(fq2_mul(y, z2), z), z};
  };
  auto tod = [](const g2j& a) { return g2jd{fq2d_from_fq2(a.x), fq2d_from_fq2(a.y), fq2d_from_fq2(a.z)}; };
  const g2j Pj = jac(P, false), Qj = g2_from_affine(Q), Pn = jac(P, true), O = g2_identity();
  const g2j cases[6][2] = {{Pj, Qj}, {Pj, g2_from_affine(P)}, {Pj, Pn}, {O, Pj}, {Qj, O}, {O, O}};
  int mask = 0;
  for (int c = 0; c < 6; c++) {
    const g2a want = g2_to_affine(g2_add(cases[c][0], cases[c][1]));
    const g2a got = g2_to_affine(g2jd_to_g2j(g2d_add(tod(cases[c][0]), tod(cases[c][1]))));
    const bool ok = want.inf || got.inf ? want.inf == got.inf : fq2_eq(want.x, got.x) && fq2_eq(want.y, got.y);
    mask |= ok ? 1 << c : 0;
  }
  return mask;
}
// fqd_is_zero_mod over digit vectors of k p + e (k = -2..3, e = 0 or 1), unnormalised by moving
// 2^28 between neighbouring digits: 1 if every answer is right.
int hc_fqd_is_zero_mod() {
  for (int k = -2; k <= 3; k++)
    for (int e = 0; e <= 1; e++)
      for (int sh = 0; sh < 13; sh++) {
        fqd a;
        for (int i = 0; i < 14; i++) a.d[i] = k * (int32_t)FQ_P28[i];
        a.d[0] += e;
        a.d[sh] += 1 << 28;
        a.d[sh + 1] -= 1;
        if (fqd_is_zero_mod(a) != (e == 0)) return 0;
      }
  return 1;
}
}
extern "C" {
// miller_loop_gen_d (inlined steps, two-lane coin check) against miller_loop_mixed_d with pair A
// off: the same Fq12 element and the same final T.  1 if both agree.
int hc_miller_gen_cmp(const uint8_t* q96, int parked) {
  g2a Q;
  if (g2_decompress(q96, Q) != HBX_PT_OK) return -1;
  const fqd z = fqd_zero();
  const fqd bx = fqd_from_fq(fq_from_const(G1_MGEN_X)), by = fqd_from_fq(fq_neg(fq_from_const(G1_MGEN_Y)));
  g2jd T1, T2;
  const fq12d f1 = miller_loop_mixed_d(nullptr, z, z, false, fq2d_from_fq2(Q.x), fq2d_from_fq2(Q.y), bx, by, true, &T1);
  uint32_t park[6 * 14];
  const fq12d f2 = parked ? miller_loop_gen_parked_d(fq2d_from_fq2(Q.x), fq2d_from_fq2(Q.y), bx, by, park, T2)
                          : miller_loop_gen_d(fq2d_from_fq2(Q.x), fq2d_from_fq2(Q.y), bx, by, T2);
  const fqd* a = &f1.c0.c0.c0;
  const fqd* b = &f2.c0.c0.c0;
  for (int q = 0; q < 12; q++)
    if (!fq_eq(fq_canon(fqd_to_fq(a[q])), fq_canon(fqd_to_fq(b[q])))) return 0;
  const g2j t1{fq2d_to_fq2(T1.x), fq2d_to_fq2(T1.y), fq2d_to_fq2(T1.z)}, t2{fq2d_to_fq2(T2.x), fq2d_to_fq2(T2.y), fq2d_to_fq2(T2.z)};
  return g2j_eq(t1, t2) ? 1 : 0;
}
}
extern "C" {
// the digit-tower square roots of the hash chains against field.hpp's: 1 if all agree
int hc_sqrt_d_cmp(const uint8_t* x48) {
  fq a = fq_to_mont(fq_from_be(x48));
  fq s1, s2;
  const bool r1 = fq_sqrt(a, s1), r2 = fq_sqrt_d(a, s2);
  if (r1 != r2 || (r1 && !fq_eq(fq_canon(s1), fq_canon(s2)))) return 0;
  const fq2 b{a, fq_add(a, fq_one())};
  fq n1, n2;
  const bool q1 = fq2_norm_sqrt(b, n1), q2 = fq2_norm_sqrt_d(b, n2);
  if (q1 != q2) return 0;
  if (q1) {
    if (!fq_eq(fq_canon(n1), fq_canon(n2))) return 0;
    const fq2 y1 = fq2_sqrt_from_norm(b, n1), y2 = fq2_sqrt_from_norm_d(b, n2);
    if (!fq_eq(fq_canon(y1.c0), fq_canon(y2.c0)) || !fq_eq(fq_canon(y1.c1), fq_canon(y2.c1))) return 0;
  }
  return 1;
}
}
