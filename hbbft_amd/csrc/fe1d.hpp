// The one-lane share check's final exponentiation as a chain of STEP kernels (k_fe1<STEP>), in the
// signed-digit tower (fieldd.hpp).  Same element as pairingd.hpp final_exponentiation_d (and
// pairing.hpp final_exponentiation): f^(3 (p^12 - 1)/r), compared with 1 -- the verdict of
// PublicKeyShare::verify_decryption_share (honey_badger.rs:229 via threshold_crypto; SURVEY.md
// §8(a) rows A1, A9).
//
// Why a chain of kernels.  Inside one kernel the exponentiation's Fq12 values crossed out-of-line
// calls through the lane's scratch stack: 8.7 KB/lane of frames, 18.7 GB of scratch traffic per
// N=256 launch and ~20 % of the wave's cycles waiting on it.  Here nothing leaves
// the registers inside a kernel except through explicit slots:
//   * the running value r (one Fq12, 168 registers) stays in registers for a whole step;
//   * the exponentiation base / product operand sits in the lane's LDS slot A (one packed Fq12,
//     156 dwords, lane-interleaved: one wave per SIMD fills a CU's 160 KB), streamed one Fq2
//     coefficient at a time into the products (fq12d_mul_slot), so a product holds r, three Fq6
//     accumulators and one Fq2 product's temporaries;
//   * the values that live across exponentiations (t^3 then d, a, b) go to coalesced global slots
//     between kernels: 3 packed Fq12 per check, [wave][slot][word][64 lanes] (~7.5 KB of traffic
//     per check in total instead of ~285 KB of frames).
// Every step is one kernel, so the register allocator sees at most one exponentiation loop and
// two products at a time, and there are no call frames at all.
//
// Chain (pairing.hpp final_exponentiation, regrouped as pairing2d.hpp FE2_PROG), four kernels
// (F0, F1 + F2, F3 + F4, F5 + F6; a pair shares one kernel: its hand-over stays in registers and
// LDS):
//   F0  t0 = conj(f)^2 / N(f) (= conj(f) f^-1, N(f) = f0^2 - v f1^2 in Fq6: one Fq6 inverse);
//       t = frob2(t0) t0                                                      -> slot G
//   F1  a = conj(t^|x| t); t^3 is the value after the first run of t^|x|      -> slot G, T
//   F2  a = conj(a^|x| a)                                                      -> slot G
//   F3  b = conj(a^|x|) frob(a) -> slot F, then (same kernel, b from registers)
//       d = t^3 conj(b) frob2(b)                                               -> slot T
//   F5  u = b^|x|                                                              -> slot G
//   F6  u^|x| d == 1  (= b^(x^2) d = f^(3 (p^12 - 1)/r))
#pragma once
#include "pairingd.hpp"

namespace hbx {

// ---- one-lane slots: a packed Fq12 (12 Fq x 13 dwords, pairingd.hpp lds_put_fq12d's packing),
// word k of this lane at p[k * S] ------------------------------------------------------------------
constexpr int FE1_WORDS = 156;

// The lane's LDS slot, addressed afresh at every access.  Held as a pointer, the slot address is one
// more VGPR live across every product; at the steps' register peak the allocator spilled exactly
// that value and reloaded it from scratch before each operand fetch -- 456 of the 525 scratch
// reloads of one Fq12 slot product (tools/microbench/fe_probe.hip), each waited on before its
// ds_read.  Here the lane index comes from v_mbcnt (two VALU ops, no register input) in a volatile
// asm, so it is recomputed where needed and never held: nothing to spill.
#if defined(__HIPCC__)
struct lane_lds {
  lds_u32* base;  // the block's slot array (wave-uniform); lane l's word k at base[k * 64 + l]
};
__device__ __forceinline__ lds_u32* slot_ptr(lane_lds s) {
  uint32_t l;
  __asm__ volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return s.base + l;
}
#endif
template <class T>
HBX_HD T* slot_ptr(T* p) {
  return p;
}

template <int S, class P>
HBX_HD fqd s1_get_fqd(P p_, int word) {
  const auto p = slot_ptr(p_);
  uint32_t w[13];
#pragma unroll
  for (int k = 0; k < 13; k++) w[k] = p[(word + k) * S];
  fqd e;
#pragma unroll
  for (int i = 0; i < 13; i++) {
    const int off = 28 * i, wd = off >> 5, sh = off & 31;
    uint32_t d = w[wd] >> sh;
    if (sh > 4) d |= w[wd + 1] << (32 - sh);
    e.d[i] = (int32_t)(d & (uint32_t)DMASK);
    HBX_LAUNDER(e.d[i]);
  }
  e.d[13] = (int32_t)w[12];
  return e;
}
// e normalised: digits 0..12 in [0, 2^28), digit 13 whole
template <int S, class P>
HBX_HD void s1_put_fqd(P p_, int word, const fqd& e) {
  uint32_t w[13];
#pragma unroll
  for (int k = 0; k < 12; k++) w[k] = 0;
#pragma unroll
  for (int i = 0; i < 13; i++) {
    const int off = 28 * i, wd = off >> 5, sh = off & 31;
    const uint32_t d = (uint32_t)e.d[i];
    w[wd] |= d << sh;
    if (sh > 4) w[wd + 1] |= d >> (32 - sh);
  }
  w[12] = (uint32_t)e.d[13];
  const auto p = slot_ptr(p_);
#pragma unroll
  for (int k = 0; k < 13; k++) p[(word + k) * S] = w[k];
}
// Fq2 coefficient q (0..5: c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2)
template <int S, class P>
HBX_HD fq2d s1_get_fq2d(P p, int q) {
  return fq2d{s1_get_fqd<S>(p, 26 * q), s1_get_fqd<S>(p, 26 * q + 13)};
}
template <int S, class P>
HBX_HD void s1_put_fq2d(P p, int q, const fq2d& a) {
  s1_put_fqd<S>(p, 26 * q, a.c0);
  s1_put_fqd<S>(p, 26 * q + 13, a.c1);
}
// Whole-Fq12 loads / stores go one Fq2 coefficient at a time behind fences: unfenced, the
// scheduler issues all 156 loads (or packs all 12 elements) at once, and those temporaries beside
// a live Fq12 are what made the steps spill.
template <int S, class P>
HBX_HD fq12d s1_get_fq12d(P p) {
  const fq2d c0 = s1_get_fq2d<S>(p, 0);
  HBX_SEQ();
  const fq2d c1 = s1_get_fq2d<S>(p, 1);
  HBX_SEQ();
  const fq2d c2 = s1_get_fq2d<S>(p, 2);
  HBX_SEQ();
  const fq2d c3 = s1_get_fq2d<S>(p, 3);
  HBX_SEQ();
  const fq2d c4 = s1_get_fq2d<S>(p, 4);
  HBX_SEQ();
  const fq2d c5 = s1_get_fq2d<S>(p, 5);
  HBX_SEQ();
  return fq12d{fq6d{c0, c1, c2}, fq6d{c3, c4, c5}};
}
template <int S, class P>
HBX_HD void s1_put_fq12d(P p, const fq12d& a) {
  s1_put_fq2d<S>(p, 0, a.c0.c0);
  HBX_SEQ();
  s1_put_fq2d<S>(p, 1, a.c0.c1);
  HBX_SEQ();
  s1_put_fq2d<S>(p, 2, a.c0.c2);
  HBX_SEQ();
  s1_put_fq2d<S>(p, 3, a.c1.c0);
  HBX_SEQ();
  s1_put_fq2d<S>(p, 4, a.c1.c1);
  HBX_SEQ();
  s1_put_fq2d<S>(p, 5, a.c1.c2);
  HBX_SEQ();
}
// slot-to-slot copy (global -> LDS), 52 words (two Fq2 coefficients) in flight at a time
template <int SD, int SS, class PD, class PS>
HBX_HD void s1_copy(PD d_, PS s_) {
#pragma unroll 1
  for (int k0 = 0; k0 < FE1_WORDS; k0 += 52) {
    const auto d = slot_ptr(d_);
    const auto s = slot_ptr(s_);
#pragma unroll
    for (int k = 0; k < 52; k++) d[(k0 + k) * SD] = s[(k0 + k) * SS];
    HBX_SEQ();
  }
}

// fq6d_zero_ and fq6d_mul_acc1 (acc += a * y, y streamed): pairingd.hpp

// acc_p += a * y and acc_m -= a * y at once (pairingd.hpp fq6d_mul_acc1's Karatsuba, every Fq2
// product folded into both accumulators): both normalised (or zero) on entry, carry-normalised on exit.
template <class Y>
HBX_HD void fq6d_mul_acc_pm(fq6d& acc_p, fq6d& acc_m, const fq6d& a, Y y) {
  auto fold = [&](int k, const fq2d& t, int sign) __attribute__((always_inline)) {
    fq2d& p = k == 0 ? acc_p.c0 : k == 1 ? acc_p.c1 : acc_p.c2;
    fq2d& m = k == 0 ? acc_m.c0 : k == 1 ? acc_m.c1 : acc_m.c2;
    if (sign > 0) {
      p = fq2d_add(p, t);
      m = fq2d_sub(m, t);
    } else {
      p = fq2d_sub(p, t);
      m = fq2d_add(m, t);
    }
  };
  {
    const fq2d t0 = fq2d_mul(a.c0, y(0));
    fold(0, t0, 1);
    fold(1, t0, -1);
    fold(2, t0, -1);
  }
  HBX_SEQ();
  {
    const fq2d t1 = fq2d_mul(a.c1, y(1));
    fold(0, fq2d_mul_xi(t1), -1);
    fold(1, t1, -1);
    fold(2, t1, 1);
  }
  HBX_SEQ();
  {
    const fq2d t2 = fq2d_mul(a.c2, y(2));
    const fq2d xt2 = fq2d_mul_xi(t2);
    fold(0, xt2, -1);
    fold(1, xt2, 1);
    fold(2, t2, -1);
  }
  HBX_SEQ();
  fold(0, fq2d_mul_xi(fq2d_mul(fq2d_add(a.c1, a.c2), fq2d_add(y(1), y(2)))), 1);
  HBX_SEQ();
  fold(1, fq2d_mul(fq2d_add(a.c0, a.c1), fq2d_add(y(0), y(1))), 1);
  HBX_SEQ();
  fold(2, fq2d_mul(fq2d_add(a.c0, a.c2), fq2d_add(y(0), y(2))), 1);
  HBX_SEQ();
  acc_p = fq6d_norm(acc_p);
  acc_m = fq6d_norm(acc_m);
}

// X * Y, X in registers (reduced, or its conjugate), Y the packed value in slot y.  Reduced.
// Karatsuba over w: c0 = X0 Y0 + v X1 Y1, c1 = (X0 + X1)(Y0 + Y1) - X0 Y0 - X1 Y1.
#ifndef HBX_FE1_MUL_ORDER
#define HBX_FE1_MUL_ORDER 0  // 1: the three-Fq6 order below (tools/build_variant.py measures it)
#endif
#if HBX_FE1_MUL_ORDER
// The order keeps at most three Fq6 values beside a product's temporaries (the round-5 order held
// X, X0 + X1 and three accumulators, ~500 registers): B = X1 Y1 first; X0 + X1 replaces X1; B
// seeds both outputs (c0 = v B, c1 = -B) and dies; c1 += (X0 + X1)(Y0 + Y1), then X0 Y0 goes into
// c0 and out of c1 in one pass.  Same element.
template <int S, class P>
HBX_HD fq12d fq12d_mul_slot(const fq12d& X, P y) {
  fq6d c0, c1;
  fq6d Xs;
  {
    fq6d B = fq6d_zero_();
    fq6d_mul_acc1(B, X.c1, [&](int q) { return s1_get_fq2d<S>(y, 3 + q); });
    HBX_SEQ();
    Xs = fq6d_norm(fq6d_add(X.c0, X.c1));
    c0 = fq6d_norm(fq6d_mul_v(B));
    c1 = fq6d_neg(B);
  }
  HBX_SEQ();
  fq6d_mul_acc1(c1, Xs, [&](int q) { return fq2d_norm(fq2d_add(s1_get_fq2d<S>(y, q), s1_get_fq2d<S>(y, 3 + q))); });
  HBX_SEQ();
  fq6d_mul_acc_pm(c0, c1, X.c0, [&](int q) { return s1_get_fq2d<S>(y, q); });
  return fq12d{fq6d_reduce(c0), fq6d_reduce(c1)};
}
#else
template <int S, class P>
HBX_HD fq12d fq12d_mul_slot(const fq12d& X, P y) {
  fq6d A = fq6d_zero_();
  fq6d_mul_acc1(A, X.c0, [&](int q) { return s1_get_fq2d<S>(y, q); });
  HBX_SEQ();
  fq6d B = fq6d_zero_();
  fq6d_mul_acc1(B, X.c1, [&](int q) { return s1_get_fq2d<S>(y, 3 + q); });
  HBX_SEQ();
  fq6d C = fq6d_zero_();
  const fq6d Xs = fq6d_norm(fq6d_add(X.c0, X.c1));
  fq6d_mul_acc1(C, Xs, [&](int q) { return fq2d_norm(fq2d_add(s1_get_fq2d<S>(y, q), s1_get_fq2d<S>(y, 3 + q))); });
  return fq12d{fq6d_reduce(fq6d_add(A, fq6d_mul_v(B))), fq6d_reduce(fq6d_sub(fq6d_sub(C, A), B))};
}
#endif

// Granger-Scott cyclotomic squaring (fieldd.hpp fq12d_cyclotomic_sqr) with a fence after every Fq2
// squaring: the nine squarings are independent, and unfenced the scheduler interleaves them until
// the temporaries of all of them are live at once (440 VGPRs spilled around a bare loop of them).
#ifndef HBX_FE1_CYC_FENCE
#define HBX_FE1_CYC_FENCE 2  // 2: after every Fq2 squaring, 1: after every Fq4 squaring, 0: none
#endif
#if HBX_FE1_CYC_FENCE >= 2
#define HBX_CYC_SEQ2() HBX_SEQ()
#else
#define HBX_CYC_SEQ2() ((void)0)
#endif
#if HBX_FE1_CYC_FENCE >= 1
#define HBX_CYC_SEQ1() HBX_SEQ()
#else
#define HBX_CYC_SEQ1() ((void)0)
#endif
#ifndef HBX_FE1_LAZY
#define HBX_FE1_LAZY 1  // 1: Fq4 squarings by fq4d_sqr_lazy (one reduction per output coordinate)
#endif
HBX_HD void fq4d_sqr_seq(const fq2d& a, const fq2d& b, fq2d& c0, fq2d& c1) {
#if HBX_FE1_LAZY
  fq4d_sqr_lazy(a, b, c0, c1);
  HBX_CYC_SEQ1();
#else
  const fq2d t0 = fq2d_sqr(a);
  HBX_CYC_SEQ2();
  const fq2d t1 = fq2d_sqr(b);
  HBX_CYC_SEQ2();
  c0 = fq2d_norm(fq2d_add(fq2d_mul_xi(t1), t0));
  c1 = fq2d_norm(fq2d_sub(fq2d_sub(fq2d_sqr(fq2d_add(a, b)), t0), t1));
  HBX_CYC_SEQ1();
#endif
}
HBX_HD fq12d fq12d_cyclotomic_sqr_seq(const fq12d& f) {
  fq2d z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2;
  fq2d z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
  fq2d t0, t1;
  fq4d_sqr_seq(z0, z1, t0, t1);
  z0 = fq2d_reduce(fq2d_add(fq2d_dbl(fq2d_sub(t0, z0)), t0));
  z1 = fq2d_reduce(fq2d_add(fq2d_dbl(fq2d_add(t1, z1)), t1));
  fq4d_sqr_seq(z4, z5, t0, t1);  // (z4, z5) before they are replaced: t2, t3 of fieldd.hpp
  const fq2d n3 = fq2d_reduce(fq2d_add(fq2d_dbl(fq2d_sub(t0, z3)), t0));
  t0 = fq2d_mul_xi(t1);
  const fq2d n2 = fq2d_reduce(fq2d_add(fq2d_dbl(fq2d_add(t0, z2)), t0));
  fq4d_sqr_seq(z2, z3, t0, t1);
  z4 = fq2d_reduce(fq2d_add(fq2d_dbl(fq2d_sub(t0, z4)), t0));
  z5 = fq2d_reduce(fq2d_add(fq2d_dbl(fq2d_add(t1, z5)), t1));
  return fq12d{fq6d{z0, z4, n3}, fq6d{n2, z1, z5}};
}

// ---- Karabina compressed squarings (the exp-by-|x| runs of 32 and 16 squarings) ---------------
// An element of the cyclotomic subgroup is determined by four of its six Fq2 coefficients,
// g1 = c0.c1, g2 = c0.c2, g3 = c1.c0, g5 = c1.c2, and its square's four from them with six Fq2
// squarings (Granger-Scott: nine):
//   g1' = 3 (g3^2 + xi g2^2) - 2 g1        g2' = 3 (g1^2 + xi g5^2) - 2 g2
//   g3' = 6 xi g1 g5 + 2 g3                g5' = 6 g2 g3 + 2 g5
// (2 g1 g5 = (g1 + g5)^2 - g1^2 - g5^2, 2 g2 g3 likewise).  Decompression recovers
//   g4 = c1.c1 = (xi g5^2 + 3 g1^2 - 2 g2) / (4 g3),   g0 = c0.c0 = xi (2 g4^2 + g3 g5 - 3 g1 g2) + 1,
// one Fq2 inversion per run (checked against the oracle's squarings, tools/hostcheck).  g3 = 0
// makes the division impossible; such a lane is flagged and re-checked by the single-kernel path.
// For a run that starts at the identity (t = 1 after the easy part) g3 = 0 always: a proposer can
// cause that on purpose (fe1_step0 explains how), so step 0 decides t = 1 itself.  Otherwise g3 = 0
// needs an element with a zero Fq2 coefficient at a run's end (~2^-760 for values not chosen so).
struct fq12c {
  fq2d g1, g2, g3, g5;
};
HBX_HD fq2d fq2d_lin(const fq2d& a3, const fq2d& b2, bool minus) {  // reduce(3 a +/- 2 b), a, b normalised
  const fq2d a = fq2d_add(fq2d_dbl(a3), a3);
  const fq2d b = fq2d_dbl(b2);
  return fq2d_reduce(minus ? fq2d_sub(a, b) : fq2d_add(a, b));
}
HBX_HD void karabina_sqr(fq12c& c) {
#if HBX_FE1_LAZY
  // (g3 + g2 Y)^2 = (g3^2 + xi g2^2) + 2 g2 g3 Y and (g1 + g5 Y)^2 = (g1^2 + xi g5^2) + 2 g1 g5 Y:
  // the six squarings as two lazily reduced Fq4 squarings (fieldd.hpp fq4d_sqr_lazy)
  fq2d p1, x23, p2, x15;
  fq4d_sqr_lazy(c.g3, c.g2, p1, x23);
  HBX_SEQ();
  fq4d_sqr_lazy(c.g1, c.g5, p2, x15);
  HBX_SEQ();
  const fq2d n1 = fq2d_lin(p1, c.g1, true);
  const fq2d n2 = fq2d_lin(p2, c.g2, true);
  const fq2d n3 = fq2d_lin(fq2d_norm(fq2d_mul_xi(x15)), c.g3, false);
  const fq2d n5 = fq2d_lin(x23, c.g5, false);
  c = fq12c{n1, n2, n3, n5};
#else
  const fq2d s1 = fq2d_sqr(c.g1);
  HBX_SEQ();
  const fq2d s5 = fq2d_sqr(c.g5);
  HBX_SEQ();
  const fq2d x15 = fq2d_norm(fq2d_sub(fq2d_sub(fq2d_sqr(fq2d_add(c.g1, c.g5)), s1), s5));  // 2 g1 g5
  HBX_SEQ();
  const fq2d s3 = fq2d_sqr(c.g3);
  HBX_SEQ();
  const fq2d s2 = fq2d_sqr(c.g2);
  HBX_SEQ();
  const fq2d x23 = fq2d_norm(fq2d_sub(fq2d_sub(fq2d_sqr(fq2d_add(c.g2, c.g3)), s2), s3));  // 2 g2 g3
  HBX_SEQ();
  const fq2d n1 = fq2d_lin(fq2d_norm(fq2d_add(s3, fq2d_mul_xi(s2))), c.g1, true);
  const fq2d n2 = fq2d_lin(fq2d_norm(fq2d_add(s1, fq2d_mul_xi(s5))), c.g2, true);
  const fq2d n3 = fq2d_lin(fq2d_norm(fq2d_mul_xi(x15)), c.g3, false);
  const fq2d n5 = fq2d_lin(x23, c.g5, false);
  c = fq12c{n1, n2, n3, n5};
#endif
}
// decompressed element (reduced); `degenerate` set when g3 = 0
#ifndef HBX_KARA_INV_CALL
#define HBX_KARA_INV_CALL 0
#endif
HBX_HD fq12d karabina_decompress(const fq12c& c, bool& degenerate) {
  fq2d g4;
  {
    const fq2d t1 = fq2d_norm(fq2d_sub(fq2d_add(fq2d_dbl(fq2d_sqr(c.g1)), fq2d_sqr(c.g1)), fq2d_dbl(c.g2)));
    HBX_SEQ();
    const fq2d num = fq2d_reduce(fq2d_add(fq2d_mul_xi(fq2d_sqr(c.g5)), t1));
    HBX_SEQ();
    const fq2d den = fq2d_reduce(fq2d_dbl(fq2d_dbl(c.g3)));
    const fqd nrm = fqd_reduce(fqd_add(fqd_sqr(den.c0), fqd_sqr(den.c1)));
    HBX_SEQ();
    bool zero;
#if HBX_KARA_INV_CALL
    const fqd ni = fqd_inv_ni(nrm, zero);  // out of line (fieldd.hpp): its loop sees only its own state
#else
    const fqd ni = fqd_inv(nrm, zero);
#endif
    degenerate = degenerate || zero;
    HBX_SEQ();
    g4 = fq2d_mul(num, fq2d_mul_fq(fq2d_conj(den), ni));
  }
  HBX_SEQ();
  const fq2d t12 = fq2d_mul(c.g2, c.g1);
  HBX_SEQ();
  const fq2d s4 = fq2d_sqr(g4);
  HBX_SEQ();
  const fq2d t35 = fq2d_mul(c.g3, c.g5);
  HBX_SEQ();
  // 2 g4^2 - 3 g1 g2 + g3 g5, then xi (..) + 1
  const fq2d u = fq2d_norm(fq2d_add(fq2d_sub(fq2d_dbl(s4), fq2d_add(fq2d_dbl(t12), t12)), t35));
  fq2d g0 = fq2d_mul_xi(u);
  g0.c0 = fqd_add(g0.c0, fqd_const(FQD_ONE));
  return fq12d{fq6d{fq2d_reduce(g0), c.g1, c.g2}, fq6d{c.g3, fq2d_reduce(g4), c.g5}};
}

// r^|x| with r's value also in slot a (the base): squaring runs between the one bits of |x| (63,
// 62, 60, 57, 48, 16), a product by the base after each run but the last; the runs of 32 and 16
// squarings in compressed form.  (A compressed squaring is ~7.1k VALU instructions against ~10.3k
// for Granger-Scott, and a decompression ~38k, most of it the Fq inversion: the break-even run is
// ~12 squarings, so the run of 9 stays uncompressed.)  If t3 is given, the value after the first run and product (r^3)
// is stored there.  `degenerate`: see karabina_decompress.
template <int S, int SG, class P, class PG>
HBX_HD fq12d cyc_exp_abs_x_slot(fq12d r, P a, PG t3, bool& degenerate) {
  static_assert(BLS_X == 0xd201000000010000ull, "square-and-multiply runs are specific to |x|");
  int q0 = 0;
  if (t3) {
    // the first run (one squaring) and its product outside the loop, so that the loop body holds
    // no store of r (with it inside, F1 spilled 446 VGPRs against F2's 132)
    r = fq12d_cyclotomic_sqr_seq(r);
    HBX_SEQ();
    r = fq12d_mul_slot<S>(r, a);
    HBX_SEQ();
    s1_put_fq12d<SG>(t3, r);
    q0 = 1;
  }
#pragma unroll 1
  for (int q = q0; q < 6; q++) {
    const int run = q == 0 ? 1 : q == 1 ? 2 : q == 2 ? 3 : q == 3 ? 9 : q == 4 ? 32 : 16;
    if (q >= 4) {
      fq12c c{r.c0.c1, r.c0.c2, r.c1.c0, r.c1.c2};
#pragma unroll 1
      for (int i = 0; i < run; i++) karabina_sqr(c);
      HBX_SEQ();
      r = karabina_decompress(c, degenerate);
    } else {
#pragma unroll 1
      for (int i = 0; i < run; i++) r = fq12d_cyclotomic_sqr_seq(r);
    }
    if (q < 5) {
      HBX_SEQ();
      r = fq12d_mul_slot<S>(r, a);
    }
  }
  return r;
}

// slot a <- map(slot a) in place, one Fq2 coefficient at a time: MAP 1 = f^p, 2 = f^(p^2)
// (fieldd.hpp fq12d_frobenius / fq12d_frobenius2: coefficient c_h.c_k is gamma index 2k + h)
template <int S, int MAP, class P>
HBX_HD void s1_frob_inplace(P a) {
#pragma unroll 1
  for (int q = 0; q < 6; q++) {
    const int i = 2 * (q % 3) + q / 3;
    fq2d y = s1_get_fq2d<S>(a, q);
    if (MAP == 1) {
      y = fq2d_conj(y);
      if (i) {
        const int32_t* k0 = i == 1 ? FROBD1_C1_0 : i == 2 ? FROBD1_C2_0 : i == 3 ? FROBD1_C3_0 : i == 4 ? FROBD1_C4_0 : FROBD1_C5_0;
        const int32_t* k1 = i == 1 ? FROBD1_C1_1 : i == 2 ? FROBD1_C2_1 : i == 3 ? FROBD1_C3_1 : i == 4 ? FROBD1_C4_1 : FROBD1_C5_1;
        y = fq2d_mul(y, fq2d_const(k0, k1));
      } else {
        y = fq2d_norm(y);
      }
    } else if (i) {
      const int32_t* kk = i == 1 ? FROBD2_C1 : i == 2 ? FROBD2_C2 : i == 3 ? FROBD2_C3 : i == 4 ? FROBD2_C4 : FROBD2_C5;
      y = fq2d_mul_fq(y, fqd_const(kk));
    }
    s1_put_fq2d<S>(a, q, y);
  }
}

// ---- STEP 0 pieces ---------------------------------------------------------------------------
// Fq6 inverse of a (reduced) into slot words [0, 78) of y (fieldd.hpp tower; one Fq inversion):
// c0 = a0^2 - xi a1 a2, c1 = xi a2^2 - a0 a1, c2 = a1^2 - a0 a2, t = a0 c0 + xi (a2 c1 + a1 c2),
// a^-1 = (c0, c1, c2) conj(t) / (t0^2 + t1^2).  The packed coefficients are normalised.
template <int S, class P>
HBX_HD void fq6d_inv_to_slot(const fq6d& a, P y) {
  fq2d t;
  {
    const fq2d c0 = fq2d_reduce(fq2d_sub(fq2d_sqr(a.c0), fq2d_mul_xi(fq2d_mul(a.c1, a.c2))));
    s1_put_fq2d<S>(y, 0, c0);
    t = fq2d_mul(a.c0, c0);
  }
  HBX_SEQ();
  {
    const fq2d c1 = fq2d_reduce(fq2d_sub(fq2d_mul_xi(fq2d_sqr(a.c2)), fq2d_mul(a.c0, a.c1)));
    s1_put_fq2d<S>(y, 1, c1);
    t = fq2d_add(t, fq2d_mul_xi(fq2d_mul(a.c2, c1)));
  }
  HBX_SEQ();
  {
    const fq2d c2 = fq2d_reduce(fq2d_sub(fq2d_sqr(a.c1), fq2d_mul(a.c0, a.c2)));
    s1_put_fq2d<S>(y, 2, c2);
    t = fq2d_reduce(fq2d_add(t, fq2d_mul_xi(fq2d_mul(a.c1, c2))));
  }
  HBX_SEQ();
  const fqd nrm = fqd_reduce(fqd_add(fqd_sqr(t.c0), fqd_sqr(t.c1)));
  HBX_SEQ();
  bool zero;  // (N(f) != 0: f is a nonzero Miller value)
  const fqd ni = fqd_inv(nrm, zero);
  HBX_SEQ();
  const fq2d ti = fq2d_mul_fq(fq2d_conj(t), ni);
#pragma unroll 1
  for (int q = 0; q < 3; q++) {
    HBX_SEQ();
    s1_put_fq2d<S>(y, q, fq2d_reduce(fq2d_mul(s1_get_fq2d<S>(y, q), ti)));
  }
}

// t0 = conj(f) / f = conj(f)^2 / N(f) with N(f) = f0^2 - v f1^2 (f reduced, f != 0); slot a is
// scratch.  Reduced.
template <int S, class P>
HBX_HD fq12d fe1_easy_first(const fq12d& f, P a) {
  {
    const fq6d n = fq6d_reduce(fq6d_sub(fq6d_mul(f.c0, f.c0), fq6d_mul_v(fq6d_mul(f.c1, f.c1))));
    HBX_SEQ();
    fq6d_inv_to_slot<S>(n, a);  // words [0, 78): N^-1
  }
  HBX_SEQ();
  const fq12d g = fq12d_sqr(fq12d_conj(f));
  HBX_SEQ();
  fq6d A = fq6d_zero_(), B = fq6d_zero_();
  fq6d_mul_acc1(A, g.c0, [&](int q) { return s1_get_fq2d<S>(a, q); });
  HBX_SEQ();
  fq6d_mul_acc1(B, g.c1, [&](int q) { return s1_get_fq2d<S>(a, q); });
  return fq12d{fq6d_reduce(A), fq6d_reduce(B)};
}

// fq12d_is_one with the conversions one Fq at a time (no Fq12 in a call frame)
HBX_HD bool fq12d_is_one_seq(const fq12d& a) {
  const fqd* e = &a.c0.c0.c0;
  bool ok = true;
#pragma unroll
  for (int q = 0; q < 12; q++) {
    const fq v = fq_canon(fqd_to_fq(e[q]));
    ok = ok && (q == 0 ? fq_eq(v, fq_one()) : fq_is_zero(v));
  }
  return ok;
}

// ---- the seven steps over a lane's slots: a = LDS (or host) slot, gf / gt / gg = global slots F
// (Miller output, later b), T (t^3, later d), G (t, a, u) ------------------------------------------
constexpr int FE1_STEPS = 7;  // F0..F6; run as four kernels: k_fe1<0>, <1> (F1 + F2), <3> (F3 + F4), <5> (F5 + F6)
constexpr int FE1_LAST = 5;   // the kernel that decides the verdict
// F0: t = frob2(t0) t0, t0 = conj(f) / f  -> G
template <int SG, class PG>
HBX_HD fq6d s1_get_half(PG p, int h) {
  return fq6d{s1_get_fq2d<SG>(p, 3 * h), s1_get_fq2d<SG>(p, 3 * h + 1), s1_get_fq2d<SG>(p, 3 * h + 2)};
}
// fe1_easy_first restated over the slots with at most two Fq6 values in registers at a time (the
// round-4 version held f's halves beside an Fq12 squaring: 224 spilled VGPRs, 0.46 GB of scratch
// traffic per N=256 launch).  With A = f0^2, B = v f1^2, C = f0 f1 (three Fq6 products, each
// streaming its second operand from the lane's LDS slot): N(f) = A - B, conj(f)^2 = (A + B) -
// 2 C w, and t0 = conj(f)^2 / N(f) -- three Fq6 products for N(f) and conj(f)^2 instead of four.
// f is copied into slot a first, so the products stream it from LDS (streamed from slot F in
// global memory, every Fq2 operand read behind a fence exposed a global load's latency: the step
// waited 29 % of its cycles); B and C wait in slot T's halves (free until F1 writes t^3), A + B in
// slot G's half 0, and N^-1 replaces f in slot a once the three products are done.
template <int S, int SG, class P, class PG>
HBX_HD bool fe1_step0(P a, PG gf, PG gt, PG gg) {
  s1_copy<S, SG>(a, gf);
  HBX_SEQ();
  {
    // B = v f1^2 -> slot T half 0
    fq6d B = fq6d_zero_();
    fq6d_mul_acc1(B, s1_get_half<S>(a, 1), [&](int q) { return s1_get_fq2d<S>(a, 3 + q); });
    B = fq6d_norm(fq6d_mul_v(B));
    s1_put_fq2d<SG>(gt, 0, B.c0);
    s1_put_fq2d<SG>(gt, 1, B.c1);
    s1_put_fq2d<SG>(gt, 2, B.c2);
  }
  HBX_SEQ();
  {
    // C' = -2 f0 f1 -> slot T half 1
    fq6d C = fq6d_zero_();
    fq6d_mul_acc1(C, s1_get_half<S>(a, 0), [&](int q) { return s1_get_fq2d<S>(a, 3 + q); });
    C = fq6d_reduce(fq6d_neg(fq6d_add(C, C)));
    s1_put_fq2d<SG>(gt, 3, C.c0);
    s1_put_fq2d<SG>(gt, 4, C.c1);
    s1_put_fq2d<SG>(gt, 5, C.c2);
  }
  HBX_SEQ();
  {
    // A = f0^2; N = A - B (kept), A + B -> slot G half 0; N^-1 -> slot a words [0, 78) (f is
    // no longer needed)
    fq6d A = fq6d_zero_();
    fq6d_mul_acc1(A, s1_get_half<S>(a, 0), [&](int q) { return s1_get_fq2d<S>(a, q); });
    HBX_SEQ();
    fq6d n;
#pragma unroll 1
    for (int q = 0; q < 3; q++) {  // one Fq2 coefficient at a time (B from slot T)
      const fq2d b = s1_get_fq2d<SG>(gt, q);
      const fq2d aq = q == 0 ? A.c0 : q == 1 ? A.c1 : A.c2;
      s1_put_fq2d<SG>(gg, q, fq2d_reduce(fq2d_add(aq, b)));
      const fq2d nq = fq2d_reduce(fq2d_sub(aq, b));
      if (q == 0) n.c0 = nq;
      else if (q == 1) n.c1 = nq;
      else n.c2 = nq;
    }
    HBX_SEQ();
    fq6d_inv_to_slot<S>(n, a);  // words [0, 78): N^-1
  }
  HBX_SEQ();
  fq12d r;
  {
    // t0.c1 = -2 C N^-1
    fq6d T1 = fq6d_zero_();
    fq6d_mul_acc1(T1, s1_get_half<SG>(gt, 1), [&](int q) { return s1_get_fq2d<S>(a, q); });
    r.c1 = fq6d_reduce(T1);
  }
  HBX_SEQ();
  {
    // t0.c0 = (A + B) N^-1
    fq6d T0 = fq6d_zero_();
    fq6d_mul_acc1(T0, s1_get_half<SG>(gg, 0), [&](int q) { return s1_get_fq2d<S>(a, q); });
    r.c0 = fq6d_reduce(T0);  // t0 = conj(f) / f
  }
  HBX_SEQ();
  s1_put_fq12d<S>(a, r);
  HBX_SEQ();
  r = fq12d_mul_slot<S>(fq12d_frobenius2(r), a);
  s1_put_fq12d<SG>(gg, r);
  HBX_SEQ();
  // t = 1: the hard part of 1 is 1, so the check holds and no compressed squaring runs (they would
  // start at g3 = 0 and send the lane to the fallback).  Reachable on purpose: a ciphertext with
  // r = 3(x^2 - 1) makes W = H' and every honest share S_i = [m] pk_i, so f = f_H'(P) f_H'(-P) lies
  // in Fq6 and t = 1 (tests/test_gpu_threshold.py::test_degenerate_ciphertext_r_m).
  return fq12d_is_one_seq(r);
}
// F1 + F2 in one kernel: x -> conj(x^|x| x) twice (x = t, t^3 -> T on the way; then x = a), the
// intermediate a handed over in registers and slot a (no store / reload through G, no kernel
// boundary); the loop keeps one copy of the code
template <int S, int SG, class P, class PG>
HBX_HD void fe1_step12(P a, PG gt, PG gg, bool& degenerate) {
  s1_copy<S, SG>(a, gg);
  HBX_SEQ();
  fq12d r = s1_get_fq12d<S>(a);
#pragma unroll 1
  for (int rep = 0; rep < 2; rep++) {
    r = cyc_exp_abs_x_slot<S, SG>(r, a, rep == 0 ? gt : (PG) nullptr, degenerate);
    HBX_SEQ();
    r = fq12d_mul_slot<S>(r, a);
    r = fq12d{r.c0, fq6d_norm(fq6d_neg(r.c1))};
    HBX_SEQ();
    if (rep == 0) s1_put_fq12d<S>(a, r);
    HBX_SEQ();
  }
  s1_put_fq12d<SG>(gg, r);
}
// F3 + F4 in one kernel: b = conj(a^|x|) frob(a) -> F, then d = t^3 conj(b) frob2(b) -> T with b
// still in registers and put into slot a directly (no reload of F, no kernel boundary)
template <int S, int SG, class P, class PG>
HBX_HD void fe1_step34(P a, PG gf, PG gt, PG gg, bool& degenerate) {
  s1_copy<S, SG>(a, gg);
  HBX_SEQ();
  fq12d r = s1_get_fq12d<S>(a);
  r = cyc_exp_abs_x_slot<S, SG>(r, a, (PG) nullptr, degenerate);
  HBX_SEQ();
  s1_frob_inplace<S, 1>(a);
  HBX_SEQ();
  r = fq12d_mul_slot<S>(fq12d_conj(r), a);  // b
  s1_put_fq12d<SG>(gf, r);
  HBX_SEQ();
  s1_put_fq12d<S>(a, r);
  HBX_SEQ();
  s1_frob_inplace<S, 2>(a);
  HBX_SEQ();
  r = fq12d_mul_slot<S>(fq12d_conj(r), a);
  HBX_SEQ();
  s1_copy<S, SG>(a, gt);
  HBX_SEQ();
  r = fq12d_mul_slot<S>(r, a);
  s1_put_fq12d<SG>(gt, r);
}
// F5 + F6 in one kernel: u = b^|x|, then u^|x| d (= b^(x^2) d = f^(3 (p^12 - 1)/r)), == 1 iff the
// check holds; u handed over in registers and slot a
template <int S, int SG, class P, class PG>
HBX_HD fq12d fe1_step56(P a, PG gf, PG gt, bool& degenerate) {
  s1_copy<S, SG>(a, gf);
  HBX_SEQ();
  fq12d r = s1_get_fq12d<S>(a);
#pragma unroll 1
  for (int rep = 0; rep < 2; rep++) {
    r = cyc_exp_abs_x_slot<S, SG>(r, a, (PG) nullptr, degenerate);
    HBX_SEQ();
    if (rep == 0) s1_put_fq12d<S>(a, r);
    HBX_SEQ();
  }
  s1_copy<S, SG>(a, gt);
  HBX_SEQ();
  return fq12d_mul_slot<S>(r, a);
}
// the whole chain on one lane (host checks; the kernels run one step each)
template <int S, int SG, class P, class PG>
HBX_HD fq12d fe1_chain(P a, PG gf, PG gt, PG gg, bool& degenerate) {
  fe1_step0<S, SG>(a, gf, gt, gg);
  fe1_step12<S, SG>(a, gt, gg, degenerate);
  fe1_step34<S, SG>(a, gf, gt, gg, degenerate);
  return fe1_step56<S, SG>(a, gf, gt, degenerate);
}

}  // namespace hbx
