// Signed 28-bit digit form of the BLS12-381 tower, for the share-check kernel (k_verify_shares).
//
// Same field, same tower (Fq2 = Fq[u]/(u^2+1), Fq6 = Fq2[v]/(v^3-(u+1)), Fq12 = Fq6[w]/(w^2-v)) as
// field.hpp -- the values a check computes are the same elements; only their representation in
// registers differs:
//  * an Fq element is 14 signed 32-bit digits of weight 2^(28 i), Montgomery with R' = 2^392, so
//    a product's result digits come out on the same digit grid as its inputs (no re-cutting of
//    12 x 32-bit limbs into digits and back around every product, field.hpp's fq_mul);
//  * additions, subtractions and negations are digit-wise and carry-free (14 independent VALU
//    ops; the 12-limb carry chain of fq_add / fq_sub is 36 ops plus the wait states gfx950
//    inserts between carry-dependent instructions);
//  * an Fq2 product is ONE fused column loop computing both Montgomery reductions: per column
//    a0 b0 - a1 b1 and (a0 + a1)(b0 + b1) - a0 b0 - a1 b1 from three digit convolutions (Karatsuba)
//    -- 3 x 196 + 2 x 196 = 980 v_mad instead of 3 x 392 = 1176.
// Bounds (all arithmetic on a column is exact modulo 2^64, so only the TRUE column value must fit
// a signed 64-bit word -- intermediate wrap-around of the Karatsuba sum is harmless):
//  * "normalised" (fqd_norm, every product output): digits 0..12 in [0, 2^28), digit 13 signed;
//    value in (-p, 2p);
//  * fqd_mul(a, b): max|a_i| max|b_i| <= 2^59;  fq2d_mul / fq2d_sqr: max|a_i| max|b_i| <= 2^58,
//    i.e. operands that are sums of at most two normalised values.  The tower functions below
//    take normalised inputs and return normalised outputs; host builds with HBX_DCHECK assert
//    the operand bounds (tools/hostcheck).
// Values: a product needs |a b| < p 2^392; operands here stay below 2^386.  Digit sums between
// normalisations stay below 8 x 2^28 (int32).
#pragma once
#include <math.h>
#include "field.hpp"

#if defined(HBX_DCHECK) && !defined(__HIP_DEVICE_COMPILE__)
#include <cstdio>
#include <cstdlib>
#define HBX_DBOUND(a, lim)                                                                  \
  do {                                                                                      \
    for (int i_ = 0; i_ < 14; i_++)                                                         \
      if ((a).d[i_] > (int64_t)(lim) || (a).d[i_] < -(int64_t)(lim)) {                      \
        fprintf(stderr, "fqd bound %s:%d digit %d = %d > %lld\n", __FILE__, __LINE__, i_,   \
                (a).d[i_], (long long)(lim));                                               \
        abort();                                                                            \
      }                                                                                     \
  } while (0)
#else
#define HBX_DBOUND(a, lim) ((void)0)
#endif

namespace hbx {

// A fence between field products whose operands stream from LDS (pairing2d.hpp): the memory
// clobber makes every later operand read a fresh load (otherwise the compiler keeps an operand
// loaded for one product live until its reuse several products later), and the scheduling
// barrier keeps the next product's loads and sums below the current one.  Without it the
// temporaries of several products are live at once and overflow the register file.
#if defined(__HIP_DEVICE_COMPILE__)
#define HBX_SEQ()                          \
  do {                                     \
    __asm__ volatile("" ::: "memory");     \
    __builtin_amdgcn_sched_barrier(0);     \
  } while (0)
#else
#define HBX_SEQ() ((void)0)
#endif

// Digit laundering.  `(int64_t)a * (int64_t)b` of two sign-extended digits is ONE v_mad_i64_i32 --
// unless the compiler has proved one operand non-negative (a digit masked to 28 bits by a
// normalisation, a reduction, a product or an unpacking): it then turns that sign extension into a
// zero extension and expands the mixed-sign product into v_mad_u64_u32 plus a correction
// multiply-add by the other operand's sign word and register moves (a cyclotomic squaring in the
// final exponentiation steps measured 8,979 multiply-adds and 3,622 v_mov_b32 instead of ~7,100 and
// ~0).  Every place that masks a digit passes it through an empty asm with the digit as an in/out
// VGPR operand, which hides what is known about its value and emits nothing.  (Laundering the
// product operands instead forced the Miller loop's wave-uniform line coefficients out of SGPRs
// into VGPRs: more registers, spills.)  The six-lane check's unit is built with HBX_NO_LAUNDER
// (tools/build.py TU_FLAGS): there the laundered digits raised its spills from 8 to 130 VGPRs.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(HBX_NO_LAUNDER)
#define HBX_LAUNDER(x) __asm__("" : "+v"(x))
#else
#define HBX_LAUNDER(x) ((void)0)
#endif

struct fqd {
  int32_t d[14];
};
struct fq2d {
  fqd c0, c1;
};
struct fq6d {
  fq2d c0, c1, c2;
};
struct fq12d {
  fq6d c0, c1;
};

constexpr int32_t DMASK = 0x0FFFFFFF;
constexpr int64_t DN = 1ll << 28;  // bound of a normalised digit

HBX_HD fqd fqd_const(const int32_t* c) {
  fqd r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = c[i];
  return r;
}
HBX_HD fqd fqd_zero() {
  fqd r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = 0;
  return r;
}
HBX_HD fqd fqd_add(const fqd& a, const fqd& b) {
  fqd r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = a.d[i] + b.d[i];
  return r;
}
HBX_HD fqd fqd_sub(const fqd& a, const fqd& b) {
  fqd r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = a.d[i] - b.d[i];
  return r;
}
HBX_HD fqd fqd_neg(const fqd& a) {
  fqd r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = -a.d[i];
  return r;
}
HBX_HD fqd fqd_dbl(const fqd& a) { return fqd_add(a, a); }
// carry propagation: digits 0..12 into [0, 2^28), the signed carry into digit 13 (value kept)
HBX_HD fqd fqd_norm(const fqd& a) {
  fqd r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 13; i++) {
    const int32_t v = a.d[i] + c;
    r.d[i] = v & DMASK;
    c = v >> 28;  // arithmetic: floor division
    HBX_LAUNDER(r.d[i]);
  }
  r.d[13] = a.d[13] + c;
  return r;
}
// Value reduction + carry propagation: x - q p with q = floor(d13 / p13) estimated from the top
// digit (p13 = p >> 364), then digits 0..12 into [0, 2^28).  For |digits| < 2^31 and |q| < 2^14
// the result lies in (-1.3 p, 2.3 p) ("reduced"): what keeps values bounded across the tower,
// since the carry-free additions never subtract p.
HBX_HD fqd fqd_reduce(const fqd& a) {
  const int32_t q = (int32_t)floorf((float)a.d[13] * (1.0f / (float)FQ_P28[13]));
  fqd r;
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 13; i++) {
    acc += (int64_t)a.d[i] - (int64_t)q * (int64_t)FQ_P28[i];
    r.d[i] = (int32_t)((uint32_t)acc & (uint32_t)DMASK);
    acc >>= 28;
    HBX_LAUNDER(r.d[i]);
  }
  r.d[13] = (int32_t)(acc + (int64_t)a.d[13] - (int64_t)q * (int64_t)FQ_P28[13]);
  return r;
}

// One parallel carry step ("relaxed" form for latency-bound chains: groupd.hpp, g1d.hpp):
// d_i <- (d_i mod 2^28) + floor(d_(i-1) / 2^28), the top digit keeps the rest.  Input digits below
// 2^31 in magnitude; output digits in (-2^28 - 8, 2^28 + 8); the value is unchanged.  Three VALU
// levels, against fqd_norm's 13-step carry chain.
HBX_HD fqd fqd_relax(const fqd& a) {
  fqd r;
  r.d[0] = a.d[0] & DMASK;
  HBX_LAUNDER(r.d[0]);
#pragma unroll
  for (int i = 1; i < 13; i++) {
    r.d[i] = (a.d[i] & DMASK) + (a.d[i - 1] >> 28);
    HBX_LAUNDER(r.d[i]);
  }
  r.d[13] = a.d[13] + (a.d[12] >> 28);
  return r;
}

// Montgomery product a b / 2^392 (signed digits; see the bounds above).  Column k of the digit
// convolution accumulates in int64 (v_mad_i64_i32), the reduction digits m_k = -acc p^-1 mod 2^28
// in unsigned (v_mad_u64_u32); three a*b and two m*p chains per column for ILP, as fq_mul_body.
HBX_HD fqd fqd_mul(const fqd& a, const fqd& b) {
  HBX_COUNT_FQMUL();
  uint32_t m[14];
  fqd r;
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    const int jlo = k < 14 ? 0 : k - 13;
    const int jhi = k < 14 ? k : 13;
    int64_t s0 = acc, s1 = 0, s2 = 0;
    uint64_t t0 = 0, t1 = 0;
#pragma unroll
    for (int j = jlo; j <= jhi; j++) {
      const int64_t pr = (int64_t)a.d[j] * (int64_t)b.d[k - j];
      if (j % 3 == 0) s0 += pr;
      else if (j % 3 == 1) s1 += pr;
      else s2 += pr;
    }
#pragma unroll
    for (int j = jlo; j <= jhi; j++)
      if (j < k - 1) {
        if (j & 1) t1 = (uint64_t)m[j] * FQ_P28[k - j] + t1;
        else t0 = (uint64_t)m[j] * FQ_P28[k - j] + t0;
      }
    acc = s0 + s1 + s2 + (int64_t)(t0 + t1);
    if (k >= 1 && k <= 14) acc += (int64_t)((uint64_t)m[k - 1] * FQ_P28[1]);
    if (k < 14) {
      m[k] = ((uint32_t)acc * FQ_INV28) & (uint32_t)DMASK;
      acc += (int64_t)((uint64_t)m[k] * FQ_P28[0]);  // low 28 bits cancel
      acc >>= 28;
    } else {
      r.d[k - 14] = (int32_t)((uint32_t)acc & (uint32_t)DMASK);
      acc >>= 28;
      HBX_LAUNDER(r.d[k - 14]);
    }
  }
  r.d[13] = (int32_t)acc;
  return r;
}
// a^2: the a_i a_j (i != j) column terms taken once, doubled
HBX_HD fqd fqd_sqr(const fqd& a) {
  HBX_COUNT_FQMUL();
  uint32_t m[14];
  int32_t a2[14];
#pragma unroll
  for (int i = 0; i < 14; i++) a2[i] = a.d[i] * 2;
  fqd r;
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    const int jlo = k < 14 ? 0 : k - 13;
    const int jhi = k < 14 ? k : 13;
    int64_t s0 = acc, s1 = 0, s2 = 0;
    uint64_t t0 = 0, t1 = 0;
#pragma unroll
    for (int j = jlo; j <= jhi; j++) {
      if (j > k - j) continue;
      const int64_t pr = j == k - j ? (int64_t)a.d[j] * (int64_t)a.d[j] : (int64_t)a2[j] * (int64_t)a.d[k - j];
      if (j % 3 == 0) s0 += pr;
      else if (j % 3 == 1) s1 += pr;
      else s2 += pr;
    }
#pragma unroll
    for (int j = jlo; j <= jhi; j++)
      if (j < k - 1) {
        if (j & 1) t1 = (uint64_t)m[j] * FQ_P28[k - j] + t1;
        else t0 = (uint64_t)m[j] * FQ_P28[k - j] + t0;
      }
    acc = s0 + s1 + s2 + (int64_t)(t0 + t1);
    if (k >= 1 && k <= 14) acc += (int64_t)((uint64_t)m[k - 1] * FQ_P28[1]);
    if (k < 14) {
      m[k] = ((uint32_t)acc * FQ_INV28) & (uint32_t)DMASK;
      acc += (int64_t)((uint64_t)m[k] * FQ_P28[0]);
      acc >>= 28;
    } else {
      r.d[k - 14] = (int32_t)((uint32_t)acc & (uint32_t)DMASK);
      acc >>= 28;
      HBX_LAUNDER(r.d[k - 14]);
    }
  }
  r.d[13] = (int32_t)acc;
  return r;
}

// HBX_REDC_FENCE (set per translation unit): a scheduling barrier after every column of the fused
// Fq2 product loops, so the scheduler cannot hoist later columns' multiply-adds -- at one wave per
// SIMD it otherwise fills ~190 VGPRs with a single Fq2 product's partial sums, which leaves no
// room for a live Fq12 (fe1d.hpp).
#if defined(HBX_REDC_FENCE) && defined(__HIP_DEVICE_COMPILE__)
#define HBX_COL_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define HBX_COL_FENCE() ((void)0)
#endif

// Two Montgomery reductions driven by one column loop: (x, y) with x = sum_k X_k 2^(28k),
// y = sum_k Y_k 2^(28k) given column by column by `col` (X_k, Y_k exact in int64), returns
// (x / 2^392, y / 2^392) mod p, normalised.
template <class Col>
HBX_HD void fqd_redc2(Col col, fqd& rx, fqd& ry) {
  uint32_t mx[14], my[14];
  int64_t ax = 0, ay = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    const int jlo = k < 14 ? 0 : k - 13;
    const int jhi = k < 14 ? k : 13;
    int64_t X, Y;
    col(k, jlo, jhi, X, Y);
    uint64_t ux = 0, uy = 0;
#pragma unroll
    for (int j = jlo; j <= jhi; j++)
      if (j < k - 1) {
        ux = (uint64_t)mx[j] * FQ_P28[k - j] + ux;
        uy = (uint64_t)my[j] * FQ_P28[k - j] + uy;
      }
    ax += X + (int64_t)ux;
    ay += Y + (int64_t)uy;
    if (k >= 1 && k <= 14) {
      ax += (int64_t)((uint64_t)mx[k - 1] * FQ_P28[1]);
      ay += (int64_t)((uint64_t)my[k - 1] * FQ_P28[1]);
    }
    if (k < 14) {
      mx[k] = ((uint32_t)ax * FQ_INV28) & (uint32_t)DMASK;
      my[k] = ((uint32_t)ay * FQ_INV28) & (uint32_t)DMASK;
      ax += (int64_t)((uint64_t)mx[k] * FQ_P28[0]);
      ay += (int64_t)((uint64_t)my[k] * FQ_P28[0]);
      ax >>= 28;
      ay >>= 28;
    } else {
      rx.d[k - 14] = (int32_t)((uint32_t)ax & (uint32_t)DMASK);
      ry.d[k - 14] = (int32_t)((uint32_t)ay & (uint32_t)DMASK);
      ax >>= 28;
      ay >>= 28;
      HBX_LAUNDER(rx.d[k - 14]);
      HBX_LAUNDER(ry.d[k - 14]);
    }
    HBX_COL_FENCE();
  }
  rx.d[13] = (int32_t)ax;
  ry.d[13] = (int32_t)ay;
}

// N Montgomery reductions driven by one column loop (fqd_redc2 for any N): col(k, jlo, jhi, X)
// gives column k of each of the N double-width values (X[q] exact in int64); r[q] = x_q / 2^392 mod
// p, normalised.  A product whose outputs are sums of several digit convolutions reduces each
// output ONCE (lazy reduction) instead of once per convolution's Fq2 product.
template <int N, class Col>
HBX_HD void fqd_redcn(Col col, fqd (&r)[N]) {
  uint32_t mm[N][14];
  int64_t acc[N];
#pragma unroll
  for (int q = 0; q < N; q++) acc[q] = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    const int jlo = k < 14 ? 0 : k - 13;
    const int jhi = k < 14 ? k : 13;
    int64_t X[N];
    col(k, jlo, jhi, X);
#pragma unroll
    for (int q = 0; q < N; q++) {
      uint64_t u = 0;
#pragma unroll
      for (int j = jlo; j <= jhi; j++)
        if (j < k - 1) u = (uint64_t)mm[q][j] * FQ_P28[k - j] + u;
      acc[q] += X[q] + (int64_t)u;
      if (k >= 1 && k <= 14) acc[q] += (int64_t)((uint64_t)mm[q][k - 1] * FQ_P28[1]);
      if (k < 14) {
        mm[q][k] = ((uint32_t)acc[q] * FQ_INV28) & (uint32_t)DMASK;
        acc[q] += (int64_t)((uint64_t)mm[q][k] * FQ_P28[0]);
        acc[q] >>= 28;
      } else {
        r[q].d[k - 14] = (int32_t)((uint32_t)acc[q] & (uint32_t)DMASK);
        acc[q] >>= 28;
        HBX_LAUNDER(r[q].d[k - 14]);
      }
    }
    HBX_COL_FENCE();
  }
#pragma unroll
  for (int q = 0; q < N; q++) r[q].d[13] = (int32_t)acc[q];
}

// ----------------------------------------------------------------------------------------------
// Fq2
// ----------------------------------------------------------------------------------------------
HBX_HD fq2d fq2d_add(const fq2d& a, const fq2d& b) { return fq2d{fqd_add(a.c0, b.c0), fqd_add(a.c1, b.c1)}; }
HBX_HD fq2d fq2d_sub(const fq2d& a, const fq2d& b) { return fq2d{fqd_sub(a.c0, b.c0), fqd_sub(a.c1, b.c1)}; }
HBX_HD fq2d fq2d_neg(const fq2d& a) { return fq2d{fqd_neg(a.c0), fqd_neg(a.c1)}; }
HBX_HD fq2d fq2d_dbl(const fq2d& a) { return fq2d{fqd_dbl(a.c0), fqd_dbl(a.c1)}; }
HBX_HD fq2d fq2d_conj(const fq2d& a) { return fq2d{a.c0, fqd_neg(a.c1)}; }
HBX_HD fq2d fq2d_norm(const fq2d& a) { return fq2d{fqd_norm(a.c0), fqd_norm(a.c1)}; }
HBX_HD fq2d fq2d_reduce(const fq2d& a) { return fq2d{fqd_reduce(a.c0), fqd_reduce(a.c1)}; }
HBX_HD fq2d fq2d_relax(const fq2d& a) { return fq2d{fqd_relax(a.c0), fqd_relax(a.c1)}; }
// times xi = 1 + u
HBX_HD fq2d fq2d_mul_xi(const fq2d& a) { return fq2d{fqd_sub(a.c0, a.c1), fqd_add(a.c0, a.c1)}; }

// (a0 + a1 u)(b0 + b1 u): column k of  a0 b0 - a1 b1  and  (a0 + a1)(b0 + b1) - a0 b0 - a1 b1.
// Operands: max|digit| products <= 2^58 (sums of two normalised values).  Output normalised.
HBX_HD fq2d fq2d_mul(const fq2d& a, const fq2d& b) {
  HBX_DBOUND(a.c0, 2 * DN); HBX_DBOUND(a.c1, 2 * DN); HBX_DBOUND(b.c0, 2 * DN); HBX_DBOUND(b.c1, 2 * DN);
  HBX_COUNT_FQMUL(); HBX_COUNT_FQMUL(); HBX_COUNT_FQMUL();
  int32_t sa[14], sb[14];
#pragma unroll
  for (int i = 0; i < 14; i++) {
    sa[i] = a.c0.d[i] + a.c1.d[i];
    sb[i] = b.c0.d[i] + b.c1.d[i];
  }
  fq2d r;
  fqd_redc2(
      [&](int k, int jlo, int jhi, int64_t& X, int64_t& Y) {
        int64_t t0 = 0, t1 = 0, t2 = 0;
#pragma unroll
        for (int j = jlo; j <= jhi; j++) {
          t0 += (int64_t)a.c0.d[j] * (int64_t)b.c0.d[k - j];
          t1 += (int64_t)a.c1.d[j] * (int64_t)b.c1.d[k - j];
          t2 += (int64_t)sa[j] * (int64_t)sb[k - j];
        }
        X = t0 - t1;
        Y = t2 - t0 - t1;
      },
      r.c0, r.c1);
  return r;
}
// a^2 = (a0 + a1)(a0 - a1) + 2 a0 a1 u, both columns in one loop.  Operand bound as fq2d_mul.
HBX_HD fq2d fq2d_sqr(const fq2d& a) {
  HBX_DBOUND(a.c0, 2 * DN); HBX_DBOUND(a.c1, 2 * DN);
  HBX_COUNT_FQMUL(); HBX_COUNT_FQMUL();
  int32_t s[14], df[14], a2[14];
#pragma unroll
  for (int i = 0; i < 14; i++) {
    s[i] = a.c0.d[i] + a.c1.d[i];
    df[i] = a.c0.d[i] - a.c1.d[i];
    a2[i] = a.c0.d[i] * 2;
  }
  fq2d r;
  fqd_redc2(
      [&](int k, int jlo, int jhi, int64_t& X, int64_t& Y) {
        int64_t x = 0, y = 0;
#pragma unroll
        for (int j = jlo; j <= jhi; j++) {
          x += (int64_t)s[j] * (int64_t)df[k - j];
          y += (int64_t)a2[j] * (int64_t)a.c1.d[k - j];
        }
        X = x;
        Y = y;
      },
      r.c0, r.c1);
  return r;
}
// (a + b Y)^2 in Fq4 = Fq2[Y]/(Y^2 - xi): c0 = a^2 + xi b^2, c1 = 2 a b (the Fq4 squaring of the
// Granger-Scott and Karabina cyclotomic squarings).  ONE column loop of six digit convolutions --
// a^2, b^2 and e^2 = (a + b)^2 each as (x0 + x1)(x0 - x1) and x0 x1 -- combined per column into
// the four output coordinates (c1 = e^2 - a^2 - b^2) and four Montgomery reductions: 6 + 4
// reductions' worth of multiply-adds instead of three Fq2 squarings' 6 + 6.  a, b normalised;
// every convolution column is below 14 x 2^57, an output's true column below 2^62.4 (the
// combination is exact modulo 2^64, so only the true value must fit).  Normalised outputs.
HBX_HD void fq4d_sqr_lazy(const fq2d& a, const fq2d& b, fq2d& c0, fq2d& c1) {
  HBX_DBOUND(a.c0, DN); HBX_DBOUND(a.c1, DN); HBX_DBOUND(b.c0, DN); HBX_DBOUND(b.c1, DN);
  HBX_COUNT_FQMUL(); HBX_COUNT_FQMUL(); HBX_COUNT_FQMUL(); HBX_COUNT_FQMUL(); HBX_COUNT_FQMUL();
  const fq2d e = fq2d_norm(fq2d_add(a, b));
  int32_t sa[14], da[14], sb[14], db[14], se[14], de[14];
#pragma unroll
  for (int i = 0; i < 14; i++) {
    sa[i] = a.c0.d[i] + a.c1.d[i];
    da[i] = a.c0.d[i] - a.c1.d[i];
    sb[i] = b.c0.d[i] + b.c1.d[i];
    db[i] = b.c0.d[i] - b.c1.d[i];
    se[i] = e.c0.d[i] + e.c1.d[i];
    de[i] = e.c0.d[i] - e.c1.d[i];
  }
  fqd r[4];
  fqd_redcn<4>(
      [&](int k, int jlo, int jhi, int64_t (&X)[4]) {
        int64_t ar = 0, ai = 0, br = 0, bi = 0, er = 0, ei = 0;
#pragma unroll
        for (int j = jlo; j <= jhi; j++) {
          ar += (int64_t)sa[j] * (int64_t)da[k - j];
          ai += (int64_t)a.c0.d[j] * (int64_t)a.c1.d[k - j];
          br += (int64_t)sb[j] * (int64_t)db[k - j];
          bi += (int64_t)b.c0.d[j] * (int64_t)b.c1.d[k - j];
          er += (int64_t)se[j] * (int64_t)de[k - j];
          ei += (int64_t)e.c0.d[j] * (int64_t)e.c1.d[k - j];
        }
        // a^2 = (ar, 2 ai), b^2 = (br, 2 bi), e^2 = (er, 2 ei); xi (x + y u) = (x - y) + (x + y) u
        X[0] = ar + br - 2 * bi;
        X[1] = 2 * ai + br + 2 * bi;
        X[2] = er - ar - br;
        X[3] = 2 * (ei - ai - bi);
      },
      r);
  c0 = fq2d{r[0], r[1]};
  c1 = fq2d{r[2], r[3]};
}
// a * s, s in Fq (two products sharing s)
HBX_HD fq2d fq2d_mul_fq(const fq2d& a, const fqd& s) {
  HBX_DBOUND(a.c0, 2 * DN); HBX_DBOUND(a.c1, 2 * DN); HBX_DBOUND(s, 2 * DN);
  HBX_COUNT_FQMUL(); HBX_COUNT_FQMUL();
  fq2d r;
  fqd_redc2(
      [&](int k, int jlo, int jhi, int64_t& X, int64_t& Y) {
        int64_t x = 0, y = 0;
#pragma unroll
        for (int j = jlo; j <= jhi; j++) {
          x += (int64_t)a.c0.d[j] * (int64_t)s.d[k - j];
          y += (int64_t)a.c1.d[j] * (int64_t)s.d[k - j];
        }
        X = x;
        Y = y;
      },
      r.c0, r.c1);
  return r;
}

// ----------------------------------------------------------------------------------------------
// Fq6, Fq12.  Fq12-level functions take reduced (or conjugated reduced) inputs and return reduced
// outputs; the Fq6 products inside return carry-normalised sums of at most 7 product outputs
// (fq6d_norm: digits back to [0, 2^28), value not reduced), which the Fq12 level combines and
// reduces.
// ----------------------------------------------------------------------------------------------
HBX_HD fq6d fq6d_add(const fq6d& a, const fq6d& b) { return fq6d{fq2d_add(a.c0, b.c0), fq2d_add(a.c1, b.c1), fq2d_add(a.c2, b.c2)}; }
HBX_HD fq6d fq6d_sub(const fq6d& a, const fq6d& b) { return fq6d{fq2d_sub(a.c0, b.c0), fq2d_sub(a.c1, b.c1), fq2d_sub(a.c2, b.c2)}; }
HBX_HD fq6d fq6d_neg(const fq6d& a) { return fq6d{fq2d_neg(a.c0), fq2d_neg(a.c1), fq2d_neg(a.c2)}; }
HBX_HD fq6d fq6d_norm(const fq6d& a) { return fq6d{fq2d_norm(a.c0), fq2d_norm(a.c1), fq2d_norm(a.c2)}; }
HBX_HD fq6d fq6d_reduce(const fq6d& a) { return fq6d{fq2d_reduce(a.c0), fq2d_reduce(a.c1), fq2d_reduce(a.c2)}; }
HBX_HD fq6d fq6d_mul_v(const fq6d& a) { return fq6d{fq2d_mul_xi(a.c2), a.c0, a.c1}; }

// Karatsuba (6 Fq2 products); the operand sums are sums of two normalised values
HBX_HD fq6d fq6d_mul(const fq6d& a, const fq6d& b) {
  const fq2d t0 = fq2d_mul(a.c0, b.c0);
  const fq2d t1 = fq2d_mul(a.c1, b.c1);
  const fq2d t2 = fq2d_mul(a.c2, b.c2);
  const fq2d u0 = fq2d_mul(fq2d_add(a.c1, a.c2), fq2d_add(b.c1, b.c2));
  const fq2d u1 = fq2d_mul(fq2d_add(a.c0, a.c1), fq2d_add(b.c0, b.c1));
  const fq2d u2 = fq2d_mul(fq2d_add(a.c0, a.c2), fq2d_add(b.c0, b.c2));
  const fq2d c0 = fq2d_add(t0, fq2d_mul_xi(fq2d_sub(fq2d_sub(u0, t1), t2)));
  const fq2d c1 = fq2d_add(fq2d_sub(fq2d_sub(u1, t0), t1), fq2d_mul_xi(t2));
  const fq2d c2 = fq2d_add(fq2d_sub(fq2d_sub(u2, t0), t2), t1);
  return fq6d_norm(fq6d{c0, c1, c2});
}
// a * (b0 + b1 v)   (5 Fq2 products)
HBX_HD fq6d fq6d_mul_by_01(const fq6d& a, const fq2d& b0, const fq2d& b1) {
  const fq2d t0 = fq2d_mul(a.c0, b0);
  const fq2d t1 = fq2d_mul(a.c1, b1);
  const fq2d c0 = fq2d_add(t0, fq2d_mul_xi(fq2d_mul(a.c2, b1)));
  const fq2d c1 = fq2d_sub(fq2d_sub(fq2d_mul(fq2d_add(a.c0, a.c1), fq2d_add(b0, b1)), t0), t1);
  const fq2d c2 = fq2d_add(fq2d_mul(a.c2, b0), t1);
  return fq6d_norm(fq6d{c0, c1, c2});
}
// a * (s v), s in Fq
HBX_HD fq6d fq6d_mul_by_1_fq(const fq6d& a, const fqd& s) {
  return fq6d{fq2d_mul_xi(fq2d_mul_fq(a.c2, s)), fq2d_mul_fq(a.c0, s), fq2d_mul_fq(a.c1, s)};
}

HBX_HD fq12d fq12d_conj(const fq12d& a) { return fq12d{a.c0, fq6d_neg(a.c1)}; }
// conj keeps digits within [-2^28, 2^28]: still "normalised" for the product bounds (|digit| <=
// 2^28); fq6d_norm restores non-negative low digits where a value feeds additions repeatedly.

HBX_HD fq12d fq12d_mul(const fq12d& a, const fq12d& b) {
  const fq6d t0 = fq6d_mul(a.c0, b.c0);
  const fq6d t1 = fq6d_mul(a.c1, b.c1);
  const fq6d s = fq6d_mul(fq6d_norm(fq6d_add(a.c0, a.c1)), fq6d_norm(fq6d_add(b.c0, b.c1)));
  return fq12d{fq6d_reduce(fq6d_add(t0, fq6d_mul_v(t1))), fq6d_reduce(fq6d_sub(fq6d_sub(s, t0), t1))};
}
// complex squaring: c0 = (a0 + a1)(a0 + v a1) - ab - v ab, c1 = 2 ab
HBX_HD fq12d fq12d_sqr(const fq12d& a) {
  const fq6d ab = fq6d_mul(a.c0, a.c1);
  const fq6d t = fq6d_mul(fq6d_norm(fq6d_add(a.c0, a.c1)), fq6d_norm(fq6d_add(a.c0, fq6d_mul_v(a.c1))));
  const fq6d c0 = fq6d_sub(fq6d_sub(t, ab), fq6d_mul_v(ab));
  return fq12d{fq6d_reduce(c0), fq6d_reduce(fq6d_add(ab, ab))};
}
// f * (c0 + c1 v + c4 v w), c4 in Fq (a prepared line at a G1 point; field.hpp fq12_mul_by_014_t)
HBX_HD fq12d fq12d_mul_by_014(const fq12d& f, const fq2d& c0, const fq2d& c1, const fqd& c4) {
  const fq6d aa = fq6d_mul_by_01(f.c0, c0, c1);
  const fq6d bb = fq6d_mul_by_1_fq(f.c1, c4);
  const fq2d o = fq2d{fqd_add(c1.c0, c4), c1.c1};
  const fq6d s = fq6d_mul_by_01(fq6d_norm(fq6d_add(f.c1, f.c0)), c0, fq2d_norm(o));
  return fq12d{fq6d_reduce(fq6d_add(fq6d_mul_v(bb), aa)), fq6d_reduce(fq6d_sub(fq6d_sub(s, aa), bb))};
}

// f * (c0 + c1 v + v w): fq12d_mul_by_014 with c4 = 1 -- a line divided by y_P (an Fq factor the
// final exponentiation maps to 1).  The c4 product becomes f.c1 v, a coefficient shift: 10 Fq2
// products instead of 10 plus three Fq-by-Fq2 products.
HBX_HD fq12d fq12d_mul_by_01v(const fq12d& f, const fq2d& c0, const fq2d& c1) {
  const fq6d aa = fq6d_mul_by_01(f.c0, c0, c1);
  const fq2d o = fq2d_norm(fq2d{fqd_add(c1.c0, fqd_const(FQD_ONE)), c1.c1});
  const fq6d s = fq6d_mul_by_01(fq6d_norm(fq6d_add(f.c1, f.c0)), c0, o);
  const fq6d bv = fq6d_mul_v(f.c1);  // f.c1 v
  return fq12d{fq6d_reduce(fq6d_add(fq6d_mul_v(bv), aa)), fq6d_reduce(fq6d_sub(fq6d_sub(s, aa), bv))};
}

// Granger-Scott cyclotomic squaring (field.hpp fq12_cyclotomic_sqr_t)
HBX_HD void fq4d_sqr(const fq2d& a, const fq2d& b, fq2d& c0, fq2d& c1) {
  const fq2d t0 = fq2d_sqr(a);
  const fq2d t1 = fq2d_sqr(b);
  // carry-normalised (3 product outputs each): the callers take 3 c - 2 z, which must stay
  // within int32 digits
  c0 = fq2d_norm(fq2d_add(fq2d_mul_xi(t1), t0));
  c1 = fq2d_norm(fq2d_sub(fq2d_sub(fq2d_sqr(fq2d_add(a, b)), t0), t1));
}
HBX_HD fq12d fq12d_cyclotomic_sqr(const fq12d& f) {
  fq2d z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2;
  fq2d z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
  fq2d t0, t1, t2, t3;
  fq4d_sqr(z0, z1, t0, t1);
  z0 = fq2d_reduce(fq2d_add(fq2d_dbl(fq2d_sub(t0, z0)), t0));
  z1 = fq2d_reduce(fq2d_add(fq2d_dbl(fq2d_add(t1, z1)), t1));
  fq4d_sqr(z2, z3, t0, t1);
  fq4d_sqr(z4, z5, t2, t3);
  z4 = fq2d_reduce(fq2d_add(fq2d_dbl(fq2d_sub(t0, z4)), t0));
  z5 = fq2d_reduce(fq2d_add(fq2d_dbl(fq2d_add(t1, z5)), t1));
  t0 = fq2d_mul_xi(t3);
  z2 = fq2d_reduce(fq2d_add(fq2d_dbl(fq2d_add(t0, z2)), t0));
  z3 = fq2d_reduce(fq2d_add(fq2d_dbl(fq2d_sub(t2, z3)), t2));
  return fq12d{fq6d{z0, z4, z3}, fq6d{z2, z1, z5}};
}

// Frobenius maps (field.hpp fq12_frobenius / fq12_frobenius2) with the digit-form constants
HBX_HD fq2d fq2d_const(const int32_t* c0, const int32_t* c1) { return fq2d{fqd_const(c0), fqd_const(c1)}; }
HBX_HD fq12d fq12d_frobenius(const fq12d& a) {
  fq12d r;
  r.c0.c0 = fq2d_norm(fq2d_conj(a.c0.c0));
  r.c1.c0 = fq2d_mul(fq2d_conj(a.c1.c0), fq2d_const(FROBD1_C1_0, FROBD1_C1_1));
  r.c0.c1 = fq2d_mul(fq2d_conj(a.c0.c1), fq2d_const(FROBD1_C2_0, FROBD1_C2_1));
  r.c1.c1 = fq2d_mul(fq2d_conj(a.c1.c1), fq2d_const(FROBD1_C3_0, FROBD1_C3_1));
  r.c0.c2 = fq2d_mul(fq2d_conj(a.c0.c2), fq2d_const(FROBD1_C4_0, FROBD1_C4_1));
  r.c1.c2 = fq2d_mul(fq2d_conj(a.c1.c2), fq2d_const(FROBD1_C5_0, FROBD1_C5_1));
  return r;
}
HBX_HD fq12d fq12d_frobenius2(const fq12d& a) {
  fq12d r;
  r.c0.c0 = a.c0.c0;
  r.c1.c0 = fq2d_mul_fq(a.c1.c0, fqd_const(FROBD2_C1));
  r.c0.c1 = fq2d_mul_fq(a.c0.c1, fqd_const(FROBD2_C2));
  r.c1.c1 = fq2d_mul_fq(a.c1.c1, fqd_const(FROBD2_C3));
  r.c0.c2 = fq2d_mul_fq(a.c0.c2, fqd_const(FROBD2_C4));
  r.c1.c2 = fq2d_mul_fq(a.c1.c2, fqd_const(FROBD2_C5));
  return r;
}

// ----------------------------------------------------------------------------------------------
// Conversions with field.hpp's 12 x 32-bit form (R = 2^384, lazy [0, 2p])
// ----------------------------------------------------------------------------------------------
HBX_HD fqd fqd_from_fq(const fq& a) {
  fqd raw;  // the 384-bit integer a R in 28-bit digits (non-negative, < 2^384)
#pragma unroll
  for (int j = 0; j < 14; j++) {
    const int bit = 28 * j, w = bit >> 5, sh = bit & 31;
    uint32_t v = a.l[w] >> sh;
    if (sh > 4 && w + 1 < 12) v |= a.l[w + 1] << (32 - sh);
    raw.d[j] = (int32_t)(j == 13 ? v : (v & (uint32_t)DMASK));
  }
  return fqd_mul(raw, fqd_const(FQD_CONV));  // (x R) 2^400 / 2^392 = x R 2^8 = x R'
}
HBX_HD fq fqd_to_fq(const fqd& a) {
  // x R' * 2^384 / 2^392 = x R, value in (-p, 2p); + 2p -> (p, 4p), then into [0, 2p)
  const fqd b = fqd_norm(fqd_add(fqd_mul(a, fqd_const(FQD_BACK)), fqd_const(FQD_2P)));
  fq r;
#pragma unroll
  for (int w = 0; w < 12; w++) {
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int off = 28 * i;
      if (off + 28 <= 32 * w && i != 13) continue;
      if (off >= 32 * w + 32) continue;
      const uint32_t di = (uint32_t)b.d[i];
      if (off >= 32 * w) v |= di << (off - 32 * w);
      else v |= di >> (32 * w - off);
    }
    r.l[w] = v;
  }
  return fq_csub(r, FQ_2P);
}
HBX_HD fq2d fq2d_from_fq2(const fq2& a) { return fq2d{fqd_from_fq(a.c0), fqd_from_fq(a.c1)}; }

// ---- Fq inversion on the digits themselves ---------------------------------------------------------
// field.hpp binv_limbs' half-delta divsteps (Bernstein-Yang; the step bound of libsecp256k1's
// safegcd analysis), batched 28 at a time so that a batch's division by 2^28 is a shift of the
// digit index: 28 divsteps on digit 0 of f and g give the matrix T (|entries| <= 2^28), then
// (f, g) <- T (f, g) / 2^28 exactly and (d, e) <- (T (d, e) + k p) / 2^28 with k = -(T (d, e))_0
// p^-1 mod 2^28, one signed v_mad_i64_i32 per digit product and one carry step per digit.  The
// 12-limb route (fqd_to_fq, fq_canon, binv_limbs on 32-bit limbs, whose signed x unsigned limb
// products the compiler expands, fq_mul by R^3, fqd_from_fq) measured 100.5 us per lone wave
// (profiles/r06i_fq_inversion.txt).  d, e grow by at most p per batch (|d'| <= max(|d|, |e|) + p:
// 33 batches stay below 34 p, digit 13 below 2^22), f, g stay within [-p, p].
// In: a in digit Montgomery form (x R', any normalised-range value); out: x^-1 R' (normalised,
// value in (-p, 2p)), 0 for x = 0 (zero set).
HBX_HD fqd fqd_addp_if(const fqd& v, bool add, int sign) {  // v + sign p when add, carry-normalised
  fqd r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const int32_t t = v.d[i] + (add ? sign * (int32_t)FQ_P28[i] : 0) + c;
    if (i < 13) {
      r.d[i] = t & DMASK;
      c = t >> 28;
      HBX_LAUNDER(r.d[i]);
    } else {
      r.d[i] = t;
    }
  }
  return r;
}
// the representative of v in [0, p), digits normalised (v's value within (-2p, 3p))
HBX_HD fqd fqd_canon(const fqd& v_) {
  fqd v = fqd_norm(v_);
  v = fqd_addp_if(v, v.d[13] < 0, 1);
  v = fqd_addp_if(v, v.d[13] < 0, 1);
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const fqd t = fqd_addp_if(v, true, -1);
    const bool ge = t.d[13] >= 0;
#pragma unroll
    for (int i = 0; i < 14; i++) v.d[i] = ge ? t.d[i] : v.d[i];
  }
  return v;
}
// (ca a + cb b [+ k p]) / 2^28, exact; a, b digits normalised; |ca| + |cb| <= 2^28
template <bool MODP>
HBX_HD fqd fqd_lincomb28(const fqd& a, const fqd& b, int32_t ca, int32_t cb) {
  int64_t acc = (int64_t)ca * a.d[0] + (int64_t)cb * b.d[0];
  int32_t k = 0;
  if (MODP) {
    k = (int32_t)(((uint32_t)acc * FQ_INV28) & (uint32_t)DMASK);
    acc += (int64_t)k * (int64_t)FQ_P28[0];  // low 28 bits now zero
  }
  acc >>= 28;
  fqd r;
#pragma unroll
  for (int i = 1; i < 14; i++) {
    acc += (int64_t)ca * a.d[i];
    acc += (int64_t)cb * b.d[i];
    if (MODP) acc += (int64_t)k * (int64_t)FQ_P28[i];
    r.d[i - 1] = (int32_t)((uint32_t)acc & (uint32_t)DMASK);
    HBX_LAUNDER(r.d[i - 1]);
    acc >>= 28;
  }
  r.d[13] = (int32_t)acc;
  return r;
}
HBX_HD fqd fqd_inv(const fqd& a, bool& zero) {
  constexpr int BATCHES = ((45907 * 381 + 26313) / 19929 + 28 + 27) / 28;  // hddivsteps bound + one batch
  fqd g = fqd_canon(a), f, d = fqd_zero(), e = fqd_zero();
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    f.d[i] = (int32_t)FQ_P28[i];
    nz |= (uint32_t)g.d[i];
  }
  zero = nz == 0;
  e.d[0] = 1;
  int32_t delta = 1;  // 2 delta, delta = 1/2
#pragma unroll 1
  for (int b = 0; b < BATCHES; b++) {
    int32_t u, v, q, r;
    divsteps_n<28>(delta, (uint32_t)f.d[0], (uint32_t)g.d[0], u, v, q, r);
    const fqd nf = fqd_lincomb28<false>(f, g, u, v);
    const fqd ng = fqd_lincomb28<false>(f, g, q, r);
    const fqd nd = fqd_lincomb28<true>(d, e, u, v);
    e = fqd_lincomb28<true>(d, e, q, r);
    f = nf;
    g = ng;
    d = nd;
  }
  // g = 0, f = +-1 (f = p, d = 0 for x = 0): x^-1 = f d, then times R'^3 / R'
  const bool fneg = f.d[0] != 1;
  return fqd_mul(fneg ? fqd_neg(d) : d, fqd_const(FQD_R3));
}
HBX_HDNI fqd fqd_inv_ni(const fqd& a, bool& zero) { return fqd_inv(a, zero); }

// a^e (e a 384-bit constant, 12 LE words) in the digit tower: field.hpp fq_pow_const's 4-bit
// fixed windows, with the squarings and products as fqd_sqr / fqd_mul (no re-cutting of 12 limbs
// into digits around every product).  In and out in field.hpp's 12-limb form.  The hash chains'
// square roots (hash.hpp hash_g2_group) run on it.
HBX_HDNI fq fq_pow_const_d(const fq& a_, const uint32_t* e) {
  const fqd a = fqd_from_fq(a_);
  fqd tab[16];
  tab[0] = fqd_const(FQD_ONE);
  tab[1] = a;
  for (int i = 2; i < 16; i++) tab[i] = fqd_mul(tab[i - 1], a);
  fqd r = tab[0];
  bool started = false;
  for (int w = 95; w >= 0; w--) {
    const uint32_t nib = (e[w >> 3] >> ((w & 7) * 4)) & 0xF;
    if (started) {
#pragma unroll 1
      for (int q = 0; q < 4; q++) r = fqd_sqr(r);
    }
    if (nib) {
      fqd t = tab[1];
      for (int k = 2; k < 16; k++)
        if ((uint32_t)k == nib) t = tab[k];
      r = started ? fqd_mul(r, t) : t;
      started = true;
    }
  }
  return fqd_to_fq(r);
}
// field.hpp fq_sqrt / fq2_norm_sqrt / fq2_sqrt_from_norm with fq_pow_const_d
HBX_HD bool fq_sqrt_d(const fq& a, fq& out) {
  const fq s = fq_pow_const_d(a, FQ_SQRT_EXP);
  out = s;
  return fq_eq(fq_sqr(s), a);
}
HBX_HD bool fq2_norm_sqrt_d(const fq2& a, fq& s) {
  const fq n = fq_add(fq_sqr(a.c0), fq_sqr(a.c1));
  return fq_sqrt_d(n, s);
}
HBX_HDNI fq2 fq2_sqrt_from_norm_d(const fq2& a, const fq& s) {
  const fq half = fq_from_const(FQ_HALF_MONT);
  const fq alpha = fq_mul(fq_add(a.c0, s), half);
  const fq e = fq_pow_const_d(alpha, FQ_P_MINUS_3_DIV_4);
  const fq t = fq_mul(alpha, e);
  const fq c = fq_mul(t, e);
  const fq h = fq_mul(fq_mul(a.c1, e), half);
  if (fq_eq(c, fq_one())) return fq2{t, h};
  return fq2{fq_neg(h), t};
}
HBX_HD fq2 fq2d_to_fq2(const fq2d& a) { return fq2{fqd_to_fq(a.c0), fqd_to_fq(a.c1)}; }
HBX_HD fq6d fq6d_from_fq6(const fq6& a) { return fq6d{fq2d_from_fq2(a.c0), fq2d_from_fq2(a.c1), fq2d_from_fq2(a.c2)}; }
HBX_HD fq6 fq6d_to_fq6(const fq6d& a) { return fq6{fq2d_to_fq2(a.c0), fq2d_to_fq2(a.c1), fq2d_to_fq2(a.c2)}; }
HBX_HD fq12d fq12d_from_fq12(const fq12& a) { return fq12d{fq6d_from_fq6(a.c0), fq6d_from_fq6(a.c1)}; }
HBX_HD fq12 fq12d_to_fq12(const fq12d& a) { return fq12{fq6d_to_fq6(a.c0), fq6d_to_fq6(a.c1)}; }
HBX_HD fq12d fq12d_one() {
  fq12d r;
  const fqd z = fqd_zero();
  r.c0 = fq6d{fq2d{fqd_const(FQD_ONE), z}, fq2d{z, z}, fq2d{z, z}};
  r.c1 = fq6d{fq2d{z, z}, fq2d{z, z}, fq2d{z, z}};
  return r;
}
// Inversion (once per check) through field.hpp's binary-Euclid inverse
HBX_HDNI fq12d fq12d_inv(const fq12d& a) { return fq12d_from_fq12(fq12_inv(fq12d_to_fq12(a))); }
HBX_HDNI bool fq12d_is_one(const fq12d& a) { return fq12_is_one(fq12d_to_fq12(a)); }

}  // namespace hbx
