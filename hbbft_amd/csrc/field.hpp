// BLS12-381 base-field tower for gfx950: Fq (381-bit) / Fq2 / Fq6 / Fq12, and the scalar field Fr.
//
// What this replaces: the `pairing = 0.14.2` field types (reference Cargo.toml:28) that
// threshold_crypto drives on hbbft's hot path.  The tower is the same
// one pairing builds: Fq2 = Fq[u]/(u^2+1), Fq6 = Fq2[v]/(v^3-(u+1)), Fq12 = Fq6[w]/(w^2-v).
//
// Representation (MI355X-first):
//  * 12 x 32-bit limbs, little-endian, Montgomery form with R = 2^384 (the same value pairing
//    stores in 6 x u64).  Every multiply is a 12x12 CIOS loop of v_mad_u64_u32 (measured ~half
//    rate on gfx950, tools/microbench/mad_rate.hip) -- integer VALU, not MFMA: this is not a
//    dense contraction.
//  * "Lazy" range [0, 2p]: p < 2^381 leaves 3 spare bits, so the no-carry CIOS takes inputs
//    <= 2p and returns < 2p without a final subtraction (bounds checked numerically).  Add/sub
//    fold back into [0, 2p) with one conditional 2p correction.  Canonical [0, p) form is only
//    produced for encodings and equality tests (fq_canon).
//  * Everything is __host__ __device__ so tools/hostcheck can unit-test the arithmetic on a CPU;
//    the product path only ever runs it on the GPU.
#pragma once
#include <stdint.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define HBX_HD __host__ __device__ __forceinline__
#define HBX_HDNI __host__ __device__ __noinline__ inline
#else
#define HBX_HD inline
#define HBX_HDNI inline
#endif
#include "constants.hpp"

// Operation counter for the roofline's algorithmic work (tools/opcount, host builds only).
#if defined(HBX_OPCOUNT) && !defined(__HIP_DEVICE_COMPILE__)
extern unsigned long long hbx_opcount_fqmul;
#define HBX_COUNT_FQMUL() (++hbx_opcount_fqmul)
#else
#define HBX_COUNT_FQMUL() ((void)0)
#endif

namespace hbx {

// Load of read-only data at a wave-uniform address through the constant address space, so it
// is issued as scalar (SMEM) loads through the scalar cache: a plain global load after an
// out-of-line call cannot be proven unclobbered and would be a vector load per lane.
template <class T>
HBX_HD T ld_uniform(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((address_space(4))) const T* cptr;
  return *(cptr)p;
#else
  return *p;
#endif
}

struct fq {
  uint32_t l[12];
};
struct fq2 {
  fq c0, c1;
};
struct fq6 {
  fq2 c0, c1, c2;
};
struct fq12 {
  fq6 c0, c1;
};
struct fr {
  uint32_t l[8];
};

// ----------------------------------------------------------------------------------------------
// Fq
// ----------------------------------------------------------------------------------------------
HBX_HD fq fq_zero() {
  fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = 0;
  return r;
}
HBX_HD fq fq_one() {
  fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = FQ_ONE[i];
  return r;
}
HBX_HD fq fq_from_const(const uint32_t* c) {
  fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = c[i];
  return r;
}

// Montgomery product, inputs <= 2p, output < 2p.
//
// Digit-sliced product scanning.  The operands stay 12 x 32-bit limbs with R = 2^384 everywhere
// else; inside the product they are re-cut into 14 digits of 28 bits (13 x 28 + 20 = 384), so a
// column of <= 14 a*b products plus <= 14 m*p products (each < 2^56) fits a 64-bit accumulator:
// every partial product is ONE v_mad_u64_u32 with no carry word.  (With 32-bit digits each
// product needed a v_mad_u64_u32 plus a v_addc_co_u32 into a third word and the loop carried
// ~100 moves; measured on MI355X at one wave per SIMD: 1.9 us -> 1.5 us per product,
// tools/microbench/fq28.hip.)  The Montgomery digits m_0..m_12 are 28-bit, m_13 is 20-bit, so
// the reduction divides by exactly 2^(13*28 + 20) = 2^384 = R.
// Bounds: a, b < 2p and M = sum m_j 2^(28 j) < 2^384 give (ab + Mp)/R < 4p^2/R + p < 2p.
// The same C++ runs on the host (tools/hostcheck, tools/opcount), so the host check exercises
// exactly this digit schedule.
HBX_HD void fq_unpack28(const fq& a, uint32_t* d) {
#pragma unroll
  for (int j = 0; j < 14; j++) {
    const int bit = 28 * j, w = bit >> 5, sh = bit & 31;
    uint32_t v = a.l[w] >> sh;
    if (sh > 4 && w + 1 < 12) v |= a.l[w + 1] << (32 - sh);
    d[j] = j == 13 ? v : (v & 0x0FFFFFFFu);
  }
}
// Independent accumulator chains per column of the digit product (a*b terms, m*p terms).
#ifndef HBX_FQ_NA
#define HBX_FQ_NA 3
#endif
#ifndef HBX_FQ_NP
#define HBX_FQ_NP 2
#endif
#if defined(__HIP_DEVICE_COMPILE__) && defined(HBX_FQ_INLINE)
#define HBX_FQMUL_ATTR __device__ __forceinline__
#elif defined(__HIP_DEVICE_COMPILE__)
#define HBX_FQMUL_ATTR __device__ __noinline__
#else
#define HBX_FQMUL_ATTR inline
#endif
// One out-of-line copy on the device (inlined at every call site the tower code would not fit
// the instruction cache).  Limbs travel as 24 scalar arguments so the call passes them in VGPRs.
#define HBX_L12(x) x##0, x##1, x##2, x##3, x##4, x##5, x##6, x##7, x##8, x##9, x##10, x##11
#define HBX_P12(x)                                                                                  \
  uint32_t x##0, uint32_t x##1, uint32_t x##2, uint32_t x##3, uint32_t x##4, uint32_t x##5, uint32_t x##6, \
      uint32_t x##7, uint32_t x##8, uint32_t x##9, uint32_t x##10, uint32_t x##11
HBX_HD fq fq_mul_body(HBX_P12(a), HBX_P12(b)) {
  const fq a = {{HBX_L12(a)}};
  const fq b = {{HBX_L12(b)}};
  uint32_t A[14], B[14], m[14], o[15];
  fq_unpack28(a, A);
  fq_unpack28(b, B);
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    const int jlo = k < 14 ? 0 : k - 13;
    const int jhi = k < 14 ? k : 13;
    // HBX_FQ_NA interleaved a*b chains and HBX_FQ_NP m*p chains (independent accumulators, so
    // one wave keeps several v_mad_u64_u32 in flight); m_{k-1} p_1 (the only term that waits on
    // the previous digit) is added last
    uint64_t s[HBX_FQ_NA], t[HBX_FQ_NP];
#pragma unroll
    for (int q = 0; q < HBX_FQ_NA; q++) s[q] = q == 0 ? acc : 0;
#pragma unroll
    for (int q = 0; q < HBX_FQ_NP; q++) t[q] = 0;
#pragma unroll
    for (int j = jlo; j <= jhi; j++) s[j % HBX_FQ_NA] = (uint64_t)A[j] * B[k - j] + s[j % HBX_FQ_NA];
#pragma unroll
    for (int j = jlo; j <= jhi; j++)
      if (j < k - 1) t[j % HBX_FQ_NP] = (uint64_t)m[j] * FQ_P28[k - j] + t[j % HBX_FQ_NP];
    acc = 0;
#pragma unroll
    for (int q = 0; q < HBX_FQ_NA; q++) acc += s[q];
#pragma unroll
    for (int q = 0; q < HBX_FQ_NP; q++) acc += t[q];
    if (k >= 1 && k <= 14) acc = (uint64_t)m[k - 1] * FQ_P28[1] + acc;
    if (k < 13) {
      m[k] = ((uint32_t)acc * FQ_INV28) & 0x0FFFFFFFu;
      acc = (uint64_t)m[k] * FQ_P28[0] + acc;  // low 28 bits cancel
      acc >>= 28;
    } else if (k == 13) {
      m[k] = ((uint32_t)acc * FQ_INV28) & 0x000FFFFFu;
      acc = (uint64_t)m[k] * FQ_P28[0] + acc;  // low 20 bits cancel: R = 2^384 reached
      o[0] = (uint32_t)(acc >> 20) & 0xFFu;    // result bits 0..7
      acc >>= 28;
    } else {
      o[k - 13] = (uint32_t)acc & 0x0FFFFFFFu;  // result bits 8 + 28 (k - 14) ..
      acc >>= 28;
    }
  }
  o[14] = (uint32_t)acc;  // result bits 372..
  fq r;
#pragma unroll
  for (int w = 0; w < 12; w++) {
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 15; i++) {
      const int off = i == 0 ? 0 : 8 + 28 * (i - 1);
      const int width = i == 0 ? 8 : (i == 14 ? 32 : 28);
      if (off + width <= 32 * w || off >= 32 * w + 32) continue;
      if (off >= 32 * w) v |= o[i] << (off - 32 * w);
      else v |= o[i] >> (32 * w - off);
    }
    r.l[w] = v;
  }
  return r;
}
// Montgomery square, input <= 2p, output < 2p: the product above with the a*a column sums
// taken once per pair, sum_{i<j} (2 a_i) a_j + a_{k/2}^2, i.e. 105 instead of 196 digit products
// (the reduction's 196 m*p products are unchanged): 301 v_mad_u64_u32 instead of 392.
// (2 a_i) < 2^29, so a column holds < 8 * 2^57 from the square plus < 14 * 2^56 from m*p.
HBX_HD fq fq_sqr_body(HBX_P12(a)) {
  const fq a = {{HBX_L12(a)}};
  uint32_t A[14], A2[14], m[14], o[15];
  fq_unpack28(a, A);
#pragma unroll
  for (int j = 0; j < 14; j++) A2[j] = A[j] << 1;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    const int jlo = k < 14 ? 0 : k - 13;
    const int jhi = k < 14 ? k : 13;
    uint64_t s[HBX_FQ_NA], t[HBX_FQ_NP];
#pragma unroll
    for (int q = 0; q < HBX_FQ_NA; q++) s[q] = q == 0 ? acc : 0;
#pragma unroll
    for (int q = 0; q < HBX_FQ_NP; q++) t[q] = 0;
#pragma unroll
    for (int j = jlo; j <= jhi; j++)
      if (j < k - j) s[j % HBX_FQ_NA] = (uint64_t)A2[j] * A[k - j] + s[j % HBX_FQ_NA];
    if ((k & 1) == 0 && k / 2 <= 13) s[(k / 2) % HBX_FQ_NA] = (uint64_t)A[k / 2] * A[k / 2] + s[(k / 2) % HBX_FQ_NA];
#pragma unroll
    for (int j = jlo; j <= jhi; j++)
      if (j < k - 1) t[j % HBX_FQ_NP] = (uint64_t)m[j] * FQ_P28[k - j] + t[j % HBX_FQ_NP];
    acc = 0;
#pragma unroll
    for (int q = 0; q < HBX_FQ_NA; q++) acc += s[q];
#pragma unroll
    for (int q = 0; q < HBX_FQ_NP; q++) acc += t[q];
    if (k >= 1 && k <= 14) acc = (uint64_t)m[k - 1] * FQ_P28[1] + acc;
    if (k < 13) {
      m[k] = ((uint32_t)acc * FQ_INV28) & 0x0FFFFFFFu;
      acc = (uint64_t)m[k] * FQ_P28[0] + acc;
      acc >>= 28;
    } else if (k == 13) {
      m[k] = ((uint32_t)acc * FQ_INV28) & 0x000FFFFFu;
      acc = (uint64_t)m[k] * FQ_P28[0] + acc;
      o[0] = (uint32_t)(acc >> 20) & 0xFFu;
      acc >>= 28;
    } else {
      o[k - 13] = (uint32_t)acc & 0x0FFFFFFFu;
      acc >>= 28;
    }
  }
  o[14] = (uint32_t)acc;
  fq r;
#pragma unroll
  for (int w = 0; w < 12; w++) {
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 15; i++) {
      const int off = i == 0 ? 0 : 8 + 28 * (i - 1);
      const int width = i == 0 ? 8 : (i == 14 ? 32 : 28);
      if (off + width <= 32 * w || off >= 32 * w + 32) continue;
      if (off >= 32 * w) v |= o[i] << (off - 32 * w);
      else v |= o[i] >> (32 * w - off);
    }
    r.l[w] = v;
  }
  return r;
}
#if defined(HBX_HOST_INT128) && !defined(__HIPCC__)
// Host-only alternative for the CPU baseline port (tools/cpu_baseline): textbook 6 x 64-bit CIOS
// with unsigned __int128, the limb shape pairing 0.14 (u128-support) uses on x86-64.  Same
// Montgomery value (R = 2^384, output < 2p); the GPU and tools/hostcheck never use it.
inline fq fq_mul_cios64(const fq& a, const fq& b) {
  typedef unsigned __int128 u128;
  uint64_t A[6], B[6], P6[6], t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 6; i++) {
    A[i] = (uint64_t)a.l[2 * i] | ((uint64_t)a.l[2 * i + 1] << 32);
    B[i] = (uint64_t)b.l[2 * i] | ((uint64_t)b.l[2 * i + 1] << 32);
    P6[i] = (uint64_t)FQ_P[2 * i] | ((uint64_t)FQ_P[2 * i + 1] << 32);
  }
  const uint64_t pinv = 0x89f3fffcfffcfffdull;  // -p^-1 mod 2^64
  for (int i = 0; i < 6; i++) {
    u128 c = 0;
    for (int j = 0; j < 6; j++) {
      c = (u128)A[j] * B[i] + t[j] + (uint64_t)(c >> 64);
      t[j] = (uint64_t)c;
    }
    u128 s = (u128)t[6] + (uint64_t)(c >> 64);
    t[6] = (uint64_t)s;
    t[7] = (uint64_t)(s >> 64);
    const uint64_t m = t[0] * pinv;
    c = (u128)m * P6[0] + t[0];
    for (int j = 1; j < 6; j++) {
      c = (u128)m * P6[j] + t[j] + (uint64_t)(c >> 64);
      t[j - 1] = (uint64_t)c;
    }
    s = (u128)t[6] + (uint64_t)(c >> 64);
    t[5] = (uint64_t)s;
    t[6] = t[7] + (uint64_t)(s >> 64);
  }
  fq r;
  for (int i = 0; i < 6; i++) {
    r.l[2 * i] = (uint32_t)t[i];
    r.l[2 * i + 1] = (uint32_t)(t[i] >> 32);
  }
  return r;
}
#endif
// The out-of-line copies (one each on the device): called from everything that is not a hot
// inner loop, which keeps the code of the rarely-run paths small.
HBX_FQMUL_ATTR fq fq_mul_limbs(HBX_P12(a), HBX_P12(b)) { return fq_mul_body(HBX_L12(a), HBX_L12(b)); }
HBX_FQMUL_ATTR fq fq_sqr_limbs(HBX_P12(a)) { return fq_sqr_body(HBX_L12(a)); }
// Inlined copies for the hot loops (the Miller loop, the cyclotomic squarings): a call costs a
// wave far more than its argument moves at one wave per SIMD -- the s_waitcnt at the callee's
// entry, two jumps, and no overlap of the product with the caller's independent work
// (tools/microbench/parts.hip: 1.50 -> 1.00 us per dependent product, Miller loop -13 %).
HBX_HD fq fq_mul_inl(const fq& a, const fq& b) {
  HBX_COUNT_FQMUL();
#if defined(HBX_HOST_INT128) && !defined(__HIPCC__)
  return fq_mul_cios64(a, b);
#endif
  return fq_mul_body(a.l[0], a.l[1], a.l[2], a.l[3], a.l[4], a.l[5], a.l[6], a.l[7], a.l[8], a.l[9], a.l[10], a.l[11],
                     b.l[0], b.l[1], b.l[2], b.l[3], b.l[4], b.l[5], b.l[6], b.l[7], b.l[8], b.l[9], b.l[10], b.l[11]);
}
HBX_HD fq fq_sqr_inl(const fq& a) {
  HBX_COUNT_FQMUL();
#if defined(HBX_HOST_INT128) && !defined(__HIPCC__)
  return fq_mul_cios64(a, a);
#endif
  return fq_sqr_body(a.l[0], a.l[1], a.l[2], a.l[3], a.l[4], a.l[5], a.l[6], a.l[7], a.l[8], a.l[9], a.l[10], a.l[11]);
}
HBX_HD fq fq_mul(const fq& a, const fq& b) {
  HBX_COUNT_FQMUL();
#if defined(HBX_HOST_INT128) && !defined(__HIPCC__)
  return fq_mul_cios64(a, b);
#endif
  return fq_mul_limbs(a.l[0], a.l[1], a.l[2], a.l[3], a.l[4], a.l[5], a.l[6], a.l[7], a.l[8], a.l[9], a.l[10],
                      a.l[11], b.l[0], b.l[1], b.l[2], b.l[3], b.l[4], b.l[5], b.l[6], b.l[7], b.l[8], b.l[9],
                      b.l[10], b.l[11]);
}
#undef HBX_L12
#undef HBX_P12
#undef HBX_FQMUL_ATTR

HBX_HD fq fq_sqr(const fq& a) {
  HBX_COUNT_FQMUL();
#if defined(HBX_HOST_INT128) && !defined(__HIPCC__)
  return fq_mul_cios64(a, a);
#endif
  return fq_sqr_limbs(a.l[0], a.l[1], a.l[2], a.l[3], a.l[4], a.l[5], a.l[6], a.l[7], a.l[8], a.l[9], a.l[10],
                      a.l[11]);
}

// 32-bit add/sub with carry.  Device: clang's carry builtins lower to one v_addc_co_u32 /
// v_subb_co_u32 per limb with the carry in VCC (the portable 64-bit form compiled to ~10 VALU
// instructions per limb on gfx950: v_lshl_add_u64 + shifts + moves).
HBX_HD uint32_t addc32(uint32_t a, uint32_t b, uint32_t& c) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t co;
  const uint32_t r = __builtin_addc(a, b, c, &co);
  c = co;
  return r;
#else
  const uint64_t v = (uint64_t)a + b + c;
  c = (uint32_t)(v >> 32);
  return (uint32_t)v;
#endif
}
HBX_HD uint32_t subb32(uint32_t a, uint32_t b, uint32_t& br) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t bo;
  const uint32_t r = __builtin_subc(a, b, br, &bo);
  br = bo;
  return r;
#else
  const uint64_t v = (uint64_t)a - b - br;
  br = (uint32_t)(v >> 32) & 1u;
  return (uint32_t)v;
#endif
}

// r = a + b reduced into [0, 2p) (inputs <= 2p).
HBX_HD fq fq_add(const fq& a, const fq& b) {
  fq s, d;
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) s.l[i] = addc32(a.l[i], b.l[i], carry);
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d.l[i] = subb32(s.l[i], FQ_2P[i], borrow);
  // a + b < 4p < 2^384 so no carry out; keep s if s < 2p (borrow), else d
  fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = borrow ? s.l[i] : d.l[i];
  return r;
}

// r = a - b (+2p if negative), result in [0, 2p].
HBX_HD fq fq_sub(const fq& a, const fq& b) {
  fq d;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d.l[i] = subb32(a.l[i], b.l[i], borrow);
  const uint32_t mask = 0u - borrow;
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d.l[i] = addc32(d.l[i], FQ_2P[i] & mask, carry);
  return d;
}

HBX_HD fq fq_neg(const fq& a) { return fq_sub(fq_zero(), a); }
HBX_HD fq fq_dbl(const fq& a) { return fq_add(a, a); }

// Conditional subtract of a 12-limb constant if x >= c.
HBX_HD fq fq_csub(const fq& x, const uint32_t* c) {
  fq d;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d.l[i] = subb32(x.l[i], c[i], borrow);
  fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = borrow ? x.l[i] : d.l[i];
  return r;
}

// Canonical representative in [0, p) of a lazy value in [0, 2p].
HBX_HD fq fq_canon(const fq& a) { return fq_csub(fq_csub(a, FQ_P), FQ_P); }

HBX_HD bool fq_is_zero(const fq& a) {
  fq c = fq_canon(a);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) o |= c.l[i];
  return o == 0;
}
HBX_HD bool fq_eq(const fq& a, const fq& b) { return fq_is_zero(fq_sub(a, b)); }

HBX_HD fq fq_to_mont(const fq& a) { return fq_mul(a, fq_from_const(FQ_R2)); }
HBX_HD fq fq_from_mont(const fq& a) {
  fq one = fq_zero();
  one.l[0] = 1;
  return fq_canon(fq_mul(a, one));
}

// a^e for a fixed 12-limb exponent, left-to-right, 4-bit fixed window (~381 S + ~95 M).
HBX_HDNI fq fq_pow_const(const fq& a, const uint32_t* e) {
  fq tab[16];
  tab[0] = fq_one();
  tab[1] = a;
  for (int i = 2; i < 16; i++) tab[i] = fq_mul(tab[i - 1], a);
  fq r = fq_one();
  bool started = false;
  for (int w = 95; w >= 0; w--) {
    const uint32_t nib = (e[w >> 3] >> ((w & 7) * 4)) & 0xF;
    if (started) {
#pragma unroll 1
      for (int q = 0; q < 4; q++) r = fq_sqr_inl(r);
    }
    if (nib) {
      // select tab[nib] without dynamic register indexing
      fq t = tab[1];
      for (int k = 2; k < 16; k++)
        if ((uint32_t)k == nib) t = tab[k];
      r = started ? fq_mul_inl(r, t) : t;
      started = true;
    }
  }
  return r;
}

// x^-1 mod m (x canonical, m odd, N limbs) by Bernstein-Yang divsteps ("safegcd"), batched 30
// at a time: with delta = 1, (f, g) = (m, x), (d, e) = (0, 1) and the invariants f = d x,
// g = e x (mod m), a divstep is
//   delta > 0 and g odd:  (delta, f, g) <- (1 - delta, g, (g - f) / 2)
//   g odd otherwise:      (delta, f, g) <- (1 + delta, f, (g + f) / 2)
//   g even:               (delta, f, g) <- (1 + delta, f, g / 2)
// and depends only on delta and the parity of g, so 30 steps run on the low words of f and g and
// give an integer matrix T with 2^30 (f', g') = T (f, g) (|entries| <= 2^30); T then updates the
// full f, g (exact shift) and d, e (mod m, made divisible by 2^30 with a multiple of m).
// Half-delta variant ("hddivsteps"): delta starts at 1/2 (the steps hold `delta` = 2 delta: start
// 1, updates 2 - delta / 2 + delta), which lowers the step bound from Bernstein-Yang's
// floor((49 b + 57) / 17) to floor((45907 b + 26313) / 19929) (b = 32N bits; the bound libsecp256k1's
// safegcd uses, 590 steps at 256 bits): 886 steps at 381 bits, run as 31 batches of 30 with a
// margin of one batch (Bernstein-Yang's bound: 37).  After them g = 0, f = +-1 and x^-1 = +-d.
// Fixed step count and selects only: every lane of a wave runs the same instructions (~30k VALU
// ops for N = 12, against ~150k for the bit-by-bit binary Euclid this replaced, whose
// data-dependent branch split the wave).  x = 0 gives 0.
// NS steps (NS <= 30; the digit-form inversion of fieldd.hpp runs 28 on a 28-bit digit)
template <int NS>
HBX_HD void divsteps_n(int32_t& delta, uint32_t f, uint32_t g, int32_t& u, int32_t& v, int32_t& q, int32_t& r) {
  int32_t uu = 1, vv = 0, qq = 0, rr = 1;
  constexpr int UR = NS % 7 == 0 ? 7 : 6;  // 30 steps: 5 x 6 as before; 28: 4 x 7
#pragma unroll UR
  for (int i = 0; i < NS; i++) {
    const bool godd = (g & 1u) != 0;
    const bool sw = godd && delta > 0;
    const uint32_t nf = sw ? g : f;
    const uint32_t ng = sw ? g - f : (godd ? g + f : g);
    const int32_t nu = sw ? qq : uu, nv = sw ? rr : vv;
    const int32_t nq = sw ? qq - uu : (godd ? qq + uu : qq);
    const int32_t nr = sw ? rr - vv : (godd ? rr + vv : rr);
    delta = sw ? 2 - delta : 2 + delta;  // 2 delta (half-delta steps)
    f = nf;
    g = ng >> 1;
    uu = nu * 2;
    vv = nv * 2;
    qq = nq;
    rr = nr;
  }
  u = uu;
  v = vv;
  q = qq;
  r = rr;
}
HBX_HD void divsteps30(int32_t& delta, uint32_t f, uint32_t g, int32_t& u, int32_t& v, int32_t& q, int32_t& r) {
  divsteps_n<30>(delta, f, g, u, v, q, r);
}
// out = (ca a + cb b) / 2^30 for L-limb two's complement a, b (top limb signed); exact.
template <int L>
HBX_HD void lincomb_shr30(const uint32_t* a, const uint32_t* b, int32_t ca, int32_t cb, uint32_t* out) {
  int64_t acc = 0;
  uint32_t prev = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int64_t ai = i == L - 1 ? (int64_t)(int32_t)a[i] : (int64_t)a[i];
    const int64_t bi = i == L - 1 ? (int64_t)(int32_t)b[i] : (int64_t)b[i];
    acc += (int64_t)ca * ai + (int64_t)cb * bi;
    const uint32_t lo = (uint32_t)acc;
    acc >>= 32;
    if (i > 0) out[i - 1] = (prev >> 30) | (lo << 2);
    prev = lo;
  }
  out[L - 1] = (prev >> 30) | ((uint32_t)acc << 2);
}
// out = (ca d + cb e) / 2^30 mod m in [0, m) for d, e in [0, m) (L = N + 1 limbs, top limb 0);
// minv = m^-1 mod 2^32.
template <int L>
HBX_HD void lincomb_mod_shr30(const uint32_t* d, const uint32_t* e, int32_t ca, int32_t cb, const uint32_t* m,
                              uint32_t minv, uint32_t* out) {
  const uint32_t tlo = (uint32_t)ca * d[0] + (uint32_t)cb * e[0];
  const uint32_t k = ((0u - tlo) * minv) & 0x3FFFFFFFu;  // t + k m = 0 mod 2^30
  int64_t acc = 0;
  uint32_t prev = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const uint32_t mi = i < L - 1 ? m[i] : 0u;
    acc += (int64_t)ca * (int64_t)d[i] + (int64_t)cb * (int64_t)e[i] + (int64_t)((uint64_t)k * mi);
    const uint32_t lo = (uint32_t)acc;
    acc >>= 32;
    if (i > 0) out[i - 1] = (prev >> 30) | (lo << 2);
    prev = lo;
  }
  out[L - 1] = (prev >> 30) | ((uint32_t)acc << 2);
  // out in (-m, 2m): add m if negative, then subtract m if still >= m
  uint32_t t[L];
  const uint32_t neg = 0u - (out[L - 1] >> 31);
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) out[i] = addc32(out[i], (i < L - 1 ? m[i] : 0u) & neg, c);
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < L; i++) t[i] = subb32(out[i], i < L - 1 ? m[i] : 0u, br);
  const bool ge = (t[L - 1] >> 31) == 0;
#pragma unroll
  for (int i = 0; i < L; i++) out[i] = ge ? t[i] : out[i];
}
template <int N>
HBX_HD void binv_limbs(const uint32_t* x, const uint32_t* m, uint32_t* out) {
  constexpr int L = N + 1;
  constexpr int BATCHES = ((45907 * 32 * N + 26313) / 19929 + 30 + 29) / 30;  // hddivsteps bound + one batch
  uint32_t f[L], g[L], d[L], e[L];
#pragma unroll
  for (int i = 0; i < L; i++) {
    f[i] = i < N ? m[i] : 0u;
    g[i] = i < N ? x[i] : 0u;
    d[i] = 0;
    e[i] = i == 0 ? 1u : 0u;
  }
  uint32_t minv = m[0];  // Newton: 3 -> 6 -> 12 -> 24 -> 48 correct low bits
#pragma unroll
  for (int i = 0; i < 4; i++) minv *= 2u - m[0] * minv;
  int32_t delta = 1;  // 2 delta, delta = 1/2
#pragma unroll 1
  for (int b = 0; b < BATCHES; b++) {
    int32_t u, v, q, r;
    divsteps30(delta, f[0], g[0], u, v, q, r);
    uint32_t nf[L], ng[L], nd[L], ne[L];
    lincomb_shr30<L>(f, g, u, v, nf);
    lincomb_shr30<L>(f, g, q, r, ng);
    lincomb_mod_shr30<L>(d, e, u, v, m, minv, nd);
    lincomb_mod_shr30<L>(d, e, q, r, m, minv, ne);
#pragma unroll
    for (int i = 0; i < L; i++) {
      f[i] = nf[i];
      g[i] = ng[i];
      d[i] = nd[i];
      e[i] = ne[i];
    }
  }
  // f = +-1: x^-1 = d or m - d (d = 0 stays 0: x = 0)
  const bool fneg = (f[L - 1] >> 31) != 0;
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < N; i++) nz |= d[i];
  uint32_t t[N], br = 0;
#pragma unroll
  for (int i = 0; i < N; i++) t[i] = subb32(m[i], d[i], br);
#pragma unroll
  for (int i = 0; i < N; i++) out[i] = (fneg && nz != 0) ? t[i] : d[i];
}

// Montgomery inverse: a = x R  ->  binv(a) = x^-1 R^-1, times R^3 in the Montgomery product
// gives x^-1 R.
HBX_HD fq fq_inv_i(const fq& a) {  // inlined copy (no call frame: pairing2d.hpp)
  const fq c = fq_canon(a);
  fq r;
  binv_limbs<12>(c.l, FQ_P, r.l);
  return fq_mul(r, fq_from_const(FQ_R3));
}
HBX_HDNI fq fq_inv(const fq& a) { return fq_inv_i(a); }

// Square root for p = 3 mod 4.  Returns false if a is a non-residue.
HBX_HD bool fq_sqrt(const fq& a, fq& out) {
  fq s = fq_pow_const(a, FQ_SQRT_EXP);
  out = s;
  return fq_eq(fq_sqr(s), a);
}

// Lexicographic "largest" flag of the zcash encoding: canonical(y) > (p-1)/2.
HBX_HD bool fq_lex_largest(const fq& y_mont) {
  fq y = fq_from_mont(y_mont);
  // y > (p-1)/2  <=>  (p-1)/2 - y borrows
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) (void)subb32(FQ_P_MINUS_1_HALF[i], y.l[i], borrow);
  return borrow != 0;
}

// Big-endian 48-byte encoding <-> canonical limbs (not Montgomery).
HBX_HD fq fq_from_be(const uint8_t* b) {
  fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint8_t* q = b + 44 - 4 * i;
    r.l[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
  return r;
}
HBX_HD void fq_to_be(const fq& a, uint8_t* b) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint8_t* q = b + 44 - 4 * i;
    q[0] = (uint8_t)(a.l[i] >> 24);
    q[1] = (uint8_t)(a.l[i] >> 16);
    q[2] = (uint8_t)(a.l[i] >> 8);
    q[3] = (uint8_t)a.l[i];
  }
}
// true iff canonical value < p
HBX_HD bool fq_lt_p(const fq& a) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) (void)subb32(a.l[i], FQ_P[i], borrow);
  return borrow != 0;
}

// ----------------------------------------------------------------------------------------------
// Fq2 = Fq[u]/(u^2 + 1)
// ----------------------------------------------------------------------------------------------
HBX_HD fq2 fq2_zero() { return fq2{fq_zero(), fq_zero()}; }
HBX_HD fq2 fq2_one() { return fq2{fq_one(), fq_zero()}; }
HBX_HD fq2 fq2_add(const fq2& a, const fq2& b) { return fq2{fq_add(a.c0, b.c0), fq_add(a.c1, b.c1)}; }
HBX_HD fq2 fq2_sub(const fq2& a, const fq2& b) { return fq2{fq_sub(a.c0, b.c0), fq_sub(a.c1, b.c1)}; }
HBX_HD fq2 fq2_neg(const fq2& a) { return fq2{fq_neg(a.c0), fq_neg(a.c1)}; }
HBX_HD fq2 fq2_dbl(const fq2& a) { return fq2{fq_dbl(a.c0), fq_dbl(a.c1)}; }
HBX_HD fq2 fq2_conj(const fq2& a) { return fq2{a.c0, fq_neg(a.c1)}; }

// Product policy of the tower templates below: FqCall = the out-of-line Fq product (compact code),
// FqInl = the inlined one (hot loops).  Same values either way.
struct FqCall {
  static HBX_HD fq mul(const fq& a, const fq& b) { return fq_mul(a, b); }
  static HBX_HD fq sqr(const fq& a) { return fq_sqr(a); }
};
struct FqInl {
  static HBX_HD fq mul(const fq& a, const fq& b) { return fq_mul_inl(a, b); }
  static HBX_HD fq sqr(const fq& a) { return fq_sqr_inl(a); }
};

template <class M>
HBX_HD fq2 fq2_mul_t(const fq2& a, const fq2& b) {
  const fq t0 = M::mul(a.c0, b.c0);
  const fq t1 = M::mul(a.c1, b.c1);
  const fq t2 = M::mul(fq_add(a.c0, a.c1), fq_add(b.c0, b.c1));
  return fq2{fq_sub(t0, t1), fq_sub(fq_sub(t2, t0), t1)};
}
template <class M>
HBX_HD fq2 fq2_sqr_t(const fq2& a) {
  // (a0 + a1)(a0 - a1), 2 a0 a1
  const fq t0 = M::mul(fq_add(a.c0, a.c1), fq_sub(a.c0, a.c1));
  const fq t1 = M::mul(a.c0, a.c1);
  return fq2{t0, fq_dbl(t1)};
}
template <class M>
HBX_HD fq2 fq2_mul_fq_t(const fq2& a, const fq& s) { return fq2{M::mul(a.c0, s), M::mul(a.c1, s)}; }
HBX_HD fq2 fq2_mul(const fq2& a, const fq2& b) { return fq2_mul_t<FqCall>(a, b); }
HBX_HD fq2 fq2_sqr(const fq2& a) {
  return fq2_sqr_t<FqCall>(a);
}
HBX_HD fq2 fq2_mul_fq(const fq2& a, const fq& s) { return fq2_mul_fq_t<FqCall>(a, s); }
// multiply by the Fq6 non-residue xi = 1 + u
HBX_HD fq2 fq2_mul_xi(const fq2& a) { return fq2{fq_sub(a.c0, a.c1), fq_add(a.c0, a.c1)}; }
HBX_HD bool fq2_is_zero(const fq2& a) { return fq_is_zero(a.c0) && fq_is_zero(a.c1); }
HBX_HD bool fq2_eq(const fq2& a, const fq2& b) { return fq_eq(a.c0, b.c0) && fq_eq(a.c1, b.c1); }
HBX_HD fq2 fq2_canon(const fq2& a) { return fq2{fq_canon(a.c0), fq_canon(a.c1)}; }

HBX_HDNI fq2 fq2_inv(const fq2& a) {
  const fq n = fq_add(fq_sqr(a.c0), fq_sqr(a.c1));
  const fq ni = fq_inv(n);
  return fq2{fq_mul(a.c0, ni), fq_neg(fq_mul(a.c1, ni))};
}

// pairing 0.14 Ord on Fq2 (c1 first, then c0) applied to (y, -y): is y the larger root?
HBX_HD int fq_cmp_canon(const fq& a, const fq& b) {  // canonical inputs
  for (int i = 11; i >= 0; i--) {
    if (a.l[i] != b.l[i]) return a.l[i] > b.l[i] ? 1 : -1;
  }
  return 0;
}
HBX_HD bool fq2_lex_largest(const fq2& y_mont) {
  const fq y0 = fq_from_mont(y_mont.c0), y1 = fq_from_mont(y_mont.c1);
  const fq2 n = fq2_neg(y_mont);
  const fq n0 = fq_from_mont(n.c0), n1 = fq_from_mont(n.c1);
  int c = fq_cmp_canon(y1, n1);
  if (c == 0) c = fq_cmp_canon(y0, n0);
  return c > 0;
}

// Fq2 square root (p = 3 mod 4), norm method, two fixed exponentiations:
//   a = a0 + a1 u is a square iff N(a) = a0^2 + a1^2 is a square in Fq (-1 is a non-residue);
//   s = sqrt(N(a)), alpha = (a0 + s)/2, e = alpha^((p-3)/4), t = alpha e = alpha^((p+1)/4),
//   c = t e = alpha^((p-1)/2) = +-1 and 1/t = c e, so
//     c = +1:  x0 = t,          x1 = a1 e / 2   (x0^2 = alpha)
//     c = -1:  x0 = -a1 e / 2,  x1 = t          (x1^2 = -alpha)
// (pairing's Fq2::sqrt returns one of the two roots; callers normalise the sign, so the choice
// of root does not affect any output).  a1 = 0 never reaches the norm path.
// Step 1: the residuosity test; s is reused by step 2.
HBX_HD bool fq2_norm_sqrt(const fq2& a, fq& s) {
  const fq n = fq_add(fq_sqr(a.c0), fq_sqr(a.c1));
  return fq_sqrt(n, s);
}
// Step 2 for a known square with a1 != 0.
HBX_HDNI fq2 fq2_sqrt_from_norm(const fq2& a, const fq& s) {
  const fq half = fq_from_const(FQ_HALF_MONT);
  const fq alpha = fq_mul(fq_add(a.c0, s), half);
  const fq e = fq_pow_const(alpha, FQ_P_MINUS_3_DIV_4);
  const fq t = fq_mul(alpha, e);
  const fq c = fq_mul(t, e);
  const fq h = fq_mul(fq_mul(a.c1, e), half);
  if (fq_eq(c, fq_one())) return fq2{t, h};
  return fq2{fq_neg(h), t};
}
// Square root in Fq; false for a non-residue.
HBX_HDNI bool fq2_sqrt(const fq2& a, fq2& out) {
  if (fq_is_zero(a.c1)) {
    // one exponentiation: s^2 = a0 if a0 is a square, else s^2 = -a0 and (s u)^2 = a0
    const fq sq = fq_pow_const(a.c0, FQ_SQRT_EXP);
    if (fq_eq(fq_sqr(sq), a.c0)) out = fq2{sq, fq_zero()};
    else out = fq2{fq_zero(), sq};
    return true;
  }
  fq s;
  if (!fq2_norm_sqrt(a, s)) return false;
  out = fq2_sqrt_from_norm(a, s);
  return true;
}

// ----------------------------------------------------------------------------------------------
// Fq6 = Fq2[v]/(v^3 - xi)
// ----------------------------------------------------------------------------------------------
HBX_HD fq6 fq6_zero() { return fq6{fq2_zero(), fq2_zero(), fq2_zero()}; }
HBX_HD fq6 fq6_one() { return fq6{fq2_one(), fq2_zero(), fq2_zero()}; }
HBX_HD fq6 fq6_add(const fq6& a, const fq6& b) {
  return fq6{fq2_add(a.c0, b.c0), fq2_add(a.c1, b.c1), fq2_add(a.c2, b.c2)};
}
HBX_HD fq6 fq6_sub(const fq6& a, const fq6& b) {
  return fq6{fq2_sub(a.c0, b.c0), fq2_sub(a.c1, b.c1), fq2_sub(a.c2, b.c2)};
}
HBX_HD fq6 fq6_neg(const fq6& a) { return fq6{fq2_neg(a.c0), fq2_neg(a.c1), fq2_neg(a.c2)}; }
// multiply by v: (c0, c1, c2) v = (xi c2, c0, c1)
HBX_HD fq6 fq6_mul_v(const fq6& a) { return fq6{fq2_mul_xi(a.c2), a.c0, a.c1}; }

// Karatsuba-style Fq6 product (6 Fq2 mults).
template <class M>
HBX_HD fq6 fq6_mul_t(const fq6& a, const fq6& b) {
  const fq2 t0 = fq2_mul_t<M>(a.c0, b.c0);
  const fq2 t1 = fq2_mul_t<M>(a.c1, b.c1);
  const fq2 t2 = fq2_mul_t<M>(a.c2, b.c2);
  // c0 = t0 + xi((a1+a2)(b1+b2) - t1 - t2)
  fq2 c0 = fq2_mul_t<M>(fq2_add(a.c1, a.c2), fq2_add(b.c1, b.c2));
  c0 = fq2_add(t0, fq2_mul_xi(fq2_sub(fq2_sub(c0, t1), t2)));
  // c1 = (a0+a1)(b0+b1) - t0 - t1 + xi t2
  fq2 c1 = fq2_mul_t<M>(fq2_add(a.c0, a.c1), fq2_add(b.c0, b.c1));
  c1 = fq2_add(fq2_sub(fq2_sub(c1, t0), t1), fq2_mul_xi(t2));
  // c2 = (a0+a2)(b0+b2) - t0 - t2 + t1
  fq2 c2 = fq2_mul_t<M>(fq2_add(a.c0, a.c2), fq2_add(b.c0, b.c2));
  c2 = fq2_add(fq2_sub(fq2_sub(c2, t0), t2), t1);
  return fq6{c0, c1, c2};
}
HBX_HD fq6 fq6_mul_i(const fq6& a, const fq6& b) { return fq6_mul_t<FqCall>(a, b); }
HBX_HDNI fq6 fq6_mul(const fq6& a, const fq6& b) { return fq6_mul_i(a, b); }

HBX_HD fq6 fq6_sqr_i(const fq6& a) {
  // CH-SQR2
  const fq2 s0 = fq2_sqr(a.c0);
  const fq2 ab = fq2_mul(a.c0, a.c1);
  const fq2 s1 = fq2_dbl(ab);
  const fq2 s2 = fq2_sqr(fq2_add(fq2_sub(a.c0, a.c1), a.c2));
  const fq2 bc = fq2_mul(a.c1, a.c2);
  const fq2 s3 = fq2_dbl(bc);
  const fq2 s4 = fq2_sqr(a.c2);
  const fq2 c0 = fq2_add(s0, fq2_mul_xi(s3));
  const fq2 c1 = fq2_add(s1, fq2_mul_xi(s4));
  const fq2 c2 = fq2_sub(fq2_sub(fq2_add(fq2_add(s1, s2), s3), s0), s4);
  return fq6{c0, c1, c2};
}
HBX_HDNI fq6 fq6_sqr(const fq6& a) { return fq6_sqr_i(a); }

// a * (b0 + b1 v)   (5 Fq2 mults)
template <class M>
HBX_HD fq6 fq6_mul_by_01_t(const fq6& a, const fq2& b0, const fq2& b1) {
  const fq2 t0 = fq2_mul_t<M>(a.c0, b0);
  const fq2 t1 = fq2_mul_t<M>(a.c1, b1);
  // c0 = t0 + xi * (a2 * b1)
  const fq2 c0 = fq2_add(t0, fq2_mul_xi(fq2_mul_t<M>(a.c2, b1)));
  // c1 = (a0 + a1)(b0 + b1) - t0 - t1
  const fq2 c1 = fq2_sub(fq2_sub(fq2_mul_t<M>(fq2_add(a.c0, a.c1), fq2_add(b0, b1)), t0), t1);
  // c2 = a2 * b0 + t1
  const fq2 c2 = fq2_add(fq2_mul_t<M>(a.c2, b0), t1);
  return fq6{c0, c1, c2};
}
HBX_HD fq6 fq6_mul_by_01_i(const fq6& a, const fq2& b0, const fq2& b1) { return fq6_mul_by_01_t<FqCall>(a, b0, b1); }
HBX_HDNI fq6 fq6_mul_by_01(const fq6& a, const fq2& b0, const fq2& b1) { return fq6_mul_by_01_i(a, b0, b1); }

// a * (s v) with s in Fq: (xi a2 s, a0 s, a1 s)
template <class M>
HBX_HD fq6 fq6_mul_by_1_fq_t(const fq6& a, const fq& s) {
  return fq6{fq2_mul_xi(fq2_mul_fq_t<M>(a.c2, s)), fq2_mul_fq_t<M>(a.c0, s), fq2_mul_fq_t<M>(a.c1, s)};
}
HBX_HD fq6 fq6_mul_by_1_fq(const fq6& a, const fq& s) { return fq6_mul_by_1_fq_t<FqCall>(a, s); }

HBX_HDNI fq6 fq6_inv(const fq6& a) {
  const fq2 c0 = fq2_sub(fq2_sqr(a.c0), fq2_mul_xi(fq2_mul(a.c1, a.c2)));
  const fq2 c1 = fq2_sub(fq2_mul_xi(fq2_sqr(a.c2)), fq2_mul(a.c0, a.c1));
  const fq2 c2 = fq2_sub(fq2_sqr(a.c1), fq2_mul(a.c0, a.c2));
  const fq2 t = fq2_add(fq2_mul(a.c0, c0), fq2_mul_xi(fq2_add(fq2_mul(a.c2, c1), fq2_mul(a.c1, c2))));
  const fq2 ti = fq2_inv(t);
  return fq6{fq2_mul(c0, ti), fq2_mul(c1, ti), fq2_mul(c2, ti)};
}

// ----------------------------------------------------------------------------------------------
// Fq12 = Fq6[w]/(w^2 - v)
// ----------------------------------------------------------------------------------------------
HBX_HD fq12 fq12_one() { return fq12{fq6_one(), fq6_zero()}; }
HBX_HD fq12 fq12_conj(const fq12& a) { return fq12{a.c0, fq6_neg(a.c1)}; }

HBX_HD fq12 fq12_mul_i(const fq12& a, const fq12& b) {
  const fq6 t0 = fq6_mul_i(a.c0, b.c0);
  const fq6 t1 = fq6_mul_i(a.c1, b.c1);
  const fq6 c1 = fq6_sub(fq6_sub(fq6_mul_i(fq6_add(a.c0, a.c1), fq6_add(b.c0, b.c1)), t0), t1);
  return fq12{fq6_add(t0, fq6_mul_v(t1)), c1};
}
HBX_HDNI fq12 fq12_mul(const fq12& a, const fq12& b) { return fq12_mul_i(a, b); }

template <class M>
HBX_HD fq12 fq12_sqr_t(const fq12& a) {
  // complex squaring: c0 = (a0 + a1)(a0 + v a1) - ab - v ab, c1 = 2 ab
  const fq6 ab = fq6_mul_t<M>(a.c0, a.c1);
  const fq6 t = fq6_mul_t<M>(fq6_add(a.c0, a.c1), fq6_add(a.c0, fq6_mul_v(a.c1)));
  const fq6 c0 = fq6_sub(fq6_sub(t, ab), fq6_mul_v(ab));
  return fq12{c0, fq6_add(ab, ab)};
}
HBX_HD fq12 fq12_sqr_i(const fq12& a) { return fq12_sqr_t<FqCall>(a); }
HBX_HDNI fq12 fq12_sqr(const fq12& a) { return fq12_sqr_i(a); }

// f * (c0 + c1 v + c4 v w) with c0, c1 in Fq2 and c4 in Fq -- the shape of a prepared line
// evaluated at a G1 point (pairing's mul_by_014, with c4 real).
template <class M>
HBX_HD fq12 fq12_mul_by_014_t(const fq12& f, const fq2& c0, const fq2& c1, const fq& c4) {
  const fq6 aa = fq6_mul_by_01_t<M>(f.c0, c0, c1);
  const fq6 bb = fq6_mul_by_1_fq_t<M>(f.c1, c4);
  const fq2 o = fq2{fq_add(c1.c0, c4), c1.c1};
  fq6 s = fq6_add(f.c1, f.c0);
  s = fq6_mul_by_01_t<M>(s, c0, o);
  const fq6 n1 = fq6_sub(fq6_sub(s, aa), bb);
  const fq6 n0 = fq6_add(fq6_mul_v(bb), aa);
  return fq12{n0, n1};
}
HBX_HD fq12 fq12_mul_by_014_i(const fq12& f, const fq2& c0, const fq2& c1, const fq& c4) {
  return fq12_mul_by_014_t<FqCall>(f, c0, c1, c4);
}
HBX_HDNI fq12 fq12_mul_by_014(const fq12& f, const fq2& c0, const fq2& c1, const fq& c4) { return fq12_mul_by_014_i(f, c0, c1, c4); }

HBX_HDNI fq12 fq12_inv(const fq12& a) {
  const fq6 t = fq6_sub(fq6_sqr(a.c0), fq6_mul_v(fq6_sqr(a.c1)));
  const fq6 ti = fq6_inv(t);
  return fq12{fq6_mul(a.c0, ti), fq6_neg(fq6_mul(a.c1, ti))};
}

// Frobenius maps.  With f = sum g_i w^i (g0..g5 = c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2),
// (g w^i)^p = conj(g) gamma_1,i w^i and (g w^i)^(p^2) = g gamma_2,i w^i.
HBX_HD fq2 fq2_frob_coef1(const fq2& g, int i) {
  const uint32_t* k0 = i == 1 ? FROB1_C1_0 : i == 2 ? FROB1_C2_0 : i == 3 ? FROB1_C3_0 : i == 4 ? FROB1_C4_0 : FROB1_C5_0;
  const uint32_t* k1 = i == 1 ? FROB1_C1_1 : i == 2 ? FROB1_C2_1 : i == 3 ? FROB1_C3_1 : i == 4 ? FROB1_C4_1 : FROB1_C5_1;
  return fq2_mul(fq2_conj(g), fq2{fq_from_const(k0), fq_from_const(k1)});
}
HBX_HDNI fq12 fq12_frobenius(const fq12& a) {
  fq12 r;
  r.c0.c0 = fq2_conj(a.c0.c0);
  r.c1.c0 = fq2_frob_coef1(a.c1.c0, 1);
  r.c0.c1 = fq2_frob_coef1(a.c0.c1, 2);
  r.c1.c1 = fq2_frob_coef1(a.c1.c1, 3);
  r.c0.c2 = fq2_frob_coef1(a.c0.c2, 4);
  r.c1.c2 = fq2_frob_coef1(a.c1.c2, 5);
  return r;
}
HBX_HDNI fq12 fq12_frobenius2(const fq12& a) {
  fq12 r;
  r.c0.c0 = a.c0.c0;
  r.c1.c0 = fq2_mul_fq(a.c1.c0, fq_from_const(FROB2_C1));
  r.c0.c1 = fq2_mul_fq(a.c0.c1, fq_from_const(FROB2_C2));
  r.c1.c1 = fq2_mul_fq(a.c1.c1, fq_from_const(FROB2_C3));
  r.c0.c2 = fq2_mul_fq(a.c0.c2, fq_from_const(FROB2_C4));
  r.c1.c2 = fq2_mul_fq(a.c1.c2, fq_from_const(FROB2_C5));
  return r;
}

// Granger-Scott squaring, valid in the cyclotomic subgroup (after the easy part).
template <class M>
HBX_HD void fq4_sqr_t(const fq2& a, const fq2& b, fq2& c0, fq2& c1) {
  const fq2 t0 = fq2_sqr_t<M>(a);
  const fq2 t1 = fq2_sqr_t<M>(b);
  c0 = fq2_add(fq2_mul_xi(t1), t0);
  c1 = fq2_sub(fq2_sub(fq2_sqr_t<M>(fq2_add(a, b)), t0), t1);
}
HBX_HD void fq4_sqr(const fq2& a, const fq2& b, fq2& c0, fq2& c1) { fq4_sqr_t<FqCall>(a, b, c0, c1); }
template <class M>
HBX_HD fq12 fq12_cyclotomic_sqr_t(const fq12& f) {
  fq2 z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2;
  fq2 z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
  fq2 t0, t1, t2, t3;
  fq4_sqr_t<M>(z0, z1, t0, t1);
  z0 = fq2_sub(t0, z0);
  z0 = fq2_add(fq2_dbl(z0), t0);
  z1 = fq2_add(t1, z1);
  z1 = fq2_add(fq2_dbl(z1), t1);
  fq4_sqr_t<M>(z2, z3, t0, t1);
  fq4_sqr_t<M>(z4, z5, t2, t3);
  z4 = fq2_sub(t0, z4);
  z4 = fq2_add(fq2_dbl(z4), t0);
  z5 = fq2_add(t1, z5);
  z5 = fq2_add(fq2_dbl(z5), t1);
  t0 = fq2_mul_xi(t3);
  z2 = fq2_add(t0, z2);
  z2 = fq2_add(fq2_dbl(z2), t0);
  z3 = fq2_sub(t2, z3);
  z3 = fq2_add(fq2_dbl(z3), t2);
  return fq12{fq6{z0, z4, z3}, fq6{z2, z1, z5}};
}
HBX_HD fq12 fq12_cyclotomic_sqr_i(const fq12& f) { return fq12_cyclotomic_sqr_t<FqCall>(f); }
HBX_HDNI fq12 fq12_cyclotomic_sqr(const fq12& f) { return fq12_cyclotomic_sqr_i(f); }

HBX_HD bool fq12_is_one(const fq12& a) {
  const fq12 o = fq12_one();
  return fq2_eq(a.c0.c0, o.c0.c0) && fq2_is_zero(a.c0.c1) && fq2_is_zero(a.c0.c2) &&
         fq2_is_zero(a.c1.c0) && fq2_is_zero(a.c1.c1) && fq2_is_zero(a.c1.c2);
}

// ----------------------------------------------------------------------------------------------
// Fr (255-bit scalar field): 8 limbs, Montgomery R = 2^256, canonical outputs (< r).
// ----------------------------------------------------------------------------------------------
HBX_HD fr fr_from_const(const uint32_t* c) {
  fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = c[i];
  return r;
}
HBX_HD fr fr_csub(const fr& x) {
  fr d;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d.l[i] = subb32(x.l[i], FR_R[i], borrow);
  fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = borrow ? x.l[i] : d.l[i];
  return r;
}
// Montgomery product with a full carry word (r's top limb is large: no lazy trick), output < r.
HBX_HDNI fr fr_mul(const fr& a, const fr& b) {
  uint32_t t[10];
#pragma unroll
  for (int j = 0; j < 10; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      c = (uint64_t)a.l[j] * b.l[i] + t[j] + (c >> 32);
      t[j] = (uint32_t)c;
    }
    uint64_t s = (uint64_t)t[8] + (c >> 32);
    t[8] = (uint32_t)s;
    t[9] = (uint32_t)(s >> 32);
    const uint32_t m = t[0] * FR_INV;
    c = (uint64_t)m * FR_R[0] + t[0];
#pragma unroll
    for (int j = 1; j < 8; j++) {
      c = (uint64_t)m * FR_R[j] + t[j] + (c >> 32);
      t[j - 1] = (uint32_t)c;
    }
    s = (uint64_t)t[8] + (c >> 32);
    t[7] = (uint32_t)s;
    t[8] = t[9] + (uint32_t)(s >> 32);
  }
  fr r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.l[j] = t[j];
  // t < 2r; t[8] may hold the top carry
  if (t[8]) {
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.l[i] = subb32(r.l[i], FR_R[i], borrow);
    return r;
  }
  return fr_csub(r);
}
HBX_HD fr fr_add(const fr& a, const fr& b) {
  fr s;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s.l[i] = addc32(a.l[i], b.l[i], c);
  return fr_csub(s);  // a + b < 2r < 2^256
}
HBX_HD fr fr_sub(const fr& a, const fr& b) {
  fr d;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d.l[i] = subb32(a.l[i], b.l[i], borrow);
  if (borrow) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d.l[i] = addc32(d.l[i], FR_R[i], c);
  }
  return d;
}
HBX_HD fr fr_to_mont(const fr& a) { return fr_mul(a, fr_from_const(FR_R2)); }
HBX_HD fr fr_from_mont(const fr& a) {
  fr one;
#pragma unroll
  for (int i = 0; i < 8; i++) one.l[i] = 0;
  one.l[0] = 1;
  return fr_mul(a, one);
}
HBX_HDNI fr fr_pow_const(const fr& a, const uint32_t* e) {
  fr r = fr_from_const(FR_ONE);
  for (int i = 255; i >= 0; i--) {
    r = fr_mul(r, r);
    if ((e[i >> 5] >> (i & 31)) & 1) r = fr_mul(r, a);
  }
  return r;
}
// Montgomery inverse over Fr by binary extended Euclid (binv_limbs), R = 2^256.
HBX_HDNI fr fr_inv(const fr& a) {
  const fr c = fr_csub(a);
  fr r;
  binv_limbs<8>(c.l, FR_R, r.l);
  return fr_mul(r, fr_from_const(FR_R3));
}

}  // namespace hbx
