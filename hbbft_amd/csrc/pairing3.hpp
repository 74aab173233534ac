// Three-lane cooperative pairing check for gfx950: one share check e(PA, QA) e(PB, QB) == 1 on a
// group of 3 lanes of a wave (21 groups per wave, lane 63 idle), the same bits as pairing.hpp's
// one-lane check2 (pairing 0.14 `Bls12::pairing` twice, compared; reference honey_badger.rs:229
// via threshold_crypto).
//
// Why: one lane per check needs 65,536 checks to fill the chip (N = 256 on one GPU).  A shard of
// an epoch (N = 256 over 8 GPUs: 8,192 checks per GPU) fills an eighth of the SIMDs and its
// latency is one lane's whole check.  Three lanes per check cut that latency ~2.5x, and the
// per-lane state is 24 dwords instead of 144, so several waves fit on a SIMD.
//
// Representation.  Fq12 = Fq4[X]/(X^3 - Y) with Fq4 = Fq2[Y]/(Y^2 - xi), X = w, Y = w^3: the
// element sum_{i<6} g_i w^i of the Fq6[w] tower (field.hpp; g_i = c0.c0, c1.c0, c0.c1, c1.c1,
// c0.c2, c1.c2) is a0 + a1 X + a2 X^2 with a_k = g_k + g_{k+3} Y.  Lane k of the group holds a_k.
// Every Fq12 operation becomes: each lane computes the Fq4 products that feed its own
// coefficient, with at most a few Fq4 values fetched from the other two lanes by ds_bpermute
// (24 dwords each):
//   * Miller squaring:   a_k^2 and a_k a_{k+1} per lane (15 Fq products), 3 fetches;
//   * line product:      l = L0 + L2 X^2 (L0 = c0 + y_P Y, L2 = c1 x_P), a_k L0 and a_k L2 per lane
//                        (16), 1 fetch;
//   * cyclotomic square: Granger-Scott, a_k^2 per lane (6), 1 fetch;
//   * general product:   a_k b_0, a_{k+1} b_2, a_{k+2} b_1 per lane (27), 5 fetches;
//   * Frobenius maps and conjugation are coefficient-wise (no fetch).
// Control flow is group-uniform; a group's shuffles only read lanes of the same group.
#pragma once
#include "pairing.hpp"

namespace hbx {
#if defined(__HIPCC__)

constexpr int G3 = 3;            // lanes per check
constexpr int G3_PER_WAVE = 21;  // groups per 64-lane wave

struct fq4 {
  fq2 c0, c1;  // c0 + c1 Y,  Y^2 = xi
};

__device__ __forceinline__ fq4 fq4_add(const fq4& a, const fq4& b) { return fq4{fq2_add(a.c0, b.c0), fq2_add(a.c1, b.c1)}; }
__device__ __forceinline__ fq4 fq4_sub(const fq4& a, const fq4& b) { return fq4{fq2_sub(a.c0, b.c0), fq2_sub(a.c1, b.c1)}; }
__device__ __forceinline__ fq4 fq4_dbl(const fq4& a) { return fq4{fq2_dbl(a.c0), fq2_dbl(a.c1)}; }
__device__ __forceinline__ fq4 fq4_conj(const fq4& a) { return fq4{a.c0, fq2_neg(a.c1)}; }
// times Y: (a0 + a1 Y) Y = xi a1 + a0 Y
__device__ __forceinline__ fq4 fq4_mul_y(const fq4& a) { return fq4{fq2_mul_xi(a.c1), a.c0}; }
__device__ __forceinline__ fq4 fq4_sel(bool c, const fq4& a, const fq4& b) {
  fq4 r;
  const uint32_t* pa = reinterpret_cast<const uint32_t*>(&a);
  const uint32_t* pb = reinterpret_cast<const uint32_t*>(&b);
  uint32_t* pr = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
  for (int i = 0; i < 48; i++) pr[i] = c ? pa[i] : pb[i];
  return r;
}
// Karatsuba: 3 Fq2 products
__device__ __forceinline__ fq4 fq4_mul(const fq4& a, const fq4& b) {
  const fq2 t0 = fq2_mul(a.c0, b.c0);
  const fq2 t1 = fq2_mul(a.c1, b.c1);
  const fq2 s = fq2_mul(fq2_add(a.c0, a.c1), fq2_add(b.c0, b.c1));
  return fq4{fq2_add(t0, fq2_mul_xi(t1)), fq2_sub(fq2_sub(s, t0), t1)};
}
// 3 Fq2 squarings (field.hpp fq4_sqr)
__device__ __forceinline__ fq4 fq4_square(const fq4& a) {
  fq4 r;
  fq4_sqr(a.c0, a.c1, r.c0, r.c1);
  return r;
}
__device__ __forceinline__ fq4 fq4_shfl(const fq4& v, int src) {
  fq4 r;
  const uint32_t* pv = reinterpret_cast<const uint32_t*>(&v);
  uint32_t* pr = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
  for (int i = 0; i < 48; i++) pr[i] = (uint32_t)__shfl((int)pv[i], src & 63, 64);
  return r;
}
__device__ __forceinline__ fq4 fq4_one() { return fq4{fq2_one(), fq2_zero()}; }
__device__ __forceinline__ fq4 fq4_zero() { return fq4{fq2_zero(), fq2_zero()}; }

// Position of this lane in its group.
struct grp3 {
  int gl;    // 0, 1, 2 (lane 63: 0, a group of one whose results are discarded)
  int base;  // first lane of the group
  __device__ int nxt() const { return base + (gl == 2 ? 0 : gl + 1); }
  __device__ int prv() const { return base + (gl == 0 ? 2 : gl - 1); }
};
__device__ __forceinline__ grp3 grp3_of_lane() {
  const int lane = (int)(threadIdx.x & 63);
  grp3 g;
  g.gl = lane == 63 ? 0 : lane % 3;
  g.base = lane - g.gl;
  return g;
}

// Fq12 (Fq6[w]) conjugation: g1, g3, g5 negated.
__device__ __forceinline__ fq4 conj3(const fq4& a, const grp3& g) {
  return g.gl == 1 ? fq4{fq2_neg(a.c0), a.c1} : fq4{a.c0, fq2_neg(a.c1)};
}

// Miller-loop squaring: (a0 + a1 X + a2 X^2)^2 =
//   (a0^2 + 2Y a1 a2) + (2 a0 a1 + Y a2^2) X + (a1^2 + 2 a0 a2) X^2.
// Lane k computes S_k = a_k^2 and P_k = a_k a_{k+1}.
__device__ __forceinline__ fq4 sqr3(const fq4& a, const grp3 g) {
  const fq4 an = fq4_shfl(a, g.nxt());
  const fq4 S = fq4_square(a);
  const fq4 P = fq4_mul(a, an);
  // lane 0 <- P_1, lane 1 <- P_0, lane 2 <- P_2;  lane 0 <- S_0, lane 1 <- S_2, lane 2 <- S_1
  const fq4 Pf = fq4_shfl(P, g.gl == 0 ? g.nxt() : g.gl == 1 ? g.prv() : g.base + 2);
  const fq4 Sf = fq4_shfl(S, g.gl == 0 ? g.base : g.gl == 1 ? g.nxt() : g.prv());
  const fq4 U = fq4_sel(g.gl == 1, fq4_mul_y(Sf), Sf);
  const fq4 V = fq4_sel(g.gl == 0, fq4_mul_y(Pf), Pf);
  return fq4_add(U, fq4_dbl(V));
}

// f *= l with l = L0 + L2 X^2, L0 = c0 + y Y (y in Fq), L2 = c1x (the prepared line c0 + (c1 x_P)
// v + y_P v w of pairing.hpp in this basis):
//   c0' = a0 L0 + Y a1 L2,  c1' = a1 L0 + Y a2 L2,  c2' = a2 L0 + a0 L2.
__device__ __forceinline__ fq4 line3(const fq4& a, const fq2& c0, const fq2& c1x, const fq& y, const grp3 g) {
  const fq4 T = fq4{fq2_add(fq2_mul(a.c0, c0), fq2_mul_xi(fq2_mul_fq(a.c1, y))),
                    fq2_add(fq2_mul_fq(a.c0, y), fq2_mul(a.c1, c0))};
  const fq4 Q = fq4{fq2_mul(a.c0, c1x), fq2_mul(a.c1, c1x)};
  const fq4 Qn = fq4_shfl(Q, g.nxt());
  return fq4_add(T, fq4_sel(g.gl == 2, Qn, fq4_mul_y(Qn)));
}

// Granger-Scott squaring in the cyclotomic subgroup:
//   a0' = 3 a0^2 - 2 conj(a0),  a1' = 3 Y a2^2 + 2 conj(a1),  a2' = 3 a1^2 - 2 conj(a2).
__device__ __forceinline__ fq4 cyc_sqr3(const fq4& a, const grp3 g) {
  const fq4 S = fq4_square(a);
  const fq4 Sf = fq4_shfl(S, g.gl == 0 ? g.base : g.gl == 1 ? g.base + 2 : g.base + 1);
  const fq4 U = fq4_sel(g.gl == 1, fq4_mul_y(Sf), Sf);
  const fq4 U3 = fq4_add(fq4_dbl(U), U);
  const fq4 C2 = fq4_dbl(fq4_conj(a));
  return fq4_sel(g.gl == 1, fq4_add(U3, C2), fq4_sub(U3, C2));
}

// General product: c_m = a_m b_0 + [Y if m <= 1] a_{m+1} b_2 + [Y if m == 0] a_{m+2} b_1.
__device__ __noinline__ fq4 mul3(const fq4& a, const fq4& b, const grp3 g) {
  const fq4 a1 = fq4_shfl(a, g.nxt());
  const fq4 a2 = fq4_shfl(a, g.prv());
  const fq4 b0 = fq4_shfl(b, g.base);
  const fq4 b1 = fq4_shfl(b, g.base + 1);
  const fq4 b2 = fq4_shfl(b, g.base + 2);
  const fq4 t0 = fq4_mul(a, b0);
  fq4 t1 = fq4_mul(a1, b2);
  fq4 t2 = fq4_mul(a2, b1);
  t1 = fq4_sel(g.gl <= 1, fq4_mul_y(t1), t1);
  t2 = fq4_sel(g.gl == 0, fq4_mul_y(t2), t2);
  return fq4_add(fq4_add(t0, t1), t2);
}

// f^p: g_i -> conj(g_i) gamma_1,i (field.hpp fq12_frobenius); lane k holds g_k, g_{k+3}.
__device__ __forceinline__ fq4 frob3(const fq4& a, const grp3 g) {
  const uint32_t* k00 = g.gl == 0 ? FROB1_C0_0 : g.gl == 1 ? FROB1_C1_0 : FROB1_C2_0;
  const uint32_t* k01 = g.gl == 0 ? FROB1_C0_1 : g.gl == 1 ? FROB1_C1_1 : FROB1_C2_1;
  const uint32_t* k10 = g.gl == 0 ? FROB1_C3_0 : g.gl == 1 ? FROB1_C4_0 : FROB1_C5_0;
  const uint32_t* k11 = g.gl == 0 ? FROB1_C3_1 : g.gl == 1 ? FROB1_C4_1 : FROB1_C5_1;
  return fq4{fq2_mul(fq2_conj(a.c0), fq2{fq_from_const(k00), fq_from_const(k01)}),
             fq2_mul(fq2_conj(a.c1), fq2{fq_from_const(k10), fq_from_const(k11)})};
}
// f^(p^2): g_i -> g_i gamma_2,i (gamma_2,i in Fq)
__device__ __forceinline__ fq4 frob2_3(const fq4& a, const grp3 g) {
  const uint32_t* k0 = g.gl == 0 ? FROB2_C0 : g.gl == 1 ? FROB2_C1 : FROB2_C2;
  const uint32_t* k1 = g.gl == 0 ? FROB2_C3 : g.gl == 1 ? FROB2_C4 : FROB2_C5;
  return fq4{fq2_mul_fq(a.c0, fq_from_const(k0)), fq2_mul_fq(a.c1, fq_from_const(k1))};
}

// (x0 + x1 Y)^-1 = (x0 - x1 Y) / (x0^2 - xi x1^2)
__device__ __noinline__ fq4 fq4_inv(const fq4& a) {
  const fq2 d = fq2_sub(fq2_sqr(a.c0), fq2_mul_xi(fq2_sqr(a.c1)));
  const fq2 di = fq2_inv(d);
  return fq4{fq2_mul(a.c0, di), fq2_neg(fq2_mul(a.c1, di))};
}

// Inverse in the cubic extension: B = (a0^2 - Y a1 a2, Y a2^2 - a0 a1, a1^2 - a0 a2),
// N = a0 B0 + Y (a2 B1 + a1 B2) in Fq4, A^-1 = B / N.
__device__ __noinline__ fq4 inv3(const fq4& a, const grp3 g) {
  const fq4 an1 = fq4_shfl(a, g.nxt());  // a_{m+1}
  const fq4 an2 = fq4_shfl(a, g.prv());  // a_{m+2}
  const fq4 X = g.gl == 0 ? a : g.gl == 1 ? an1 : an2;
  const fq4 Yv = g.gl == 1 ? an2 : an1;
  const fq4 Zv = g.gl == 0 ? an2 : a;
  const fq4 X2 = fq4_square(X);
  const fq4 YZ = fq4_mul(Yv, Zv);
  const fq4 B = fq4_sub(fq4_sel(g.gl == 1, fq4_mul_y(X2), X2), fq4_sel(g.gl == 0, fq4_mul_y(YZ), YZ));
  const fq4 m = fq4_mul(g.gl == 0 ? a : g.gl == 1 ? an1 : an2, B);
  const fq4 term = fq4_sel(g.gl == 0, m, fq4_mul_y(m));
  const fq4 N = fq4_add(fq4_add(term, fq4_shfl(term, g.nxt())), fq4_shfl(term, g.prv()));
  return fq4_mul(B, fq4_inv(N));
}

// f == 1: lane 0 holds (1, 0), lanes 1, 2 hold 0 -- decided for the whole group.
__device__ __forceinline__ bool is_one3(const fq4& a, const grp3 g) {
  const bool mine = g.gl == 0 ? (fq2_eq(a.c0, fq2_one()) && fq2_is_zero(a.c1))
                              : (fq2_is_zero(a.c0) && fq2_is_zero(a.c1));
  const uint64_t bal = __ballot(mine);
  const uint64_t gm = (g.base == 63 ? 1ull : 7ull) << g.base;
  return (bal & gm) == gm;
}

// Two Miller loops over prepared lines (pairing.hpp miller_loop2), conjugated for x < 0.
// UNIFORM: the line arrays are the same for every group of the wave (scalar loads); otherwise
// each group reads its own lines (vector loads).
template <bool UNIFORM = true>
__device__ fq4 miller3(const line_pre* LA, const g1a& PA, bool useA, const line_pre* LB, const g1a& PB, bool useB,
                       const grp3 g) {
  fq4 f = g.gl == 0 ? fq4_one() : fq4_zero();
  int k = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (i != 62) f = sqr3(f, g);
    const int steps = ((BLS_X >> i) & 1) ? 4 : 2;
#pragma unroll 1
    for (int s = 0; s < steps; s++) {
      const bool b = (s & 1) != 0;
      const line_pre* lp = (b ? LB : LA) + k;
      const line_pre L = UNIFORM ? ld_uniform(lp) : *lp;
      if (b ? useB : useA) {
        const fq px = b ? PB.x : PA.x;
        const fq py = b ? PB.y : PA.y;
        f = line3(f, L.c0, fq2_mul_fq(L.c1, px), py, g);
      }
      if (b) k++;
    }
  }
  return conj3(f, g);
}

// g^|x| in the cyclotomic subgroup: runs of squarings between the one bits of |x| (63, 62, 60,
// 57, 48, 16), as pairing.hpp cyc_exp_abs_x_lds.
__device__ __noinline__ fq4 cyc_exp_abs_x3(const fq4& gin, const grp3 g) {
  static_assert(BLS_X == 0xd201000000010000ull, "square-and-multiply runs are specific to |x|");
  const int runs[6] = {1, 2, 3, 9, 32, 16};
  fq4 r = gin;
#pragma unroll 1
  for (int q = 0; q < 6; q++) {
#pragma unroll 1
    for (int i = 0; i < runs[q]; i++) r = cyc_sqr3(r, g);
    if (q < 5) r = mul3(r, gin, g);
  }
  return r;
}
__device__ __forceinline__ fq4 cyc_exp_x3(const fq4& a, const grp3 g) { return conj3(cyc_exp_abs_x3(a, g), g); }

// f^(3 (p^12 - 1)/r) (pairing.hpp final_exponentiation, same chain)
__device__ __noinline__ fq4 final_exp3(const fq4& f, const grp3 g) {
  fq4 t = mul3(conj3(f, g), inv3(f, g), g);
  t = mul3(frob2_3(t, g), t, g);
  fq4 a = mul3(cyc_exp_x3(t, g), conj3(t, g), g);
  a = mul3(cyc_exp_x3(a, g), conj3(a, g), g);
  const fq4 b = mul3(cyc_exp_x3(a, g), frob3(a, g), g);
  fq4 c = mul3(cyc_exp_x3(cyc_exp_x3(b, g), g), frob2_3(b, g), g);
  c = mul3(c, conj3(b, g), g);
  const fq4 t3 = mul3(cyc_sqr3(t, g), t, g);
  return mul3(c, t3, g);
}

// e(PA, QA) e(PB, QB) == 1 with identity handling (check2 of hbx_kernels.hip); group-uniform.
template <bool UNIFORM = true>
__device__ __forceinline__ bool check2_g3(const line_pre* LA, const g1a& PA, bool qa_inf, const line_pre* LB,
                                          const g1a& PB, bool qb_inf, const grp3 g) {
  const bool skipA = PA.inf || qa_inf;
  const bool skipB = PB.inf || qb_inf;
  if (skipA && skipB) return true;
  const fq4 f = miller3<UNIFORM>(LA, PA, !skipA, LB, PB, !skipB, g);
  return is_one3(final_exp3(f, g), g);
}

#endif  // __HIPCC__
}  // namespace hbx
