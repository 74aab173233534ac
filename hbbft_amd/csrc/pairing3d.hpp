// The three-lane cooperative share check (pairing3.hpp) in the signed-digit tower (fieldd.hpp).
//
// Same representation and the same formulas as pairing3.hpp -- Fq12 = Fq4[X]/(X^3 - Y), lane k
// of a 3-lane group holding a_k = g_k + g_{k+3} Y -- with Fq2 products as fieldd.hpp's fused
// column loops and carry-free additions; Fq4 products return carry-normalised sums (fq4d level),
// the Fq12-level operations (sqr3, line3, cyc_sqr3, mul3) return reduced values.  The inversion
// and the final "== 1" test go through pairing3.hpp's 12-limb versions.  Same bits as
// check2_g3 (and as two pairing 0.14 pairings compared).
#pragma once
#include "pairing3.hpp"
#include "pairingd.hpp"

namespace hbx {
#if defined(__HIPCC__)

struct fq4d {
  fq2d c0, c1;  // c0 + c1 Y,  Y^2 = xi
};

__device__ __forceinline__ fq4d fq4d_add(const fq4d& a, const fq4d& b) { return fq4d{fq2d_add(a.c0, b.c0), fq2d_add(a.c1, b.c1)}; }
__device__ __forceinline__ fq4d fq4d_sub(const fq4d& a, const fq4d& b) { return fq4d{fq2d_sub(a.c0, b.c0), fq2d_sub(a.c1, b.c1)}; }
__device__ __forceinline__ fq4d fq4d_dbl(const fq4d& a) { return fq4d{fq2d_dbl(a.c0), fq2d_dbl(a.c1)}; }
__device__ __forceinline__ fq4d fq4d_conj(const fq4d& a) { return fq4d{a.c0, fq2d_neg(a.c1)}; }
__device__ __forceinline__ fq4d fq4d_norm(const fq4d& a) { return fq4d{fq2d_norm(a.c0), fq2d_norm(a.c1)}; }
__device__ __forceinline__ fq4d fq4d_reduce(const fq4d& a) { return fq4d{fq2d_reduce(a.c0), fq2d_reduce(a.c1)}; }
__device__ __forceinline__ fq4d fq4d_mul_y(const fq4d& a) { return fq4d{fq2d_mul_xi(a.c1), a.c0}; }
__device__ __forceinline__ fq4d fq4d_sel(bool c, const fq4d& a, const fq4d& b) {
  fq4d r;
  const int32_t* pa = reinterpret_cast<const int32_t*>(&a);
  const int32_t* pb = reinterpret_cast<const int32_t*>(&b);
  int32_t* pr = reinterpret_cast<int32_t*>(&r);
#pragma unroll
  for (int i = 0; i < 56; i++) pr[i] = c ? pa[i] : pb[i];
  return r;
}
__device__ __forceinline__ fq4d fq4d_shfl(const fq4d& v, int src) {
  fq4d r;
  const int32_t* pv = reinterpret_cast<const int32_t*>(&v);
  int32_t* pr = reinterpret_cast<int32_t*>(&r);
#pragma unroll
  for (int i = 0; i < 56; i++) pr[i] = __shfl(pv[i], src & 63, 64);
  return r;
}
// Karatsuba over Fq2 (3 fused Fq2 products), carry-normalised output
__device__ __forceinline__ fq4d fq4d_mul(const fq4d& a, const fq4d& b) {
  const fq2d t0 = fq2d_mul(a.c0, b.c0);
  const fq2d t1 = fq2d_mul(a.c1, b.c1);
  const fq2d s = fq2d_mul(fq2d_add(a.c0, a.c1), fq2d_add(b.c0, b.c1));
  return fq4d_norm(fq4d{fq2d_add(t0, fq2d_mul_xi(t1)), fq2d_sub(fq2d_sub(s, t0), t1)});
}
// (a0 + a1 Y)^2 by three Fq2 squarings (fq4d_sqr of fieldd.hpp), carry-normalised output
__device__ __forceinline__ fq4d fq4d_square(const fq4d& a) {
  fq4d r;
  fq4d_sqr(a.c0, a.c1, r.c0, r.c1);
  return r;
}
__device__ __forceinline__ fq4d fq4d_one() {
  const fqd z = fqd_zero();
  return fq4d{fq2d{fqd_const(FQD_ONE), z}, fq2d{z, z}};
}
__device__ __forceinline__ fq4d fq4d_zero() {
  const fqd z = fqd_zero();
  return fq4d{fq2d{z, z}, fq2d{z, z}};
}
__device__ __forceinline__ fq4 fq4d_to_fq4(const fq4d& a) { return fq4{fq2d_to_fq2(a.c0), fq2d_to_fq2(a.c1)}; }
__device__ __forceinline__ fq4d fq4d_from_fq4(const fq4& a) { return fq4d{fq2d_from_fq2(a.c0), fq2d_from_fq2(a.c1)}; }

__device__ __forceinline__ fq4d conj3d(const fq4d& a, const grp3& g) {
  return g.gl == 1 ? fq4d{fq2d_neg(a.c0), a.c1} : fq4d{a.c0, fq2d_neg(a.c1)};
}

// pairing3.hpp sqr3
__device__ __forceinline__ fq4d sqr3d(const fq4d& a, const grp3 g) {
  const fq4d an = fq4d_shfl(a, g.nxt());
  const fq4d S = fq4d_square(a);
  const fq4d P = fq4d_mul(a, an);
  const fq4d Pf = fq4d_shfl(P, g.gl == 0 ? g.nxt() : g.gl == 1 ? g.prv() : g.base + 2);
  const fq4d Sf = fq4d_shfl(S, g.gl == 0 ? g.base : g.gl == 1 ? g.nxt() : g.prv());
  const fq4d U = fq4d_sel(g.gl == 1, fq4d_mul_y(Sf), Sf);
  const fq4d V = fq4d_sel(g.gl == 0, fq4d_mul_y(Pf), Pf);
  return fq4d_reduce(fq4d_add(U, fq4d_dbl(V)));
}
// pairing3.hpp line3: f *= L0 + L2 X^2, L0 = c0 + y Y, L2 = c1x
__device__ __forceinline__ fq4d line3d(const fq4d& a, const fq2d& c0, const fq2d& c1x, const fqd& y, const grp3 g) {
  const fq4d T = fq4d{fq2d_add(fq2d_mul(a.c0, c0), fq2d_mul_xi(fq2d_mul_fq(a.c1, y))),
                      fq2d_add(fq2d_mul_fq(a.c0, y), fq2d_mul(a.c1, c0))};
  const fq4d Q = fq4d{fq2d_mul(a.c0, c1x), fq2d_mul(a.c1, c1x)};
  const fq4d Qn = fq4d_shfl(Q, g.nxt());
  return fq4d_reduce(fq4d_add(T, fq4d_sel(g.gl == 2, Qn, fq4d_mul_y(Qn))));
}
// pairing3.hpp cyc_sqr3 (Granger-Scott)
__device__ __forceinline__ fq4d cyc_sqr3d(const fq4d& a, const grp3 g) {
  const fq4d S = fq4d_square(a);
  const fq4d Sf = fq4d_shfl(S, g.gl == 0 ? g.base : g.gl == 1 ? g.base + 2 : g.base + 1);
  const fq4d U = fq4d_norm(fq4d_sel(g.gl == 1, fq4d_mul_y(Sf), Sf));
  const fq4d U3 = fq4d_add(fq4d_dbl(U), U);
  const fq4d C2 = fq4d_dbl(fq4d_conj(a));
  return fq4d_reduce(fq4d_sel(g.gl == 1, fq4d_add(U3, C2), fq4d_sub(U3, C2)));
}
// pairing3.hpp mul3
__device__ __noinline__ fq4d mul3d(const fq4d& a, const fq4d& b, const grp3 g) {
  const fq4d a1 = fq4d_shfl(a, g.nxt());
  const fq4d a2 = fq4d_shfl(a, g.prv());
  const fq4d b0 = fq4d_shfl(b, g.base);
  const fq4d b1 = fq4d_shfl(b, g.base + 1);
  const fq4d b2 = fq4d_shfl(b, g.base + 2);
  const fq4d t0 = fq4d_mul(a, b0);
  fq4d t1 = fq4d_mul(a1, b2);
  fq4d t2 = fq4d_mul(a2, b1);
  t1 = fq4d_sel(g.gl <= 1, fq4d_mul_y(t1), t1);
  t2 = fq4d_sel(g.gl == 0, fq4d_mul_y(t2), t2);
  return fq4d_reduce(fq4d_add(fq4d_add(t0, t1), t2));
}
// pairing3.hpp frob3 / frob2_3 with the digit-form constants
__device__ __forceinline__ fq4d frob3d(const fq4d& a, const grp3 g) {
  const int32_t* k00 = g.gl == 0 ? FROBD1_C0_0 : g.gl == 1 ? FROBD1_C1_0 : FROBD1_C2_0;
  const int32_t* k01 = g.gl == 0 ? FROBD1_C0_1 : g.gl == 1 ? FROBD1_C1_1 : FROBD1_C2_1;
  const int32_t* k10 = g.gl == 0 ? FROBD1_C3_0 : g.gl == 1 ? FROBD1_C4_0 : FROBD1_C5_0;
  const int32_t* k11 = g.gl == 0 ? FROBD1_C3_1 : g.gl == 1 ? FROBD1_C4_1 : FROBD1_C5_1;
  return fq4d{fq2d_mul(fq2d_conj(a.c0), fq2d_const(k00, k01)), fq2d_mul(fq2d_conj(a.c1), fq2d_const(k10, k11))};
}
__device__ __forceinline__ fq4d frob2_3d(const fq4d& a, const grp3 g) {
  const int32_t* k0 = g.gl == 0 ? FROBD2_C0 : g.gl == 1 ? FROBD2_C1 : FROBD2_C2;
  const int32_t* k1 = g.gl == 0 ? FROBD2_C3 : g.gl == 1 ? FROBD2_C4 : FROBD2_C5;
  return fq4d{fq2d_mul_fq(a.c0, fqd_const(k0)), fq2d_mul_fq(a.c1, fqd_const(k1))};
}
// inversion once per check, through pairing3.hpp's 12-limb inv3
__device__ __noinline__ fq4d inv3d(const fq4d& a, const grp3 g) { return fq4d_from_fq4(inv3(fq4d_to_fq4(a), g)); }

// pairing3.hpp miller3 over digit-form prepared lines (wave-uniform loads)
__device__ fq4d miller3d(const line_pre_d* LA, const fqd& ax, const fqd& ay, bool useA, const line_pre_d* LB,
                         const fqd& bx, const fqd& by, bool useB, const grp3 g) {
  fq4d f = g.gl == 0 ? fq4d_one() : fq4d_zero();
  int k = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (i != 62) f = sqr3d(f, g);
    const int steps = ((BLS_X >> i) & 1) ? 4 : 2;
#pragma unroll 1
    for (int s = 0; s < steps; s++) {
      const bool b = (s & 1) != 0;
      const line_pre_d L = ld_uniform((b ? LB : LA) + k);
      if (b ? useB : useA) f = line3d(f, L.c0, fq2d_mul_fq(L.c1, b ? bx : ax), b ? by : ay, g);
      if (b) k++;
    }
  }
  return conj3d(f, g);
}

__device__ __noinline__ fq4d cyc_exp_abs_x3d(const fq4d& gin, const grp3 g) {
  static_assert(BLS_X == 0xd201000000010000ull, "square-and-multiply runs are specific to |x|");
  fq4d r = gin;
#pragma unroll 1
  for (int q = 0; q < 6; q++) {
    const int run = q == 0 ? 1 : q == 1 ? 2 : q == 2 ? 3 : q == 3 ? 9 : q == 4 ? 32 : 16;
#pragma unroll 1
    for (int i = 0; i < run; i++) r = cyc_sqr3d(r, g);
    if (q < 5) r = mul3d(r, gin, g);
  }
  return r;
}
__device__ __forceinline__ fq4d cyc_exp_x3d(const fq4d& a, const grp3 g) { return conj3d(cyc_exp_abs_x3d(a, g), g); }

// pairing3.hpp final_exp3
__device__ __noinline__ fq4d final_exp3d(const fq4d& f, const grp3 g) {
  fq4d t = mul3d(conj3d(f, g), inv3d(f, g), g);
  t = mul3d(frob2_3d(t, g), t, g);
  fq4d a = mul3d(cyc_exp_x3d(t, g), conj3d(t, g), g);
  a = mul3d(cyc_exp_x3d(a, g), conj3d(a, g), g);
  const fq4d b = mul3d(cyc_exp_x3d(a, g), frob3d(a, g), g);
  fq4d c = mul3d(cyc_exp_abs_x3d(cyc_exp_abs_x3d(b, g), g), frob2_3d(b, g), g);
  c = mul3d(c, conj3d(b, g), g);
  const fq4d t3 = mul3d(cyc_sqr3d(t, g), t, g);
  return mul3d(c, t3, g);
}

// check2_g3 in the digit tower; group-uniform.
__device__ __forceinline__ bool check2_g3d(const line_pre_d* LA, const g1a& PA, bool qa_inf, const line_pre_d* LB,
                                           const g1a& PB, bool qb_inf, const grp3 g) {
  const bool skipA = PA.inf || qa_inf;
  const bool skipB = PB.inf || qb_inf;
  if (skipA && skipB) return true;
  const fq4d f = miller3d(LA, fqd_from_fq(PA.x), fqd_from_fq(PA.y), !skipA, LB, fqd_from_fq(PB.x),
                          fqd_from_fq(PB.y), !skipB, g);
  return is_one3(fq4d_to_fq4(final_exp3d(f, g)), g);
}

// ---- six lanes per check: the two Miller loops side by side ------------------------------------
// A 6-lane group is two 3-lane groups: triplet 0 (lanes 0..2) runs the Miller loop of pair A,
// triplet 1 (lanes 3..5) the loop of pair B, in ONE instruction stream -- each step multiplies by
// one line per lane, the lane's own pair's (both lines are loaded wave-uniform and selected per
// lane), so a step costs a squaring and one line instead of a squaring and two.  Then each triplet
// fetches the other's value (3 lanes away) and both hold f_A f_B; the final exponentiation runs
// on both (the same instructions; triplet 0's result is used).  ~1/3 of the Miller loop's line
// products per lane fewer than check2_g3d, on twice the lanes: for launches that leave SIMDs idle
// at three lanes per check.  Same bits as check2_g3d.
constexpr int G6_PER_WAVE = 10;  // lanes 60..63 idle
__device__ __forceinline__ line_pre_d line_d_sel(bool c, const line_pre_d& a, const line_pre_d& b) {
  line_pre_d r;
  const int32_t* pa = reinterpret_cast<const int32_t*>(&a);
  const int32_t* pb = reinterpret_cast<const int32_t*>(&b);
  int32_t* pr = reinterpret_cast<int32_t*>(&r);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(line_pre_d) / 4); i++) pr[i] = c ? pa[i] : pb[i];
  return r;
}
__device__ fq4d miller3d_split(const line_pre_d* LA, const line_pre_d* LB, const fqd& px, const fqd& py, bool use,
                               bool second, const grp3 g) {
  fq4d f = g.gl == 0 ? fq4d_one() : fq4d_zero();
  int k = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (i != 62) f = sqr3d(f, g);
    const int steps = ((BLS_X >> i) & 1) ? 2 : 1;
#pragma unroll 1
    for (int s = 0; s < steps; s++) {
      const line_pre_d L = line_d_sel(second, ld_uniform(LB + k), ld_uniform(LA + k));
      if (use) f = line3d(f, L.c0, fq2d_mul_fq(L.c1, px), py, g);
      k++;
    }
  }
  f = conj3d(f, g);
  const int lane = (int)(threadIdx.x & 63);
  return mul3d(f, fq4d_shfl(f, second ? lane - 3 : lane + 3), g);
}
// check2_g3d on a 6-lane group: triplet `second` brings pair B (PB, LB), the other pair A.  The
// skip flags are group-uniform (both triplets evaluate the same four values).
__device__ __forceinline__ bool check2_g6d(const line_pre_d* LA, const g1a& PA, bool qa_inf, const line_pre_d* LB,
                                           const g1a& PB, bool qb_inf, bool second, const grp3 g) {
  const bool skipA = PA.inf || qa_inf;
  const bool skipB = PB.inf || qb_inf;
  if (skipA && skipB) return true;
  const g1a& P = second ? PB : PA;
  const fq4d f = miller3d_split(LA, LB, fqd_from_fq(P.x), fqd_from_fq(P.y), second ? !skipB : !skipA, second, g);
  return is_one3(fq4d_to_fq4(final_exp3d(f, g)), g);
}

#endif  // __HIPCC__
}  // namespace hbx
