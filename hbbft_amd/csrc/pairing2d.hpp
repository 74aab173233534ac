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
//     lane k computes A_k (c0' + c1' v) (5 Fq2 products) + v^(2-k) A_(1-k) -- 10 Fq2 products a
//     line instead of the one-lane sparse product's 10 plus 3 Fq-by-Fq2 products for the y term;
//   * general product (final exponentiation): lane k computes its own output half as two Fq6
//     products, X_k Y_0 + [v] X_(1-k) Y_1;
//   * cyclotomic squaring (Granger-Scott): each lane produces its own three Fq2 coefficients, each
//     from ONE fused column loop of four digit convolutions and two reductions (lane 0:
//     a^2 + xi b^2, lane 1: 2 a b; operands selected per lane), the one-lane squaring's 9 Fq2
//     squarings split evenly;
//   * Frobenius maps and conjugation are coefficient-wise.
// Register budget: every Fq6 product streams one operand from LDS (the per-lane region of the
// block, 156 dwords = one wave per SIMD), one Fq2 coefficient at a time behind a scheduling fence,
// so a product holds its register operand, three accumulators and one Fq2 product's temporaries
// (~300 registers: nothing spills).  The Miller loop uses the region unpacked as scratch; the final
// exponentiation as two packed slots (FE2_PROG).
// The per-check scalars: lane 0 holds 1/y of both G1 points, lane 1 x/y (one Fq inversion each).
// Control flow is pair-uniform; every exchange reads the partner lane of the same pair.
#pragma once
#include "pairingd.hpp"
#include "fe1d.hpp"
#include "dpp.hpp"

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
  dpp_guard_pairs();
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
// (selects, not a branch: a conditional on an aggregate compiles to divergent control flow with
// both values live, which made the allocator spill)
__device__ __forceinline__ fq6d conj2d(const fq6d& a, bool l1) { return sel_t(l1, fq6d_neg(a), a); }

// ---- the per-lane LDS region: 156 dwords, word k of lane L at k * 64 + L -------------------
constexpr int LDS2_DWORDS = 156;
typedef lds_u32* lds2;  // this lane's word 0

__device__ __forceinline__ void lds_put_fq2d_raw(lds2 base, int word, const fq2d& a) {
  const int32_t* p = reinterpret_cast<const int32_t*>(&a);
#pragma unroll
  for (int i = 0; i < 28; i++) base[(word + i) * 64] = (uint32_t)p[i];
}
__device__ __forceinline__ fq2d lds_get_fq2d_raw(const lds_u32* base, int word) {
  fq2d a;
  int32_t* p = reinterpret_cast<int32_t*>(&a);
#pragma unroll
  for (int i = 0; i < 28; i++) p[i] = (int32_t)base[(word + i) * 64];
  return a;
}
// packed: a reduced Fq as 13 dwords (digits 0..12 as 28-bit fields, digit 13 whole), pairingd.hpp
__device__ __forceinline__ void lds_put_fqd_packed(lds2 base, int word, const fqd& e) {
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
#pragma unroll
  for (int k = 0; k < 13; k++) base[(word + k) * 64] = w[k];
}
__device__ __forceinline__ fqd lds_get_fqd_packed(const lds_u32* base, int word) {
  uint32_t w[13];
#pragma unroll
  for (int k = 0; k < 13; k++) w[k] = base[(word + k) * 64];
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
constexpr int LDS_FQ6D_PACKED = 78;  // one packed Fq6 half
__device__ __forceinline__ void lds_put_fq6d_packed(lds2 base, int word, const fq6d& a) {
  const fqd* e = &a.c0.c0;
#pragma unroll
  for (int q = 0; q < 6; q++) lds_put_fqd_packed(base, word + 13 * q, e[q]);
}
__device__ __forceinline__ fq2d lds_get_fq2d_packed(const lds_u32* base, int word, int q) {
  return fq2d{lds_get_fqd_packed(base, word + 26 * q), lds_get_fqd_packed(base, word + 26 * q + 13)};
}
__device__ __forceinline__ fq6d lds_get_fq6d_packed(const lds_u32* base, int word) {
  return fq6d{lds_get_fq2d_packed(base, word, 0), lds_get_fq2d_packed(base, word, 1), lds_get_fq2d_packed(base, word, 2)};
}

// ---- Fq6 products with the second operand streamed: y(q) returns its Fq2 coefficient q --------
// Karatsuba (fieldd.hpp fq6d_mul) with each product folded into the output accumulators at once
// (c0 = t0 + xi (u0 - t1 - t2), c1 = u1 - t0 - t1 + xi t2, c2 = u2 - t0 - t2 + t1); inputs
// normalised (y's coefficients: sums are formed here); carry-normalised output added to `acc`.
template <class Y>
__device__ __forceinline__ void fq6d_mul_acc(fq6d& acc, const fq6d& a, Y y) {
  {
    const fq2d t0 = fq2d_mul(a.c0, y(0));
    acc.c0 = fq2d_add(acc.c0, t0);
    acc.c1 = fq2d_sub(acc.c1, t0);
    acc.c2 = fq2d_sub(acc.c2, t0);
  }
  HBX_SEQ();
  {
    const fq2d t1 = fq2d_mul(a.c1, y(1));
    acc.c0 = fq2d_sub(acc.c0, fq2d_mul_xi(t1));
    acc.c1 = fq2d_sub(acc.c1, t1);
    acc.c2 = fq2d_add(acc.c2, t1);
  }
  HBX_SEQ();
  {
    const fq2d t2 = fq2d_mul(a.c2, y(2));
    acc.c0 = fq2d_sub(acc.c0, fq2d_mul_xi(t2));
    acc.c1 = fq2d_add(acc.c1, fq2d_mul_xi(t2));
    acc.c2 = fq2d_sub(acc.c2, t2);
  }
  HBX_SEQ();
  acc.c0 = fq2d_add(acc.c0, fq2d_mul_xi(fq2d_mul(fq2d_add(a.c1, a.c2), fq2d_add(y(1), y(2)))));
  HBX_SEQ();
  acc.c1 = fq2d_add(acc.c1, fq2d_mul(fq2d_add(a.c0, a.c1), fq2d_add(y(0), y(1))));
  HBX_SEQ();
  acc.c2 = fq2d_add(acc.c2, fq2d_mul(fq2d_add(a.c0, a.c2), fq2d_add(y(0), y(2))));
  HBX_SEQ();
  acc = fq6d_norm(acc);
}

// ---- Miller loop -------------------------------------------------------------------------
// LDS scratch words of the Miller loop: Y of the squaring (unpacked, 84), the scaled line (56)
constexpr int ML_Y = 0, ML_C0 = 84, ML_C1 = 112;

// (A0 + A1 w)^2 = (t - ab - v ab) + 2 ab w, ab = A0 A1, t = (A0 + A1)(A0 + v A1).  Reduced output.
// Y2REG: Y's third coefficient stays in registers (words ML_Y .. ML_Y + 55 only).
template <bool Y2REG = false>
__device__ __forceinline__ fq6d sqr2d(const fq6d& A, bool l1, lds2 lds) {
  fq6d X;
  fq2d y2;
  {
    const fq6d B = xchg_t(A);
    X = sel_t(l1, fq6d_norm(fq6d_add(A, B)), A);
    const fq6d Y = sel_t(l1, fq6d_norm(fq6d_add(B, fq6d_mul_v(A))), B);
    lds_put_fq2d_raw(lds, ML_Y, Y.c0);
    lds_put_fq2d_raw(lds, ML_Y + 28, Y.c1);
    if (Y2REG) y2 = Y.c2;
    else lds_put_fq2d_raw(lds, ML_Y + 56, Y.c2);
  }
  HBX_SEQ();
  fq6d P = fq6d_zero();  // lane 0: ab, lane 1: t
  fq6d_mul_acc(P, X, [&](int q) { return Y2REG && q == 2 ? y2 : lds_get_fq2d_raw(lds, ML_Y + 28 * q); });
  const fq6d Q = xchg_t(P);
  const fq6d r0 = fq6d_sub(fq6d_sub(Q, P), fq6d_mul_v(P));
  const fq6d r1 = fq6d_add(Q, Q);
  return fq6d_reduce(sel_t(l1, r1, r0));
}

// f * ((c0s + c1s v) + v w) with the scaled line in LDS: lane 0 A0 L0 + v^2 A1, lane 1
// A1 L0 + v A0.  A0 L0 by fieldd.hpp fq6d_mul_by_01's Karatsuba (5 Fq2 products).  Reduced output.
__device__ __forceinline__ fq6d line2d(const fq6d& A, bool l1, lds2 lds) {
  fq2d c0, c1, c2;
  {
    const fq2d t0 = fq2d_mul(A.c0, lds_get_fq2d_raw(lds, ML_C0));
    c0 = t0;
    c1 = fq2d_neg(t0);
  }
  HBX_SEQ();
  {
    const fq2d t1 = fq2d_mul(A.c1, lds_get_fq2d_raw(lds, ML_C1));
    c1 = fq2d_sub(c1, t1);
    c2 = t1;
  }
  HBX_SEQ();
  c0 = fq2d_add(c0, fq2d_mul_xi(fq2d_mul(A.c2, lds_get_fq2d_raw(lds, ML_C1))));
  HBX_SEQ();
  c1 = fq2d_add(c1, fq2d_mul(fq2d_add(A.c0, A.c1), fq2d_add(lds_get_fq2d_raw(lds, ML_C0), lds_get_fq2d_raw(lds, ML_C1))));
  HBX_SEQ();
  c2 = fq2d_add(c2, fq2d_mul(A.c2, lds_get_fq2d_raw(lds, ML_C0)));
  HBX_SEQ();
  const fq6d T = fq6d_norm(fq6d{c0, c1, c2});
  const fq6d vB = fq6d_mul_v(xchg_t(A));
  return fq6d_reduce(fq6d_add(T, sel_t(l1, vB, fq6d_mul_v(vB))));
}

// The scaled line's (c0 / y, c1 x / y) into LDS: lane 0 holds s = 1/y, lane 1 s = x/y.
__device__ __forceinline__ void line_eval2d(const line_pre_d& L, const fqd& s, bool l1, lds2 lds) {
  const fq2d mine = fq2d_mul_fq(sel_t(l1, L.c1, L.c0), s);
  const fq2d other = xchg_t(mine);
  lds_put_fq2d_raw(lds, ML_C0, sel_t(l1, other, mine));
  lds_put_fq2d_raw(lds, ML_C1, sel_t(l1, mine, other));
}

// Two Miller loops over prepared lines (pairingd.hpp miller_loop2_d), conjugated for x < 0.
__device__ __forceinline__ fq6d miller2d(const line_pre_d* LA, const fqd& sA, bool useA, const line_pre_d* LB,
                                         const fqd& sB, bool useB, bool l1, lds2 lds) {
  fq6d f = sel_t(l1, fq6d_zero(), fq6d_one());
  int k = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (i != 62) f = sqr2d(f, l1, lds);
    const int steps = ((BLS_X >> i) & 1) ? 4 : 2;  // (A, B) lines of the doubling [+ addition]
#pragma unroll 1
    for (int s = 0; s < steps; s++) {
      const bool b = (s & 1) != 0;
      if (b ? useB : useA) {
        line_eval2d(ld_uniform((b ? LB : LA) + k), b ? sB : sA, l1, lds);
        HBX_SEQ();
        f = line2d(f, l1, lds);
      }
      if (b) k++;
    }
  }
  return conj2d(f, l1);
}

// ---- final exponentiation --------------------------------------------------------------------
// Granger-Scott halves: lane 0 a^2 + xi b^2, lane 1 2 a b, as ONE column loop of four digit
// convolutions re = C1 + C2 - C3, im = C4 + C2 + C3 with
//   lane 0: C1 = (a0 + a1)(a0 - a1), C2 = (b0 + b1)(b0 - b1), C3 = (2 b0) b1,      C4 = (2 a0) a1;
//   lane 1: C1 = (2 a0) b0,          C2 = (a0 - a1) b1,        C3 = (a0 + a1) b1, C4 = (2 a1) b0
// (lane 1: re = 2 a0 b0 - 2 a1 b1, im = 2 a1 b0 + 2 a0 b1).  Inputs reduced (digits 0..12 in
// [0, 2^28)): every operand digit is below 2^29 in magnitude, a column of one convolution below
// 14 x 2^57, re / im below 2^62.4.  Normalised output.
__device__ __forceinline__ fq2d cyc_pair2d(const fq2d& a, const fq2d& b, bool l1) {
  HBX_COUNT_FQMUL(); HBX_COUNT_FQMUL(); HBX_COUNT_FQMUL(); HBX_COUNT_FQMUL();
  int32_t p1[14], q1[14], p2[14], q2[14], p3[14], p4[14], q4[14], q3[14];
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
    q3[i] = b1;
  }
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
  HBX_SEQ();
  const fq2d T1 = cyc_pair2d(B.c0, sel_t(l1, A.c1, A.c2), l1);
  HBX_SEQ();
  const fq2d T2 = cyc_pair2d(sel_t(l1, A.c0, A.c1), B.c2, l1);
  T0 = sel_t(l1, fq2d_mul_xi(T0), T0);
  const fq6d T{T0, T1, T2};
  const fq6d T3 = fq6d_add(fq6d_add(T, T), T);
  const fq6d A2 = fq6d_add(A, A);
  return fq6d_reduce(sel_t(l1, fq6d_add(T3, A2), fq6d_sub(T3, A2)));
}

// ---- Final exponentiation over slots --------------------------------------------------------
// The working value r lives in LDS slot B between operations, beside slot A (the current
// exponentiation base or operand); the long-lived t^3 / d sit in a third slot G in global memory
// (written twice and read twice per check).  Every operation reads its operands from slots and
// writes its result to a slot, so no large value stays in registers from one operation to the
// next: each operation is register-allocated on its own (a loop carrying r in registers across
// its alternative operations spilled the product's operands).  A slot holds this lane's half
// packed (78 dwords); the pair's halves are at lanes 2m (half 0) and 2m + 1 (half 1).
// Slot addressing: word k of half h at half_base(h)[k * stride].
template <class P>
struct slot2 {
  P h0;             // half 0 of this pair (the lane-0 column)
  uint32_t stride;  // dword distance between consecutive words
  __device__ __forceinline__ P half(int h) const { return h0 + h; }
};
template <class P>
__device__ __forceinline__ fqd slot_get_fqd(P base, uint32_t stride, int word) {
  uint32_t w[13];
#pragma unroll
  for (int k = 0; k < 13; k++) w[k] = base[(word + k) * stride];
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
template <class P>
__device__ __forceinline__ void slot_put_fqd(P base, uint32_t stride, int word, const fqd& e) {
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
#pragma unroll
  for (int k = 0; k < 13; k++) base[(word + k) * stride] = w[k];
}
template <class P>
__device__ __forceinline__ fq2d slot_get_fq2d(P base, uint32_t stride, int q) {
  return fq2d{slot_get_fqd(base, stride, 26 * q), slot_get_fqd(base, stride, 26 * q + 13)};
}
template <class P>
__device__ __forceinline__ void slot_put_fq2d(P base, uint32_t stride, int q, const fq2d& a) {
  slot_put_fqd(base, stride, 26 * q, a.c0);
  slot_put_fqd(base, stride, 26 * q + 13, a.c1);
}
template <class P>
__device__ __forceinline__ fq6d slot_get_fq6d(P base, uint32_t stride) {
  return fq6d{slot_get_fq2d(base, stride, 0), slot_get_fq2d(base, stride, 1), slot_get_fq2d(base, stride, 2)};
}
template <class P>
__device__ __forceinline__ void slot_put_fq6d(P base, uint32_t stride, const fq6d& a) {
  slot_put_fq2d(base, stride, 0, a.c0);
  slot_put_fq2d(base, stride, 1, a.c1);
  slot_put_fq2d(base, stride, 2, a.c2);
}

// Fq6 product with BOTH operands streamed (x(q), y(q): Fq2 coefficient q), Karatsuba as
// fq6d_mul_acc; inputs normalised (or negated normalised); carry-normalised sum added to acc.
template <class X, class Y>
__device__ __forceinline__ void fq6d_mul_acc2(fq6d& acc, X x, Y y) {
  {
    const fq2d t0 = fq2d_mul(x(0), y(0));
    acc.c0 = fq2d_add(acc.c0, t0);
    acc.c1 = fq2d_sub(acc.c1, t0);
    acc.c2 = fq2d_sub(acc.c2, t0);
  }
  HBX_SEQ();
  {
    const fq2d t1 = fq2d_mul(x(1), y(1));
    acc.c0 = fq2d_sub(acc.c0, fq2d_mul_xi(t1));
    acc.c1 = fq2d_sub(acc.c1, t1);
    acc.c2 = fq2d_add(acc.c2, t1);
  }
  HBX_SEQ();
  {
    const fq2d t2 = fq2d_mul(x(2), y(2));
    acc.c0 = fq2d_sub(acc.c0, fq2d_mul_xi(t2));
    acc.c1 = fq2d_add(acc.c1, fq2d_mul_xi(t2));
    acc.c2 = fq2d_sub(acc.c2, t2);
  }
  HBX_SEQ();
  acc.c0 = fq2d_add(acc.c0, fq2d_mul_xi(fq2d_mul(fq2d_add(x(1), x(2)), fq2d_add(y(1), y(2)))));
  HBX_SEQ();
  acc.c1 = fq2d_add(acc.c1, fq2d_mul(fq2d_add(x(0), x(1)), fq2d_add(y(0), y(1))));
  HBX_SEQ();
  acc.c2 = fq2d_add(acc.c2, fq2d_mul(fq2d_add(x(0), x(2)), fq2d_add(y(0), y(2))));
  HBX_SEQ();
  acc = fq6d_norm(acc);
}

// B = X * Y with X = slot B (conj first if cx), Y = slot `ys`: lane k's half X_k Y_0 +
// [v if k = 0] X_(1-k) Y_1; conj of the product if co.  Reads of B all precede the write (one
// wave, in-order LDS), so the pair's two lanes see the old value.
template <class P>
__device__ __forceinline__ void op_mul(const slot2<lds_u32*>& B, const slot2<P>& ys, bool cx, bool co, bool l1) {
  const lds_u32* xk = B.half(l1 ? 1 : 0);
  const lds_u32* xo = B.half(l1 ? 0 : 1);
  fq6d acc = fq6d_zero();
  // X_k (negated for k = 1 under cx)
  fq6d_mul_acc2(
      acc,
      [&](int q) {
        const fq2d v = slot_get_fq2d(xk, B.stride, q);
        return sel_t(cx && l1, fq2d_neg(v), v);
      },
      [&](int q) { return slot_get_fq2d(ys.half(0), ys.stride, q); });
  HBX_SEQ();
  // W = v X_1 on lane 0 (v (w0, w1, w2) = (xi w2, w0, w1); X_1 negated under cx), X_0 on lane 1
  fq6d_mul_acc2(
      acc,
      [&](int q) {
        const int qq = l1 ? q : (q + 2) % 3;
        fq2d v = slot_get_fq2d(xo, B.stride, qq);
        v = sel_t(cx && !l1, fq2d_neg(v), v);
        return sel_t(!l1 && q == 0, fq2d_norm(fq2d_mul_xi(v)), v);
      },
      [&](int q) { return slot_get_fq2d(ys.half(1), ys.stride, q); });
  slot_put_fq6d(B.half(l1 ? 1 : 0), B.stride, fq6d_reduce(sel_t(co && l1, fq6d_neg(acc), acc)));
}

// ---- Karabina compressed squarings on a pair (fe1d.hpp karabina_sqr split over the lanes) ----
// fe1d.hpp's numbering: g1 = c0.c1, g2 = c0.c2, g3 = c1.c0, g5 = c1.c2 (lane 0 holds c0, lane 1
// c1).  During a run lane 0 keeps (a, b) = (g3, g2) and lane 1 (g1, g5), and a squaring is ONE
// lazily reduced Fq4 squaring per lane -- lane 0 (g3 + g2 Y)^2 = (p1, x23), lane 1 (g1 + g5 Y)^2 =
// (p2, x15) -- plus an exchange of the two results (DPP):
//   lane 0: g3' = 3 xi x15 + 2 g3,  g2' = 3 p2 - 2 g2;    lane 1: g1' = 3 p1 - 2 g1,  g5' = 3 x23 + 2 g5
// (six convolutions and four reductions per lane against cyc_sqr2d's twelve and six).  A run ends
// in one decompression (an Fq inversion, ~38k instructions), so only the runs of 32 and 16 use it.
struct kara2 {
  fq2d a, b;
};
__device__ __forceinline__ fq2d kara2_lin(const fq2d& a3, const fq2d& b2, bool minus) {  // reduce(3 a +/- 2 b)
  const fq2d a = fq2d_add(fq2d_dbl(a3), a3);
  const fq2d b = fq2d_dbl(b2);
  return fq2d_reduce(sel_t(minus, fq2d_sub(a, b), fq2d_add(a, b)));
}
__device__ __forceinline__ kara2 kara2_sqr(const kara2& s, bool l1) {
  fq2d P, X;
  fq4d_sqr_lazy(s.a, s.b, P, X);
  const fq2d Po = xchg_t(P), Xo = xchg_t(X);
  const fq2d first = sel_t(l1, Po, fq2d_norm(fq2d_mul_xi(Xo)));
  const fq2d second = sel_t(l1, Xo, Po);
  return kara2{kara2_lin(first, s.a, l1), kara2_lin(second, s.b, !l1)};
}
// back to the split form: the pair swaps its coefficients, both lanes recover g4 and g0 (fe1d.hpp
// karabina_decompress, the same values on both lanes), lane 0 keeps (g0, g1, g2), lane 1 (g3, g4,
// g5).  `degenerate` (g3 = 0, the division impossible) is pair-uniform.
__device__ __forceinline__ fq6d kara2_decompress(const kara2& s, bool l1, bool& degenerate) {
  const fq2d oa = xchg_t(s.a), ob = xchg_t(s.b);
  fq12c c;
  c.g1 = sel_t(l1, s.a, oa);
  c.g5 = sel_t(l1, s.b, ob);
  c.g3 = sel_t(l1, oa, s.a);
  c.g2 = sel_t(l1, ob, s.b);
  const fq12d r = karabina_decompress(c, degenerate);
  return sel_t(l1, r.c1, r.c0);
}

// B = B^(2^n) by cyclotomic squarings in registers: Granger-Scott, or compressed (KARA, n >= 16)
template <bool KARA>
__device__ __forceinline__ void op_sqr(const slot2<lds_u32*>& B, uint32_t n, bool l1, bool& degenerate) {
  lds_u32* mine = B.half(l1 ? 1 : 0);
  if (KARA && n >= 16) {
    // lane 0 takes g3 from lane 1 (its c0), lane 1 takes g1 from lane 0 (its c1); b = own c2
    kara2 s{xchg_t(slot_get_fq2d(mine, B.stride, l1 ? 0 : 1)), slot_get_fq2d(mine, B.stride, 2)};
#pragma unroll 1
    for (uint32_t i = 0; i < n; i++) s = kara2_sqr(s, l1);
    HBX_SEQ();
    slot_put_fq6d(mine, B.stride, kara2_decompress(s, l1, degenerate));
    return;
  }
  fq6d r = slot_get_fq6d(mine, B.stride);
#pragma unroll 1
  for (uint32_t i = 0; i < n; i++) r = cyc_sqr2d(r, l1);
  slot_put_fq6d(mine, B.stride, r);
}

// dst = src (own half), or frob / frob2 of it: own coefficient q becomes conj^c(g) K_q with
// (c, K) = (1, gamma_{1, 2q + k}) for f^p and (0, gamma_{2, 2q + k}) for f^(p^2) (fieldd.hpp
// fq12d_frobenius / fq12d_frobenius2; gamma_0 = 1; k = this lane's half).  map: 0 copy, 1 frob,
// 2 frob2.
template <class PS, class PD>
__device__ __forceinline__ void op_map(const slot2<PS>& src, const slot2<PD>& dst, int map, bool l1) {
  const int k = l1 ? 1 : 0;
  if (map == 0) {
    const PS s = src.half(k);
    const PD d = dst.half(k);
#pragma unroll 6
    for (int w = 0; w < LDS_FQ6D_PACKED; w++) d[w * dst.stride] = s[w * src.stride];
    return;
  }
#pragma unroll 1
  for (int q = 0; q < 3; q++) {
    const int i = 2 * q + k;
    fq2d c{fqd_const(FQD_ONE), fqd_zero()};
    if (map == 1) {
      const int32_t* k0 = i == 1 ? FROBD1_C1_0 : i == 2 ? FROBD1_C2_0 : i == 3 ? FROBD1_C3_0 : i == 4 ? FROBD1_C4_0 : FROBD1_C5_0;
      const int32_t* k1 = i == 1 ? FROBD1_C1_1 : i == 2 ? FROBD1_C2_1 : i == 3 ? FROBD1_C3_1 : i == 4 ? FROBD1_C4_1 : FROBD1_C5_1;
      if (i) c = fq2d_const(k0, k1);
    } else {
      const int32_t* kk = i == 1 ? FROBD2_C1 : i == 2 ? FROBD2_C2 : i == 3 ? FROBD2_C3 : i == 4 ? FROBD2_C4 : FROBD2_C5;
      if (i) c = fq2d{fqd_const(kk), fqd_zero()};
    }
    fq2d y = slot_get_fq2d(src.half(k), src.stride, q);
    if (map == 1) y = fq2d_conj(y);
    slot_put_fq2d(dst.half(k), dst.stride, q, fq2d_mul(y, c));
  }
}

// The chain of pairingd.hpp final_exponentiation_d as a program over the slots (regrouped:
// t^3 is the value after the first step of t^|x|; conj(x^|x|) conj(x) = conj(x^|x| x);
// d = conj(conj(t^3) b) frob2(b) = t^3 conj(b) frob2(b) before the last two exponentiations).
// Products always take B * A; the global slots G1 (t^3, then d) and G2 (b) are only copied in and
// out.  Entry: B = f, A = f^-1.
enum : uint32_t { FE2_SQR = 0, FE2_MUL = 1, FE2_MAP = 2 };
enum : uint32_t { FE2_CX = 1, FE2_CO = 2 };  // MUL: conj(X) first, conj of the product
enum : uint32_t { FE2_S_A = 0, FE2_S_B = 1, FE2_S_G1 = 2, FE2_S_G2 = 3 };  // MAP slots
#define FE2_MULF(fl) ((uint32_t)FE2_MUL | ((uint32_t)(fl) << 4))
#define FE2_SQRN(n) ((uint32_t)FE2_SQR | ((uint32_t)(n) << 8))
#define FE2_MAPOP(m, s, d) ((uint32_t)FE2_MAP | ((uint32_t)(m) << 4) | ((uint32_t)(s) << 8) | ((uint32_t)(d) << 12))
// B <- B^|x| with the base in A: the runs of squarings between the one bits of |x| (63, 62, 60,
// 57, 48, 16) and a product by the base after each run but the last
#define FE2_EXP_TAIL FE2_SQRN(2), FE2_MULF(0), FE2_SQRN(3), FE2_MULF(0), FE2_SQRN(9), FE2_MULF(0), FE2_SQRN(32), \
    FE2_MULF(0), FE2_SQRN(16)
#define FE2_EXP FE2_SQRN(1), FE2_MULF(0), FE2_EXP_TAIL
__constant__ static const uint32_t FE2_PROG[] = {
    FE2_MULF(FE2_CX),                                            // t0 = conj(f) f^-1
    FE2_MAPOP(2, FE2_S_B, FE2_S_A), FE2_MULF(0),                 // t = t0 frob2(t0)
    FE2_MAPOP(0, FE2_S_B, FE2_S_A),                              // A = t
    FE2_SQRN(1), FE2_MULF(0), FE2_MAPOP(0, FE2_S_B, FE2_S_G1),   // B = t^3 = G1
    FE2_EXP_TAIL, FE2_MULF(FE2_CO),                              // a = conj(t^|x| t)
    FE2_MAPOP(0, FE2_S_B, FE2_S_A), FE2_EXP, FE2_MULF(FE2_CO),   // a = conj(a^|x| a)
    FE2_MAPOP(0, FE2_S_B, FE2_S_A), FE2_EXP,                     // B = a^|x|
    FE2_MAPOP(1, FE2_S_A, FE2_S_A), FE2_MULF(FE2_CX),            // b = conj(a^|x|) frob(a)
    FE2_MAPOP(0, FE2_S_B, FE2_S_G2),                             // G2 = b
    FE2_MAPOP(0, FE2_S_B, FE2_S_A), FE2_MAPOP(0, FE2_S_G1, FE2_S_B),  // A = b, B = t^3
    FE2_MULF(FE2_CX | FE2_CO),                                   // B = conj(conj(t^3) b)
    FE2_MAPOP(2, FE2_S_G2, FE2_S_A), FE2_MULF(0),                // B = t^3 conj(b) frob2(b) = d
    FE2_MAPOP(0, FE2_S_B, FE2_S_G1),                             // G1 = d
    FE2_MAPOP(0, FE2_S_G2, FE2_S_A), FE2_MAPOP(0, FE2_S_G2, FE2_S_B),  // A = B = b
    FE2_EXP, FE2_MAPOP(0, FE2_S_B, FE2_S_A), FE2_EXP,            // B = b^(x^2)
    FE2_MAPOP(0, FE2_S_G1, FE2_S_A), FE2_MULF(0)};               // b^(x^2) d
#undef FE2_EXP
#undef FE2_EXP_TAIL
#undef FE2_MAPOP
#undef FE2_SQRN
#undef FE2_MULF
constexpr int FE2_STEPS = (int)(sizeof(FE2_PROG) / sizeof(FE2_PROG[0]));

// Fq6 inverse in digit form (one Fq inversion, field.hpp's divsteps, inlined: no call frame):
// c0 = a0^2 - xi a1 a2, c1 = xi a2^2 - a0 a1, c2 = a1^2 - a0 a2, t = a0 c0 + xi (a2 c1 + a1 c2),
// a^-1 = (c0, c1, c2) / t with t^-1 = conj(t) / (t0^2 + t1^2).  Input reduced; the reduced result
// goes to `dst` (own half; it also parks (c0, c1, c2) meanwhile).
template <class PD>
__device__ __forceinline__ void fq6d_inv_to(const fq6d& a, PD dst, uint32_t stride) {
  fq2d t;
  {
    const fq2d c0 = fq2d_reduce(fq2d_sub(fq2d_sqr(a.c0), fq2d_mul_xi(fq2d_mul(a.c1, a.c2))));
    slot_put_fq2d(dst, stride, 0, c0);
    t = fq2d_mul(a.c0, c0);
  }
  HBX_SEQ();
  {
    const fq2d c1 = fq2d_reduce(fq2d_sub(fq2d_mul_xi(fq2d_sqr(a.c2)), fq2d_mul(a.c0, a.c1)));
    slot_put_fq2d(dst, stride, 1, c1);
    t = fq2d_add(t, fq2d_mul_xi(fq2d_mul(a.c2, c1)));
  }
  HBX_SEQ();
  {
    const fq2d c2 = fq2d_reduce(fq2d_sub(fq2d_sqr(a.c1), fq2d_mul(a.c0, a.c2)));
    slot_put_fq2d(dst, stride, 2, c2);
    t = fq2d_reduce(fq2d_add(t, fq2d_mul_xi(fq2d_mul(a.c1, c2))));
  }
  HBX_SEQ();
  const fqd nrm = fqd_reduce(fqd_add(fqd_sqr(t.c0), fqd_sqr(t.c1)));
  HBX_SEQ();
  bool zero;
  const fqd ni = fqd_inv(nrm, zero);
  HBX_SEQ();
  const fq2d ti = fq2d_mul_fq(fq2d_conj(t), ni);
#pragma unroll 1
  for (int q = 0; q < 3; q++) {
    HBX_SEQ();
    slot_put_fq2d(dst, stride, q, fq2d_reduce(fq2d_mul(slot_get_fq2d(dst, stride, q), ti)));
  }
}

// A = f^-1 = (f0 - f1 w) / (f0^2 - v f1^2) with f in B (own halves).
template <class PA>
__device__ __forceinline__ void op_inv(const slot2<PA>& A, const slot2<lds_u32*>& B, bool l1) {
  const lds_u32* fb = B.half(l1 ? 1 : 0);
  PA ao = A.half(l1 ? 1 : 0);
  fq6d S = fq6d_zero();  // lane 0: f0^2, lane 1: f1^2
  fq6d_mul_acc2(
      S, [&](int q) { return slot_get_fq2d(fb, B.stride, q); }, [&](int q) { return slot_get_fq2d(fb, B.stride, q); });
  const fq6d So = xchg_t(S);
  fq6d_inv_to(fq6d_reduce(fq6d_sub(sel_t(l1, So, S), fq6d_mul_v(sel_t(l1, S, So)))), ao, A.stride);
  HBX_SEQ();
  fq6d R = fq6d_zero();
  fq6d_mul_acc2(
      R, [&](int q) { return slot_get_fq2d(fb, B.stride, q); }, [&](int q) { return slot_get_fq2d(ao, A.stride, q); });
  slot_put_fq6d(ao, A.stride, fq6d_reduce(conj2d(R, l1)));
}

// f^(3 (p^12 - 1)/r) == 1 with f (reduced) in B; A, G1, G2 as above.  KARA: the runs of 32 and
// 16 squarings compressed; `degenerate` is then set (pair-uniformly) when a decompression met
// g3 = 0, and the verdict is not valid -- the caller decides that pair again with KARA = false.
__device__ __forceinline__ bool is_one2d(const fq6d& A, bool l1);
template <bool KARA, class PA = lds_u32*>
__device__ __forceinline__ bool final_exp2d_is_one(const slot2<PA>& A, const slot2<lds_u32*>& B,
                                                  const slot2<uint32_t*>& G1, const slot2<uint32_t*>& G2, bool l1,
                                                  bool& degenerate) {
  op_inv(A, B, l1);
#pragma unroll 1
  for (int pc = 0; pc < FE2_STEPS; pc++) {
    const uint32_t st = FE2_PROG[pc];
    const uint32_t op = st & 15;
    HBX_SEQ();
    if (op == FE2_SQR) {
      op_sqr<KARA>(B, st >> 8, l1, degenerate);
    } else if (op == FE2_MUL) {
      op_mul(B, A, ((st >> 4) & FE2_CX) != 0, ((st >> 4) & FE2_CO) != 0, l1);
    } else {
      const int map = (int)((st >> 4) & 15), src = (int)((st >> 8) & 15), dst = (int)((st >> 12) & 15);
      if (src == FE2_S_B) {
        if (dst == FE2_S_A) op_map(B, A, map, l1);
        else if (dst == FE2_S_G1) op_map(B, G1, map, l1);
        else op_map(B, G2, map, l1);
      } else if (src == FE2_S_A) {
        op_map(A, A, map, l1);
      } else {
        const slot2<uint32_t*>& g = src == FE2_S_G1 ? G1 : G2;
        if (dst == FE2_S_A) op_map(g, A, map, l1);
        else op_map(g, B, map, l1);
      }
    }
  }
  HBX_SEQ();
  return is_one2d(slot_get_fq6d(B.half(l1 ? 1 : 0), B.stride), l1);
}

// The pair's per-check scalars of point P (12-limb affine, not the identity): lane 0 1/y,
// lane 1 x/y.  `neg`: use -P.
__device__ __forceinline__ fqd point_scalar2d(const g1a& P, bool neg, bool l1) {
  const fq y = neg ? fq_neg(P.y) : P.y;
#if HBX_ML_INV
  bool zero;
#if HBX_ML_INV == 2
  const fqd yi = fqd_inv_ni(fqd_from_fq(y), zero);
#else
  const fqd yi = fqd_inv(fqd_from_fq(y), zero);  // digit form (fieldd.hpp fqd_inv)
#endif
  return l1 ? fqd_mul(fqd_from_fq(P.x), yi) : yi;
#else
  const fq yi = fq_inv_i(y);  // (the digit form inline: coin Miller kernel 4.06 -> 4.14 ms)
  return fqd_from_fq(l1 ? fq_mul(P.x, yi) : yi);
#endif
}

// ---- the coin's check: lines generated on the fly, f split over the pair ----------------------
// A lane's LDS words: its own line c0 + c1 v + c4 v w (c4 in Fq2: an un-normalised line at a G1
// point; packed, words 0..77), and one packed park (words MG_PARK..155) holding whichever of T and
// f is idle -- T while the pair multiplies, f while the lane generates its line.  The squaring
// uses words 0..55 (sqr2d<true>).  In registers at any time: f or T, and one step's temporaries.
constexpr int MG_PARK = 78;

// f * (c0 + c1 v + c4 v w) with the packed line in the lane column `ln` (either lane of the pair):
// lane 0 A0 L0 + v^2 c4 A1, lane 1 A1 L0 + v c4 A0 (L0 = c0 + c1 v; w^2 = v).  8 Fq2 products per
// lane against the one-lane sparse product's 13; the partner's half comes over one coefficient at
// a time.  Reduced output.
// C4ONE: the line is c0 + c1 v + v w (a prepared line scaled by 1 / y_P, the coin's H' lines since
// round 6): E = A_(1-k) itself, no c4 products.
template <bool C4ONE = false>
__device__ __forceinline__ fq6d line2d_f2(const fq6d& A, bool l1, const lds_u32* ln) {
  fq6d acc;  // v^(2-k) c4 A_(1-k), then + A_k L0 (fieldd.hpp fq6d_mul_by_01's Karatsuba)
  if (C4ONE) {
    const fq6d vE = fq6d_mul_v(fq6d{xchg_t(A.c0), xchg_t(A.c1), xchg_t(A.c2)});
    acc = sel_t(l1, vE, fq6d_mul_v(vE));
  } else {
    const fq2d c4 = slot_get_fq2d(ln, 64u, 2);
    fq6d E;
    E.c0 = fq2d_mul(xchg_t(A.c0), c4);
    HBX_SEQ();
    E.c1 = fq2d_mul(xchg_t(A.c1), c4);
    HBX_SEQ();
    E.c2 = fq2d_mul(xchg_t(A.c2), c4);
    const fq6d vE = fq6d_mul_v(E);
    acc = sel_t(l1, vE, fq6d_mul_v(vE));
  }
  HBX_SEQ();
  const fq2d c0 = slot_get_fq2d(ln, 64u, 0), c1 = slot_get_fq2d(ln, 64u, 1);
  {
    const fq2d t0 = fq2d_mul(A.c0, c0);
    acc.c0 = fq2d_add(acc.c0, t0);
    acc.c1 = fq2d_sub(acc.c1, t0);
  }
  HBX_SEQ();
  {
    const fq2d t1 = fq2d_mul(A.c1, c1);
    acc.c1 = fq2d_sub(acc.c1, t1);
    acc.c2 = fq2d_add(acc.c2, t1);
  }
  HBX_SEQ();
  acc.c0 = fq2d_add(acc.c0, fq2d_mul_xi(fq2d_mul(A.c2, c1)));
  HBX_SEQ();
  acc.c1 = fq2d_add(acc.c1, fq2d_mul(fq2d_add(A.c0, A.c1), fq2d_add(c0, c1)));
  HBX_SEQ();
  acc.c2 = fq2d_add(acc.c2, fq2d_mul(A.c2, c0));
  HBX_SEQ();
  return fq6d_reduce(acc);  // digit sums of a few normalised values: below 2^31
}

// The coin check's two Miller loops on a pair (pairingd.hpp miller_loop_gen_parked_d, both pairs):
// lane k generates the lines of its own pair (Q = *q, P = (px, py); lane 0 (H', pk_i), lane 1
// (sigma_i, -[m] g1)) into its LDS words, and the pair multiplies the split f by lane 0's line and
// then lane 1's.  Returns this lane's half of f_A f_B, conjugated for x < 0; T = [|x|] Q.  An
// unused pair (`use` false: a point at infinity) contributes lines equal to 1.  The one-lane loop
// held a whole Fq12 plus the sparse product's temporaries per lane and spilled (367 VGPRs,
// 10.6 GB of scratch traffic per coin launch).
__device__ __forceinline__ fq6d miller_gen2d(const g2a* q, const fqd& px, const fqd& py, bool use, bool l1, lds2 lds,
                                             const lds_u32* pair0, g2jd& Tout) {
  const fq2d one{fqd_const(FQD_ONE), fqd_zero()}, zero{fqd_zero(), fqd_zero()};
  lds_u32* park = lds + MG_PARK * 64;
  {
    const g2a Q = *q;
    slot_put_fq6d(park, 64u, fq6d{fq2d_from_fq2(Q.x), fq2d_from_fq2(Q.y), one});  // T
  }
  fq6d f = sel_t(l1, fq6d_zero(), fq6d_one());
  // one line step: T from the park, f to it, the line (doubling, or addition of Q), f back, T to
  // the park, the pair's two line products
  auto step = [&](bool add) __attribute__((always_inline)) {
    HBX_SEQ();
    g2jd T;
    {
      const fq6d t = slot_get_fq6d(park, 64u);
      T = g2jd{t.c0, t.c1, t.c2};
    }
    HBX_SEQ();
    slot_put_fq6d(park, 64u, f);
    HBX_SEQ();
    fq2d c0, c1, c2;
    if (!add) {
      line_dbl_step_di(T, c0, c1, c2);
    } else {
      const g2a Q = *q;  // the five addition steps re-read the base point
      line_add_step_call(T, fq2d_from_fq2(Q.x), fq2d_from_fq2(Q.y), c0, c1, c2);
    }
    HBX_SEQ();
    slot_put_fq2d(lds, 64u, 0, sel_t(use, c0, one));
    slot_put_fq2d(lds, 64u, 1, sel_t(use, fq2d_mul_fq(c1, px), zero));
    slot_put_fq2d(lds, 64u, 2, sel_t(use, fq2d_mul_fq(c2, py), zero));
    HBX_SEQ();
    f = slot_get_fq6d(park, 64u);
    HBX_SEQ();
    slot_put_fq6d(park, 64u, fq6d{T.x, T.y, T.z});
    HBX_SEQ();
    f = line2d_f2(f, l1, pair0);
    HBX_SEQ();
    f = line2d_f2(f, l1, pair0 + 1);
  };
  // |x| = 0xd201000000010000: the doubling steps i = 62..0 in runs, an addition step after each run
  // but the last (bits 62, 60, 57, 48, 16).  The addition is an out-of-line call, kept out of the
  // runs' loops: inside the loop the values live across it spilled (139 VGPRs).
  static_assert(BLS_X == 0xd201000000010000ull, "the runs below follow |x|'s bits");
  constexpr int RUN[6] = {1, 2, 3, 9, 32, 16};
  bool first = true;
#pragma unroll 1
  for (int r = 0; r < 6; r++) {
#pragma unroll 1
    for (int t = 0; t < RUN[r]; t++) {
      if (!first) f = sqr2d<true>(f, l1, lds);
      first = false;
      step(false);
    }
    if (r < 5) step(true);
  }
  HBX_SEQ();
  {
    const fq6d t = slot_get_fq6d(park, 64u);
    Tout = g2jd{t.c0, t.c1, t.c2};
  }
  return conj2d(f, l1);
}

// ---- the coin check with H''s lines prepared once per instance (round 6) ---------------------
// The 128 checks of an instance share H': its 68 Miller lines are prepared once (k_prepare_lines +
// k_normalise_lines, as the decryption checks' are) and each pair only loads them, scaled by
// 1 / y_pk (c4 = 1: line2d_f2<true> skips the three c4 products).  Both lanes then generate
// sigma's lines TOGETHER: each doubling step is split into rounds of one Fq2 product per lane
// whose results the pair exchanges (6 rounds instead of pairingd.hpp line_dbl_step_di's 11
// products), so both lanes hold sigma's T and line.

// one product round on the pair: lane 0 computes a0 b0, lane 1 a1 b1; both get (r0, r1)
__device__ __forceinline__ void round2_mul(bool l1, const fq2d& a0, const fq2d& b0, const fq2d& a1, const fq2d& b1,
                                           fq2d& r0, fq2d& r1) {
  const fq2d mine = fq2d_mul(sel_t(l1, a1, a0), sel_t(l1, b1, b0));
  const fq2d other = xchg_t(mine);
  r0 = sel_t(l1, other, mine);
  r1 = sel_t(l1, mine, other);
}
__device__ __forceinline__ void round2_sqr(bool l1, const fq2d& a0, const fq2d& a1, fq2d& r0, fq2d& r1) {
  const fq2d mine = fq2d_sqr(sel_t(l1, a1, a0));
  const fq2d other = xchg_t(mine);
  r0 = sel_t(l1, other, mine);
  r1 = sel_t(l1, mine, other);
}
__device__ __forceinline__ void round2_mul_fq(bool l1, const fq2d& a0, const fqd& s0, const fq2d& a1, const fqd& s1,
                                              fq2d& r0, fq2d& r1) {
  const fq2d mine = fq2d_mul_fq(sel_t(l1, a1, a0), sel_t(l1, s1, s0));
  const fq2d other = xchg_t(mine);
  r0 = sel_t(l1, other, mine);
  r1 = sel_t(l1, mine, other);
}
// pairingd.hpp line_dbl_step_di on the pair (both lanes hold T; the same T', c0, c1, c2 result):
// A = X^2 | B = Y^2;  ZZ = Z^2 | YZ;  C = B^2 | F = E^2;  (X + B)^2 | E X;  E ZZ | Z3 ZZ;  E (D - X3)
__device__ __forceinline__ void line_dbl_step_2s(g2jd& T, bool l1, fq2d& c0, fq2d& c1, fq2d& c2) {
  fq2d A, B, ZZ, YZ, C, F, S, EX, EZZ;
  round2_sqr(l1, T.x, T.y, A, B);
  HBX_SEQ();
  round2_mul(l1, T.z, T.z, T.y, T.z, ZZ, YZ);
  HBX_SEQ();
  const fq2d E = fq2d_norm(fq2d_add(fq2d_dbl(A), A));
  const fq2d XB = fq2d_add(T.x, B);
  const fq2d Z3 = fq2d_reduce(fq2d_dbl(YZ));
  round2_sqr(l1, B, E, C, F);
  HBX_SEQ();
  round2_mul(l1, XB, XB, E, T.x, S, EX);
  HBX_SEQ();
  round2_mul(l1, E, ZZ, Z3, ZZ, EZZ, c2);
  HBX_SEQ();
  c0 = fq2d_reduce(fq2d_sub(EX, fq2d_dbl(B)));
  c1 = fq2d_neg(EZZ);
  const fq2d D = fq2d_reduce(fq2d_dbl(fq2d_sub(fq2d_sub(S, A), C)));
  const fq2d X3 = fq2d_reduce(fq2d_sub(F, fq2d_dbl(D)));
  const fq2d C8 = fq2d_dbl(fq2d_reduce(fq2d_dbl(fq2d_dbl(C))));
  const fq2d Y3 = fq2d_reduce(fq2d_sub(fq2d_mul(E, fq2d_sub(D, X3)), C8));
  T = g2jd{X3, Y3, Z3};
}

// pairingd.hpp line_add_step_di on the pair (T + Q with Q = (qx, qy) affine; both lanes hold T and
// Q): 7 rounds instead of 14 products, inline -- the round-5 kernel called the one-lane step out of
// line, through scratch frames (0.93 GB of scratch traffic per coin launch,
// profiles/r06m_final_pmc_coin.json)
__device__ __forceinline__ void line_add_step_2s(g2jd& T, const fq2d& qx, const fq2d& qy, bool l1, fq2d& c0,
                                                 fq2d& c1, fq2d& c2) {
  fq2d Z1Z1, qyZ, U2, S2, ZH, HH, nqx, ZpH2, r2, qyden, J, V, YJ, W;
  round2_mul(l1, T.z, T.z, qy, T.z, Z1Z1, qyZ);
  HBX_SEQ();
  round2_mul(l1, qx, Z1Z1, qyZ, Z1Z1, U2, S2);
  HBX_SEQ();
  const fq2d H = fq2d_reduce(fq2d_sub(U2, T.x));
  const fq2d num = fq2d_reduce(fq2d_sub(T.y, S2));
  const fq2d r = fq2d_reduce(fq2d_dbl(fq2d_sub(S2, T.y)));
  round2_mul(l1, T.z, H, H, H, ZH, HH);
  HBX_SEQ();
  const fq2d ZpH = fq2d_norm(fq2d_add(T.z, H));
  round2_mul(l1, num, qx, ZpH, ZpH, nqx, ZpH2);
  HBX_SEQ();
  const fq2d den = fq2d_neg(ZH);
  round2_mul(l1, r, r, qy, den, r2, qyden);
  HBX_SEQ();
  const fq2d I = fq2d_reduce(fq2d_dbl(fq2d_dbl(HH)));
  c0 = fq2d_reduce(fq2d_sub(nqx, qyden));
  c1 = fq2d_neg(num);
  c2 = den;
  const fq2d Z3 = fq2d_reduce(fq2d_sub(fq2d_sub(ZpH2, Z1Z1), HH));
  round2_mul(l1, H, I, T.x, I, J, V);
  HBX_SEQ();
  const fq2d X3 = fq2d_reduce(fq2d_sub(fq2d_sub(r2, J), fq2d_dbl(V)));
  round2_mul(l1, T.y, J, r, fq2d_sub(V, X3), YJ, W);
  HBX_SEQ();
  const fq2d Y3 = fq2d_reduce(fq2d_sub(W, fq2d_dbl(YJ)));
  T = g2jd{X3, Y3, Z3};
}

// The coin check's two Miller loops on a pair with H''s prepared lines LH (68, Miller order; the
// instance's, wave-uniform): lane 0 holds s = 1 / y_pk, lane 1 s = x_pk / y_pk (point_scalar2d of
// pk_i); useH false: the H' pair contributes 1.  sigma (*q) at -[m] g1 = (px, py) in digit form;
// useS false: sigma's lines are 1.  Returns this lane's half of f_H f_sigma (conjugated for x < 0);
// T = [|x|] sigma on both lanes.  LDS: lane 0's column holds H''s scaled line (words 0..55), lane
// 1's sigma's (c0, c1 px, c2 py); both columns' park (words MG_PARK..) holds whichever of T and f is
// idle, as in miller_gen2d.
__device__ __forceinline__ fq6d miller_gen2s(const line_pre_d* LH, const fqd& s, bool useH, const g2a* q,
                                             const fqd& px, const fqd& py, bool useS, bool l1, lds2 lds,
                                             const lds_u32* pair0, g2jd& Tout) {
  const fq2d one{fqd_const(FQD_ONE), fqd_zero()}, zero{fqd_zero(), fqd_zero()};
  lds_u32* park = lds + MG_PARK * 64;
  {
    const g2a Q = *q;
    slot_put_fq6d(park, 64u, fq6d{fq2d_from_fq2(Q.x), fq2d_from_fq2(Q.y), one});  // T
  }
  fq6d f = sel_t(l1, fq6d_zero(), fq6d_one());
  int k = 0;
  auto step = [&](bool add) __attribute__((always_inline)) {
    HBX_SEQ();
    g2jd T;
    {
      const fq6d t = slot_get_fq6d(park, 64u);
      T = g2jd{t.c0, t.c1, t.c2};
    }
    HBX_SEQ();
    slot_put_fq6d(park, 64u, f);
    HBX_SEQ();
    fq2d c0, c1, c2;
    if (!add) {
      line_dbl_step_2s(T, l1, c0, c1, c2);
    } else {
      const g2a Q = *q;  // sigma's addition step, split over the pair like the doubling
      line_add_step_2s(T, fq2d_from_fq2(Q.x), fq2d_from_fq2(Q.y), l1, c0, c1, c2);
    }
    HBX_SEQ();
    // sigma's (c1 px | c2 py) and H''s scaled (h0 / y | h1 x / y), one product per lane each
    fq2d c1p, c2p, h0s, h1s;
    round2_mul_fq(l1, c1, px, c2, py, c1p, c2p);
    HBX_SEQ();
    {
      const line_pre_d L = ld_uniform(LH + k);
      round2_mul_fq(l1, L.c0, s, L.c1, s, h0s, h1s);
    }
    k++;
    HBX_SEQ();
    // lane 0's column: H''s line; lane 1's: sigma's (each lane writes its own column)
    slot_put_fq2d(lds, 64u, 0, sel_t(l1, sel_t(useS, c0, one), h0s));
    slot_put_fq2d(lds, 64u, 1, sel_t(l1, sel_t(useS, c1p, zero), h1s));
    slot_put_fq2d(lds, 64u, 2, sel_t(useS, c2p, zero));  // (lane 0's word 2 unused: c4 = 1)
    HBX_SEQ();
    f = slot_get_fq6d(park, 64u);
    HBX_SEQ();
    slot_put_fq6d(park, 64u, fq6d{T.x, T.y, T.z});
    HBX_SEQ();
    {
      const fq6d fh = line2d_f2<true>(f, l1, pair0);
      f = sel_t(useH, fh, f);  // pair-uniform (both lanes know pk_i and H')
    }
    HBX_SEQ();
    f = line2d_f2(f, l1, pair0 + 1);
  };
  static_assert(BLS_X == 0xd201000000010000ull, "the runs below follow |x|'s bits");
  constexpr int RUN[6] = {1, 2, 3, 9, 32, 16};
  bool first = true;
#pragma unroll 1
  for (int r = 0; r < 6; r++) {
#pragma unroll 1
    for (int t = 0; t < RUN[r]; t++) {
      if (!first) f = sqr2d<true>(f, l1, lds);
      first = false;
      step(false);
    }
    if (r < 5) step(true);
  }
  HBX_SEQ();
  {
    const fq6d t = slot_get_fq6d(park, 64u);
    Tout = g2jd{t.c0, t.c1, t.c2};
  }
  return conj2d(f, l1);
}

// ---- the whole check ------------------------------------------------------------------------
// Miller stage: the scalars of both points, the two Miller loops (Miller scratch in the LDS
// region), f (reduced) to slot B.  flags: bit 0 = this lane is lane 1 of its pair, bit 1 = use
// pair A (S, H'), bit 2 = use pair B (-[m] pk, W).
__device__ __forceinline__ void check2d_miller(const line_pre_d* LA, const g1a& PA, const line_pre_d* LB, const g1a& PB,
                                               uint32_t flags, lds2 lds, const slot2<lds_u32*>& B) {
  const bool l1 = (flags & 1) != 0, useA = (flags & 2) != 0, useB = (flags & 4) != 0;
  fqd sA = fqd_zero(), sB = fqd_zero();
  if (useA) sA = point_scalar2d(PA, false, l1);
  if (useB) sB = point_scalar2d(PB, true, l1);  // the B point enters negated: -[m] pk_i
  const fq6d f = miller2d(LA, sA, useA, LB, sB, useB, l1, lds);
  HBX_SEQ();
  slot_put_fq6d(B.half(l1 ? 1 : 0), B.stride, fq6d_reduce(f));
}

// f == 1 for the pair: lane 0 holds (1, 0, 0), lane 1 holds 0
__device__ __forceinline__ bool is_one2d(const fq6d& A, bool l1) {
  const fq6 a = fq6d_to_fq6(A);
  const bool c0ok = l1 ? fq2_is_zero(a.c0) : (fq_eq(a.c0.c0, fq_one()) && fq_is_zero(a.c0.c1));
  const bool mine = c0ok && fq2_is_zero(a.c1) && fq2_is_zero(a.c2);
  dpp_guard_pairs();
  return mine && xchg_i32(mine ? 1 : 0) != 0;
}

#endif  // __HIPCC__
}  // namespace hbx
