// G1 / G2 group arithmetic for BLS12-381 on gfx950 (pairing 0.14.2 G1/G2, reference
// Cargo.toml:28; used through threshold_crypto at honey_badger.rs:229/:340/:403 and
// common_coin.rs:142/:151/:190).
//
// Points are Jacobian (X, Y, Z) with x = X/Z^2, y = Y/Z^3 in Montgomery form; Z = 0 is the
// identity.  Affine points carry an explicit infinity flag.  Encodings follow the zcash format
// pairing uses.
#pragma once
#include "field.hpp"

namespace hbx {

struct g1a {
  fq x, y;
  bool inf;
};
struct g1j {
  fq x, y, z;
};
struct g2a {
  fq2 x, y;
  bool inf;
};
struct g2j {
  fq2 x, y, z;
};

// Decode status codes (same values as include/hbx.h HBX_PT_*).
#ifndef HBX_PT_OK
#define HBX_PT_OK 0
#define HBX_PT_BAD_FLAGS 1
#define HBX_PT_NOT_IN_FIELD 2
#define HBX_PT_NOT_ON_CURVE 3
#define HBX_PT_INFINITY 4
#define HBX_PT_NOT_IN_SUBGROUP 5
#endif

// ----------------------------------------------------------------------------------------------
// G1
// ----------------------------------------------------------------------------------------------
HBX_HD g1j g1_identity() { return g1j{fq_one(), fq_one(), fq_zero()}; }
HBX_HD bool g1j_is_identity(const g1j& p) { return fq_is_zero(p.z); }
HBX_HD g1j g1_from_affine(const g1a& a) {
  if (a.inf) return g1_identity();
  return g1j{a.x, a.y, fq_one()};
}

// dbl-2009-l (a = 0); g1_dbl_i inlined into hot loops, g1_dbl one out-of-line copy
HBX_HD g1j g1_dbl_i(const g1j& p) {
  const fq A = fq_sqr_inl(p.x);
  const fq B = fq_sqr_inl(p.y);
  const fq C = fq_sqr_inl(B);
  fq D = fq_sub(fq_sub(fq_sqr_inl(fq_add(p.x, B)), A), C);
  D = fq_dbl(D);
  const fq E = fq_add(fq_dbl(A), A);
  const fq F = fq_sqr_inl(E);
  const fq X3 = fq_sub(F, fq_dbl(D));
  const fq C8 = fq_dbl(fq_dbl(fq_dbl(C)));
  const fq Y3 = fq_sub(fq_mul_inl(E, fq_sub(D, X3)), C8);
  const fq Z3 = fq_dbl(fq_mul_inl(p.y, p.z));
  return g1j{X3, Y3, Z3};
}
HBX_HDNI g1j g1_dbl(const g1j& p) { return g1_dbl_i(p); }

// add-2007-bl, complete for P == Q / P == -Q / identities.
HBX_HD g1j g1_add_i(const g1j& p, const g1j& q) {
  if (g1j_is_identity(p)) return q;
  if (g1j_is_identity(q)) return p;
  const fq Z1Z1 = fq_sqr_inl(p.z);
  const fq Z2Z2 = fq_sqr_inl(q.z);
  const fq U1 = fq_mul_inl(p.x, Z2Z2);
  const fq U2 = fq_mul_inl(q.x, Z1Z1);
  const fq S1 = fq_mul_inl(fq_mul_inl(p.y, q.z), Z2Z2);
  const fq S2 = fq_mul_inl(fq_mul_inl(q.y, p.z), Z1Z1);
  if (fq_eq(U1, U2)) {
    if (fq_eq(S1, S2)) return g1_dbl(p);
    return g1_identity();
  }
  const fq H = fq_sub(U2, U1);
  const fq I = fq_sqr_inl(fq_dbl(H));
  const fq J = fq_mul_inl(H, I);
  const fq r = fq_dbl(fq_sub(S2, S1));
  const fq V = fq_mul_inl(U1, I);
  const fq X3 = fq_sub(fq_sub(fq_sqr_inl(r), J), fq_dbl(V));
  const fq Y3 = fq_sub(fq_mul_inl(r, fq_sub(V, X3)), fq_dbl(fq_mul_inl(S1, J)));
  const fq Z3 = fq_mul_inl(fq_sub(fq_sub(fq_sqr_inl(fq_add(p.z, q.z)), Z1Z1), Z2Z2), H);
  return g1j{X3, Y3, Z3};
}
HBX_HDNI g1j g1_add(const g1j& p, const g1j& q) { return g1_add_i(p, q); }

HBX_HD g1j g1_neg(const g1j& p) { return g1j{p.x, fq_neg(p.y), p.z}; }

HBX_HDNI g1a g1_to_affine(const g1j& p) {
  g1a r;
  if (g1j_is_identity(p)) {
    r.x = fq_zero();
    r.y = fq_zero();
    r.inf = true;
    return r;
  }
  const fq zi = fq_inv(p.z);
  const fq zi2 = fq_sqr(zi);
  r.x = fq_mul(p.x, zi2);
  r.y = fq_mul(fq_mul(p.y, zi2), zi);
  r.inf = false;
  return r;
}

// 255-bit scalar (canonical, 8 limbs) times point, left-to-right double-and-add.
HBX_HDNI g1j g1_mul_scalar(const g1j& p, const uint32_t* k8) {
  g1j acc = g1_identity();
  bool started = false;
  for (int i = 255; i >= 0; i--) {
    if (started) acc = g1_dbl(acc);
    if ((k8[i >> 5] >> (i & 31)) & 1) {
      acc = started ? g1_add(acc, p) : p;
      started = true;
    }
  }
  return acc;
}

// madd-2007-bl: Jacobian + affine (7M + 4S), complete for identities and P == +-Q.
HBX_HD g1j g1_add_mixed_i(const g1j& p, const g1a& q) {
  if (q.inf) return p;
  if (g1j_is_identity(p)) return g1j{q.x, q.y, fq_one()};
  const fq Z1Z1 = fq_sqr_inl(p.z);
  const fq U2 = fq_mul_inl(q.x, Z1Z1);
  const fq S2 = fq_mul_inl(fq_mul_inl(q.y, p.z), Z1Z1);
  const fq H = fq_sub(U2, p.x);
  const fq r = fq_dbl(fq_sub(S2, p.y));
  if (fq_is_zero(H)) {
    if (fq_is_zero(r)) return g1_dbl(p);
    return g1_identity();
  }
  const fq HH = fq_sqr_inl(H);
  const fq I = fq_dbl(fq_dbl(HH));
  const fq J = fq_mul_inl(H, I);
  const fq V = fq_mul_inl(p.x, I);
  const fq X3 = fq_sub(fq_sub(fq_sqr_inl(r), J), fq_dbl(V));
  const fq Y3 = fq_sub(fq_mul_inl(r, fq_sub(V, X3)), fq_dbl(fq_mul_inl(p.y, J)));
  const fq Z3 = fq_sub(fq_sub(fq_sqr_inl(fq_add(p.z, H)), Z1Z1), HH);
  return g1j{X3, Y3, Z3};
}

// k * P for a 128-bit scalar (4 limbs) and affine P: one inlined doubling and one inlined mixed
// addition in a non-unrolled loop (the accumulator stays in registers).
HBX_HDNI g1j g1_mul_u128(const g1a& P, const uint32_t* k4) {
  const g1a q = P;
  g1j acc = g1_identity();
#pragma unroll 1
  for (int i = 127; i >= 0; i--) {
    acc = g1_dbl_i(acc);
    if ((k4[i >> 5] >> (i & 31)) & 1) acc = g1_add_mixed_i(acc, q);
  }
  return acc;
}

// Same product with a fixed 4-bit window, for scalars that differ across the lanes of a wave
// (the Lagrange combine): double-and-add issues the addition whenever ANY lane has a 1 bit,
// i.e. ~128 mixed additions per wave, while here every lane adds its own table entry once per
// window: 124 doublings + 31 additions + 14 table additions.  The table (0..15) P sits in
// per-lane scratch (dynamically indexed); a zero digit takes g1_add's identity early-out.
HBX_HDNI g1j g1_mul_u128_w4(const g1a& P, const uint32_t* k4) {
  g1j tab[16];
  tab[0] = g1_identity();
  tab[1] = g1_from_affine(P);
#pragma unroll 1
  for (int i = 2; i < 16; i++) tab[i] = g1_add_mixed_i(tab[i - 1], P);
  g1j acc = tab[k4[3] >> 28];
  // the next window's table entry is loaded before this window's doublings, so the scratch read
  // lands while they run
  g1j nxt = tab[(k4[3] >> 24) & 0xFu];
#pragma unroll 1
  for (int w = 30; w >= 0; w--) {
    const g1j cur = nxt;
    if (w > 0) nxt = tab[(k4[(w - 1) >> 3] >> (((w - 1) & 7) * 4)) & 0xFu];
#pragma unroll 1
    for (int q = 0; q < 4; q++) acc = g1_dbl_i(acc);  // one inlined copy each: acc stays in VGPRs
    acc = g1_add_i(acc, cur);
  }
  return acc;
}

// k * P for a 64-bit scalar: g1_mul_u128_w4's 4-bit fixed window over 16 windows (60 doublings)
HBX_HDNI g1j g1_mul_u64_w4(const g1a& P, uint64_t k) {
  g1j tab[16];
  tab[0] = g1_identity();
  tab[1] = g1_from_affine(P);
#pragma unroll 1
  for (int i = 2; i < 16; i++) tab[i] = g1_add_mixed_i(tab[i - 1], P);
  g1j acc = tab[k >> 60];
  g1j nxt = tab[(k >> 56) & 0xFu];
#pragma unroll 1
  for (int w = 14; w >= 0; w--) {
    const g1j cur = nxt;
    if (w > 0) nxt = tab[(k >> (4 * (w - 1))) & 0xFu];
#pragma unroll 1
    for (int q = 0; q < 4; q++) acc = g1_dbl_i(acc);
    acc = g1_add_i(acc, cur);
  }
  return acc;
}

// GLV split of a canonical scalar k < r: k = k1 + k2 lambda with lambda = x^2 - 1 (128 bits),
// k1 = k mod lambda, k2 = k div lambda (< lambda + 2 < 2^128 since r = lambda^2 + lambda + 1).
// Then k P = k1 P + k2 phi(P), phi(x, y) = (beta x, y).
HBX_HD void g1_glv_split(const uint32_t* k8, uint32_t* k1, uint32_t* k2) {
  uint32_t rem[5] = {0, 0, 0, 0, 0};
  uint32_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 255; i >= 0; i--) {
    // rem = 2 rem + bit
    uint32_t c = (k8[i >> 5] >> (i & 31)) & 1u;
#pragma unroll
    for (int w = 0; w < 5; w++) {
      const uint32_t nc = rem[w] >> 31;
      rem[w] = (rem[w] << 1) | c;
      c = nc;
    }
    // if rem >= lambda: rem -= lambda
    uint32_t d[5], br = 0;
#pragma unroll
    for (int w = 0; w < 5; w++) d[w] = subb32(rem[w], w < 4 ? G1_GLV_LAMBDA[w] : 0u, br);
    if (!br) {
#pragma unroll
      for (int w = 0; w < 5; w++) rem[w] = d[w];
      q[i >> 5] |= 1u << (i & 31);
    }
  }
  for (int w = 0; w < 4; w++) {
    k1[w] = rem[w];
    k2[w] = q[w];
  }
}

// P in G1 (the order-r subgroup) for an affine point on the curve -- what pairing 0.14's
// into_affine checks on deserialisation (is_in_correct_subgroup_assuming_on_curve).
// Criterion (eprint 2021/1130 sec. 6, proof in 2022/352): phi'(P) == -[x^2] P with
// phi'(x, y) = (beta^2 x, y).  One 128-bit double-and-add instead of a 255-bit [r] P.
HBX_HDNI bool g1_is_torsion_free(const g1a& P) {
  if (P.inf) return true;
  const g1j m = g1_mul_u128(P, G1_X2);  // [x^2] P
  if (g1j_is_identity(m)) return false;  // phi'(P) is never O for P != O
  // (beta^2 x_P, y_P) == -(X/Z^2, Y/Z^3)  <=>  X == beta^2 x_P Z^2  and  Y == -y_P Z^3
  const fq z2 = fq_sqr(m.z);
  const fq z3 = fq_mul(z2, m.z);
  return fq_eq(m.x, fq_mul(fq_mul(P.x, fq_from_const(G1_BETA2)), z2)) && fq_eq(m.y, fq_neg(fq_mul(P.y, z3)));
}

// zcash compressed G1 -> affine (Montgomery).  No subgroup check.
// `sqrt(a, y)`: a square root of a, false if none (fq_sqrt; g1d.hpp passes the digit-tower one).
template <class Sqrt>
HBX_HD int32_t g1_decompress_t(const uint8_t* b48, g1a& out, Sqrt sqrt) {
  const uint8_t flags = b48[0];
  out.inf = false;
  if (!(flags & 0x80)) return HBX_PT_BAD_FLAGS;
  if (flags & 0x40) {
    bool clean = !(flags & 0x20) && !(flags & 0x1F);
    for (int i = 1; i < 48; i++) clean = clean && b48[i] == 0;
    if (!clean) return HBX_PT_BAD_FLAGS;
    out.x = fq_zero();
    out.y = fq_zero();
    out.inf = true;
    return HBX_PT_INFINITY;
  }
  uint8_t tmp[48];
  for (int i = 0; i < 48; i++) tmp[i] = b48[i];
  tmp[0] &= 0x1F;
  const fq xc = fq_from_be(tmp);
  if (!fq_lt_p(xc)) return HBX_PT_NOT_IN_FIELD;
  const fq x = fq_to_mont(xc);
  const fq rhs = fq_add(fq_mul(fq_sqr(x), x), fq_from_const(FQ_B1));
  fq y;
  if (!sqrt(rhs, y)) return HBX_PT_NOT_ON_CURVE;
  if (fq_lex_largest(y) != ((flags & 0x20) != 0)) y = fq_neg(y);
  out.x = x;
  out.y = y;
  return HBX_PT_OK;
}
HBX_HDNI int32_t g1_decompress(const uint8_t* b48, g1a& out) {
  return g1_decompress_t(b48, out, [](const fq& a, fq& y) { return fq_sqrt(a, y); });
}

HBX_HD void g1_compress(const g1a& p, uint8_t* b48) {
  if (p.inf) {
    for (int i = 0; i < 48; i++) b48[i] = 0;
    b48[0] = 0xC0;
    return;
  }
  fq_to_be(fq_from_mont(p.x), b48);
  b48[0] |= 0x80;
  if (fq_lex_largest(p.y)) b48[0] |= 0x20;
}

// ----------------------------------------------------------------------------------------------
// G2 (twist y^2 = x^3 + 4(u+1))
// ----------------------------------------------------------------------------------------------
HBX_HD fq2 g2_b() {
  const fq four = fq_from_const(FQ_B1);
  return fq2{four, four};
}
HBX_HD g2j g2_identity() { return g2j{fq2_one(), fq2_one(), fq2_zero()}; }
HBX_HD bool g2j_is_identity(const g2j& p) { return fq2_is_zero(p.z); }
HBX_HD g2j g2_from_affine(const g2a& a) {
  if (a.inf) return g2_identity();
  return g2j{a.x, a.y, fq2_one()};
}

HBX_HDNI g2j g2_dbl(const g2j& p) {
  const fq2 A = fq2_sqr_t<FqInl>(p.x);
  const fq2 B = fq2_sqr_t<FqInl>(p.y);
  const fq2 C = fq2_sqr_t<FqInl>(B);
  fq2 D = fq2_sub(fq2_sub(fq2_sqr_t<FqInl>(fq2_add(p.x, B)), A), C);
  D = fq2_dbl(D);
  const fq2 E = fq2_add(fq2_dbl(A), A);
  const fq2 F = fq2_sqr_t<FqInl>(E);
  const fq2 X3 = fq2_sub(F, fq2_dbl(D));
  const fq2 C8 = fq2_dbl(fq2_dbl(fq2_dbl(C)));
  const fq2 Y3 = fq2_sub(fq2_mul_t<FqInl>(E, fq2_sub(D, X3)), C8);
  const fq2 Z3 = fq2_dbl(fq2_mul_t<FqInl>(p.y, p.z));
  return g2j{X3, Y3, Z3};
}

HBX_HDNI g2j g2_add(const g2j& p, const g2j& q) {
  if (g2j_is_identity(p)) return q;
  if (g2j_is_identity(q)) return p;
  const fq2 Z1Z1 = fq2_sqr_t<FqInl>(p.z);
  const fq2 Z2Z2 = fq2_sqr_t<FqInl>(q.z);
  const fq2 U1 = fq2_mul_t<FqInl>(p.x, Z2Z2);
  const fq2 U2 = fq2_mul_t<FqInl>(q.x, Z1Z1);
  const fq2 S1 = fq2_mul_t<FqInl>(fq2_mul_t<FqInl>(p.y, q.z), Z2Z2);
  const fq2 S2 = fq2_mul_t<FqInl>(fq2_mul_t<FqInl>(q.y, p.z), Z1Z1);
  if (fq2_eq(U1, U2)) {
    if (fq2_eq(S1, S2)) return g2_dbl(p);
    return g2_identity();
  }
  const fq2 H = fq2_sub(U2, U1);
  const fq2 I = fq2_sqr_t<FqInl>(fq2_dbl(H));
  const fq2 J = fq2_mul_t<FqInl>(H, I);
  const fq2 r = fq2_dbl(fq2_sub(S2, S1));
  const fq2 V = fq2_mul_t<FqInl>(U1, I);
  const fq2 X3 = fq2_sub(fq2_sub(fq2_sqr_t<FqInl>(r), J), fq2_dbl(V));
  const fq2 Y3 = fq2_sub(fq2_mul_t<FqInl>(r, fq2_sub(V, X3)), fq2_dbl(fq2_mul_t<FqInl>(S1, J)));
  const fq2 Z3 = fq2_mul_t<FqInl>(fq2_sub(fq2_sub(fq2_sqr_t<FqInl>(fq2_add(p.z, q.z)), Z1Z1), Z2Z2), H);
  return g2j{X3, Y3, Z3};
}

HBX_HD g2j g2_neg(const g2j& p) { return g2j{p.x, fq2_neg(p.y), p.z}; }

// p + q for an affine q (Z2 = 1): 7M + 4S instead of 12M + 4S.
HBX_HDNI g2j g2_add_mixed(const g2j& p, const g2a& q) {
  if (q.inf) return p;
  if (g2j_is_identity(p)) return g2j{q.x, q.y, fq2_one()};
  const fq2 Z1Z1 = fq2_sqr_t<FqInl>(p.z);
  const fq2 U2 = fq2_mul_t<FqInl>(q.x, Z1Z1);
  const fq2 S2 = fq2_mul_t<FqInl>(fq2_mul_t<FqInl>(q.y, p.z), Z1Z1);
  if (fq2_eq(p.x, U2)) {
    if (fq2_eq(p.y, S2)) return g2_dbl(p);
    return g2_identity();
  }
  const fq2 H = fq2_sub(U2, p.x);
  const fq2 HH = fq2_sqr_t<FqInl>(H);
  const fq2 I = fq2_dbl(fq2_dbl(HH));
  const fq2 J = fq2_mul_t<FqInl>(H, I);
  const fq2 r = fq2_dbl(fq2_sub(S2, p.y));
  const fq2 V = fq2_mul_t<FqInl>(p.x, I);
  const fq2 X3 = fq2_sub(fq2_sub(fq2_sqr_t<FqInl>(r), J), fq2_dbl(V));
  const fq2 Y3 = fq2_sub(fq2_mul_t<FqInl>(r, fq2_sub(V, X3)), fq2_dbl(fq2_mul_t<FqInl>(p.y, J)));
  const fq2 Z3 = fq2_sub(fq2_sub(fq2_sqr_t<FqInl>(fq2_add(p.z, H)), Z1Z1), HH);
  return g2j{X3, Y3, Z3};
}

// k P for a 64-bit k and an affine P, left to right over the non-adjacent form of k (65 digits,
// about a third nonzero; the negation of an affine point is free).  One addition site per digit
// with the point selected by sign, so lanes with different scalars share it.
HBX_HDNI g2j g2_mul_u64_naf(const g2a& P, uint64_t k) {
  // NAF(k): c = 3k (66 bits as hi:lo), np = c ^ k; digit i is +1 where bit i+1 of np & c is
  // set, -1 where bit i+1 of np & k is set
  const uint64_t lo = k + (k << 1);
  const uint64_t hi = (k >> 63) + (lo < k ? 1u : 0u);  // carry of k + 2k into bit 64
  const uint64_t np_lo = lo ^ k, np_hi = hi;           // k has no bits >= 64
  const uint64_t pos_lo = np_lo & lo, pos_hi = np_hi & hi;
  const uint64_t neg_lo = np_lo & k;
  g2a negP = P;
  negP.y = fq2_neg(P.y);
  g2j acc = g2_identity();
  for (int i = 65; i >= 0; i--) {  // bit i+1 of the masks <-> digit i
    const int b = i + 1;
    const bool pos = b >= 64 ? ((pos_hi >> (b - 64)) & 1) != 0 : ((pos_lo >> b) & 1) != 0;
    const bool neg = b >= 64 ? false : ((neg_lo >> b) & 1) != 0;
    if (!g2j_is_identity(acc)) acc = g2_dbl(acc);
    if (pos || neg) acc = g2_add_mixed(acc, neg ? negP : P);
  }
  return acc;
}

// k P for a 64-bit k and an affine P by 4-bit fixed windows (g1_mul_u64_w4's schedule in G2): a
// table (0..15) P in per-lane scratch, then 15 x (4 doublings + 1 addition).  Every lane adds its
// own table entry once per window, so a wave of lanes with different scalars issues 15 additions
// -- g2_mul_u64_naf's addition site is taken whenever ANY lane has a nonzero digit (~66 additions
// per wave): k_combine_sigs' 64-bit multiplications 5.3 -> ~3.5 ms at one wave per SIMD
// (tools/microbench/combsig.hip).
HBX_HDNI g2j g2_mul_u64_w4(const g2a& P, uint64_t k) {
  g2j tab[16];
  tab[0] = g2_identity();
  tab[1] = g2_from_affine(P);
#pragma unroll 1
  for (int i = 2; i < 16; i++) tab[i] = g2_add_mixed(tab[i - 1], P);
  g2j acc = tab[k >> 60];
  g2j nxt = tab[(k >> 56) & 0xFu];
#pragma unroll 1
  for (int w = 14; w >= 0; w--) {
    const g2j cur = nxt;
    if (w > 0) nxt = tab[(k >> (4 * (w - 1))) & 0xFu];
#pragma unroll 1
    for (int q = 0; q < 4; q++) acc = g2_dbl(acc);
    acc = g2_add(acc, cur);
  }
  return acc;
}

HBX_HDNI g2a g2_to_affine(const g2j& p) {
  g2a r;
  if (g2j_is_identity(p)) {
    r.x = fq2_zero();
    r.y = fq2_zero();
    r.inf = true;
    return r;
  }
  const fq2 zi = fq2_inv(p.z);
  const fq2 zi2 = fq2_sqr(zi);
  r.x = fq2_mul(p.x, zi2);
  r.y = fq2_mul(fq2_mul(p.y, zi2), zi);
  r.inf = false;
  return r;
}

// Scalar given as little-endian 32-bit limbs with an explicit bit length.
HBX_HDNI g2j g2_mul_bits(const g2j& p, const uint32_t* k, int nbits) {
  g2j acc = g2_identity();
  bool started = false;
  for (int i = nbits - 1; i >= 0; i--) {
    if (started) acc = g2_dbl(acc);
    if ((k[i >> 5] >> (i & 31)) & 1) {
      acc = started ? g2_add(acc, p) : p;
      started = true;
    }
  }
  return acc;
}

HBX_HD g2j g2_sub(const g2j& p, const g2j& q) { return g2_add(p, g2_neg(q)); }

// k * P for a 64-bit k > 0 (left-to-right double-and-add)
HBX_HDNI g2j g2_mul_u64(const g2j& p, uint64_t k) {
  g2j acc = p;
  const int top = 63 - __builtin_clzll(k);
  for (int i = top - 1; i >= 0; i--) {
    acc = g2_dbl(acc);
    if ((k >> i) & 1) acc = g2_add(acc, p);
  }
  return acc;
}

HBX_HD g2j g2_dbl_n(g2j p, int n) {
  for (int i = 0; i < n; i++) p = g2_dbl(p);
  return p;
}
// [D] P for D = GLS_D = 0x4600_5555_5555_AAAB by its 16-bit digits: with Z = 0x5555 P
// (= 5 * 17 * 257 P) and W = 0xAAAB P = 2Z + P,  D P = ((70 P * 2^8 * 2^16 + Z) 2^16 + Z) 2^16 + W.
// 77 doublings + 9 additions instead of 62 + 27 for binary double-and-add (an addition costs
// ~2.7 doublings).
HBX_HDNI g2j g2_mul_gls_d(const g2j& P) {
  static_assert(GLS_D == 0x460055555555aaabull, "addition chain is specific to D");
  const g2j P2 = g2_dbl(P);
  const g2j P4 = g2_dbl(P2);
  g2j Z = g2_add(P4, P);                 // 5P
  Z = g2_add(g2_dbl_n(Z, 4), Z);         // 0x55 P
  Z = g2_add(g2_dbl_n(Z, 8), Z);         // 0x5555 P
  const g2j W = g2_add(g2_dbl(Z), P);    // 0xAAAB P
  g2j acc = g2_add(g2_dbl_n(P2, 3), P);  // 17 P
  acc = g2_add(g2_dbl(acc), P);          // 35 P
  acc = g2_dbl_n(acc, 1 + 8 + 16);       // 0x4600 P << 16
  acc = g2_add(acc, Z);
  acc = g2_add(g2_dbl_n(acc, 16), Z);
  return g2_add(g2_dbl_n(acc, 16), W);
}

// psi(x, y) = (C1 conj(x), C2 conj(y)) on E'(Fq2), in Jacobian form (conj(Z) keeps x = X/Z^2).
HBX_HD g2j g2_psi(const g2j& p) {
  const fq2 c1 = fq2{fq_from_const(PSI_C1_0), fq_from_const(PSI_C1_1)};
  const fq2 c2 = fq2{fq_from_const(PSI_C2_0), fq_from_const(PSI_C2_1)};
  return g2j{fq2_mul(fq2_conj(p.x), c1), fq2_mul(fq2_conj(p.y), c2), fq2_conj(p.z)};
}

// h2 * P for any P on E'(Fq2) -- the value pairing 0.14's scale_by_cofactor computes with a
// 507-bit double-and-add, here in ~4x fewer operations:
//   Q = h_eff P by the psi formula of Budroni-Pintore / IETF hash-to-curve, h_eff = 3(x^2-1) h2;
//   h2 P = s Q with s = (3(x^2-1))^-1 mod r = D (1 + x - x^2 - x^3), psi = [x] on G2 (Q in G2).
// Q = h_eff P (the first half of g2_clear_cofactor)
HBX_HDNI g2j g2_heff(const g2j& P) {
  const g2j t1 = g2_neg(g2_mul_u64(P, BLS_X));  // [x] P, x = -|x|
  g2j t2 = g2_psi(P);
  g2j t3 = g2_psi(g2_psi(g2_dbl(P)));
  t3 = g2_sub(t3, t2);
  t2 = g2_add(t1, t2);
  t2 = g2_neg(g2_mul_u64(t2, BLS_X));
  t3 = g2_add(t3, t2);
  t3 = g2_sub(t3, t1);
  return g2_sub(t3, P);
}
// h2 P from Q = h_eff P (the second half): s Q, s = (3(x^2-1))^-1 mod r
HBX_HDNI g2j g2_heff_to_h2(const g2j& Q) {
  const g2j q1 = g2_psi(Q);
  const g2j q2 = g2_psi(q1);
  const g2j q3 = g2_psi(q2);
  const g2j Rp = g2_sub(g2_sub(g2_add(Q, q1), q2), q3);
  return g2_mul_gls_d(Rp);
}
HBX_HDNI g2j g2_clear_cofactor(const g2j& P) {
  const g2j Q = g2_heff(P);
  const g2j q1 = g2_psi(Q);
  const g2j q2 = g2_psi(q1);
  const g2j q3 = g2_psi(q2);
  const g2j Rp = g2_sub(g2_sub(g2_add(Q, q1), q2), q3);
  return g2_mul_gls_d(Rp);
}

// Jacobian equality (identities included).
// Jacobian equality in G1 (X1 Z2^2 == X2 Z1^2 and Y1 Z2^3 == Y2 Z1^3, identities apart)
HBX_HD bool g1j_eq(const g1j& a, const g1j& b) {
  const bool ia = g1j_is_identity(a), ib = g1j_is_identity(b);
  if (ia || ib) return ia && ib;
  const fq za2 = fq_sqr(a.z), zb2 = fq_sqr(b.z);
  if (!fq_eq(fq_mul(a.x, zb2), fq_mul(b.x, za2))) return false;
  return fq_eq(fq_mul(a.y, fq_mul(zb2, b.z)), fq_mul(b.y, fq_mul(za2, a.z)));
}
// k P for a small scalar (Horner steps of the bivariate commitment evaluation): left-to-right
// double-and-add on a Jacobian base
HBX_HDNI g1j g1j_mul_u64(const g1j& p, uint64_t k) {
  if (k == 0 || g1j_is_identity(p)) return g1_identity();
  g1j acc = p;
  const int top = 63 - __builtin_clzll(k);
#pragma unroll 1
  for (int i = top - 1; i >= 0; i--) {
    acc = g1_dbl_i(acc);
    if ((k >> i) & 1) acc = g1_add_i(acc, p);
  }
  return acc;
}

HBX_HD bool g2j_eq(const g2j& a, const g2j& b) {
  const bool ia = g2j_is_identity(a), ib = g2j_is_identity(b);
  if (ia || ib) return ia && ib;
  const fq2 za2 = fq2_sqr(a.z), zb2 = fq2_sqr(b.z);
  if (!fq2_eq(fq2_mul(a.x, zb2), fq2_mul(b.x, za2))) return false;
  return fq2_eq(fq2_mul(a.y, fq2_mul(zb2, b.z)), fq2_mul(b.y, fq2_mul(za2, a.z)));
}

// Q in G2 for an affine point on the twist (pairing's into_affine subgroup check).  Criterion
// (eprint 2021/1130 sec. 4, proof in 2022/352): psi(Q) == [x] Q -- one 64-bit multiplication.
HBX_HDNI bool g2_is_torsion_free(const g2a& Q) {
  if (Q.inf) return true;
  const g2j q = g2_from_affine(Q);
  return g2j_eq(g2_neg(g2_mul_u64(q, BLS_X)), g2_psi(q));  // [x] Q with x = -|x|
}

// zcash compressed G2 (x.c1 || x.c0) -> affine (Montgomery).  No subgroup check here; the
// ciphertext decode (k_prepare_ct) adds g2_is_torsion_free.
HBX_HDNI int32_t g2_decompress(const uint8_t* b96, g2a& out) {
  const uint8_t flags = b96[0];
  out.inf = false;
  if (!(flags & 0x80)) return HBX_PT_BAD_FLAGS;
  if (flags & 0x40) {
    bool clean = !(flags & 0x20) && !(flags & 0x1F);
    for (int i = 1; i < 96; i++) clean = clean && b96[i] == 0;
    if (!clean) return HBX_PT_BAD_FLAGS;
    out.x = fq2_zero();
    out.y = fq2_zero();
    out.inf = true;
    return HBX_PT_INFINITY;
  }
  uint8_t tmp[48];
  for (int i = 0; i < 48; i++) tmp[i] = b96[i];
  tmp[0] &= 0x1F;
  const fq x1c = fq_from_be(tmp);
  const fq x0c = fq_from_be(b96 + 48);
  if (!fq_lt_p(x1c) || !fq_lt_p(x0c)) return HBX_PT_NOT_IN_FIELD;
  const fq2 x = fq2{fq_to_mont(x0c), fq_to_mont(x1c)};
  const fq2 rhs = fq2_add(fq2_mul(fq2_sqr(x), x), g2_b());
  fq2 y;
  if (!fq2_sqrt(rhs, y)) return HBX_PT_NOT_ON_CURVE;
  if (fq2_lex_largest(y) != ((flags & 0x20) != 0)) y = fq2_neg(y);
  out.x = x;
  out.y = y;
  return HBX_PT_OK;
}

HBX_HD void g2_compress(const g2a& p, uint8_t* b96) {
  if (p.inf) {
    for (int i = 0; i < 96; i++) b96[i] = 0;
    b96[0] = 0xC0;
    return;
  }
  fq_to_be(fq_from_mont(p.x.c1), b96);
  fq_to_be(fq_from_mont(p.x.c0), b96 + 48);
  b96[0] |= 0x80;
  if (fq2_lex_largest(p.y)) b96[0] |= 0x20;
}

// Uncompressed G2 (x.c1 || x.c0 || y.c1 || y.c0), as Signature::parity reads it.
HBX_HD void g2_uncompressed(const g2a& p, uint8_t* b192) {
  if (p.inf) {
    for (int i = 0; i < 192; i++) b192[i] = 0;
    b192[0] = 0x40;
    return;
  }
  fq_to_be(fq_from_mont(p.x.c1), b192);
  fq_to_be(fq_from_mont(p.x.c0), b192 + 48);
  fq_to_be(fq_from_mont(p.y.c1), b192 + 96);
  fq_to_be(fq_from_mont(p.y.c0), b192 + 144);
}

}  // namespace hbx
