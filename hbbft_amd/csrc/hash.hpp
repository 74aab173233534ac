// Byte-level primitives on the hot path:
//  * SHA-256 (FIPS 180-4) -- the digest threshold_crypto applies inside hash_g2 / hash_g1_g2 /
//    hash_bytes (DIGEST default = SHA-256, the reference's own `ring`
//    dependency, Cargo.toml:32) and the Merkle hash of broadcast.rs:381/:683;
//  * SHA3-256 (FIPS 202) -- the opt-in DIGEST variant (tiny-keccak) and the SHA3 Merkle variant;
//  * ChaCha20 as `rand 0.4` ChaChaRng emits it (Cargo.toml:29): key = 8 seed words, 128-bit
//    block counter in words 12..15, words returned in block order, next_u64 = hi<<32 | lo;
//  * hash_g2 / hash_g1_g2 (threshold_crypto): digest -> 8 big-endian seed words -> ChaChaRng ->
//    pairing 0.14 `G2::rand` (Fq2 sampled in raw Montgomery representation, bool `greatest`,
//    lift, multiply by the full cofactor h2, retry).
#pragma once
#include "curve.hpp"
#include "fieldd.hpp"
#include "dpp.hpp"
#include "groupd.hpp"

namespace hbx {

// ----------------------------------------------------------------------------------------------
// SHA-256
// ----------------------------------------------------------------------------------------------
HBX_CONST uint32_t SHA256_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

HBX_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
HBX_HD uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
// SHA-2 Ch / Maj and a three-way XOR: one v_bitop3_b32 each on the device (truth tables 0xCA,
// 0xE8, 0x96; the compiler builds Maj from three ops), plain logic in the host build
HBX_HD uint32_t sha_ch(uint32_t e, uint32_t f, uint32_t g) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
#else
  return (e & f) ^ (~e & g);
#endif
}
HBX_HD uint32_t sha_maj(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
#else
  return (a & b) ^ (a & c) ^ (b & c);
#endif
}
HBX_HD uint32_t sha_xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

struct sha256_state {
  uint32_t h[8];
};

HBX_HD void sha256_init(sha256_state& s) {
  s.h[0] = 0x6a09e667u; s.h[1] = 0xbb67ae85u; s.h[2] = 0x3c6ef372u; s.h[3] = 0xa54ff53au;
  s.h[4] = 0x510e527fu; s.h[5] = 0x9b05688cu; s.h[6] = 0x1f83d9abu; s.h[7] = 0x5be0cd19u;
}

// One compression over 16 big-endian message words (inlined form: the Merkle node hash, whose
// second block is constant but for one word, folds its schedule; sha256_compress is the call).
HBX_HD void sha256_compress_il(sha256_state& s, const uint32_t* w16) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = w16[i];
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      const uint32_t s0 = sha_xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
      const uint32_t s1 = sha_xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
      wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
      w[i & 15] = wi;
    }
    const uint32_t S1 = sha_xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
    const uint32_t ch = sha_ch(e, f, g);
    const uint32_t t1 = h + SHA256_K[i] + wi + S1 + ch;
    const uint32_t S0 = sha_xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
    const uint32_t mj = sha_maj(a, b, c);
    const uint32_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
  s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}
HBX_HDNI void sha256_compress(sha256_state& s, const uint32_t* w16) { sha256_compress_il(s, w16); }

// Streaming SHA-256 over a concatenation of up to two byte ranges (enough for hash_g1_g2's
// "message || compress(g1)"), one lane.  Output: 32-byte digest.
HBX_HD void sha256_2(const uint8_t* m0, uint64_t n0, const uint8_t* m1, uint64_t n1, uint8_t* out32) {
  sha256_state s;
  sha256_init(s);
  const uint64_t total = n0 + n1;
  const uint64_t nblocks = (total + 9 + 63) / 64;
  for (uint64_t blk = 0; blk < nblocks; blk++) {
    uint32_t w[16];
    for (int i = 0; i < 16; i++) {
      uint32_t word = 0;
      for (int k = 0; k < 4; k++) {
        const uint64_t pos = blk * 64 + (uint64_t)(4 * i + k);
        uint8_t byte;
        if (pos < n0) byte = m0[pos];
        else if (pos < total) byte = m1[pos - n0];
        else if (pos == total) byte = 0x80;
        else if (pos >= nblocks * 64 - 8) byte = (uint8_t)((total * 8) >> (8 * (nblocks * 64 - 1 - pos)));
        else byte = 0;
        word = (word << 8) | byte;
      }
      w[i] = word;
    }
    sha256_compress(s, w);
  }
  for (int i = 0; i < 8; i++) {
    out32[4 * i] = (uint8_t)(s.h[i] >> 24);
    out32[4 * i + 1] = (uint8_t)(s.h[i] >> 16);
    out32[4 * i + 2] = (uint8_t)(s.h[i] >> 8);
    out32[4 * i + 3] = (uint8_t)s.h[i];
  }
}

// ----------------------------------------------------------------------------------------------
// SHA3-256 (FIPS 202): Keccak-f[1600], rate 136 bytes, domain padding 0x06 .. 0x80.
// The opt-in DIGEST of SURVEY.md App. A.3: threshold_crypto revisions that hash with tiny-keccak's
// sha3_256 instead of SHA-256 (reference Cargo.toml:35 pins no revision), and the digest of the
// SHA3 Merkle variant (later hbbft's src/broadcast/merkle.rs).  State: 25 x u64 lanes in
// registers; every 64-bit rotate is two v_alignbit_b32.
// ----------------------------------------------------------------------------------------------
HBX_CONST uint64_t KECCAK_RC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

HBX_HD uint64_t rotl64(uint64_t x, int n) { return n == 0 ? x : (x << n) | (x >> (64 - n)); }

// Keccak-f[1600] on a[5 * y + x].
HBX_HDNI void keccak_f1600(uint64_t* st) {
  uint64_t a[25];
#pragma unroll
  for (int i = 0; i < 25; i++) a[i] = st[i];
  // rho offsets and the pi permutation as one table: b[pi(i)] = rotl(a[i], rho(i))
  constexpr int RHO[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
#pragma unroll 1
  for (int r = 0; r < 24; r++) {
    uint64_t c[5], b[25];
#pragma unroll
    for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
#pragma unroll
    for (int x = 0; x < 5; x++) {
      const uint64_t d = c[(x + 4) % 5] ^ rotl64(c[(x + 1) % 5], 1);
#pragma unroll
      for (int y = 0; y < 5; y++) a[5 * y + x] ^= d;
    }
#pragma unroll
    for (int x = 0; x < 5; x++)
#pragma unroll
      for (int y = 0; y < 5; y++) {
        // (x, y) -> (y, 2x + 3y)
        const int X = y, Y = (2 * x + 3 * y) % 5;
        b[5 * Y + X] = rotl64(a[5 * y + x], RHO[5 * y + x]);
      }
#pragma unroll
    for (int y = 0; y < 5; y++)
#pragma unroll
      for (int x = 0; x < 5; x++) a[5 * y + x] = b[5 * y + x] ^ (~b[5 * y + (x + 1) % 5] & b[5 * y + (x + 2) % 5]);
    a[0] ^= KECCAK_RC[r];
  }
#pragma unroll
  for (int i = 0; i < 25; i++) st[i] = a[i];
}

// SHA3-256 over a concatenation of up to two byte ranges (like sha256_2), one lane.
HBX_HD void sha3_256_2(const uint8_t* m0, uint64_t n0, const uint8_t* m1, uint64_t n1, uint8_t* out32) {
  uint64_t st[25];
#pragma unroll
  for (int i = 0; i < 25; i++) st[i] = 0;
  const uint64_t total = n0 + n1;
  const uint64_t nblocks = total / 136 + 1;  // the padding always fits the last block (>= 1 byte)
  for (uint64_t blk = 0; blk < nblocks; blk++) {
    for (int i = 0; i < 17; i++) {
      uint64_t lane = 0;
      for (int k = 0; k < 8; k++) {
        const uint64_t pos = blk * 136 + (uint64_t)(8 * i + k);
        uint8_t byte;
        if (pos < n0) byte = m0[pos];
        else if (pos < total) byte = m1[pos - n0];
        else byte = 0;
        if (pos == total) byte ^= 0x06;
        if (blk == nblocks - 1 && 8 * i + k == 135) byte ^= 0x80;
        lane |= (uint64_t)byte << (8 * k);
      }
      st[i] ^= lane;
    }
    keccak_f1600(st);
  }
  for (int i = 0; i < 32; i++) out32[i] = (uint8_t)(st[i >> 3] >> (8 * (i & 7)));
}

// The DIGEST of threshold_crypto's hash_g2 / hash_g1_g2 / hash_bytes (include/hbx.h
// HBX_DIGEST_*): a per-context switch, SHA-256 by default.
constexpr int DIGEST_SHA256 = 0;
constexpr int DIGEST_SHA3_256 = 1;
HBX_HD void digest2(int variant, const uint8_t* m0, uint64_t n0, const uint8_t* m1, uint64_t n1, uint8_t* out32) {
  if (variant == DIGEST_SHA3_256) sha3_256_2(m0, n0, m1, n1, out32);
  else sha256_2(m0, n0, m1, n1, out32);
}

// ----------------------------------------------------------------------------------------------
// ChaCha20 / rand 0.4 ChaChaRng
// ----------------------------------------------------------------------------------------------
#define HBX_QR(a, b, c, d)       \
  a += b; d = rotl32(d ^ a, 16); \
  c += d; b = rotl32(b ^ c, 12); \
  a += b; d = rotl32(d ^ a, 8);  \
  c += d; b = rotl32(b ^ c, 7);

// One 16-word output block for key words k[8] and 128-bit counter (ctr_lo, ctr_hi).
HBX_HDNI void chacha20_block(const uint32_t* k, uint64_t ctr_lo, uint64_t ctr_hi, uint32_t* out16) {
  uint32_t st[16] = {0x61707865u, 0x3320646Eu, 0x79622D32u, 0x6B206574u, k[0], k[1], k[2], k[3],
                     k[4], k[5], k[6], k[7], (uint32_t)ctr_lo, (uint32_t)(ctr_lo >> 32),
                     (uint32_t)ctr_hi, (uint32_t)(ctr_hi >> 32)};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = st[i];
#pragma unroll
  for (int r = 0; r < 10; r++) {
    HBX_QR(x[0], x[4], x[8], x[12]);
    HBX_QR(x[1], x[5], x[9], x[13]);
    HBX_QR(x[2], x[6], x[10], x[14]);
    HBX_QR(x[3], x[7], x[11], x[15]);
    HBX_QR(x[0], x[5], x[10], x[15]);
    HBX_QR(x[1], x[6], x[11], x[12]);
    HBX_QR(x[2], x[7], x[8], x[13]);
    HBX_QR(x[3], x[4], x[9], x[14]);
  }
#pragma unroll
  for (int i = 0; i < 16; i++) out16[i] = x[i] + st[i];
}

struct chacha_rng {
  uint32_t key[8];
  uint32_t buf[16];
  uint64_t ctr;  // next block number (low 64 bits of the 128-bit counter suffice here)
  int idx;
};

HBX_HD void chacha_rng_from_digest(chacha_rng& r, const uint8_t* d32) {
  for (int i = 0; i < 8; i++)
    r.key[i] = ((uint32_t)d32[4 * i] << 24) | ((uint32_t)d32[4 * i + 1] << 16) |
               ((uint32_t)d32[4 * i + 2] << 8) | d32[4 * i + 3];
  r.ctr = 0;
  r.idx = 16;
}
HBX_HD uint32_t chacha_next_u32(chacha_rng& r) {
  if (r.idx == 16) {
    chacha20_block(r.key, r.ctr, 0, r.buf);
    r.ctr++;
    r.idx = 0;
  }
  return r.buf[r.idx++];
}
HBX_HD uint64_t chacha_next_u64(chacha_rng& r) {
  const uint64_t hi = chacha_next_u32(r);
  const uint64_t lo = chacha_next_u32(r);
  return (hi << 32) | lo;
}

// pairing 0.14 `Fq::rand`: 6 x next_u64 limbs, top limb masked to 61 bits, rejection-sampled,
// the raw limbs ARE the Montgomery representation.
HBX_HD fq fq_rand(chacha_rng& r) {
  for (;;) {
    fq v;
    for (int i = 0; i < 6; i++) {
      const uint64_t w = chacha_next_u64(r);
      v.l[2 * i] = (uint32_t)w;
      v.l[2 * i + 1] = (uint32_t)(w >> 32);
    }
    v.l[11] &= 0x1FFFFFFFu;
    if (fq_lt_p(v)) return v;
  }
}

// G2::rand + scale_by_cofactor (h2 * P; computed by g2_clear_cofactor, same point).
// SIMT shape: the rejection loop only draws x and runs the residuosity test (one Fq
// exponentiation per draw); the square root and the cofactor clearing run once, after every
// lane of the wave has found its point, instead of once per loop trip inside the divergent loop.
HBX_HDNI g2j g2_rand_from_rng(chacha_rng& r) {
  for (;;) {
    fq2 x, rhs;
    fq s;
    bool greatest;
    for (;;) {
      const fq c0 = fq_rand(r);
      const fq c1 = fq_rand(r);
      x = fq2{c0, c1};
      greatest = (chacha_next_u32(r) & 1u) != 0;
      rhs = fq2_add(fq2_mul(fq2_sqr(x), x), g2_b());
      if (fq_is_zero(rhs.c1)) {
        // measure-zero branch (x^3 + b in Fq); handled exactly by the general square root
        fq2 y0;
        if (fq2_sqrt(rhs, y0)) break;
        continue;
      }
      if (fq2_norm_sqrt(rhs, s)) break;
    }
    fq2 y;
    if (fq_is_zero(rhs.c1)) fq2_sqrt(rhs, y);
    else y = fq2_sqrt_from_norm(rhs, s);
    // pairing: y if (y < -y) ^ greatest else -y  ==  pick the larger root iff greatest
    if (fq2_lex_largest(y) != greatest) y = fq2_neg(y);
    const g2j p = g2_clear_cofactor(g2j{x, y, fq2_one()});
    if (!g2j_is_identity(p)) return p;
  }
}

#if defined(__HIPCC__)
// ---- group-cooperative G2 doubling for the cofactor clearing --------------------------------
// The cofactor clearing is ~200 sequential doublings on one point: a latency chain, run by one
// lane per proposer while the other lanes of its hash group idle.  Here the 8 lanes of the group
// (all holding the same point) split each doubling's 16 Fq products into three rounds of
// independent products, one per lane, exchanged through ds_bpermute (__shfl).  Same formulas
// as g2_dbl (dbl-2009-l); Fq2 products by schoolbook (four Fq products on four lanes), so the
// coordinates are equal mod p to g2_dbl's.  Control flow must be group-uniform.
__device__ __forceinline__ fq fq_from_lane(const fq& v, int src) {
  fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = (uint32_t)__shfl((int)v.l[i], src, 64);
  return r;
}
// Lane K of the calling lane's 16-lane row (= its group: groups here are 16 aligned lanes), to
// every lane of the row: a DPP row_newbcast move per limb -- VALU, no LDS round trip as with
// __shfl.  K must be a constant; all 16 lanes of the row must be active.
template <int K>
__device__ __forceinline__ fq fq_from_row(const fq& v) {
  static_assert(K >= 0 && K < 16, "row lane");
  dpp_guard_src<16, K>();
  fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.l[i], 0x150 + K, 0xf, 0xf, false);
  return r;
}
__device__ __forceinline__ fq fq_sel8(int s, const fq& v0, const fq& v1, const fq& v2, const fq& v3, const fq& v4,
                                      const fq& v5, const fq& v6, const fq& v7) {
  fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint32_t lo = (s & 2) ? ((s & 1) ? v3.l[i] : v2.l[i]) : ((s & 1) ? v1.l[i] : v0.l[i]);
    const uint32_t hi = (s & 2) ? ((s & 1) ? v7.l[i] : v6.l[i]) : ((s & 1) ? v5.l[i] : v4.l[i]);
    r.l[i] = (s & 4) ? hi : lo;
  }
  return r;
}
__device__ __forceinline__ fq fq_sel16(int s, const fq (&v)[16]) {
  fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint32_t t = v[0].l[i];
#pragma unroll
    for (int k = 1; k < 16; k++) t = (s == k) ? v[k].l[i] : t;
    r.l[i] = t;
  }
  return r;
}

#ifndef HBX_DBL_MARK
#define HBX_DBL_MARK(k)  // timing hooks (tools/microbench/dblstamp.hip: clock stamps between the
#define HBX_DBL_USE(v)   // segments; USE pins a product's result before the next stamp)
#endif
__device__ __forceinline__ g2j g2_dbl_group(const g2j& p, int gl, int gbase) {
  const int s = gl & 7;
  const fq x0 = p.x.c0, x1 = p.x.c1, y0 = p.y.c0, y1 = p.y.c1, z0 = p.z.c0, z1 = p.z.c1;
  // round 1: A = X^2 (lanes 0, 1), B = Y^2 (2, 3), Y Z (4..7)
  HBX_DBL_MARK(0);
  const fq a1 = fq_sel8(s, fq_add(x0, x1), x0, fq_add(y0, y1), y0, y0, y1, y0, y1);
  const fq b1 = fq_sel8(s, fq_sub(x0, x1), x1, fq_sub(y0, y1), y1, z0, z1, z1, z0);
  HBX_DBL_USE(a1);
  HBX_DBL_USE(b1);
  HBX_DBL_MARK(1);
  fq r = fq_mul_inl(a1, b1);
  HBX_DBL_USE(r);
  HBX_DBL_MARK(2);
  const fq2 A = fq2{fq_from_row<0>(r), fq_dbl(fq_from_row<1>(r))};
  const fq2 B = fq2{fq_from_row<2>(r), fq_dbl(fq_from_row<3>(r))};
  const fq2 YZ = fq2{fq_sub(fq_from_row<4>(r), fq_from_row<5>(r)),
                     fq_add(fq_from_row<6>(r), fq_from_row<7>(r))};
  // round 2: C = B^2 (0, 1), T = (X + B)^2 (2, 3), F = E^2 with E = 3A (4, 5)
  const fq2 S = fq2_add(p.x, B);
  const fq2 E = fq2_add(fq2_dbl(A), A);
  const fq a2 = fq_sel8(s, fq_add(B.c0, B.c1), B.c0, fq_add(S.c0, S.c1), S.c0, fq_add(E.c0, E.c1), E.c0, E.c0, E.c0);
  const fq b2 = fq_sel8(s, fq_sub(B.c0, B.c1), B.c1, fq_sub(S.c0, S.c1), S.c1, fq_sub(E.c0, E.c1), E.c1, E.c1, E.c1);
  HBX_DBL_USE(a2);
  HBX_DBL_USE(b2);
  HBX_DBL_MARK(3);
  r = fq_mul_inl(a2, b2);
  HBX_DBL_USE(r);
  HBX_DBL_MARK(4);
  const fq2 C = fq2{fq_from_row<0>(r), fq_dbl(fq_from_row<1>(r))};
  const fq2 T = fq2{fq_from_row<2>(r), fq_dbl(fq_from_row<3>(r))};
  const fq2 F = fq2{fq_from_row<4>(r), fq_dbl(fq_from_row<5>(r))};
  const fq2 D = fq2_dbl(fq2_sub(fq2_sub(T, A), C));
  const fq2 X3 = fq2_sub(F, fq2_dbl(D));
  // round 3: E (D - X3) (0..3)
  const fq2 G = fq2_sub(D, X3);
  const fq a3 = fq_sel8(s, E.c0, E.c1, E.c0, E.c1, E.c0, E.c1, E.c0, E.c1);
  const fq b3 = fq_sel8(s, G.c0, G.c1, G.c1, G.c0, G.c0, G.c1, G.c1, G.c0);
  HBX_DBL_USE(a3);
  HBX_DBL_USE(b3);
  HBX_DBL_MARK(5);
  r = fq_mul_inl(a3, b3);
  HBX_DBL_USE(r);
  HBX_DBL_MARK(6);
  const fq2 EG = fq2{fq_sub(fq_from_row<0>(r), fq_from_row<1>(r)),
                     fq_add(fq_from_row<2>(r), fq_from_row<3>(r))};
  const fq2 C8 = fq2_dbl(fq2_dbl(fq2_dbl(C)));
  const g2j out{X3, fq2_sub(EG, C8), fq2_dbl(YZ)};
  HBX_DBL_USE(out.x.c0);
  HBX_DBL_USE(out.x.c1);
  HBX_DBL_USE(out.y.c0);
  HBX_DBL_USE(out.y.c1);
  HBX_DBL_USE(out.z.c0);
  HBX_DBL_USE(out.z.c1);
  HBX_DBL_MARK(7);
  return out;
}
__device__ __forceinline__ g2j g2_dbl_n_group(g2j p, int n, int gl, int gbase) {
  for (int i = 0; i < n; i++) p = g2_dbl_group(p, gl, gbase);
  return p;
}
// g2_add (add-2007-bl) on 16 lanes of a group holding the same p and q: its 16 Fq2 products
// (43 Fq products) as five rounds of independent Fq products, one per lane.  Same special cases
// as g2_add (identities, P = Q, P = -Q), decided group-uniformly.
struct round16 {
  fq a[16], b[16];
};
__device__ __forceinline__ void r16_mul(round16& R, int k, const fq2& x, const fq2& y) {
  R.a[k] = x.c0; R.b[k] = y.c0;
  R.a[k + 1] = x.c1; R.b[k + 1] = y.c1;
  R.a[k + 2] = x.c0; R.b[k + 2] = y.c1;
  R.a[k + 3] = x.c1; R.b[k + 3] = y.c0;
}
__device__ __forceinline__ void r16_sqr(round16& R, int k, const fq2& x) {
  R.a[k] = fq_add(x.c0, x.c1); R.b[k] = fq_sub(x.c0, x.c1);
  R.a[k + 1] = x.c0; R.b[k + 1] = x.c1;
}
__device__ __forceinline__ fq r16_run(const round16& R, int gl) { return fq_mul_inl(fq_sel16(gl, R.a), fq_sel16(gl, R.b)); }
template <int K>
__device__ __forceinline__ fq2 r16_get_mul(const fq& r) {
  return fq2{fq_sub(fq_from_row<K>(r), fq_from_row<K + 1>(r)), fq_add(fq_from_row<K + 2>(r), fq_from_row<K + 3>(r))};
}
template <int K>
__device__ __forceinline__ fq2 r16_get_sqr(const fq& r) {
  return fq2{fq_from_row<K>(r), fq_dbl(fq_from_row<K + 1>(r))};
}
__device__ __forceinline__ void r16_clear(round16& R) {
#pragma unroll
  for (int i = 0; i < 16; i++) {
    R.a[i] = fq_zero();
    R.b[i] = fq_zero();
  }
}
__device__ __noinline__ g2j g2_add_group(const g2j& p, const g2j& q, int gl, int gbase) {
  if (g2j_is_identity(p)) return q;
  if (g2j_is_identity(q)) return p;
  round16 R;
  r16_clear(R);
  // round 1: Z1^2, Z2^2, Y1 Z2, Y2 Z1, (Z1 + Z2)^2
  r16_sqr(R, 0, p.z);
  r16_sqr(R, 2, q.z);
  r16_mul(R, 4, p.y, q.z);
  r16_mul(R, 8, q.y, p.z);
  r16_sqr(R, 12, fq2_add(p.z, q.z));
  fq r = r16_run(R, gl);
  const fq2 Z1Z1 = r16_get_sqr<0>(r), Z2Z2 = r16_get_sqr<2>(r);
  const fq2 Y1Z2 = r16_get_mul<4>(r), Y2Z1 = r16_get_mul<8>(r);
  const fq2 ZS = r16_get_sqr<12>(r);
  // round 2: U1, U2, S1, S2
  r16_mul(R, 0, p.x, Z2Z2);
  r16_mul(R, 4, q.x, Z1Z1);
  r16_mul(R, 8, Y1Z2, Z2Z2);
  r16_mul(R, 12, Y2Z1, Z1Z1);
  r = r16_run(R, gl);
  const fq2 U1 = r16_get_mul<0>(r), U2 = r16_get_mul<4>(r);
  const fq2 S1 = r16_get_mul<8>(r), S2 = r16_get_mul<12>(r);
  if (fq2_eq(U1, U2)) {
    if (fq2_eq(S1, S2)) return g2_dbl_group(p, gl, gbase);
    return g2_identity();
  }
  const fq2 H = fq2_sub(U2, U1);
  const fq2 rr = fq2_dbl(fq2_sub(S2, S1));
  // round 3: I = (2H)^2, r^2, Z3 = ((Z1 + Z2)^2 - Z1Z1 - Z2Z2) H
  r16_sqr(R, 0, fq2_dbl(H));
  r16_sqr(R, 2, rr);
  r16_mul(R, 4, fq2_sub(fq2_sub(ZS, Z1Z1), Z2Z2), H);
  r = r16_run(R, gl);
  const fq2 I = r16_get_sqr<0>(r), RR = r16_get_sqr<2>(r), Z3 = r16_get_mul<4>(r);
  // round 4: J = H I, V = U1 I
  r16_mul(R, 0, H, I);
  r16_mul(R, 4, U1, I);
  r = r16_run(R, gl);
  const fq2 J = r16_get_mul<0>(r), V = r16_get_mul<4>(r);
  const fq2 X3 = fq2_sub(fq2_sub(RR, J), fq2_dbl(V));
  // round 5: r (V - X3), S1 J
  r16_mul(R, 0, rr, fq2_sub(V, X3));
  r16_mul(R, 4, S1, J);
  r = r16_run(R, gl);
  const fq2 Y3 = fq2_sub(r16_get_mul<0>(r), fq2_dbl(r16_get_mul<4>(r)));
  return g2j{X3, Y3, Z3};
}
__device__ __forceinline__ g2j g2_sub_group(const g2j& p, const g2j& q, int gl, int gbase) {
  return g2_add_group(p, g2_neg(q), gl, gbase);
}

// g2_mul_u64 / g2_mul_gls_d / g2_clear_cofactor (curve.hpp) with the group doubling and addition
#define GADD(a, b) g2_add_group(a, b, gl, gbase)
#define GSUB(a, b) g2_sub_group(a, b, gl, gbase)
__device__ g2j g2_mul_u64_group(const g2j& p, uint64_t k, int gl, int gbase) {
  g2j acc = p;
  const int top = 63 - __builtin_clzll(k);
  for (int i = top - 1; i >= 0; i--) {
    acc = g2_dbl_group(acc, gl, gbase);
    if ((k >> i) & 1) acc = GADD(acc, p);
  }
  return acc;
}
__device__ g2j g2_mul_gls_d_group(const g2j& P, int gl, int gbase) {
  const g2j P2 = g2_dbl_group(P, gl, gbase);
  const g2j P4 = g2_dbl_group(P2, gl, gbase);
  g2j Z = GADD(P4, P);
  Z = GADD(g2_dbl_n_group(Z, 4, gl, gbase), Z);
  Z = GADD(g2_dbl_n_group(Z, 8, gl, gbase), Z);
  const g2j W = GADD(g2_dbl_group(Z, gl, gbase), P);
  g2j acc = GADD(g2_dbl_n_group(P2, 3, gl, gbase), P);
  acc = GADD(g2_dbl_group(acc, gl, gbase), P);
  acc = g2_dbl_n_group(acc, 1 + 8 + 16, gl, gbase);
  acc = GADD(acc, Z);
  acc = GADD(g2_dbl_n_group(acc, 16, gl, gbase), Z);
  return GADD(g2_dbl_n_group(acc, 16, gl, gbase), W);
}
// full = false stops at Q = h_eff P = [3(x^2-1)] h2 P (k_prepare_ct: the checks carry the factor
// on their G1 side, hbx_api.hip pk_m / G1_MGEN)
__device__ g2j g2_clear_cofactor_group(const g2j& P, int gl, int gbase, bool full = true) {
  const g2j t1 = g2_neg(g2_mul_u64_group(P, BLS_X, gl, gbase));
  g2j t2 = g2_psi(P);
  g2j t3 = g2_psi(g2_psi(g2_dbl_group(P, gl, gbase)));
  t3 = GSUB(t3, t2);
  t2 = GADD(t1, t2);
  t2 = g2_neg(g2_mul_u64_group(t2, BLS_X, gl, gbase));
  t3 = GADD(t3, t2);
  t3 = GSUB(t3, t1);
  const g2j Q = GSUB(t3, P);
  if (!full) return Q;
  const g2j q1 = g2_psi(Q);
  const g2j q2 = g2_psi(q1);
  const g2j q3 = g2_psi(q2);
  const g2j Rp = GSUB(GSUB(GADD(Q, q1), q2), q3);
  return g2_mul_gls_d_group(Rp, gl, gbase);
}
#undef GADD
#undef GSUB

// hash_g2 by a GROUP of K aligned lanes of one wave (K | 64), same point as g2_rand_from_rng.
//
// Why.  One lane per hash leaves a wave waiting for its unluckiest lane: every lane draws
// candidates x from the ChaCha stream until x^3 + b is a square (probability 1/2 each), so a wave
// runs ~log2(64) + 1 residuosity exponentiations instead of the 2 a lane needs on average.  Here
// lane g of the group draws the stream itself (cheap) but tests only candidate base + g, all K tests
// run as ONE exponentiation, and the lowest passing index wins -- exactly the candidate the
// sequential loop would stop at.  Only the winner lane runs the square root and the cofactor
// clearing.  A cleared point equal to the identity makes the sequential loop continue with the next
// candidate; so does this one (base = winner + 1).  `active` must be group-uniform.
// Returns true on the lane that holds the result in `out`.
#ifndef HBX_HASH_GROUPD
#define HBX_HASH_GROUPD 1  // 1: the cofactor clearing in the digit tower (groupd.hpp), 0: 12-limb rounds
#endif
#ifndef HBX_PHASE
#define HBX_PHASE(k)  // profiling hook (tools/microbench/hashg2.hip records wall-clock stamps)
#endif
template <int K>
__device__ bool hash_g2_group(const uint8_t* d32, bool active, g2j& out, bool full = true) {
  static_assert(K >= 8 && K <= 32 && (64 % K) == 0, "group size (the cofactor clearing uses 8 lanes)");
  if (!active) return false;
  const int lane = (int)(threadIdx.x & 63);
  const int gl = lane % K;
  const int gbase = lane - gl;
  const uint64_t gmask = ((1ull << K) - 1) << gbase;
  chacha_rng r;
  chacha_rng_from_digest(r, d32);
  uint32_t drawn = 0, base = 0;
  fq2 x = fq2_zero();
  bool greatest = false;
  for (;;) {
    // draw up to candidate base + gl (monotone: base only grows)
    while (drawn <= base + (uint32_t)gl) {
      const fq c0 = fq_rand(r);
      const fq c1 = fq_rand(r);
      x = fq2{c0, c1};
      greatest = (chacha_next_u32(r) & 1u) != 0;
      drawn++;
    }
    HBX_PHASE(1);
    const fq2 rhs = fq2_add(fq2_mul(fq2_sqr(x), x), g2_b());
    const bool c1zero = fq_is_zero(rhs.c1);
    fq s = fq_zero();
    fq2 y0 = fq2_zero();
    bool sq;
    if (c1zero) sq = fq2_sqrt(rhs, y0);  // measure-zero branch, exact general square root
    else sq = fq2_norm_sqrt_d(rhs, s);
    HBX_PHASE(2);
    const uint64_t pass = __ballot(sq) & gmask;
    if (pass == 0) {
      base += K;
      continue;
    }
    const int win = __builtin_ctzll(pass) - gbase;
    fq2 y = fq2_zero();
    if (gl == win) {
      y = c1zero ? y0 : fq2_sqrt_from_norm_d(rhs, s);
      // pairing: y if (y < -y) ^ greatest else -y  ==  pick the larger root iff greatest
      if (fq2_lex_largest(y) != greatest) y = fq2_neg(y);
    }
    HBX_PHASE(3);
    // the winner's point to every lane of the group, then the cooperative cofactor clearing
    const int src = gbase + win;
    const fq2 xw = fq2{fq_from_lane(x.c0, src), fq_from_lane(x.c1, src)};
    const fq2 yw = fq2{fq_from_lane(y.c0, src), fq_from_lane(y.c1, src)};
#if HBX_HASH_GROUPD
    {
      const fq2d one{fqd_const(FQD_ONE), fqd_zero()};
      out = g2jd_to_g2j(g2d_clear_cofactor_group(g2jd{fq2d_from_fq2(xw), fq2d_from_fq2(yw), one}, gl, full));
    }
#else
    out = g2_clear_cofactor_group(g2j{xw, yw, fq2_one()}, gl, gbase, full);
#endif
    HBX_PHASE(4);
    const bool ident = g2j_is_identity(out);
    if ((__ballot(ident) & gmask) == 0) return gl == win;
    base += (uint32_t)win + 1;
  }
}
#endif

// hash_g2(digest) where the digest is already computed.
HBX_HD g2j hash_g2_from_digest(const uint8_t* d32) {
  chacha_rng r;
  chacha_rng_from_digest(r, d32);
  return g2_rand_from_rng(r);
}

// hash_g1_g2(u, v): m = (|v| > 64 ? DIGEST(v) : v) || u_comp48; H = hash_g2(m), whose seed is
// DIGEST(m).
HBX_HD void hash_g1_g2_digest(const uint8_t* u_comp48, const uint8_t* v, uint64_t vlen, uint8_t* d,
                              int variant = DIGEST_SHA256) {
  if (vlen > 64) {
    uint8_t dv[32];
    digest2(variant, v, vlen, nullptr, 0, dv);
    digest2(variant, dv, 32, u_comp48, 48, d);
  } else {
    digest2(variant, v, vlen, u_comp48, 48, d);
  }
}
HBX_HD g2j hash_g1_g2(const uint8_t* u_comp48, const uint8_t* v, uint64_t vlen, int variant = DIGEST_SHA256) {
  uint8_t d[32];
  hash_g1_g2_digest(u_comp48, v, vlen, d, variant);
  return hash_g2_from_digest(d);
}

}  // namespace hbx
