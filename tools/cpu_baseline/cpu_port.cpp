// CPU baseline ("port"): threshold_crypto's PublicKeyShare::verify_decryption_share in the shape the
// reference runs it (honey_badger.rs:229 -> threshold_crypto -> pairing 0.14), timed on host cores.
// Per share, exactly as the reference does it:
//   * H = hash_g1_g2(U, V) recomputed for every share, with pairing 0.14's scale_by_cofactor shape
//     (507-bit double-and-add of h2, not the kernels' psi shortcut);
//   * two independent pairings e(S, H) and e(pk_i, W), each = G2 line preparation + Miller loop +
//     its own final exponentiation, compared in Fq12.
// The tower/curve code is the kernels' __host__ __device__ C++ compiled by g++; the Fq product is the
// 6 x 64-bit __int128 CIOS (HBX_HOST_INT128), the limb shape pairing 0.14 uses on x86-64.
// std::thread spreads independent shares over host cores (the reference is single-threaded per
// node; the thread count is reported).  NOT part of the product; built by tools/build.py into
// oracle/_build/ and loaded only by bench.py's cpu_baseline legs.
// Also: the Common Coin's signature-share checks and combine (common_coin.rs:151, :190, :196, :173;
// BASELINE.md §2 row C4) and reed-solomon-erasure 3.1.0's encode / reconstruct by its
// multiplication-table shape (galois_8 MUL_TABLE rows, one byte per lookup; row C5).
#include <atomic>
#include <cstring>
#include <thread>
#define HBX_HOST_INT128 1
#include <vector>
#include "../../hbbft_amd/csrc/pairing.hpp"
#include "../../hbbft_amd/csrc/hash.hpp"
using namespace hbx;

namespace {
// G2::rand + scale_by_cofactor as pairing 0.14 computes it (h2 * P by double-and-add).
g2j g2_rand_reference_shape(chacha_rng& r) {
  for (;;) {
    const fq c0 = fq_rand(r);
    const fq c1 = fq_rand(r);
    const fq2 x{c0, c1};
    const bool greatest = (chacha_next_u32(r) & 1u) != 0;
    const fq2 rhs = fq2_add(fq2_mul(fq2_sqr(x), x), g2_b());
    fq2 y;
    if (!fq2_sqrt(rhs, y)) continue;
    if (fq2_lex_largest(y) != greatest) y = fq2_neg(y);
    const g2j p = g2_mul_bits(g2j{x, y, fq2_one()}, G2_COFACTOR, G2_COFACTOR_BITS);
    if (!g2j_is_identity(p)) return p;
  }
}
fq12 pairing(const g1a& P, const g2a& Q) {
  if (P.inf || Q.inf) return fq12_one();  // e(O, Q) = e(P, O) = 1
  line_pre L[MILLER_LINES];
  fq2 scratch[2 * MILLER_LINES];
  g2_prepare_lines(Q, L, scratch);
  return final_exponentiation(miller_loop2(L, P, true, L, P, false));
}
bool fq12_eq(const fq12& a, const fq12& b) {
  const fq2* x = &a.c0.c0;
  const fq2* y = &b.c0.c0;
  for (int i = 0; i < 6; i++)
    if (!fq2_eq(x[i], y[i])) return false;
  return true;
}
}  // namespace

extern "C" {
// jobs: (proposer j, sender i) pairs.  out[k] = verify_decryption_share result (1/0).
int cpu_verify_dec_shares(const uint8_t* pk48, uint32_t n, const uint8_t* u48, const uint8_t* v_blob,
                          const uint64_t* v_off, const uint8_t* w96, const uint8_t* shares48,
                          const uint32_t* jobs, uint32_t njobs, int threads, uint8_t* out) {
  std::atomic<uint32_t> next{0};
  auto work = [&]() {
    for (;;) {
      const uint32_t k = next.fetch_add(1);
      if (k >= njobs) return;
      const uint32_t j = jobs[2 * k], i = jobs[2 * k + 1];
      g1a pk, S, U;
      g2a W;
      // deserialisation (the identity decodes; HBX_PT_INFINITY sets .inf)
      auto ok1 = [](int st) { return st == HBX_PT_OK || st == HBX_PT_INFINITY; };
      if (!ok1(g1_decompress(pk48 + (size_t)i * 48, pk)) || !ok1(g1_decompress(u48 + (size_t)j * 48, U)) ||
          !ok1(g2_decompress(w96 + (size_t)j * 96, W)) ||
          !ok1(g1_decompress(shares48 + ((size_t)j * n + i) * 48, S))) {
        out[k] = 0;
        continue;
      }
      uint8_t d[32];
      hash_g1_g2_digest(u48 + (size_t)j * 48, v_blob + v_off[j], v_off[j + 1] - v_off[j], d);
      chacha_rng r;
      chacha_rng_from_digest(r, d);
      const g2a H = g2_to_affine(g2_rand_reference_shape(r));
      out[k] = fq12_eq(pairing(S, H), pairing(pk, W)) ? 1 : 0;
    }
  };
  if (threads < 1) threads = 1;
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; t++) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
  return 0;
}

// CPU baseline row (b) of BASELINE.md §2: the same verify_decryption_share bits computed the way
// a CPU implementation would batch them -- H_j = hash_g1_g2(U_j, V_j) hoisted to once per proposer
// (with its Miller lines prepared once, like the kernels' k_prepare_lines), and each share checked
// as e(S, H_j) e(-pk_i, W_j) == 1 with ONE two-pair Miller loop and ONE final exponentiation.
// jobs are (proposer, sender) pairs; the per-proposer preparation of every proposer the jobs touch
// is included in the time (it is part of the work), spread over the same threads.
int cpu_verify_dec_shares_fused(const uint8_t* pk48, uint32_t n, const uint8_t* u48, const uint8_t* v_blob,
                                const uint64_t* v_off, const uint8_t* w96, const uint8_t* shares48, uint32_t p,
                                const uint32_t* jobs, uint32_t njobs, int threads, uint8_t* out) {
  if (threads < 1) threads = 1;
  struct prep {
    bool used = false, ok = false, h_inf = false, w_inf = false;
    std::vector<line_pre> lh, lw;
  };
  std::vector<prep> P(p);
  for (uint32_t k = 0; k < njobs; k++) P[jobs[2 * k]].used = true;
  std::vector<uint32_t> props;
  for (uint32_t j = 0; j < p; j++)
    if (P[j].used) props.push_back(j);
  auto ok1 = [](int st) { return st == HBX_PT_OK || st == HBX_PT_INFINITY; };
  {
    std::atomic<uint32_t> next{0};
    auto work = [&]() {
      for (;;) {
        const uint32_t q = next.fetch_add(1);
        if (q >= props.size()) return;
        const uint32_t j = props[q];
        prep& pr = P[j];
        g1a U;
        g2a W;
        if (!ok1(g1_decompress(u48 + (size_t)j * 48, U)) || !ok1(g2_decompress(w96 + (size_t)j * 96, W))) continue;
        uint8_t d[32];
        hash_g1_g2_digest(u48 + (size_t)j * 48, v_blob + v_off[j], v_off[j + 1] - v_off[j], d);
        const g2a H = g2_to_affine(hash_g2_from_digest(d));
        pr.lh.resize(MILLER_LINES);
        pr.lw.resize(MILLER_LINES);
        fq2 scratch[2 * MILLER_LINES];
        pr.h_inf = H.inf;
        pr.w_inf = W.inf;
        if (!H.inf) g2_prepare_lines(H, pr.lh.data(), scratch);
        if (!W.inf) g2_prepare_lines(W, pr.lw.data(), scratch);
        pr.ok = true;
      }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; t++) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
  }
  std::atomic<uint32_t> next{0};
  auto work = [&]() {
    for (;;) {
      const uint32_t k = next.fetch_add(1);
      if (k >= njobs) return;
      const uint32_t j = jobs[2 * k], i = jobs[2 * k + 1];
      const prep& pr = P[j];
      g1a pk, S;
      if (!pr.ok || !ok1(g1_decompress(pk48 + (size_t)i * 48, pk)) ||
          !ok1(g1_decompress(shares48 + ((size_t)j * n + i) * 48, S))) {
        out[k] = 0;
        continue;
      }
      pk.y = fq_neg(pk.y);
      const bool useA = !S.inf && !pr.h_inf, useB = !pk.inf && !pr.w_inf;
      if (!useA && !useB) {
        out[k] = 1;
        continue;
      }
      const fq12 f = miller_loop2(pr.lh.data(), S, useA, pr.lw.data(), pk, useB);
      out[k] = fq12_is_one(final_exponentiation(f)) ? 1 : 0;
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; t++) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
  return 0;
}
}

namespace {
template <class F>
void run_pool(int threads, F&& work) {
  if (threads < 1) threads = 1;
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; t++) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
}
bool ok1(int st) { return st == HBX_PT_OK || st == HBX_PT_INFINITY; }
// into_affine as serde runs it on a signature share: on the curve AND in G2
bool g2_decode_sub(const uint8_t* b96, g2a& q) {
  const int st = g2_decompress(b96, q);
  if (st == HBX_PT_INFINITY) return true;
  return st == HBX_PT_OK && g2_is_torsion_free(q);
}
void hash_g2_msg(const uint8_t* msg, uint64_t len, uint8_t* d) { digest2(DIGEST_SHA256, msg, len, nullptr, 0, d); }
}  // namespace

extern "C" {
// PublicKeyShare::verify(sig, nonce) (common_coin.rs:151): e(pk_i, H) == e(g1, sig_i).
//  fused = 0: the reference's shape -- hash_g2(nonce) per share with pairing 0.14's cofactor
//             multiplication, two pairings compared;
//  fused = 1: H and its Miller lines once per instance, sig's lines generated inside one mixed
//             two-pair Miller loop, one final exponentiation.
// jobs: (instance, signer) pairs; out[k] = 1/0.
int cpu_verify_sig_shares(const uint8_t* pk48, uint32_t n, const uint8_t* nonce_blob, const uint64_t* nonce_off,
                          uint32_t inst, const uint8_t* sig96, const uint32_t* jobs, uint32_t njobs, int threads,
                          int fused, uint8_t* out) {
  struct prep {
    bool used = false, ok = false;
    g2a H;
    std::vector<line_pre> lh;
  };
  std::vector<prep> P(inst);
  if (fused) {
    for (uint32_t k = 0; k < njobs; k++) P[jobs[2 * k]].used = true;
    std::vector<uint32_t> todo;
    for (uint32_t j = 0; j < inst; j++)
      if (P[j].used) todo.push_back(j);
    std::atomic<uint32_t> next{0};
    run_pool(threads, [&]() {
      for (;;) {
        const uint32_t q = next.fetch_add(1);
        if (q >= todo.size()) return;
        prep& pr = P[todo[q]];
        uint8_t d[32];
        hash_g2_msg(nonce_blob + nonce_off[todo[q]], nonce_off[todo[q] + 1] - nonce_off[todo[q]], d);
        pr.H = g2_to_affine(hash_g2_from_digest(d));
        pr.lh.resize(MILLER_LINES);
        fq2 scratch[2 * MILLER_LINES];
        g2_prepare_lines(pr.H, pr.lh.data(), scratch);
        pr.ok = true;
      }
    });
  }
  g1a g1{fq_from_const(G1_GEN_X), fq_from_const(G1_GEN_Y), false};
  g1a ng = g1;
  ng.y = fq_neg(ng.y);
  std::atomic<uint32_t> next{0};
  run_pool(threads, [&]() {
    for (;;) {
      const uint32_t k = next.fetch_add(1);
      if (k >= njobs) return;
      const uint32_t j = jobs[2 * k], i = jobs[2 * k + 1];
      g1a pk;
      g2a S;
      if (!ok1(g1_decompress(pk48 + (size_t)i * 48, pk)) || !g2_decode_sub(sig96 + ((size_t)j * n + i) * 96, S)) {
        out[k] = 0;
        continue;
      }
      if (!fused) {
        uint8_t d[32];
        hash_g2_msg(nonce_blob + nonce_off[j], nonce_off[j + 1] - nonce_off[j], d);
        chacha_rng r;
        chacha_rng_from_digest(r, d);
        const g2a H = g2_to_affine(g2_rand_reference_shape(r));
        out[k] = fq12_eq(pairing(pk, H), pairing(g1, S)) ? 1 : 0;
        continue;
      }
      const prep& pr = P[j];
      const bool useA = !pk.inf, useB = !S.inf;
      if (!useA && !useB) {
        out[k] = 1;
        continue;
      }
      const fq12 f = miller_loop_mixed(pr.lh.data(), pk, useA, S, ng, useB);
      out[k] = fq12_is_one(final_exponentiation(f)) ? 1 : 0;
    }
  });
  return 0;
}

// combine_signatures over the first t valid shares of each instance (Lagrange at 0 in Fr, G2
// double-and-add), PublicKey::verify of the result against the master key (two pairings) and
// Signature::parity (common_coin.rs:183-207, :173).  valid: u8[inst][n]; out: per instance
// 1 = master check passed (0 = failed or fewer than t valid shares), parity[j].
int cpu_combine_sigs(const uint8_t* sig96, const uint8_t* valid, uint32_t n, uint32_t inst, uint32_t t,
                     const uint8_t* master48, const uint8_t* nonce_blob, const uint64_t* nonce_off, int threads,
                     uint8_t* ok, uint8_t* parity) {
  g1a mpk;
  if (g1_decompress(master48, mpk) != HBX_PT_OK) return -1;
  g1a g1{fq_from_const(G1_GEN_X), fq_from_const(G1_GEN_Y), false};
  std::atomic<uint32_t> next{0};
  run_pool(threads, [&]() {
    std::vector<uint32_t> idx;
    for (;;) {
      const uint32_t j = next.fetch_add(1);
      if (j >= inst) return;
      idx.clear();
      for (uint32_t i = 0; i < n && idx.size() < t; i++)
        if (valid[(size_t)j * n + i] == 1) idx.push_back(i);
      ok[j] = 0;
      parity[j] = 0;
      if (idx.size() < t) continue;
      g2j acc = g2_identity();
      for (uint32_t a = 0; a < t; a++) {
        fr num = fr_from_const(FR_ONE), den = fr_from_const(FR_ONE), xa{};
        xa.l[0] = idx[a] + 1;
        xa = fr_to_mont(xa);
        for (uint32_t b = 0; b < t; b++) {
          if (b == a) continue;
          fr xb{};
          xb.l[0] = idx[b] + 1;
          xb = fr_to_mont(xb);
          num = fr_mul(num, xb);
          den = fr_mul(den, fr_sub(xb, xa));
        }
        const fr lam = fr_from_mont(fr_mul(num, fr_inv(den)));
        g2a S;
        g2_decompress(sig96 + ((size_t)j * n + idx[a]) * 96, S);
        acc = g2_add(acc, g2_mul_bits(g2_from_affine(S), lam.l, 255));
      }
      const g2a sig = g2_to_affine(acc);
      uint8_t d[32];
      hash_g2_msg(nonce_blob + nonce_off[j], nonce_off[j + 1] - nonce_off[j], d);
      const g2a H = g2_to_affine(hash_g2_from_digest(d));
      ok[j] = fq12_eq(pairing(mpk, H), pairing(g1, sig)) ? 1 : 0;
      uint8_t u[192];
      g2_uncompressed(sig, u);
      uint8_t x = 0;
      for (int q = 0; q < 192; q++) x ^= u[q];
      parity[j] = (uint8_t)(__builtin_popcount(x) & 1);
    }
  });
  return 0;
}

// PublicKeySet::decrypt (honey_badger.rs:340) as threshold_crypto runs it: per proposer, the first t
// valid decryption shares in node order, Lagrange coefficients at 0 in Fr, sum of lambda_i S_i by
// 255-bit double-and-add in G1, then hash_bytes (ChaCha keystream seeded by SHA-256 of the compressed
// point) XOR V.  shares48 u8[p][n][48], valid u8[p][n]; out = plaintexts at v_off; status[j] = 0 or
// -3 (NotEnoughShares).  BASELINE.md §2 row C3 "ms per epoch (verify + combine)".
int cpu_combine_decrypt(const uint8_t* shares48, const uint8_t* valid, uint32_t n, uint32_t p, uint32_t t,
                        const uint8_t* v_blob, const uint64_t* v_off, int threads, uint8_t* out, int32_t* status) {
  std::atomic<uint32_t> next{0};
  run_pool(threads, [&]() {
    std::vector<uint32_t> idx;
    for (;;) {
      const uint32_t j = next.fetch_add(1);
      if (j >= p) return;
      idx.clear();
      for (uint32_t i = 0; i < n && idx.size() < t; i++)
        if (valid[(size_t)j * n + i] == 1) idx.push_back(i);
      status[j] = 0;
      if (idx.size() < t) {
        status[j] = -3;
        continue;
      }
      g1j acc = g1_identity();
      for (uint32_t a = 0; a < t; a++) {
        fr num = fr_from_const(FR_ONE), den = fr_from_const(FR_ONE), xa{};
        xa.l[0] = idx[a] + 1;
        xa = fr_to_mont(xa);
        for (uint32_t b = 0; b < t; b++) {
          if (b == a) continue;
          fr xb{};
          xb.l[0] = idx[b] + 1;
          xb = fr_to_mont(xb);
          num = fr_mul(num, xb);
          den = fr_mul(den, fr_sub(xb, xa));
        }
        const fr lam = fr_from_mont(fr_mul(num, fr_inv(den)));
        g1a S;
        g1_decompress(shares48 + ((size_t)j * n + idx[a]) * 48, S);
        acc = g1_add(acc, g1_mul_scalar(g1_from_affine(S), lam.l));
      }
      uint8_t comp[48], d[32];
      g1_compress(g1_to_affine(acc), comp);
      digest2(DIGEST_SHA256, comp, 48, nullptr, 0, d);
      uint32_t key[8];
      for (int q = 0; q < 8; q++)
        key[q] = ((uint32_t)d[4 * q] << 24) | ((uint32_t)d[4 * q + 1] << 16) | ((uint32_t)d[4 * q + 2] << 8) | d[4 * q + 3];
      const uint64_t off = v_off[j], len = v_off[j + 1] - off;
      for (uint64_t b = 0; 16 * b < len; b++) {
        uint32_t ks[16];
        chacha20_block(key, b, 0, ks);
        for (uint64_t q = 16 * b; q < len && q < 16 * b + 16; q++) out[off + q] = v_blob[off + q] ^ (uint8_t)ks[q - 16 * b];
      }
    }
  });
  return 0;
}

// ---- reed-solomon-erasure 3.1.0 shape: GF(2^8) with poly 0x11D, MUL_TABLE rows -----------------
namespace {
struct gf8 {
  uint8_t mul[256][256];
  uint8_t inv[256];
  gf8() {
    uint8_t ex[512];
    int lg[256];
    uint32_t x = 1;
    for (int i = 0; i < 255; i++) {
      ex[i] = ex[i + 255] = (uint8_t)x;
      lg[x] = i;
      x <<= 1;
      if (x & 0x100) x ^= 0x11D;
    }
    for (int a = 0; a < 256; a++)
      for (int b = 0; b < 256; b++) mul[a][b] = (a && b) ? ex[lg[a] + lg[b]] : 0;
    inv[0] = 0;
    for (int a = 1; a < 256; a++) inv[a] = ex[255 - lg[a]];
  }
};
const gf8& GF() {
  static gf8 g;
  return g;
}
// galois_8::mul_slice_xor: out[i] ^= c * in[i]
void mul_slice_xor(uint8_t c, const uint8_t* in, uint8_t* out, size_t len) {
  const uint8_t* row = GF().mul[c];
  for (size_t i = 0; i < len; i++) out[i] ^= row[in[i]];
}
void mul_slice(uint8_t c, const uint8_t* in, uint8_t* out, size_t len) {
  const uint8_t* row = GF().mul[c];
  for (size_t i = 0; i < len; i++) out[i] = row[in[i]];
}
// Gauss-Jordan inverse of a k x k matrix (false if singular)
bool gf_invert(std::vector<uint8_t>& a, uint32_t k) {
  const gf8& g = GF();
  std::vector<uint8_t> m(k * 2 * k, 0);
  for (uint32_t r = 0; r < k; r++) {
    for (uint32_t c = 0; c < k; c++) m[r * 2 * k + c] = a[r * k + c];
    m[r * 2 * k + k + r] = 1;
  }
  for (uint32_t r = 0; r < k; r++) {
    uint32_t b = r;
    while (b < k && !m[b * 2 * k + r]) b++;
    if (b == k) return false;
    if (b != r)
      for (uint32_t c = 0; c < 2 * k; c++) std::swap(m[r * 2 * k + c], m[b * 2 * k + c]);
    const uint8_t iv = g.inv[m[r * 2 * k + r]];
    for (uint32_t c = 0; c < 2 * k; c++) m[r * 2 * k + c] = g.mul[iv][m[r * 2 * k + c]];
    for (uint32_t i = 0; i < k; i++) {
      const uint8_t f = m[i * 2 * k + r];
      if (i == r || !f) continue;
      for (uint32_t c = 0; c < 2 * k; c++) m[i * 2 * k + c] ^= g.mul[f][m[r * 2 * k + c]];
    }
  }
  for (uint32_t r = 0; r < k; r++)
    for (uint32_t c = 0; c < k; c++) a[r * k + c] = m[r * 2 * k + k + c];
  return true;
}
// systematic encoding matrix V * inverse(V[0..k]) with V[r][c] = r^c, (k + m) x k
std::vector<uint8_t> rs_matrix(uint32_t k, uint32_t m) {
  const gf8& g = GF();
  auto pw = [&](uint8_t a, uint32_t e) {
    uint8_t r = 1;
    for (uint32_t q = 0; q < e; q++) r = g.mul[r][a];
    return r;
  };
  const uint32_t n = k + m;
  std::vector<uint8_t> V(n * k), top(k * k), M(n * k, 0);
  for (uint32_t r = 0; r < n; r++)
    for (uint32_t c = 0; c < k; c++) V[r * k + c] = pw((uint8_t)r, c);
  for (uint32_t q = 0; q < k * k; q++) top[q] = V[q];
  gf_invert(top, k);
  for (uint32_t r = 0; r < n; r++)
    for (uint32_t c = 0; c < k; c++) {
      uint8_t acc = 0;
      for (uint32_t q = 0; q < k; q++) acc ^= g.mul[V[r * k + q]][top[q * k + c]];
      M[r * k + c] = acc;
    }
  return M;
}
}  // namespace

// ReedSolomon::encode of `inst` instances: shards u8[inst][k + m][L], data rows filled, parity
// rows written (for each parity row: mul_slice of the first input, mul_slice_xor of the rest).
int cpu_rs_encode(uint8_t* shards, uint32_t inst, uint32_t k, uint32_t m, uint32_t L, int threads) {
  const std::vector<uint8_t> M = rs_matrix(k, m);
  std::atomic<uint32_t> next{0};
  run_pool(threads, [&]() {
    for (;;) {
      const uint32_t j = next.fetch_add(1);
      if (j >= inst) return;
      uint8_t* base = shards + (size_t)j * (k + m) * L;
      for (uint32_t o = 0; o < m; o++) {
        uint8_t* out = base + (size_t)(k + o) * L;
        const uint8_t* row = &M[(size_t)(k + o) * k];
        mul_slice(row[0], base, out, L);
        for (uint32_t q = 1; q < k; q++) mul_slice_xor(row[q], base + (size_t)q * L, out, L);
      }
    }
  });
  return 0;
}

// ReedSolomon::reconstruct_shards: present u8[inst][k + m]; the first k present rows (in index
// order) give the decode matrix (inverted per call, as rse does), missing data rows are rebuilt
// from them, then missing parity rows from the data.  status[j] = 0 or -1 (TooFewShardsPresent).
int cpu_rs_reconstruct(uint8_t* shards, const uint8_t* present, uint32_t inst, uint32_t k, uint32_t m, uint32_t L,
                       int threads, int32_t* status) {
  const std::vector<uint8_t> M = rs_matrix(k, m);
  const uint32_t n = k + m;
  std::atomic<uint32_t> next{0};
  run_pool(threads, [&]() {
    std::vector<uint32_t> sub;
    std::vector<uint8_t> D;
    for (;;) {
      const uint32_t j = next.fetch_add(1);
      if (j >= inst) return;
      uint8_t* base = shards + (size_t)j * n * L;
      const uint8_t* pr = present + (size_t)j * n;
      sub.clear();
      for (uint32_t i = 0; i < n && sub.size() < k; i++)
        if (pr[i]) sub.push_back(i);
      status[j] = 0;
      if (sub.size() < k) {
        status[j] = -1;
        continue;
      }
      D.assign(k * k, 0);
      for (uint32_t r = 0; r < k; r++)
        for (uint32_t c = 0; c < k; c++) D[r * k + c] = M[(size_t)sub[r] * k + c];
      gf_invert(D, k);
      for (uint32_t d = 0; d < k; d++) {
        if (pr[d]) continue;
        uint8_t* out = base + (size_t)d * L;
        mul_slice(D[d * k], base + (size_t)sub[0] * L, out, L);
        for (uint32_t q = 1; q < k; q++) mul_slice_xor(D[d * k + q], base + (size_t)sub[q] * L, out, L);
      }
      for (uint32_t o = k; o < n; o++) {
        if (pr[o]) continue;
        uint8_t* out = base + (size_t)o * L;
        mul_slice(M[(size_t)o * k], base, out, L);
        for (uint32_t q = 1; q < k; q++) mul_slice_xor(M[(size_t)o * k + q], base + (size_t)q * L, out, L);
      }
    }
  });
  return 0;
}
}  // extern "C"
