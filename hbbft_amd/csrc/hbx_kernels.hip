// HIP kernels for the threshold-decryption hot path on gfx950.
//
// Layout in HBM (per context, sized for one epoch of p proposers x n senders):
//   pk      : g1a[n]                 affine Montgomery pk_i (replicated once per era)
//   U       : g1a[p]                 ciphertext U_j
//   G2pts   : g2a[2p]                (H_j, W_j) interleaved
//   lines   : line_pre[2p][68]       prepared Miller-loop lines of H_j and W_j (26 KiB / proposer)
//   S       : g1a[p][n]              decompressed shares (kept for the Lagrange combine)
//   valid   : u8[p][n]               verification result per share
//   keys    : u32[p][8]              ChaCha keys of hash_bytes(g_j) after the combine
// Kernel geometry: one lane per independent check (share, ciphertext, G2 point); the verify
// grid is (ceil(n/64), p) single-wave workgroups so all lanes of a wave share proposer j and
// read its prepared lines at wave-uniform addresses.
#include <hip/hip_runtime.h>
#include "hash.hpp"
#include "pairing.hpp"

namespace hbx {

struct line_block {  // lines of one proposer: H then W
  line_pre h[MILLER_LINES];
  line_pre w[MILLER_LINES];
};

// e(PA, QA) * e(PB, QB) == 1 with identity handling (pairing with the identity is 1).
__device__ __forceinline__ bool check2(const line_pre* LA, const g1a& PA, bool qa_inf,
                                       const line_pre* LB, const g1a& PB, bool qb_inf) {
  const bool skipA = PA.inf || qa_inf;
  const bool skipB = PB.inf || qb_inf;
  if (skipA && skipB) return true;
  const fq12 f = miller_loop2(LA, PA, !skipA, LB, PB, !skipB);
  return fq12_is_one(final_exponentiation(f));
}

__global__ void __launch_bounds__(64) k_decompress_g1(const uint8_t* __restrict__ comp, uint32_t n,
                                                      g1a* __restrict__ out, int32_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1a p;
  const int32_t st = g1_decompress(comp + (size_t)i * 48, p);
  out[i] = p;
  status[i] = st;
}

// One lane per proposer: decode U_j and W_j, compute H_j = hash_g1_g2(U_j, V_j).
__global__ void __launch_bounds__(64) k_prepare_ct(const uint8_t* __restrict__ u_comp,
                                                   const uint8_t* __restrict__ v_blob,
                                                   const uint64_t* __restrict__ v_off,
                                                   const uint8_t* __restrict__ w_comp, uint32_t p,
                                                   g1a* __restrict__ U, g2a* __restrict__ G2pts,
                                                   uint8_t* __restrict__ ct_ok) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= p) return;
  g1a u;
  g2a w;
  const int32_t su = g1_decompress(u_comp + (size_t)j * 48, u);
  const int32_t sw = g2_decompress(w_comp + (size_t)j * 96, w);
  const bool ok = (su == HBX_PT_OK || su == HBX_PT_INFINITY) && (sw == HBX_PT_OK || sw == HBX_PT_INFINITY);
  g2a h;
  h.x = fq2_zero();
  h.y = fq2_zero();
  h.inf = true;
  if (ok) {
    const uint64_t off = v_off[j];
    const uint64_t len = v_off[j + 1] - off;
    h = g2_to_affine(hash_g1_g2(u_comp + (size_t)j * 48, v_blob + off, len));
  }
  U[j] = u;
  G2pts[2 * j] = h;
  G2pts[2 * j + 1] = w;
  ct_ok[j] = ok ? 1 : 0;
}

// One lane per G2 point: the 68 normalised lines.
__global__ void __launch_bounds__(64) k_prepare_lines(const g2a* __restrict__ pts, uint32_t count,
                                                      line_pre* __restrict__ lines, fq2* __restrict__ scratch) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  const g2a q = pts[k];
  if (q.inf) return;
  g2_prepare_lines(q, lines + (size_t)k * MILLER_LINES, scratch + (size_t)k * 2 * MILLER_LINES);
}

// Ciphertext::verify: e(-U, H) * e(g1, W) == 1.
__global__ void __launch_bounds__(64) k_verify_ct(const g1a* __restrict__ U, const g2a* __restrict__ G2pts,
                                                  const line_block* __restrict__ lines, uint32_t p,
                                                  const uint8_t* __restrict__ ct_ok, uint8_t* __restrict__ ct_valid) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= p) return;
  bool valid = false;
  if (ct_ok[j]) {
    g1a nu = U[j];
    nu.y = fq_neg(nu.y);
    g1a g;
    g.x = fq_from_const(G1_GEN_X);
    g.y = fq_from_const(G1_GEN_Y);
    g.inf = false;
    valid = check2(lines[j].h, nu, G2pts[2 * j].inf, lines[j].w, g, G2pts[2 * j + 1].inf);
  }
  ct_valid[j] = valid ? 1 : 0;
}

// Share verification: lane = sender i, blockIdx.y = proposer j.
__global__ void __launch_bounds__(64) k_verify_shares(const uint8_t* __restrict__ shares,
                                                      const uint8_t* __restrict__ present,
                                                      const g1a* __restrict__ pk, uint32_t n_keys,
                                                      const g2a* __restrict__ G2pts,
                                                      const line_block* __restrict__ lines,
                                                      const uint8_t* __restrict__ ct_ok, uint32_t n,
                                                      g1a* __restrict__ S, uint8_t* __restrict__ valid) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = blockIdx.y;
  if (i >= n) return;
  const size_t idx = (size_t)j * n + i;
  g1a s;
  const int32_t st = g1_decompress(shares + idx * 48, s);
  S[idx] = s;
  bool ok = (st == HBX_PT_OK || st == HBX_PT_INFINITY) && i < n_keys && ct_ok[j] &&
            (present == nullptr || present[idx]);
  bool v = false;
  if (ok) {
    g1a npk = pk[i];
    npk.y = fq_neg(npk.y);
    v = check2(lines[j].h, s, G2pts[2 * j].inf, lines[j].w, npk, G2pts[2 * j + 1].inf);
  }
  valid[idx] = v ? 1 : 0;
}

// Lagrange combine of the first t valid shares of proposer j (one 256-thread block per
// proposer), then the hash_bytes key = SHA-256(compress(g)).
constexpr int COMBINE_THREADS = 256;
constexpr int COMBINE_MAX_T = 4096;

__global__ void __launch_bounds__(COMBINE_THREADS) k_combine(const uint8_t* __restrict__ valid,
                                                             const g1a* __restrict__ S, uint32_t n,
                                                             uint32_t t, const uint8_t* __restrict__ ct_valid,
                                                             uint32_t* __restrict__ keys,
                                                             int32_t* __restrict__ status) {
  __shared__ uint16_t idx[COMBINE_MAX_T];
  __shared__ int s_count;
  __shared__ g1j red[COMBINE_THREADS];
  const uint32_t j = blockIdx.x;
  const int tid = threadIdx.x;
  if (tid == 0) {
    int c = 0;
    for (uint32_t i = 0; i < n && c < (int)t; i++)
      if (valid[(size_t)j * n + i]) idx[c++] = (uint16_t)i;
    s_count = c;
  }
  __syncthreads();
  const int count = s_count;
  if (!ct_valid[j] || count < (int)t) {
    if (tid == 0) status[j] = !ct_valid[j] ? -7 : -3;
    return;
  }
  g1j acc = g1_identity();
  for (int k = tid; k < (int)t; k += COMBINE_THREADS) {
    // lambda_k(0) = prod_{m != k} x_m / (x_m - x_k), x = index + 1
    fr num = fr_from_const(FR_ONE), den = fr_from_const(FR_ONE);
    fr xk;
    for (int q = 0; q < 8; q++) xk.l[q] = 0;
    xk.l[0] = (uint32_t)idx[k] + 1;
    xk = fr_to_mont(xk);
    for (int m = 0; m < (int)t; m++) {
      if (m == k) continue;
      fr xm;
      for (int q = 0; q < 8; q++) xm.l[q] = 0;
      xm.l[0] = (uint32_t)idx[m] + 1;
      xm = fr_to_mont(xm);
      num = fr_mul(num, xm);
      den = fr_mul(den, fr_sub(xm, xk));
    }
    const fr lam = fr_from_mont(fr_mul(num, fr_inv(den)));
    const g1a sp = S[(size_t)j * n + idx[k]];
    const g1j part = g1_mul_scalar(g1_from_affine(sp), lam.l);
    acc = g1_add(acc, part);
  }
  red[tid] = acc;
  __syncthreads();
  for (int stride = COMBINE_THREADS / 2; stride > 0; stride >>= 1) {
    if (tid < stride) red[tid] = g1_add(red[tid], red[tid + stride]);
    __syncthreads();
  }
  if (tid == 0) {
    const g1a g = g1_to_affine(red[0]);
    uint8_t comp[48], d[32];
    g1_compress(g, comp);
    sha256_2(comp, 48, nullptr, 0, d);
    for (int q = 0; q < 8; q++)
      keys[(size_t)j * 8 + q] = ((uint32_t)d[4 * q] << 24) | ((uint32_t)d[4 * q + 1] << 16) |
                                ((uint32_t)d[4 * q + 2] << 8) | d[4 * q + 3];
    status[j] = 0;
  }
}

// plaintext_j = V_j XOR hash_bytes(g_j, |V_j|): lane = 16-byte keystream block (one ChaCha20
// block of 16 words, one word per byte as rand 0.4 gen::<u8>() consumes them).
__global__ void __launch_bounds__(64) k_keystream_xor(const uint32_t* __restrict__ keys,
                                                      const int32_t* __restrict__ status,
                                                      const uint8_t* __restrict__ v_blob,
                                                      const uint64_t* __restrict__ v_off,
                                                      uint8_t* __restrict__ out) {
  const uint32_t j = blockIdx.y;
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t off = v_off[j];
  const uint64_t len = v_off[j + 1] - off;
  if (16 * b >= len) return;
  if (status[j] != 0) return;
  uint32_t key[8];
  for (int q = 0; q < 8; q++) key[q] = keys[(size_t)j * 8 + q];
  uint32_t ks[16];
  chacha20_block(key, b, 0, ks);
  const uint64_t end = (16 * b + 16 < len) ? 16 * b + 16 : len;
  for (uint64_t q = 16 * b; q < end; q++) out[off + q] = v_blob[off + q] ^ (uint8_t)ks[q - 16 * b];
}


// ----------------------------------------------------------------------------------------------
// Producer side: scalar multiplications that make the
// inputs of the verification path.  Scalars are canonical Fr values, 8 little-endian u32 limbs.
// ----------------------------------------------------------------------------------------------

// 32-byte big-endian canonical scalar -> 8 LE limbs.
__device__ __forceinline__ void fr_from_be32(const uint8_t* b, uint32_t* k8) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint8_t* q = b + 28 - 4 * i;
    k8[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}

__device__ __forceinline__ g1a g1_generator() {
  g1a g;
  g.x = fq_from_const(G1_GEN_X);
  g.y = fq_from_const(G1_GEN_Y);
  g.inf = false;
  return g;
}

// SecretKey::public_key (threshold_crypto): pk = g1 * sk, one lane per key.
__global__ void __launch_bounds__(64) k_public_keys(const uint8_t* __restrict__ sk32, uint32_t n,
                                                    uint8_t* __restrict__ pk48) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  fr_from_be32(sk32 + (size_t)i * 32, k);
  const g1a pk = g1_to_affine(g1_mul_scalar(g1_from_affine(g1_generator()), k));
  g1_compress(pk, pk48 + (size_t)i * 48);
}

// SecretKeyShare::decrypt_share_no_verify (honey_badger.rs:403): S_ji = sk_i * U_j.
// Lane = node i, blockIdx.y = proposer j; output proposer-major like the verify input.
__global__ void __launch_bounds__(64) k_decrypt_shares(const uint8_t* __restrict__ sk32, uint32_t n,
                                                       const g1a* __restrict__ U, uint8_t* __restrict__ out48) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = blockIdx.y;
  if (i >= n) return;
  uint32_t k[8];
  fr_from_be32(sk32 + (size_t)i * 32, k);
  const g1a s = g1_to_affine(g1_mul_scalar(g1_from_affine(U[j]), k));
  g1_compress(s, out48 + ((size_t)j * n + i) * 48);
}

// PublicKey::encrypt (honey_badger.rs:116) with explicit randomness r_j (threshold_crypto draws
// it from thread_rng):  U = g1 r, V = M xor hash_bytes(pk r, |M|), W = hash_g1_g2(U, V) r.
// One lane per message.
__global__ void __launch_bounds__(64) k_encrypt(const g1a* __restrict__ pk, const uint8_t* __restrict__ r32,
                                                const uint8_t* __restrict__ msg, const uint64_t* __restrict__ off,
                                                uint32_t p, uint8_t* __restrict__ u48, uint8_t* __restrict__ v,
                                                uint8_t* __restrict__ w96) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= p) return;
  uint32_t k[8];
  fr_from_be32(r32 + (size_t)j * 32, k);
  const g1a u = g1_to_affine(g1_mul_scalar(g1_from_affine(g1_generator()), k));
  const g1a g = g1_to_affine(g1_mul_scalar(g1_from_affine(pk[0]), k));
  uint8_t* uc = u48 + (size_t)j * 48;
  g1_compress(u, uc);
  uint8_t gc[48], d[32];
  g1_compress(g, gc);
  sha256_2(gc, 48, nullptr, 0, d);
  chacha_rng rng;
  chacha_rng_from_digest(rng, d);
  const uint64_t o = off[j], len = off[j + 1] - o;
  for (uint64_t q = 0; q < len; q++) v[o + q] = msg[o + q] ^ (uint8_t)chacha_next_u32(rng);
  const g2j h = hash_g1_g2(uc, v + o, len);
  g2_compress(g2_to_affine(g2_mul_bits(h, k, 256)), w96 + (size_t)j * 96);
}

}  // namespace hbx
