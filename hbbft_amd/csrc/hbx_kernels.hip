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
#include "../../include/hbx.h"
#include "hash.hpp"
#include "pairing.hpp"
#include "pairing3.hpp"
#include "pairingd.hpp"
#include "pairing3d.hpp"
#include "pairing2d.hpp"
#include "fe1d.hpp"
#include "g2d.hpp"
#include "g1d.hpp"
#include "curve4.hpp"
#include "wide.hpp"

// Split build (tools/build.py): the kernels compile in groups, one translation unit per group
// (-DHBX_TU=1..10: epoch, share checks, producer, wide checks, coin, broadcast, two-lane share
// checks, the one-lane checks' final-exponentiation steps in three units); TU 0 is the host
// API, which sees only their declarations (_kdecl.hpp, generated from these sources).
#if !defined(HBX_TU)
#define HBX_IN_TU(n) 1
#else
#define HBX_IN_TU(n) (HBX_TU == (n))
#endif

namespace hbx {

struct line_block {  // lines of one proposer: H then W
  line_pre h[MILLER_LINES];
  line_pre w[MILLER_LINES];
};
struct line_block_d {  // the same lines in the share check's digit form (pairingd.hpp)
  line_pre_d h[MILLER_LINES];
  line_pre_d w[MILLER_LINES];
};

// Status of a share before its pairing check (include/hbx.h HBX_SHARE_*): HBX_SHARE_VALID means
// "check it"; precedence follows what the reference would see first: no message, a message from
// a non-validator (UnknownSender), a message serde cannot decode, a proposer whose ciphertext was
// rejected (its shares are never verified).
__device__ __forceinline__ uint8_t share_precheck(int32_t dec_status, bool present, bool known_sender, bool ct_ok) {
  if (!present) return HBX_SHARE_ABSENT;
  if (!known_sender) return HBX_SHARE_UNKNOWN_SENDER;
  if (dec_status != HBX_PT_OK && dec_status != HBX_PT_INFINITY) return HBX_SHARE_UNDECODABLE;
  if (!ct_ok) return HBX_SHARE_SKIPPED_CT;
  return HBX_SHARE_VALID;
}

#ifndef HBX_ML_SCALED
#define HBX_ML_SCALED 1  // the one-lane Miller kernel over lines divided by y_P (pairingd.hpp)
#endif

// Internal status of a share whose pairing check waits for its final exponentiation
// (k_verify_shares_ml -> k_fe1<6>); never visible outside a verification call.
constexpr uint8_t SHARE_PENDING = 0xFE;
// A one-lane check whose compressed squarings met g3 = 0 (fe1d.hpp karabina_decompress): decided
// again by the single-kernel check (k_verify_shares with fallback_only).
constexpr uint8_t SHARE_FALLBACK = 0xFD;

// e(PA, QA) * e(PB, QB) == 1 with identity handling (pairing with the identity is 1).
__device__ __forceinline__ bool check2(const line_pre* LA, const g1a& PA, bool qa_inf,
                                       const line_pre* LB, const g1a& PB, bool qb_inf) {
  const bool skipA = PA.inf || qa_inf;
  const bool skipB = PB.inf || qb_inf;
  if (skipA && skipB) return true;
  const fq12 f = miller_loop2(LA, PA, !skipA, LB, PB, !skipB);
  return fq12_is_one(final_exponentiation(f));
}
// check2 with the final exponentiation's base in this lane's LDS slot (pairing.hpp)
__device__ __forceinline__ bool check2_lds(const line_pre* LA, const g1a& PA, bool qa_inf, const line_pre* LB,
                                           const g1a& PB, bool qb_inf, lds_u32* gslot) {
  const bool skipA = PA.inf || qa_inf;
  const bool skipB = PB.inf || qb_inf;
  if (skipA && skipB) return true;
  const fq12 f = miller_loop2(LA, PA, !skipA, LB, PB, !skipB);
  return fq12_is_one(final_exponentiation_lds(f, gslot));
}

#if HBX_IN_TU(1)
__global__ void __launch_bounds__(64) k_decompress_g1(const uint8_t* __restrict__ comp, uint32_t n,
                                                      g1a* __restrict__ out, int32_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1a p;
  const int32_t st = g1_decompress_d(comp + (size_t)i * 48, p);
  out[i] = p;
  status[i] = st;
}
#endif

// Fixed-base tables of the key shares (k_g1_tables): 64 windows of 4 bits, digits 1..15.
constexpr int G1TAB_W = 64, G1TAB_D = 15;

// Lanes per hash_g2 group (hash.hpp hash_g2_group).
constexpr int HASH_K = 16;

#if HBX_IN_TU(1)
// H_j = hash_g1_g2(U_j, V_j) for every proposer, plus the decoding of U_j and W_j, in ONE launch:
//  * blocks [0, hash_blocks): HASH_K-lane groups, one per proposer (hash_g2_group); the hash reads
//    only the compressed bytes of U_j, so it does not wait for the decode;
//  * blocks [hash_blocks, ...): one lane per point decodes U_j (j < p) or W_j (p <= j < 2p), in
//    waves of their own, concurrently with the hash waves; in own-share mode lanes [2p, 4p)
//    compute the two GLV halves of sk_me U_j (summed by k_prepare_lines).
// ct_ok and the identity substitution for undecodable ciphertexts (H_j = O) are applied by
// k_prepare_lines, which runs after both.
__global__ void __launch_bounds__(64) k_prepare_ct(const uint8_t* __restrict__ u_comp,
                                                   const uint8_t* __restrict__ v_blob,
                                                   const uint64_t* __restrict__ v_off,
                                                   const uint8_t* __restrict__ w_comp, uint32_t p,
                                                   uint32_t hash_blocks, g1a* __restrict__ U,
                                                   g2a* __restrict__ G2pts, int32_t* __restrict__ dec_st,
                                                   const uint32_t* __restrict__ own_sk, g1j* __restrict__ own_part,
                                                   g2j* __restrict__ Hj, int digest, uint32_t block0, uint32_t dec_blocks,
                                                   const uint8_t* __restrict__ shares, size_t share_count,
                                                   uint32_t n, uint32_t me, g1a* __restrict__ S,
                                                   int32_t* __restrict__ S_status) {
  const uint32_t bid = blockIdx.x + block0;  // block0 > 0: the decode part launched on its own
  if (bid >= hash_blocks + dec_blocks) {
    // early share decode (hbx_decrypt_epoch_d): k_decompress_shares' work in waves of this
    // launch, beside the hash chains (which leave most SIMDs idle) instead of after them.  The
    // own-share entries are filled by k_prepare_lines.
    const size_t i = (size_t)(bid - hash_blocks - dec_blocks) * blockDim.x + threadIdx.x;
    if (i >= share_count || (uint32_t)(i % n) == me) return;
    g1a q;
    int32_t st = g1_decompress_d(shares + i * 48, q);
    if (st == HBX_PT_OK && !g1_is_torsion_free_d(q)) st = HBX_PT_NOT_IN_SUBGROUP;
    S_status[i] = st;
    S[i] = q;
    return;
  }
  if (bid >= hash_blocks) {
    // decode = pairing 0.14's into_affine: on-curve AND subgroup membership (U in G1, W in G2).
    // Each part starts on a wave boundary (pw = p rounded up to 64) so no wave mixes the G1 and
    // G2 chains (a mixed wave runs both back to back): U_j at lane j, W_j at pw + j, the own
    // share halves at 2 pw + h.
    const uint32_t pw = (p + 63) & ~63u;
    const uint32_t k = (bid - hash_blocks) * blockDim.x + threadIdx.x;
    if (k < p) {
      g1a u;
      int32_t st = g1_decompress_d(u_comp + (size_t)k * 48, u);
      if (st == HBX_PT_OK && !g1_is_torsion_free_d(u)) st = HBX_PT_NOT_IN_SUBGROUP;
      dec_st[k] = st;
      U[k] = u;
    } else if (own_sk && k >= 2 * pw && k < 2 * pw + 2 * p) {
      // this node's own decryption share sk_me * U_j (decrypt_share_no_verify,
      // honey_badger.rs:403), GLV k = k1 + k2 lambda, phi(x, y) = (beta x, y), one half per lane:
      // lane 2j computes k1 U_j, lane 2j + 1 computes k2 phi(U_j), each decoding U_j itself so
      // neither waits for the subgroup check (k_prepare_lines adds the halves where U_j is valid)
      const uint32_t h = k - 2 * pw, j = h >> 1;
      g1a u;
      g1j part = g1_identity();
      if (g1_decompress_d(u_comp + (size_t)j * 48, u) == HBX_PT_OK) {
        uint32_t k1[4], k2[4];
        g1_glv_split(own_sk, k1, k2);
        if (h & 1) u.x = fq_mul(u.x, fq_from_const(G1_BETA));
        part = g1_mul_u128(u, (h & 1) ? k2 : k1);
      }
      own_part[h] = part;
    } else if (k >= pw && k < pw + p) {
      const uint32_t j = k - pw;
      g2a w;
      int32_t st = g2_decompress(w_comp + (size_t)j * 96, w);
      if (st == HBX_PT_OK && !g2_is_torsion_free(w)) st = HBX_PT_NOT_IN_SUBGROUP;
      dec_st[p + j] = st;
      G2pts[2 * j + 1] = w;
    }
    return;
  }
  const uint32_t gid = bid * blockDim.x + threadIdx.x;
  const uint32_t j = gid / HASH_K;
  if (j >= p) return;  // whole groups only (HASH_K | 64)
  const uint64_t off = v_off[j];
  const uint64_t len = v_off[j + 1] - off;
  uint8_t d[32];
  hash_g1_g2_digest(u_comp + (size_t)j * 48, v_blob + off, len, d, digest);
  g2j h;
  // H'_j = h_eff P = [3(x^2-1)] H_j: the checks use [3(x^2-1)] pk_i and [3(x^2-1)] g1 (k_scale_keys,
  // G1_MGEN), e(S, H') e(-[m] pk, W) = (e(S, H) e(-pk, W))^m with m invertible mod r -- the same
  // bit, without the last third of the cofactor clearing
  // kept in Jacobian form (Hj): the lines are made from (X, Y) on the isomorphic twist and
  // corrected by Z in k_normalise_lines (g2_normalise_line_z), so no inversion sits on this chain;
  // G2pts[2j] carries only the identity flag
  if (hash_g2_group<HASH_K>(d, true, h, false)) {
    Hj[j] = h;
    g2a flag;
    flag.x = fq2_zero();
    flag.y = fq2_zero();
    flag.inf = g2j_is_identity(h);
    G2pts[2 * j] = flag;
  }
}
#endif

// Lanes per G2 point in k_prepare_lines.
constexpr int LINE_K = 16;


#if HBX_IN_TU(1)
// LINE_K lanes per G2 point: the 68 raw lines (c2 into `scratch`, count x 68 Fq2), normalised by
// k_normalise_lines.  With `dec_st` (ciphertext points), the group of point 2j also
// settles ct_ok[j]: U_j and W_j must decode (threshold_crypto deserialisation); otherwise H_j is
// replaced by the identity and the proposer's checks are gated off.
template <bool GADD>
__global__ void __launch_bounds__(64) k_prepare_lines(g2a* __restrict__ pts, uint32_t count,
                                                      line_pre_d* __restrict__ raw, fq2d* __restrict__ scratch,
                                                      const int32_t* __restrict__ dec_st, uint32_t p,
                                                      uint8_t* __restrict__ ct_ok, const g1j* __restrict__ own_part,
                                                      g1a* __restrict__ own_S, uint32_t n, uint32_t me,
                                                      g1a* __restrict__ S, int32_t* __restrict__ S_status,
                                                      const g2j* __restrict__ Hj) {
  const uint32_t line_blocks = (count * LINE_K + 63) / 64;
  if (blockIdx.x >= line_blocks) {
    // own share S_j,me = k1 U_j + k2 phi(U_j) (k_prepare_ct's two halves) where U_j decoded
    const uint32_t j = (blockIdx.x - line_blocks) * blockDim.x + threadIdx.x;
    if (j >= p) return;
    g1a sh;
    sh.x = fq_zero();
    sh.y = fq_zero();
    sh.inf = true;
    if (dec_st[j] == HBX_PT_OK) sh = g1_to_affine(g1_add(own_part[2 * j], own_part[2 * j + 1]));
    own_S[j] = sh;
    if (S) {  // shares decoded early (k_prepare_ct): the own entry as k_decompress_shares writes it
      S[(size_t)j * n + me] = sh;
      S_status[(size_t)j * n + me] = sh.inf ? HBX_PT_INFINITY : HBX_PT_OK;
    }
    return;
  }
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t k = gid / LINE_K;
  const int gl = (int)(gid % LINE_K);
  const int gbase = (int)(threadIdx.x & 63) - gl;
  if (k >= count) return;  // whole groups (LINE_K | 64)
  g2a q = pts[k];
  if (Hj && (k & 1) == 0) {  // (X, Y) of the Jacobian hash point; Z enters in k_normalise_lines
    q.x = Hj[k >> 1].x;
    q.y = Hj[k >> 1].y;
  }
  if (dec_st) {
    const uint32_t j = k >> 1;
    const int32_t su = dec_st[j], sw = dec_st[p + j];
    const bool ok = (su == HBX_PT_OK || su == HBX_PT_INFINITY) && (sw == HBX_PT_OK || sw == HBX_PT_INFINITY);
    if ((k & 1) == 0) {
      if (gl == 0) ct_ok[j] = ok ? 1 : 0;
      if (!ok) {
        q.x = fq2_zero();
        q.y = fq2_zero();
        q.inf = true;
        if (gl == 0) pts[k] = q;
      }
    }
  }
  if (q.inf) {
    if (gl == 0) {
      const fq2d one{fqd_const(FQD_ONE), fqd_zero()}, zero{fqd_zero(), fqd_zero()};
      for (int i = 0; i < MILLER_LINES; i++) {
        raw[(size_t)k * MILLER_LINES + i] = line_pre_d{one, zero};
        scratch[(size_t)k * MILLER_LINES + i] = one;
      }
    }
    return;
  }
  // the steps in the digit tower on the group (groupd.hpp); raw lines in digit form
  (void)gbase;
  g2d_raw_lines_group<GADD>(fq2d_from_fq2(q.x), fq2d_from_fq2(q.y), raw + (size_t)k * MILLER_LINES,
                            scratch + (size_t)k * MILLER_LINES, gl);
}
template __global__ void k_prepare_lines<true>(g2a*, uint32_t, line_pre_d*, fq2d*, const int32_t*, uint32_t, uint8_t*,
                                               const g1j*, g1a*, uint32_t, uint32_t, g1a*, int32_t*, const g2j*);
template __global__ void k_prepare_lines<false>(g2a*, uint32_t, line_pre_d*, fq2d*, const int32_t*, uint32_t, uint8_t*,
                                                const g1j*, g1a*, uint32_t, uint32_t, g1a*, int32_t*, const g2j*);

// Second half of the line preparation: one lane per raw line, (c0, c1) /= c2.  68 independent
// Fq2 inversions replace the batched inversion (3 x 68 Fq2 products plus one inversion) that
// used to sit at the end of each point's sequential chain: the chain of k_prepare_lines is the
// 68 T steps only, and this launch is 68x wider and one inversion deep.
// The raw lines come in digit form (k_prepare_lines: (c0, c1) in lines_d, c2 in `c2`); the
// normalised lines go out in both forms, lines_d overwritten in place.
__global__ void __launch_bounds__(64) k_normalise_lines(line_pre* __restrict__ lines,
                                                        const fq2d* __restrict__ c2, uint32_t count,
                                                        line_pre_d* __restrict__ lines_d,
                                                        const g2a* __restrict__ pts, const g2j* __restrict__ Hj) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  const line_pre_d rd = lines_d[k];
  line_pre l{fq2d_to_fq2(rd.c0), fq2d_to_fq2(rd.c1)};
  const uint32_t pt = k / MILLER_LINES;
  // lines of a Jacobian hash point (k_prepare_lines with Hj) unless it was replaced by the
  // identity; z = 1 otherwise (one code path for the wave: a branch would run both inversions)
  fq2 z = fq2_one();
  if (Hj && (pt & 1) == 0 && !pts[pt].inf) z = Hj[pt >> 1].z;
  g2_normalise_line_z(l, fq2d_to_fq2(c2[k]), z);
  lines[k] = l;
  lines_d[k] = line_to_d(l);
}
#endif

#if HBX_IN_TU(2)
// Share verification, one lane per share (lane = sender i, blockIdx.y = proposer j):
// e(S_ji, H_j) * e(-pk_i, W_j) == 1 over the prepared lines of H_j / W_j (wave-uniform loads)
// with one shared final exponentiation.  At N=256 one epoch is 65,536 independent checks: one
// lane each keeps every lane of every wave busy with useful work (the throughput-optimal
// mapping; the 16-lane group executor is kept for the latency-bound per-proposer checks).
//
// Own-share mode (me < n, hbx_set_own_share): sender `me` is this node and its share S_j,me =
// sk_me U_j was computed by k_prepare_ct, not received.  With U_j in G1, W_j and H_j in G2 (the
// decode checks membership), e(sk U, H) e(-sk g1, W) = (e(U, H) / e(g1, W))^sk and sk != 0 mod r,
// so that lane's check is exactly Ciphertext::verify (honey_badger.rs:371): its result is also
// written to ct_valid[j], and the separate 256 ciphertext checks are not needed.
__global__ void __launch_bounds__(64) k_verify_shares(const g1a* __restrict__ S, const int32_t* __restrict__ s_status,
                                                      const uint8_t* __restrict__ present,
                                                      const g1a* __restrict__ pk, uint32_t n_keys,
                                                      const g2a* __restrict__ G2pts,
                                                      const line_block_d* __restrict__ lines,
                                                      const uint8_t* __restrict__ ct_ok, uint32_t n,
                                                      uint8_t* __restrict__ valid, uint32_t me,
                                                      uint8_t* __restrict__ ct_valid, uint32_t fallback_only,
                                                      uint32_t* __restrict__ fallback_lanes) {
  __shared__ uint32_t gslots[LDS_FQ12D_DWORDS * LDS_FQ12_STRIDE];  // final-exp base, one slot per lane
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = blockIdx.y;
  if (i >= n) return;
  const size_t idx = (size_t)j * n + i;
  if (fallback_only) {
    if (valid[idx] != SHARE_FALLBACK) return;  // the lanes k_fe1 could not decide
    if (fallback_lanes) atomicAdd(fallback_lanes, 1u);  // hbx_get_fallback_lanes
  }
  const uint8_t res = share_precheck(s_status[idx], present == nullptr || present[idx] || i == me, i < n_keys,
                                     ct_ok[j] != 0);
  bool v = false;
  if (res == HBX_SHARE_VALID) {
    // check2_lds in the signed-digit tower (pairingd.hpp): Miller loop and final exponentiation
    const g1a sh = S[idx], pki = pk[i];
    const bool skipA = sh.inf || G2pts[2 * j].inf;
    const bool skipB = pki.inf || G2pts[2 * j + 1].inf;
    if (skipA && skipB) {
      v = true;
    } else {
      // the G1 coordinates wait in this lane's LDS slot during the Miller loop (pairingd.hpp)
      lds_u32* slot = (lds_u32*)(gslots + threadIdx.x);
      park_put_fqd(slot, 0, fqd_from_fq(sh.x));
      park_put_fqd(slot, 1, fqd_from_fq(sh.y));
      park_put_fqd(slot, 2, fqd_from_fq(pki.x));
      park_put_fqd(slot, 3, fqd_neg(fqd_from_fq(pki.y)));
      const fq12d fd = miller_loop2_parked_d(lines[j].h, !skipA, lines[j].w, !skipB, slot);
      v = fq12d_is_one(final_exponentiation_d(fd, slot));
    }
  }
  valid[idx] = res == HBX_SHARE_VALID ? (v ? HBX_SHARE_VALID : HBX_SHARE_INVALID) : res;
  if (i == me && ct_valid) ct_valid[j] = !ct_ok[j] ? HBX_CT_UNDECODABLE : v ? HBX_CT_VALID : HBX_CT_INVALID;
}

// One lane per share, the Miller loop only (k_verify_shares up to its final exponentiation): the
// Miller value conj(f) goes to the lane's global slot F (fe1d.hpp) for the four k_fe1 kernels, the
// share status byte is final unless it is SHARE_PENDING (k_fe1<5> decides those).
__global__ void __launch_bounds__(64) k_verify_shares_ml(const g1a* __restrict__ S, const int32_t* __restrict__ s_status,
                                                         const uint8_t* __restrict__ present,
                                                         const g1a* __restrict__ pk, uint32_t n_keys,
                                                         const g2a* __restrict__ G2pts,
                                                         const line_block_d* __restrict__ lines,
                                                         const uint8_t* __restrict__ ct_ok, uint32_t n,
                                                         uint8_t* __restrict__ valid, uint32_t me,
                                                         uint32_t* __restrict__ gslot) {
  __shared__ uint32_t park[LDS_FQ12D_DWORDS * LDS_FQ12_STRIDE];  // the G1 points, one slot per lane
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = blockIdx.y;
  if (i >= n) return;
  const size_t idx = (size_t)j * n + i;
  uint8_t res = share_precheck(s_status[idx], present == nullptr || present[idx] || i == me, i < n_keys,
                               ct_ok[j] != 0);
  if (res == HBX_SHARE_VALID) {
    const g1a sh = S[idx], pki = pk[i];
    const bool skipA = sh.inf || G2pts[2 * j].inf;
    const bool skipB = pki.inf || G2pts[2 * j + 1].inf;
    if (!(skipA && skipB)) {
      lds_u32* slot = (lds_u32*)(park + threadIdx.x);
#if HBX_ML_SCALED
      // lines divided by y_P (pairingd.hpp miller_loop2_scaled_d): (x/y, 1/y) of S and of -[m] pk_i
      park_scaled_points(slot, sh.x, sh.y, sh.inf, pki.x, fq_neg(pki.y), pki.inf);
      const fq12d fd = miller_loop2_scaled_d(lines[j].h, !skipA, lines[j].w, !skipB, slot);
#else
      park_put_fqd(slot, 0, fqd_from_fq(sh.x));
      park_put_fqd(slot, 1, fqd_from_fq(sh.y));
      park_put_fqd(slot, 2, fqd_from_fq(pki.x));
      park_put_fqd(slot, 3, fqd_neg(fqd_from_fq(pki.y)));
      const fq12d fd = miller_loop2_parked_d(lines[j].h, !skipA, lines[j].w, !skipB, slot);
#endif
      uint32_t* gf = gslot + (size_t)(blockIdx.y * gridDim.x + blockIdx.x) * (3 * FE1_WORDS * 64) + threadIdx.x;
      s1_put_fq12d<64>(gf, fq12d{fd.c0, fq6d_norm(fd.c1)});
      res = SHARE_PENDING;
    }
  }
  valid[idx] = res;
}

#ifndef HBX_V3_WAVES
#define HBX_V3_WAVES 1
#endif
// k_verify_shares with THREE lanes per share (pairing3.hpp): 21 checks per wave, ~2.5x lower
// latency per check.  Used when a launch has too few shares to fill the chip one lane per share
// (an epoch shard on one of several GPUs).  Same inputs, outputs and own-share semantics.
__global__ void __launch_bounds__(64, HBX_V3_WAVES) k_verify_shares3(const g1a* __restrict__ S, const int32_t* __restrict__ s_status,
                                                       const uint8_t* __restrict__ present,
                                                       const g1a* __restrict__ pk, uint32_t n_keys,
                                                       const g2a* __restrict__ G2pts,
                                                       const line_block_d* __restrict__ lines,
                                                       const uint8_t* __restrict__ ct_ok, uint32_t n,
                                                       uint8_t* __restrict__ valid, uint32_t me,
                                                       uint8_t* __restrict__ ct_valid) {
  const int lane = (int)(threadIdx.x & 63);
  const grp3 g = grp3_of_lane();
  const uint32_t i = blockIdx.x * G3_PER_WAVE + (uint32_t)(lane / G3);
  const uint32_t j = blockIdx.y;
  if (lane == 63 || i >= n) return;  // whole groups
  const size_t idx = (size_t)j * n + i;
  const uint8_t res = share_precheck(s_status[idx], present == nullptr || present[idx] || i == me, i < n_keys,
                                     ct_ok[j] != 0);
  bool v = false;
  if (res == HBX_SHARE_VALID) {
    g1a npk = pk[i];
    npk.y = fq_neg(npk.y);
    v = check2_g3d(lines[j].h, S[idx], G2pts[2 * j].inf, lines[j].w, npk, G2pts[2 * j + 1].inf, g);
  }
  if (g.gl == 0) {
    valid[idx] = res == HBX_SHARE_VALID ? (v ? HBX_SHARE_VALID : HBX_SHARE_INVALID) : res;
    if (i == me && ct_valid) ct_valid[j] = !ct_ok[j] ? HBX_CT_UNDECODABLE : v ? HBX_CT_VALID : HBX_CT_INVALID;
  }
}
#endif

#if HBX_IN_TU(8) || HBX_IN_TU(9) || HBX_IN_TU(10)
// The final-exponentiation steps F0..F6 of the one-lane share checks (fe1d.hpp) as four kernels
// (k_fe1<0>, <1>, <3>, <5>), over the same grid as k_verify_shares_ml (lane = sender i, blockIdx.y =
// proposer j).  Lanes whose status is not SHARE_PENDING have nothing to do.  The last kernel (F5 +
// F6) turns SHARE_PENDING into HBX_SHARE_VALID / INVALID and,
// in own-share mode, writes the own lane's verdict as Ciphertext::verify (k_verify_shares).
#ifndef HBX_FE1_LANE_LDS
#define HBX_FE1_LANE_LDS 0
#endif
template <int STEP>
__global__ void __launch_bounds__(64) k_fe1(uint32_t* __restrict__ gslot, uint32_t n, uint8_t* __restrict__ valid,
                                            const uint8_t* __restrict__ ct_ok, uint32_t me,
                                            uint8_t* __restrict__ ct_valid, uint32_t force_fallback) {
  __shared__ uint32_t slots[FE1_WORDS * 64];  // slot A, lane-interleaved (one wave per SIMD)
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = blockIdx.y;
  if (i >= n) return;
  const size_t idx = (size_t)j * n + i;
  const uint8_t st = valid[idx];
  if (st != SHARE_PENDING) {
    if (STEP == FE1_LAST && i == me && ct_valid && st != SHARE_FALLBACK)
      ct_valid[j] = !ct_ok[j] ? HBX_CT_UNDECODABLE : st == HBX_SHARE_VALID ? HBX_CT_VALID : HBX_CT_INVALID;
    return;
  }
#if HBX_FE1_LANE_LDS
  const lane_lds a{(lds_u32*)slots};  // the slot addressed afresh at every access (fe1d.hpp)
#else
  lds_u32* a = (lds_u32*)(slots + threadIdx.x);
#endif
  uint32_t* gf = gslot + (size_t)(blockIdx.y * gridDim.x + blockIdx.x) * (3 * FE1_WORDS * 64) + threadIdx.x;
  uint32_t* gt = gf + FE1_WORDS * 64;
  uint32_t* gg = gt + FE1_WORDS * 64;
  // force_fallback (tests only, hbx_debug_force_fallback): every force_fallback-th sender's lane
  // takes the degenerate path, so the fallback check is exercised
  bool degenerate = STEP == 1 && force_fallback && (i % force_fallback) == 0;
  if (STEP == 0) {
    if (fe1_step0<64, 64>(a, gf, gt, gg)) {  // t = 1 after the easy part: the check holds (fe1d.hpp)
      valid[idx] = HBX_SHARE_VALID;
      if (i == me && ct_valid) ct_valid[j] = !ct_ok[j] ? HBX_CT_UNDECODABLE : HBX_CT_VALID;
      return;
    }
  } else if (STEP == 1) {  // F1 + F2
    fe1_step12<64, 64>(a, gt, gg, degenerate);
  } else if (STEP == 3) {  // F3 + F4
    fe1_step34<64, 64>(a, gf, gt, gg, degenerate);
  } else {  // F5 + F6: the verdict
    const bool v = fq12d_is_one_seq(fe1_step56<64, 64>(a, gf, gt, degenerate));
    if (!degenerate) {
      valid[idx] = v ? HBX_SHARE_VALID : HBX_SHARE_INVALID;
      if (i == me && ct_valid) ct_valid[j] = !ct_ok[j] ? HBX_CT_UNDECODABLE : v ? HBX_CT_VALID : HBX_CT_INVALID;
    }
  }
  if (degenerate) valid[idx] = SHARE_FALLBACK;
}
// the four step kernels compile in three translation units (tools/build.py): each is a large kernel
#if HBX_IN_TU(8)
template __global__ void k_fe1<0>(uint32_t*, uint32_t, uint8_t*, const uint8_t*, uint32_t, uint8_t*, uint32_t);
template __global__ void k_fe1<5>(uint32_t*, uint32_t, uint8_t*, const uint8_t*, uint32_t, uint8_t*, uint32_t);
#elif HBX_IN_TU(9)
template __global__ void k_fe1<1>(uint32_t*, uint32_t, uint8_t*, const uint8_t*, uint32_t, uint8_t*, uint32_t);
#else
template __global__ void k_fe1<3>(uint32_t*, uint32_t, uint8_t*, const uint8_t*, uint32_t, uint8_t*, uint32_t);
#endif
#endif

#if HBX_IN_TU(7)
// k_verify_shares with TWO lanes per share (pairing2d.hpp): lane pair = sender i, blockIdx.y =
// proposer j, 32 checks per wave.  The throughput kernel of a whole epoch on one GPU: per check the
// same Fq2-product count as one lane (a little less: scaled lines), half of it on each lane, with
// the Fq12 state split so that nothing spills; the final exponentiation's saved values sit in two
// packed LDS slots per lane (FE2_PROG).  Same inputs, outputs and own-share semantics.
__global__ void __launch_bounds__(64) k_verify_shares2(const g1a* __restrict__ S, const int32_t* __restrict__ s_status,
                                                       const uint8_t* __restrict__ present,
                                                       const g1a* __restrict__ pk, uint32_t n_keys,
                                                       const g2a* __restrict__ G2pts,
                                                       const line_block_d* __restrict__ lines,
                                                       const uint8_t* __restrict__ ct_ok, uint32_t n,
                                                       uint8_t* __restrict__ valid, uint32_t me,
                                                       uint8_t* __restrict__ ct_valid, uint32_t* __restrict__ gslot) {
  // per lane: the Miller loop's scratch, then the final exponentiation's slots A (words 0..77)
  // and B (78..155); slots G1 (t^3, then d) and G2 (b) in global memory
  __shared__ uint32_t region[LDS2_DWORDS * 64];
  const int lane = (int)(threadIdx.x & 63);
  const bool l1 = (lane & 1) != 0;
  const uint32_t i = blockIdx.x * 32 + (uint32_t)(lane >> 1);
  const uint32_t j = blockIdx.y;
  if (i >= n) return;  // whole pairs
  const size_t idx = (size_t)j * n + i;
  const uint8_t res = share_precheck(s_status[idx], present == nullptr || present[idx] || i == me, i < n_keys,
                                     ct_ok[j] != 0);
  bool v = false;
  if (res == HBX_SHARE_VALID) {
    const g1a sh = S[idx], pki = pk[i];
    const bool skipA = sh.inf || G2pts[2 * j].inf;
    const bool skipB = pki.inf || G2pts[2 * j + 1].inf;
    if (skipA && skipB) {
      v = true;
    } else {
      lds_u32* reg = (lds_u32*)region;
      const int pl = lane & ~1;
      const slot2<lds_u32*> A{reg + pl, 64u}, B{reg + LDS_FQ6D_PACKED * 64 + pl, 64u};
      // global slots: [block][slot][word][64 lanes], so a wave's accesses are contiguous
      uint32_t* gb = gslot + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * (2 * LDS_FQ6D_PACKED * 64) + pl;
      const slot2<uint32_t*> G1{gb, 64u}, G2{gb + LDS_FQ6D_PACKED * 64, 64u};
      const uint32_t flags = (l1 ? 1u : 0u) | (skipA ? 0u : 2u) | (skipB ? 0u : 4u);
      check2d_miller(lines[j].h, sh, lines[j].w, pki, flags, (lds2)(reg + lane), B);
      bool dg = false;  // Granger-Scott squarings only: no decompression, never degenerate
      v = final_exp2d_is_one<false>(A, B, G1, G2, l1, dg);
    }
  }
  if (!l1) {
    valid[idx] = res == HBX_SHARE_VALID ? (v ? HBX_SHARE_VALID : HBX_SHARE_INVALID) : res;
    if (i == me && ct_valid) ct_valid[j] = !ct_ok[j] ? HBX_CT_UNDECODABLE : v ? HBX_CT_VALID : HBX_CT_INVALID;
  }
}
#endif

// B1 on TWO lanes per check (k_verify_sig_shares2): the check's two Miller loops are independent,
// so lane 2m runs f_A = f_{|x|,H}(pk_i) and lane 2m + 1 runs f_B = f_{|x|,sigma_i}(-g1), each with
// its lines generated on the fly (pairingd.hpp miller_loop_mixed_d with one pair: the same code on
// both lanes, different data -- no divergence), then the pair multiplies the two results into the
// split form f = A0 + A1 w in LDS slot B (pairing2d.hpp op_mul) and runs the two-lane final
// exponentiation (final_exp2d_is_one, no scratch).  Per lane the Miller loop is ~74 % of the
// one-lane check's (one pair's lines, the squarings on both lanes), and 32,768 checks fill 1,024
// waves instead of 512.  Same verdicts as k_verify_sig_shares (common_coin.rs:151).
#if HBX_IN_TU(7)
// Split in two kernels, each register-allocated on its own: k_verify_sig_shares2 runs the pair's
// Miller loops (sigma's membership in G2 from lane 1's T) and the pair product, and leaves the
// product's halves in the pair's global slot G1 with status SHARE_PENDING; k_verify_sig_shares2_fe
// runs the two-lane final exponentiation of the pending pairs.  Same grid for both.
// Since round 6 H''s lines come prepared (Hlines: [instance][68], k_prepare_lines +
// k_normalise_lines once per instance) and the pair generates sigma's lines together
// (pairing2d.hpp miller_gen2s); the round-5 schedule -- each lane generating its own pair's lines
// (miller_gen2d) -- remains for Hlines = nullptr.
__global__ void __launch_bounds__(64) k_verify_sig_shares2(const g2a* __restrict__ H, const g1a* __restrict__ pk,
                                                           uint32_t n_keys, const g2a* __restrict__ sig,
                                                           const int32_t* __restrict__ sig_status,
                                                           const uint8_t* __restrict__ present, uint32_t n,
                                                           uint8_t* __restrict__ valid, uint32_t* __restrict__ gslot,
                                                           uint32_t retry, const line_pre_d* __restrict__ Hlines) {
  __shared__ uint32_t region[LDS2_DWORDS * 64];
  const int lane = (int)(threadIdx.x & 63);
  const bool l1 = (lane & 1) != 0;
  const uint32_t i = blockIdx.x * 32 + (uint32_t)(lane >> 1);
  const uint32_t inst = blockIdx.y;
  if (i >= n) return;  // whole pairs
  const size_t idx = (size_t)inst * n + i;
  // retry: only the pairs k_verify_sig_shares2_fe<true> sent back (SHARE_FALLBACK), Miller again
  if (retry && valid[idx] != SHARE_FALLBACK) return;  // pair-uniform
  const uint8_t res = share_precheck(sig_status[idx], present == nullptr || present[idx], i < n_keys, true);
  bool tf = true;
  if (res == HBX_SHARE_VALID) {
    // lane 0: e(pk_i, H'); lane 1: e(-[m] g1, sigma_i)  (H' = [m] H: the same verdict)
    const g2a* qp = l1 ? sig + idx : H + inst;
    const g2a Q = *qp;
    g1a P;
    if (l1) {
      P.x = fq_from_const(G1_MGEN_X);
      P.y = fq_neg(fq_from_const(G1_MGEN_Y));
      P.inf = false;
    } else {
      P = pk[i];
    }
    const bool use = !(Q.inf || P.inf);  // a pairing with the identity contributes 1
    lds_u32* reg = (lds_u32*)region;
    const int pl = lane & ~1;
    g2jd T;
    fq6d f;
    if (Hlines) {
      // both lanes: pk_i's scalars (lane 0 1 / y, lane 1 x / y), sigma at -[m] g1 (pair-uniform flags)
      const g1a pki = pk[i];
      const g2a Hq = H[inst], Sq = sig[idx];
      fqd sc = fqd_zero();
      if (!pki.inf) sc = point_scalar2d(pki, false, l1);
      f = miller_gen2s(Hlines + (size_t)inst * MILLER_LINES, sc, !(Hq.inf || pki.inf), sig + idx,
                       fqd_from_fq(fq_from_const(G1_MGEN_X)), fqd_from_fq(fq_neg(fq_from_const(G1_MGEN_Y))), !Sq.inf,
                       l1, (lds2)(reg + lane), reg + pl, T);
    } else {
      f = miller_gen2d(qp, fqd_from_fq(P.x), fqd_from_fq(P.y), use, l1, (lds2)(reg + lane), reg + pl, T);
    }
    // sigma's membership in G2 from lane 1's T = [|x|] sigma (decode skipped it); lane 0's is H's
    tf = !l1 || g2_torsion_free_from_T(T, Q);
    // this lane's half of f_A f_B to the pair's global slot
    uint32_t* gb = gslot + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * (2 * LDS_FQ6D_PACKED * 64) + pl;
    slot_put_fq6d(gb + (l1 ? 1 : 0), 64u, fq6d_reduce(f));
  }
  // lane 1's membership bit to lane 0 (the pair is active or inactive together).  The exchange runs
  // on every lane before the bits are combined: inside `tf && ...` lane 1 (tf false) would skip it
  // and lane 0 would read lane 1's unwritten operand register.
  const int tf_other = __shfl_xor((int)tf, 1);
  const bool tf_pair = tf && tf_other != 0;
  if (!l1) valid[idx] = res != HBX_SHARE_VALID ? res : tf_pair ? SHARE_PENDING : (uint8_t)HBX_SHARE_UNDECODABLE;
}
// KARA: the final exponentiation's runs of 32 and 16 squarings compressed (pairing2d.hpp kara2);
// a pair whose decompression meets g3 = 0 -- or every force_fallback-th share (tests only,
// hbx_debug_force_fallback) -- becomes SHARE_FALLBACK and is counted in *fb; the host then runs
// k_verify_sig_shares2 (retry) and k_verify_sig_shares2_fe<false> on those pairs alone.
template <bool KARA>
__global__ void __launch_bounds__(64) k_verify_sig_shares2_fe(uint32_t n, uint8_t* __restrict__ valid,
                                                              uint32_t* __restrict__ gslot, uint32_t force_fallback,
                                                              uint32_t* __restrict__ fb) {
  __shared__ uint32_t region[LDS2_DWORDS * 64];
  const int lane = (int)(threadIdx.x & 63);
  const bool l1 = (lane & 1) != 0;
  const uint32_t i = blockIdx.x * 32 + (uint32_t)(lane >> 1);
  if (i >= n) return;
  const size_t idx = (size_t)blockIdx.y * n + i;
  if (valid[idx] != SHARE_PENDING) return;  // pair-uniform
  lds_u32* reg = (lds_u32*)region;
  const int pl = lane & ~1;
  const slot2<lds_u32*> A{reg + pl, 64u}, B{reg + LDS_FQ6D_PACKED * 64 + pl, 64u};
  uint32_t* gb = gslot + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * (2 * LDS_FQ6D_PACKED * 64) + pl;
  const slot2<uint32_t*> G1{gb, 64u}, G2{gb + LDS_FQ6D_PACKED * 64, 64u};
  const int h = l1 ? 1 : 0;
#pragma unroll 6
  for (int k = 0; k < LDS_FQ6D_PACKED; k++) B.half(h)[k * 64] = gb[h + k * 64];
  HBX_SEQ();
  bool degenerate = KARA && force_fallback && (i % force_fallback) == 0;
  const bool v = final_exp2d_is_one<KARA>(A, B, G1, G2, l1, degenerate);
  if (!l1) {
    if (KARA && degenerate) {
      valid[idx] = SHARE_FALLBACK;
      atomicAdd(fb, 1u);
    } else {
      valid[idx] = v ? HBX_SHARE_VALID : HBX_SHARE_INVALID;
    }
  }
}
template __global__ void k_verify_sig_shares2_fe<true>(uint32_t, uint8_t*, uint32_t*, uint32_t, uint32_t*);
template __global__ void k_verify_sig_shares2_fe<false>(uint32_t, uint8_t*, uint32_t*, uint32_t, uint32_t*);
#endif

constexpr int COMBINE_THREADS = 256;
constexpr int COMBQ_TERMS = 16;  // k_combine_q: terms (quads) per one-wave block
constexpr int COMBINE_MAX_T = 4096;
constexpr int COMBINE_LDS_T = 512;  // Lagrange x_k cached in LDS up to this threshold
// threshold_crypto interpolate: lambda_k(0) = prod_{m != k} x_m / (x_m - x_k) over Fr with
// x = index + 1 (canonical, little-endian limbs out).
__device__ fr lagrange_at_zero(const uint16_t* idx, int t, int k) {
  fr num = fr_from_const(FR_ONE), den = fr_from_const(FR_ONE);
  fr xk;
  for (int q = 0; q < 8; q++) xk.l[q] = 0;
  xk.l[0] = (uint32_t)idx[k] + 1;
  xk = fr_to_mont(xk);
  for (int m = 0; m < t; m++) {
    if (m == k) continue;
    fr xm;
    for (int q = 0; q < 8; q++) xm.l[q] = 0;
    xm.l[0] = (uint32_t)idx[m] + 1;
    xm = fr_to_mont(xm);
    num = fr_mul(num, xm);
    den = fr_mul(den, fr_sub(xm, xk));
  }
  return fr_from_mont(fr_mul(num, fr_inv(den)));
}

#if HBX_IN_TU(1)
// Lagrange combine of the first t valid shares of proposer j (one 256-thread block per
// proposer), then the hash_bytes key = SHA-256(compress(g)).

__global__ void __launch_bounds__(COMBINE_THREADS) k_combine(const uint8_t* __restrict__ valid,
                                                             const g1a* __restrict__ S, uint32_t n,
                                                             uint32_t t, const uint8_t* __restrict__ ct_valid,
                                                             uint32_t* __restrict__ keys,
                                                             int32_t* __restrict__ status, int digest) {
  __shared__ uint16_t idx[COMBINE_MAX_T];
  __shared__ int wcnt[COMBINE_THREADS / 64];
  __shared__ fr xm[COMBINE_LDS_T];  // Montgomery x_k = idx_k + 1 (t <= COMBINE_LDS_T)
  __shared__ fr nall;               // prod_k x_k
  __shared__ fr tp[COMBINE_LDS_T];  // its product tree
  __shared__ g1j red[COMBINE_THREADS];
  const uint32_t j = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // the first t valid senders in index order (BTreeMap order, honey_badger.rs:328-340): a
  // block-wide ballot compaction, 256 senders per step
  int count = 0;
  for (uint32_t i0 = 0; i0 < n && count < (int)t; i0 += COMBINE_THREADS) {
    const uint32_t i = i0 + (uint32_t)tid;
    const bool ok = i < n && valid[(size_t)j * n + i] == HBX_SHARE_VALID;
    const uint64_t b = __ballot(ok);
    if (lane == 0) wcnt[wv] = __popcll(b);
    __syncthreads();
    int before = count, total = 0;
    for (int q = 0; q < COMBINE_THREADS / 64; q++) {
      if (q < wv) before += wcnt[q];
      total += wcnt[q];
    }
    const int pos = before + __popcll(b & ((1ull << lane) - 1));
    if (ok && pos < (int)t) idx[pos] = (uint16_t)i;
    count += total;
    __syncthreads();
  }
  const bool ctv = ct_valid[j] == HBX_CT_VALID;
  if (!ctv || count < (int)t) {
    if (tid == 0) status[j] = !ctv ? -7 : -3;
    return;
  }
  // Lagrange numerators shared through LDS: lambda_k = N / (x_k prod_{m != k} (x_m - x_k)) with
  // N = prod_m x_m (one product per block instead of t - 1 per lane)
  const bool lds_lag = t <= (uint32_t)COMBINE_LDS_T;
  if (lds_lag) {
    for (int k = tid; k < (int)t; k += COMBINE_THREADS) {
      fr x;
      for (int q = 0; q < 8; q++) x.l[q] = 0;
      x.l[0] = (uint32_t)idx[k] + 1;
      xm[k] = fr_to_mont(x);
    }
    for (int k = tid; k < (int)t; k += COMBINE_THREADS) tp[k] = xm[k];
    __syncthreads();
    // N = prod_k x_k by a product tree (ceil(log2 t) levels instead of t - 1 products on one lane)
    for (int cnt = (int)t; cnt > 1;) {
      const int half = (cnt + 1) >> 1;
      for (int i = tid; i < cnt - half; i += COMBINE_THREADS) tp[i] = fr_mul(tp[i], tp[i + half]);
      __syncthreads();
      cnt = half;
    }
    if (tid == 0) nall = tp[0];
    __syncthreads();
  }
  // two lanes per share (GLV): lane 2k computes k1 S_k, lane 2k+1 computes k2 phi(S_k) with
  // lambda_k = k1 + k2 lambda -- two independent 128-bit scalar multiplications instead of one
  // 255-bit one, halving the latency of the per-proposer combine
  g1j acc = g1_identity();
  for (int q = tid; q < 2 * (int)t; q += COMBINE_THREADS) {
    const int k = q >> 1;
    fr lam;
    if (lds_lag) {
      // the denominator x_k prod_{m != k} (x_m - x_k) split over the lane pair of share k (lane 2k
      // takes m < t/2, lane 2k + 1 the rest), the halves multiplied after one exchange
      const fr xk = xm[k];
      const int h = q & 1, m0 = h ? (int)t / 2 : 0, m1 = h ? (int)t : (int)t / 2;
      fr den = h ? fr_from_const(FR_ONE) : xk;
      for (int m = m0; m < m1; m++)
        if (m != k) den = fr_mul(den, fr_sub(xm[m], xk));
      fr other;
#pragma unroll
      for (int w = 0; w < 8; w++) other.l[w] = (uint32_t)__shfl_xor((int)den.l[w], 1);
      den = fr_mul(den, other);
      lam = fr_from_mont(fr_mul(nall, fr_inv(den)));
    } else {
      lam = lagrange_at_zero(idx, (int)t, k);
    }
    uint32_t k1[4], k2[4];
    g1_glv_split(lam.l, k1, k2);
    g1a sp = S[(size_t)j * n + idx[k]];
    if (q & 1) sp.x = fq_mul(sp.x, fq_from_const(G1_BETA));
    acc = g1_add(acc, g1d_mul_u128_w4(sp, (q & 1) ? k2 : k1));  // digit tower (g1d.hpp)
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
    digest2(digest, comp, 48, nullptr, 0, d);  // hash_bytes seed = DIGEST(compress(g))
    for (int q = 0; q < 8; q++)
      keys[(size_t)j * 8 + q] = ((uint32_t)d[4 * q] << 24) | ((uint32_t)d[4 * q + 1] << 16) |
                                ((uint32_t)d[4 * q + 2] << 8) | d[4 * q + 3];
    status[j] = 0;
  }
}

// k_combine for launches that leave most of the chip idle (an epoch shard: p x 172 terms at
// t = 86 on 1024 SIMDs): the 2t GLV terms of proposer j spread over COMBQ_TERMS-term one-wave
// blocks (blockIdx.x), a QUAD of lanes per term (curve4.hpp: the doubling in 3 product rounds, the
// addition in 5 -- 1.5 instead of 2.0 ms per 128-bit multiplication for a lone wave,
// profiles/r03l_microbench_combine.txt); each block computes the Lagrange coefficients of its own
// 8 shares (8 lanes per share), sums its terms, and the last block of the proposer to finish
// (a device-scope counter) sums the partials and derives the key.  Same index set, the same
// lambda_k and the same sum as k_combine, so the same keys and statuses.  t <= COMBINE_LDS_T.
__device__ __forceinline__ g1j g1j_shfl_xor_q(const g1j& a, int m) {
  g1j r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.x.l[i] = (uint32_t)__shfl_xor((int)a.x.l[i], m);
    r.y.l[i] = (uint32_t)__shfl_xor((int)a.y.l[i], m);
    r.z.l[i] = (uint32_t)__shfl_xor((int)a.z.l[i], m);
  }
  return r;
}
__global__ void __launch_bounds__(64, 1) k_combine_q(const uint8_t* __restrict__ valid, const g1a* __restrict__ S,
                                                     uint32_t n, uint32_t t, const uint8_t* __restrict__ ct_valid,
                                                     uint32_t* __restrict__ keys, int32_t* __restrict__ status,
                                                     int digest, g1j* __restrict__ partial,
                                                     uint32_t* __restrict__ done) {
  __shared__ uint16_t idx[COMBINE_LDS_T];
  __shared__ fr xm[COMBINE_LDS_T];
  __shared__ uint32_t lk[COMBQ_TERMS / 2][8];
  const uint32_t j = blockIdx.y, b = blockIdx.x, nb = gridDim.x;
  const int lane = threadIdx.x, s = lane & 3, qd = lane >> 2;
  // the first t valid senders in index order, 64 per step (as k_combine)
  int count = 0;
  for (uint32_t i0 = 0; i0 < n && count < (int)t; i0 += 64) {
    const uint32_t i = i0 + (uint32_t)lane;
    const bool ok = i < n && valid[(size_t)j * n + i] == HBX_SHARE_VALID;
    const uint64_t bal = __ballot(ok);
    const int pos = count + __popcll(bal & ((1ull << lane) - 1));
    if (ok && pos < (int)t) idx[pos] = (uint16_t)i;
    count += __popcll(bal);
  }
  const bool ctv = ct_valid[j] == HBX_CT_VALID;
  if (!ctv || count < (int)t) {
    if (b == 0 && lane == 0) status[j] = !ctv ? -7 : -3;
    return;  // every block of the proposer returns here: the counter is untouched
  }
  __syncthreads();
  for (int k = lane; k < (int)t; k += 64) {
    fr x;
#pragma unroll
    for (int q = 0; q < 8; q++) x.l[q] = 0;
    x.l[0] = (uint32_t)idx[k] + 1;
    xm[k] = fr_to_mont(x);
  }
  __syncthreads();
  // lambda_k = N / (x_k prod_{m != k} (x_m - x_k)) for this block's shares k = 8b + kk: 8 lanes per
  // share, each a slice of N's factors and of the denominator's, multiplied across the 8 lanes
  {
    const int kk = lane >> 3, part = lane & 7;
    const int k = (int)(COMBQ_TERMS / 2 * b) + kk;
    const bool have = k < (int)t;
    const fr xk = xm[have ? k : 0];
    fr num = fr_from_const(FR_ONE), den = part == 0 ? xk : fr_from_const(FR_ONE);
    for (int m = part; m < (int)t; m += 8) {
      num = fr_mul(num, xm[m]);
      if (m != k) den = fr_mul(den, fr_sub(xm[m], xk));
    }
#pragma unroll
    for (int w = 1; w < 8; w <<= 1) {
      fr on, od;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        on.l[q] = (uint32_t)__shfl_xor((int)num.l[q], w);
        od.l[q] = (uint32_t)__shfl_xor((int)den.l[q], w);
      }
      num = fr_mul(num, on);
      den = fr_mul(den, od);
    }
    if (have && part == 0) {
      const fr lam = fr_from_mont(fr_mul(num, fr_inv(den)));
      uint32_t k1[4], k2[4];
      g1_glv_split(lam.l, k1, k2);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        lk[kk][q] = k1[q];
        lk[kk][4 + q] = k2[q];
      }
    }
  }
  __syncthreads();
  // one term per quad: GLV half h of share k, lambda_k's half times S_k (h = 0) or phi(S_k)
  const int term = (int)(COMBQ_TERMS * b) + qd;
  g1j acc = g1_identity();
  if (term < 2 * (int)t) {
    const int k = term >> 1, h = term & 1;
    uint32_t kh[4];
#pragma unroll
    for (int q = 0; q < 4; q++) kh[q] = lk[k - COMBQ_TERMS / 2 * (int)b][4 * h + q];
    g1a sp = S[(size_t)j * n + idx[k]];
    if (h) sp.x = fq_mul(sp.x, fq_from_const(G1_BETA));
    acc = g1_mul_u128_w4_q4(sp, kh, s);
  }
  // the block's 16 quads: butterfly over quads (lane xor 4, 8, 16, 32), every quad ends with the sum
#pragma unroll 1
  for (int m = 4; m < 64; m <<= 1) acc = g1_add_q4(acc, g1j_shfl_xor_q(acc, m), s);
  __shared__ uint32_t last;
  if (lane == 0) {
    partial[(size_t)j * nb + b] = acc;
    __threadfence();
    last = atomicAdd(&done[j], 1u) == nb - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  // the last block of proposer j: the nb partials, a quad each, by the same butterfly
  g1j tot = g1_identity();
  if (qd < (int)nb) {
    const volatile g1j* vp = partial + (size_t)j * nb + qd;
#pragma unroll
    for (int i = 0; i < 12; i++) {
      tot.x.l[i] = vp->x.l[i];
      tot.y.l[i] = vp->y.l[i];
      tot.z.l[i] = vp->z.l[i];
    }
  }
#pragma unroll 1
  for (int m = 4; m < 64; m <<= 1) tot = g1_add_q4(tot, g1j_shfl_xor_q(tot, m), s);
  if (lane == 0) {
    done[j] = 0;  // ready for the next launch
    const g1a g = g1_to_affine(tot);
    uint8_t comp[48], d[32];
    g1_compress(g, comp);
    digest2(digest, comp, 48, nullptr, 0, d);  // hash_bytes seed = DIGEST(compress(g))
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

#endif

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

#if HBX_IN_TU(3)
// k_verify_shares with SIX lanes per share (pairing3d.hpp check2_g6d: the two Miller loops on
// two triplets side by side): 10 checks per wave.  For launches small enough that twice the
// three-lane wave count still leaves at most one wave per SIMD (an epoch shard).  Same inputs,
// outputs and own-share semantics.
__global__ void __launch_bounds__(64, 1) k_verify_shares6(const g1a* __restrict__ S, const int32_t* __restrict__ s_status,
                                                          const uint8_t* __restrict__ present,
                                                          const g1a* __restrict__ pk, uint32_t n_keys,
                                                          const g2a* __restrict__ G2pts,
                                                          const line_block_d* __restrict__ lines,
                                                          const uint8_t* __restrict__ ct_ok, uint32_t n,
                                                          uint8_t* __restrict__ valid, uint32_t me,
                                                          uint8_t* __restrict__ ct_valid) {
  const int lane = (int)(threadIdx.x & 63);
  if (lane >= 6 * G6_PER_WAVE) return;
  grp3 g;
  g.gl = lane % 3;
  g.base = lane - g.gl;
  const bool second = ((lane / 3) & 1) != 0;
  const uint32_t i = blockIdx.x * G6_PER_WAVE + (uint32_t)(lane / 6);
  const uint32_t j = blockIdx.y;
  if (i >= n) return;  // whole groups
  const size_t idx = (size_t)j * n + i;
  const uint8_t res = share_precheck(s_status[idx], present == nullptr || present[idx] || i == me, i < n_keys,
                                     ct_ok[j] != 0);
  bool v = false;
  if (res == HBX_SHARE_VALID) {
    g1a npk = pk[i];
    npk.y = fq_neg(npk.y);
    v = check2_g6d(lines[j].h, S[idx], G2pts[2 * j].inf, lines[j].w, npk, G2pts[2 * j + 1].inf, second, g);
  }
  if (lane % 6 == 0) {
    valid[idx] = res == HBX_SHARE_VALID ? (v ? HBX_SHARE_VALID : HBX_SHARE_INVALID) : res;
    if (i == me && ct_valid) ct_valid[j] = !ct_ok[j] ? HBX_CT_UNDECODABLE : v ? HBX_CT_VALID : HBX_CT_INVALID;
  }
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
                                                uint8_t* __restrict__ w96, int digest) {
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
  digest2(digest, gc, 48, nullptr, 0, d);
  chacha_rng rng;
  chacha_rng_from_digest(rng, d);
  const uint64_t o = off[j], len = off[j + 1] - o;
  for (uint64_t q = 0; q < len; q++) v[o + q] = msg[o + q] ^ (uint8_t)chacha_next_u32(rng);
  const g2j h = hash_g1_g2(uc, v + o, len, digest);
  g2_compress(g2_to_affine(g2_mul_bits(h, k, 256)), w96 + (size_t)j * 96);
}

// ----------------------------------------------------------------------------------------------
// SyncKeyGen commitment checks (reference src/sync_key_gen.rs): a Part's
// BivarCommitment C (symmetric, degree t, (t+1)(t+2)/2 G1 points in threshold_crypto's
// coeff_pos order, j (j + 1)/2 + i for i <= j) and the Ack values sent to this node.
// ----------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bivar_pos(uint32_t i, uint32_t j) {
  return i <= j ? j * (j + 1) / 2 + i : i * (i + 1) / 2 + j;
}
// BivarCommitment::row(x) (sync_key_gen.rs:313, :401): R_j = sum_i C_ij x^i by Horner in x, one
// lane per (proposer, j).  pst[q] = HBX_SHARE_UNDECODABLE if any of q's points failed to decode.
__global__ void __launch_bounds__(64) k_bivar_rows(const g1a* __restrict__ C, const int32_t* __restrict__ cst,
                                                   uint32_t p, uint32_t t, uint64_t x, g1j* __restrict__ rows,
                                                   uint8_t* __restrict__ rows48, uint8_t* __restrict__ pst) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= p * (t + 1)) return;
  const uint32_t q = k / (t + 1), j = k % (t + 1);
  const uint32_t M = (t + 1) * (t + 2) / 2;
  const g1a* Cq = C + (size_t)q * M;
  bool ok = true;  // the whole commitment decodes (every lane of q decides the same)
  for (uint32_t m = 0; m < M; m++) {
    const int32_t st = cst[(size_t)q * M + m];
    ok = ok && (st == HBX_PT_OK || st == HBX_PT_INFINITY);
  }
  g1j acc = g1_identity();
  if (ok) {
    for (int i = (int)t; i >= 0; i--) acc = g1_add_mixed_i(g1j_mul_u64(acc, x), Cq[bivar_pos((uint32_t)i, j)]);
  }
  rows[k] = acc;
  if (rows48) g1_compress(g1_to_affine(acc), rows48 + (size_t)k * 48);
  if (j == 0) pst[q] = ok ? HBX_SHARE_VALID : HBX_SHARE_UNDECODABLE;
}
// handle_ack's value check (sync_key_gen.rs:449): commit.evaluate(x, y) = sum_j R_j y^j (Horner in
// y) == g1 * val, one lane per ack.  val must be a canonical Fr (big-endian); otherwise, or when
// the proposer's commitment did not decode, HBX_SHARE_UNDECODABLE.
__global__ void __launch_bounds__(64) k_bivar_check(const g1j* __restrict__ rows, const uint8_t* __restrict__ pst,
                                                    uint32_t t, const uint32_t* __restrict__ ack_p,
                                                    const uint64_t* __restrict__ ack_y,
                                                    const uint8_t* __restrict__ vals32, uint32_t count,
                                                    uint8_t* __restrict__ out) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  const uint32_t q = ack_p[k];
  uint32_t v[8];
  fr_from_be32(vals32 + (size_t)k * 32, v);
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) (void)subb32(v[i], FR_R[i], br);
  if (pst[q] != HBX_SHARE_VALID || !br) {
    out[k] = HBX_SHARE_UNDECODABLE;
    return;
  }
  const g1j* R = rows + (size_t)q * (t + 1);
  g1j acc = g1_identity();
  for (int j = (int)t; j >= 0; j--) acc = g1_add(g1j_mul_u64(acc, ack_y[k]), R[j]);
  const g1j rhs = g1_mul_scalar(g1_from_affine(g1_generator()), v);
  out[k] = g1j_eq(acc, rhs) ? HBX_SHARE_VALID : HBX_SHARE_INVALID;
}
#endif

// ----------------------------------------------------------------------------------------------
// Wide pairing checks: a 16-lane group per check, 8 checks of ONE
// proposer per 128-thread block sharing that proposer's prepared lines through LDS.
//   job q <  n : share check  e(S_jq, H_j) e(-pk_q, W_j) == 1   (verify_decryption_share)
//   job q == n : ct check     e(-U_j, H_j) e(g1, W_j) == 1      (Ciphertext::verify)
// Jobs with a point at infinity are flagged for k_pair_fallback (the identity cases of check2).
// ----------------------------------------------------------------------------------------------
constexpr int WG_GROUPS = 8;
constexpr int WG_THREADS = WG_GROUPS * wide::G;
constexpr int PRIV_SLOTS = prog::MAX_SCRATCH + 12 * prog::NUM_REGIONS + 4;
constexpr int SH_SLOTS = prog::NUM_K + 16;
constexpr int WIDE_LDS_DWORDS = (SH_SLOTS + WG_GROUPS * PRIV_SLOTS) * wide::SLOT;
constexpr uint8_t JOB_FALLBACK = 1;

#if HBX_IN_TU(4)
__device__ __forceinline__ void put_fq(uint32_t* lds, uint32_t off, const fq& a) { wide::lds_store_fq(lds, off, a); }

__global__ void __launch_bounds__(WG_THREADS) k_verify_wide(
    const g1a* __restrict__ S, const int32_t* __restrict__ s_status, const uint8_t* __restrict__ present,
    const g1a* __restrict__ pk, uint32_t n_keys, const g1a* __restrict__ U, const g2a* __restrict__ G2pts,
    const line_block* __restrict__ lines, const uint8_t* __restrict__ ct_ok, uint32_t n, uint32_t q_first,
    uint32_t q_last, uint8_t* __restrict__ valid, uint8_t* __restrict__ ct_valid, uint8_t* __restrict__ fallback) {
  __shared__ uint4 lds4[WIDE_LDS_DWORDS / 4];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  const int tid = threadIdx.x;
  const int grp = tid / wide::G;
  const int lane = tid % wide::G;
  const uint32_t j = blockIdx.y;
  const uint32_t q = q_first + blockIdx.x * WG_GROUPS + grp;
  for (int t = tid; t < prog::NUM_K * wide::SLOT; t += WG_THREADS) lds[t] = prog::KCONST[t / wide::SLOT][t % wide::SLOT];
  const uint32_t gbase = (SH_SLOTS + grp * PRIV_SLOTS) * wide::SLOT;
  const uint32_t rbase = gbase + prog::MAX_SCRATCH * wide::SLOT;
  const uint32_t pbase = rbase + prog::NUM_REGIONS * 12 * wide::SLOT;
  const uint32_t lbase0 = prog::NUM_K * wide::SLOT;

  // ---- job setup: decide what this group computes ----
  const bool in_range = q <= q_last && q <= n;
  const bool ct_job = q == n;
  const bool qa_inf = G2pts[2 * j].inf, qb_inf = G2pts[2 * j + 1].inf;
  bool decodable = ct_ok[j] != 0;
  g1a PA, PB;
  PA.inf = PB.inf = true;
  if (in_range && decodable) {
    if (ct_job) {
      PA = U[j];
      PA.y = fq_neg(PA.y);
      PB.x = fq_from_const(G1_MGEN_X);  // [m] g1 against H' = [m] H
      PB.y = fq_from_const(G1_MGEN_Y);
      PB.inf = false;
    } else {
      const size_t idx = (size_t)j * n + q;
      const int32_t st = s_status[idx];
      decodable = (st == HBX_PT_OK || st == HBX_PT_INFINITY) && q < n_keys && (present == nullptr || present[idx]);
      if (decodable) {
        PA = S[idx];
        PB = pk[q];
        PB.y = fq_neg(PB.y);
      }
    }
  }
  const bool needs_fallback = in_range && decodable && (PA.inf || PB.inf || qa_inf || qb_inf);
  // points: P[0..1] = P_A, P[2..3] = P_B  (any finite value for idle groups)
  if (lane < 4) {
    const g1a& pt = lane < 2 ? PA : PB;
    fq v = (lane & 1) ? pt.y : pt.x;
    if (pt.inf) v = fq_zero();
    put_fq(lds, pbase + lane * wide::SLOT, v);
  }
  if (lane < 12) put_fq(lds, rbase + lane * wide::SLOT, lane == 0 ? fq_one() : fq_zero());
  __syncthreads();

  // ---- the schedule: Miller loop with line loads, then the final exponentiation ----
  wide::bases b;
  b.cls[prog::SCR] = gbase;
  b.cls[prog::PT] = pbase;
  b.cls[prog::K] = 0;
  b.cls[prog::L] = lbase0;
  const line_pre* la = lines[j].h;
  const line_pre* lb = lines[j].w;
  for (int e = 0; e < prog::SCHED_LEN; e++) {
    const uint32_t ent = prog::SCHED[e];
    const int line = (int)(ent >> 16) - 1;
    if (line >= 0) {
      const uint32_t buf = lbase0 + (line & 1) * 8 * wide::SLOT;
      if (tid < 96) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(tid < 48 ? &la[line] : &lb[line]);
        lds[buf + tid] = src[tid % 48];
      }
      b.cls[prog::L] = buf;
      __syncthreads();
    }
    b.cls[prog::X] = rbase + ((ent >> 4) & 0xF) * 12 * wide::SLOT;
    b.cls[prog::Y] = rbase + ((ent >> 8) & 0xF) * 12 * wide::SLOT;
    b.cls[prog::O] = rbase + ((ent >> 12) & 0xF) * 12 * wide::SLOT;
    wide::run(lds, (int)(ent & 0xF), lane, b);
  }

  // ---- result == 1 ? ----
  bool eq = true;
  if (lane < 12) {
    const fq v = fq_canon(wide::lds_load_fq(lds, rbase + (prog::SCHED_RESULT_REGION * 12 + lane) * wide::SLOT));
    const fq one = fq_one();
#pragma unroll
    for (int k = 0; k < 12; k++) eq = eq && v.l[k] == (lane == 0 ? one.l[k] : 0u);
  }
  const uint64_t bal = __ballot(eq);
  const bool ok = ((bal >> ((tid & 63) & ~15)) & 0xFFFFull) == 0xFFFFull;
  if (lane == 0 && in_range) {
    const uint8_t res = (decodable && !needs_fallback && ok) ? 1 : 0;
    if (ct_job) ct_valid[j] = ct_ok[j] ? res : HBX_CT_UNDECODABLE;
    else valid[(size_t)j * n + q] = res;
    fallback[(size_t)j * (n + 1) + q] = needs_fallback ? JOB_FALLBACK : 0;
  }
}
#endif

#if HBX_IN_TU(1)
// One lane per share: decompress S_ji (kept for the verification and the Lagrange combine).
// Decode = pairing 0.14's into_affine (on-curve and G1 membership), as the reference deserialises
// a DecryptionShare.  In own-share mode the entry of sender `me` is this node's own share from
// k_prepare_ct instead of the received bytes.
__global__ void __launch_bounds__(256) k_decompress_shares(const uint8_t* __restrict__ shares, size_t count,
                                                           g1a* __restrict__ S, int32_t* __restrict__ status,
                                                           uint32_t n, uint32_t me, const g1a* __restrict__ own_S) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  if (own_S && (uint32_t)(i % n) == me) {
    const g1a o = own_S[i / n];
    S[i] = o;
    status[i] = o.inf ? HBX_PT_INFINITY : HBX_PT_OK;
    return;
  }
  g1a p;
  int32_t st = g1_decompress_d(shares + i * 48, p);
  if (st == HBX_PT_OK && !g1_is_torsion_free_d(p)) st = HBX_PT_NOT_IN_SUBGROUP;
  status[i] = st;
  S[i] = p;
}
#endif

#if HBX_IN_TU(4)
// Identity cases (a point at infinity on either side) that the wide kernel flagged: e(O, Q) = 1.
__global__ void __launch_bounds__(64) k_pair_fallback(const uint8_t* __restrict__ fallback, const g1a* __restrict__ S,
                                                      const g1a* __restrict__ pk, const g1a* __restrict__ U,
                                                      const g2a* __restrict__ G2pts,
                                                      const line_block* __restrict__ lines, uint32_t n, uint32_t p,
                                                      uint8_t* __restrict__ valid, uint8_t* __restrict__ ct_valid) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (size_t)p * (n + 1) || fallback[k] != JOB_FALLBACK) return;
  const uint32_t j = (uint32_t)(k / (n + 1)), q = (uint32_t)(k % (n + 1));
  g1a PA, PB;
  if (q == n) {
    PA = U[j];
    PA.y = fq_neg(PA.y);
    PB.x = fq_from_const(G1_MGEN_X);  // [m] g1 against H' = [m] H
    PB.y = fq_from_const(G1_MGEN_Y);
    PB.inf = false;
  } else {
    PA = S[(size_t)j * n + q];
    PB = pk[q];
    PB.y = fq_neg(PB.y);
  }
  const bool v = check2(lines[j].h, PA, G2pts[2 * j].inf, lines[j].w, PB, G2pts[2 * j + 1].inf);
  if (q == n) ct_valid[j] = v ? 1 : 0;
  else valid[(size_t)j * n + q] = v ? 1 : 0;
}
#endif

#if HBX_IN_TU(1)
// pk_m[i] = [3(x^2-1)] pk_i (once per key set): the G1 side of the share checks against
// H' = [3(x^2-1)] H (k_prepare_ct).
// pk64[i] = [2^64] pk_i: the coin combine's master identity splits each 128-bit GLV half of
// lambda_k into two 64-bit multiplications, of pk_k and of pk64_k (k_combine_sigs).
__global__ void __launch_bounds__(64) k_scale_keys(const g1a* __restrict__ pk, uint32_t n, g1a* __restrict__ pk_m,
                                                   g1a* __restrict__ pk64) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  pk_m[i] = g1_to_affine(g1_mul_scalar(g1_from_affine(pk[i]), HEFF_M));
  g1j q = g1_from_affine(pk[i]);
#pragma unroll 1
  for (int d = 0; d < 64; d++) q = g1_dbl(q);
  pk64[i] = g1_to_affine(q);
}
// Fixed-base tables of the key shares (once per key set, hbx_set_pk_shares): tab[(i * 64 + w) * 15 +
// d - 1] = [d 16^w] pk_i (affine), d = 1..15, w = 0..63 -- the coin combine's master identity
// sum_k lambda_k pk_k then costs one mixed addition per nonzero 4-bit digit of lambda_k and no
// doublings (k_combine_sigs).  One lane per (key, window): 4w doublings, 14 additions.
__global__ void __launch_bounds__(64) k_g1_tables(const g1a* __restrict__ pk, uint32_t n, g1a* __restrict__ tab) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t i = gid / G1TAB_W, w = gid % G1TAB_W;
  if (i >= n) return;
  g1j b = g1_from_affine(pk[i]);
#pragma unroll 1
  for (uint32_t d = 0; d < 4 * w; d++) b = g1_dbl(b);
  const g1a ba = g1_to_affine(b);
  g1a* out = tab + ((size_t)i * G1TAB_W + w) * G1TAB_D;
  out[0] = ba;
  g1j acc = b;
#pragma unroll 1
  for (int d = 2; d <= G1TAB_D; d++) {
    acc = g1_add_mixed_i(acc, ba);
    out[d - 1] = g1_to_affine(acc);
  }
}
// H_j = hash_g1_g2(U_j, V_j) itself from H'_j = h_eff P (hbx_get_ct_hashes), compressed.
__global__ void __launch_bounds__(64) k_true_hashes(const g2a* __restrict__ G2pts, const g2j* __restrict__ Hj,
                                                    uint32_t count, uint8_t* __restrict__ out96) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= count) return;
  const g2j q = G2pts[2 * j].inf ? g2_identity() : Hj[j];
  g2_compress(g2_to_affine(g2_heff_to_h2(q)), out96 + (size_t)j * 96);
}

// Shares of a ciphertext that failed Ciphertext::verify become HBX_SHARE_SKIPPED_CT: the
// reference never verifies them (honey_badger.rs:371-376), so they are neither valid nor a fault.
__global__ void __launch_bounds__(256) k_gate_by_ct(uint8_t* __restrict__ valid, const uint8_t* __restrict__ ct_valid,
                                                    uint32_t n, uint32_t p) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (size_t)n * p) return;
  if (ct_valid[k / n] != HBX_CT_VALID && valid[k] <= HBX_SHARE_VALID) valid[k] = HBX_SHARE_SKIPPED_CT;
}
#endif

// ----------------------------------------------------------------------------------------------
// Common Coin (reference src/common_coin.rs)
// ----------------------------------------------------------------------------------------------
#if HBX_IN_TU(5)
// combine_signatures over a caller-chosen subset of the verified shares (the shares a node held
// when try_output ran, common_coin.rs:163-190): out[k] = valid[k] where use[k], else ABSENT
__global__ void __launch_bounds__(256) k_coin_use(const uint8_t* __restrict__ valid, const uint8_t* __restrict__ use,
                                                  size_t m, uint8_t* __restrict__ out) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= m) return;
  out[k] = use[k] ? valid[k] : (uint8_t)HBX_SHARE_ABSENT;
}
// H_i = hash_g2(nonce_i) (threshold_crypto; the nonce of agreement/mod.rs:155-165), one HASH_K-lane
// group each.  full = 0: H'_i = h_eff P = [m] H_i (m = 3(x^2 - 1), the decryption checks' trick,
// DESIGN.md §4.2): the coin's share checks take H' with [m] g1 on the G1 side, and the true H_i
// (for SecretKeyShare::sign and the API's output) comes from k_h2_from_heff, off the checks' path.
__global__ void __launch_bounds__(64) k_hash_nonces(const uint8_t* __restrict__ blob, const uint64_t* __restrict__ off,
                                                    uint32_t count, g2a* __restrict__ H, int digest, int full) {
  const uint32_t j = (blockIdx.x * blockDim.x + threadIdx.x) / HASH_K;
  if (j >= count) return;  // whole groups only
  uint8_t d[32];
  digest2(digest, blob + off[j], off[j + 1] - off[j], nullptr, 0, d);
  g2j h;
  if (hash_g2_group<HASH_K>(d, true, h, full != 0)) H[j] = g2_to_affine(h);
}
// H = h2 P from H' = h_eff P (hash.hpp g2_heff_to_h2), one lane per point
__global__ void __launch_bounds__(64) k_h2_from_heff(const g2a* __restrict__ Hp, uint32_t count, g2a* __restrict__ H) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= count) return;
  H[j] = Hp[j].inf ? Hp[j] : g2_to_affine(g2_heff_to_h2(g2_from_affine(Hp[j])));
}

// subgroup = 0: curve membership only -- the coin's share checks (k_verify_sig_shares[2]) take G2
// membership from their Miller loop's [|x|] sigma and report HBX_SHARE_UNDECODABLE themselves.
__global__ void __launch_bounds__(64) k_decompress_g2(const uint8_t* __restrict__ comp, size_t count,
                                                      g2a* __restrict__ out, int32_t* __restrict__ status,
                                                      uint32_t subgroup) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  g2a p;
  // decode = pairing 0.14's into_affine, as a SignatureShare is deserialised: on the curve AND in
  // G2.  A share sig_i + T (T of cofactor order) could otherwise pass the ate check and carry T
  // into the combined signature and its parity bit.
  int32_t st = g2_decompress(comp + i * 96, p);
  if (subgroup && st == HBX_PT_OK && !g2_is_torsion_free(p)) st = HBX_PT_NOT_IN_SUBGROUP;
  status[i] = st;
  out[i] = p;
}

// check_mixed in the signed-digit tower (pairingd.hpp): the same verdict; `slot` is this lane's
// LDS slot for the final exponentiation's base.
__device__ __forceinline__ bool check_mixed_d(const line_pre_d* LA, const g1a& PA, bool qa_inf, const g2a& QB,
                                              const g1a& PB, lds_u32* slot) {
  const bool skipA = PA.inf || qa_inf;
  const bool skipB = PB.inf || QB.inf;
  if (skipA && skipB) return true;
  const fq12d f = miller_loop_mixed_d(LA, fqd_from_fq(PA.x), fqd_from_fq(PA.y), !skipA, fq2d_from_fq2(QB.x),
                                      fq2d_from_fq2(QB.y), fqd_from_fq(PB.x), fqd_from_fq(PB.y), !skipB);
  return fq12d_is_one(final_exponentiation_d(f, slot));
}

// e(PA, QA) e(PB, QB) == 1 with QA prepared and QB's lines on the fly; pairings with the
// identity contribute 1.
__device__ __forceinline__ bool check_mixed(const line_pre* LA, const g1a& PA, bool qa_inf, const g2a& QB,
                                            const g1a& PB) {
  const bool skipA = PA.inf || qa_inf;
  const bool skipB = PB.inf || QB.inf;
  if (skipA && skipB) return true;
  const fq12 f = skipB ? miller_loop2(LA, PA, true, LA, PA, false) : miller_loop_mixed(LA, PA, !skipA, QB, PB, true);
  return fq12_is_one(final_exponentiation(f));
}

// B1: PublicKeyShare::verify(share, nonce) (common_coin.rs:151): e(pk_i, H) == e(g1, sig_i),
// i.e. e(pk_i, H) e(-g1, sig_i) == 1.  Lane = node i, blockIdx.y = coin instance.
__global__ void __launch_bounds__(64) k_verify_sig_shares(const line_pre_d* __restrict__ lines, const g2a* __restrict__ H,
                                                          const g1a* __restrict__ pk, uint32_t n_keys,
                                                          const g2a* __restrict__ sig,
                                                          const int32_t* __restrict__ sig_status,
                                                          const uint8_t* __restrict__ present, uint32_t n,
                                                          uint8_t* __restrict__ valid) {
  __shared__ uint32_t gslots[LDS_FQ12D_DWORDS * LDS_FQ12_STRIDE];  // final-exp base, one slot per lane
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t inst = blockIdx.y;
  if (i >= n) return;
  const size_t idx = (size_t)inst * n + i;
  uint8_t res = share_precheck(sig_status[idx], present == nullptr || present[idx], i < n_keys, true);
  bool v = false;
  if (res == HBX_SHARE_VALID) {
    g1a ng;  // -[m] g1 against H' = [m] H
    ng.x = fq_from_const(G1_MGEN_X);
    ng.y = fq_neg(fq_from_const(G1_MGEN_Y));
    ng.inf = false;
    // check_mixed_d with sigma's membership in G2 from the loop's final T (decode skipped it)
    const g1a PA = pk[i];
    const g2a QB = sig[idx];
    const bool skipA = PA.inf || H[inst].inf, skipB = QB.inf;
    g2jd T;
    const fq12d f = miller_loop_mixed_d(lines + (size_t)inst * MILLER_LINES, fqd_from_fq(PA.x), fqd_from_fq(PA.y), !skipA,
                                        fq2d_from_fq2(QB.x), fq2d_from_fq2(QB.y), fqd_from_fq(ng.x), fqd_from_fq(ng.y),
                                        !skipB, &T);
    if (!skipB && !g2_torsion_free_from_T(T, QB)) {
      res = HBX_SHARE_UNDECODABLE;
    } else {
      v = (skipA && skipB) || fq12d_is_one(final_exponentiation_d(f, (lds_u32*)(gslots + threadIdx.x)));
    }
  }
  valid[idx] = res == HBX_SHARE_VALID ? (v ? HBX_SHARE_VALID : HBX_SHARE_INVALID) : res;
}

// PublicKey::verify(sig, msg) for independent (key, message, signature) items -- Dynamic
// HoneyBadger's signed votes (src/dynamic_honey_badger/votes.rs:151-156) and key-generation
// messages (dynamic_honey_badger.rs:395-410), SURVEY.md §8(f) row 4: e(pk, H_i) e(-g1, sig) == 1
// with H_i = hash_g2(msg_i) prepared by k_hash_nonces + k_prepare_lines.  One lane per item (the
// lines differ per lane, so the mixed loop's plain loads).  The key is decoded here as pairing's
// into_affine does (curve + G1 membership); an identity key or signature reduces the check to
// "both are the identity" (e(O, H) = 1, and e(pk, H) = 1 only for pk = O since H != O).
__global__ void __launch_bounds__(64) k_verify_sigs(const uint8_t* __restrict__ pk48, const line_pre_d* __restrict__ lines,
                                                    const g2a* __restrict__ H, const g2a* __restrict__ sig,
                                                    const int32_t* __restrict__ sig_st, uint32_t count,
                                                    uint8_t* __restrict__ status) {
  __shared__ uint32_t gslots[LDS_FQ12D_DWORDS * LDS_FQ12_STRIDE];  // final-exp base, one slot per lane
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  g1a pk;
  int32_t st = g1_decompress_d(pk48 + (size_t)i * 48, pk);
  if (st == HBX_PT_OK && !g1_is_torsion_free_d(pk)) st = HBX_PT_NOT_IN_SUBGROUP;
  const bool pk_ok = st == HBX_PT_OK || st == HBX_PT_INFINITY;
  const bool sig_ok = sig_st[i] == HBX_PT_OK || sig_st[i] == HBX_PT_INFINITY;
  if (!pk_ok || !sig_ok) {
    status[i] = HBX_SHARE_UNDECODABLE;
    return;
  }
  const g2a s = sig[i];
  bool v;
  if (pk.inf || s.inf) {
    v = pk.inf && s.inf;
  } else {
    g1a ng;
    ng.x = fq_from_const(G1_GEN_X);
    ng.y = fq_neg(fq_from_const(G1_GEN_Y));
    ng.inf = false;
    v = check_mixed_d(lines + (size_t)i * MILLER_LINES, pk, H[i].inf, s, ng, (lds_u32*)(gslots + threadIdx.x));
  }
  status[i] = v ? HBX_SHARE_VALID : HBX_SHARE_INVALID;
}

// lambda (canonical Fr, 8 LE limbs) in base X = |x| = 0xd201000000010000: lambda = d0 + d1 X +
// d2 X^2 + d3 X^3 (lambda < r < X^4), by binary long division (the remainder needs 65 bits
// between steps: its top bit is carried in `top`).
__device__ void fr_base_x_digits(const uint32_t* lam, uint64_t* d) {
  uint32_t v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = lam[i];
  for (int q = 0; q < 4; q++) {
    uint64_t rem = 0;
    for (int bit = 255; bit >= 0; bit--) {
      const uint32_t w = (uint32_t)bit >> 5, sh = (uint32_t)bit & 31;
      const uint64_t top = rem >> 63;
      rem = (rem << 1) | ((v[w] >> sh) & 1u);
      const bool ge = top != 0 || rem >= BLS_X;
      if (ge) rem -= BLS_X;
      v[w] = (v[w] & ~(1u << sh)) | ((ge ? 1u : 0u) << sh);  // quotient bit replaces the dividend bit
    }
    d[q] = rem;
  }
}

// g2j sum over the lanes of a block (tree: lane pairs by shuffles inside each wave, then the
// per-wave partial sums through LDS).  Every lane must call it; the result is valid in thread 0.
__device__ __forceinline__ fq fq_shfl_xor(const fq& a, int m) {
  fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = (uint32_t)__shfl_xor((int)a.l[i], m);
  return r;
}
__device__ __forceinline__ fqd fqd_shfl_xor(const fqd& a, int m) {
  fqd r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = __shfl_xor(a.d[i], m);
  return r;
}
__device__ __forceinline__ g2jd g2jd_shfl_xor(const g2jd& a, int m) {
  return g2jd{fq2d{fqd_shfl_xor(a.x.c0, m), fqd_shfl_xor(a.x.c1, m)}, fq2d{fqd_shfl_xor(a.y.c0, m), fqd_shfl_xor(a.y.c1, m)},
              fq2d{fqd_shfl_xor(a.z.c0, m), fqd_shfl_xor(a.z.c1, m)}};
}
__device__ __forceinline__ g2j g2j_shfl_xor(const g2j& a, int m) {
  return g2j{fq2{fq_shfl_xor(a.x.c0, m), fq_shfl_xor(a.x.c1, m)}, fq2{fq_shfl_xor(a.y.c0, m), fq_shfl_xor(a.y.c1, m)},
             fq2{fq_shfl_xor(a.z.c0, m), fq_shfl_xor(a.z.c1, m)}};
}

// B3: PublicKeySet::combine_signatures over the first t valid shares in node-index order
// (common_coin.rs:190; received_shares is a BTreeMap): sig = sum lambda_k S_k, Lagrange at 0 in
// G2.  Each S_k is in G2 (the decode checks membership), where psi acts as [x] = [-X]; with
// lambda_k = d0 + d1 X + d2 X^2 + d3 X^3 (|d_i| < X < 2^64),
//     lambda_k S_k = d0 S_k - d1 psi(S_k) + d2 psi^2(S_k) - d3 psi^3(S_k),
// four independent 64-bit scalar multiplications instead of one 255-bit multiplication: a quarter
// of the doubling chain; 4-bit fixed windows (g2d.hpp g2d_mul_u64_w4), so the tasks' different
// digits do not serialise the additions; the point arithmetic in the digit tower.
//
// B3 master check (PublicKey::verify(sig, nonce), common_coin.rs:196) in the same block, on its
// last wave: every S_k was verified, e(pk_k, H) = e(g1, S_k), so by bilinearity
//     e(g1, sig) = prod e(g1, S_k)^lambda_k = e(sum lambda_k pk_k, H),
// and e(master_pk, H) = e(g1, sig)  <=>  sum lambda_k pk_k = master_pk  (H != O, prime order):
// the same bit as the pairing check, from a G1 Lagrange sum over the same index set (GLV halves
// on two lanes, 4-bit windows, like k_combine) -- concurrent with the G2 sum instead of a pairing
// after it.  master_ok = 0 where the combine fails.  One block per instance.
// status: 0 or -3 (NotEnoughShares).
#endif
constexpr int SIGCOMB_THREADS = 256;
#if HBX_IN_TU(5)
__device__ __forceinline__ g1j g1j_shfl_xor(const g1j& a, int m) {
  return g1j{fq_shfl_xor(a.x, m), fq_shfl_xor(a.y, m), fq_shfl_xor(a.z, m)};
}
__global__ void __launch_bounds__(SIGCOMB_THREADS) k_combine_sigs(const uint8_t* __restrict__ valid,
                                                                  const g2a* __restrict__ sig, uint32_t n, uint32_t t,
                                                                  const g1a* __restrict__ pk,
                                                                  const g1a* __restrict__ pk64,
                                                                  const g1a* __restrict__ master_pk,
                                                                  g2a* __restrict__ out, int32_t* __restrict__ status,
                                                                  uint8_t* __restrict__ master_ok,
                                                                  const g1a* __restrict__ g1tab) {
  // One block per instance: waves 0..2 the G2 combine (four psi-digit lanes per share), wave 3 the
  // G1 master identity (64 fixed-base window lanes).  At t = 43 that is 172 G2 tasks on 192 lanes
  // in ONE round of blocks, one wave per SIMD.  (Lane pairs splitting every Fq2 product, g2d.hpp
  // style, on 448 threads: 5.13 ms against 4.07 -- at two waves per SIMD the 256-VGPR budget
  // spilled and the waves waited 57 % of their cycles.)
  constexpr int G2_THREADS = SIGCOMB_THREADS - 64;
  __shared__ uint16_t idx[COMBINE_MAX_T];
  __shared__ int s_count;
  __shared__ g2j red2[G2_THREADS / 64];
  __shared__ fr lam_s[COMBINE_LDS_T];  // lambda_k, once per share (t <= COMBINE_LDS_T)
  const uint32_t inst = blockIdx.x;
  const int tid = threadIdx.x;
  const bool g1_part = tid >= G2_THREADS;  // the last wave
  if (tid == 0) {
    int c = 0;
    for (uint32_t i = 0; i < n && c < (int)t; i++)
      if (valid[(size_t)inst * n + i] == HBX_SHARE_VALID) idx[c++] = (uint16_t)i;
    s_count = c;
  }
  __syncthreads();
  if (s_count < (int)t) {
    if (tid == 0) {
      master_ok[inst] = 0;
      status[inst] = -3;
      out[inst].inf = true;
    }
    return;
  }
  // lambda_k once per share, shared by its four G2 digit lanes and its four G1 tasks
  const bool lds_lam = t <= (uint32_t)COMBINE_LDS_T;
  if (lds_lam) {
    for (int k = tid; k < (int)t; k += SIGCOMB_THREADS) lam_s[k] = lagrange_at_zero(idx, (int)t, k);
    __syncthreads();
  }
  g1j acc1 = g1_identity();
  if (g1_part && g1tab) {
    // fixed-base tables (k_g1_tables): lane w sums window w of every term,
    // sum_k [nibble_w(lambda_k) 16^w] pk_k, one mixed addition per nonzero nibble; the tree below
    // adds the 64 window sums
    const int w = tid - G2_THREADS;
#pragma unroll 1
    for (int k = 0; k < (int)t; k++) {
      const fr lam = lds_lam ? lam_s[k] : lagrange_at_zero(idx, (int)t, k);
      const uint32_t nib = (lam.l[w >> 3] >> ((w & 7) * 4)) & 15u;
      if (nib) acc1 = g1_add_mixed_i(acc1, g1tab[((size_t)idx[k] * G1TAB_W + w) * G1TAB_D + nib - 1]);
    }
#pragma unroll 1
    for (int m = 1; m < 64; m <<= 1) acc1 = g1_add(acc1, g1j_shfl_xor(acc1, m));
  } else if (g1_part) {
    // four 64-bit tasks per share: GLV half h of lambda_k = lo + 2^64 hi, [lo] P_h + [hi] [2^64] P_h
    // with P_0 = pk_k, P_1 = phi(pk_k) (4t tasks of 60 doublings on the wave's 64 lanes instead of
    // 2t of 124: the master identity no longer outlasts the G2 sum)
    for (int q = tid - G2_THREADS; q < 4 * (int)t; q += 64) {
      const int k = q >> 2, h = (q >> 1) & 1, part = q & 1;
      const fr lam = lds_lam ? lam_s[k] : lagrange_at_zero(idx, (int)t, k);
      uint32_t kk[2][4];
      g1_glv_split(lam.l, kk[0], kk[1]);
      const uint32_t* kh = kk[h];
      const uint64_t piece = part ? ((uint64_t)kh[3] << 32 | kh[2]) : ((uint64_t)kh[1] << 32 | kh[0]);
      g1a pp = part ? pk64[idx[k]] : pk[idx[k]];
      if (h) pp.x = fq_mul(pp.x, fq_from_const(G1_BETA));
      if (piece != 0) acc1 = g1_add(acc1, g1_mul_u64_w4(pp, piece));
    }
#pragma unroll 1
    for (int m = 1; m < 64; m <<= 1) acc1 = g1_add(acc1, g1j_shfl_xor(acc1, m));
  } else {
    // the G2 half in the digit tower (g2d.hpp): the 64-bit multiplications and the lane tree
    g2jd a2 = g2d_identity();
    for (int q = tid; q < 4 * (int)t; q += G2_THREADS) {
      const int k = q >> 2, i = q & 3;
      const fr lam = lds_lam ? lam_s[k] : lagrange_at_zero(idx, (int)t, k);
      uint64_t d[4];
      fr_base_x_digits(lam.l, d);
      const g2a S = sig[(size_t)inst * n + idx[k]];
      if (d[i] == 0 || S.inf) continue;
      g2j P = g2_from_affine(S);
      for (int e = 0; e < i; e++) P = g2_psi(P);  // affine in, affine out (Z = 1)
      bool rinf;
      const g2jd R = g2d_mul_u64_w4(fq2d_from_fq2(P.x), fq2d_from_fq2(i & 1 ? fq2_neg(P.y) : P.y), d[i], rinf);
      if (!rinf) a2 = g2d_add(a2, R);
    }
#pragma unroll 1
    for (int m = 1; m < 64; m <<= 1) a2 = g2d_add(a2, g2jd_shfl_xor(a2, m));
    if ((tid & 63) == 0) red2[tid >> 6] = g2jd_to_g2j(a2);
  }
  __syncthreads();
  if (tid == 0) {
    g2j sum = red2[0];
    for (int w = 1; w < G2_THREADS / 64; w++) sum = g2_add(sum, red2[w]);
    out[inst] = g2_to_affine(sum);
    status[inst] = 0;
  } else if (tid == G2_THREADS) {
    // the G1 Lagrange sum == master_pk (affine, not the identity): X = x Z^2, Y = y Z^3
    const g1a M = master_pk[0];
    bool eq = !g1j_is_identity(acc1) && !M.inf;
    if (eq) {
      const fq zz = fq_sqr(acc1.z);
      eq = fq_eq(acc1.x, fq_mul(M.x, zz)) && fq_eq(acc1.y, fq_mul(M.y, fq_mul(zz, acc1.z)));
    }
    master_ok[inst] = eq ? 1 : 0;
  }
}

// B4 Signature::parity (common_coin.rs:173) and the compressed signature, one lane per instance.
__global__ void __launch_bounds__(64) k_sig_parity(const g2a* __restrict__ sig, const int32_t* __restrict__ status,
                                                   uint32_t count, uint8_t* __restrict__ parity,
                                                   uint8_t* __restrict__ sig96) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= count) return;
  if (status[j] != 0) {
    parity[j] = 0;
    for (int q = 0; q < 96; q++) sig96[(size_t)j * 96 + q] = 0;
    return;
  }
  const g2a s = sig[j];
  uint8_t u[192];
  g2_uncompressed(s, u);
  uint8_t x = 0;
  for (int q = 0; q < 192; q++) x ^= u[q];
  parity[j] = (uint8_t)(__builtin_popcount(x) & 1);
  g2_compress(s, sig96 + (size_t)j * 96);
}

// compressed encodings of pts[j * stride], j < count
__global__ void __launch_bounds__(64) k_compress_g2(const g2a* __restrict__ pts, uint32_t count, uint32_t stride,
                                                    uint8_t* __restrict__ out96) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < count) g2_compress(pts[(size_t)j * stride], out96 + (size_t)j * 96);
}

// SecretKeyShare::sign (common_coin.rs:142): sig[inst][i] = sk_i * H_inst, compressed.
__global__ void __launch_bounds__(64) k_sign(const uint8_t* __restrict__ sk32, uint32_t n, const g2a* __restrict__ H,
                                             uint8_t* __restrict__ out96) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t inst = blockIdx.y;
  if (i >= n) return;
  uint32_t k[8];
  fr_from_be32(sk32 + (size_t)i * 32, k);
  g2_compress(g2_to_affine(g2_mul_bits(g2_from_affine(H[inst]), k, 256)), out96 + ((size_t)inst * n + i) * 96);
}

#endif
}  // namespace hbx
