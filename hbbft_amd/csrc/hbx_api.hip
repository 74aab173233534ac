// C-ABI implementation (include/hbx.h): context, device buffers, kernel launches.
// Host code only orchestrates -- every verification, combine and hash runs in the HIP kernels of
// hbx_kernels.hip.  There is no CPU fallback: without a usable HIP device every call fails with
// HBX_E_DEVICE.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/hbx.h"
#include "hbx_kernels.hip"
#include "broadcast.hpp"
#if defined(HBX_TU) && HBX_TU == 0
#include "_kdecl.hpp"  // the kernels live in translation units 1..6 (tools/build.py)
#endif

#if !defined(HBX_TU) || HBX_TU == 0
using namespace hbx;

namespace {

// one wave per SIMD: a one-lane-per-check launch with fewer waves leaves SIMDs idle, and the
// three-lane kernel finishes it sooner (MI355X: 256 CUs x 4 SIMDs)
constexpr int VERIFY_FILL_WAVES = 1024;

struct dbuf {
  void* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t bytes) {
    if (bytes <= cap && p) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (bytes == 0) bytes = 16;
    if (hipMalloc(&p, bytes) != hipSuccess) return false;
    cap = bytes;
    return true;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

}  // namespace

struct hbx_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool coin_h_ready = false;  // coin_H (the true hash_g2 of the prepared nonces) computed
  hipEvent_t coin_ready_ev = nullptr;  // end of hbx_prepare_nonces' work: later coin calls on any stream wait on it
  std::string err = "ok";
  int digest = DIGEST_SHA256;         // hbx_set_digest: threshold_crypto's DIGEST
  int merkle = 0;                     // hbx_set_merkle_digest: HBX_MERKLE_*
  int verify_lanes = 0;               // hbx_set_verify_lanes: 0 auto, 1, 2, 3 or 6 lanes per share check
  int combine_lanes = 0;              // hbx_set_combine_lanes: 0 auto, 1 or 4 lanes per Lagrange term
  int coin_lanes_used = 0;            // lanes per check of the last signature-share launch
  int lanes_used = 0;                 // lanes per check of the last share-check launch
  // era state
  uint32_t n_keys = 0;
  dbuf comb_partial, comb_done;  // k_combine_q: per-block partial sums, per-proposer block counters
  dbuf pk, pk_m, pk64, pk_status, pk_comp;  // pk_m = [3(x^2-1)] pk, pk64 = [2^64] pk (k_scale_keys)
  dbuf g1tab;  // fixed-base tables of the key shares, [n][64][15] affine (k_g1_tables; coin master identity)
  // epoch state
  uint32_t p_ct = 0;
  dbuf U, G2pts, Hj, lines, lines_d, scratch, ct_ok, ct_valid, dec_st;
  // own-share mode (hbx_set_own_share): this node's index and secret share (8 LE limbs), and its
  // own decryption shares of the prepared ciphertexts
  uint32_t own_me = UINT32_MAX;
  dbuf own_sk, own_S, own_part;
  bool own_ready = false;  // own_S computed by the last prepare
  bool ct_known = false;  // ct_valid computed (else deferred into the next share verification)
  const uint8_t* d_v_blob = nullptr;  // device V blob used by the combine (caller-owned for _d)
  const uint64_t* d_v_off = nullptr;
  uint64_t max_v_len = 0;
  dbuf v_blob_own, v_off_own, u_comp_own, w_comp_own;
  // verification state: n_shares / verified_p of the last verify after the latest prepare
  // (0 = none: a prepare invalidates S / valid for the combine)
  uint32_t n_shares = 0, verified_p = 0;
  dbuf S, S_status, fallback, valid, shares_own, present_own, gslot;
  dbuf fe1slot;  // one-lane checks: the final exponentiation's global slots F, T, G (fe1d.hpp)
  uint32_t force_fallback = 0;  // hbx_debug_force_fallback (tests only)
  // u32 counters of the checks the fallback path decided: one for the one-lane decryption-share
  // checks, one for the two-lane coin checks (launches of the two kinds on different streams must
  // not mix their counts); fb_last names the counter of the last share-check launch of either kind,
  // or none when that launch used a lane count without a fallback path
  dbuf fb_lanes, fb_coin;
  dbuf* fb_last = nullptr;
  dbuf hs[6];                   // staging of the host-pointer broadcast calls
  // combine state
  dbuf keys, status, out_own;
  // broadcast state: GF(2^8) tables, encoding matrix of (rs_k, rs_m), reconstruct jobs, Merkle
  dbuf gf_log, gf_exp;
  uint32_t rs_k = 0, rs_m = 0;
  dbuf rs_enc, rs_enc_job, rs_enc_coef, rs_enc_ptab, rs_ptab_d, rs_ptab_p, rs_jobs_d, rs_jobs_p, rs_coef_d, rs_coef_p, leaf_hash, leaf_slots, val_digest, roots;
  // common coin state: nonces' hash_g2 points and lines, signature shares, combined signatures
  uint32_t coin_I = 0, coin_n = 0;
  dbuf coin_blob, coin_off, coin_H, coin_Hp, coin_lines, coin_scratch, coin_sk, coin_sig96, coin_sig, coin_sig_st, coin_present,
      coin_valid, coin_comb, coin_comb_st, coin_mpk_comp, coin_mpk, coin_mpk_st, coin_ok, coin_par, coin_out96;
  // PublicKey::verify batches (hbx_verify_sigs)
  dbuf vs_pk, vs_blob, vs_off, vs_H, vs_lines, vs_lines_d, vs_scratch, vs_sig96, vs_sig, vs_sig_st, vs_status;
  dbuf coin_lines_d;  // the nonces' lines in the coin check's digit form
  bool coin_lines_ready = false;  // coin_lines_d computed for the prepared nonces (one-lane checks only)
  uint8_t coin_mpk48[48] = {0};   // the master key coin_mpk was decoded from
  bool coin_mpk_known = false;
  dbuf coin_use;      // hbx_combine_signatures_d: the verified shares masked by the caller's subset
  // SyncKeyGen commitment checks (hbx_bivar_rows / hbx_bivar_check_acks)
  dbuf bv_commit48, bv_C, bv_cst, bv_rows, bv_rows48, bv_pst, bv_ackp, bv_acky, bv_vals, bv_out;
  // opt-in kernel timing: event pairs per timed kernel (hbx_set_timing / hbx_kernel_time)
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> tev[HBX_K_COUNT];
  std::vector<hipEvent_t> ev_pool;
  // ordering of this context's work across streams: every entry point waits on `ev_last` before
  // enqueuing on its stream and records it after (stream_scope), so a host call on `stream`
  // after a _d call on the caller's stream (or on NULL, which does not order against the
  // non-blocking `stream`) sees that call's results; readouts wait on this event only, not on
  // the whole device (other contexts' epochs in flight keep running)
  hipEvent_t ev_last = nullptr;
  bool ev_recorded = false;
};

static hipEvent_t ev_get(hbx_ctx* c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}
static void timing_reset(hbx_ctx* c) {
  for (auto& v : c->tev) {
    for (auto& pr : v) {
      c->ev_pool.push_back(pr.first);
      c->ev_pool.push_back(pr.second);
    }
    v.clear();
  }
}
// Records a start event before and a stop event after one kernel launch on stream s.
struct timed {
  hbx_ctx* c;
  int id;
  hipStream_t s;
  hipEvent_t e0 = nullptr;
  timed(hbx_ctx* c_, int id_, hipStream_t s_) : c(c_), id(id_), s(s_) {
    if (c->timing && (e0 = ev_get(c))) (void)hipEventRecord(e0, s);
  }
  ~timed() {
    if (!e0) return;
    hipEvent_t e1 = ev_get(c);
    if (!e1) return;
    (void)hipEventRecord(e1, s);
    c->tev[id].emplace_back(e0, e1);
  }
};

static int fail(hbx_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define HIPCHK(ctx, expr)                                                                      \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess) return fail(ctx, HBX_E_DEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// _d API: the caller's stream; NULL is the HIP null stream (a framework's default stream), so the
// enqueued work is ordered with the caller's own work on it.  The stream first waits for this
// context's previous work on any stream (ev_last).
static hipStream_t pick(hbx_ctx* c, void* s) {
  hipStream_t st = static_cast<hipStream_t>(s);
  if (c && c->ev_recorded) (void)hipStreamWaitEvent(st, c->ev_last, 0);
  return st;
}
// Records ev_last on the entry point's stream when it returns (on every return path).
struct stream_scope {
  hbx_ctx* c;
  hipStream_t s;
  ~stream_scope() {
    if (c && c->ev_last && hipEventRecord(c->ev_last, s) == hipSuccess) c->ev_recorded = true;
  }
};
// Host-side wait for everything this context has enqueued (its own stream and callers' streams).
static hipError_t quiesce(hbx_ctx* c) {
  if (c->ev_recorded) {
    const hipError_t e = hipEventSynchronize(c->ev_last);
    if (e != hipSuccess) return e;
  }
  return hipStreamSynchronize(c->stream);
}

// bit k = (bytes[k] == 1): status bytes (HBX_SHARE_VALID, HBX_CT_VALID) and 0/1 flags alike
static void pack_bits(const uint8_t* bytes, size_t n, uint8_t* bits) {
  memset(bits, 0, (n + 7) / 8);
  for (size_t k = 0; k < n; k++)
    if (bytes[k] == 1) bits[k >> 3] |= (uint8_t)(1u << (k & 7));
}

static bool scalars_canonical(const uint8_t* s32, size_t count);

// Pairing checks of jobs [q_first, q_last] of every proposer (q < n: shares, q == n: ciphertext).
static int launch_pair_checks(hbx_ctx* c, hipStream_t s, uint32_t n, uint32_t p, uint32_t q_first, uint32_t q_last,
                              const uint8_t* d_present) {
  if (!c->fallback.ensure((size_t)p * (n + 1)))
    return fail(c, HBX_E_OUT_OF_MEMORY, "out of device memory (fallback flags)");
  HIPCHK(c, hipMemsetAsync(c->fallback.p, 0, (size_t)p * (n + 1), s));
  const uint32_t jobs = q_last - q_first + 1;
  {
    timed t_(c, HBX_K_CT_CHECKS, s);
    hipLaunchKernelGGL(k_verify_wide, dim3((jobs + WG_GROUPS - 1) / WG_GROUPS, p), dim3(WG_THREADS), 0, s,
                       c->S.as<g1a>(), c->S_status.as<int32_t>(), d_present, c->pk_m.as<g1a>(), c->n_keys,
                       c->U.as<g1a>(), c->G2pts.as<g2a>(), c->lines.as<line_block>(), c->ct_ok.as<uint8_t>(), n,
                       q_first, q_last, c->valid.as<uint8_t>(), c->ct_valid.as<uint8_t>(), c->fallback.as<uint8_t>());
  }
  HIPCHK(c, hipGetLastError());
  const size_t all = (size_t)p * (n + 1);
  hipLaunchKernelGGL(k_pair_fallback, dim3((unsigned)((all + 63) / 64)), dim3(64), 0, s, c->fallback.as<uint8_t>(),
                     c->S.as<g1a>(), c->pk_m.as<g1a>(), c->U.as<g1a>(), c->G2pts.as<g2a>(), c->lines.as<line_block>(),
                     n, p, c->valid.as<uint8_t>(), c->ct_valid.as<uint8_t>());
  HIPCHK(c, hipGetLastError());
  return HBX_OK;
}

// ---- broadcast: host-side set-up (ReedSolomon::new; tables and matrices only, no shard data) ----
struct gf_host {
  uint16_t lg[256];
  uint8_t ex[768];
  uint8_t mul(uint8_t a, uint8_t b) const { return (a == 0 || b == 0) ? 0 : ex[lg[a] + lg[b]]; }
  uint8_t inv(uint8_t a) const { return ex[255 - lg[a]]; }
  uint8_t pow(uint8_t a, uint32_t n) const {  // galois_8::exp, 0^0 = 1
    if (n == 0) return 1;
    if (a == 0) return 0;
    return ex[(lg[a] * n) % 255];
  }
};

static const gf_host& gf() {
  static gf_host g = [] {
    gf_host t{};
    uint32_t x = 1;
    for (int i = 0; i < 768; i++) t.ex[i] = 0;
    for (int i = 0; i < 255; i++) {
      t.ex[i] = (uint8_t)x;
      t.ex[i + 255] = (uint8_t)x;
      t.lg[x] = (uint16_t)i;
      x <<= 1;
      if (x & 0x100) x ^= 0x11D;
    }
    t.lg[0] = GF_LOG_ZERO;
    return t;
  }();
  return g;
}

// Byte-permute tables of one coefficient (layout in broadcast.hpp, k_rs_code_perm).
static gf_ptab gf_perm_table(uint8_t c) {
  const gf_host& g = gf();
  uint8_t b[20];
  for (int i = 0; i < 8; i++) {
    b[i] = g.mul(c, (uint8_t)i);
    b[8 + i] = g.mul(c, (uint8_t)(i << 3));
  }
  for (int i = 0; i < 4; i++) b[16 + i] = g.mul(c, (uint8_t)(i << 6));
  gf_ptab t{};
  for (int w = 0; w < 5; w++)
    t.w[w] = (uint32_t)b[4 * w] | ((uint32_t)b[4 * w + 1] << 8) | ((uint32_t)b[4 * w + 2] << 16) |
             ((uint32_t)b[4 * w + 3] << 24);
  return t;
}

// Output rows x dwords per lane of the byte-permute kernel; HBX_RS_TILE (0..7) pins one of the
// compiled variants for tuning, -1 (unset) picks by output count (rs_auto_tile).
static int rs_tile() {
  static const int t = [] {
    const char* e = getenv("HBX_RS_TILE");
    return e ? atoi(e) : -1;
  }();
  return t;
}

// HBX_RS_K3=0 keeps the pair kernel (k_rs_code_perm) where the triple one would run.
static bool rs_k3() {
  static const bool t = [] {
    const char* e = getenv("HBX_RS_K3");
    return !e || atoi(e) != 0;
  }();
  return t;
}

static const int rs_tile_ch[] = {32, 32, 64, 24, 48, 28, 28, 44};

// The tile whose row count wastes the fewest computed rows on `no` outputs per instance (each
// pass over the k input rows yields CH outputs; a short last pass still reads all k rows), ties
// to the larger tile.  r06q_rs_tiles: m = 84 parity rows run 740 GB/s on 32-row tiles (96 rows
// computed) and 810 GB/s on 28-row ones (84).
static int rs_auto_tile(uint32_t k, uint32_t no) {
  static const int cand[] = {2, 4, 7, 0, 5, 3};  // 64, 48, 44, 32, 28, 24 rows, two dwords per lane but 24
  int best = 3, best_rows = 1 << 30;
  for (int t : cand) {
    const int ch = rs_tile_ch[t];
    if (rs_perm_lds_bytes(k, ch) > 65536) continue;
    const int rows = (int)((no + ch - 1) / ch) * ch;
    if (rows < best_rows) best = t, best_rows = rows;
  }
  return best;
}

// One coding pass: the byte-permute kernel when rows are whole dwords, else the LDS log/exp one.
// `no` is the outputs one instance's pass is expected to write: m on encode; on a reconstruct pass
// the f = m / 2 erasures of hbbft's fault bound (the bench's pattern; up to m still runs, in more passes).
static void rs_code(hbx_ctx* c, uint8_t* d_shards, size_t stride, uint32_t L, uint32_t k, uint32_t inst,
                    const rs_job* jobs, const uint16_t* coef, const gf_ptab* ptab, uint32_t job_stride, uint32_t no,
                    hipStream_t s) {
  timed t_(c, HBX_K_RS_CODE, s);
  if (no == 0) no = 1;  // grid.z >= 1; the kernels read the true count from the job
  if (L % 4 == 0 && rs_k3() && rs_tile() < 0) {
    // triple kernel (4.0 VALU ops per coefficient-dword): tile by output count as below
    const uint32_t Ld = L / 4;
    // fewest computed rows, ties to the earlier entry: the 21-row tile runs 88 VGPRs (5 waves per
    // SIMD) against 105 for 28 rows and 130 for 42 (r06t21: encode 0.405 -> 0.387-0.398 ms, the
    // decode with spread erasures 1.33 -> 1.22 ms)
    static const int ch3[] = {21, 14, 12, 28, 42};
    int ch = 0, best_rows = 1 << 30;
    for (int t : ch3) {
      if (rs_perm3_lds_bytes(k, t) > 65536) continue;
      const int rows = (int)((no + t - 1) / t) * t;
      if (rows < best_rows) ch = t, best_rows = rows;
    }
    static const int pin = [] {
      const char* e = getenv("HBX_RS_CH3");  // tuning: 100 * D + CH of a compiled triple tile
      return e ? atoi(e) : 0;
    }();
    int d3 = 2;
    if (pin && rs_perm3_lds_bytes(k, pin % 100) <= 65536) ch = pin % 100, d3 = pin / 100;
    if (ch) {
      switch (d3 * 100 + ch) {
#define HBX_RS_TILE3(c3, d)                                                                                         \
  hipLaunchKernelGGL((k_rs_code_perm3<c3, d>), dim3((Ld + 256 * d - 1) / (256 * d), inst, (no + c3 - 1) / c3), dim3(256), \
                     rs_perm3_lds_bytes(k, c3), s, d_shards, stride, L, k, jobs, ptab, job_stride);                  \
  break;
        case 242: HBX_RS_TILE3(42, 2)
        case 228: HBX_RS_TILE3(28, 2)
        case 214: HBX_RS_TILE3(14, 2)
        case 212: HBX_RS_TILE3(12, 2)
        default: HBX_RS_TILE3(21, 2)
#undef HBX_RS_TILE3
      }
      return;
    }
  }
  if (L % 4 == 0) {
    const uint32_t Ld = L / 4;
    int tile = rs_tile();
    if (tile < 0 || tile > 7) tile = rs_auto_tile(k, no);
    if (rs_perm_lds_bytes(k, rs_tile_ch[tile]) > 65536) tile = 3;  // 24 x 128 x 20 B fits any k
    switch (tile) {
#define HBX_RS_TILE(ch, d)                                                                                        \
  hipLaunchKernelGGL((k_rs_code_perm<ch, d>), dim3((Ld + 256 * d - 1) / (256 * d), inst, (no + ch - 1) / ch), dim3(256), \
                     rs_perm_lds_bytes(k, ch), s, d_shards, stride, L, k, jobs, ptab, job_stride);                 \
  break;
      case 1: HBX_RS_TILE(32, 4)
      case 2: HBX_RS_TILE(64, 2)
      case 3: HBX_RS_TILE(24, 4)
      case 4: HBX_RS_TILE(48, 2)
      case 5: HBX_RS_TILE(28, 2)
      case 6: HBX_RS_TILE(28, 4)
      case 7: HBX_RS_TILE(44, 2)
      default: HBX_RS_TILE(32, 2)
#undef HBX_RS_TILE
    }
  } else {
    hipLaunchKernelGGL(k_rs_code, dim3((L + 1023) / 1024, inst), dim3(256), 0, s, d_shards, stride, L, k, jobs, coef,
                       job_stride, c->gf_log.as<uint16_t>(), c->gf_exp.as<uint8_t>());
  }
}

// Encoding matrix V * inverse(V[0..k]) with V[r][c] = r^c ((k + m) x k, reed-solomon-erasure 3.1.0).
static bool rs_matrix(uint32_t k, uint32_t m, std::vector<uint8_t>& out) {
  const gf_host& g = gf();
  const uint32_t n = k + m;
  std::vector<uint8_t> V(n * k), A(k * 2 * k);
  for (uint32_t r = 0; r < n; r++)
    for (uint32_t c = 0; c < k; c++) V[r * k + c] = g.pow((uint8_t)r, c);
  for (uint32_t r = 0; r < k; r++)
    for (uint32_t c = 0; c < 2 * k; c++) A[r * 2 * k + c] = c < k ? V[r * k + c] : (c - k == r ? 1 : 0);
  for (uint32_t r = 0; r < k; r++) {
    if (A[r * 2 * k + r] == 0) {
      uint32_t b = r + 1;
      while (b < k && A[b * 2 * k + r] == 0) b++;
      if (b == k) return false;
      for (uint32_t c = 0; c < 2 * k; c++) std::swap(A[r * 2 * k + c], A[b * 2 * k + c]);
    }
    const uint8_t inv = g.inv(A[r * 2 * k + r]);
    for (uint32_t c = 0; c < 2 * k; c++) A[r * 2 * k + c] = g.mul(A[r * 2 * k + c], inv);
    for (uint32_t i = 0; i < k; i++) {
      const uint8_t f = A[i * 2 * k + r];
      if (i == r || !f) continue;
      for (uint32_t c = 0; c < 2 * k; c++) A[i * 2 * k + c] ^= g.mul(f, A[r * 2 * k + c]);
    }
  }
  out.assign(n * k, 0);
  for (uint32_t r = 0; r < n; r++)
    for (uint32_t c = 0; c < k; c++) {
      uint8_t acc = 0;
      for (uint32_t q = 0; q < k; q++) acc ^= g.mul(V[r * k + q], A[q * 2 * k + k + c]);
      out[r * k + c] = acc;
    }
  return true;
}

static int rs_setup(hbx_ctx* c, uint32_t k, uint32_t m, hipStream_t s) {
  if (k == 0 || k > (uint32_t)RS_MAX_K || k + m > (uint32_t)RS_MAX_N)
    return fail(c, HBX_E_INVALID_ARG, "rs: need 1 <= k <= %d and k + m <= %d (k=%u m=%u)", RS_MAX_K, RS_MAX_N, k, m);
  if (!c->gf_log.p) {
    if (!c->gf_log.ensure(512) || !c->gf_exp.ensure(768)) return fail(c, HBX_E_OUT_OF_MEMORY, "rs: tables");
    HIPCHK(c, hipMemcpyAsync(c->gf_log.p, gf().lg, 512, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->gf_exp.p, gf().ex, 768, hipMemcpyHostToDevice, s));
  }
  if (c->rs_k == k && c->rs_m == m) return HBX_OK;
  std::vector<uint8_t> M;
  if (m > 0 && !rs_matrix(k, m, M)) return fail(c, HBX_E_INVALID_ARG, "rs: singular Vandermonde block");
  if (m == 0) M.assign((size_t)k * k, 0);
  rs_job job{};
  job.n_out = (int32_t)m;
  for (uint32_t q = 0; q < k; q++) job.in_idx[q] = (int32_t)q;
  for (uint32_t o = 0; o < m; o++) job.out_idx[o] = (int32_t)(k + o);
  std::vector<uint16_t> coef((size_t)RS_MAX_N * k, GF_COEF_ZERO);
  for (uint32_t o = 0; o < m; o++)
    for (uint32_t q = 0; q < k; q++) {
      const uint8_t v = M[(size_t)(k + o) * k + q];
      coef[(size_t)o * k + q] = v ? gf().lg[v] : GF_COEF_ZERO;
    }
  std::vector<gf_ptab> ptab((size_t)m * k);
  for (uint32_t o = 0; o < m; o++)
    for (uint32_t q = 0; q < k; q++) ptab[(size_t)o * k + q] = gf_perm_table(M[(size_t)(k + o) * k + q]);
  if (!c->rs_enc.ensure(M.size()) || !c->rs_enc_job.ensure(sizeof(rs_job)) || !c->rs_enc_coef.ensure(coef.size() * 2) ||
      !c->rs_enc_ptab.ensure(ptab.size() * sizeof(gf_ptab) + sizeof(gf_ptab)))
    return fail(c, HBX_E_OUT_OF_MEMORY, "rs: matrix");
  HIPCHK(c, hipMemcpyAsync(c->rs_enc_ptab.p, ptab.data(), ptab.size() * sizeof(gf_ptab), hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(c->rs_enc.p, M.data(), M.size(), hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(c->rs_enc_job.p, &job, sizeof(rs_job), hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(c->rs_enc_coef.p, coef.data(), coef.size() * 2, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipStreamSynchronize(s));  // host staging buffers die at return
  c->rs_k = k;
  c->rs_m = m;
  return HBX_OK;
}

static int rs_reconstruct(hbx_ctx* c, uint8_t* d_shards, const uint8_t* d_present, uint32_t inst, uint32_t k,
                          uint32_t m, uint32_t L, int32_t* d_status, hipStream_t s) {
  const size_t stride = (size_t)(k + m) * L;
  if (!c->rs_jobs_d.ensure((size_t)inst * sizeof(rs_job)) || !c->rs_jobs_p.ensure((size_t)inst * sizeof(rs_job)) ||
      !c->rs_coef_d.ensure((size_t)inst * RS_MAX_N * k * 2) || !c->rs_coef_p.ensure((size_t)inst * RS_MAX_N * k * 2))
    return fail(c, HBX_E_OUT_OF_MEMORY, "rs_reconstruct: out of device memory");
  hipLaunchKernelGGL(k_rs_setup_reconstruct, dim3(inst), dim3(256), 0, s, d_present, k, m, c->rs_enc.as<uint8_t>(),
                     c->gf_log.as<uint16_t>(), c->gf_exp.as<uint8_t>(), c->rs_jobs_d.as<rs_job>(),
                     c->rs_coef_d.as<uint16_t>(), c->rs_jobs_p.as<rs_job>(), c->rs_coef_p.as<uint16_t>(), d_status);
  HIPCHK(c, hipGetLastError());
  if (L % 4 == 0) {
    if (!c->rs_ptab_d.ensure((size_t)inst * RS_MAX_N * k * sizeof(gf_ptab)) ||
        !c->rs_ptab_p.ensure((size_t)inst * RS_MAX_N * k * sizeof(gf_ptab)))
      return fail(c, HBX_E_OUT_OF_MEMORY, "rs_reconstruct: out of device memory");
    const dim3 tg((RS_MAX_N * k + 255) / 256, inst);
    hipLaunchKernelGGL(k_rs_perm_tables, tg, dim3(256), 0, s, c->rs_jobs_d.as<rs_job>(), c->rs_coef_d.as<uint16_t>(), k,
                       c->gf_log.as<uint16_t>(), c->gf_exp.as<uint8_t>(), c->rs_ptab_d.as<gf_ptab>());
    hipLaunchKernelGGL(k_rs_perm_tables, tg, dim3(256), 0, s, c->rs_jobs_p.as<rs_job>(), c->rs_coef_p.as<uint16_t>(), k,
                       c->gf_log.as<uint16_t>(), c->gf_exp.as<uint8_t>(), c->rs_ptab_p.as<gf_ptab>());
    HIPCHK(c, hipGetLastError());
  }
  rs_code(c, d_shards, stride, L, k, inst, c->rs_jobs_d.as<rs_job>(), c->rs_coef_d.as<uint16_t>(),
          c->rs_ptab_d.as<gf_ptab>(), 1u, (m + 1) / 2, s);
  HIPCHK(c, hipGetLastError());
  rs_code(c, d_shards, stride, L, k, inst, c->rs_jobs_p.as<rs_job>(), c->rs_coef_p.as<uint16_t>(),
          c->rs_ptab_p.as<gf_ptab>(), 1u, (m + 1) / 2, s);
  HIPCHK(c, hipGetLastError());
  return HBX_OK;
}

static int merkle_roots(hbx_ctx* c, const uint8_t* d_shards, uint32_t inst, uint32_t n, uint32_t L, uint8_t* d_roots,
                        hipStream_t s, uint8_t* d_nodes = nullptr) {
  if (n == 0 || n > (uint32_t)RS_MAX_N) return fail(c, HBX_E_INVALID_ARG, "merkle: need 1 <= n <= 256");
  if (!c->leaf_hash.ensure((size_t)inst * n * 32)) return fail(c, HBX_E_OUT_OF_MEMORY, "merkle: leaf hashes");
  {
    timed t_(c, HBX_K_MERKLE_LEAVES, s);
    if (c->merkle == HBX_MERKLE_SHA256)
      hipLaunchKernelGGL(k_merkle_leaves_sha256, dim3((n + 63) / 64, inst), dim3(128), 0, s, d_shards, (size_t)n * L,
                         n, L, c->leaf_hash.as<uint32_t>(), (const uint16_t*)nullptr, 0u, 0u);
    else
      hipLaunchKernelGGL(k_merkle_leaves_sha3, dim3((n + 31) / 32, inst), dim3(64), 0, s, d_shards, (size_t)n * L, n,
                         L, c->leaf_hash.as<uint32_t>(), (const uint16_t*)nullptr, 0u, 0u);
  }
  HIPCHK(c, hipGetLastError());
  hipLaunchKernelGGL(k_merkle_tree, dim3(inst), dim3(128), 0, s, c->leaf_hash.as<uint32_t>(), n, d_roots, d_nodes,
                     c->merkle);
  HIPCHK(c, hipGetLastError());
  return HBX_OK;
}

extern "C" {

const char* hbx_version(void) { return "hbx 0.1.0 gfx950"; }
#ifndef HBX_SOURCE_HASH
#define HBX_SOURCE_HASH "unknown"
#endif
const char* hbx_build_id(void) { return HBX_SOURCE_HASH; }

const char* hbx_last_error(const hbx_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int hbx_ctx_create(int device, hbx_ctx** out) {
  if (!out) return HBX_E_INVALID_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return HBX_E_DEVICE;
  if (device < 0 || device >= count) return HBX_E_INVALID_ARG;
  if (hipSetDevice(device) != hipSuccess) return HBX_E_DEVICE;
  hbx_ctx* c = new hbx_ctx();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return HBX_E_DEVICE;
  }
  if (hipEventCreateWithFlags(&c->ev_last, hipEventDisableTiming) != hipSuccess) {
    (void)hipStreamDestroy(c->stream);
    delete c;
    return HBX_E_DEVICE;
  }
  *out = c;
  return HBX_OK;
}

int hbx_ctx_destroy(hbx_ctx* c) {
  if (!c) return HBX_E_INVALID_ARG;
  (void)hipSetDevice(c->device);
  (void)quiesce(c);
  timing_reset(c);
  for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
  c->ev_pool.clear();
  dbuf* bufs[] = {&c->comb_partial, &c->comb_done, &c->pk,       &c->pk_m,       &c->pk64,       &c->g1tab,      &c->pk_status,  &c->pk_comp,     &c->U,         &c->G2pts, &c->Hj,
                  &c->lines,    &c->scratch,    &c->ct_ok,       &c->ct_valid,  &c->v_blob_own,
                  &c->v_off_own, &c->u_comp_own, &c->w_comp_own, &c->S,         &c->valid,
                  &c->S_status, &c->fallback, &c->gslot,
                  &c->shares_own, &c->present_own, &c->keys,     &c->status,    &c->out_own,
                  &c->gf_log,   &c->gf_exp,     &c->rs_enc,      &c->rs_enc_job, &c->rs_enc_coef, &c->rs_enc_ptab, &c->rs_ptab_d, &c->rs_ptab_p,
                  &c->rs_jobs_d, &c->rs_jobs_p, &c->rs_coef_d,   &c->rs_coef_p, &c->leaf_hash, &c->leaf_slots, &c->val_digest, &c->roots,
                  &c->coin_blob, &c->coin_off,  &c->coin_H, &c->coin_Hp,      &c->coin_lines, &c->coin_scratch, &c->coin_sk,
                  &c->coin_sig96, &c->coin_sig, &c->coin_sig_st, &c->coin_present, &c->coin_valid, &c->coin_comb,
                  &c->coin_comb_st, &c->coin_mpk_comp, &c->coin_mpk, &c->coin_mpk_st, &c->coin_ok, &c->coin_par,
                  &c->coin_out96, &c->dec_st, &c->own_sk, &c->own_S, &c->own_part, &c->lines_d,
                  &c->vs_pk, &c->vs_lines_d, &c->coin_lines_d, &c->vs_blob, &c->vs_off, &c->vs_H, &c->vs_lines, &c->vs_scratch, &c->vs_sig96,
                  &c->vs_sig, &c->vs_sig_st, &c->vs_status, &c->fe1slot, &c->fb_lanes, &c->fb_coin, &c->hs[0], &c->hs[1], &c->hs[2], &c->hs[3], &c->hs[4], &c->hs[5], &c->coin_use, &c->bv_commit48, &c->bv_C, &c->bv_cst, &c->bv_rows,
                  &c->bv_rows48, &c->bv_pst, &c->bv_ackp, &c->bv_acky, &c->bv_vals, &c->bv_out};
  for (dbuf* b : bufs) b->release();
  (void)hipEventDestroy(c->ev_last);
  if (c->coin_ready_ev) (void)hipEventDestroy(c->coin_ready_ev);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return HBX_OK;
}

int hbx_set_digest(hbx_ctx* c, int variant) {
  if (!c || (variant != HBX_DIGEST_SHA256 && variant != HBX_DIGEST_SHA3_256))
    return fail(c, HBX_E_INVALID_ARG, "hbx_set_digest: unknown variant %d", variant);
  c->digest = variant == HBX_DIGEST_SHA3_256 ? DIGEST_SHA3_256 : DIGEST_SHA256;
  c->p_ct = 0;  // hashes prepared under the other digest are void
  c->ct_known = false;
  c->n_shares = 0;
  c->verified_p = 0;
  c->coin_I = 0;
  c->coin_n = 0;
  return HBX_OK;
}

int hbx_set_verify_lanes(hbx_ctx* c, int lanes) {
  if (!c || lanes < 0 || lanes > 7 || lanes == 4 || lanes == 5)
    return fail(c, HBX_E_INVALID_ARG, "hbx_set_verify_lanes: 0 (auto), 1, 2, 3, 6 or 7, not %d", lanes);
  c->verify_lanes = lanes;
  return HBX_OK;
}

int hbx_get_verify_lanes_used(const hbx_ctx* c) { return c ? c->lanes_used : 0; }

int hbx_debug_force_fallback(hbx_ctx* c, uint32_t every) {
  if (!c) return HBX_E_INVALID_ARG;
  c->force_fallback = every;
  return HBX_OK;
}

int64_t hbx_get_fallback_lanes(hbx_ctx* c) {
  if (!c) return HBX_E_INVALID_ARG;
  if (!c->fb_last) return 0;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, quiesce(c));
  uint32_t v = 0;
  HIPCHK(c, hipMemcpy(&v, c->fb_last->p, 4, hipMemcpyDeviceToHost));
  return v;
}

int hbx_set_combine_lanes(hbx_ctx* c, int lanes) {
  if (!c || (lanes != 0 && lanes != 1 && lanes != 4))
    return fail(c, HBX_E_INVALID_ARG, "hbx_set_combine_lanes: 0 (auto), 1 or 4, not %d", lanes);
  c->combine_lanes = lanes;
  return HBX_OK;
}

int hbx_set_merkle_digest(hbx_ctx* c, int variant) {
  if (!c || (variant != HBX_MERKLE_SHA256 && variant != HBX_MERKLE_SHA3))
    return fail(c, HBX_E_INVALID_ARG, "hbx_set_merkle_digest: unknown variant %d", variant);
  c->merkle = variant;
  return HBX_OK;
}

int hbx_set_pk_shares(hbx_ctx* c, const uint8_t* pk_comp, uint32_t n, int32_t* status) {
  if (!c || (!pk_comp && n)) return fail(c, HBX_E_INVALID_ARG, "hbx_set_pk_shares: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  // era change: nothing enqueued earlier (on any stream) may still read the old keys, and every
  // state derived from them is void -- the own share (its pk_me check was against the old keys)
  // and the current epoch's prepared ciphertexts / verified shares
  HIPCHK(c, quiesce(c));
  stream_scope ss_{c, pick(c, c->stream)};
  c->own_me = UINT32_MAX;
  c->own_ready = false;
  c->p_ct = 0;
  c->ct_known = false;
  c->n_shares = 0;
  c->verified_p = 0;
  c->coin_n = 0;
  if (!c->pk.ensure((size_t)n * sizeof(g1a)) || !c->pk_m.ensure((size_t)n * sizeof(g1a)) ||
      !c->pk64.ensure((size_t)n * sizeof(g1a)) || !c->pk_status.ensure((size_t)n * 4) || !c->pk_comp.ensure((size_t)n * 48))
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_set_pk_shares: out of device memory");
  HIPCHK(c, hipMemcpyAsync(c->pk_comp.p, pk_comp, (size_t)n * 48, hipMemcpyHostToDevice, c->stream));
  if (n) {
    hipLaunchKernelGGL(k_decompress_g1, dim3((n + 63) / 64), dim3(64), 0, c->stream, c->pk_comp.as<uint8_t>(),
                       n, c->pk.as<g1a>(), c->pk_status.as<int32_t>());
    HIPCHK(c, hipGetLastError());
    // [3(x^2-1)] pk_i: the decryption-share checks' G1 side against H' = h_eff P (k_prepare_ct)
    hipLaunchKernelGGL(k_scale_keys, dim3((n + 63) / 64), dim3(64), 0, c->stream, c->pk.as<g1a>(), n,
                       c->pk_m.as<g1a>(), c->pk64.as<g1a>());
    HIPCHK(c, hipGetLastError());
    // [d 16^w] pk_i for the coin combine's master identity (k_combine_sigs): era set-up, not per round
    if (!c->g1tab.ensure((size_t)n * G1TAB_W * G1TAB_D * sizeof(g1a)))
      return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_set_pk_shares: out of device memory (key tables)");
    hipLaunchKernelGGL(k_g1_tables, dim3((n * G1TAB_W + 63) / 64), dim3(64), 0, c->stream, c->pk.as<g1a>(), n,
                       c->g1tab.as<g1a>());
    HIPCHK(c, hipGetLastError());
  } else {
    c->g1tab.release();  // no tables of an older key set
  }
  std::vector<int32_t> st(n);
  HIPCHK(c, hipMemcpyAsync(st.data(), c->pk_status.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (status) memcpy(status, st.data(), (size_t)n * 4);
  c->n_keys = n;
  return HBX_OK;
}

int hbx_set_own_share(hbx_ctx* c, uint32_t me, const uint8_t* sk32) {
  if (!c) return HBX_E_INVALID_ARG;
  if (!sk32) {  // clear: back to separate Ciphertext::verify checks
    c->own_me = UINT32_MAX;
    c->own_ready = false;
    return HBX_OK;
  }
  if (c->n_keys == 0 || me >= c->n_keys) return fail(c, HBX_E_NO_KEYS, "hbx_set_own_share: me=%u, n=%u", me, c->n_keys);
  static const uint8_t ZERO[32] = {0};
  if (!scalars_canonical(sk32, 1) || memcmp(sk32, ZERO, 32) == 0)
    return fail(c, HBX_E_INVALID_ARG, "hbx_set_own_share: scalar must be in [1, r)");
  // the secret share must match pk_me: the fused ciphertext check relies on pk_me = sk_me g1
  uint8_t pk48[48], want[48];
  int rc = hbx_public_keys(c, sk32, 1, pk48);
  if (rc) return rc;
  HIPCHK(c, hipMemcpy(want, static_cast<uint8_t*>(c->pk_comp.p) + (size_t)me * 48, 48, hipMemcpyDeviceToHost));
  if (memcmp(pk48, want, 48) != 0) return fail(c, HBX_E_INVALID_ARG, "hbx_set_own_share: sk does not match pk[%u]", me);
  uint32_t limbs[8];
  for (int q = 0; q < 8; q++)
    limbs[q] = ((uint32_t)sk32[31 - 4 * q - 3] << 24) | ((uint32_t)sk32[31 - 4 * q - 2] << 16) |
               ((uint32_t)sk32[31 - 4 * q - 1] << 8) | sk32[31 - 4 * q];
  if (!c->own_sk.ensure(32)) return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_set_own_share: out of device memory");
  // a prepare enqueued earlier on any stream may still read own_sk
  HIPCHK(c, quiesce(c));
  HIPCHK(c, hipMemcpy(c->own_sk.p, limbs, 32, hipMemcpyHostToDevice));
  c->own_me = me;
  c->own_ready = false;
  return HBX_OK;
}

// Ciphertext preparation; with `early_shares` (the fused epoch call) the received shares of the
// epoch are decoded in the same launch, in waves beside the hash chains.
static int prepare_impl(hbx_ctx* c, const uint8_t* d_u_comp, const uint8_t* d_v_blob, const uint64_t* d_v_off,
                        const uint8_t* d_w_comp, uint32_t p, uint64_t max_v_len, uint8_t* d_ct_valid,
                        void* stream, const uint8_t* early_shares, uint32_t early_n) {
  if (!c || p == 0 || !d_u_comp || !d_v_off || !d_w_comp)
    return fail(c, HBX_E_INVALID_ARG, "hbx_prepare_ciphertexts_d: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  stream_scope ss_{c, s};
  if (!c->U.ensure((size_t)p * sizeof(g1a)) || !c->G2pts.ensure((size_t)2 * p * sizeof(g2a)) || !c->Hj.ensure((size_t)p * sizeof(g2j)) ||
      !c->lines.ensure((size_t)p * sizeof(line_block)) || !c->lines_d.ensure((size_t)p * sizeof(line_block_d)) ||
      !c->scratch.ensure((size_t)2 * p * MILLER_LINES * sizeof(fq2d)) || !c->ct_ok.ensure(p) ||
      !c->ct_valid.ensure(p) || !c->dec_st.ensure((size_t)2 * p * 4))
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_prepare_ciphertexts_d: out of device memory");
  const size_t m_early = early_shares ? (size_t)early_n * p : 0;
  if (m_early && (!c->S.ensure(m_early * sizeof(g1a)) || !c->S_status.ensure(m_early * 4)))
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_prepare_ciphertexts_d: out of device memory");
  const dim3 b64(64);
  const bool own = c->own_me != UINT32_MAX;
  // own entry of the early-decoded matrix (written by k_prepare_lines), as hbx_verify_dec_shares_d
  const uint32_t me_early = (own && c->own_me < early_n) ? c->own_me : UINT32_MAX;
  {
    timed t_(c, HBX_K_PREPARE_CT, s);
    const uint32_t hash_blocks = (uint32_t)(((size_t)p * HASH_K + 63) / 64);
    const uint32_t dec_blocks = (own ? 4 : 2) * ((p + 63) / 64);  // wave-aligned parts (k_prepare_ct)
    const uint32_t share_blocks = (uint32_t)((m_early + 63) / 64);
    if (own && (!c->own_S.ensure((size_t)p * sizeof(g1a)) || !c->own_part.ensure((size_t)2 * p * sizeof(g1j))))
      return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_prepare_ciphertexts_d: out of device memory");
    // HBX_SPLIT_PREP=1 (profiling): the hash part and the decode parts as two launches, so a
    // kernel trace times each chain on its own
    static const bool split = getenv("HBX_SPLIT_PREP") != nullptr;
    const uint32_t parts = split ? 2 : 1;
    for (uint32_t q = 0; q < parts; q++) {
      const uint32_t b0 = split && q == 1 ? hash_blocks : 0;
      const uint32_t nb = split ? (q == 0 ? hash_blocks : dec_blocks + share_blocks)
                                : hash_blocks + dec_blocks + share_blocks;
      hipLaunchKernelGGL(k_prepare_ct, dim3(nb), b64, 0, s, d_u_comp, d_v_blob, d_v_off, d_w_comp, p, hash_blocks,
                         c->U.as<g1a>(), c->G2pts.as<g2a>(), c->dec_st.as<int32_t>(),
                         own ? c->own_sk.as<uint32_t>() : nullptr, own ? c->own_part.as<g1j>() : nullptr, c->Hj.as<g2j>(), c->digest,
                         b0, dec_blocks, early_shares, m_early, early_n ? early_n : 1u, me_early, c->S.as<g1a>(),
                         c->S_status.as<int32_t>());
    }
    c->own_ready = own;
  }
  HIPCHK(c, hipGetLastError());
  {
    timed t_(c, HBX_K_PREPARE_LINES, s);
    const uint32_t line_blocks = (2 * p * LINE_K + 63) / 64, own_blocks = own ? (p + 63) / 64 : 0;
    const bool own_entry = m_early && me_early != UINT32_MAX;
    // grouped addition steps (g2_raw_lines_group<true>) at every size: since the group rounds pick
    // their operands by blocks (groupd.hpp gd_round) the grouped kernel is the faster one at N=256
    // too (lines 1.00 -> 0.85 ms, epoch 23.43 -> 23.27 ms averaged over two runs each), and two
    // epochs in flight stay within the runs' spread (22.7-23.4 ms per epoch either way).  Round 3
    // had kept it to launches below a full chip: its register footprint then slowed two epochs in
    // flight 28.2 -> 32.5 ms per epoch (profiles/r03n_bisect_*).
    auto kpl = k_prepare_lines<true>;
    hipLaunchKernelGGL(kpl, dim3(line_blocks + own_blocks), b64, 0, s, c->G2pts.as<g2a>(), 2 * p,
                       c->lines_d.as<line_pre_d>(), c->scratch.as<fq2d>(), c->dec_st.as<int32_t>(), p,
                       c->ct_ok.as<uint8_t>(), own ? c->own_part.as<g1j>() : nullptr,
                       own ? c->own_S.as<g1a>() : nullptr, early_n, me_early,
                       own_entry ? c->S.as<g1a>() : nullptr, own_entry ? c->S_status.as<int32_t>() : nullptr,
                       c->Hj.as<g2j>());
    HIPCHK(c, hipGetLastError());
    const uint32_t nl = 2 * p * MILLER_LINES;
    hipLaunchKernelGGL(k_normalise_lines, dim3((nl + 63) / 64), b64, 0, s, c->lines.as<line_pre>(),
                       c->scratch.as<fq2d>(), nl, c->lines_d.as<line_pre_d>(), c->G2pts.as<g2a>(),
                       c->Hj.as<g2j>());
  }
  HIPCHK(c, hipGetLastError());
  c->p_ct = p;
  c->ct_known = false;
  c->n_shares = 0;  // S / valid of an earlier verify belong to other ciphertexts
  c->verified_p = 0;
  if (d_ct_valid) {
    // Ciphertext::verify now: one check per proposer (n = 0 share jobs, job 0 = the ciphertext)
    if (!c->S.ensure(sizeof(g1a)) || !c->S_status.ensure(4) || !c->valid.ensure(16))
      return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_prepare_ciphertexts_d: out of device memory");
    int rc = launch_pair_checks(c, s, 0, p, 0, 0, nullptr);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(d_ct_valid, c->ct_valid.p, p, hipMemcpyDeviceToDevice, s));
    c->ct_known = true;
  }
  c->d_v_blob = d_v_blob;
  c->d_v_off = d_v_off;
  c->max_v_len = max_v_len;
  return HBX_OK;
}

int hbx_prepare_ciphertexts_d(hbx_ctx* c, const uint8_t* d_u_comp, const uint8_t* d_v_blob,
                              const uint64_t* d_v_off, const uint8_t* d_w_comp, uint32_t p,
                              uint64_t max_v_len, uint8_t* d_ct_valid, void* stream) {
  return prepare_impl(c, d_u_comp, d_v_blob, d_v_off, d_w_comp, p, max_v_len, d_ct_valid, stream, nullptr, 0);
}

int hbx_prepare_ciphertexts(hbx_ctx* c, const uint8_t* u_comp, const uint8_t* v_blob, const uint64_t* v_off,
                            const uint8_t* w_comp, uint32_t p, uint8_t* ct_valid_bits) {
  if (!c || p == 0 || !u_comp || !v_off || !w_comp)
    return fail(c, HBX_E_INVALID_ARG, "hbx_prepare_ciphertexts: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  stream_scope ss_{c, pick(c, c->stream)};
  const uint64_t vbytes = v_off[p];
  uint64_t maxv = 0;
  for (uint32_t j = 0; j < p; j++) {
    if (v_off[j + 1] < v_off[j]) return fail(c, HBX_E_INVALID_ARG, "v_off not monotone");
    maxv = std::max<uint64_t>(maxv, v_off[j + 1] - v_off[j]);
  }
  if (!c->u_comp_own.ensure((size_t)p * 48) || !c->w_comp_own.ensure((size_t)p * 96) ||
      !c->v_off_own.ensure((size_t)(p + 1) * 8) || !c->v_blob_own.ensure(vbytes ? vbytes : 16))
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_prepare_ciphertexts: out of device memory");
  HIPCHK(c, hipMemcpyAsync(c->u_comp_own.p, u_comp, (size_t)p * 48, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->w_comp_own.p, w_comp, (size_t)p * 96, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->v_off_own.p, v_off, (size_t)(p + 1) * 8, hipMemcpyHostToDevice, c->stream));
  if (vbytes) HIPCHK(c, hipMemcpyAsync(c->v_blob_own.p, v_blob, vbytes, hipMemcpyHostToDevice, c->stream));
  if (!c->ct_valid.ensure(p)) return fail(c, HBX_E_OUT_OF_MEMORY, "out of device memory");
  int rc = hbx_prepare_ciphertexts_d(c, c->u_comp_own.as<uint8_t>(), c->v_blob_own.as<uint8_t>(),
                                     c->v_off_own.as<uint64_t>(), c->w_comp_own.as<uint8_t>(), p, maxv,
                                     c->ct_valid.as<uint8_t>(), c->stream);
  if (rc) return rc;
  std::vector<uint8_t> ok(p);
  HIPCHK(c, hipMemcpyAsync(ok.data(), c->ct_valid.p, p, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (ct_valid_bits) pack_bits(ok.data(), p, ct_valid_bits);
  return HBX_OK;
}

// Share checks of the prepared ciphertexts.  `predecoded`: the fused epoch call (hbx_decrypt_epoch_d)
// had prepare_impl decode exactly these shares into S / S_status already.
static int verify_impl(hbx_ctx* c, const uint8_t* d_shares, const uint8_t* d_present, uint32_t n, uint32_t p,
                       uint8_t* d_valid, void* stream, bool predecoded) {
  if (!c || !d_shares || n == 0 || p == 0) return fail(c, HBX_E_INVALID_ARG, "hbx_verify_dec_shares_d: bad args");
  if (c->n_keys == 0) return fail(c, HBX_E_NO_KEYS, "hbx_set_pk_shares has not been called");
  if (p != c->p_ct) return fail(c, HBX_E_NO_CIPHERTEXTS, "p=%u but %u ciphertexts prepared", p, c->p_ct);
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  stream_scope ss_{c, s};
  const size_t m = (size_t)n * p;
  if (!c->S.ensure(m * sizeof(g1a)) || !c->S_status.ensure(m * 4) || !c->valid.ensure(m))
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_verify_dec_shares_d: out of device memory");
  // own-share mode: this node's share is the one computed in prepare, and its check IS
  // Ciphertext::verify (k_verify_shares); otherwise the ciphertext checks run separately
  const bool own = c->own_ready && c->own_me < n;
  if (!predecoded) {
    hipLaunchKernelGGL(k_decompress_shares, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, d_shares, m,
                       c->S.as<g1a>(), c->S_status.as<int32_t>(), n, own ? c->own_me : UINT32_MAX,
                       own ? c->own_S.as<g1a>() : nullptr);
    HIPCHK(c, hipGetLastError());
  }
  // ciphertext checks (if prepare deferred them): latency-bound, p checks -> 16-lane groups
  if (!c->ct_known && !own) {
    int rc = launch_pair_checks(c, s, n, p, n, n, d_present);
    if (rc) return rc;
    c->ct_known = true;
  }
  // share checks: one lane per check when the launch fills the chip (throughput), else six lanes
  // per check when that still leaves at most one wave per SIMD, else three (latency: an epoch
  // shard on one of several GPUs; pairing3.hpp / pairing3d.hpp).  The two-lane
  // check (no scratch) measured slower than the one-lane check at N=256 (26.6 vs 24.0 ms,
  // profiles/r03a_bench.json), so it is only used when asked for.
  {
    timed t_(c, HBX_K_VERIFY_SHARES, s);
    // below a full chip: the most lanes per check that still fit one wave per SIMD -- six, three,
    // then two (an N=256 epoch over 2 GPUs: 1,024 two-lane waves, 11.0 ms against 17.4 for the
    // three-lane check in two rounds of waves, profiles/r04w_lanes.txt)
    const size_t waves1 = (size_t)((n + 63) / 64) * p;
    const size_t waves2 = (size_t)((n + 31) / 32) * p;
    const size_t waves3 = (size_t)((n + G3_PER_WAVE - 1) / G3_PER_WAVE) * p;
    const size_t waves6 = (size_t)((n + G6_PER_WAVE - 1) / G6_PER_WAVE) * p;
    const size_t fill = (size_t)VERIFY_FILL_WAVES;
    const int lanes = c->verify_lanes   ? c->verify_lanes
                      : waves1 >= fill ? 1
                      : waves6 <= fill ? 6
                      : waves3 <= fill ? 3
                      : waves2 <= fill ? 2
                                       : 3;
    c->lanes_used = lanes;
    c->fb_last = nullptr;  // set again below by the one-lane path, the only one with a fallback
    if (lanes == 2) {
      // global slots of the final exponentiation: 2 x 78 dwords per lane of the launch
      const size_t glanes = (size_t)((n + 31) / 32) * p * 64;
      if (!c->gslot.ensure(glanes * 2 * LDS_FQ6D_PACKED * 4))
        return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_verify_dec_shares_d: out of device memory (slots)");
      hipLaunchKernelGGL(k_verify_shares2, dim3((n + 31) / 32, p), dim3(64), 0, s, c->S.as<g1a>(),
                         c->S_status.as<int32_t>(), d_present, c->pk_m.as<g1a>(), c->n_keys, c->G2pts.as<g2a>(),
                         c->lines_d.as<line_block_d>(), c->ct_ok.as<uint8_t>(), n, c->valid.as<uint8_t>(),
                         own ? c->own_me : UINT32_MAX,
                         (own && !c->ct_known) ? c->ct_valid.as<uint8_t>() : nullptr, c->gslot.as<uint32_t>());
    }
    else if (lanes == 6)
      hipLaunchKernelGGL(k_verify_shares6, dim3((n + G6_PER_WAVE - 1) / G6_PER_WAVE, p), dim3(64), 0, s,
                         c->S.as<g1a>(), c->S_status.as<int32_t>(), d_present, c->pk_m.as<g1a>(), c->n_keys,
                         c->G2pts.as<g2a>(), c->lines_d.as<line_block_d>(), c->ct_ok.as<uint8_t>(), n,
                         c->valid.as<uint8_t>(), own ? c->own_me : UINT32_MAX,
                         (own && !c->ct_known) ? c->ct_valid.as<uint8_t>() : nullptr);
    else if (lanes == 3)
      hipLaunchKernelGGL(k_verify_shares3, dim3((n + G3_PER_WAVE - 1) / G3_PER_WAVE, p), dim3(64), 0, s,
                         c->S.as<g1a>(), c->S_status.as<int32_t>(), d_present, c->pk_m.as<g1a>(), c->n_keys,
                         c->G2pts.as<g2a>(), c->lines_d.as<line_block_d>(), c->ct_ok.as<uint8_t>(), n,
                         c->valid.as<uint8_t>(), own ? c->own_me : UINT32_MAX,
                         (own && !c->ct_known) ? c->ct_valid.as<uint8_t>() : nullptr);
    else if (lanes == 7)  // the one-lane check as one kernel (final exponentiation through call frames)
      hipLaunchKernelGGL(k_verify_shares, dim3((n + 63) / 64, p), dim3(64), 0, s, c->S.as<g1a>(),
                         c->S_status.as<int32_t>(), d_present, c->pk_m.as<g1a>(), c->n_keys, c->G2pts.as<g2a>(),
                         c->lines_d.as<line_block_d>(), c->ct_ok.as<uint8_t>(), n, c->valid.as<uint8_t>(),
                         own ? c->own_me : UINT32_MAX,
                         (own && !c->ct_known) ? c->ct_valid.as<uint8_t>() : nullptr, 0u, nullptr);
    else {
      // one lane per check: the Miller loops, then the final exponentiation's seven steps as four
      // kernels over per-lane slots (fe1d.hpp: no Fq12 ever crosses a call frame)
      const dim3 grid((n + 63) / 64, p);
      if (!c->fe1slot.ensure((size_t)grid.x * grid.y * 64 * 3 * FE1_WORDS * 4))
        return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_verify_dec_shares_d: out of device memory (slots)");
      uint8_t* ctv = (own && !c->ct_known) ? c->ct_valid.as<uint8_t>() : nullptr;
      const uint32_t me = own ? c->own_me : UINT32_MAX;
      uint32_t* gs = c->fe1slot.as<uint32_t>();
      if (!c->fb_lanes.ensure(4)) return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_verify_dec_shares_d: out of device memory");
      HIPCHK(c, hipMemsetAsync(c->fb_lanes.p, 0, 4, s));
      c->fb_last = &c->fb_lanes;
      hipLaunchKernelGGL(k_verify_shares_ml, grid, dim3(64), 0, s, c->S.as<g1a>(), c->S_status.as<int32_t>(),
                         d_present, c->pk_m.as<g1a>(), c->n_keys, c->G2pts.as<g2a>(), c->lines_d.as<line_block_d>(),
                         c->ct_ok.as<uint8_t>(), n, c->valid.as<uint8_t>(), me, gs);
      const uint8_t* ctok = c->ct_ok.as<uint8_t>();
      uint8_t* vd = c->valid.as<uint8_t>();
      hipLaunchKernelGGL(k_fe1<0>, grid, dim3(64), 0, s, gs, n, vd, ctok, me, ctv, c->force_fallback);
      hipLaunchKernelGGL(k_fe1<1>, grid, dim3(64), 0, s, gs, n, vd, ctok, me, ctv, c->force_fallback);  // F1 + F2
      hipLaunchKernelGGL(k_fe1<3>, grid, dim3(64), 0, s, gs, n, vd, ctok, me, ctv, c->force_fallback);  // F3 + F4
      hipLaunchKernelGGL(k_fe1<5>, grid, dim3(64), 0, s, gs, n, vd, ctok, me, ctv, c->force_fallback);  // F5 + F6
      // lanes whose compressed squarings met g3 = 0 (never expected): the single-kernel check
      hipLaunchKernelGGL(k_verify_shares, grid, dim3(64), 0, s, c->S.as<g1a>(), c->S_status.as<int32_t>(), d_present,
                         c->pk_m.as<g1a>(), c->n_keys, c->G2pts.as<g2a>(), c->lines_d.as<line_block_d>(), ctok, n, vd,
                         me, ctv, 1u, c->fb_lanes.as<uint32_t>());
    }
  }
  HIPCHK(c, hipGetLastError());
  c->ct_known = true;
  hipLaunchKernelGGL(k_gate_by_ct, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, c->valid.as<uint8_t>(),
                     c->ct_valid.as<uint8_t>(), n, p);
  HIPCHK(c, hipGetLastError());
  if (d_valid) HIPCHK(c, hipMemcpyAsync(d_valid, c->valid.p, m, hipMemcpyDeviceToDevice, s));
  c->n_shares = n;
  c->verified_p = p;
  return HBX_OK;
}

int hbx_verify_dec_shares_d(hbx_ctx* c, const uint8_t* d_shares, const uint8_t* d_present, uint32_t n,
                            uint32_t p, uint8_t* d_valid, void* stream) {
  return verify_impl(c, d_shares, d_present, n, p, d_valid, stream, false);
}

int hbx_verify_dec_shares(hbx_ctx* c, const uint8_t* shares, const uint8_t* present_bits, uint32_t n,
                          uint32_t p, uint8_t* valid_bits) {
  if (!c || !shares || n == 0 || p == 0) return fail(c, HBX_E_INVALID_ARG, "hbx_verify_dec_shares: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  stream_scope ss_{c, pick(c, c->stream)};
  const size_t m = (size_t)n * p;
  if (!c->shares_own.ensure(m * 48) || (present_bits && !c->present_own.ensure(m)))
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_verify_dec_shares: out of device memory");
  HIPCHK(c, hipMemcpyAsync(c->shares_own.p, shares, m * 48, hipMemcpyHostToDevice, c->stream));
  std::vector<uint8_t> pres;
  if (present_bits) {
    pres.resize(m);
    for (size_t k = 0; k < m; k++) pres[k] = (present_bits[k >> 3] >> (k & 7)) & 1;
    HIPCHK(c, hipMemcpyAsync(c->present_own.p, pres.data(), m, hipMemcpyHostToDevice, c->stream));
  }
  int rc = hbx_verify_dec_shares_d(c, c->shares_own.as<uint8_t>(),
                                   present_bits ? c->present_own.as<uint8_t>() : nullptr, n, p, nullptr,
                                   c->stream);
  if (rc) return rc;
  std::vector<uint8_t> v(m);
  HIPCHK(c, hipMemcpyAsync(v.data(), c->valid.p, m, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (valid_bits) pack_bits(v.data(), m, valid_bits);
  return HBX_OK;
}

int hbx_rs_encode_d(hbx_ctx* c, uint8_t* d_shards, uint32_t inst, uint32_t k, uint32_t m, uint32_t L, void* stream) {
  if (!c || !d_shards || inst == 0 || L == 0) return fail(c, HBX_E_INVALID_ARG, "hbx_rs_encode_d: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  stream_scope ss_{c, s};
  if (m == 0) return HBX_OK;  // Coding::Trivial
  int rc = rs_setup(c, k, m, s);
  if (rc) return rc;
  rs_code(c, d_shards, (size_t)(k + m) * L, L, k, inst, c->rs_enc_job.as<rs_job>(), c->rs_enc_coef.as<uint16_t>(),
          c->rs_enc_ptab.as<gf_ptab>(), 0u, m, s);
  HIPCHK(c, hipGetLastError());
  return HBX_OK;
}

int hbx_rs_reconstruct_d(hbx_ctx* c, uint8_t* d_shards, const uint8_t* d_present, uint32_t inst, uint32_t k,
                         uint32_t m, uint32_t L, int32_t* d_status, void* stream) {
  if (!c || !d_shards || !d_present || !d_status || inst == 0 || L == 0)
    return fail(c, HBX_E_INVALID_ARG, "hbx_rs_reconstruct_d: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  stream_scope ss_{c, s};
  int rc = rs_setup(c, k, m, s);
  if (rc) return rc;
  return rs_reconstruct(c, d_shards, d_present, inst, k, m, L, d_status, s);
}

int hbx_merkle_roots_d(hbx_ctx* c, const uint8_t* d_shards, uint32_t inst, uint32_t n, uint32_t L, uint8_t* d_roots,
                       void* stream) {
  if (!c || !d_shards || !d_roots || inst == 0) return fail(c, HBX_E_INVALID_ARG, "hbx_merkle_roots_d: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  stream_scope ss_{c, s};
  return merkle_roots(c, d_shards, inst, n, L, d_roots, s);
}

int hbx_merkle_validate_d(hbx_ctx* c, const uint8_t* d_values, uint32_t vlen, const uint8_t* d_node_hash,
                          const uint8_t* d_sib_hash, const uint32_t* d_sides, const uint32_t* d_depth,
                          const uint8_t* d_root, const uint32_t* d_sender, uint32_t count, uint32_t nproofs,
                          uint8_t* d_valid, void* stream) {
  if (!c || !d_values || !d_node_hash || !d_sib_hash || !d_sides || !d_depth || !d_root || !d_sender || !d_valid ||
      nproofs == 0 || vlen == 0)
    return fail(c, HBX_E_INVALID_ARG, "hbx_merkle_validate_d: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  stream_scope ss_{c, s};
  // long values (Echo proofs of real shards): their leaf digests first, by the leaf kernels (the
  // producer/consumer SHA-256 or the two-lane SHA3 schedule) instead of one lane per value inside
  // the path check
  const uint32_t* vdigest = nullptr;
  if (vlen > 256) {
    if (!c->val_digest.ensure((size_t)nproofs * 32))
      return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_merkle_validate_d: out of device memory");
    timed t_(c, HBX_K_MERKLE_LEAVES, s);
    if (c->merkle == HBX_MERKLE_SHA256)
      hipLaunchKernelGGL(k_merkle_leaves_sha256, dim3((nproofs + 63) / 64, 1), dim3(128), 0, s, d_values + 1, (size_t)0,
                         nproofs, vlen - 1, c->val_digest.as<uint32_t>(), (const uint16_t*)nullptr, 0u, vlen);
    else
      hipLaunchKernelGGL(k_merkle_leaves_sha3, dim3((nproofs + 31) / 32, 1), dim3(64), 0, s, d_values + 1, (size_t)0,
                         nproofs, vlen - 1, c->val_digest.as<uint32_t>(), (const uint16_t*)nullptr, 0u, vlen);
    HIPCHK(c, hipGetLastError());
    vdigest = c->val_digest.as<uint32_t>();
  }
  hipLaunchKernelGGL(k_merkle_validate, dim3((nproofs + 63) / 64), dim3(64), 0, s, d_values, vlen,
                     d_node_hash, d_sib_hash, d_sides, d_depth, d_root, d_sender, count, nproofs, d_valid, c->merkle,
                     vdigest);
  HIPCHK(c, hipGetLastError());
  return HBX_OK;
}

uint32_t hbx_merkle_node_count(uint32_t n) { return n ? merkle_node_count(n) : 0; }

int hbx_merkle_build_d(hbx_ctx* c, const uint8_t* d_shards, uint32_t inst, uint32_t n, uint32_t L, uint8_t* d_nodes,
                       uint8_t* d_roots, void* stream) {
  if (!c || !d_shards || !d_nodes || inst == 0) return fail(c, HBX_E_INVALID_ARG, "hbx_merkle_build_d: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  stream_scope ss_{c, s};
  uint8_t* roots = d_roots;
  if (!roots) {
    if (!c->roots.ensure((size_t)inst * 32)) return fail(c, HBX_E_OUT_OF_MEMORY, "merkle: roots");
    roots = c->roots.as<uint8_t>();
  }
  return merkle_roots(c, d_shards, inst, n, L, roots, s, d_nodes);
}

int hbx_merkle_proofs_d(hbx_ctx* c, const uint8_t* d_nodes, uint32_t n, const uint32_t* d_req, uint32_t count,
                        uint8_t* d_node_hash, uint8_t* d_sib_hash, uint32_t* d_sides, uint32_t* d_depth,
                        uint8_t* d_root, void* stream) {
  if (!c || !d_nodes || !d_req || !d_node_hash || !d_sib_hash || !d_sides || !d_depth || !d_root || count == 0 ||
      n == 0 || n > (uint32_t)RS_MAX_N)
    return fail(c, HBX_E_INVALID_ARG, "hbx_merkle_proofs_d: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  stream_scope ss_{c, s};
  hipLaunchKernelGGL(k_merkle_proofs, dim3((count + 63) / 64), dim3(64), 0, s, d_nodes, n, d_req, count,
                     d_node_hash, d_sib_hash, d_sides, d_depth, d_root);
  HIPCHK(c, hipGetLastError());
  return HBX_OK;
}

// decode_from_shards + glue for `inst` instances; with d_leaf_hash the present shards' leaf digests
// are taken from it (validated Echo proofs) and only the reconstructed shards are hashed.
static int broadcast_decode(hbx_ctx* c, uint8_t* d_shards, const uint8_t* d_present, const uint8_t* d_leaf_hash,
                            const uint8_t* d_root_expect, uint32_t inst, uint32_t k, uint32_t m, uint32_t L,
                            uint8_t* d_out, uint64_t out_stride, uint64_t* d_out_len, int32_t* d_status, void* stream) {
  if (!c || !d_shards || !d_present || !d_root_expect || !d_out || !d_out_len || !d_status || inst == 0 || L == 0)
    return fail(c, HBX_E_INVALID_ARG, "hbx_broadcast_decode_d: bad args");
  // the payload length comes from the (untrusted) big-endian header: k L - 4 bytes is the most
  // glue_shards can take, so every output row must hold that many
  if ((uint64_t)k * L >= 4 && out_stride < (uint64_t)k * L - 4)
    return fail(c, HBX_E_INVALID_ARG, "hbx_broadcast_decode_d: out_stride %llu < k L - 4 = %llu",
                (unsigned long long)out_stride, (unsigned long long)((uint64_t)k * L - 4));
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  stream_scope ss_{c, s};
  int rc = rs_setup(c, k, m, s);
  if (rc) return rc;
  rc = rs_reconstruct(c, d_shards, d_present, inst, k, m, L, d_status, s);
  if (rc) return rc;
  if (!c->roots.ensure((size_t)inst * 32)) return fail(c, HBX_E_OUT_OF_MEMORY, "decode: roots");
  if (d_leaf_hash) {
    const uint32_t n = k + m;
    if (n > (uint32_t)RS_MAX_N) return fail(c, HBX_E_INVALID_ARG, "merkle: need 1 <= n <= 256");
    if (!c->leaf_hash.ensure((size_t)inst * n * 32) || !c->leaf_slots.ensure((size_t)inst * (m ? m : 1) * 2))
      return fail(c, HBX_E_OUT_OF_MEMORY, "decode: leaf hashes");
    const uint32_t words = inst * n * 8;
    hipLaunchKernelGGL(k_import_leaf_hashes, dim3((words + 255) / 256), dim3(256), 0, s, d_leaf_hash, d_present,
                       inst * n, c->leaf_hash.as<uint32_t>());
    if (m) {  // Coding::Trivial reconstructs nothing: every shard is present or the status is an error
      hipLaunchKernelGGL(k_missing_slots, dim3(inst), dim3(64), 0, s, d_present, n, d_status, m,
                         c->leaf_slots.as<uint16_t>());
      timed t_(c, HBX_K_MERKLE_LEAVES, s);
      if (c->merkle == HBX_MERKLE_SHA256)
        hipLaunchKernelGGL(k_merkle_leaves_sha256, dim3((m + 63) / 64, inst), dim3(128), 0, s, d_shards,
                           (size_t)n * L, n, L, c->leaf_hash.as<uint32_t>(), c->leaf_slots.as<uint16_t>(), m, 0u);
      else
        hipLaunchKernelGGL(k_merkle_leaves_sha3, dim3((m + 31) / 32, inst), dim3(64), 0, s, d_shards, (size_t)n * L,
                           n, L, c->leaf_hash.as<uint32_t>(), c->leaf_slots.as<uint16_t>(), m, 0u);
    }
    HIPCHK(c, hipGetLastError());
    hipLaunchKernelGGL(k_merkle_tree, dim3(inst), dim3(128), 0, s, c->leaf_hash.as<uint32_t>(), n,
                       c->roots.as<uint8_t>(), (uint8_t*)nullptr, c->merkle);
    HIPCHK(c, hipGetLastError());
  } else {
    rc = merkle_roots(c, d_shards, inst, k + m, L, c->roots.as<uint8_t>(), s);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(k_root_check, dim3((inst + 63) / 64), dim3(64), 0, s, c->roots.as<uint8_t>(), d_root_expect, inst,
                     d_status);
  HIPCHK(c, hipGetLastError());
  const uint64_t glue_blocks = ((uint64_t)k * L + 4095) / 4096;
  hipLaunchKernelGGL(k_glue, dim3((unsigned)glue_blocks, inst), dim3(256), 0, s, d_shards, (size_t)(k + m) * L, k, L, d_out,
                     (size_t)out_stride, d_out_len, d_status);
  HIPCHK(c, hipGetLastError());
  return HBX_OK;
}

int hbx_broadcast_decode_d(hbx_ctx* c, uint8_t* d_shards, const uint8_t* d_present, const uint8_t* d_root_expect,
                           uint32_t inst, uint32_t k, uint32_t m, uint32_t L, uint8_t* d_out, uint64_t out_stride,
                           uint64_t* d_out_len, int32_t* d_status, void* stream) {
  return broadcast_decode(c, d_shards, d_present, nullptr, d_root_expect, inst, k, m, L, d_out, out_stride, d_out_len,
                          d_status, stream);
}

int hbx_broadcast_decode_leaves_d(hbx_ctx* c, uint8_t* d_shards, const uint8_t* d_present, const uint8_t* d_leaf_hash,
                                  const uint8_t* d_root_expect, uint32_t inst, uint32_t k, uint32_t m, uint32_t L,
                                  uint8_t* d_out, uint64_t out_stride, uint64_t* d_out_len, int32_t* d_status,
                                  void* stream) {
  if (!d_leaf_hash) return fail(c, HBX_E_INVALID_ARG, "hbx_broadcast_decode_leaves_d: d_leaf_hash is NULL");
  return broadcast_decode(c, d_shards, d_present, d_leaf_hash, d_root_expect, inst, k, m, L, d_out, out_stride,
                          d_out_len, d_status, stream);
}

// ---- Broadcast, host-pointer forms (include/hbx.h): the _d calls above on context-owned staging
// buffers (c->hs[]), on the context's own stream, blocking until the outputs are on the host -- the
// shape a thin Rust FFI drives from Vec<u8> / &[u8] ------------
static uint8_t* stage(hbx_ctx* c, int slot, size_t bytes) {
  return c->hs[slot].ensure(bytes ? bytes : 1) ? c->hs[slot].as<uint8_t>() : nullptr;
}
#define HBX_STAGE(ptr, slot, bytes, what)                                                      \
  uint8_t* ptr = stage(c, slot, bytes);                                                      \
  if (!ptr) return fail(c, HBX_E_OUT_OF_MEMORY, "%s: out of device memory (staging)", what)
#define HBX_H2D(dst, src, bytes) HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream))
#define HBX_D2H(dst, src, bytes) HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream))

int hbx_rs_encode(hbx_ctx* c, uint8_t* shards, uint32_t inst, uint32_t k, uint32_t m, uint32_t L) {
  if (!c || !shards || inst == 0 || L == 0) return fail(c, HBX_E_INVALID_ARG, "hbx_rs_encode: bad args");
  if (m == 0) return HBX_OK;  // Coding::Trivial
  HIPCHK(c, hipSetDevice(c->device));
  stream_scope ss_{c, pick(c, c->stream)};
  const size_t row = (size_t)(k + m) * L;
  HBX_STAGE(d, 0, row * inst, "hbx_rs_encode");
  // the k data shards of every instance in, the m parity shards out (one strided copy each way)
  HIPCHK(c, hipMemcpy2DAsync(d, row, shards, row, (size_t)k * L, inst, hipMemcpyHostToDevice, c->stream));
  int rc = hbx_rs_encode_d(c, d, inst, k, m, L, c->stream);
  if (rc) return rc;
  HIPCHK(c, hipMemcpy2DAsync(shards + (size_t)k * L, row, d + (size_t)k * L, row, (size_t)m * L, inst,
                             hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return HBX_OK;
}

int hbx_rs_reconstruct(hbx_ctx* c, uint8_t* shards, const uint8_t* present, uint32_t inst, uint32_t k, uint32_t m,
                       uint32_t L, int32_t* status) {
  if (!c || !shards || !present || !status || inst == 0 || L == 0)
    return fail(c, HBX_E_INVALID_ARG, "hbx_rs_reconstruct: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  stream_scope ss_{c, pick(c, c->stream)};
  const size_t n = (size_t)k + m, all = n * L * inst;
  HBX_STAGE(d, 0, all, "hbx_rs_reconstruct");
  HBX_STAGE(dp, 1, n * inst, "hbx_rs_reconstruct");
  HBX_STAGE(ds, 2, (size_t)inst * 4, "hbx_rs_reconstruct");
  HBX_H2D(d, shards, all);
  HBX_H2D(dp, present, n * inst);
  int rc = hbx_rs_reconstruct_d(c, d, dp, inst, k, m, L, (int32_t*)ds, c->stream);
  if (rc) return rc;
  HBX_D2H(shards, d, all);
  HBX_D2H(status, ds, (size_t)inst * 4);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return HBX_OK;
}

int hbx_merkle_roots(hbx_ctx* c, const uint8_t* shards, uint32_t inst, uint32_t n, uint32_t L, uint8_t* roots) {
  if (!c || !shards || !roots || inst == 0) return fail(c, HBX_E_INVALID_ARG, "hbx_merkle_roots: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  stream_scope ss_{c, pick(c, c->stream)};
  const size_t all = (size_t)n * L * inst;
  HBX_STAGE(d, 0, all, "hbx_merkle_roots");
  HBX_STAGE(dr, 1, (size_t)inst * 32, "hbx_merkle_roots");
  HBX_H2D(d, shards, all);
  int rc = hbx_merkle_roots_d(c, d, inst, n, L, dr, c->stream);
  if (rc) return rc;
  HBX_D2H(roots, dr, (size_t)inst * 32);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return HBX_OK;
}

int hbx_merkle_build(hbx_ctx* c, const uint8_t* shards, uint32_t inst, uint32_t n, uint32_t L, uint8_t* nodes,
                     uint8_t* roots) {
  if (!c || !shards || !nodes || inst == 0 || n == 0) return fail(c, HBX_E_INVALID_ARG, "hbx_merkle_build: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  stream_scope ss_{c, pick(c, c->stream)};
  const size_t all = (size_t)n * L * inst, nb = (size_t)inst * merkle_node_count(n) * 32;
  HBX_STAGE(d, 0, all, "hbx_merkle_build");
  HBX_STAGE(dn, 1, nb, "hbx_merkle_build");
  HBX_STAGE(dr, 2, (size_t)inst * 32, "hbx_merkle_build");
  HBX_H2D(d, shards, all);
  int rc = hbx_merkle_build_d(c, d, inst, n, L, dn, dr, c->stream);
  if (rc) return rc;
  HBX_D2H(nodes, dn, nb);
  if (roots) HBX_D2H(roots, dr, (size_t)inst * 32);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return HBX_OK;
}

int hbx_merkle_proofs(hbx_ctx* c, const uint8_t* nodes, uint32_t inst, uint32_t n, const uint32_t* req, uint32_t count,
                      uint8_t* node_hash, uint8_t* sib_hash, uint32_t* sides, uint32_t* depth, uint8_t* root) {
  if (!c || !nodes || !req || !node_hash || !sib_hash || !sides || !depth || !root || inst == 0 || count == 0 ||
      n == 0 || n > (uint32_t)RS_MAX_N)
    return fail(c, HBX_E_INVALID_ARG, "hbx_merkle_proofs: bad args");
  for (uint32_t q = 0; q < count; q++)
    if (req[2 * q] >= inst || req[2 * q + 1] >= n)
      return fail(c, HBX_E_INVALID_ARG, "hbx_merkle_proofs: request %u names leaf %u of instance %u (inst %u, n %u)",
                  q, req[2 * q + 1], req[2 * q], inst, n);
  HIPCHK(c, hipSetDevice(c->device));
  stream_scope ss_{c, pick(c, c->stream)};
  const size_t nb = (size_t)inst * merkle_node_count(n) * 32;
  HBX_STAGE(dn, 0, nb, "hbx_merkle_proofs");
  HBX_STAGE(dq, 1, (size_t)count * 8, "hbx_merkle_proofs");
  HBX_STAGE(dh, 2, (size_t)count * 17 * 32, "hbx_merkle_proofs");
  HBX_STAGE(dsib, 3, (size_t)count * 16 * 32, "hbx_merkle_proofs");
  HBX_STAGE(dsd, 4, (size_t)count * 8, "hbx_merkle_proofs");
  HBX_STAGE(dr, 5, (size_t)count * 32, "hbx_merkle_proofs");
  HBX_H2D(dn, nodes, nb);
  HBX_H2D(dq, req, (size_t)count * 8);
  // levels below a proof's depth are not written: zeros, as in a freshly allocated output
  HIPCHK(c, hipMemsetAsync(dh, 0, (size_t)count * 17 * 32, c->stream));
  HIPCHK(c, hipMemsetAsync(dsib, 0, (size_t)count * 16 * 32, c->stream));
  int rc = hbx_merkle_proofs_d(c, dn, n, (const uint32_t*)dq, count, dh, dsib, (uint32_t*)dsd,
                               (uint32_t*)dsd + count, dr, c->stream);
  if (rc) return rc;
  HBX_D2H(node_hash, dh, (size_t)count * 17 * 32);
  HBX_D2H(sib_hash, dsib, (size_t)count * 16 * 32);
  HBX_D2H(sides, dsd, (size_t)count * 4);
  HBX_D2H(depth, dsd + (size_t)count * 4, (size_t)count * 4);
  HBX_D2H(root, dr, (size_t)count * 32);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return HBX_OK;
}

int hbx_merkle_validate(hbx_ctx* c, const uint8_t* values, uint32_t vlen, const uint8_t* node_hash,
                        const uint8_t* sib_hash, const uint32_t* sides, const uint32_t* depth, const uint8_t* root,
                        const uint32_t* sender, uint32_t count, uint32_t nproofs, uint8_t* valid) {
  if (!c || !values || !node_hash || !sib_hash || !sides || !depth || !root || !sender || !valid || nproofs == 0 ||
      vlen == 0)
    return fail(c, HBX_E_INVALID_ARG, "hbx_merkle_validate: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  stream_scope ss_{c, pick(c, c->stream)};
  const size_t P = nproofs;
  HBX_STAGE(dv, 0, P * vlen, "hbx_merkle_validate");
  HBX_STAGE(dh, 1, P * 17 * 32, "hbx_merkle_validate");
  HBX_STAGE(dsib, 2, P * 16 * 32, "hbx_merkle_validate");
  HBX_STAGE(du, 3, P * 12, "hbx_merkle_validate");  // sides | depth | sender
  HBX_STAGE(dr, 4, P * 32, "hbx_merkle_validate");
  HBX_STAGE(dok, 5, P, "hbx_merkle_validate");
  HBX_H2D(dv, values, P * vlen);
  HBX_H2D(dh, node_hash, P * 17 * 32);
  HBX_H2D(dsib, sib_hash, P * 16 * 32);
  HBX_H2D(du, sides, P * 4);
  HBX_H2D(du + P * 4, depth, P * 4);
  HBX_H2D(du + P * 8, sender, P * 4);
  HBX_H2D(dr, root, P * 32);
  const uint32_t* u = (const uint32_t*)du;
  int rc = hbx_merkle_validate_d(c, dv, vlen, dh, dsib, u, u + P, dr, u + 2 * P, count, nproofs, dok, c->stream);
  if (rc) return rc;
  HBX_D2H(valid, dok, P);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return HBX_OK;
}

static int broadcast_decode_host(hbx_ctx* c, uint8_t* shards, const uint8_t* present, const uint8_t* leaf_hash,
                                 const uint8_t* root_expect, uint32_t inst, uint32_t k, uint32_t m, uint32_t L,
                                 uint8_t* out, uint64_t out_stride, uint64_t* out_len, int32_t* status,
                                 const char* what) {
  if (!c || !shards || !present || !root_expect || !out || !out_len || !status || inst == 0 || L == 0)
    return fail(c, HBX_E_INVALID_ARG, "%s: bad args", what);
  HIPCHK(c, hipSetDevice(c->device));
  stream_scope ss_{c, pick(c, c->stream)};
  const size_t n = (size_t)k + m, all = n * L * inst;
  HBX_STAGE(d, 0, all, what);
  HBX_STAGE(dp, 1, n * inst, what);
  HBX_STAGE(dre, 2, (size_t)inst * 32, what);
  HBX_STAGE(dout, 3, (size_t)inst * out_stride, what);
  HBX_STAGE(dlen, 4, (size_t)inst * 12, what);  // out_len (u64) | status (i32)
  uint8_t* dl = nullptr;
  if (leaf_hash) {
    dl = stage(c, 5, n * inst * 32);
    if (!dl) return fail(c, HBX_E_OUT_OF_MEMORY, "%s: out of device memory (staging)", what);
    HBX_H2D(dl, leaf_hash, n * inst * 32);
  }
  HBX_H2D(d, shards, all);
  HBX_H2D(dp, present, n * inst);
  HBX_H2D(dre, root_expect, (size_t)inst * 32);
  HIPCHK(c, hipMemsetAsync(dout, 0, (size_t)inst * out_stride, c->stream));  // bytes past a payload: 0
  int rc = broadcast_decode(c, d, dp, dl, dre, inst, k, m, L, dout, out_stride, (uint64_t*)dlen,
                            (int32_t*)(dlen + (size_t)inst * 8), c->stream);
  if (rc) return rc;
  HBX_D2H(shards, d, all);
  HBX_D2H(out, dout, (size_t)inst * out_stride);
  HBX_D2H(out_len, dlen, (size_t)inst * 8);
  HBX_D2H(status, dlen + (size_t)inst * 8, (size_t)inst * 4);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return HBX_OK;
}

int hbx_broadcast_decode(hbx_ctx* c, uint8_t* shards, const uint8_t* present, const uint8_t* root_expect, uint32_t inst,
                         uint32_t k, uint32_t m, uint32_t L, uint8_t* out, uint64_t out_stride, uint64_t* out_len,
                         int32_t* status) {
  return broadcast_decode_host(c, shards, present, nullptr, root_expect, inst, k, m, L, out, out_stride, out_len,
                               status, "hbx_broadcast_decode");
}

int hbx_broadcast_decode_leaves(hbx_ctx* c, uint8_t* shards, const uint8_t* present, const uint8_t* leaf_hash,
                                const uint8_t* root_expect, uint32_t inst, uint32_t k, uint32_t m, uint32_t L,
                                uint8_t* out, uint64_t out_stride, uint64_t* out_len, int32_t* status) {
  if (!leaf_hash) return fail(c, HBX_E_INVALID_ARG, "hbx_broadcast_decode_leaves: leaf_hash is NULL");
  return broadcast_decode_host(c, shards, present, leaf_hash, root_expect, inst, k, m, L, out, out_stride, out_len,
                               status, "hbx_broadcast_decode_leaves");
}
#undef HBX_STAGE
#undef HBX_H2D
#undef HBX_D2H

// ---- Common Coin ----------------------------------------------------------------------------
// The true H = hash_g2(nonce) of the prepared nonces from H' = [m] H (k_h2_from_heff), once, on s.
static int coin_true_h(hbx_ctx* c, hipStream_t s) {
  if (c->coin_h_ready) return HBX_OK;
  hipLaunchKernelGGL(k_h2_from_heff, dim3((c->coin_I + 63) / 64), dim3(64), 0, s, c->coin_Hp.as<g2a>(), c->coin_I,
                     c->coin_H.as<g2a>());
  HIPCHK(c, hipGetLastError());
  c->coin_h_ready = true;
  return HBX_OK;
}

int hbx_prepare_nonces(hbx_ctx* c, const uint8_t* nonce_blob, const uint64_t* nonce_off, uint32_t count,
                       uint8_t* h96) {
  if (!c || !nonce_off || count == 0) return fail(c, HBX_E_INVALID_ARG, "hbx_prepare_nonces: bad args");
  for (uint32_t j = 0; j < count; j++)
    if (nonce_off[j + 1] < nonce_off[j]) return fail(c, HBX_E_INVALID_ARG, "nonce_off not monotone");
  const uint64_t total = nonce_off[count];
  if (total && !nonce_blob) return fail(c, HBX_E_INVALID_ARG, "hbx_prepare_nonces: null blob");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, c->stream);
  stream_scope ss_{c, s};
  if (!c->coin_blob.ensure(total ? total : 16) || !c->coin_off.ensure((size_t)(count + 1) * 8) ||
      !c->coin_H.ensure((size_t)count * sizeof(g2a)) || !c->coin_Hp.ensure((size_t)count * sizeof(g2a)) ||
      !c->coin_lines.ensure((size_t)count * MILLER_LINES * sizeof(line_pre)) ||
      !c->coin_lines_d.ensure((size_t)count * MILLER_LINES * sizeof(line_pre_d)) ||
      !c->coin_scratch.ensure((size_t)count * MILLER_LINES * sizeof(fq2d)) || !c->coin_out96.ensure((size_t)count * 96))
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_prepare_nonces: out of device memory");
  if (total) HIPCHK(c, hipMemcpyAsync(c->coin_blob.p, nonce_blob, total, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(c->coin_off.p, nonce_off, (size_t)(count + 1) * 8, hipMemcpyHostToDevice, s));
  // the caller's host buffers are free once the uploads are done; the hashing itself is enqueued
  // and the call returns without waiting for it (unless h96 asks for the hashes)
  HIPCHK(c, hipStreamSynchronize(s));
  {
    timed t_(c, HBX_K_HASH_NONCES, s);
    hipLaunchKernelGGL(k_hash_nonces, dim3((unsigned)(((size_t)count * HASH_K + 63) / 64)), dim3(64), 0, s, c->coin_blob.as<uint8_t>(),
                       c->coin_off.as<uint64_t>(), count, c->coin_Hp.as<g2a>(), c->digest, 0);
  }
  HIPCHK(c, hipGetLastError());
  // the Miller lines of H' are prepared on demand by the one-lane share checks (the two-lane
  // kernel, the default for a coin round, generates both pairs' lines itself); the true H only for
  // hbx_sign and h96 (coin_true_h): the share checks and the combine work on H' = [m] H
  c->coin_lines_ready = false;
  c->coin_h_ready = false;
  c->coin_I = count;
  if (h96) {
    if (int rc = coin_true_h(c, s)) return rc;
    hipLaunchKernelGGL(k_compress_g2, dim3((count + 63) / 64), dim3(64), 0, s, c->coin_H.as<g2a>(), count, 1u,
                       c->coin_out96.as<uint8_t>());
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(h96, c->coin_out96.p, (size_t)count * 96, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
  }
  if (!c->coin_ready_ev) HIPCHK(c, hipEventCreateWithFlags(&c->coin_ready_ev, hipEventDisableTiming));
  HIPCHK(c, hipEventRecord(c->coin_ready_ev, s));
  c->coin_I = count;
  return HBX_OK;
}

int hbx_sign(hbx_ctx* c, const uint8_t* sk32, uint32_t n, uint8_t* sig96) {
  if (!c || !sk32 || !sig96 || n == 0) return fail(c, HBX_E_INVALID_ARG, "hbx_sign: bad args");
  if (c->coin_I == 0) return fail(c, HBX_E_NO_CIPHERTEXTS, "hbx_prepare_nonces has not been called");
  if (!scalars_canonical(sk32, n)) return fail(c, HBX_E_INVALID_ARG, "hbx_sign: scalar >= r");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, c->stream);
  stream_scope ss_{c, s};
  const size_t m = (size_t)n * c->coin_I;
  if (!c->coin_sk.ensure((size_t)n * 32) || !c->coin_sig96.ensure(m * 96))
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_sign: out of device memory");
  HIPCHK(c, hipMemcpyAsync(c->coin_sk.p, sk32, (size_t)n * 32, hipMemcpyHostToDevice, s));
  if (int rc = coin_true_h(c, s)) return rc;
  hipLaunchKernelGGL(k_sign, dim3((n + 63) / 64, c->coin_I), dim3(64), 0, s, c->coin_sk.as<uint8_t>(), n,
                     c->coin_H.as<g2a>(), c->coin_sig96.as<uint8_t>());
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(sig96, c->coin_sig96.p, m * 96, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return HBX_OK;
}

// Signature-share checks of the prepared nonces on device buffers: d_sig96 [count][n][96],
// d_present [count][n] bytes (NULL = all present); statuses in c->coin_valid.
static int verify_sig_impl(hbx_ctx* c, const uint8_t* d_sig96, const uint8_t* d_present, uint32_t n, uint32_t count,
                           hipStream_t s) {
  const size_t m = (size_t)n * count;
  if (!c->coin_sig.ensure(m * sizeof(g2a)) || !c->coin_sig_st.ensure(m * 4) || !c->coin_valid.ensure(m))
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_verify_sig_shares: out of device memory");
  if (c->coin_ready_ev) HIPCHK(c, hipStreamWaitEvent(s, c->coin_ready_ev, 0));  // the nonces' hashes are in
  {
    timed t_(c, HBX_K_DECODE_SIGS, s);
    // curve membership only: the share checks test G2 membership on their Miller loop's [|x|] sigma
    hipLaunchKernelGGL(k_decompress_g2, dim3((unsigned)((m + 63) / 64)), dim3(64), 0, s, d_sig96, m, c->coin_sig.as<g2a>(),
                       c->coin_sig_st.as<int32_t>(), 0u);
  }
  HIPCHK(c, hipGetLastError());
  // two lanes per check when one lane per check would leave SIMDs idle (a coin round of 256
  // instances at N = 128 is 512 one-lane waves on 1,024 SIMDs), or when asked for
  // (hbx_set_verify_lanes 2); one lane otherwise
  const size_t waves1 = (size_t)((n + 63) / 64) * count;
  const int lanes = c->verify_lanes == 1 || c->verify_lanes == 2 ? c->verify_lanes
                    : waves1 < (size_t)VERIFY_FILL_WAVES ? 2 : 1;
  c->coin_lanes_used = lanes;
  if (!c->coin_lines_ready) {
    // H''s prepared lines (wave-uniform loads): the one-lane kernel's mixed loop, and since round 6
    // the two-lane kernel's H' pair (its lanes then generate only sigma's lines, together)
    timed t_(c, HBX_K_PREPARE_LINES, s);
    hipLaunchKernelGGL(k_prepare_lines<true>, dim3((count * LINE_K + 63) / 64), dim3(64), 0, s, c->coin_Hp.as<g2a>(), count,
                       c->coin_lines_d.as<line_pre_d>(), c->coin_scratch.as<fq2d>(), nullptr, 0u, nullptr, nullptr, nullptr, 1u,
                       UINT32_MAX, nullptr, nullptr, nullptr);
    HIPCHK(c, hipGetLastError());
    const uint32_t nl = count * MILLER_LINES;
    hipLaunchKernelGGL(k_normalise_lines, dim3((nl + 63) / 64), dim3(64), 0, s, c->coin_lines.as<line_pre>(),
                       c->coin_scratch.as<fq2d>(), nl, c->coin_lines_d.as<line_pre_d>(), nullptr, nullptr);
    HIPCHK(c, hipGetLastError());
    c->coin_lines_ready = true;
    // the lines are built on this call's stream: move the prepare event past them, so a later
    // one-lane check on another stream (which waits on coin_ready_ev) is ordered after the build
    if (!c->coin_ready_ev) HIPCHK(c, hipEventCreateWithFlags(&c->coin_ready_ev, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(c->coin_ready_ev, s));
  }
  {
    timed t_(c, HBX_K_VERIFY_SIG, s);
    if (lanes == 2) {
      const size_t glanes = (size_t)((n + 31) / 32) * count * 64;
      if (!c->gslot.ensure(glanes * 2 * LDS_FQ6D_PACKED * 4))
        return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_verify_sig_shares: out of device memory (slots)");
      if (!c->fb_coin.ensure(4)) return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_verify_sig_shares: out of device memory");
      HIPCHK(c, hipMemsetAsync(c->fb_coin.p, 0, 4, s));
      c->fb_last = &c->fb_coin;
      const dim3 grid((n + 31) / 32, count);
      // Miller loops; the final exponentiation with compressed runs; then the pairs whose
      // decompression met g3 = 0 (SHARE_FALLBACK) once more, Miller and Granger-Scott squarings
      // only (both launches return at once per pair when there are none)
      for (uint32_t retry = 0; retry < 2; retry++) {
        hipLaunchKernelGGL(k_verify_sig_shares2, grid, dim3(64), 0, s, c->coin_Hp.as<g2a>(), c->pk.as<g1a>(), c->n_keys,
                           c->coin_sig.as<g2a>(), c->coin_sig_st.as<int32_t>(), d_present, n, c->coin_valid.as<uint8_t>(),
                           c->gslot.as<uint32_t>(), retry, c->coin_lines_d.as<line_pre_d>());
        HIPCHK(c, hipGetLastError());
        if (retry == 0)
          hipLaunchKernelGGL(k_verify_sig_shares2_fe<true>, grid, dim3(64), 0, s, n, c->coin_valid.as<uint8_t>(),
                             c->gslot.as<uint32_t>(), c->force_fallback, c->fb_coin.as<uint32_t>());
        else
          hipLaunchKernelGGL(k_verify_sig_shares2_fe<false>, grid, dim3(64), 0, s, n, c->coin_valid.as<uint8_t>(),
                             c->gslot.as<uint32_t>(), 0u, c->fb_coin.as<uint32_t>());
        HIPCHK(c, hipGetLastError());
      }
    } else {
      c->fb_last = nullptr;  // the one-lane coin check has no fallback path
      hipLaunchKernelGGL(k_verify_sig_shares, dim3((n + 63) / 64, count), dim3(64), 0, s, c->coin_lines_d.as<line_pre_d>(),
                         c->coin_Hp.as<g2a>(), c->pk.as<g1a>(), c->n_keys, c->coin_sig.as<g2a>(),
                         c->coin_sig_st.as<int32_t>(), d_present, n, c->coin_valid.as<uint8_t>());
    }
  }
  HIPCHK(c, hipGetLastError());
  c->coin_n = n;
  return HBX_OK;
}

static int verify_sig_check(hbx_ctx* c, uint32_t n, uint32_t count) {
  if (c->n_keys == 0) return fail(c, HBX_E_NO_KEYS, "hbx_set_pk_shares has not been called");
  if (count != c->coin_I) return fail(c, HBX_E_NO_CIPHERTEXTS, "%u instances but %u nonces prepared", count, c->coin_I);
  return HBX_OK;
}

int hbx_verify_sig_shares(hbx_ctx* c, const uint8_t* sig96, const uint8_t* present_bits, uint32_t n, uint32_t count,
                          uint8_t* valid_bits) {
  if (!c || !sig96 || n == 0 || count == 0) return fail(c, HBX_E_INVALID_ARG, "hbx_verify_sig_shares: bad args");
  if (int rc = verify_sig_check(c, n, count)) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, c->stream);
  stream_scope ss_{c, s};
  const size_t m = (size_t)n * count;
  if (!c->coin_sig96.ensure(m * 96) || (present_bits && !c->coin_present.ensure(m)))
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_verify_sig_shares: out of device memory");
  HIPCHK(c, hipMemcpyAsync(c->coin_sig96.p, sig96, m * 96, hipMemcpyHostToDevice, s));
  std::vector<uint8_t> pres;
  if (present_bits) {
    pres.resize(m);
    for (size_t k = 0; k < m; k++) pres[k] = (present_bits[k >> 3] >> (k & 7)) & 1;
    HIPCHK(c, hipMemcpyAsync(c->coin_present.p, pres.data(), m, hipMemcpyHostToDevice, s));
  }
  if (int rc = verify_sig_impl(c, c->coin_sig96.as<uint8_t>(), present_bits ? c->coin_present.as<uint8_t>() : nullptr,
                               n, count, s))
    return rc;
  std::vector<uint8_t> v(m);
  HIPCHK(c, hipMemcpyAsync(v.data(), c->coin_valid.p, m, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  if (valid_bits) pack_bits(v.data(), m, valid_bits);
  return HBX_OK;
}

int hbx_verify_sig_shares_d(hbx_ctx* c, const uint8_t* d_sig96, const uint8_t* d_present, uint32_t n, uint32_t count,
                            uint8_t* d_status, void* stream) {
  if (!c || !d_sig96 || n == 0 || count == 0) return fail(c, HBX_E_INVALID_ARG, "hbx_verify_sig_shares_d: bad args");
  if (int rc = verify_sig_check(c, n, count)) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  stream_scope ss_{c, s};
  if (int rc = verify_sig_impl(c, d_sig96, d_present, n, count, s)) return rc;
  if (d_status) HIPCHK(c, hipMemcpyAsync(d_status, c->coin_valid.p, (size_t)n * count, hipMemcpyDeviceToDevice, s));
  return HBX_OK;
}

int hbx_get_coin_lanes_used(const hbx_ctx* c) { return c ? c->coin_lanes_used : 0; }

int hbx_verify_sigs(hbx_ctx* c, const uint8_t* pk48, const uint8_t* msg_blob, const uint64_t* msg_off,
                    const uint8_t* sig96, uint32_t count, uint8_t* status) {
  if (!c || !pk48 || !msg_off || !sig96 || !status || count == 0)
    return fail(c, HBX_E_INVALID_ARG, "hbx_verify_sigs: bad args");
  for (uint32_t i = 0; i < count; i++)
    if (msg_off[i + 1] < msg_off[i]) return fail(c, HBX_E_INVALID_ARG, "hbx_verify_sigs: msg_off not monotone");
  const uint64_t total = msg_off[count];
  if (total && !msg_blob) return fail(c, HBX_E_INVALID_ARG, "hbx_verify_sigs: null blob");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, c->stream);
  stream_scope ss_{c, s};
  if (!c->vs_pk.ensure((size_t)count * 48) || !c->vs_blob.ensure(total ? total : 16) ||
      !c->vs_off.ensure((size_t)(count + 1) * 8) || !c->vs_H.ensure((size_t)count * sizeof(g2a)) ||
      !c->vs_lines.ensure((size_t)count * MILLER_LINES * sizeof(line_pre)) ||
      !c->vs_lines_d.ensure((size_t)count * MILLER_LINES * sizeof(line_pre_d)) ||
      !c->vs_scratch.ensure((size_t)count * MILLER_LINES * sizeof(fq2d)) || !c->vs_sig96.ensure((size_t)count * 96) ||
      !c->vs_sig.ensure((size_t)count * sizeof(g2a)) || !c->vs_sig_st.ensure((size_t)count * 4) ||
      !c->vs_status.ensure(count))
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_verify_sigs: out of device memory");
  HIPCHK(c, hipMemcpyAsync(c->vs_pk.p, pk48, (size_t)count * 48, hipMemcpyHostToDevice, s));
  if (total) HIPCHK(c, hipMemcpyAsync(c->vs_blob.p, msg_blob, total, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(c->vs_off.p, msg_off, (size_t)(count + 1) * 8, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(c->vs_sig96.p, sig96, (size_t)count * 96, hipMemcpyHostToDevice, s));
  // H_i = hash_g2(msg_i) on lane groups, its Miller lines, the signatures' decode
  hipLaunchKernelGGL(k_hash_nonces, dim3((unsigned)(((size_t)count * HASH_K + 63) / 64)), dim3(64), 0, s,
                     c->vs_blob.as<uint8_t>(), c->vs_off.as<uint64_t>(), count, c->vs_H.as<g2a>(), c->digest, 1);
  HIPCHK(c, hipGetLastError());
  hipLaunchKernelGGL(k_decompress_g2, dim3((count + 63) / 64), dim3(64), 0, s, c->vs_sig96.as<uint8_t>(), (size_t)count,
                     c->vs_sig.as<g2a>(), c->vs_sig_st.as<int32_t>(), 1u);
  HIPCHK(c, hipGetLastError());
  hipLaunchKernelGGL(k_prepare_lines<true>, dim3((count * LINE_K + 63) / 64), dim3(64), 0, s, c->vs_H.as<g2a>(), count,
                     c->vs_lines_d.as<line_pre_d>(), c->vs_scratch.as<fq2d>(), nullptr, 0u, nullptr, nullptr, nullptr, 1u,
                     UINT32_MAX, nullptr, nullptr, nullptr);
  HIPCHK(c, hipGetLastError());
  const uint32_t nl = count * MILLER_LINES;
  hipLaunchKernelGGL(k_normalise_lines, dim3((nl + 63) / 64), dim3(64), 0, s, c->vs_lines.as<line_pre>(),
                     c->vs_scratch.as<fq2d>(), nl, c->vs_lines_d.as<line_pre_d>(), nullptr, nullptr);
  HIPCHK(c, hipGetLastError());
  {
    timed t_(c, HBX_K_VERIFY_SIG, s);
    hipLaunchKernelGGL(k_verify_sigs, dim3((count + 63) / 64), dim3(64), 0, s, c->vs_pk.as<uint8_t>(),
                       c->vs_lines_d.as<line_pre_d>(), c->vs_H.as<g2a>(), c->vs_sig.as<g2a>(), c->vs_sig_st.as<int32_t>(),
                       count, c->vs_status.as<uint8_t>());
  }
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(status, c->vs_status.p, count, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return HBX_OK;
}

// Decode p commitments of degree t and compute their rows at x (device state for the checks).
static int bivar_rows_impl(hbx_ctx* c, const uint8_t* commit48, uint32_t p, uint32_t t, uint64_t x, bool want48) {
  if (!c || !commit48 || p == 0 || t > 4095) return fail(c, HBX_E_INVALID_ARG, "hbx_bivar: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, c->stream);
  stream_scope ss_{c, s};
  const size_t M = (size_t)(t + 1) * (t + 2) / 2, nr = (size_t)p * (t + 1);
  if (!c->bv_commit48.ensure(p * M * 48) || !c->bv_C.ensure(p * M * sizeof(g1a)) || !c->bv_cst.ensure(p * M * 4) ||
      !c->bv_rows.ensure(nr * sizeof(g1j)) || !c->bv_rows48.ensure(nr * 48) || !c->bv_pst.ensure(p))
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_bivar: out of device memory");
  HIPCHK(c, hipMemcpyAsync(c->bv_commit48.p, commit48, p * M * 48, hipMemcpyHostToDevice, s));
  // decode = into_affine (curve + G1 membership), as a Part's commitment deserialises
  hipLaunchKernelGGL(k_decompress_shares, dim3((unsigned)((p * M + 255) / 256)), dim3(256), 0, s,
                     c->bv_commit48.as<uint8_t>(), p * M, c->bv_C.as<g1a>(), c->bv_cst.as<int32_t>(), 1u, UINT32_MAX,
                     nullptr);
  HIPCHK(c, hipGetLastError());
  hipLaunchKernelGGL(k_bivar_rows, dim3((unsigned)((nr + 63) / 64)), dim3(64), 0, s, c->bv_C.as<g1a>(),
                     c->bv_cst.as<int32_t>(), p, t, x, c->bv_rows.as<g1j>(), want48 ? c->bv_rows48.as<uint8_t>() : nullptr,
                     c->bv_pst.as<uint8_t>());
  HIPCHK(c, hipGetLastError());
  return HBX_OK;
}

int hbx_bivar_rows(hbx_ctx* c, const uint8_t* commit48, uint32_t p, uint32_t t, uint64_t x, uint8_t* rows48,
                   uint8_t* status) {
  if (!rows48 || !status) return fail(c, HBX_E_INVALID_ARG, "hbx_bivar_rows: null output");
  int rc = bivar_rows_impl(c, commit48, p, t, x, true);
  if (rc) return rc;
  hipStream_t s = pick(c, c->stream);
  stream_scope ss_{c, s};
  HIPCHK(c, hipMemcpyAsync(rows48, c->bv_rows48.p, (size_t)p * (t + 1) * 48, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipMemcpyAsync(status, c->bv_pst.p, p, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return HBX_OK;
}

int hbx_bivar_check_acks(hbx_ctx* c, const uint8_t* commit48, uint32_t p, uint32_t t, uint64_t x,
                         const uint32_t* ack_proposer, const uint64_t* ack_y, const uint8_t* vals32, uint32_t count,
                         uint8_t* status) {
  if (!ack_proposer || !ack_y || !vals32 || !status || count == 0)
    return fail(c, HBX_E_INVALID_ARG, "hbx_bivar_check_acks: bad args");
  for (uint32_t k = 0; k < count; k++)
    if (ack_proposer[k] >= p) return fail(c, HBX_E_INVALID_ARG, "hbx_bivar_check_acks: proposer %u >= p", ack_proposer[k]);
  int rc = bivar_rows_impl(c, commit48, p, t, x, false);
  if (rc) return rc;
  hipStream_t s = pick(c, c->stream);
  stream_scope ss_{c, s};
  if (!c->bv_ackp.ensure((size_t)count * 4) || !c->bv_acky.ensure((size_t)count * 8) ||
      !c->bv_vals.ensure((size_t)count * 32) || !c->bv_out.ensure(count))
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_bivar_check_acks: out of device memory");
  HIPCHK(c, hipMemcpyAsync(c->bv_ackp.p, ack_proposer, (size_t)count * 4, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(c->bv_acky.p, ack_y, (size_t)count * 8, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(c->bv_vals.p, vals32, (size_t)count * 32, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_bivar_check, dim3((count + 63) / 64), dim3(64), 0, s, c->bv_rows.as<g1j>(),
                     c->bv_pst.as<uint8_t>(), t, c->bv_ackp.as<uint32_t>(), c->bv_acky.as<uint64_t>(),
                     c->bv_vals.as<uint8_t>(), count, c->bv_out.as<uint8_t>());
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(status, c->bv_out.p, count, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return HBX_OK;
}

// combine_signatures + master check + parity of every prepared nonce over the valid shares of
// the last signature-share verification (masked by d_use [I][n] when given): results in
// coin_out96 / coin_comb_st / coin_ok / coin_par.
static int combine_sigs_impl(hbx_ctx* c, const uint8_t* master_pk48, uint32_t t, const uint8_t* d_use, hipStream_t s) {
  if (!master_pk48 || t == 0 || t > (uint32_t)COMBINE_MAX_T) return fail(c, HBX_E_INVALID_ARG, "hbx_combine_signatures: bad args");
  if (c->coin_n == 0) return fail(c, HBX_E_NO_CIPHERTEXTS, "no verified signature shares");
  const uint32_t I = c->coin_I;
  const size_t m = (size_t)I * c->coin_n;
  if (!c->coin_comb.ensure((size_t)I * sizeof(g2a)) || !c->coin_comb_st.ensure((size_t)I * 4) ||
      !c->coin_mpk_comp.ensure(48) || !c->coin_mpk.ensure(sizeof(g1a)) || !c->coin_mpk_st.ensure(4) ||
      !c->coin_ok.ensure(I) || !c->coin_par.ensure(I) || !c->coin_out96.ensure((size_t)I * 96) ||
      (d_use && !c->coin_use.ensure(m)))
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_combine_signatures: out of device memory");
  if (c->coin_ready_ev) HIPCHK(c, hipStreamWaitEvent(s, c->coin_ready_ev, 0));
  // the master key: decoded once per distinct value (era state; checked on the host)
  if (!c->coin_mpk_known || memcmp(c->coin_mpk48, master_pk48, 48) != 0) {
    HIPCHK(c, hipMemcpyAsync(c->coin_mpk_comp.p, master_pk48, 48, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_decompress_g1, dim3(1), dim3(64), 0, s, c->coin_mpk_comp.as<uint8_t>(), 1u, c->coin_mpk.as<g1a>(),
                       c->coin_mpk_st.as<int32_t>());
    HIPCHK(c, hipGetLastError());
    int32_t mst = 0;
    HIPCHK(c, hipMemcpyAsync(&mst, c->coin_mpk_st.p, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (mst != HBX_PT_OK) return fail(c, HBX_E_INVALID_ARG, "master public key does not decode (status %d)", mst);
    memcpy(c->coin_mpk48, master_pk48, 48);
    c->coin_mpk_known = true;
  }
  const uint8_t* valid = c->coin_valid.as<uint8_t>();
  if (d_use) {
    hipLaunchKernelGGL(k_coin_use, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, valid, d_use, m,
                       c->coin_use.as<uint8_t>());
    HIPCHK(c, hipGetLastError());
    valid = c->coin_use.as<uint8_t>();
  }
  {
    // the G2 combine (waves 0..2) and the master-key identity (wave 3), one block per instance
    timed t_(c, HBX_K_COMBINE_SIGS, s);
    hipLaunchKernelGGL(k_combine_sigs, dim3(I), dim3(SIGCOMB_THREADS), 0, s, valid, c->coin_sig.as<g2a>(), c->coin_n, t,
                       c->pk.as<g1a>(), c->pk64.as<g1a>(), c->coin_mpk.as<g1a>(), c->coin_comb.as<g2a>(),
                       c->coin_comb_st.as<int32_t>(), c->coin_ok.as<uint8_t>(),
                       c->g1tab.p ? c->g1tab.as<g1a>() : nullptr);
  }
  HIPCHK(c, hipGetLastError());
  hipLaunchKernelGGL(k_sig_parity, dim3((I + 63) / 64), dim3(64), 0, s, c->coin_comb.as<g2a>(), c->coin_comb_st.as<int32_t>(),
                     I, c->coin_par.as<uint8_t>(), c->coin_out96.as<uint8_t>());
  HIPCHK(c, hipGetLastError());
  return HBX_OK;
}

int hbx_combine_signatures(hbx_ctx* c, const uint8_t* master_pk48, uint32_t t, uint8_t* sig96, int32_t* status,
                           uint8_t* master_ok_bits, uint8_t* parity_bits) {
  if (!c) return HBX_E_INVALID_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, c->stream);
  stream_scope ss_{c, s};
  if (int rc = combine_sigs_impl(c, master_pk48, t, nullptr, s)) return rc;
  const uint32_t I = c->coin_I;
  std::vector<uint8_t> ok(I), par(I);
  std::vector<int32_t> st(I);
  if (sig96) HIPCHK(c, hipMemcpyAsync(sig96, c->coin_out96.p, (size_t)I * 96, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipMemcpyAsync(ok.data(), c->coin_ok.p, I, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipMemcpyAsync(par.data(), c->coin_par.p, I, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipMemcpyAsync(st.data(), c->coin_comb_st.p, (size_t)I * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  if (status) memcpy(status, st.data(), (size_t)I * 4);
  if (master_ok_bits) pack_bits(ok.data(), I, master_ok_bits);
  if (parity_bits) pack_bits(par.data(), I, parity_bits);
  return HBX_OK;
}

int hbx_combine_signatures_d(hbx_ctx* c, const uint8_t* master_pk48, uint32_t t, const uint8_t* d_use, uint8_t* d_sig96,
                             int32_t* d_status, uint8_t* d_master_ok, uint8_t* d_parity, void* stream) {
  if (!c) return HBX_E_INVALID_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  stream_scope ss_{c, s};
  if (int rc = combine_sigs_impl(c, master_pk48, t, d_use, s)) return rc;
  const uint32_t I = c->coin_I;
  if (d_sig96) HIPCHK(c, hipMemcpyAsync(d_sig96, c->coin_out96.p, (size_t)I * 96, hipMemcpyDeviceToDevice, s));
  if (d_status) HIPCHK(c, hipMemcpyAsync(d_status, c->coin_comb_st.p, (size_t)I * 4, hipMemcpyDeviceToDevice, s));
  if (d_master_ok) HIPCHK(c, hipMemcpyAsync(d_master_ok, c->coin_ok.p, I, hipMemcpyDeviceToDevice, s));
  if (d_parity) HIPCHK(c, hipMemcpyAsync(d_parity, c->coin_par.p, I, hipMemcpyDeviceToDevice, s));
  return HBX_OK;
}

int hbx_get_ct_valid_d(hbx_ctx* c, uint8_t* d_ct_valid, void* stream) {
  if (!c || !d_ct_valid) return fail(c, HBX_E_INVALID_ARG, "hbx_get_ct_valid_d: bad args");
  if (c->p_ct == 0 || !c->ct_known) return fail(c, HBX_E_NO_CIPHERTEXTS, "ciphertext validity not computed yet");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  stream_scope ss_{c, s};
  HIPCHK(c, hipMemcpyAsync(d_ct_valid, c->ct_valid.p, c->p_ct, hipMemcpyDeviceToDevice, s));
  return HBX_OK;
}

int hbx_combine_decrypt_d(hbx_ctx* c, uint32_t t, uint8_t* d_out_blob, int32_t* d_status, void* stream) {
  if (!c || t == 0 || t > (uint32_t)COMBINE_MAX_T || !d_out_blob)
    return fail(c, HBX_E_INVALID_ARG, "hbx_combine_decrypt_d: bad args");
  if (c->n_shares == 0 || c->p_ct == 0 || !c->ct_known || c->verified_p != c->p_ct)
    return fail(c, HBX_E_NO_CIPHERTEXTS, "no verified shares for the prepared ciphertexts");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  stream_scope ss_{c, s};
  const uint32_t p = c->p_ct;
  if (!c->keys.ensure((size_t)p * 32) || !c->status.ensure((size_t)p * 4))
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_combine_decrypt_d: out of device memory");
  {
    timed t_(c, HBX_K_COMBINE, s);
    // a quad of lanes per GLV term over one-wave blocks when that still leaves at most one wave per
    // SIMD (an epoch shard; k_combine_q), else one lane per term in one block per proposer
    const uint32_t nb = (2 * t + COMBQ_TERMS - 1) / COMBQ_TERMS;
    const bool quads = c->combine_lanes == 4 ? nb <= 16
                       : c->combine_lanes == 1 ? false
                                               : nb <= 16 && (size_t)nb * p <= (size_t)VERIFY_FILL_WAVES;
    if (quads) {
      if (!c->comb_partial.ensure((size_t)p * nb * sizeof(g1j)) || !c->comb_done.ensure((size_t)p * 4))
        return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_combine_decrypt_d: out of device memory");
      HIPCHK(c, hipMemsetAsync(c->comb_done.p, 0, (size_t)p * 4, s));
      hipLaunchKernelGGL(k_combine_q, dim3(nb, p), dim3(64), 0, s, c->valid.as<uint8_t>(), c->S.as<g1a>(),
                         c->n_shares, t, c->ct_valid.as<uint8_t>(), c->keys.as<uint32_t>(), c->status.as<int32_t>(),
                         c->digest, c->comb_partial.as<g1j>(), c->comb_done.as<uint32_t>());
    } else
    hipLaunchKernelGGL(k_combine, dim3(p), dim3(COMBINE_THREADS), 0, s, c->valid.as<uint8_t>(), c->S.as<g1a>(),
                       c->n_shares, t, c->ct_valid.as<uint8_t>(), c->keys.as<uint32_t>(), c->status.as<int32_t>(),
                       c->digest);
  }
  HIPCHK(c, hipGetLastError());
  const uint64_t blocks = (c->max_v_len + 15) / 16;
  if (blocks) {
    hipLaunchKernelGGL(k_keystream_xor, dim3((unsigned)((blocks + 63) / 64), p), dim3(64), 0, s,
                       c->keys.as<uint32_t>(), c->status.as<int32_t>(), c->d_v_blob, c->d_v_off, d_out_blob);
    HIPCHK(c, hipGetLastError());
  }
  if (d_status) HIPCHK(c, hipMemcpyAsync(d_status, c->status.p, (size_t)p * 4, hipMemcpyDeviceToDevice, s));
  return HBX_OK;
}

int hbx_decrypt_epoch_d(hbx_ctx* c, const uint8_t* d_u_comp, const uint8_t* d_v_blob, const uint64_t* d_v_off,
                        const uint8_t* d_w_comp, uint32_t p, uint64_t max_v_len, const uint8_t* d_shares,
                        const uint8_t* d_present, uint32_t n, uint32_t t, uint8_t* d_valid, uint8_t* d_ct_valid,
                        uint8_t* d_out_blob, int32_t* d_status, void* stream) {
  if (!c || !d_shares || n == 0 || p == 0 || t == 0 || t > (uint32_t)COMBINE_MAX_T || !d_out_blob)
    return fail(c, HBX_E_INVALID_ARG, "hbx_decrypt_epoch_d: bad args");
  if (c->n_keys == 0) return fail(c, HBX_E_NO_KEYS, "hbx_set_pk_shares has not been called");
  // Stages in stream order.  (Running Ciphertext::verify on the aux stream beside a speculative
  // combine was measured on MI355X and gained nothing: the combine's 4 waves per proposer already
  // occupy every SIMD, and two single-wave-per-SIMD kernels only time-share the VALU.)
  int rc = prepare_impl(c, d_u_comp, d_v_blob, d_v_off, d_w_comp, p, max_v_len, nullptr, stream, d_shares, n);
  if (rc) return rc;
  rc = verify_impl(c, d_shares, d_present, n, p, d_valid, stream, true);
  if (rc) return rc;
  if (d_ct_valid) {
    rc = hbx_get_ct_valid_d(c, d_ct_valid, stream);
    if (rc) return rc;
  }
  return hbx_combine_decrypt_d(c, t, d_out_blob, d_status, stream);
}

int hbx_combine_decrypt(hbx_ctx* c, uint32_t t, uint8_t* out_blob, int32_t* status) {
  if (!c || !out_blob) return fail(c, HBX_E_INVALID_ARG, "hbx_combine_decrypt: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  stream_scope ss_{c, pick(c, c->stream)};
  if (c->p_ct == 0) return fail(c, HBX_E_NO_CIPHERTEXTS, "no ciphertexts prepared");
  std::vector<uint64_t> off(c->p_ct + 1);
  HIPCHK(c, hipMemcpyAsync(off.data(), c->d_v_off, off.size() * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const uint64_t total = off[c->p_ct];
  if (!c->out_own.ensure(total ? total : 16)) return fail(c, HBX_E_OUT_OF_MEMORY, "out of device memory");
  HIPCHK(c, hipMemsetAsync(c->out_own.p, 0, total ? total : 16, c->stream));
  int rc = hbx_combine_decrypt_d(c, t, c->out_own.as<uint8_t>(), nullptr, c->stream);
  if (rc) return rc;
  if (total) HIPCHK(c, hipMemcpyAsync(out_blob, c->out_own.p, total, hipMemcpyDeviceToHost, c->stream));
  std::vector<int32_t> st(c->p_ct);
  HIPCHK(c, hipMemcpyAsync(st.data(), c->status.p, (size_t)c->p_ct * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (status) memcpy(status, st.data(), st.size() * 4);
  return HBX_OK;
}

// ---- status readout ---------------------------------------------------------------------------
static int copy_status(hbx_ctx* c, const dbuf& b, size_t have, uint8_t* out, size_t count, const char* what) {
  if (!out) return fail(c, HBX_E_INVALID_ARG, "%s: null output", what);
  if (have == 0) return fail(c, HBX_E_NO_CIPHERTEXTS, "%s: nothing computed yet", what);
  if (count != have) return fail(c, HBX_E_INVALID_ARG, "%s: count %zu, expected %zu", what, count, have);
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, quiesce(c));  // the last results may have been enqueued on a caller's stream
  HIPCHK(c, hipMemcpy(out, b.p, have, hipMemcpyDeviceToHost));
  return HBX_OK;
}

int hbx_get_share_status(hbx_ctx* c, uint8_t* status, size_t count) {
  if (!c) return HBX_E_INVALID_ARG;
  return copy_status(c, c->valid, (size_t)c->n_shares * c->verified_p, status, count, "hbx_get_share_status");
}

int hbx_get_ct_status(hbx_ctx* c, uint8_t* status, size_t count) {
  if (!c) return HBX_E_INVALID_ARG;
  return copy_status(c, c->ct_valid, c->ct_known ? c->p_ct : 0, status, count, "hbx_get_ct_status");
}

int hbx_get_ct_hashes(hbx_ctx* c, uint8_t* h96, size_t count) {
  if (!c || !h96) return fail(c, HBX_E_INVALID_ARG, "hbx_get_ct_hashes: bad args");
  if (c->p_ct == 0) return fail(c, HBX_E_NO_CIPHERTEXTS, "hbx_get_ct_hashes: no ciphertexts prepared");
  if (count != c->p_ct) return fail(c, HBX_E_INVALID_ARG, "hbx_get_ct_hashes: count %zu, expected %u", count, c->p_ct);
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, quiesce(c));
  dbuf out;
  if (!out.ensure(count * 96)) return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_get_ct_hashes: out of device memory");
  // Hj holds H' = h_eff P = [3(x^2-1)] H (k_prepare_ct); the reference's H = h2 P from it
  hipLaunchKernelGGL(k_true_hashes, dim3((unsigned)((count + 63) / 64)), dim3(64), 0, c->stream, c->G2pts.as<g2a>(),
                     c->Hj.as<g2j>(), (uint32_t)count, out.as<uint8_t>());
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess) e = hipMemcpy(h96, out.p, count * 96, hipMemcpyDeviceToHost);
  out.release();
  if (e != hipSuccess) return fail(c, HBX_E_DEVICE, "hbx_get_ct_hashes: %s", hipGetErrorString(e));
  return HBX_OK;
}

int hbx_get_sig_share_status(hbx_ctx* c, uint8_t* status, size_t count) {
  if (!c) return HBX_E_INVALID_ARG;
  return copy_status(c, c->coin_valid, (size_t)c->coin_n * c->coin_I, status, count, "hbx_get_sig_share_status");
}

// ---- producer side --------------------------------------------------------------------------
static bool scalars_canonical(const uint8_t* s32, size_t count) {
  static const uint8_t R_BE[32] = {0x73, 0xed, 0xa7, 0x53, 0x29, 0x9d, 0x7d, 0x48, 0x33, 0x39, 0xd8,
                                   0x08, 0x09, 0xa1, 0xd8, 0x05, 0x53, 0xbd, 0xa4, 0x02, 0xff, 0xfe,
                                   0x5b, 0xfe, 0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x01};
  for (size_t k = 0; k < count; k++)
    if (memcmp(s32 + 32 * k, R_BE, 32) >= 0) return false;
  return true;
}

int hbx_public_keys(hbx_ctx* c, const uint8_t* sk32, uint32_t n, uint8_t* pk48) {
  if (!c || !sk32 || !pk48 || n == 0) return fail(c, HBX_E_INVALID_ARG, "hbx_public_keys: bad args");
  if (!scalars_canonical(sk32, n)) return fail(c, HBX_E_INVALID_ARG, "hbx_public_keys: scalar >= r");
  HIPCHK(c, hipSetDevice(c->device));
  stream_scope ss_{c, pick(c, c->stream)};
  dbuf dsk, dpk;
  if (!dsk.ensure((size_t)n * 32) || !dpk.ensure((size_t)n * 48)) {
    dsk.release();
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_public_keys: out of device memory");
  }
  int rc = HBX_OK;
  if (hipMemcpyAsync(dsk.p, sk32, (size_t)n * 32, hipMemcpyHostToDevice, c->stream) != hipSuccess) rc = HBX_E_DEVICE;
  if (rc == HBX_OK) {
    hipLaunchKernelGGL(k_public_keys, dim3((n + 63) / 64), dim3(64), 0, c->stream, dsk.as<uint8_t>(), n,
                       dpk.as<uint8_t>());
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(pk48, dpk.p, (size_t)n * 48, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
      rc = HBX_E_DEVICE;
  }
  dsk.release();
  dpk.release();
  return rc ? fail(c, rc, "hbx_public_keys: device error") : HBX_OK;
}

int hbx_encrypt(hbx_ctx* c, const uint8_t* pk48, const uint8_t* msg_blob, const uint64_t* msg_off, uint32_t p,
                const uint8_t* r32, uint8_t* u48, uint8_t* v_blob, uint8_t* w96) {
  if (!c || !pk48 || !msg_off || !r32 || !u48 || !w96 || p == 0)
    return fail(c, HBX_E_INVALID_ARG, "hbx_encrypt: bad args");
  if (!scalars_canonical(r32, p)) return fail(c, HBX_E_INVALID_ARG, "hbx_encrypt: scalar >= r");
  for (uint32_t j = 0; j < p; j++)
    if (msg_off[j + 1] < msg_off[j]) return fail(c, HBX_E_INVALID_ARG, "hbx_encrypt: msg_off not monotone");
  const uint64_t total = msg_off[p];
  if (total && (!msg_blob || !v_blob)) return fail(c, HBX_E_INVALID_ARG, "hbx_encrypt: bad args");
  HIPCHK(c, hipSetDevice(c->device));
  stream_scope ss_{c, pick(c, c->stream)};
  dbuf dpkc, dpk, dst, dr, dm, doff, du, dv, dw;
  dbuf* all[] = {&dpkc, &dpk, &dst, &dr, &dm, &doff, &du, &dv, &dw};
  auto cleanup = [&]() { for (dbuf* b : all) b->release(); };
  if (!dpkc.ensure(48) || !dpk.ensure(sizeof(g1a)) || !dst.ensure(4) || !dr.ensure((size_t)p * 32) ||
      !dm.ensure(total) || !doff.ensure((size_t)(p + 1) * 8) || !du.ensure((size_t)p * 48) || !dv.ensure(total) ||
      !dw.ensure((size_t)p * 96)) {
    cleanup();
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_encrypt: out of device memory");
  }
  int rc = HBX_OK;
  int32_t st = 0;
  bool ok = hipMemcpyAsync(dpkc.p, pk48, 48, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
            hipMemcpyAsync(dr.p, r32, (size_t)p * 32, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
            hipMemcpyAsync(doff.p, msg_off, (size_t)(p + 1) * 8, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
            (total == 0 || hipMemcpyAsync(dm.p, msg_blob, total, hipMemcpyHostToDevice, c->stream) == hipSuccess);
  if (ok) {
    hipLaunchKernelGGL(k_decompress_g1, dim3(1), dim3(64), 0, c->stream, dpkc.as<uint8_t>(), 1u, dpk.as<g1a>(),
                       dst.as<int32_t>());
    ok = hipGetLastError() == hipSuccess &&
         hipMemcpyAsync(&st, dst.p, 4, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
         hipStreamSynchronize(c->stream) == hipSuccess;
  }
  if (ok && st != HBX_PT_OK) {
    cleanup();
    return fail(c, HBX_E_INVALID_ARG, "hbx_encrypt: public key does not decode (status %d)", st);
  }
  if (ok) {
    hipLaunchKernelGGL(k_encrypt, dim3((p + 63) / 64), dim3(64), 0, c->stream, dpk.as<g1a>(), dr.as<uint8_t>(),
                       dm.as<uint8_t>(), doff.as<uint64_t>(), p, du.as<uint8_t>(), dv.as<uint8_t>(), dw.as<uint8_t>(),
                       c->digest);
    ok = hipGetLastError() == hipSuccess &&
         hipMemcpyAsync(u48, du.p, (size_t)p * 48, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
         hipMemcpyAsync(w96, dw.p, (size_t)p * 96, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
         (total == 0 || hipMemcpyAsync(v_blob, dv.p, total, hipMemcpyDeviceToHost, c->stream) == hipSuccess) &&
         hipStreamSynchronize(c->stream) == hipSuccess;
  }
  if (!ok) rc = HBX_E_DEVICE;
  cleanup();
  return rc ? fail(c, rc, "hbx_encrypt: device error") : HBX_OK;
}

int hbx_decrypt_shares(hbx_ctx* c, const uint8_t* sk32, uint32_t n, const uint8_t* u48, uint32_t p,
                       uint8_t* shares48) {
  if (!c || !sk32 || !u48 || !shares48 || n == 0 || p == 0)
    return fail(c, HBX_E_INVALID_ARG, "hbx_decrypt_shares: bad args");
  if (!scalars_canonical(sk32, n)) return fail(c, HBX_E_INVALID_ARG, "hbx_decrypt_shares: scalar >= r");
  HIPCHK(c, hipSetDevice(c->device));
  stream_scope ss_{c, pick(c, c->stream)};
  const size_t m = (size_t)n * p;
  dbuf dsk, duc, du, dst, dout;
  dbuf* all[] = {&dsk, &duc, &du, &dst, &dout};
  auto cleanup = [&]() { for (dbuf* b : all) b->release(); };
  if (!dsk.ensure((size_t)n * 32) || !duc.ensure((size_t)p * 48) || !du.ensure((size_t)p * sizeof(g1a)) ||
      !dst.ensure((size_t)p * 4) || !dout.ensure(m * 48)) {
    cleanup();
    return fail(c, HBX_E_OUT_OF_MEMORY, "hbx_decrypt_shares: out of device memory");
  }
  std::vector<int32_t> st(p);
  bool ok = hipMemcpyAsync(dsk.p, sk32, (size_t)n * 32, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
            hipMemcpyAsync(duc.p, u48, (size_t)p * 48, hipMemcpyHostToDevice, c->stream) == hipSuccess;
  if (ok) {
    hipLaunchKernelGGL(k_decompress_g1, dim3((p + 63) / 64), dim3(64), 0, c->stream, duc.as<uint8_t>(), p,
                       du.as<g1a>(), dst.as<int32_t>());
    ok = hipGetLastError() == hipSuccess &&
         hipMemcpyAsync(st.data(), dst.p, (size_t)p * 4, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
         hipStreamSynchronize(c->stream) == hipSuccess;
  }
  for (uint32_t j = 0; ok && j < p; j++)
    if (st[j] != HBX_PT_OK && st[j] != HBX_PT_INFINITY) {
      cleanup();
      return fail(c, HBX_E_INVALID_ARG, "hbx_decrypt_shares: U_%u does not decode (status %d)", j, st[j]);
    }
  if (ok) {
    hipLaunchKernelGGL(k_decrypt_shares, dim3((n + 63) / 64, p), dim3(64), 0, c->stream, dsk.as<uint8_t>(), n,
                       du.as<g1a>(), dout.as<uint8_t>());
    ok = hipGetLastError() == hipSuccess &&
         hipMemcpyAsync(shares48, dout.p, m * 48, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
         hipStreamSynchronize(c->stream) == hipSuccess;
  }
  cleanup();
  return ok ? HBX_OK : fail(c, HBX_E_DEVICE, "hbx_decrypt_shares: device error");
}

}  // extern "C"

int hbx_set_timing(hbx_ctx* c, int on) {
  if (!c) return HBX_E_INVALID_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  timing_reset(c);
  c->timing = on != 0;
  return HBX_OK;
}

int hbx_kernel_time(hbx_ctx* c, int kernel, double* total_ms, uint32_t* launches) {
  if (!c || kernel < 0 || kernel >= HBX_K_COUNT || !total_ms) return fail(c, HBX_E_INVALID_ARG, "hbx_kernel_time: bad argument");
  HIPCHK(c, hipSetDevice(c->device));
  double tot = 0;
  for (auto& pr : c->tev[kernel]) {
    HIPCHK(c, hipEventSynchronize(pr.second));
    float ms = 0;
    HIPCHK(c, hipEventElapsedTime(&ms, pr.first, pr.second));
    tot += ms;
  }
  *total_ms = tot;
  if (launches) *launches = (uint32_t)c->tev[kernel].size();
  return HBX_OK;
}
#endif  // host translation unit
