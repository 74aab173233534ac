// Broadcast byte path on gfx950: Reed-Solomon
// GF(2^8) coding as reed-solomon-erasure 3.1.0 defines it and the SHA-256 Merkle tree of the
// afck/merkle.rs fork (or the opt-in SHA3-256 tree of later hbbft), for whole batches of
// broadcast instances (reference src/broadcast.rs).
//
// HBM layout: one instance = n shards of L bytes, contiguous ([inst][n][L]); leaf i of an
// instance is the index byte i followed by shard i (broadcast.rs:373-377), never materialised.
// All of it is byte/integer work: the roofline is HBM bandwidth for RS (k reads + m writes per
// column) and the integer VALU for SHA-256 (64 rounds per 64-byte block); no MFMA.
#pragma once
#include "hash.hpp"
#include "dpp.hpp"
#ifndef HBX_IN_TU
#define HBX_IN_TU(n) 1  // single-TU build (hbx_kernels.hip defines the split)
#endif

namespace hbx {

// ---------------------------------------------------------------------------------------------
// GF(2^8): tables built on the host (hbx_api.hip) and staged in LDS.  log[0] = 512 (sentinel);
// exp has 768 entries, zero from index 510 on, so exp[log a + log c] is a*c for every byte a and
// nonzero coefficient c (zero coefficients are skipped: log = 0xFFFF).
// ---------------------------------------------------------------------------------------------
constexpr uint16_t GF_LOG_ZERO = 512;
constexpr uint16_t GF_COEF_ZERO = 0xFFFF;
constexpr int RS_OUT_CHUNK = 16;
constexpr int RS_MAX_K = 128;
constexpr int RS_MAX_N = 256;

struct gf_tab {
  uint16_t lg[256];
  uint8_t ex[768];
};

__device__ __forceinline__ void gf_stage(gf_tab& T, const uint16_t* glog, const uint8_t* gexp) {
  for (int i = threadIdx.x; i < 256; i += blockDim.x) T.lg[i] = glog[i];
  for (int i = threadIdx.x; i < 768; i += blockDim.x) T.ex[i] = gexp[i];
}

__device__ __forceinline__ uint8_t gf_mul(const gf_tab& T, uint8_t a, uint8_t b) {
  return (a == 0 || b == 0) ? 0 : T.ex[T.lg[a] + T.lg[b]];
}

// Per-instance coding job: out rows = XOR_c coef[o][c] * in rows c  (byte columns).
struct rs_job {
  int32_t n_out;
  int32_t in_idx[RS_MAX_K];
  int32_t out_idx[RS_MAX_N];
};

// grid (ceil(L / (4 * 256)), inst); thread = 4 consecutive byte columns of one instance.
// coef: [inst][RS_MAX_N][k] logs (GF_COEF_ZERO for 0).  Coefficient reads are wave-uniform.
// job_stride = 0: every instance runs job 0 (encode); 1: per-instance jobs (reconstruct).
#if HBX_IN_TU(6)
__global__ void __launch_bounds__(256) k_rs_code(uint8_t* __restrict__ shards, size_t inst_stride, uint32_t L,
                                                 uint32_t k, const rs_job* __restrict__ jobs,
                                                 const uint16_t* __restrict__ coef, uint32_t job_stride,
                                                 const uint16_t* __restrict__ glog, const uint8_t* __restrict__ gexp) {
  __shared__ gf_tab T;
  gf_stage(T, glog, gexp);
  __syncthreads();
  const uint32_t inst = blockIdx.y;
  const rs_job& J = jobs[inst * job_stride];
  const int no = J.n_out;
  const uint32_t col = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (no == 0 || col >= L) return;
  uint8_t* base = shards + (size_t)inst * inst_stride;
  const uint16_t* cl = coef + (size_t)inst * job_stride * RS_MAX_N * k;
  const uint32_t nb = L - col < 4 ? L - col : 4;
  for (int o0 = 0; o0 < no; o0 += RS_OUT_CHUNK) {
    uint32_t acc[RS_OUT_CHUNK];
#pragma unroll
    for (int o = 0; o < RS_OUT_CHUNK; o++) acc[o] = 0;
    for (uint32_t c = 0; c < k; c++) {
      const uint8_t* src = base + (size_t)J.in_idx[c] * L + col;
      uint32_t lg4[4];
      if (nb == 4 && ((uintptr_t)src & 3) == 0) {
        const uint32_t d = *reinterpret_cast<const uint32_t*>(src);
#pragma unroll
        for (int q = 0; q < 4; q++) lg4[q] = T.lg[(d >> (8 * q)) & 0xFF];
      } else {
#pragma unroll
        for (int q = 0; q < 4; q++) lg4[q] = (uint32_t)q < nb ? T.lg[src[q]] : GF_LOG_ZERO;
      }
#pragma unroll
      for (int o = 0; o < RS_OUT_CHUNK; o++) {
        if (o0 + o < no) {
          const uint32_t lc = cl[(o0 + o) * k + c];
          if (lc != GF_COEF_ZERO)
            acc[o] ^= (uint32_t)T.ex[lg4[0] + lc] | ((uint32_t)T.ex[lg4[1] + lc] << 8) |
                      ((uint32_t)T.ex[lg4[2] + lc] << 16) | ((uint32_t)T.ex[lg4[3] + lc] << 24);
        }
      }
    }
#pragma unroll
    for (int o = 0; o < RS_OUT_CHUNK; o++) {
      if (o0 + o < no) {
        uint8_t* dst = base + (size_t)J.out_idx[o0 + o] * L + col;
        if (nb == 4 && ((uintptr_t)dst & 3) == 0) {
          *reinterpret_cast<uint32_t*>(dst) = acc[o];
        } else {
          for (uint32_t q = 0; q < nb; q++) dst[q] = (uint8_t)(acc[o] >> (8 * q));
        }
      }
    }
  }
}
#endif

// ---------------------------------------------------------------------------------------------
// GF(2^8) coding by byte permutes.  Multiplication by a fixed coefficient c is GF(2)-linear, so
// c * d = c * (d & 0x07) ^ c * (d & 0x38) ^ c * (d & 0xC0): three lookups in tables of 8, 8 and 4
// bytes, and an 8-byte table is exactly what one v_perm_b32 selects from (selector bytes 0..7
// over two dwords) -- for four packed data bytes at once.  Per (output, input) coefficient and
// data dword: 3 perms and 1.5 xors (v_xor3), no LDS, no per-byte work.  The 32-byte table of a
// coefficient is wave-uniform (one s_load_dwordx8); the two 8-byte tables need VGPR copies
// (one constant-bus operand per VALU op), which D data dwords per lane share.  The selector
// words depend on the data only and are computed once per input dword.
// tables: u32[jobs][RS_MAX_N][k][8] = {T0 lo, T0 hi, T1 lo, T1 hi, T2, 0, 0, 0}, T0[i] = c*i,
// T1[i] = c*(i << 3) (i < 8), T2[i] = c*(i << 6) (i < 4).
// ---------------------------------------------------------------------------------------------
struct alignas(32) gf_ptab {
  uint32_t w[8];
};

// Perm tables for per-instance jobs (reconstruct): one lane per coefficient of jobs[inst]
// (logs in coef, GF_COEF_ZERO = 0).  grid (ceil(RS_MAX_N * k / 256), inst).
#if HBX_IN_TU(6)
__global__ void __launch_bounds__(256) k_rs_perm_tables(const rs_job* __restrict__ jobs, const uint16_t* __restrict__ coef,
                                                        uint32_t k, const uint16_t* __restrict__ glog,
                                                        const uint8_t* __restrict__ gexp, gf_ptab* __restrict__ tables) {
  __shared__ gf_tab T;
  gf_stage(T, glog, gexp);
  __syncthreads();
  const uint32_t inst = blockIdx.y;
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t no = (uint32_t)jobs[inst].n_out;
  if (e >= no * k) return;
  const uint16_t lc = coef[(size_t)inst * RS_MAX_N * k + e];
  uint8_t b[20];
  for (int i = 0; i < 8; i++) {
    b[i] = lc == GF_COEF_ZERO || i == 0 ? 0 : T.ex[T.lg[i] + lc];
    b[8 + i] = lc == GF_COEF_ZERO || i == 0 ? 0 : T.ex[T.lg[i << 3] + lc];
  }
  for (int i = 0; i < 4; i++) b[16 + i] = lc == GF_COEF_ZERO || i == 0 ? 0 : T.ex[T.lg[i << 6] + lc];
  gf_ptab t;
  for (int w = 0; w < 5; w++)
    t.w[w] = (uint32_t)b[4 * w] | ((uint32_t)b[4 * w + 1] << 8) | ((uint32_t)b[4 * w + 2] << 16) |
             ((uint32_t)b[4 * w + 3] << 24);
  t.w[5] = t.w[6] = t.w[7] = 0;
  tables[(size_t)inst * RS_MAX_N * k + e] = t;
}
#endif

// 3-input XOR in one VALU op (gfx950 v_bitop3_b32, truth table 0x96).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// out rows = XOR_c coef[o][c] * in rows c, byte columns; needs L % 4 == 0 (dword rows).  A wave
// covers 64 * D consecutive dwords of every row (lane l: dwords l, l + 64, ...) and accumulates
// CH output rows per pass over the inputs, two inputs per step so the 6 lookups of a step fold
// into the accumulator with 3 v_bitop3 (4.5 VALU ops per coefficient and data dword).  The
// pass's tables are staged in LDS ([c][o]: T0/T1 as one 16-byte entry, T2 packed 4 per entry;
// wave-uniform broadcast reads); outputs past n_out get zero tables and are not stored, inputs
// are read one step ahead of use.  grid (ceil(L / (4 * 256 * D)), inst), dynamic LDS
// rs_perm_lds_bytes(k, CH); job_stride as k_rs_code (0: job 0 / tables[0] for all instances).
__host__ __device__ constexpr size_t rs_perm_lds_bytes(uint32_t k, int ch) {
  return (size_t)((k + 1) & ~1u) * ch * 20;
}

#ifndef HBX_RS_LOADS
#define HBX_RS_LOADS 0  // 1: branch-free clamped loads (r06s: 0.474 vs 0.467 ms on encode, kept off)
#endif
#if HBX_IN_TU(6)
template <int CH, int D>
__global__ void __launch_bounds__(256) k_rs_code_perm(uint8_t* __restrict__ shards, size_t inst_stride, uint32_t L,
                                                      uint32_t k, const rs_job* __restrict__ jobs,
                                                      const gf_ptab* __restrict__ tables, uint32_t job_stride) {
  static_assert(CH % 4 == 0, "T2 entries are packed four per 16 bytes");
  extern __shared__ uint4 rs_lds[];
  const uint32_t kp = (k + 1) & ~1u;
  uint4* tab01 = rs_lds;                 // [kp][CH]
  uint4* tab2 = rs_lds + (size_t)kp * CH;  // [kp][CH / 4]
  const uint32_t inst = blockIdx.y;
  const rs_job* J = jobs + (size_t)inst * job_stride;
  const int no = ld_uniform(&J->n_out);
  if (no == 0) return;
  const uint32_t Ld = L >> 2;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 64 * D;
  uint32_t* base = reinterpret_cast<uint32_t*>(shards + (size_t)inst * inst_stride);
  const gf_ptab* tb = tables + (size_t)inst * job_stride * RS_MAX_N * k;
  bool ok[D];
#pragma unroll
  for (int j = 0; j < D; j++) ok[j] = wave0 + lane + 64 * j < Ld;
#if HBX_RS_LOADS
  // Branch-free loads: lanes past the row end read its last dword and inputs past k (the odd
  // k's pad row) re-read row k - 1 -- their results are not stored / their tables are zero.
  uint32_t off[D];
#pragma unroll
  for (int j = 0; j < D; j++) off[j] = min(wave0 + lane + 64 * j, Ld - 1);
  auto load_in = [&](uint32_t c, uint32_t* d) {
    const uint32_t* src = base + (size_t)ld_uniform(&J->in_idx[c < k ? c : k - 1]) * Ld;
#pragma unroll
    for (int j = 0; j < D; j++) d[j] = src[off[j]];
  };
#else
  auto load_in = [&](uint32_t c, uint32_t* d) {
    if (c < k) {
      const uint32_t* src = base + (size_t)ld_uniform(&J->in_idx[c]) * Ld + wave0 + lane;
#pragma unroll
      for (int j = 0; j < D; j++) d[j] = ok[j] ? src[64 * j] : 0u;
    } else {
#pragma unroll
      for (int j = 0; j < D; j++) d[j] = 0u;
    }
  };
#endif
  // passes of CH outputs spread over grid.z (host: ceil(expected outputs / CH)); more outputs
  // than the grid covers loop here
  for (int o0 = blockIdx.z * CH; o0 < no; o0 += gridDim.z * CH) {
    __syncthreads();  // previous pass done with the tables
    for (uint32_t e = threadIdx.x; e < kp * CH; e += blockDim.x) {
      const uint32_t c = e / CH, o = e % CH;
      gf_ptab t{};
      if (c < k && o0 + (int)o < no) t = tb[(size_t)(o0 + o) * k + c];
      tab01[e] = make_uint4(t.w[0], t.w[1], t.w[2], t.w[3]);
      reinterpret_cast<uint32_t*>(tab2)[e] = t.w[4];
    }
    __syncthreads();
    uint32_t acc[CH][D];
#pragma unroll
    for (int o = 0; o < CH; o++)
#pragma unroll
      for (int j = 0; j < D; j++) acc[o][j] = 0;
    uint32_t na[D], nb[D];
    load_in(0, na);
    load_in(1, nb);
#pragma unroll 1
    for (uint32_t c = 0; c < kp; c += 2) {
      uint32_t a0[D], a1[D], a2[D], b0[D], b1[D], b2[D];
#pragma unroll
      for (int j = 0; j < D; j++) {
        a0[j] = na[j] & 0x07070707u;
        a1[j] = (na[j] >> 3) & 0x07070707u;
        a2[j] = (na[j] >> 6) & 0x03030303u;
        b0[j] = nb[j] & 0x07070707u;
        b1[j] = (nb[j] >> 3) & 0x07070707u;
        b2[j] = (nb[j] >> 6) & 0x03030303u;
      }
      load_in(c + 2, na);
      load_in(c + 3, nb);
      const uint4* ta = tab01 + (size_t)c * CH;
      const uint4* tc = tab2 + (size_t)c * (CH / 4);
#pragma unroll
      for (int o4 = 0; o4 < CH; o4 += 4) {
        const uint4 t2a = tc[o4 / 4], t2b = tc[CH / 4 + o4 / 4];
        const uint32_t t2av[4] = {t2a.x, t2a.y, t2a.z, t2a.w}, t2bv[4] = {t2b.x, t2b.y, t2b.z, t2b.w};
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int o = o4 + q;
          const uint4 A = ta[o], B = ta[CH + o];
#pragma unroll
          for (int j = 0; j < D; j++) {
            uint32_t x = xor3(acc[o][j], __builtin_amdgcn_perm(A.y, A.x, a0[j]), __builtin_amdgcn_perm(A.w, A.z, a1[j]));
            x = xor3(x, __builtin_amdgcn_perm(0u, t2av[q], a2[j]), __builtin_amdgcn_perm(B.y, B.x, b0[j]));
            acc[o][j] = xor3(x, __builtin_amdgcn_perm(B.w, B.z, b1[j]), __builtin_amdgcn_perm(0u, t2bv[q], b2[j]));
          }
        }
      }
    }
#pragma unroll
    for (int o = 0; o < CH; o++) {
      if (o0 + o < no) {
        uint32_t* dst = base + (size_t)ld_uniform(&J->out_idx[o0 + o]) * Ld + wave0 + lane;
#pragma unroll
        for (int j = 0; j < D; j++)
          if (ok[j]) dst[64 * j] = acc[o][j];
      }
    }
  }
}
#endif

// The same product over input TRIPLES: a byte's 8 bits split 3 + 3 + 2, and the two 2-bit tops
// of a triple's three inputs (6 bits) are regrouped as two 3-bit lookups into mixed 8-entry
// tables -- M1[a7 a6 | b6] = c_a (a_top << 6) ^ c_b (b6 << 6), M2[b7 | c7 c6] = c_b (b7 << 7) ^
// c_c (c_top << 6) -- so a triple costs 8 v_perm + 4 v_bitop3 per output dword: 4.0 VALU ops per
// coefficient and data dword against the pair kernel's 4.5 (which spends 3 perms on every
// byte).  LDS per pass: [triple][CH] x 64 B ({T0,T1} of a, b, c; {M1, M2}), staged from the
// per-coefficient gf_ptab tables; inputs past k (pad of the last triple) have zero tables.
__host__ __device__ constexpr size_t rs_perm3_lds_bytes(uint32_t k, int ch) {
  return (size_t)((k + 2) / 3) * ch * 64;
}

#if HBX_IN_TU(6)
#ifndef HBX_RS3_WPE
#define HBX_RS3_WPE 1  // tuning: minimum waves per EU of the triple kernel (__launch_bounds__'s second bound)
#endif
template <int CH, int D>
__global__ void __launch_bounds__(256, HBX_RS3_WPE) k_rs_code_perm3(uint8_t* __restrict__ shards, size_t inst_stride, uint32_t L,
                                                       uint32_t k, const rs_job* __restrict__ jobs,
                                                       const gf_ptab* __restrict__ tables, uint32_t job_stride) {
  extern __shared__ uint4 rs_lds[];
  const uint32_t nt = (k + 2) / 3;
  const uint32_t inst = blockIdx.y;
  const rs_job* J = jobs + (size_t)inst * job_stride;
  const int no = ld_uniform(&J->n_out);
  if (no == 0) return;
  const uint32_t Ld = L >> 2;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 64 * D;
  uint32_t* base = reinterpret_cast<uint32_t*>(shards + (size_t)inst * inst_stride);
  const gf_ptab* tb = tables + (size_t)inst * job_stride * RS_MAX_N * k;
  bool ok[D];
#pragma unroll
  for (int j = 0; j < D; j++) ok[j] = wave0 + lane + 64 * j < Ld;
  auto load_in = [&](uint32_t c, uint32_t* d) {
    if (c < k) {
      const uint32_t* src = base + (size_t)ld_uniform(&J->in_idx[c]) * Ld + wave0 + lane;
#pragma unroll
      for (int j = 0; j < D; j++) d[j] = ok[j] ? src[64 * j] : 0u;
    } else {
#pragma unroll
      for (int j = 0; j < D; j++) d[j] = 0u;
    }
  };
  auto tbyte = [](uint32_t w, int i) { return (w >> (8 * i)) & 0xffu; };
  // passes of CH outputs spread over grid.z (host: ceil(expected outputs / CH)); more outputs
  // than the grid covers loop here
  for (int o0 = blockIdx.z * CH; o0 < no; o0 += gridDim.z * CH) {
    __syncthreads();  // previous pass done with the tables
    for (uint32_t e = threadIdx.x; e < nt * CH; e += blockDim.x) {
      const uint32_t t = e / CH, o = e % CH;
      gf_ptab g[3];
#pragma unroll
      for (int i = 0; i < 3; i++) {
        const uint32_t c = 3 * t + i;
        g[i] = gf_ptab{};
        if (c < k && o0 + (int)o < no) g[i] = tb[(size_t)(o0 + o) * k + c];
      }
      // T2 (w[4]) byte i = c * (i << 6): byte 1 = c * 0x40, byte 2 = c * 0x80
      uint32_t m1[2] = {0, 0}, m2[2] = {0, 0};
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const uint32_t v1 = tbyte(g[0].w[4], j & 3) ^ ((j & 4) ? tbyte(g[1].w[4], 1) : 0u);
        const uint32_t v2 = ((j & 1) ? tbyte(g[1].w[4], 2) : 0u) ^ tbyte(g[2].w[4], j >> 1);
        m1[j >> 2] |= v1 << (8 * (j & 3));
        m2[j >> 2] |= v2 << (8 * (j & 3));
      }
      uint4* dst = rs_lds + (size_t)e * 4;
      dst[0] = make_uint4(g[0].w[0], g[0].w[1], g[0].w[2], g[0].w[3]);
      dst[1] = make_uint4(g[1].w[0], g[1].w[1], g[1].w[2], g[1].w[3]);
      dst[2] = make_uint4(g[2].w[0], g[2].w[1], g[2].w[2], g[2].w[3]);
      dst[3] = make_uint4(m1[0], m1[1], m2[0], m2[1]);
    }
    __syncthreads();
    if (wave0 >= Ld) continue;  // a wave wholly past the row end only stages tables (uniform)
    uint32_t acc[CH][D];
#pragma unroll
    for (int o = 0; o < CH; o++)
#pragma unroll
      for (int j = 0; j < D; j++) acc[o][j] = 0;
    uint32_t na[D], nb[D], nc[D];
    load_in(0, na);
    load_in(1, nb);
    load_in(2, nc);
#pragma unroll 1
    for (uint32_t t = 0; t < nt; t++) {
      uint32_t a0[D], a1[D], b0[D], b1[D], c0[D], c1[D], s1[D], s2[D];
#pragma unroll
      for (int j = 0; j < D; j++) {
        a0[j] = na[j] & 0x07070707u;
        a1[j] = (na[j] >> 3) & 0x07070707u;
        b0[j] = nb[j] & 0x07070707u;
        b1[j] = (nb[j] >> 3) & 0x07070707u;
        c0[j] = nc[j] & 0x07070707u;
        c1[j] = (nc[j] >> 3) & 0x07070707u;
        s1[j] = ((na[j] >> 6) & 0x03030303u) | ((nb[j] >> 4) & 0x04040404u);
        s2[j] = ((nb[j] >> 7) & 0x01010101u) | ((nc[j] >> 5) & 0x06060606u);
      }
      load_in(3 * t + 3, na);
      load_in(3 * t + 4, nb);
      load_in(3 * t + 5, nc);
      const uint4* tp = rs_lds + (size_t)t * CH * 4;
#pragma unroll
      for (int o = 0; o < CH; o++) {
        const uint4 A = tp[4 * o], B = tp[4 * o + 1], C = tp[4 * o + 2], M = tp[4 * o + 3];
#pragma unroll
        for (int j = 0; j < D; j++) {
          uint32_t x = xor3(acc[o][j], __builtin_amdgcn_perm(A.y, A.x, a0[j]), __builtin_amdgcn_perm(A.w, A.z, a1[j]));
          x = xor3(x, __builtin_amdgcn_perm(B.y, B.x, b0[j]), __builtin_amdgcn_perm(B.w, B.z, b1[j]));
          x = xor3(x, __builtin_amdgcn_perm(C.y, C.x, c0[j]), __builtin_amdgcn_perm(C.w, C.z, c1[j]));
          acc[o][j] = xor3(x, __builtin_amdgcn_perm(M.y, M.x, s1[j]), __builtin_amdgcn_perm(M.w, M.z, s2[j]));
        }
      }
    }
#pragma unroll
    for (int o = 0; o < CH; o++) {
      if (o0 + o < no) {
        uint32_t* dst = base + (size_t)ld_uniform(&J->out_idx[o0 + o]) * Ld + wave0 + lane;
#pragma unroll
        for (int j = 0; j < D; j++)
          if (ok[j]) dst[64 * j] = acc[o][j];
      }
    }
  }
}
#endif
#if defined(HBX_TU) && HBX_TU == 6
// the tiles rs_code() (hbx_api.hip) launches, instantiated in this translation unit
#define HBX_RS_INST(ch, d)                                                                                   \
  template __global__ void k_rs_code_perm<ch, d>(uint8_t* __restrict__, size_t, uint32_t, uint32_t,            \
                                                  const rs_job* __restrict__, const gf_ptab* __restrict__, uint32_t);
HBX_RS_INST(32, 2)
HBX_RS_INST(32, 4)
HBX_RS_INST(64, 2)
HBX_RS_INST(24, 4)
HBX_RS_INST(48, 2)
HBX_RS_INST(28, 2)
HBX_RS_INST(28, 4)
HBX_RS_INST(44, 2)
#undef HBX_RS_INST
#define HBX_RS_INST3(ch, d)                                                                                  \
  template __global__ void k_rs_code_perm3<ch, d>(uint8_t* __restrict__, size_t, uint32_t, uint32_t,           \
                                                   const rs_job* __restrict__, const gf_ptab* __restrict__, uint32_t);
HBX_RS_INST3(12, 2)
HBX_RS_INST3(14, 2)
HBX_RS_INST3(21, 2)
HBX_RS_INST3(28, 2)
HBX_RS_INST3(42, 2)
#undef HBX_RS_INST3
#endif

// reconstruct_shards set-up, one block per instance (reed-solomon-erasure 3.1.0):
// first k present shards -> invert that k x k sub-matrix of the encoding matrix (Gauss-Jordan in
// LDS) -> job 0: rebuild missing data shards from the k sub shards; job 1: re-encode missing
// parity shards from the (then complete) data shards.  status: 0, or HBX_E_TOO_FEW_SHARDS.
#if HBX_IN_TU(6)
__global__ void __launch_bounds__(256) k_rs_setup_reconstruct(const uint8_t* __restrict__ present, uint32_t k,
                                                              uint32_t m, const uint8_t* __restrict__ enc,
                                                              const uint16_t* __restrict__ glog,
                                                              const uint8_t* __restrict__ gexp,
                                                              rs_job* __restrict__ jobs_data,
                                                              uint16_t* __restrict__ coef_data,
                                                              rs_job* __restrict__ jobs_par,
                                                              uint16_t* __restrict__ coef_par,
                                                              int32_t* __restrict__ status) {
  __shared__ gf_tab T;
  __shared__ uint8_t A[RS_MAX_K][2 * RS_MAX_K];
  __shared__ int32_t sub[RS_MAX_K];
  __shared__ int32_t s_count, s_nmd, s_nmp, s_swap;
  __shared__ int32_t missing_data[RS_MAX_K], missing_par[RS_MAX_N];
  __shared__ uint8_t factor[RS_MAX_K];
  __shared__ int32_t wcnt[4][3];
  gf_stage(T, glog, gexp);
  const uint32_t inst = blockIdx.x;
  const uint32_t n = k + m;
  const uint8_t* pr = present + (size_t)inst * n;
  const int tid = threadIdx.x;
  // classification by ballots (n <= RS_MAX_N = blockDim): the rank of each shard among the
  // present / missing-data / missing-parity ones, in index order
  const uint32_t lane = tid & 63, wv = tid >> 6;
  const bool in = (uint32_t)tid < n, p = in && pr[tid] != 0;
  const bool md = in && !p && (uint32_t)tid < k, mp = in && !p && (uint32_t)tid >= k;
  const uint64_t bp = __ballot(p), bd = __ballot(md), bm = __ballot(mp);
  const uint64_t below = (1ull << lane) - 1;
  if (lane == 0) {
    wcnt[wv][0] = __popcll(bp);
    wcnt[wv][1] = __popcll(bd);
    wcnt[wv][2] = __popcll(bm);
  }
  __syncthreads();
  int op = 0, od = 0, om = 0;
  for (uint32_t w = 0; w < wv; w++) op += wcnt[w][0], od += wcnt[w][1], om += wcnt[w][2];
  if (p && op + __popcll(bp & below) < (int)k) sub[op + __popcll(bp & below)] = tid;
  if (md) missing_data[od + __popcll(bd & below)] = tid;
  if (mp) missing_par[om + __popcll(bm & below)] = tid;
  if (tid == 0) {
    s_count = wcnt[0][0] + wcnt[1][0] + wcnt[2][0] + wcnt[3][0];
    s_nmd = wcnt[0][1] + wcnt[1][1] + wcnt[2][1] + wcnt[3][1];
    s_nmp = wcnt[0][2] + wcnt[1][2] + wcnt[2][2] + wcnt[3][2];
  }
  __syncthreads();
  rs_job& JD = jobs_data[inst];
  rs_job& JP = jobs_par[inst];
  if (s_count < (int)k || s_count == (int)n) {
    if (tid == 0) {
      JD.n_out = 0;
      JP.n_out = 0;
      status[inst] = s_count < (int)k ? -9 : 0;
    }
    return;
  }
  // The sub-matrix of the first k present rows is [[I, 0], [E_p, E_m]] with the present data
  // shards first (sub[0, npd)) and the first nmd present parity shards after them, columns as
  // (present data D_p, missing data D_m).  Only its rows for D_m are needed:
  //   x_m = E_m^-1 y_s + (E_m^-1 E_p) x_p,
  // so Gauss-Jordan runs on the nmd x nmd block E_m (nmd = missing data shards; none when only
  // parity is missing) instead of the whole k x k matrix -- the same unique coefficients.
  const int nmd = s_nmd, npd = (int)k - nmd;
  if (nmd > 0) {
    for (uint32_t e = tid; e < (uint32_t)(nmd * 2 * nmd); e += blockDim.x) {  // [E_m | I]
      const int r = (int)e / (2 * nmd), c = (int)e % (2 * nmd);
      A[r][c] = c < nmd ? enc[(size_t)sub[npd + r] * k + missing_data[c]] : (c - nmd == r ? 1 : 0);
    }
    __syncthreads();
    for (int r = 0; r < nmd; r++) {
      if (tid == 0) {
        s_swap = -1;
        if (A[r][r] == 0)
          for (int b2 = r + 1; b2 < nmd; b2++)
            if (A[b2][r]) {
              s_swap = b2;
              break;
            }
      }
      __syncthreads();
      if (s_swap >= 0)
        for (int c = tid; c < 2 * nmd; c += blockDim.x) {
          const uint8_t t = A[r][c];
          A[r][c] = A[s_swap][c];
          A[s_swap][c] = t;
        }
      __syncthreads();
      const uint8_t piv = A[r][r];
      const uint8_t inv = piv ? T.ex[255 - T.lg[piv]] : 0;  // MDS: E_m is invertible
      __syncthreads();
      for (int c = tid; c < 2 * nmd; c += blockDim.x) A[r][c] = gf_mul(T, A[r][c], inv);
      for (int i = tid; i < nmd; i += blockDim.x) factor[i] = A[i][r];
      __syncthreads();
      for (uint32_t e = tid; e < (uint32_t)(nmd * 2 * nmd); e += blockDim.x) {
        const int i = (int)e / (2 * nmd), c = (int)e % (2 * nmd);
        if (i != r && factor[i]) A[i][c] ^= gf_mul(T, factor[i], A[r][c]);
      }
      __syncthreads();
    }
  }
  // job 0: missing data rows from the k sub shards
  if (tid == 0) {
    JD.n_out = s_nmd;
    JP.n_out = s_nmp;
    status[inst] = 0;
  }
  for (uint32_t c = tid; c < k; c += blockDim.x) {
    JD.in_idx[c] = sub[c];
    JP.in_idx[c] = (int32_t)c;
  }
  for (int o = tid; o < s_nmd; o += blockDim.x) JD.out_idx[o] = missing_data[o];
  for (int o = tid; o < s_nmp; o += blockDim.x) JP.out_idx[o] = missing_par[o];
  uint16_t* cd = coef_data + (size_t)inst * RS_MAX_N * k;
  for (uint32_t e = tid; e < (uint32_t)s_nmd * k; e += blockDim.x) {
    const int o = (int)(e / k), c = (int)(e % k);
    uint8_t v;
    if (c >= npd) {
      v = A[o][nmd + (c - npd)];  // E_m^-1 on the present parity shards
    } else {                      // (E_m^-1 E_p) on the present data shards
      v = 0;
      for (int r = 0; r < nmd; r++) v ^= gf_mul(T, A[o][nmd + r], enc[(size_t)sub[npd + r] * k + sub[c]]);
    }
    cd[o * k + c] = v ? T.lg[v] : GF_COEF_ZERO;
  }
  uint16_t* cp = coef_par + (size_t)inst * RS_MAX_N * k;
  for (uint32_t e = tid; e < (uint32_t)s_nmp * k; e += blockDim.x) {
    const uint32_t o = e / k, c = e % k;
    const uint8_t v = enc[(size_t)missing_par[o] * k + c];
    cp[o * k + c] = v ? T.lg[v] : GF_COEF_ZERO;
  }
}
#endif

// ---------------------------------------------------------------------------------------------
// SHA-256 of (prefix bytes) || data[len]: one lane per message; the bulk of the data is read as
// aligned dwords and realigned with v_alignbyte (leaves start at an index-byte offset).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ uint8_t msg_byte(uint32_t prefix, int plen, const uint8_t* data, uint64_t len, uint64_t q) {
  if (q < (uint64_t)plen) return (uint8_t)(prefix >> (8 * q));
  q -= plen;
  return q < len ? data[q] : 0;
}

__device__ void sha256_prefixed(uint32_t prefix, int plen, const uint8_t* data, uint64_t len, uint32_t* h8) {
  sha256_state s;
  sha256_init(s);
  const uint64_t total = (uint64_t)plen + len;
  const uint64_t nblocks = (total + 9 + 63) / 64;
  for (uint64_t blk = 0; blk < nblocks; blk++) {
    uint32_t w[16];
    const uint64_t b0 = blk * 64;
    if (b0 >= (uint64_t)plen && b0 + 64 <= total) {
      // fast path: the whole block is data; 17 aligned dwords cover it
      const uint8_t* p = data + (b0 - plen);
      const uintptr_t a = (uintptr_t)p;
      const uint32_t* pa = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
      const uint32_t sh = (uint32_t)(a & 3);
      uint32_t d[17];
      const int nd = sh ? 17 : 16;
#pragma unroll
      for (int i = 0; i < 17; i++) d[i] = i < nd ? pa[i] : 0;
#pragma unroll
      for (int i = 0; i < 16; i++) w[i] = bswap32(__builtin_amdgcn_alignbyte(d[i + 1], d[i], sh));
    } else {
#pragma unroll 1
      for (int i = 0; i < 16; i++) {
        uint32_t word = 0;
        for (int q = 0; q < 4; q++) {
          const uint64_t pos = b0 + 4 * i + q;
          uint8_t byte;
          if (pos < total) byte = msg_byte(prefix, plen, data, len, pos);
          else if (pos == total) byte = 0x80;
          else if (pos >= nblocks * 64 - 8) byte = (uint8_t)((total * 8) >> (8 * (nblocks * 64 - 1 - pos)));
          else byte = 0;
          word = (word << 8) | byte;
        }
        w[i] = word;
      }
    }
    sha256_compress(s, w);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) h8[i] = s.h[i];
}

// SHA3-256 of (prefix bytes) || data[len] (the SHA3 Merkle variant's leaf: SHA3(index byte ||
// shard)), one lane; full 136-byte blocks of data are read as aligned dwords realigned with
// v_alignbyte (little-endian lanes, no byte swap).  Digest as 8 big-endian words like
// sha256_prefixed, so both variants share the tree and output code.
__device__ void sha3_prefixed(uint32_t prefix, int plen, const uint8_t* data, uint64_t len, uint32_t* h8) {
  uint64_t st[25];
#pragma unroll
  for (int i = 0; i < 25; i++) st[i] = 0;
  const uint64_t total = (uint64_t)plen + len;
  const uint64_t nblocks = total / 136 + 1;
  for (uint64_t blk = 0; blk < nblocks; blk++) {
    const uint64_t b0 = blk * 136;
    if (b0 >= (uint64_t)plen && b0 + 136 <= total) {
      const uint8_t* q = data + (b0 - plen);
      const uintptr_t a = (uintptr_t)q;
      const uint32_t* pa = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
      const uint32_t sh = (uint32_t)(a & 3);
      uint32_t d[35];
      const int nd = sh ? 35 : 34;
#pragma unroll
      for (int i = 0; i < 35; i++) d[i] = i < nd ? pa[i] : 0;
#pragma unroll
      for (int i = 0; i < 17; i++) {
        const uint32_t lo = __builtin_amdgcn_alignbyte(d[2 * i + 1], d[2 * i], sh);
        const uint32_t hi = __builtin_amdgcn_alignbyte(d[2 * i + 2], d[2 * i + 1], sh);
        st[i] ^= (uint64_t)lo | ((uint64_t)hi << 32);
      }
    } else {
#pragma unroll 1
      for (int i = 0; i < 17; i++) {
        uint64_t lane = 0;
        for (int k = 0; k < 8; k++) {
          const uint64_t pos = b0 + 8 * i + k;
          uint8_t byte = pos < total ? msg_byte(prefix, plen, data, len, pos) : 0;
          if (pos == total) byte ^= 0x06;
          if (blk == nblocks - 1 && 8 * i + k == 135) byte ^= 0x80;
          lane |= (uint64_t)byte << (8 * k);
        }
        st[i] ^= lane;
      }
    }
    keccak_f1600(st);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) h8[i] = bswap32((uint32_t)(st[i >> 1] >> (32 * (i & 1))));
}

// node = SHA-256(0x01 || left || right) on big-endian word digests (2 blocks)
__device__ void sha256_node(const uint32_t* l8, const uint32_t* r8, uint32_t* out8) {
  sha256_state s;
  sha256_init(s);
  uint32_t w[16];
  // bytes: 01 | L(32) | R(32) | 80 | zeros | len=65*8
  w[0] = 0x01000000u | (l8[0] >> 8);
#pragma unroll
  for (int i = 1; i < 8; i++) w[i] = (l8[i - 1] << 24) | (l8[i] >> 8);
  w[8] = (l8[7] << 24) | (r8[0] >> 8);
#pragma unroll
  for (int i = 9; i < 16; i++) w[i] = (r8[i - 9] << 24) | (r8[i - 8] >> 8);
  sha256_compress_il(s, w);
  w[0] = (r8[7] << 24) | 0x00800000u;
#pragma unroll
  for (int i = 1; i < 15; i++) w[i] = 0;
  w[15] = 65 * 8;
  sha256_compress_il(s, w);
#pragma unroll
  for (int i = 0; i < 8; i++) out8[i] = s.h[i];
}

// node = SHA3-256(left || right) (the SHA3 Merkle variant: no domain prefixes)
__device__ void sha3_node(const uint32_t* l8, const uint32_t* r8, uint32_t* out8) {
  uint64_t st[25];
#pragma unroll
  for (int i = 0; i < 25; i++) st[i] = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    st[i] = (uint64_t)bswap32(l8[2 * i]) | ((uint64_t)bswap32(l8[2 * i + 1]) << 32);
    st[4 + i] = (uint64_t)bswap32(r8[2 * i]) | ((uint64_t)bswap32(r8[2 * i + 1]) << 32);
  }
  st[8] = 0x06;                      // padding right after the 64 message bytes
  st[16] = 0x8000000000000000ull;    // last byte of the 136-byte block
  keccak_f1600(st);
#pragma unroll
  for (int i = 0; i < 8; i++) out8[i] = bswap32((uint32_t)(st[i >> 1] >> (32 * (i & 1))));
}

// Merkle digests by variant (include/hbx.h HBX_MERKLE_*):
//   HBX_MERKLE_SHA256  merkle (afck fork) + ring: leaf SHA-256(0x00 || v), node SHA-256(0x01 || l || r)
//   HBX_MERKLE_SHA3    later hbbft's merkle.rs:  leaf SHA3-256(v),         node SHA3-256(l || r)
// Leaves of the broadcast are index-prefixed shards: v = [i as u8] || shard_i (broadcast.rs:373-377).
constexpr int MERKLE_SHA256 = 0;
constexpr int MERKLE_SHA3 = 1;
__device__ __forceinline__ void merkle_leaf_value(int variant, const uint8_t* v, uint64_t len, uint32_t* h) {
  if (variant == MERKLE_SHA3) sha3_prefixed(0, 0, v, len, h);
  else sha256_prefixed(0, 1, v, len, h);
}
__device__ __forceinline__ void merkle_node(int variant, const uint32_t* l8, const uint32_t* r8, uint32_t* out8) {
  if (variant == MERKLE_SHA3) sha3_node(l8, r8, out8);
  else sha256_node(l8, r8, out8);
}

// Leaf hashes of the index-prefixed shards: leaf(i) = H_leaf([i] || shard_i), out u32[inst][n][8]
// (digest words, big-endian order), by k_merkle_leaves_sha256 / k_merkle_leaves_sha3.  With
// `slots` (u16[inst][nslots], MERKLE_NO_SLOT = unused) only the listed leaves are hashed: the
// decode of validated Echo values hashes only the shards it reconstructed (the others' digests
// come from the Echo proofs, k_import_leaf_hashes).  With `row` != 0 the rows are proof values
// of `row` bytes (hbx_merkle_validate_d): leaf i hashes the whole value, its first byte in the
// prefix position and the other L = row - 1 bytes as the data.
constexpr uint32_t MERKLE_NO_SLOT = 0xFFFFu;

// SHA-256 Merkle leaves (HBX_MERKLE_SHA256), two waves per 64 leaves of one instance:
//  * wave 1 (producer) loads each leaf's next 64-byte block, expands the message schedule and
//    writes K[t] + W[t] for t < 64 to LDS, one block ahead of the consumer, with the raw words of
//    the block after that already in flight (register prefetch);
//  * wave 0 (consumer) runs only the 64 rounds from LDS: the serial chain of a leaf -- the
//    bound of this kernel, since a C5 epoch has just n x inst = 16,384 independent leaves of 373
//    blocks each -- carries no global loads, no schedule and no scratch round trips.
// leaf = SHA-256(0x00 || i || shard_i) (merkle.rs with ring).
// grid (ceil(n / 64), inst), 128 threads.
__device__ __forceinline__ uint32_t sha_sig(uint32_t x, int r1, int r2, int r3) {
  return xor3(rotr32(x, r1), rotr32(x, r2), rotr32(x, r3));
}

#if HBX_IN_TU(6)
__global__ void __launch_bounds__(128) k_merkle_leaves_sha256(const uint8_t* __restrict__ shards, size_t inst_stride,
                                                              uint32_t n, uint32_t L, uint32_t* __restrict__ leaf_hash,
                                                              const uint16_t* __restrict__ slots, uint32_t nslots,
                                                              uint32_t row) {
  __shared__ uint4 kw[2][16][64];  // [slot][rounds / 4][lane]
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t inst = blockIdx.y;
  uint32_t i = blockIdx.x * 64 + lane;
  if (slots) i = i < nslots ? slots[(size_t)inst * nslots + i] : MERKLE_NO_SLOT;
  const bool live = i < n;
  // a block with no leaf to hash (all its slots unused) leaves at once, both waves together
  if (!__syncthreads_or(live ? 1 : 0)) return;
  const uint8_t* data = shards + (size_t)inst * inst_stride + (size_t)(live ? i : 0) * (row ? row : L);
  // bytes 0x00, i -- or, for proof values (row != 0: rows of `row` bytes, the data after their
  // first byte), 0x00, value[0]
  const uint32_t prefix = (row ? (live ? (uint32_t)data[-1] : 0u) : (i & 0xFF)) << 8;
  const uint64_t total = 2 + (uint64_t)L;
  const uint64_t nblocks = (total + 9 + 63) / 64;
  // producer state: raw dwords of the next block (fast blocks: whole 64 bytes of shard data)
  uint32_t raw[17];
  auto fast = [&](uint64_t b) { return b * 64 >= 2 && b * 64 + 64 <= total; };
  auto fetch = [&](uint64_t b) {
    if (b < nblocks && fast(b)) {
      const uint8_t* q = data + (b * 64 - 2);
      const uint32_t* pa = reinterpret_cast<const uint32_t*>((uintptr_t)q & ~(uintptr_t)3);
#pragma unroll
      for (int k = 0; k < 16; k++) raw[k] = pa[k];
      // a misaligned block needs a 17th dword (it holds block bytes, so it is inside the buffer)
      raw[16] = ((uintptr_t)q & 3) ? pa[16] : 0u;
    }
  };
  auto produce = [&](uint64_t b, int slot) {
    uint32_t w[16];
    if (fast(b)) {
      const uint32_t sh = (uint32_t)(((uintptr_t)data + b * 64 - 2) & 3);
#pragma unroll
      for (int k = 0; k < 16; k++) w[k] = bswap32(__builtin_amdgcn_alignbyte(raw[k + 1], raw[k], sh));
    } else {
      const uint64_t b0 = b * 64;
#pragma unroll 1
      for (int k = 0; k < 16; k++) {
        uint32_t word = 0;
        for (int q = 0; q < 4; q++) {
          const uint64_t pos = b0 + 4 * k + q;
          uint8_t byte;
          if (pos < total) byte = msg_byte(prefix, 2, data, L, pos);
          else if (pos == total) byte = 0x80;
          else if (pos >= nblocks * 64 - 8) byte = (uint8_t)((total * 8) >> (8 * (nblocks * 64 - 1 - pos)));
          else byte = 0;
          word = (word << 8) | byte;
        }
        w[k] = word;
      }
    }
    fetch(b + 1);  // next block's raw words load while this schedule is expanded
#pragma unroll
    for (int t4 = 0; t4 < 16; t4++) {
      uint32_t o[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int t = 4 * t4 + q;
        uint32_t wt;
        if (t < 16) {
          wt = w[t];
        } else {
          const uint32_t w15 = w[(t + 1) & 15], w2 = w[(t + 14) & 15];
          const uint32_t s0 = xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
          const uint32_t s1 = xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
          wt = w[t & 15] + s0 + w[(t + 9) & 15] + s1;
          w[t & 15] = wt;
        }
        o[q] = wt + SHA256_K[t];
      }
      kw[slot][t4][lane] = make_uint4(o[0], o[1], o[2], o[3]);
    }
  };
  uint32_t H[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  if (wave == 1) {
    fetch(0);
    produce(0, 0);
  }
  __syncthreads();
  for (uint64_t b = 0; b < nblocks; b++) {
    const int slot = (int)(b & 1);
    if (wave == 0) {
      uint32_t a = H[0], bb = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma unroll
      for (int t4 = 0; t4 < 16; t4++) {
        const uint4 k4 = kw[slot][t4][lane];
        const uint32_t kv[4] = {k4.x, k4.y, k4.z, k4.w};
#pragma unroll
        for (int q = 0; q < 4; q++) {
          // Ch and Maj as one v_bitop3 each (truth tables 0xCA: e ? f : g, 0xE8: majority); the
          // compiler's own Maj took three ops (14 VALU per round instead of 16)
          const uint32_t t1 = h + kv[q] + sha_sig(e, 6, 11, 25) + __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
          const uint32_t t2 = sha_sig(a, 2, 13, 22) + __builtin_amdgcn_bitop3_b32(a, bb, c, 0xE8);
          h = g; g = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + t2;
        }
      }
      H[0] += a; H[1] += bb; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
    } else if (b + 1 < nblocks) {
      produce(b + 1, slot ^ 1);
    }
    __syncthreads();
  }
  if (wave == 0 && live) {
    uint32_t* o = leaf_hash + ((size_t)inst * n + i) * 8;
#pragma unroll
    for (int q = 0; q < 8; q++) o[q] = H[q];
  }
}
#endif

// Leaf digests handed in by the caller (the Echo proofs' leaf hashes, bytes as on the wire) for
// every present shard: leaf_hash[inst][i] = BE words of given[inst][i] where present[inst][i].
#if HBX_IN_TU(6)
__global__ void k_import_leaf_hashes(const uint8_t* __restrict__ given, const uint8_t* __restrict__ present,
                                     uint32_t total, uint32_t* __restrict__ leaf_hash) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;  // one digest word
  if (e >= total * 8 || !present[e / 8]) return;
  const uint8_t* p = given + (size_t)e * 4;
  leaf_hash[e] = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// The leaves a decode must hash: slots[inst][0..nslots) = the absent shard indices in order, the
// rest MERKLE_NO_SLOT; none for an instance whose status is already an error (too few shards).
// One wave per instance (ballot compaction in 64-leaf steps).
__global__ void __launch_bounds__(64) k_missing_slots(const uint8_t* __restrict__ present, uint32_t n,
                                                      const int32_t* __restrict__ status, uint32_t nslots,
                                                      uint16_t* __restrict__ slots) {
  const uint32_t inst = blockIdx.x, lane = threadIdx.x;
  uint16_t* out = slots + (size_t)inst * nslots;
  uint32_t filled = 0;
  if (status[inst] == 0) {
    for (uint32_t b = 0; b < n; b += 64) {
      const uint32_t i = b + lane;
      const bool miss = i < n && !present[(size_t)inst * n + i];
      const uint64_t mask = __ballot(miss);
      const uint32_t pos = filled + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
      if (miss && pos < nslots) out[pos] = (uint16_t)i;
      filled += (uint32_t)__popcll(mask);
    }
  }
  for (uint32_t q = filled + lane; q < nslots; q += 64) out[q] = (uint16_t)MERKLE_NO_SLOT;
}
#endif

// SHA3 Merkle leaves (HBX_MERKLE_SHA3), TWO lanes per leaf, bit-interleaved Keccak-f[1600]: the
// lane pair (2m, 2m + 1) holds the even bits (lane 2m) and the odd bits (lane 2m + 1) of all 25
// state words as 32-bit halves (the classic 32-bit technique).  A 64-bit rotation by 2k is a 32-bit
// rotation by k of both halves; by 2k + 1 it swaps the halves between the lanes (one DPP quad
// permutation) with rotations by k + 1 (even) and k (odd).  pi, chi and iota are half-local, so a
// round costs a lane ~115 VALU ops against ~190 for a whole-word round, and a C5 epoch's 16,384
// leaves fill 512 waves instead of 256 (the one-lane kernel left three SIMDs of four idle).
// leaf = SHA3-256([i] || shard_i), as sha3_prefixed computes it on one lane (k_merkle_validate).
// grid (ceil(n / 32), inst) [or ceil(nslots / 32) with slots], 64 threads.
#if HBX_IN_TU(6)
__device__ __forceinline__ uint32_t k_xchg(uint32_t v) {  // quad_perm [1, 0, 3, 2]: the pair partner
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t rotl32c(uint32_t x, uint32_t k) { return __builtin_amdgcn_alignbit(x, x, (32u - k) & 31u); }
__device__ __forceinline__ uint32_t even16(uint32_t x) {  // bits 0, 2, .., 30 -> bits 0..15
  x &= 0x55555555u;
  x = (x | (x >> 1)) & 0x33333333u;
  x = (x | (x >> 2)) & 0x0F0F0F0Fu;
  x = (x | (x >> 4)) & 0x00FF00FFu;
  return (x | (x >> 8)) & 0x0000FFFFu;
}
__device__ __forceinline__ uint32_t spread16(uint32_t x) {  // bits 0..15 -> bits 0, 2, .., 30
  x &= 0xFFFFu;
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x = (x | (x << 2)) & 0x33333333u;
  return (x | (x << 1)) & 0x55555555u;
}
// this lane's half of the 64-bit word (lo, hi): h = 0 the even bits, h = 1 the odd bits
__device__ __forceinline__ uint32_t ileave_half(uint32_t lo, uint32_t hi, uint32_t h) {
  return even16(lo >> h) | (even16(hi >> h) << 16);
}
constexpr uint32_t rc_half(uint64_t rc, int h) {
  uint32_t r = 0;
  for (int b = 0; b < 32; b++) r |= (uint32_t)((rc >> (2 * b + h)) & 1u) << b;
  return r;
}
struct keccak_rc_halves {
  uint32_t e[24], o[24];
  constexpr keccak_rc_halves() : e(), o() {
    constexpr uint64_t RC[24] = {
        0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
        0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
        0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
        0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
        0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
        0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
    for (int r = 0; r < 24; r++) {
      e[r] = rc_half(RC[r], 0);
      o[r] = rc_half(RC[r], 1);
    }
  }
};
// Keccak-f[1600] on this lane's halves a[5 y + x]; both lanes of every active pair active (the
// swaps are DPP moves: dpp.hpp), checked once per permutation
__device__ __forceinline__ void keccak_f1600_il(uint32_t* a, uint32_t h) {
  constexpr keccak_rc_halves RCH{};
  dpp_guard_pairs();
  constexpr int RHO[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
#pragma unroll
  for (int r = 0; r < 24; r++) {
    uint32_t c[5], rc1[5], b[25];
#pragma unroll
    for (int x = 0; x < 5; x++) c[x] = xor3(xor3(a[x], a[x + 5], a[x + 10]), a[x + 15], a[x + 20]);
    // rotl64(C, 1): the even half is the odd half rotated by 1, the odd half is the even half
#pragma unroll
    for (int x = 0; x < 5; x++) {
      const uint32_t p = k_xchg(c[x]);
      rc1[x] = __builtin_amdgcn_alignbit(p, p, 31u + h);  // rotl by 1 - h
    }
#pragma unroll
    for (int x = 0; x < 5; x++)  // a ^= D[x] = C[x - 1] ^ rotl(C[x + 1], 1), one v_bitop3 per word
#pragma unroll
      for (int y = 0; y < 5; y++) a[5 * y + x] = xor3(a[5 * y + x], c[(x + 4) % 5], rc1[(x + 1) % 5]);
    // rho + pi: b[pi(i)] = rotl64(a[i], RHO[i])
#pragma unroll
    for (int x = 0; x < 5; x++)
#pragma unroll
      for (int y = 0; y < 5; y++) {
        const int i = 5 * y + x, rho = RHO[i], k = rho >> 1;
        uint32_t v;
        if ((rho & 1) == 0) {
          v = rotl32c(a[i], (uint32_t)k);
        } else {
          const uint32_t p = k_xchg(a[i]);
          v = __builtin_amdgcn_alignbit(p, p, (uint32_t)(31 - k) + h);  // rotl by k + 1 - h
        }
        b[5 * ((2 * x + 3 * y) % 5) + y] = v;
      }
#pragma unroll
    for (int y = 0; y < 5; y++)
#pragma unroll
      for (int x = 0; x < 5; x++) a[5 * y + x] = b[5 * y + x] ^ (~b[5 * y + (x + 1) % 5] & b[5 * y + (x + 2) % 5]);
    a[0] ^= h ? RCH.o[r] : RCH.e[r];
  }
}

__global__ void __launch_bounds__(64) k_merkle_leaves_sha3(const uint8_t* __restrict__ shards, size_t inst_stride,
                                                           uint32_t n, uint32_t L, uint32_t* __restrict__ leaf_hash,
                                                           const uint16_t* __restrict__ slots, uint32_t nslots,
                                                           uint32_t row) {
  const uint32_t inst = blockIdx.y, lane = threadIdx.x, h = lane & 1u;
  uint32_t i = blockIdx.x * 32 + (lane >> 1);
  if (slots) i = i < nslots ? slots[(size_t)inst * nslots + i] : MERKLE_NO_SLOT;
  if (i >= n) return;  // whole pairs
  const uint8_t* data = shards + (size_t)inst * inst_stride + (size_t)i * (row ? row : L);
  const uint32_t prefix = row ? (uint32_t)data[-1] : (i & 0xFF);  // the index byte / value[0] (plen = 1)
  const uint64_t total = 1 + (uint64_t)L;
  const uint64_t nblocks = total / 136 + 1;
  uint32_t a[25];
#pragma unroll
  for (int q = 0; q < 25; q++) a[q] = 0;
  for (uint64_t blk = 0; blk < nblocks; blk++) {
    const uint64_t b0 = blk * 136;
    if (b0 >= 1 && b0 + 136 <= total) {
      const uint8_t* q = data + (b0 - 1);
      const uintptr_t ad = (uintptr_t)q;
      const uint32_t* pa = reinterpret_cast<const uint32_t*>(ad & ~(uintptr_t)3);
      const uint32_t sh = (uint32_t)(ad & 3);
      uint32_t d[35];
#pragma unroll
      for (int k = 0; k < 34; k++) d[k] = pa[k];
      d[34] = sh ? pa[34] : 0u;
#pragma unroll
      for (int w = 0; w < 17; w++) {
        const uint32_t lo = __builtin_amdgcn_alignbyte(d[2 * w + 1], d[2 * w], sh);
        const uint32_t hi = __builtin_amdgcn_alignbyte(d[2 * w + 2], d[2 * w + 1], sh);
        a[w] ^= ileave_half(lo, hi, h);
      }
    } else {
#pragma unroll 1
      for (int w = 0; w < 17; w++) {
        uint32_t lo = 0, hi = 0;
        for (int k = 0; k < 8; k++) {
          const uint64_t pos = b0 + 8 * w + k;
          uint8_t byte = pos < total ? msg_byte(prefix, 1, data, L, pos) : 0;
          if (pos == total) byte ^= 0x06;
          if (blk == nblocks - 1 && 8 * w + k == 135) byte ^= 0x80;
          if (k < 4) lo |= (uint32_t)byte << (8 * k);
          else hi |= (uint32_t)byte << (8 * (k - 4));
        }
        a[w] ^= ileave_half(lo, hi, h);
      }
    }
    keccak_f1600_il(a, h);
  }
  // digest bytes 0..31 = state words 0..3, little-endian; out as 8 big-endian words
  uint32_t out[8];
  dpp_guard_pairs();
#pragma unroll
  for (int w = 0; w < 4; w++) {
    const uint32_t mine = a[w], other = k_xchg(a[w]);
    const uint32_t e = h ? other : mine, o = h ? mine : other;
    const uint32_t lo = spread16(e) | (spread16(o) << 1);
    const uint32_t hi = spread16(e >> 16) | (spread16(o >> 16) << 1);
    out[2 * w] = bswap32(lo);
    out[2 * w + 1] = bswap32(hi);
  }
  if (h == 0) {
    uint32_t* o = leaf_hash + ((size_t)inst * n + i) * 8;
#pragma unroll
    for (int q = 0; q < 8; q++) o[q] = out[q];
  }
}
#endif

// Number of stored tree nodes for n leaves: every level from the leaves (n) to the root (1),
// with a promoted odd node stored again on the level it moves to.
__host__ __device__ inline uint32_t merkle_node_count(uint32_t n) {
  uint32_t total = 0, c = n;
  while (true) {
    total += c;
    if (c <= 1) break;
    c = (c + 1) / 2;
  }
  return total;
}

// MerkleTree::from_vec levels (pairs left to right, odd trailing node promoted): one block per
// instance, the level in LDS.  roots: u8[inst][32]; nodes (optional): u8[inst][node_count][32],
// level-major from the leaf level up, the root last (the `(2n - 1) x 32` tree of SURVEY.md
// §8(b) hbx_merkle_build, plus the promoted copies).
#if HBX_IN_TU(6)
__global__ void __launch_bounds__(128) k_merkle_tree(const uint32_t* __restrict__ leaf_hash, uint32_t n,
                                                     uint8_t* __restrict__ roots, uint8_t* __restrict__ nodes,
                                                     int variant) {
  __shared__ uint32_t lvl[2][RS_MAX_N][8];
  const uint32_t inst = blockIdx.x;
  for (uint32_t e = threadIdx.x; e < n * 8; e += blockDim.x) lvl[0][e / 8][e % 8] = leaf_hash[(size_t)inst * n * 8 + e];
  __syncthreads();
  uint8_t* out = nodes ? nodes + (size_t)inst * merkle_node_count(n) * 32 : nullptr;
  auto store = [&](int cur, uint32_t cnt, uint32_t base) {
    if (!out) return;
    for (uint32_t e = threadIdx.x; e < cnt * 32; e += blockDim.x) {
      const uint32_t wv = lvl[cur][e / 32][(e % 32) / 4];
      out[(size_t)(base + e / 32) * 32 + e % 32] = (uint8_t)(wv >> (8 * (3 - e % 4)));
    }
  };
  uint32_t cnt = n, base = 0;
  int cur = 0;
  store(cur, cnt, base);
  while (cnt > 1) {
    const uint32_t nxt = (cnt + 1) / 2;
    for (uint32_t j = threadIdx.x; j < nxt; j += blockDim.x) {
      if (2 * j + 1 < cnt) {
        merkle_node(variant, lvl[cur][2 * j], lvl[cur][2 * j + 1], lvl[cur ^ 1][j]);
      } else {
#pragma unroll
        for (int q = 0; q < 8; q++) lvl[cur ^ 1][j][q] = lvl[cur][2 * j][q];
      }
    }
    __syncthreads();
    base += cnt;
    cur ^= 1;
    cnt = nxt;
    store(cur, cnt, base);
  }
  if (threadIdx.x < 32) {
    const uint32_t wv = lvl[cur][0][threadIdx.x / 4];
    roots[(size_t)inst * 32 + threadIdx.x] = (uint8_t)(wv >> (8 * (3 - threadIdx.x % 4)));
  }
}
#endif

// MerkleTree::gen_proof (broadcast.rs:389-401 asks one per node) from the stored tree: proof q
// is for leaf req[2q + 1] of instance req[2q]; like merkle.rs it is the proof of the FIRST leaf
// whose digest equals that leaf's (equal leaves cannot occur for index-prefixed shards of N <= 256,
// broadcast.rs:371-372, but the semantics are kept).  Output in the layout k_merkle_validate
// reads: node path root first ... leaf digest (depth + 1 entries of 32 B), the sibling of each
// lemma level, `sides` bit l = the level-l sibling is Positioned::Left, depth, root.
#if HBX_IN_TU(6)
__global__ void __launch_bounds__(64) k_merkle_proofs(const uint8_t* __restrict__ nodes, uint32_t n,
                                                      const uint32_t* __restrict__ req, uint32_t count,
                                                      uint8_t* __restrict__ node_hash, uint8_t* __restrict__ sib_hash,
                                                      uint32_t* __restrict__ sides, uint32_t* __restrict__ depth,
                                                      uint8_t* __restrict__ root) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= count) return;
  const uint32_t inst = req[2 * q];
  uint32_t pos = req[2 * q + 1];
  const uint32_t total = merkle_node_count(n);
  const uint8_t* T = nodes + (size_t)inst * total * 32;
  auto eq32 = [](const uint8_t* a, const uint8_t* b) {
    bool e = true;
    for (int k = 0; k < 32; k++) e = e && a[k] == b[k];
    return e;
  };
  for (uint32_t j = 0; j < pos; j++)
    if (eq32(T + (size_t)j * 32, T + (size_t)pos * 32)) {
      pos = j;
      break;
    }
  // walk up: (node on the path, sibling, side) for every level where the node has a sibling
  uint32_t path[16], sib[16], left_bits = 0, d = 0;
  uint32_t cnt = n, base = 0;
  while (cnt > 1) {
    const bool promoted = (pos % 2 == 0) && pos == cnt - 1;
    if (!promoted) {
      path[d] = base + pos;
      sib[d] = base + (pos ^ 1u);
      if (pos & 1u) left_bits |= 1u << d;  // sibling on the left
      d++;
    }
    base += cnt;
    pos /= 2;
    cnt = (cnt + 1) / 2;
  }
  const uint32_t root_idx = total - 1;
  uint8_t* nh = node_hash + (size_t)q * 17 * 32;
  uint8_t* sh = sib_hash + (size_t)q * 16 * 32;
  uint32_t side_out = 0;
  for (int k = 0; k < 32; k++) nh[k] = T[(size_t)root_idx * 32 + k];
  for (uint32_t lv = 0; lv < d; lv++) {
    const uint32_t up = d - 1 - lv;  // lemma level lv (root first) = walk step d - 1 - lv
    for (int k = 0; k < 32; k++) {
      sh[(size_t)lv * 32 + k] = T[(size_t)sib[up] * 32 + k];
      nh[(size_t)(lv + 1) * 32 + k] = T[(size_t)path[up] * 32 + k];
    }
    if ((left_bits >> up) & 1u) side_out |= 1u << lv;
  }
  for (int k = 0; k < 32; k++) root[(size_t)q * 32 + k] = T[(size_t)root_idx * 32 + k];
  sides[q] = side_out;
  depth[q] = d;
}
#endif

// Broadcast::validate_proof (broadcast.rs:555-575) over a batch of proofs:
//   Proof::validate(root): root == lemma[0].node_hash == the proof's root_hash, every
//   lemma[k].node_hash == H(01 || left || right) of its child and sibling, and the leaf lemma's
//   hash == SHA-256(0x00 || value); then value[0] == sender index == Proof::index(count).
// Per proof j: value = values + j * vlen (the index byte first), depth[j] <= 16,
// nodes = node_hash + j * 17 * 32 (root first, leaf hash last), sibs = sib_hash + j * 16 * 32,
// sides bit k set = sibling at level k is on the LEFT (merkle.rs Positioned::Left).
#if HBX_IN_TU(6)
__global__ void __launch_bounds__(64) k_merkle_validate(const uint8_t* __restrict__ values, uint32_t vlen,
                                                        const uint8_t* __restrict__ node_hash,
                                                        const uint8_t* __restrict__ sib_hash,
                                                        const uint32_t* __restrict__ sides,
                                                        const uint32_t* __restrict__ depth,
                                                        const uint8_t* __restrict__ root_hash,
                                                        const uint32_t* __restrict__ sender, uint32_t count,
                                                        uint32_t nproofs, uint8_t* __restrict__ valid, int variant,
                                                        const uint32_t* __restrict__ vdigest) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nproofs) return;
  const uint32_t d = depth[j];
  const uint8_t* nodes = node_hash + (size_t)j * 17 * 32;
  const uint8_t* sibs = sib_hash + (size_t)j * 16 * 32;
  const uint8_t* val = values + (size_t)j * vlen;
  bool ok = d <= 16 && vlen >= 1;
  for (int q = 0; q < 32 && ok; q++) ok = root_hash[(size_t)j * 32 + q] == nodes[q];
  auto be8 = [](const uint8_t* p, uint32_t* w) {
    for (int q = 0; q < 8; q++)
      w[q] = ((uint32_t)p[4 * q] << 24) | ((uint32_t)p[4 * q + 1] << 16) | ((uint32_t)p[4 * q + 2] << 8) | p[4 * q + 3];
  };
  uint32_t h[8], want[8], a[8], b[8];
  if (ok) {
    if (vdigest) {  // the values' leaf digests, hashed beforehand by the leaf kernels
#pragma unroll
      for (int q = 0; q < 8; q++) h[q] = vdigest[(size_t)j * 8 + q];
    } else {
      merkle_leaf_value(variant, val, vlen, h);
    }
    be8(nodes + (size_t)d * 32, want);
    for (int q = 0; q < 8; q++) ok = ok && h[q] == want[q];
  }
  for (uint32_t lv = 0; lv < d && ok; lv++) {
    be8(sibs + (size_t)lv * 32, a);
    be8(nodes + (size_t)(lv + 1) * 32, b);
    if ((sides[j] >> lv) & 1) merkle_node(variant, a, b, h);
    else merkle_node(variant, b, a, h);
    be8(nodes + (size_t)lv * 32, want);
    for (int q = 0; q < 8; q++) ok = ok && h[q] == want[q];
  }
  // Proof::index(count) from the Left/Right path
  uint32_t idx = 0, c = count;
  for (uint32_t lv = 0; lv < d; lv++) {
    const uint32_t left = c > 1 ? 1u << (31 - __clz(c - 1)) : 1u;
    if ((sides[j] >> lv) & 1) {
      idx += left;
      c -= left;
    } else {
      c = left;
    }
  }
  ok = ok && val[0] == sender[j] && idx == val[0];
  valid[j] = ok ? 1 : 0;
}
#endif

// glue_shards (broadcast.rs:697-707): the payload is bytes [4, 4 + len) of the first k shards
// (contiguous), len = the big-endian u32 header clamped to the available bytes.  grid
// (ceil(max_len / 4096), inst): thread = 16 output bytes, dword loads/stores when source and
// destination rows are dword-aligned (byte copy otherwise).
#if HBX_IN_TU(6)
__global__ void __launch_bounds__(256) k_glue(const uint8_t* __restrict__ shards, size_t inst_stride, uint32_t k,
                                              uint32_t L, uint8_t* __restrict__ out, size_t out_stride,
                                              uint64_t* __restrict__ out_len, int32_t* __restrict__ status) {
  const uint32_t inst = blockIdx.y;
  const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
  if (status[inst] != 0) {
    if (lead) out_len[inst] = 0;
    return;
  }
  const uint8_t* base = shards + (size_t)inst * inst_stride;  // shards 0..k-1 are contiguous
  const uint64_t total = (uint64_t)k * L;
  if (total < 4) {
    if (lead) {  // the other blocks of the instance return here or above either way
      status[inst] = -11;
      out_len[inst] = 0;
    }
    return;
  }
  const uint64_t want = ((uint64_t)base[0] << 24) | ((uint64_t)base[1] << 16) | ((uint64_t)base[2] << 8) | base[3];
  // glue_shards takes at most the bytes there are (broadcast.rs:704); the row holds out_stride
  uint64_t len = want < total - 4 ? want : total - 4;
  if (len > out_stride) len = out_stride;
  if (lead) out_len[inst] = len;
  const uint64_t q0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (q0 >= len) return;
  const uint8_t* src = base + 4 + q0;
  uint8_t* dst = out + (size_t)inst * out_stride + q0;
  if (q0 + 16 <= len && (((uintptr_t)src | (uintptr_t)dst) & 3) == 0) {
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d4 = reinterpret_cast<uint32_t*>(dst);
    const uint32_t v0 = s4[0], v1 = s4[1], v2 = s4[2], v3 = s4[3];
    d4[0] = v0;
    d4[1] = v1;
    d4[2] = v2;
    d4[3] = v3;
  } else {
    const uint64_t end = q0 + 16 < len ? 16 : len - q0;
    for (uint64_t q = 0; q < end; q++) dst[q] = src[q];
  }
}
#endif

// status = root(inst) == expected ? status : HBX_E_ROOT_MISMATCH
#if HBX_IN_TU(6)
__global__ void k_root_check(const uint8_t* __restrict__ roots, const uint8_t* __restrict__ expect, uint32_t inst,
                             int32_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= inst || status[i] != 0) return;
  bool eq = true;
  for (int q = 0; q < 32; q++) eq = eq && roots[(size_t)i * 32 + q] == expect[(size_t)i * 32 + q];
  if (!eq) status[i] = -10;
}
#endif

}  // namespace hbx
