// Group executor for the wide-tower programs (tools/gen_programs.py -> programs.hpp).
//
// A pairing check is run by a GROUP of 16 lanes.  Its tower state lives in LDS slots (one Fq
// element = 12 x u32, Montgomery form, lazily reduced to [0, 2p]); each program is a list of
// rounds, each round at most 16 independent instructions, lane k of the group running
// instruction k:
//     MUL  dst = (sum c_i slot_i) * (sum d_j slot_j)      LIN  dst = sum c_i slot_i
//     INV  dst = (sum c_i slot_i)^(p-2)
// Every lane first loads all its operands, then computes, then stores (after the wave has
// reconverged), so within a round all reads precede all writes; rounds are separated by a
// wave-level fence.  A group never spans two waves (16 | 64), so no workgroup barrier is needed
// inside a program.  The generator guarantees that a slot written in round r is not read by
// another instruction of round r.
//
// Slot classes: SCR (group scratch), X, Y, P, O (group regions with runtime bases), L (block
// shared line coefficients), K (block shared constants).  Bases are LDS dword offsets.
#pragma once
#include "field.hpp"
#include "programs.hpp"

namespace hbx {
namespace wide {

constexpr int G = 16;           // lanes per group
constexpr int SLOT = 12;        // dwords per slot

struct bases {
  uint32_t cls[7];  // dword offset of slot 0 of each class
};

__device__ __forceinline__ fq lds_load_fq(const uint32_t* lds, uint32_t off) {
  fq r;
  const uint4* p = reinterpret_cast<const uint4*>(lds + off);
#pragma unroll
  for (int q = 0; q < 3; q++) {
    const uint4 v = p[q];
    r.l[4 * q] = v.x;
    r.l[4 * q + 1] = v.y;
    r.l[4 * q + 2] = v.z;
    r.l[4 * q + 3] = v.w;
  }
  return r;
}

__device__ __forceinline__ void lds_store_fq(uint32_t* lds, uint32_t off, const fq& a) {
  uint4* p = reinterpret_cast<uint4*>(lds + off);
#pragma unroll
  for (int q = 0; q < 3; q++) p[q] = make_uint4(a.l[4 * q], a.l[4 * q + 1], a.l[4 * q + 2], a.l[4 * q + 3]);
}

__device__ __forceinline__ uint32_t slot_off(const bases& b, uint32_t cls, uint32_t idx) {
  uint32_t base = b.cls[0];
#pragma unroll
  for (int c = 1; c < 7; c++) base = cls == (uint32_t)c ? b.cls[c] : base;
  return base + idx * SLOT;
}

// Operand accumulation in raw 13-limb form: every slot holds a value v <= 2p; a term c*slot adds
// |c| * v (c > 0) or |c| * (2p - v) (c < 0), so a sum of terms with S = sum |c| is < S * 2p + 1 and
// nonnegative.  No modular reduction per term; one conditional-subtract ladder at the end.
struct acc13 {
  uint32_t l[13];
};

__device__ __forceinline__ void acc_add(acc13& acc, const uint32_t* x) {  // acc += x (12 limbs)
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) acc.l[i] = addc32(acc.l[i], x[i], c);
  acc.l[12] += c;
}

// 2^k * 2p for k = 0..6 (13 limbs each) -- the reduction ladder
__device__ constexpr uint32_t LADDER[7][13] = {
#define HBX_L(k)                                                                                   \
  {(FQ_2P[0] << k), (FQ_2P[1] << k) | (k ? FQ_2P[0] >> (32 - k) : 0u),                             \
   (FQ_2P[2] << k) | (k ? FQ_2P[1] >> (32 - k) : 0u), (FQ_2P[3] << k) | (k ? FQ_2P[2] >> (32 - k) : 0u), \
   (FQ_2P[4] << k) | (k ? FQ_2P[3] >> (32 - k) : 0u), (FQ_2P[5] << k) | (k ? FQ_2P[4] >> (32 - k) : 0u), \
   (FQ_2P[6] << k) | (k ? FQ_2P[5] >> (32 - k) : 0u), (FQ_2P[7] << k) | (k ? FQ_2P[6] >> (32 - k) : 0u), \
   (FQ_2P[8] << k) | (k ? FQ_2P[7] >> (32 - k) : 0u), (FQ_2P[9] << k) | (k ? FQ_2P[8] >> (32 - k) : 0u), \
   (FQ_2P[10] << k) | (k ? FQ_2P[9] >> (32 - k) : 0u), (FQ_2P[11] << k) | (k ? FQ_2P[10] >> (32 - k) : 0u), \
   (k ? FQ_2P[11] >> (32 - k) : 0u)}
    HBX_L(0), HBX_L(1), HBX_L(2), HBX_L(3), HBX_L(4), HBX_L(5), HBX_L(6)
#undef HBX_L
};

// acc < 2^K * 2p  ->  [0, 2p)
__device__ __forceinline__ fq acc_reduce(acc13 acc, int K) {
  for (int k = 6; k >= 0; k--) {
    if (k >= K) continue;
    uint32_t d[13];
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 13; i++) d[i] = subb32(acc.l[i], LADDER[k][i], br);
#pragma unroll
    for (int i = 0; i < 13; i++) acc.l[i] = br ? acc.l[i] : d[i];
  }
  fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = acc.l[i];
  return r;
}

// Instruction words live in registers (loaded once per round, prefetched a round ahead); the
// term loop is unrolled so every word index is static.
struct insn {
  uint4 w[4];
};
__device__ __forceinline__ uint32_t insn_word(const insn& I, int k) {
  const uint4 v = I.w[k >> 2];
  return (k & 3) == 0 ? v.x : (k & 3) == 1 ? v.y : (k & 3) == 2 ? v.z : v.w;
}
__device__ __forceinline__ insn load_insn(uint32_t idx) {
  insn I;
  const uint4* p = reinterpret_cast<const uint4*>(prog::INSNS[idx]);
#pragma unroll
  for (int q = 0; q < 4; q++) I.w[q] = p[q];
  return I;
}

// Raw sums of the A terms [0, na) and B terms [na, na + nb); S = sum |c| of each.
__device__ __forceinline__ void sum_terms(const uint32_t* lds, const bases& b, const insn& I, int na, int nb,
                                          acc13& ra, int& SA, acc13& rb, int& SB) {
#pragma unroll
  for (int i = 0; i < 13; i++) ra.l[i] = rb.l[i] = 0;
  SA = SB = 0;
#pragma unroll
  for (int t = 0; t < 15; t++) {
    if (t < na + nb) {
    const uint32_t term = insn_word(I, 1 + t);
    fq v = lds_load_fq(lds, slot_off(b, (term >> 16) & 0xF, term & 0xFFFF));
    const int c = (int)(int8_t)(term >> 24);
    if (c < 0) {  // 2p - v
      uint64_t br = 0;
#pragma unroll
      for (int i = 0; i < 12; i++) {
        const uint64_t x = (uint64_t)FQ_2P[i] - v.l[i] - br;
        v.l[i] = (uint32_t)x;
        br = (x >> 32) & 1;
      }
    }
    const int m = c < 0 ? -c : c;
    if (t < na) {
      SA += m;
      for (int q = 0; q < m; q++) acc_add(ra, v.l);
    } else {
      SB += m;
      for (int q = 0; q < m; q++) acc_add(rb, v.l);
    }
    }
  }
}

__device__ __forceinline__ int ladder_steps(int S) { return S <= 1 ? 0 : 32 - __clz(S - 1); }

// a^(p-2) with a 2-bit fixed window and a small register footprint (the INV instruction: one lane
// of the group, once per pairing check).  Exponent bits come from a wave-uniform constant.
__device__ __forceinline__ fq fq_inv_lowreg(const fq& a) {
  const fq a2 = fq_sqr(a);
  const fq a3 = fq_mul(a2, a);
  fq r = a;  // top 2-bit digit of p-2 is 1 (bits 380..381 = 0b01)
#pragma unroll 1
  for (int w = 189; w >= 0; w--) {
    const uint32_t d = (FQ_P_MINUS_2[(2 * w) >> 5] >> ((2 * w) & 31)) & 3u;
    r = fq_sqr(r);
    r = fq_sqr(r);
    if (d) r = fq_mul(r, d == 1 ? a : d == 2 ? a2 : a3);
  }
  return r;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Run program `prog` for this lane's group.  `lane` = lane index within the group (0..15).
__device__ __forceinline__ void run(uint32_t* lds, int prog, int lane, const bases& b) {
  const uint32_t s0 = prog::PROG_STAGES[prog][0];
  const uint32_t ns = prog::PROG_STAGES[prog][1];
  uint32_t cnt = prog::STAGES[s0][1];
  insn cur = load_insn(prog::STAGES[s0][0] + ((uint32_t)lane < cnt ? lane : 0));
  for (uint32_t s = s0; s < s0 + ns; s++) {
    const bool act = (uint32_t)lane < cnt;
    // prefetch the next round's instruction while this one computes
    const uint32_t ncnt = s + 1 < s0 + ns ? prog::STAGES[s + 1][1] : 0;
    const insn nxt = load_insn(s + 1 < s0 + ns ? prog::STAGES[s + 1][0] + ((uint32_t)lane < ncnt ? lane : 0)
                                               : prog::STAGES[s][0]);
    fq r = fq_zero();
    uint32_t dst = 0;
    if (act) {
      const uint32_t hdr = cur.w[0].x;
      const uint32_t op = hdr & 0xF, na = (hdr >> 4) & 0xF, nb = (hdr >> 8) & 0xF;
      dst = slot_off(b, (hdr >> 12) & 0xF, hdr >> 16);
      acc13 ra, rb;
      int SA, SB;
      sum_terms(lds, b, cur, (int)na, (int)nb, ra, SA, rb, SB);
      if (op == 0) {
        // MUL: A may stay raw while < 2^383 (S <= 2: 2 * 2p < 2^383; then A*B < p R and the product < 2p);
        // B must be < 2p
        const fq fa = acc_reduce(ra, SA <= 2 ? 0 : ladder_steps(SA));
        const fq fb = acc_reduce(rb, ladder_steps(SB));
        r = fq_mul(fa, fb);
      } else {
        const fq fa = acc_reduce(ra, ladder_steps(SA));
        r = op == 2 ? fq_inv_lowreg(fa) : fa;
      }
    }
    // every lane of the wave has finished its loads before any store of this round
    __builtin_amdgcn_wave_barrier();
    if (act) lds_store_fq(lds, dst, r);
    wave_sync();
    cur = nxt;
    cnt = ncnt;
  }
}

}  // namespace wide
}  // namespace hbx
