// Issue cost of the digit tower's two multiply-adds on gfx950, forced by inline asm (the compiler
// rewrites C-level signed products of known-range operands into unsigned expansions, which is what
// issue.hip's mad_i64 row measured): v_mad_i64_i32 (the signed digit convolutions of fieldd.hpp)
// against v_mad_u64_u32 (the Montgomery reduction digits), one wave per SIMD (1,024 one-wave
// blocks) and four, with 8 independent accumulators per lane (throughput) or 1 (dependent latency).
//   hipcc -O3 --offload-arch=gfx950 -o madrate2 madrate2.hip && ./madrate2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096

// SD: the carry-out (sdst) of the MADs -- 0: vcc for every MAD, 1: a distinct SGPR pair per
// chain (s[40:41] .. s[54:55]), 2: two pairs alternating.  Every MAD writes its sdst, so a single
// wave's consecutive MADs may wait on each other's SGPR write even when their VGPRs are independent.
#define MADI(OP, SDST, i) __asm__ volatile(OP " %0, " SDST ", %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b + i) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "vcc")
template <bool SIGNED, int CH, int SD>
__global__ void __launch_bounds__(64) k_mad_sd(uint64_t* out, uint32_t a0) {
  uint32_t a = a0 + threadIdx.x, b = a0 ^ 0x9e3779b9u;
  uint64_t acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
    if (SD == 1) {
      MADI("v_mad_u64_u32", "s[40:41]", 0); MADI("v_mad_u64_u32", "s[42:43]", 1);
      MADI("v_mad_u64_u32", "s[44:45]", 2); MADI("v_mad_u64_u32", "s[46:47]", 3);
      MADI("v_mad_u64_u32", "s[48:49]", 4); MADI("v_mad_u64_u32", "s[50:51]", 5);
      MADI("v_mad_u64_u32", "s[52:53]", 6); MADI("v_mad_u64_u32", "s[54:55]", 7);
    } else {
      MADI("v_mad_u64_u32", "s[40:41]", 0); MADI("v_mad_u64_u32", "s[42:43]", 1);
      MADI("v_mad_u64_u32", "s[40:41]", 2); MADI("v_mad_u64_u32", "s[42:43]", 3);
      MADI("v_mad_u64_u32", "s[40:41]", 4); MADI("v_mad_u64_u32", "s[42:43]", 5);
      MADI("v_mad_u64_u32", "s[40:41]", 6); MADI("v_mad_u64_u32", "s[42:43]", 7);
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// MIX: 1 = four u64 and four i64 chains interleaved; 2 = eight u64 chains, each MAD followed by an
// independent 32-bit add; 3 = eight u64 chains, each MAD followed by an independent 64-bit shift
template <int MIX>
__global__ void __launch_bounds__(64) k_mix(uint64_t* out, uint32_t a0) {
  uint32_t a = a0 + threadIdx.x, b = a0 ^ 0x9e3779b9u;
  uint64_t acc[8];
  uint32_t t[8];
  uint64_t u[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc[i] = i * 7 + threadIdx.x;
    t[i] = i * 3 + threadIdx.x;
    u[i] = acc[i] << 20;
  }
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (MIX == 1 && (i & 1))
        __asm__ volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b + i) : "vcc");
      else
        __asm__ volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b + i) : "vcc");
      if (MIX == 2) __asm__ volatile("v_add_u32_e32 %0, %1, %0" : "+v"(t[i]) : "v"(a));
      if (MIX == 3) __asm__ volatile("v_ashrrev_i64 %0, 1, %0" : "+v"(u[i]));
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= acc[i] ^ t[i] ^ u[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <bool SIGNED, int CH>
__global__ void __launch_bounds__(64) k_mad(uint64_t* out, uint32_t a0) {
  uint32_t a = a0 + threadIdx.x, b = a0 ^ 0x9e3779b9u;
  uint64_t acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      if (SIGNED)
        __asm__ volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b + i) : "vcc");
      else
        __asm__ volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b + i) : "vcc");
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <bool SIGNED, int CH, int SD = 0>
static void run(uint64_t* d, int waves_per_simd, const char* name) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int blocks = 1024 * waves_per_simd;
  float best = 1e30f;
  for (int r = 0; r < 3; r++) {
    (void)hipEventRecord(e0, 0);
    if (SD >= 10)
      hipLaunchKernelGGL((k_mix<SD - 10>), dim3(blocks), dim3(64), 0, 0, d, 1u + r);
    else if (SD == 0)
      hipLaunchKernelGGL((k_mad<SIGNED, CH>), dim3(blocks), dim3(64), 0, 0, d, 1u + r);
    else
      hipLaunchKernelGGL((k_mad_sd<SIGNED, CH, SD>), dim3(blocks), dim3(64), 0, 0, d, 1u + r);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  // SIMD cycles per wave-instruction at 2.4 GHz (each SIMD runs waves_per_simd waves)
  const double ops = (double)ITERS * CH * waves_per_simd;  // MAD count (the mixes' other ops not counted)
  printf("%-16s chains %d  waves/SIMD %d  %.3f ms  %.2f SIMD-cycles per wave-op\n", name, CH, waves_per_simd, best,
         best * 1e-3 * 2.4e9 / ops);
}

int main() {
  uint64_t* d;
  if (hipMalloc(&d, 4096 * 64 * 8) != hipSuccess) return 2;
  for (int w : {1, 4}) {
    run<false, 8>(d, w, "v_mad_u64_u32");
    run<true, 8>(d, w, "v_mad_i64_i32");
    run<false, 1>(d, w, "v_mad_u64_u32");
    run<true, 1>(d, w, "v_mad_i64_i32");
    run<false, 8, 1>(d, w, "u64 sdst x8 pairs");
    run<false, 8, 2>(d, w, "u64 sdst x2 pairs");
    run<false, 8, 11>(d, w, "mix u64+i64 4+4");
    run<false, 8, 12>(d, w, "mad + add_u32 (per mad)");
    run<false, 8, 13>(d, w, "mad + ashr_i64 (per mad)");
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 3;
}
