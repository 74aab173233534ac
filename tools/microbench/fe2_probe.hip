// Register-pressure / throughput probe of the two-lane final exponentiation (pairing2d.hpp
// final_exp2d_is_one) compiled for one or two waves per SIMD (-DPROBE_WAVES=1|2): does a pair
// of lanes per check fit 256 registers (one wave per SIMD issues a 64-bit
// multiply-add only every ~10.5 cycles against ~5.5 for the SIMD with several waves,
// profiles/r06d_madrate2.txt)?  Slot A in global memory when PROBE_A_GLOBAL (LDS for two waves per
// SIMD holds one packed Fq12 per pair, not two).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../../hbbft_amd/csrc/pairing2d.hpp"

using namespace hbx;
#ifndef PROBE_WAVES
#define PROBE_WAVES 2
#endif
#ifndef PROBE_A_GLOBAL
#define PROBE_A_GLOBAL 1
#endif

__global__ void __launch_bounds__(64, PROBE_WAVES) p_fe2(uint32_t* g, uint8_t* out) {
#if PROBE_A_GLOBAL
  __shared__ uint32_t region[LDS_FQ6D_PACKED * 64];  // slot B only
#else
  __shared__ uint32_t region[2 * LDS_FQ6D_PACKED * 64];
#endif
  const int lane = (int)(threadIdx.x & 63);
  const bool l1 = (lane & 1) != 0;
  const int pl = lane & ~1;
  lds_u32* reg = (lds_u32*)region;
  uint32_t* gb = g + (size_t)blockIdx.x * (4 * LDS_FQ6D_PACKED * 64) + pl;
  const slot2<lds_u32*> B{reg + pl, 64u};
  const slot2<uint32_t*> G1{gb, 64u}, G2{gb + LDS_FQ6D_PACKED * 64, 64u};
  // B = f (the pair's halves from global words)
  for (int w = 0; w < LDS_FQ6D_PACKED; w++) B.half(l1 ? 1 : 0)[w * 64] = gb[2 * LDS_FQ6D_PACKED * 64 + w * 64 + (l1 ? 1 : 0)];
  bool dg = false;
#if PROBE_A_GLOBAL
  const slot2<uint32_t*> A{gb + 3 * LDS_FQ6D_PACKED * 64, 64u};
  const bool v = final_exp2d_is_one<true, uint32_t*>(A, B, G1, G2, l1, dg);
#else
  const slot2<lds_u32*> A{reg + LDS_FQ6D_PACKED * 64 + pl, 64u};
  const bool v = final_exp2d_is_one<true>(A, B, G1, G2, l1, dg);
#endif
  out[blockIdx.x * 64 + lane] = (v ? 1 : 0) | (dg ? 2 : 0);
}

int main() {
  const int blocks = 2048;  // 65,536 checks on pairs: the N=256 epoch
  const size_t words = (size_t)blocks * 4 * LDS_FQ6D_PACKED * 64;
  std::vector<uint32_t> h(words);
  uint32_t s = 99;
  for (size_t i = 0; i < words; i++) {
    s = s * 1664525u + 1013904223u;
    h[i] = (s >> 4) & 0x0FFFFFFFu;
  }
  uint32_t* g;
  uint8_t* o;
  if (hipMalloc(&g, words * 4) != hipSuccess || hipMalloc(&o, blocks * 64) != hipSuccess) return 2;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int it = 0; it < 3; it++) {
    if (hipMemcpy(g, h.data(), words * 4, hipMemcpyHostToDevice) != hipSuccess) return 3;
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(p_fe2, dim3(blocks), dim3(64), 0, 0, g, o);
    (void)hipEventRecord(e1, 0);
    if (hipEventSynchronize(e1) != hipSuccess) return 4;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  printf("two-lane final exponentiation, 65,536 checks (2,048 waves), compiled for %d wave(s)/SIMD, slot A in %s: %.3f ms\n",
         PROBE_WAVES, PROBE_A_GLOBAL ? "global" : "LDS", best);
  return 0;
}
