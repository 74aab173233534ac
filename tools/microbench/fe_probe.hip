// Register-pressure probe of the one-lane final exponentiation's pieces (fe1d.hpp), each in a kernel
// of its own with the same slot layout as k_fe1 (slot A in LDS, lane-interleaved; global slots
// [block][slot][word][64 lanes]).  Compiled device-only and read with tools/kres.py: which piece sets
// the step kernels' VGPR peak and spills.  Also runnable: every kernel writes its
// result, so a timing harness can launch it (grid = 1024 one-wave blocks like the N=256 epoch).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 --cuda-device-only -c -o /tmp/fe_probe.co fe_probe.hip
//   python tools/kres.py /tmp/fe_probe.co
#include <hip/hip_runtime.h>
#include "../../hbbft_amd/csrc/fe1d.hpp"

using namespace hbx;

#ifndef PROBE_WAVES
#define PROBE_WAVES 1  // min waves per SIMD the kernels are compiled for (2: at most 256 registers)
#endif
#ifndef PROBE_LANE_LDS
#define PROBE_LANE_LDS 1  // 1: the slot addressed afresh (fe1d.hpp lane_lds), 0: a held pointer
#endif
#if PROBE_LANE_LDS
#define PROBE_LDS_SLOT const lane_lds a { (lds_u32*)slots }
#else
#define PROBE_LDS_SLOT lds_u32* a = (lds_u32*)(slots + threadIdx.x)
#endif
#define PROBE_SLOTS                                                                                   \
  __shared__ uint32_t slots[FE1_WORDS * 64];                                                         \
  PROBE_LDS_SLOT;                                                                                     \
  uint32_t* gf = g + (size_t)blockIdx.x * (3 * FE1_WORDS * 64) + threadIdx.x;                        \
  uint32_t* gt = gf + FE1_WORDS * 64;                                                                \
  uint32_t* gg = gt + FE1_WORDS * 64;                                                                \
  (void)gt;                                                                                           \
  (void)gg

#ifndef PROBE
#define PROBE 0  // 0: every kernel; k: only kernel k (parallel compiles)
#endif
#define PROBE_ON(k) (PROBE == 0 || PROBE == (k))

#ifdef PROBE_CHOOSE
#undef PROBE_ON
#define PROBE_ON(k) (((PROBE_CHOOSE) >> (k)) & 1)  // a bit mask of kernels
#endif

#if PROBE_ON(1)
// one Fq12 product by the slot, `reps` times
__global__ void __launch_bounds__(64, PROBE_WAVES) p_mul(uint32_t* g, int reps) {
  PROBE_SLOTS;
  s1_copy<64, 64>(a, gg);
  HBX_SEQ();
  fq12d r = s1_get_fq12d<64>(gf);
#pragma unroll 1
  for (int k = 0; k < reps; k++) {
    HBX_SEQ();
    r = fq12d_mul_slot<64>(r, a);
  }
  s1_put_fq12d<64>(gf, r);
}
#endif

#if PROBE_ON(2)
// `reps` Granger-Scott squarings
__global__ void __launch_bounds__(64, PROBE_WAVES) p_cyc(uint32_t* g, int reps) {
  PROBE_SLOTS;
  fq12d r = s1_get_fq12d<64>(gf);
#pragma unroll 1
  for (int k = 0; k < reps; k++) r = fq12d_cyclotomic_sqr_seq(r);
  s1_put_fq12d<64>(gf, r);
}
#endif

#if PROBE_ON(3)
// `reps` compressed squarings and the decompression
__global__ void __launch_bounds__(64, PROBE_WAVES) p_kara(uint32_t* g, int reps) {
  PROBE_SLOTS;
  fq12d r = s1_get_fq12d<64>(gf);
  fq12c c{r.c0.c1, r.c0.c2, r.c1.c0, r.c1.c2};
#pragma unroll 1
  for (int k = 0; k < reps; k++) karabina_sqr(c);
  HBX_SEQ();
  bool deg = false;
  r = karabina_decompress(c, deg);
  s1_put_fq12d<64>(gf, r);
  if (deg) gg[0] = 1;
}
#endif

#if PROBE_ON(6)
// `reps` compressed squarings alone
__global__ void __launch_bounds__(64, PROBE_WAVES) p_kloop(uint32_t* g, int reps) {
  PROBE_SLOTS;
  fq12d r = s1_get_fq12d<64>(gf);
  fq12c c{r.c0.c1, r.c0.c2, r.c1.c0, r.c1.c2};
#pragma unroll 1
  for (int k = 0; k < reps; k++) karabina_sqr(c);
  s1_put_fq2d<64>(gf, 0, c.g1);
  s1_put_fq2d<64>(gf, 1, c.g2);
  s1_put_fq2d<64>(gf, 2, c.g3);
  s1_put_fq2d<64>(gf, 3, c.g5);
}
#endif

#if PROBE_ON(7)
// the decompression alone
__global__ void __launch_bounds__(64, PROBE_WAVES) p_decomp(uint32_t* g, int reps) {
  PROBE_SLOTS;
  (void)reps;
  fq12c c{s1_get_fq2d<64>(gf, 0), s1_get_fq2d<64>(gf, 1), s1_get_fq2d<64>(gf, 2), s1_get_fq2d<64>(gf, 3)};
  bool deg = false;
  const fq12d r = karabina_decompress(c, deg);
  s1_put_fq12d<64>(gf, r);
  if (deg) gg[0] = 1;
}
#endif

#if PROBE_ON(8)
// one Fq2 product alone (operands from the slots): the product's own register need
__global__ void __launch_bounds__(64, PROBE_WAVES) p_fq2(uint32_t* g, int reps) {
  PROBE_SLOTS;
  (void)reps;
  const fq2d x = s1_get_fq2d<64>(gf, 0), y = s1_get_fq2d<64>(gf, 1);
  s1_put_fq2d<64>(gg, 0, fq2d_mul(x, y));
}
#endif

#if PROBE_ON(9)
// one Fq6 product by a streamed operand into an accumulator
__global__ void __launch_bounds__(64, PROBE_WAVES) p_fq6(uint32_t* g, int reps) {
  PROBE_SLOTS;
  (void)reps;
  const fq6d x = s1_get_half<64>(gf, 0);
  fq6d acc = fq6d_zero_();
  fq6d_mul_acc1(acc, x, [&](int q) { return s1_get_fq2d<64>(gt, q); });
  s1_put_fq2d<64>(gg, 0, acc.c0);
  s1_put_fq2d<64>(gg, 1, acc.c1);
  s1_put_fq2d<64>(gg, 2, acc.c2);
}
#endif

#if PROBE_ON(10)
// `reps` dependent Fq inversions (field.hpp fq_inv_i: batched divsteps), the decompression's core
__global__ void __launch_bounds__(64, PROBE_WAVES) p_inv(uint32_t* g, int reps) {
  PROBE_SLOTS;
#if PROBE_INV_DIGITS
  fqd x = s1_get_fqd<64>(gf, 0);  // fieldd.hpp fqd_inv (divsteps on the 28-bit digits)
  bool z = false;
#pragma unroll 1
  for (int k = 0; k < reps; k++) x = fqd_norm(fqd_add(fqd_inv(x, z), fqd_const(FQD_ONE)));
  s1_put_fqd<64>(gg, 0, x);
  if (z) gg[64] = 1;
#else
  fq x = fqd_to_fq(s1_get_fqd<64>(gf, 0));  // field.hpp fq_inv_i (12-limb divsteps)
#pragma unroll 1
  for (int k = 0; k < reps; k++) x = fq_add(fq_inv_i(x), fq_one());
  s1_put_fqd<64>(gg, 0, fqd_from_fq(x));
#endif
}
#endif

#if PROBE_ON(4)
// one exp-by-|x| with the base in slot a
__global__ void __launch_bounds__(64, PROBE_WAVES) p_exp(uint32_t* g, int reps) {
  PROBE_SLOTS;
  (void)reps;
  s1_copy<64, 64>(a, gf);
  HBX_SEQ();
  fq12d r = s1_get_fq12d<64>(a);
  bool deg = false;
  r = cyc_exp_abs_x_slot<64, 64>(r, a, (uint32_t*)nullptr, deg);
  s1_put_fq12d<64>(gf, r);
  if (deg) gg[0] = 1;
}
#endif

#if PROBE_ON(5)
// the F1 + F2 step kernel's body
__global__ void __launch_bounds__(64, PROBE_WAVES) p_step12(uint32_t* g, int reps) {
  PROBE_SLOTS;
  (void)reps;
  bool deg = false;
  fe1_step12<64, 64>(a, gt, gg, deg);
  if (deg) gf[0] = 1;
}
#endif

#if !defined(__HIP_DEVICE_COMPILE__) || 1
#include <cstdio>
#include <vector>
// Timing harness (the pieces this build has, -DPROBE=k for one): each over 1,024 one-wave blocks (one wave per SIMD, the N=256 epoch's
// share-check grid), HIP events, best of 3; per-unit microseconds = time / reps.
int main() {
  const int blocks = 1024 * PROBE_WAVES;  // PROBE_WAVES waves per SIMD
  const size_t words = (size_t)blocks * 3 * FE1_WORDS * 64;
  std::vector<uint32_t> h(words);
  uint32_t s = 12345;
  for (size_t i = 0; i < words; i++) {
    s = s * 1664525u + 1013904223u;
    h[i] = (s >> 4) & 0x0FFFFFFFu;  // 28-bit words: digits stay in range after unpacking
  }
  uint32_t* g;
  if (hipMalloc(&g, words * 4) != hipSuccess) return 2;
  struct K {
    const char* name;
    void (*fn)(uint32_t*, int);
    int reps;
  } ks[] = {
#if PROBE_ON(1)
      {"p_mul (Fq12 x slot)", p_mul, 5},
#endif
#if PROBE_ON(2)
      {"p_cyc (Granger-Scott)", p_cyc, 15},
#endif
#if PROBE_ON(6)
      {"p_kloop (Karabina sqr)", p_kloop, 48},
#endif
#if PROBE_ON(7)
      {"p_decomp (decompression)", p_decomp, 1},
#endif
#if PROBE_ON(10)
      {"p_inv (Fq inversion)", p_inv, 8},
#endif
#if PROBE_ON(3)
      {"p_kara (48 sqr + decomp)", p_kara, 48},
#endif
#if PROBE_ON(4)
      {"p_exp (exp by |x|)", p_exp, 1},
#endif
#if PROBE_ON(5)
      {"p_step12 (F1 + F2)", p_step12, 1},
#endif
  };
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (auto& k : ks) {
    float best = 1e30f;
    for (int it = 0; it < 3; it++) {
      if (hipMemcpy(g, h.data(), words * 4, hipMemcpyHostToDevice) != hipSuccess) return 3;
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(64), 0, 0, g, k.reps);
      (void)hipEventRecord(e1, 0);
      if (hipEventSynchronize(e1) != hipSuccess) return 4;
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    // per unit of one wave-per-SIMD's work: time / (reps * waves per SIMD)
    printf("%-28s reps %3d  waves/SIMD %d  %8.3f ms  %8.2f us/unit per 1024 waves\n", k.name, k.reps, PROBE_WAVES, best,
           best * 1e3 / k.reps / PROBE_WAVES);
  }
  return 0;
}
#endif
