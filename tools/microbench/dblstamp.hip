// Where one lane-group G2 doubling of the hash-to-G2 cofactor clearing spends its time (VERDICT r4
// item 3): s_memtime stamps between the segments of hash.hpp g2_dbl_group -- operand selection,
// the Fq product of each of the three rounds, the DPP broadcasts and additions between them --
// summed over 4096 dependent doublings of one 16-lane group (one wave on the chip, as a hash
// chain runs) and over the same on 64 waves (as k_prepare_ct's 256 hashes run).
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ unsigned long long g_seg[8];
__device__ unsigned long long g_last;
#define HBX_DBL_MARK(k)                                                                 \
  do {                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                                          \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                       \
      if ((k) > 0) g_seg[(k)] += t_ - g_last;                                           \
      g_last = t_;                                                                      \
    }                                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                                  \
  } while (0)
// a value's limbs as asm operands: computed before the stamp that follows
#define HBX_DBL_USE(v)                                                   \
  do {                                                                   \
    for (int i_ = 0; i_ < 12; i_++) __asm__ volatile("" ::"v"((v).l[i_])); \
  } while (0)
#include "../../hbbft_amd/csrc/hash.hpp"
using namespace hbx;

__global__ void __launch_bounds__(64) k_dbl(g2a* io, int n) {
  const int lane = threadIdx.x & 63, gl = lane % 16, gbase = lane - gl;
  g2j p = g2_from_affine(io[blockIdx.x]);
  for (int i = 0; i < n; i++) p = g2_dbl_group(p, gl, gbase);
  if (gl == 0) io[blockIdx.x * 4 + (lane >> 4)] = g2a{p.x, p.y, false};
}

int main() {
  const int n = 4096;
  g2a* d;
  if (hipMalloc(&d, 256 * sizeof(g2a)) != hipSuccess) return 1;
  g2a h[256];
  for (int i = 0; i < 256; i++) h[i] = g2a{fq2_one(), fq2_add(fq2_one(), fq2_one()), false};  // timing only: any (x, y)
  const char* names[8] = {"", "select r1", "product r1", "bcast+adds+select r2", "product r2",
                          "bcast+adds+select r3", "product r3", "bcast+adds tail"};
  for (int waves : {1, 64}) {
    if (hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 1;
    unsigned long long z[8] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_seg), z, sizeof(z));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_dbl, dim3(waves), dim3(64), 0, 0, d, n);
    hipEventRecord(e1);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long seg[8];
    hipMemcpyFromSymbol(seg, HIP_SYMBOL(g_seg), sizeof(seg));
    unsigned long long tot = 0;
    for (int k = 1; k < 8; k++) tot += seg[k];
    printf("== %d wave(s), %d dependent doublings: %.3f ms = %.2f us per doubling\n", waves, n, ms, 1e3 * ms / n);
    for (int k = 1; k < 8; k++)
      printf("  %-24s %8.1f cycles per doubling (%4.1f %%)\n", names[k], (double)seg[k] / n, 100.0 * seg[k] / tot);
  }
  return 0;
}
