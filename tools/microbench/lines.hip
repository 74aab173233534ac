// k_prepare_lines' chain (hbx_kernels.hip g2_raw_lines_group: 63 grouped doubling steps + 5
// one-lane addition steps per G2 point, LINE_K = 16 lanes per point) with wall-clock stamps, on
// the shard-of-8 load: 64 points = 16 one-wave blocks.  Also the hash's grouped G2 doubling
// (hash.hpp g2_dbl_group) and a chain of dependent Fq products, for scale.  Inputs are arbitrary
// field elements (the instruction stream, not the value, is measured).
//
// Round 3 (profiles/r03l_microbench_lines.txt): 17.4 us per grouped doubling step (3 product
// rounds: ~5,600 instructions, of which ~1,600 are the products -- the 12-limb additions' carry
// chains, the 16-way selects and their wait states are the rest), 57.6 us per one-lane addition
// step, 9.9 us per hash doubling, 0.93 us per dependent product.  A digit-form (fieldd.hpp)
// version of both steps measured 15.4 us / doubling and 17.9 us / addition step, but its DPP
// row broadcasts gave wrong lines inside the full step (each round alone was exact; the same code
// with ds_bpermute exchanges was exact at 18.2 / 22.4 us): not adopted.
#include <hip/hip_runtime.h>
#include <cstdio>
#define HBX_TU 1
#include "../../hbbft_amd/csrc/hbx_kernels.hip"

using namespace hbx;

__device__ fq seed_fq(uint32_t s) {
  fq a;
  for (int i = 0; i < 12; i++) a.l[i] = (s * 2654435761u + i * 40503u) & (i == 11 ? 0x0fffffffu : 0xffffffffu);
  return a;
}

__global__ void __launch_bounds__(64) k_lines_parts(uint64_t* st, fq2* sink) {
  const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
  const int gl = (int)(gid % LINE_K);
  const int gbase = (int)(threadIdx.x & 63) - gl;
  const uint32_t k = gid / LINE_K;
  g2a Q{fq2{seed_fq(k), seed_fq(k + 1)}, fq2{seed_fq(k + 2), seed_fq(k + 3)}, false};
  g2j T = g2_from_affine(Q);
  fq2 acc = fq2_zero();
  if (threadIdx.x == 0) st[blockIdx.x * 8 + 0] = wall_clock64();
  for (int i = 0; i < 63; i++) {
    fq2 c0, c1, c2;
    line_dbl_step_group(T, c0, c1, c2, gl, gbase);
    acc = fq2_add(acc, c0);
  }
  if (threadIdx.x == 0) st[blockIdx.x * 8 + 1] = wall_clock64();
  for (int i = 0; i < 5; i++) {
    fq2 c0, c1, c2;
    line_add_step(T, Q, c0, c1, c2);
    acc = fq2_add(acc, c1);
  }
  if (threadIdx.x == 0) st[blockIdx.x * 8 + 2] = wall_clock64();
  g2j H = T;
  for (int i = 0; i < 63; i++) H = g2_dbl_group(H, gl, gbase);
  if (threadIdx.x == 0) st[blockIdx.x * 8 + 3] = wall_clock64();
  fq a = H.y.c0, b = H.z.c1;
  for (int i = 0; i < 100; i++) {
    a = fq_mul_inl(a, b);
    b = fq_mul_inl(b, a);
  }
  if (threadIdx.x == 0) st[blockIdx.x * 8 + 4] = wall_clock64();
  sink[gid] = fq2_add(acc, fq2_add(H.x, fq2{a, b}));
}

#define CK(x)                                               \
  do {                                                      \
    hipError_t e_ = (x);                                    \
    if (e_ != hipSuccess) {                                 \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_)); \
      return 1;                                             \
    }                                                       \
  } while (0)

int main() {
  uint64_t* d_st;
  fq2* d_sink;
  const int blocks = 16;
  CK(hipMalloc(&d_st, blocks * 8 * 8));
  CK(hipMalloc(&d_sink, blocks * 64 * sizeof(fq2)));
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_lines_parts, dim3(blocks), dim3(64), 0, 0, d_st, d_sink);
    CK(hipDeviceSynchronize());
  }
  uint64_t st[8];
  CK(hipMemcpy(st, d_st, sizeof(st), hipMemcpyDeviceToHost));
  printf("63 grouped line doubling steps  %8.3f ms (%.2f us / step)\n", (st[1] - st[0]) / 100e3, (st[1] - st[0]) / 100.0 / 63);
  printf("5 one-lane line addition steps  %8.3f ms (%.2f us / step)\n", (st[2] - st[1]) / 100e3, (st[2] - st[1]) / 100.0 / 5);
  printf("63 hash g2_dbl_group doublings  %8.3f ms (%.2f us / step)\n", (st[3] - st[2]) / 100e3, (st[3] - st[2]) / 100.0 / 63);
  printf("200 dependent fq_mul_inl         %8.3f ms (%.2f us / product)\n", (st[4] - st[3]) / 100e3, (st[4] - st[3]) / 100.0 / 200);
  return 0;
}
