// The Lagrange combine (k_combine, hbx_kernels.hip) split into its phases, one 256-thread block per
// proposer and 32 proposers (the shard-of-8 slice), t = 86 (N = 256): wall-clock stamps of block 0
// after each phase, so the ~2.6 ms of k_combine can be attributed.  Variants of the per-lane scalar
// multiplication are timed beside it.  Inputs are arbitrary field elements (the instruction stream,
// not the value, is measured).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../hbbft_amd/csrc/curve.hpp"
#include "../../hbbft_amd/csrc/hash.hpp"

using namespace hbx;

constexpr int TH = 256, T = 86, MAXST = 8;

__device__ fq seed_fq(uint32_t s) {
  fq a;
  for (int i = 0; i < 12; i++) a.l[i] = (s * 2654435761u + i * 40503u) & (i == 11 ? 0x0fffffffu : 0xffffffffu);
  return a;
}

#define STAMP(k)                                                 \
  do {                                                           \
    __syncthreads();                                             \
    if (threadIdx.x == 0) st[blockIdx.x * MAXST + (k)] = wall_clock64(); \
  } while (0)

template <int MODE>
__global__ void __launch_bounds__(TH) k_comb(uint64_t* st, uint32_t* out) {
  __shared__ fr xm[T];
  __shared__ fr nall;
  __shared__ g1j red[TH];
  const int tid = threadIdx.x;
  STAMP(0);
  for (int k = tid; k < T; k += TH) {
    fr x;
    for (int q = 0; q < 8; q++) x.l[q] = 0;
    x.l[0] = (uint32_t)(k * 3 + blockIdx.x) + 1;
    xm[k] = fr_to_mont(x);
  }
  __syncthreads();
  if (tid == 0) {
    fr nn = xm[0];
    for (int k = 1; k < T; k++) nn = fr_mul(nn, xm[k]);
    nall = nn;
  }
  STAMP(1);
  fr lam;
  for (int q = 0; q < 8; q++) lam.l[q] = 0;
  const int k = tid >> 1;
  if (tid < 2 * T) {
    const fr xk = xm[k];
    fr den = xk;
    for (int m = 0; m < T; m++)
      if (m != k) den = fr_mul(den, fr_sub(xm[m], xk));
    lam = fr_mul(nall, den);
  }
  STAMP(2);
  if (tid < 2 * T) lam = fr_from_mont(fr_inv(lam));
  STAMP(3);
  g1j acc = g1_identity();
  if (tid < 2 * T) {
    uint32_t k1[4], k2[4];
    g1_glv_split(lam.l, k1, k2);
    g1a sp{seed_fq(tid + 1000 * blockIdx.x), seed_fq(tid + 7), false};
    if (MODE == 0) acc = g1_mul_u128_w4(sp, (tid & 1) ? k2 : k1);
    else acc = g1_mul_u128(sp, (tid & 1) ? k2 : k1);
  }
  STAMP(4);
  red[tid] = acc;
  __syncthreads();
  for (int stride = TH / 2; stride > 0; stride >>= 1) {
    if (tid < stride) red[tid] = g1_add(red[tid], red[tid + stride]);
    __syncthreads();
  }
  STAMP(5);
  if (tid == 0) {
    const g1a g = g1_to_affine(red[0]);
    uint8_t comp[48], d[32];
    g1_compress(g, comp);
    digest2(DIGEST_SHA256, comp, 48, nullptr, 0, d);
    out[blockIdx.x] = d[0] | (d[31] << 8);
  }
  STAMP(6);
}

#define CK(x)                                               \
  do {                                                      \
    hipError_t e_ = (x);                                    \
    if (e_ != hipSuccess) {                                 \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_)); \
      return 1;                                             \
    }                                                       \
  } while (0)

template <int MODE>
int run(const char* name, int blocks, uint64_t* d_st, uint32_t* d_out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float ms = 0;
  for (int rep = 0; rep < 2; rep++) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_comb<MODE>, dim3(blocks), dim3(TH), 0, 0, d_st, d_out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
  }
  uint64_t st[MAXST];
  CK(hipMemcpy(st, d_st, sizeof(st), hipMemcpyDeviceToHost));
  const char* ph[6] = {"x_k + numerator", "denominators (t-1 fr_mul)", "fr_inv + from_mont", "glv split + scalar mul",
                       "tree reduction (8 g1_add)", "to_affine + compress + sha"};
  printf("%s, %d blocks: %.3f ms\n", name, blocks, ms);
  for (int i = 0; i < 6; i++) printf("  %-28s %8.3f ms\n", ph[i], (st[i + 1] - st[i]) / 100e3);  // 100 MHz
  return 0;
}

int main() {
  uint64_t* d_st;
  uint32_t* d_out;
  CK(hipMalloc(&d_st, 256 * MAXST * 8));
  CK(hipMalloc(&d_out, 256 * 4));
  if (run<0>("w4 window (k_combine)", 32, d_st, d_out)) return 1;
  if (run<0>("w4 window (k_combine)", 256, d_st, d_out)) return 1;
  if (run<1>("double-and-add", 32, d_st, d_out)) return 1;
  return 0;
}
