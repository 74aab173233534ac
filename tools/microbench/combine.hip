// The Lagrange combine (k_combine, hbx_kernels.hip) split into its phases, one 256-thread block per
// proposer and 32 proposers (the shard-of-8 slice), t = 86 (N = 256): wall-clock stamps of block 0
// after each phase, so the ~2.6 ms of k_combine can be attributed.  Variants of the per-lane scalar
// multiplication are timed beside it.  Inputs are arbitrary field elements (the instruction stream,
// not the value, is measured).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../hbbft_amd/csrc/curve4.hpp"
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

// quads: one 4-lane group per GLV term, lambda once per share (LDS), quad tree reduction
constexpr int TH4 = 768, NQ = TH4 / 4;
__global__ void __launch_bounds__(TH4) k_comb4(uint64_t* st, uint32_t* out) {
  __shared__ fr xm[T];
  __shared__ fr nall;
  __shared__ uint32_t lk[T][8];
  __shared__ g1j red[256];
  const int tid = threadIdx.x, qd = tid >> 2, s = tid & 3;
  STAMP(0);
  for (int k = tid; k < T; k += TH4) {
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
  if (tid < T) {
    const fr xk = xm[tid];
    fr den = xk;
    for (int m = 0; m < T; m++)
      if (m != tid) den = fr_mul(den, fr_sub(xm[m], xk));
    lam = fr_mul(nall, den);
  }
  STAMP(2);
  if (tid < T) {
    lam = fr_from_mont(fr_inv(lam));
    uint32_t k1[4], k2[4];
    g1_glv_split(lam.l, k1, k2);
    for (int q = 0; q < 4; q++) {
      lk[tid][q] = k1[q];
      lk[tid][4 + q] = k2[q];
    }
  }
  STAMP(3);
  g1j acc = g1_identity();
  if (qd < 2 * T) {
    uint32_t kk[4];
    for (int q = 0; q < 4; q++) kk[q] = lk[qd >> 1][(qd & 1) * 4 + q];
    g1a sp{seed_fq(qd + 1000 * blockIdx.x), seed_fq(qd + 7), false};
    acc = g1_mul_u128_w4_q4(sp, kk, s);
  }
  STAMP(4);
  if (s == 0) red[qd] = acc;
  if (tid < 256 - NQ) red[NQ + tid] = g1_identity();
  __syncthreads();
  for (int stride = 128; stride > 0; stride >>= 1) {
    if (qd < stride) {
      const g1j r = g1_add_q4(red[qd], red[qd + stride], s);
      if (s == 0) red[qd] = r;
    }
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

// the quad product equals the one-lane product (same formulas): 64 terms, affine results compared
__global__ void __launch_bounds__(256) k_check(uint32_t* bad) {
  const int tid = threadIdx.x, qd = tid >> 2, s = tid & 3;
  uint32_t kk[4];
  for (int q = 0; q < 4; q++) kk[q] = (qd * 2654435761u + q * 97531u) ^ (q == 3 ? 0x80000000u : 0u);
  if (qd == 5) kk[3] = 0;  // short scalar
  const g1a sp{seed_fq(qd + 11), seed_fq(qd + 5), false};
  const g1a a = g1_to_affine(g1_mul_u128_w4_q4(sp, kk, s));
  const g1a b = g1_to_affine(g1_mul_u128_w4(sp, kk));
  if (!fq_eq(a.x, b.x) || !fq_eq(a.y, b.y) || a.inf != b.inf) atomicAdd(bad, 1u);
}

// the scalar multiplication alone, one wave per block, 352 blocks (<= 1 wave per SIMD): one lane
// per term vs a quad per term
template <int QUAD>
__global__ void __launch_bounds__(64) k_sm(uint32_t* out) {
  const int tid = threadIdx.x, qd = QUAD ? tid >> 2 : tid, s = tid & 3;
  uint32_t kk[4];
  for (int q = 0; q < 4; q++) kk[q] = (qd * 2654435761u + q * 97531u + blockIdx.x) | 0x10000000u;
  const g1a sp{seed_fq(qd + 11), seed_fq(qd + 5), false};
  const g1j r = QUAD ? g1_mul_u128_w4_q4(sp, kk, s) : g1_mul_u128_w4(sp, kk);
  out[blockIdx.x * 64 + tid] = r.x.l[0];
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
  auto kern = MODE == 2 ? k_comb4 : k_comb<MODE>;
  const int th = MODE == 2 ? TH4 : TH;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float ms = 0;
  for (int rep = 0; rep < 2; rep++) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(th), 0, 0, d_st, d_out);
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
  CK(hipMemset(d_out, 0, 4));
  hipLaunchKernelGGL(k_check, dim3(1), dim3(256), 0, 0, d_out);
  uint32_t bad = 1;
  CK(hipMemcpy(&bad, d_out, 4, hipMemcpyDeviceToHost));
  printf("quad vs one-lane scalar multiplication: %u of 256 lanes differ\n", bad);
  {
    uint32_t* d_big;
    CK(hipMalloc(&d_big, 1024 * 64 * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int blocks : {352, 1024}) {
      for (int quad = 0; quad < 2; quad++) {
        float ms = 0;
        for (int rep = 0; rep < 2; rep++) {
          CK(hipEventRecord(a));
          if (quad) hipLaunchKernelGGL(k_sm<1>, dim3(blocks), dim3(64), 0, 0, d_big);
          else hipLaunchKernelGGL(k_sm<0>, dim3(blocks), dim3(64), 0, 0, d_big);
          CK(hipEventRecord(b));
          CK(hipEventSynchronize(b));
          CK(hipEventElapsedTime(&ms, a, b));
        }
        printf("scalar mult alone, %s, %d one-wave blocks: %.3f ms\n", quad ? "quad per term" : "lane per term", blocks, ms);
      }
    }
  }
  if (run<0>("w4 window (k_combine)", 32, d_st, d_out)) return 1;
  if (run<0>("w4 window (k_combine)", 256, d_st, d_out)) return 1;
  if (run<1>("double-and-add", 32, d_st, d_out)) return 1;
  if (run<2>("quads (curve4.hpp)", 32, d_st, d_out)) return 1;
  if (run<2>("quads (curve4.hpp)", 256, d_st, d_out)) return 1;
  return 0;
}
