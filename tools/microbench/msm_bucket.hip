// The north_star's bucket MSM measured against the combine's current multi-scalar multiplication
// (VERDICT r3 item 7).  One proposer's PublicKeySet::decrypt at N = 256 is sum_k lambda_k S_k over
// t = 86 shares; after the GLV split (curve.hpp g1_glv_split) that is 172 points with 128-bit
// scalars.  Both kernels below compute exactly that sum, one block per proposer:
//   K_lane    the current method (k_combine): one lane per term, 4-bit fixed windows
//             (g1_mul_u128_w4: 128 doublings + 32 additions + 7 table additions), then an LDS tree
//             reduction (8 levels);
//   K_bucket  Pippenger with LDS-staged buckets: 4-bit windows -> 32 windows x 15 buckets, one lane
//             per (window, bucket) builds its bucket's term list in LDS and sums its points (mixed
//             additions); one lane per window forms sum_b b B_b by running sums (30 additions); lane
//             w doubles its window sum 4w times, and an LDS tree adds the 32 windows.
// The scalars and points are the same for both (valid points [s] g1', s seeded), and the results
// are compared.  Timed at 256 blocks (the whole N = 256 epoch) and 32 blocks (a shard-of-8 slice).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o msm_bucket msm_bucket.hip && ./msm_bucket
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../hbbft_amd/csrc/curve.hpp"

using namespace hbx;

constexpr int TERMS = 172;  // 2 x 86 GLV halves
constexpr int WIN = 32, BUCKETS = 15, CAP = 64;  // CAP: list slots per bucket (~11.5 expected)

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
      return 1;                                                                \
    }                                                                          \
  } while (0)

__device__ uint32_t mix(uint32_t a) {
  a ^= a >> 16;
  a *= 0x7feb352du;
  a ^= a >> 15;
  a *= 0x846ca68bu;
  return a ^ (a >> 16);
}

// inputs: points[p][TERMS] affine, scalars[p][TERMS][4]
__global__ void __launch_bounds__(64) k_setup(g1a* pts, uint32_t* sc, int blocks) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= blocks * TERMS) return;
  const g1a base{fq_from_const(G1_MGEN_X), fq_from_const(G1_MGEN_Y), false};
  uint32_t s[4] = {mix(i * 4 + 1) | 1u, mix(i * 4 + 2), 0, 0};
  pts[i] = g1_to_affine(g1_mul_u128_w4(base, s));
  for (int q = 0; q < 4; q++) sc[i * 4 + q] = mix(i * 4 + q + 977);
}

__global__ void __launch_bounds__(256) k_lane(const g1a* pts, const uint32_t* sc, fq* out) {
  __shared__ g1j red[256];
  const int tid = threadIdx.x;
  const size_t b0 = (size_t)blockIdx.x * TERMS;
  g1j acc = g1_identity();
  if (tid < TERMS) acc = g1_mul_u128_w4(pts[b0 + tid], sc + (b0 + tid) * 4);
  red[tid] = acc;
  __syncthreads();
  for (int stride = 128; stride > 0; stride >>= 1) {
    if (tid < stride) red[tid] = g1_add(red[tid], red[tid + stride]);
    __syncthreads();
  }
  if (tid == 0) out[blockIdx.x] = fq_canon(g1_to_affine(red[0]).x);
}

__global__ void __launch_bounds__(512) k_bucket(const g1a* pts, const uint32_t* sc, fq* out) {
  __shared__ g1a P[TERMS];
  __shared__ uint32_t S[TERMS][4];
  __shared__ uint8_t list[WIN * BUCKETS][CAP];
  __shared__ g1j B[WIN * BUCKETS];  // bucket sums, later the window sums in B[w * BUCKETS]
  const int tid = threadIdx.x;
  const size_t b0 = (size_t)blockIdx.x * TERMS;
  for (int k = tid; k < TERMS; k += 512) {
    P[k] = pts[b0 + k];
    for (int q = 0; q < 4; q++) S[k][q] = sc[(b0 + k) * 4 + q];
  }
  __syncthreads();
  // bucket (w, b + 1): its term list, then the sum of its points
  if (tid < WIN * BUCKETS) {
    const int w = tid / BUCKETS, b = tid % BUCKETS + 1;
    int cnt = 0;
    for (int k = 0; k < TERMS; k++) {
      const uint32_t d = (S[k][w >> 3] >> (4 * (w & 7))) & 15u;
      if ((int)d == b) {
        if (cnt == CAP) __builtin_trap();  // never at these sizes; a trap, not a silent wrong sum
        list[tid][cnt++] = (uint8_t)k;
      }
    }
    g1j acc = g1_identity();
    for (int q = 0; q < cnt; q++) acc = g1_add_mixed_i(acc, P[list[tid][q]]);
    B[tid] = acc;
  }
  __syncthreads();
  // window w: sum_b b B_b = sum over b of (B_15 + ... + B_b)
  g1j win = g1_identity();
  if (tid < WIN) {
    g1j run = g1_identity();
    for (int b = BUCKETS - 1; b >= 0; b--) {
      run = g1_add(run, B[tid * BUCKETS + b]);
      win = g1_add(win, run);
    }
    for (int i = 0; i < 4 * tid; i++) win = g1_dbl(win);  // 2^(4w) W_w
  }
  __syncthreads();
  if (tid < WIN) B[tid] = win;
  __syncthreads();
  for (int stride = WIN / 2; stride > 0; stride >>= 1) {
    if (tid < stride) B[tid] = g1_add(B[tid], B[tid + stride]);
    __syncthreads();
  }
  if (tid == 0) out[blockIdx.x] = fq_canon(g1_to_affine(B[0]).x);
}

int main() {
  const int maxb = 256;
  g1a* pts;
  uint32_t* sc;
  fq *o1, *o2;
  CK(hipMalloc(&pts, (size_t)maxb * TERMS * sizeof(g1a)));
  CK(hipMalloc(&sc, (size_t)maxb * TERMS * 16));
  CK(hipMalloc(&o1, maxb * sizeof(fq)));
  CK(hipMalloc(&o2, maxb * sizeof(fq)));
  hipLaunchKernelGGL(k_setup, dim3((maxb * TERMS + 63) / 64), dim3(64), 0, 0, pts, sc, maxb);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int blocks : {256, 32}) {
    for (int v = 0; v < 2; v++) {
      float best = 1e9f;
      for (int r = 0; r < 3; r++) {
        CK(hipEventRecord(e0));
        if (v == 0) hipLaunchKernelGGL(k_lane, dim3(blocks), dim3(256), 0, 0, pts, sc, o1);
        else hipLaunchKernelGGL(k_bucket, dim3(blocks), dim3(512), 0, 0, pts, sc, o2);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
      }
      printf("%-9s %3d proposers x %d terms: %8.3f ms\n", v ? "K_bucket" : "K_lane", blocks, TERMS, best);
    }
  }
  fq h1[maxb], h2[maxb];
  CK(hipMemcpy(h1, o1, sizeof(h1), hipMemcpyDeviceToHost));
  CK(hipMemcpy(h2, o2, sizeof(h2), hipMemcpyDeviceToHost));
  int diff = 0;
  for (int b = 0; b < 32; b++)
    for (int q = 0; q < 12; q++) diff += h1[b].l[q] != h2[b].l[q];
  printf("results of the two methods: %s (32 proposers compared)\n", diff ? "DIFFER" : "equal");
  return diff ? 1 : 0;
}
