// The coin's combine_signatures kernel (k_combine_sigs, hbx_kernels.hip) split into its phases at
// the C4 size (256 instances, t = 43 of n = 128 shares, one 256-thread block per instance:
// waves 0..2 the G2 sum over four psi-digit lanes per share, wave 3 the G1 master identity):
// wall-clock stamps (100 MHz) of block 0 after each phase, plus the whole launch by events.
// Inputs are arbitrary field elements (the instruction stream, not the value, is measured).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o combsig combsig.hip && ./combsig
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../hbbft_amd/csrc/curve.hpp"

using namespace hbx;

constexpr int TH = 256, G2T = TH - 64, T = 43, NS = 128, MAXST = 8;

__device__ fq seed_fq(uint32_t s) {
  fq a;
  for (int i = 0; i < 12; i++) a.l[i] = (s * 2654435761u + i * 40503u) & (i == 11 ? 0x0fffffffu : 0xffffffffu);
  return a;
}
#define STAMP(k)                                                            \
  do {                                                                      \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) st[(threadIdx.x >> 6) * MAXST + (k)] = wall_clock64(); \
  } while (0)

__device__ fr lag(const uint16_t* idx, int t, int k) {
  fr num = fr_from_const(FR_ONE), den = fr_from_const(FR_ONE);
  fr xk;
  for (int q = 0; q < 8; q++) xk.l[q] = 0;
  xk.l[0] = (uint32_t)idx[k] + 1;
  xk = fr_to_mont(xk);
  for (int m = 0; m < t; m++) {
    if (m == k) continue;
    fr xm;
    for (int q = 0; q < 8; q++) xm.l[q] = 0;
    xm.l[0] = (uint32_t)idx[m] + 1;
    xm = fr_to_mont(xm);
    num = fr_mul(num, xm);
    den = fr_mul(den, fr_sub(xm, xk));
  }
  return fr_from_mont(fr_mul(num, fr_inv(den)));
}
__device__ void digits(const uint32_t* lam, uint64_t* d) {
  uint32_t v[8];
  for (int i = 0; i < 8; i++) v[i] = lam[i];
  for (int q = 0; q < 4; q++) {
    uint64_t rem = 0;
    for (int bit = 255; bit >= 0; bit--) {
      const uint32_t w = (uint32_t)bit >> 5, sh = (uint32_t)bit & 31;
      const uint64_t top = rem >> 63;
      rem = (rem << 1) | ((v[w] >> sh) & 1u);
      const bool ge = top != 0 || rem >= BLS_X;
      if (ge) rem -= BLS_X;
      v[w] = (v[w] & ~(1u << sh)) | ((ge ? 1u : 0u) << sh);
    }
    d[q] = rem;
  }
}
__device__ fq fq_shfl(const fq& a, int m) {
  fq r;
  for (int i = 0; i < 12; i++) r.l[i] = (uint32_t)__shfl_xor((int)a.l[i], m);
  return r;
}

__global__ void __launch_bounds__(TH) k_cs(uint64_t* st, uint32_t* out) {
  __shared__ uint16_t idx[T];
  __shared__ fr lam_s[T];
  __shared__ g2j red2[G2T / 64];
  const int tid = threadIdx.x;
  STAMP(0);
  if (tid < T) idx[tid] = (uint16_t)(3 * tid + (blockIdx.x & 1));
  __syncthreads();
  for (int k = tid; k < T; k += TH) lam_s[k] = lag(idx, T, k);
  __syncthreads();
  STAMP(1);
  g2j acc2 = g2_identity();
  g1j acc1 = g1_identity();
  if (tid >= G2T) {
    for (int q = tid - G2T; q < 4 * T; q += 64) {
      const fr lam = lam_s[q >> 2];
      uint32_t kk[2][4];
      g1_glv_split(lam.l, kk[0], kk[1]);
      const uint32_t* kh = kk[(q >> 1) & 1];
      const uint64_t piece = (q & 1) ? ((uint64_t)kh[3] << 32 | kh[2]) : ((uint64_t)kh[1] << 32 | kh[0]);
      const g1a pp{seed_fq(q + 5), seed_fq(q + 9), false};
      if (piece != 0) acc1 = g1_add(acc1, g1_mul_u64_w4(pp, piece));
    }
    STAMP(2);
    for (int m = 1; m < 64; m <<= 1) acc1 = g1_add(acc1, g1j{fq_shfl(acc1.x, m), fq_shfl(acc1.y, m), fq_shfl(acc1.z, m)});
    STAMP(3);
  } else {
    uint64_t d[4] = {0, 0, 0, 0};
    const int q = tid;
    if (q < 4 * T) digits(lam_s[q >> 2].l, d);
    STAMP(2);
    if (q < 4 * T) {
      g2j P = g2_from_affine(g2a{fq2{seed_fq(q), seed_fq(q + 1)}, fq2{seed_fq(q + 2), seed_fq(q + 3)}, false});
      for (int e = 0; e < (q & 3); e++) P = g2_psi(P);
      const g2a Pa{P.x, (q & 1) ? fq2_neg(P.y) : P.y, false};
      acc2 = g2_mul_u64_naf(Pa, d[q & 3] | 1u);
    }
    STAMP(3);
    for (int m = 1; m < 64; m <<= 1) {
      const g2j o{fq2{fq_shfl(acc2.x.c0, m), fq_shfl(acc2.x.c1, m)}, fq2{fq_shfl(acc2.y.c0, m), fq_shfl(acc2.y.c1, m)},
                  fq2{fq_shfl(acc2.z.c0, m), fq_shfl(acc2.z.c1, m)}};
      acc2 = g2_add(acc2, o);
    }
    if ((tid & 63) == 0) red2[tid >> 6] = acc2;
    STAMP(4);
  }
  __syncthreads();
  if (tid == 0) {
    g2j sum = red2[0];
    for (int w = 1; w < G2T / 64; w++) sum = g2_add(sum, red2[w]);
    out[blockIdx.x] = g2_to_affine(sum).x.c0.l[0] ^ acc1.x.l[0];
  }
  STAMP(5);
}

// the pieces alone on one wave per SIMD (1024 blocks of 64): a 64-bit G2 NAF multiplication, a
// G2 doubling chain of 64, a 64-bit G1 4-bit-window multiplication
template <int K>
__global__ void __launch_bounds__(64) k_piece(uint32_t* out) {
  const uint32_t q = blockIdx.x * 64 + threadIdx.x;
  if (K == 0) {
    const g2a Pa{fq2{seed_fq(q), seed_fq(q + 1)}, fq2{seed_fq(q + 2), seed_fq(q + 3)}, false};
    out[q] = g2_mul_u64_naf(Pa, 0xd201000000010000ull ^ (q * 2654435761ull)).x.c0.l[0];
  } else if (K == 1) {
    g2j P = g2_from_affine(g2a{fq2{seed_fq(q), seed_fq(q + 1)}, fq2{seed_fq(q + 2), seed_fq(q + 3)}, false});
    for (int i = 0; i < 64; i++) P = g2_dbl(P);
    out[q] = P.x.c0.l[0];
  } else {
    const g1a pp{seed_fq(q + 5), seed_fq(q + 9), false};
    out[q] = g1_mul_u64_w4(pp, 0xd201000000010000ull ^ (q * 2654435761ull)).x.l[0];
  }
}

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                             \
    }                                                                       \
  } while (0)

int main() {
  uint64_t* d_st;
  uint32_t* d_out;
  CK(hipMalloc(&d_st, 4 * MAXST * 8));
  CK(hipMalloc(&d_out, 1024 * 64 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float ms = 0;
  for (int rep = 0; rep < 2; rep++) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_cs, dim3(256), dim3(TH), 0, 0, d_st, d_out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
  }
  uint64_t st[4 * MAXST];
  CK(hipMemcpy(st, d_st, sizeof(st), hipMemcpyDeviceToHost));
  printf("k_combine_sigs replica, 256 instances, t = %d: %.3f ms\n", T, ms);
  printf("  lambda (lagrange_at_zero)            %8.3f ms\n", (st[1] - st[0]) / 100e3);
  printf("  G2 wave 0: base-X digits             %8.3f ms\n", (st[2] - st[1]) / 100e3);
  printf("  G2 wave 0: 64-bit NAF multiplication %8.3f ms\n", (st[3] - st[2]) / 100e3);
  printf("  G2 wave 0: shuffle tree              %8.3f ms\n", (st[4] - st[3]) / 100e3);
  printf("  G1 wave 3: 3 x 64-bit mult + adds    %8.3f ms\n", (st[3 * MAXST + 2] - st[3 * MAXST + 1]) / 100e3);
  printf("  G1 wave 3: shuffle tree              %8.3f ms\n", (st[3 * MAXST + 3] - st[3 * MAXST + 2]) / 100e3);
  printf("  end of block 0 (thread 0 final sum)  %8.3f ms after start\n", (st[5] - st[0]) / 100e3);
  const char* nm[3] = {"G2 64-bit NAF mult", "G2 64 doublings", "G1 64-bit w4 mult"};
  for (int k = 0; k < 3; k++) {
    for (int rep = 0; rep < 2; rep++) {
      CK(hipEventRecord(a));
      if (k == 0) hipLaunchKernelGGL(k_piece<0>, dim3(1024), dim3(64), 0, 0, d_out);
      if (k == 1) hipLaunchKernelGGL(k_piece<1>, dim3(1024), dim3(64), 0, 0, d_out);
      if (k == 2) hipLaunchKernelGGL(k_piece<2>, dim3(1024), dim3(64), 0, 0, d_out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
    }
    printf("  alone, 1024 one-wave blocks: %-20s %8.3f ms\n", nm[k], ms);
  }
  return 0;
}
