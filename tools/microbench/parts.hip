// Pairing-check parts in isolation, one lane per check, 1024 waves (one per SIMD) like the N=256
// k_verify_shares launch: the fused Miller loop alone, the final exponentiation alone, a chain of
// Fq products, a chain of cyclotomic squarings.  For rocprofv3 --kernel-trace / --pmc (which part
// carries the SQ_WAIT_ANY cycles).  Inputs are arbitrary field elements: the instruction stream,
// not the value, is what is measured.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../hbbft_amd/csrc/pairing.hpp"
#ifndef PARTS_WAVES
#define PARTS_WAVES 1
#endif

using namespace hbx;

__device__ fq seed_fq(uint32_t s) {
  fq a;
  for (int i = 0; i < 12; i++) a.l[i] = (s * 2654435761u + i * 40503u) & (i == 11 ? 0x0fffffffu : 0xffffffffu);
  return a;
}

__global__ void __launch_bounds__(64, PARTS_WAVES) k_miller(const line_pre* lines, uint32_t* out) {
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  g1a P{seed_fq(t), seed_fq(t + 7), false}, Q{seed_fq(t + 3), seed_fq(t + 9), false};
  const fq12 f = miller_loop2(lines, P, true, lines + MILLER_LINES, Q, true);
  out[t] = f.c0.c0.c0.l[0] ^ f.c1.c2.c1.l[11];
}

__global__ void __launch_bounds__(64, PARTS_WAVES) k_finalexp(uint32_t* out) {
  __shared__ uint32_t gslots[144 * LDS_FQ12_STRIDE];
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  fq12 f;
  uint32_t* p = reinterpret_cast<uint32_t*>(&f);
  for (int i = 0; i < 144; i++) p[i] = (t * 2654435761u + i * 97u) & ((i % 12) == 11 ? 0x0fffffffu : 0xffffffffu);
  const fq12 r = final_exponentiation_lds(f, (lds_u32*)(gslots + threadIdx.x));
  out[t] = r.c0.c0.c0.l[0] ^ r.c1.c2.c1.l[11];
}

__global__ void __launch_bounds__(64) k_fqchain(uint32_t* out, int n) {
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  fq a = seed_fq(t), b = seed_fq(t + 1);
  for (int i = 0; i < n; i++) {
    a = fq_mul(a, b);
    b = fq_mul(b, a);
  }
  out[t] = a.l[0] ^ b.l[3];
}

__global__ void __launch_bounds__(64) k_cycsqr(uint32_t* out, int n) {
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  fq12 f;
  uint32_t* p = reinterpret_cast<uint32_t*>(&f);
  for (int i = 0; i < 144; i++) p[i] = (t * 2654435761u + i * 97u) & ((i % 12) == 11 ? 0x0fffffffu : 0xffffffffu);
#pragma unroll 1
  for (int i = 0; i < n; i++) f = fq12_cyclotomic_sqr_i(f);
  out[t] = f.c0.c0.c0.l[0] ^ f.c1.c2.c1.l[11];
}

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));               \
      return 1;                                                           \
    }                                                                     \
  } while (0)

int main() {
  const int blocks = 1024;  // 1024 waves of 64 lanes
  uint32_t* out;
  line_pre* lines;
  CK(hipMalloc(&out, blocks * 64 * 4));
  CK(hipMalloc(&lines, 2 * MILLER_LINES * sizeof(line_pre)));
  CK(hipMemset(lines, 0x11, 2 * MILLER_LINES * sizeof(line_pre)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float ms;
  const int NCHAIN = 2000, NCYC = 200;
  for (int rep = 0; rep < 2; rep++) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_miller, dim3(blocks), dim3(64), 0, 0, lines, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep) printf("miller_loop2        %8.3f ms\n", ms);
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_finalexp, dim3(blocks), dim3(64), 0, 0, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep) printf("final_exp_lds       %8.3f ms\n", ms);
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_fqchain, dim3(blocks), dim3(64), 0, 0, out, NCHAIN);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep) printf("fq_mul chain x%d   %8.3f ms  (%.3f us per fq_mul per lane)\n", 2 * NCHAIN, ms, ms * 1e3 / (2 * NCHAIN));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_cycsqr, dim3(blocks), dim3(64), 0, 0, out, NCYC);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep) printf("cyc_sqr x%d         %8.3f ms  (%.3f us per cyclotomic square)\n", NCYC, ms, ms * 1e3 / NCYC);
  }
  return 0;
}
