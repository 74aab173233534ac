#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "/root/repo/hbbft_amd/csrc/field.hpp"
using namespace hbx;
#define ITERS 256
struct f28 { uint32_t l[14]; };
__constant__ uint32_t P28[14];
constexpr uint32_t M28 = (1u << 28) - 1;
__device__ __noinline__ f28 mul28(f28 a, f28 b, const uint32_t* __restrict__ P, uint32_t pinv) {
  uint32_t m[14];
  f28 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    const int jlo = k < 14 ? 0 : k - 13, jhi = k < 14 ? k : 13;
    uint64_t s1 = acc, s2 = 0;
#pragma unroll
    for (int j = jlo; j <= jhi; j++) s1 = (uint64_t)a.l[j] * b.l[k - j] + s1;
#pragma unroll
    for (int j = jlo; j <= jhi; j++) if (j < k) s2 = (uint64_t)m[j] * P[k - j] + s2;
    acc = s1 + s2;
    if (k < 14) {
      m[k] = ((uint32_t)acc * pinv) & M28;
      acc = (uint64_t)m[k] * P[0] + acc;
    } else {
      r.l[k - 14] = (uint32_t)acc & M28;
    }
    acc >>= 28;
  }
  r.l[13] = (uint32_t)acc;
  return r;
}
__global__ void __launch_bounds__(64) k_chain28(uint32_t* out, uint32_t seed, uint32_t pinv) {
  f28 x, y;
  for (int i = 0; i < 14; i++) { x.l[i] = (seed * 2654435761u + i * 40503u + threadIdx.x) & M28; y.l[i] = (seed * 97u + i) & M28; }
  x.l[13] &= 0xffff; y.l[13] &= 0xffff;
  for (int i = 0; i < ITERS; i++) x = mul28(x, y, P28, pinv);
  for (int k = 0; k < 14; k++) out[(blockIdx.x * 64 + threadIdx.x) * 14 + k] = x.l[k];
}
__global__ void __launch_bounds__(64) k_chain32(uint32_t* out, uint32_t seed, uint32_t pinv) {
  fq x = fq_one(), y = fq_one();
  x.l[0] ^= seed + threadIdx.x; y.l[1] ^= seed * 3;
  for (int i = 0; i < ITERS; i++) x = fq_mul(x, y);
  for (int k = 0; k < 12; k++) out[(blockIdx.x * 64 + threadIdx.x) * 14 + k] = x.l[k];
}
__global__ void __launch_bounds__(64) k_chain28x4(uint32_t* out, uint32_t seed, uint32_t pinv) {
  f28 x[4], y;
  for (int c = 0; c < 4; c++) for (int i = 0; i < 14; i++) x[c].l[i] = (seed * 2654435761u + i * 40503u + threadIdx.x + c) & M28;
  for (int i = 0; i < 14; i++) y.l[i] = (seed * 97u + i) & M28;
  for (int c = 0; c < 4; c++) x[c].l[13] &= 0xffff;
  y.l[13] &= 0xffff;
  for (int i = 0; i < ITERS; i++) for (int c = 0; c < 4; c++) x[c] = mul28(x[c], y, P28, pinv);
  for (int k = 0; k < 14; k++) out[(blockIdx.x * 64 + threadIdx.x) * 14 + k] = x[0].l[k] ^ x[1].l[k] ^ x[2].l[k] ^ x[3].l[k];
}
typedef void (*kfn)(uint32_t*, uint32_t, uint32_t);
static void run(const char* name, kfn f, int blocks, int chains, uint32_t pinv) {
  uint32_t* d; (void)hipMalloc(&d, (size_t)blocks * 64 * 56);
  hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, d, 1u, pinv);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, d, 2u, pinv);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  const double muls = (double)blocks * 64 * ITERS * chains;
  printf("%-10s waves=%6d  %8.3f ms  per-wave mul latency %.0f ns  chip %.3f T mul/s\n", name, blocks, ms,
         ms * 1e6 / (ITERS * chains), muls / (ms * 1e-3) / 1e12);
  (void)hipFree(d);
}
int main() {
  // p in base 2^28
  const char* ph = "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab";
  unsigned __int128 dummy = 0; (void)dummy;
  uint32_t p32[12] = {0};
  for (int i = 0; i < 96; i++) { char c = ph[95 - i]; uint32_t v = c <= '9' ? c - '0' : c - 'a' + 10; p32[i / 8] |= v << (4 * (i % 8)); }
  uint32_t p28[14] = {0};
  for (int bit = 0; bit < 384; bit++) if ((p32[bit / 32] >> (bit % 32)) & 1) p28[bit / 28] |= 1u << (bit % 28);
  // pinv = -p^-1 mod 2^28
  uint32_t inv = 1; for (int i = 0; i < 5; i++) inv *= 2 - p28[0] * inv;
  const uint32_t pinv = (0u - inv) & M28;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(P28), p28, sizeof p28);
  run("chain32", k_chain32, 1024, 1, pinv);
  run("chain28", k_chain28, 1024, 1, pinv);
  run("chain28x4", k_chain28x4, 1024, 4, pinv);
  run("chain32", k_chain32, 4096, 1, pinv);
  run("chain28", k_chain28, 4096, 1, pinv);
  return 0;
}
