// Microbenchmark: latency / throughput of the kernels' fq_mul (12x32-bit CIOS Montgomery) on MI355X.
// chain1: one dependent chain per lane; chain4: four independent chains per lane (ILP).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../hbbft_amd/csrc/field.hpp"
using namespace hbx;
#define ITERS 256
__global__ void __launch_bounds__(64) k_chain1(uint32_t* out, uint32_t seed) {
  fq x = fq_one(), y = fq_one();
  x.l[0] ^= seed + threadIdx.x; y.l[1] ^= seed * 3;
  for (int i = 0; i < ITERS; i++) x = fq_mul(x, y);
  for (int k = 0; k < 12; k++) out[(blockIdx.x * 64 + threadIdx.x) * 12 + k] = x.l[k];
}
__global__ void __launch_bounds__(64) k_chain4(uint32_t* out, uint32_t seed) {
  fq x0 = fq_one(), x1 = fq_one(), x2 = fq_one(), x3 = fq_one(), y = fq_one();
  x0.l[0] ^= seed + threadIdx.x; x1.l[0] ^= seed + 7; x2.l[2] ^= seed; x3.l[3] ^= seed; y.l[1] ^= seed * 3;
  for (int i = 0; i < ITERS; i++) { x0 = fq_mul(x0, y); x1 = fq_mul(x1, y); x2 = fq_mul(x2, y); x3 = fq_mul(x3, y); }
  fq s = fq_add(fq_add(x0, x1), fq_add(x2, x3));
  for (int k = 0; k < 12; k++) out[(blockIdx.x * 64 + threadIdx.x) * 12 + k] = s.l[k];
}
typedef void (*kfn)(uint32_t*, uint32_t);
static void run(const char* name, kfn f, int blocks, int chains) {
  uint32_t* d; hipMalloc(&d, (size_t)blocks * 64 * 48);
  hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, d, 1u);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, d, 2u);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double muls = (double)blocks * 64 * ITERS * chains;
  printf("%-8s waves=%6d  %8.3f ms  per-wave fq_mul latency %.0f ns  chip %.3f T fq_mul/s = %.2f T MAD/s\n", name, blocks, ms,
         ms * 1e6 / (ITERS * chains), muls / (ms * 1e-3) / 1e12, muls * 288 / (ms * 1e-3) / 1e12);
  hipFree(d);
}
int main() {
  run("chain1", k_chain1, 1024, 1);
  run("chain1", k_chain1, 4096, 1);
  run("chain1", k_chain1, 16384, 1);
  run("chain4", k_chain4, 1024, 4);
  run("chain4", k_chain4, 4096, 4);
  return 0;
}
