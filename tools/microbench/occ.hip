// Occupancy microbenchmark: chip throughput of the engine's Fq product (field.hpp fq_mul, the
// 28-bit digit-sliced Montgomery product) and of Fq additions at 1, 2 and 4 waves per SIMD, and
// with 1 or 2 independent chains per lane.  Question it answers: does a second wave on a SIMD
// (or a second independent chain in one lane) raise the issue rate of the product, i.e. is a
// lane-split share check (2 lanes per check -> 2 waves per SIMD at N=256) worth building?
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o occ occ.hip && ./occ
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../hbbft_amd/csrc/field.hpp"
using namespace hbx;
#define ITERS 512

template <int CH>
__global__ void __launch_bounds__(64) k_mul(uint32_t* out, uint32_t seed) {
  fq x[CH], y = fq_one();
  for (int c = 0; c < CH; c++) {
    x[c] = fq_one();
    x[c].l[0] ^= seed + threadIdx.x + 17 * c;
  }
  y.l[1] ^= seed * 3;
  for (int i = 0; i < ITERS; i++)
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = fq_mul(x[c], y);
  uint32_t s = 0;
  for (int c = 0; c < CH; c++)
    for (int k = 0; k < 12; k++) s ^= x[c].l[k];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int CH>
__global__ void __launch_bounds__(64) k_add(uint32_t* out, uint32_t seed) {
  fq x[CH], y = fq_one();
  for (int c = 0; c < CH; c++) {
    x[c] = fq_one();
    x[c].l[0] ^= seed + threadIdx.x + 17 * c;
  }
  y.l[1] ^= seed * 3;
  for (int i = 0; i < ITERS * 8; i++)
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = fq_sub(fq_add(x[c], y), x[c ^ (CH > 1)]);
  uint32_t s = 0;
  for (int c = 0; c < CH; c++)
    for (int k = 0; k < 12; k++) s ^= x[c].l[k];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

typedef void (*kfn)(uint32_t*, uint32_t);
static void run(const char* name, kfn f, int waves, double ops_per_lane) {
  uint32_t* d;
  (void)hipMalloc(&d, (size_t)waves * 64 * 4);
  hipLaunchKernelGGL(f, dim3(waves), dim3(64), 0, 0, d, 1u);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int r = 0; r < 3; r++) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(f, dim3(waves), dim3(64), 0, 0, d, 2u + r);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  const double ops = (double)waves * 64 * ops_per_lane;
  printf("%-12s waves=%5d (%.0f/SIMD)  %8.3f ms  chip %.3f T op/s  per-wave op latency %.0f ns\n", name, waves,
         waves / 1024.0, best, ops / (best * 1e-3) / 1e12, best * 1e6 / ops_per_lane);
  (void)hipFree(d);
}

int main() {
  for (int w : {1024, 2048, 4096}) {
    run("mul x1", k_mul<1>, w, ITERS);
    run("mul x2", k_mul<2>, w, 2.0 * ITERS);
    run("add+sub x1", k_add<1>, w, 8.0 * ITERS);
    run("add+sub x2", k_add<2>, w, 16.0 * ITERS);
  }
  return 0;
}
