// Microbenchmark: SIMD issue rate of the share check's instruction classes at 1, 2 and 4 waves per
// SIMD (grid = 1024 x W one-wave blocks), and of the digit tower's Fq2 products themselves.
// Question it answers: is a lone wave per SIMD (the one-lane check at N=256: 1,024 waves) issue
// bound below what the SIMD sustains with two waves -- i.e. would a check over two lanes at two
// waves per SIMD raise the chip's multiply-add rate?
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o issue issue.hip && ./issue
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../hbbft_amd/csrc/fieldd.hpp"
using namespace hbx;
#define ITERS 2048

__global__ void __launch_bounds__(64) k_mad_u64(uint64_t* out, uint32_t a0) {
  uint32_t a = a0 + threadIdx.x, b = a0 ^ 0x9e3779b9u;
  uint64_t acc[8];
  for (int i = 0; i < 8; i++) acc[i] = i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = (uint64_t)a * (uint32_t)(b + i) + acc[i];
    a += 1;
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(64) k_mad_i64(uint64_t* out, uint32_t a0) {
  int32_t a = (int32_t)(a0 + threadIdx.x), b = (int32_t)(a0 ^ 0x9e3779b9u);
  int64_t acc[8];
  for (int i = 0; i < 8; i++) acc[i] = i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      int32_t bi = b + i;
      __asm__("" : "+v"(bi));
      acc[i] = (int64_t)a * (int64_t)bi + acc[i];
    }
    a += 1;
  }
  int64_t s = 0;
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}
__global__ void __launch_bounds__(64) k_add_u32(uint64_t* out, uint32_t a0) {
  uint32_t acc[8];
  uint32_t a = a0 + threadIdx.x;
  for (int i = 0; i < 8; i++) acc[i] = i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) __asm__ volatile("v_add_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(a));
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(64) k_ashr_i64(uint64_t* out, uint32_t a0) {
  int64_t acc[8];
  for (int i = 0; i < 8; i++) acc[i] = (int64_t)(i * 7 + threadIdx.x + a0) << 40;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) __asm__ volatile("v_ashrrev_i64 %0, 1, %0" : "+v"(acc[i]));
  }
  int64_t s = 0;
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}
__global__ void __launch_bounds__(64) k_lshl_add_u64(uint64_t* out, uint32_t a0) {
  uint64_t acc[8];
  uint64_t a = a0 + threadIdx.x;
  for (int i = 0; i < 8; i++) acc[i] = i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) __asm__ volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[i]) : "v"(a));
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// the real thing: a chain of fq2d_sqr / fq2d_mul (fieldd.hpp), CH independent chains per lane
template <int CH>
__global__ void __launch_bounds__(64) k_fq2d_sqr(uint64_t* out, uint32_t a0) {
  fq2d x[CH];
#pragma unroll
  for (int c = 0; c < CH; c++) {
    x[c] = fq2d{fqd_const(FQD_ONE), fqd_zero()};
    x[c].c1.d[0] = (int32_t)((a0 + threadIdx.x + 17 * c) & 0xFFFFF);
  }
  for (int it = 0; it < ITERS / 8; it++)
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = fq2d_sqr(x[c]);
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++)
#pragma unroll
    for (int k = 0; k < 14; k++) s ^= x[c].c0.d[k] ^ x[c].c1.d[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int CH>
__global__ void __launch_bounds__(64) k_fq2d_mul(uint64_t* out, uint32_t a0) {
  fq2d x[CH], y{fqd_const(FQD_ONE), fqd_const(FQD_ONE)};
#pragma unroll
  for (int c = 0; c < CH; c++) {
    x[c] = fq2d{fqd_const(FQD_ONE), fqd_zero()};
    x[c].c1.d[0] = (int32_t)((a0 + threadIdx.x + 17 * c) & 0xFFFFF);
  }
  y.c1.d[1] = (int32_t)(a0 & 0xFFF);
  for (int it = 0; it < ITERS / 8; it++)
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = fq2d_mul(x[c], y);
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++)
#pragma unroll
    for (int k = 0; k < 14; k++) s ^= x[c].c0.d[k] ^ x[c].c1.d[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint64_t*, uint32_t);
static void run(const char* name, kfn f, double ops_per_wave, int W) {
  const int blocks = 1024 * W;
  uint64_t* d;
  hipMalloc(&d, (size_t)blocks * 64 * 8);
  hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, d, 1u);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, d, 1u + r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // SIMD cycles per wave-operation at 2.4 GHz (all W waves of a SIMD counted)
  const double cyc = ms * 1e-3 / 5 * 2.4e9 / (W * ops_per_wave);
  printf("%-14s W=%d  %8.3f ms/launch  %7.2f SIMD-cycles per wave-op  (%.2f per wave-op of one wave)\n", name, W,
         ms / 5, cyc, cyc * W);
  hipFree(d);
}
int main() {
  for (int W = 1; W <= 4; W *= 2) {
    run("mad_u64_u32", k_mad_u64, 8.0 * ITERS, W);
    run("mad_i64_i32", k_mad_i64, 8.0 * ITERS, W);
    run("add_u32", k_add_u32, 8.0 * ITERS, W);
    run("ashrrev_i64", k_ashr_i64, 8.0 * ITERS, W);
    run("lshl_add_u64", k_lshl_add_u64, 8.0 * ITERS, W);
    run("fq2d_sqr x1", k_fq2d_sqr<1>, 1.0 * (ITERS / 8), W);
    run("fq2d_sqr x2", k_fq2d_sqr<2>, 2.0 * (ITERS / 8), W);
    run("fq2d_mul x1", k_fq2d_mul<1>, 1.0 * (ITERS / 8), W);
    run("fq2d_mul x2", k_fq2d_mul<2>, 2.0 * (ITERS / 8), W);
  }
  return 0;
}
