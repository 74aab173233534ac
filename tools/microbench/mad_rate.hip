// Microbenchmark: per-CU issue rate of the integer/fp ops a 384-bit Montgomery multiply uses.
// Each lane runs independent chains (8 accumulators) so the loop is throughput-bound.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 4096
__global__ void k_mad64(uint64_t* out, uint32_t a0) {
  uint32_t a = a0 + threadIdx.x, b = a0 ^ 0x9e3779b9u;
  uint64_t acc[8];
  for (int i = 0; i < 8; i++) acc[i] = i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = (uint64_t)a * (uint32_t)(b + i) + acc[i];
    // prevent hoisting: perturb a slightly (1 extra add per 8 mads)
    a += 1;
  }
  uint64_t s = 0; for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mulhi(uint64_t* out, uint32_t a0) {
  uint32_t a = a0 + threadIdx.x;
  uint32_t acc[8];
  for (int i = 0; i < 8; i++) acc[i] = i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = __umulhi(acc[i], a) ;
    a += 1;
  }
  uint64_t s = 0; for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mullo(uint64_t* out, uint32_t a0) {
  uint32_t a = a0 + threadIdx.x;
  uint32_t acc[8];
  for (int i = 0; i < 8; i++) acc[i] = i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = acc[i] * a;
    a += 1;
  }
  uint64_t s = 0; for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fma64(uint64_t* out, uint32_t a0) {
  double a = 1.0000001 + threadIdx.x * 1e-9, b = 0.9999999;
  double acc[8];
  for (int i = 0; i < 8; i++) acc[i] = i + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = __builtin_fma(acc[i], a, b);
  }
  double s = 0; for (int i = 0; i < 8; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}
__global__ void k_addc(uint64_t* out, uint32_t a0) {
  // 32-bit add with carry chains: acc (64-bit) += a as u32 pairs -> v_add_co/v_addc_co
  uint64_t acc[8];
  uint64_t a = a0 + threadIdx.x;
  for (int i = 0; i < 8; i++) acc[i] = i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] += a;
    a ^= acc[it & 7];
  }
  uint64_t s = 0; for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_add32(uint64_t* out, uint32_t a0) {
  uint32_t acc[8];
  uint32_t a = a0 + threadIdx.x;
  for (int i = 0; i < 8; i++) acc[i] = i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = (acc[i] + a) ^ i;
  }
  uint64_t s = 0; for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
typedef void (*kfn)(uint64_t*, uint32_t);
static void run(const char* name, kfn f, double ops_per_lane_iter) {
  int blocks = 256 * 8, threads = 256;
  uint64_t* d; hipMalloc(&d, blocks * threads * 8);
  hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, 1u + r);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double ops = 5.0 * blocks * threads * (double)ITERS * ops_per_lane_iter;
  double rate = ops / (ms * 1e-3);
  printf("%-8s %8.3f ms  %.3f Tops/s  = %.1f lane-ops/clk/CU @2.4GHz\n", name, ms, rate / 1e12,
         rate / (256 * 2.4e9));
  hipFree(d);
}
int main() {
  run("mad64", k_mad64, 8);
  run("mulhi", k_mulhi, 8);
  run("mullo", k_mullo, 8);
  run("fma64", k_fma64, 8);
  run("add64", k_addc, 8);
  run("add32", k_add32, 8);
  return 0;
}
