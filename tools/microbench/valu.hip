// VALU issue-rate microbenchmark: v_perm_b32, v_bitop3_b32, v_xor_b32, v_alignbit_b32 and
// v_mad_u64_u32 chains (8 independent per lane), 4 waves per SIMD.  Prints lane-ops/s per op.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;

template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint32_t seed) {
  uint32_t v[8];
  for (int i = 0; i < 8; i++) v[i] = seed * (threadIdx.x + i + 1);
  const uint32_t s = seed ^ 0x03020100u;
#pragma unroll 1
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
#pragma unroll
      for (int i = 0; i < 8; i++) {
        if (OP == 0) v[i] = __builtin_amdgcn_perm(v[(i + 1) & 7], s, v[i] & 0x07070707u);
        if (OP == 1) v[i] = __builtin_amdgcn_bitop3_b32(v[i], v[(i + 1) & 7], s, 0x96);
        if (OP == 2) v[i] = v[i] ^ v[(i + 1) & 7];
        if (OP == 3) v[i] = __builtin_amdgcn_alignbit(v[i], v[(i + 1) & 7], 7);
        if (OP == 4) v[i] = (uint32_t)((uint64_t)v[i] * v[(i + 1) & 7] + s);
      }
    }
  }
  uint32_t acc = 0;
  for (int i = 0; i < 8; i++) acc ^= v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP>
static void run(const char* name, uint32_t* d, int blocks, int extra_per_op) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 7u);
  hipEventRecord(a);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 9u);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double ops = (double)blocks * 256 * ITERS * 64;  // 8 rounds x 8 chains
  printf("%-10s %8.3f ms  %7.2f T lane-ops/s (instr per op incl. %d helper)\n", name, ms, ops / (ms * 1e-3) / 1e12,
         extra_per_op);
}

int main() {
  uint32_t* d;
  const int blocks = 256 * 4;  // 4 blocks (16 waves) per CU = 4 waves per SIMD
  hipMalloc(&d, (size_t)blocks * 256 * 4);
  run<0>("v_perm", d, blocks, 1);  // + v_and for the selector
  run<1>("v_bitop3", d, blocks, 0);
  run<2>("v_xor", d, blocks, 0);
  run<3>("v_alignbit", d, blocks, 0);
  run<4>("mad_u64", d, blocks, 0);
  return 0;
}
