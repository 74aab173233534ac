// Latency of the hash chain's group operations in the digit tower (groupd.hpp): one 16-lane group
// running n dependent doublings, n dependent additions (acc + P), and the cofactor clearing.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../hbbft_amd/csrc/hash.hpp"
using namespace hbx;

__global__ void __launch_bounds__(64) k_op(g2a* io, int n, int op) {
  const int gl = (int)(threadIdx.x & 15);
  const g2a q = io[blockIdx.x];
  const fq2d one{fqd_const(FQD_ONE), fqd_zero()};
  const g2jd P{fq2d_from_fq2(q.x), fq2d_from_fq2(q.y), one};
  g2jd acc = g2d_dbl_group(P, gl);
  if (op == 0) {
    for (int i = 0; i < n; i++) acc = g2d_dbl_group(acc, gl);
  } else if (op == 1) {
    for (int i = 0; i < n; i++) acc = g2d_add_group(acc, P, gl);
  } else {
    for (int i = 0; i < n; i++) acc = g2d_clear_cofactor_group(acc, gl, false);
  }
  const g2a a = g2_to_affine(g2jd_to_g2j(acc));
  if (threadIdx.x == 0) io[blockIdx.x] = a;
}

int main() {
  g2a* d;
  if (hipMalloc(&d, 64 * sizeof(g2a)) != hipSuccess) return 1;
  static g2a h[64];
  for (int i = 0; i < 64; i++) {
    fq2 x = fq2_one();
    x.c0.l[0] += (uint32_t)i;
    h[i] = g2a{x, fq2_add(fq2_one(), fq2_one()), false};
  }
  const char* names[3] = {"doubling", "addition", "cofactor clearing (h_eff)"};
  const int ns[3] = {4096, 1024, 16};
  for (int op = 0; op < 3; op++) {
    if (hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_op, dim3(64), dim3(64), 0, 0, d, ns[op], op);
    hipEventRecord(e1);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %8.2f us each (%d dependent, 64 groups)\n", names[op], 1e3 * ms / ns[op], ns[op]);
  }
  return 0;
}
