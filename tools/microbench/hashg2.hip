// hash_g2 latency by phase (HBX_PHASE hooks in hash.hpp): one 16-lane group per digest, 256
// digests like the N=256 prepare_ct launch; wall-clock stamps (100 MHz) of group 0's lane 0.
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ long long g_stamp[8];
#define HBX_PHASE(k)                                              \
  do {                                                            \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_stamp[k] = wall_clock64(); \
  } while (0)
#include "../../hbbft_amd/csrc/hash.hpp"
using namespace hbx;

__global__ void __launch_bounds__(64) k_hash(const uint8_t* digests, uint32_t count, g2a* out) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = gid / 16;
  if (j >= count) return;
  HBX_PHASE(0);
  g2j h;
  if (hash_g2_group<16>(digests + 32 * j, true, h, false)) {  // stops at h_eff P, as k_prepare_ct does
    const g2a a = g2_to_affine(h);
    out[j] = a;
  }
  HBX_PHASE(5);
}

int main() {
  const uint32_t count = 256;
  uint8_t* d;
  g2a* o;
  if (hipMalloc(&d, count * 32) != hipSuccess || hipMalloc(&o, count * sizeof(g2a)) != hipSuccess) return 1;
  uint8_t h[count * 32];
  for (uint32_t i = 0; i < count * 32; i++) h[i] = (uint8_t)(i * 131 + 7);
  if (hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 1;
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_hash, dim3(count * 16 / 64), dim3(64), 0, 0, d, count, o);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
  }
  long long st[8];
  if (hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamp), sizeof(st)) != hipSuccess) return 1;
  const char* names[6] = {"start", "drawn", "residuosity exp", "sqrt from norm", "cofactor clearing", "to_affine+store"};
  for (int k = 1; k < 6; k++) printf("%-20s %8.3f ms\n", names[k], (st[k] - st[k - 1]) / 100e3);
  printf("total                %8.3f ms\n", (st[5] - st[0]) / 100e3);
  // checksum of the affine results (builds with -DHBX_G2_GROUP_DIGITS=0/1 must agree)
  g2a* ho = new g2a[count];
  if (hipMemcpy(ho, o, count * sizeof(g2a), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  uint64_t sum = 0;
  for (uint32_t j = 0; j < count; j++) {
    const fq x = fq_canon(ho[j].x.c0), y = fq_canon(ho[j].y.c1);
    for (int q = 0; q < 12; q++) sum = sum * 1000003u + x.l[q] + 7u * y.l[q];
  }
  printf("checksum             %016llx\n", (unsigned long long)sum);
  return 0;
}
