// Where the two-lane coin check's time goes (k_verify_sig_shares2, hbx_kernels.hip): at the coin
// round's size (32,768 checks = 1,024 one-wave blocks of 32 pairs) time
//   K_ml   the per-lane Miller loop alone (miller_loop_mixed_d, one pair, lines generated),
//   K_full the Miller loop + the pair product + the two-lane final exponentiation,
//   K_ml1  the one-lane mixed Miller loop (prepared H lines + sigma's lines generated) on 512 waves,
// so FE2 = K_full - K_ml.  Inputs are arbitrary digit-form values (the instruction stream, not the
// value, is measured; no data-dependent branches on these paths).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o coin_parts coin_parts.hip && ./coin_parts
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../hbbft_amd/csrc/pairingd.hpp"
#include "../../hbbft_amd/csrc/pairing2d.hpp"

using namespace hbx;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
      return 1;                                                                \
    }                                                                          \
  } while (0)

__device__ fqd seed_fqd(uint32_t s) {
  fqd a;
  for (int i = 0; i < 13; i++) a.d[i] = (int32_t)((s * 2654435761u + (uint32_t)i * 40503u) & (uint32_t)DMASK);
  a.d[13] = (int32_t)((s * 97u) & 0xFFFFu);
  return a;
}

template <bool FULL>
__global__ void __launch_bounds__(64) k_coin2(uint32_t* out, uint32_t* gslot) {
  __shared__ uint32_t region[LDS2_DWORDS * 64];
  const int lane = (int)(threadIdx.x & 63);
  const bool l1 = (lane & 1) != 0;
  const uint32_t s = blockIdx.x * 64 + lane;
  const fq2d qx{seed_fqd(s), seed_fqd(s + 1)}, qy{seed_fqd(s + 2), seed_fqd(s + 3)};
  const fqd z = fqd_zero();
  const fq12d f = miller_loop_mixed_d(nullptr, z, z, false, qx, qy, seed_fqd(s + 5), seed_fqd(s + 6), true);
  if (!FULL) {
    uint32_t acc = 0;
    for (int i = 0; i < 14; i++) acc ^= (uint32_t)f.c0.c0.c0.d[i] ^ (uint32_t)f.c1.c2.c1.d[i];
    out[s] = acc;
    return;
  }
  lds_u32* reg = (lds_u32*)region;
  const int pl = lane & ~1;
  const slot2<lds_u32*> A{reg + pl, 64u}, B{reg + LDS_FQ6D_PACKED * 64 + pl, 64u};
  uint32_t* gb = gslot + (size_t)blockIdx.x * (2 * LDS_FQ6D_PACKED * 64) + pl;
  const slot2<uint32_t*> G1{gb, 64u}, G2{gb + LDS_FQ6D_PACKED * 64, 64u};
  const slot2<lds_u32*>& mine = l1 ? B : A;
  slot_put_fq6d(mine.half(0), mine.stride, fq6d_reduce(f.c0));
  slot_put_fq6d(mine.half(1), mine.stride, fq6d_reduce(f.c1));
  HBX_SEQ();
  op_mul(B, A, false, false, l1);
  HBX_SEQ();
  const bool v = final_exp2d_is_one(A, B, G1, G2, l1);
  out[s] = v ? 1u : 0u;
}

// one lane per check: prepared H lines (wave-uniform: one instance per block) + sigma generated
__global__ void __launch_bounds__(64) k_coin1(const line_pre_d* lines, uint32_t* out) {
  const int lane = (int)(threadIdx.x & 63);
  const uint32_t s = blockIdx.x * 64 + lane;
  const fq2d qx{seed_fqd(s), seed_fqd(s + 1)}, qy{seed_fqd(s + 2), seed_fqd(s + 3)};
  const fq12d f = miller_loop_mixed_d(lines + (size_t)(blockIdx.x >> 1) * MILLER_LINES, seed_fqd(s + 7), seed_fqd(s + 8),
                                      true, qx, qy, seed_fqd(s + 5), seed_fqd(s + 6), true);
  uint32_t acc = 0;
  for (int i = 0; i < 14; i++) acc ^= (uint32_t)f.c0.c0.c0.d[i] ^ (uint32_t)f.c1.c2.c1.d[i];
  out[s] = acc;
}

int main() {
  const int blocks2 = 1024, blocks1 = 512;
  uint32_t *out, *gslot;
  line_pre_d* lines;
  CK(hipMalloc(&out, (size_t)blocks2 * 64 * 4));
  CK(hipMalloc(&gslot, (size_t)blocks2 * 2 * LDS_FQ6D_PACKED * 64 * 4));
  CK(hipMalloc(&lines, (size_t)256 * MILLER_LINES * sizeof(line_pre_d)));
  CK(hipMemset(lines, 0x11, (size_t)256 * MILLER_LINES * sizeof(line_pre_d)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) -> int {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e9f;
    for (int r = 0; r < 3; r++) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("%-44s %8.3f ms\n", name, best);
    return 0;
  };
  timeit("K_ml   two-lane Miller only (1024 waves)", [&] { hipLaunchKernelGGL(k_coin2<false>, dim3(blocks2), dim3(64), 0, 0, out, gslot); });
  timeit("K_full two-lane Miller + pair mul + FE2", [&] { hipLaunchKernelGGL(k_coin2<true>, dim3(blocks2), dim3(64), 0, 0, out, gslot); });
  timeit("K_ml1  one-lane mixed Miller (512 waves)", [&] { hipLaunchKernelGGL(k_coin1, dim3(blocks1), dim3(64), 0, 0, lines, out); });
  CK(hipGetLastError());
  return 0;
}
