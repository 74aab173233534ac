// k_prepare_lines' chain (hbx_kernels.hip g2_raw_lines_group: 63 grouped doubling steps + 5
// one-lane addition steps per G2 point, LINE_K = 16 lanes per point) with wall-clock stamps, on
// the shard-of-8 load: 64 points = 16 one-wave blocks.  Also times the kernels of the hash
// (hash.hpp g2_dbl_group) step alone.  Inputs are arbitrary field elements.
#include <hip/hip_runtime.h>
#include <cstdio>
#define HBX_TU 1
#include "../../hbbft_amd/csrc/hbx_kernels.hip"

using namespace hbx;

__device__ fq seed_fq(uint32_t s) {
  fq a;
  for (int i = 0; i < 12; i++) a.l[i] = (s * 2654435761u + i * 40503u) & (i == 11 ? 0x0fffffffu : 0xffffffffu);
  return a;
}

// stamps: [0] start, [1] after the 63 doubling steps (no additions), [2] after 5 addition steps,
// [3] after 63 g2_dbl_group (hash) doublings
__global__ void __launch_bounds__(64) k_lines_parts(uint64_t* st, fq2* sink) {
  const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
  const int gl = (int)(gid % LINE_K);
  const int gbase = (int)(threadIdx.x & 63) - gl;
  const uint32_t k = gid / LINE_K;
  g2a Q{fq2{seed_fq(k), seed_fq(k + 1)}, fq2{seed_fq(k + 2), seed_fq(k + 3)}, false};
  const fq2d xq = fq2d_from_fq2(Q.x), yq = fq2d_from_fq2(Q.y);
  g2jd_t Td{xq, yq, fq2d{fqd_const(FQD_ONE), fqd_zero()}};
  fq2d accd{fqd_zero(), fqd_zero()};
  if (threadIdx.x == 0) st[blockIdx.x * 8 + 0] = wall_clock64();
#pragma unroll 1
  for (int i = 0; i < 63; i++) {
    fq2d c0, c1, c2;
    line_dbl_step_gd(Td, c0, c1, c2, gl);
    accd = fq2d_norm(fq2d_add(accd, c0));
  }
  if (threadIdx.x == 0) st[blockIdx.x * 8 + 1] = wall_clock64();
#pragma unroll 1
  for (int i = 0; i < 5; i++) {
    fq2d c0, c1, c2;
    line_add_step_gd(Td, xq, yq, c0, c1, c2, gl);
    accd = fq2d_norm(fq2d_add(accd, c1));
  }
  if (threadIdx.x == 0) st[blockIdx.x * 8 + 2] = wall_clock64();
  const fq2 acc = fq2d_to_fq2(accd);
  g2j H = g2j{fq2d_to_fq2(Td.x), fq2d_to_fq2(Td.y), fq2d_to_fq2(Td.z)};
  for (int i = 0; i < 63; i++) H = g2_dbl_group(H, gl, gbase);
  if (threadIdx.x == 0) st[blockIdx.x * 8 + 3] = wall_clock64();
  fq a = H.y.c0, b = H.z.c1;
  for (int i = 0; i < 100; i++) {
    a = fq_mul_inl(a, b);
    b = fq_mul_inl(b, a);
  }
  if (threadIdx.x == 0) st[blockIdx.x * 8 + 4] = wall_clock64();
  sink[gid] = fq2_add(acc, fq2_add(H.x, fq2{a, b}));
}

// device parity: the grouped digit steps' 68 raw lines against pairing.hpp g2_raw_lines (one lane)
// for the same point; per group, the first differing line index (-1 = none) after normalising
__global__ void __launch_bounds__(64, 1) k_lines_parity(int* first_bad, line_pre_d* raw, fq2d* rc2) {
  const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
  const int gl = (int)(gid % LINE_K);
  const uint32_t k = gid / LINE_K;
  g2a Q{fq2{seed_fq(k), seed_fq(k + 1)}, fq2{seed_fq(k + 2), seed_fq(k + 3)}, false};
  g2_raw_lines_group(Q, raw + (size_t)k * MILLER_LINES, rc2 + (size_t)k * MILLER_LINES, gl);
  if (gl != 0) return;
  line_pre a[MILLER_LINES];
  fq2 ca[MILLER_LINES];
  g2_raw_lines(Q, a, ca);
  int bad = -1;
  for (int i = MILLER_LINES - 1; i >= 0; i--) {
    const line_pre_d r = raw[(size_t)k * MILLER_LINES + i];
    line_pre l{fq2d_to_fq2(r.c0), fq2d_to_fq2(r.c1)};
    g2_normalise_line(l, fq2d_to_fq2(rc2[(size_t)k * MILLER_LINES + i]));
    g2_normalise_line(a[i], ca[i]);
    if (!fq2_eq(l.c0, a[i].c0) || !fq2_eq(l.c1, a[i].c1)) bad = i;
  }
  first_bad[k] = bad;
}

template <int K>
__device__ int row_bad(const rdres& r, const fqd (&a)[14], const fqd (&b)[14]) {
  const fqd g = fqd_from_row<K>(r), p = fqd_mul(a[K], b[K]);
  int bad = 0;
  for (int i = 0; i < 14; i++) bad |= g.d[i] != p.d[i];
  return bad << K;
}
__global__ void __launch_bounds__(64, 1) k_round_dbg(int* out) {
  const int gl = (int)(threadIdx.x % LINE_K);
  const fq2d x = fq2d_from_fq2(fq2{seed_fq(1), seed_fq(2)});
  const fq2d y = fq2d_from_fq2(fq2{seed_fq(3), seed_fq(4)});
  const fq2d z = fq2d_from_fq2(fq2{seed_fq(5), seed_fq(6)});
  const fqd x0 = x.c0, x1 = x.c1, y0 = y.c0, y1 = y.c1, z0 = z.c0, z1 = z.c1;
  const fqd a[14] = {fqd_add(x0, x1), x0, fqd_add(y0, y1), y0, fqd_add(z0, z1), z0, y0, y1, y0, y1, x0, x1, y0, z1};
  const fqd b[14] = {fqd_sub(x0, x1), x1, fqd_sub(y0, y1), y1, fqd_sub(z0, z1), z1, z0, z1, z1, z0, y1, x0, z0, x1};
  const rdres r = rd_run<14>(gl, a, b);
  out[threadIdx.x] = row_bad<0>(r, a, b) | row_bad<1>(r, a, b) | row_bad<2>(r, a, b) | row_bad<3>(r, a, b) |
                     row_bad<4>(r, a, b) | row_bad<5>(r, a, b) | row_bad<6>(r, a, b) | row_bad<7>(r, a, b) |
                     row_bad<8>(r, a, b) | row_bad<9>(r, a, b) | row_bad<10>(r, a, b) | row_bad<11>(r, a, b) |
                     row_bad<12>(r, a, b) | row_bad<13>(r, a, b);
}

#define CK(x)                                               \
  do {                                                      \
    hipError_t e_ = (x);                                    \
    if (e_ != hipSuccess) {                                 \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_)); \
      return 1;                                             \
    }                                                       \
  } while (0)

int main() {
  uint64_t* d_st;
  fq2* d_sink;
  const int blocks = 16;
  CK(hipMalloc(&d_st, blocks * 8 * 8));
  CK(hipMalloc(&d_sink, blocks * 64 * sizeof(fq2)));
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_lines_parts, dim3(blocks), dim3(64), 0, 0, d_st, d_sink);
    CK(hipDeviceSynchronize());
  }
  {
    int* d_bad;
    line_pre_d* d_raw;
    fq2d* d_c2;
    CK(hipMalloc(&d_bad, 64 * 4));
    CK(hipMalloc(&d_raw, 64 * MILLER_LINES * sizeof(line_pre_d)));
    CK(hipMalloc(&d_c2, 64 * MILLER_LINES * sizeof(fq2d)));
    hipLaunchKernelGGL(k_lines_parity, dim3(16), dim3(64), 0, 0, d_bad, d_raw, d_c2);
    CK(hipDeviceSynchronize());
    int bad[64];
    CK(hipMemcpy(bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost));
    printf("digit group lines vs g2_raw_lines, first differing line per point:");
    for (int i = 0; i < 64; i++) printf(" %d", bad[i]);
    printf("\n");
  }
  {
    int* d_o;
    CK(hipMalloc(&d_o, 64 * 4));
    hipLaunchKernelGGL(k_round_dbg, dim3(1), dim3(64), 0, 0, d_o);
    CK(hipDeviceSynchronize());
    int o[64];
    CK(hipMemcpy(o, d_o, sizeof(o), hipMemcpyDeviceToHost));
    printf("round debug: bitmask of wrong rows per lane:");
    for (int i = 0; i < 64; i++) printf(" %x", o[i]);
    printf("\n");
  }
  uint64_t st[8];
  CK(hipMemcpy(st, d_st, sizeof(st), hipMemcpyDeviceToHost));
  printf("63 grouped digit doubling steps  %8.3f ms (%.2f us / step)\n", (st[1] - st[0]) / 100e3, (st[1] - st[0]) / 100.0 / 63);
  printf("5 grouped digit addition steps  %8.3f ms (%.2f us / step)\n", (st[2] - st[1]) / 100e3, (st[2] - st[1]) / 100.0 / 5);
  printf("63 hash g2_dbl_group doublings  %8.3f ms (%.2f us / step)\n", (st[3] - st[2]) / 100e3, (st[3] - st[2]) / 100.0 / 63);
  printf("200 dependent fq_mul_inl         %8.3f ms (%.2f us / product)\n", (st[4] - st[3]) / 100e3, (st[4] - st[3]) / 100.0 / 200);
  return 0;
}
