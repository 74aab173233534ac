// A lane-group G2 doubling with digit-form operands (fieldd.hpp) where every addition is followed
// by at most ONE parallel carry step (fqd_relax: digits back under 2^28 + 8 in one VALU level, the
// value kept) instead of hash.hpp's 12-limb modular additions (two carry chains each): per-doubling
// latency of one 16-lane group against g2_dbl_group's, same points checked at the end.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../hbbft_amd/csrc/hash.hpp"
#include "../../hbbft_amd/csrc/g2d.hpp"
using namespace hbx;
// fqd_relax (fieldd.hpp), fqd_from_row / fqd_sel8 / rows_* (groupd.hpp): the helpers this
// prototype introduced, now in the headers

// inputs: relaxed digits (< 2^28 + 8), values < 2^386; outputs the same
__device__ __forceinline__ g2jd g2d_dbl_group_r(const g2jd& p, int gl) {
  const int s = gl & 7;
  const fqd x0 = p.x.c0, x1 = p.x.c1, y0 = p.y.c0, y1 = p.y.c1, z0 = p.z.c0, z1 = p.z.c1;
  fqd r = fqd_mul(fqd_sel8(s, fqd_add(x0, x1), x0, fqd_add(y0, y1), y0, y0, y1, y0, y1),
                  fqd_sel8(s, fqd_sub(x0, x1), x1, fqd_sub(y0, y1), y1, z0, z1, z1, z0));
  const fq2d A = rows_sqr<0>(r), B = rows_sqr<2>(r), YZ = rows_mul<4>(r);
  const fq2d S = fq2d_relax(fq2d_add(p.x, B));
  const fq2d E = fq2d_relax(fq2d_add(fq2d_dbl(A), A));
  r = fqd_mul(fqd_sel8(s, fqd_add(B.c0, B.c1), B.c0, fqd_add(S.c0, S.c1), S.c0, fqd_add(E.c0, E.c1), E.c0, E.c0, E.c0),
              fqd_sel8(s, fqd_sub(B.c0, B.c1), B.c1, fqd_sub(S.c0, S.c1), S.c1, fqd_sub(E.c0, E.c1), E.c1, E.c1, E.c1));
  const fq2d C = rows_sqr<0>(r), T = rows_sqr<2>(r), F = rows_sqr<4>(r);
  const fq2d D = fq2d_dbl(fq2d_relax(fq2d_sub(fq2d_sub(T, A), C)));
  const fq2d X3 = fq2d_relax(fq2d_sub(F, fq2d_dbl(D)));
  const fq2d G = fq2d_sub(D, X3);
  r = fqd_mul(fqd_sel8(s, E.c0, E.c1, E.c0, E.c1, E.c0, E.c1, E.c0, E.c1),
              fqd_sel8(s, G.c0, G.c1, G.c1, G.c0, G.c0, G.c1, G.c1, G.c0));
  const fq2d EG = rows_mul<0>(r);
  const fq2d C8 = fq2d_dbl(fq2d_dbl(fq2d_relax(fq2d_dbl(C))));
  return g2jd{X3, fq2d_relax(fq2d_sub(EG, C8)), fq2d_relax(fq2d_dbl(YZ))};
}

__global__ void __launch_bounds__(64) k_dbl12(g2a* io, int n) {
  const int lane = threadIdx.x & 63, gl = lane % 16, gbase = lane - gl;
  g2j p = g2_from_affine(io[blockIdx.x]);
  for (int i = 0; i < n; i++) p = g2_dbl_group(p, gl, gbase);
  const g2a a = g2_to_affine(p);
  if (lane == 0) io[blockIdx.x] = a;
}
__global__ void __launch_bounds__(64) k_dbld(g2a* io, int n) {
  const int lane = threadIdx.x & 63, gl = lane % 16;
  const g2a q = io[blockIdx.x];
  g2jd p{fq2d_from_fq2(q.x), fq2d_from_fq2(q.y), fq2d{fqd_const(FQD_ONE), fqd_zero()}};
  for (int i = 0; i < n; i++) p = g2d_dbl_group_r(p, gl);
  const g2a a = g2_to_affine(g2jd_to_g2j(p));
  if (lane == 0) io[blockIdx.x] = a;
}

int main() {
  const int n = 4096, waves = 64;
  g2a* d;
  if (hipMalloc(&d, 2 * waves * sizeof(g2a)) != hipSuccess) return 1;
  static g2a h[waves];
  for (int i = 0; i < waves; i++) {
    fq2 x = fq2_one();
    x.c0.l[0] += (uint32_t)i;  // any (x, y): doubling formulas do not need a curve point
    h[i] = g2a{x, fq2_add(fq2_one(), fq2_one()), false};
  }
  g2a out[2][waves];
  for (int v = 0; v < 2; v++) {
    if (hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    if (v == 0) hipLaunchKernelGGL(k_dbl12, dim3(waves), dim3(64), 0, 0, d, n);
    else hipLaunchKernelGGL(k_dbld, dim3(waves), dim3(64), 0, 0, d, n);
    hipEventRecord(e1);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-40s %8.3f ms = %6.2f us per doubling\n", v == 0 ? "12-limb g2_dbl_group" : "digit form, one-step carries",
           ms, 1e3 * ms / n);
    if (hipMemcpy(out[v], d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  }
  int same = 0;
  for (int i = 0; i < waves; i++) same += fq2_eq(out[0][i].x, out[1][i].x) && fq2_eq(out[0][i].y, out[1][i].y);
  printf("same affine points: %d of %d\n", same, waves);
  return 0;
}
