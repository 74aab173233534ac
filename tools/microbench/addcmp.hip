// old (round16 arrays) vs new (fqd_pick) digit group addition on the same inputs
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../hbbft_amd/csrc/hash.hpp"
using namespace hbx;
__device__ fqd g_dbg[2][16][64];
__device__ __forceinline__ fqd fqd_sel16x(int s, const fqd (&v)[16]) {
  fqd r;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    int32_t t = v[0].d[i];
#pragma unroll
    for (int k = 1; k < 16; k++) t = (s == k) ? v[k].d[i] : t;
    r.d[i] = t;
  }
  return r;
}
struct round16x {
  fqd a[16], b[16];
};
__device__ __forceinline__ void r16x_mul(round16x& R, int k, const fq2d& x, const fq2d& y) {
  R.a[k] = x.c0; R.b[k] = y.c0;
  R.a[k + 1] = x.c1; R.b[k + 1] = y.c1;
  R.a[k + 2] = x.c0; R.b[k + 2] = y.c1;
  R.a[k + 3] = x.c1; R.b[k + 3] = y.c0;
}
__device__ __forceinline__ void r16x_sqr(round16x& R, int k, const fq2d& x) {
  R.a[k] = fqd_add(x.c0, x.c1); R.b[k] = fqd_sub(x.c0, x.c1);
  R.a[k + 1] = x.c0; R.b[k + 1] = x.c1;
}
__device__ __forceinline__ void r16x_clear(round16x& R) {
#pragma unroll
  for (int i = 0; i < 16; i++) {
    R.a[i] = fqd_zero();
    R.b[i] = fqd_zero();
  }
}
__device__ __forceinline__ fqd r16x_run(const round16x& R, int gl) { return fqd_mul(fqd_sel16x(gl, R.a), fqd_sel16x(gl, R.b)); }

// P + Q on the 16 lanes of a group (hash.hpp g2_add_group, add-2007-bl) in five rounds, the same
// special cases as g2_add by exact tests.  Relaxed in and out.
__device__ __forceinline__ g2jd g2d_add_old(const g2jd& p, const g2jd& q, int gl) {
  if (fq2d_is_zero_mod(p.z)) return q;
  if (fq2d_is_zero_mod(q.z)) return p;
  round16x R;
  r16x_clear(R);
  // round 1: Z1^2, Z2^2, Y1 Z2, Y2 Z1, (Z1 + Z2)^2
  r16x_sqr(R, 0, p.z);
  r16x_sqr(R, 2, q.z);
  r16x_mul(R, 4, p.y, q.z);
  r16x_mul(R, 8, q.y, p.z);
  r16x_sqr(R, 12, fq2d_relax(fq2d_add(p.z, q.z)));
  fqd r = r16x_run(R, gl);
  const fq2d Z1Z1 = rows_sqr<0>(r), Z2Z2 = rows_sqr<2>(r);
  const fq2d Y1Z2 = rows_mul<4>(r), Y2Z1 = rows_mul<8>(r);
  const fq2d ZS = rows_sqr<12>(r);
  g_dbg[0][8][threadIdx.x] = Z1Z1.c0; g_dbg[0][9][threadIdx.x] = Z2Z2.c0; g_dbg[0][10][threadIdx.x] = Y1Z2.c0; g_dbg[0][11][threadIdx.x] = Y2Z1.c0; g_dbg[0][12][threadIdx.x] = p.x.c0; g_dbg[0][13][threadIdx.x] = q.x.c0;
  g_dbg[0][0][threadIdx.x] = ZS.c0;
  // round 2: U1, U2, S1, S2
  r16x_mul(R, 0, p.x, Z2Z2);
  r16x_mul(R, 4, q.x, Z1Z1);
  r16x_mul(R, 8, Y1Z2, Z2Z2);
  r16x_mul(R, 12, Y2Z1, Z1Z1);
  r = r16x_run(R, gl);
  const fq2d U1 = rows_mul<0>(r), U2 = rows_mul<4>(r);
  const fq2d S1 = rows_mul<8>(r), S2 = rows_mul<12>(r);
  g_dbg[0][14][threadIdx.x] = U1.c0; g_dbg[0][15][threadIdx.x] = S1.c0;
  const fq2d H = fq2d_relax(fq2d_sub(U2, U1));
  const fq2d dS = fq2d_relax(fq2d_sub(S2, S1));
  g_dbg[0][2][threadIdx.x] = dS.c0;
  g_dbg[0][1][threadIdx.x] = H.c0;
  if (fq2d_is_zero_mod(H)) {
    if (fq2d_is_zero_mod(dS)) return g2d_dbl_group(p, gl);
    return g2d_identity();
  }
  const fq2d rr = fq2d_dbl(dS);
  // round 3: I = (2H)^2 = 4 H^2, r^2 = 4 dS^2, Z3 = ((Z1 + Z2)^2 - Z1Z1 - Z2Z2) H
  r16x_sqr(R, 0, H);
  r16x_sqr(R, 2, dS);
  r16x_mul(R, 4, fq2d_relax(fq2d_sub(fq2d_sub(ZS, Z1Z1), Z2Z2)), H);
  r = r16x_run(R, gl);
  const fq2d I = fq2d_dbl(fq2d_relax(fq2d_dbl(rows_sqr<0>(r))));
  const fq2d RR = fq2d_dbl(fq2d_relax(fq2d_dbl(rows_sqr<2>(r))));
  const fq2d Z3 = fq2d_relax(rows_mul<4>(r));
  g_dbg[0][4][threadIdx.x] = Z3.c0;
  g_dbg[0][3][threadIdx.x] = I.c0;
  // round 4: J = H I, V = U1 I
  r16x_mul(R, 0, H, I);
  r16x_mul(R, 4, U1, I);
  r = r16x_run(R, gl);
  const fq2d J = rows_mul<0>(r), V = rows_mul<4>(r);
  const fq2d X3 = fq2d_relax(fq2d_sub(fq2d_relax(fq2d_sub(RR, J)), fq2d_dbl(V)));
  g_dbg[0][6][threadIdx.x] = X3.c0;
  g_dbg[0][5][threadIdx.x] = J.c0;
  // round 5: r (V - X3), S1 J
  r16x_mul(R, 0, rr, fq2d_sub(V, X3));
  r16x_mul(R, 4, S1, J);
  r = r16x_run(R, gl);
  const fq2d Y3 = fq2d_relax(fq2d_sub(rows_mul<0>(r), fq2d_dbl(rows_mul<4>(r))));
  g_dbg[0][7][threadIdx.x] = Y3.c0;
  return g2jd{X3, Y3, Z3};
}
__device__ __forceinline__ g2jd g2d_add_new(const g2jd& p, const g2jd& q, int gl) {
  if (fq2d_is_zero_mod(p.z)) return q;
  if (fq2d_is_zero_mod(q.z)) return p;
  const fqd z = fqd_zero();
  // round 1: Z1^2 (0, 1), Z2^2 (2, 3), Y1 Z2 (4..7), Y2 Z1 (8..11), (Z1 + Z2)^2 (12, 13)
  fqd r;
  {
    const fq2d zs = fq2d_relax(fq2d_add(p.z, q.z));
    r = fqd_mul(fqd_pick(gl, GD_SQRA(p.z), GD_SQRA(q.z), GD_MULA(p.y), GD_MULA(q.y), GD_SQRA(zs), z, z),
                fqd_pick(gl, GD_SQRB(p.z), GD_SQRB(q.z), GD_MULB(q.z), GD_MULB(p.z), GD_SQRB(zs), z, z));
  }
  const fq2d Z1Z1 = rows_sqr<0>(r), Z2Z2 = rows_sqr<2>(r);
  const fq2d Y1Z2 = rows_mul<4>(r), Y2Z1 = rows_mul<8>(r);
  const fq2d ZS = rows_sqr<12>(r);
  g_dbg[1][8][threadIdx.x] = Z1Z1.c0; g_dbg[1][9][threadIdx.x] = Z2Z2.c0; g_dbg[1][10][threadIdx.x] = Y1Z2.c0; g_dbg[1][11][threadIdx.x] = Y2Z1.c0; g_dbg[1][12][threadIdx.x] = p.x.c0; g_dbg[1][13][threadIdx.x] = q.x.c0;
  g_dbg[1][0][threadIdx.x] = ZS.c0;
  // round 2: U1 (0..3), U2 (4..7), S1 (8..11), S2 (12..15)
  r = fqd_mul(fqd_pick(gl, GD_MULA(p.x), GD_MULA(q.x), GD_MULA(Y1Z2), GD_MULA(Y2Z1)),
              fqd_pick(gl, GD_MULB(Z2Z2), GD_MULB(Z1Z1), GD_MULB(Z2Z2), GD_MULB(Z1Z1)));
  const fq2d U1 = rows_mul<0>(r), S1 = rows_mul<8>(r);
  g_dbg[1][14][threadIdx.x] = U1.c0; g_dbg[1][15][threadIdx.x] = S1.c0;
  const fq2d H = fq2d_relax(fq2d_sub(rows_mul<4>(r), U1));
  const fq2d dS = fq2d_relax(fq2d_sub(rows_mul<12>(r), S1));
  g_dbg[1][2][threadIdx.x] = dS.c0;
  g_dbg[1][1][threadIdx.x] = H.c0;
  if (fq2d_is_zero_mod(H)) {
    if (fq2d_is_zero_mod(dS)) return g2d_dbl_group(p, gl);
    return g2d_identity();
  }
  const fq2d rr = fq2d_dbl(dS);
  // round 3: H^2 (0, 1), dS^2 (2, 3), ((Z1 + Z2)^2 - Z1Z1 - Z2Z2) H (4..7)
  {
    const fq2d zz = fq2d_relax(fq2d_sub(fq2d_sub(ZS, Z1Z1), Z2Z2));
    r = fqd_mul(fqd_pick(gl, GD_SQRA(H), GD_SQRA(dS), GD_MULA(zz), z, z, z, z, z, z, z, z),
                fqd_pick(gl, GD_SQRB(H), GD_SQRB(dS), GD_MULB(H), z, z, z, z, z, z, z, z));
  }
  const fq2d I = fq2d_dbl(fq2d_relax(fq2d_dbl(rows_sqr<0>(r))));   // (2H)^2
  const fq2d RR = fq2d_dbl(fq2d_relax(fq2d_dbl(rows_sqr<2>(r))));  // rr^2
  const fq2d Z3 = fq2d_relax(rows_mul<4>(r));
  g_dbg[1][4][threadIdx.x] = Z3.c0;
  g_dbg[1][3][threadIdx.x] = I.c0;
  // round 4: J = H I (0..3), V = U1 I (4..7)
  r = fqd_mul(fqd_pick(gl, GD_MULA(H), GD_MULA(U1), z, z, z, z, z, z, z, z),
              fqd_pick(gl, GD_MULB(I), GD_MULB(I), z, z, z, z, z, z, z, z));
  const fq2d J = rows_mul<0>(r), V = rows_mul<4>(r);
  const fq2d X3 = fq2d_relax(fq2d_sub(fq2d_relax(fq2d_sub(RR, J)), fq2d_dbl(V)));
  g_dbg[1][6][threadIdx.x] = X3.c0;
  g_dbg[1][5][threadIdx.x] = J.c0;
  // round 5: rr (V - X3) (0..3), S1 J (4..7)
  {
    const fq2d w = fq2d_sub(V, X3);
    r = fqd_mul(fqd_pick(gl, GD_MULA(rr), GD_MULA(S1), z, z, z, z, z, z, z, z),
                fqd_pick(gl, GD_MULB(w), GD_MULB(J), z, z, z, z, z, z, z, z));
  }
  const fq2d Y3 = fq2d_relax(fq2d_sub(rows_mul<0>(r), fq2d_dbl(rows_mul<4>(r))));
  g_dbg[1][7][threadIdx.x] = Y3.c0;
  return g2jd{X3, Y3, Z3};
}

__device__ int g_bad[8];
__device__ void chk(int round, const fqd& x, const fqd& y) {
  for (int i = 0; i < 14; i++)
    if (x.d[i] != y.d[i]) { atomicAdd(&g_bad[round], 1); return; }
}
__global__ void __launch_bounds__(64) k_cmp(const g2a* pts, g2a* out) {
  const int gl = (int)(threadIdx.x & 15);
  const int g = (int)(threadIdx.x >> 4);
  const fq2d one{fqd_const(FQD_ONE), fqd_zero()};
  const g2a a = pts[2 * g], b = pts[2 * g + 1];
  g2jd p{fq2d_from_fq2(a.x), fq2d_from_fq2(a.y), one};
  g2jd q{fq2d_from_fq2(b.x), fq2d_from_fq2(b.y), one};
  p = g2d_dbl_group(p, gl);
  q = g2d_dbl_group(g2d_dbl_group(q, gl), gl);
  const fqd z = fqd_zero();
  round16x R;
  r16x_clear(R);
  r16x_sqr(R, 0, p.z);
  r16x_sqr(R, 2, q.z);
  r16x_mul(R, 4, p.y, q.z);
  r16x_mul(R, 8, q.y, p.z);
  const fq2d zs = fq2d_relax(fq2d_add(p.z, q.z));
  r16x_sqr(R, 12, zs);
  const fqd oa = fqd_sel16x(gl, R.a), ob = fqd_sel16x(gl, R.b);
  const fqd na = fqd_pick(gl, GD_SQRA(p.z), GD_SQRA(q.z), GD_MULA(p.y), GD_MULA(q.y), GD_SQRA(zs), z, z);
  const fqd nb = fqd_pick(gl, GD_SQRB(p.z), GD_SQRB(q.z), GD_MULB(q.z), GD_MULB(p.z), GD_SQRB(zs), z, z);
  chk(0, oa, na);
  chk(1, ob, nb);
  const fqd ro = fqd_mul(oa, ob), rn = fqd_mul(na, nb);
  chk(2, ro, rn);
  chk(3, rows_mul<4>(ro).c0, rows_mul<4>(rn).c0);
  {
    const g2jd A = g2d_add_old(p, q, gl);
    const g2jd B = g2d_add_new(p, q, gl);
    if (gl == 0) out[g] = g2a{fq2d_to_fq2(A.x), fq2d_to_fq2(B.x), false};
  }
  {
    const fqd r = ro;
    const fq2d Z1Z1 = rows_sqr<0>(r), Z2Z2 = rows_sqr<2>(r);
    const fq2d Y1Z2 = rows_mul<4>(r), Y2Z1 = rows_mul<8>(r);
    r16x_mul(R, 0, p.x, Z2Z2);
    r16x_mul(R, 4, q.x, Z1Z1);
    r16x_mul(R, 8, Y1Z2, Z2Z2);
    r16x_mul(R, 12, Y2Z1, Z1Z1);
    const fqd oa2 = fqd_sel16x(gl, R.a), ob2 = fqd_sel16x(gl, R.b);
    const fqd na2 = fqd_pick(gl, GD_MULA(p.x), GD_MULA(q.x), GD_MULA(Y1Z2), GD_MULA(Y2Z1));
    const fqd nb2 = fqd_pick(gl, GD_MULB(Z2Z2), GD_MULB(Z1Z1), GD_MULB(Z2Z2), GD_MULB(Z1Z1));
    chk(4, oa2, na2);
    chk(5, ob2, nb2);
  }
}
int main() {
  g2a h[8], o[12];
  uint8_t* p = (uint8_t*)h;
  for (size_t i = 0; i < sizeof(h); i++) p[i] = (uint8_t)(i * 37 + 11);
  for (int k = 0; k < 8; k++) { h[k].inf = false; h[k].x.c0.l[11] &= 0xfff; h[k].x.c1.l[11] &= 0xfff; h[k].y.c0.l[11] &= 0xfff; h[k].y.c1.l[11] &= 0xfff; }
  g2a *d, *od;
  if (hipMalloc(&d, sizeof(h)) != hipSuccess || hipMalloc(&od, sizeof(o)) != hipSuccess) return 1;
  if (hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 1;
  hipLaunchKernelGGL(k_cmp, dim3(1), dim3(64), 0, 0, d, od);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  if (hipMemcpy(o, od, sizeof(o), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int hb[8];
  if (hipMemcpyFromSymbol(hb, HIP_SYMBOL(g_bad), sizeof(hb)) != hipSuccess) return 1;
  for (int k = 0; k < 6; k++) printf("check %d: %d lanes differ\n", k, hb[k]);
  int bad = hb[0] + hb[1] + hb[2] + hb[3];
  static fqd dbg[2][16][64];
  if (hipMemcpyFromSymbol(dbg, HIP_SYMBOL(g_dbg), sizeof(dbg)) != hipSuccess) return 1;
  const char* nm[8] = {"ZS", "H", "dS", "I", "Z3", "J", "X3", "Y3"};
  const char* nm2[16] = {"ZS", "H", "dS", "I", "Z3", "J", "X3", "Y3", "Z1Z1", "Z2Z2", "Y1Z2", "Y2Z1", "px", "qx", "U1", "S1"};
  for (int k = 0; k < 16; k++) {
    int nd = 0;
    for (int t = 0; t < 64; t++)
      for (int i = 0; i < 14; i++) nd += dbg[0][k][t].d[i] != dbg[1][k][t].d[i];
    printf("%-5s differing digits %d\n", nm2[k], nd);
  }
  return bad != 0;
}
