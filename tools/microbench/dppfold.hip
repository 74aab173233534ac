// Is a DPP row broadcast folded into a 32-bit VOP2 consumer exact on gfx950?  (VERDICT r5 item 2:
// with the group rounds' broadcasts unpinned the compiler combined `v_mov_b32_dpp t, s
// row_newbcast:K` + `v_add_u32 d, t, x` into one `v_add_u32_dpp d, s, x row_newbcast:K`, and the
// group addition's sums came out wrong; tools/microbench/addcmp.hip.)
//
// Every case computes, per lane, op(s[row lane K], x[own lane]) on distinct per-lane values, once
// through the unfolded pair (the reference: the VOP1 move with the broadcast, then the plain VOP2
// op) and once as the single DPP-modified VOP2 instruction, both as inline asm so the encodings are
// exactly the ones named.  Control cases: the same folds with quad_perm (the form the compiler
// also emits) and a row_newbcast move alone.  Prints, per case, the lanes whose folded result differs.
//   hipcc -O3 --offload-arch=gfx950 -o dppfold dppfold.hip && ./dppfold
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define NCASE 15
static const char* kName[NCASE] = {
    "v_add_u32_dpp    row_newbcast:1", "v_sub_u32_dpp    row_newbcast:1", "v_subrev_u32_dpp row_newbcast:1",
    "v_xor_b32_dpp    row_newbcast:1", "v_add_u32_dpp    row_newbcast:9", "v_add_u32_dpp    quad_perm:[1,1,1,1]",
    "v_sub_u32_dpp    quad_perm:[1,1,1,1]", "v_mov_b32_dpp    row_newbcast:1 (alone)",
    "v_add_u32_dpp    row_newbcast:1, src written by the previous VALU op, no wait states",
    "v_add_u32_dpp    row_newbcast:1, src written by the previous VALU op, s_nop 1",
    "v_subrev_u32_dpp quad_perm:[1,1,1,1]", "v_lshlrev_b32_dpp row_newbcast:1 (x << (bcast & 31))",
    "v_subrev_u32_dpp row_newbcast:1 vs x - s (no broadcast)",
    "v_add_u32_dpp    row_newbcast:3 bound_ctrl:1 (the compiler's fold)", "v_mov_b32_dpp    row_newbcast:3 bound_ctrl:1 (alone)"};

__global__ void k_dppfold(uint32_t* out_ref, uint32_t* out_fold) {
  const uint32_t lane = threadIdx.x;
  const uint32_t s = 0x01000193u * (lane + 1) ^ 0x5bd1e995u;  // distinct per lane
  const uint32_t x = 0x9e3779b9u * (lane + 7);
  uint32_t r[NCASE], f[NCASE], t;
  // reference: move with the broadcast, then the op on plain registers
  asm volatile("s_nop 4\n\tv_mov_b32_dpp %0, %1 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(t) : "v"(s));
  r[0] = t + x; r[1] = t - x; r[2] = x - t; r[3] = t ^ x; r[7] = t;
  asm volatile("s_nop 4\n\tv_mov_b32_dpp %0, %1 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(t) : "v"(s));
  r[4] = t + x;
  asm volatile("s_nop 4\n\tv_mov_b32_dpp %0, %1 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(t) : "v"(s));
  r[5] = t + x; r[6] = t - x;
  // folded: one DPP-modified VOP2 instruction (src0 through the DPP network)
  asm volatile("s_nop 4\n\tv_add_u32_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(f[0]) : "v"(s), "v"(x));
  asm volatile("s_nop 4\n\tv_sub_u32_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(f[1]) : "v"(s), "v"(x));
  asm volatile("s_nop 4\n\tv_subrev_u32_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(f[2]) : "v"(s), "v"(x));
  asm volatile("s_nop 4\n\tv_xor_b32_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(f[3]) : "v"(s), "v"(x));
  asm volatile("s_nop 4\n\tv_add_u32_dpp %0, %1, %2 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(f[4]) : "v"(s), "v"(x));
  asm volatile("s_nop 4\n\tv_add_u32_dpp %0, %1, %2 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(f[5]) : "v"(s), "v"(x));
  asm volatile("s_nop 4\n\tv_sub_u32_dpp %0, %1, %2 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(f[6]) : "v"(s), "v"(x));
  asm volatile("s_nop 4\n\tv_mov_b32_dpp %0, %1 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(f[7]) : "v"(s));
  // the DPP source written by the VALU instruction right before it (the hazard the ISA requires
  // two wait states for on GFX9): without, then with them
  uint32_t u;
  r[8] = r[9] = r[0] + 1u;  // (s + 1) of row lane 1, plus x
  asm volatile("s_nop 4\n\tv_add_u32 %1, 1, %2\n\tv_add_u32_dpp %0, %1, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\ts_nop 1"
               : "=&v"(f[8]), "=&v"(u) : "v"(s), "v"(x));
  asm volatile("s_nop 4\n\tv_add_u32 %1, 1, %2\n\ts_nop 1\n\tv_add_u32_dpp %0, %1, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\ts_nop 1"
               : "=&v"(f[9]), "=&v"(u) : "v"(s), "v"(x));
  // the rev forms: src0 (through DPP) is the SECOND operand of the operation
  asm volatile("s_nop 4\n\tv_mov_b32_dpp %0, %1 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(t) : "v"(s));
  r[10] = x - t;
  asm volatile("s_nop 4\n\tv_subrev_u32_dpp %0, %1, %2 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(f[10]) : "v"(s), "v"(x));
  asm volatile("s_nop 4\n\tv_mov_b32_dpp %0, %1 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(t) : "v"(s));
  r[11] = x << (t & 31u);
  asm volatile("s_nop 4\n\tv_lshlrev_b32_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(f[11]) : "v"(s), "v"(x));
  // what the folded subrev computed: compare with the subtraction WITHOUT the broadcast
  r[12] = x - s;
  f[12] = f[2];
  // the compiler's folded form (tools/microbench/addcmp.hip built with HBX_ROW_PIN=0): the move's
  // old = 0 became bound_ctrl:1 (disabled source lanes read 0) on the combined add
  asm volatile("s_nop 4\n\tv_mov_b32_dpp %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=&v"(t) : "v"(s));
  r[13] = t + x;
  r[14] = t;
  asm volatile("s_nop 4\n\tv_add_u32_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 1" : "=&v"(f[13]) : "v"(s), "v"(x));
  asm volatile("s_nop 4\n\tv_mov_b32_dpp %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 1" : "=&v"(f[14]) : "v"(s));
  for (int c = 0; c < NCASE; c++) {
    out_ref[c * 64 + lane] = r[c];
    out_fold[c * 64 + lane] = f[c];
  }
}

int main() {
  uint32_t *dr, *df;
  uint32_t hr[NCASE * 64], hf[NCASE * 64];
  if (hipMalloc(&dr, sizeof(hr)) != hipSuccess || hipMalloc(&df, sizeof(hf)) != hipSuccess) return 2;
  hipLaunchKernelGGL(k_dppfold, dim3(1), dim3(64), 0, 0, dr, df);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  if (hipMemcpy(hr, dr, sizeof(hr), hipMemcpyDeviceToHost) != hipSuccess) return 4;
  if (hipMemcpy(hf, df, sizeof(hf), hipMemcpyDeviceToHost) != hipSuccess) return 4;
  int bad_total = 0;
  for (int c = 0; c < NCASE; c++) {
    int bad = 0, first = -1;
    for (int l = 0; l < 64; l++)
      if (hr[c * 64 + l] != hf[c * 64 + l]) {
        bad++;
        if (first < 0) first = l;
      }
    bad_total += bad;
    printf("%-40s lanes differing: %2d", kName[c], bad);
    if (first >= 0)
      printf("  (lane %d: unfolded %08x folded %08x)", first, hr[c * 64 + first], hf[c * 64 + first]);
    printf("\n");
  }
  printf("%s\n", bad_total ? "FOLDED DPP DIFFERS" : "all folded forms exact");
  return 0;
}
