// Developer tool: counts the Fq multiplications (squarings included) the kernels' algorithms
// perform per work unit, by running the same __host__ __device__ code on the CPU with a counter
// in fq_mul.  The counts are the "algorithmic work" of the roofline:
// MADs per unit = Fq-muls x 288 (12x12 product + 12x12 Montgomery reduction, 32-bit limbs).
// Not part of the product.
#define HBX_OPCOUNT 1
unsigned long long hbx_opcount_fqmul = 0;
#include <cstdio>
#include <cstring>
#include "../../hbbft_amd/csrc/pairing.hpp"
#include "../../hbbft_amd/csrc/pairingd.hpp"
#include "../../hbbft_amd/csrc/hash.hpp"
using namespace hbx;

static g1a g1gen() { g1a g; g.x = fq_from_const(G1_GEN_X); g.y = fq_from_const(G1_GEN_Y); g.inf = false; return g; }

int main() {
  // a G2 point: hash of a fixed digest
  uint8_t d[32];
  for (int i = 0; i < 32; i++) d[i] = (uint8_t)(i * 7 + 1);
  hbx_opcount_fqmul = 0;
  const g2a Q = g2_to_affine(hash_g2_from_digest(d));
  const unsigned long long c_hash = hbx_opcount_fqmul;
  static line_pre L1[MILLER_LINES], L2[MILLER_LINES];
  static fq2 scratch[2 * MILLER_LINES];
  hbx_opcount_fqmul = 0;
  g2_prepare_lines(Q, L1, scratch);
  const unsigned long long c_lines = hbx_opcount_fqmul;
  g2_prepare_lines(Q, L2, scratch);
  g1a P = g1gen();
  g1a nP = P;
  nP.y = fq_neg(nP.y);
  hbx_opcount_fqmul = 0;
  const fq12 f = miller_loop2(L1, P, true, L2, nP, true);
  const unsigned long long c_miller = hbx_opcount_fqmul;
  hbx_opcount_fqmul = 0;
  const bool ok = fq12_is_one(final_exponentiation(f));
  const unsigned long long c_fexp = hbx_opcount_fqmul;
  uint8_t comp[48];
  g1_compress(P, comp);
  hbx_opcount_fqmul = 0;
  g1a tmp;
  g1_decompress(comp, tmp);
  const unsigned long long c_dec = hbx_opcount_fqmul;
  uint32_t k[8];
  for (int i = 0; i < 8; i++) k[i] = 0x9e3779b9u * (i + 1);
  k[7] &= 0x3fffffffu;
  hbx_opcount_fqmul = 0;
  g1_to_affine(g1_mul_scalar(g1_from_affine(P), k));
  const unsigned long long c_g1mul = hbx_opcount_fqmul;
  // the share check as k_verify_shares runs it (digit tower; same algorithm, same count expected)
  static line_pre_d D1[MILLER_LINES], D2[MILLER_LINES];
  for (int i = 0; i < MILLER_LINES; i++) { D1[i] = line_to_d(L1[i]); D2[i] = line_to_d(L2[i]); }
  const fqd px = fqd_from_fq(P.x), py = fqd_from_fq(P.y), ny = fqd_from_fq(nP.y);
  hbx_opcount_fqmul = 0;
  const fq12d fdd = miller_loop2_d(D1, px, py, true, D2, px, ny, true);
  const unsigned long long c_miller_d = hbx_opcount_fqmul;
  static uint32_t slot[LDS_FQ12D_DWORDS];
  hbx_opcount_fqmul = 0;
  (void)final_exponentiation_d(fdd, slot);
  const unsigned long long c_fexp_d = hbx_opcount_fqmul;
  fprintf(stderr, "digit tower: miller %llu final_exp %llu (conversions and inversion included)\n", c_miller_d, c_fexp_d);
  // the coin's signature-share check: pair A over prepared lines, pair B's lines on the fly
  hbx_opcount_fqmul = 0;
  const fq12 fm = miller_loop_mixed(L1, P, true, Q, nP, true);
  const unsigned long long c_mixed = hbx_opcount_fqmul;
  hbx_opcount_fqmul = 0;
  (void)fq12_is_one(final_exponentiation(fm));
  const unsigned long long c_fexp2 = hbx_opcount_fqmul;
  printf("{\"check_ok\": %d, \"hash_g2\": %llu, \"prepare_lines\": %llu, \"miller_loop2\": %llu, "
         "\"final_exp\": %llu, \"g1_decompress\": %llu, \"g1_mul_255\": %llu, "
         "\"verify_share\": %llu, \"miller_loop_mixed\": %llu, \"verify_sig_share\": %llu}\n",
         ok ? 1 : 0, c_hash, c_lines, c_miller, c_fexp, c_dec, c_g1mul, c_dec + c_miller + c_fexp, c_mixed,
         c_mixed + c_fexp2);
  return 0;
}
