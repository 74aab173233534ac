// EXEC guards for the DPP lane exchanges.
//
// A DPP move reads its source lane through the crossbar only if that lane is active: with
// bound_ctrl = 0 a disabled source leaves the destination's `old` value, with bound_ctrl = 1 it
// reads 0 -- either way a silently wrong operand, where ds_bpermute would still have read the
// register.  Every DPP helper of the engine therefore requires that, for each ACTIVE lane, the lane
// it reads from is active too.  The check is on the wave-uniform EXEC mask in scalar registers
// (a few SALU instructions beside the VALU stream, no VALU work) and traps when it fails, so a
// build whose control flow breaks the precondition stops with a GPU trap instead of computing
// wrong lines (the failure of the reverted digit-form line preparation: DESIGN.md §5).
#pragma once
#include <stdint.h>

namespace hbx {
#if defined(__HIPCC__)
// every active lane of a group of G lanes (G = 2, 4 or 16; groups aligned) reads group lane K
template <int G, int K>
__device__ __forceinline__ void dpp_guard_src() {
  static_assert(G == 2 || G == 4 || G == 16, "DPP group");
  static_assert(K >= 0 && K < G, "group lane");
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr uint64_t lane0 = G == 2 ? 0x5555555555555555ull : G == 4 ? 0x1111111111111111ull : 0x0001000100010001ull;
  constexpr uint64_t fill = (G == 16 ? 0xFFFFull : (1ull << G) - 1);
  const uint64_t e = __builtin_amdgcn_read_exec();
  const uint64_t src = (e >> K) & lane0;  // group g's bit 0 = is its lane K active
  if (e & ~(src * fill)) __builtin_trap();
#endif
}
// the pair exchange (quad_perm [1, 0, 3, 2]): both lanes of a pair active, or neither
__device__ __forceinline__ void dpp_guard_pairs() {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t e = __builtin_amdgcn_read_exec();
  if (((e ^ (e >> 1)) & 0x5555555555555555ull) != 0) __builtin_trap();
#endif
}
#endif
}  // namespace hbx
