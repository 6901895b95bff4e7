// Cross-lane helpers of the row-parallel field code (bn254_row.h, fe25519_row.h): a 16-lane DPP
// row holds one field element, limb i in row lane i.  Device versions are DPP moves (row_newbcast,
// row_shr / row_shl with zero fill) and ds_bpermute; tests/cpp/row_emu.h defines the same names
// over 64-lane host vectors, so the arithmetic templates run unchanged as an exact host emulation.
#pragma once
#include <stdint.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#endif

#if defined(__HIPCC__)
#define RF_HD __device__ __forceinline__
#else
#define RF_HD inline
#endif

// ------------------------------------------------------------------------------ lane ops
#if defined(__HIPCC__)
template <int I>
RF_HD uint32_t rl_bcast(uint32_t x) {  // lane I of each row -> the whole row
  // row_newbcast writes every lane, so no "old" operand: update_dpp(0, ...) would cost a v_mov 0
  // per broadcast for a destination value no lane keeps
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150 + I, 0xF, 0xF, false);
}
template <int I>
RF_HD uint32_t rl_bcast_w(uint32_t x) {  // alias (fe25519_row.h)
  return rl_bcast<I>(x);
}
template <int I>
RF_HD uint32_t rl_shr(uint32_t x) {  // lane k <- lane k - I of the row, 0 below
  if (I == 0) return x;
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x110 + I, 0xF, 0xF, true);
}
template <int I>
RF_HD uint32_t rl_shl(uint32_t x) {  // lane k <- lane k + I of the row, 0 above
  if (I == 0) return x;
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x100 + I, 0xF, 0xF, true);
}
RF_HD uint32_t rl_index(uint32_t) { return __lane_id() & 15u; }
RF_HD uint32_t rl_row(uint32_t) { return __lane_id() >> 4; }
// every row's value to every row: r[s] = x of row s (same row lane), s = 0..3, by one
// v_permlane16_swap (odd rows of one copy <-> even rows of the other: [x0 x0 x2 x2] and
// [x1 x1 x3 x3]) and two v_permlane32_swap (upper <-> lower 32 lanes: [x0 x0 x0 x0] and
// [x2 x2 x2 x2] from the first, x1 / x3 from the second).  gfx950 VALU lane swaps: no LDS
// crossbar trip, no s_waitcnt.
RF_HD void rl_all_rows(uint32_t x, uint32_t* r) {
  const auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  const auto q0 = __builtin_amdgcn_permlane32_swap(p[0], p[0], false, false);
  const auto q1 = __builtin_amdgcn_permlane32_swap(p[1], p[1], false, false);
  r[0] = q0[0];
  r[1] = q1[0];
  r[2] = q0[1];
  r[3] = q1[1];
}
// the value the same row lane holds in row S (ds_bpermute: the LDS crossbar, no LDS memory)
template <int S>
RF_HD uint32_t rl_from_row(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((S << 6) | ((__lane_id() & 15u) << 2)), (int)x);
}
RF_HD uint32_t rf_lo(uint64_t w) { return (uint32_t)w; }
RF_HD uint32_t rf_hi(uint64_t w) { return (uint32_t)(w >> 32); }
RF_HD uint64_t rf_w(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }
RF_HD uint64_t rf_mad(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }
RF_HD uint32_t rf_sel(bool c, uint32_t a, uint32_t b) { return c ? a : b; }
RF_HD uint64_t rf_sel(bool c, uint64_t a, uint64_t b) { return c ? a : b; }
RF_HD uint32_t rf_const(uint32_t, uint32_t v) { return v; }
RF_HD uint64_t rf_const64(uint32_t, uint64_t v) { return v; }
// 64-bit lane shifts by 29 as 32-bit funnel shifts (v_alignbit_b32) of the register halves
RF_HD uint64_t rf_shr29(uint64_t w) {
  const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
  return (uint64_t)__builtin_amdgcn_alignbit(hi, lo, 29) | ((uint64_t)(hi >> 29) << 32);
}
RF_HD uint64_t rf_sra29(uint64_t w) {
  const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
  return (uint64_t)__builtin_amdgcn_alignbit(hi, lo, 29) | ((uint64_t)(uint32_t)((int32_t)hi >> 29) << 32);
}
RF_HD uint64_t rf_ballot(bool c) { return __ballot(c); }
RF_HD uint32_t rl_lane(uint32_t) { return __lane_id(); }
RF_HD uint64_t rf_widen(uint32_t x) { return x; }
RF_HD uint64_t rf_mul64(uint32_t a, uint32_t b) { return (uint64_t)a * b; }
RF_HD uint32_t rf_bit(uint64_t mask, uint32_t lane) { return (uint32_t)(mask >> lane) & 1u; }
#endif
