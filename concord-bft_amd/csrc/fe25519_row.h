// Row-parallel GF(2^255 - 19) for latency-bound chains (gfx950 device code, and a host SIMD
// emulation for tests): the R decode of the small-batch kernels (a square root: 254 squarings
// and 11 multiplications in series, ~80 % of a lone verify's decode wave).
//
// An element lives in ONE 16-lane DPP row: limb i (radix 2^29, the limbs of fe25519.h) in row
// lane i, lanes 9..15 zero.  A product is, per lane, 9 v_mad_u64_u32 (lane k accumulates column
// k = sum_i a_i b_(k-i): a_i by row_newbcast, b shifted by row_shr) + one for column 16, two carry
// passes over the columns, one fold of columns 9..17 into 0..8 (2^261 == 1216), one carry pass.
// That is ~11 mads and ~50 single-rate lane ops against the one-lane fe_sq's 55 mads and ~65
// ops (fe25519.h, ISA of ed25519_small_kernel): on a lone wave, which issues every instruction
// at its rate and waits on nothing else (fe25519.h notes), ~2x less time per squaring.
//
// Bounds (row lanes 0..8; lanes 9..15 are zero in every input and output):
//   "row-reduced"  limbs <= 2^29 + 2^23   (outputs of rfe_mul / rfe_sq / rfe_carry / rfe_sub)
//   "row-lazy"     limbs <= 2^30 + 2^24   (a sum of two row-reduced)
// rfe_mul takes row-reduced or row-lazy operands: a column is <= 9 (2^30 + 2^24)^2 < 2^63.3,
// carry pass 1 leaves limbs <= 2^29 + 2^34.3, pass 2 <= 2^29 + 2^6 (32-bit); column 16 + its
// carries <= 2^60.1, so its high part (column 17) is < 2^31.1; after the fold a lane holds
// <= 2^29 + 2^6 + 1216 * 2^31.1 < 2^41.4, and the last pass (lane 8's carry, weight 2^261, back
// into lane 0 times 1216) leaves lane 0 <= 2^29 + 1216 * 2^12.4 < 2^29 + 2^22.7, the others
// <= 2^29 + 2^12.4.  tests/test_fe_row.py checks the host emulation of every function here
// against Python integers mod p, with operands at these bounds.
#pragma once
#include "row_lanes.h"

#define RFE_MASK 0x1fffffffu

// r = a * b (mod p), row-reduced
template <class U, class W>
RF_HD U rfe_mul(U a, U b) {
  const U rl = rl_index(a);
  W col = rf_const64(a, 0ull);
#define RFE_PROD(I) col = rf_mad(rl_bcast_w<I>(a), rl_shr<I>(b), col);
  RFE_PROD(0) RFE_PROD(1) RFE_PROD(2) RFE_PROD(3) RFE_PROD(4) RFE_PROD(5) RFE_PROD(6) RFE_PROD(7) RFE_PROD(8)
#undef RFE_PROD
  W c16 = rf_mul64(rl_bcast_w<8>(a), rl_bcast_w<8>(b));  // column 16 (every lane)
  // carry pass 1 on 64-bit columns; lane 15's carry joins column 16
  const W cy = rf_shr29(col);
  const U cy_lo = rf_lo(cy), cy_hi = rf_hi(cy);
  c16 = c16 + rf_w(rl_bcast_w<15>(cy_lo), rl_bcast_w<15>(cy_hi));
  col = (col & rf_const64(a, (uint64_t)RFE_MASK)) + rf_w(rl_shr<1>(cy_lo), rl_shr<1>(cy_hi));
  // carry pass 2: carries < 2^6, columns now fit 32 bits
  const U c2 = rf_lo(rf_shr29(col));
  c16 = c16 + rf_widen(rl_bcast_w<15>(c2));
  const U colu = (rf_lo(col) & rf_const(a, RFE_MASK)) + rl_shr<1>(c2);
  // fold: columns 9..15 from lanes 0..6, column 16's low 29 bits into lane 7, its top (column 17)
  // into lane 8; r = low column + 1216 * high column
  U hi = rl_shl<9>(colu);
  hi = rf_sel(rl == rf_const(a, 7u), rf_lo(c16) & rf_const(a, RFE_MASK), hi);
  hi = rf_sel(rl == rf_const(a, 8u), rf_lo(rf_shr29(c16)), hi);
  const U lo = rf_sel(rl < rf_const(a, 9u), colu, rf_const(a, 0u));
  const W r = rf_mad(hi, rf_const(a, 1216u), rf_widen(lo));
  // last pass: lane 8's carry has weight 2^261 == 1216 and goes to lane 0
  const U c3 = rf_lo(rf_shr29(r));
  U out = (rf_lo(r) & rf_const(a, RFE_MASK)) + rl_shr<1>(c3);
  out = out + rf_sel(rl == rf_const(a, 0u), rl_bcast_w<8>(c3) * rf_const(a, 1216u), rf_const(a, 0u));
  return rf_sel(rl < rf_const(a, 9u), out, rf_const(a, 0u));
}

template <class U, class W>
RF_HD U rfe_sq(U a) {
  return rfe_mul<U, W>(a, a);
}

// carry pass on 32-bit limbs (< 2^32 - 2^12) -> row-reduced
template <class U>
RF_HD U rfe_carry(U x) {
  const U rl = rl_index(x);
  const U c = x >> 29;
  U out = (x & rf_const(x, RFE_MASK)) + rl_shr<1>(c);
  out = out + rf_sel(rl == rf_const(x, 0u), rl_bcast_w<8>(c) * rf_const(x, 1216u), rf_const(x, 0u));
  return rf_sel(rl < rf_const(x, 9u), out, rf_const(x, 0u));
}

// a + b (row-lazy for row-reduced operands; no carry)
template <class U>
RF_HD U rfe_add(U a, U b) {
  return a + b;
}

// a - b (mod p) for row-lazy a, b -> row-reduced: adds 256p = (2^31 - 4864, 2^31 - 4, ...), as
// fe_sub (every digit >= any row-lazy limb)
template <class U>
RF_HD U rfe_sub(U a, U b) {
  const U rl = rl_index(a);
  U k = rf_sel(rl == rf_const(a, 0u), rf_const(a, 0x80000000u - 4864u), rf_const(a, 0x80000000u - 4u));
  k = rf_sel(rl < rf_const(a, 9u), k, rf_const(a, 0u));
  return rfe_carry((a + k) - b);
}

// z^(2^n)
template <class U, class W>
RF_HD U rfe_sqn(U z, int n) {
#pragma nounroll
  for (int i = 0; i < n; i++) z = rfe_sq<U, W>(z);
  return z;
}

// z^((p - 5) / 8) = z^(2^252 - 3): the chain of fe_pow22523 (fe25519.h).  mid() runs after ~80 of
// its 265 operations (a caller's workgroup barrier placed inside the chain).
struct RfeNoop {
  RF_HD void operator()() const {}
};
template <class U, class W, class F = RfeNoop>
RF_HD U rfe_pow22523(U z, F mid = F()) {
  const U z2 = rfe_sq<U, W>(z);                              // 2
  const U z9 = rfe_mul<U, W>(rfe_sqn<U, W>(z2, 2), z);       // 9
  const U z11 = rfe_mul<U, W>(z9, z2);                       // 11
  U t0 = rfe_mul<U, W>(rfe_sq<U, W>(z11), z9);               // 2^5 - 1
  t0 = rfe_mul<U, W>(rfe_sqn<U, W>(t0, 5), t0);              // 2^10 - 1
  U t1 = rfe_mul<U, W>(rfe_sqn<U, W>(t0, 10), t0);           // 2^20 - 1
  t1 = rfe_mul<U, W>(rfe_sqn<U, W>(t1, 20), t1);             // 2^40 - 1
  t0 = rfe_mul<U, W>(rfe_sqn<U, W>(t1, 10), t0);             // 2^50 - 1
  t1 = rfe_sqn<U, W>(t0, 25);
  mid();                                                     // ~80 of the chain's 265 operations
  t1 = rfe_mul<U, W>(rfe_sqn<U, W>(t1, 25), t0);             // 2^100 - 1
  t1 = rfe_mul<U, W>(rfe_sqn<U, W>(t1, 100), t1);            // 2^200 - 1
  t0 = rfe_mul<U, W>(rfe_sqn<U, W>(t1, 50), t0);             // 2^250 - 1
  return rfe_mul<U, W>(rfe_sqn<U, W>(t0, 2), z);             // 2^252 - 3
}

// limb i of a 9-limb constant in row lane i (0 elsewhere)
template <class U>
RF_HD U rfe_row_const(const uint32_t* c, U tag) {
  const U rl = rl_index(tag);
  U r = rf_const(tag, 0u);
#pragma unroll
  for (int i = 0; i < 9; i++) r = rf_sel(rl == rf_const(tag, (uint32_t)i), rf_const(tag, c[i]), r);
  return r;
}
