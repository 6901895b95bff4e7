// Row-parallel BN-P254 Fp arithmetic (gfx950 device code, and a host SIMD emulation for tests).
//
// An Fp element lives in ONE 16-lane DPP row: limb i (29 bits, the same Montgomery form as
// bn254_field.h, R = 2^261) in row lane i, lanes 9..15 zero.  Each lane therefore holds one
// 32-bit word of the element instead of nine, and the four rows of a wave compute four
// independent products in the same instruction stream (the "quad" of bn254_g1quad.h, but with
// the limbs spread too).  A product is 9 row_newbcast/row_shr DPP moves + 9 v_mad_u64_u32 per
// lane for the columns, then a word-serial Montgomery reduction across the row (m_i broadcast
// from lane i, the carry handed to lane i + 1 with row_shr:1), then a lane-parallel carry
// normalisation: about 3x fewer issue slots than the one-lane f_mul.  Additions and
// subtractions are one lane op plus one carry pass.
//
// Bounds ("row-normal"): limbs <= 2^29 + 8, lanes 9..15 zero.  rf_mul maps two row-normal inputs
// with (a / q)(b / q) < R / q = 221 (e.g. both < 14q) to a row-normal output < 2q (the REDC bound
// a b / R + q < 2q holds while a b < q R); columns stay < 18 (2^29 + 8)^2 + carries < 2^63.
// Callers track value bounds: rf_add(a, b) = a + b, rf_sub(a, b) = a - b + 8q for b < 4q,
// rf_sub32(a, b) = a - b + 32q for b < 16q, rf_reduce(x) < 4q for any x < 2^261.
//
// The code is written once over a lane-vector type: on the device U = uint32_t / W = uint64_t
// are the lane's own registers and the cross-lane helpers are DPP moves; on the host (tests/cpp/
// bn254_shim.cpp) U / W are 64-lane vectors and the same templates run as an exact SIMD
// emulation, checked against f_mul.
#pragma once
#include "bn254_field.h"

#include "row_lanes.h"

// 8q in the redundant limb form used by rf_sub: limb i in [2^30, 2^31) for i < 8 (limb 8 =
// 8q's top limb - 2), so a + Q8R - b is limb-wise non-negative for any row-normal b < 4q.
struct RfConsts {
  static constexpr uint32_t Q8R[9] = {0x40000098u, 0x3ffffffeu, 0x4000274cu, 0x4ffffffeu, 0x4004308eu,
                                      0x55fffffeu, 0x40374687u, 0x423ffffeu, 0x01291b22u};
  // 32q in the same redundant form: a + Q32R - b for any row-normal b < 16q
  static constexpr uint32_t Q32R[9] = {0x40000260u, 0x3ffffffeu, 0x40009d36u, 0x3ffffffeu, 0x4010c240u,
                                       0x57fffffeu, 0x40dd1a24u, 0x48fffffeu, 0x04a46c8eu};
  // 7q, 8q, 9q with normalised limbs: H = U2 - U1 + 8q (|U2 - U1| < 2q) is 0 mod q iff it is one
  static constexpr uint32_t Q7N[9] = {0x00000085u, 0x08000000u, 0x00002264u, 0x0e000000u, 0x0003aa7eu,
                                      0x0f400000u, 0x00305db8u, 0x11f80000u, 0x0103f7bfu};
  static constexpr uint32_t Q8N[9] = {0x00000098u, 0x00000000u, 0x0000274eu, 0x10000000u, 0x00043090u,
                                      0x16000000u, 0x00374689u, 0x02400000u, 0x01291b24u};
  static constexpr uint32_t Q9N[9] = {0x000000abu, 0x18000000u, 0x00002c37u, 0x12000000u, 0x0004b6a2u,
                                      0x1cc00000u, 0x003e2f5au, 0x12880000u, 0x014e3e88u};
  // 64q, limbs 0..7 raised by 2^38 (and 2^9 borrowed from the next): rf_reduce subtracts up to
  // ~285 q limb-wise from x + 64q without a negative limb below the top one
  static constexpr uint64_t Q64R[9] = {0x040000004c0ull, 0x03ffffffe00ull, 0x04000013870ull, 0x03ffffffe00ull,
                                       0x04000218284ull, 0x0400ffffe00ull, 0x04001ba324dull, 0x04011fffe00ull,
                                       0x0000948d720ull};
  static constexpr uint32_t TOP_RECIP = 1764;  // floor(2^32 / (floor(q / 2^232) + 1))
};


// ------------------------------------------------------------------------------ arithmetic
// limb i of a 9-limb constant in row lane i (0 elsewhere)
template <class U>
RF_HD U rf_row_const(const uint32_t* c, U tag) {
  const U rl = rl_index(tag);
  U r = rf_const(tag, 0u);
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) r = rf_sel(rl == rf_const(tag, (uint32_t)i), rf_const(tag, c[i]), r);
  return r;
}

// carry pass on 64-bit lanes: x = (x & mask) + carry of the lane below
template <class U, class W>
RF_HD W rf_carry64(W x) {
  const W x29 = rf_shr29(x);
  const U c_lo = rl_shr<1>(rf_lo(x29)), c_hi = rl_shr<1>(rf_hi(x29));
  return (x & rf_const64(c_lo, (uint64_t)BN_MASK)) + rf_w(c_lo, c_hi);
}
template <class U>
RF_HD U rf_carry32(U x) {
  return (x & rf_const(x, BN_MASK)) + rl_shr<1>(x >> 29);
}

#ifndef RF_MUL_CHECK
#define RF_MUL_CHECK(a, b)  // host emulation builds check every product's bounds (tests/cpp/bn254_shim.cpp)
#endif

// r = a * b * 2^-261 mod q (row-normal in, row-normal out, value < 2q).  qrow = rf_row_const(Q).
template <class U, class W>
RF_HD U rf_mul(U a, U b, U qrow) {
  RF_MUL_CHECK(a, b);
  const U rl = rl_index(a);
  W col = rf_const64(a, 0ull);
  // product columns 0..15 in lanes 0..15; column 16 (= a8 b8 + m8 q8) separately
#define RF_PROD(I) col = rf_mad(rl_bcast<I>(a), rl_shr<I>(b), col);
  RF_PROD(0) RF_PROD(1) RF_PROD(2) RF_PROD(3) RF_PROD(4) RF_PROD(5) RF_PROD(6) RF_PROD(7) RF_PROD(8)
#undef RF_PROD
  W c16 = rf_mad(rl_bcast<8>(a), rl_bcast<8>(b), rf_const64(a, 0ull));
  // word-serial REDC: m_i from lane i's column, m_i q added into columns i..i+8, lane i's carry
  // (its low 29 bits are now 0) into lane i + 1
#define RF_REDC(I)                                                                         \
  {                                                                                        \
    const U m = rl_bcast<I>((rf_lo(col) * rf_const(a, FpParams::NPRIME)) & rf_const(a, BN_MASK)); \
    col = rf_mad(m, rl_shr<I>(qrow), col);                                                 \
    if (I == 8) c16 = rf_mad(m, rl_bcast<8>(qrow), c16);                                   \
    const W c = rf_shr29(col);                                                             \
    const U c_lo = rl_shr<1>(rf_lo(c)), c_hi = rl_shr<1>(rf_hi(c));                        \
    col = col + rf_sel(rl == rf_const(a, (uint32_t)(I + 1)), rf_w(c_lo, c_hi), rf_const64(a, 0ull)); \
  }
  RF_REDC(0) RF_REDC(1) RF_REDC(2) RF_REDC(3) RF_REDC(4) RF_REDC(5) RF_REDC(6) RF_REDC(7) RF_REDC(8)
#undef RF_REDC
  // columns 9..15 -> lanes 0..6, column 16 -> lane 7, then carry passes
  W r = rf_w(rl_shl<9>(rf_lo(col)), rl_shl<9>(rf_hi(col)));
  r = r + rf_sel(rl == rf_const(a, 7u), c16, rf_const64(a, 0ull));
  r = rf_carry64<U, W>(r);
  r = rf_carry64<U, W>(r);
  return rf_carry32(rf_lo(r));
}

template <class U>
RF_HD U rf_add(U a, U b) {  // value a + b
  return rf_carry32(a + b);
}
template <class U>
RF_HD U rf_sub(U a, U b, U q8r) {  // a - b + 8q for b < 4q; q8r = rf_row_const(RfConsts::Q8R)
  return rf_carry32((a + q8r) - b);
}
template <class U>
RF_HD U rf_sub32(U a, U b, U q32r) {  // a - b + 32q for b < 16q; q32r = rf_row_const(RfConsts::Q32R)
  return rf_carry32((a + q32r) - b);
}

// 9-limb 64-bit constant in row lane i
template <class U, class W>
RF_HD W rf_row_const64(const uint64_t* c, U tag) {
  const U rl = rl_index(tag);
  W r = rf_const64(tag, 0ull);
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) r = rf_sel(rl == rf_const(tag, (uint32_t)i), rf_const64(tag, c[i]), r);
  return r;
}

// x mod q, up to 4q: x < 2^261 with limbs <= 2^29 + 8.  m = floor(x / q) is estimated from the
// top limb (low by at most 3), and x + 64q - (m + 64) q is formed limb-wise (limbs 0..7 stay
// non-negative; the top limb may go negative and takes the carries from below).  Result < 4q,
// row-normal.  q64r = rf_row_const64(Q64R).
template <class U, class W>
RF_HD U rf_reduce(U x, U qrow, W q64r) {
  const U rl = rl_index(x);
  const U t8 = rl_bcast<8>(x);
  U m = rf_hi(rf_mul64(t8, rf_const(x, RfConsts::TOP_RECIP)));  // <= floor(x / q) + 1
  m = m + rf_const(x, 63u);  // (m - 1) + 64: the estimate lowered by one, plus the 64q added
  W y = rf_widen(x) + q64r;
  y = y + (rf_const64(x, 0ull) - rf_mul64(m, qrow));  // x + 64q - (m + 63) q, limbs 0..7 >= 0
  const auto low = rl < rf_const(x, 8u);
#pragma unroll
  for (int pass = 0; pass < 2; pass++) {
    const W c = rf_sel(low, rf_sra29(y), rf_const64(x, 0ull));
    const U c_lo = rl_shr<1>(rf_lo(c)), c_hi = rl_shr<1>(rf_hi(c));
    y = rf_sel(low, y & rf_const64(x, (uint64_t)BN_MASK), y) + rf_w(c_lo, c_hi);
  }
  return rf_carry32(rf_lo(y));
}

// exact normalisation: limbs < 2^29 (x row-normal, value < 2^261); carries resolved with one
// carry-lookahead over the wave's ballot masks (lanes 9..15 are zero and stop them at rows)
template <class U>
RF_HD U rf_normalize(U x) {
  x = rf_carry32(x);  // limbs <= 2^29
  const uint64_t g = rf_ballot(x > rf_const(x, BN_MASK)), p = rf_ballot(x == rf_const(x, BN_MASK));
  const uint64_t t = g | p, cin = (t + g) ^ t ^ g;
  return (x + rf_bit(cin, rl_lane(x))) & rf_const(x, BN_MASK);
}

// wave-uniform: does row 0 of the normalised x equal the row constant c (normalised limbs)?
template <class U>
RF_HD bool rf_row0_equals(U xn, U c) {
  return (rf_ballot(xn == c) & 0xFFFFull) == 0xFFFFull;
}

// a^e on row-parallel Fp for the window schedule of f_pow_sw (bn254_field.h: same windows, same
// table of odd powers), each product on the row: ~2x less latency than the one-lane chain.
// a row-normal < 2q; result row-normal < 2q.  The window index is uniform across the wave.
template <class Sched, class U, class W>
RF_HD U rf_pow_sw(U a, U qrow) {
  U t[8];
  t[0] = a;
  const U a2 = rf_mul<U, W>(a, a, qrow);
#pragma unroll
  for (int k = 1; k < 8; k++) t[k] = rf_mul<U, W>(t[k - 1], a2, qrow);
  U acc = t[0];
  for (int w = 0; w < Sched::S.n; w++) {
    for (int q = 0; q < Sched::S.nsq[w]; q++) acc = rf_mul<U, W>(acc, acc, qrow);
    const int idx = Sched::S.v[w] >> 1;
    U e = t[0];
#pragma unroll
    for (int k = 1; k < 8; k++)
      if (idx == k) e = t[k];
    acc = w == 0 ? e : rf_mul<U, W>(acc, e, qrow);
  }
  for (int q = 0; q < Sched::S.tail; q++) acc = rf_mul<U, W>(acc, acc, qrow);
  return acc;
}

// ------------------------------------------------------------------------------ conversions
// one-lane fp (every lane the same value) <-> row element
template <class U, class F>
RF_HD U rf_from_fe(const Fe<F>& x, U tag) {
  const U rl = rl_index(tag);
  U r = rf_const(tag, 0u);
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) r = rf_sel(rl == rf_const(tag, (uint32_t)i), rf_const(tag, x.v[i]), r);
  return r;
}

#if defined(__HIPCC__)
// row element -> one-lane fp in every lane of the row (limbs gathered with row_newbcast, then
// normalised; value unchanged)
template <class F>
RF_HD void rf_to_fe(Fe<F>& r, uint32_t x) {
  uint32_t v[BN_LIMBS] = {rl_bcast<0>(x), rl_bcast<1>(x), rl_bcast<2>(x), rl_bcast<3>(x), rl_bcast<4>(x),
                          rl_bcast<5>(x), rl_bcast<6>(x), rl_bcast<7>(x), rl_bcast<8>(x)};
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
    const uint32_t t = v[i] + c;
    r.v[i] = i == BN_LIMBS - 1 ? t : (t & BN_MASK);
    c = t >> 29;
  }
}
#endif
