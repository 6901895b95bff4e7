// Host SIMD emulation of the lane-vector operations bn254_row.h is written over: a U / W is the
// 64 lanes' 32 / 64-bit values of one wave, cross-lane helpers move values exactly as the gfx950
// DPP controls do (row_newbcast, row_shr / row_shl with zero fill, ds_bpermute by row).  The
// row-parallel arithmetic then runs unchanged on the host and is compared with the one-lane
// field code (tests/cpp/bn254_shim.cpp, tests/test_bn254_inv.py).
#pragma once
#include <array>
#include <cstdint>

struct HU {
  std::array<uint32_t, 64> x{};
};
struct HW {
  std::array<uint64_t, 64> x{};
};
struct HB {
  std::array<bool, 64> x{};
};

#define HU_BIN(OP)                                         \
  inline HU operator OP(const HU& a, const HU& b) {        \
    HU r;                                                  \
    for (int l = 0; l < 64; l++) r.x[l] = a.x[l] OP b.x[l]; \
    return r;                                              \
  }
HU_BIN(+)
HU_BIN(-)
HU_BIN(*)
HU_BIN(&)
HU_BIN(|)
#undef HU_BIN
inline HU operator>>(const HU& a, int s) {
  HU r;
  for (int l = 0; l < 64; l++) r.x[l] = a.x[l] >> s;
  return r;
}
inline HW operator>>(const HW& a, int s) {
  HW r;
  for (int l = 0; l < 64; l++) r.x[l] = a.x[l] >> s;
  return r;
}
inline HW operator+(const HW& a, const HW& b) {
  HW r;
  for (int l = 0; l < 64; l++) r.x[l] = a.x[l] + b.x[l];
  return r;
}
inline HW operator&(const HW& a, const HW& b) {
  HW r;
  for (int l = 0; l < 64; l++) r.x[l] = a.x[l] & b.x[l];
  return r;
}
inline HB operator==(const HU& a, const HU& b) {
  HB r;
  for (int l = 0; l < 64; l++) r.x[l] = a.x[l] == b.x[l];
  return r;
}

inline HU rf_const(const HU&, uint32_t v) {
  HU r;
  r.x.fill(v);
  return r;
}
inline HW rf_const64(const HU&, uint64_t v) {
  HW r;
  r.x.fill(v);
  return r;
}
inline HU rf_lo(const HW& w) {
  HU r;
  for (int l = 0; l < 64; l++) r.x[l] = (uint32_t)w.x[l];
  return r;
}
inline HU rf_hi(const HW& w) {
  HU r;
  for (int l = 0; l < 64; l++) r.x[l] = (uint32_t)(w.x[l] >> 32);
  return r;
}
inline HW rf_w(const HU& lo, const HU& hi) {
  HW r;
  for (int l = 0; l < 64; l++) r.x[l] = (uint64_t)lo.x[l] | ((uint64_t)hi.x[l] << 32);
  return r;
}
inline HW rf_mad(const HU& a, const HU& b, const HW& c) {
  HW r;
  for (int l = 0; l < 64; l++) r.x[l] = (uint64_t)a.x[l] * b.x[l] + c.x[l];
  return r;
}
inline HU rf_sel(const HB& c, const HU& a, const HU& b) {
  HU r;
  for (int l = 0; l < 64; l++) r.x[l] = c.x[l] ? a.x[l] : b.x[l];
  return r;
}
inline HW rf_sel(const HB& c, const HW& a, const HW& b) {
  HW r;
  for (int l = 0; l < 64; l++) r.x[l] = c.x[l] ? a.x[l] : b.x[l];
  return r;
}
inline HU rl_index(const HU&) {
  HU r;
  for (int l = 0; l < 64; l++) r.x[l] = (uint32_t)(l & 15);
  return r;
}
inline HU rl_row(const HU&) {
  HU r;
  for (int l = 0; l < 64; l++) r.x[l] = (uint32_t)(l >> 4);
  return r;
}
template <int I>
inline HU rl_bcast(const HU& a) {
  HU r;
  for (int l = 0; l < 64; l++) r.x[l] = a.x[(l & ~15) + I];
  return r;
}
template <int I>
inline HU rl_bcast_w(const HU& a) {
  return rl_bcast<I>(a);
}
template <int I>
inline HU rl_shr(const HU& a) {
  HU r;
  for (int l = 0; l < 64; l++) r.x[l] = (l & 15) >= I ? a.x[l - I] : 0u;
  return r;
}
template <int I>
inline HU rl_shl(const HU& a) {
  HU r;
  for (int l = 0; l < 64; l++) r.x[l] = (l & 15) + I < 16 ? a.x[l + I] : 0u;
  return r;
}
inline void rl_all_rows(const HU& a, HU* r) {
  for (int s = 0; s < 4; s++)
    for (int l = 0; l < 64; l++) r[s].x[l] = a.x[16 * s + (l & 15)];
}
template <int S>
inline HU rl_from_row(const HU& a) {
  HU r;
  for (int l = 0; l < 64; l++) r.x[l] = a.x[S * 16 + (l & 15)];
  return r;
}

inline HB operator>(const HU& a, const HU& b) {
  HB r;
  for (int l = 0; l < 64; l++) r.x[l] = a.x[l] > b.x[l];
  return r;
}
inline HW operator-(const HW& a, const HW& b) {
  HW r;
  for (int l = 0; l < 64; l++) r.x[l] = a.x[l] - b.x[l];
  return r;
}
inline HW rf_shr29(const HW& w) {
  HW r;
  for (int l = 0; l < 64; l++) r.x[l] = w.x[l] >> 29;
  return r;
}
inline HW rf_sra29(const HW& w) {
  HW r;
  for (int l = 0; l < 64; l++) r.x[l] = (uint64_t)((int64_t)w.x[l] >> 29);
  return r;
}
inline uint64_t rf_ballot(const HB& c) {
  uint64_t m = 0;
  for (int l = 0; l < 64; l++) m |= (uint64_t)c.x[l] << l;
  return m;
}
inline HU rl_lane(const HU&) {
  HU r;
  for (int l = 0; l < 64; l++) r.x[l] = (uint32_t)l;
  return r;
}
inline HW rf_widen(const HU& x) {
  HW r;
  for (int l = 0; l < 64; l++) r.x[l] = x.x[l];
  return r;
}
inline HW rf_mul64(const HU& a, const HU& b) {
  HW r;
  for (int l = 0; l < 64; l++) r.x[l] = (uint64_t)a.x[l] * b.x[l];
  return r;
}
inline HU rf_bit(uint64_t mask, const HU& lane) {
  HU r;
  for (int l = 0; l < 64; l++) r.x[l] = (uint32_t)(mask >> lane.x[l]) & 1u;
  return r;
}
inline HB operator<(const HU& a, const HU& b) {
  HB r;
  for (int l = 0; l < 64; l++) r.x[l] = a.x[l] < b.x[l];
  return r;
}
