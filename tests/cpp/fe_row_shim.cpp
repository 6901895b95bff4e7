// Host build of the row-parallel GF(2^255 - 19) code (concord-bft_amd/csrc/fe25519_row.h) on the
// SIMD emulation of tests/cpp/row_emu.h, exposed to tests/test_fe_row.py through ctypes: the SAME
// templates the small-batch kernels' R decode runs on gfx950, checked against Python integers.
// Every entry point takes four row elements (4 x 9 limbs: the four rows of one wave) and returns
// the 4 x 16 lanes of the result, so a test also sees that lanes 9..15 stay zero.
#include <cstring>

#include "row_emu.h"
#include "fe25519_row.h"

static HU load_rows(const uint32_t* x36) {
  HU r;
  for (int row = 0; row < 4; row++)
    for (int l = 0; l < 9; l++) r.x[16 * row + l] = x36[9 * row + l];
  return r;
}
static void store_lanes(uint32_t* out64, const HU& r) { std::memcpy(out64, r.x.data(), 64 * sizeof(uint32_t)); }

extern "C" {
void fe_row_mul(const uint32_t* a36, const uint32_t* b36, uint32_t* out64) {
  store_lanes(out64, rfe_mul<HU, HW>(load_rows(a36), load_rows(b36)));
}
void fe_row_sq(const uint32_t* a36, uint32_t* out64) { store_lanes(out64, rfe_sq<HU, HW>(load_rows(a36))); }
void fe_row_sub(const uint32_t* a36, const uint32_t* b36, uint32_t* out64) {
  store_lanes(out64, rfe_sub(load_rows(a36), load_rows(b36)));
}
void fe_row_carry(const uint32_t* a36, uint32_t* out64) { store_lanes(out64, rfe_carry(load_rows(a36))); }
void fe_row_pow22523(const uint32_t* a36, uint32_t* out64) {
  store_lanes(out64, rfe_pow22523<HU, HW>(load_rows(a36)));
}
}
