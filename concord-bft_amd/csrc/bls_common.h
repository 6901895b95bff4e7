// Helpers shared by the BLS kernel translation units (internal).
#pragma once
#include <hip/hip_runtime.h>

#include "bls_kernels.h"
#include "bls_ops.h"
#include "bn254_row.h"

#define LINES_PER_KEY (BN_ATE_LINES * BN_LINE_WORDS)

__device__ __forceinline__ void g1a_store(uint32_t* o, const g1a& a) {
  for (int i = 0; i < 9; i++) {
    o[i] = a.x.v[i];
    o[9 + i] = a.y.v[i];
  }
  o[18] = a.inf ? 1u : 0u;
}
__device__ __forceinline__ void g1a_load(g1a& a, const uint32_t* o) {
  for (int i = 0; i < 9; i++) {
    a.x.v[i] = o[i];
    a.y.v[i] = o[9 + i];
  }
  a.inf = o[18] != 0;
}

__device__ __forceinline__ void g2a_store(uint32_t* o, const g2a& a) {
  for (int i = 0; i < 9; i++) {
    o[i] = a.x.a.v[i];
    o[9 + i] = a.x.b.v[i];
    o[18 + i] = a.y.a.v[i];
    o[27 + i] = a.y.b.v[i];
  }
  o[36] = a.inf ? 1u : 0u;
}
__device__ __forceinline__ void g2a_load(g2a& a, const uint32_t* o) {
  for (int i = 0; i < 9; i++) {
    a.x.a.v[i] = o[i];
    a.x.b.v[i] = o[9 + i];
    a.y.a.v[i] = o[18 + i];
    a.y.b.v[i] = o[27 + i];
  }
  a.inf = o[36] != 0;
}


// g1_map (bls_ops.h) with the try-and-increment candidates x, x + 1, ..., x + 63 tried on the
// 64 lanes of a wave at once: the lowest lane whose x^3 + 2 is a square wins, which is the point
// the sequential loop returns; every lane gets it.  One sqrt latency instead of two on average
// (half of all x are abscissas).  All 64 lanes must call it together.
__device__ __forceinline__ void g1_map_wave(g1a& r, const uint8_t* msg, uint32_t len) {
  uint8_t d[32];
  sha256(d, msg, len);
  uint32_t w[8];
  be32_to_words(w, d);
  fp x, two, rhs, y, off, step;
  f_from_words(x, w);
  const uint32_t lane = threadIdx.x & 63;
  uint32_t t[8] = {2, 0, 0, 0, 0, 0, 0, 0};
  f_from_words(two, t);
  t[0] = lane;
  f_from_words(off, t);
  t[0] = 64;
  f_from_words(step, t);
  f_add(x, x, off);
  for (;;) {
    f_sqr(rhs, x);
    f_mul(rhs, rhs, x);
    f_add(rhs, rhs, two);
    const bool ok = fp_sqrt(y, rhs);
    const unsigned long long m = __ballot(ok);
    if (m) {
      const int src = __ffsll(m) - 1;
      for (int i = 0; i < BN_LIMBS; i++) {
        r.x.v[i] = (uint32_t)__shfl((int)x.v[i], src);
        r.y.v[i] = (uint32_t)__shfl((int)y.v[i], src);
      }
      break;
    }
    f_add(x, x, step);
  }
  r.inf = false;
}

// Jacobian G2 point <-> 54 words (X | Y | Z, Fp2 = a | b, 9 limbs each): key-sum partials
__device__ __forceinline__ void g2j_store(uint32_t* o, const g2j& a) {
  const fp2* src[3] = {&a.X, &a.Y, &a.Z};
  for (int c = 0; c < 3; c++)
    for (int q = 0; q < 9; q++) {
      o[18 * c + q] = src[c]->a.v[q];
      o[18 * c + 9 + q] = src[c]->b.v[q];
    }
}
__device__ __forceinline__ void g2j_load(g2j& a, const uint32_t* o) {
  fp2* dst[3] = {&a.X, &a.Y, &a.Z};
  for (int c = 0; c < 3; c++)
    for (int q = 0; q < 9; q++) {
      dst[c]->a.v[q] = o[18 * c + q];
      dst[c]->b.v[q] = o[18 * c + 9 + q];
    }
}

// fp_sqrt (bn254_field.h) on the lane's DPP row: y = a^((p+1)/4) by rf_pow_sw, true iff y^2 == a.
// Every lane of a row must hold the same a, and all 64 lanes of the wave must call it together.
__device__ __forceinline__ bool fp_sqrt_row(fp& y, const fp& a) {
  const uint32_t tag = 0;
  const uint32_t qrow = rf_row_const(FpParams::Q, tag);
  rf_to_fe(y, rf_pow_sw<FpSqrtSchedule, uint32_t, uint64_t>(rf_from_fe(a, tag), qrow));
  fp t;
  f_sqr(t, y);
  return f_eq(t, a);
}

// g1_decompress (bn254_pairing.h: RELIC ep_read_bin, pack = 1) with the square root on the lane's
// DPP row: the same point and verdict for every 33-byte input.  Every lane of a row must hold the
// same bytes and all 64 lanes of the wave must call it together: the root is taken whatever the
// encoding (a malformed one is rejected after it), so no row leaves the row-parallel code early.
__device__ __forceinline__ bool g1_decompress_row(g1a& r, const uint8_t* b) {
  const uint8_t pre = b[0];
  uint8_t o = 0;
  for (int i = 1; i < 33; i++) o |= b[i];
  uint32_t w[8];
  be32_to_words(w, b + 1);
  fp x, rhs, b2, y;
  f_from_words(x, w);  // any 256-bit value: used only when x < p
  f_sqr(rhs, x);
  f_mul(rhs, rhs, x);
  uint32_t two[8] = {2, 0, 0, 0, 0, 0, 0, 0};
  f_from_words(b2, two);
  f_add(rhs, rhs, b2);
  const bool sq = fp_sqrt_row(y, rhs);
  if (pre == 0) {  // infinity: 0x00 || 0^32
    r.inf = true;
    f_zero(r.x);
    f_zero(r.y);
    return o == 0;
  }
  r.inf = false;
  if ((pre != 2 && pre != 3) || !words_lt_p(w) || !sq) return false;
  r.x = x;
  if (f_relic_bit(y) != (uint32_t)(pre & 1)) f_neg(y, y);
  r.y = y;
  return true;
}

// bls_parse_share (bls_ops.h) with g1_decompress_row: the same contract as g1_decompress_row
__device__ __forceinline__ bool bls_parse_share_row(uint32_t& id, g1a& s, const uint8_t* b) {
  id = ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
  return g1_decompress_row(s, b + 4);
}

// g1_map with the try-and-increment candidates tried four at a time, one per DPP row, the square
// root on row-parallel Fp: candidate x + 4 i + row in row `row`; the lowest row whose x^3 + 2 is a
// square wins (the point the sequential loop returns), every lane gets it.  1.07 rounds on
// average (a round fails with probability 1/16), each ~2x shorter than g1_map_wave's one-lane
// root.  All 64 lanes must call it together.
__device__ __forceinline__ void g1_map_row(g1a& r, const uint8_t* msg, uint32_t len) {
  uint8_t d[32];
  sha256(d, msg, len);
  uint32_t w[8];
  be32_to_words(w, d);
  fp x, two, rhs, y, off, step;
  f_from_words(x, w);
  const uint32_t row = (threadIdx.x & 63) >> 4;
  uint32_t t[8] = {2, 0, 0, 0, 0, 0, 0, 0};
  f_from_words(two, t);
  t[0] = row;
  f_from_words(off, t);
  t[0] = 4;
  f_from_words(step, t);
  f_add(x, x, off);
  for (;;) {
    f_sqr(rhs, x);
    f_mul(rhs, rhs, x);
    f_add(rhs, rhs, two);
    const bool ok = fp_sqrt_row(y, rhs);
    const unsigned long long m = __ballot(ok);
    if (m) {
      const int src = __ffsll(m) - 1;
      for (int i = 0; i < BN_LIMBS; i++) {
        r.x.v[i] = (uint32_t)__shfl((int)x.v[i], src);
        r.y.v[i] = (uint32_t)__shfl((int)y.v[i], src);
      }
      break;
    }
    f_add(x, x, step);
  }
  r.inf = false;
}
