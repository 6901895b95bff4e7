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
  fp x, two, rhs, y, off, step, t2;
  f_from_words(x, w);
  const uint32_t tag = 0;
  const uint32_t row = (threadIdx.x & 63) >> 4;
  uint32_t t[8] = {2, 0, 0, 0, 0, 0, 0, 0};
  f_from_words(two, t);
  t[0] = row;
  f_from_words(off, t);
  t[0] = 4;
  f_from_words(step, t);
  f_add(x, x, off);
  const uint32_t qrow = rf_row_const(FpParams::Q, tag);
  for (;;) {
    f_sqr(rhs, x);
    f_mul(rhs, rhs, x);
    f_add(rhs, rhs, two);
    rf_to_fe(y, rf_pow_sw<FpSqrtSchedule, uint32_t, uint64_t>(rf_from_fe(rhs, tag), qrow));
    f_sqr(t2, y);
    const bool ok = f_eq(t2, rhs);
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
