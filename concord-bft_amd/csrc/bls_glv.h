// GLV decomposition and signed radix-16 digits for the BN-P254 G1 MSM (shared by the quad and
// row-parallel MSM kernels; internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// ---- GLV (Gallant-Lambert-Vanstone) on BN-P254 G1: phi(x, y) = (beta x, y) = [lam] P with
// beta^3 = 1 in Fp, lam^2 + lam + 1 = 0 mod r.  k = k1 + k2 lam (mod r) with |k1|, |k2| < 2^128
// from the short lattice basis v1 = (a1, b1), v2 = (a2, b2) of {(x, y): x + y lam = 0 mod r}
// (extended Euclid on (r, lam)): c1 = floor(k g1 / 2^256), c2 = floor(k g2 / 2^256) with
// g1 = floor(b2 2^256 / r), g2 = floor(-b1 2^256 / r); k1 = k - c1 a1 - c2 a2, k2 = -c1 b1 - c2 b2.
// (Constants derived with the Python oracle; any decomposition with k1 + k2 lam = k mod r gives
// the same point, the bound only sizes the ladder.)
static __constant__ const uint32_t kGlvG1[3] = {0x8a6b4904u, 0x7937ca68u, 0x00000003u};
static __constant__ const uint32_t kGlvG2[5] = {0x36bf3357u, 0xc0eb31ffu, 0x04a017b9u, 0xa01fab7eu, 0x00000002u};
static __constant__ const uint32_t kGlvA1[2] = {0x00000001u, 0x81000000u};
static __constant__ const uint32_t kGlvA2[4] = {0x00000004u, 0x85000000u, 0x00000002u, 0x61818000u};
static __constant__ const uint32_t kGlvB1[4] = {0x00000003u, 0x04000000u, 0x00000002u, 0x61818000u};  // |b1|, b1 < 0
static __constant__ const uint32_t kGlvB2[2] = {0x00000001u, 0x81000000u};
static __constant__ const uint32_t kGlvBeta[8] = {0x00000007u, 0xcd800000u, 0x00000006u, 0x49090000u,
                                           0x00000002u, 0x49b36240u, 0x00000000u, 0x00000000u};

// out[0..no) = (a[0..na) * b[0..nb)) words [shift, shift + no) (schoolbook, 32-bit words)
template <int NA, int NB, int NO>
__device__ __forceinline__ void mp_mul(uint32_t* out, const uint32_t* a, const uint32_t* b, int shift) {
  uint32_t t[NA + NB];
#pragma unroll
  for (int i = 0; i < NA + NB; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < NA; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < NB; j++) {
      c += (uint64_t)a[i] * b[j] + t[i + j];
      t[i + j] = (uint32_t)c;
      c >>= 32;
    }
    t[i + NB] = (uint32_t)c;
  }
#pragma unroll
  for (int i = 0; i < NO; i++) out[i] = (shift + i < NA + NB) ? t[shift + i] : 0u;
}

// a -= b (mod 2^256), 8 words
__device__ __forceinline__ void mp_sub8(uint32_t* a, const uint32_t* b) {
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int64_t d = (int64_t)a[i] - b[i] + br;
    a[i] = (uint32_t)d;
    br = d >> 32;
  }
}
// |a| and its sign (a as two's complement mod 2^256)
__device__ __forceinline__ bool mp_abs8(uint32_t* a) {
  const bool neg = (a[7] >> 31) != 0;
  if (neg) {
    uint64_t c = 1;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      c += (uint32_t)~a[i];
      a[i] = (uint32_t)c;
      c >>= 32;
    }
  }
  return neg;
}

// k (8 LE words, < r) -> |k1|, |k2| (5 words each, < 2^129 with the window offset headroom) and
// their signs
__device__ __forceinline__ void glv_split(const uint32_t* k, uint32_t* k1, uint32_t* k2, bool& n1, bool& n2) {
  uint32_t c1[3], c2[5], g1[3], g2[5], a1[2], a2[4], b1[4], b2[2];
#pragma unroll
  for (int i = 0; i < 3; i++) g1[i] = kGlvG1[i];
#pragma unroll
  for (int i = 0; i < 5; i++) g2[i] = kGlvG2[i];
#pragma unroll
  for (int i = 0; i < 2; i++) {
    a1[i] = kGlvA1[i];
    b2[i] = kGlvB2[i];
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    a2[i] = kGlvA2[i];
    b1[i] = kGlvB1[i];
  }
  mp_mul<8, 3, 3>(c1, k, g1, 8);
  mp_mul<8, 5, 5>(c2, k, g2, 8);
  uint32_t t[8], p[8];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = k[i];
  mp_mul<3, 2, 8>(p, c1, a1, 0);
  mp_sub8(t, p);
  mp_mul<5, 4, 8>(p, c2, a2, 0);
  mp_sub8(t, p);  // k1 = k - c1 a1 - c2 a2
  n1 = mp_abs8(t);
#pragma unroll
  for (int i = 0; i < 5; i++) k1[i] = t[i];
  mp_mul<3, 4, 8>(t, c1, b1, 0);  // -c1 b1 = c1 |b1|
  mp_mul<5, 2, 8>(p, c2, b2, 0);
  mp_sub8(t, p);  // k2 = c1 |b1| - c2 b2
  n2 = mp_abs8(t);
#pragma unroll
  for (int i = 0; i < 5; i++) k2[i] = t[i];
}

// signed radix-16 digits of a < 2^128 scalar: s + 8 (16^0 + ... + 16^31), nibble i minus 8 for
// i < 32, the carry into bit 128 as digit 32 (0 or 1)
__device__ __forceinline__ int glv_digit(const uint32_t* so, int i) {
  const int nib = (int)((so[i >> 3] >> (4 * (i & 7))) & 15u);
  return i < 32 ? nib - 8 : nib;
}
__device__ __forceinline__ void glv_offset(uint32_t* s) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    c += (uint64_t)s[i] + (i < 4 ? 0x88888888u : 0u);
    s[i] = (uint32_t)c;
    c >>= 32;
  }
}

