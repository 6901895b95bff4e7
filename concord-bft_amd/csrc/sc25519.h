// Scalars modulo the group order L = 2^252 + 27742317777372353535851937790883648493
// (RFC 8032 §5.1), as little-endian 32-bit words.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __constant__ const uint32_t kScL[9] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u,
                                                  0u,          0u,          0x10000000u, 0u};
// mu = floor(2^512 / L)  (Barrett constant, 261 bits)
__device__ __constant__ const uint32_t kScMu[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu,
                                                   0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu};

// S < L ? (strict, as OpenSSL's check on the signature's S half)
__device__ __forceinline__ bool sc_is_canonical(const uint32_t* s) {
  // lexicographic compare from the top word
  bool lt = false, decided = false;
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    bool l = s[i] < kScL[i], g = s[i] > kScL[i];
    lt = decided ? lt : l;
    decided = decided || l || g;
  }
  return lt;  // equal -> not canonical
}

// r (8 words) = x (16 words, 512-bit) mod L, Barrett reduction (HAC 14.42, b = 2^32, k = 8).
__device__ __forceinline__ void sc_reduce512(uint32_t* r, const uint32_t* x) {
  // q1 = x >> 224 (9 words); q3 = (q1 * mu) >> 288
  uint32_t q2[18];
#pragma unroll
  for (int i = 0; i < 18; i++) q2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) {
      uint64_t t = (uint64_t)x[7 + i] * kScMu[j] + q2[i + j] + carry;
      q2[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    q2[i + 9] = (uint32_t)carry;
  }
  const uint32_t* q3 = q2 + 9;
  // r2 = (q3 * L) mod 2^288
  uint32_t r2[9];
#pragma unroll
  for (int i = 0; i < 9; i++) r2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j + i < 9; j++) {
      uint64_t t = (uint64_t)q3[i] * kScL[j] + r2[i + j] + carry;
      r2[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
  }
  // t = (x mod 2^288) - r2  (mod 2^288)
  uint32_t t[9];
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    int64_t d = (int64_t)x[i] - (int64_t)r2[i] + br;
    t[i] = (uint32_t)d;
    br = d >> 32;
  }
  // at most two subtractions of L
#pragma unroll
  for (int rep = 0; rep < 2; rep++) {
    uint32_t u[9];
    int64_t b2 = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      int64_t d = (int64_t)t[i] - (int64_t)kScL[i] + b2;
      u[i] = (uint32_t)d;
      b2 = d >> 32;
    }
    bool ge = (b2 == 0);  // no borrow -> t >= L
#pragma unroll
    for (int i = 0; i < 9; i++) t[i] = ge ? u[i] : t[i];
  }
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = t[i];
}

// Signed fixed-window recoding constant C_w,n = 2^(w-1) * sum_{i<n} 2^(w i).
// k + C has n windows whose w-bit values minus 2^(w-1) are the signed digits of k
// (in [-2^(w-1), 2^(w-1)-1]); requires k + C < 2^(n w).
struct RecodeConst {
  uint32_t w[9];
};
constexpr RecodeConst make_recode_const(int W, int N) {
  RecodeConst c{};
  for (int i = 0; i < N; i++) {
    int bit = W * i + (W - 1);
    c.w[bit >> 5] |= 1u << (bit & 31);
  }
  return c;
}

// kp (9 words) = (k + C) << (288 - N*W): the top window sits at bits [288-W, 288).
template <int W, int N>
__device__ __forceinline__ void sc_recode_prepare(uint32_t* kp, const uint32_t* k8) {
  constexpr RecodeConst C = make_recode_const(W, N);
  uint32_t s[9];
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t t = (uint64_t)(i < 8 ? k8[i] : 0u) + C.w[i] + carry;
    s[i] = (uint32_t)t;
    carry = t >> 32;
  }
  constexpr int SH = 288 - N * W;
  constexpr int WO = SH / 32, BO = SH % 32;
  static_assert(SH >= 0 && SH < 64, "window layout");
#pragma unroll
  for (int i = 8; i >= 0; i--) {
    int src = i - WO;
    uint32_t hi = src >= 0 ? s[src] : 0u;
    uint32_t lo = src >= 1 ? s[src - 1] : 0u;
    kp[i] = BO == 0 ? hi : ((hi << BO) | (lo >> ((32 - BO) & 31)));
  }
}

// Pop the top signed digit and shift the remaining windows up.
template <int W>
__device__ __forceinline__ int sc_recode_pop(uint32_t* kp) {
  int d = (int)(kp[8] >> (32 - W)) - (1 << (W - 1));
#pragma unroll
  for (int i = 8; i > 0; i--) kp[i] = (kp[i] << W) | (kp[i - 1] >> (32 - W));
  kp[0] <<= W;
  return d;
}
