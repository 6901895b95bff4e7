// BN-P254 prime fields (Fp: base field, Fr: group order) for gfx950 and for the host, one
// element per lane.  Same source compiles as HIP device code and as plain C++ (the host build
// is used for tests and for the labelled "not RELIC" CPU baseline).
//
// Representation: Montgomery form, 9 limbs x 29 bits (R = 2^261), limbs normalised (< 2^29),
// value < 2q ("reduced", q = the modulus).  Multiplication is FIPS (finely integrated product
// scanning): column k accumulates every a_i b_j and m_j q_(k-j) into one 64-bit accumulator
// with v_mad_u64_u32, so there is no per-product carry chain: 81 + 81 mads per multiply,
// 45 + 81 per square.  Column bound: 18 products < 2^58 plus carry < 2^63 (normalised inputs).
// Output of mont_mul for inputs < 2q is < 2q (R = 2^261 > 4q).
#pragma once
#include <stdint.h>
#include "safegcd30.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BN_HD __host__ __device__ __forceinline__
// Heavy tower/curve/pairing routines are compiled once and called (objects pass through
// scratch): fully inlining the pairing into its kernels makes the code object explode
// (a > 40 min compile measured); field-level ops stay inlined inside each routine.
#define BN_HDN static __host__ __device__ __noinline__
#else
#define BN_HD inline
#define BN_HDN inline
#endif

#define BN_LIMBS 9
#define BN_MASK 0x1fffffffu

struct FpParams {  // p = 36u^4 + 36u^3 + 24u^2 + 6u + 1, u = -(2^62 + 2^55 + 1)
  static constexpr uint32_t Q[9] = {0x00000013u, 0x18000000u, 0x000004e9u, 0x02000000u, 0x00008612u,
                                    0x06c00000u, 0x0006e8d1u, 0x10480000u, 0x00252364u};
  static constexpr uint32_t NPRIME = 0x179435e5u;  // -q^-1 mod 2^29
  static constexpr uint32_t R2[9] = {0x011cbcb5u, 0x18ce8a6eu, 0x03e367a8u, 0x097460e6u, 0x124f515fu,
                                     0x123f0d2au, 0x1e665acbu, 0x19981d1du, 0x0014cc78u};
  static constexpr uint32_t ONE[9] = {0x1fffefacu, 0x1fffffffu, 0x1ffbc71eu, 0x07ffffffu, 0x1f8cc87au,
                                      0x12ffffffu, 0x1a0fec35u, 0x021fffffu, 0x001595a0u};
};
struct FrParams {  // r = 36u^4 + 36u^3 + 18u^2 + 6u + 1 (the order of G1, G2, GT)
  static constexpr uint32_t Q[9] = {0x0000000du, 0x08000000u, 0x00000428u, 0x1f000000u, 0x00007ff9u,
                                    0x06c00000u, 0x0006e8d1u, 0x10480000u, 0x00252364u};
  static constexpr uint32_t NPRIME = 0x1b13b13bu;
  static constexpr uint32_t R2[9] = {0x0a9e505bu, 0x0ad6de81u, 0x1eb35b9fu, 0x1d971118u, 0x1c3bba09u,
                                     0x05eebab4u, 0x00bd2046u, 0x0b27c81au, 0x001934a7u};
  static constexpr uint32_t ONE[9] = {0x1ffff4d4u, 0x1fffffffu, 0x1ffc6d68u, 0x1bffffffu, 0x1f92052eu,
                                      0x12ffffffu, 0x1a0fec35u, 0x021fffffu, 0x001595a0u};
};

template <class F>
struct Fe {
  uint32_t v[BN_LIMBS];
};
using fp = Fe<FpParams>;
using fr = Fe<FrParams>;

BN_HD uint64_t bn_mad(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * (uint64_t)b + c; }

template <class F>
BN_HD void f_zero(Fe<F>& r) {
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) r.v[i] = 0;
}
template <class F>
BN_HD void f_one(Fe<F>& r) {
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) r.v[i] = F::ONE[i];
}

// Montgomery reduction of 17 product columns c[0..16] (each < 2^61.2, c[17] = 0 spare):
// word-serial REDC, m_k = c_k * (-q^-1) mod 2^29, then m_k q added into columns k..k+8.  The
// only serial dependency is column k -> m_k -> column k+1 (about 4 instructions per step);
// the 9 mads of each step are independent.  Columns stay < 2^62.2 + carries.
// A modulus limb that is a power of two (p's limb 3 is 2^25) is passed to its mad as an opaque
// SGPR: LLVM would otherwise strength-reduce m_k * 2^25 + c into a 64-bit shift plus a 64-bit add,
// two half-rate instructions where the mad is one.
template <class F>
BN_HD uint32_t bn_qlimb(int i) {
  uint32_t q = F::Q[i];
#if defined(__HIP_DEVICE_COMPILE__)
  if ((q & (q - 1u)) == 0u) asm("" : "+s"(q));
#endif
  return q;
}
template <class F>
BN_HD void f_redc(Fe<F>& r, uint64_t* c) {
#pragma unroll
  for (int k = 0; k < BN_LIMBS; k++) {
    const uint32_t mk = ((uint32_t)c[k] * F::NPRIME) & BN_MASK;
    c[k] = bn_mad(mk, F::Q[0], c[k]);  // low 29 bits become 0
    c[k + 1] = bn_mad(mk, F::Q[1], c[k + 1]) + (c[k] >> 29);
#pragma unroll
    for (int i = 2; i < BN_LIMBS; i++) c[k + i] = bn_mad(mk, bn_qlimb<F>(i), c[k + i]);
  }
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < BN_LIMBS - 1; i++) {
    acc += c[BN_LIMBS + i];
    r.v[i] = (uint32_t)acc & BN_MASK;
    acc >>= 29;
  }
  r.v[BN_LIMBS - 1] = (uint32_t)(acc + c[2 * BN_LIMBS - 1]);  // value < 2q < 2^255
}

// r = a * b * 2^-261 mod q (a, b < 2q, normalised)  ->  r < 2q, normalised.  Product columns
// first (17 independent mad chains), then f_redc: bit-identical to the interleaved FIPS form
// (the same m_k), but with a dependency chain ~4x shorter, which is what a pairing running on
// few lanes waits on.
//
// Accumulation order is row-wise (a_i against every b_j): consecutive mads update different
// columns, so a lone wave (a pairing check runs one wave per SIMD) issues them back to back
// instead of waiting out the v_mad_u64_u32 latency of a column chain.
template <class F>
BN_HD void f_mul(Fe<F>& r, const Fe<F>& a, const Fe<F>& b) {
  uint64_t c[2 * BN_LIMBS];
#pragma unroll
  for (int k = 0; k < 2 * BN_LIMBS; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
#pragma unroll
    for (int j = 0; j < BN_LIMBS; j++) c[i + j] = bn_mad(a.v[i], b.v[j], c[i + j]);
  }
  f_redc(r, c);
}

// r = (a b + c d) 2^-261 mod q: both products' columns in one set of accumulators and ONE
// f_redc (half the reductions of two f_mul and a sum).  a, b normalised (< 2q); c may have limbs
// up to 2^30 (a redundant negation, value < 4q), d normalised.  Columns < 9 2^58 + 9 2^59 < 2^62.6
// (+ the REDC terms, < 2^63.1); the value ab + cd < 12 q^2 < q 2^261, so the result is < 2q.
template <class F>
BN_HD void f_mul_sum2(Fe<F>& r, const Fe<F>& a, const Fe<F>& b, const Fe<F>& c, const Fe<F>& d) {
  uint64_t t[2 * BN_LIMBS];
#pragma unroll
  for (int k = 0; k < 2 * BN_LIMBS; k++) t[k] = 0;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
#pragma unroll
    for (int j = 0; j < BN_LIMBS; j++) t[i + j] = bn_mad(a.v[i], b.v[j], t[i + j]);
  }
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
#pragma unroll
    for (int j = 0; j < BN_LIMBS; j++) t[i + j] = bn_mad(c.v[i], d.v[j], t[i + j]);
  }
  f_redc(r, t);
}

template <class F>
BN_HD void f_sqr(Fe<F>& r, const Fe<F>& a) {
  uint32_t a2[BN_LIMBS];
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) a2[i] = a.v[i] << 1;
  uint64_t c[2 * BN_LIMBS];
#pragma unroll
  for (int k = 0; k < 2 * BN_LIMBS; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {  // row-wise, as f_mul
    c[2 * i] = bn_mad(a.v[i], a.v[i], c[2 * i]);
#pragma unroll
    for (int j = i + 1; j < BN_LIMBS; j++) c[i + j] = bn_mad(a2[i], a.v[j], c[i + j]);
  }
  f_redc(r, c);
}

// t = a - c*q for the selected c (c = 0 or 1 times q or 2q via `sub`), keep if non-negative
template <class F>
BN_HD void f_csub(Fe<F>& a, const uint32_t* s) {  // a -= s if a >= s (a, s normalised)
  uint32_t t[BN_LIMBS];
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
    int32_t d = (int32_t)a.v[i] - (int32_t)s[i] + br;
    t[i] = (uint32_t)d & BN_MASK;
    br = d >> 29;  // 0 or -1
  }
  const bool keep = br == 0;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) a.v[i] = keep ? t[i] : a.v[i];
}

template <class F>
BN_HD void f_2q(uint32_t* s) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
    uint32_t x = (F::Q[i] << 1) + c;
    s[i] = x & BN_MASK;
    c = x >> 29;
  }
}

// true in every lane of the wave when any lane's pred holds (device); pred itself on the host
BN_HD bool bn_any(bool pred) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __any(pred);
#else
  return pred;
#endif
}

// r += 2q where fix (the correction pass of f_add / f_sub, rarely taken)
template <class F>
BN_HD void f_add_2q_where(Fe<F>& r, bool fix) {
  uint32_t q2[BN_LIMBS];
  f_2q<F>(q2);
  const uint32_t msk = fix ? BN_MASK : 0u;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
    const uint32_t x = r.v[i] + (q2[i] & msk) + c;
    r.v[i] = x & BN_MASK;
    c = x >> 29;
  }
}

// r = a + b reduced below 2q (a, b < 2q, normalised).  The reduction is decided from the top
// limbs: with T = top limb of 2q, a + b lies in [t, t + 2) 2^232 for t = a8 + b8, so t + 2 <= T
// means a + b < 2q (keep); otherwise 2q is subtracted in the same signed carry pass as the add
// (~40 instructions against ~70 for add + trial subtraction).  Only for t in {T - 1, T} can
// that go negative (probability ~2^-21 per random operand pair): the final carry says so and a
// correction pass adds 2q back, executed by a wave only when one of its lanes needs it.  The
// result is the same reduced value as the trial-subtraction form.
template <class F>
BN_HD void f_add(Fe<F>& r, const Fe<F>& a, const Fe<F>& b) {
  uint32_t q2[BN_LIMBS];
  f_2q<F>(q2);
  const uint32_t t = a.v[BN_LIMBS - 1] + b.v[BN_LIMBS - 1];
  const uint32_t msk = t + 2 > q2[BN_LIMBS - 1] ? BN_MASK : 0u;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
    const int32_t x = (int32_t)(a.v[i] + b.v[i]) - (int32_t)(q2[i] & msk) + c;
    r.v[i] = (uint32_t)x & BN_MASK;
    c = x >> 29;
  }
  if (bn_any(c < 0)) f_add_2q_where(r, c < 0);
}

// r = a - b reduced below 2q (a, b < 2q, normalised): a8 < b8 means a < b, so 2q is added in
// the same signed pass; otherwise nothing is added, and when the top limbs were equal and
// a < b after all, the final borrow triggers the correction pass.
template <class F>
BN_HD void f_sub(Fe<F>& r, const Fe<F>& a, const Fe<F>& b) {
  uint32_t q2[BN_LIMBS];
  f_2q<F>(q2);
  const uint32_t msk = a.v[BN_LIMBS - 1] < b.v[BN_LIMBS - 1] ? BN_MASK : 0u;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
    const int32_t x = (int32_t)a.v[i] - (int32_t)b.v[i] + (int32_t)(q2[i] & msk) + c;
    r.v[i] = (uint32_t)x & BN_MASK;
    c = x >> 29;
  }
  if (bn_any(c < 0)) f_add_2q_where(r, c < 0);
}

// r = add ? a + b : a - b, reduced below 2q (a, b < 2q, normalised), for lanes that pick one
// of the two per lane (the Fp2 / Fp12 component formulas): one signed pass instead of both
// operations and a select.  Same reduction rule as f_add / f_sub, so the same results.
template <class F>
BN_HD void f_addsub(Fe<F>& r, const Fe<F>& a, const Fe<F>& b, bool add) {
  uint32_t q2[BN_LIMBS];
  f_2q<F>(q2);
  const uint32_t a8 = a.v[BN_LIMBS - 1], b8 = b.v[BN_LIMBS - 1];
  const bool corr = add ? a8 + b8 + 2 > q2[BN_LIMBS - 1] : a8 < b8;  // -2q (add) / +2q (sub)
  const int32_t bs = add ? 0 : -1;  // b's sign: (b ^ bs) - bs = +-b
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
    const int32_t bi = ((int32_t)b.v[i] ^ bs) - bs;
    const int32_t qi = corr ? (add ? -(int32_t)q2[i] : (int32_t)q2[i]) : 0;
    const int32_t x = (int32_t)a.v[i] + bi + qi + c;
    r.v[i] = (uint32_t)x & BN_MASK;
    c = x >> 29;
  }
  if (bn_any(c < 0)) f_add_2q_where(r, c < 0);
}

template <class F>
BN_HD void f_neg(Fe<F>& r, const Fe<F>& a) {
  Fe<F> z;
  f_zero(z);
  f_sub(r, z, a);
}

template <class F>
BN_HD void f_dbl(Fe<F>& r, const Fe<F>& a) {
  f_add(r, a, a);
}

// canonical value in [0, q) (still Montgomery form)
template <class F>
BN_HD void f_canon(Fe<F>& a) {
  f_csub(a, F::Q);
}

template <class F>
BN_HD bool f_eq(const Fe<F>& a, const Fe<F>& b) {
  Fe<F> x = a, y = b;
  f_canon(x);
  f_canon(y);
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) d |= x.v[i] ^ y.v[i];
  return d == 0;
}

template <class F>
BN_HD bool f_is_zero(const Fe<F>& a) {
  Fe<F> x = a;
  f_canon(x);
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) d |= x.v[i];
  return d == 0;
}

// integer (8 little-endian 32-bit words, < q) -> Montgomery
template <class F>
BN_HD void f_from_words(Fe<F>& r, const uint32_t* w) {
  Fe<F> t, r2;
  t.v[0] = w[0] & BN_MASK;
  t.v[1] = ((w[0] >> 29) | (w[1] << 3)) & BN_MASK;
  t.v[2] = ((w[1] >> 26) | (w[2] << 6)) & BN_MASK;
  t.v[3] = ((w[2] >> 23) | (w[3] << 9)) & BN_MASK;
  t.v[4] = ((w[3] >> 20) | (w[4] << 12)) & BN_MASK;
  t.v[5] = ((w[4] >> 17) | (w[5] << 15)) & BN_MASK;
  t.v[6] = ((w[5] >> 14) | (w[6] << 18)) & BN_MASK;
  t.v[7] = ((w[6] >> 11) | (w[7] << 21)) & BN_MASK;
  t.v[8] = (w[7] >> 8);
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) r2.v[i] = F::R2[i];
  f_mul(r, t, r2);
}

// Montgomery -> canonical integer words
template <class F>
BN_HD void f_to_words(uint32_t* w, const Fe<F>& a) {
  Fe<F> one, t;
  f_zero(one);
  one.v[0] = 1;
  f_mul(t, a, one);
  f_canon(t);
  w[0] = t.v[0] | (t.v[1] << 29);
  w[1] = (t.v[1] >> 3) | (t.v[2] << 26);
  w[2] = (t.v[2] >> 6) | (t.v[3] << 23);
  w[3] = (t.v[3] >> 9) | (t.v[4] << 20);
  w[4] = (t.v[4] >> 12) | (t.v[5] << 17);
  w[5] = (t.v[5] >> 15) | (t.v[6] << 14);
  w[6] = (t.v[6] >> 18) | (t.v[7] << 11);
  w[7] = (t.v[7] >> 21) | (t.v[8] << 8);
}

// r = a^e, e given as 8 little-endian words (left-to-right binary, runtime loop)
template <class F>
BN_HDN void f_pow(Fe<F>& r, const Fe<F>& a, const uint32_t* e) {
  Fe<F> acc;
  f_one(acc);
  for (int i = 255; i >= 0; i--) {
    f_sqr(acc, acc);
    if ((e[i >> 5] >> (i & 31)) & 1) f_mul(acc, acc, a);
  }
  r = acc;
}

// exponents as words
struct FpExp {
  // p - 2
  static constexpr uint32_t PM2[8] = {0x00000011u, 0xa7000000u, 0x00000013u, 0x61210000u,
                                      0x00000008u, 0xba344d80u, 0x40000001u, 0x25236482u};
  // (p + 1) / 4
  static constexpr uint32_t SQRT[8] = {0x00000005u, 0xe9c00000u, 0x00000004u, 0x18484000u,
                                       0x00000002u, 0x6e8d1360u, 0x90000000u, 0x0948d920u};
  // r - 2 (inversion in Fr)
  static constexpr uint32_t RM2[8] = {0x0000000bu, 0xa1000000u, 0x00000010u, 0xff9f8000u,
                                      0x00000007u, 0xba344d80u, 0x40000001u, 0x25236482u};
};

// exponent word arrays must live in registers on the device: copy from the constexpr table
template <class F>
BN_HD void f_inv_fp(Fe<F>& r, const Fe<F>& a) {
  uint32_t e[8];
#pragma unroll
  for (int i = 0; i < 8; i++) e[i] = FpExp::PM2[i];
  f_pow(r, a, e);
}

// Left-to-right sliding-window schedule (window 4) of a fixed public exponent: acc = a^v[0],
// then for each further window nsq[w] squarings and a multiplication by a^v[w] (v odd, < 16),
// then `tail` squarings.  Built at compile time; the schedule depends on the exponent only.
struct SwSchedule {
  int n, tail;
  uint8_t nsq[80], v[80];
};
constexpr SwSchedule sw_schedule(const uint32_t (&e)[8]) {
  SwSchedule s{};
  int i = 255;
  while (!((e[i >> 5] >> (i & 31)) & 1u)) i--;
  int pend = 0;  // squarings owed before the next window
  while (i >= 0) {
    if (!((e[i >> 5] >> (i & 31)) & 1u)) {
      pend++;
      i--;
      continue;
    }
    int j = i - 3 < 0 ? 0 : i - 3;
    while (!((e[j >> 5] >> (j & 31)) & 1u)) j++;
    uint32_t v = 0;
    for (int b = i; b >= j; b--) v = 2 * v + ((e[b >> 5] >> (b & 31)) & 1u);
    s.nsq[s.n] = (uint8_t)(s.n == 0 ? 0 : pend + (i - j + 1));
    s.v[s.n] = (uint8_t)v;
    s.n++;
    pend = 0;
    i = j - 1;
  }
  s.tail = pend;
  return s;
}
struct FpSqrtSchedule {
  static constexpr SwSchedule S = sw_schedule(FpExp::SQRT);  // 19 windows instead of 42 multiplications
};

// a^e for the schedule S: 8 odd powers a, a^3, .., a^15, then the windows (the table entry is
// picked by a wave-uniform switch, so it stays in registers)
template <class F, class Sched>
BN_HDN void f_pow_sw(Fe<F>& r, const Fe<F>& a) {
  Fe<F> t[8], a2, acc;
  t[0] = a;
  f_sqr(a2, a);
#pragma unroll
  for (int k = 1; k < 8; k++) f_mul(t[k], t[k - 1], a2);
  for (int w = 0; w < Sched::S.n; w++) {
    for (int q = 0; q < Sched::S.nsq[w]; q++) f_sqr(acc, acc);
    const int idx = Sched::S.v[w] >> 1;
    if (w == 0) {
      acc = t[0];
#pragma unroll
      for (int k = 1; k < 8; k++)
        if (idx == k) acc = t[k];
      continue;
    }
    switch (idx) {
      case 0: f_mul(acc, acc, t[0]); break;
      case 1: f_mul(acc, acc, t[1]); break;
      case 2: f_mul(acc, acc, t[2]); break;
      case 3: f_mul(acc, acc, t[3]); break;
      case 4: f_mul(acc, acc, t[4]); break;
      case 5: f_mul(acc, acc, t[5]); break;
      case 6: f_mul(acc, acc, t[6]); break;
      default: f_mul(acc, acc, t[7]); break;
    }
  }
  for (int q = 0; q < Sched::S.tail; q++) f_sqr(acc, acc);
  r = acc;
}

// square root for p = 3 mod 4: y = a^((p+1)/4); returns false if a is not a square
BN_HDN bool fp_sqrt(fp& y, const fp& a) {
  f_pow_sw<FpParams, FpSqrtSchedule>(y, a);
  fp t;
  f_sqr(t, y);
  return f_eq(t, a);
}

BN_HDN void fp_inv(fp& r, const fp& a) { f_inv_fp(r, a); }

// ---- variable-time inversion in Fp, for PUBLIC values only (the final exponentiation of a
// pairing check: signatures, message hashes, public keys): safegcd30.h.
struct BnS30Mod {  // p in signed-30 limbs, p^-1 mod 2^30, R^3 mod p (R = 2^261) in 29-bit limbs
  static constexpr int32_t P[9] = {0x00000013, 0x1c000000, 0x0000013a, 0x08400000, 0x00000861,
                                   0x11360000, 0x00001ba3, 0x19209000, 0x00002523};
  static constexpr uint32_t PINV30 = 0x286bca1bu;
  static constexpr uint32_t R3[9] = {0x1b6b46eeu, 0x090454c7u, 0x1074d76du, 0x0c39e3dcu, 0x0cbd1a82u,
                                     0x1c75654du, 0x0a20d59bu, 0x174dc09au, 0x0008606fu};
};

// r = a^-1 (Montgomery form in and out; a^-1 of 0 is 0, as Fermat's).  VARIABLE TIME.
BN_HDN void fp_inv_var(fp& r, const fp& a) {
  fp c = a;
  f_canon(c);  // [0, q): the integer A = a R mod q
  Sg30 x;
  sg_from_limbs29(x, c.v);
  sg_inv30_var<BnS30Mod>(x);  // A^-1 mod q
  fp y;
  sg_to_limbs29(y.v, x);
  fp r3;
#pragma unroll
  for (int i = 0; i < 9; i++) r3.v[i] = BnS30Mod::R3[i];
  f_mul(r, y, r3);  // A^-1 R^3 / R = a^-1 R
}

#if defined(__HIP_DEVICE_COMPILE__)
// the same for a value every lane of the wave holds, the whole wave active (a pairing check's
// norm): safegcd30.h sg_inv30_var_wave -- scalar divsteps, lane-parallel limb updates
__device__ __forceinline__ void fp_inv_var_wave(fp& r, const fp& a) {
  fp c = a;
  f_canon(c);
  Sg30 x;
  sg_from_limbs29(x, c.v);
  sg_inv30_var_wave<BnS30Mod>(x);
  fp y;
  sg_to_limbs29(y.v, x);
  fp r3;
#pragma unroll
  for (int i = 0; i < 9; i++) r3.v[i] = BnS30Mod::R3[i];
  f_mul(r, y, r3);
}
#endif

BN_HDN void fr_inv(fr& r, const fr& a) {
  uint32_t e[8];
#pragma unroll
  for (int i = 0; i < 8; i++) e[i] = FpExp::RM2[i];
  f_pow(r, a, e);
}
