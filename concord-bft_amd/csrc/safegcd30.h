// Variable-time modular inversion for PUBLIC values (verification only): Bernstein-Yang
// "safegcd" divsteps, the variable-time form (eta = -delta, up to 8 bits of g cancelled per step
// with -f^-1 mod 2^8), in batches of 30 on 9 signed radix-2^30 limbs, as published for
// libsecp256k1's modinv32_var.  Any odd modulus below 2^269 (BN-P254's p, 2^255 - 19).
// About 13 batches of ~450 instructions for a 255-bit modulus, against ~300 squarings and
// multiplications for Fermat.  Host and device (one lane per inversion; lanes of a wave with
// different inputs diverge in the loop counts only).
#pragma once
#include <stdint.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SG_HD __host__ __device__ __forceinline__
#else
#define SG_HD inline
#endif
#define SG_M30 0x3fffffff

struct Sg30 {
  int32_t v[9];
};

// f^-1 mod 2^10 for odd f: (3 f) ^ 2 is the inverse mod 2^5, one Newton step doubles that
SG_HD uint32_t sg_inv10(uint32_t f) {
  const uint32_t x = (3u * f) ^ 2u;
  return x * (2u - f * x);
}
// 30 divsteps on the low words of f (odd) and g: eta' and the transition matrix t = (u, v, q, r)
// with (f', g') = (u f + v g, q f + r g) / 2^30.
SG_HD int32_t sg_divsteps30_var(int32_t eta, uint32_t f, uint32_t g, int32_t* t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  uint32_t nfi = 0u - sg_inv10(f);  // -f^-1 mod 2^8 and above; f changes only at a swap
  int i = 30;
  for (;;) {
    const int zeros = __builtin_ctz(g | (0xffffffffu << i));  // sentinel: at most i zeros
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    if (eta < 0) {  // (f, g) <- (g, -f) and the matrix rows with them
      uint32_t x;
      eta = -eta;
      x = f;
      f = g;
      g = 0u - x;
      x = u;
      u = q;
      q = 0u - x;
      x = v;
      v = r;
      r = 0u - x;
      nfi = 0u - sg_inv10(f);
    }
    const int limit = (eta + 1) > i ? i : (eta + 1);
    const uint32_t m = (0xffffffffu >> (32 - limit)) & 255u;
    const uint32_t w = (g * nfi) & m;  // cancels the low min(limit, 8) bits of g
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t[0] = (int32_t)u;
  t[1] = (int32_t)v;
  t[2] = (int32_t)q;
  t[3] = (int32_t)r;
  return eta;
}

// (d, e) <- (t [d, e] + p [md, me]) / 2^30 with md, me chosen to clear the low 30 bits
template <class M>
SG_HD void sg_update_de30(Sg30& d, Sg30& e, const int32_t* t) {
  const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
  const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
  int32_t md = (u & sd) + (v & se), me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d.v[0] + (int64_t)v * e.v[0];
  int64_t ce = (int64_t)q * d.v[0] + (int64_t)r * e.v[0];
  md -= (int32_t)((M::PINV30 * (uint32_t)cd + (uint32_t)md) & SG_M30);
  me -= (int32_t)((M::PINV30 * (uint32_t)ce + (uint32_t)me) & SG_M30);
  cd += (int64_t)M::P[0] * md;
  ce += (int64_t)M::P[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    cd += (int64_t)u * d.v[i] + (int64_t)v * e.v[i] + (int64_t)M::P[i] * md;
    ce += (int64_t)q * d.v[i] + (int64_t)r * e.v[i] + (int64_t)M::P[i] * me;
    d.v[i - 1] = (int32_t)cd & SG_M30;
    cd >>= 30;
    e.v[i - 1] = (int32_t)ce & SG_M30;
    ce >>= 30;
  }
  d.v[8] = (int32_t)cd;
  e.v[8] = (int32_t)ce;
}

// (f, g) <- t [f, g] / 2^30
SG_HD void sg_update_fg30(Sg30& f, Sg30& g, const int32_t* t) {
  const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
  int64_t cf = (int64_t)u * f.v[0] + (int64_t)v * g.v[0];
  int64_t cg = (int64_t)q * f.v[0] + (int64_t)r * g.v[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    cf += (int64_t)u * f.v[i] + (int64_t)v * g.v[i];
    cg += (int64_t)q * f.v[i] + (int64_t)r * g.v[i];
    f.v[i - 1] = (int32_t)cf & SG_M30;
    cf >>= 30;
    g.v[i - 1] = (int32_t)cg & SG_M30;
    cg >>= 30;
  }
  f.v[8] = (int32_t)cf;
  g.v[8] = (int32_t)cg;
}

// d in (-2p, p) -> (sign < 0 ? -d : d) mod p in [0, p)
template <class M>
SG_HD void sg_normalize30(Sg30& d, int32_t sign) {
  const int32_t neg = sign >> 31;
  int32_t add = d.v[8] >> 31;
#pragma unroll
  for (int i = 0; i < 9; i++) d.v[i] = ((d.v[i] + (M::P[i] & add)) ^ neg) - neg;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    d.v[i + 1] += d.v[i] >> 30;
    d.v[i] &= SG_M30;
  }
  add = d.v[8] >> 31;
#pragma unroll
  for (int i = 0; i < 9; i++) d.v[i] += M::P[i] & add;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    d.v[i + 1] += d.v[i] >> 30;
    d.v[i] &= SG_M30;
  }
}

// x in [0, p) (signed-30 limbs, each in [0, 2^30)) -> x^-1 mod p in [0, p); 0 -> 0.  VARIABLE TIME.
// M: P[9] (the odd modulus in signed-30 limbs), PINV30 = P^-1 mod 2^30.
template <class M>
SG_HD void sg_inv30_var(Sg30& x) {
  Sg30 f, g = x, d, e;
#pragma unroll
  for (int j = 0; j < 9; j++) {
    f.v[j] = M::P[j];
    d.v[j] = 0;
    e.v[j] = j == 0 ? 1 : 0;
  }
  int32_t eta = -1;
  for (int it = 0; it < 64; it++) {  // g = 0 after <= 25 batches for 255 bits (bound 741 divsteps)
    int32_t t[4];
    eta = sg_divsteps30_var(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    sg_update_de30<M>(d, e, t);
    sg_update_fg30(f, g, t);
    int32_t any = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) any |= g.v[j];
    if (any == 0) break;
  }
  sg_normalize30<M>(d, f.v[8]);  // f = +-1: d = +-x^-1
  x = d;
}

// ---- the same inversion spread over a wave (sg_inv30_var_wave) ---------------------------------
// For a value every lane holds (a finish block's tree root, a pairing check's norm).  The divsteps
// run on the scalar unit (their inputs are the low limbs, read from lane 0); the four updates
// (d, e, f, g) <- (t [d, e] + p [md, me], t [f, g]) / 2^30 run lane-parallel: lane j < 9 holds limb
// j of d, e, f and g (lanes >= 9 hold 0), forms its column c_j = u d_j + v e_j + P_j md (one int64 per
// vector), and the division by 2^30 is two limb splits with a neighbour exchange each:
//   pass 1  c_j = hi_j 2^30 + lo_j, lo in [0, 2^30):        x_k = lo_(k+1) + hi_k    (|x_k| < 2^33)
//   pass 2  x_k = hi'_k 2^30 + lo'_k (top lane 8 kept whole): limb_k = lo'_k + hi'_(k-1)
// so limbs below the top end in [-4, 2^30 + 4] (redundant; limb 0 exact mod 2^30, all the divsteps
// read) instead of the sequential 9-limb carry chain the scalar form runs 4 times per batch.
// Bounds: |u| + |v| <= 2^30, |md| <= 2^31, limbs <= 2^30 + 4: |c_j| < 2^60 (1 + 2^-27) + 2^61 < 2^63.
// The sign of d (which of p's multiples md adds) is read from the top limb as before; with
// redundant lower limbs a value within 2^214 of 0 can read the wrong sign, which moves the result's
// range (-2p, p) by less than 2^214 for that batch and never compounds (the next update scales it
// by (|u| + |v|) / 2^30 <= 1); sg_canon30 takes the final d from any such range to [0, p).
// g = 0 is tested exactly (a zero value often has redundant limbs, 2^30 next to -1): a cheap
// per-lane test that every limb could belong to a zero, then the scalar carry chain.

// pass 1 of one lane: c = hi 2^30 + lo
SG_HD void sg_w_split1(int64_t c, uint32_t& lo, int64_t& hi) {
  lo = (uint32_t)c & SG_M30;
  hi = c >> 30;
}
// pass 2 of one lane: x = hi + lo of the lane above; the top lane keeps x whole
SG_HD void sg_w_split2(int64_t hi, uint32_t lo_above, bool top, int32_t& lo2, int32_t& hi2) {
  const int64_t x = hi + (int64_t)lo_above;
  lo2 = top ? (int32_t)x : (int32_t)((uint32_t)x & SG_M30);
  hi2 = top ? 0 : (int32_t)(x >> 30);
}
// a limb that can be part of a zero value (limbs in [-4, 2^30 + 4], carries in {-1, 0, 1}):
// 0, +-1, 2^30, 2^30 +- 1.  The loop's cheap test; the exact one (sg_is_zero30) runs only when
// every limb passes it.
SG_HD bool sg_w_zero_limb(int32_t x) {
  return (uint32_t)(x + 1) <= 2u || (uint32_t)(x - (1 << 30) + 1) <= 2u;
}
SG_HD bool sg_is_zero30(Sg30 x) {
  int32_t any = 0;
  for (int i = 0; i < 8; i++) {
    x.v[i + 1] += x.v[i] >> 30;
    any |= x.v[i] & SG_M30;
  }
  return (any | x.v[8]) == 0;
}
// md, me of sg_update_de30 from d's and e's low limbs and top limbs (the low 32 bits of the
// column-0 sums suffice: only their residues mod 2^30 are used)
template <class M>
SG_HD void sg_w_m(int32_t& md, int32_t& me, const int32_t* t, int32_t d0, int32_t e0, int32_t d8, int32_t e8) {
  const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
  const int32_t sd = d8 >> 31, se = e8 >> 31;
  md = (u & sd) + (v & se);
  me = (q & sd) + (r & se);
  const uint32_t cd = (uint32_t)u * (uint32_t)d0 + (uint32_t)v * (uint32_t)e0;
  const uint32_t ce = (uint32_t)q * (uint32_t)d0 + (uint32_t)r * (uint32_t)e0;
  md -= (int32_t)((M::PINV30 * cd + (uint32_t)md) & SG_M30);
  me -= (int32_t)((M::PINV30 * ce + (uint32_t)me) & SG_M30);
}
// (sign < 0 ? -d : d) mod p in [0, p) for d with any int32 limbs whose value lies in (-3p, 3p)
template <class M>
SG_HD void sg_canon30(Sg30& d, int32_t sign) {
  auto carry = [&d]() {
    for (int i = 0; i < 8; i++) {
      d.v[i + 1] += d.v[i] >> 30;
      d.v[i] &= SG_M30;
    }
  };
  carry();
  if (sign < 0) {
    for (int i = 0; i < 9; i++) d.v[i] = -d.v[i];
    carry();
  }
  while (d.v[8] < 0) {  // the top limb's sign is the value's once the low limbs are in [0, 2^30)
    for (int i = 0; i < 9; i++) d.v[i] += M::P[i];
    carry();
  }
  for (;;) {  // subtract p while d >= p
    Sg30 t;
    for (int i = 0; i < 9; i++) t.v[i] = d.v[i] - M::P[i];
    for (int i = 0; i < 8; i++) {
      t.v[i + 1] += t.v[i] >> 30;
      t.v[i] &= SG_M30;
    }
    if (t.v[8] < 0) break;
    d = t;
  }
}

#if defined(__HIP_DEVICE_COMPILE__)
// one lane's update column c -> its limb of c / 2^30 (passes 1 and 2 with the DPP row shifts:
// row_shl:1 reads the lane above, row_shr:1 the lane below, 0 past the row's edge)
__device__ __forceinline__ int32_t sg_w_column(int64_t c, bool top) {
  uint32_t lo;
  int64_t hi;
  sg_w_split1(c, lo, hi);
  const uint32_t la = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0x101, 0xF, 0xF, true);
  int32_t lo2, hi2;
  sg_w_split2(hi, la, top, lo2, hi2);
  return lo2 + __builtin_amdgcn_update_dpp(0, hi2, 0x111, 0xF, 0xF, true);
}

// x^-1 mod p in [0, p) for x in [0, p) held (the same) by every lane; 0 -> 0.  The whole wave must
// be active (lanes 0..9 take part in the exchanges).  VARIABLE TIME.  Result: wave-uniform.
template <class M>
__device__ __forceinline__ void sg_inv30_var_wave(Sg30& x) {
  const uint32_t ln = __lane_id();
  const bool top = ln == 8;
  int32_t P = 0, g = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    P = ln == (uint32_t)k ? M::P[k] : P;
    g = ln == (uint32_t)k ? x.v[k] : g;
  }
  int32_t f = P, d = 0, e = ln == 0 ? 1 : 0;
  int32_t eta = -1;
  for (int it = 0; it < 64; it++) {  // <= 25 batches for 255 bits, + <= 8 for a redundant zero
    int32_t t[4];
    eta = sg_divsteps30_var(eta, (uint32_t)__builtin_amdgcn_readlane(f, 0), (uint32_t)__builtin_amdgcn_readlane(g, 0),
                            t);
    int32_t md, me;
    sg_w_m<M>(md, me, t, __builtin_amdgcn_readlane(d, 0), __builtin_amdgcn_readlane(e, 0),
              __builtin_amdgcn_readlane(d, 8), __builtin_amdgcn_readlane(e, 8));
    const int64_t cd = (int64_t)t[0] * d + (int64_t)t[1] * e + (int64_t)P * md;
    const int64_t ce = (int64_t)t[2] * d + (int64_t)t[3] * e + (int64_t)P * me;
    const int64_t cf = (int64_t)t[0] * f + (int64_t)t[1] * g;
    const int64_t cg = (int64_t)t[2] * f + (int64_t)t[3] * g;
    d = sg_w_column(cd, top);
    e = sg_w_column(ce, top);
    f = sg_w_column(cf, top);
    g = sg_w_column(cg, top);
    if (__ballot(!sg_w_zero_limb(g)) == 0) {
      Sg30 gg;
#pragma unroll
      for (int k = 0; k < 9; k++) gg.v[k] = __builtin_amdgcn_readlane(g, k);
      if (sg_is_zero30(gg)) break;
    }
  }
  // f = +-1: its exact limb 0 is 1 or 2^30 - 1
  const int32_t fsign = __builtin_amdgcn_readlane(f, 0) == 1 ? 1 : -1;
#pragma unroll
  for (int k = 0; k < 9; k++) x.v[k] = __builtin_amdgcn_readlane(d, k);
  sg_canon30<M>(x, fsign);
}
#endif

// value of 9 29-bit limbs (< 2^261, < p here) <-> 9 signed-30 limbs
SG_HD void sg_from_limbs29(Sg30& x, const uint32_t* c) {
#pragma unroll
  for (int j = 0; j < 9; j++) {
    const int b = 30 * j, i = b / 29, s = b % 29;
    const uint64_t w = ((uint64_t)(i + 1 < 9 ? c[i + 1] : 0u) << 29) | c[i];
    x.v[j] = (int32_t)((w >> s) & SG_M30);
  }
}
SG_HD void sg_to_limbs29(uint32_t* c, const Sg30& x) {
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int b = 29 * i, j = b / 30, s = b % 30;
    const uint64_t w = ((uint64_t)(uint32_t)(j + 1 < 9 ? x.v[j + 1] : 0) << 30) | (uint32_t)x.v[j];
    c[i] = (uint32_t)(w >> s) & 0x1fffffffu;
  }
}
