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

// 30 divsteps on the low words of f (odd) and g: eta' and the transition matrix t = (u, v, q, r)
// with (f', g') = (u f + v g, q f + r g) / 2^30.
SG_HD int32_t sg_divsteps30_var(int32_t eta, uint32_t f, uint32_t g, int32_t* t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
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
    }
    const int limit = (eta + 1) > i ? i : (eta + 1);
    const uint32_t m = (0xffffffffu >> (32 - limit)) & 255u;
    uint32_t fi = f;  // f^-1 mod 2^12 by two Newton steps (f odd: f f == 1 mod 8)
    fi *= 2u - f * fi;
    fi *= 2u - f * fi;
    const uint32_t w = (g * (0u - fi)) & m;  // cancels the low min(limit, 8) bits of g
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

#if defined(__HIP_DEVICE_COMPILE__)
// The same inversion of a value every lane of the wave holds (a finish block's shared tree root, a
// pairing check's norm): the limbs are taken from the first active lane, so the whole chain is
// wave-uniform and compiles to scalar (SALU) code -- one scalar instruction stream with scalar
// branches instead of one lane's VALU stream under an exec mask.
template <class M>
__device__ __forceinline__ void sg_inv30_var_uniform(Sg30& x) {
#pragma unroll
  for (int j = 0; j < 9; j++) x.v[j] = __builtin_amdgcn_readfirstlane(x.v[j]);
  sg_inv30_var<M>(x);
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
