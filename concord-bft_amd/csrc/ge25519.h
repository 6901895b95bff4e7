// Edwards25519 group arithmetic (-x^2 + y^2 = 1 + d x^2 y^2) on the radix-2^29 field.
//
// Coordinate systems (the standard extended-coordinates family, RFC 8032 §5.1.4):
//   ge_p2    (X:Y:Z)          x = X/Z, y = Y/Z
//   ge_p3    (X:Y:Z:T)        additionally xy = T/Z
//   ge_p1p1  ((X:Z),(Y:T))    x = X/Z, y = Y/T   ("completed", output of dbl/add)
//   ge_cached (Y+X, Y-X, Z, 2dT)   addend form of a p3 point
// Limb bounds of every field value are annotated (R = reduced, Lz = lazy), see fe25519.h.
#pragma once
#include "fe25519.h"
#include "fe25519_row.h"

struct ge_p2 {
  fe X, Y, Z;
};
struct ge_p3 {
  fe X, Y, Z, T;
};
struct ge_p1p1 {
  fe X, Y, Z, T;
};
struct ge_cached {
  fe YpX, YmX, Z, T2d;
};

__device__ __constant__ const uint32_t kFeD[9] = {0x135978a3u, 0x0f5a6e50u, 0x10762addu, 0x00149a82u, 0x1e898007u,
                                                  0x003cbbbcu, 0x19ce331du, 0x1dc56dffu, 0x0052036cu};
__device__ __constant__ const uint32_t kFeD2[9] = {0x06b2f159u, 0x1eb4dca1u, 0x00ec55bau, 0x00293505u, 0x1d13000eu,
                                                   0x00797779u, 0x139c663au, 0x1b8adbffu, 0x002406d9u};
__device__ __constant__ const uint32_t kFeSqrtM1[9] = {0x0a0ea0b0u, 0x0770d93au, 0x0bf91e31u, 0x06300d5au, 0x1d7a72f4u,
                                                       0x004c9efdu, 0x1c2cad34u, 0x1009f83bu, 0x002b8324u};

FE_INLINE void fe_load_const(fe& r, const uint32_t* c) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) r.v[i] = c[i];
}

FE_INLINE void ge_p3_0(ge_p3& h) {
  fe_0(h.X);
  fe_1(h.Y);
  fe_1(h.Z);
  fe_0(h.T);
}

FE_INLINE void ge_cached_0(ge_cached& c) {
  fe_1(c.YpX);
  fe_1(c.YmX);
  fe_1(c.Z);
  fe_0(c.T2d);
}

// p1p1 -> p2 (3M).  Inputs: X,Z,T reduced, Y lazy.
FE_INLINE void ge_p1p1_to_p2(ge_p2& r, const ge_p1p1& p) {
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
}

// p1p1 -> p3 (4M)
FE_INLINE void ge_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) {
  fe_mul(r.T, p.X, p.Y);
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
}

// 2*p (p given in p2 or p3 form; only X,Y,Z read).  4S.
//   XX = X^2, YY = Y^2, B = 2Z^2, AA = (X+Y)^2
//   X' = AA - (YY+XX), Y' = YY+XX, Z' = YY-XX, T' = B - (YY-XX)
FE_INLINE void ge_dbl(ge_p1p1& r, const fe& X, const fe& Y, const fe& Z) {
  fe XX, YY, B, A;
  fe_sq(XX, X);
  fe_sq(YY, Y);
  fe_sq(B, Z);
  fe_add(B, B, B);        // Lz
  fe_add(A, X, Y);        // Lz
  fe_sq(A, A);            // R
  fe_add(r.Y, YY, XX);    // Lz
  fe_sub(r.Z, YY, XX);    // R
  fe_sub(r.X, A, r.Y);    // R
  fe_sub(r.T, B, r.Z);    // R
}

// p + q (q cached).  4M (3M when q.Z == 1 is known: zIsOne).
FE_INLINE void ge_add(ge_p1p1& r, const ge_p3& p, const ge_cached& q, bool zIsOne) {
  fe A, B, C, D, t;
  fe_add(t, p.Y, p.X);    // Lz
  fe_mul(A, t, q.YpX);
  fe_sub(t, p.Y, p.X);    // R
  fe_mul(B, t, q.YmX);
  fe_mul(C, q.T2d, p.T);
  if (zIsOne) {
    fe_copy(D, p.Z);
  } else {
    fe_mul(D, p.Z, q.Z);
  }
  fe_add(D, D, D);        // Lz
  fe_sub(r.X, A, B);      // R
  fe_add(r.Y, A, B);      // Lz
  fe_add(r.Z, D, C);      // 3R -> carry
  fe_carry(r.Z);          // R
  fe_sub(r.T, D, C);      // R
}

FE_INLINE void ge_p3_to_cached(ge_cached& c, const ge_p3& p) {
  fe_add(c.YpX, p.Y, p.X);
  fe_carry(c.YpX);
  fe_sub(c.YmX, p.Y, p.X);
  fe_copy(c.Z, p.Z);
  fe d2;
  fe_load_const(d2, kFeD2);
  fe_mul(c.T2d, p.T, d2);
}

// Conditionally negate a cached point: -(x,y) = (-x,y): swap Y+X <-> Y-X, T2d -> -T2d.
FE_INLINE void ge_cached_cneg(ge_cached& c, bool neg) {
  fe n;
  fe_neg(n, c.T2d);
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) {
    uint32_t a = c.YpX.v[i], b = c.YmX.v[i];
    c.YpX.v[i] = neg ? b : a;
    c.YmX.v[i] = neg ? a : b;
    c.T2d.v[i] = neg ? n.v[i] : c.T2d.v[i];
  }
}

// Decode a 32-byte point with OpenSSL 3.0.2 ge_frombytes_vartime semantics:
//   y = low 255 bits, NOT required canonical; x from the (p+3)/8 root; off-curve -> fail;
//   sign bit applied by negation (x == 0 with sign 1 is accepted).  Returns true on success.
FE_INLINE bool ge_frombytes(ge_p3& h, const uint32_t* w) {
  fe u, v, v3, vxx, chk, one, d;
  fe_from_words(h.Y, w);
  fe_1(h.Z);
  fe_1(one);
  fe_load_const(d, kFeD);
  fe_sq(u, h.Y);
  fe_mul(v, u, d);
  fe_sub(u, u, one);      // u = y^2 - 1
  fe_add(v, v, one);      // v = d y^2 + 1 (Lz)
  fe_carry(v);
  fe_sq(v3, v);
  fe_mul(v3, v3, v);      // v^3
  fe_sq(h.X, v3);
  fe_mul(h.X, h.X, v);
  fe_mul(h.X, h.X, u);    // u v^7
  fe_pow22523(h.X, h.X);  // (u v^7)^((p-5)/8)
  fe_mul(h.X, h.X, v3);
  fe_mul(h.X, h.X, u);    // x = u v^3 (u v^7)^((p-5)/8)
  fe_sq(vxx, h.X);
  fe_mul(vxx, vxx, v);
  fe_sub(chk, vxx, u);
  bool ok = true;
  if (!fe_iszero(chk)) {
    fe_add(chk, vxx, u);
    if (!fe_iszero(chk)) ok = false;
    fe sm1;
    fe_load_const(sm1, kFeSqrtM1);
    fe_mul(h.X, h.X, sm1);
  }
  uint32_t sign = w[7] >> 31;
  if (fe_isnegative(h.X) != sign) fe_neg(h.X, h.X);
  fe_mul(h.T, h.X, h.Y);
  return ok;
}

// ge_frombytes for a whole 16-lane DPP row holding the same w: the square-root chain runs in the
// row-parallel field (fe25519_row.h, ~2x less latency per squaring on a lone wave), the checks
// and the sign in the one-lane field as above.  Same point, same verdict; X and Y only (the small
// kernels' projective comparison needs no T).
FE_INLINE void rfe_to_fe(fe& r, uint32_t x) {
  r.v[0] = rl_bcast_w<0>(x);
  r.v[1] = rl_bcast_w<1>(x);
  r.v[2] = rl_bcast_w<2>(x);
  r.v[3] = rl_bcast_w<3>(x);
  r.v[4] = rl_bcast_w<4>(x);
  r.v[5] = rl_bcast_w<5>(x);
  r.v[6] = rl_bcast_w<6>(x);
  r.v[7] = rl_bcast_w<7>(x);
  r.v[8] = rl_bcast_w<8>(x);
  fe_carry(r);
}
// SYNC: one __syncthreads() inside the square-root chain (the three-wave fused kernel's
// "schedules written" barrier, which the decode waves reach ~12 us in, when waves 0 and 1 do)
template <bool SYNC = false>
FE_INLINE bool ge_frombytes_row(fe& X, fe& Y, const uint32_t* w) {
  typedef uint32_t U;
  typedef uint64_t W;
  fe_from_words(Y, w);
  const U tag = 0u;
  const U one = rl_index(tag) == 0u ? 1u : 0u;
  const U y = rfe_row_const(Y.v, tag);
  const U yy = rfe_sq<U, W>(y);
  const U u = rfe_sub(yy, one);                                   // y^2 - 1
  const U v = rfe_carry(rfe_mul<U, W>(yy, rfe_row_const(kFeD, tag)) + one);  // d y^2 + 1
  const U v3 = rfe_mul<U, W>(rfe_sq<U, W>(v), v);
  U x = rfe_mul<U, W>(rfe_mul<U, W>(rfe_sq<U, W>(v3), v), u);    // u v^7
  x = rfe_pow22523<U, W>(x, [] {
    if (SYNC) __syncthreads();
  });
  x = rfe_mul<U, W>(rfe_mul<U, W>(x, v3), u);                     // u v^3 (u v^7)^((p-5)/8)
  const U vxx = rfe_mul<U, W>(rfe_sq<U, W>(x), v);
  fe fu, fvxx, chk;
  rfe_to_fe(X, x);
  rfe_to_fe(fu, u);
  rfe_to_fe(fvxx, vxx);
  fe_sub(chk, fvxx, fu);
  bool ok = true;
  if (!fe_iszero(chk)) {
    fe_add(chk, fvxx, fu);
    if (!fe_iszero(chk)) ok = false;
    fe sm1;
    fe_load_const(sm1, kFeSqrtM1);
    fe_mul(X, X, sm1);
  }
  const uint32_t sign = w[7] >> 31;
  if (fe_isnegative(X) != sign) fe_neg(X, X);
  return ok;
}

// Canonical encoding of (X:Y:Z) into 8 little-endian words.
template <bool C = CBFT_FE_CHAIN>
FE_INLINE void ge_tobytes(uint32_t* out, const fe& X, const fe& Y, const fe& Z) {
  fe zi, x, y;
  fe_invert<C>(zi, Z);
  fe_mul<C>(x, X, zi);
  fe_mul<C>(y, Y, zi);
  fe_to_words(out, y);
  out[7] ^= fe_isnegative(x) << 31;
}
