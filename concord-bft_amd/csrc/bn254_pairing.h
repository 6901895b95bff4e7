// BN-P254 groups and the optimal ate pairing (host + device).
//
//   G1: E(Fp): y^2 = x^3 + 2, Jacobian coordinates.
//   G2: D-type twist E'(Fp2): y^2 = x^3 + (1 - i).  G2 points are fixed per key set (share
//       verification keys, the group public key, the generator), so their Miller-loop lines are
//       PRECOMPUTED once in affine form: per step (lambda, mu = lambda x_T - y_T), and the
//       per-signature work only evaluates l(P) = y_P + (-lambda x_P) w + mu w^3 (2 Fp mul).
//   pairing check  prod_k e(P_k, Q_k) == 1  with one shared Miller loop and one final
//   exponentiation (hard part by the u-decomposition of (p^4 - p^2 + 1)/r, lambda_0..3,
//   checked in tools/gen_bn254_consts.py).
#pragma once
#include "bn254_tower.h"

// |6u + 2| = 2^64 + 2^63 + 2^57 + 2^56 + 4: 64 doubling steps, additions after bits 63,57,56,2
#define BN_ATE_DBL 64
#define BN_ATE_LINES 70  // 64 doubling + 4 addition + 2 Frobenius lines
#define BN_LINE_WORDS 36  // lambda (fp2) | mu (fp2)

BN_HD bool bn_ate_bit(int i) {  // bit i (0..63) of |6u+2|
  return i == 63 || i == 57 || i == 56 || i == 2;
}

struct g1j {
  fp X, Y, Z;  // Jacobian; Z = 0 is infinity
};
struct g1a {
  fp x, y;
  bool inf;
};
struct g2a {
  fp2 x, y;
  bool inf;
};
struct g2j {
  fp2 X, Y, Z;
};

// ------------------------------------------------------------------------------ G1
BN_HD void g1_set_inf(g1j& r) {
  f_one(r.X);
  f_one(r.Y);
  f_zero(r.Z);
}
BN_HD bool g1_is_inf(const g1j& p) { return f_is_zero(p.Z); }

BN_HD void g1_dbl(g1j& r, const g1j& p) {  // a = 0 doubling (dbl-2009-l)
  fp A, B, C, D, E, F, t;
  f_sqr(A, p.X);
  f_sqr(B, p.Y);
  f_sqr(C, B);
  f_add(t, p.X, B);
  f_sqr(t, t);
  f_sub(t, t, A);
  f_sub(t, t, C);
  f_add(D, t, t);
  f_add(E, A, A);
  f_add(E, E, A);
  f_sqr(F, E);
  fp Z3;
  f_mul(Z3, p.Y, p.Z);
  f_add(r.Z, Z3, Z3);
  f_sub(r.X, F, D);
  f_sub(r.X, r.X, D);
  f_sub(t, D, r.X);
  f_mul(t, E, t);
  f_add(C, C, C);
  f_add(C, C, C);
  f_add(C, C, C);
  f_sub(r.Y, t, C);
}

// r = p + q (general Jacobian addition, add-2007-bl), handles infinity and doubling
BN_HD void g1_add(g1j& r, const g1j& p, const g1j& q) {
  if (g1_is_inf(p)) {
    r = q;
    return;
  }
  if (g1_is_inf(q)) {
    r = p;
    return;
  }
  fp Z1Z1, Z2Z2, U1, U2, S1, S2, H, I, J, rr, V, t;
  f_sqr(Z1Z1, p.Z);
  f_sqr(Z2Z2, q.Z);
  f_mul(U1, p.X, Z2Z2);
  f_mul(U2, q.X, Z1Z1);
  f_mul(S1, p.Y, q.Z);
  f_mul(S1, S1, Z2Z2);
  f_mul(S2, q.Y, p.Z);
  f_mul(S2, S2, Z1Z1);
  f_sub(H, U2, U1);
  f_sub(rr, S2, S1);
  if (f_is_zero(H)) {
    if (f_is_zero(rr)) {
      g1_dbl(r, p);
    } else {
      g1_set_inf(r);
    }
    return;
  }
  f_add(I, H, H);
  f_sqr(I, I);
  f_mul(J, H, I);
  f_add(rr, rr, rr);
  f_mul(V, U1, I);
  fp X3, Y3, Z3;
  f_sqr(X3, rr);
  f_sub(X3, X3, J);
  f_sub(X3, X3, V);
  f_sub(X3, X3, V);
  f_sub(t, V, X3);
  f_mul(Y3, rr, t);
  f_mul(t, S1, J);
  f_add(t, t, t);
  f_sub(Y3, Y3, t);
  f_add(Z3, p.Z, q.Z);
  f_sqr(Z3, Z3);
  f_sub(Z3, Z3, Z1Z1);
  f_sub(Z3, Z3, Z2Z2);
  f_mul(Z3, Z3, H);
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
}

BN_HD void g1_from_affine(g1j& r, const g1a& a) {
  if (a.inf) {
    g1_set_inf(r);
    return;
  }
  r.X = a.x;
  r.Y = a.y;
  f_one(r.Z);
}

// VAR: variable-time inversion (safegcd) -- only for points that are public anyway (a combined
// signature, sums of published shares); signing keeps the constant-time Fermat form
template <bool VAR = false>
BN_HDN void g1_to_affine(g1a& r, const g1j& p) {
  if (g1_is_inf(p)) {
    r.inf = true;
    f_zero(r.x);
    f_zero(r.y);
    return;
  }
  fp zi, zi2;
  if (VAR)
    fp_inv_var(zi, p.Z);
  else
    fp_inv(zi, p.Z);
  f_sqr(zi2, zi);
  f_mul(r.x, p.X, zi2);
  f_mul(zi2, zi2, zi);
  f_mul(r.y, p.Y, zi2);
  r.inf = false;
}

// r = k * p, k as 8 little-endian words (left-to-right double-and-add)
BN_HDN void g1_mul(g1j& r, const g1j& p, const uint32_t* k) {
  g1j acc;
  g1_set_inf(acc);
  for (int i = 255; i >= 0; i--) {
    g1_dbl(acc, acc);
    if ((k[i >> 5] >> (i & 31)) & 1) g1_add(acc, acc, p);
  }
  r = acc;
}

// ------------------------------------------------------------------------------ secret scalars
// Scalar multiplication by a SECRET scalar (signing, sk * g2) in a fixed operation sequence: a
// Montgomery ladder over k' = k + 2r, which has bit 254 set and bit 255 clear for every k < r
// (2r > 2^254, 3r < 2^255), so the loop length does not depend on k; the two ladder registers are
// exchanged by a masked select, never by a branch on a key bit.  R1 - R0 = P throughout, so the
// additions never reach their doubling or infinity cases (for P of order r and k >= 2); k'P = kP.
template <class F>
BN_HD void f_cswap(Fe<F>& a, Fe<F>& b, uint32_t mask) {
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
    const uint32_t t = (a.v[i] ^ b.v[i]) & mask;
    a.v[i] ^= t;
    b.v[i] ^= t;
  }
}

// k' = k + 2r as 8 LE words (k < r, 8 LE words)
BN_HD void bn_scalar_plus_2r(uint32_t* out, const uint32_t* k) {
  const uint32_t r2[8] = {0x0000001au, 0x42000000u, 0x00000021u, 0xff3f0000u,
                          0x0000000fu, 0x74689b00u, 0x80000003u, 0x4a46c904u};  // 2r
  uint64_t c = 0;
  for (int q = 0; q < 8; q++) {
    c += (uint64_t)k[q] + r2[q];
    out[q] = (uint32_t)c;
    c >>= 32;
  }
}

template <class PT, class SWAP, class DBL, class ADD>
BN_HD void bn_ladder(PT& r, const PT& p, const uint32_t* k, SWAP cswap, DBL dbl, ADD add) {
  uint32_t kk[8];
  bn_scalar_plus_2r(kk, k);
  PT r0 = p, r1;
  dbl(r1, p);
  for (int i = 253; i >= 0; i--) {
    const uint32_t mask = 0u - ((kk[i >> 5] >> (i & 31)) & 1u);
    cswap(r0, r1, mask);
    add(r1, r0, r1);
    dbl(r0, r0);
    cswap(r0, r1, mask);
  }
  r = r0;
}

// r = k * p for a secret k (constant operation sequence; p of order r)
BN_HDN void g1_mul_ct(g1j& r, const g1j& p, const uint32_t* k) {
  bn_ladder(
      r, p, k,
      [](g1j& a, g1j& b, uint32_t m) {
        f_cswap(a.X, b.X, m);
        f_cswap(a.Y, b.Y, m);
        f_cswap(a.Z, b.Z, m);
      },
      [](g1j& o, const g1j& a) { g1_dbl(o, a); }, [](g1j& o, const g1j& a, const g1j& b) { g1_add(o, a, b); });
}

BN_HDN bool g1_on_curve(const g1a& a) {
  if (a.inf) return true;
  fp l, rr, b;
  f_sqr(l, a.y);
  f_sqr(rr, a.x);
  f_mul(rr, rr, a.x);
  uint32_t two[8] = {2, 0, 0, 0, 0, 0, 0, 0};
  f_from_words(b, two);
  f_add(rr, rr, b);
  return f_eq(l, rr);
}

// big-endian 32 bytes -> 8 little-endian words
BN_HD void be32_to_words(uint32_t* w, const uint8_t* b) {
  for (int i = 0; i < 8; i++) {
    const uint8_t* q = b + 28 - 4 * i;
    w[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}
BN_HD void words_to_be32(uint8_t* b, const uint32_t* w) {
  for (int i = 0; i < 8; i++) {
    uint8_t* q = b + 28 - 4 * i;
    q[0] = (uint8_t)(w[i] >> 24);
    q[1] = (uint8_t)(w[i] >> 16);
    q[2] = (uint8_t)(w[i] >> 8);
    q[3] = (uint8_t)w[i];
  }
}
BN_HD bool words_lt_p(const uint32_t* w) {  // w < p ?
  const uint32_t p[8] = {0x00000013u, 0xa7000000u, 0x00000013u, 0x61210000u,
                         0x00000008u, 0xba344d80u, 0x40000001u, 0x25236482u};
  for (int i = 7; i >= 0; i--) {
    if (w[i] < p[i]) return true;
    if (w[i] > p[i]) return false;
  }
  return false;
}

// The y "parity" of RELIC's compressed encodings: fp_get_bit(y, 0) on RELIC's raw Montgomery
// digits (R = 2^256 for FP_PRIME = 254 on 64-bit digits), i.e. lsb(y * 2^256 mod p) — not lsb(y).
// Pinned for G2 by the reference's RELIC-generated key files (tests/simpleKVBC/scripts/
// set{A,B}_replica_*, 40/40 vks, tests/golden/relic_bls_keys.json); G1 (ep_write_bin) uses the
// same fp_get_bit rule (oracle/bn254_ref.py relic_bit).  Our own Montgomery radix is 2^261, so
// y * (2^256 mod p) is formed with one field multiplication and read back canonically.
BN_HDN uint32_t f_relic_bit(const fp& y) {
  const uint32_t r256[8] = {0xffffff8eu, 0x15ffffffu, 0xffffff8au, 0xb939ffffu,
                            0xffffffcdu, 0xa2c62effu, 0x7ffffff5u, 0x212ba4f2u};
  fp c, t;
  f_from_words(c, r256);
  f_mul(t, y, c);
  uint32_t w[8];
  f_to_words(w, t);
  return w[0] & 1u;
}

// RELIC ep_read_bin(pack = 1) semantics as restated in oracle/bn254_ref.py: 33 bytes,
// 0x00 || 0^32 = infinity; prefix 2 | f_relic_bit(y); x < p; x^3 + 2 must be a square.
BN_HDN bool g1_decompress(g1a& r, const uint8_t* b) {
  r.inf = false;
  if (b[0] == 0) {
    uint8_t o = 0;
    for (int i = 1; i < 33; i++) o |= b[i];
    r.inf = true;
    f_zero(r.x);
    f_zero(r.y);
    return o == 0;
  }
  if (b[0] != 2 && b[0] != 3) return false;
  uint32_t w[8];
  be32_to_words(w, b + 1);
  if (!words_lt_p(w)) return false;
  f_from_words(r.x, w);
  fp rhs, b2;
  f_sqr(rhs, r.x);
  f_mul(rhs, rhs, r.x);
  uint32_t two[8] = {2, 0, 0, 0, 0, 0, 0, 0};
  f_from_words(b2, two);
  f_add(rhs, rhs, b2);
  if (!fp_sqrt(r.y, rhs)) return false;
  if (f_relic_bit(r.y) != (uint32_t)(b[0] & 1)) f_neg(r.y, r.y);
  return true;
}

BN_HDN void g1_compress(uint8_t* out, const g1a& a) {
  if (a.inf) {
    for (int i = 0; i < 33; i++) out[i] = 0;
    return;
  }
  uint32_t xw[8];
  f_to_words(xw, a.x);
  out[0] = (uint8_t)(2 | f_relic_bit(a.y));
  words_to_be32(out + 1, xw);
}

// ------------------------------------------------------------------------------ G2 (twist)
BN_HD void fp2_from_be(fp2& r, const uint8_t* b, bool* ok) {  // x0 || x1, 64 bytes
  uint32_t w0[8], w1[8];
  be32_to_words(w0, b);
  be32_to_words(w1, b + 32);
  if (!words_lt_p(w0) || !words_lt_p(w1)) *ok = false;
  f_from_words(r.a, w0);
  f_from_words(r.b, w1);
}

// Fp2 square root (p = 3 mod 4, i^2 = -1), false if not a square
BN_HDN bool fp2_sqrt(fp2& r, const fp2& a) {
  if (fp2_is_zero(a)) {
    fp2_zero(r);
    return true;
  }
  // a1 = a^((p-3)/4)
  const uint32_t e[8] = {0x00000004u, 0xe9c00000u, 0x00000004u, 0x18484000u,
                         0x00000002u, 0x6e8d1360u, 0x90000000u, 0x0948d920u};
  fp2 a1, alpha, x0, t;
  fp2_one(a1);
  for (int i = 255; i >= 0; i--) {
    fp2_sqr(a1, a1);
    if ((e[i >> 5] >> (i & 31)) & 1) fp2_mul(a1, a1, a);
  }
  fp2_sqr(alpha, a1);
  fp2_mul(alpha, alpha, a);
  fp2_mul(x0, a1, a);
  fp2 m1;
  fp2_one(m1);
  fp2_neg(m1, m1);
  if (fp2_eq(alpha, m1)) {
    // x = i * x0
    t.a = x0.b;
    f_neg(t.a, t.a);
    t.b = x0.a;
    r = t;
  } else {
    // b = (1 + alpha)^((p-1)/2)
    const uint32_t h[8] = {0x00000009u, 0xd3800000u, 0x00000009u, 0x30908000u,
                           0x00000004u, 0xdd1a26c0u, 0x20000000u, 0x1291b241u};
    fp2 one, bb;
    fp2_one(one);
    fp2_add(t, one, alpha);
    fp2_one(bb);
    for (int i = 255; i >= 0; i--) {
      fp2_sqr(bb, bb);
      if ((h[i >> 5] >> (i & 31)) & 1) fp2_mul(bb, bb, t);
    }
    fp2_mul(r, bb, x0);
  }
  fp2_sqr(t, r);
  return fp2_eq(t, a);
}

BN_HDN void g2_dbl_j(g2j& r, const g2j& p) {
  fp2 A, B, C, D, E, F, t, Z3;
  fp2_sqr(A, p.X);
  fp2_sqr(B, p.Y);
  fp2_sqr(C, B);
  fp2_add(t, p.X, B);
  fp2_sqr(t, t);
  fp2_sub(t, t, A);
  fp2_sub(t, t, C);
  fp2_add(D, t, t);
  fp2_add(E, A, A);
  fp2_add(E, E, A);
  fp2_sqr(F, E);
  fp2_mul(Z3, p.Y, p.Z);
  fp2_add(r.Z, Z3, Z3);
  fp2_sub(r.X, F, D);
  fp2_sub(r.X, r.X, D);
  fp2_sub(t, D, r.X);
  fp2_mul(t, E, t);
  fp2_dbl(C, C);
  fp2_dbl(C, C);
  fp2_dbl(C, C);
  fp2_sub(r.Y, t, C);
}

// The Jacobian addition's body, inlinable where the caller has registers to spare (the multisig
// key-sum tree: as a called function it gets a 128-VGPR budget and spills every product to
// scratch).  g2_add_j below is the out-of-line form.
BN_HD void g2_add_j_body(g2j& r, const g2j& p, const g2j& q) {
  if (fp2_is_zero(p.Z)) {
    r = q;
    return;
  }
  if (fp2_is_zero(q.Z)) {
    r = p;
    return;
  }
  fp2 Z1Z1, Z2Z2, U1, U2, S1, S2, H, I, J, rr, V, t, X3, Y3, Z3;
  fp2_sqr(Z1Z1, p.Z);
  fp2_sqr(Z2Z2, q.Z);
  fp2_mul(U1, p.X, Z2Z2);
  fp2_mul(U2, q.X, Z1Z1);
  fp2_mul(S1, p.Y, q.Z);
  fp2_mul(S1, S1, Z2Z2);
  fp2_mul(S2, q.Y, p.Z);
  fp2_mul(S2, S2, Z1Z1);
  fp2_sub(H, U2, U1);
  fp2_sub(rr, S2, S1);
  if (fp2_is_zero(H)) {
    if (fp2_is_zero(rr)) {
      g2_dbl_j(r, p);
    } else {
      fp2_one(r.X);
      fp2_one(r.Y);
      fp2_zero(r.Z);
    }
    return;
  }
  fp2_add(I, H, H);
  fp2_sqr(I, I);
  fp2_mul(J, H, I);
  fp2_add(rr, rr, rr);
  fp2_mul(V, U1, I);
  fp2_sqr(X3, rr);
  fp2_sub(X3, X3, J);
  fp2_sub(X3, X3, V);
  fp2_sub(X3, X3, V);
  fp2_sub(t, V, X3);
  fp2_mul(Y3, rr, t);
  fp2_mul(t, S1, J);
  fp2_add(t, t, t);
  fp2_sub(Y3, Y3, t);
  fp2_add(Z3, p.Z, q.Z);
  fp2_sqr(Z3, Z3);
  fp2_sub(Z3, Z3, Z1Z1);
  fp2_sub(Z3, Z3, Z2Z2);
  fp2_mul(Z3, Z3, H);
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
}
BN_HDN void g2_add_j(g2j& r, const g2j& p, const g2j& q) { g2_add_j_body(r, p, q); }

// VAR: variable-time inversion, for public points only (a multisig key sum)
template <bool VAR = false>
BN_HDN void g2_to_affine(g2a& r, const g2j& p) {
  if (fp2_is_zero(p.Z)) {
    r.inf = true;
    fp2_zero(r.x);
    fp2_zero(r.y);
    return;
  }
  fp2 zi, zi2;
  fp2_inv<VAR>(zi, p.Z);
  fp2_sqr(zi2, zi);
  fp2_mul(r.x, p.X, zi2);
  fp2_mul(zi2, zi2, zi);
  fp2_mul(r.y, p.Y, zi2);
  r.inf = false;
}

// r = k * p for a secret k (G2 form of g1_mul_ct)
BN_HDN void g2_mul_ct(g2j& r, const g2j& p, const uint32_t* k) {
  bn_ladder(
      r, p, k,
      [](g2j& a, g2j& b, uint32_t m) {
        f_cswap(a.X.a, b.X.a, m);
        f_cswap(a.X.b, b.X.b, m);
        f_cswap(a.Y.a, b.Y.a, m);
        f_cswap(a.Y.b, b.Y.b, m);
        f_cswap(a.Z.a, b.Z.a, m);
        f_cswap(a.Z.b, b.Z.b, m);
      },
      [](g2j& o, const g2j& a) { g2_dbl_j(o, a); }, [](g2j& o, const g2j& a, const g2j& b) { g2_add_j(o, a, b); });
}

BN_HDN bool g2_in_subgroup(const g2a& q) {  // r * Q == O
  const uint32_t rw[8] = {0x0000000du, 0xa1000000u, 0x00000010u, 0xff9f8000u,
                          0x00000007u, 0xba344d80u, 0x40000001u, 0x25236482u};
  g2j P, acc;
  P.X = q.x;
  P.Y = q.y;
  fp2_one(P.Z);
  fp2_one(acc.X);
  fp2_one(acc.Y);
  fp2_zero(acc.Z);
  for (int i = 255; i >= 0; i--) {
    g2_dbl_j(acc, acc);
    if ((rw[i >> 5] >> (i & 31)) & 1) g2_add_j(acc, acc, P);
  }
  return fp2_is_zero(acc.Z);
}

// RELIC ep2_read_bin(pack = 1) as restated: 65 bytes, prefix 2 | f_relic_bit(y.a), x0 || x1 < p,
// on E' -- without the subgroup check (g2_decompress adds it; bls_keys.hip runs it wave-wide).
BN_HDN bool g2_decode_on_curve(g2a& r, const uint8_t* b) {
  r.inf = false;
  if (b[0] == 0) {
    uint8_t o = 0;
    for (int i = 1; i < 65; i++) o |= b[i];
    r.inf = true;
    fp2_zero(r.x);
    fp2_zero(r.y);
    return o == 0;
  }
  if (b[0] != 2 && b[0] != 3) return false;
  bool ok = true;
  fp2_from_be(r.x, b + 1, &ok);
  if (!ok) return false;
  fp2 rhs, b2;
  fp2_sqr(rhs, r.x);
  fp2_mul(rhs, rhs, r.x);
  fp2_load(b2, Bn254Consts::B2);
  fp2_add(rhs, rhs, b2);
  if (!fp2_sqrt(r.y, rhs)) return false;
  if (f_relic_bit(r.y.a) != (uint32_t)(b[0] & 1)) fp2_neg(r.y, r.y);
  return true;
}

// ... and (CHECK) in the order-r subgroup (r Q == O; infinity decodes, for the caller to judge)
BN_HDN bool g2_decompress(g2a& r, const uint8_t* b) {
  if (!g2_decode_on_curve(r, b)) return false;
  return r.inf || g2_in_subgroup(r);
}

BN_HDN void g2_compress(uint8_t* out, const g2a& a) {
  if (a.inf) {
    for (int i = 0; i < 65; i++) out[i] = 0;
    return;
  }
  uint32_t w[8];
  out[0] = (uint8_t)(2 | f_relic_bit(a.y.a));
  f_to_words(w, a.x.a);
  words_to_be32(out + 1, w);
  f_to_words(w, a.x.b);
  words_to_be32(out + 33, w);
}

// ------------------------------------------------------------------------------ lines
BN_HD void line_store(uint32_t* out, const fp2& lam, const fp2& mu) {
  for (int i = 0; i < 9; i++) {
    out[i] = lam.a.v[i];
    out[9 + i] = lam.b.v[i];
    out[18 + i] = mu.a.v[i];
    out[27 + i] = mu.b.v[i];
  }
}

// affine step T <- T + Q (or 2T when dbl), emitting (lambda, mu = lambda x_T - y_T)
BN_HDN void line_step(uint32_t* out, fp2& tx, fp2& ty, const fp2& qx, const fp2& qy, bool dbl) {
  fp2 lam, t, x3, y3, mu;
  if (dbl) {
    fp2_sqr(t, tx);
    fp2_add(lam, t, t);
    fp2_add(lam, lam, t);  // 3x^2
    fp2_add(t, ty, ty);
    fp2_inv(t, t);
    fp2_mul(lam, lam, t);
  } else {
    fp2_sub(lam, qy, ty);
    fp2_sub(t, qx, tx);
    fp2_inv(t, t);
    fp2_mul(lam, lam, t);
  }
  fp2_mul(mu, lam, tx);
  fp2_sub(mu, mu, ty);
  line_store(out, lam, mu);
  fp2_sqr(x3, lam);
  fp2_sub(x3, x3, tx);
  fp2_sub(x3, x3, dbl ? tx : qx);
  fp2_sub(t, tx, x3);
  fp2_mul(y3, lam, t);
  fp2_sub(y3, y3, ty);
  tx = x3;
  ty = y3;
}

// All BN_ATE_LINES line coefficients of Q (affine, not infinity) in Miller-loop order.
BN_HDN void g2_precompute_lines(uint32_t* out, const g2a& q) {
  fp2 tx = q.x, ty = q.y;
  int k = 0;
  for (int i = BN_ATE_DBL - 1; i >= 0; i--) {
    line_step(out + (k++) * BN_LINE_WORDS, tx, ty, q.x, q.y, true);
    if (bn_ate_bit(i)) line_step(out + (k++) * BN_LINE_WORDS, tx, ty, q.x, q.y, false);
  }
  // 6u + 2 < 0: T = -T (f is conjugated in the loop)
  fp2_neg(ty, ty);
  fp2 q1x, q1y, q2x, q2y, c;
  fp2_conj(q1x, q.x);
  fp2_load(c, Bn254Consts::TWX1);
  fp2_mul(q1x, q1x, c);
  fp2_conj(q1y, q.y);
  fp2_load(c, Bn254Consts::TWY1);
  fp2_mul(q1y, q1y, c);
  line_step(out + (k++) * BN_LINE_WORDS, tx, ty, q1x, q1y, false);
  fp2_load(c, Bn254Consts::TWX2);
  fp2_mul(q2x, q.x, c);
  fp2_load(c, Bn254Consts::TWY2);
  fp2_mul(q2y, q.y, c);
  fp2_neg(q2y, q2y);
  line_step(out + (k++) * BN_LINE_WORDS, tx, ty, q2x, q2y, false);
}

// ---- the same lines without an inversion per step (Jacobian T), normalised by ONE batched
// inversion.  Step k of the Miller loop records the line through T (and T or Q) scaled by a
// non-zero A_k in Fp2:  A_k yP + B_k xP w + C_k w^3, with (T = (X, Y, Z), x_T = X/Z^2,
// y_T = Y/Z^3; affine slope lambda = n/d):
//   doubling  n = 3X^2, d = 2YZ:         A = d Z^2 = 2YZ^3,  B = -n Z^2,  C = 3X^3 - 2Y^2
//   addition  n = qy Z^3 - Y, d = Z (qx Z^2 - X):   A = d,  B = -n,  C = qy Z X - qx Y
// (C = A (lambda x_T - y_T) in both cases).  lambda_k = -B_k / A_k and mu_k = C_k / A_k are then
// exactly the affine line_step values (the same field elements; the limbs may hold the other
// representative < 2p), with Montgomery's trick over the
// A_k: 3 multiplications per line and one Fp2 inversion in place of 70 inversions.
// scratch: BN_ATE_LINES x 36 words (A_k, then its prefix product).
BN_HD void fp2_store(uint32_t* o, const fp2& x) {
  for (int i = 0; i < 9; i++) {
    o[i] = x.a.v[i];
    o[9 + i] = x.b.v[i];
  }
}
BN_HD void fp2_fetch(fp2& x, const uint32_t* o) {
  for (int i = 0; i < 9; i++) {
    x.a.v[i] = o[i];
    x.b.v[i] = o[9 + i];
  }
}

// doubling step: records (A, B, C) of the tangent at T, T <- 2T
BN_HD void line_dbl_j(uint32_t* ln, uint32_t* sa, g2j& T) {
  fp2 XX, YY, ZZ, YYYY, t, A, B, C, D, E, F;
  fp2_sqr(XX, T.X);
  fp2_sqr(YY, T.Y);
  fp2_sqr(ZZ, T.Z);
  fp2_mul(t, T.Y, T.Z);
  fp2_dbl(t, t);  // 2YZ = Z3
  fp2_mul(A, t, ZZ);
  fp2_add(E, XX, XX);
  fp2_add(E, E, XX);  // 3X^2
  fp2_mul(B, E, ZZ);
  fp2_neg(B, B);
  fp2_mul(C, E, T.X);
  fp2_dbl(D, YY);
  fp2_sub(C, C, D);  // 3X^3 - 2Y^2
  fp2_store(sa, A);
  fp2_store(ln, B);
  fp2_store(ln + 18, C);
  // dbl-2009-l
  fp2_sqr(YYYY, YY);
  fp2_add(D, T.X, YY);
  fp2_sqr(D, D);
  fp2_sub(D, D, XX);
  fp2_sub(D, D, YYYY);
  fp2_dbl(D, D);
  fp2_sqr(F, E);
  fp2_sub(T.X, F, D);
  fp2_sub(T.X, T.X, D);
  fp2_sub(D, D, T.X);
  fp2_mul(D, E, D);
  fp2_dbl(YYYY, YYYY);
  fp2_dbl(YYYY, YYYY);
  fp2_dbl(YYYY, YYYY);
  fp2_sub(T.Y, D, YYYY);
  T.Z = t;
}

// addition step with affine (qx, qy): records (A, B, C) of the line through T and Q, T <- T + Q
BN_HD void line_add_j(uint32_t* ln, uint32_t* sa, g2j& T, const fp2& qx, const fp2& qy) {
  fp2 ZZ, U2, S2, H, R, A, C, t, HH, I, J, V, r;
  fp2_sqr(ZZ, T.Z);
  fp2_mul(U2, qx, ZZ);
  fp2_mul(S2, qy, T.Z);
  fp2_mul(S2, S2, ZZ);
  fp2_sub(H, U2, T.X);
  fp2_sub(R, S2, T.Y);
  fp2_mul(A, T.Z, H);
  fp2_mul(C, qy, T.Z);
  fp2_mul(C, C, T.X);
  fp2_mul(t, qx, T.Y);
  fp2_sub(C, C, t);
  fp2_neg(t, R);
  fp2_store(sa, A);
  fp2_store(ln, t);
  fp2_store(ln + 18, C);
  // madd-2007-bl
  fp2_sqr(HH, H);
  fp2_dbl(I, HH);
  fp2_dbl(I, I);
  fp2_mul(J, H, I);
  fp2_dbl(r, R);
  fp2_mul(V, T.X, I);
  fp2_sqr(t, r);
  fp2_sub(t, t, J);
  fp2_sub(t, t, V);
  fp2_sub(t, t, V);  // X3
  fp2_sub(V, V, t);
  fp2_mul(V, r, V);
  fp2_mul(J, T.Y, J);
  fp2_dbl(J, J);
  fp2_sub(T.Y, V, J);
  fp2_add(V, T.Z, H);
  fp2_sqr(V, V);
  fp2_sub(V, V, ZZ);
  fp2_sub(T.Z, V, HH);
  T.X = t;
}

BN_HDN void g2_precompute_lines_batch(uint32_t* out, const g2a& q, uint32_t* scratch) {
  g2j T;
  T.X = q.x;
  T.Y = q.y;
  fp2_one(T.Z);
  int k = 0;
  for (int i = BN_ATE_DBL - 1; i >= 0; i--) {
    line_dbl_j(out + k * BN_LINE_WORDS, scratch + 36 * k, T);
    k++;
    if (bn_ate_bit(i)) {
      line_add_j(out + k * BN_LINE_WORDS, scratch + 36 * k, T, q.x, q.y);
      k++;
    }
  }
  fp2_neg(T.Y, T.Y);  // 6u + 2 < 0
  fp2 q1x, q1y, q2x, q2y, c;
  fp2_conj(q1x, q.x);
  fp2_load(c, Bn254Consts::TWX1);
  fp2_mul(q1x, q1x, c);
  fp2_conj(q1y, q.y);
  fp2_load(c, Bn254Consts::TWY1);
  fp2_mul(q1y, q1y, c);
  line_add_j(out + k * BN_LINE_WORDS, scratch + 36 * k, T, q1x, q1y);
  k++;
  fp2_load(c, Bn254Consts::TWX2);
  fp2_mul(q2x, q.x, c);
  fp2_load(c, Bn254Consts::TWY2);
  fp2_mul(q2y, q.y, c);
  fp2_neg(q2y, q2y);
  line_add_j(out + k * BN_LINE_WORDS, scratch + 36 * k, T, q2x, q2y);
  k++;
  // Montgomery's trick over the A_k
  fp2 acc, a;
  fp2_one(acc);
  for (int j = 0; j < k; j++) {
    fp2_fetch(a, scratch + 36 * j);
    fp2_mul(acc, acc, a);
    fp2_store(scratch + 36 * j + 18, acc);
  }
  fp2 inv;
  fp2_inv(inv, acc);
  for (int j = k - 1; j >= 0; j--) {
    fp2 ai, pre, b, cc, lam, mu;
    if (j > 0) {
      fp2_fetch(pre, scratch + 36 * (j - 1) + 18);
      fp2_mul(ai, inv, pre);
    } else {
      ai = inv;
    }
    fp2_fetch(a, scratch + 36 * j);
    fp2_mul(inv, inv, a);
    fp2_fetch(b, out + j * BN_LINE_WORDS);
    fp2_fetch(cc, out + j * BN_LINE_WORDS + 18);
    fp2_mul(lam, b, ai);
    fp2_neg(lam, lam);
    fp2_mul(mu, cc, ai);
    line_store(out + j * BN_LINE_WORDS, lam, mu);
  }
}

// f <- f * l(P) for a precomputed line
BN_HDN void line_eval_mul(fp12& f, const uint32_t* ln, const g1a& P) {
  fp2 lam, mu, s;
  for (int i = 0; i < 9; i++) {
    lam.a.v[i] = ln[i];
    lam.b.v[i] = ln[9 + i];
    mu.a.v[i] = ln[18 + i];
    mu.b.v[i] = ln[27 + i];
  }
  fp2_mul_fp(s, lam, P.x);
  fp2_neg(s, s);
  fp12_mul_line(f, P.y, s, mu);
}

// Miller loop of prod_{k<NP} e(P_k, Q_k), Q_k given by precomputed lines (infinite P_k must be
// excluded by the caller: e(O, Q) = 1).
template <int NP>
BN_HDN void miller_multi(fp12& f, const g1a* P, const uint32_t* const* lines) {
  fp12_one(f);
  int k = 0;
  for (int i = BN_ATE_DBL - 1; i >= 0; i--) {
    fp12_sqr(f, f);
    for (int j = 0; j < NP; j++) line_eval_mul(f, lines[j] + k * BN_LINE_WORDS, P[j]);
    k++;
    if (bn_ate_bit(i)) {
      for (int j = 0; j < NP; j++) line_eval_mul(f, lines[j] + k * BN_LINE_WORDS, P[j]);
      k++;
    }
  }
  fp12_conj(f, f);
  for (int t = 0; t < 2; t++) {
    for (int j = 0; j < NP; j++) line_eval_mul(f, lines[j] + k * BN_LINE_WORDS, P[j]);
    k++;
  }
}

// ------------------------------------------------------------------------------ final exp
BN_HDN void fp12_pow_small(fp12& r, const fp12& x, uint32_t e) {  // e >= 1
  fp12 acc = x;
  int top = 31;
  while (!((e >> top) & 1)) top--;
  for (int i = top - 1; i >= 0; i--) {
    fp12_sqr(acc, acc);
    if ((e >> i) & 1) fp12_mul(acc, acc, x);
  }
  r = acc;
}

// x^u for x in the cyclotomic subgroup: u = -(2^62 + 2^55 + 1) -> conj(x^(2^62+2^55+1))
BN_HDN void fp12_pow_u(fp12& r, const fp12& x) {
  fp12 acc = x;
  for (int i = 61; i >= 0; i--) {
    fp12_sqr(acc, acc);
    if (i == 55 || i == 0) fp12_mul(acc, acc, x);
  }
  fp12_conj(r, acc);
}

// f^((p^12 - 1)/r)
BN_HDN void final_exp(fp12& r, const fp12& f) {
  fp12 t, g;
  // easy part: g = f^((p^6 - 1)(p^2 + 1))
  fp12_inv(t, f);
  fp12_conj(g, f);
  fp12_mul(g, g, t);
  fp12_frob2(t, g);
  fp12_mul(g, t, g);
  // hard part: g^(l0 + l1 p + l2 p^2 + p^3), l0 = -36u^3-30u^2-18u-2, l1 = -36u^3-18u^2-12u+1,
  // l2 = 6u^2 + 1; a = g^u, b = g^(u^2), c = g^(u^3)
  fp12 a, b, c, c36, b6, b18, b30, a12, a18, g2;
  fp12_pow_u(a, g);
  fp12_pow_u(b, a);
  fp12_pow_u(c, b);
  fp12_pow_small(c36, c, 36);
  fp12_pow_small(b6, b, 6);
  fp12_pow_small(b18, b6, 3);
  fp12_mul(b30, b18, b6);
  fp12_mul(b30, b30, b6);
  fp12_pow_small(a12, a, 12);
  fp12_pow_small(a18, a, 18);
  fp12_sqr(g2, g);
  // t0 = g^l0 = conj(c36 b30 a18 g2)
  fp12 t0, t1, t2, t3;
  fp12_mul(t0, c36, b30);
  fp12_mul(t0, t0, a18);
  fp12_mul(t0, t0, g2);
  fp12_conj(t0, t0);
  // t1 = g^l1 = conj(c36 b18 a12) g
  fp12_mul(t1, c36, b18);
  fp12_mul(t1, t1, a12);
  fp12_conj(t1, t1);
  fp12_mul(t1, t1, g);
  // t2 = g^l2 = b6 g
  fp12_mul(t2, b6, g);
  fp12_frob(t1, t1);
  fp12_frob2(t2, t2);
  fp12_frob3(t3, g);
  fp12_mul(t0, t0, t1);
  fp12_mul(t0, t0, t2);
  fp12_mul(r, t0, t3);
}

// prod_k e(P_k, Q_k) == 1 ?
template <int NP>
BN_HDN bool pairing_check(const g1a* P, const uint32_t* const* lines) {
  fp12 f, e;
  miller_multi<NP>(f, P, lines);
  final_exp(e, f);
  return fp12_is_one(e);
}
