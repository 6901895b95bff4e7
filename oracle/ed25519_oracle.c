/* Ed25519 CPU oracle in plain C — TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library
 * (oracle/libcbft_oracle.so); it is never linked into or called by libcbft_hipcrypto.
 *
 * Restates the verify semantics the product must match: OpenSSL 3.0.2 EVP_DigestVerify with
 * EVP_PKEY_ED25519 (third-party library the reference's OpenSSL idiom binds,
 * util/src/openssl_crypto.cpp:229-253 — success only on == 1; the reference snapshot has no
 * Ed25519 code of its own):
 *   1. S < L (strict)                          2. A: low 255 bits as y, NOT reduced-checked,
 *   3. h = SHA-512(R || A || M) mod L             x by the (p+3)/8 root, off-curve -> reject,
 *   4. R' = [S]B - [h]A, cofactorless             sign applied by negation (x = 0, sign 1 ok)
 *   5. accept iff encode(R') == R bytewise
 * Pinned by tests/golden/ed25519_vectors.bin (verdicts from the container's OpenSSL 3.0.2) and
 * the RFC 8032 test vectors 1-3 (tests/test_oracle.py).
 *
 * Field: radix 2^51, 5 limbs, unsigned __int128 products.  Scalar multiplication: plain
 * binary double-and-add in extended coordinates (clarity over speed; ~0.3 ms per verify).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "sha512_oracle.h"

typedef unsigned __int128 u128;
typedef struct {
  uint64_t v[5];
} fo;
#define M51 ((1ULL << 51) - 1)

static void fo_carry(fo* r) {
  for (int k = 0; k < 2; k++) {
    uint64_t c = 0;
    for (int i = 0; i < 5; i++) {
      r->v[i] += c;
      c = r->v[i] >> 51;
      r->v[i] &= M51;
    }
    r->v[0] += 19 * c;
  }
}
static void fo_add(fo* r, const fo* a, const fo* b) {
  for (int i = 0; i < 5; i++) r->v[i] = a->v[i] + b->v[i];
  fo_carry(r);
}
static void fo_sub(fo* r, const fo* a, const fo* b) {
  /* + 4p: limbs 4*(2^51-19), 4*(2^51-1) */
  r->v[0] = a->v[0] + 0x1FFFFFFFFFFFB4ULL - b->v[0];
  for (int i = 1; i < 5; i++) r->v[i] = a->v[i] + 0x1FFFFFFFFFFFFCULL - b->v[i];
  fo_carry(r);
}
static void fo_mul(fo* r, const fo* a, const fo* b) {
  u128 t[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < 5; i++)
    for (int j = 0; j < 5; j++) {
      u128 p = (u128)a->v[i] * b->v[j];
      if (i + j < 5)
        t[i + j] += p;
      else
        t[i + j - 5] += p * 19;
    }
  uint64_t c = 0;
  for (int i = 0; i < 5; i++) {
    t[i] += c;
    r->v[i] = (uint64_t)t[i] & M51;
    c = (uint64_t)(t[i] >> 51);
  }
  r->v[0] += 19 * c;
  fo_carry(r);
}
static void fo_set(fo* r, uint64_t x) {
  memset(r, 0, sizeof *r);
  r->v[0] = x;
}
static void fo_frombytes(fo* r, const uint8_t s[32]) { /* low 255 bits, not reduced */
  uint64_t w[4];
  for (int i = 0; i < 4; i++) {
    w[i] = 0;
    for (int k = 7; k >= 0; k--) w[i] = (w[i] << 8) | s[8 * i + k];
  }
  w[3] &= 0x7FFFFFFFFFFFFFFFULL;
  r->v[0] = w[0] & M51;
  r->v[1] = ((w[0] >> 51) | (w[1] << 13)) & M51;
  r->v[2] = ((w[1] >> 38) | (w[2] << 26)) & M51;
  r->v[3] = ((w[2] >> 25) | (w[3] << 39)) & M51;
  r->v[4] = (w[3] >> 12) & M51;
}
static void fo_tobytes(uint8_t s[32], const fo* a) { /* canonical */
  fo t = *a;
  fo_carry(&t);
  /* t < 2^255 + small; subtract p if t >= p */
  uint64_t u[5], c = 19;
  for (int i = 0; i < 5; i++) {
    u[i] = t.v[i] + c;
    c = u[i] >> 51;
    u[i] &= M51;
  }
  if (c) memcpy(t.v, u, sizeof u); /* t + 19 >= 2^255  <=>  t >= p */
  uint64_t w[4];
  w[0] = t.v[0] | (t.v[1] << 51);
  w[1] = (t.v[1] >> 13) | (t.v[2] << 38);
  w[2] = (t.v[2] >> 26) | (t.v[3] << 25);
  w[3] = (t.v[3] >> 39) | (t.v[4] << 12);
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 8; k++) s[8 * i + k] = (uint8_t)(w[i] >> (8 * k));
}
static int fo_iszero(const fo* a) {
  uint8_t s[32];
  fo_tobytes(s, a);
  uint8_t o = 0;
  for (int i = 0; i < 32; i++) o |= s[i];
  return o == 0;
}
static int fo_isneg(const fo* a) {
  uint8_t s[32];
  fo_tobytes(s, a);
  return s[0] & 1;
}
static void fo_pow(fo* r, const fo* a, const uint8_t e[32]) { /* e little-endian */
  fo acc, base = *a;
  fo_set(&acc, 1);
  for (int i = 0; i < 256; i++) {
    if ((e[i >> 3] >> (i & 7)) & 1) fo_mul(&acc, &acc, &base);
    fo_mul(&base, &base, &base);
  }
  *r = acc;
}
static void fo_neg(fo* r, const fo* a) {
  fo z;
  fo_set(&z, 0);
  fo_sub(r, &z, a);
}

/* constants */
static fo D, D2, SQRTM1;
static uint8_t EXP_P58[32], EXP_PM2[32];
static int consts_ready;
static void init_consts(void) {
  if (consts_ready) return;
  /* p - 2 and (p - 5)/8 as little-endian byte strings */
  memset(EXP_PM2, 0xff, 32);
  EXP_PM2[0] = 0xeb;
  EXP_PM2[31] = 0x7f;
  memset(EXP_P58, 0xff, 32); /* (2^255-24)/8 = 2^252 - 3 */
  EXP_P58[0] = 0xfd;
  EXP_P58[31] = 0x0f;
  fo n, dd, t;
  fo_set(&n, 121665);
  fo_neg(&n, &n);
  fo_set(&dd, 121666);
  fo_pow(&t, &dd, EXP_PM2);
  fo_mul(&D, &n, &t);
  fo_add(&D2, &D, &D);
  /* sqrt(-1) = 2^((p-1)/4) ; (p-1)/4 = 2^253 - 5 */
  uint8_t e[32];
  memset(e, 0xff, 32);
  e[0] = 0xfb;
  e[31] = 0x1f;
  fo two;
  fo_set(&two, 2);
  fo_pow(&SQRTM1, &two, e);
  consts_ready = 1;
}

typedef struct {
  fo X, Y, Z, T;
} pt;

static void pt_add(pt* r, const pt* p, const pt* q) {
  fo a, b, c, d, e, f, g, h, t1, t2;
  fo_sub(&t1, &p->Y, &p->X);
  fo_sub(&t2, &q->Y, &q->X);
  fo_mul(&a, &t1, &t2);
  fo_add(&t1, &p->Y, &p->X);
  fo_add(&t2, &q->Y, &q->X);
  fo_mul(&b, &t1, &t2);
  fo_mul(&c, &p->T, &q->T);
  fo_mul(&c, &c, &D2);
  fo_mul(&d, &p->Z, &q->Z);
  fo_add(&d, &d, &d);
  fo_sub(&e, &b, &a);
  fo_sub(&f, &d, &c);
  fo_add(&g, &d, &c);
  fo_add(&h, &b, &a);
  fo_mul(&r->X, &e, &f);
  fo_mul(&r->Y, &g, &h);
  fo_mul(&r->Z, &f, &g);
  fo_mul(&r->T, &e, &h);
}
static void pt_zero(pt* r) {
  fo_set(&r->X, 0);
  fo_set(&r->Y, 1);
  fo_set(&r->Z, 1);
  fo_set(&r->T, 0);
}
static void pt_smul(pt* r, const uint8_t k[32], const pt* p) {
  pt acc, base = *p;
  pt_zero(&acc);
  for (int i = 0; i < 256; i++) {
    if ((k[i >> 3] >> (i & 7)) & 1) pt_add(&acc, &acc, &base);
    pt_add(&base, &base, &base);
  }
  *r = acc;
}
static void pt_encode(uint8_t s[32], const pt* p) {
  fo zi, x, y;
  fo_pow(&zi, &p->Z, EXP_PM2);
  fo_mul(&x, &p->X, &zi);
  fo_mul(&y, &p->Y, &zi);
  fo_tobytes(s, &y);
  s[31] |= (uint8_t)(fo_isneg(&x) << 7);
}
/* OpenSSL ge_frombytes_vartime semantics */
static int pt_decode(pt* r, const uint8_t s[32]) {
  fo u, v, v3, vxx, chk, one, x, y;
  fo_set(&one, 1);
  fo_frombytes(&y, s);
  fo_mul(&u, &y, &y);
  fo_mul(&v, &u, &D);
  fo_sub(&u, &u, &one);
  fo_add(&v, &v, &one);
  fo_mul(&v3, &v, &v);
  fo_mul(&v3, &v3, &v);
  fo_mul(&x, &v3, &v3);
  fo_mul(&x, &x, &v);
  fo_mul(&x, &x, &u);
  fo_pow(&x, &x, EXP_P58);
  fo_mul(&x, &x, &v3);
  fo_mul(&x, &x, &u);
  fo_mul(&vxx, &x, &x);
  fo_mul(&vxx, &vxx, &v);
  fo_sub(&chk, &vxx, &u);
  if (!fo_iszero(&chk)) {
    fo_add(&chk, &vxx, &u);
    if (!fo_iszero(&chk)) return -1;
    fo_mul(&x, &x, &SQRTM1);
  }
  if (fo_isneg(&x) != (s[31] >> 7)) fo_neg(&x, &x);
  r->X = x;
  r->Y = y;
  fo_set(&r->Z, 1);
  fo_mul(&r->T, &x, &y);
  return 0;
}

/* scalars mod L: 512-bit little-endian byte string reduced by bitwise long division */
static const uint8_t L_BYTES[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7,
                                    0xa2, 0xde, 0xf9, 0xde, 0x14, 0,    0,    0,    0,    0,    0,
                                    0,    0,    0,    0,    0,    0,    0,    0,    0,    0x10};
static int cmp_le(const uint8_t* a, const uint8_t* b, int n) {
  for (int i = n - 1; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  }
  return 0;
}
static void sc_reduce(uint8_t r[32], const uint8_t x[64]) {
  uint8_t acc[33];
  memset(acc, 0, sizeof acc);
  uint8_t l33[33];
  memcpy(l33, L_BYTES, 32);
  l33[32] = 0;
  for (int bit = 511; bit >= 0; bit--) {
    /* acc = acc*2 + bit */
    int c = (x[bit >> 3] >> (bit & 7)) & 1;
    for (int i = 0; i < 33; i++) {
      int nc = acc[i] >> 7;
      acc[i] = (uint8_t)((acc[i] << 1) | c);
      c = nc;
    }
    if (cmp_le(acc, l33, 33) >= 0) {
      int br = 0;
      for (int i = 0; i < 33; i++) {
        int d = acc[i] - l33[i] - br;
        br = d < 0;
        acc[i] = (uint8_t)(d + (br ? 256 : 0));
      }
    }
  }
  memcpy(r, acc, 32);
}

static const uint8_t B_ENC[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                  0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                  0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};

int cbft_oracle_ed25519_verify(const uint8_t pk[32], const uint8_t* msg, size_t len, const uint8_t sig[64]) {
  init_consts();
  const uint8_t* S = sig + 32;
  if (cmp_le(S, L_BYTES, 32) >= 0) return 0;
  pt A, B, sB, hA, R;
  if (pt_decode(&A, pk) != 0) return 0;
  pt_decode(&B, B_ENC);
  sha512o_ctx c;
  uint8_t dig[64], h[32], enc[32];
  sha512o_init(&c);
  sha512o_update(&c, sig, 32);
  sha512o_update(&c, pk, 32);
  sha512o_update(&c, msg, len);
  sha512o_final(&c, dig);
  sc_reduce(h, dig);
  pt_smul(&sB, S, &B);
  pt_smul(&hA, h, &A);
  fo_neg(&hA.X, &hA.X);
  fo_neg(&hA.T, &hA.T);
  pt_add(&R, &sB, &hA);
  pt_encode(enc, &R);
  return memcmp(enc, sig, 32) == 0;
}

/* Batch form with the C ABI's layout (blob + offsets + lengths, keys by index); writes one
 * byte per signature (0/1). */
void cbft_oracle_ed25519_verify_many(const uint8_t* pk, const uint32_t* key_idx, const uint8_t* sig,
                                     const uint8_t* blob, const uint64_t* off, const uint32_t* len, size_t n,
                                     uint8_t* out) {
  for (size_t i = 0; i < n; i++) {
    const uint8_t* k = pk + 32 * (size_t)(key_idx ? key_idx[i] : i);
    out[i] = (uint8_t)cbft_oracle_ed25519_verify(k, blob + off[i], len[i], sig + 64 * i);
  }
}

/* RFC 8032 §5.1.5 / §5.1.6 key derivation and signing (fixture generation). */
static void expand(const uint8_t sk[32], uint8_t a[32], uint8_t prefix[32]) {
  sha512o_ctx c;
  uint8_t d[64];
  sha512o_init(&c);
  sha512o_update(&c, sk, 32);
  sha512o_final(&c, d);
  memcpy(a, d, 32);
  a[0] &= 248;
  a[31] &= 127;
  a[31] |= 64;
  memcpy(prefix, d + 32, 32);
}
void cbft_oracle_ed25519_pubkey(const uint8_t sk[32], uint8_t pk[32]) {
  init_consts();
  uint8_t a[32], pre[32];
  expand(sk, a, pre);
  pt B, A;
  pt_decode(&B, B_ENC);
  pt_smul(&A, a, &B);
  pt_encode(pk, &A);
}
static void sc_muladd(uint8_t s[32], const uint8_t a[32], const uint8_t b[32], const uint8_t c[32]) {
  /* s = (a*b + c) mod L via 512-bit schoolbook */
  uint32_t t[64] = {0};
  for (int i = 0; i < 32; i++)
    for (int j = 0; j < 32; j++) t[i + j] += (uint32_t)a[i] * b[j];
  for (int i = 0; i < 32; i++) t[i] += c[i];
  uint8_t x[64];
  uint32_t carry = 0;
  for (int i = 0; i < 64; i++) {
    uint32_t v = t[i] + carry;
    x[i] = (uint8_t)v;
    carry = v >> 8;
  }
  sc_reduce(s, x);
}
void cbft_oracle_ed25519_sign(const uint8_t sk[32], const uint8_t* msg, size_t len, uint8_t sig[64]) {
  init_consts();
  uint8_t a[32], pre[32], pk[32], dig[64], r[32], h[32];
  expand(sk, a, pre);
  pt B, Rp;
  pt_decode(&B, B_ENC);
  cbft_oracle_ed25519_pubkey(sk, pk);
  sha512o_ctx c;
  sha512o_init(&c);
  sha512o_update(&c, pre, 32);
  sha512o_update(&c, msg, len);
  sha512o_final(&c, dig);
  sc_reduce(r, dig);
  pt_smul(&Rp, r, &B);
  pt_encode(sig, &Rp);
  sha512o_init(&c);
  sha512o_update(&c, sig, 32);
  sha512o_update(&c, pk, 32);
  sha512o_update(&c, msg, len);
  sha512o_final(&c, dig);
  sc_reduce(h, dig);
  sc_muladd(sig + 32, h, a, r);
}
