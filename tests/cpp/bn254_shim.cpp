// Host build of the BN-P254 device code (concord-bft_amd/csrc/bn254_*.h), exposed to the
// Python tests through ctypes: the SAME source that runs on gfx950, checked on the CPU against
// oracle/bn254_ref.py.  Test infrastructure; also the labelled "not RELIC" CPU baseline.
#include <cstring>
#include <memory>
#include <random>
#include <thread>
#include <vector>

#include "bls_ops.h"
#include "bn254_cycsq.h"

static void fp12_flat(uint8_t* out, const fp12& x) {  // 12 x 32-byte big-endian, oracle basis
  const fp2* e[6] = {&x.c0.c0, &x.c1.c0, &x.c0.c1, &x.c1.c1, &x.c0.c2, &x.c1.c2};
  for (int k = 0; k < 6; k++) {
    fp lo;
    f_sub(lo, e[k]->a, e[k]->b);
    uint32_t w[8];
    f_to_words(w, lo);
    words_to_be32(out + 32 * k, w);
    f_to_words(w, e[k]->b);
    words_to_be32(out + 32 * (k + 6), w);
  }
}

#include "row_emu.h"
// every rf_mul's operands checked against its precondition: row-normal limbs and
// (a / q)(b / q) < 221 in every row (counted in g_rf_bound_violations)
static void rf_mul_check(const HU& a, const HU& b);
#define RF_MUL_CHECK(a, b) rf_mul_check(a, b)
#include "bn254_row.h"
#include "bn254_g1row.h"
#include "bn254_g2row.h"

static long g_rf_bound_violations = 0;
static long double rf_row_over_q(const HU& x, int row) {
  static const long double q = [] {
    long double v = 0;
    for (int i = BN_LIMBS - 1; i >= 0; i--) v = v * 536870912.0L + FpParams::Q[i];
    return v;
  }();
  long double v = 0;
  for (int i = BN_LIMBS - 1; i >= 0; i--) v = v * 536870912.0L + x.x[16 * row + i];
  return v / q;
}
static void rf_mul_check(const HU& a, const HU& b) {
  for (int row = 0; row < 4; row++) {
    for (int l = 0; l < 16; l++) {
      const uint32_t lim = l < 9 ? (1u << 29) + 8 : 0u;
      if (a.x[16 * row + l] > lim || b.x[16 * row + l] > lim) g_rf_bound_violations++;
    }
    if (rf_row_over_q(a, row) * rf_row_over_q(b, row) >= 221.0L) g_rf_bound_violations++;
  }
}

// ---- safegcd30.h's wave inversion (sg_inv30_var_wave) over an emulated 64-lane wave: the same
// stage functions (sg_w_split1 / sg_w_split2 / sg_w_m / sg_canon30 / sg_divsteps30_var) with the
// DPP row shifts written out (row_shl:1 / row_shr:1 within 16-lane rows, 0 past a row's edge)
struct Sg25519 {
  static constexpr int32_t P[9] = {0x3fffffed, 0x3fffffff, 0x3fffffff, 0x3fffffff, 0x3fffffff,
                                   0x3fffffff, 0x3fffffff, 0x3fffffff, 0x00007fff};
  static constexpr uint32_t PINV30 = 0x179435e5u;
};
static long g_sgw_batches = 0, g_sgw_redundant = 0;
static void sgw_column(int32_t* out, const int64_t* c) {
  uint32_t lo[64], la[64];
  int64_t hi[64];
  int32_t lo2[64], hi2[64];
  for (int l = 0; l < 64; l++) sg_w_split1(c[l], lo[l], hi[l]);
  for (int l = 0; l < 64; l++) la[l] = (l & 15) == 15 ? 0u : lo[l + 1];
  for (int l = 0; l < 64; l++) sg_w_split2(hi[l], la[l], l == 8, lo2[l], hi2[l]);
  for (int l = 0; l < 64; l++) out[l] = lo2[l] + ((l & 15) == 0 ? 0 : hi2[l - 1]);
}
template <class M>
static void sgw_inv(Sg30& x) {
  int32_t P[64] = {0}, f[64], g[64] = {0}, d[64] = {0}, e[64] = {0};
  for (int k = 0; k < 9; k++) {
    P[k] = M::P[k];
    g[k] = x.v[k];
  }
  std::memcpy(f, P, sizeof f);
  e[0] = 1;
  int32_t eta = -1;
  for (int it = 0; it < 64; it++) {
    g_sgw_batches++;
    int32_t t[4], md, me;
    eta = sg_divsteps30_var(eta, (uint32_t)f[0], (uint32_t)g[0], t);
    sg_w_m<M>(md, me, t, d[0], e[0], d[8], e[8]);
    int64_t cd[64], ce[64], cf[64], cg[64];
    for (int l = 0; l < 64; l++) {
      cd[l] = (int64_t)t[0] * d[l] + (int64_t)t[1] * e[l] + (int64_t)P[l] * md;
      ce[l] = (int64_t)t[2] * d[l] + (int64_t)t[3] * e[l] + (int64_t)P[l] * me;
      cf[l] = (int64_t)t[0] * f[l] + (int64_t)t[1] * g[l];
      cg[l] = (int64_t)t[2] * f[l] + (int64_t)t[3] * g[l];
    }
    sgw_column(d, cd);
    sgw_column(e, ce);
    sgw_column(f, cf);
    sgw_column(g, cg);
    for (int l = 0; l < 8; l++)
      if (d[l] < 0 || d[l] > (int32_t)SG_M30 || e[l] < 0 || e[l] > (int32_t)SG_M30) g_sgw_redundant++;
    bool far = false;  // some limb cannot be part of a zero value
    for (int l = 0; l < 64; l++) far = far || !sg_w_zero_limb(g[l]);
    if (!far) {
      Sg30 gg;
      for (int k = 0; k < 9; k++) gg.v[k] = g[k];
      if (sg_is_zero30(gg)) break;
    }
  }
  const int32_t fsign = f[0] == 1 ? 1 : -1;
  for (int k = 0; k < 9; k++) x.v[k] = d[k];
  sg_canon30<M>(x, fsign);
}

extern "C" {

// sg_inv30_var_wave's emulation on x (32-byte big-endian, < p; which = 0: BN-P254's p, 1:
// 2^255 - 19): out = x^-1 (big-endian, canonical).  Returns the batches run; *redundant counts the
// batches that left some low limb of d or e outside [0, 2^30).
long shim_sg_wave_inv(int which, const uint8_t* x32, uint8_t* out32, long* redundant) {
  uint32_t w[8];
  be32_to_words(w, x32);
  Sg30 x;
  for (int j = 0; j < 9; j++) {
    const int b = 30 * j, i = b >> 5, sh = b & 31;
    const uint64_t v = ((uint64_t)(i + 1 < 8 ? w[i + 1] : 0u) << 32) | (i < 8 ? w[i] : 0u);
    x.v[j] = (int32_t)((v >> sh) & SG_M30);
  }
  g_sgw_batches = 0;
  g_sgw_redundant = 0;
  if (which == 0)
    sgw_inv<BnS30Mod>(x);
  else
    sgw_inv<Sg25519>(x);
  for (int i = 0; i < 8; i++) {
    const int b = 32 * i, j = b / 30, sh = b % 30;
    const uint64_t v = ((uint64_t)(uint32_t)(j + 2 < 9 ? x.v[j + 2] : 0) << 60) |
                       ((uint64_t)(uint32_t)(j + 1 < 9 ? x.v[j + 1] : 0) << 30) | (uint32_t)x.v[j];
    w[i] = (uint32_t)(v >> sh);
  }
  words_to_be32(out32, w);
  *redundant = g_sgw_redundant;
  return g_sgw_batches;
}

// f_add / f_sub / f_addsub on Montgomery forms of a, b (< p, 32-byte big-endian): writes the
// canonical results of add, sub, addsub(add = 1), addsub(add = 0); returns 1 if the reduced
// representations of addsub equal f_add's / f_sub's limb for limb.
int shim_fp_addsub(const uint8_t* a32, const uint8_t* b32, uint8_t* out128) {
  uint32_t w[8];
  fp a, b, r[4];
  be32_to_words(w, a32);
  f_from_words(a, w);
  be32_to_words(w, b32);
  f_from_words(b, w);
  f_add(r[0], a, b);
  f_sub(r[1], a, b);
  f_addsub(r[2], a, b, true);
  f_addsub(r[3], a, b, false);
  for (int k = 0; k < 4; k++) {
    f_to_words(w, r[k]);
    words_to_be32(out128 + 32 * k, w);
  }
  return std::memcmp(&r[0], &r[2], sizeof(fp)) == 0 && std::memcmp(&r[1], &r[3], sizeof(fp)) == 0;
}

// fp_inv_var and fp_inv of the canonical integer x (32-byte big-endian, < p): out_var, out_fermat
// (big-endian canonical).  Returns 1 if both agree.
int shim_fp_inv(const uint8_t* x32, uint8_t* out_var, uint8_t* out_fermat) {
  uint32_t w[8];
  be32_to_words(w, x32);
  fp a, r1, r2;
  f_from_words(a, w);
  fp_inv_var(r1, a);
  fp_inv(r2, a);
  f_to_words(w, r1);
  words_to_be32(out_var, w);
  uint32_t w2[8];
  f_to_words(w2, r2);
  words_to_be32(out_fermat, w2);
  return std::memcmp(w, w2, sizeof w) == 0 ? 1 : 0;
}

// rf_pow_sw (bn254_row.h) for the square-root schedule on four emulated rows against the one-lane
// f_pow_sw, for four values x (32-byte big-endian, < p): writes the four row results (big-endian
// canonical) and returns 1 when each equals the one-lane result and no product broke its bounds.
int shim_rf_sqrt_pow(const uint8_t* x128, uint8_t* out128) {
  HU in;
  fp lane[4];
  for (int r = 0; r < 4; r++) {
    uint32_t w[8];
    be32_to_words(w, x128 + 32 * r);
    f_from_words(lane[r], w);
    for (int i = 0; i < BN_LIMBS; i++) in.x[16 * r + i] = lane[r].v[i];
  }
  const long v0 = g_rf_bound_violations;
  const HU qrow = rf_row_const(FpParams::Q, in);
  const HU y = rf_pow_sw<FpSqrtSchedule, HU, HW>(in, qrow);
  int ok = g_rf_bound_violations == v0;
  for (int r = 0; r < 4; r++) {
    fp a, b;
    uint32_t c = 0;
    for (int i = 0; i < BN_LIMBS; i++) {
      const uint32_t t = y.x[16 * r + i] + c;
      a.v[i] = i < BN_LIMBS - 1 ? (t & BN_MASK) : t;
      c = t >> 29;
    }
    f_pow_sw<FpParams, FpSqrtSchedule>(b, lane[r]);
    uint32_t wa[8], wb[8];
    f_to_words(wa, a);
    f_to_words(wb, b);
    words_to_be32(out128 + 32 * r, wa);
    ok = ok && std::memcmp(wa, wb, sizeof wa) == 0;
  }
  return ok;
}

// sha256_key_msg (sha256.h: the BLS blinds' register-resident SHA-256) -> 32-byte digest
void shim_sha256_key_msg(const uint32_t* key8, uint32_t x, const uint8_t* msg, uint32_t m, uint8_t* out32) {
  uint32_t h[8];
  sha256_key_msg(h, key8, (uint8_t)x, msg, m);
  for (int i = 0; i < 8; i++)
    for (int q = 0; q < 4; q++) out32[4 * i + q] = (uint8_t)(h[i] >> (24 - 8 * q));
}

// ---- the lazy cyclotomic squaring (bn254_cycsq.h) on an emulated pair36 wave ----------------
static uint64_t sm64(uint64_t& x) {
  uint64_t z = (x += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
static void fp_random(fp& r, uint64_t& st) {
  uint32_t w[8];
  for (int i = 0; i < 8; i++) w[i] = (uint32_t)sm64(st);
  w[7] &= 0x1fffffffu;  // < 2^253 < p
  f_from_words(r, w);
}
static int cs_src(int k, int h, int s) { return 12 * s + 2 * k + h; }
static fp2* fp12_coef(fp12& x, int k) {
  fp2* e[6] = {&x.c0.c0, &x.c1.c0, &x.c0.c1, &x.c1.c1, &x.c0.c2, &x.c1.c2};
  return e[k];
}
// normalised limbs and value < 2q
static bool fp_reduced(const fp& x) {
  for (int i = 0; i < BN_LIMBS - 1; i++)
    if (x.v[i] > BN_MASK) return false;
  uint32_t q2[BN_LIMBS];
  f_2q<FpParams>(q2);
  for (int i = BN_LIMBS - 1; i >= 0; i--) {
    if (x.v[i] != q2[i]) return x.v[i] < q2[i];
  }
  return false;
}

// fp_reduce64 on raw limbs x9 -> out9; returns 1 when the output is normalised and < 2q
int shim_fp_reduce64(const uint32_t* x9, uint32_t* out9) {
  fp x, r;
  std::memcpy(x.v, x9, sizeof x.v);
  fp_reduce64(r, x);
  std::memcpy(out9, r.v, sizeof r.v);
  return fp_reduced(r) ? 1 : 0;
}

// f_mul on raw limbs (the cyclotomic squaring's unreduced operands); 1 when normalised, < 2q
int shim_fp_mul_raw(const uint32_t* a9, const uint32_t* b9, uint32_t* out9) {
  fp a, b, r;
  std::memcpy(a.v, a9, sizeof a.v);
  std::memcpy(b.v, b9, sizeof b.v);
  f_mul(r, a, b);
  std::memcpy(out9, r.v, sizeof r.v);
  return fp_reduced(r) ? 1 : 0;
}

// A random element of the cyclotomic subgroup (f^((p^6 - 1)(p^2 + 1))) squared `iters` times by
// the lane stages of p36_cyc_sqr over an emulated 36-lane wave, against fp12_sqr.  Returns 1 on
// success; -1 a lane left the reduced form, -2 the sub-lane replicas differ, -3 a value differs.
int shim_cyc_sqr_emul(uint64_t seed, int iters) {
  uint64_t st = seed;
  fp12 f, fi, g, t;
  for (int k = 0; k < 6; k++) {
    fp_random(fp12_coef(f, k)->a, st);
    fp_random(fp12_coef(f, k)->b, st);
  }
  fp12_inv(fi, f);
  fp12_conj(g, f);
  fp12_mul(g, g, fi);
  fp12_frob2(t, g);
  fp12_mul(g, t, g);
  fp lane[36];
  for (int L = 0; L < 36; L++) {
    const int c = L % 12, k = c >> 1, h = c & 1;
    const fp2* e = fp12_coef(g, k);
    lane[L] = h ? e->b : e->a;
  }
  fp12 ref = g;
  for (int it = 0; it < iters; it++) {
    fp R[36], T[36], v[36], r[36];
    for (int L = 0; L < 36; L++) {
      const int c = L % 12, s = L / 12, k = c >> 1, h = c & 1;
      cs_pre(R[L], lane[L], lane[cs_src(k < 3 ? k + 3 : k - 3, h, s)], s);
    }
    for (int L = 0; L < 36; L++) {
      const int c = L % 12, s = L / 12, k = c >> 1, h = c & 1;
      const int sx = (k == 0 || k == 3) ? 0 : ((k == 1 || k == 4) ? 2 : 1);
      const int cc = s == 1 ? sx + 3 : sx;
      fp U, V;
      cs_operands(U, V, R[cs_src(cc, h, s)], R[cs_src(cc, 1 - h, s)], h);
      f_mul(T[L], U, V);
    }
    for (int L = 0; L < 36; L++) {
      const int c = L % 12, k = c >> 1, h = c & 1;
      const bool odd = (k & 1) != 0;
      cs_combine(v[L], T[cs_src(k, h, 0)], T[cs_src(k, h, 1)], odd ? T[cs_src(k, h, 2)] : T[cs_src(k, 1 - h, 1)], k, h);
    }
    for (int L = 0; L < 36; L++) {
      const int c = L % 12, s = L / 12, k = c >> 1, h = c & 1;
      cs_finish(r[L], v[L], v[cs_src(k, 1 - h, s)], lane[L], k, h);
    }
    for (int L = 0; L < 36; L++) {
      if (!fp_reduced(r[L])) return -1;
      if (std::memcmp(&r[L], &r[L % 12], sizeof(fp)) != 0) return -2;
      lane[L] = r[L];
    }
    fp12_sqr(ref, ref);
  }
  for (int k = 0; k < 6; k++) {
    const fp2* e = fp12_coef(ref, k);
    if (!f_eq(lane[2 * k], e->a) || !f_eq(lane[2 * k + 1], e->b)) return -3;
  }
  return 1;
}

// p36_mul's lane stages (cm_terms, cm_xi, cm_sum3) over an emulated 36-lane wave: x <- x * y
// `iters` times from random x, y, against fp12_mul.  Return codes as shim_cyc_sqr_emul.
int shim_p36_mul_emul(uint64_t seed, int iters) {
  uint64_t st = seed;
  fp12 x, y;
  for (int k = 0; k < 6; k++) {
    fp_random(fp12_coef(x, k)->a, st);
    fp_random(fp12_coef(x, k)->b, st);
    fp_random(fp12_coef(y, k)->a, st);
    fp_random(fp12_coef(y, k)->b, st);
  }
  fp la[36], lb[36];
  for (int L = 0; L < 36; L++) {
    const int c = L % 12, k = c >> 1, h = c & 1;
    la[L] = h ? fp12_coef(x, k)->b : fp12_coef(x, k)->a;
    lb[L] = h ? fp12_coef(y, k)->b : fp12_coef(y, k)->a;
  }
  fp12 ref = x;
  for (int it = 0; it < iters; it++) {
    fp acc[36], accw[36], z[36], r[36];
    for (int L = 0; L < 36; L++) {
      const int c = L % 12, s = L / 12, k = c >> 1, h = c & 1;
      fp T[4];
      bool wrap[2];
      for (int t = 0; t < 2; t++) {
        const int i = 2 * s + t;
        int j = k - i;
        wrap[t] = j < 0;
        if (wrap[t]) j += 6;
        const fp& am = la[cs_src(i, h, s)];
        const fp& ao = la[cs_src(i, 1 - h, s)];
        const fp& bm = lb[cs_src(j, h, s)];
        const fp& bo = lb[cs_src(j, 1 - h, s)];
        f_mul(T[2 * t], h ? ao : am, bm);
        f_mul(T[2 * t + 1], h ? am : ao, bo);
      }
      cm_terms(acc[L], accw[L], T[0], T[1], T[2], T[3], h, wrap[0], wrap[1]);
    }
    for (int L = 0; L < 36; L++) {
      const int c = L % 12, s = L / 12, k = c >> 1, h = c & 1;
      cm_xi(z[L], acc[L], accw[L], accw[cs_src(k, 1 - h, s)], h);
    }
    for (int L = 0; L < 36; L++) {
      const int c = L % 12, k = c >> 1, h = c & 1;
      cm_sum3(r[L], z[cs_src(k, h, 0)], z[cs_src(k, h, 1)], z[cs_src(k, h, 2)]);
    }
    for (int L = 0; L < 36; L++) {
      if (!fp_reduced(r[L])) return -1;
      if (std::memcmp(&r[L], &r[L % 12], sizeof(fp)) != 0) return -2;
      la[L] = r[L];
    }
    fp12_mul(ref, ref, y);
  }
  for (int k = 0; k < 6; k++) {
    const fp2* e = fp12_coef(ref, k);
    if (!f_eq(la[2 * k], e->a) || !f_eq(la[2 * k + 1], e->b)) return -3;
  }
  return 1;
}

// p36_sqr's lane stages (sq_operands, cm_terms, cm_xi, cm_sum3) over an emulated wave: x <- x^2
// `iters` times from a random (non-cyclotomic) x, against fp12_sqr.  kSq = bn254_pair12.h's
// kP12Sq term table (i, j, flags: bit 1 = times xi), repeated here for the host build.
static const uint8_t kSq[6][4][3] = {
    {{0, 0, 4}, {3, 3, 6}, {1, 5, 7}, {2, 4, 7}}, {{0, 1, 5}, {2, 5, 7}, {3, 4, 7}, {0, 0, 0}},
    {{1, 1, 4}, {4, 4, 6}, {0, 2, 5}, {3, 5, 7}}, {{0, 3, 5}, {1, 2, 5}, {4, 5, 7}, {0, 0, 0}},
    {{2, 2, 4}, {5, 5, 6}, {0, 4, 5}, {1, 3, 5}}, {{0, 5, 5}, {1, 4, 5}, {2, 3, 5}, {0, 0, 0}},
};
int shim_p36_sqr_emul(uint64_t seed, int iters) {
  uint64_t st = seed;
  fp12 x;
  for (int k = 0; k < 6; k++) {
    fp_random(fp12_coef(x, k)->a, st);
    fp_random(fp12_coef(x, k)->b, st);
  }
  fp la[36];
  for (int L = 0; L < 36; L++) {
    const int c = L % 12, k = c >> 1, h = c & 1;
    la[L] = h ? fp12_coef(x, k)->b : fp12_coef(x, k)->a;
  }
  fp12 ref = x;
  fp zero;
  f_zero(zero);
  for (int it = 0; it < iters; it++) {
    fp acc[36], accw[36], z[36], r[36];
    for (int L = 0; L < 36; L++) {
      const int c = L % 12, s = L / 12, k = c >> 1, h = c & 1;
      const bool even = (k & 1) == 0, diag = even && s == 0;
      const int tt = even ? s + 1 : s;
      const int f1 = diag ? kSq[k][0][0] : kSq[k][tt][0];
      const int f2 = diag ? kSq[k][1][0] : kSq[k][tt][1];
      const bool cwrap = (kSq[k][tt][2] & 2) != 0;
      fp U1, V1, U2, V2, P1, P2;
      sq_operands(U1, V1, U2, V2, la[cs_src(f1, h, s)], la[cs_src(f1, 1 - h, s)], la[cs_src(f2, h, s)],
                  la[cs_src(f2, 1 - h, s)], diag, h);
      f_mul(P1, U1, V1);
      f_mul(P2, U2, V2);
      cm_terms(acc[L], accw[L], P1, diag ? zero : P2, diag ? P2 : zero, zero, h, !diag && cwrap, true);
    }
    for (int L = 0; L < 36; L++) {
      const int c = L % 12, s = L / 12, k = c >> 1, h = c & 1;
      cm_xi(z[L], acc[L], accw[L], accw[cs_src(k, 1 - h, s)], h);
    }
    for (int L = 0; L < 36; L++) {
      const int c = L % 12, k = c >> 1, h = c & 1;
      cm_sum3(r[L], z[cs_src(k, h, 0)], z[cs_src(k, h, 1)], z[cs_src(k, h, 2)]);
    }
    for (int L = 0; L < 36; L++) {
      if (!fp_reduced(r[L])) return -1;
      if (std::memcmp(&r[L], &r[L % 12], sizeof(fp)) != 0) return -2;
      la[L] = r[L];
    }
    fp12_sqr(ref, ref);
  }
  for (int k = 0; k < 6; k++) {
    const fp2* e = fp12_coef(ref, k);
    if (!f_eq(la[2 * k], e->a) || !f_eq(la[2 * k + 1], e->b)) return -3;
  }
  return 1;
}

// g1_dbl_lazy (the stages of g1q_dbl) against g1_dbl, `iters` doublings deep from g1_map(seed):
// 1 when every step gives the same affine point and reduced coordinates, else a negative code
int shim_g1_dbl_lazy(uint64_t seed, int iters) {
  uint8_t msg[8];
  for (int i = 0; i < 8; i++) msg[i] = (uint8_t)(seed >> (8 * i));
  g1a h;
  g1_map(h, msg, 8);
  g1j p, q;
  g1_from_affine(p, h);
  q = p;
  for (int it = 0; it < iters; it++) {
    g1_dbl(p, p);
    g1_dbl_lazy(q, q);
    if (!fp_reduced(q.X) || !fp_reduced(q.Y) || !fp_reduced(q.Z)) return -1;
    g1a a, b;
    g1_to_affine(a, p);
    g1_to_affine(b, q);
    if (a.inf != b.inf || !f_eq(a.x, b.x) || !f_eq(a.y, b.y)) return -3;
  }
  return 1;
}

// fp_lin3 for the coefficient sets the G2 line steps use, on canonical inputs a, b, c (32-byte
// big-endian, < p): out = 5 x 32-byte canonical results; 1 when every result is reduced
int shim_fp_lin3(const uint8_t* a32, const uint8_t* b32, const uint8_t* c32, uint8_t* out160) {
  uint32_t w[8];
  fp a, b, c, r[5];
  be32_to_words(w, a32);
  f_from_words(a, w);
  be32_to_words(w, b32);
  f_from_words(b, w);
  be32_to_words(w, c32);
  f_from_words(c, w);
  f_add(a, a, a);  // inputs up to 2q: a + a reduced
  fp_lin3<3, 0, 0, 0>(r[0], a, b, c);
  fp_lin3<1, -2, 0, 4>(r[1], a, b, c);
  fp_lin3<2, -2, -2, 8>(r[2], a, b, c);
  fp_lin3<1, -4, 0, 8>(r[3], a, b, c);
  fp_lin3<1, -1, -1, 4>(r[4], a, b, c);
  int ok = 1;
  for (int k = 0; k < 5; k++) {
    if (!fp_reduced(r[k])) ok = 0;
    f_to_words(w, r[k]);
    words_to_be32(out160 + 32 * k, w);
  }
  return ok;
}

int shim_g1_decompress(const uint8_t* in33, uint8_t* out64) {
  g1a a;
  if (!g1_decompress(a, in33)) return 0;
  uint32_t w[8];
  f_to_words(w, a.x);
  words_to_be32(out64, w);
  f_to_words(w, a.y);
  words_to_be32(out64 + 32, w);
  return a.inf ? 2 : 1;
}

void shim_g1_mul(const uint8_t* in33, const uint8_t* kbe, uint8_t* out33) {
  g1a a;
  g1_decompress(a, in33);
  g1j p, r;
  g1_from_affine(p, a);
  uint32_t k[8];
  be32_to_words(k, kbe);
  g1_mul(r, p, k);
  g1a o;
  g1_to_affine(o, r);
  g1_compress(out33, o);
}

// the constant-sequence ladders (g1_mul_ct / g2_mul_ct, used for secret scalars on the GPU)
void shim_g1_mul_ct(const uint8_t* in33, const uint8_t* kbe, uint8_t* out33) {
  g1a a;
  g1_decompress(a, in33);
  g1j p, r;
  g1_from_affine(p, a);
  uint32_t k[8];
  be32_to_words(k, kbe);
  g1_mul_ct(r, p, k);
  g1a o;
  g1_to_affine(o, r);
  g1_compress(out33, o);
}

void shim_g2_mul_gen_ct(const uint8_t* skbe, uint8_t* out65) {
  uint32_t k[8];
  be32_to_words(k, skbe);
  g2j P, acc;
  fp2_load(P.X, Bn254Consts::G2X);
  fp2_load(P.Y, Bn254Consts::G2Y);
  fp2_one(P.Z);
  g2_mul_ct(acc, P, k);
  g2a a;
  g2_to_affine(a, acc);
  g2_compress(out65, a);
}

// Row-parallel Fp (bn254_row.h) over the host SIMD emulation: random chains of rf_mul / rf_add /
// rf_sub in the four rows of a wave against f_mul / f_add / f_sub on one-lane elements.  Returns
// the number of mismatches (0 = pass); edge operands (0, 1, q-1, 2q-1 and limbs at 2^29 + 8)
// included.
static HU row_of4(const fp* x) {
  HU r;
  for (int row = 0; row < 4; row++)
    for (int i = 0; i < BN_LIMBS; i++) r.x[16 * row + i] = x[row].v[i];
  return r;
}
static void fe_of_row(fp& r, const HU& x, int row) {  // normalise row `row` into a one-lane element
  uint64_t c = 0;
  for (int i = 0; i < BN_LIMBS; i++) {
    const uint64_t t = (uint64_t)x.x[16 * row + i] + c;
    r.v[i] = i == BN_LIMBS - 1 ? (uint32_t)t : (uint32_t)(t & BN_MASK);
    c = t >> 29;
  }
  for (int i = 9; i < 16; i++)
    if (x.x[16 * row + i]) r.v[0] = 0xFFFFFFFFu;  // lanes 9..15 must stay zero
}
static bool fe_same(const fp& a, const fp& b) {  // equal mod q
  uint32_t wa[8], wb[8];
  f_to_words(wa, a);
  f_to_words(wb, b);
  for (int i = 0; i < 8; i++)
    if (wa[i] != wb[i]) return false;
  return true;
}
int shim_rf_check(uint64_t seed, int iters) {
  std::mt19937_64 g(seed);
  auto rnd = [&](fp& x) {
    uint32_t w[8];
    for (int i = 0; i < 8; i++) w[i] = (uint32_t)g();
    w[7] &= 0x1FFFFFFF;
    f_from_words(x, w);  // Montgomery form of a value < 2^253 (< q)
  };
  HU tag;
  const HU qrow = rf_row_const(FpParams::Q, tag), q8r = rf_row_const(RfConsts::Q8R, tag);
  fp a[4], b[4];
  for (int r = 0; r < 4; r++) {
    rnd(a[r]);
    rnd(b[r]);
  }
  f_zero(a[1]);                                    // 0
  f_one(b[2]);                                     // 1 (Montgomery)
  for (int i = 0; i < BN_LIMBS; i++) a[3].v[i] = FpParams::Q[i];  // q (= 0), unreduced operand
  HU ra = row_of4(a), rb = row_of4(b);
  int bad = 0;
  for (int it = 0; it < iters; it++) {
    const int op = it % 4;
    HU rr;
    fp e[4];
    if (op == 0 || op == 3) {
      rr = rf_mul<HU, HW>(ra, rb, qrow);
      for (int r = 0; r < 4; r++) f_mul(e[r], a[r], b[r]);
    } else if (op == 1) {
      // a + b with a, b < 2q: a row-normal value < 4q
      rr = rf_add(ra, rb);
      for (int r = 0; r < 4; r++) f_add(e[r], a[r], b[r]);
    } else {
      rr = rf_sub(ra, rb, q8r);
      for (int r = 0; r < 4; r++) f_sub(e[r], a[r], b[r]);
    }
    for (int r = 0; r < 4; r++) {
      fp got;
      fe_of_row(got, rr, r);
      if (!fe_same(got, e[r])) bad++;
      for (int l = 0; l < 16; l++)
        if (l < 9 ? rr.x[16 * r + l] > (1u << 29) + 8 : rr.x[16 * r + l] != 0) bad++;
    }
    // next operands: the row results (reduced below 2q by a multiplication so the bounds hold)
    if (op == 0 || op == 3) {
      ra = rb;
      for (int r = 0; r < 4; r++) a[r] = b[r];
      rb = rr;
      for (int r = 0; r < 4; r++) b[r] = e[r];
    } else {
      const HU m = rf_mul<HU, HW>(rr, ra, qrow);
      for (int r = 0; r < 4; r++) f_mul(a[r], e[r], a[r]);
      ra = m;
    }
  }
  return bad;
}

// G1 row-parallel dbl / add (bn254_g1row.h) over the host emulation against g1_dbl / g1_add:
// random points (multiples of g1_map outputs) including p + p (the doubling branch) and
// p + (-p) (infinity).  Returns the number of mismatches.
static HU row_all(const fp& x) {
  HU r;
  for (int row = 0; row < 4; row++)
    for (int i = 0; i < BN_LIMBS; i++) r.x[16 * row + i] = x.v[i];
  return r;
}
static bool rows_consistent(const HU& x) {  // every row holds the same element, lanes 9..15 zero
  for (int row = 1; row < 4; row++)
    for (int i = 0; i < 16; i++)
      if (x.x[16 * row + i] != x.x[i]) return false;
  for (int i = 9; i < 16; i++)
    if (x.x[i]) return false;
  return true;
}
static void g1j_of_row(g1j& r, const G1R<HU>& p) {
  fe_of_row(r.X, p.X, 0);
  fe_of_row(r.Y, p.Y, 0);
  fe_of_row(r.Z, p.Z, 0);
  const fp one = [] { fp o; f_one(o); return o; }();
  f_mul(r.X, r.X, one);  // values < 4q -> < 2q (reduced, as the one-lane code expects)
  f_mul(r.Y, r.Y, one);
  f_mul(r.Z, r.Z, one);
}
static bool same_point(const g1j& a, const g1j& b) {
  g1a x, y;
  g1_to_affine(x, a);
  g1_to_affine(y, b);
  uint8_t ba[33], bb[33];
  g1_compress(ba, x);
  g1_compress(bb, y);
  return std::memcmp(ba, bb, 33) == 0;
}
int shim_g1r_check(uint64_t seed, int iters) {
  std::mt19937_64 g(seed);
  HU tag;
  const RowCtx<HU, HW> c(tag);
  int bad = 0;
  for (int it = 0; it < iters; it++) {
    uint8_t msg[8];
    for (auto& m : msg) m = (uint8_t)g();
    g1a h;
    g1_map(h, msg, 8);
    g1j P, Q;
    g1_from_affine(P, h);
    uint32_t k[8] = {(uint32_t)g(), (uint32_t)g(), (uint32_t)g(), 0, 0, 0, 0, 0};
    g1_mul(Q, P, k);  // a Jacobian Z != 1
    const int kind = it % 5;
    if (kind == 3) Q = P;                      // doubling branch
    if (kind == 4) {                           // -P: infinity
      Q = P;
      f_neg(Q.Y, P.Y);
    }
    G1R<HU> rp{row_all(P.X), row_all(P.Y), row_all(P.Z)}, rq{row_all(Q.X), row_all(Q.Y), row_all(Q.Z)}, rr;
    // doubling
    g1r_dbl(rr, rq, c);
    g1j e, got;
    g1_dbl(e, Q);
    g1j_of_row(got, rr);
    if (!same_point(got, e) || !rows_consistent(rr.X) || !rows_consistent(rr.Y) || !rows_consistent(rr.Z)) bad++;
    // addition (and a chain: the doubled point added to p)
    const G1rAddResult res = g1r_add(rr, rp, rq, c);
    g1_add(e, P, Q);
    if (kind == 4) {
      if (res != G1R_INF || !g1_is_inf(e)) bad++;
      continue;
    }
    g1j_of_row(got, rr);
    if (res != G1R_SUM || !same_point(got, e) || !rows_consistent(rr.X)) bad++;
    G1R<HU> r2;
    g1r_add(r2, rr, rp, c);
    g1j e2;
    g1_add(e2, e, P);
    g1j_of_row(got, r2);
    if (!same_point(got, e2)) bad++;
    G1R<HU> rn;
    g1r_neg(rn, rp, c);
    g1j n = P;
    f_neg(n.Y, P.Y);
    g1j_of_row(got, rn);
    if (!same_point(got, n)) bad++;
  }
  return bad;
}

// G2 row-parallel arithmetic (bn254_g2row.h) over the host emulation against the one-lane G2
// code: g2r_dbl<LINE> vs line_dbl_j / g2_dbl_j, g2r_madd<LINE> vs line_add_j / g2_add_j_body,
// g2r_add vs g2_add_j_body (incl. T + T and T + (-T)), g2r_accum chains, and g2r_in_subgroup
// vs g2_in_subgroup on points of G2 and off it.  Lines compared as field values (A, B, C), points
// projectively.  Returns the mismatches plus every rf_mul bound violation seen.
static F2R<HU> f2r_of(const fp2& x) { return {row_all(x.a), row_all(x.b)}; }
static void fp2_of_row(fp2& r, const F2R<HU>& x) {
  const fp one = [] { fp o; f_one(o); return o; }();
  fe_of_row(r.a, x.a, 0);
  fe_of_row(r.b, x.b, 0);
  f_mul(r.a, r.a, one);  // value < 4q -> < 2q
  f_mul(r.b, r.b, one);
}
static G2R<HU> g2r_of(const g2j& p) { return {f2r_of(p.X), f2r_of(p.Y), f2r_of(p.Z)}; }
static void g2j_of_row(g2j& r, const G2R<HU>& p) {
  fp2_of_row(r.X, p.X);
  fp2_of_row(r.Y, p.Y);
  fp2_of_row(r.Z, p.Z);
}
static bool fp2_same(const fp2& a, const fp2& b) { return fe_same(a.a, b.a) && fe_same(a.b, b.b); }
static bool f2r_consistent(const F2R<HU>& x) { return rows_consistent(x.a) && rows_consistent(x.b); }
static bool g2_same(const g2j& a, const g2j& b) {
  g2a x, y;
  g2_to_affine(x, a);
  g2_to_affine(y, b);
  uint8_t ba[65], bb[65];
  g2_compress(ba, x);
  g2_compress(bb, y);
  return std::memcmp(ba, bb, 65) == 0;
}
static bool line_same(const F2R<HU>* l, const uint32_t* ln, const uint32_t* sa) {
  fp2 A, B, C, eA, eB, eC;
  fp2_of_row(A, l[0]);
  fp2_of_row(B, l[1]);
  fp2_of_row(C, l[2]);
  fp2_fetch(eA, sa);
  fp2_fetch(eB, ln);
  fp2_fetch(eC, ln + 18);
  return fp2_same(A, eA) && fp2_same(B, eB) && fp2_same(C, eC) && f2r_consistent(l[0]) && f2r_consistent(l[1]) &&
         f2r_consistent(l[2]);
}
int shim_g2r_check(uint64_t seed, int iters) {
  std::mt19937_64 g(seed);
  HU tag;
  const G2RowCtx<HU, HW> c(tag);
  g_rf_bound_violations = 0;
  int bad = 0;
  g2j G;
  fp2_load(G.X, Bn254Consts::G2X);
  fp2_load(G.Y, Bn254Consts::G2Y);
  fp2_one(G.Z);
  for (int it = 0; it < iters; it++) {
    uint32_t k[8] = {(uint32_t)g(), (uint32_t)g(), (uint32_t)g(), (uint32_t)g(), 0, 0, 0, 0};
    g2j P, Q;
    g2_mul_ct(P, G, k);  // Jacobian, Z != 1
    k[0] ^= 0x5a5a;
    g2_mul_ct(Q, G, k);
    g2a qa;
    g2_to_affine(qa, Q);
    // doubling with / without the line
    {
      g2j T = P, e = P;
      uint32_t ln[36], sa[36];
      line_dbl_j(ln, sa, e);
      G2R<HU> rt = g2r_of(T);
      F2R<HU> l[3];
      g2r_dbl<true>(l, rt, c);
      g2j got;
      g2j_of_row(got, rt);
      if (!g2_same(got, e) || !line_same(l, ln, sa) || !f2r_consistent(rt.X) || !f2r_consistent(rt.Y) ||
          !f2r_consistent(rt.Z))
        bad++;
      G2R<HU> r2 = g2r_of(T);
      g2r_dbl<false>((F2R<HU>*)nullptr, r2, c);
      g2j_of_row(got, r2);
      g2j e2;
      g2_dbl_j(e2, T);
      if (!g2_same(got, e2)) bad++;
    }
    // mixed addition with / without the line
    {
      g2j e = P;
      uint32_t ln[36], sa[36];
      line_add_j(ln, sa, e, qa.x, qa.y);
      G2R<HU> rt = g2r_of(P);
      F2R<HU> l[3];
      bool same = false;
      g2r_madd<true>(l, rt, f2r_of(qa.x), f2r_of(qa.y), c, same);
      g2j got;
      g2j_of_row(got, rt);
      if (!g2_same(got, e) || !line_same(l, ln, sa)) bad++;
      G2R<HU> r2 = g2r_of(P);
      if (!g2r_madd<false>((F2R<HU>*)nullptr, r2, f2r_of(qa.x), f2r_of(qa.y), c, same)) bad++;
      g2j_of_row(got, r2);
      if (!g2_same(got, e)) bad++;
    }
    // full addition, and its exceptional cases
    {
      G2R<HU> rt = g2r_of(P);
      bool same = false;
      if (!g2r_add(rt, g2r_of(Q), c, same)) bad++;
      g2j e, got;
      g2_add_j(e, P, Q);
      g2j_of_row(got, rt);
      if (!g2_same(got, e)) bad++;
      // both affine (Z = 1): the key sum's first additions
      g2a pa;
      g2_to_affine(pa, P);
      g2j Pa{pa.x, pa.y, G.Z}, Qa{qa.x, qa.y, G.Z};
      G2R<HU> ra = g2r_of(Pa);
      if (!g2r_add(ra, g2r_of(Qa), c, same)) bad++;
      g2j_of_row(got, ra);
      if (!g2_same(got, e)) bad++;
      g2j P2;  // P in another Jacobian representation
      g2_add_j(P2, P, G);
      g2j nG = G;
      fp2_neg(nG.Y, G.Y);
      g2_add_j(P2, P2, nG);
      G2R<HU> a = g2r_of(P);
      if (g2r_add(a, g2r_of(P2), c, same) || !same) bad++;  // P + P: the doubling case
      g2j nP = P2;
      fp2_neg(nP.Y, P2.Y);
      G2R<HU> b = g2r_of(P);
      if (g2r_add(b, g2r_of(nP), c, same) || same) bad++;  // P + (-P): infinity
      // accumulate chains with the flags: P + P + (-2P) + Q == Q
      G2R<HU> acc{};
      bool inf = true;
      g2r_accum(acc, inf, g2r_of(P), false, c);
      g2r_accum(acc, inf, g2r_of(P2), false, c);
      g2j m2;
      g2_dbl_j(m2, P);
      fp2_neg(m2.Y, m2.Y);
      g2r_accum(acc, inf, g2r_of(m2), false, c);
      if (!inf) bad++;
      g2r_accum_aff(acc, inf, f2r_of(qa.x), f2r_of(qa.y), c);
      g2j_of_row(got, acc);
      if (inf || !g2_same(got, Q)) bad++;
    }
    // subgroup membership: a point of G2, and (every 4th iteration) a twist point off it
    if (it % 4 == 0) {
      g2a pa;
      g2_to_affine(pa, P);
      if (!g2r_in_subgroup(f2r_of(pa.x), f2r_of(pa.y), c)) bad++;
      uint8_t enc[65] = {0x02};
      for (uint32_t x = 1 + (uint32_t)(g() & 0xffff);; x++) {
        enc[64] = (uint8_t)x;
        enc[63] = (uint8_t)(x >> 8);
        enc[62] = (uint8_t)(x >> 16);
        enc[32] = 1;
        g2a t;
        if (!g2_decode_on_curve(t, enc)) continue;
        if (g2r_in_subgroup(f2r_of(t.x), f2r_of(t.y), c) != g2_in_subgroup(t)) bad++;
        break;
      }
    }
  }
  return bad + (int)g_rf_bound_violations;
}

// g2r_in_subgroup (the psi(Q) = [6u^2]Q test) against r Q == O on twist points multiplied by
// k1 then k2 (8 LE words each; e.g. r and h2 / ell land in the cofactor's order-ell subgroup, h2
// and 1 in G2): returns mismatches, *tested = points that were not infinity.
int shim_g2r_subgroup_scaled(uint64_t seed, int n, const uint32_t* k1, const uint32_t* k2, int* tested) {
  std::mt19937_64 g(seed);
  HU tag;
  const G2RowCtx<HU, HW> c(tag);
  int bad = 0;
  *tested = 0;
  for (int it = 0; it < n; it++) {
    uint8_t enc[65] = {0x02};
    for (uint32_t x = 1 + (uint32_t)(g() & 0xffffff);; x++) {
      enc[64] = (uint8_t)x;
      enc[63] = (uint8_t)(x >> 8);
      enc[62] = (uint8_t)(x >> 16);
      enc[32] = (uint8_t)(1 + (g() & 7));
      g2a t;
      if (!g2_decode_on_curve(t, enc)) continue;
      g2j p, q;
      p.X = t.x;
      p.Y = t.y;
      fp2_one(p.Z);
      g2_mul_ct(q, p, k1);
      g2_mul_ct(p, q, k2);
      g2a a;
      g2_to_affine(a, p);
      if (!a.inf) {
        ++*tested;
        if (g2r_in_subgroup(f2r_of(a.x), f2r_of(a.y), c) != g2_in_subgroup(a)) bad++;
      }
      break;
    }
  }
  return bad + (int)g_rf_bound_violations;
}

// the key-sum kernel's flow (bls_g2_sum_row_kernel) on the host emulation: waves of 8 ids each
// (mixed additions from affine keys), then a pairwise tree through one-lane words (the LDS
// exchange) -> compressed; 1 iff equal to the one-lane g2_add_j sum of the same keys
int shim_g2r_sum_check(uint64_t seed, int nkeys, int stride) {
  std::mt19937_64 g(seed);
  HU tag;
  const G2RowCtx<HU, HW> c(tag);
  g2j G;
  fp2_load(G.X, Bn254Consts::G2X);
  fp2_load(G.Y, Bn254Consts::G2Y);
  fp2_one(G.Z);
  std::vector<g2a> keys(nkeys);
  g2j ref;
  fp2_one(ref.X);
  fp2_one(ref.Y);
  fp2_zero(ref.Z);
  for (int i = 0; i < nkeys; i++) {
    uint32_t k[8] = {(uint32_t)g(), (uint32_t)g(), 0, 0, 0, 0, 0, 0};
    g2j P;
    g2_mul_ct(P, G, k);
    g2_to_affine(keys[i], P);
    if (i % stride == 0) {
      g2j t;
      t.X = keys[i].x;
      t.Y = keys[i].y;
      fp2_one(t.Z);
      g2_add_j(ref, ref, t);
    }
  }
  const int W = (nkeys + 7) / 8;
  std::vector<G2R<HU>> acc(W);
  std::unique_ptr<bool[]> inf(new bool[W]);
  for (int w = 0; w < W; w++) inf[w] = true;
  for (int w = 0; w < W; w++)
    for (int i = 8 * w; i < 8 * w + 8 && i < nkeys; i++)
      if (i % stride == 0) g2r_accum_aff(acc[w], inf[w], f2r_of(keys[i].x), f2r_of(keys[i].y), c);
  for (int st = 1; st < W; st *= 2)
    for (int w = 0; w + st < W; w += 2 * st) {
      // the LDS round trip: normalised one-lane words back into rows
      g2j o;
      g2j_of_row(o, acc[w + st]);
      g2r_accum(acc[w], inf[w], g2r_of(o), inf[w + st], c);
    }
  g2j got;
  g2j_of_row(got, acc[0]);
  if (inf[0]) fp2_zero(got.Z);
  g2a a, b;
  g2_to_affine(a, got);
  g2_to_affine(b, ref);
  uint8_t ea[65], eb[65];
  g2_compress(ea, a);
  g2_compress(eb, b);
  return std::memcmp(ea, eb, 65) == 0 && g_rf_bound_violations == 0;
}

// G + 2G through g2r_add on the host emulation, compressed (debug aid)
void shim_g2r_3g(uint8_t* out65) {
  HU tag;
  const G2RowCtx<HU, HW> c(tag);
  g2j G, Q2;
  fp2_load(G.X, Bn254Consts::G2X);
  fp2_load(G.Y, Bn254Consts::G2Y);
  fp2_one(G.Z);
  g2_dbl_j(Q2, G);
  g2a qa;
  g2_to_affine(qa, Q2);
  g2j Qa{qa.x, qa.y, G.Z};
  G2R<HU> t = g2r_of(G);
  bool sy = false;
  g2r_add(t, g2r_of(Qa), c, sy);
  g2j r;
  g2j_of_row(r, t);
  g2a a;
  g2_to_affine(a, r);
  g2_compress(out65, a);
}

int shim_g2_decompress(const uint8_t* in65, uint8_t* out65) {
  g2a q;
  if (!g2_decompress(q, in65)) return 0;
  g2_compress(out65, q);
  return 1;
}

// 1 iff the inversion-free, batch-normalised line precomputation equals the affine one word for
// word (both kernels' formats), 0 if they differ, -1 if the key does not decode
int shim_lines_match(const uint8_t* in65) {
  g2a q;
  if (!g2_decompress(q, in65) || q.inf) return -1;
  std::vector<uint32_t> a(BN_ATE_LINES * BN_LINE_WORDS), b(a.size()), scr(BN_ATE_LINES * 36);
  g2_precompute_lines(a.data(), q);
  g2_precompute_lines_batch(b.data(), q, scr.data());
  // compare the field elements canonically (limbs hold a value < 2p: either representative)
  for (size_t e = 0; e < a.size(); e += 9) {
    fp x, y;
    for (int i = 0; i < 9; i++) {
      x.v[i] = a[e + i];
      y.v[i] = b[e + i];
    }
    uint32_t wx[8], wy[8];
    f_to_words(wx, x);
    f_to_words(wy, y);
    for (int i = 0; i < 8; i++)
      if (wx[i] != wy[i]) return 0;
  }
  return 1;
}

void shim_g1_map(const uint8_t* msg, uint32_t len, uint8_t* out33) {
  g1a h;
  g1_map(h, msg, len);
  g1_compress(out33, h);
}

// full pairing value e(P, Q) in the oracle's flat Fp12 basis (12 x 32 bytes)
int shim_pairing(const uint8_t* p33, const uint8_t* q65, uint8_t* out384) {
  g1a P;
  g2a Q;
  if (!g1_decompress(P, p33) || !g2_decompress(Q, q65)) return 0;
  std::vector<uint32_t> lines(BN_ATE_LINES * BN_LINE_WORDS);
  g2_precompute_lines(lines.data(), Q);
  const uint32_t* l[1] = {lines.data()};
  fp12 f, e;
  miller_multi<1>(f, &P, l);
  final_exp(e, f);
  fp12_flat(out384, e);
  return 1;
}

// e(P1, Q1) * e(P2, Q2) == 1 ?
int shim_pairing_check2(const uint8_t* p1, const uint8_t* q1, const uint8_t* p2, const uint8_t* q2) {
  g1a P[2];
  g2a Q[2];
  if (!g1_decompress(P[0], p1) || !g1_decompress(P[1], p2) || !g2_decompress(Q[0], q1) ||
      !g2_decompress(Q[1], q2))
    return -1;
  std::vector<uint32_t> l0(BN_ATE_LINES * BN_LINE_WORDS), l1(BN_ATE_LINES * BN_LINE_WORDS);
  g2_precompute_lines(l0.data(), Q[0]);
  g2_precompute_lines(l1.data(), Q[1]);
  const uint32_t* l[2] = {l0.data(), l1.data()};
  return pairing_check<2>(P, l) ? 1 : 0;
}

// vk = sk * g2 (65 bytes), sk big-endian 32 bytes
void shim_g2_mul_gen(const uint8_t* skbe, uint8_t* out65) {
  uint32_t k[8];
  be32_to_words(k, skbe);
  g2j P, acc;
  fp2_load(P.X, Bn254Consts::G2X);
  fp2_load(P.Y, Bn254Consts::G2Y);
  fp2_one(P.Z);
  fp2_one(acc.X);
  fp2_one(acc.Y);
  fp2_zero(acc.Z);
  for (int i = 255; i >= 0; i--) {
    g2_dbl_j(acc, acc);
    if ((k[i >> 5] >> (i & 31)) & 1) g2_add_j(acc, acc, P);
  }
  g2a a;
  g2_to_affine(a, acc);
  g2_compress(out65, a);
}

// BlsThresholdSigner::signData: id (4 B big-endian) || sk * g1_map(msg)
void shim_sign_share(const uint8_t* skbe, uint32_t id, const uint8_t* msg, uint32_t len, uint8_t* out37) {
  g1a h;
  g1_map(h, msg, len);
  g1j p, r;
  g1_from_affine(p, h);
  uint32_t k[8];
  be32_to_words(k, skbe);
  g1_mul(r, p, k);
  g1a a;
  g1_to_affine(a, r);
  out37[0] = (uint8_t)(id >> 24);
  out37[1] = (uint8_t)(id >> 16);
  out37[2] = (uint8_t)(id >> 8);
  out37[3] = (uint8_t)id;
  g1_compress(out37 + 4, a);
}

// many shares / keys on host threads (test-set generation)
void shim_sign_shares_mt(const uint8_t* sks, const uint32_t* ids, uint32_t k, const uint8_t* msg, uint32_t len,
                         uint8_t* out, int threads) {
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++)
    th.emplace_back([=] {
      for (uint32_t j = t; j < k; j += threads) shim_sign_share(sks + 32 * j, ids[j], msg, len, out + 37 * j);
    });
  for (auto& x : th) x.join();
}
// CPU baseline of share verification (labelled "not RELIC"): per share, decompress, G2 line
// precomputation for vk_id (as RELIC's pc_map recomputes the G2 side every call) and the
// 2-pairing check e(H, vk) e(-sigma, g2) == 1, shares split over host threads.
void shim_verify_shares_mt(const uint8_t* h33, const uint8_t* vks65, uint32_t n, const uint8_t* shares37,
                           uint32_t k, uint8_t* out, int threads) {
  g1a H;
  g1_decompress(H, h33);
  g2a G;
  fp2_load(G.x, Bn254Consts::G2X);
  fp2_load(G.y, Bn254Consts::G2Y);
  G.inf = false;
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++)
    th.emplace_back([=] {
      std::vector<uint32_t> l0(BN_ATE_LINES * BN_LINE_WORDS), l1(BN_ATE_LINES * BN_LINE_WORDS);
      for (uint32_t j = t; j < k; j += threads) {
        uint32_t id;
        g1a P[2];
        g2a Q;
        bool ok = bls_parse_share(id, P[1], shares37 + 37 * (size_t)j) && id >= 1 && id <= n &&
                  g2_decompress(Q, vks65 + 65 * (size_t)(id - 1)) && !Q.inf;
        if (ok) {
          P[0] = H;
          g2_precompute_lines(l0.data(), Q);
          g2_precompute_lines(l1.data(), G);
          const uint32_t* l[2] = {l0.data(), l1.data()};
          if (P[1].inf) {
            ok = pairing_check<1>(P, l);
          } else {
            f_neg(P[1].y, P[1].y);
            ok = pairing_check<2>(P, l);
          }
        }
        out[j] = ok ? 1 : 0;
      }
    });
  for (auto& x : th) x.join();
}

void shim_g2_mul_gen_mt(const uint8_t* sks, uint32_t n, uint8_t* out, int threads) {
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++)
    th.emplace_back([=] {
      for (uint32_t j = t; j < n; j += threads) shim_g2_mul_gen(sks + 32 * j, out + 65 * j);
    });
  for (auto& x : th) x.join();
}

}  // extern "C"
