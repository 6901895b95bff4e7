// Lazy-reduction lane arithmetic of the cyclotomic squaring on the pair36 layout
// (bn254_pair36.h: p36_cyc_sqr).  Host + device: tests/cpp/bn254_shim.cpp runs the same stage
// functions on the CPU over an emulated 36-lane wave and checks them against fp12_sqr.
//
// A final exponentiation is one wave issuing one dependent instruction stream (a lone wave on
// gfx950: ~6 cycles per VALU instruction, 10.6 per v_mad_u64_u32, profiles/r02_intrate2.txt), so
// its cost is the instruction count per lane.  The reduced form (f_add / f_sub: a carry pass, a
// reduction decision and a branch each) cost ~14 x 45 instructions per squaring against ~210 for
// the one Fp multiplication.  Here the squaring carries unreduced values between its gathers
// (sums of a few reduced values, limbs kept non-negative by redundant representations of
// multiples of q) and reduces ONCE, at the end (fp_reduce64: the multiple of q estimated from the
// top limb, subtracted with 24-bit products).  Every bound is stated at the function.
#pragma once
#include "bn254_pairing.h"  // g1j (the lazy G1 doubling); bn254_field.h for the rest

// ---- constants: k q as limbs, and redundant forms of k q with every low limb >= L ----------
struct CsLimbs {
  uint32_t v[BN_LIMBS];
};

// k q normalised (limbs 0..7 < 2^29)
constexpr CsLimbs cs_kq(uint32_t k) {
  CsLimbs r{};
  uint64_t c = 0;
  for (int i = 0; i < BN_LIMBS; i++) {
    const uint64_t x = (uint64_t)k * FpParams::Q[i] + c;
    r.v[i] = i < BN_LIMBS - 1 ? (uint32_t)(x & BN_MASK) : (uint32_t)x;
    c = x >> 29;
  }
  return r;
}

// the same value (k q, or 0 for k = 0) with limbs 0..7 in [L, L + 2^29) and the rest (signed)
// in the top limb: added to a limb-wise difference it keeps every low limb non-negative
constexpr CsLimbs cs_redundant(uint32_t k, int64_t L) {
  const CsLimbs n = cs_kq(k);
  CsLimbs r{};
  int64_t b = 0;  // borrowed from this limb (in units of its weight)
  for (int i = 0; i < BN_LIMBS - 1; i++) {
    const int64_t cur = (int64_t)n.v[i] - b;
    int64_t d = (cur - L) % (int64_t)(1 << 29);
    if (d < 0) d += (int64_t)1 << 29;
    const int64_t di = L + d;
    r.v[i] = (uint32_t)di;
    b = (di - cur) >> 29;
  }
  r.v[BN_LIMBS - 1] = (uint32_t)(int32_t)((int64_t)n.v[BN_LIMBS - 1] - b);
  return r;
}

struct CsConst {
  static constexpr CsLimbs Q4R = cs_redundant(4, (1 << 30) - 2);   // cs_operands: Wm - Wo + 4q
  static constexpr CsLimbs Z3 = cs_redundant(0, 3 << 29);          // cs_combine: +-(X2 + Y2) +- G3
  static constexpr CsLimbs Z4 = cs_redundant(0, 1 << 29);          // cs_finish: v +- vo
  static constexpr CsLimbs D28M = cs_redundant(28, (1 << 30) - 2);  // cs_finish: 3w - 2a + 28q
  static constexpr CsLimbs D28P = cs_kq(28);                        // cs_finish: 3w + 2a + 28q
  // floor(2^32 / (Q8 + 1)): m = umulhi(x8, MINV) estimates floor(x / q) from the top limb
  static constexpr uint32_t MINV = (uint32_t)((1ull << 32) / (FpParams::Q[BN_LIMBS - 1] + 1));
};

constexpr int cs_ctz(uint32_t x) {
  int n = 0;
  while (!(x & 1u)) {
    x >>= 1;
    n++;
  }
  return n;
}
constexpr int cs_bitlen(uint32_t x) {
  int n = 0;
  while (x) {
    x >>= 1;
    n++;
  }
  return n;
}

// ---- lane-role selects ----------------------------------------------------------------------
// A lane condition (h, diag, s == 2, ...) as an all-ones / zero mask that LLVM cannot see through:
// with the plain ternaries it merged the limb-wise selects of one condition into ONE divergent
// branch around both limb loops (exec-mask save / restore, both sides issued anyway: ~40 % of the
// p36_sqr operand code); with an opaque mask every select is one v_bfi_b32.
BN_HD uint32_t cs_mask(bool c) {
  uint32_t m = c ? ~0u : 0u;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(m));
#endif
  return m;
}
BN_HD uint32_t cs_sel(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }  // m ? a : b

// ---- carry passes -------------------------------------------------------------------------
// limbs 0..7 non-negative (as uint32, any size): -> [0, 2^29), carries into the top limb
// (two's complement, so a signed top limb stays signed).  Sequential, 3 instructions a limb.
BN_HD void cs_carry(fp& x) {
#pragma unroll
  for (int i = 0; i < BN_LIMBS - 1; i++) {
    x.v[i + 1] += x.v[i] >> 29;
    x.v[i] &= BN_MASK;
  }
}
// limbs 0..7 signed (|x_i| < 2^31): the same with arithmetic shifts
BN_HD void cs_carry_s(fp& x) {
#pragma unroll
  for (int i = 0; i < BN_LIMBS - 1; i++) {
    x.v[i + 1] += (uint32_t)((int32_t)x.v[i] >> 29);
    x.v[i] &= BN_MASK;
  }
}

// ---- the single reduction -------------------------------------------------------------------
// r = x mod q, r < 2q and normalised, for 0 <= x < 64 q given with limbs 0..7 in [0, 2^29 + 8)
// (the top limb then within 1 of floor(x / 2^232) from below).
//   m = umulhi(x8, MINV) satisfies floor(x/q) - 1 <= m <= floor(x/q): m <= x8 / (Q8 + 1) <= x/q,
//   and x8 MINV / 2^32 > x8 / (Q8 + 1) - 2^-4 > x/q - 2^-4 - 66 / (Q8 + 1)  (x8 < 2^28).
// m q is subtracted limb by limb: Q_i = s_i 2^sh_i with s_i < 2^22, so every m s_i (m < 64) is
// one 24-bit product, placed as (m s_i << sh_i) & mask into limb i and m s_i >> (29 - sh_i)
// into limb i + 1.  One signed carry pass normalises (x - m q in [0, 2q)).
BN_HD void fp_reduce64(fp& r, fp& x) {
  const uint32_t x8 = x.v[BN_LIMBS - 1];
  const uint32_t m = (uint32_t)(((uint64_t)x8 * CsConst::MINV) >> 32) & 63u;
#pragma unroll
  for (int i = 0; i < BN_LIMBS - 1; i++) {
    const int sh = cs_ctz(FpParams::Q[i]);
    const uint32_t s = FpParams::Q[i] >> sh;
    const uint32_t p = m * s;  // < 2^28
    if (sh == 0) {
      x.v[i] -= p;  // s < 2^23 here: m s < 2^29, no spill into limb i + 1
    } else {
      x.v[i] -= (p << sh) & BN_MASK;
      if (cs_bitlen(s) + 6 + sh > 29) x.v[i + 1] -= p >> (29 - sh);
    }
  }
  x.v[BN_LIMBS - 1] -= m * FpParams::Q[BN_LIMBS - 1];
  cs_carry_s(x);
  r = x;
}

// ---- the four lane stages of p36_cyc_sqr -------------------------------------------------
// Lane (k, h, s) of the pair36 layout; a = its component of the input (reduced, < 2q).
// Granger-Scott: for (x, y) = (e_sx, e_sx+3), sub-lane s squares w = x | y | x + y (s = 0, 1, 2);
// the component h of e_k^2-part then combines x^2, y^2, (x + y)^2 (bn254_pair12.h: p12_cyc_sqr).

// stage 1 (source side): R = a, plus a_{k+3} (t, gathered from coefficient k + 3) on sub-lane 2,
// so one gather per component gives w: x from (sx, h, 0), y from (sx + 3, h, 1), x + y from
// (sx, h, 2).  Limbs < 2^30, value < 4q.
BN_HD void cs_pre(fp& R, const fp& a, const fp& t, int s) {
  const uint32_t msk = s == 2 ? ~0u : 0u;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) R.v[i] = a.v[i] + (t.v[i] & msk);
}

// stage 2: the operands of the one multiplication from my (Wm) and the other (Wo) component of w:
//   h = 0: (Wm + Wo)(Wm - Wo) = w_0^2 - w_1^2;  h = 1: (2 Wm) Wo = 2 w_0 w_1.
// U stays raw (limbs < 2^31, value < 8q); V = Wm - Wo + 4q (h = 0; low limbs of Q4R >= 2^30 - 2
// >= Wo_i, so non-negative) or Wo (h = 1), then carried (value < 8q).  f_mul(U, V): product
// columns < 9 2^60 + 9 2^58 + 2^35 < 2^64, result T < 64 q^2 / 2^261 + q < 1.3 q, normalised.
BN_HD void cs_operands(fp& U, fp& V, const fp& Wm, const fp& Wo, int h) {
  const uint32_t mh = cs_mask(h != 0);
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
    U.v[i] = Wm.v[i] + cs_sel(mh, Wm.v[i], Wo.v[i]);
    V.v[i] = cs_sel(mh, Wo.v[i], Wm.v[i] - Wo.v[i] + CsConst::Q4R.v[i]);
  }
  cs_carry(V);
}

// stage 3: v = x^2 + xi y^2 (even k) or (x + y)^2 - x^2 - y^2 = 2xy (odd k), my component, from
// X2 = x^2_h, Y2 = y^2_h and G3 = y^2_h' (even k) | (x + y)^2_h (odd k), each < 1.3 q:
//   even, h = 0: X2 + Y2 - G3;  even, h = 1: X2 + Y2 + G3;  odd: G3 - X2 - Y2.
// Negation as (z ^ -1) + 1; Z3 (a redundant zero, low limbs >= 3 2^29) keeps the low limbs
// non-negative.  Carried: low limbs normalised, signed top, |v| < 3.9 q.
BN_HD void cs_combine(fp& v, const fp& X2, const fp& Y2, const fp& G3, int k, int h) {
  const bool odd = (k & 1) != 0;
  const uint32_t mP = odd ? ~0u : 0u;
  const uint32_t mG = (!odd && h == 0) ? ~0u : 0u;
  const uint32_t c = (mP & 1u) + (mG & 1u);
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) v.v[i] = ((X2.v[i] + Y2.v[i]) ^ mP) + (G3.v[i] ^ mG) + (CsConst::Z3.v[i] + c);
  cs_carry(v);
}

// stage 4: r = 3 v' + 2a (odd k) | 3 v' - 2a (even k), reduced below 2q, where v' = xi v for k = 1
// (xi = 1 + i: component 0 v_0 - v_1, component 1 v_0 + v_1; vo = the other component's v) and
// v' = v otherwise.  w = v' with Z4 (low limbs >= 2^29) is carried (|w| < 7.8 q); then
// 3w +- 2a + 28q has low limbs in [0, 3 2^30) (D28M's low limbs >= 2^30 - 2 >= 2a_i) and value in
// (0, 56 q): one carry pass and fp_reduce64.
BN_HD void cs_finish(fp& r, const fp& v, const fp& vo, const fp& a, int k, int h) {
  const uint32_t use = k == 1 ? ~0u : 0u;
  const uint32_t neg = (k == 1 && h == 0) ? ~0u : 0u;
  fp w;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) w.v[i] = v.v[i] + ((vo.v[i] & use) ^ neg) + (CsConst::Z4.v[i] + (neg & 1u));
  cs_carry(w);
  const bool odd = (k & 1) != 0;
  const uint32_t sa = odd ? 0u : ~0u;
  fp x;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
    const uint32_t d = (odd ? CsConst::D28P.v[i] : CsConst::D28M.v[i]) + (sa & 1u);
    x.v[i] = 3u * w.v[i] + ((a.v[i] << 1) ^ sa) + d;
  }
  cs_carry(x);
  fp_reduce64(r, x);
}

// ---- the lazy Fp12 multiplication (bn254_pair36.h: p36_mul) ------------------------------
// Lane (k, h, s) forms the terms i = 2s, 2s + 1 of c_k = sum_i a_i b_{k-i} (xi on wrap), each an
// Fp2 product's component h from two Fp multiplications (t1 = u b_m, t2 = v b_o, all < 1.02 q:
// inputs < 2q); the sums stay unreduced up to one reduction after the sub-lane sum.

struct CmConst {
  static constexpr CsLimbs Z2 = cs_redundant(0, 1 << 30);  // cm_terms: up to two negated terms
  static constexpr CsLimbs Z1 = cs_redundant(0, 1 << 29);  // cm_xi: one negated term
};

// stage 1: e_t = t1_t + t2_t (h = 1) | t1_t - t2_t (h = 0), summed into acc (no wrap) or accw (wrap).
// Low limbs of e in (-2^29, 2^30); Z2 keeps them >= 0, below 3.5 2^30; both carried.
BN_HD void cm_terms(fp& acc, fp& accw, const fp& t1a, const fp& t2a, const fp& t1b, const fp& t2b, int h, bool wa,
                    bool wb) {
  const uint32_t sg = h ? 0u : ~0u;
  const uint32_t ma = wa ? ~0u : 0u, mb = wb ? ~0u : 0u;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
    const uint32_t ea = t1a.v[i] + (t2a.v[i] ^ sg) + (sg & 1u);
    const uint32_t eb = t1b.v[i] + (t2b.v[i] ^ sg) + (sg & 1u);
    acc.v[i] = CmConst::Z2.v[i] + (ea & ~ma) + (eb & ~mb);
    accw.v[i] = CmConst::Z2.v[i] + (ea & ma) + (eb & mb);
  }
  cs_carry(acc);
  cs_carry(accw);
}

// stage 2: z = acc + xi accw, my component (xi = 1 + i: accw +- the other component's accw, ao)
BN_HD void cm_xi(fp& z, const fp& acc, const fp& accw, const fp& ao, int h) {
  const uint32_t sg = h ? 0u : ~0u;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) z.v[i] = acc.v[i] + accw.v[i] + (ao.v[i] ^ sg) + (CmConst::Z1.v[i] + (sg & 1u));
  cs_carry(z);
}

// stage 3: r = z_0 + z_1 + z_2 over the sub-lanes (|sum| < 24.5 q) + 28 q, reduced below 2q
BN_HD void cm_sum3(fp& r, const fp& z0, const fp& z1, const fp& z2) {
  fp x;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) x.v[i] = z0.v[i] + z1.v[i] + (z2.v[i] + CsConst::D28P.v[i]);
  cs_carry(x);
  fp_reduce64(r, x);
}

// ---- the lazy Fp12 squaring (bn254_pair36.h: p36_sqr) ------------------------------------
// Two multiplications per lane: diag (even k, s = 0) squares x = a_f1 and z = a_f2 (component h:
// (m + o)(m - o) for h = 0, (2m) o for h = 1); a cross lane forms 2 (x z)_h = (2u) z_m +- (2v) z_o
// (u = h ? x_o : x_m, v = h ? x_m : x_o).  The doublings ride in the raw left operands (limbs
// < 2^30, values < 4q); the right operands are carried (m - o + 2q: Q2R's low limbs >= 2^29).
// Products < 16 q^2 / 2^261 + q < 1.08 q.  The products then go through cm_terms (diag: x^2 term
// to acc, z^2 term to accw; cross: P1 +- P2 to acc or accw), cm_xi and cm_sum3 (sum < 26 q).
struct SqConst {
  static constexpr CsLimbs Q2R = cs_redundant(2, 1 << 29);
};
BN_HD void sq_operands(fp& U1, fp& V1, fp& U2, fp& V2, const fp& xm, const fp& xo, const fp& zm, const fp& zo,
                       bool diag, int h) {
  const uint32_t mh = cs_mask(h != 0), md = cs_mask(diag);
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
    const uint32_t du1 = xm.v[i] + cs_sel(mh, xm.v[i], xo.v[i]);
    const uint32_t dv1 = cs_sel(mh, xo.v[i], xm.v[i] - xo.v[i] + SqConst::Q2R.v[i]);
    const uint32_t du2 = zm.v[i] + cs_sel(mh, zm.v[i], zo.v[i]);
    const uint32_t dv2 = cs_sel(mh, zo.v[i], zm.v[i] - zo.v[i] + SqConst::Q2R.v[i]);
    const uint32_t cu1 = cs_sel(mh, xo.v[i], xm.v[i]) << 1;
    const uint32_t cu2 = cs_sel(mh, xm.v[i], xo.v[i]) << 1;
    U1.v[i] = cs_sel(md, du1, cu1);
    V1.v[i] = cs_sel(md, dv1, zm.v[i]);
    U2.v[i] = cs_sel(md, du2, cu2);
    V2.v[i] = cs_sel(md, dv2, zo.v[i]);
  }
  cs_carry(V1);
  cs_carry(V2);
}

// ---- the lazy G1 doubling (bn254_g1quad.h: g1q_dbl, dbl-2009-l, a = 0) --------------------
// Rounds of products: {A = X^2, B = Y^2, YZ} -> {C = B^2, T2 = t^2, F = E^2} -> {E w}, with
// E = 3A, t = X + B, D = 2(T2 - A - C), X3 = F - 2D, w = D - X3, Y3 = E w - 8C, Z3 = 2 YZ.
// Inputs < 2q: A, B, YZ, C < 1.02 q; E < 3.06 q and t < 3.02 q carried (T2, F < 1.04 q).
// D' = D + 5q in (0.92 q, 7.08 q) is carried, X3 and Y3 are reduced once each (fp_reduce64),
// w' = D' - X3 + 2q = w + 7q in (0.92 q, 9.08 q) feeds E w' (< 28 q^2: product < 1.13 q).
struct G1dConst {
  static constexpr CsLimbs D5 = cs_redundant(5, (int64_t)1 << 31);   // 2T2 - 2A - 2C + 5q
  static constexpr CsLimbs D16 = cs_redundant(16, (int64_t)1 << 30); // F - 2D' + 16q
  static constexpr CsLimbs D2 = cs_redundant(2, (int64_t)1 << 29);   // D' - X3 + 2q
  static constexpr CsLimbs D9 = cs_redundant(9, (int64_t)1 << 29);   // E w' - 8C + 9q
};
BN_HD void g1d_et(fp& E, fp& t, const fp& A, const fp& X, const fp& B) {
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
    E.v[i] = 3u * A.v[i];
    t.v[i] = X.v[i] + B.v[i];
  }
  cs_carry(E);
  cs_carry(t);
}
BN_HD void g1d_x3w(fp& X3, fp& w, const fp& T2, const fp& A, const fp& C, const fp& F) {
  fp Dp, x;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) Dp.v[i] = 2u * (T2.v[i] - A.v[i] - C.v[i]) + G1dConst::D5.v[i];
  cs_carry(Dp);
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) x.v[i] = F.v[i] - 2u * Dp.v[i] + G1dConst::D16.v[i];
  cs_carry(x);
  fp_reduce64(X3, x);
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) w.v[i] = Dp.v[i] - X3.v[i] + G1dConst::D2.v[i];
  cs_carry(w);
}
BN_HD void g1d_y3(fp& Y3, const fp& Ew, const fp& C) {
  fp c8, x;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) c8.v[i] = C.v[i] << 3;
  cs_carry(c8);
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) x.v[i] = Ew.v[i] - c8.v[i] + G1dConst::D9.v[i];
  cs_carry(x);
  fp_reduce64(Y3, x);
}

// one lane's lazy doubling (the same stages with the products inline): the host check of g1q_dbl
BN_HD void g1_dbl_lazy(g1j& r, const g1j& p) {
  fp A, B, YZ, Z3, E, t, C, T2, F, X3, w, Ew;
  f_mul(A, p.X, p.X);
  f_mul(B, p.Y, p.Y);
  f_mul(YZ, p.Y, p.Z);
  f_add(Z3, YZ, YZ);
  g1d_et(E, t, A, p.X, B);
  f_mul(C, B, B);
  f_mul(T2, t, t);
  f_mul(F, E, E);
  g1d_x3w(X3, w, T2, A, C, F);
  f_mul(Ew, E, w);
  g1d_y3(r.Y, Ew, C);
  r.X = X3;
  r.Z = Z3;
}

// unreduced operand sums (bn254_g2wave.h, bn254_g1quad.h): a + b, and a - b + 2q (low limbs of
// Q2R >= 2^29 > b_i), for a, b < 2q normalised: limbs < 2^30 / < 1.5 2^30, values < 4q -- f_mul
// takes either on both sides (tests/test_bn254_inv.py: test_fp_mul_raw_both_operands)
BN_HD void fl_sum(fp& r, const fp& a, const fp& b) {
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) r.v[i] = a.v[i] + b.v[i];
}
BN_HD void fl_diff2q(fp& r, const fp& a, const fp& b) {
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) r.v[i] = a.v[i] - b.v[i] + SqConst::Q2R.v[i];
}

// ---- small linear combinations with one reduction ------------------------------------------
// r = C0 a0 + C1 a1 + C2 a2 (mod q), reduced below 2q, for a_j normalised with values < 2q:
// K q (K >= 2 * the negative coefficients' sum) keeps the value in (0, 64q), and a redundant form
// of K q with low limbs >= 2^29 * that sum keeps every low limb in [0, 7 2^29).
template <int K, int NEG>
struct CsRed {
  static constexpr CsLimbs V = cs_redundant(K, (int64_t)NEG << 29);
};
template <int C0, int C1, int C2, int K>
BN_HD void fp_lin3(fp& r, const fp& a0, const fp& a1, const fp& a2) {
  constexpr int NEG = (C0 < 0 ? -C0 : 0) + (C1 < 0 ? -C1 : 0) + (C2 < 0 ? -C2 : 0);
  constexpr int POS = (C0 > 0 ? C0 : 0) + (C1 > 0 ? C1 : 0) + (C2 > 0 ? C2 : 0);
  static_assert(NEG + POS <= 6 && K >= 2 * NEG && K + 2 * POS <= 62, "fp_lin3 bounds");
  fp x;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++)
    x.v[i] = (uint32_t)C0 * a0.v[i] + (uint32_t)C1 * a1.v[i] + (uint32_t)C2 * a2.v[i] + CsRed<K, NEG>::V.v[i];
  cs_carry(x);
  fp_reduce64(r, x);
}
