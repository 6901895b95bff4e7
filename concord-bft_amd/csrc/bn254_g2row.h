// G2 (E'(Fp2)) Jacobian arithmetic on row-parallel Fp (bn254_row.h): one point per wave,
// replicated in the four rows, Fp2 = two row elements (a + b i); each step's independent Fp
// products are dealt one per ROW, four per pass (g1r_round), and gathered back to every row.
// Same formulas and special cases as the one-lane G2 code (bn254_pairing.h: g2_dbl_j,
// g2_add_j_body, line_dbl_j, line_add_j) and the lane-per-product wave form (bn254_g2wave.h);
// the host emulation compares them value for value (tests/cpp/bn254_shim.cpp).
//
// Why rows: in the lane-per-product form every lane holds all of a step's Fp2 values in nine
// limbs, so each round pays a 15-way operand select (2 x 9 cndmasks per product), nine
// ds_bpermutes per product for the gather, and ~40-instruction reduced adds for the Fp2 sums, on
// top of the ~250-instruction one-lane multiply.  Here each lane holds ONE limb: a select is 6
// instructions per pass, a gather one ds_bpermute per product, an add or subtraction one carry
// pass, a multiply ~110 instructions -- a G2 doubling with its line is 8 passes.
//
// Value bounds (bn254_row.h: products need (a/q)(b/q) < 221; rf_sub needs b < 4q, rf_sub32
// b < 16q; rf_reduce x < 2^261 -> < 4q): point coordinates leave every function below 4q (R4);
// line coefficients are left unreduced (< 50q: a one-lane f_mul against a value < 2q still
// returns < 2q, and the key-table normalisation reduces them as it loads them); Karatsuba operand sums are formed from R4 values (< 8q), the worst
// product is (8q)(24q) = 192 q^2 (E (D - X3), r (V - X3)); every bound is noted where it is used.
#pragma once
#include "bn254_g1row.h"
#include "bn254_tower.h"

template <class U>
struct F2R {
  U a, b;
};
template <class U>
struct G2R {
  F2R<U> X, Y, Z;
};

struct RfMult {  // q, 2q, 3q with normalised limbs: a value < 4q is 0 mod q iff it is one of 0, q, 2q, 3q
  static constexpr uint32_t Q2N[9] = {0x00000026u, 0x10000000u, 0x000009d3u, 0x04000000u, 0x00010c24u,
                                      0x0d800000u, 0x000dd1a2u, 0x00900000u, 0x004a46c9u};
  static constexpr uint32_t Q3N[9] = {0x00000039u, 0x08000000u, 0x00000ebdu, 0x06000000u, 0x00019236u,
                                      0x14400000u, 0x0014ba73u, 0x10d80000u, 0x006f6a2du};
};

template <class U, class W>
struct G2RowCtx : RowCtx<U, W> {
  U q1n, q2n, q3n, zero;
  RF_HD explicit G2RowCtx(U tag)
      : RowCtx<U, W>(tag),
        q1n(rf_row_const(FpParams::Q, tag)),
        q2n(rf_row_const(RfMult::Q2N, tag)),
        q3n(rf_row_const(RfMult::Q3N, tag)),
        zero(rf_const(tag, 0u)) {}
  // x row-normal, value < 4q: x == 0 mod q?  (wave-uniform: row 0 decides, all rows are equal)
  RF_HD bool zero4(U x) const {
    const U n = rf_normalize(x);
    return rf_row0_equals(n, zero) || rf_row0_equals(n, q1n) || rf_row0_equals(n, q2n) || rf_row0_equals(n, q3n);
  }
  RF_HD bool zero4(const F2R<U>& x) const { return zero4(x.a) && zero4(x.b); }
};

// N <= 16 products, four per pass; every row receives all N
template <int N, class U, class W>
RF_HD void r_prods(U* o, const U* a, const U* b, const RowCtx<U, W>& c) {
  if constexpr (N > 4) {
    g1r_round<4>(o, a, b, c);
    r_prods<N - 4>(o + 4, a + 4, b + 4, c);
  } else {
    g1r_round<N>(o, a, b, c);
  }
}

// ---- Fp2 pieces.  Operand slots of x * y (Karatsuba: x0 y0, x1 y1, (x0 + x1)(y0 + y1)) and x^2
// ((x0 + x1)(x0 - x1 + 8q), x0 x1), then the results from the gathered products.
template <class U>
RF_HD void f2r_mul_ops(U* A, U* B, int o, const F2R<U>& x, const F2R<U>& y) {
  A[o] = x.a;
  B[o] = y.a;
  A[o + 1] = x.b;
  B[o + 1] = y.b;
  A[o + 2] = rf_add(x.a, x.b);
  B[o + 2] = rf_add(y.a, y.b);
}
template <class U, class W>
RF_HD void f2r_sqr_ops(U* A, U* B, int o, const F2R<U>& x, const RowCtx<U, W>& c) {  // x R4: (8q)(12q)
  A[o] = rf_add(x.a, x.b);
  B[o] = c.sub(x.a, x.b);
  A[o + 1] = x.a;
  B[o + 1] = x.b;
}
// x * y reduced: (p0 - p1, p2 - p0 - p1) -> R4
template <class U, class W>
RF_HD void f2r_mul_res(F2R<U>& r, const U* p, int o, const RowCtx<U, W>& c) {
  r.a = c.red(c.sub(p[o], p[o + 1]));
  r.b = c.red(c.sub(c.sub(p[o + 2], p[o]), p[o + 1]));
}
// x * y unreduced: a < 10q, b < 18q (for a subtrahend-free use: the minuend of a subtraction, a
// line coefficient, or one more reduction after further sums)
template <class U, class W>
RF_HD void f2r_mul_raw(F2R<U>& r, const U* p, int o, const RowCtx<U, W>& c) {
  r.a = c.sub(p[o], p[o + 1]);
  r.b = c.sub(c.sub(p[o + 2], p[o]), p[o + 1]);
}
// x^2: a < 2q (a product), b = 2 x0 x1 < 4q
template <class U>
RF_HD void f2r_sqr_res(F2R<U>& r, const U* p, int o) {
  r.a = p[o];
  r.b = rf_add(p[o + 1], p[o + 1]);
}
template <class U, class W>
RF_HD F2R<U> f2r_red(const F2R<U>& x, const RowCtx<U, W>& c) {
  return {c.red(x.a), c.red(x.b)};
}
template <class U>
RF_HD F2R<U> f2r_add(const F2R<U>& x, const F2R<U>& y) {
  return {rf_add(x.a, y.a), rf_add(x.b, y.b)};
}
template <class U, class W>
RF_HD F2R<U> f2r_sub(const F2R<U>& x, const F2R<U>& y, const RowCtx<U, W>& c) {  // y < 4q: + 8q
  return {c.sub(x.a, y.a), c.sub(x.b, y.b)};
}
template <class U, class W>
RF_HD F2R<U> f2r_sub32(const F2R<U>& x, const F2R<U>& y, const RowCtx<U, W>& c) {  // y < 16q: + 32q
  return {c.sub32(x.a, y.a), c.sub32(x.b, y.b)};
}

// ---- T <- 2T (dbl-2009-l).  LINE: also the tangent's (A, B, C) = (2YZ^3, -3X^2 Z^2, 3X^3 - 2Y^2)
// of line_dbl_j / g2w_dbl, each R4.  Passes: 3 + 4 + 1 with the line; without it 1 + 2 + 1 (the
// three products of YZ, needed only for Z3, fill the spare slots of the later passes).
template <bool LINE, class U, class W>
RF_HD void g2r_dbl(F2R<U>* line, G2R<U>& T, const G2RowCtx<U, W>& c) {
  U A[15], B[15], P[15];
  f2r_sqr_ops(A, B, 0, T.X, c);
  f2r_sqr_ops(A, B, 2, T.Y, c);
  F2R<U> XX, YY, ZZ, YZ;
  if constexpr (LINE) {
    f2r_sqr_ops(A, B, 4, T.Z, c);
    f2r_mul_ops(A, B, 6, T.Y, T.Z);
    r_prods<9>(P, A, B, c);
    f2r_sqr_res(ZZ, P, 4);
    f2r_mul_raw(YZ, P, 6, c);  // < 18q: only 2YZ is used, reduced
  } else {
    r_prods<4>(P, A, B, c);
  }
  f2r_sqr_res(XX, P, 0);
  f2r_sqr_res(YY, P, 2);
  const F2R<U> E = f2r_red(f2r_add(f2r_add(XX, XX), XX), c);  // 3X^2 (XX.b < 4q: < 12q)
  const F2R<U> D0 = f2r_red(f2r_add(T.X, YY), c);             // X + Y^2 < 8q
  F2R<U> t;
  int o = 0;
  if constexpr (LINE) {
    t = f2r_red(f2r_add(YZ, YZ), c);                            // Z3 = 2YZ
    const F2R<U> nZZ = f2r_sub(F2R<U>{c.zero, c.zero}, ZZ, c);  // -Z^2 + 8q: (4q, 8q]
    f2r_mul_ops(A, B, 0, t, ZZ);     // A = 2YZ Z^2: (8q)(6q)
    f2r_mul_ops(A, B, 3, E, nZZ);    // B = 3X^2 (-Z^2): (8q)(16q)
    f2r_mul_ops(A, B, 6, E, T.X);    // 3X^3: (8q)(8q)
    o = 9;
  }
  f2r_sqr_ops(A, B, o, YY, c);      // Y^4 (YY.a < 2q, YY.b < 4q: (6q)(10q))
  f2r_sqr_ops(A, B, o + 2, D0, c);  // (X + Y^2)^2
  f2r_sqr_ops(A, B, o + 4, E, c);   // F = E^2
  U yz2 = {};
  if constexpr (LINE) {
    r_prods<15>(P, A, B, c);
    f2r_mul_raw(line[0], P, 0, c);  // line coefficients stay unreduced: < 18q, < 18q, < 50q
    f2r_mul_raw(line[1], P, 3, c);
    F2R<U> X3E;
    f2r_mul_raw(X3E, P, 6, c);
    line[2] = f2r_sub32(X3E, f2r_add(YY, YY), c);  // 3X^3 - 2Y^2 (2YY < 8q)
  } else {
    f2r_mul_ops(A, B, 6, T.Y, T.Z);  // Y Z: two of its products here, the third in the last pass
    yz2 = A[8];
    const U yz2b = B[8];
    r_prods<8>(P, A, B, c);
    A[8] = yz2;
    B[8] = yz2b;
  }
  F2R<U> YYYY, DD, F;
  f2r_sqr_res(YYYY, P, o);
  f2r_sqr_res(DD, P, o + 2);
  f2r_sqr_res(F, P, o + 4);
  U yz01[2] = {P[6], P[7]};
  // D = 2((X + YY)^2 - XX - YYYY) (< 2 (4q + 64q)), X3 = F - 2D, w = D - X3
  const F2R<U> D1 = f2r_sub32(f2r_sub32(DD, XX, c), YYYY, c);
  const F2R<U> D = f2r_red(f2r_add(D1, D1), c);
  const F2R<U> X3 = f2r_red(f2r_sub32(F, f2r_add(D, D), c), c);
  const F2R<U> w = f2r_sub(D, X3, c);  // < 12q
  f2r_mul_ops(A, B, 0, E, w);          // (8q)(24q) = 192 q^2
  F2R<U> Y3;
  if constexpr (LINE) {
    r_prods<3>(P, A, B, c);
  } else {
    A[3] = A[8];
    B[3] = B[8];
    r_prods<4>(P, A, B, c);
    const U yzp[3] = {yz01[0], yz01[1], P[3]};
    f2r_mul_raw(YZ, yzp, 0, c);
    t = f2r_red(f2r_add(YZ, YZ), c);  // Z3 = 2YZ (< 36q before the reduction)
  }
  (void)yz2;
  f2r_mul_raw(Y3, P, 0, c);
  const F2R<U> Y4 = f2r_add(f2r_add(YYYY, YYYY), f2r_add(YYYY, YYYY));  // 4 YYYY < 16q
  T.Y = f2r_red(f2r_sub32(f2r_sub32(Y3, Y4, c), Y4, c), c);              // E (D - X3) - 8 YYYY < 82q
  T.X = X3;
  T.Z = t;
}

// ---- T <- T + Q for affine Q = (qx, qy) R4 (madd-2007-bl).  LINE: also the line through T and
// Q, (A, B, C) = (Z H, -R, qy Z X - qx Y) of line_add_j / g2w_add, and no exceptional-case test
// (never taken by the Miller loop of a point of order r).  Without LINE, T = +-Q (H = 0) returns
// false with same_y = (T == Q), T untouched.  Passes: 2 + 3 + 3 + 2 + 2 with the line,
// 2 + 2 + 2 + 2 + 2 without.
template <bool LINE, class U, class W>
RF_HD bool g2r_madd(F2R<U>* line, G2R<U>& T, const F2R<U>& qx, const F2R<U>& qy, const G2RowCtx<U, W>& c,
                    bool& same_y) {
  U A[9], B[9], P[9];
  f2r_sqr_ops(A, B, 0, T.Z, c);
  f2r_mul_ops(A, B, 2, qy, T.Z);
  F2R<U> ZZ, QZ, QXY, U2, S2;
  if constexpr (LINE) {
    f2r_mul_ops(A, B, 5, qx, T.Y);
    r_prods<8>(P, A, B, c);
    f2r_mul_res(QXY, P, 5, c);
  } else {
    r_prods<5>(P, A, B, c);
  }
  f2r_sqr_res(ZZ, P, 0);
  f2r_mul_res(QZ, P, 2, c);
  f2r_mul_ops(A, B, 0, qx, ZZ);  // U2: (8q)(6q)
  f2r_mul_ops(A, B, 3, QZ, ZZ);  // S2
  if constexpr (LINE) {
    f2r_mul_ops(A, B, 6, QZ, T.X);  // qy Z X
    r_prods<9>(P, A, B, c);
    F2R<U> QZX;
    f2r_mul_raw(QZX, P, 6, c);
    line[2] = f2r_sub(QZX, QXY, c);  // < 26q, unreduced
  } else {
    r_prods<6>(P, A, B, c);
  }
  f2r_mul_raw(U2, P, 0, c);  // minuends: reduced after the subtraction
  f2r_mul_raw(S2, P, 3, c);
  const F2R<U> H = f2r_red(f2r_sub(U2, T.X, c), c);
  const F2R<U> R = f2r_red(f2r_sub(S2, T.Y, c), c);
  if constexpr (!LINE) {
    if (c.zero4(H)) {
      same_y = c.zero4(R);
      return false;
    }
  } else {
    line[1] = f2r_sub(F2R<U>{c.zero, c.zero}, R, c);  // -R + 8q < 8q, unreduced
  }
  const F2R<U> r = f2r_red(f2r_add(R, R), c);
  const F2R<U> ZH = f2r_red(f2r_add(T.Z, H), c);
  int o = 0;
  if constexpr (LINE) {
    f2r_mul_ops(A, B, 0, T.Z, H);  // A = Z H
    o = 3;
  }
  f2r_sqr_ops(A, B, o, H, c);
  f2r_sqr_ops(A, B, o + 2, r, c);
  f2r_sqr_ops(A, B, o + 4, ZH, c);
  r_prods<LINE ? 9 : 6>(P, A, B, c);
  if constexpr (LINE) f2r_mul_raw(line[0], P, 0, c);
  F2R<U> HH, rr, ZH2;
  f2r_sqr_res(HH, P, o);
  f2r_sqr_res(rr, P, o + 2);
  f2r_sqr_res(ZH2, P, o + 4);
  const F2R<U> I = f2r_red(f2r_add(f2r_add(HH, HH), f2r_add(HH, HH)), c);  // 4 HH < 16q
  f2r_mul_ops(A, B, 0, H, I);    // J
  f2r_mul_ops(A, B, 3, T.X, I);  // V
  r_prods<6>(P, A, B, c);
  F2R<U> J, V;
  f2r_mul_res(J, P, 0, c);
  f2r_mul_res(V, P, 3, c);
  const F2R<U> X3 = f2r_red(f2r_sub32(f2r_sub(rr, J, c), f2r_add(V, V), c), c);
  const F2R<U> w = f2r_sub(V, X3, c);  // < 12q
  f2r_mul_ops(A, B, 0, r, w);          // (8q)(24q)
  f2r_mul_ops(A, B, 3, T.Y, J);
  r_prods<6>(P, A, B, c);
  F2R<U> Y3, YJ;
  f2r_mul_raw(Y3, P, 0, c);
  f2r_mul_res(YJ, P, 3, c);
  T.Y = f2r_red(f2r_sub32(Y3, f2r_add(YJ, YJ), c), c);    // < 18q + 32q
  T.Z = f2r_red(f2r_sub(f2r_sub(ZH2, ZZ, c), HH, c), c);  // (Z + H)^2 - ZZ - HH < 20q
  T.X = X3;
  return true;
}

// ---- T <- T + Q, both Jacobian and finite (add-2007-bl, g2_add_j_body / g2w_add_full).  T = +-Q
// (U1 = U2) returns false with same_y = (S1 = S2), T untouched.  Passes 1 + 3 + 3 + 3 + 2.
template <class U, class W>
RF_HD bool g2r_add(G2R<U>& T, const G2R<U>& Q, const G2RowCtx<U, W>& c, bool& same_y) {
  U A[12], B[12], P[12];
  f2r_sqr_ops(A, B, 0, T.Z, c);
  f2r_sqr_ops(A, B, 2, Q.Z, c);
  r_prods<4>(P, A, B, c);
  F2R<U> Z1Z1, Z2Z2;
  f2r_sqr_res(Z1Z1, P, 0);
  f2r_sqr_res(Z2Z2, P, 2);
  f2r_mul_ops(A, B, 0, T.X, Z2Z2);  // U1: (8q)(6q)
  f2r_mul_ops(A, B, 3, Q.X, Z1Z1);  // U2
  f2r_mul_ops(A, B, 6, T.Y, Q.Z);
  f2r_mul_ops(A, B, 9, Q.Y, T.Z);
  r_prods<12>(P, A, B, c);
  F2R<U> U1, U2, Y1Z2, Y2Z1;
  f2r_mul_res(U1, P, 0, c);
  f2r_mul_res(U2, P, 3, c);
  f2r_mul_res(Y1Z2, P, 6, c);
  f2r_mul_res(Y2Z1, P, 9, c);
  const F2R<U> H = f2r_red(f2r_sub(U2, U1, c), c);
  const F2R<U> H2 = f2r_red(f2r_add(H, H), c);
  const F2R<U> ZS = f2r_red(f2r_add(T.Z, Q.Z), c);
  f2r_mul_ops(A, B, 0, Y1Z2, Z2Z2);  // S1
  f2r_mul_ops(A, B, 3, Y2Z1, Z1Z1);  // S2
  f2r_sqr_ops(A, B, 6, H2, c);       // I = (2H)^2
  f2r_sqr_ops(A, B, 8, ZS, c);       // (Z1 + Z2)^2
  r_prods<10>(P, A, B, c);
  F2R<U> S1, S2, I, ZS2;
  f2r_mul_res(S1, P, 0, c);
  f2r_mul_res(S2, P, 3, c);
  const F2R<U> R = f2r_red(f2r_sub(S2, S1, c), c);
  if (c.zero4(H)) {
    same_y = c.zero4(R);
    return false;
  }
  f2r_sqr_res(I, P, 6);
  f2r_sqr_res(ZS2, P, 8);
  const F2R<U> ZZ = f2r_red(f2r_sub(f2r_sub(ZS2, Z1Z1, c), Z2Z2, c), c);  // < 20q
  const F2R<U> r = f2r_red(f2r_add(R, R), c);
  f2r_mul_ops(A, B, 0, H, I);    // J: (8q)(6q)
  f2r_mul_ops(A, B, 3, U1, I);   // V
  f2r_mul_ops(A, B, 6, ZZ, H);   // Z3
  f2r_sqr_ops(A, B, 9, r, c);    // r^2
  r_prods<11>(P, A, B, c);
  F2R<U> J, V, rr;
  f2r_mul_res(J, P, 0, c);
  f2r_mul_res(V, P, 3, c);
  f2r_mul_res(T.Z, P, 6, c);
  f2r_sqr_res(rr, P, 9);
  const F2R<U> X3 = f2r_red(f2r_sub32(f2r_sub(rr, J, c), f2r_add(V, V), c), c);
  const F2R<U> w = f2r_sub(V, X3, c);
  f2r_mul_ops(A, B, 0, r, w);
  f2r_mul_ops(A, B, 3, S1, J);
  r_prods<6>(P, A, B, c);
  F2R<U> Y3, SJ;
  f2r_mul_res(Y3, P, 0, c);
  f2r_mul_res(SJ, P, 3, c);
  T.Y = f2r_red(f2r_sub32(Y3, f2r_add(SJ, SJ), c), c);
  T.X = X3;
  return true;
}

// acc += o / acc += (qx, qy) with wave-uniform infinity flags: every case of g2_add_j_body (O + o,
// acc + O, acc = o -> doubling, acc = -o -> O); a doubling that lands on O sets the flag
template <class U, class W>
RF_HD void g2r_accum(G2R<U>& acc, bool& inf, const G2R<U>& o, bool oinf, const G2RowCtx<U, W>& c) {
  if (oinf) return;
  if (inf) {
    acc = o;
    inf = false;
    return;
  }
  bool same_y = false;
  if (!g2r_add(acc, o, c, same_y)) {
    if (same_y) {
      g2r_dbl<false>((F2R<U>*)nullptr, acc, c);
      inf = c.zero4(acc.Z);
    } else {
      inf = true;
    }
  }
}
template <class U, class W>
RF_HD void g2r_accum_aff(G2R<U>& acc, bool& inf, const F2R<U>& qx, const F2R<U>& qy, const G2RowCtx<U, W>& c) {
  if (inf) {
    acc.X = qx;
    acc.Y = qy;
    acc.Z = F2R<U>{c.one, c.zero};
    inf = false;
    return;
  }
  bool same_y = false;
  if (!g2r_madd<false>((F2R<U>*)nullptr, acc, qx, qy, c, same_y)) {
    if (same_y) {
      g2r_dbl<false>((F2R<U>*)nullptr, acc, c);
      inf = c.zero4(acc.Z);
    } else {
      inf = true;
    }
  }
}

// Q in G2 (Q a decoded point of E'(Fp2), not infinity) by the endomorphism psi = twist^-1 o
// Frobenius o twist: psi(Q) = [6u^2] Q.  psi satisfies psi^2 - t psi + p = 0 with t = 6u^2 + 1
// (the trace of E over Fp, #E(Fp) = r), so psi(Q) = [6u^2] Q gives [(6u^2)^2 - t 6u^2 + p] Q =
// [r] Q = O; conversely G2 is psi's eigenspace for p = r + 6u^2 on E'[r].  So the verdict is
// r Q == O's (g2_in_subgroup), for half the doublings: [6u^2] Q is 126 doublings and 11 mixed
// additions of Q (exact in every case, g2r_accum_aff), then psi(Q) = (conj(x) g_x, conj(y) g_y)
// against T = (X : Y : Z): X = x' Z^2, Y = y' Z^3.  Wave-uniform.
template <class U, class W>
RF_HD bool g2r_in_subgroup(const F2R<U>& qx, const F2R<U>& qy, const G2RowCtx<U, W>& c) {
  const uint32_t k[4] = {0x00000006u, 0x06000000u, 0x00000003u, 0x61818000u};  // 6u^2, bit 126 on top
  G2R<U> T{qx, qy, F2R<U>{c.one, c.zero}};
  bool inf = false;
#pragma nounroll
  for (int i = 125; i >= 0; i--) {
    if (!inf) {
      g2r_dbl<false>((F2R<U>*)nullptr, T, c);
      inf = c.zero4(T.Z);
    }
    if ((k[i >> 5] >> (i & 31)) & 1u) g2r_accum_aff(T, inf, qx, qy, c);
  }
  if (inf) return false;  // [6u^2] Q = O but psi(Q) is not O
  fp2 g;
  fp2_load(g, Bn254Consts::TWX1);
  const F2R<U> gx{rf_from_fe(g.a, c.zero), rf_from_fe(g.b, c.zero)};
  fp2_load(g, Bn254Consts::TWY1);
  const F2R<U> gy{rf_from_fe(g.a, c.zero), rf_from_fe(g.b, c.zero)};
  const F2R<U> cx{qx.a, c.sub(c.zero, qx.b)}, cy{qy.a, c.sub(c.zero, qy.b)};  // conjugates, b < 8q
  U A[8], B[8], P[8];
  F2R<U> ZZ, xs, ys, ZZZ, xz, yz;
  f2r_sqr_ops(A, B, 0, T.Z, c);  // Z R4: (8q)(12q)
  f2r_mul_ops(A, B, 2, cx, gx);  // (12q)(4q)
  f2r_mul_ops(A, B, 5, cy, gy);
  r_prods<8>(P, A, B, c);
  f2r_sqr_res(ZZ, P, 0);  // a < 2q, b < 4q
  f2r_mul_res(xs, P, 2, c);
  f2r_mul_res(ys, P, 5, c);
  f2r_mul_ops(A, B, 0, ZZ, T.Z);  // (6q)(8q)
  f2r_mul_ops(A, B, 3, xs, ZZ);   // (8q)(6q)
  r_prods<6>(P, A, B, c);
  f2r_mul_res(ZZZ, P, 0, c);
  f2r_mul_res(xz, P, 3, c);
  f2r_mul_ops(A, B, 0, ys, ZZZ);  // (8q)(8q)
  r_prods<3>(P, A, B, c);
  f2r_mul_res(yz, P, 0, c);
  return c.zero4(f2r_red(f2r_sub(T.X, xz, c), c)) && c.zero4(f2r_red(f2r_sub(T.Y, yz, c), c));
}

#if defined(__HIPCC__)
// ---- device memory <-> rows: 9 one-lane limb words (bn254_field.h layout) per Fp
__device__ __forceinline__ uint32_t rf_ld9(const uint32_t* p) {  // lane i of each row takes p[i]
  const uint32_t rl = __lane_id() & 15u;
  return rl < 9 ? p[rl] : 0u;
}
__device__ __forceinline__ F2R<uint32_t> f2r_ld(const uint32_t* p) { return {rf_ld9(p), rf_ld9(p + 9)}; }
// normalised limbs (value unchanged) of EACH row to that row's p[0..8] (p may differ per row)
__device__ __forceinline__ void rf_st9(uint32_t* p, uint32_t x) {
  const uint32_t n = rf_normalize(x), rl = __lane_id() & 15u;
  if (rl < 9) p[rl] = n;
}
__device__ __forceinline__ void f2r_st(uint32_t* p, const F2R<uint32_t>& x) {
  rf_st9(p, x.a);
  rf_st9(p + 9, x.b);
}
// the same from row 0 only (all rows hold the element)
__device__ __forceinline__ void rf_st9_row0(uint32_t* p, uint32_t x) {
  const uint32_t n = rf_normalize(x), l = __lane_id();
  if (l < 9) p[l] = n;
}
__device__ __forceinline__ void f2r_st_row0(uint32_t* p, const F2R<uint32_t>& x) {
  rf_st9_row0(p, x.a);
  rf_st9_row0(p + 9, x.b);
}
__device__ __forceinline__ F2R<uint32_t> f2r_from(const fp2& x) { return {rf_from_fe(x.a, 0u), rf_from_fe(x.b, 0u)}; }
#endif
