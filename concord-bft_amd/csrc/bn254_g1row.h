// G1 Jacobian arithmetic on row-parallel Fp (bn254_row.h): one point per wave, replicated in the
// four rows; each step's independent products are dealt one per ROW (four per round), each row
// computing its product with the limbs spread over its 16 lanes, then every row gathers the
// round's products (ds_bpermute).  Same formulas and special cases as g1_dbl / g1_add
// (bn254_pairing.h); host emulation compares them point for point (tests/cpp/bn254_shim.cpp).
//
// Value bounds (see bn254_row.h, products need (a/q)(b/q) < 221): X and Y leave every operation
// reduced (< 4q: X feeds X^2, Y feeds -Y); Z < 4q; intermediate values stay unreduced where the
// products they feed allow it (noted per line), two rf_reduce per doubling and per addition.  Infinity is not encoded in Z:
// callers carry a wave-uniform flag (a point of the MSM is infinity only before its first
// addition).
#pragma once
#include "bn254_row.h"

template <class U>
struct G1R {
  U X, Y, Z;
};

template <class U, class W>
struct RowCtx {
  U qrow, q8r, q32r, q7n, q8n, q9n, one, rowid;
  W q64r;
  RF_HD explicit RowCtx(U tag)
      : qrow(rf_row_const(FpParams::Q, tag)),
        q8r(rf_row_const(RfConsts::Q8R, tag)),
        q32r(rf_row_const(RfConsts::Q32R, tag)),
        q7n(rf_row_const(RfConsts::Q7N, tag)),
        q8n(rf_row_const(RfConsts::Q8N, tag)),
        q9n(rf_row_const(RfConsts::Q9N, tag)),
        one(rf_row_const(FpParams::ONE, tag)),
        rowid(rl_row(tag)),
        q64r(rf_row_const64<U, W>(RfConsts::Q64R, tag)) {}
  RF_HD U red(U x) const { return rf_reduce<U, W>(x, qrow, q64r); }
  RF_HD U sub(U a, U b) const { return rf_sub(a, b, q8r); }
  RF_HD U sub32(U a, U b) const { return rf_sub32(a, b, q32r); }
  RF_HD U mul(U a, U b) const { return rf_mul<U, W>(a, b, qrow); }
  // h = a - b + 8q with |a - b| < 2q (a, b products): is it 0 mod q?
  RF_HD bool zero_diff(U h) const {
    const U n = rf_normalize(h);
    return rf_row0_equals(n, q7n) || rf_row0_equals(n, q8n) || rf_row0_equals(n, q9n);
  }
};

// one round: row r multiplies a[r] * b[r] (r < N <= 4); every row receives all N products
template <int N, class U, class W>
RF_HD void g1r_round(U* o, const U* a, const U* b, const RowCtx<U, W>& c) {
  U ua = a[0], ub = b[0];
#pragma unroll
  for (int r = 1; r < N; r++) {
    const auto here = c.rowid == rf_const(ua, (uint32_t)r);
    ua = rf_sel(here, a[r], ua);
    ub = rf_sel(here, b[r], ub);
  }
  const U p = c.mul(ua, ub);
  if (N == 1) {
    o[0] = p;
    return;
  }
  U r[4];
  rl_all_rows(p, r);  // lane swaps (row_lanes.h), not the LDS crossbar
#pragma unroll
  for (int k = 0; k < N; k++) o[k] = r[k];
}

// r = 2p, a = 0 (dbl-2009-l with D = 4XB taken as one product: (X + B)^2 - A - C = 2XB)
template <class U, class W>
RF_HD void g1r_dbl(G1R<U>& r, const G1R<U>& p, const RowCtx<U, W>& c) {
  U o[3];
  {
    const U a[3] = {p.X, p.Y, p.Y}, b[3] = {p.X, p.Y, p.Z};
    g1r_round<3>(o, a, b, c);
  }
  const U A = o[0], B = o[1], T1 = o[2];
  const U E = rf_add(rf_add(A, A), A);  // < 6q
  {
    const U a[3] = {B, p.X, E}, b[3] = {B, B, E};
    g1r_round<3>(o, a, b, c);
  }
  const U C = o[0], XB = o[1], F = o[2];
  const U XB2 = rf_add(XB, XB), XB4 = rf_add(XB2, XB2);  // 4XB = D < 8q
  const U X3 = c.red(c.sub32(F, rf_add(XB4, XB4)));      // F - 2D
  const U Wv = c.sub(XB4, X3);                            // D - X3 < 16q (E W: 6 x 16 < 221)
  {
    const U a[1] = {E}, b[1] = {Wv};
    g1r_round<1>(o, a, b, c);
  }
  const U C2 = rf_add(C, C), C4 = rf_add(C2, C2);
  r.Y = c.red(c.sub32(o[0], rf_add(C4, C4)));  // E (D - X3) - 8C
  r.X = X3;
  r.Z = rf_add(T1, T1);  // 2YZ < 4q
}

enum G1rAddResult { G1R_SUM, G1R_INF };

// r = p + q (add-2007-bl with r = 2 Rd: r^2 = 4 Rd^2, r (V - X3) = 2 Rd (V - X3)), p, q finite.
// p == q -> doubling; p == -q -> returns G1R_INF.
template <class U, class W>
RF_HD G1rAddResult g1r_add(G1R<U>& r, const G1R<U>& p, const G1R<U>& q, const RowCtx<U, W>& c) {
  U o[4];
  {
    const U a[2] = {p.Z, q.Z};
    g1r_round<2>(o, a, a, c);
  }
  const U Z1Z1 = o[0], Z2Z2 = o[1];
  {
    const U a[4] = {p.X, q.X, p.Y, q.Y}, b[4] = {Z2Z2, Z1Z1, q.Z, p.Z};
    g1r_round<4>(o, a, b, c);
  }
  const U U1 = o[0];
  const U Hd = c.sub(o[1], U1);     // H = U2 - U1 (+ 8q), < 10q
  const U ZS = rf_add(p.Z, q.Z);    // < 8q
  {
    const U a[4] = {o[2], o[3], Hd, ZS}, b[4] = {Z2Z2, Z1Z1, Hd, ZS};
    g1r_round<4>(o, a, b, c);
  }
  const U S1 = o[0];
  const U Rd = c.sub(o[1], S1);  // (S2 - S1) + 8q, < 10q
  if (c.zero_diff(Hd)) {         // same x (wave-uniform)
    if (c.zero_diff(Rd)) {
      g1r_dbl(r, p, c);
      return G1R_SUM;
    }
    return G1R_INF;
  }
  const U H2 = rf_add(o[2], o[2]), I = rf_add(H2, H2);  // (2H)^2 < 8q
  const U ZZb = c.sub(c.sub(o[3], Z1Z1), Z2Z2);          // (Z1 + Z2)^2 - Z1Z1 - Z2Z2 < 18q (x H: 180 < 221)
  {
    const U a[4] = {Hd, U1, Rd, ZZb}, b[4] = {I, I, Rd, Hd};
    g1r_round<4>(o, a, b, c);
  }
  const U J = o[0], V = o[1];
  const U R2 = rf_add(o[2], o[2]), RR = rf_add(R2, R2);  // r^2 < 8q
  const U X3 = c.red(c.sub(c.sub(RR, J), rf_add(V, V)));
  const U Wv = c.sub(V, X3);  // < 10q
  r.Z = o[3];
  {
    const U a[2] = {Rd, S1}, b[2] = {Wv, J};
    g1r_round<2>(o, a, b, c);
  }
  r.Y = c.red(c.sub(rf_add(o[0], o[0]), rf_add(o[1], o[1])));  // r (V - X3) - 2 S1 J
  r.X = X3;
  return G1R_SUM;
}

// -p
template <class U, class W>
RF_HD void g1r_neg(G1R<U>& r, const G1R<U>& p, const RowCtx<U, W>& c) {
  r.X = p.X;
  r.Z = p.Z;
  r.Y = c.red(c.sub(rf_const(p.Y, 0u), p.Y));
}
