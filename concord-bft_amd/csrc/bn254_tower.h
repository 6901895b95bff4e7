// BN-P254 extension tower (host + device): Fp2 = Fp[i]/(i^2 + 1), Fp6 = Fp2[v]/(v^3 - xi),
// Fp12 = Fp6[w]/(w^2 - v), xi = 1 + i.  Frobenius maps use the generated constants of
// bn254_consts.h (gamma_k = xi^(k(p^j - 1)/6)).
#pragma once
#include "bn254_consts.h"
#include "bn254_field.h"

struct fp2 {
  fp a, b;  // a + b i
};
struct fp6 {
  fp2 c0, c1, c2;  // c0 + c1 v + c2 v^2
};
struct fp12 {
  fp6 c0, c1;  // c0 + c1 w
};

template <int N>
BN_HD void fp_load(fp& r, const uint32_t (&c)[N], int off) {
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) r.v[i] = c[off + i];
}
template <int N>
BN_HD void fp2_load(fp2& r, const uint32_t (&c)[N]) {
  fp_load(r.a, c, 0);
  fp_load(r.b, c, 9);
}

// ------------------------------------------------------------------------------ Fp2
BN_HD void fp2_zero(fp2& r) {
  f_zero(r.a);
  f_zero(r.b);
}
BN_HD void fp2_one(fp2& r) {
  f_one(r.a);
  f_zero(r.b);
}
BN_HD void fp2_add(fp2& r, const fp2& x, const fp2& y) {
  f_add(r.a, x.a, y.a);
  f_add(r.b, x.b, y.b);
}
BN_HD void fp2_sub(fp2& r, const fp2& x, const fp2& y) {
  f_sub(r.a, x.a, y.a);
  f_sub(r.b, x.b, y.b);
}
BN_HD void fp2_neg(fp2& r, const fp2& x) {
  f_neg(r.a, x.a);
  f_neg(r.b, x.b);
}
BN_HD void fp2_dbl(fp2& r, const fp2& x) {
  f_add(r.a, x.a, x.a);
  f_add(r.b, x.b, x.b);
}
BN_HD void fp2_conj(fp2& r, const fp2& x) {
  r.a = x.a;
  f_neg(r.b, x.b);
}
BN_HD void fp2_mul(fp2& r, const fp2& x, const fp2& y) {  // Karatsuba, 3 M
  fp t0, t1, s0, s1;
  f_mul(t0, x.a, y.a);
  f_mul(t1, x.b, y.b);
  f_add(s0, x.a, x.b);
  f_add(s1, y.a, y.b);
  f_mul(s0, s0, s1);
  f_sub(r.a, t0, t1);
  f_sub(s0, s0, t0);
  f_sub(r.b, s0, t1);
}
BN_HD void fp2_sqr(fp2& r, const fp2& x) {  // complex squaring, 2 M
  fp s, d, m;
  f_add(s, x.a, x.b);
  f_sub(d, x.a, x.b);
  f_mul(m, x.a, x.b);
  f_mul(r.a, s, d);
  f_add(r.b, m, m);
}
BN_HD void fp2_mul_fp(fp2& r, const fp2& x, const fp& k) {
  f_mul(r.a, x.a, k);
  f_mul(r.b, x.b, k);
}
BN_HD void fp2_mul_xi(fp2& r, const fp2& x) {  // (a + b i)(1 + i) = (a - b) + (a + b) i
  fp t;
  f_sub(t, x.a, x.b);
  f_add(r.b, x.a, x.b);
  r.a = t;
}
// VAR: variable-time inversion (fp_inv_var) -- public values only (final exponentiations)
template <bool VAR = false>
BN_HDN void fp2_inv(fp2& r, const fp2& x) {
  fp n, t;
  f_sqr(n, x.a);
  f_sqr(t, x.b);
  f_add(n, n, t);
  if (VAR)
    fp_inv_var(n, n);
  else
    fp_inv(n, n);
  f_mul(r.a, x.a, n);
  f_mul(t, x.b, n);
  f_neg(r.b, t);
}
BN_HD bool fp2_eq(const fp2& x, const fp2& y) { return f_eq(x.a, y.a) && f_eq(x.b, y.b); }
BN_HD bool fp2_is_zero(const fp2& x) { return f_is_zero(x.a) && f_is_zero(x.b); }

// ------------------------------------------------------------------------------ Fp6
BN_HD void fp6_zero(fp6& r) {
  fp2_zero(r.c0);
  fp2_zero(r.c1);
  fp2_zero(r.c2);
}
BN_HD void fp6_one(fp6& r) {
  fp2_one(r.c0);
  fp2_zero(r.c1);
  fp2_zero(r.c2);
}
BN_HD void fp6_add(fp6& r, const fp6& x, const fp6& y) {
  fp2_add(r.c0, x.c0, y.c0);
  fp2_add(r.c1, x.c1, y.c1);
  fp2_add(r.c2, x.c2, y.c2);
}
BN_HD void fp6_sub(fp6& r, const fp6& x, const fp6& y) {
  fp2_sub(r.c0, x.c0, y.c0);
  fp2_sub(r.c1, x.c1, y.c1);
  fp2_sub(r.c2, x.c2, y.c2);
}
BN_HD void fp6_neg(fp6& r, const fp6& x) {
  fp2_neg(r.c0, x.c0);
  fp2_neg(r.c1, x.c1);
  fp2_neg(r.c2, x.c2);
}
BN_HDN void fp6_mul(fp6& r, const fp6& x, const fp6& y) {  // 6 Fp2 M
  fp2 t0, t1, t2, s0, s1, c0, c1, c2;
  fp2_mul(t0, x.c0, y.c0);
  fp2_mul(t1, x.c1, y.c1);
  fp2_mul(t2, x.c2, y.c2);
  // c0 = t0 + xi((x1+x2)(y1+y2) - t1 - t2)
  fp2_add(s0, x.c1, x.c2);
  fp2_add(s1, y.c1, y.c2);
  fp2_mul(s0, s0, s1);
  fp2_sub(s0, s0, t1);
  fp2_sub(s0, s0, t2);
  fp2_mul_xi(s0, s0);
  fp2_add(c0, s0, t0);
  // c1 = (x0+x1)(y0+y1) - t0 - t1 + xi t2
  fp2_add(s0, x.c0, x.c1);
  fp2_add(s1, y.c0, y.c1);
  fp2_mul(s0, s0, s1);
  fp2_sub(s0, s0, t0);
  fp2_sub(s0, s0, t1);
  fp2_mul_xi(s1, t2);
  fp2_add(c1, s0, s1);
  // c2 = (x0+x2)(y0+y2) - t0 - t2 + t1
  fp2_add(s0, x.c0, x.c2);
  fp2_add(s1, y.c0, y.c2);
  fp2_mul(s0, s0, s1);
  fp2_sub(s0, s0, t0);
  fp2_sub(s0, s0, t2);
  fp2_add(c2, s0, t1);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
BN_HD void fp6_mul_v(fp6& r, const fp6& x) {  // x * v = (xi c2, c0, c1)
  fp2 t;
  fp2_mul_xi(t, x.c2);
  r.c2 = x.c1;
  r.c1 = x.c0;
  r.c0 = t;
}
BN_HD void fp6_mul_fp2(fp6& r, const fp6& x, const fp2& k) {
  fp2_mul(r.c0, x.c0, k);
  fp2_mul(r.c1, x.c1, k);
  fp2_mul(r.c2, x.c2, k);
}
BN_HD void fp6_mul_fp(fp6& r, const fp6& x, const fp& k) {
  fp2_mul_fp(r.c0, x.c0, k);
  fp2_mul_fp(r.c1, x.c1, k);
  fp2_mul_fp(r.c2, x.c2, k);
}
// x * (s0 + s1 v) (sparse, 5 Fp2 M)
BN_HDN void fp6_mul_01(fp6& r, const fp6& x, const fp2& s0, const fp2& s1) {
  fp2 t0, t1, u, w, c0, c1, c2;
  fp2_mul(t0, x.c0, s0);
  fp2_mul(t1, x.c1, s1);
  // c0 = t0 + xi * x2 s1
  fp2_mul(u, x.c2, s1);
  fp2_mul_xi(u, u);
  fp2_add(c0, t0, u);
  // c1 = (x0 + x1)(s0 + s1) - t0 - t1
  fp2_add(u, x.c0, x.c1);
  fp2_add(w, s0, s1);
  fp2_mul(u, u, w);
  fp2_sub(u, u, t0);
  fp2_sub(c1, u, t1);
  // c2 = x2 s0 + t1
  fp2_mul(u, x.c2, s0);
  fp2_add(c2, u, t1);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
template <bool VAR = false>
BN_HDN void fp6_inv(fp6& r, const fp6& x) {
  fp2 t0, t1, t2, u, v, n;
  // t0 = c0^2 - xi c1 c2, t1 = xi c2^2 - c0 c1, t2 = c1^2 - c0 c2
  fp2_sqr(t0, x.c0);
  fp2_mul(u, x.c1, x.c2);
  fp2_mul_xi(u, u);
  fp2_sub(t0, t0, u);
  fp2_sqr(t1, x.c2);
  fp2_mul_xi(t1, t1);
  fp2_mul(u, x.c0, x.c1);
  fp2_sub(t1, t1, u);
  fp2_sqr(t2, x.c1);
  fp2_mul(u, x.c0, x.c2);
  fp2_sub(t2, t2, u);
  // n = c0 t0 + xi (c2 t1 + c1 t2)
  fp2_mul(u, x.c2, t1);
  fp2_mul(v, x.c1, t2);
  fp2_add(u, u, v);
  fp2_mul_xi(u, u);
  fp2_mul(n, x.c0, t0);
  fp2_add(n, n, u);
  fp2_inv<VAR>(n, n);
  fp2_mul(r.c0, t0, n);
  fp2_mul(r.c1, t1, n);
  fp2_mul(r.c2, t2, n);
}

// ------------------------------------------------------------------------------ Fp12
BN_HD void fp12_one(fp12& r) {
  fp6_one(r.c0);
  fp6_zero(r.c1);
}
BN_HDN void fp12_mul(fp12& r, const fp12& x, const fp12& y) {  // 18 Fp2 M
  fp6 t0, t1, s0, s1;
  fp6_mul(t0, x.c0, y.c0);
  fp6_mul(t1, x.c1, y.c1);
  fp6_add(s0, x.c0, x.c1);
  fp6_add(s1, y.c0, y.c1);
  fp6_mul(s0, s0, s1);
  fp6_sub(s0, s0, t0);
  fp6_sub(r.c1, s0, t1);
  fp6_mul_v(t1, t1);
  fp6_add(r.c0, t0, t1);
}
BN_HDN void fp12_sqr(fp12& r, const fp12& x) {  // complex squaring, 12 Fp2 M
  fp6 t, s0, s1;
  fp6_mul(t, x.c0, x.c1);
  fp6_add(s0, x.c0, x.c1);
  fp6_mul_v(s1, x.c1);
  fp6_add(s1, s1, x.c0);
  fp6_mul(s0, s0, s1);  // (c0 + c1)(c0 + v c1) = c0^2 + v c1^2 + (1 + v) t
  fp6_sub(s0, s0, t);
  fp6_mul_v(s1, t);
  fp6_sub(r.c0, s0, s1);
  fp6_add(r.c1, t, t);
}
BN_HD void fp12_conj(fp12& r, const fp12& x) {
  r.c0 = x.c0;
  fp6_neg(r.c1, x.c1);
}
// Only the final exponentiations invert in Fp12, always of a Miller value computed from public
// inputs (signatures, hashes, keys), so the variable-time Fp inversion is used.
BN_HDN void fp12_inv(fp12& r, const fp12& x) {  // (c0 - c1 w) / (c0^2 - v c1^2)
  fp6 t0, t1;
  fp6_mul(t0, x.c0, x.c0);
  fp6_mul(t1, x.c1, x.c1);
  fp6_mul_v(t1, t1);
  fp6_sub(t0, t0, t1);
  fp6_inv<true>(t0, t0);
  fp6_mul(r.c0, x.c0, t0);
  fp6_mul(t1, x.c1, t0);
  fp6_neg(r.c1, t1);
}
BN_HDN bool fp12_is_one(const fp12& x) {
  fp2 one;
  fp2_one(one);
  return fp2_eq(x.c0.c0, one) && fp2_is_zero(x.c0.c1) && fp2_is_zero(x.c0.c2) && fp2_is_zero(x.c1.c0) &&
         fp2_is_zero(x.c1.c1) && fp2_is_zero(x.c1.c2);
}

// f * l for a D-type line l = y_P + (s) w + (mu) w^3, s, mu in Fp2, y_P in Fp:
//   l = L0 + L1 w with L0 = (yP, 0, 0), L1 = (s, mu, 0)
BN_HDN void fp12_mul_line(fp12& f, const fp& yP, const fp2& s, const fp2& mu) {
  fp6 a0L0, a1L1, t;
  fp6_mul_fp(a0L0, f.c0, yP);
  fp6_mul_01(a1L1, f.c1, s, mu);
  // c1 = (a0 + a1)(L0 + L1) - a0L0 - a1L1 ; L0 + L1 = (yP + s, mu, 0)
  fp2 s0;
  s0 = s;
  f_add(s0.a, s0.a, yP);
  fp6_add(t, f.c0, f.c1);
  fp6_mul_01(t, t, s0, mu);
  fp6_sub(t, t, a0L0);
  fp6_sub(f.c1, t, a1L1);
  fp6_mul_v(a1L1, a1L1);
  fp6_add(f.c0, a0L0, a1L1);
}

// Frobenius x -> x^(p^j), j = 1, 2, 3, on the basis e_k w^k, k = 0..5
// (e_0 = c0.c0, e_1 = c1.c0, e_2 = c0.c1, e_3 = c1.c1, e_4 = c0.c2, e_5 = c1.c2)
BN_HDN void fp12_frob(fp12& r, const fp12& x) {
  fp2 g;
  fp2_conj(r.c0.c0, x.c0.c0);
  fp2_conj(r.c1.c0, x.c1.c0);
  fp2_load(g, Bn254Consts::G1_1);
  fp2_mul(r.c1.c0, r.c1.c0, g);
  fp2_conj(r.c0.c1, x.c0.c1);
  fp2_load(g, Bn254Consts::G1_2);
  fp2_mul(r.c0.c1, r.c0.c1, g);
  fp2_conj(r.c1.c1, x.c1.c1);
  fp2_load(g, Bn254Consts::G1_3);
  fp2_mul(r.c1.c1, r.c1.c1, g);
  fp2_conj(r.c0.c2, x.c0.c2);
  fp2_load(g, Bn254Consts::G1_4);
  fp2_mul(r.c0.c2, r.c0.c2, g);
  fp2_conj(r.c1.c2, x.c1.c2);
  fp2_load(g, Bn254Consts::G1_5);
  fp2_mul(r.c1.c2, r.c1.c2, g);
}
BN_HDN void fp12_frob2(fp12& r, const fp12& x) {
  fp g;
  r.c0.c0 = x.c0.c0;
  fp_load(g, Bn254Consts::G2_1, 0);
  fp2_mul_fp(r.c1.c0, x.c1.c0, g);
  fp_load(g, Bn254Consts::G2_2, 0);
  fp2_mul_fp(r.c0.c1, x.c0.c1, g);
  fp_load(g, Bn254Consts::G2_3, 0);
  fp2_mul_fp(r.c1.c1, x.c1.c1, g);
  fp_load(g, Bn254Consts::G2_4, 0);
  fp2_mul_fp(r.c0.c2, x.c0.c2, g);
  fp_load(g, Bn254Consts::G2_5, 0);
  fp2_mul_fp(r.c1.c2, x.c1.c2, g);
}
BN_HDN void fp12_frob3(fp12& r, const fp12& x) {
  fp2 g;
  fp2_conj(r.c0.c0, x.c0.c0);
  fp2_conj(r.c1.c0, x.c1.c0);
  fp2_load(g, Bn254Consts::G3_1);
  fp2_mul(r.c1.c0, r.c1.c0, g);
  fp2_conj(r.c0.c1, x.c0.c1);
  fp2_load(g, Bn254Consts::G3_2);
  fp2_mul(r.c0.c1, r.c0.c1, g);
  fp2_conj(r.c1.c1, x.c1.c1);
  fp2_load(g, Bn254Consts::G3_3);
  fp2_mul(r.c1.c1, r.c1.c1, g);
  fp2_conj(r.c0.c2, x.c0.c2);
  fp2_load(g, Bn254Consts::G3_4);
  fp2_mul(r.c0.c2, r.c0.c2, g);
  fp2_conj(r.c1.c2, x.c1.c2);
  fp2_load(g, Bn254Consts::G3_5);
  fp2_mul(r.c1.c2, r.c1.c2, g);
}
