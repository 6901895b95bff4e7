// Pairing check with one Fp12 spread over TWELVE lanes (gfx950 device code only).
//
// A pairing check's latency is one lane's instruction stream: with the 6-lane layout
// (bn254_pair6.h, one Fp2 coefficient e_k of f = sum_k e_k w^k per lane) a lone wave issued
// ~2.0 M VALU instructions per check (rocprofv3 PMC, bls_verify_kernel), about half of them at the
// issue limit.  Here each Fp2 coefficient is split over a lane PAIR: lane 2k + h of a 16-lane group
// holds component h (0 = real, 1 = imaginary) of e_k, so every Fp2 product costs a lane two Fp
// multiplications instead of three (schoolbook halves: h = 0 forms a0 b0 - a1 b1, h = 1 forms
// a0 b1 + a1 b0), an Fp2 square one instead of two, and additions one instead of two:
//   mul        6 split products per lane (12 Fp M; 18 in the 6-lane layout)
//   sqr        4 products per lane (8 Fp M; 12)
//   cyc_sqr    3 split squares per lane (3 Fp M; 6)             -- Granger-Scott, as p6_cyc_sqr
//   line       yP, lambda, mu terms (6 Fp M; 10)
// Partner components move with ds_bpermute (__shfl) inside the group; xi = 1 + i multiplications
// of a split value need the partner's component too (one extra gather).  Lanes 12..15 of a group
// shadow lanes 0..3 (results discarded).  Results equal the 6-lane and one-lane pairing checks
// exactly (same GT element; tests/test_bls_gpu.py against the Python oracle).
#pragma once
#include "bn254_pairing.h"

struct P12 {
  int k;     // coefficient 0..5
  int h;     // component: 0 = real, 1 = imaginary
  int base;  // first lane of the 16-lane group within the wave
  int lane;  // this lane's index within the wave
};

__device__ __forceinline__ P12 p12_lane() {
  P12 g;
  g.lane = threadIdx.x & 63;
  g.base = g.lane & ~15;
  const int q = g.lane & 15;
  const int e = q < 12 ? q : q - 12;
  g.k = e >> 1;
  g.h = e & 1;
  return g;
}

__device__ __forceinline__ void fp_shfl(fp& r, const fp& x, int src) {
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) r.v[i] = (uint32_t)__shfl((int)x.v[i], src);
}
__device__ __forceinline__ void fp_sel(fp& r, const fp& x, bool c) {  // r = c ? x : r
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) r.v[i] = c ? x.v[i] : r.v[i];
}
__device__ __forceinline__ void p12_sel2(fp2& r, const fp2& x, bool c) {
  fp_sel(r.a, x.a, c);
  fp_sel(r.b, x.b, c);
}
// component h2 of coefficient k2 (its lane in the group)
__device__ __forceinline__ int p12_src(const P12& g, int k2, int h2) { return g.base + 2 * k2 + h2; }

// my component of x * y, given my and the other component of each (xm, xo, ym, yo)
__device__ __forceinline__ void p12_cmul(fp& r, const fp& xm, const fp& xo, const fp& ym, const fp& yo, int h) {
  fp u = h ? xo : xm, v = h ? xm : xo, t1, t2;
  f_mul(t1, u, ym);
  f_mul(t2, v, yo);
  f_addsub(r, t1, t2, h != 0);
}
// my component of x^2 (xm, xo): h = 0: (x0 + x1)(x0 - x1); h = 1: 2 x0 x1
__device__ __forceinline__ void p12_csqr(fp& r, const fp& xm, const fp& xo, int h) {
  fp a, b, t;
  f_add(a, xm, xo);
  f_sub(b, xm, xo);
  fp u = h ? xm : a, v = h ? xo : b;
  f_mul(t, u, v);
  fp t2;
  f_add(t2, t, t);
  r = h ? t2 : t;
}
// my component of xi * z from my and the other component: h = 0: z0 - z1; h = 1: z0 + z1
__device__ __forceinline__ void p12_cxi(fp& r, const fp& zm, const fp& zo, int h) { f_addsub(r, zm, zo, h != 0); }
__device__ __forceinline__ void p12_xi(fp& r, const fp& z, const P12& g) {
  fp zo;
  fp_shfl(zo, z, g.lane ^ 1);
  p12_cxi(r, z, zo, g.h);
}

// r = a * b (both distributed): c_k = sum_{i+j=k} a_i b_j + xi sum_{i+j=k+6} a_i b_j
__device__ __forceinline__ void p12_mul(fp& r, const fp& a, const fp& b, const P12& g) {
  fp acc, accw;
  f_zero(acc);
  f_zero(accw);
#pragma nounroll
  for (int i = 0; i < 6; i++) {
    int j = g.k - i;
    const bool wrap = j < 0;
    if (wrap) j += 6;
    fp am, ao, bm, bo, t, s;
    fp_shfl(am, a, p12_src(g, i, g.h));
    fp_shfl(ao, a, p12_src(g, i, 1 - g.h));
    fp_shfl(bm, b, p12_src(g, j, g.h));
    fp_shfl(bo, b, p12_src(g, j, 1 - g.h));
    p12_cmul(t, am, ao, bm, bo, g.h);
    f_add(s, wrap ? accw : acc, t);
    fp_sel(acc, s, !wrap);
    fp_sel(accw, s, wrap);
  }
  fp w;
  p12_xi(w, accw, g);
  f_add(r, acc, w);
}

// Squaring terms per coefficient (same table as bn254_pair6.h): (i, j, flags) with
// i + j == k (mod 6); flags bit 0 = double (i != j), bit 1 = times xi, bit 2 = valid
__constant__ const uint8_t kP12Sq[6][4][3] = {
    {{0, 0, 4}, {3, 3, 6}, {1, 5, 7}, {2, 4, 7}},
    {{0, 1, 5}, {2, 5, 7}, {3, 4, 7}, {0, 0, 0}},
    {{1, 1, 4}, {4, 4, 6}, {0, 2, 5}, {3, 5, 7}},
    {{0, 3, 5}, {1, 2, 5}, {4, 5, 7}, {0, 0, 0}},
    {{2, 2, 4}, {5, 5, 6}, {0, 4, 5}, {1, 3, 5}},
    {{0, 5, 5}, {1, 4, 5}, {2, 3, 5}, {0, 0, 0}},
};

__device__ __forceinline__ void p12_sqr(fp& r, const fp& a, const P12& g) {
  fp acc, accw;
  f_zero(acc);
  f_zero(accw);
#pragma nounroll
  for (int t = 0; t < 4; t++) {
    const int i = kP12Sq[g.k][t][0], j = kP12Sq[g.k][t][1], fl = kP12Sq[g.k][t][2];
    fp im, io, jm, jo, p, q;
    fp_shfl(im, a, p12_src(g, i, g.h));
    fp_shfl(io, a, p12_src(g, i, 1 - g.h));
    fp_shfl(jm, a, p12_src(g, j, g.h));
    fp_shfl(jo, a, p12_src(g, j, 1 - g.h));
    p12_cmul(p, im, io, jm, jo, g.h);
    f_add(q, p, p);
    fp_sel(p, q, (fl & 1) != 0);
    if (!(fl & 4)) f_zero(p);
    const bool wrap = (fl & 2) != 0;
    f_add(q, wrap ? accw : acc, p);
    fp_sel(acc, q, !wrap);
    fp_sel(accw, q, wrap);
  }
  fp w;
  p12_xi(w, accw, g);
  f_add(r, acc, w);
}

// Granger-Scott cyclotomic squaring (see p6_cyc_sqr): lane (k, h) forms its component of
// P = x^2 + xi y^2 (even k) or Q = 2xy (odd k) from three split squares, then 3 (P|Q) -+ 2 e_k
// (xi (.) once more for k = 1).
__device__ __forceinline__ void p12_cyc_sqr(fp& r, const fp& a, const P12& g) {
  const int sx = (g.k == 0 || g.k == 3) ? 0 : ((g.k == 1 || g.k == 4) ? 2 : 1);
  fp xm, xo, ym, yo, x2, y2, s2, sm, so;
  fp_shfl(xm, a, p12_src(g, sx, g.h));
  fp_shfl(xo, a, p12_src(g, sx, 1 - g.h));
  fp_shfl(ym, a, p12_src(g, sx + 3, g.h));
  fp_shfl(yo, a, p12_src(g, sx + 3, 1 - g.h));
  p12_csqr(x2, xm, xo, g.h);
  p12_csqr(y2, ym, yo, g.h);
  f_add(sm, xm, ym);
  f_add(so, xo, yo);
  p12_csqr(s2, sm, so, g.h);
  fp xy2, p, q;
  p12_xi(xy2, y2, g);
  f_add(p, x2, xy2);  // P = x^2 + xi y^2
  f_sub(q, s2, x2);
  f_sub(q, q, y2);  // Q = 2xy
  const bool odd = (g.k & 1) != 0;
  fp_sel(p, q, odd);
  fp_shfl(q, p, g.lane ^ 1);  // (xi p for k = 1: every lane gathers, so the shuffle is uniform)
  fp px;
  p12_cxi(px, p, q, g.h);
  fp_sel(p, px, g.k == 1);
  fp three, two;
  f_add(three, p, p);
  f_add(three, three, p);
  f_add(two, a, a);
  f_addsub(r, three, two, odd);
}

// f <- f * (yP + s w + mu w^3) with s = -lambda xP: c_k = f_k yP - xP f_{k-1} lambda + f_{k-3} mu
// (xi on wrap-around: k - 1 < 0 for k = 0, k - 3 < 0 for k < 3)
__device__ __forceinline__ void p12_line_eval(fp& f, const uint32_t* ln, const g1a& P, const P12& g) {
  fp lm, lo, mm, mo;  // lambda, mu: my and the other component
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint32_t l0 = ln[i], l1 = ln[9 + i], m0 = ln[18 + i], m1 = ln[27 + i];
    lm.v[i] = g.h ? l1 : l0;
    lo.v[i] = g.h ? l0 : l1;
    mm.v[i] = g.h ? m1 : m0;
    mo.v[i] = g.h ? m0 : m1;
  }
  const int k1 = (g.k + 5) % 6, k3 = (g.k + 3) % 6;
  fp f1m, f1o, f3m, f3o, t0, t1, t3, w;
  fp_shfl(f1m, f, p12_src(g, k1, g.h));
  fp_shfl(f1o, f, p12_src(g, k1, 1 - g.h));
  fp_shfl(f3m, f, p12_src(g, k3, g.h));
  fp_shfl(f3o, f, p12_src(g, k3, 1 - g.h));
  f_mul(t0, f, P.y);
  p12_cmul(t1, f1m, f1o, lm, lo, g.h);
  f_mul(t1, t1, P.x);
  f_neg(t1, t1);
  p12_cmul(t3, f3m, f3o, mm, mo, g.h);
  p12_xi(w, t1, g);
  fp_sel(t1, w, g.k == 0);
  p12_xi(w, t3, g);
  fp_sel(t3, w, g.k < 3);
  f_add(f, t0, t1);
  f_add(f, f, t3);
}

__device__ __forceinline__ void p12_one(fp& r, const P12& g) {
  f_zero(r);
  fp one;
  f_one(one);
  fp_sel(r, one, g.k == 0 && g.h == 0);
}

__device__ __forceinline__ void p12_conj(fp& r, const fp& x, const P12& g) {  // negate odd w powers
  fp n;
  f_neg(n, x);
  r = x;
  fp_sel(r, n, (g.k & 1) != 0);
}

// Frobenius x -> x^(p^J): e_k -> conj^J(e_k) * gamma_{J,k} (bn254_consts.h); gamma_{J,0} = 1
template <int J>
__device__ __forceinline__ void p12_frob(fp& r, const fp& x, const P12& g) {
  fp c = x;
  if (J & 1) {  // conjugate: negate the imaginary component
    fp n;
    f_neg(n, x);
    fp_sel(c, n, g.h == 1);
  }
  if (J == 2) {  // constants in Fp: component-wise
    fp q, gm;
    f_one(gm);
    fp_load(q, Bn254Consts::G2_1, 0);
    fp_sel(gm, q, g.k == 1);
    fp_load(q, Bn254Consts::G2_2, 0);
    fp_sel(gm, q, g.k == 2);
    fp_load(q, Bn254Consts::G2_3, 0);
    fp_sel(gm, q, g.k == 3);
    fp_load(q, Bn254Consts::G2_4, 0);
    fp_sel(gm, q, g.k == 4);
    fp_load(q, Bn254Consts::G2_5, 0);
    fp_sel(gm, q, g.k == 5);
    f_mul(r, c, gm);
    return;
  }
  fp2 gm, t;
  fp2_one(gm);
  if (J == 1) {
    fp2_load(t, Bn254Consts::G1_1);
    p12_sel2(gm, t, g.k == 1);
    fp2_load(t, Bn254Consts::G1_2);
    p12_sel2(gm, t, g.k == 2);
    fp2_load(t, Bn254Consts::G1_3);
    p12_sel2(gm, t, g.k == 3);
    fp2_load(t, Bn254Consts::G1_4);
    p12_sel2(gm, t, g.k == 4);
    fp2_load(t, Bn254Consts::G1_5);
    p12_sel2(gm, t, g.k == 5);
  } else {
    fp2_load(t, Bn254Consts::G3_1);
    p12_sel2(gm, t, g.k == 1);
    fp2_load(t, Bn254Consts::G3_2);
    p12_sel2(gm, t, g.k == 2);
    fp2_load(t, Bn254Consts::G3_3);
    p12_sel2(gm, t, g.k == 3);
    fp2_load(t, Bn254Consts::G3_4);
    p12_sel2(gm, t, g.k == 4);
    fp2_load(t, Bn254Consts::G3_5);
    p12_sel2(gm, t, g.k == 5);
  }
  fp co;
  fp_shfl(co, c, g.lane ^ 1);
  fp gmm = g.h ? gm.b : gm.a, gmo = g.h ? gm.a : gm.b;
  p12_cmul(r, c, co, gmm, gmo, g.h);
}

// the whole element on every lane (tower layout) for the one-off inversion
__device__ __forceinline__ void p12_gather2(fp2& e, const fp& x, const P12& g, int k) {
  fp_shfl(e.a, x, p12_src(g, k, 0));
  fp_shfl(e.b, x, p12_src(g, k, 1));
}
__device__ __noinline__ void p12_inv(fp& r, const fp& x, const P12& g) {
  fp12 f, t;
  p12_gather2(f.c0.c0, x, g, 0);
  p12_gather2(f.c1.c0, x, g, 1);
  p12_gather2(f.c0.c1, x, g, 2);
  p12_gather2(f.c1.c1, x, g, 3);
  p12_gather2(f.c0.c2, x, g, 4);
  p12_gather2(f.c1.c2, x, g, 5);
  fp12_inv(t, f);
  const fp2* e[6] = {&t.c0.c0, &t.c1.c0, &t.c0.c1, &t.c1.c1, &t.c0.c2, &t.c1.c2};
  fp2 pick = t.c0.c0;
#pragma unroll
  for (int k = 1; k < 6; k++) p12_sel2(pick, *e[k], g.k == k);
  r = g.h ? pick.b : pick.a;
}

// x^u for x in the cyclotomic subgroup: u = -(2^62 + 2^55 + 1)
__device__ __forceinline__ void p12_pow_u(fp& r, const fp& x, const P12& g) {
  fp acc = x;
#pragma nounroll
  for (int i = 61; i >= 0; i--) {
    p12_cyc_sqr(acc, acc, g);
    if (i == 55 || i == 0) p12_mul(acc, acc, x, g);
  }
  p12_conj(r, acc, g);
}

__device__ __forceinline__ void p12_pow_small(fp& r, const fp& x, uint32_t e, const P12& g) {
  fp acc = x;
  int top = 31;
  while (!((e >> top) & 1)) top--;
#pragma nounroll
  for (int i = top - 1; i >= 0; i--) {
    p12_cyc_sqr(acc, acc, g);
    if ((e >> i) & 1) p12_mul(acc, acc, x, g);
  }
  r = acc;
}

// f^((p^12 - 1)/r), the decomposition of p6_final_exp / final_exp
__device__ __forceinline__ void p12_final_exp(fp& r, const fp& f, const P12& g) {
  fp t, gg;
  p12_inv(t, f, g);
  p12_conj(gg, f, g);
  p12_mul(gg, gg, t, g);
  p12_frob<2>(t, gg, g);
  p12_mul(gg, t, gg, g);
  fp a, b, c, c36, b6, b18, b30, a12, a18, g2;
  p12_pow_u(a, gg, g);
  p12_pow_u(b, a, g);
  p12_pow_u(c, b, g);
  p12_pow_small(c36, c, 36, g);
  p12_pow_small(b6, b, 6, g);
  p12_pow_small(b18, b6, 3, g);
  p12_mul(b30, b18, b6, g);
  p12_mul(b30, b30, b6, g);
  p12_pow_small(a12, a, 12, g);
  p12_pow_small(a18, a, 18, g);
  p12_cyc_sqr(g2, gg, g);
  fp t0, t1, t2, t3;
  p12_mul(t0, c36, b30, g);
  p12_mul(t0, t0, a18, g);
  p12_mul(t0, t0, g2, g);
  p12_conj(t0, t0, g);
  p12_mul(t1, c36, b18, g);
  p12_mul(t1, t1, a12, g);
  p12_conj(t1, t1, g);
  p12_mul(t1, t1, gg, g);
  p12_mul(t2, b6, gg, g);
  p12_frob<1>(t1, t1, g);
  p12_frob<2>(t2, t2, g);
  p12_frob<3>(t3, gg, g);
  p12_mul(t0, t0, t1, g);
  p12_mul(t0, t0, t2, g);
  p12_mul(r, t0, t3, g);
}

// prod_{j < np} e(P_j, Q_j) == 1 ?  Lines of Q_j precomputed (lines[j]); P_j not infinity.
// Every lane of the 16-lane group returns the verdict.
template <int NP>
__device__ __forceinline__ bool p12_pairing_check(const g1a* P, const uint32_t* const* lines, const P12& g) {
  fp f;
  p12_one(f, g);
  int k = 0;
#pragma nounroll
  for (int i = BN_ATE_DBL - 1; i >= 0; i--) {
    p12_sqr(f, f, g);
#pragma unroll
    for (int j = 0; j < NP; j++) p12_line_eval(f, lines[j] + k * BN_LINE_WORDS, P[j], g);
    k++;
    if (bn_ate_bit(i)) {
#pragma unroll
      for (int j = 0; j < NP; j++) p12_line_eval(f, lines[j] + k * BN_LINE_WORDS, P[j], g);
      k++;
    }
  }
  p12_conj(f, f, g);
  for (int t = 0; t < 2; t++) {
#pragma unroll
    for (int j = 0; j < NP; j++) p12_line_eval(f, lines[j] + k * BN_LINE_WORDS, P[j], g);
    k++;
  }
  fp e;
  p12_final_exp(e, f, g);
  fp want;
  p12_one(want, g);
  const bool mine = f_eq(e, want);
  bool all = true;
#pragma unroll
  for (int q = 0; q < 12; q++) all = all && (__shfl((int)mine, g.base + q) != 0);
  return all;
}
