// Pairing check with one Fp12 spread over SIX lanes (gfx950 device code only).
//
// A single pairing check on one lane is a dependent chain of ~17 K Fp multiplications whose
// Fp12 temporaries do not fit in VGPRs (10 KB of scratch per lane): 26 ms on MI355X, which is
// the latency of a BLS certificate's final verify.  Here an 8-lane group owns one check; lane
// k = 0..5 holds coefficient e_k of f = sum_k e_k w^k in the w-basis of
// Fp12 = Fp2[w]/(w^6 - xi) (the tower's Fp6[w]/(w^2 - v) with v = w^2, so
// e_0 = c0.c0, e_1 = c1.c0, e_2 = c0.c1, e_3 = c1.c1, e_4 = c0.c2, e_5 = c1.c2 -- the basis of
// the Frobenius constants in bn254_consts.h).  Products gather the partner coefficients with
// ds_bpermute (__shfl) inside the group:
//   mul   c_k = sum_{i+j=k} a_i b_j + xi sum_{i+j=k+6} a_i b_j   6 Fp2 M per lane
//   sqr   the same sum folded by symmetry                       4 Fp2 M per lane
//   line  f * (yP + s w + mu w^3)                                1 Fp2xFp + 2 Fp2 M per lane
// so each Fp12 step costs a lane 3-4x fewer dependent multiplications than the one-lane tower
// code, and a lane's state is a few Fp2 (no scratch).  Lanes 6 and 7 shadow lane 0 (their
// results are discarded).  Results equal the one-lane pairing_check exactly (same GT element,
// same verdict): tests/test_bls_gpu.py compares both against the Python oracle.
#pragma once
#include "bn254_pairing.h"

struct P6 {
  int k;     // coefficient index 0..5 (lanes 6, 7 of the group act as 0)
  int base;  // first lane of the 8-lane group within the wave
};

__device__ __forceinline__ P6 p6_lane() {
  const int l = threadIdx.x & 63;
  P6 g;
  g.base = l & ~7;
  const int q = l & 7;
  g.k = q < 6 ? q : 0;
  return g;
}

__device__ __forceinline__ void fp2_shfl(fp2& r, const fp2& x, int src) {
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
    r.a.v[i] = (uint32_t)__shfl((int)x.a.v[i], src);
    r.b.v[i] = (uint32_t)__shfl((int)x.b.v[i], src);
  }
}

__device__ __forceinline__ void fp2_select(fp2& r, const fp2& x, bool c) {  // r = c ? x : r
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) {
    r.a.v[i] = c ? x.a.v[i] : r.a.v[i];
    r.b.v[i] = c ? x.b.v[i] : r.b.v[i];
  }
}

// r = a * b (both distributed)
__device__ __forceinline__ void p6_mul(fp2& r, const fp2& a, const fp2& b, const P6& g) {
  fp2 acc;
  fp2_zero(acc);
#pragma nounroll
  for (int i = 0; i < 6; i++) {
    int j = g.k - i;
    const bool wrap = j < 0;
    if (wrap) j += 6;
    fp2 ai, bj, t, tx;
    fp2_shfl(ai, a, g.base + i);
    fp2_shfl(bj, b, g.base + j);
    fp2_mul(t, ai, bj);
    fp2_mul_xi(tx, t);
    fp2_select(t, tx, wrap);
    fp2_add(acc, acc, t);
  }
  r = acc;
}

// Squaring terms per coefficient k: (i, j, flags) with i + j == k (mod 6);
// flags bit 0 = double (i != j), bit 1 = times xi (i + j >= 6), bit 2 = valid
__constant__ const uint8_t kP6Sq[6][4][3] = {
    {{0, 0, 4}, {3, 3, 6}, {1, 5, 7}, {2, 4, 7}},
    {{0, 1, 5}, {2, 5, 7}, {3, 4, 7}, {0, 0, 0}},
    {{1, 1, 4}, {4, 4, 6}, {0, 2, 5}, {3, 5, 7}},
    {{0, 3, 5}, {1, 2, 5}, {4, 5, 7}, {0, 0, 0}},
    {{2, 2, 4}, {5, 5, 6}, {0, 4, 5}, {1, 3, 5}},
    {{0, 5, 5}, {1, 4, 5}, {2, 3, 5}, {0, 0, 0}},
};

__device__ __forceinline__ void p6_sqr(fp2& r, const fp2& a, const P6& g) {
  fp2 acc;
  fp2_zero(acc);
#pragma nounroll  // unrolling measured no faster (share verify 4.06 vs 4.01 ms) and compiles slower
  for (int t = 0; t < 4; t++) {
    const int i = kP6Sq[g.k][t][0], j = kP6Sq[g.k][t][1], fl = kP6Sq[g.k][t][2];
    fp2 ai, aj, p, q;
    fp2_shfl(ai, a, g.base + i);
    fp2_shfl(aj, a, g.base + j);
    fp2_mul(p, ai, aj);
    fp2_add(q, p, p);
    fp2_select(p, q, (fl & 1) != 0);
    fp2_mul_xi(q, p);
    fp2_select(p, q, (fl & 2) != 0);
    fp2_add(q, acc, p);
    fp2_select(acc, q, (fl & 4) != 0);
  }
  r = acc;
}

// f <- f * (yP + s w + mu w^3): c_k = f_k yP + f_{k-1} s + f_{k-3} mu (xi on wrap-around)
__device__ __forceinline__ void p6_mul_line(fp2& f, const fp& yP, const fp2& s, const fp2& mu, const P6& g) {
  fp2 a1, a3, t0, t1, t3, tx;
  fp2_shfl(a1, f, g.base + (g.k + 5) % 6);
  fp2_shfl(a3, f, g.base + (g.k + 3) % 6);
  fp2_mul_fp(t0, f, yP);
  fp2_mul(t1, a1, s);
  fp2_mul_xi(tx, t1);
  fp2_select(t1, tx, g.k == 0);
  fp2_mul(t3, a3, mu);
  fp2_mul_xi(tx, t3);
  fp2_select(t3, tx, g.k < 3);
  fp2_add(f, t0, t1);
  fp2_add(f, f, t3);
}

__device__ __forceinline__ void p6_line_eval(fp2& f, const uint32_t* ln, const g1a& P, const P6& g) {
  fp2 lam, mu, s;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    lam.a.v[i] = ln[i];
    lam.b.v[i] = ln[9 + i];
    mu.a.v[i] = ln[18 + i];
    mu.b.v[i] = ln[27 + i];
  }
  fp2_mul_fp(s, lam, P.x);
  fp2_neg(s, s);
  p6_mul_line(f, P.y, s, mu, g);
}

__device__ __forceinline__ void p6_one(fp2& r, const P6& g) {
  fp2_zero(r);
  fp2 one;
  fp2_one(one);
  fp2_select(r, one, g.k == 0);
}

__device__ __forceinline__ void p6_conj(fp2& r, const fp2& x, const P6& g) {  // negate odd w powers
  fp2 n;
  fp2_neg(n, x);
  r = x;
  fp2_select(r, n, (g.k & 1) != 0);
}

// Frobenius x -> x^(p^J): e_k -> conj^J(e_k) * gamma_{J,k}; gamma_{J,0} = 1
template <int J>
__device__ __forceinline__ void p6_frob(fp2& r, const fp2& x, const P6& g) {
  fp2 c = x;
  if (J & 1) fp2_conj(c, x);
  fp2 gm, t;
  fp2_one(gm);
  if (J == 2) {  // Fp constants
    fp q;
    fp_load(q, Bn254Consts::G2_1, 0);
    if (g.k == 1) gm.a = q;
    fp_load(q, Bn254Consts::G2_2, 0);
    if (g.k == 2) gm.a = q;
    fp_load(q, Bn254Consts::G2_3, 0);
    if (g.k == 3) gm.a = q;
    fp_load(q, Bn254Consts::G2_4, 0);
    if (g.k == 4) gm.a = q;
    fp_load(q, Bn254Consts::G2_5, 0);
    if (g.k == 5) gm.a = q;
    if (g.k != 0) f_zero(gm.b);
  } else if (J == 1) {
    fp2_load(t, Bn254Consts::G1_1);
    fp2_select(gm, t, g.k == 1);
    fp2_load(t, Bn254Consts::G1_2);
    fp2_select(gm, t, g.k == 2);
    fp2_load(t, Bn254Consts::G1_3);
    fp2_select(gm, t, g.k == 3);
    fp2_load(t, Bn254Consts::G1_4);
    fp2_select(gm, t, g.k == 4);
    fp2_load(t, Bn254Consts::G1_5);
    fp2_select(gm, t, g.k == 5);
  } else {
    fp2_load(t, Bn254Consts::G3_1);
    fp2_select(gm, t, g.k == 1);
    fp2_load(t, Bn254Consts::G3_2);
    fp2_select(gm, t, g.k == 2);
    fp2_load(t, Bn254Consts::G3_3);
    fp2_select(gm, t, g.k == 3);
    fp2_load(t, Bn254Consts::G3_4);
    fp2_select(gm, t, g.k == 4);
    fp2_load(t, Bn254Consts::G3_5);
    fp2_select(gm, t, g.k == 5);
  }
  fp2_mul(r, c, gm);
}

// full element on every lane (tower layout) for the one-off inversion
__device__ __forceinline__ void p6_gather(fp12& f, const fp2& x, const P6& g) {
  fp2_shfl(f.c0.c0, x, g.base + 0);
  fp2_shfl(f.c1.c0, x, g.base + 1);
  fp2_shfl(f.c0.c1, x, g.base + 2);
  fp2_shfl(f.c1.c1, x, g.base + 3);
  fp2_shfl(f.c0.c2, x, g.base + 4);
  fp2_shfl(f.c1.c2, x, g.base + 5);
}
__device__ __forceinline__ void p6_pick(fp2& r, const fp12& f, const P6& g) {
  const fp2* e[6] = {&f.c0.c0, &f.c1.c0, &f.c0.c1, &f.c1.c1, &f.c0.c2, &f.c1.c2};
  r = f.c0.c0;
#pragma unroll
  for (int k = 1; k < 6; k++) fp2_select(r, *e[k], g.k == k);
}

__device__ __noinline__ void p6_inv(fp2& r, const fp2& x, const P6& g) {
  fp12 f, t;
  p6_gather(f, x, g);
  fp12_inv(t, f);
  p6_pick(r, t, g);
}

// x^2 for x in the cyclotomic subgroup of Fp12 (every value of the final exponentiation after
// its easy part), Granger-Scott: view f = A + B w + C w^2 over Fp4 = Fp2[t]/(t^2 - xi), t = w^3
// (A = e0 + e3 t, B = e1 + e4 t, C = e2 + e5 t); then
//   f^2 = (3A^2 - 2 conj A) + (3 t C^2 + 2 conj B) w + (3B^2 - 2 conj C) w^2
// (checked against the oracle's F12).  Each lane needs one half of one Fp4 square of a pair
// (x, y): P = x^2 + xi y^2 (even k) or Q = 2xy (odd k), formed uniformly from three Fp2 squares
// (x^2, y^2, (x + y)^2): 6 Fp multiplications and 2 gathers per lane instead of p6_sqr's 12 and 8.
__device__ __forceinline__ void p6_cyc_sqr(fp2& r, const fp2& a, const P6& g) {
  // sources of (x, y) per k: A for k = 0, 3; C for k = 4, 1; B for k = 2, 5
  const int sx = (g.k == 0 || g.k == 3) ? 0 : ((g.k == 1 || g.k == 4) ? 2 : 1);
  fp2 x, y, x2, y2, s, p, q;
  fp2_shfl(x, a, g.base + sx);
  fp2_shfl(y, a, g.base + sx + 3);
  fp2_sqr(x2, x);
  fp2_sqr(y2, y);
  fp2_add(s, x, y);
  fp2_sqr(s, s);
  fp2_mul_xi(p, y2);
  fp2_add(p, p, x2);  // P = x^2 + xi y^2
  fp2_sub(q, s, x2);
  fp2_sub(q, q, y2);  // Q = 2xy
  const bool odd = (g.k & 1) != 0;
  fp2_select(p, q, odd);
  fp2_mul_xi(q, p);
  fp2_select(p, q, g.k == 1);  // the t C^2 term: t (cx + cy t) = xi cy + cx t
  fp2 three, two;
  fp2_add(three, p, p);
  fp2_add(three, three, p);
  fp2_add(two, a, a);
  fp2 plus, minus;
  fp2_add(plus, three, two);
  fp2_sub(minus, three, two);
  r = minus;
  fp2_select(r, plus, odd);
}

// x^u for x in the cyclotomic subgroup: u = -(2^62 + 2^55 + 1)
__device__ __forceinline__ void p6_pow_u(fp2& r, const fp2& x, const P6& g) {
  fp2 acc = x;
#pragma nounroll
  for (int i = 61; i >= 0; i--) {
    p6_cyc_sqr(acc, acc, g);
    if (i == 55 || i == 0) p6_mul(acc, acc, x, g);
  }
  p6_conj(r, acc, g);
}

__device__ __forceinline__ void p6_pow_small(fp2& r, const fp2& x, uint32_t e, const P6& g) {
  fp2 acc = x;
  int top = 31;
  while (!((e >> top) & 1)) top--;
#pragma nounroll
  for (int i = top - 1; i >= 0; i--) {
    p6_cyc_sqr(acc, acc, g);
    if ((e >> i) & 1) p6_mul(acc, acc, x, g);
  }
  r = acc;
}

// f^((p^12 - 1)/r), same decomposition as final_exp (bn254_pairing.h)
__device__ __forceinline__ void p6_final_exp(fp2& r, const fp2& f, const P6& g) {
  fp2 t, gg;
  p6_inv(t, f, g);
  p6_conj(gg, f, g);
  p6_mul(gg, gg, t, g);
  p6_frob<2>(t, gg, g);
  p6_mul(gg, t, gg, g);
  fp2 a, b, c, c36, b6, b18, b30, a12, a18, g2;
  p6_pow_u(a, gg, g);
  p6_pow_u(b, a, g);
  p6_pow_u(c, b, g);
  p6_pow_small(c36, c, 36, g);
  p6_pow_small(b6, b, 6, g);
  p6_pow_small(b18, b6, 3, g);
  p6_mul(b30, b18, b6, g);
  p6_mul(b30, b30, b6, g);
  p6_pow_small(a12, a, 12, g);
  p6_pow_small(a18, a, 18, g);
  p6_cyc_sqr(g2, gg, g);
  fp2 t0, t1, t2, t3;
  p6_mul(t0, c36, b30, g);
  p6_mul(t0, t0, a18, g);
  p6_mul(t0, t0, g2, g);
  p6_conj(t0, t0, g);
  p6_mul(t1, c36, b18, g);
  p6_mul(t1, t1, a12, g);
  p6_conj(t1, t1, g);
  p6_mul(t1, t1, gg, g);
  p6_mul(t2, b6, gg, g);
  p6_frob<1>(t1, t1, g);
  p6_frob<2>(t2, t2, g);
  p6_frob<3>(t3, gg, g);
  p6_mul(t0, t0, t1, g);
  p6_mul(t0, t0, t2, g);
  p6_mul(r, t0, t3, g);
}

// prod_{j < np} e(P_j, Q_j) == 1 ?  Lines of Q_j precomputed (lines[j]); P_j not infinity.
// Every lane of the group returns the verdict.
template <int NP>
__device__ __forceinline__ bool p6_pairing_check(const g1a* P, const uint32_t* const* lines, const P6& g) {
  fp2 f;
  p6_one(f, g);
  int k = 0;
#pragma nounroll
  for (int i = BN_ATE_DBL - 1; i >= 0; i--) {
    p6_sqr(f, f, g);
#pragma unroll
    for (int j = 0; j < NP; j++) p6_line_eval(f, lines[j] + k * BN_LINE_WORDS, P[j], g);
    k++;
    if (bn_ate_bit(i)) {
#pragma unroll
      for (int j = 0; j < NP; j++) p6_line_eval(f, lines[j] + k * BN_LINE_WORDS, P[j], g);
      k++;
    }
  }
  p6_conj(f, f, g);
  for (int t = 0; t < 2; t++) {
#pragma unroll
    for (int j = 0; j < NP; j++) p6_line_eval(f, lines[j] + k * BN_LINE_WORDS, P[j], g);
    k++;
  }
  fp2 e;
  p6_final_exp(e, f, g);
  fp2 want;
  p6_one(want, g);
  const bool mine = fp2_eq(e, want);
  // AND over the 6 coefficient lanes of the group
  bool all = true;
#pragma unroll
  for (int q = 0; q < 6; q++) all = all && (__shfl((int)mine, g.base + q) != 0);
  return all;
}
