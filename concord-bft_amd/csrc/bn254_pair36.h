// Pairing check with one Fp12 spread over a whole wave (gfx950 device code only).
//
// Latency of one pairing check is the instruction stream of one lane.  bn254_pair12.h gives
// each of the 12 Fp components of f = sum_k e_k w^k (e_k in Fp2) its own lane; here every
// component gets THREE lanes (sub-lanes s = 0, 1, 2; lane 12 s + 2 k + h holds component h of
// e_k, lanes 36..63 shadow lanes 0..27) and the products an Fp12 operation needs are dealt out
// to the sub-lanes, then summed.  The other component of a lane's coefficient sits in the partner
// lane (lane ^ 1): a DPP quad_perm move; the coefficient fetches and the sub-lane sums are
// ds_bpermute gathers.  (Sub-lane s in DPP row s, the sub-lane sum one permlane gather, measured
// 1.3 % (verify) to 2 % (multisig verify) slower than the bpermute sums.)
//   op          Fp mults per lane   (bn254_pair12.h)
//   mul         4                   12    6 split products per component, 2 per sub-lane
//   sqr         2                    8    even k: two diagonal squares on s = 0, one cross
//                                         term on s = 1, 2; odd k: one cross term per sub-lane
//   cyc_sqr     1                    3    x^2, y^2, (x + y)^2 on s = 0, 1, 2 (Granger-Scott)
//   line        3                    6    f_k yP | xP (f_{k-1} lambda) | f_{k-3} mu
// All three sub-lanes of a component end every operation with the same bits (the sub-lane
// partials are summed in the order s = 0, 1, 2 on every lane), so the state is replicated and
// any sub-lane can serve a gather.  Results equal the 12-lane and one-lane pairing checks
// exactly (same GT element; tests/test_bls_gpu.py and tests/test_relic_gpu.py against the
// Python oracle).
#pragma once
#include "bn254_cycsq.h"
#include "bn254_pair12.h"
#include "row_lanes.h"

struct P36 {
  int k;     // coefficient 0..5
  int h;     // component: 0 = real, 1 = imaginary
  int s;     // sub-lane 0..2
  int lane;  // lane within the wave
  int e;     // 12 s + 2 k + h: the lane's slot among the 36 (Miller value exchange)
  bool own;  // not a shadow: the lane owning slot e
};

__device__ __forceinline__ P36 p36_lane() {
  P36 g;
  g.lane = threadIdx.x & 63;
  const int e = g.lane < 36 ? g.lane : g.lane - 36;
  const int c = e % 12;
  g.s = e / 12;
  g.own = g.lane < 36;
  g.k = c >> 1;
  g.h = c & 1;
  g.e = 12 * g.s + c;
  return g;
}

__device__ __forceinline__ int p36_src(int k2, int h2, int s2) {
  return 12 * s2 + 2 * k2 + h2;
}

// (q0, q1, q2) = part of sub-lanes 0, 1, 2 of this lane's component
__device__ __forceinline__ void p36_gather3(fp& q0, fp& q1, fp& q2, const fp& part, const P36& g) {
  fp_shfl(q0, part, p36_src(g.k, g.h, 0));
  fp_shfl(q1, part, p36_src(g.k, g.h, 1));
  fp_shfl(q2, part, p36_src(g.k, g.h, 2));
}

// r = x of the partner lane (same k and s, the other component h): lane ^ 1, shadows included, as a
// DPP quad_perm [1, 0, 3, 2] move instead of a ds_bpermute
__device__ __forceinline__ void fp_swap_h(fp& r, const fp& x, const P36& g) {
  (void)g;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)x.v[i], 0xB1, 0xF, 0xF, false);
}

// (my component, the other component) of coefficient k2 of x.  The partner lane fetches the same
// coefficient (k2 depends on k and s only), so its result is my other component.
__device__ __forceinline__ void p36_fetch(fp& m, fp& o, const fp& x, int k2, const P36& g) {
  fp_shfl(m, x, p36_src(k2, g.h, g.s));
  fp_swap_h(o, m, g);
}

// r = sum over the three sub-lanes of component (k, h) of part, in the order 0, 1, 2: one limb-wise
// three-term sum (< 6q), one carry pass and fp_reduce64 (two reduced additions would each pay their
// own conditional 2q subtraction and wave vote)
__device__ __forceinline__ void p36_sum3(fp& r, const fp& part, const P36& g) {
  fp q0, q1, q2;
  p36_gather3(q0, q1, q2, part, g);
  fp x;
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) x.v[i] = q0.v[i] + q1.v[i] + q2.v[i];  // inputs < 2q, normalised
  cs_carry(x);
  fp_reduce64(r, x);
}

// my component of xi * z, z held componentwise by this lane and its partner (same k, s)
__device__ __forceinline__ void p36_xi(fp& r, const fp& z, const P36& g) {
  fp zo;
  fp_swap_h(zo, z, g);
  p12_cxi(r, z, zo, g.h);
}

struct P36Const {
  static constexpr CsLimbs Q4N = cs_redundant(4, 1 << 29);  // 4q, low limbs in [2^29, 2^30): 4q - v >= 0 limb-wise
};
// v' = -v (as 4q - v) where neg, else v
__device__ __forceinline__ void p36_cneg4(fp& r, const fp& v, bool neg) {
  const uint32_t m = cs_mask(neg);
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) r.v[i] = cs_sel(m, P36Const::Q4N.v[i] - v.v[i], v.v[i]);
}

// r = a * b: sub-lane s forms the terms i = 2s, 2s + 1 of c_k = sum_i a_i b_{k-i} (xi on wrap);
// lazy sums and one reduction (bn254_cycsq.h: cm_terms, cm_xi, cm_sum3).  Each term's Fp2-product
// component u b_m +- v b_o is ONE two-product reduction (f_mul_sum2, v negated beforehand on the
// h = 0 lanes, as the lines): two reductions per lane instead of four; cm_terms then only sums
// (h = 1, zero second terms).
__device__ __forceinline__ void p36_mul(fp& r, const fp& a, const fp& b, const P36& g) {
  fp T[4];
  bool wrap[2];
#pragma unroll
  for (int t = 0; t < 2; t++) {
    const int i = 2 * g.s + t;
    int j = g.k - i;
    wrap[t] = j < 0;
    if (wrap[t]) j += 6;
    fp am, ao, bm, bo;
    p36_fetch(am, ao, a, i, g);
    p36_fetch(bm, bo, b, j, g);
    const fp u = g.h ? ao : am, v = g.h ? am : ao;
    fp vn;
    p36_cneg4(vn, v, g.h == 0);
    f_mul_sum2(T[2 * t], u, bm, vn, bo);
    f_zero(T[2 * t + 1]);
  }
  fp acc, accw, ao, z, z0, z1, z2;
  cm_terms(acc, accw, T[0], T[1], T[2], T[3], 1, wrap[0], wrap[1]);
  fp_swap_h(ao, accw, g);
  cm_xi(z, acc, accw, ao, g.h);
  p36_gather3(z0, z1, z2, z, g);
  cm_sum3(r, z0, z1, z2);
}

// r = a^2 (the term table kP12Sq of bn254_pair12.h).  Even k: s = 0 squares the two diagonal
// terms (a_i^2, one component each: (x0 + x1)(x0 - x1) or 2 x0 x1), s = 1, 2 the cross terms
// 2 a_i a_j; odd k: one cross term per sub-lane.  Two multiplications per lane.
__device__ __forceinline__ void p36_sqr(fp& r, const fp& a, const P36& g) {
  const bool even = (g.k & 1) == 0;
  const bool diag = even && g.s == 0;
  const int tt = even ? g.s + 1 : g.s;  // cross term index
  const int f1 = diag ? kP12Sq[g.k][0][0] : kP12Sq[g.k][tt][0];
  const int f2 = diag ? kP12Sq[g.k][1][0] : kP12Sq[g.k][tt][1];
  const bool cwrap = (kP12Sq[g.k][tt][2] & 2) != 0;
  fp xm, xo, zm, zo;
  p36_fetch(xm, xo, a, f1, g);
  p36_fetch(zm, zo, a, f2, g);
  // lazy form (bn254_cycsq.h: sq_operands, then p36_mul's cm_* stages)
  fp U1, V1, U2, V2, P1, P2;
  sq_operands(U1, V1, U2, V2, xm, xo, zm, zo, diag, g.h);
  f_mul(P1, U1, V1);
  f_mul(P2, U2, V2);
  fp zero, acc, accw, ao, z, z0, z1, z2;
  f_zero(zero);
  // diag: x^2 term -> acc, z^2 term -> accw (the second diagonal term wraps); cross: P1 +- P2
  cm_terms(acc, accw, P1, diag ? zero : P2, diag ? P2 : zero, zero, g.h, !diag && cwrap, true);
  fp_swap_h(ao, accw, g);
  cm_xi(z, acc, accw, ao, g.h);
  p36_gather3(z0, z1, z2, z, g);
  cm_sum3(r, z0, z1, z2);
}

// Granger-Scott cyclotomic squaring (p6_cyc_sqr's formulas): s = 0, 1, 2 square x, y, x + y
// (one component each), then P = x^2 + xi y^2 (even k) or Q = (x + y)^2 - x^2 - y^2 (odd k)
__device__ __forceinline__ void p36_cyc_sqr(fp& r, const fp& a, const P36& g) {
  // lazy form (bn254_cycsq.h): 4 gathers of 9 limbs, one Fp multiplication, one reduction
  const int k3 = g.k >= 3 ? g.k - 3 : g.k;  // sx = 0, 2, 1 for k mod 3 = 0, 1, 2 (arithmetic, no branch)
  const int sx = k3 == 0 ? 0 : 3 - k3;
  const bool odd = (g.k & 1) != 0;
  fp t, R, Wm, Wo, U, V, T, X2, Y2, G3, v, vo, Z3;
  fp_shfl(t, a, p36_src(g.k < 3 ? g.k + 3 : g.k - 3, g.h, g.s));
  cs_pre(R, a, t, g.s);
  const int c = g.s == 1 ? sx + 3 : sx;
  fp_shfl(Wm, R, p36_src(c, g.h, g.s));
  fp_swap_h(Wo, Wm, g);
  cs_operands(U, V, Wm, Wo, g.h);
  f_mul(T, U, V);
  // (x+y)^2_h (odd k) | y^2_h' (even k: the partner's sub-lane 1)
  fp_shfl(X2, T, p36_src(g.k, g.h, 0));
  fp_shfl(Y2, T, p36_src(g.k, g.h, 1));
  fp_shfl(G3, T, odd ? p36_src(g.k, g.h, 2) : p36_src(g.k, 1 - g.h, 1));
  (void)Z3;
  cs_combine(v, X2, Y2, G3, g.k, g.h);
  fp_swap_h(vo, v, g);
  cs_finish(r, v, vo, a, g.k, g.h);
}

__device__ __forceinline__ void p36_coef(fp& m, fp& o, const uint32_t* c, int h) {
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint32_t x0 = c[i], x1 = c[9 + i];
    m.v[i] = h ? x1 : x0;
    o.v[i] = h ? x0 : x1;
  }
}

// f <- f * (yP + s w + mu w^3), s = -lambda xP, for one precomputed line:
//   s = 0: f_k yP;  s = 1: -xP (f_{k-1} lambda) (xi for k = 0);  s = 2: f_{k-3} mu (xi for k < 3)
// this lane's (my, other) components of the line coefficient it multiplies by (lambda for s < 2,
// mu for s = 2): the line's global-memory read
__device__ __forceinline__ void p36_line_coef(fp& cm, fp& co, const uint32_t* ln, const P36& g) {
  p36_coef(cm, co, ln + (g.s == 2 ? 18 : 0), g.h);
}

// A line's component C = u c_m +- v c_o (the Fp2 product's component h) is ONE two-product
// reduction (f_mul_sum2) with v negated beforehand (4q - v, redundant limbs, on the h = 0 lanes)
// instead of two f_mul and f_addsub; s = 0 lanes zero their second product.
// P: the G1 point with its x NEGATED (p36_neg_x), so the s = 1 term -xP (f_{k-1} lambda) is one
// product; the Miller loops negate once, before their first line.
__device__ __forceinline__ g1a p36_neg_x(const g1a& P) {
  g1a n = P;
  f_neg(n.x, P.x);
  return n;
}
__device__ __forceinline__ void p36_line1c(fp& f, const fp& cm, const fp& co, const g1a& P, const P36& g) {
  fp om, oo;
  p36_fetch(om, oo, f, g.s == 1 ? (g.k + 5) % 6 : (g.k + 3) % 6, g);
  const fp u = g.h ? oo : om, v = g.h ? om : oo;
  fp X1 = g.s == 0 ? f : u;
  fp Y1 = g.s == 0 ? P.y : cm;
  fp P3, C;
  fp vn, cz;
  p36_cneg4(vn, v, g.h == 0);
  const uint32_t mz = cs_mask(g.s != 0);
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) cz.v[i] = co.v[i] & mz;
  f_mul_sum2(C, X1, Y1, vn, cz);  // s = 0: f_k yP; else u c_m +- v c_o
  f_mul(P3, C, P.x);              // P.x holds -xP (p36_line1: the caller negates once per loop)
  fp T = C;
  fp_sel(T, P3, g.s == 1);
  const bool wrap = (g.s == 1 && g.k == 0) || (g.s == 2 && g.k < 3);
  fp w;
  p36_xi(w, T, g);
  fp_sel(T, w, wrap);
  p36_sum3(f, T, g);
}

__device__ __forceinline__ void p36_line1(fp& f, const uint32_t* ln, const g1a& P, const P36& g) {
  fp cm, co;
  p36_line_coef(cm, co, ln, g);
  p36_line1c(f, cm, co, P, g);
}

// Lambda records: with LDS room (lx) the Miller loops first form lambda' = -xP lambda for every
// normalised line they will read (p36_lambda_x: 140 Fp products per pair over the wave's 64 lanes,
// into LDS); a line's s = 1 term -xP (f_{k-1} lambda) = f_{k-1} lambda' is then the same two-product
// reduction as the s = 2 term, and no lane multiplies by xP inside the loop (two products per lane
// per line instead of three).  The record also holds xi lambda' and xi mu, so the lanes whose term
// wraps (s = 1, k = 0; s = 2, k < 3) read pre-twisted coefficients and no lane applies xi after the
// product.
#define P36_LX_WORDS 54  // per line: lambda' | xi lambda' | xi mu (9-limb components)
// lx[(j (k1 - k0) + k - k0) P36_LX_WORDS + ...] for pair j's line k in [k0, k1): lambda' = -xP lambda
// (components 0, 1), then xi lambda', xi mu; Pn[j].x holds -xP_j.  One lane per (pair, line); the
// whole wave calls it.
template <int NP>
__device__ __forceinline__ void p36_lambda_x(uint32_t* lx, const g1a* Pn, const uint32_t* const* lines, int k0, int k1,
                                             const P36& g) {
  const int nl = k1 - k0, total = NP * nl;
#pragma nounroll
  for (int base = 0; base < total; base += 64) {
    const int item = base + g.lane;
    const bool on = item < total;
    const int it = on ? item : 0;
    const int j = it / nl, kk = it - j * nl;
    const uint32_t* src = lines[0];
    fp x = Pn[0].x;
#pragma unroll
    for (int q = 1; q < NP; q++) {
      if (j == q) src = lines[q];
      fp_sel(x, Pn[q].x, j == q);
    }
    src += (k0 + kk) * BN_LINE_WORDS;
    fp2 l, r;
#pragma unroll
    for (int i = 0; i < BN_LIMBS; i++) {
      l.a.v[i] = src[i];
      l.b.v[i] = src[9 + i];
    }
    f_mul(r.a, l.a, x);
    f_mul(r.b, l.b, x);
    uint32_t* dst = lx + (j * nl + kk) * P36_LX_WORDS;
    if (on)
#pragma unroll
      for (int i = 0; i < BN_LIMBS; i++) {
        dst[i] = r.a.v[i];
        dst[9 + i] = r.b.v[i];
      }
    {
      fp2 m, t;
#pragma unroll
      for (int i = 0; i < BN_LIMBS; i++) {
        m.a.v[i] = src[18 + i];
        m.b.v[i] = src[27 + i];
      }
      fp2_mul_xi(t, r);
      fp2_mul_xi(m, m);
      if (on)
#pragma unroll
        for (int i = 0; i < BN_LIMBS; i++) {
          dst[18 + i] = t.a.v[i];
          dst[27 + i] = t.b.v[i];
          dst[36 + i] = m.a.v[i];
          dst[45 + i] = m.b.v[i];
        }
    }
  }
}

// the normalised line k with lambda' from p36_lambda_x (lxk: its record) and mu from the table
__device__ __forceinline__ void p36_line_lx(fp& f, const uint32_t* lxk, const uint32_t* ln, const g1a& P, const P36& g) {
  fp om, oo;
  p36_fetch(om, oo, f, g.s == 1 ? (g.k + 5) % 6 : (g.k + 3) % 6, g);
  const bool wrap = (g.s == 1 && g.k == 0) || (g.s == 2 && g.k < 3);
  fp lm, lo, mm, mo;
  // s = 1: lambda' (xi lambda' on wrap); s = 2 on wrap: xi mu; else mu from the table
  const int off = g.s == 2 ? 36 : (wrap ? 18 : 0);
  p36_coef(lm, lo, lxk + off, g.h);
  p36_coef(mm, mo, ln + 18, g.h);
  const bool use_lds = g.s == 1 || wrap;
  const fp u = g.h ? oo : om, v = g.h ? om : oo;
  fp X1 = g.s == 0 ? f : u;
  fp Y1 = g.s == 0 ? P.y : (use_lds ? lm : mm);
  fp cz = use_lds ? lo : mo;
  const uint32_t mz = cs_mask(g.s != 0);
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) cz.v[i] &= mz;
  fp vn;
  p36_cneg4(vn, v, g.h == 0);
  fp T;
  f_mul_sum2(T, X1, Y1, vn, cz);  // s = 0: f_k yP; s = 1: f_{k-1} lambda'; s = 2: f_{k-3} mu
  p36_sum3(f, T, g);
}

// f <- f * (A yP + B xP w + C w^3) for an unnormalised line (bn254_g2wave.h, 54 words):
//   s = 0: yP (f_k A);  s = 1: xP (f_{k-1} B) (xi for k = 0);  s = 2: f_{k-3} C (xi for k < 3)
// Three multiplications per lane, as p36_line1.
__device__ __forceinline__ void p36_line_abc(fp& f, const uint32_t* ln, const g1a& P, const P36& g) {
  fp om, oo, cm, co;
  p36_fetch(om, oo, f, g.s == 0 ? g.k : (g.s == 1 ? (g.k + 5) % 6 : (g.k + 3) % 6), g);
  p36_coef(cm, co, ln + 18 * g.s, g.h);
  const fp u = g.h ? oo : om, v = g.h ? om : oo;
  fp P3, C;
  fp vn;
  p36_cneg4(vn, v, g.h == 0);
  f_mul_sum2(C, u, cm, vn, co);
  f_mul(P3, C, g.s == 0 ? P.y : P.x);
  fp T = g.s == 2 ? C : P3;
  const bool wrap = (g.s == 1 && g.k == 0) || (g.s == 2 && g.k < 3);
  fp w;
  p36_xi(w, T, g);
  fp_sel(T, w, wrap);
  p36_sum3(f, T, g);
}

__device__ __forceinline__ void p36_one(fp& r, const P36& g) {
  f_zero(r);
  fp one;
  f_one(one);
  fp_sel(r, one, g.k == 0 && g.h == 0);
}

__device__ __forceinline__ void p36_conj(fp& r, const fp& x, const P36& g) {
  fp n;
  f_neg(n, x);
  r = x;
  fp_sel(r, n, (g.k & 1) != 0);
}

// x -> x^(p^J) (see p12_frob)
template <int J>
__device__ __forceinline__ void p36_frob(fp& r, const fp& x, const P36& g) {
  fp c = x;
  if (J & 1) {
    fp n;
    f_neg(n, x);
    fp_sel(c, n, g.h == 1);
  }
  if (J == 2) {
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
  fp_swap_h(co, c, g);
  const fp gmm = g.h ? gm.b : gm.a, gmo = g.h ? gm.a : gm.b;
  p12_cmul(r, c, co, gmm, gmo, g.h);
}

// x^-1 = conj(x) / N with N = x conj(x) in Fp6 (the even w-coefficients; the odd ones vanish):
// N on the wave (one p36_mul), N^-1 by the Fp6 tower on every lane (variable-time Fp inversion:
// x is a Miller value of public inputs), then conj(x) N^-1 on the wave.  Half the one-lane tower
// work of inverting in Fp12 directly.
//
// The Fp6 inversion's Fp2 products are spread over lanes (fp6_inv's formulas): six lanes form c0^2,
// c1 c2, c2^2, c0 c1, c1^2, c0 c2 at once, three lanes c2 t1, c1 t2, c0 t0, and each lane its own
// t_(k/2) N^-1 -- 3 Fp2 products on the critical path between the gathers and the one Fp2
// inversion instead of 12.
__device__ __forceinline__ void fp2_shfl(fp2& r, const fp2& x, int src) {
  fp_shfl(r.a, x.a, src);
  fp_shfl(r.b, x.b, src);
}
__device__ __noinline__ void p36_inv(fp& r, const fp& x, const P36& g) {
  fp xc, n;
  p36_conj(xc, x, g);
  p36_mul(n, x, xc, g);
  fp6 t;
  fp_shfl(t.c0.a, n, p36_src(0, 0, 0));
  fp_shfl(t.c0.b, n, p36_src(0, 1, 0));
  fp_shfl(t.c1.a, n, p36_src(2, 0, 0));
  fp_shfl(t.c1.b, n, p36_src(2, 1, 0));
  fp_shfl(t.c2.a, n, p36_src(4, 0, 0));
  fp_shfl(t.c2.b, n, p36_src(4, 1, 0));
  fp2 pick;
  {
    const int j = g.lane;
    // lane j < 6: (c0 c0, c1 c2, c2 c2, c0 c1, c1 c1, c0 c2)[j]
    fp2 X = t.c0, Y = t.c0, R, R0, R1, R2, R3, R4, R5;
    p12_sel2(X, t.c1, j == 1 || j == 4);
    p12_sel2(X, t.c2, j == 2);
    p12_sel2(Y, t.c2, j == 1 || j == 2 || j == 5);
    p12_sel2(Y, t.c1, j == 3 || j == 4);
    fp2_mul(R, X, Y);
    fp2_shfl(R0, R, 0);
    fp2_shfl(R1, R, 1);
    fp2_shfl(R2, R, 2);
    fp2_shfl(R3, R, 3);
    fp2_shfl(R4, R, 4);
    fp2_shfl(R5, R, 5);
    fp2 t0, t1, t2, u;
    fp2_mul_xi(u, R1);  // t0 = c0^2 - xi c1 c2
    fp2_sub(t0, R0, u);
    fp2_mul_xi(u, R2);  // t1 = xi c2^2 - c0 c1
    fp2_sub(t1, u, R3);
    fp2_sub(t2, R4, R5);  // t2 = c1^2 - c0 c2
    // lane j < 3: (c2 t1, c1 t2, c0 t0)[j]; N = c0 t0 + xi (c2 t1 + c1 t2)
    X = t.c2;
    Y = t1;
    p12_sel2(X, t.c1, j == 1);
    p12_sel2(Y, t2, j == 1);
    p12_sel2(X, t.c0, j == 2);
    p12_sel2(Y, t0, j == 2);
    fp2_mul(R, X, Y);
    fp2_shfl(R0, R, 0);
    fp2_shfl(R1, R, 1);
    fp2_shfl(R2, R, 2);
    fp2 nn;
    fp2_add(u, R0, R1);
    fp2_mul_xi(u, u);
    fp2_add(nn, R2, u);
    {  // nn^-1: every lane holds nn (gathered from lanes 0..2), so the Fp inversion is the wave form
      fp n2, t2;
      f_sqr(n2, nn.a);
      f_sqr(t2, nn.b);
      f_add(n2, n2, t2);
#if defined(__HIP_DEVICE_COMPILE__)
      fp_inv_var_wave(n2, n2);
#endif
      f_mul(nn.a, nn.a, n2);
      f_mul(t2, nn.b, n2);
      f_neg(nn.b, t2);
    }
    // this lane's coefficient of the inverse: t_(k/2) N^-1 (k odd: unused)
    fp2 tk = t0;
    p12_sel2(tk, t1, g.k == 2 || g.k == 3);
    p12_sel2(tk, t2, g.k >= 4);
    fp2_mul(pick, tk, nn);
  }
  fp ninv = g.h ? pick.b : pick.a;
  if (g.k & 1) f_zero(ninv);
  p36_mul(r, xc, ninv, g);
}

__device__ __forceinline__ void p36_pow_u(fp& r, const fp& x, const P36& g) {
  fp acc = x;
#pragma nounroll
  for (int i = 61; i >= 0; i--) {
    p36_cyc_sqr(acc, acc, g);
    if (i == 55 || i == 0) p36_mul(acc, acc, x, g);
  }
  p36_conj(r, acc, g);
}

__device__ __forceinline__ void p36_pow_small(fp& r, const fp& x, uint32_t e, const P36& g) {
  fp acc = x;
  int top = 31;
  while (!((e >> top) & 1)) top--;
#pragma nounroll
  for (int i = top - 1; i >= 0; i--) {
    p36_cyc_sqr(acc, acc, g);
    if ((e >> i) & 1) p36_mul(acc, acc, x, g);
  }
  r = acc;
}

// The hard part's tail as a vectorial addition chain (gg^d = y0 y1^2 y2^6 y3^12
// y4^18 y5^30 y6^36 with y0 = gg^(p + p^2 + p^3), y1 = 1/gg, y2 = b^(p^2), y3 = a^-p, y4 = 1/(a b^p),
// y5 = 1/b, y6 = 1/(c c^p): 4 squarings, 13 products, 7 Frobenius maps) instead of raising c, b, a
// to 36, 30, 18, 12, 6 separately (16 squarings, 17 products, 3 maps).  The same exponent d, so
// the same GT element.
__device__ __forceinline__ void p36_final_exp(fp& r, const fp& f, const P36& g) {
  fp t, gg;
  p36_inv(t, f, g);
  p36_conj(gg, f, g);
  p36_mul(gg, gg, t, g);
  p36_frob<2>(t, gg, g);
  p36_mul(gg, t, gg, g);
  fp a, b, c;
  p36_pow_u(a, gg, g);
  p36_pow_u(b, a, g);
  p36_pow_u(c, b, g);
  {
    fp y0, y1, y2, y3, y4, y5, y6, u, T0, T1;
    p36_frob<1>(y0, gg, g);
    p36_frob<2>(u, gg, g);
    p36_mul(y0, y0, u, g);
    p36_frob<3>(u, gg, g);
    p36_mul(y0, y0, u, g);
    p36_conj(y1, gg, g);
    p36_frob<2>(y2, b, g);
    p36_frob<1>(y3, a, g);
    p36_conj(y3, y3, g);
    p36_frob<1>(y4, b, g);
    p36_mul(y4, y4, a, g);
    p36_conj(y4, y4, g);
    p36_conj(y5, b, g);
    p36_frob<1>(y6, c, g);
    p36_mul(y6, y6, c, g);
    p36_conj(y6, y6, g);
    p36_cyc_sqr(T0, y6, g);  // y6^2 y4 y5
    p36_mul(T0, T0, y4, g);
    p36_mul(T0, T0, y5, g);
    p36_mul(T1, y3, y5, g);  // y6^2 y5^2 y4 y3
    p36_mul(T1, T1, T0, g);
    p36_mul(T0, T0, y2, g);  // y6^2 y5 y4 y2
    p36_cyc_sqr(T1, T1, g);
    p36_mul(T1, T1, T0, g);  // y6^6 y5^5 y4^3 y3^2 y2
    p36_cyc_sqr(T1, T1, g);
    p36_mul(T0, T1, y1, g);
    p36_mul(T1, T1, y0, g);
    p36_cyc_sqr(T0, T0, g);  // y6^24 y5^20 y4^12 y3^8 y2^4 y1^2
    p36_mul(r, T0, T1, g);
  }
}

// f = prod_{j < NP} of the Miller values of (P_j, Q_j) (lines of Q_j precomputed, normalised or
// ABC; P_j not infinity), conjugation and the two Frobenius lines included: the value final_exp takes.
// Miller values of disjoint pair sets multiply (the loop squares and conjugates a product), so
// two waves may run one pair each and multiply their f.  All 64 lanes of the wave call it.
// progress (nullable, LDS): lines are still being produced by another wave of the block
// (g2w_lines_abc); line k is read once progress > k.  (Reading each line's coefficients one line
// ahead measured equal or 1-2 % slower: the line tables are L2-resident and the load latency is not
// what a lone wave waits on.)
// lx (nullable, LDS, NP x 70 x P36_LX_WORDS words, normalised lines only): room for p36_lambda_x
template <int NP, bool ABC = false>
__device__ __forceinline__ void p36_miller(fp& f, const g1a* P, const uint32_t* const* lines, const P36& g,
                                           const volatile int* progress = nullptr, uint32_t* lx = nullptr) {
  constexpr int W = ABC ? 54 : BN_LINE_WORDS;  // ABC: unnormalised lines (bn254_g2wave.h)
  p36_one(f, g);
  int k = 0;
  g1a Pn[NP];  // normalised lines take -xP (p36_line1c)
#pragma unroll
  for (int j = 0; j < NP; j++) Pn[j] = ABC ? P[j] : p36_neg_x(P[j]);
  if (!ABC && !progress && lx) {
    p36_lambda_x<NP>(lx, Pn, lines, 0, BN_ATE_LINES, g);
    auto lline = [&](int j) { p36_line_lx(f, lx + (j * BN_ATE_LINES + k) * P36_LX_WORDS, lines[j] + k * W, P[j], g); };
#pragma nounroll
    for (int i = BN_ATE_DBL - 1; i >= 0; i--) {
      p36_sqr(f, f, g);
#pragma unroll
      for (int j = 0; j < NP; j++) lline(j);
      k++;
      if (bn_ate_bit(i)) {
#pragma unroll
        for (int j = 0; j < NP; j++) lline(j);
        k++;
      }
    }
    p36_conj(f, f, g);
    for (int t = 0; t < 2; t++) {
#pragma unroll
      for (int j = 0; j < NP; j++) lline(j);
      k++;
    }
    return;
  }
  auto line = [&](int j) {
    if (progress) {
      while (*progress <= k) __builtin_amdgcn_s_sleep(2);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    if (ABC)
      p36_line_abc(f, lines[j] + k * W, P[j], g);
    else
      p36_line1(f, lines[j] + k * W, Pn[j], g);
  };
#pragma nounroll
  for (int i = BN_ATE_DBL - 1; i >= 0; i--) {
    p36_sqr(f, f, g);
#pragma unroll
    for (int j = 0; j < NP; j++) line(j);
    k++;
    if (bn_ate_bit(i)) {
#pragma unroll
      for (int j = 0; j < NP; j++) line(j);
      k++;
    }
  }
  p36_conj(f, f, g);
  for (int t = 0; t < 2; t++) {
#pragma unroll
    for (int j = 0; j < NP; j++) line(j);
    k++;
  }
}

// One pair's Miller loop split over two waves: the TOP part runs iterations 63..s and then s
// more squarings, the BOTTOM part iterations s-1..0 (starting from 1), the conjugation and the
// two Frobenius lines; F_top^(2^s) F_bottom is the whole loop's value (squaring distributes over
// the product), conjugation applied to both.  With s = 40 both parts cost 209 Fp multiplications
// per lane (sqr 2, line 3) against 320 for the whole loop on one wave.
#define P36_MILLER_SPLIT 40
// ABC: unnormalised lines (54 words, bn254_g2wave.h) read once progress > k (nullable: all present)
// lx (nullable, LDS, up to 70 x P36_LX_WORDS words, normalised lines only): room for p36_lambda_x
template <bool TOP, bool ABC = false>
__device__ __forceinline__ void p36_miller_part(fp& f, const g1a& P, const uint32_t* lines, const P36& g,
                                                const volatile int* progress = nullptr, uint32_t* lx = nullptr) {
  constexpr int W = ABC ? 54 : BN_LINE_WORDS;
  p36_one(f, g);
  int k = 0;
  const int hi = TOP ? BN_ATE_DBL - 1 : P36_MILLER_SPLIT - 1, lo = TOP ? P36_MILLER_SPLIT : 0;
  for (int i = BN_ATE_DBL - 1; i > hi; i--) k += bn_ate_bit(i) ? 2 : 1;
  if (!ABC && !progress && lx) {
    int k1 = k;  // this part's lines: [k, k1)
    for (int i = hi; i >= lo; i--) k1 += bn_ate_bit(i) ? 2 : 1;
    if (!TOP) k1 += 2;  // the two Frobenius lines
    const int k0 = k;
    const g1a Pn = p36_neg_x(P);
    const uint32_t* l1[1] = {lines};
    p36_lambda_x<1>(lx, &Pn, l1, k0, k1, g);
    auto lline = [&]() {
      p36_line_lx(f, lx + (k - k0) * P36_LX_WORDS, lines + k * W, P, g);
      k++;
    };
#pragma nounroll
    for (int i = hi; i >= lo; i--) {
      p36_sqr(f, f, g);
      lline();
      if (bn_ate_bit(i)) lline();
    }
    if (TOP) {
#pragma nounroll
      for (int t = 0; t < P36_MILLER_SPLIT; t++) p36_sqr(f, f, g);
    }
    p36_conj(f, f, g);
    if (!TOP) {
      lline();
      lline();
    }
    return;
  }
  const g1a Pn = ABC ? P : p36_neg_x(P);  // normalised lines take -xP (p36_line1c)
  auto line = [&]() {
    if (progress) {
      while (*progress <= k) __builtin_amdgcn_s_sleep(2);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    if (ABC)
      p36_line_abc(f, lines + k * W, P, g);
    else
      p36_line1(f, lines + k * W, Pn, g);
    k++;
  };
#pragma nounroll
  for (int i = hi; i >= lo; i--) {
    p36_sqr(f, f, g);
    line();
    if (bn_ate_bit(i)) line();
  }
  if (TOP) {
#pragma nounroll
    for (int t = 0; t < P36_MILLER_SPLIT; t++) p36_sqr(f, f, g);
  }
  p36_conj(f, f, g);
  if (!TOP) {
    line();
    line();
  }
}

// final_exp(f) == 1 ?  Every lane returns the verdict.
__device__ __forceinline__ bool p36_is_one_after_final_exp(const fp& f, const P36& g) {
  fp e;
  p36_final_exp(e, f, g);
  fp want;
  p36_one(want, g);
  const bool mine = f_eq(e, want);
  bool all = true;
#pragma unroll
  for (int q = 0; q < 12; q++) all = all && (__shfl((int)mine, q) != 0);
  return all;
}

// ---- the final exponentiation on two waves of a block ----
// The hard part's three u-powers a = gg^u, b = a^u, c = b^u are one serial chain; everything
// else p36_final_exp derives from gg, a and b (a^12, a^18, b^6, b^18, b^30, gg^2 and two of the
// Frobenius terms) runs on a helper wave while the lead wave is still raising to u, so the lead's
// tail after c is c^36 and six products instead of 16 squarings and 17 products.  Same GT element
// as p36_final_exp (products reassociated; f_eq compares canonical forms).  Values pass through
// an LDS mailbox: the writer's owning lanes store, release-fence, then lane 0 raises the slot's
// flag; the reader spins on the flag (s_sleep) and acquire-fences.
struct FeMail {
  enum { GG = 0, A = 1, B = 2, X = 3, Y = 4, Z = 5, SLOTS = 6 };
  uint32_t v[SLOTS][36][BN_LIMBS];
  int flag[SLOTS];
};
__device__ __forceinline__ void femail_init(FeMail& m) {  // one thread; a barrier before any use
  for (int i = 0; i < FeMail::SLOTS; i++) m.flag[i] = 0;
}
__device__ __forceinline__ void femail_write(FeMail& m, int slot, const fp& x, const P36& g) {
  if (g.own)
#pragma unroll
    for (int i = 0; i < BN_LIMBS; i++) m.v[slot][g.e][i] = x.v[i];
}
__device__ __forceinline__ void femail_raise(FeMail& m, int slot, const P36& g) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (g.lane == 0) *(volatile int*)&m.flag[slot] = 1;
}
__device__ __forceinline__ void femail_wait(const FeMail& m, int slot) {
  while (*(const volatile int*)&m.flag[slot] == 0) __builtin_amdgcn_s_sleep(2);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ void femail_read(fp& x, const FeMail& m, int slot, const P36& g) {
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) x.v[i] = m.v[slot][g.e][i];  // shadows read the slot they mirror
}

// lead wave: r = final_exp(f), with p36_fe2_helper running on another wave of the block
__device__ __forceinline__ void p36_final_exp_lead(fp& r, const fp& f, FeMail& m, const P36& g) {
  fp t, gg;
  p36_inv(t, f, g);
  p36_conj(gg, f, g);
  p36_mul(gg, gg, t, g);
  p36_frob<2>(t, gg, g);
  p36_mul(gg, t, gg, g);
  femail_write(m, FeMail::GG, gg, g);
  femail_raise(m, FeMail::GG, g);
  fp a, b, c;
  p36_pow_u(a, gg, g);
  femail_write(m, FeMail::A, a, g);
  femail_raise(m, FeMail::A, g);
  p36_pow_u(b, a, g);
  femail_write(m, FeMail::B, b, g);
  femail_raise(m, FeMail::B, g);
  p36_pow_u(c, b, g);
  fp c36, X, Y, Z, t0, t1;
  p36_pow_small(c36, c, 36, g);
  femail_wait(m, FeMail::Z);  // X, Y, Z raised together
  femail_read(X, m, FeMail::X, g);
  femail_read(Y, m, FeMail::Y, g);
  femail_read(Z, m, FeMail::Z, g);
  p36_mul(t0, c36, X, g);  // c^36 b^30 a^18 gg^2
  p36_conj(t0, t0, g);
  p36_mul(t1, c36, Y, g);  // c^36 b^18 a^12
  p36_conj(t1, t1, g);
  p36_mul(t1, t1, gg, g);
  p36_frob<1>(t1, t1, g);
  p36_mul(t0, t0, t1, g);
  p36_mul(r, t0, Z, g);  // Z = frob2(b^6 gg) frob3(gg)
}

// helper wave: X = b^30 a^18 gg^2, Y = b^18 a^12, Z = frob2(b^6 gg) frob3(gg) from the lead's gg, a, b
__device__ __forceinline__ void p36_fe2_helper(FeMail& m, const P36& g) {
  fp gg, g2, t3, a, a12, a18, P1, b, b6, b18, b30, t2, X, Y, Z;
  femail_wait(m, FeMail::GG);
  femail_read(gg, m, FeMail::GG, g);
  p36_cyc_sqr(g2, gg, g);
  p36_frob<3>(t3, gg, g);
  femail_wait(m, FeMail::A);
  femail_read(a, m, FeMail::A, g);
  p36_pow_small(a12, a, 12, g);
  p36_pow_small(a18, a, 18, g);
  p36_mul(P1, a18, g2, g);
  femail_wait(m, FeMail::B);
  femail_read(b, m, FeMail::B, g);
  p36_pow_small(b6, b, 6, g);
  p36_pow_small(b18, b6, 3, g);
  p36_mul(b30, b18, b6, g);
  p36_mul(b30, b30, b6, g);
  p36_mul(t2, b6, gg, g);
  p36_frob<2>(t2, t2, g);
  p36_mul(X, b30, P1, g);
  p36_mul(Y, b18, a12, g);
  p36_mul(Z, t2, t3, g);
  femail_write(m, FeMail::X, X, g);
  femail_write(m, FeMail::Y, Y, g);
  femail_write(m, FeMail::Z, Z, g);
  femail_raise(m, FeMail::Z, g);
}

// final_exp(f) == 1 by the lead wave (every lane of it gets the verdict); another wave of the block
// must run p36_fe2_helper on the same mailbox (initialised, then a barrier, before either starts)
__device__ __forceinline__ bool p36_is_one_after_final_exp_lead(const fp& f, FeMail& m, const P36& g) {
  fp e;
  p36_final_exp_lead(e, f, m, g);
  fp want;
  p36_one(want, g);
  const bool mine = f_eq(e, want);
  bool all = true;
#pragma unroll
  for (int q = 0; q < 12; q++) all = all && (__shfl((int)mine, q) != 0);
  return all;
}

// prod_{j < NP} e(P_j, Q_j) == 1 on one wave
template <int NP>
__device__ __forceinline__ bool p36_pairing_check(const g1a* P, const uint32_t* const* lines, const P36& g,
                                                  uint32_t* lx = nullptr) {
  fp f;
  p36_miller<NP>(f, P, lines, g, nullptr, lx);
  return p36_is_one_after_final_exp(f, g);
}
