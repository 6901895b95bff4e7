// Miller-loop lines of a fresh G2 point computed by a whole wave (gfx950 device code only).
//
// A multisig verify needs the lines of PK = sum vk_i, a key used once.  On one lane the 70
// Jacobian line steps are ~1,900 dependent Fp multiplications (plus ~1,000 more to normalise
// the lines by a batched inversion): milliseconds at one lane's issue rate.  Here every Fp
// product of a step is dealt to its own lane: the doubling step's 27 products (Fp2 Karatsuba:
// 3 per Fp2 product, 2 per square) fall into 3 rounds of independent products (9, 15, 3), the
// mixed addition's 38 into 5 rounds; after each round all lanes gather the products
// (ds_bpermute) and form the Fp2 sums redundantly, so the whole wave holds T.
//
// The lines are left UNNORMALISED, (A, B, C) with line(P) = A yP + B xP w + C w^3 (the same
// A_k, B_k, C_k as g2_precompute_lines_batch, bn254_pairing.h, before it divides by A_k):
// A_k is a non-zero Fp2 factor, which the final exponentiation maps to 1
// ((p^12 - 1)/r is a multiple of p^2 - 1), so the pairing is unchanged and no inversion is
// needed.  bn254_pair36.h evaluates them at the same cost as normalised lines.
#pragma once
#include "bn254_cycsq.h"
#include "bn254_g2row.h"
#include "bn254_pairing.h"

#define BN_ABC_WORDS 54  // A | B | C (fp2 each)

// r[i] = U[i] * V[i], i < N (N <= 64): product i on lane i, gathered to every lane
template <int N>
__device__ __forceinline__ void g2w_round(fp* r, const fp* U, const fp* V, int lane) {
  fp u = U[0], v = V[0];
#pragma unroll
  for (int i = 1; i < N; i++) {
#pragma unroll
    for (int q = 0; q < BN_LIMBS; q++) {
      u.v[q] = lane == i ? U[i].v[q] : u.v[q];
      v.v[q] = lane == i ? V[i].v[q] : v.v[q];
    }
  }
  fp p;
  f_mul(p, u, v);
#pragma unroll
  for (int i = 0; i < N; i++)
#pragma unroll
    for (int q = 0; q < BN_LIMBS; q++) r[i].v[q] = (uint32_t)__shfl((int)p.v[q], i);
}

// operand slots of an Fp2 product x*y (Karatsuba: x0 y0, x1 y1, (x0 + x1)(y0 + y1)) and square
// x^2 ((x0 + x1)(x0 - x1), x0 x1), written at U/V + o.  The sums stay unreduced (bn254_cycsq.h:
// fl_sum / fl_diff2q): limbs < 2^30 (sum) and < 1.5 2^30 (difference), values < 4q, keep
// f_mul's columns below 2^64 (at most 7 full-size products: 7 1.5 2^60 + 9 2^58 + 2^35) and its
// result below 2q (16 q^2 < q 2^261), so no reduction is spent on an operand
// (tests/test_bn254_inv.py: test_fp_mul_raw_both_operands).
__device__ __forceinline__ void g2w_mul_ops(fp* U, fp* V, int o, const fp2& x, const fp2& y) {
  U[o] = x.a;
  V[o] = y.a;
  U[o + 1] = x.b;
  V[o + 1] = y.b;
  fl_sum(U[o + 2], x.a, x.b);
  fl_sum(V[o + 2], y.a, y.b);
}
__device__ __forceinline__ void g2w_sqr_ops(fp* U, fp* V, int o, const fp2& x) {
  fl_sum(U[o], x.a, x.b);
  fl_diff2q(V[o], x.a, x.b);
  U[o + 1] = x.a;
  V[o + 1] = x.b;
}
__device__ __forceinline__ void g2w_mul_res(fp2& r, const fp* p, int o) {
  f_sub(r.a, p[o], p[o + 1]);
  fp_lin3<1, -1, -1, 4>(r.b, p[o + 2], p[o], p[o + 1]);  // one reduction (bn254_cycsq.h)
}
__device__ __forceinline__ void g2w_sqr_res(fp2& r, const fp* p, int o) {
  r.a = p[o];
  f_add(r.b, p[o + 1], p[o + 1]);
}

// lines write: word w of the 54-word (A, B, C) record on lane w (coalesced)
__device__ __forceinline__ void g2w_store(uint32_t* ln, const fp2& A, const fp2& B, const fp2& C, int lane) {
  uint32_t wv[BN_ABC_WORDS];
#pragma unroll
  for (int q = 0; q < BN_LIMBS; q++) {
    wv[q] = A.a.v[q];
    wv[9 + q] = A.b.v[q];
    wv[18 + q] = B.a.v[q];
    wv[27 + q] = B.b.v[q];
    wv[36 + q] = C.a.v[q];
    wv[45 + q] = C.b.v[q];
  }
  uint32_t w = wv[0];
#pragma unroll
  for (int i = 1; i < BN_ABC_WORDS; i++) w = lane == i ? wv[i] : w;
  if (lane < BN_ABC_WORDS) ln[lane] = w;
}

// tangent at T (line_dbl_j's A, B, C), T <- 2T (dbl-2009-l)
__device__ __forceinline__ void g2w_dbl(uint32_t* ln, g2j& T, int lane) {
  fp U[15], V[15], p[15];
  g2w_sqr_ops(U, V, 0, T.X);
  g2w_sqr_ops(U, V, 2, T.Y);
  g2w_sqr_ops(U, V, 4, T.Z);
  g2w_mul_ops(U, V, 6, T.Y, T.Z);
  g2w_round<9>(p, U, V, lane);
  fp2 XX, YY, ZZ, t, E, D0;
  g2w_sqr_res(XX, p, 0);
  g2w_sqr_res(YY, p, 2);
  g2w_sqr_res(ZZ, p, 4);
  g2w_mul_res(t, p, 6);
  fp2_dbl(t, t);  // 2YZ = Z3
  fp_lin3<3, 0, 0, 0>(E.a, XX.a, XX.a, XX.a);  // 3X^2 (one reduction per component)
  fp_lin3<3, 0, 0, 0>(E.b, XX.b, XX.b, XX.b);
  fp2_add(D0, T.X, YY);
  g2w_mul_ops(U, V, 0, t, ZZ);    // A = 2YZ^3
  g2w_mul_ops(U, V, 3, E, ZZ);    // -B = 3X^2 Z^2
  g2w_mul_ops(U, V, 6, E, T.X);   // 3X^3
  g2w_sqr_ops(U, V, 9, YY);       // YYYY
  g2w_sqr_ops(U, V, 11, D0);      // (X + YY)^2
  g2w_sqr_ops(U, V, 13, E);       // F = E^2
  g2w_round<15>(p, U, V, lane);
  fp2 A, B, C, YYYY, D, F, X3, w;
  g2w_mul_res(A, p, 0);
  g2w_mul_res(B, p, 3);
  fp2_neg(B, B);
  g2w_mul_res(C, p, 6);
  fp_lin3<1, -2, 0, 4>(C.a, C.a, YY.a, YY.a);  // 3X^3 - 2Y^2
  fp_lin3<1, -2, 0, 4>(C.b, C.b, YY.b, YY.b);
  g2w_store(ln, A, B, C, lane);
  g2w_sqr_res(YYYY, p, 9);
  g2w_sqr_res(D, p, 11);
  g2w_sqr_res(F, p, 13);
  fp_lin3<2, -2, -2, 8>(D.a, D.a, XX.a, YYYY.a);  // D = 2((X + YY)^2 - XX - YYYY)
  fp_lin3<2, -2, -2, 8>(D.b, D.b, XX.b, YYYY.b);
  fp_lin3<1, -2, 0, 4>(X3.a, F.a, D.a, D.a);  // X3 = F - 2D
  fp_lin3<1, -2, 0, 4>(X3.b, F.b, D.b, D.b);
  fp2_sub(w, D, X3);
  g2w_mul_ops(U, V, 0, E, w);
  g2w_round<3>(p, U, V, lane);
  fp2 Y3;
  g2w_mul_res(Y3, p, 0);
  fp u;  // Y3 - 8 YYYY as two reductions of - 4 YYYY
  fp_lin3<1, -4, 0, 8>(u, Y3.a, YYYY.a, YYYY.a);
  fp_lin3<1, -4, 0, 8>(T.Y.a, u, YYYY.a, YYYY.a);
  fp_lin3<1, -4, 0, 8>(u, Y3.b, YYYY.b, YYYY.b);
  fp_lin3<1, -4, 0, 8>(T.Y.b, u, YYYY.b, YYYY.b);
  T.X = X3;
  T.Z = t;
}

// line through T and affine (qx, qy) (line_add_j's A, B, C), T <- T + Q (madd-2007-bl)
__device__ __forceinline__ void g2w_add(uint32_t* ln, g2j& T, const fp2& qx, const fp2& qy, int lane) {
  fp U[9], V[9], p[9];
  g2w_sqr_ops(U, V, 0, T.Z);
  g2w_mul_ops(U, V, 2, qy, T.Z);
  g2w_mul_ops(U, V, 5, qx, T.Y);
  g2w_round<8>(p, U, V, lane);
  fp2 ZZ, QZ, QXY;
  g2w_sqr_res(ZZ, p, 0);
  g2w_mul_res(QZ, p, 2);
  g2w_mul_res(QXY, p, 5);
  g2w_mul_ops(U, V, 0, qx, ZZ);   // U2
  g2w_mul_ops(U, V, 3, QZ, ZZ);   // S2
  g2w_mul_ops(U, V, 6, QZ, T.X);  // qy Z X
  g2w_round<9>(p, U, V, lane);
  fp2 U2, S2, C, H, R, B, r;
  g2w_mul_res(U2, p, 0);
  g2w_mul_res(S2, p, 3);
  g2w_mul_res(C, p, 6);
  fp2_sub(C, C, QXY);
  fp2_sub(H, U2, T.X);
  fp2_sub(R, S2, T.Y);
  fp2_neg(B, R);
  fp2_dbl(r, R);
  fp2 ZH;
  fp2_add(ZH, T.Z, H);
  g2w_mul_ops(U, V, 0, T.Z, H);  // A = Z H
  g2w_sqr_ops(U, V, 3, H);       // HH
  g2w_sqr_ops(U, V, 5, r);       // r^2
  g2w_sqr_ops(U, V, 7, ZH);      // (Z + H)^2
  g2w_round<9>(p, U, V, lane);
  fp2 A, HH, rr, I;
  g2w_mul_res(A, p, 0);
  g2w_sqr_res(HH, p, 3);
  g2w_sqr_res(rr, p, 5);
  g2w_sqr_res(ZH, p, 7);
  g2w_store(ln, A, B, C, lane);
  fp2_dbl(I, HH);
  fp2_dbl(I, I);
  g2w_mul_ops(U, V, 0, H, I);    // J
  g2w_mul_ops(U, V, 3, T.X, I);  // V
  g2w_round<6>(p, U, V, lane);
  fp2 J, Vv, X3, w;
  g2w_mul_res(J, p, 0);
  g2w_mul_res(Vv, p, 3);
  fp2_sub(X3, rr, J);
  fp2_sub(X3, X3, Vv);
  fp2_sub(X3, X3, Vv);
  fp2_sub(w, Vv, X3);
  g2w_mul_ops(U, V, 0, r, w);
  g2w_mul_ops(U, V, 3, T.Y, J);
  g2w_round<6>(p, U, V, lane);
  fp2 Y3, YJ;
  g2w_mul_res(Y3, p, 0);
  g2w_mul_res(YJ, p, 3);
  fp2_dbl(YJ, YJ);
  fp2_sub(T.Y, Y3, YJ);
  fp2_sub(ZH, ZH, ZZ);
  fp2_sub(T.Z, ZH, HH);
  T.X = X3;
}

// Streaming hand-over of lines to a consumer wave of the same block (progress in LDS): after
// line k is stored, progress = k + 1 (release at workgroup scope).
__device__ __forceinline__ void g2w_publish(volatile int* progress, int k, int lane) {
  if (!progress) return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane == 0) *progress = k;
}

// all BN_ATE_LINES (A, B, C) lines of affine q (not infinity), in Miller-loop order
// (g2_precompute_lines_batch's step sequence); every lane of the wave calls it.  progress
// (nullable): published after every line (g2w_publish).
__device__ __noinline__ void g2w_lines_abc(uint32_t* out, const g2a& q, volatile int* progress = nullptr) {
  const int lane = threadIdx.x & 63;
  g2j T;
  T.X = q.x;
  T.Y = q.y;
  fp2_one(T.Z);
  int k = 0;
#pragma nounroll
  for (int i = BN_ATE_DBL - 1; i >= 0; i--) {
    g2w_dbl(out + (k++) * BN_ABC_WORDS, T, lane);
    g2w_publish(progress, k, lane);
    if (bn_ate_bit(i)) {
      g2w_add(out + (k++) * BN_ABC_WORDS, T, q.x, q.y, lane);
      g2w_publish(progress, k, lane);
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
  g2w_add(out + (k++) * BN_ABC_WORDS, T, q1x, q1y, lane);
  g2w_publish(progress, k, lane);
  fp2_load(c, Bn254Consts::TWX2);
  fp2_mul(q2x, q.x, c);
  fp2_load(c, Bn254Consts::TWY2);
  fp2_mul(q2y, q.y, c);
  fp2_neg(q2y, q2y);
  g2w_add(out + (k++) * BN_ABC_WORDS, T, q2x, q2y, lane);
  g2w_publish(progress, k, lane);
}

// ---- the same lines on row-parallel Fp (bn254_g2row.h): T in rows, each step's Fp products four
// per pass; each (A, B, C) record is written from row 0 as normalised limbs (values < 4q, which
// p36_line_abc's products take).  Same records as g2w_lines_abc (field values; host emulation:
// tests/cpp/bn254_shim.cpp against line_dbl_j / line_add_j).
__device__ __forceinline__ void g2r_store_abc(uint32_t* ln, const F2R<uint32_t>* l) {
  f2r_st_row0(ln, l[0]);
  f2r_st_row0(ln + 18, l[1]);
  f2r_st_row0(ln + 36, l[2]);
}
__device__ __noinline__ void g2r_lines_abc(uint32_t* out, const g2a& q, volatile int* progress = nullptr) {
  const int lane = threadIdx.x & 63;
  const G2RowCtx<uint32_t, uint64_t> c(0u);
  const F2R<uint32_t> qx = f2r_from(q.x), qy = f2r_from(q.y);
  G2R<uint32_t> T{qx, qy, F2R<uint32_t>{c.one, c.zero}};
  F2R<uint32_t> l[3];
  bool same_y;
  int k = 0;
#pragma nounroll
  for (int i = BN_ATE_DBL - 1; i >= 0; i--) {
    g2r_dbl<true>(l, T, c);
    g2r_store_abc(out + (k++) * BN_ABC_WORDS, l);
    g2w_publish(progress, k, lane);
    if (bn_ate_bit(i)) {
      g2r_madd<true>(l, T, qx, qy, c, same_y);
      g2r_store_abc(out + (k++) * BN_ABC_WORDS, l);
      g2w_publish(progress, k, lane);
    }
  }
  T.Y = f2r_red(f2r_sub(F2R<uint32_t>{c.zero, c.zero}, T.Y, c), c);  // 6u + 2 < 0
  fp2 q1x, q1y, q2x, q2y, cc;
  fp2_conj(q1x, q.x);
  fp2_load(cc, Bn254Consts::TWX1);
  fp2_mul(q1x, q1x, cc);
  fp2_conj(q1y, q.y);
  fp2_load(cc, Bn254Consts::TWY1);
  fp2_mul(q1y, q1y, cc);
  fp2_load(cc, Bn254Consts::TWX2);
  fp2_mul(q2x, q.x, cc);
  fp2_load(cc, Bn254Consts::TWY2);
  fp2_mul(q2y, q.y, cc);
  fp2_neg(q2y, q2y);
  g2r_madd<true>(l, T, f2r_from(q1x), f2r_from(q1y), c, same_y);
  g2r_store_abc(out + (k++) * BN_ABC_WORDS, l);
  g2w_publish(progress, k, lane);
  g2r_madd<true>(l, T, f2r_from(q2x), f2r_from(q2y), c, same_y);
  g2r_store_abc(out + (k++) * BN_ABC_WORDS, l);
  g2w_publish(progress, k, lane);
}
