// G1 Jacobian arithmetic on a lane QUAD (gfx950 device code only).
//
// One lane's point chain (the Lagrange MSM: 132 doublings + 66 additions per share, all
// dependent) runs at one lane's issue rate.  Here the four lanes of a quad hold the same point
// and each step's independent field products are dealt out one per lane, then broadcast back
// with DPP quad_perm (a VALU move, no LDS): the doubling (2M + 5S, depth 3) becomes 3 rounds,
// the general addition (11M + 5S) 5 rounds of at most 4 products.  Every lane of the quad ends
// with the same bits, so the state stays replicated.  Results equal g1_dbl / g1_add
// (bn254_pairing.h) as points (same field elements; tests/test_bls_gpu.py compares the
// combined signature with the oracle byte for byte).
#pragma once
#include "bn254_cycsq.h"
#include "bn254_pairing.h"

template <int CTRL>
__device__ __forceinline__ void g1q_bcast(fp& r, const fp& a) {
#pragma unroll
  for (int k = 0; k < BN_LIMBS; k++) r.v[k] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a.v[k], CTRL, 0xF, 0xF, false);
}

// r[i] = U[i] * V[i] for i < N (N <= 4): product i on quad lane i, broadcast to the quad
template <int N>
__device__ __forceinline__ void g1q_round(fp* r, const fp* U, const fp* V, int q) {
  fp u = U[0], v = V[0];
#pragma unroll
  for (int i = 1; i < N; i++) {
#pragma unroll
    for (int k = 0; k < BN_LIMBS; k++) {
      u.v[k] = q == i ? U[i].v[k] : u.v[k];
      v.v[k] = q == i ? V[i].v[k] : v.v[k];
    }
  }
  fp p;
  f_mul(p, u, v);
  g1q_bcast<0x00>(r[0], p);
  if (N > 1) g1q_bcast<0x55>(r[1], p);
  if (N > 2) g1q_bcast<0xAA>(r[2], p);
  if (N > 3) g1q_bcast<0xFF>(r[3], p);
}

// r = 2p (dbl-2009-l, a = 0); infinity (Z = 0) stays infinity.  Lazy sums between the rounds
// and one reduction per output coordinate (bn254_cycsq.h: g1d_*, checked on the host as
// g1_dbl_lazy against g1_dbl).
__device__ __forceinline__ void g1q_dbl(g1j& r, const g1j& p, int q) {
  fp U[3], V[3], o[3];
  U[0] = p.X;
  V[0] = p.X;
  U[1] = p.Y;
  V[1] = p.Y;
  U[2] = p.Y;
  V[2] = p.Z;
  g1q_round<3>(o, U, V, q);
  fp A = o[0], B = o[1], E, Z3, t;
  f_add(Z3, o[2], o[2]);
  g1d_et(E, t, A, p.X, B);
  U[0] = B;
  V[0] = B;
  U[1] = t;
  V[1] = t;
  U[2] = E;
  V[2] = E;
  g1q_round<3>(o, U, V, q);
  fp C = o[0], X3, w;
  g1d_x3w(X3, w, o[1], A, C, o[2]);
  U[0] = E;
  V[0] = w;
  g1q_round<1>(o, U, V, q);
  g1d_y3(r.Y, o[0], C);
  r.X = X3;
  r.Z = Z3;
}

// r = p + q (add-2007-bl) with g1_add's special cases: infinity operands, p = q (doubling),
// p = -q (infinity).  The special branches are quad-uniform (replicated state).
__device__ __forceinline__ void g1q_add(g1j& r, const g1j& p, const g1j& qq, int q) {
  const bool pinf = g1_is_inf(p), qinf = g1_is_inf(qq);
  fp U[4], V[4], o[4];
  U[0] = p.Z;
  V[0] = p.Z;
  U[1] = qq.Z;
  V[1] = qq.Z;
  g1q_round<2>(o, U, V, q);
  const fp Z1Z1 = o[0], Z2Z2 = o[1];
  U[0] = p.X;
  V[0] = Z2Z2;
  U[1] = qq.X;
  V[1] = Z1Z1;
  U[2] = p.Y;
  V[2] = qq.Z;
  U[3] = qq.Y;
  V[3] = p.Z;
  g1q_round<4>(o, U, V, q);
  const fp U1 = o[0], U2 = o[1];
  fp H, H2, ZS;
  f_sub(H, U2, U1);
  fl_sum(H2, H, H);  // unreduced operands of H2^2 and ZS^2 (limbs < 2^30, values < 4q)
  fl_sum(ZS, p.Z, qq.Z);
  U[0] = o[2];
  V[0] = Z2Z2;
  U[1] = o[3];
  V[1] = Z1Z1;
  U[2] = H2;
  V[2] = H2;
  U[3] = ZS;
  V[3] = ZS;
  g1q_round<4>(o, U, V, q);
  const fp S1 = o[0], I = o[2];
  fp rr, ZZ;
  f_sub(rr, o[1], S1);
  f_add(rr, rr, rr);
  f_sub(ZZ, o[3], Z1Z1);
  f_sub(ZZ, ZZ, Z2Z2);
  g1j res;
  if (!pinf && !qinf && f_is_zero(H)) {  // same x: p = q (double) or p = -q (infinity)
    if (f_is_zero(rr)) {
      g1q_dbl(res, p, q);
    } else {
      g1_set_inf(res);
    }
  } else {
    U[0] = H;
    V[0] = I;
    U[1] = U1;
    V[1] = I;
    U[2] = rr;
    V[2] = rr;
    U[3] = ZZ;
    V[3] = H;
    g1q_round<4>(o, U, V, q);
    const fp J = o[0], Vv = o[1];
    fp X3, w;
    f_sub(X3, o[2], J);
    f_sub(X3, X3, Vv);
    f_sub(X3, X3, Vv);
    f_sub(w, Vv, X3);
    res.Z = o[3];
    U[0] = rr;
    V[0] = w;
    U[1] = S1;
    V[1] = J;
    g1q_round<2>(o, U, V, q);
    fp SJ;
    f_add(SJ, o[1], o[1]);
    f_sub(res.Y, o[0], SJ);
    res.X = X3;
  }
  r = pinf ? qq : (qinf ? p : res);
}
