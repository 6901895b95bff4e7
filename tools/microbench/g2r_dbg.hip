// Device check of the row-parallel G2 full addition (bn254_g2row.h: g2r_add) step by step
// against the one-lane formulas (debug aid).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I concord-bft_amd/csrc tools/microbench/g2r_dbg.hip -o tools/microbench/g2r_dbg
#include <hip/hip_runtime.h>

#include <cstdio>

#include "bn254_g2row.h"
#include "bn254_pairing.h"

using C2 = G2RowCtx<uint32_t, uint64_t>;
__device__ __noinline__ bool add_noinline(G2R<uint32_t>& T, const G2R<uint32_t>& Q, bool& sy) {
  const C2 c(0u);
  return g2r_add(T, Q, c, sy);
}
__device__ bool same(uint32_t x, const fp& e, const C2& c) {
  const uint32_t r = c.mul(x, c.one);
  fp f;
  rf_to_fe(f, r);
  uint32_t w1[8], w2[8];
  f_to_words(w1, f);
  f_to_words(w2, e);
  bool eq = true;
  for (int i = 0; i < 8; i++) eq = eq && w1[i] == w2[i];
  return eq;
}
__device__ void chk(const char* n, const F2R<uint32_t>& x, const fp2& e, const C2& c) {
  const bool a = same(x.a, e.a, c), b = same(x.b, e.b, c);
  if (threadIdx.x == 0) printf("%-6s %s %s\n", n, a ? "ok" : "BAD", b ? "ok" : "BAD");
}
template <class U, class W>
__device__ bool g2r_add_dbg(G2R<U>& T, const G2R<U>& Q, const G2RowCtx<U, W>& c, bool& same_y, const fp2* ex) {
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
  chk("fU1", U1, ex[0], c);
  chk("fU2", U2, ex[1], c);
  const F2R<U> H = f2r_red(f2r_sub(U2, U1, c), c);
  chk("fH", H, ex[2], c);
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
  chk("fS1", S1, ex[3], c);
  chk("fS2", S2, ex[4], c);
  chk("fI", I, ex[5], c);
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
  chk("fJ", J, ex[6], c);
  chk("fV", V, ex[7], c);
  chk("frr", rr, ex[8], c);
  const F2R<U> X3 = f2r_red(f2r_sub32(f2r_sub(rr, J, c), f2r_add(V, V), c), c);
  const F2R<U> w = f2r_sub(V, X3, c);
  f2r_mul_ops(A, B, 0, r, w);
  f2r_mul_ops(A, B, 3, S1, J);
  r_prods<6>(P, A, B, c);
  F2R<U> Y3, SJ;
  f2r_mul_res(Y3, P, 0, c);
  f2r_mul_res(SJ, P, 3, c);
  chk("fX3", X3, ex[9], c);
  chk("fY3'", Y3, ex[10], c);
  chk("fSJ", SJ, ex[11], c);
  T.Y = f2r_red(f2r_sub32(Y3, f2r_add(SJ, SJ), c), c);
  T.X = X3;
  return true;
}


__global__ void k_dbg() {
  const C2 c(0u);
  g2j G, Q2;
  fp2_load(G.X, Bn254Consts::G2X);
  fp2_load(G.Y, Bn254Consts::G2Y);
  fp2_one(G.Z);
  g2_dbl_j(Q2, G);
  g2a qa;
  g2_to_affine(qa, Q2);
  g2j Q{qa.x, qa.y, G.Z};
  // one-lane reference intermediates (g2_add_j_body)
  fp2 Z1Z1, Z2Z2, U1, U2, S1, S2, H, I, J, rr, V, X3, Y3, Z3, t;
  fp2_sqr(Z1Z1, G.Z);
  fp2_sqr(Z2Z2, Q.Z);
  fp2_mul(U1, G.X, Z2Z2);
  fp2_mul(U2, Q.X, Z1Z1);
  fp2_mul(S1, G.Y, Q.Z);
  fp2_mul(S1, S1, Z2Z2);
  fp2_mul(S2, Q.Y, G.Z);
  fp2_mul(S2, S2, Z1Z1);
  fp2_sub(H, U2, U1);
  fp2_sub(rr, S2, S1);
  fp2_add(I, H, H);
  fp2_sqr(I, I);
  fp2_mul(J, H, I);
  fp2_add(rr, rr, rr);
  fp2_mul(V, U1, I);
  // row form, g2r_add's steps
  G2R<uint32_t> T{f2r_from(G.X), f2r_from(G.Y), f2r_from(G.Z)}, R{f2r_from(Q.X), f2r_from(Q.Y), f2r_from(Q.Z)};
  uint32_t A[12], B[12], P[12];
  f2r_sqr_ops(A, B, 0, T.Z, c);
  f2r_sqr_ops(A, B, 2, R.Z, c);
  r_prods<4>(P, A, B, c);
  F2R<uint32_t> rZ1Z1, rZ2Z2;
  f2r_sqr_res(rZ1Z1, P, 0);
  f2r_sqr_res(rZ2Z2, P, 2);
  chk("Z1Z1", rZ1Z1, Z1Z1, c);
  chk("Z2Z2", rZ2Z2, Z2Z2, c);
  f2r_mul_ops(A, B, 0, T.X, rZ2Z2);
  f2r_mul_ops(A, B, 3, R.X, rZ1Z1);
  f2r_mul_ops(A, B, 6, T.Y, R.Z);
  f2r_mul_ops(A, B, 9, R.Y, T.Z);
  r_prods<12>(P, A, B, c);
  F2R<uint32_t> rU1, rU2, rY1Z2, rY2Z1;
  f2r_mul_res(rU1, P, 0, c);
  f2r_mul_res(rU2, P, 3, c);
  f2r_mul_res(rY1Z2, P, 6, c);
  f2r_mul_res(rY2Z1, P, 9, c);
  chk("U1", rU1, U1, c);
  chk("U2", rU2, U2, c);
  const F2R<uint32_t> rH = f2r_red(f2r_sub(rU2, rU1, c), c);
  chk("H", rH, H, c);
  const F2R<uint32_t> rH2 = f2r_red(f2r_add(rH, rH), c);
  const F2R<uint32_t> ZS = f2r_red(f2r_add(T.Z, R.Z), c);
  f2r_mul_ops(A, B, 0, rY1Z2, rZ2Z2);
  f2r_mul_ops(A, B, 3, rY2Z1, rZ1Z1);
  f2r_sqr_ops(A, B, 6, rH2, c);
  f2r_sqr_ops(A, B, 8, ZS, c);
  r_prods<10>(P, A, B, c);
  F2R<uint32_t> rS1, rS2, rI, rZS2;
  f2r_mul_res(rS1, P, 0, c);
  f2r_mul_res(rS2, P, 3, c);
  f2r_sqr_res(rI, P, 6);
  f2r_sqr_res(rZS2, P, 8);
  chk("S1", rS1, S1, c);
  chk("S2", rS2, S2, c);
  chk("I", rI, I, c);
  // R4 of g2r_add
  fp2 ZSf, ZZ3;
  fp2_add(ZSf, G.Z, Q.Z);
  fp2_sqr(ZSf, ZSf);
  fp2_sub(ZSf, ZSf, Z1Z1);
  fp2_sub(ZZ3, ZSf, Z2Z2);
  const F2R<uint32_t> rR = f2r_red(f2r_sub(rS2, rS1, c), c);
  const F2R<uint32_t> rZZ = f2r_red(f2r_sub(f2r_sub(rZS2, rZ1Z1, c), rZ2Z2, c), c);
  chk("ZZ", rZZ, ZZ3, c);
  const F2R<uint32_t> rr2 = f2r_red(f2r_add(rR, rR), c);
  chk("r", rr2, rr, c);
  f2r_mul_ops(A, B, 0, rH, rI);
  f2r_mul_ops(A, B, 3, rU1, rI);
  f2r_mul_ops(A, B, 6, rZZ, rH);
  f2r_sqr_ops(A, B, 9, rr2, c);
  r_prods<11>(P, A, B, c);
  F2R<uint32_t> rJ, rV, rZ3, rrr;
  f2r_mul_res(rJ, P, 0, c);
  f2r_mul_res(rV, P, 3, c);
  f2r_mul_res(rZ3, P, 6, c);
  f2r_sqr_res(rrr, P, 9);
  fp2 rsq;
  fp2_sqr(rsq, rr);
  chk("J", rJ, J, c);
  chk("V", rV, V, c);
  chk("rr", rrr, rsq, c);
  {
    fp e8, e9, e10;
    fp2 t8;
    fp2_mul(t8, ZZ3, H);  // product slots: 8 = (ZZ.a + ZZ.b)(H.a + H.b), 9 = (r.a + r.b)(r.a - r.b), 10 = r.a r.b
    fp s1, s2;
    f_add(s1, rr.a, rr.b);
    f_sub(s2, rr.a, rr.b);
    f_mul(e9, s1, s2);
    f_mul(e10, rr.a, rr.b);
    const bool ok9 = same(P[9], e9, c), ok10 = same(P[10], e10, c);
    if (threadIdx.x == 0) printf("P9 %s P10 %s\n", ok9 ? "ok" : "BAD", ok10 ? "ok" : "BAD");
    (void)e8;
  }
  {
    const F2R<uint32_t> mX3 = f2r_red(f2r_sub32(f2r_sub(rrr, rJ, c), f2r_add(rV, rV), c), c);
    fp2 eX3;
    fp2_sub(eX3, rsq, J);
    fp2_sub(eX3, eX3, V);
    fp2_sub(eX3, eX3, V);
    chk("mX3", mX3, eX3, c);
    {
      g2j ee;
      g2_add_j(ee, G, Q);
      uint32_t w1[8], w2[8], w3[8];
      f_to_words(w1, ee.X.b);
      f_to_words(w2, eX3.b);
      fp tmp;
      rf_to_fe(tmp, c.mul(mX3.b, c.one));
      f_to_words(w3, tmp);
      if (threadIdx.x == 0)
        for (int i = 0; i < 8; i++) printf("w%d add_j %08x repl %08x row %08x\n", i, w1[i], w2[i], w3[i]);
      g2j P2;
      g2_dbl_j(P2, G);
      g2j e3;
      g2_add_j(e3, P2, G);  // 3G both ways
      g2j e4;
      g2_add_j(e4, G, P2);
      g2a a3, a4, aq;
      g2_to_affine(a3, e3);
      g2_to_affine(a4, e4);
      g2j ee2;
      g2_add_j(ee2, G, Q);
      g2_to_affine(aq, ee2);
      if (threadIdx.x == 0) printf("3G consistent %d, G+Q == 3G %d\n", (int)fp2_eq(a3.x, a4.x), (int)fp2_eq(aq.x, a3.x));
    }
    const F2R<uint32_t> s1 = f2r_sub(rrr, rJ, c);
    fp2 e1;
    fp2_sub(e1, rsq, J);
    chk("rr-J", f2r_red(s1, c), e1, c);
    const F2R<uint32_t> v2 = f2r_add(rV, rV);
    fp2 e2;
    fp2_add(e2, V, V);
    chk("2V", f2r_red(v2, c), e2, c);
    const F2R<uint32_t> s3 = f2r_sub32(s1, v2, c);
    fp2 e3;
    fp2_sub(e3, e1, e2);
    chk("s32", f2r_red(s3, c), e3, c);
    // R5 replicated
    const F2R<uint32_t> mw = f2r_sub(rV, mX3, c);
    fp2 ew;
    fp2_sub(ew, V, eX3);
    chk("w", mw, ew, c);
    f2r_mul_ops(A, B, 0, rr2, mw);
    f2r_mul_ops(A, B, 3, rS1, rJ);
    r_prods<6>(P, A, B, c);
    F2R<uint32_t> mY3, mSJ;
    f2r_mul_res(mY3, P, 0, c);
    f2r_mul_res(mSJ, P, 3, c);
    fp2 eY3, eSJ;
    fp2_mul(eY3, rr, ew);
    fp2_mul(eSJ, S1, J);
    chk("rw", mY3, eY3, c);
    chk("SJ", mSJ, eSJ, c);
    const F2R<uint32_t> fY3 = f2r_red(f2r_sub32(mY3, f2r_add(mSJ, mSJ), c), c);
    fp2 t2;
    fp2_add(t2, eSJ, eSJ);
    fp2_sub(eY3, eY3, t2);
    chk("mY3", fY3, eY3, c);
    G2R<uint32_t> T4 = T;
    bool sy4;
    g2r_add(T4, R, c, sy4);
    const uint32_t d1 = rf_normalize(c.mul(T4.X.b, c.one)), d2 = rf_normalize(c.mul(mX3.b, c.one));
    const uint32_t z1 = rf_normalize(c.mul(T4.Z.b, c.one)), z2 = rf_normalize(c.mul(rZ3.b, c.one));
    if (threadIdx.x < 9) printf("lane %d fnX3.b %08x myX3.b %08x | fnZ3.b %08x myZ3.b %08x\n", threadIdx.x, d1, d2, z1, z2);
    if (threadIdx.x < 0) printf("lane %2d s3.b %08x red %08x rrr.b %08x J.b %08x V.b %08x\n", threadIdx.x, s3.b, c.red(s3.b), rrr.b, rJ.b, rV.b);
  }
  bool sy;
  {
    fp2 ex[12];
    ex[0] = U1; ex[1] = U2; ex[2] = H; ex[3] = S1; ex[4] = S2; ex[5] = I; ex[6] = J; ex[7] = V;
    fp2_sqr(ex[8], rr);
    fp2_sub(ex[9], ex[8], J); fp2_sub(ex[9], ex[9], V); fp2_sub(ex[9], ex[9], V);
    fp2 w9; fp2_sub(w9, V, ex[9]); fp2_mul(ex[10], rr, w9); fp2_mul(ex[11], S1, J);
    G2R<uint32_t> T9 = T;
    g2r_add_dbg(T9, R, c, sy, ex);
    chk("T9.X", T9.X, ex[9], c);


    const uint64_t nz = __ballot(T9.X.b != 0);
    if (threadIdx.x == 0) printf("T9 X.b nonzero lanes %016llx\n", (unsigned long long)nz);
  }
  G2R<uint32_t> T2 = T;
  const bool okadd = g2r_add(T2, R, c, sy);
  g2j e;
  g2_add_j(e, G, Q);
  g2j got;
  fp2 zero2;
  fp2_zero(zero2);
  (void)zero2;
  {
    const uint32_t v[6] = {T2.X.a, T2.X.b, T2.Y.a, T2.Y.b, T2.Z.a, T2.Z.b};
    for (int k = 0; k < 6; k++) {
      const uint64_t nz = __ballot(v[k] != 0);
      if (threadIdx.x == 0) printf("coord %d nonzero lanes %016llx\n", k, (unsigned long long)nz);
    }
    uint32_t w1[8], w2[8];
    f_to_words(w1, e.X.b);
    fp f;
    rf_to_fe(f, c.mul(T2.X.b, c.one));
    f_to_words(w2, f);
    if (threadIdx.x == 0) for (int i = 0; i < 8; i++) printf("T2.X.b w%d e %08x row %08x\n", i, w1[i], w2[i]);
  }
  chk("X3", T2.X, e.X, c);
  G2R<uint32_t> T3 = T;
  add_noinline(T3, R, sy);
  chk("nX3", T3.X, e.X, c);
  chk("nY3", T3.Y, e.Y, c);  // Jacobian coordinates equal when the formulas match
  chk("Y3", T2.Y, e.Y, c);
  chk("Z3", T2.Z, e.Z, c);
  if (threadIdx.x == 0) printf("add returned %d\n", (int)okadd);
  (void)got;
}
int main() {
  hipLaunchKernelGGL(k_dbg, dim3(1), dim3(64), 0, 0);
  return hipDeviceSynchronize() != hipSuccess;
}
