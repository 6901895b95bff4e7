// Device check of the key-sum data path: rows -> partial words -> rows -> g2r_add -> words ->
// one-lane affine, against the one-lane sum (debug aid).
#include <hip/hip_runtime.h>

#include <cstdio>

#include "bn254_g2row.h"
#include "bn254_pairing.h"
#include "bls_common.h"

using C2 = G2RowCtx<uint32_t, uint64_t>;
__device__ void part_store(uint32_t* o, const G2R<uint32_t>& p, const C2& c) {
  uint32_t A[6] = {p.X.a, p.X.b, p.Y.a, p.Y.b, p.Z.a, p.Z.b}, B[6], P[6];
  for (int i = 0; i < 6; i++) B[i] = c.one;
  r_prods<6>(P, A, B, c);
  for (int i = 0; i < 6; i++) rf_st9_row0(o + 9 * i, P[i]);
}
__device__ void part_load(G2R<uint32_t>& p, const uint32_t* o) {
  p.X = f2r_ld(o);
  p.Y = f2r_ld(o + 18);
  p.Z = f2r_ld(o + 36);
}
__global__ void k_dbg(uint32_t* mem) {
  const C2 c(0u);
  g2j G, Q2;
  fp2_load(G.X, Bn254Consts::G2X);
  fp2_load(G.Y, Bn254Consts::G2Y);
  fp2_one(G.Z);
  g2_dbl_j(Q2, G);
  g2a qa;
  g2_to_affine(qa, Q2);
  G2R<uint32_t> T{f2r_from(G.X), f2r_from(G.Y), f2r_from(G.Z)}, R{f2r_from(qa.x), f2r_from(qa.y), f2r_from(G.Z)};
  part_store(mem, T, c);
  part_store(mem + 64, R, c);
  __syncthreads();
  G2R<uint32_t> a, b;
  part_load(a, mem);
  part_load(b, mem + 64);
  bool sy;
  const bool r1 = g2r_add(a, b, c, sy);
  G2R<uint32_t> a2 = T;
  const bool r2 = g2r_add(a2, R, c, sy);
  part_store(mem + 128, a, c);
  part_store(mem + 192, a2, c);
  __syncthreads();
  g2j s1, s2, e;
  g2j_load(s1, mem + 128);
  g2j_load(s2, mem + 192);
  g2j Qj{qa.x, qa.y, G.Z};
  g2_add_j(e, G, Qj);
  g2a x1, x2, xe;
  g2_to_affine(x1, s1);
  g2_to_affine(x2, s2);
  g2_to_affine(xe, e);
  uint8_t b1[65], b2[65], be[65];
  g2_compress(b1, x1);
  g2_compress(b2, x2);
  g2_compress(be, xe);
  int d1 = 0, d2 = 0;
  for (int i = 0; i < 65; i++) {
    d1 |= b1[i] != be[i];
    d2 |= b2[i] != be[i];
  }
  if (threadIdx.x == 0) printf("ret %d %d  via memory %s  registers %s\n", r1, r2, d1 ? "BAD" : "ok", d2 ? "BAD" : "ok");
  if (threadIdx.x == 0)
    for (int i = 0; i < 65; i++) {
      mem[256 + i] = b1[i];
      mem[384 + i] = b2[i];
      mem[512 + i] = be[i];
    }
  if (threadIdx.x == 0)
    for (int i = 0; i < 54; i++)
      if (mem[i] != 0 || mem[64 + i] != 0) {}
  // compare loaded operands with the registers they came from
  const uint32_t dx = rf_normalize(c.mul(a2.X.a, c.one)) ^ rf_normalize(c.mul(a.X.a, c.one));
  if (threadIdx.x < 9) printf("lane %d diff Xa %08x\n", threadIdx.x, dx);
}
int main() {
  uint32_t* m;
  hipMalloc(&m, 4096);
  hipMemset(m, 0, 4096);
  hipLaunchKernelGGL(k_dbg, dim3(1), dim3(64), 0, 0, m);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  uint32_t h[640];
  hipMemcpy(h, m, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[3] = {"row_mem", "row_reg", "onelane"};
  for (int k = 0; k < 3; k++) {
    printf("%s ", names[k]);
    for (int i = 0; i < 65; i++) printf("%02x", h[256 + 128 * k + i]);
    printf("\n");
  }
  return 0;
}
