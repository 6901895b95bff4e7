// Single-lane latency of the BN-P254 building blocks on gfx950 (design input for the BLS
// kernels: a certificate's critical path is chains of these on one lane or one wave).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iconcord-bft_amd/csrc -Iinclude \
//          tools/microbench/bn254_ops.hip -o tools/microbench/bn254_ops
// Prints one JSON object: microseconds per operation (one lane of one wave, REPS in a chain).
#include <hip/hip_runtime.h>

#include <cstdio>

#include "bls_common.h"

#define REPS 64

template <int OP>
__global__ void k_op(uint32_t* io) {
  if (threadIdx.x != 0) return;
  fp a, b;
  for (int i = 0; i < 9; i++) {
    a.v[i] = io[i] & BN_MASK;
    b.v[i] = io[9 + i] & BN_MASK;
  }
  a.v[8] &= 0xfffff;
  b.v[8] &= 0xfffff;
  g1j P;
  P.X = a;
  P.Y = b;
  f_one(P.Z);
  g1a A;
  A.x = a;
  A.y = b;
  A.inf = false;
  uint8_t buf[33];
  for (int r = 0; r < REPS; r++) {
    if (OP == 0) f_mul(a, a, b);
    if (OP == 1) f_sqr(a, a);
    if (OP == 2) fp_inv(a, a);
    if (OP == 3) fp_inv_vt(a, a);
    if (OP == 4) fp_sqrt(a, a);
    if (OP == 5) g1_dbl(P, P);
    if (OP == 6) {
      g1j Q = P;
      Q.X = b;
      g1_add(P, P, Q);
    }
    if (OP == 7) {
      g1_to_affine(A, P, true);
      P.X = A.y;
    }
    if (OP == 8) {
      g1_compress(buf, A);
      A.x.v[0] ^= buf[3];
    }
    if (OP == 9) {
      a.v[0] ^= f_relic_bit(a);
    }
  }
  for (int i = 0; i < 9; i++) io[18 + i] = a.v[i] ^ P.X.v[i] ^ A.x.v[i] ^ buf[i];
}

template <int OP>
static float run(uint32_t* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k_op<OP>, dim3(1), dim3(64), 0, 0, d);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k_op<OP>, dim3(1), dim3(64), 0, 0, d);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / REPS;
}

int main() {
  uint32_t h[27];
  for (int i = 0; i < 27; i++) h[i] = 0x1234567u * (i + 3) + 0x9e3779b9u;
  uint32_t* d;
  hipMalloc(&d, sizeof(h));
  hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  printf("{\"us_per_op\": {\"f_mul\": %.3f, \"f_sqr\": %.3f, \"fp_inv\": %.2f, \"fp_inv_vt\": %.2f, \"fp_sqrt\": %.2f, ",
         run<0>(d), run<1>(d), run<2>(d), run<3>(d), run<4>(d));
  printf("\"g1_dbl\": %.2f, \"g1_add\": %.2f, \"g1_to_affine_vt\": %.2f, \"g1_compress\": %.2f, \"relic_bit\": %.2f}}\n",
         run<5>(d), run<6>(d), run<7>(d), run<8>(d), run<9>(d));
  hipFree(d);
  return 0;
}
