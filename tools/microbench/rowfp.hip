// Latency of one dependent BN-P254 Fp multiplication on a lone wave: the one-lane f_mul
// (bn254_field.h, what bn254_g1quad.h runs per round) against the row-parallel rf_mul
// (bn254_row.h).  Both chains start from the same operands; the results must agree mod q.
//   hipcc --offload-arch=gfx950 -O3 -I concord-bft_amd/csrc tools/microbench/rowfp.hip -o tools/microbench/rowfp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "bn254_row.h"

__global__ void __launch_bounds__(64) chain_fmul(const uint32_t* in, uint32_t* out, int n) {
  fp x, y;
  for (int i = 0; i < 9; i++) {
    x.v[i] = in[i];
    y.v[i] = in[9 + i];
  }
#pragma unroll 1
  for (int k = 0; k < n; k++) f_mul(x, x, y);
  uint32_t w[8];
  f_to_words(w, x);
  if (threadIdx.x == 0)
    for (int i = 0; i < 8; i++) out[i] = w[i];
}

__global__ void __launch_bounds__(64) chain_rfmul(const uint32_t* in, uint32_t* out, int n) {
  fp x, y;
  for (int i = 0; i < 9; i++) {
    x.v[i] = in[i];
    y.v[i] = in[9 + i];
  }
  const uint32_t tag = 0;
  uint32_t rx = rf_from_fe(x, tag), ry = rf_from_fe(y, tag);
  const uint32_t qrow = rf_row_const(FpParams::Q, tag);
#pragma unroll 1
  for (int k = 0; k < n; k++) rx = rf_mul<uint32_t, uint64_t>(rx, ry, qrow);
  fp r;
  rf_to_fe(r, rx);
  uint32_t w[8];
  f_to_words(w, r);
  if (threadIdx.x == 0)
    for (int i = 0; i < 8; i++) out[i] = w[i];
}

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(1);                                                    \
    }                                                                  \
  } while (0)

int main() {
  uint32_t h_in[18];
  fp a, b;
  uint32_t wa[8] = {0x12345678, 0x9abcdef0, 0x0fedcba9, 0x87654321, 0x11111111, 0x22222222, 0x33333333, 0x01234567};
  uint32_t wb[8] = {0xdeadbeef, 0xcafebabe, 0x01010101, 0x10203040, 0x55555555, 0x66666666, 0x77777777, 0x0abcdef1};
  f_from_words(a, wa);
  f_from_words(b, wb);
  for (int i = 0; i < 9; i++) {
    h_in[i] = a.v[i];
    h_in[9 + i] = b.v[i];
  }
  uint32_t *d_in, *d_out;
  CK(hipMalloc(&d_in, sizeof h_in));
  CK(hipMalloc(&d_out, 64));
  CK(hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int n = 20000;
  uint32_t res[2][8];
  float ms[2];
  for (int mode = 0; mode < 2; mode++) {
    for (int rep = 0; rep < 2; rep++) {  // second run timed
      CK(hipEventRecord(e0));
      if (mode == 0)
        hipLaunchKernelGGL(chain_fmul, dim3(1), dim3(64), 0, 0, d_in, d_out, n);
      else
        hipLaunchKernelGGL(chain_rfmul, dim3(1), dim3(64), 0, 0, d_in, d_out, n);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms[mode], e0, e1));
    }
    CK(hipMemcpy(res[mode], d_out, 32, hipMemcpyDeviceToHost));
  }
  bool same = true;
  for (int i = 0; i < 8; i++) same &= res[0][i] == res[1][i];
  std::printf("{\"chain\": %d, \"f_mul_ns\": %.1f, \"rf_mul_ns\": %.1f, \"speedup\": %.2f, \"results_equal\": %s}\n", n,
              ms[0] * 1e6 / n, ms[1] * 1e6 / n, ms[0] / ms[1], same ? "true" : "false");
  return same ? 0 : 1;
}
