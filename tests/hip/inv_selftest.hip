// Test-only device harness (not part of the product library): the wave-cooperative variable-time
// inversion of safegcd30.h (sg_inv30_var_wave) and the one-lane form (sg_inv30_var), one wave per
// value, for BN-P254's p and 2^255 - 19, so tests/test_inv_gpu.py can check the primitive itself
// on gfx950 against Python integers -- adversarial values included, not only the values the
// finish kernel and the pairing checks happen to feed it.
#include <hip/hip_runtime.h>

#include "safegcd30.h"

struct BnMod {  // p in signed-30 limbs and p^-1 mod 2^30 (bn254_field.h: BnS30Mod)
  static constexpr int32_t P[9] = {0x00000013, 0x1c000000, 0x0000013a, 0x08400000, 0x00000861,
                                   0x11360000, 0x00001ba3, 0x19209000, 0x00002523};
  static constexpr uint32_t PINV30 = 0x286bca1bu;
};
struct EdMod {  // 2^255 - 19 (fe25519.h: Fe25519S30)
  static constexpr int32_t P[9] = {0x3fffffed, 0x3fffffff, 0x3fffffff, 0x3fffffff, 0x3fffffff,
                                   0x3fffffff, 0x3fffffff, 0x3fffffff, 0x00007fff};
  static constexpr uint32_t PINV30 = 0x179435e5u;
};

template <class M>
__global__ void __launch_bounds__(64) inv_kernel(const int32_t* in, int32_t* wave_out, int32_t* lane_out) {
#if defined(__HIP_DEVICE_COMPILE__)  // (sg_inv30_var_wave is device code only)
  const int i = blockIdx.x;
  Sg30 x, y;
#pragma unroll
  for (int j = 0; j < 9; j++) x.v[j] = in[9 * i + j];
  y = x;
  sg_inv30_var_wave<M>(x);  // every lane of the wave takes part
  if (threadIdx.x == 5) sg_inv30_var<M>(y);  // the one-lane form on one lane
  if (threadIdx.x == 5) {
#pragma unroll
    for (int j = 0; j < 9; j++) {
      wave_out[9 * i + j] = x.v[j];
      lane_out[9 * i + j] = y.v[j];
    }
  }
#endif
}

// n values of 9 signed-30 limbs each (canonical, < p): which = 0 BN-P254, 1 2^255 - 19.  0 or a HIP error.
extern "C" int inv_selftest(const int32_t* h_in, int32_t* h_wave, int32_t* h_lane, int n, int which) {
  if (n <= 0) return 0;
  const size_t bytes = (size_t)n * 9 * sizeof(int32_t);
  int32_t *d_in = nullptr, *d_w = nullptr, *d_l = nullptr;
  hipError_t e = hipMalloc(&d_in, bytes);
  if (e == hipSuccess) e = hipMalloc(&d_w, bytes);
  if (e == hipSuccess) e = hipMalloc(&d_l, bytes);
  if (e == hipSuccess) e = hipMemcpy(d_in, h_in, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    if (which == 0)
      hipLaunchKernelGGL(inv_kernel<BnMod>, dim3(n), dim3(64), 0, 0, d_in, d_w, d_l);
    else
      hipLaunchKernelGGL(inv_kernel<EdMod>, dim3(n), dim3(64), 0, 0, d_in, d_w, d_l);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(h_wave, d_w, bytes, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(h_lane, d_l, bytes, hipMemcpyDeviceToHost);
  (void)hipFree(d_in);
  (void)hipFree(d_w);
  (void)hipFree(d_l);
  return (int)e;
}
