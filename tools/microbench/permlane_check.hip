// Device check of rl_all_rows (row_lanes.h): every lane of every row must receive each row's
// value of its own row lane.  Prints "permlane ok" or the first mismatch.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "row_lanes.h"

__global__ void k(uint32_t* out) {
  const uint32_t l = threadIdx.x;
  uint32_t r[4];
  rl_all_rows(1000u * l + 7u, r);
  for (int s = 0; s < 4; s++) out[4 * l + s] = r[s];
}

int main() {
  uint32_t* d;
  if (hipMalloc(&d, 256 * 4) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  uint32_t h[256];
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int l = 0; l < 64; l++)
    for (int s = 0; s < 4; s++) {
      const uint32_t want = 1000u * (16 * s + (l & 15)) + 7u;
      if (h[4 * l + s] != want) {
        std::printf("permlane MISMATCH lane %d row %d: %u want %u\n", l, s, h[4 * l + s], want);
        return 2;
      }
    }
  std::printf("permlane ok\n");
  return 0;
}
