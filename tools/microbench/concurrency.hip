// Do kernels on two HIP streams co-run on MI355X?  Two "lone-wave" ALU kernels (256 blocks x
// 256 threads = 1 wave per SIMD each, ~100 VGPRs) launched on two streams vs back-to-back on one.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) alu(uint32_t* out, int iters) {
  uint32_t a = threadIdx.x, b = blockIdx.x, c = 7, d = 11;
  for (int i = 0; i < iters; i++) {
    a = a * 2654435761u + b;
    b = b ^ (a >> 7);
    c = c * 40503u + d;
    d = d + (c >> 3);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d;
}

int main() {
  uint32_t* buf;
  hipMalloc(&buf, 1 << 24);
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int rep = 0; rep < 2; rep++) {
    for (int mode = 0; mode < 2; mode++) {
      hipDeviceSynchronize();
      hipEventRecord(e0, 0);
      hipDeviceSynchronize();
      for (int k = 0; k < 4; k++) {
        hipLaunchKernelGGL(alu, dim3(256), dim3(256), 0, s1, buf, iters);
        hipLaunchKernelGGL(alu, dim3(256), dim3(256), 0, mode ? s2 : s1, buf + (1 << 20), iters);
      }
      hipDeviceSynchronize();
      hipEventRecord(e1, 0);
      hipDeviceSynchronize();
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("%s: 8 kernels in %.3f ms\n", mode ? "two streams" : "one stream ", ms);
    }
  }
  return 0;
}
