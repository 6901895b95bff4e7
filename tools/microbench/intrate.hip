// Integer VALU issue-rate microbenchmark for gfx950 (design input for the field arithmetic).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
#define CH 8

__global__ void k_mad64(uint32_t* out, uint32_t seed) {
  uint64_t acc[CH]; uint32_t a = threadIdx.x ^ seed, b = seed * 3 + 1;
#pragma unroll
  for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++)
      { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(cc) : "v"(a), "v"(b)); }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}
__global__ void k_mullo(uint32_t* out, uint32_t seed) {
  uint32_t acc[CH]; uint32_t b = seed * 3 + 1;
#pragma unroll
  for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mulhi(uint32_t* out, uint32_t seed) {
  uint32_t acc[CH]; uint32_t b = seed * 3 + 1;
#pragma unroll
  for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mad24(uint32_t* out, uint32_t seed) {
  uint32_t acc[CH]; uint32_t a = threadIdx.x ^ seed, b = seed * 3 + 1;
#pragma unroll
  for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mulhi24(uint32_t* out, uint32_t seed) {
  uint32_t acc[CH]; uint32_t b = seed * 3 + 1;
#pragma unroll
  for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_add(uint32_t* out, uint32_t seed) {
  uint32_t acc[CH]; uint32_t b = seed * 3 + 1;
#pragma unroll
  for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_addco(uint32_t* out, uint32_t seed) {
  uint32_t acc[CH]; uint32_t b = seed * 3 + 1;
#pragma unroll
  for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CH; c += 2)
      asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc" : "+v"(acc[c]), "+v"(acc[c+1]) : "v"(b) : "vcc");
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fma64(uint32_t* out, uint32_t seed) {
  double acc[CH]; double a = 1.0000001 + threadIdx.x * 1e-9, b = 0.9999999;
#pragma unroll
  for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(acc[c]) : "v"(a), "v"(b));
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}
__global__ void k_fma32(uint32_t* out, uint32_t seed) {
  float acc[CH]; float a = 1.0001f, b = 0.9999f;
#pragma unroll
  for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(acc[c]) : "v"(a), "v"(b));
  }
  float s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}

typedef void (*kfn)(uint32_t*, uint32_t);
int main() {
  const int blocks = 256 * 16, threads = 256;
  uint32_t* d; hipMalloc(&d, (size_t)blocks * threads * 4);
  struct { const char* name; kfn f; int instrs_per_iter; } ks[] = {
    {"v_mad_u64_u32", k_mad64, CH}, {"v_mul_lo_u32", k_mullo, CH}, {"v_mul_hi_u32", k_mulhi, CH},
    {"v_mad_u32_u24", k_mad24, CH}, {"v_mul_hi_u32_u24", k_mulhi24, CH}, {"v_add_u32", k_add, CH},
    {"v_add_co+addc (per instr)", k_addco, CH}, {"v_fma_f64", k_fma64, CH}, {"v_fma_f32", k_fma32, CH}};
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int clk = 0; hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  printf("clock attr kHz=%d\n", clk);
  for (auto& k : ks) {
    for (int rep = 0; rep < 3; rep++) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 7u);
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 7u);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double ops = (double)blocks * threads * ITERS * k.instrs_per_iter;
      if (rep == 2) printf("%-28s %8.3f ms  %.3e lane-ops/s  = %.3f of 256CUx4x32x2.4GHz\n", k.name, ms, ops / (ms * 1e-3), ops / (ms * 1e-3) / 7.864e13);
    }
  }
  return 0;
}
