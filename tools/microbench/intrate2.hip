// gfx950 issue-rate microbenchmark, part 2: the 64-bit integer helpers the compiler emits in the
// field multiply (v_lshrrev_b64, v_lshl_add_u64), the 32-bit glue (and, alignbit, add3, cndmask),
// mixes of v_mad_u64_u32 with 32-bit glue (do they overlap?), and the mad rate at 1/2/4/8 waves
// per SIMD with and without instruction-level parallelism inside the wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 2048
#define CH 8

#define KERNEL32(name, ASM)                                                  \
  __global__ void name(uint32_t* out, uint32_t seed) {                       \
    uint32_t acc[CH];                                                        \
    uint32_t b = seed * 3 + 1, c2 = seed ^ 0x55;                             \
    _Pragma("unroll") for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x; \
    for (int i = 0; i < ITERS; i++) {                                        \
      _Pragma("unroll") for (int c = 0; c < CH; c++) asm volatile(ASM : "+v"(acc[c]) : "v"(b), "v"(c2)); \
    }                                                                        \
    uint32_t s = 0;                                                          \
    _Pragma("unroll") for (int c = 0; c < CH; c++) s += acc[c];              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                          \
  }

KERNEL32(k_and, "v_and_b32 %0, %0, %1")
KERNEL32(k_alignbit, "v_alignbit_b32 %0, %0, %1, 29")
KERNEL32(k_add3, "v_add3_u32 %0, %0, %1, %2")
KERNEL32(k_lshr32, "v_lshrrev_b32 %0, 3, %0")

#define KERNEL64(name, ASM)                                                  \
  __global__ void name(uint32_t* out, uint32_t seed) {                       \
    uint64_t acc[CH];                                                        \
    uint64_t b = seed * 3 + 1;                                               \
    _Pragma("unroll") for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x; \
    for (int i = 0; i < ITERS; i++) {                                        \
      _Pragma("unroll") for (int c = 0; c < CH; c++) asm volatile(ASM : "+v"(acc[c]) : "v"(b)); \
    }                                                                        \
    uint64_t s = 0;                                                          \
    _Pragma("unroll") for (int c = 0; c < CH; c++) s += acc[c];              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32); \
  }

KERNEL64(k_lshr64, "v_lshrrev_b64 %0, 3, %0")
KERNEL64(k_lshladd64, "v_lshl_add_u64 %0, %0, 0, %1")

// v_mad_u64_u32 with CH independent chains (ILP = CH)
__global__ void k_mad64(uint32_t* out, uint32_t seed) {
  uint64_t acc[CH];
  uint32_t a = threadIdx.x ^ seed, b = seed * 3 + 1;
#pragma unroll
  for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) {
      uint64_t cc;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(cc) : "v"(a), "v"(b));
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}
// one dependent chain (ILP = 1)
__global__ void k_mad64_dep(uint32_t* out, uint32_t seed) {
  uint64_t acc = threadIdx.x;
  uint32_t a = threadIdx.x ^ seed, b = seed * 3 + 1;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) {
      uint64_t cc;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(a), "v"(b));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)acc ^ (uint32_t)(acc >> 32);
}
// mad64 interleaved 1:1 with a 32-bit and (independent registers)
__global__ void k_mix_mad_and(uint32_t* out, uint32_t seed) {
  uint64_t acc[CH];
  uint32_t g[CH];
  uint32_t a = threadIdx.x ^ seed, b = seed * 3 + 1;
#pragma unroll
  for (int c = 0; c < CH; c++) { acc[c] = c + threadIdx.x; g[c] = c ^ threadIdx.x; }
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) {
      uint64_t cc;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(cc) : "v"(a), "v"(b));
      asm volatile("v_and_b32 %0, %0, %1" : "+v"(g[c]) : "v"(b));
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s += acc[c] + g[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}
// mad64 interleaved 1:1 with a 64-bit shift
__global__ void k_mix_mad_lshr64(uint32_t* out, uint32_t seed) {
  uint64_t acc[CH], g[CH];
  uint32_t a = threadIdx.x ^ seed, b = seed * 3 + 1;
#pragma unroll
  for (int c = 0; c < CH; c++) { acc[c] = c + threadIdx.x; g[c] = c ^ threadIdx.x; }
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) {
      uint64_t cc;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(cc) : "v"(a), "v"(b));
      asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(g[c]));
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s += acc[c] + g[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

typedef void (*kfn)(uint32_t*, uint32_t);
int main() {
  const int threads = 256;
  uint32_t* d;
  hipMalloc(&d, (size_t)256 * 64 * threads * 4);
  struct {
    const char* name;
    kfn f;
    int instrs_per_iter;
  } ks[] = {{"v_and_b32", k_and, CH},           {"v_alignbit_b32", k_alignbit, CH},
            {"v_add3_u32", k_add3, CH},         {"v_lshrrev_b32", k_lshr32, CH},
            {"v_lshrrev_b64", k_lshr64, CH},    {"v_lshl_add_u64", k_lshladd64, CH},
            {"v_mad_u64_u32 ilp8", k_mad64, CH}, {"v_mad_u64_u32 dep", k_mad64_dep, CH},
            {"mad64+and (per pair)", k_mix_mad_and, CH}, {"mad64+lshr64 (per pair)", k_mix_mad_lshr64, CH}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  printf("clock attr kHz=%d; wave-instr cycles per SIMD assume 2.4 GHz\n", clk);
  for (int wps : {1, 2, 4, 8, 16}) {
    const int blocks = 256 * wps;  // 4 waves per block, 1024 SIMDs: wps waves per SIMD
    for (auto& k : ks) {
      float ms = 0;
      for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 7u);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 7u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
      }
      const double winstr = (double)blocks * (threads / 64) * ITERS * k.instrs_per_iter;  // wave-instructions
      const double per_simd = winstr / 1024.0;
      printf("waves/SIMD %2d  %-26s %8.3f ms  %6.2f cycles per wave-instr per SIMD\n", wps, k.name, ms,
             ms * 1e-3 * 2.4e9 / per_simd);
    }
  }
  return 0;
}
