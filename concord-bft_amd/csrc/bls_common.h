// Helpers shared by the BLS kernel translation units (internal).
#pragma once
#include <hip/hip_runtime.h>

#include "bls_kernels.h"
#include "bls_ops.h"

#define LINES_PER_KEY (BN_ATE_LINES * BN_LINE_WORDS)

__device__ __forceinline__ void g1a_store(uint32_t* o, const g1a& a) {
  for (int i = 0; i < 9; i++) {
    o[i] = a.x.v[i];
    o[9 + i] = a.y.v[i];
  }
  o[18] = a.inf ? 1u : 0u;
}
__device__ __forceinline__ void g1a_load(g1a& a, const uint32_t* o) {
  for (int i = 0; i < 9; i++) {
    a.x.v[i] = o[i];
    a.y.v[i] = o[9 + i];
  }
  a.inf = o[18] != 0;
}

__device__ __forceinline__ void g2a_store(uint32_t* o, const g2a& a) {
  for (int i = 0; i < 9; i++) {
    o[i] = a.x.a.v[i];
    o[9 + i] = a.x.b.v[i];
    o[18 + i] = a.y.a.v[i];
    o[27 + i] = a.y.b.v[i];
  }
  o[36] = a.inf ? 1u : 0u;
}
__device__ __forceinline__ void g2a_load(g2a& a, const uint32_t* o) {
  for (int i = 0; i < 9; i++) {
    a.x.a.v[i] = o[i];
    a.x.b.v[i] = o[9 + i];
    a.y.a.v[i] = o[18 + i];
    a.y.b.v[i] = o[27 + i];
  }
  a.inf = o[36] != 0;
}

