// BLS BN-P254 G1 / scalar kernels for gfx950 (threshsign path).
//
//   bls_hash_kernel          H = g1_map(digest)            (BlsAccumulatorBase.cpp:55-60)
//   bls_inv_table_kernel     inverses of 1..2048 mod r (once per context)
//   bls_lagrange_kernel      one wave per share: lambda_i = prod_{j!=i} j/(j-i) mod r
//                            (lagrangeCoeffAccumReduced, LagrangeInterpolation.cpp:202-292)
//   (the MSM itself, fastMultExp FastMultExp.cpp:26-59, is bls_msm_row.hip's row-parallel GLV form)
//   bls_msm_finish_kernel    sum of partials -> 33-byte compressed G1 (or one Jacobian partial)
#include <cstdlib>
#include <cstring>

#include "bls_common.h"
#include "bn254_g1quad.h"

// one wave: the candidates are tried four at a time, one per DPP row (g1_map_row)
__global__ void __launch_bounds__(64) bls_hash_kernel(const uint8_t* msg, uint32_t len, uint32_t* H) {
  if (blockIdx.x != 0) return;
  g1a h;
  g1_map_row(h, msg, len);
  if (threadIdx.x == 0) g1a_store(H, h);
}

// inv[d] = d^-1 mod r (Montgomery form), d = 1 .. BLS_INV_TABLE (the reference keeps the same
// table of small inverses, Library.cpp:22-41); built once per context.
__global__ void __launch_bounds__(64) bls_inv_table_kernel(uint32_t* inv) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x + 1;
  if (d > BLS_INV_TABLE) return;
  uint32_t w[8] = {d, 0, 0, 0, 0, 0, 0, 0};
  fr x;
  f_from_words(x, w);
  fr_inv(x, x);
  for (int q = 0; q < 9; q++) inv[9 * (size_t)(d - 1) + q] = x.v[q];
}

__device__ __forceinline__ void fr_shfl_xor(fr& r, const fr& x, int m) {
#pragma unroll
  for (int q = 0; q < 9; q++) r.v[q] = (uint32_t)__shfl_xor((int)x.v[q], m);
}

// lambda_i = prod_{j != i} id_j / (id_j - id_i) mod r over the shares with use[j] != 0
// (lagrangeCoeffAccumReduced, LagrangeInterpolation.cpp:202-292; the coefficients are unique, so
// any evaluation order gives the reference's values).  One wave per coefficient: lane l takes
// j = l, l + 64, ..., multiplying id_j into the numerator and inv[|id_j - id_i|] into the
// inverted denominator and counting the j with id_j < id_i (each flips the sign); a butterfly
// over the wave combines the lanes.  No inversion at run time: O(k / 64 + 6) multiplications of
// latency per coefficient, k waves in flight.  Words out (LE).
__global__ void __launch_bounds__(64) bls_lagrange_kernel(const uint32_t* ids, const uint8_t* use, uint32_t k,
                                                          const uint32_t* inv, uint32_t* lambda) {
  const uint32_t i = blockIdx.x;
  const int ln = threadIdx.x;
  if (i >= k) return;
  const uint32_t me = ids[i];
  fr num, den;
  f_one(num);
  f_one(den);
  uint32_t below = 0;
  const bool on = use[i] != 0;
  for (uint32_t j = ln; on && j < k; j += 64) {
    if (j == i || !use[j]) continue;
    const uint32_t o = ids[j];
    uint32_t v[8] = {o, 0, 0, 0, 0, 0, 0, 0};
    fr t;
    f_from_words(t, v);
    f_mul(num, num, t);
    const uint32_t d = o > me ? o - me : me - o;  // 1 <= d < BLS_INV_TABLE (distinct ids <= 2048)
    fr iv;
#pragma unroll
    for (int q = 0; q < 9; q++) iv.v[q] = inv[9 * (size_t)(d - 1) + q];
    f_mul(den, den, iv);
    below += o < me ? 1u : 0u;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    fr a, b;
    fr_shfl_xor(a, num, m);
    fr_shfl_xor(b, den, m);
    f_mul(num, num, a);
    f_mul(den, den, b);
    below += (uint32_t)__shfl_xor((int)below, m);
  }
  if (ln != 0) return;
  uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (on) {
    f_mul(num, num, den);
    if (below & 1u) f_neg(num, num);  // each id_j < id_i contributes 1 / (negative)
    f_to_words(w, num);
  }
  for (int q = 0; q < 8; q++) lambda[8 * (size_t)i + q] = w[q];
}

#define MSM_QUADS 16  // shares (lane quads) per 64-lane MSM block

__device__ __forceinline__ void g1j_put(uint32_t* o, int stride, const g1j& a, int q) {
#pragma unroll
  for (int w = 0; w < 27; w++) {
    const uint32_t v = w < 9 ? a.X.v[w] : (w < 18 ? a.Y.v[w - 9] : a.Z.v[w - 18]);
    if ((w & 3) == q) o[w * stride] = v;
  }
}
__device__ __forceinline__ void g1j_get(g1j& a, const uint32_t* o, int stride) {
#pragma unroll
  for (int w = 0; w < 9; w++) {
    a.X.v[w] = o[w * stride];
    a.Y.v[w] = o[(9 + w) * stride];
    a.Z.v[w] = o[(18 + w) * stride];
  }
}

// sum of the MSM_QUADS quads' points of a 64-lane block (LDS tree, quad adds); quad 0 ends
// with it
__device__ __forceinline__ void g1q_block_sum(g1j& acc, uint32_t (*sp)[27], int qd, int q) {
#pragma unroll 1
  for (int stride = MSM_QUADS / 2; stride >= 1; stride >>= 1) {
    if (qd >= stride && qd < 2 * stride) g1j_put(sp[qd - stride], 1, acc, q);
    __syncthreads();
    if (qd < stride) {
      g1j o;
      g1j_get(o, sp[qd], 1);
      g1q_add(acc, acc, o, q);
    }
    __syncthreads();
  }
}

// Sum of nparts Jacobian partials (27 words each): compressed into out33, or (out_jac) left as
// one Jacobian partial -- the form ranks exchange when a combine is sharded across GPUs.  One
// block of 16 quads: quad qd sums partials qd, qd + 16, ..., then the LDS tree.
__global__ void __launch_bounds__(64) bls_msm_finish_kernel(const uint32_t* partial, uint32_t nparts, uint8_t* out33,
                                                            uint32_t* sig_aff, uint32_t* out_jac) {
  __shared__ uint32_t sp[MSM_QUADS / 2][27];
  if (blockIdx.x != 0) return;
  const int qd = threadIdx.x >> 2, q = threadIdx.x & 3;
  g1j acc;
  if (nparts == 1) {  // the row MSM's single partial: no sum (the 16-quad tree cost ~32 us)
    if (qd != 0) return;
    g1j_get(acc, partial, 1);
  } else {
    g1_set_inf(acc);
#pragma unroll 1
    for (uint32_t b = qd; b < nparts; b += MSM_QUADS) {
      g1j o;
      g1j_get(o, partial + 27 * (size_t)b, 1);
      g1q_add(acc, acc, o, q);
    }
    g1q_block_sum(acc, sp, qd, q);
    if (qd != 0) return;
  }
  if (out_jac) {
    g1j_put(out_jac, 1, acc, q);
    return;
  }
  g1a a;
  g1_to_affine<true>(a, acc);  // the combined signature is public: variable-time inversion
  if (q == 0) {
    g1_compress(out33, a);
    if (sig_aff) g1a_store(sig_aff, a);
  }
}

// use[j] = a[j] && b[j] (first occurrence of an id && share verified), k bytes
__global__ void __launch_bounds__(256) bls_and_kernel(const uint8_t* a, const uint8_t* b, uint8_t* use, uint32_t k) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < k) use[j] = (a[j] && b[j]) ? 1 : 0;
}

// ------------------------------------------------------------------------------ launchers
hipError_t cbft_bls_launch_and(const uint8_t* d_a, const uint8_t* d_b, uint8_t* d_use, uint32_t k, hipStream_t s) {
  if (!k) return hipSuccess;
  hipLaunchKernelGGL(bls_and_kernel, dim3((k + 255) / 256), dim3(256), 0, s, d_a, d_b, d_use, k);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_hash(const uint8_t* d_msg, uint32_t len, uint32_t* d_H, hipStream_t s) {
  hipLaunchKernelGGL(bls_hash_kernel, dim3(1), dim3(64), 0, s, d_msg, len, d_H);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_inv_table(uint32_t* d_inv, hipStream_t s) {
  hipLaunchKernelGGL(bls_inv_table_kernel, dim3((BLS_INV_TABLE + 63) / 64), dim3(64), 0, s, d_inv);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_combine(const uint32_t* d_sig, const uint32_t* d_ids, const uint8_t* d_use, uint32_t k,
                                   uint32_t lo, uint32_t hi, int multisig, const uint32_t* d_inv, uint32_t* d_lambda,
                                   uint32_t* d_partial, uint8_t* d_out33, uint32_t* d_sig_aff, uint32_t* d_out_jac,
                                   hipStream_t s) {
  if (!multisig && k)
    hipLaunchKernelGGL(bls_lagrange_kernel, dim3(k), dim3(64), 0, s, d_ids, d_use, k, d_inv, d_lambda);
  hi = hi < k ? hi : k;
  lo = lo < hi ? lo : hi;
  const uint32_t m = hi - lo;  // the MSM runs over shares [lo, hi) only
  uint32_t* fin = nullptr;
  hipError_t e = cbft_bls_launch_msm_row(d_sig + BLS_SIG_WORDS * (size_t)lo, d_lambda + 8 * (size_t)lo, d_use + lo,
                                         m, multisig, d_partial, &fin, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(bls_msm_finish_kernel, dim3(1), dim3(64), 0, s, fin, 1u, d_out33, d_sig_aff, d_out_jac);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_g1_parts(const uint32_t* d_parts, uint32_t count, uint8_t* d_out33, hipStream_t s) {
  hipLaunchKernelGGL(bls_msm_finish_kernel, dim3(1), dim3(64), 0, s, d_parts, count, d_out33, nullptr, nullptr);
  return hipGetLastError();
}
