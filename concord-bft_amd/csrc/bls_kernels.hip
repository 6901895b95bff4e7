// BLS BN-P254 G1 / scalar kernels for gfx950 (threshsign path).
//
//   bls_hash_kernel          H = g1_map(digest)            (BlsAccumulatorBase.cpp:55-60)
//   bls_inv_table_kernel     inverses of 1..2048 mod r (once per context)
//   bls_lagrange_kernel      one wave per share: lambda_i = prod_{j!=i} j/(j-i) mod r
//                            (lagrangeCoeffAccumReduced, LagrangeInterpolation.cpp:202-292)
//   bls_msm_kernel           lane quad per share: lambda_i sigma_i, LDS tree sum per block
//                            (fastMultExp, FastMultExp.cpp:26-59; multisig: lambda = 1)
//   bls_msm_finish_kernel    sum of block partials -> 33-byte compressed G1
//   bls_sign_kernel          sigma = sk * g1_map(msg)     (BlsThresholdSigner.cpp:32-47)
#include <cstdlib>
#include <cstring>

#include "bls_common.h"
#include "bn254_g1quad.h"
#ifndef CBFT_BLS_PHASES
#define CBFT_BLS_PHASES 0  // probe builds: bls_msm_finish_kernel prints its phase times
#endif

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

#include "bls_glv.h"

__device__ __forceinline__ void g1j_neg_if(g1j& p, bool neg) {
  fp n;
  f_neg(n, p.Y);
#pragma unroll
  for (int q = 0; q < 9; q++) p.Y.v[q] = neg ? n.v[q] : p.Y.v[q];
}

// Jacobian point <-> 27 LDS / global words, the quad's lane q moving words q, q + 4, ...
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

// partial[b] = sum over this block's 16 shares of lambda_j sigma_j (Jacobian, 27 words).  One lane
// QUAD per share (bn254_g1quad.h: the independent products of each doubling / addition on
// separate lanes).  lambda_j sigma_j = k1 sigma_j + k2 phi(sigma_j) (GLV): 33 signed radix-16
// windows, each 4 doublings + one addition from the share's LDS table {1..8} sigma (+ one from
// the phi table {1..8} phi(sigma), phi: X -> beta X) -- 132 doublings and 66 additions instead
// of 256 and ~128 for fastMultExp's double-and-add (FastMultExp.cpp:26-59).  Multisig (unit
// scalars): sum sigma_j.
__global__ void __launch_bounds__(64) bls_msm_kernel(const uint32_t* sig, const uint32_t* lambda, const uint8_t* use,
                                                     uint32_t k, int unit_scalars, uint32_t* partial) {
  __shared__ uint32_t sp[MSM_QUADS / 2][27];
  __shared__ uint32_t tbl[2][8][27][MSM_QUADS];  // [phi][multiple - 1][word][quad]
  const int qd = threadIdx.x >> 2, q = threadIdx.x & 3;
  const uint32_t j = blockIdx.x * MSM_QUADS + qd;
  g1j acc;
  g1_set_inf(acc);
  const bool live = j < k && use[j];
  if (live && unit_scalars) {
    g1a s;
    g1a_load(s, sig + 19 * (size_t)j);
    g1_from_affine(acc, s);
  }
  if (!unit_scalars) {  // block-uniform
    g1a s;
    uint32_t lw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (live) {
      g1a_load(s, sig + 19 * (size_t)j);
      for (int w = 0; w < 8; w++) lw[w] = lambda[8 * (size_t)j + w];
    } else {
      s.inf = true;
    }
    g1j P;
    g1_from_affine(P, s);
    fp beta;
    {
      uint32_t bw[8];
      for (int w = 0; w < 8; w++) bw[w] = kGlvBeta[w];
      f_from_words(beta, bw);
    }
    // tables m * sigma and phi(m * sigma), m = 1..8
    g1j T = P;
#pragma unroll 1
    for (int m = 1; m <= 8; m++) {
      if (m == 2)
        g1q_dbl(T, P, q);
      else if (m > 2)
        g1q_add(T, T, P, q);
      g1j_put(&tbl[0][m - 1][0][qd], MSM_QUADS, T, q);
      g1j F = T;
      f_mul(F.X, T.X, beta);
      g1j_put(&tbl[1][m - 1][0][qd], MSM_QUADS, F, q);
    }
    uint32_t k1[5], k2[5];
    bool n1, n2;
    glv_split(lw, k1, k2, n1, n2);
    glv_offset(k1);
    glv_offset(k2);
#pragma nounroll
    for (int w = 32; w >= 0; w--) {
      if (w != 32)
#pragma unroll 1
        for (int d = 0; d < 4; d++) g1q_dbl(acc, acc, q);
#pragma unroll
      for (int half = 0; half < 2; half++) {
        const int dg = glv_digit(half ? k2 : k1, w);
        if (dg == 0) continue;  // quad-uniform
        const int m = (dg < 0 ? -dg : dg) - 1;
        g1j E;
        g1j_get(E, &tbl[half][m][0][qd], MSM_QUADS);
        g1j_neg_if(E, (dg < 0) != (half ? n2 : n1));
        g1q_add(acc, acc, E, q);
      }
    }
  }
  __syncthreads();
  g1q_block_sum(acc, sp, qd, q);
  if (qd == 0) g1j_put(partial + 27 * (size_t)blockIdx.x, 1, acc, q);
}

// Sum of nparts Jacobian partials (27 words each): compressed into out33, or (out_jac) left as
// one Jacobian partial -- the form ranks exchange when a combine is sharded across GPUs.  One
// block of 16 quads: quad qd sums partials qd, qd + 16, ..., then the LDS tree.
__global__ void __launch_bounds__(64) bls_msm_finish_kernel(const uint32_t* partial, uint32_t nparts, uint8_t* out33,
                                                            uint32_t* sig_aff, uint32_t* out_jac) {
  __shared__ uint32_t sp[MSM_QUADS / 2][27];
  if (blockIdx.x != 0) return;
#if CBFT_BLS_PHASES
  uint64_t ph[5];
  ph[0] = wall_clock64();
#endif
  const int qd = threadIdx.x >> 2, q = threadIdx.x & 3;
  g1j acc;
  if (nparts == 1) {  // the row MSM's single partial: no sum (the 16-quad tree cost ~32 us)
    if (qd != 0) return;
    g1j_get(acc, partial, 1);
#if CBFT_BLS_PHASES
    ph[1] = ph[2] = wall_clock64();
#endif
  } else {
    g1_set_inf(acc);
#pragma unroll 1
    for (uint32_t b = qd; b < nparts; b += MSM_QUADS) {
      g1j o;
      g1j_get(o, partial + 27 * (size_t)b, 1);
      g1q_add(acc, acc, o, q);
    }
#if CBFT_BLS_PHASES
    ph[1] = wall_clock64();
#endif
    g1q_block_sum(acc, sp, qd, q);
#if CBFT_BLS_PHASES
    ph[2] = wall_clock64();
#endif
    if (qd != 0) return;
  }
  if (out_jac) {
    g1j_put(out_jac, 1, acc, q);
    return;
  }
  g1a a;
  g1_to_affine<true>(a, acc);  // the combined signature is public: variable-time inversion
#if CBFT_BLS_PHASES
  ph[3] = wall_clock64();
#endif
  if (q == 0) {
    g1_compress(out33, a);
    if (sig_aff) g1a_store(sig_aff, a);
  }
#if CBFT_BLS_PHASES
  ph[4] = wall_clock64();
  if (threadIdx.x == 0)
    printf("msm finish (us): partials %.1f block-sum %.1f to-affine %.1f compress %.1f (nparts %u)\n",
           (ph[1] - ph[0]) * 0.01, (ph[2] - ph[1]) * 0.01, (ph[3] - ph[2]) * 0.01, (ph[4] - ph[3]) * 0.01, nparts);
#endif
}

// sigma_i = sk_i * g1_map(msg) as a 37-byte share (BlsThresholdSigner::signData,
// BlsThresholdSigner.cpp:32-47): 4-byte big-endian id || 33-byte compressed G1.  sk: 8 LE words.
__global__ void bls_sign_kernel(const uint8_t* msg, uint32_t len, const uint32_t* sk, uint32_t id, uint8_t* out37) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  g1a h;
  g1_map(h, msg, len);
  g1j p, r;
  g1_from_affine(p, h);
  uint32_t k[8];
  for (int q = 0; q < 8; q++) k[q] = sk[q];
  g1_mul_ct(r, p, k);  // secret scalar: constant operation sequence
  g1a a;
  g1_to_affine(a, r);
  out37[0] = (uint8_t)(id >> 24);
  out37[1] = (uint8_t)(id >> 16);
  out37[2] = (uint8_t)(id >> 8);
  out37[3] = (uint8_t)id;
  g1_compress(out37 + 4, a);
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
  static const bool quad = [] {  // $CBFT_BLS_MSM=quad: the lane-quad MSM (A/B reference)
    const char* e = getenv("CBFT_BLS_MSM");
    return e && strcmp(e, "quad") == 0;
  }();
  if (!quad) {
    uint32_t* fin = nullptr;
    hipError_t e = cbft_bls_launch_msm_row(d_sig + BLS_SIG_WORDS * (size_t)lo, d_lambda + 8 * (size_t)lo,
                                           d_use + lo, m, multisig, d_partial, &fin, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(bls_msm_finish_kernel, dim3(1), dim3(64), 0, s, fin, 1u, d_out33, d_sig_aff, d_out_jac);
    return hipGetLastError();
  }
  const uint32_t nparts = (m + MSM_QUADS - 1) / MSM_QUADS;
  if (m)
    hipLaunchKernelGGL(bls_msm_kernel, dim3(nparts), dim3(64), 0, s, d_sig + 19 * (size_t)lo,
                       d_lambda + 8 * (size_t)lo, d_use + lo, m, multisig, d_partial);
  hipLaunchKernelGGL(bls_msm_finish_kernel, dim3(1), dim3(64), 0, s, d_partial, nparts, d_out33, d_sig_aff,
                     d_out_jac);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_g1_parts(const uint32_t* d_parts, uint32_t count, uint8_t* d_out33, hipStream_t s) {
  hipLaunchKernelGGL(bls_msm_finish_kernel, dim3(1), dim3(64), 0, s, d_parts, count, d_out33, nullptr, nullptr);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_sign(const uint8_t* d_msg, uint32_t len, const uint32_t* d_sk, uint32_t id,
                                uint8_t* d_out37, hipStream_t s) {
  hipLaunchKernelGGL(bls_sign_kernel, dim3(1), dim3(64), 0, s, d_msg, len, d_sk, id, d_out37);
  return hipGetLastError();
}
