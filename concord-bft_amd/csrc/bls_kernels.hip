// BLS BN-P254 threshold-signature kernels for gfx950 (threshsign path).
//
//   bls_keys_kernel          per G2 key: decompress + subgroup check + 70 Miller-loop lines
//                            (BlsThresholdVerifier ctor; lines make per-share work G2-free)
//   bls_hash_kernel          H = g1_map(digest)            (BlsAccumulatorBase.cpp:55-60)
//   bls_share_verify_kernel  lane per share: parse, e(H, vk_id) e(-sigma, g2) == 1
//                            (BlsAccumulatorBase::verifyShare, BlsAccumulatorBase.cpp:62-84)
//   bls_lagrange_kernel      lane per share: lambda_i = prod_{j!=i} j/(j-i) mod r
//                            (lagrangeCoeffAccumReduced, LagrangeInterpolation.cpp:202-292)
//   bls_msm_kernel           lane per share: lambda_i sigma_i, LDS tree sum per block
//                            (fastMultExp, FastMultExp.cpp:26-59; multisig: lambda = 1)
//   bls_msm_finish_kernel    sum of block partials -> 33-byte compressed G1
//   bls_g2_sum_kernel        multisig PK = sum vk_i over the signer bitmap, + its lines
//   bls_verify_kernel        e(H, PK) e(-sigma, g2) == 1   (BlsThresholdVerifier.cpp:69-96)
// One lane per pairing check: the per-lane state (an Fp12 accumulator + temporaries) lives in
// VGPRs/scratch; the G2 side is entirely precomputed.
#include <hip/hip_runtime.h>

#include "bls_kernels.h"
#include "bls_ops.h"
#include "bn254_pair6.h"

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

__global__ void __launch_bounds__(64) bls_keys_kernel(const uint8_t* keys65, uint32_t nkeys, uint32_t* lines,
                                                      uint8_t* ok, uint32_t* aff) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nkeys) return;
  g2a q;
  bool good = g2_decompress(q, keys65 + 65 * (size_t)k) && !q.inf;
  ok[k] = good ? 1 : 0;
  if (!good) q.inf = true;
  g2a_store(aff + (size_t)k * BLS_G2A_WORDS, q);
  if (good) g2_precompute_lines(lines + (size_t)k * LINES_PER_KEY, q);
}

__global__ void bls_gen_lines_kernel(uint32_t* lines) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  g2a q;
  fp2_load(q.x, Bn254Consts::G2X);
  fp2_load(q.y, Bn254Consts::G2Y);
  q.inf = false;
  g2_precompute_lines(lines, q);
}

__global__ void bls_hash_kernel(const uint8_t* msg, uint32_t len, uint32_t* H) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  g1a h;
  g1_map(h, msg, len);
  g1a_store(H, h);
}

// shares: k x 37 bytes.  out: valid[k] (1 = verified), sig[k] (parsed affine point, 19 words),
// ids[k].  A share whose id is outside [1, n] or whose point does not decode is invalid.
// One 8-lane group per share: the pairing check runs on six lanes (bn254_pair6.h); parsing is
// done by every lane of the group (same latency as one) and lane 0 writes the results.
__global__ void __launch_bounds__(64) bls_share_verify_kernel(const uint8_t* shares, uint32_t k, uint32_t n,
                                                              const uint32_t* H, const uint32_t* vk_lines,
                                                              const uint8_t* vk_ok, const uint32_t* gen_lines,
                                                              int do_verify, uint8_t* valid, uint32_t* sig,
                                                              uint32_t* ids) {
  const uint32_t j = (blockIdx.x * blockDim.x + threadIdx.x) >> 3;
  if (j >= k) return;  // whole groups exit together
  const P6 g = p6_lane();
  const bool lead = (threadIdx.x & 7) == 0;
  uint32_t id;
  g1a s;
  bool good = bls_parse_share(id, s, shares + 37 * (size_t)j);
  good = good && id >= 1 && id <= n;
  if (lead) {
    ids[j] = id;
    g1a_store(sig + 19 * (size_t)j, s);
  }
  if (good && do_verify) {
    good = vk_ok[id - 1] != 0;
    if (good) {
      g1a P[2];
      g1a_load(P[0], H);
      P[1] = s;
      if (!s.inf) f_neg(P[1].y, s.y);
      const uint32_t* l[2] = {vk_lines + (size_t)(id - 1) * LINES_PER_KEY, gen_lines};
      // e(O, Q) = 1: an infinite sigma checks against e(H, vk) alone
      if (P[1].inf)
        good = p6_pairing_check<1>(P, l, g);
      else
        good = p6_pairing_check<2>(P, l, g);
    }
  }
  if (lead) valid[j] = good ? 1 : 0;
}

// lambda_i = prod_{j != i} j / (j - i) mod r over the shares with use[j] != 0; words out (LE)
__global__ void __launch_bounds__(64) bls_lagrange_kernel(const uint32_t* ids, const uint8_t* use, uint32_t k,
                                                          uint32_t* lambda) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (use[i]) {
    fr num, den, t, d;
    f_one(num);
    f_one(den);
    const uint32_t me = ids[i];
    for (uint32_t j = 0; j < k; j++) {
      if (j == i || !use[j]) continue;
      const uint32_t o = ids[j];
      uint32_t v[8] = {o, 0, 0, 0, 0, 0, 0, 0};
      f_from_words(t, v);
      f_mul(num, num, t);
      uint32_t dv[8] = {o > me ? o - me : me - o, 0, 0, 0, 0, 0, 0, 0};
      f_from_words(d, dv);
      if (o < me) f_neg(d, d);
      f_mul(den, den, d);
    }
    fr_inv(den, den);
    f_mul(num, num, den);
    f_to_words(w, num);
  }
  for (int q = 0; q < 8; q++) lambda[8 * (size_t)i + q] = w[q];
}

#define MSM_BLOCK 64
// partial[b] = sum over this block's lanes of lambda_j * sig_j (Jacobian, 27 words)
__global__ void __launch_bounds__(MSM_BLOCK) bls_msm_kernel(const uint32_t* sig, const uint32_t* lambda,
                                                            const uint8_t* use, uint32_t k, int unit_scalars,
                                                            uint32_t* partial) {
  __shared__ uint32_t sp[MSM_BLOCK][27];
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  g1j acc;
  g1_set_inf(acc);
  if (j < k && use[j]) {
    g1a s;
    g1a_load(s, sig + 19 * (size_t)j);
    g1j p;
    g1_from_affine(p, s);
    if (unit_scalars) {
      acc = p;
    } else {
      uint32_t lw[8];
      for (int q = 0; q < 8; q++) lw[q] = lambda[8 * (size_t)j + q];
      g1_mul(acc, p, lw);
    }
  }
  for (int stride = MSM_BLOCK / 2; stride >= 1; stride >>= 1) {
    const int t = threadIdx.x;
    if (t >= stride && t < 2 * stride) {
      for (int q = 0; q < 9; q++) {
        sp[t - stride][q] = acc.X.v[q];
        sp[t - stride][9 + q] = acc.Y.v[q];
        sp[t - stride][18 + q] = acc.Z.v[q];
      }
    }
    __syncthreads();
    if (t < stride) {
      g1j o;
      for (int q = 0; q < 9; q++) {
        o.X.v[q] = sp[t][q];
        o.Y.v[q] = sp[t][9 + q];
        o.Z.v[q] = sp[t][18 + q];
      }
      g1_add(acc, acc, o);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    uint32_t* o = partial + 27 * (size_t)blockIdx.x;
    for (int q = 0; q < 9; q++) {
      o[q] = acc.X.v[q];
      o[9 + q] = acc.Y.v[q];
      o[18 + q] = acc.Z.v[q];
    }
  }
}

// Sum of nparts Jacobian partials (27 words each): compressed into out33, or (out_jac) left as
// one Jacobian partial -- the form ranks exchange when a combine is sharded across GPUs.
__global__ void bls_msm_finish_kernel(const uint32_t* partial, uint32_t nparts, uint8_t* out33, uint32_t* sig_aff,
                                      uint32_t* out_jac) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  g1j acc;
  g1_set_inf(acc);
  for (uint32_t b = 0; b < nparts; b++) {
    g1j o;
    for (int q = 0; q < 9; q++) {
      o.X.v[q] = partial[27 * b + q];
      o.Y.v[q] = partial[27 * b + 9 + q];
      o.Z.v[q] = partial[27 * b + 18 + q];
    }
    g1_add(acc, acc, o);
  }
  if (out_jac) {
    for (int q = 0; q < 9; q++) {
      out_jac[q] = acc.X.v[q];
      out_jac[9 + q] = acc.Y.v[q];
      out_jac[18 + q] = acc.Z.v[q];
    }
    return;
  }
  g1a a;
  g1_to_affine(a, acc);
  g1_compress(out33, a);
  if (sig_aff) g1a_store(sig_aff, a);
}

// multisig public key = sum of vk_i for set bits (bit id-1, LSB first) of the 256-byte bitmap,
// then its Miller-loop lines (BlsMultisigVerifier.cpp:33-38, 89-95).  One block: each of the
// SUM_THREADS lanes adds its strided share of the (already decoded, at load) keys in Jacobian
// form, then an LDS tree halves the partial sums; lane 0 normalises, compresses and computes
// the lines.  A selected key that did not decode makes the result invalid (ok = 0).
#define SUM_THREADS 256
// normalise, compress (out65) and compute the Miller lines of a summed key; bad = a selected
// key did not decode
__device__ void g2_sum_tail(const g2j& acc, bool bad, uint32_t* lines, uint8_t* ok, uint8_t* out65) {
  g2a s;
  g2_to_affine(s, acc);
  const bool good = !bad;
  if (out65) {
    if (good) {
      g2_compress(out65, s);
    } else {
      for (int q = 0; q < 65; q++) out65[q] = 0;
    }
  }
  const bool usable = good && !s.inf;
  ok[0] = usable ? 1 : 0;
  if (usable && lines) g2_precompute_lines(lines, s);
}

__device__ __forceinline__ void g2j_store(uint32_t* o, const g2j& a) {
  const fp2* src[3] = {&a.X, &a.Y, &a.Z};
  for (int c = 0; c < 3; c++)
    for (int q = 0; q < 9; q++) {
      o[18 * c + q] = src[c]->a.v[q];
      o[18 * c + 9 + q] = src[c]->b.v[q];
    }
}
__device__ __forceinline__ void g2j_load(g2j& a, const uint32_t* o) {
  fp2* dst[3] = {&a.X, &a.Y, &a.Z};
  for (int c = 0; c < 3; c++)
    for (int q = 0; q < 9; q++) {
      dst[c]->a.v[q] = o[18 * c + q];
      dst[c]->b.v[q] = o[18 * c + 9 + q];
    }
}

// Signer ids [lo_id, hi_id) only (a rank's slice of a sharded multisig key sum).  With out_part
// the block writes its Jacobian sum (54 words) + the bad-key flag (1 word) and stops there.
__global__ void __launch_bounds__(SUM_THREADS) bls_g2_sum_kernel(const uint32_t* aff, const uint8_t* key_ok,
                                                                 uint32_t n, const uint8_t* bitmap, uint32_t lo_id,
                                                                 uint32_t hi_id, uint32_t* lines, uint8_t* ok,
                                                                 uint8_t* out65, uint32_t* out_part) {
  __shared__ uint32_t sp[SUM_THREADS / 2][54];
  __shared__ int bad;
  const int t = threadIdx.x;
  if (t == 0) bad = 0;
  __syncthreads();
  g2j acc;
  fp2_one(acc.X);
  fp2_one(acc.Y);
  fp2_zero(acc.Z);
  bool mine_bad = false;
  const uint32_t lo = lo_id < 1 ? 1 : lo_id, hi = hi_id > n + 1 ? n + 1 : hi_id;
  for (uint32_t id = lo + t; id < hi; id += SUM_THREADS) {
    if (!((bitmap[(id - 1) >> 3] >> ((id - 1) & 7)) & 1)) continue;
    if (!key_ok[id - 1]) {
      mine_bad = true;
      continue;
    }
    g2a q;
    g2a_load(q, aff + (size_t)(id - 1) * BLS_G2A_WORDS);
    g2j p;
    p.X = q.x;
    p.Y = q.y;
    fp2_one(p.Z);
    g2_add_j(acc, acc, p);
  }
  if (mine_bad) atomicOr(&bad, 1);
  for (int stride = SUM_THREADS / 2; stride >= 1; stride >>= 1) {
    if (t >= stride && t < 2 * stride) g2j_store(sp[t - stride], acc);
    __syncthreads();
    if (t < stride) {
      g2j o;
      g2j_load(o, sp[t]);
      g2_add_j(acc, acc, o);
    }
    __syncthreads();
  }
  if (t != 0) return;
  if (out_part) {
    g2j_store(out_part, acc);
    out_part[54] = bad ? 1u : 0u;
    return;
  }
  g2_sum_tail(acc, bad != 0, lines, ok, out65);
}

// Sum of count G2 partials (55 words each, from bls_g2_sum_kernel's out_part) + the tail.
__global__ void bls_g2_parts_kernel(const uint32_t* parts, uint32_t count, uint32_t* lines, uint8_t* ok,
                                    uint8_t* out65) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  g2j acc;
  fp2_one(acc.X);
  fp2_one(acc.Y);
  fp2_zero(acc.Z);
  bool bad = false;
  for (uint32_t b = 0; b < count; b++) {
    g2j o;
    g2j_load(o, parts + 55 * (size_t)b);
    bad |= parts[55 * (size_t)b + 54] != 0;
    g2_add_j(acc, acc, o);
  }
  g2_sum_tail(acc, bad, lines, ok, out65);
}

// e(H, PK) * e(-sigma, g2) == 1 for a combined signature (33 bytes); one 8-lane group
__global__ void __launch_bounds__(64) bls_verify_kernel(const uint32_t* H, const uint8_t* sig33,
                                                        const uint32_t* pk_lines, const uint8_t* pk_ok,
                                                        const uint32_t* gen_lines, uint8_t* result) {
  if (threadIdx.x >= 8 || blockIdx.x != 0) return;
  const P6 g = p6_lane();
  g1a P[2];
  g1a_load(P[0], H);
  bool good = pk_ok[0] && g1_decompress(P[1], sig33);
  if (good) {
    const uint32_t* l[2] = {pk_lines, gen_lines};
    if (P[1].inf) {
      good = p6_pairing_check<1>(P, l, g);
    } else {
      f_neg(P[1].y, P[1].y);
      good = p6_pairing_check<2>(P, l, g);
    }
  }
  if (threadIdx.x == 0) result[0] = good ? 1 : 0;
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
  g1_mul(r, p, k);
  g1a a;
  g1_to_affine(a, r);
  out37[0] = (uint8_t)(id >> 24);
  out37[1] = (uint8_t)(id >> 16);
  out37[2] = (uint8_t)(id >> 8);
  out37[3] = (uint8_t)id;
  g1_compress(out37 + 4, a);
}

// vk = sk * g2 as 65 compressed bytes: the signer's public key (BlsThresholdSigner's
// publicKey_(secretKey) -> g2_mul_gen, BlsThresholdSigner.cpp:25; IThresholdSigner::
// getShareVerificationKey).  sk: 8 LE words (< r).  One lane, double-and-add (a one-off per key).
__global__ void bls_pubkey_kernel(const uint32_t* sk, uint8_t* out65) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  g2j G, acc;
  fp2_load(G.X, Bn254Consts::G2X);
  fp2_load(G.Y, Bn254Consts::G2Y);
  fp2_one(G.Z);
  fp2_one(acc.X);
  fp2_one(acc.Y);
  fp2_zero(acc.Z);
  for (int i = 255; i >= 0; i--) {
    g2_dbl_j(acc, acc);
    if ((sk[i >> 5] >> (i & 31)) & 1) g2_add_j(acc, acc, G);
  }
  g2a a;
  g2_to_affine(a, acc);
  g2_compress(out65, a);
}

// ------------------------------------------------------------------------------ launchers
size_t cbft_bls_lines_words_per_key() { return (size_t)LINES_PER_KEY; }

hipError_t cbft_bls_launch_keys(const uint8_t* d_keys65, uint32_t nkeys, uint32_t* d_lines, uint8_t* d_ok,
                                uint32_t* d_aff, hipStream_t s) {
  if (!nkeys) return hipSuccess;
  hipLaunchKernelGGL(bls_keys_kernel, dim3((nkeys + 63) / 64), dim3(64), 0, s, d_keys65, nkeys, d_lines, d_ok,
                     d_aff);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_gen_lines(uint32_t* d_lines, hipStream_t s) {
  hipLaunchKernelGGL(bls_gen_lines_kernel, dim3(1), dim3(64), 0, s, d_lines);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_hash(const uint8_t* d_msg, uint32_t len, uint32_t* d_H, hipStream_t s) {
  hipLaunchKernelGGL(bls_hash_kernel, dim3(1), dim3(64), 0, s, d_msg, len, d_H);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_share_verify(const uint8_t* d_shares, uint32_t k, uint32_t n, const uint32_t* d_H,
                                        const uint32_t* d_vk_lines, const uint8_t* d_vk_ok,
                                        const uint32_t* d_gen_lines, int do_verify, uint8_t* d_valid,
                                        uint32_t* d_sig, uint32_t* d_ids, hipStream_t s) {
  if (!k) return hipSuccess;
  hipLaunchKernelGGL(bls_share_verify_kernel, dim3((8 * k + 63) / 64), dim3(64), 0, s, d_shares, k, n, d_H, d_vk_lines,
                     d_vk_ok, d_gen_lines, do_verify, d_valid, d_sig, d_ids);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_combine(const uint32_t* d_sig, const uint32_t* d_ids, const uint8_t* d_use, uint32_t k,
                                   uint32_t lo, uint32_t hi, int multisig, uint32_t* d_lambda, uint32_t* d_partial,
                                   uint8_t* d_out33, uint32_t* d_sig_aff, uint32_t* d_out_jac, hipStream_t s) {
  if (!multisig && k)
    hipLaunchKernelGGL(bls_lagrange_kernel, dim3((k + 63) / 64), dim3(64), 0, s, d_ids, d_use, k, d_lambda);
  hi = hi < k ? hi : k;
  lo = lo < hi ? lo : hi;
  const uint32_t m = hi - lo;  // the MSM runs over shares [lo, hi) only
  const uint32_t nparts = (m + MSM_BLOCK - 1) / MSM_BLOCK;
  if (m)
    hipLaunchKernelGGL(bls_msm_kernel, dim3(nparts), dim3(MSM_BLOCK), 0, s, d_sig + 19 * (size_t)lo,
                       d_lambda + 8 * (size_t)lo, d_use + lo, m, multisig, d_partial);
  hipLaunchKernelGGL(bls_msm_finish_kernel, dim3(1), dim3(64), 0, s, d_partial, nparts, d_out33, d_sig_aff,
                     d_out_jac);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_g1_parts(const uint32_t* d_parts, uint32_t count, uint8_t* d_out33, hipStream_t s) {
  hipLaunchKernelGGL(bls_msm_finish_kernel, dim3(1), dim3(64), 0, s, d_parts, count, d_out33, nullptr, nullptr);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_g2_sum(const uint32_t* d_aff, const uint8_t* d_key_ok, uint32_t n, const uint8_t* d_bitmap,
                                  uint32_t lo_id, uint32_t hi_id, uint32_t* d_lines, uint8_t* d_ok, uint8_t* d_out65,
                                  uint32_t* d_out_part, hipStream_t s) {
  hipLaunchKernelGGL(bls_g2_sum_kernel, dim3(1), dim3(SUM_THREADS), 0, s, d_aff, d_key_ok, n, d_bitmap, lo_id, hi_id,
                     d_lines, d_ok, d_out65, d_out_part);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_g2_parts(const uint32_t* d_parts, uint32_t count, uint32_t* d_lines, uint8_t* d_ok,
                                    uint8_t* d_out65, hipStream_t s) {
  hipLaunchKernelGGL(bls_g2_parts_kernel, dim3(1), dim3(64), 0, s, d_parts, count, d_lines, d_ok, d_out65);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_verify(const uint32_t* d_H, const uint8_t* d_sig33, const uint32_t* d_pk_lines,
                                  const uint8_t* d_pk_ok, const uint32_t* d_gen_lines, uint8_t* d_result,
                                  hipStream_t s) {
  hipLaunchKernelGGL(bls_verify_kernel, dim3(1), dim3(64), 0, s, d_H, d_sig33, d_pk_lines, d_pk_ok, d_gen_lines,
                     d_result);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_sign(const uint8_t* d_msg, uint32_t len, const uint32_t* d_sk, uint32_t id,
                                uint8_t* d_out37, hipStream_t s) {
  hipLaunchKernelGGL(bls_sign_kernel, dim3(1), dim3(64), 0, s, d_msg, len, d_sk, id, d_out37);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_pubkey(const uint32_t* d_sk, uint8_t* d_out65, hipStream_t s) {
  hipLaunchKernelGGL(bls_pubkey_kernel, dim3(1), dim3(64), 0, s, d_sk, d_out65);
  return hipGetLastError();
}
