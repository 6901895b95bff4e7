// BLS BN-P254 G2 kernels for gfx950: key decoding + Miller-loop line precomputation, the multisig
// key sum, the signer's public key (threshsign path).
//
//   bls_keys_kernel          per G2 key: decompress + subgroup check + 70 Miller-loop lines
//                            (BlsThresholdVerifier ctor; lines make per-share work G2-free)
//   bls_g2_sum_kernel        multisig PK = sum vk_i over the signer bitmap (Jacobian partial, or
//                            compressed for cbft_bls_sum_keys)
//   bls_pubkey_kernel        vk = sk * g2
#include "bls_common.h"

#define LINE_SCRATCH_WORDS (BN_ATE_LINES * 36)  // g2_precompute_lines_batch scratch per key

// scratch: nkeys x LINE_SCRATCH_WORDS words
__global__ void __launch_bounds__(64) bls_keys_kernel(const uint8_t* keys65, uint32_t nkeys, uint32_t* lines,
                                                      uint8_t* ok, uint32_t* aff, uint32_t* scratch) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nkeys) return;
  g2a q;
  bool good = g2_decompress(q, keys65 + 65 * (size_t)k) && !q.inf;
  ok[k] = good ? 1 : 0;
  if (!good) q.inf = true;
  g2a_store(aff + (size_t)k * BLS_G2A_WORDS, q);
  if (good) g2_precompute_lines_batch(lines + (size_t)k * LINES_PER_KEY, q, scratch + (size_t)k * LINE_SCRATCH_WORDS);
}

__global__ void bls_gen_lines_kernel(uint32_t* lines) {
  __shared__ uint32_t scr[LINE_SCRATCH_WORDS];
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  g2a q;
  fp2_load(q.x, Bn254Consts::G2X);
  fp2_load(q.y, Bn254Consts::G2Y);
  q.inf = false;
  g2_precompute_lines_batch(lines, q, scr);
}

// multisig public key = sum of vk_i for set bits (bit id-1, LSB first) of the 256-byte bitmap
// (BlsMultisigVerifier.cpp:33-38, 89-95).  One block: each of the SUM_THREADS lanes adds its
// strided share of the (already decoded, at load) keys in Jacobian form, then an LDS tree halves
// the partial sums.  A selected key that did not decode makes the result invalid (ok = 0).
#define SUM_THREADS 256
// normalise and compress (out65) a summed key; bad = a selected key did not decode
__device__ void g2_sum_tail(const g2j& acc, bool bad, uint8_t* ok, uint8_t* out65) {
  g2a s;
  g2_to_affine(s, acc);
  const bool good = !bad;
  if (good) {
    g2_compress(out65, s);
  } else {
    for (int q = 0; q < 65; q++) out65[q] = 0;
  }
  ok[0] = good && !s.inf ? 1 : 0;
}

// Signer ids [lo_id, hi_id) only (a rank's slice of a sharded multisig key sum).  With out_part
// the block writes its Jacobian sum (54 words) + the bad-key flag (1 word) (-> bls_verify_multisig_kernel),
// else the compressed sum into out65.
__global__ void __launch_bounds__(SUM_THREADS, 1) bls_g2_sum_kernel(const uint32_t* aff, const uint8_t* key_ok,
                                                                 uint32_t n, const uint8_t* bitmap, uint32_t lo_id,
                                                                 uint32_t hi_id, uint8_t* ok, uint8_t* out65,
                                                                 uint32_t* out_part) {
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
    g2_add_j_body(acc, acc, p);
  }
  if (mine_bad) atomicOr(&bad, 1);
  for (int stride = SUM_THREADS / 2; stride >= 1; stride >>= 1) {
    if (t >= stride && t < 2 * stride) g2j_store(sp[t - stride], acc);
    __syncthreads();
    if (t < stride) {
      g2j o;
      g2j_load(o, sp[t]);
      g2_add_j_body(acc, acc, o);
    }
    __syncthreads();
  }
  if (t != 0) return;
  if (out_part) {
    g2j_store(out_part, acc);
    out_part[54] = bad ? 1u : 0u;
    return;
  }
  g2_sum_tail(acc, bad != 0, ok, out65);
}

// vk = sk * g2 as 65 compressed bytes: the signer's public key (BlsThresholdSigner's
// publicKey_(secretKey) -> g2_mul_gen, BlsThresholdSigner.cpp:25; IThresholdSigner::
// getShareVerificationKey).  sk: 8 LE words (< r).  One lane, constant-sequence Montgomery
// ladder (g2_mul_ct: the secret key's bits select by mask, never by branch).
__global__ void bls_pubkey_kernel(const uint32_t* sk, uint8_t* out65) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  g2j G, acc;
  fp2_load(G.X, Bn254Consts::G2X);
  fp2_load(G.Y, Bn254Consts::G2Y);
  fp2_one(G.Z);
  uint32_t k[8];
  for (int q = 0; q < 8; q++) k[q] = sk[q];
  g2_mul_ct(acc, G, k);
  g2a a;
  g2_to_affine(a, acc);
  g2_compress(out65, a);
}

// ------------------------------------------------------------------------------ launchers
size_t cbft_bls_lines_words_per_key() { return (size_t)LINES_PER_KEY; }
size_t cbft_bls_keys_scratch_words(uint32_t nkeys) { return (size_t)nkeys * LINE_SCRATCH_WORDS; }
hipError_t cbft_bls_launch_keys(const uint8_t* d_keys65, uint32_t nkeys, uint32_t* d_lines, uint8_t* d_ok,
                                uint32_t* d_aff, uint32_t* d_scratch, hipStream_t s) {
  if (!nkeys) return hipSuccess;
  hipLaunchKernelGGL(bls_keys_kernel, dim3((nkeys + 63) / 64), dim3(64), 0, s, d_keys65, nkeys, d_lines, d_ok,
                     d_aff, d_scratch);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_gen_lines(uint32_t* d_lines, hipStream_t s) {
  hipLaunchKernelGGL(bls_gen_lines_kernel, dim3(1), dim3(64), 0, s, d_lines);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_g2_sum(const uint32_t* d_aff, const uint8_t* d_key_ok, uint32_t n, const uint8_t* d_bitmap,
                                  uint32_t lo_id, uint32_t hi_id, uint8_t* d_ok, uint8_t* d_out65, uint32_t* d_out_part,
                                  hipStream_t s) {
  hipLaunchKernelGGL(bls_g2_sum_kernel, dim3(1), dim3(SUM_THREADS), 0, s, d_aff, d_key_ok, n, d_bitmap, lo_id, hi_id,
                     d_ok, d_out65, d_out_part);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_pubkey(const uint32_t* d_sk, uint8_t* d_out65, hipStream_t s) {
  hipLaunchKernelGGL(bls_pubkey_kernel, dim3(1), dim3(64), 0, s, d_sk, d_out65);
  return hipGetLastError();
}
