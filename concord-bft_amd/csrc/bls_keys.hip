// BLS BN-P254 G2 kernels for gfx950: key decoding + Miller-loop line precomputation, the multisig
// key sum, the signer's public key (threshsign path).
//
//   bls_keys_wave_kernel     per G2 key, one block of two waves: decompress + subgroup check
//                            (wave 0) beside the 70 Miller-loop lines (wave 1), every step's Fp
//                            products on separate lanes (bn254_g2wave.h); also the generator's
//                            lines (BlsThresholdVerifier ctor; lines make per-share work G2-free)
//   bls_keys_kernel          the same on one lane per key (kept for A/B: $CBFT_BLS_KEYS=lane)
//   bls_g2_sum_kernel        multisig PK = sum vk_i over the signer bitmap (Jacobian partial, or
//                            compressed for cbft_bls_sum_keys)
//   bls_pubkey_kernel        vk = sk * g2
#include <cstdlib>
#include <cstring>

#include "bls_common.h"
#include "bn254_g2wave.h"

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

// Normalised lines (lambda, mu: BN_LINE_WORDS words each, g2_precompute_lines_batch's output) from
// the wave's unnormalised (A, B, C) records in LDS: lambda_k = -B_k / A_k, mu_k = C_k / A_k with
// Montgomery's trick over the A_k -- prefix products (one Fp2 product per step, its three Fp
// products on three lanes), one variable-time Fp2 inversion (public key material), the
// back-substitution (two Fp2 products per step on six lanes), then the 140 lambda / mu products
// one Fp2 product per lane.  pre: BN_ATE_LINES x 18 words of LDS.  Every lane calls it.
__device__ __noinline__ void g2w_normalise_lines(uint32_t* out, const uint32_t* abc, uint32_t* pre) {
  const int lane = threadIdx.x & 63;
  fp U[6], V[6], p[6];
  fp2 acc, a;
  fp2_fetch(acc, abc);
  if (lane < 18) pre[lane] = lane < 9 ? acc.a.v[lane] : acc.b.v[lane - 9];
#pragma nounroll
  for (int k = 1; k < BN_ATE_LINES; k++) {
    fp2_fetch(a, abc + k * BN_ABC_WORDS);
    g2w_mul_ops(U, V, 0, acc, a);
    g2w_round<3>(p, U, V, lane);
    g2w_mul_res(acc, p, 0);
    if (lane < 18) pre[18 * k + lane] = lane < 9 ? acc.a.v[lane] : acc.b.v[lane - 9];
  }
  fp2 inv;
  fp2_inv<true>(inv, acc);
#pragma nounroll
  for (int k = BN_ATE_LINES - 1; k >= 1; k--) {
    fp2 pk;
    fp2_fetch(pk, pre + 18 * (k - 1));
    fp2_fetch(a, abc + k * BN_ABC_WORDS);
    g2w_mul_ops(U, V, 0, inv, pk);  // 1 / A_k
    g2w_mul_ops(U, V, 3, inv, a);   // 1 / (A_0 .. A_{k-1})
    g2w_round<6>(p, U, V, lane);
    fp2 ai;
    g2w_mul_res(ai, p, 0);
    g2w_mul_res(inv, p, 3);
    if (lane < 18) pre[18 * k + lane] = lane < 9 ? ai.a.v[lane] : ai.b.v[lane - 9];
  }
  if (lane < 18) pre[lane] = lane < 9 ? inv.a.v[lane] : inv.b.v[lane - 9];
#pragma unroll 1
  for (int base = 0; base < 2 * BN_ATE_LINES; base += 64) {
    const int i = base + lane;
    if (i < 2 * BN_ATE_LINES) {
      const int k = i >> 1, mu = i & 1;
      fp2 x, ai, r;
      fp2_fetch(x, abc + k * BN_ABC_WORDS + (mu ? 36 : 18));
      fp2_fetch(ai, pre + 18 * k);
      fp2_mul(r, x, ai);
      if (!mu) fp2_neg(r, r);
      fp2_store(out + (size_t)k * BN_LINE_WORDS + 18 * mu, r);
    }
  }
}

// keys65 = nullptr: the generator g2's lines only (gen_lines).  Else key k = blockIdx.x: ok[k] =
// decodes && not infinity && r Q == O (g2_decompress's verdict), aff[k], lines[k] (written for
// every decodable key; only ok keys are ever read).
#define KEYS_WAVE_BLOCK 128
__global__ void __launch_bounds__(KEYS_WAVE_BLOCK) bls_keys_wave_kernel(const uint8_t* keys65, uint32_t nkeys,
                                                                        uint32_t* lines, uint8_t* ok, uint32_t* aff) {
  __shared__ uint32_t abc[BN_ATE_LINES * BN_ABC_WORDS];
  __shared__ uint32_t pre[BN_ATE_LINES * 18];
  const uint32_t k = blockIdx.x;
  if (k >= nkeys) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  g2a q;
  bool dec;
  if (keys65) {
    dec = g2_decode_on_curve(q, keys65 + 65 * (size_t)k) && !q.inf;
  } else {
    fp2_load(q.x, Bn254Consts::G2X);
    fp2_load(q.y, Bn254Consts::G2Y);
    q.inf = false;
    dec = true;
  }
  if (wave == 0) {
    if (!keys65) return;
    const bool good = dec && g2w_in_subgroup(q);
    if (lane == 0) {
      ok[k] = good ? 1 : 0;
      if (!good) q.inf = true;
      g2a_store(aff + (size_t)k * BLS_G2A_WORDS, q);
    }
    return;
  }
  if (!dec) return;
  g2w_lines_abc(abc, q);
  g2w_normalise_lines(lines + (size_t)k * LINES_PER_KEY, abc, pre);
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

// The multisig key sum on waves, every addition's Fp products on separate lanes
// (bn254_g2wave.h): a block of G2S_WAVES waves.  Level 0 (parts == nullptr): wave w of block b
// adds the selected keys among ids [lo + G2S_IDS (b G2S_WAVES + w), +G2S_IDS) within [lo, hi) by
// mixed additions (a selected key that did not decode marks the sum bad); level > 0: partials
// [G2S_PARTS (b G2S_WAVES + w), +G2S_PARTS) of count.  The block's waves then meet in an LDS
// tree and wave 0 writes the block's partial (54 words + bad flag) to out_parts[b], or, with
// out65 (a one-block launch), the compressed sum and ok (g2_sum_tail).  Group law exact in every
// case (g2w_accum), so the sum is the bls_g2_sum_kernel's point.
#define G2S_WAVES 4
#define G2S_IDS 16
#define G2S_PARTS 4
#define G2S_MAX_PARTS 64  // level-0 blocks for ids up to 4,096
__device__ __forceinline__ void g2w_part_store(uint32_t* o, const g2j& acc, bool inf, bool bad, int lane) {
  g2j a = acc;
  if (inf) {
    fp2_one(a.X);
    fp2_one(a.Y);
    fp2_zero(a.Z);
  }
  uint32_t wv[BLS_G2_PART_WORDS];
  g2j_store(wv, a);
  wv[54] = bad ? 1u : 0u;
  uint32_t w = wv[0];
#pragma unroll
  for (int i = 1; i < BLS_G2_PART_WORDS; i++) w = lane == i ? wv[i] : w;
  if (lane < BLS_G2_PART_WORDS) o[lane] = w;
}
__global__ void __launch_bounds__(64 * G2S_WAVES) bls_g2_sum_wave_kernel(const uint32_t* aff, const uint8_t* key_ok,
                                                                       const uint8_t* bitmap, uint32_t lo, uint32_t hi,
                                                                       const uint32_t* parts, uint32_t count,
                                                                       uint32_t* out_parts, uint8_t* ok,
                                                                       uint8_t* out65) {
  __shared__ uint32_t xp[G2S_WAVES][BLS_G2_PART_WORDS + 1];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t wid = blockIdx.x * G2S_WAVES + wave;
  g2j acc;
  fp2_one(acc.X);
  fp2_one(acc.Y);
  fp2_zero(acc.Z);
  bool inf = true, bad = false;
  if (!parts) {
    const uint32_t s0 = lo + wid * G2S_IDS;
#pragma nounroll
    for (uint32_t id = s0; id < s0 + G2S_IDS && id < hi; id++) {
      if (!((bitmap[(id - 1) >> 3] >> ((id - 1) & 7)) & 1)) continue;
      if (!key_ok[id - 1]) {
        bad = true;
        continue;
      }
      g2a q;
      g2a_load(q, aff + (size_t)(id - 1) * BLS_G2A_WORDS);
      g2w_accum_aff(acc, inf, q.x, q.y, lane);
    }
  } else {
#pragma nounroll
    for (uint32_t i = wid * G2S_PARTS; i < (wid + 1) * G2S_PARTS && i < count; i++) {
      g2j o;
      g2j_load(o, parts + (size_t)BLS_G2_PART_WORDS * i);
      bad |= parts[(size_t)BLS_G2_PART_WORDS * i + 54] != 0;
      g2w_accum(acc, inf, o, fp2_is_zero(o.Z), lane);
    }
  }
#pragma unroll 1
  for (int stride = G2S_WAVES / 2; stride >= 1; stride >>= 1) {
    if (wave >= stride && wave < 2 * stride) g2w_part_store(xp[wave - stride], acc, inf, bad, lane);
    __syncthreads();
    if (wave < stride) {
      g2j o;
      g2j_load(o, xp[wave]);
      bad |= xp[wave][54] != 0;
      g2w_accum(acc, inf, o, fp2_is_zero(o.Z), lane);
    }
    __syncthreads();
  }
  if (wave != 0) return;
  if (out65) {
    if (lane == 0) {
      if (inf) {
        fp2_one(acc.X);
        fp2_one(acc.Y);
        fp2_zero(acc.Z);
      }
      g2_sum_tail(acc, bad, ok, out65);
    }
    return;
  }
  g2w_part_store(out_parts + (size_t)BLS_G2_PART_WORDS * blockIdx.x, acc, inf, bad, lane);
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
// $CBFT_BLS_KEYS=lane selects the one-lane-per-key kernels (A/B), else the wave form
static bool keys_lane_form() {
  static const bool lane = [] {
    const char* e = getenv("CBFT_BLS_KEYS");
    return e && strcmp(e, "lane") == 0;
  }();
  return lane;
}
hipError_t cbft_bls_launch_keys(const uint8_t* d_keys65, uint32_t nkeys, uint32_t* d_lines, uint8_t* d_ok,
                                uint32_t* d_aff, uint32_t* d_scratch, hipStream_t s) {
  if (!nkeys) return hipSuccess;
  if (keys_lane_form())
    hipLaunchKernelGGL(bls_keys_kernel, dim3((nkeys + 63) / 64), dim3(64), 0, s, d_keys65, nkeys, d_lines, d_ok,
                       d_aff, d_scratch);
  else
    hipLaunchKernelGGL(bls_keys_wave_kernel, dim3(nkeys), dim3(KEYS_WAVE_BLOCK), 0, s, d_keys65, nkeys, d_lines,
                       d_ok, d_aff);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_gen_lines(uint32_t* d_lines, hipStream_t s) {
  if (keys_lane_form())
    hipLaunchKernelGGL(bls_gen_lines_kernel, dim3(1), dim3(64), 0, s, d_lines);
  else
    hipLaunchKernelGGL(bls_keys_wave_kernel, dim3(1), dim3(KEYS_WAVE_BLOCK), 0, s, nullptr, 1u, d_lines, nullptr,
                       nullptr);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_g2_sum(const uint32_t* d_aff, const uint8_t* d_key_ok, uint32_t n, const uint8_t* d_bitmap,
                                  uint32_t lo_id, uint32_t hi_id, uint8_t* d_ok, uint8_t* d_out65, uint32_t* d_out_part,
                                  uint32_t* d_tmp, hipStream_t s) {
  if (keys_lane_form() || !d_tmp) {
    hipLaunchKernelGGL(bls_g2_sum_kernel, dim3(1), dim3(SUM_THREADS), 0, s, d_aff, d_key_ok, n, d_bitmap, lo_id, hi_id,
                       d_ok, d_out65, d_out_part);
    return hipGetLastError();
  }
  const uint32_t lo = lo_id < 1 ? 1 : lo_id, hi = hi_id > n + 1 ? n + 1 : hi_id;
  const uint32_t span = hi > lo ? hi - lo : 0;
  uint32_t nb = (span + G2S_WAVES * G2S_IDS - 1) / (G2S_WAVES * G2S_IDS);
  if (nb == 0) nb = 1;
  // level 0: the keys -> nb partials; then G2S_WAVES * G2S_PARTS : 1 levels until one remains
  uint32_t* cur = d_tmp;
  uint32_t* nxt = d_tmp + (size_t)BLS_G2_PART_WORDS * G2S_MAX_PARTS;
  const bool one = nb == 1;
  hipLaunchKernelGGL(bls_g2_sum_wave_kernel, dim3(nb), dim3(64 * G2S_WAVES), 0, s, d_aff, d_key_ok, d_bitmap, lo, hi,
                     (const uint32_t*)nullptr, 0u, one && d_out_part ? d_out_part : cur, d_ok,
                     one ? d_out65 : (uint8_t*)nullptr);
  while (nb > 1) {
    const uint32_t nb2 = (nb + G2S_WAVES * G2S_PARTS - 1) / (G2S_WAVES * G2S_PARTS);
    const bool last = nb2 == 1;
    hipLaunchKernelGGL(bls_g2_sum_wave_kernel, dim3(nb2), dim3(64 * G2S_WAVES), 0, s, d_aff, d_key_ok, d_bitmap, lo,
                       hi, (const uint32_t*)cur, nb, last && d_out_part ? d_out_part : nxt, d_ok,
                       last ? d_out65 : (uint8_t*)nullptr);
    uint32_t* t = cur;
    cur = nxt;
    nxt = t;
    nb = nb2;
  }
  return hipGetLastError();
}
size_t cbft_bls_g2_sum_tmp_words() { return (size_t)2 * BLS_G2_PART_WORDS * G2S_MAX_PARTS; }
hipError_t cbft_bls_launch_pubkey(const uint32_t* d_sk, uint8_t* d_out65, hipStream_t s) {
  hipLaunchKernelGGL(bls_pubkey_kernel, dim3(1), dim3(64), 0, s, d_sk, d_out65);
  return hipGetLastError();
}
