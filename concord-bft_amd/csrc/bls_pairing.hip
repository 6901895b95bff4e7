// BLS BN-P254 pairing-check kernels for gfx950 (threshsign path).
//
//   bls_share_verify_kernel  one (2-wave) block per share: parse, e(H, vk_id) e(-sigma, g2) == 1
//                            (BlsAccumulatorBase::verifyShare, BlsAccumulatorBase.cpp:62-84)
//   bls_verify_kernel        H = g1_map(msg), e(H, PK) e(-sigma, g2) == 1
//                            (BlsThresholdVerifier.cpp:69-96)
// The G2 side is precomputed (bls_keys.hip); each Fp12 accumulator is spread over a whole wave,
// three lanes per Fp component (bn254_pair36.h).  The two Miller loops of a check run on two
// waves of one block (two SIMDs): wave 0 the (H, key) pair, wave 1 decodes sigma and runs the
// (-sigma, g2) pair; wave 1 hands its Miller value over through LDS, wave 0 multiplies and
// runs the final exponentiation.  A pairing check is one instruction stream per wave (a lone
// wave per SIMD, issue-bound), so splitting the pairs takes one Miller loop's line evaluations
// off the critical path, and with them the sqrt of sigma's decompression (and, in
// bls_verify_kernel, the hash to G1, which wave 0 computes while wave 1 decodes sigma).
#include <cstdlib>

#include "bls_common.h"
#include "bn254_g2wave.h"
#include "bn254_pair36.h"

#define PAIR_BLOCK 128  // two waves
#define SIMDS 1024       // 256 CUs x 4 SIMDs (MI355X)

// wave 1 -> wave 0: its Miller value (36 lanes x 9 limbs) and a flag
struct PairXchg {
  uint32_t f[36][BN_LIMBS];
  int ok;
};

__device__ __forceinline__ void xchg_put(PairXchg& x, const fp& f, const P36& g) {
  if (g.own)
    for (int i = 0; i < BN_LIMBS; i++) x.f[g.e][i] = f.v[i];
}
__device__ __forceinline__ void xchg_get(fp& f, const PairXchg& x, const P36& g) {
  for (int i = 0; i < BN_LIMBS; i++) f.v[i] = x.f[g.e][i];  // shadows read the slot they mirror
}

// shares: k x 37 bytes.  out: valid[k] (1 = verified), sig[k] (parsed affine point, 19 words),
// ids[k].  A share whose id is outside [1, n] or whose point does not decode is invalid.
// do_verify = 0: parse only, valid = decodable && id in range.
//   WAVES = 2: one 2-wave block per share (the two Miller loops in parallel): the latency form,
//              used while 2k waves fit the chip's 1,024 SIMDs;
//   WAVES = 1: one wave per share, both pairs on it: the throughput form for larger k and for
//              parse-only launches (two waves of a share would share SIMDs with other shares).
// parsed != 0: bls_prep_kernel has already decoded the shares (valid = decodable && id in range,
// sig, ids), so the check starts at the Miller loop.
template <int WAVES>
__global__ void __launch_bounds__(64 * WAVES) bls_share_verify_kernel(const uint8_t* shares, uint32_t k, uint32_t n,
                                                                      const uint32_t* H, const uint32_t* vk_lines,
                                                                      const uint8_t* vk_ok, const uint32_t* gen_lines,
                                                                      int do_verify, int parsed, uint8_t* valid,
                                                                      uint32_t* sig, uint32_t* ids) {
  __shared__ PairXchg xc;
  __shared__ FeMail fm;  // WAVES = 2: the final exponentiation's helper wave
  __shared__ uint32_t lxs[2 * BN_ATE_LINES * P36_LX_WORDS];  // lambda' (p36_lambda_x): two pairs, or one per wave
  const uint32_t j = blockIdx.x;
  if (j >= k) return;  // whole blocks exit together
  const int wave = threadIdx.x >> 6;
  const P36 g = p36_lane();
  if (WAVES == 2 && threadIdx.x == 0) femail_init(fm);
  const uint8_t* sh = shares + 37 * (size_t)j;
  const uint32_t id = ((uint32_t)sh[0] << 24) | ((uint32_t)sh[1] << 16) | ((uint32_t)sh[2] << 8) | sh[3];
  const bool id_ok = id >= 1 && id <= n;
  const bool key_ok = do_verify && id_ok && vk_ok[id - 1] != 0;
  const uint32_t* vkl = key_ok ? vk_lines + (size_t)(id - 1) * LINES_PER_KEY : nullptr;
  if (WAVES == 1) {
    g1a s;
    bool good;
    if (parsed) {
      good = valid[j] != 0;
      g1a_load(s, sig + 19 * (size_t)j);
    } else {
      uint32_t pid;
      good = bls_parse_share_row(pid, s, sh) && id_ok;
      if (g.lane == 0) {
        ids[j] = id;
        g1a_store(sig + 19 * (size_t)j, s);
      }
    }
    if (do_verify) {
      good = good && key_ok;
      if (good) {
        g1a P[2];
        g1a_load(P[0], H);
        P[1] = s;
        if (!s.inf) f_neg(P[1].y, s.y);
        const uint32_t* l[2] = {vkl, gen_lines};
        good = P[1].inf ? p36_pairing_check<1>(P, l, g, lxs) : p36_pairing_check<2>(P, l, g, lxs);
      }
    }
    if (g.lane == 0) valid[j] = good ? 1 : 0;
    return;
  }
  fp f;
  if (wave == 1) {
    g1a s;
    bool decoded;
    if (parsed) {
      decoded = valid[j] != 0;
      g1a_load(s, sig + 19 * (size_t)j);
    } else {
      uint32_t pid;
      decoded = bls_parse_share_row(pid, s, sh) && id_ok;
      if (g.lane == 0) {
        ids[j] = id;
        g1a_store(sig + 19 * (size_t)j, s);
      }
    }
    if (decoded && key_ok && !s.inf) {
      g1a P = s;
      f_neg(P.y, s.y);
      const uint32_t* l[1] = {gen_lines};
      p36_miller<1>(f, &P, l, g, nullptr, lxs + BN_ATE_LINES * P36_LX_WORDS);
    } else {
      p36_one(f, g);  // e(O, g2) = 1: an infinite sigma checks against e(H, vk) alone
    }
    xchg_put(xc, f, g);
    if (g.lane == 0) xc.ok = decoded ? 1 : 0;
  } else if (key_ok) {
    g1a P;
    g1a_load(P, H);
    const uint32_t* l[1] = {vkl};
    p36_miller<1>(f, &P, l, g, nullptr, lxs);
  }
  __syncthreads();
  bool good = xc.ok != 0;
  if (wave == 1) {
    if (do_verify && good && key_ok) p36_fe2_helper(fm, g);
    return;
  }
  if (wave != 0) return;
  if (do_verify) {
    good = good && key_ok;
    if (good) {
      fp f1;
      xchg_get(f1, xc, g);
      p36_mul(f, f, f1, g);
      good = p36_is_one_after_final_exp_lead(f, fm, g);
    }
  }
  if (g.lane == 0) valid[j] = good ? 1 : 0;
}

// H = g1_map(msg), sigma from 33 bytes: e(H, PK) * e(-sigma, g2) == 1 for a combined signature,
// in one block of FOUR waves: each pair's Miller loop is split in two (p36_miller_part: top part
// + squarings | bottom part + Frobenius lines, 209 vs 320 Fp multiplications per lane).  Waves 0
// and 1 both hash to G1 (wave 0 stores H) and run the (H, PK) parts; waves 2 and 3 both decode
// sigma and run the (-sigma, g2) parts; waves 1..3 hand their values over through LDS and wave 0
// multiplies the four and runs the final exponentiation.
#define VERIFY_BLOCK 256
__global__ void __launch_bounds__(VERIFY_BLOCK) bls_verify_kernel(const uint8_t* msg, uint32_t len, uint32_t* H_out,
                                                                  const uint8_t* sig33, const uint32_t* pk_lines,
                                                                  const uint8_t* pk_ok, const uint32_t* gen_lines,
                                                                  uint8_t* result, const uint32_t* H_in,
                                                                  const uint32_t* sig_aff) {
  __shared__ PairXchg xc[3];  // the values of waves 1, 2, 3
  __shared__ FeMail fm;       // wave 1 helps wave 0's final exponentiation
  __shared__ uint32_t lxv[4 * BN_ATE_LINES * P36_LX_WORDS];  // lambda' of each wave's Miller part
  if (blockIdx.x != 0) return;
  const int wave = threadIdx.x >> 6;
  const P36 g = p36_lane();
  if (threadIdx.x == 0) femail_init(fm);
  fp f;
  if (wave < 2) {
    g1a P;
    if (H_in)
      g1a_load(P, H_in);  // hashed by an earlier kernel of the same call
    else
      g1_map_row(P, msg, len);
    if (wave == 0 && g.lane == 0 && H_out) g1a_store(H_out, P);
    if (wave == 0)
      p36_miller_part<true>(f, P, pk_lines, g, nullptr, lxv);
    else
      p36_miller_part<false>(f, P, pk_lines, g, nullptr, lxv + BN_ATE_LINES * P36_LX_WORDS);
  } else {
    g1a s;
    bool ok = true;
    if (sig_aff)
      g1a_load(s, sig_aff);  // the combine's own point: decompressing its 33 bytes gives it back
    else
      ok = g1_decompress_row(s, sig33);
    if (ok && !s.inf) {
      g1a P = s;
      f_neg(P.y, s.y);
      if (wave == 2)
        p36_miller_part<true>(f, P, gen_lines, g, nullptr, lxv + 2 * BN_ATE_LINES * P36_LX_WORDS);
      else
        p36_miller_part<false>(f, P, gen_lines, g, nullptr, lxv + 3 * BN_ATE_LINES * P36_LX_WORDS);
    } else {
      p36_one(f, g);  // e(O, g2) = 1
    }
    if (g.lane == 0) xc[wave - 1].ok = ok ? 1 : 0;
  }
  if (wave > 0) xchg_put(xc[wave - 1], f, g);
  __syncthreads();
  bool good = xc[1].ok != 0 && pk_ok[0] != 0;
  if (wave == 1) {
    if (good) p36_fe2_helper(fm, g);
    return;
  }
  if (wave != 0) return;
  if (good) {
#pragma nounroll
    for (int w = 0; w < 3; w++) {
      fp f1;
      xchg_get(f1, xc[w], g);
      p36_mul(f, f, f1, g);
    }
    good = p36_is_one_after_final_exp_lead(f, fm, g);
  }
  if (g.lane == 0) result[0] = good ? 1 : 0;
}

// Multisig verify in one block (BlsMultisigVerifier: e(H, sum vk_i) e(-sigma, g2) == 1):
//   wave 0  PK = sum of the key-sum partials (bls_g2_sum_kernel), to affine, then its 70
//           unnormalised lines (bn254_g2wave.h) into LDS, publishing each as it lands;
//   wave 1  H = g1_map(msg), then the (H, PK) Miller loop, reading each line as soon as wave 0
//           has published it (the loop trails the line computation instead of following it);
//   wave 2  decompress sigma, the (-sigma, g2) Miller loop over the precomputed generator lines.
// Wave 1 joins the two Miller values and runs the final exponentiation, wave 2 helps it.  Every
// wave reaches the end: wave 0 publishes "all lines" even when PK is unusable (bad key, infinity).
// (Five waves with each Miller loop split in two, as bls_verify_kernel, measured 1.018 against
// 0.926 ms: the fifth wave shares a SIMD with the line computation that paces the (H, PK) loop.)
#define MS_BLOCK 192
__global__ void __launch_bounds__(MS_BLOCK) bls_verify_multisig_kernel(const uint32_t* parts, uint32_t count,
                                                                       const uint8_t* msg, uint32_t len,
                                                                       const uint8_t* sig33, const uint32_t* gen_lines,
                                                                       uint8_t* pk_ok, uint8_t* result) {
  __shared__ PairXchg xc[1];  // wave 2's value
  __shared__ uint32_t lines[BN_ATE_LINES * BN_ABC_WORDS];
  __shared__ int progress;
  __shared__ int usable;
  __shared__ FeMail fm;  // the final exponentiation's helper: wave 2
  if (blockIdx.x != 0) return;
  const int wave = threadIdx.x >> 6;
  const P36 g = p36_lane();
  if (threadIdx.x == 0) {
    progress = 0;
    usable = 0;
    xc[0].ok = 0;
    femail_init(fm);
  }
  __syncthreads();
  fp f;
  const int lead = 1, helper = 2;
  if (wave == 0) {
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
    g2a s;
    g2_to_affine<true>(s, acc);  // public point: variable-time inversion
    const bool ok = !bad && !s.inf;
    if (g.lane == 0) {
      pk_ok[0] = ok ? 1 : 0;
      usable = ok ? 1 : 0;
    }
    if (ok) g2r_lines_abc(lines, s, &progress);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (g.lane == 0) progress = BN_ATE_LINES + 1;  // release the consumers whatever happened
  } else if (wave == 1) {
    g1a P;
    g1_map_row(P, msg, len);
    const uint32_t* l[1] = {lines};
    p36_miller<1, true>(f, &P, l, g, &progress);
  } else {
    g1a s;
    const bool ok = g1_decompress_row(s, sig33);
    if (ok && !s.inf) {
      g1a P = s;
      f_neg(P.y, s.y);
      // (no lambda' here: this loop finishes before the (H, PK) loop that trails the line
      // computation, and forming it measured 12 us slower overall)
      const uint32_t* l[1] = {gen_lines};
      p36_miller<1>(f, &P, l, g);
    } else {
      p36_one(f, g);
    }
    if (g.lane == 0) xc[0].ok = ok ? 1 : 0;
  }
  if (wave == 2) xchg_put(xc[0], f, g);
  __syncthreads();
  bool good = xc[0].ok != 0 && usable != 0;  // sigma decoded (wave 2), PK usable
  if (wave == helper) {
    if (good) p36_fe2_helper(fm, g);
    return;
  }
  if (wave != lead) return;
  if (good) {
    fp f1;
    xchg_get(f1, xc[0], g);
    p36_mul(f, f, f1, g);
    good = p36_is_one_after_final_exp_lead(f, fm, g);
  }
  if (g.lane == 0) result[0] = good ? 1 : 0;
}

// H = g1_map(msg) (block 0, when H is non-null) beside the decoding of k shares, one DPP row per
// share (blocks 1..: four shares per wave, the square root on the row, ~2x shorter than one lane's):
// id, affine point, valid = decodable && id in [1, n].  The shares' square roots then run while
// the message is hashed instead of after it, inside the verify.
__global__ void __launch_bounds__(64) bls_prep_kernel(const uint8_t* msg, uint32_t len, uint32_t* H,
                                                      const uint8_t* shares, uint32_t k, uint32_t n, uint8_t* valid,
                                                      uint32_t* sig, uint32_t* ids) {
  if (blockIdx.x == 0) {
    if (!H) return;
    g1a P;
    g1_map_row(P, msg, len);
    if ((threadIdx.x & 63) == 0) g1a_store(H, P);
    return;
  }
  if (k == 0) return;
  const uint32_t j = (blockIdx.x - 1) * 4 + ((threadIdx.x & 63) >> 4);
  const uint32_t jj = j < k ? j : k - 1;  // rows past the last share decode it again, store nothing
  uint32_t id;
  g1a s;
  const bool ok = bls_parse_share_row(id, s, shares + 37 * (size_t)jj) && id >= 1 && id <= n;
  if (j < k && (threadIdx.x & 15) == 0) {
    ids[j] = id;
    g1a_store(sig + 19 * (size_t)j, s);
    valid[j] = ok ? 1 : 0;
  }
}

// ------------------------------------------------------------------------------ launchers
hipError_t cbft_bls_launch_prep(const uint8_t* d_msg, uint32_t len, uint32_t* d_H, const uint8_t* d_shares, uint32_t k,
                                uint32_t n, uint8_t* d_valid, uint32_t* d_sig, uint32_t* d_ids, hipStream_t s) {
  hipLaunchKernelGGL(bls_prep_kernel, dim3(1 + (k + 3) / 4), dim3(64), 0, s, d_msg, len, d_H, d_shares, k, n, d_valid,
                     d_sig, d_ids);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_share_verify(const uint8_t* d_shares, uint32_t k, uint32_t n, const uint32_t* d_H,
                                        const uint32_t* d_vk_lines, const uint8_t* d_vk_ok,
                                        const uint32_t* d_gen_lines, int do_verify, int parsed, uint8_t* d_valid,
                                        uint32_t* d_sig, uint32_t* d_ids, hipStream_t s) {
  if (!k) return hipSuccess;
  const bool two = 2 * (size_t)k <= SIMDS;  // two waves per share while they all fit one per SIMD
  if (do_verify && two)
    hipLaunchKernelGGL(bls_share_verify_kernel<2>, dim3(k), dim3(128), 0, s, d_shares, k, n, d_H, d_vk_lines,
                       d_vk_ok, d_gen_lines, do_verify, parsed, d_valid, d_sig, d_ids);
  else
    hipLaunchKernelGGL(bls_share_verify_kernel<1>, dim3(k), dim3(64), 0, s, d_shares, k, n, d_H, d_vk_lines,
                       d_vk_ok, d_gen_lines, do_verify, parsed, d_valid, d_sig, d_ids);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_verify(const uint8_t* d_msg, uint32_t len, uint32_t* d_H, const uint8_t* d_sig33,
                                  const uint32_t* d_pk_lines, const uint8_t* d_pk_ok,
                                  const uint32_t* d_gen_lines, uint8_t* d_result, hipStream_t s,
                                  const uint32_t* d_H_in, const uint32_t* d_sig_aff) {
  hipLaunchKernelGGL(bls_verify_kernel, dim3(1), dim3(VERIFY_BLOCK), 0, s, d_msg, len, d_H, d_sig33, d_pk_lines,
                     d_pk_ok, d_gen_lines, d_result, d_H_in, d_sig_aff);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_verify_multisig(const uint32_t* d_parts, uint32_t count, const uint8_t* d_msg, uint32_t len,
                                           const uint8_t* d_sig33, const uint32_t* d_gen_lines, uint8_t* d_pk_ok,
                                           uint8_t* d_result, hipStream_t s) {
  hipLaunchKernelGGL(bls_verify_multisig_kernel, dim3(1), dim3(MS_BLOCK), 0, s, d_parts, count, d_msg, len, d_sig33,
                     d_gen_lines, d_pk_ok, d_result);
  return hipGetLastError();
}
