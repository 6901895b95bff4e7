// BLS BN-P254 pairing-check kernels for gfx950 (threshsign path).
//
//   bls_share_verify_kernel  one wave per share: parse, e(H, vk_id) e(-sigma, g2) == 1
//                            (BlsAccumulatorBase::verifyShare, BlsAccumulatorBase.cpp:62-84)
//   bls_verify_kernel        e(H, PK) e(-sigma, g2) == 1   (BlsThresholdVerifier.cpp:69-96)
// The G2 side is precomputed (bls_keys.hip); the Fp12 accumulator is spread over a whole wave,
// three lanes per Fp component (bn254_pair36.h).
#include "bls_common.h"
#include "bn254_pair36.h"

// shares: k x 37 bytes.  out: valid[k] (1 = verified), sig[k] (parsed affine point, 19 words),
// ids[k].  A share whose id is outside [1, n] or whose point does not decode is invalid.
// One wave per share: the pairing check runs on 36 lanes (bn254_pair36.h); parsing is
// done by every lane of the group (same latency as one) and lane 0 writes the results.
__global__ void __launch_bounds__(64) bls_share_verify_kernel(const uint8_t* shares, uint32_t k, uint32_t n,
                                                              const uint32_t* H, const uint32_t* vk_lines,
                                                              const uint8_t* vk_ok, const uint32_t* gen_lines,
                                                              int do_verify, uint8_t* valid, uint32_t* sig,
                                                              uint32_t* ids) {
  const uint32_t j = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (j >= k) return;  // whole waves exit together
  const P36 g = p36_lane();
  const bool lead = (threadIdx.x & 63) == 0;
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
        good = p36_pairing_check<1>(P, l, g);
      else
        good = p36_pairing_check<2>(P, l, g);
    }
  }
  if (lead) valid[j] = good ? 1 : 0;
}

// e(H, PK) * e(-sigma, g2) == 1 for a combined signature (33 bytes); one wave
__global__ void __launch_bounds__(64) bls_verify_kernel(const uint32_t* H, const uint8_t* sig33,
                                                        const uint32_t* pk_lines, const uint8_t* pk_ok,
                                                        const uint32_t* gen_lines, uint8_t* result) {
  if (blockIdx.x != 0) return;
  const P36 g = p36_lane();
  g1a P[2];
  g1a_load(P[0], H);
  bool good = pk_ok[0] && g1_decompress(P[1], sig33);
  if (good) {
    const uint32_t* l[2] = {pk_lines, gen_lines};
    if (P[1].inf) {
      good = p36_pairing_check<1>(P, l, g);
    } else {
      f_neg(P[1].y, P[1].y);
      good = p36_pairing_check<2>(P, l, g);
    }
  }
  if (threadIdx.x == 0) result[0] = good ? 1 : 0;
}

// ------------------------------------------------------------------------------ launchers
hipError_t cbft_bls_launch_share_verify(const uint8_t* d_shares, uint32_t k, uint32_t n, const uint32_t* d_H,
                                        const uint32_t* d_vk_lines, const uint8_t* d_vk_ok,
                                        const uint32_t* d_gen_lines, int do_verify, uint8_t* d_valid,
                                        uint32_t* d_sig, uint32_t* d_ids, hipStream_t s) {
  if (!k) return hipSuccess;
  hipLaunchKernelGGL(bls_share_verify_kernel, dim3(k), dim3(64), 0, s, d_shares, k, n, d_H, d_vk_lines,
                     d_vk_ok, d_gen_lines, do_verify, d_valid, d_sig, d_ids);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_verify(const uint32_t* d_H, const uint8_t* d_sig33, const uint32_t* d_pk_lines,
                                  const uint8_t* d_pk_ok, const uint32_t* d_gen_lines, uint8_t* d_result,
                                  hipStream_t s) {
  hipLaunchKernelGGL(bls_verify_kernel, dim3(1), dim3(64), 0, s, d_H, d_sig33, d_pk_lines, d_pk_ok, d_gen_lines,
                     d_result);
  return hipGetLastError();
}
