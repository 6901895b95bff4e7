// Launch interface of the BLS BN-P254 kernels (internal to libcbft_hipcrypto).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#define BLS_SIG_WORDS 19     // affine G1 (x, y, inf flag) per parsed share
#define BLS_JAC_WORDS 27     // Jacobian G1 partial sum
#define BLS_G2A_WORDS 37     // affine G2 (x.a, x.b, y.a, y.b, inf flag) of a decoded key

size_t cbft_bls_lines_words_per_key();
// decode + subgroup-check nkeys G2 keys (d_ok, d_aff) and build their Miller-loop lines (d_lines)
hipError_t cbft_bls_launch_keys(const uint8_t* d_keys65, uint32_t nkeys, uint32_t* d_lines, uint8_t* d_ok,
                                uint32_t* d_aff, hipStream_t s);
hipError_t cbft_bls_launch_gen_lines(uint32_t* d_lines, hipStream_t s);
hipError_t cbft_bls_launch_hash(const uint8_t* d_msg, uint32_t len, uint32_t* d_H, hipStream_t s);
// H = g1_map(msg) when d_H is non-null, beside the decoding of k shares (lane per share):
// d_valid[j] = decodable && id in [1, n], d_sig (19 words each), d_ids
hipError_t cbft_bls_launch_prep(const uint8_t* d_msg, uint32_t len, uint32_t* d_H, const uint8_t* d_shares, uint32_t k,
                                uint32_t n, uint8_t* d_valid, uint32_t* d_sig, uint32_t* d_ids, hipStream_t s);
// parsed: d_valid / d_sig / d_ids already hold bls_prep's decoding (d_valid is overwritten with the verdicts)
hipError_t cbft_bls_launch_share_verify(const uint8_t* d_shares, uint32_t k, uint32_t n, const uint32_t* d_H,
                                        const uint32_t* d_vk_lines, const uint8_t* d_vk_ok,
                                        const uint32_t* d_gen_lines, int do_verify, int parsed, uint8_t* d_valid,
                                        uint32_t* d_sig, uint32_t* d_ids, hipStream_t s);
// lambda over all k shares; the MSM over shares [lo, hi); d_out_jac (nullable): write the sum as
// one Jacobian partial (BLS_JAC_WORDS) instead of compressing it into d_out33
// d_inv: the table of inverses 1..BLS_INV_TABLE mod r (cbft_bls_launch_inv_table; unused with multisig)
hipError_t cbft_bls_launch_combine(const uint32_t* d_sig, const uint32_t* d_ids, const uint8_t* d_use, uint32_t k,
                                   uint32_t lo, uint32_t hi, int multisig, const uint32_t* d_inv, uint32_t* d_lambda,
                                   uint32_t* d_partial, uint8_t* d_out33, uint32_t* d_sig_aff, uint32_t* d_out_jac,
                                   hipStream_t s);
// row-parallel combine (bls_msm_row.hip): lambda_j sigma_j per share (or the shares themselves for
// multisig) summed level by level in d_work ((2 m + 16) BLS_JAC_WORDS words); *d_final = the sum
hipError_t cbft_bls_launch_msm_row(const uint32_t* d_sig, const uint32_t* d_lambda, const uint8_t* d_use, uint32_t m,
                                   int multisig, uint32_t* d_work, uint32_t** d_final, hipStream_t s);
#define BLS_INV_TABLE 2048  // d^-1 mod r for d = 1 .. 2048 (share ids are <= 2048, IThresholdVerifier.h:36)
hipError_t cbft_bls_launch_inv_table(uint32_t* d_inv, hipStream_t s);
hipError_t cbft_bls_launch_and(const uint8_t* d_a, const uint8_t* d_b, uint8_t* d_use, uint32_t k, hipStream_t s);
hipError_t cbft_bls_launch_g1_parts(const uint32_t* d_parts, uint32_t count, uint8_t* d_out33, hipStream_t s);
#define BLS_G2_PART_WORDS 55  // Jacobian G2 partial key sum + bad-key flag
// multisig key sum over the bitmap's ids in [lo_id, hi_id): Jacobian partial (d_out_part,
// BLS_G2_PART_WORDS) or compressed (d_out65)
hipError_t cbft_bls_launch_g2_sum(const uint32_t* d_aff, const uint8_t* d_key_ok, uint32_t n, const uint8_t* d_bitmap,
                                  uint32_t lo_id, uint32_t hi_id, uint8_t* d_ok, uint8_t* d_out65, uint32_t* d_out_part,
                                  uint32_t* d_tmp, hipStream_t s);
// scratch words (d_tmp, required) cbft_bls_launch_g2_sum needs for its intermediate partials
size_t cbft_bls_g2_sum_tmp_words();
// H = g1_map(msg) (-> d_H when non-null) and e(H, PK) e(-sigma, g2) == 1 in one launch
// multisig verify in one launch: PK = sum of count key-sum partials, its lines streamed from one
// wave to the Miller loop of another, sigma's pair on a third (d_pk_ok = PK usable)
hipError_t cbft_bls_launch_verify_multisig(const uint32_t* d_parts, uint32_t count, const uint8_t* d_msg, uint32_t len,
                                           const uint8_t* d_sig33, const uint32_t* d_gen_lines, uint8_t* d_pk_ok,
                                           uint8_t* d_result, hipStream_t s);
// d_H_in (nullable): H = g1_map(msg) already on the device (the kernel does not hash);
// d_sig_aff (nullable): the signature as the affine point a combine produced (BLS_SIG_WORDS), used
// instead of decompressing d_sig33 -- the same point, and a combine's output always decodes
hipError_t cbft_bls_launch_verify(const uint8_t* d_msg, uint32_t len, uint32_t* d_H, const uint8_t* d_sig33,
                                  const uint32_t* d_pk_lines, const uint8_t* d_pk_ok,
                                  const uint32_t* d_gen_lines, uint8_t* d_result, hipStream_t s,
                                  const uint32_t* d_H_in = nullptr, const uint32_t* d_sig_aff = nullptr);
// sigma = sk * g1_map(msg) as a 37-byte share on row-parallel Fp (bls_msm_row.hip): d_H = g1_map(msg) from
// cbft_bls_launch_hash first, or nullptr (the kernel hashes); constant operation sequence in the
// secret scalar
hipError_t cbft_bls_launch_sign_row(const uint32_t* d_H, const uint32_t* d_sk, const uint8_t* d_msg, uint32_t len,
                                    uint32_t id, uint8_t* d_out37, hipStream_t s);
// vk = sk * g2 as a row-parallel fixed-base comb (bls_keys.hip): the table (cbft_bls_pub_table_words
// words) is built once by cbft_bls_launch_pub_table; constant operation sequence in sk
size_t cbft_bls_pub_table_words();
hipError_t cbft_bls_launch_pub_table(uint32_t* d_tbl, hipStream_t s);
hipError_t cbft_bls_launch_pubkey_row(const uint32_t* d_tbl, const uint32_t* d_sk, uint8_t* d_out65, hipStream_t s);
