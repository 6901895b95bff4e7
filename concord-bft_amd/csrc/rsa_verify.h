// Device-side launch interface of the RSA-2048 PKCS#1 v1.5 / SHA-256 batch-verify kernels
// (internal to libcbft_hipcrypto; the public C ABI is include/cbft_hipcrypto.h).
//
// Reference behaviour: concord::util::crypto::RSAVerifier (util/src/crypto_utils.cpp:101-117)
// = Crypto++ 8.2.0 RSASS<PKCS1v15, SHA256>::Verifier, restated in oracle/rsa_ref.py.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#define RSA_LIMBS 64        // 2048-bit modulus as 64 little-endian 32-bit limbs
#define RSA_MOD_BYTES 256
// Key record in HBM (uint32 words):
//   [0, 136)   32-bit-limb form (FIOS kernel): n[64] | R^2 mod n [64] (R = 2^2048) | -n^-1 mod 2^32 |
//              e | ok | pad
//   [136, 384) 28-bit-limb form (lane-pair kernel, R' = 2^2072): n[80] | R'^2 mod n [80] |
//              R' mod n [80] | -n^-1 mod 2^28 | pad   (limbs beyond 74 are zero)
#define RSA_KEY_WORDS 384
#define RSA_KEY_N 0
#define RSA_KEY_R2 64
#define RSA_KEY_N0INV 128
#define RSA_KEY_E 129
#define RSA_KEY_OK 130
#define RSA_NL 74           // 28-bit limbs of a value < 2^2072
#define RSA_PL 80           // 28-bit limbs stored per operand
#define RSA_KEY_P_N 136
#define RSA_KEY_P_R2 216
#define RSA_KEY_P_R1 296
#define RSA_KEY_P_N0INV 376
// One batch, all pointers in device memory.  Signature i is sig[256 i .. 256 i + 256), big-endian
// (sig must be 4-byte aligned).
struct RsaBatch {
  size_t n;
  const uint32_t* keys;     // key table (RSA_KEY_WORDS per key)
  uint32_t nkeys;
  const uint32_t* key_idx;  // n indices into the key table
  const uint8_t* sig;
  const uint8_t* msg;
  const uint64_t* msg_off;
  const uint32_t* msg_len;
};

// Build key records from nkeys big-endian moduli (256 B each) and 32-bit public exponents.
hipError_t cbft_rsa_launch_keys(const uint8_t* d_mod, const uint32_t* d_exp, uint32_t nkeys, uint32_t* d_keys,
                                hipStream_t stream);
// Verify a batch (the lane-pair radix-2^28 kernel); writes ceil(n/64) verdict words.  d_scratch:
// cbft_rsa_scratch_words(n) words.
hipError_t cbft_rsa_launch_verify(const RsaBatch& b, uint32_t* d_scratch, uint64_t* d_verdicts, hipStream_t stream);
size_t cbft_rsa_scratch_words(size_t n);
