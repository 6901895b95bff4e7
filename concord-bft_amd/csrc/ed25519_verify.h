// Device-side launch interface of the Ed25519 batch-verify kernels (internal to
// libcbft_hipcrypto; the public C ABI is include/cbft_hipcrypto.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#ifndef CBFT_WA
#define CBFT_WA 5  // signed window width for h (the -A table has 2^(WA-1)+1 entries)
#endif
#ifndef CBFT_WB
#define CBFT_WB 7  // signed window width for S (the LDS base table has 2^(WB-1)+1 entries)
#endif
#ifndef CBFT_VERIFY_BLOCK
#define CBFT_VERIFY_BLOCK 256
#endif
#ifndef CBFT_COMB8_LDS
#define CBFT_COMB8_LDS 1  // stage comb-table entries through LDS with global_load_lds
#endif
#ifndef CBFT_LADDER_MIN_WAVES
#define CBFT_LADDER_MIN_WAVES 4  // waves/SIMD the ladder is register-allocated for
#endif

// One batch of signatures, all pointers in device memory.
struct Ed25519Batch {
  size_t n;                 // signatures
  const uint8_t* pk;        // public keys, 32 B each: key of sig i = pk[key_idx ? key_idx[i] : i]
  const uint32_t* key_idx;  // nullable
  const uint8_t* sig;       // n x 64 B (R || S)
  const uint8_t* msg;       // message blob
  const uint64_t* msg_off;  // n byte offsets into msg
  const uint32_t* msg_len;  // n lengths
};

// Device work buffers of one verify launch.
struct Ed25519Work {
  const uint32_t* base_table;  // cbft_ed25519_base_table_words() words
  const uint32_t* tbl;         // windowed -A tables, indexed like pk (per-signature key mode)
  const uint32_t* comb_tbl;    // radix-256 comb tables of -A per key (key-table mode; tbl unused)
  const uint32_t* base_comb;   // radix-256 comb table of B
  const uint8_t* aok;          // A decoded OK, indexed like pk
  uint32_t* h_soa;             // 8 x n words
  uint8_t* flags;              // n bytes
  uint32_t* xyz_soa;           // 27 x n words
  uint64_t* verdict_words;     // ceil(n/64) words; bit (i % 64) of word i/64 = accept
};

size_t cbft_ed25519_table_words_per_unit();
size_t cbft_ed25519_comb8_words_per_unit();
size_t cbft_ed25519_comb8_tmp_words_per_unit();
hipError_t cbft_ed25519_launch_comb8_tables(const uint8_t* d_pk, size_t nunits, int negate, uint32_t* d_tbl,
                                           uint32_t* d_tmp, uint8_t* d_aok, hipStream_t stream);
size_t cbft_ed25519_base_table_words();
hipError_t cbft_ed25519_build_base_table(uint32_t* d_tbl, hipStream_t stream);
hipError_t cbft_ed25519_launch_prep(const uint8_t* d_pk, size_t nunits, uint32_t* d_tbl, uint8_t* d_aok,
                                    hipStream_t stream);
// ev: nullable array of 4 events recorded before K1, K2->K3, K3->K4 and after K4 (profiling)
hipError_t cbft_ed25519_launch_verify(const Ed25519Batch& b, const Ed25519Work& w, hipStream_t stream,
                                      hipEvent_t* ev = nullptr);
