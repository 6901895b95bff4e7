/*
 * libcbft_hipcrypto — C ABI of the MI355X batch signature-verification engine for concord-bft.
 *
 * This is the drop-in boundary between the reference's crypto plugin interfaces and the GPU:
 *
 *   concord::util::crypto::IVerifier::verify        util/include/crypto_utils.hpp:41-47
 *   SigManager::verifySig (per-principal verify)     bftengine/src/bftengine/SigManager.cpp:197-238
 *   serial verify loops it replaces with one batch:  PrePrepareMsg.cpp:116-125,
 *                                                    PreProcessor.cpp:557-590,
 *                                                    PreProcessBatchRequestMsg.cpp:62-75,
 *                                                    PreProcessResultMsg.cpp:57-99
 *   OpenSSL verify idiom whose verdicts it matches:  util/src/openssl_crypto.cpp:229-253
 *     (EVP_DigestVerify with EVP_PKEY_ED25519, OpenSSL 3.0.2; accept only on == 1)
 *
 * Conventions:
 *   - every function returns 0 (CBFT_OK) or a negative errno-style code; no C++ exception ever
 *     crosses this boundary;
 *   - the caller owns every buffer; host-pointer entry points are blocking unless named _async;
 *   - a context is bound to one GPU (cbft_open) or to a set of GPUs (cbft_open_mask: Ed25519
 *     batches shard statically across them); every entry point is thread-safe:
 *     submissions are serialised briefly, waiting for results is not (batches of several
 *     threads are in flight together);
 *   - a verdict never depends on batch composition (each signature is verified independently);
 *   - a bad signature is a 0 verdict bit, never an error code.
 * All integers are little-endian; keys are 32 raw bytes (RFC 8032 encoding), signatures are
 * 64 raw bytes R || S.
 */
#ifndef CBFT_HIPCRYPTO_H
#define CBFT_HIPCRYPTO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CBFT_OK 0
#define CBFT_EINVAL (-22) /* bad argument (null pointer with n > 0, unknown table id, ...) */
#define CBFT_ENOMEM (-12) /* device or host allocation failed */
#define CBFT_ENODEV (-19) /* no such GPU / HIP runtime unavailable */
#define CBFT_EIO (-5)     /* a HIP launch or copy failed */
#define CBFT_E2BIG (-7)   /* batch larger than the context was opened for */

#define CBFT_ED25519_PUBLIC_KEY_BYTES 32
#define CBFT_ED25519_SIGNATURE_BYTES 64

typedef struct cbft_ctx cbft_ctx;

/* Number of visible GPUs (>= 0), or a negative code. */
int cbft_device_count(void);

/* Human-readable text for a return code. */
const char* cbft_strerror(int code);

/* Detail of the calling thread's last CBFT_EIO/CBFT_ENOMEM failure (HIP call + error), or "". */
const char* cbft_last_error(void);

/* Open a context on GPU `device` for batches of up to `max_batch` signatures (the working
 * buffers grow on demand above that; max_batch only pre-sizes them). */
int cbft_open(cbft_ctx** out, int device, size_t max_batch);
/* Open one context over every GPU whose bit is set in device_mask (bit d = device d; SURVEY.md
 * §8(b)).  Ed25519 key tables are replicated on each device; an Ed25519 host-buffer batch is cut
 * into contiguous shards of whole 64-signature words, one per device, verified concurrently, and
 * the verdicts land in the caller's one bitmap.  BLS key sets are loaded on every device and
 * cbft_bls_verify_shares cuts the shares into contiguous slices, one per device, verified
 * concurrently (bitmaps merged).  RSA key tables are loaded on every device and an RSA
 * host-buffer batch is sharded like an Ed25519 one.  The other BLS calls and the profiling calls
 * run on the lowest device of the mask; the _device entry points need a single-GPU context
 * (CBFT_EINVAL).
 * A one-bit mask is exactly cbft_open. */
int cbft_open_mask(cbft_ctx** out, uint32_t device_mask, size_t max_batch);
/* The same over an explicit device list, in shard order; a device may repeat (several shards,
 * each with its own streams, on one GPU — how the multi-GPU geometry is tested on one GPU). */
int cbft_open_devices(cbft_ctx** out, const int* devices, int ndevices, size_t max_batch);
/* Devices of a context: returns their count and writes up to max_out device ordinals. */
int cbft_device_of(cbft_ctx* ctx, int* out_devices, int max_out);
void cbft_close(cbft_ctx* ctx);

/* ---------------------------------------------------------------- tuning ------------------
 * Every kernel a context runs is the measured default; nothing in the process environment
 * selects another kernel.  The environment variables the library and its C++ plugin layer read
 * are all here:
 *   CBFT_COMB_BUDGET_GB   HBM budget of one Ed25519 key table's comb tables (default 64 GB):
 *                         picks the widest comb radix of 13 / 11 / 8 that fits (cbft_ed25519_load_keys)
 *   CBFT_COMB_RADIX       a fixed comb radix 8..15 instead
 *   CBFT_DEVICE           the GPU the C++ verifiers open (host layer; default 0)
 *   CBFT_ENGINE_INFLIGHT  per-request engine: coalesced batches in flight (host layer)
 *   CBFT_ENGINE_SPIN_US   per-request engine: waiter spin before sleeping (host layer; default 0)
 *   CBFT_EXPECTED_KEYS    key-table sizing hint of the C++ SigManager (host layer)
 * Geometry and scheduling switches that tests exercise on purpose (both ladder layouts, other B
 * comb radices, the three-kernel path at small sizes, ...) are per-context options, set after
 * cbft_open and before the first batch that should use them; a multi-GPU context applies them
 * to every device.  CBFT_EINVAL for an unknown option or an out-of-range value. */
#define CBFT_OPT_LADDER_LANES 1     /* comb ladder lanes per signature: 0 = by batch (2 from 32K, else 4), 2, 4 */
#define CBFT_OPT_B_RADIX 2          /* radix of B's comb table, 16..26 (default 22); rebuilds it, synchronously */
#define CBFT_OPT_WORK_SLOTS 3       /* work-buffer slots big batches rotate over, 1..8 (default 4) */
#define CBFT_OPT_SMALL_MAX 4        /* key-table batches up to this size run as one fused launch (default 1024; 0 = never) */
#define CBFT_OPT_SHA_SORT_MIN 5     /* variable-length batches from this size hash in SHA-block-count order (4096; 0 = never) */
#define CBFT_OPT_STAGE_ORDER 6      /* cross-batch stage order of big batches: 0 off, 1 hash + ladder (default), 2 ladder only */
#define CBFT_OPT_HASH_ORDER_EARLY 7 /* the next batch's hash waits for the short-message hash only (default 1) */
#define CBFT_OPT_FINISH_K 8         /* signatures per finish lane: 0 = by batch (2 from 16K, else 1), 1, 2 */
int cbft_set_option(cbft_ctx* ctx, int option, int64_t value);

/* Page-locked host memory, DMA-able by every device.  A caller that builds its batches directly
 * in such memory (signatures, key indices, the message blob) saves the host copy: the
 * host-buffer entry points move any input lying inside a cbft_host_alloc block to the GPU with
 * one DMA each, and pack other (pageable) inputs into internal pinned staging first.
 * cbft_host_free only after every batch reading the block has been waited for. */
int cbft_host_alloc(cbft_ctx* ctx, size_t bytes, void** out);
int cbft_host_free(cbft_ctx* ctx, void* p);

/* ---------------------------------------------------------------- Ed25519 ----------------
 * Verdict semantics are exactly OpenSSL 3.0.2 EVP_DigestVerify(ED25519) == 1:
 * S < L, A decoded without a canonical-y check, cofactorless [S]B - [h]A, R compared bytewise
 * after re-encoding (so non-canonical R is rejected, small-order A is not).
 */

/* Upload and pre-process a key table (decoding and per-key precomputation run once here, like
 * SigManager's one-verifier-per-key cache, SigManager.cpp:139-150).  A key that does not
 * decode is accepted into the table; every signature under it verifies false. */
int cbft_ed25519_load_keys(cbft_ctx* ctx, const uint8_t* pk /* nkeys x 32 */, uint32_t nkeys,
                           uint32_t* out_key_table_id);
/* Same, choosing the radix 2^comb_radix of the per-key fixed-base comb tables (8..15; 14 and 15
 * only on explicit request: 20.9 / 41.9 MB per key).  0 = the
 * default: $CBFT_COMB_RADIX if set, else the widest of 13 / 11 / 8 whose tables fit
 * $CBFT_COMB_BUDGET_GB (default 64).  Memory per key = npos x (2^(radix-1) + 1) x 128 B:
 * radix 8: 0.53 MB (32 additions per [h]A), 11: 3.0 MB (23), 13: 10.5 MB (20).  The verdicts do
 * not depend on the radix. */
int cbft_ed25519_load_keys_ex(cbft_ctx* ctx, const uint8_t* pk, uint32_t nkeys, int comb_radix,
                              uint32_t* out_key_table_id);
int cbft_ed25519_unload_keys(cbft_ctx* ctx, uint32_t key_table_id);
/* Append nkeys keys to a loaded table (new client keys, key rotation: SigManager::
 * setClientPublicKey, SigManager.cpp:250-264; KeyExchangeManager.cpp:310-320).  The keys get
 * indices *out_first_index .. + nkeys - 1; the keys already loaded are neither moved nor rebuilt,
 * and batches against them keep running while the new keys' tables are built (only the new
 * indices are unusable until this call returns).  Up to 1,048,576 keys per table (CBFT_E2BIG).
 * The table keeps its comb radix while the grown table fits $CBFT_COMB_BUDGET_GB (default 64);
 * past it the whole table is rebuilt once at the widest radix that fits (13 -> 11 -> 8, key
 * indices unchanged, batches against the old table finish first), and past the budget at radix 8
 * the call fails with CBFT_ENOMEM leaving the table as it was.  A table loaded with nkeys = 0
 * starts empty. */
int cbft_ed25519_append_keys(cbft_ctx* ctx, uint32_t key_table_id, const uint8_t* pk, uint32_t nkeys,
                             uint32_t* out_first_index);
/* Rebuild loaded key slots idx[0..n) in place with new keys pk (n x 32 B): a rotated key reusing
 * the slot of a key nothing references any more (SigManager::setClientPublicKey replaces a
 * client's verifier, SigManager.cpp:250-264), so key rotation does not grow the table.  The
 * caller guarantees no batch names these slots while the call runs.  CBFT_EINVAL if a slot is
 * not loaded. */
int cbft_ed25519_replace_keys(cbft_ctx* ctx, uint32_t key_table_id, const uint32_t* idx, const uint8_t* pk,
                              uint32_t n);
/* Published key count and comb radix of a table. */
int cbft_ed25519_table_size(cbft_ctx* ctx, uint32_t key_table_id, uint32_t* out_nkeys, int* out_radix);

/* Verify n signatures against keys of a loaded table (blocking: _async + cbft_wait).
 *   key_idx[i]   : index of signature i's key in the table (< nkeys, else CBFT_EINVAL)
 *   sig          : n x 64 bytes
 *   msg_blob     : all messages; message i = msg_blob[msg_off[i] .. msg_off[i] + msg_len[i])
 *   verdict_bitmap: ceil(n/8) bytes, bit (i % 8) of byte i/8 = 1 iff signature i verifies
 * Bits beyond n in the last byte are written as 0. */
int cbft_ed25519_verify_batch(cbft_ctx* ctx, uint32_t key_table_id, const uint32_t* key_idx, const uint8_t* sig,
                              const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len, size_t n,
                              uint8_t* verdict_bitmap);

/* Asynchronous form: queues the batch (host -> device copy on a copy stream, kernels on compute
 * streams, so several batches overlap: batch i+1's copy runs under batch i's kernels) and returns
 * a ticket.  Inputs in cbft_host_alloc memory are read by DMA after the call returns and must stay
 * unchanged until cbft_wait(ticket); pageable inputs are copied before the call returns.
 * verdict_bitmap is written no later than when cbft_wait(ticket) returns (possibly earlier, when
 * a later submission needs the batch's slot).  n = 0 returns ticket 0. */
int cbft_ed25519_verify_batch_async(cbft_ctx* ctx, uint32_t key_table_id, const uint32_t* key_idx,
                                    const uint8_t* sig, const uint8_t* msg_blob, const uint64_t* msg_off,
                                    const uint32_t* msg_len, size_t n, uint8_t* verdict_bitmap, uint64_t* out_ticket);
/* Fixed-length messages (no offset/length arrays to move): message i = msg_blob[i * msg_len,
 * (i + 1) * msg_len). */
int cbft_ed25519_verify_fixed_async(cbft_ctx* ctx, uint32_t key_table_id, const uint32_t* key_idx,
                                    const uint8_t* sig, const uint8_t* msg_blob, uint32_t msg_len, size_t n,
                                    uint8_t* verdict_bitmap, uint64_t* out_ticket);
/* Where to place a fixed-length batch's arrays inside one cbft_host_alloc block (key indices at
 * +*off_key_idx, signatures at +*off_sig, messages at +*off_msg; *total_bytes in all) so that
 * cbft_ed25519_verify_fixed_async moves the whole batch with ONE DMA: at the PCIe bound of the
 * host path, one 21 MB copy per 64K batch instead of three. */
int cbft_ed25519_batch_layout(size_t n, uint32_t msg_len, size_t* off_key_idx, size_t* off_sig, size_t* off_msg,
                              size_t* total_bytes);
/* Wait for a ticket's batch and deliver its verdicts (0 for ticket 0 or a ticket already waited
 * for).  Any thread may wait; the context stays usable by other threads meanwhile. */
int cbft_wait(cbft_ctx* ctx, uint64_t ticket);

/* Same, with one raw 32-byte key per signature (pk = n x 32 bytes); the key is decoded per
 * signature inside the batch. */
int cbft_ed25519_verify_batch_pk(cbft_ctx* ctx, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg_blob,
                                 const uint64_t* msg_off, const uint32_t* msg_len, size_t n,
                                 uint8_t* verdict_bitmap);

/* Device-resident variant: every pointer is device memory on the context's GPU, the call is
 * asynchronous on `stream` (a hipStream_t; NULL = the context's own stream) and writes
 * ceil(n/64) 64-bit verdict words (bit i % 64 of word i / 64).  key_table_id selects a loaded
 * table (then key_idx indexes it) or is CBFT_NO_KEY_TABLE (then d_pk holds n raw keys).  A
 * key index >= the table's key count verifies false (the kernels never read past the table).
 * Messages longer than 0xFFFFFF00 bytes verify false.
 * Use cbft_sync() (or the stream) before reading the verdicts. */
#define CBFT_NO_KEY_TABLE 0xffffffffu
int cbft_ed25519_verify_batch_device(cbft_ctx* ctx, uint32_t key_table_id, const uint8_t* d_pk,
                                     const uint32_t* d_key_idx, const uint8_t* d_sig, const uint8_t* d_msg_blob,
                                     const uint64_t* d_msg_off, const uint32_t* d_msg_len, size_t n,
                                     uint64_t* d_verdict_words, void* stream);
/* The same for fixed-length messages (message i = d_msg[i * msg_len, (i + 1) * msg_len)), the
 * device-resident form of cbft_ed25519_verify_fixed_async: no offset / length arrays to read and
 * no block-count sort before the hash kernel. */
int cbft_ed25519_verify_fixed_device(cbft_ctx* ctx, uint32_t key_table_id, const uint8_t* d_pk,
                                     const uint32_t* d_key_idx, const uint8_t* d_sig, const uint8_t* d_msg,
                                     uint32_t msg_len, size_t n, uint64_t* d_verdict_words, void* stream);
int cbft_sync(cbft_ctx* ctx);

/* Instrumentation: when enabled, each verify records HIP events on its stream around its
 * three kernels; cbft_stage_times_ms() then returns (waiting for them) the last verify's
 * {hash, ladder, finish} kernel times in ms into out[0..2] (nout >= 3). */
int cbft_set_profiling(cbft_ctx* ctx, int enable);
int cbft_stage_times_ms(cbft_ctx* ctx, float* out, int nout);
/* enable = 2: every verify records its own events (a ring of the last 256 batches), so batches
 * in flight on several streams keep separate timings; cbft_stage_times_avg_ms() waits for them
 * and returns the mean {hash, ladder, finish} stage times (each stage's events sit on the
 * batch's stream, after its cross-batch waits: the in-pipeline kernel durations) and, in
 * *nbatches (nullable), how many batches were averaged.  -EINVAL unless in mode 2 with >= 1
 * batch since cbft_set_profiling. */
int cbft_stage_times_avg_ms(cbft_ctx* ctx, float* out, int nout, int* nbatches);

/* ------------------------------------------------------- RSA-2048 PKCS#1 v1.5 / SHA-256 ------
 * Replaces concord::util::crypto::RSAVerifier (util/src/crypto_utils.cpp:101-117,155-168), i.e.
 * Crypto++ 8.2.0 RSASS<PKCS1v15, SHA256>::Verifier::VerifyMessage, the verifier SigManager
 * instantiates today for replica (e = 17) and client (e = 65537) keys (SigManager.cpp:138,146,255).
 * Verdict = ((s mod n)^e mod n == 00 01 FF.. 00 || DigestInfo(SHA-256) || SHA-256(m)); as in
 * Crypto++, s is NOT required to be < n (oracle/rsa_ref.py).  Moduli are exactly 2048 bits.
 * A signature is 256 bytes big-endian (IVerifier::signatureLength() of a 2048-bit key). */
#define CBFT_RSA_MODULUS_BYTES 256
#define CBFT_RSA_SIGNATURE_BYTES 256

/* Load nkeys public keys: moduli = nkeys x 256 bytes big-endian (top bit set), exponents = nkeys
 * odd 32-bit public exponents (>= 3).  Per-key records (R^2 mod n, -n^-1 mod 2^32) are built on
 * the GPU here, once.  A key that is not a 2048-bit odd modulus with an odd e >= 3 is accepted
 * into the table and every signature under it verifies false (cbft_rsa_key_status). */
int cbft_rsa_load_keys(cbft_ctx* ctx, const uint8_t* moduli, const uint32_t* exponents, uint32_t nkeys,
                       uint32_t* out_key_table_id);
int cbft_rsa_unload_keys(cbft_ctx* ctx, uint32_t key_table_id);
/* out_ok: nkeys bytes, 1 = the key is usable */
int cbft_rsa_key_status(cbft_ctx* ctx, uint32_t key_table_id, uint8_t* out_ok);

/* Verify n signatures (sig = n x 256 bytes) against keys of a loaded table; message i =
 * msg_blob[msg_off[i] .. + msg_len[i]); verdict_bitmap as for Ed25519.  key_idx[i] >= nkeys is
 * CBFT_EINVAL. */
int cbft_rsa_verify_batch(cbft_ctx* ctx, uint32_t key_table_id, const uint32_t* key_idx, const uint8_t* sig,
                          const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len, size_t n,
                          uint8_t* verdict_bitmap);
/* Device-resident variant (asynchronous on `stream`, ceil(n/64) verdict words); an out-of-range
 * key index verifies false; d_sig must be 4-byte aligned (CBFT_EINVAL otherwise). */
int cbft_rsa_verify_batch_device(cbft_ctx* ctx, uint32_t key_table_id, const uint32_t* d_key_idx,
                                 const uint8_t* d_sig, const uint8_t* d_msg_blob, const uint64_t* d_msg_off,
                                 const uint32_t* d_msg_len, size_t n, uint64_t* d_verdict_words, void* stream);
/* With profiling enabled (cbft_set_profiling): the last RSA verify kernel's duration in ms. */
int cbft_rsa_kernel_ms(cbft_ctx* ctx, float* out_ms);

/* ------------------------------------------------------------- BLS BN-P254 (threshsign) ------
 * RELIC "BN_P254" curve (threshsign/src/bls/relic/Library.cpp:51,72): G1 compressed = 33 bytes,
 * G2 compressed = 65 bytes, share = 4-byte big-endian id || 33-byte G1 (BlsThresholdSigner.cpp:
 * 32-47), signer bitmap = 256 bytes, bit (id-1) LSB-first (VectorOfShares.cpp:136-161).
 * Compressed encodings are RELIC's ep_write_bin / ep2_write_bin (pack = 1): prefix byte
 * 2 | lsb(y * 2^256 mod p) — the parity bit of RELIC's Montgomery-form y (of y's real part in G2) —
 * then x big-endian (G2: x0 || x1).  The G2 rule is pinned by the reference's RELIC-generated key
 * files (tests/golden/relic_bls_keys.json, 40/40 vks); G1 uses the same RELIC fp_get_bit rule.
 * Hash-to-G1 follows RELIC's 2019 ep_map as restated in oracle/bn254_ref.py (SHA-256,
 * try-and-increment; parity with RELIC itself is unpinned there). */
#define CBFT_BLS_G1_BYTES 33
#define CBFT_BLS_G2_BYTES 65
#define CBFT_BLS_SHARE_BYTES 37
#define CBFT_BLS_SIGNERS_BYTES 256

/* Load a verifier key set: the group public key and n share verification keys vk_1..vk_n
 * (65 bytes each).  Decoding, subgroup checks and Miller-loop line precomputation run once
 * here (BlsThresholdVerifier's constructor, BlsThresholdVerifier.cpp:36-51).  Keys that do not
 * decode are accepted and make every check against them fail (see cbft_bls_key_status). */
int cbft_bls_load_keys(cbft_ctx* ctx, const uint8_t* pk65, const uint8_t* vks65, uint32_t n, uint32_t* out_keyset);
int cbft_bls_unload_keys(cbft_ctx* ctx, uint32_t keyset);
/* out_ok: n + 1 bytes, [0] = PK decoded, [i] = vk_i decoded */
int cbft_bls_key_status(cbft_ctx* ctx, uint32_t keyset, uint8_t* out_ok);

/* H = g1_map(msg) as 33 bytes (RELIC ep_map, 2019: SHA-256, try-and-increment). */
int cbft_bls_hash_to_g1(cbft_ctx* ctx, const uint8_t* msg, uint32_t len, uint8_t* out33);

/* Verify k shares against msg: bit j of valid_bitmap (ceil(k/8) bytes) = 1 iff share j decodes,
 * its id is in [1, n] and e(H(msg), vk_id) == e(sigma, g2)
 * (BlsAccumulatorBase::verifyShare, BlsAccumulatorBase.cpp:62-84). */
int cbft_bls_verify_shares(cbft_ctx* ctx, uint32_t keyset, const uint8_t* msg, uint32_t len, const uint8_t* shares37,
                           uint32_t k, uint8_t* valid_bitmap);

/* Combine k shares with distinct ids: threshold (multisig = 0): sum lambda_i sigma_i with
 * lambda_i = prod_{j != i} j/(j - i) mod r over the given ids (BlsThresholdAccumulator,
 * LagrangeInterpolation.cpp:202-292, FastMultExp.cpp:26-59); multisig (multisig = 1):
 * sum sigma_i (BlsMultisigAccumulator.cpp:57-65).  out33 = compressed G1.  CBFT_EINVAL if an id
 * repeats or a share does not decode. */
int cbft_bls_combine(cbft_ctx* ctx, const uint8_t* shares37, uint32_t k, int multisig, uint8_t* out33);

/* The threshold certificate in one call: the SignaturesProcessingJob policy
 * (CollectorOfThresholdSignatures.hpp:363-406; SURVEY.md §8(b) cbft_bls_combine_threshold).
 * The first share of each id is used (later duplicates are ignored, as the accumulators do).
 * optimistic = 1: combine all shares without verifying them, verify the combined signature; if
 * that fails (or a share does not decode), or optimistic = 0: verify every share, combine the
 * valid ones (Lagrange over their ids), verify.  out_sig33 = the combined signature, *out_ok = it
 * verifies under the key set's PK; bad_bitmap (ceil(k/8) bytes): bit j = share j failed share
 * verification (all zero when the optimistic combine verified). */
int cbft_bls_combine_threshold(cbft_ctx* ctx, uint32_t keyset, const uint8_t* msg, uint32_t len,
                               const uint8_t* shares37, uint32_t k, int optimistic, uint8_t* out_sig33,
                               uint8_t* bad_bitmap, int* out_ok);

/* e(H(msg), PK) == e(sig, g2) with the key set's group PK (BlsThresholdVerifier.cpp:69-96). */
int cbft_bls_verify(cbft_ctx* ctx, uint32_t keyset, const uint8_t* msg, uint32_t len, const uint8_t* sig33,
                    int* out_ok);
/* Multisig: PK = sum of vk_i over the signer bitmap (BlsMultisigVerifier.cpp:75-105). */
int cbft_bls_verify_multisig(cbft_ctx* ctx, uint32_t keyset, const uint8_t* msg, uint32_t len, const uint8_t* sig33,
                             const uint8_t* signers256, int* out_ok);

/* out65 = sum of vk_i over the signer bitmap, compressed (65 zero bytes if a selected key does
 * not decode).  The n-of-n multisig public key (BlsMultisigVerifier.cpp:33-38). */
int cbft_bls_sum_keys(cbft_ctx* ctx, uint32_t keyset, const uint8_t* signers256, uint8_t* out65);

/* Sharded combine / multisig key sum across GPUs (one process per GPU, the
 * partials are exchanged with an all-gather, concord-bft_amd/cbft_multigpu.py).  A partial is an
 * opaque fixed-size point (Jacobian, Montgomery form) meaningful only to this library:
 *   cbft_bls_combine_partial    lambda_i over ALL k shares' ids (or 1 with multisig), the sum
 *                               sum_{lo <= j < hi} lambda_j sigma_j of this rank's slice
 *   cbft_bls_combine_finish     sum of `count` partials -> the 33-byte combined signature
 *                               (equal to cbft_bls_combine over all k shares)
 *   cbft_bls_sum_keys_partial   sum of vk_id over signer-bitmap ids in [lo_id, hi_id)
 *   cbft_bls_verify_multisig_partials  sum the key partials, then verify sig33 under that key
 *                               (equal to cbft_bls_verify_multisig with the whole bitmap) */
#define CBFT_BLS_G1_PARTIAL_BYTES 108
#define CBFT_BLS_G2_PARTIAL_BYTES 220
int cbft_bls_combine_partial(cbft_ctx* ctx, const uint8_t* shares37, uint32_t k, uint32_t lo, uint32_t hi,
                             int multisig, uint8_t* out_partial);
int cbft_bls_combine_finish(cbft_ctx* ctx, const uint8_t* partials, uint32_t count, uint8_t* out33);
int cbft_bls_sum_keys_partial(cbft_ctx* ctx, uint32_t keyset, const uint8_t* signers256, uint32_t lo_id,
                              uint32_t hi_id, uint8_t* out_partial);
int cbft_bls_verify_multisig_partials(cbft_ctx* ctx, const uint8_t* msg, uint32_t len, const uint8_t* sig33,
                                      const uint8_t* key_partials, uint32_t count, int* out_ok);

/* The signer's public (share verification) key: out65 = sk * g2 compressed, sk = 32 bytes
 * big-endian (< r) (BlsThresholdSigner's publicKey_, IThresholdSigner::getShareVerificationKey). */
int cbft_bls_public_key(cbft_ctx* ctx, const uint8_t* sk32, uint8_t* out65);

/* Sign a share: out37 = 4-byte big-endian id || sk * g1_map(msg) compressed, sk = 32 bytes
 * big-endian (< r) (IThresholdSigner::signData; BlsThresholdSigner.cpp:32-47). */
int cbft_bls_sign(cbft_ctx* ctx, const uint8_t* sk32, uint32_t id, const uint8_t* msg, uint32_t len, uint8_t* out37);

#ifdef __cplusplus
}
#endif

#endif /* CBFT_HIPCRYPTO_H */
