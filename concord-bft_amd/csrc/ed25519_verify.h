// Device-side launch interface of the Ed25519 batch-verify kernels (internal to
// libcbft_hipcrypto; the public C ABI is include/cbft_hipcrypto.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

// the windowed ladder of per-signature keys (ed25519_ladder_kernel)
#define CBFT_WA 5  // signed window width for h (the -A table has 2^(WA-1)+1 entries)
#define CBFT_WB 7  // signed window width for S (the LDS base table has 2^(WB-1)+1 entries)
#define CBFT_LADDER_MIN_WAVES 4  // waves/SIMD the windowed ladder is register-allocated for
#define CBFT_VERIFY_BLOCK 256

// A loaded key table lives in chunks of CBFT_KEY_CHUNK keys, so keys can be appended without
// moving (or rebuilding) the ones already loaded: chunk c holds keys [c * CHUNK, (c + 1) * CHUNK)
// as [comb tables: CHUNK x words_per_key words][raw keys: CHUNK x 32 B][decode status: CHUNK B].
// `chunk` is a device array of chunk base pointers; entries are only ever appended.
#define CBFT_KEY_CHUNK_SHIFT 8
#define CBFT_KEY_CHUNK (1u << CBFT_KEY_CHUNK_SHIFT)
#define CBFT_MAX_KEY_CHUNKS 4096  // 1,048,576 keys per table
struct KeyChunks {
  const uint32_t* const* chunk;
  size_t wpk;  // comb words per key
#ifdef __HIPCC__
  __device__ __forceinline__ const uint32_t* base(uint32_t key) const { return chunk[key >> CBFT_KEY_CHUNK_SHIFT]; }
  __device__ __forceinline__ const uint32_t* comb(uint32_t key) const {
    return base(key) + (size_t)(key & (CBFT_KEY_CHUNK - 1)) * wpk;
  }
  __device__ __forceinline__ const uint8_t* pk(uint32_t key) const {
    return reinterpret_cast<const uint8_t*>(base(key) + (size_t)CBFT_KEY_CHUNK * wpk) + (key & (CBFT_KEY_CHUNK - 1)) * 32u;
  }
  __device__ __forceinline__ bool aok(uint32_t key) const {
    return reinterpret_cast<const uint8_t*>(base(key) + (size_t)CBFT_KEY_CHUNK * wpk)[CBFT_KEY_CHUNK * 32u +
                                                                                       (key & (CBFT_KEY_CHUNK - 1))] != 0;
  }
#endif
};
inline size_t cbft_key_chunk_bytes(size_t wpk) { return (size_t)CBFT_KEY_CHUNK * (wpk * 4 + 32 + 1); }

// One batch of signatures, all pointers in device memory.
struct Ed25519Batch {
  size_t n;                 // signatures
  const uint8_t* pk;        // per-signature keys (key_idx == nullptr): 32 B each, key of sig i = pk[i]
  const uint32_t* key_idx;  // nullable: key of sig i = keys[key_idx[i]]
  KeyChunks keys;           // the loaded key table (key_idx != nullptr)
  const uint8_t* sig;       // n x 64 B (R || S)
  const uint8_t* msg;       // message blob
  const uint64_t* msg_off;  // n byte offsets into msg; nullptr = fixed-length messages (below)
  const uint32_t* msg_len;  // n lengths (unused when msg_off is nullptr)
  uint32_t nkeys;           // keys of the table when key_idx is set: key_idx[i] >= nkeys verifies false
  uint32_t fixed_len;       // msg_off == nullptr: message i = msg[i * fixed_len, (i + 1) * fixed_len)
};
// Messages longer than this verify false (SHA-512's 64 + len byte count must not wrap 32 bits).
#define CBFT_MAX_MSG_LEN 0xFFFFFF00u

// Geometry of a fixed-base comb table with signed radix-2^w digits (8 <= w <= 26):
// npos positions of entries() = 2^(w-1) + 1 affine niels points (e * 2^(w j) * P, e = 0 ..
// 2^(w-1)), 32 words each.  npos is the least count whose top digit stays <= 2^(w-1) for every
// scalar < L (tests/test_comb_recode.py).
struct CombGeom {
  int w;
  int npos;
  __host__ __device__ int entries() const { return (1 << (w - 1)) + 1; }
  __host__ __device__ int chunks() const { return (1 << (w - 1)) / 128; }  // table-build lanes per position
  __host__ __device__ size_t words_per_unit() const { return (size_t)npos * entries() * 32; }
};
inline int cbft_comb_npos(int w) {
  static const int kPos[27] = {0,  0,  0,  0,  0,  0,  0,  0,  32, 29, 26, 23, 22, 20,
                               19, 17, 16, 15, 15, 14, 13, 13, 12, 11, 11, 11, 10};
  return (w >= 8 && w <= 26) ? kPos[w] : 0;
}
inline CombGeom cbft_comb_geom(int w) { return CombGeom{w, cbft_comb_npos(w)}; }

// Ladder parameters of the comb verify: -A tables (a), B's table (b), the recoding offsets
// 2^(w-1) sum_{j < npos-1} 2^(w j) as 8 little-endian words, and additions per lane.
struct CombLadder {
  CombGeom a, b;
  uint32_t offA[8], offB[8];
  int nper;
};
inline void cbft_comb_offset(const CombGeom& g, uint32_t* off) {
  for (int k = 0; k < 8; k++) off[k] = 0;
  for (int j = 0; j + 1 < g.npos; j++) {
    const int bit = g.w * j + g.w - 1;
    off[bit >> 5] |= 1u << (bit & 31);
  }
}
inline CombLadder cbft_comb_ladder(int wa, int wb) {
  CombLadder c{};
  c.a = cbft_comb_geom(wa);
  c.b = cbft_comb_geom(wb);
  cbft_comb_offset(c.a, c.offA);
  cbft_comb_offset(c.b, c.offB);
  c.nper = (c.a.npos + c.b.npos + 3) / 4;
  return c;
}
// B's table: radix 2^22 by default (12 positions x 2,097,153 entries, 3.2 GB per context of the
// 288 GB HBM), so a verify against a radix-2^13 key table is 20 + 12 = 32 additions: 16 per lane
// of a pair, 8 per lane of a quad (radix 2^16: 16 positions, 67 MB, 36 additions; measured on
// MI355X at 64K: pair ladder 104 us at 2^22 vs 112 us at 2^16).  $CBFT_B_RADIX selects 16..26:
// radix 2^26 is 10 positions (42.9 GB per context), so radix-2^13 keys + B = 30 additions, 15 per
// lane of a pair.
#define CBFT_COMB_B_RADIX 22
#define CBFT_COMB_MAX_RADIX 26

// Device work buffers of one verify launch.
struct Ed25519Work {
  const uint32_t* base_table;  // cbft_ed25519_base_table_words() words
  const uint32_t* tbl;         // windowed -A tables per signature (per-signature key mode)
  const uint32_t* base_comb;   // comb table of B (key-table mode; the -A combs are in Batch::keys)
  CombLadder comb;             // their geometry
  int comb_lanes;              // lanes per signature of the comb ladder: 4 (quad) or 2 (pair)
  int finish_k;                // signatures per finish lane (1 or 2; one inversion per 64 x finish_k)
  const uint8_t* aok;          // A decoded OK per signature (per-signature key mode)
  uint32_t* h_soa;             // 8 x n words
  uint8_t* flags;              // n bytes
  uint32_t* xyz_soa;           // 27 x n words
  uint64_t* verdict_words;     // ceil(n/64) words; bit (i % 64) of word i/64 = accept
  int small;                   // key-table batch in ONE launch (ed25519_small3_kernel): small batches
  // Variable-length batches: hash signatures in order of their SHA-512 block count (a counting
  // sort into perm before K1), so a wave's lanes run the same number of blocks.  Nullable.
  uint32_t* perm;              // n words
  uint32_t* buckets;           // CBFT_SHA_BUCKETS x 2 + 2 words (counts, cursors, uniform flag, n_short)
  // Messages of >= CBFT_SHA_LONG_BLOCKS SHA-512 blocks (the sorted order's tail) hash on a second
  // stream in blocks of two waves, one expanding the message schedules into LDS, the other running
  // the rounds (ed25519_hash_long_kernel); null aux = off.
  hipStream_t aux;
  hipEvent_t fork_ev, join_ev;
};
// Block-count buckets of the hash sort: bucket min(nblocks, CBFT_SHA_BUCKETS - 1).
#define CBFT_SHA_BUCKETS 256
#define CBFT_SHA_LONG_BLOCKS 12   // messages of >= 12 blocks hash in the long-message kernel
#define CBFT_SHA_LONG_GROUPS 192  // at most 192 x 64 of them (its 83-KB blocks must all be resident)

size_t cbft_ed25519_table_words_per_unit();
// staging words for `lanes` table-build lanes (18 KB each)
size_t cbft_ed25519_comb_tmp_words(size_t lanes);
// Comb tables of nunits encoded points (32 B each at d_pk), in two steps: the position points
// 2^(w j) (+-P) of every unit into d_pos (cbft_ed25519_comb_pos_words words; decode verdicts to
// d_aok when non-null), then build lanes [lane0, lane0 + nlanes) of the nunits * npos * chunks()
// lanes (lane = (unit, position, chunk of 128 multiples)) into d_tbl (units contiguous) or, with
// d_tbl null, into keys a0 .. a0 + nunits - 1 of the chunked key table whose device chunk-pointer
// array is d_chunks; d_tmp holds cbft_ed25519_comb_tmp_words(nlanes) words.
size_t cbft_ed25519_comb_pos_words(size_t nunits, const CombGeom& g);
hipError_t cbft_ed25519_launch_comb_pos(const uint8_t* d_pk, size_t nunits, int negate, const CombGeom& g,
                                        uint32_t* d_pos, uint8_t* d_aok, hipStream_t stream);
hipError_t cbft_ed25519_launch_comb_tables(const uint32_t* d_pos, size_t nunits, const CombGeom& g, uint32_t* d_tbl,
                                           void* const* d_chunks, uint32_t a0, uint32_t* d_tmp, size_t lane0,
                                           size_t nlanes, hipStream_t stream);
size_t cbft_ed25519_base_table_words();
hipError_t cbft_ed25519_build_base_table(uint32_t* d_tbl, hipStream_t stream);
hipError_t cbft_ed25519_launch_prep(const uint8_t* d_pk, size_t nunits, uint32_t* d_tbl, uint8_t* d_aok,
                                    hipStream_t stream);
// ev: nullable array of 4 events recorded before K1, K2->K3, K3->K4 and after K4 (profiling)
// Cross-batch stage order: when `wait`, the hash waits for done[0] and the ladder for done[1]
// (recorded by the previous batch, maybe on another stream); both are re-recorded here.
struct StageOrder {
  bool wait;
  bool hash;    // order the hashes
  bool ladder;  // order the ladders
  bool hash_early;  // done[0] after the short-message hash, before the long tail's join
  hipEvent_t done[2];
};
hipError_t cbft_ed25519_launch_verify(const Ed25519Batch& b, const Ed25519Work& w, hipStream_t stream,
                                      hipEvent_t* ev = nullptr, const StageOrder* order = nullptr);
