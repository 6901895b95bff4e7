// Batched Ed25519 signature verification for gfx950 (MI355X).
//
// Semantics: exactly OpenSSL 3.0.2 EVP_DigestVerify(ED25519) == 1 (see oracle/ed25519_ref.py):
//   S < L (strict);  A decoded without a canonicity check on y;  h = SHA-512(R||A||M) mod L;
//   R' = [S]B - [h]A (cofactorless);  accept iff encode(R') == R byte for byte.
//
// The verify is split into four launches so that each phase gets its own register budget
// (the ladder, ~80 % of the work, must run at >= 3-4 waves/SIMD; decode and inversion chains
// need ~160 VGPRs and would otherwise drag the whole kernel to 1 wave/SIMD).  Per-signature
// state crosses the launch boundaries through HBM in structure-of-arrays layout (coalesced):
//
//   K1 ed25519_hash_kernel    h = SHA-512(R||A||M) mod L   -> h[8][n],   flags[n] (S < L)
//   K2 ed25519_prep_kernel    decode A, table j*(-A), j = 0..2^(WA-1) (cached form)
//                             -> tbl[unit][TA][36], aok[unit]          (unit = key or signature)
//   K3 ed25519_ladder_kernel  (X:Y:Z) = [h](-A) + [S]B       -> xyz[27][n]
//   K4 ed25519_finish_kernel  encode, compare with R         -> verdict bitmap (ballot words)
//
// K2 runs once per KEY when the caller uses a key table (cbft_ed25519_load_keys: the decoded,
// pre-multiplied key is cached exactly as SigManager caches one verifier object per key), or
// once per signature for per-signature keys.
//
// K3 uses FIXED signed windows (WA bits for h, WB bits for S) in one joint double-and-add over
// bit positions 252..0: every lane adds at the same positions, so a wave never diverges (with a
// sliding window some lane of 64 is nonzero at nearly every position, so SIMT would execute an
// addition everywhere).  The B table (2^(WB-1)+1 affine entries) lives in LDS; the -A table
// entry is streamed from HBM/L2 one field element at a time inside the addition, so at most
// 9 VGPRs of it are ever live.
//
// That windowed ladder is the path for per-signature keys.  Keys loaded into a key table (and B)
// instead get fixed-base comb tables (ed25519_comb_table_kernel, below) and the comb ladders: the
// quad ladder (4 lanes per signature, ed25519_comb_ladder_kernel) below 32K signatures and the
// pair ladder (2 lanes per signature, ed25519_comb2_ladder_kernel) from 32K; hash, decode and
// finish stay one signature per lane.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ge25519.h"
#include "sc25519.h"
#include "sha512.h"
#include "ed25519_verify.h"

#define CACHED_WORDS 36  // YpX | YmX | Z | T2d, 9 limbs each
#define NIELS_WORDS 28   // YpX | YmX | T2d (+1 pad)

template <int WA, int WB>
struct VerifyShape {
  static constexpr int NA = (253 + WA) / WA;      // windows for h (< L < 2^253)
  static constexpr int NB = (253 + WB) / WB;      // windows for S (< L)
  static constexpr int TA = (1 << (WA - 1)) + 1;  // -A table entries (0 = identity)
  static constexpr int TB = (1 << (WB - 1)) + 1;  // B table entries
  static constexpr int TOP = ((NA - 1) * WA > (NB - 1) * WB) ? (NA - 1) * WA : (NB - 1) * WB;
};
using Shape = VerifyShape<CBFT_WA, CBFT_WB>;

// ---------------------------------------------------------------------------------------
// small memory helpers
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void load_words8(uint32_t* w, const uint8_t* p) {
  const uint4* p4 = reinterpret_cast<const uint4*>(p);
  uint4 a = p4[0], b = p4[1];
  w[0] = a.x;
  w[1] = a.y;
  w[2] = a.z;
  w[3] = a.w;
  w[4] = b.x;
  w[5] = b.y;
  w[6] = b.z;
  w[7] = b.w;
}

__device__ __forceinline__ void fe_load(fe& r, const uint32_t* p) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) r.v[i] = p[i];
}
__device__ __forceinline__ void fe_store(uint32_t* p, const fe& a) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) p[i] = a.v[i];
}
// SoA: element w of item i at base[w * n + i]
__device__ __forceinline__ void fe_load_soa(fe& r, const uint32_t* base, size_t n, size_t i) {
#pragma unroll
  for (int k = 0; k < FE_LIMBS; k++) r.v[k] = base[k * n + i];
}
__device__ __forceinline__ void fe_store_soa(uint32_t* base, size_t n, size_t i, const fe& a) {
#pragma unroll
  for (int k = 0; k < FE_LIMBS; k++) base[k * n + i] = a.v[k];
}

// p + q where q is read from memory (cached layout, or niels layout when NIELS) and negated
// when neg: -(x,y) swaps Y+X <-> Y-X and negates T2d, and negating C = T2d*T1 swaps the
// outputs Z' = 2D + C and T' = 2D - C.  Each field element of q is loaded right before use.
template <bool NIELS>
__device__ __forceinline__ void ge_add_mem(ge_p1p1& r, const ge_p3& p, const uint32_t* q, bool neg) {
  fe A, B, C, D, t, e;
  fe_add(t, p.Y, p.X);
  fe_load(e, q + (neg ? 9 : 0));
  fe_mul(A, t, e);
  fe_sub(t, p.Y, p.X);
  fe_load(e, q + (neg ? 0 : 9));
  fe_mul(B, t, e);
  fe_load(e, q + (NIELS ? 18 : 27));
  fe_mul(C, e, p.T);
  if (NIELS) {
    fe_copy(D, p.Z);
  } else {
    fe_load(e, q + 18);
    fe_mul(D, p.Z, e);
  }
  fe_add(D, D, D);
  fe_sub(r.X, A, B);
  fe_add(r.Y, A, B);
  fe_add(t, D, C);
  fe_carry(t);
  fe_sub(e, D, C);
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) {
    r.Z.v[i] = neg ? e.v[i] : t.v[i];
    r.T.v[i] = neg ? t.v[i] : e.v[i];
  }
}

__device__ __forceinline__ void store_cached(uint32_t* dst, const ge_cached& c) {
  fe_store(dst, c.YpX);
  fe_store(dst + 9, c.YmX);
  fe_store(dst + 18, c.Z);
  fe_store(dst + 27, c.T2d);
}

// ---------------------------------------------------------------------------------------
// K0: base-point table, entry j = j*B as (y+x, y-x, 2dxy), j = 0..TB-1.  One lane, once per
// context (65 inversions; cost irrelevant).
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) ed25519_base_table_kernel(uint32_t* tbl, int nentries) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t bw[8];  // B = (x, 4/5), x even: 0x58 0x66 ... 0x66
  bw[0] = 0x66666658u;
  for (int i = 1; i < 8; i++) bw[i] = 0x66666666u;
  ge_p3 Bp, Q;
  ge_frombytes(Bp, bw);
  ge_cached cB;
  ge_p3_to_cached(cB, Bp);
  ge_p3_0(Q);
  fe d2;
  fe_load_const(d2, kFeD2);
  for (int j = 0; j < nentries; j++) {
    fe zi, x, y, xy, ypx, ymx, t2d;
    fe_invert(zi, Q.Z);
    fe_mul(x, Q.X, zi);
    fe_mul(y, Q.Y, zi);
    fe_mul(xy, x, y);
    fe_add(ypx, y, x);
    fe_carry(ypx);
    fe_sub(ymx, y, x);
    fe_mul(t2d, xy, d2);
    uint32_t* e = tbl + (size_t)j * NIELS_WORDS;
    fe_store(e, ypx);
    fe_store(e + 9, ymx);
    fe_store(e + 18, t2d);
    e[27] = 0;
    ge_p1p1 t;
    ge_add(t, Q, cB, false);
    ge_p1p1_to_p3(Q, t);
  }
}

// ---------------------------------------------------------------------------------------
// K1: h = SHA-512(R || A || M) mod L, S < L check
// ---------------------------------------------------------------------------------------

// NW big-endian 64-bit words of (M || 0x80 || 0 ...) starting at M-relative offset base, in two
// steps so a caller can issue the loads of the next window before compressing the current one:
// fetch_msg_dwords loads the 2 NW + 1 dwords, assemble_msg_words aligns, masks and marks them.
// Only dwords that overlap [m, m+len) are loaded (an aligned dword holding >= 1 message byte
// never faults), so callers need no padding after the blob.
//
// Branch-free: dword k is read from index min(k, kmax) (kmax = last dword holding a byte of
// M), or from `safe` (any readable dword) when no dword of this window holds one; bytes at or
// past len are then masked off arithmetically, so a wave never splits on message length.
template <int NW>
__device__ __forceinline__ void fetch_msg_dwords(uint32_t* d, const uint8_t* m, uint32_t len, uint32_t base,
                                                 const uint32_t* safe) {
  const uintptr_t a = (uintptr_t)(m + base);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  const int kmax = ((int)len - 1 - (int)base + (int)sh) >> 2;  // < 0: window is past M
#pragma unroll
  for (int k = 0; k < 2 * NW + 1; k++) {
    const uint32_t* src = kmax >= 0 ? q + (k < kmax ? k : kmax) : safe;
    d[k] = *src;
  }
}
template <int NW>
__device__ __forceinline__ void assemble_msg_words(uint64_t* W, const uint32_t* d, const uint8_t* m, uint32_t len,
                                                   uint32_t base) {
  const uint32_t sh = (uint32_t)((uintptr_t)(m + base) & 3);
#pragma unroll
  for (int j = 0; j < NW; j++) {
    const uint32_t lo = __builtin_amdgcn_alignbyte(d[2 * j + 1], d[2 * j], sh);
    const uint32_t hi = __builtin_amdgcn_alignbyte(d[2 * j + 2], d[2 * j + 1], sh);
    uint64_t w = ((uint64_t)bswap32(lo) << 32) | bswap32(hi);
    // rem = bytes of M left at this word: keep the first min(rem, 8) (big-endian, high bytes
    // first), then the 0x80 marker right after M's last byte
    const int rem = (int)len - (int)(base + 8u * j);
    const int keep = rem < 0 ? 0 : (rem > 8 ? 8 : rem);
    const uint64_t mask = keep == 0 ? 0ull : (~0ull << (64 - 8 * keep));
    const uint64_t mark = (rem >= 0 && rem < 8) ? (0x80ull << (56 - 8 * rem)) : 0ull;
    W[j] = (w & mask) | mark;
  }
}

// Key-table unit of signature i.  An index outside the table reads unit 0 instead (never past
// the table) and K1 clears the signature's flag, so its verdict is false.
__device__ __forceinline__ uint32_t batch_unit(const Ed25519Batch& b, size_t i) {
  if (!b.key_idx) return (uint32_t)i;
  const uint32_t k = b.key_idx[i];
  return k < b.nkeys ? k : 0u;
}

// A decoded (the key's or the signature's own)
__device__ __forceinline__ bool unit_aok(const Ed25519Batch& b, const uint8_t* aok, uint32_t unit) {
  return b.key_idx ? b.keys.aok(unit) : aok[unit] != 0;
}

// h = SHA-512(R||A||M) mod L of signature i (hw, 8 LE words) and its flag (S < L, key index in
// range, length supported): K1's per-signature work, also run by the fused small-batch kernel.
__device__ __forceinline__ void ed25519_hash_sig(const Ed25519Batch& b, size_t i, uint32_t* hw, bool& flag) {
  const uint32_t key = batch_unit(b, i);
  const bool key_ok = !b.key_idx || b.key_idx[i] < b.nkeys;
  uint32_t Aw[8], Rw[8], Sw[8];
  load_words8(Aw, b.key_idx ? b.keys.pk(key) : b.pk + (size_t)key * 32);
  load_words8(Rw, b.sig + i * 64);
  load_words8(Sw, b.sig + i * 64 + 32);
  const uint8_t* m = b.msg_off ? b.msg + b.msg_off[i] : b.msg + i * (size_t)b.fixed_len;
  uint32_t len = b.msg_off ? b.msg_len[i] : b.fixed_len;
  const bool len_ok = len <= CBFT_MAX_MSG_LEN;
  if (!len_ok) len = 0;
  const uint32_t* safe = reinterpret_cast<const uint32_t*>(b.sig + i * 64);  // readable dword

  uint64_t H[8], W[16];
  sha512_init(H);
  const uint32_t total = 64u + len;
  const uint32_t nblocks = (total + 17u + 127u) / 128u;
  uint32_t d[33];  // the message dwords of the next block, loaded while the current one compresses
  fetch_msg_dwords<8>(d, m, len, 0u, safe);
  for (uint32_t blk = 0; blk < nblocks; blk++) {
    if (blk == 0) {  // R || A || M[0..63]
#pragma unroll
      for (int j = 0; j < 4; j++) W[j] = ((uint64_t)bswap32(Rw[2 * j]) << 32) | bswap32(Rw[2 * j + 1]);
#pragma unroll
      for (int j = 0; j < 4; j++) W[4 + j] = ((uint64_t)bswap32(Aw[2 * j]) << 32) | bswap32(Aw[2 * j + 1]);
      assemble_msg_words<8>(W + 8, d, m, len, 0u);
    } else {
      assemble_msg_words<16>(W, d, m, len, 128u * blk - 64u);
    }
    if (blk + 1 < nblocks) fetch_msg_dwords<16>(d, m, len, 128u * blk + 64u, safe);  // the next block's words
    if (blk == nblocks - 1) {
      W[14] = 0;
      W[15] = (uint64_t)total << 3;
    }
    sha512_compress(H, W);
  }
  uint32_t dig[16];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    dig[2 * k] = bswap32((uint32_t)(H[k] >> 32));
    dig[2 * k + 1] = bswap32((uint32_t)H[k]);
  }
  sc_reduce512(hw, dig);
  flag = sc_is_canonical(Sw) && key_ok && len_ok;
}

// ed25519_hash_sig split over two waves (the fused three-wave kernel): sig_sha_blocks is the
// block count of signature i's R || A || M; ed25519_sched_sig (the [S]B wave, lane q of the
// signature's quad) writes K[t] + W[t] of blocks 1 + q, 5 + q, ... into kw[block][0..80) in LDS
// while ed25519_hash_sig_kw (wave 0) compresses block 0 itself, then (after the caller's barrier,
// `sync`) runs only the rounds of blocks 1, 2, ...  Same digest, same flag.
__device__ __forceinline__ uint32_t sig_sha_blocks(const Ed25519Batch& b, size_t i) {
  uint32_t len = b.msg_off ? b.msg_len[i] : b.fixed_len;
  if (len > CBFT_MAX_MSG_LEN) len = 0;
  return (64u + len + 17u + 127u) / 128u;
}
#define KW_STRIDE 81  // 80 words + 1: the 8 signatures' rows fall on different LDS banks
__device__ __forceinline__ void ed25519_sched_sig(const Ed25519Batch& b, size_t i, uint32_t q, uint64_t* kw) {
  const uint32_t key = batch_unit(b, i);
  uint32_t Aw[8], Rw[8];
  load_words8(Aw, b.key_idx ? b.keys.pk(key) : b.pk + (size_t)key * 32);
  load_words8(Rw, b.sig + i * 64);
  const uint8_t* m = b.msg_off ? b.msg + b.msg_off[i] : b.msg + i * (size_t)b.fixed_len;
  uint32_t len = b.msg_off ? b.msg_len[i] : b.fixed_len;
  if (len > CBFT_MAX_MSG_LEN) len = 0;
  const uint32_t* safe = reinterpret_cast<const uint32_t*>(b.sig + i * 64);
  const uint32_t total = 64u + len;
  const uint32_t nblocks = (total + 17u + 127u) / 128u;
  for (uint32_t blk = 1 + q; blk < nblocks; blk += 4) {
    uint64_t W[16];
    uint32_t d[33];
    if (blk == 0) {
#pragma unroll
      for (int j = 0; j < 4; j++) W[j] = ((uint64_t)bswap32(Rw[2 * j]) << 32) | bswap32(Rw[2 * j + 1]);
#pragma unroll
      for (int j = 0; j < 4; j++) W[4 + j] = ((uint64_t)bswap32(Aw[2 * j]) << 32) | bswap32(Aw[2 * j + 1]);
      fetch_msg_dwords<8>(d, m, len, 0u, safe);
      assemble_msg_words<8>(W + 8, d, m, len, 0u);
    } else {
      fetch_msg_dwords<16>(d, m, len, 128u * blk - 64u, safe);
      assemble_msg_words<16>(W, d, m, len, 128u * blk - 64u);
    }
    if (blk == nblocks - 1) {
      W[14] = 0;
      W[15] = (uint64_t)total << 3;
    }
    sha512_schedule_kw(kw + blk * KW_STRIDE, W);
  }
}
template <class Sync>
__device__ __forceinline__ void ed25519_hash_sig_kw(const Ed25519Batch& b, size_t i, const uint64_t* kw, uint32_t* hw,
                                                    bool& flag, Sync sync) {
  const uint32_t key = batch_unit(b, i);
  const bool key_ok = !b.key_idx || b.key_idx[i] < b.nkeys;
  uint32_t Aw[8], Rw[8], Sw[8];
  load_words8(Aw, b.key_idx ? b.keys.pk(key) : b.pk + (size_t)key * 32);
  load_words8(Rw, b.sig + i * 64);
  load_words8(Sw, b.sig + i * 64 + 32);
  const uint8_t* m = b.msg_off ? b.msg + b.msg_off[i] : b.msg + i * (size_t)b.fixed_len;
  uint32_t len = b.msg_off ? b.msg_len[i] : b.fixed_len;
  const bool len_ok = len <= CBFT_MAX_MSG_LEN;
  if (!len_ok) len = 0;
  const uint32_t* safe = reinterpret_cast<const uint32_t*>(b.sig + i * 64);
  const uint32_t total = 64u + len;
  const uint32_t nblocks = (total + 17u + 127u) / 128u;
  uint64_t H[8], W[16];
  sha512_init(H);
  {  // block 0: R || A || M[0..63]
    uint32_t d[17];
#pragma unroll
    for (int j = 0; j < 4; j++) W[j] = ((uint64_t)bswap32(Rw[2 * j]) << 32) | bswap32(Rw[2 * j + 1]);
#pragma unroll
    for (int j = 0; j < 4; j++) W[4 + j] = ((uint64_t)bswap32(Aw[2 * j]) << 32) | bswap32(Aw[2 * j + 1]);
    fetch_msg_dwords<8>(d, m, len, 0u, safe);
    assemble_msg_words<8>(W + 8, d, m, len, 0u);
    if (nblocks == 1) {
      W[14] = 0;
      W[15] = (uint64_t)total << 3;
    }
    sha512_compress(H, W);
  }
  sync();  // the other blocks' schedules are in kw
  for (uint32_t blk = 1; blk < nblocks; blk++) sha512_rounds_kw(H, kw + blk * KW_STRIDE);
  uint32_t dig[16];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    dig[2 * k] = bswap32((uint32_t)(H[k] >> 32));
    dig[2 * k + 1] = bswap32((uint32_t)H[k]);
  }
  sc_reduce512(hw, dig);
  flag = sc_is_canonical(Sw) && key_ok && len_ok;
}

// SHA-512 blocks of signature i's R || A || M (what ed25519_hash_sig runs), as a sort bucket
__device__ __forceinline__ uint32_t hash_bucket(const Ed25519Batch& b, size_t i) {
  uint32_t len = b.msg_len[i];
  if (len > CBFT_MAX_MSG_LEN) len = 0;
  const uint32_t nb = (64u + len + 17u + 127u) / 128u;
  return nb < CBFT_SHA_BUCKETS - 1 ? nb : CBFT_SHA_BUCKETS - 1;
}

// Counting sort of a variable-length batch by SHA-512 block count, in three launches:
// (1) per-bucket counts (LDS histogram per block, one global atomic per non-empty bucket);
// (2) one block: exclusive scan of the counts into cursors (and counts reset for the next batch),
//     and a flag word: 1 when every signature has the same block count (fixed-size messages),
//     in which case (3) does nothing and K1 keeps the identity order (and its locality);
// (3) every signature takes a slot of its bucket (LDS ranks per block, one global atomicAdd per
//     non-empty bucket per block) and writes its index there.  Order inside a bucket is arbitrary:
//     K1 writes each signature's digest to its own index, so verdicts do not depend on it.
static_assert(CBFT_SHA_BUCKETS == 256, "the bucket kernels run one thread per bucket in 256-thread blocks");
__global__ void __launch_bounds__(256) ed25519_bucket_count_kernel(const Ed25519Batch b, uint32_t* counts) {
  __shared__ uint32_t hist[CBFT_SHA_BUCKETS];
  hist[threadIdx.x] = 0;
  __syncthreads();
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < b.n) atomicAdd(&hist[hash_bucket(b, i)], 1u);
  __syncthreads();
  if (hist[threadIdx.x]) atomicAdd(&counts[threadIdx.x], hist[threadIdx.x]);
}

__global__ void __launch_bounds__(256) ed25519_bucket_scan_kernel(uint32_t* counts, uint32_t* cursors,
                                                                  uint32_t long_groups) {
  __shared__ uint32_t v[CBFT_SHA_BUCKETS];
  const uint32_t t = threadIdx.x;
  v[t] = counts[t];
  __syncthreads();
  for (uint32_t d = 1; d < CBFT_SHA_BUCKETS; d <<= 1) {  // inclusive Hillis-Steele scan
    const uint32_t x = t >= d ? v[t - d] : 0u;
    __syncthreads();
    v[t] += x;
    __syncthreads();
  }
  const uint32_t c = counts[t];
  cursors[t] = v[t] - c;
  counts[t] = 0;  // ready for the next batch's counts
  if (t == 0) cursors[CBFT_SHA_BUCKETS] = 0;
  // n_short: signatures below CBFT_SHA_LONG_BLOCKS blocks (the long ones follow them in the order;
  // with one bucket for all, 0 or n, which the identity order also satisfies), but at most
  // long_groups (CBFT_SHA_LONG_GROUPS by default) x 64 positions for the long kernel: its blocks (83 KB of LDS each) must
  // all be resident at once, or its last groups would run a second full chain after the others
  if (t == CBFT_SHA_LONG_BLOCKS) {
    const uint32_t n = v[CBFT_SHA_BUCKETS - 1], cap = 64u * long_groups;
    const uint32_t ns = v[t] - c;
    cursors[CBFT_SHA_BUCKETS + 1] = n - ns > cap ? n - cap : ns;
  }
  __syncthreads();
  if (c != 0 && c == v[CBFT_SHA_BUCKETS - 1]) cursors[CBFT_SHA_BUCKETS] = 1;  // one bucket holds all
}

__global__ void __launch_bounds__(256) ed25519_bucket_scatter_kernel(const Ed25519Batch b, uint32_t* cursors,
                                                                     uint32_t* perm) {
  __shared__ uint32_t hist[CBFT_SHA_BUCKETS], base[CBFT_SHA_BUCKETS];
  if (cursors[CBFT_SHA_BUCKETS]) return;  // uniform: K1 keeps the identity order
  hist[threadIdx.x] = 0;
  __syncthreads();
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t k = 0, rank = 0;
  if (i < b.n) {
    k = hash_bucket(b, i);
    rank = atomicAdd(&hist[k], 1u);
  }
  __syncthreads();
  if (hist[threadIdx.x]) base[threadIdx.x] = atomicAdd(&cursors[threadIdx.x], hist[threadIdx.x]);
  __syncthreads();
  if (i < b.n) perm[base[k] + rank] = (uint32_t)i;
}

// perm: the block-count order (nullable); uniform: its flag word (perm unused when set);
// nshort (nullable): positions from *nshort on are ed25519_hash_long_kernel's.
__global__ void __launch_bounds__(CBFT_VERIFY_BLOCK) ed25519_hash_kernel(const Ed25519Batch b, const uint32_t* perm,
                                                                          const uint32_t* uniform, const uint32_t* nshort,
                                                                          uint32_t* h_soa, uint8_t* flags) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= b.n || (nshort && g >= *nshort)) return;
  const size_t i = perm && !*uniform ? (size_t)perm[g] : g;
  uint32_t hw[8];
  bool flag;
  ed25519_hash_sig(b, i, hw, flag);
#pragma unroll
  for (int k = 0; k < 8; k++) h_soa[k * b.n + i] = hw[k];
  flags[i] = flag ? 1 : 0;
}

// K1 for the sorted order's tail (messages of >= CBFT_SHA_LONG_BLOCKS blocks): 64 signatures per
// block of two waves.  Wave 1 expands block j's message schedule (K[t] + W[t], sha512_schedule_kw)
// into one of two LDS slots while wave 0 runs block j - 1's rounds from the other
// (sha512_rounds_kw): each signature's serial chain loses the schedule, ~a third of a
// compression, which is what bounds config #3's hash stage (a 4,096-B message is 33 blocks on one
// lane).  Runs on a second stream beside ed25519_hash_kernel (which skips these positions); one
// barrier per block, the same count in both waves (the group's most blocks).
#define HASH_LONG_BLOCK 128
__global__ void __launch_bounds__(HASH_LONG_BLOCK) ed25519_hash_long_kernel(const Ed25519Batch b, const uint32_t* perm,
                                                                            const uint32_t* uniform,
                                                                            const uint32_t* nshort, uint32_t* h_soa,
                                                                            uint8_t* flags) {
  __shared__ uint64_t kwl[2][64 * KW_STRIDE];
  const size_t g0 = (size_t)*nshort + (size_t)blockIdx.x * 64;
  if (g0 >= b.n) return;  // the whole block
  const uint32_t ln = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const bool ident = *uniform != 0;
  const size_t g = g0 + ln;
  const bool live = g < b.n;
  const size_t i = ident ? (live ? g : g0) : (size_t)perm[live ? g : g0];
  const uint32_t nb = live ? sig_sha_blocks(b, i) : 0u;
  uint32_t nbmax = nb;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) nbmax = max(nbmax, (uint32_t)__shfl_xor((int)nbmax, d, 64));
  uint64_t* slot0 = &kwl[0][ln * KW_STRIDE];
  uint64_t* slot1 = &kwl[1][ln * KW_STRIDE];
  if (wave == 1) {  // schedules
    const uint32_t key = batch_unit(b, i);
    uint32_t Aw[8], Rw[8];
    load_words8(Aw, b.key_idx ? b.keys.pk(key) : b.pk + (size_t)key * 32);
    load_words8(Rw, b.sig + i * 64);
    const uint8_t* m = b.msg_off ? b.msg + b.msg_off[i] : b.msg + i * (size_t)b.fixed_len;
    uint32_t len = b.msg_off ? b.msg_len[i] : b.fixed_len;
    if (len > CBFT_MAX_MSG_LEN) len = 0;
    const uint32_t* safe = reinterpret_cast<const uint32_t*>(b.sig + i * 64);
    const uint32_t total = 64u + len;
    uint32_t d[33];
    fetch_msg_dwords<8>(d, m, len, 0u, safe);
    for (uint32_t blk = 0; blk < nbmax; blk++) {
      if (blk < nb) {
        uint64_t W[16];
        if (blk == 0) {
#pragma unroll
          for (int j = 0; j < 4; j++) W[j] = ((uint64_t)bswap32(Rw[2 * j]) << 32) | bswap32(Rw[2 * j + 1]);
#pragma unroll
          for (int j = 0; j < 4; j++) W[4 + j] = ((uint64_t)bswap32(Aw[2 * j]) << 32) | bswap32(Aw[2 * j + 1]);
          assemble_msg_words<8>(W + 8, d, m, len, 0u);
        } else {
          assemble_msg_words<16>(W, d, m, len, 128u * blk - 64u);
        }
        if (blk + 1 < nb) fetch_msg_dwords<16>(d, m, len, 128u * blk + 64u, safe);  // next block's words
        if (blk == nb - 1) {
          W[14] = 0;
          W[15] = (uint64_t)total << 3;
        }
        sha512_schedule_kw((blk & 1) ? slot1 : slot0, W);
      }
      __syncthreads();  // block blk's schedules are in LDS; block blk - 1's rounds are done
    }
    return;
  }
  uint64_t H[8];  // wave 0: rounds
  sha512_init(H);
  for (uint32_t blk = 0; blk < nbmax; blk++) {
    __syncthreads();
    if (blk < nb) sha512_rounds_kw(H, (blk & 1) ? slot1 : slot0);
  }
  if (!live) return;
  uint32_t dig[16], hw[8], Sw[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    dig[2 * k] = bswap32((uint32_t)(H[k] >> 32));
    dig[2 * k + 1] = bswap32((uint32_t)H[k]);
  }
  sc_reduce512(hw, dig);
  load_words8(Sw, b.sig + i * 64 + 32);
  const uint32_t len = b.msg_off ? b.msg_len[i] : b.fixed_len;
  const bool key_ok = !b.key_idx || b.key_idx[i] < b.nkeys;
  const bool flag = sc_is_canonical(Sw) && key_ok && len <= CBFT_MAX_MSG_LEN;
#pragma unroll
  for (int k = 0; k < 8; k++) h_soa[k * b.n + i] = hw[k];
  flags[i] = flag ? 1 : 0;
}

// ---------------------------------------------------------------------------------------
// K2: decode A (OpenSSL semantics), table of j*(-A) in cached form
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(CBFT_VERIFY_BLOCK) ed25519_prep_kernel(const uint8_t* pk, size_t nunits,
                                                                          uint32_t* tbl, uint8_t* aok) {
  const size_t u = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nunits) return;
  uint32_t Aw[8];
  load_words8(Aw, pk + u * 32);
  ge_p3 Q;
  aok[u] = ge_frombytes(Q, Aw) ? 1 : 0;
  fe_neg(Q.X, Q.X);
  fe_neg(Q.T, Q.T);
  uint32_t* slab = tbl + u * (size_t)(Shape::TA * CACHED_WORDS);
  ge_cached c, c1;
  ge_cached_0(c);
  store_cached(slab, c);
  ge_p3_to_cached(c1, Q);
  store_cached(slab + CACHED_WORDS, c1);
#pragma nounroll
  for (int j = 2; j < Shape::TA; j++) {
    ge_p1p1 t;
    ge_add(t, Q, c1, false);
    ge_p1p1_to_p3(Q, t);
    ge_p3_to_cached(c, Q);
    store_cached(slab + j * CACHED_WORDS, c);
  }
}

// ---------------------------------------------------------------------------------------
// K3: (X:Y:Z) = [h](-A) + [S]B
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(CBFT_VERIFY_BLOCK, CBFT_LADDER_MIN_WAVES)
    ed25519_ladder_kernel(const Ed25519Batch b, const uint32_t* h_soa, const uint32_t* tbl,
                          const uint32_t* base_table, uint32_t* xyz_soa) {
  __shared__ uint32_t sB[Shape::TB * NIELS_WORDS];
  for (int k = threadIdx.x; k < Shape::TB * NIELS_WORDS; k += blockDim.x) sB[k] = base_table[k];
  __syncthreads();
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b.n) return;

  const uint32_t unit = batch_unit(b, i);
  const uint32_t* slab = tbl + (size_t)unit * (Shape::TA * CACHED_WORDS);
  uint32_t kA[9], kB[9];
  {
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = h_soa[k * b.n + i];
    sc_recode_prepare<CBFT_WA, Shape::NA>(kA, w);
    load_words8(w, b.sig + i * 64 + 32);
    sc_recode_prepare<CBFT_WB, Shape::NB>(kB, w);
  }
  ge_p3 P;
  ge_p3_0(P);
#pragma nounroll
  for (int p = Shape::TOP; p >= 0; --p) {
    const bool addA = (p % CBFT_WA == 0) && (p / CBFT_WA < Shape::NA);
    const bool addB = (p % CBFT_WB == 0) && (p / CBFT_WB < Shape::NB);
    // op 0 = double, op 1 = add the h digit's -A multiple, op 2 = add the S digit's B multiple
#pragma nounroll
    for (int op = 0; op < 3; op++) {
      if ((op == 1 && !addA) || (op == 2 && !addB)) continue;
      ge_p1p1 t;
      if (op == 0) {
        ge_dbl(t, P.X, P.Y, P.Z);
      } else if (op == 1) {
        const int d = sc_recode_pop<CBFT_WA>(kA);
        ge_add_mem<false>(t, P, slab + (d < 0 ? -d : d) * CACHED_WORDS, d < 0);
      } else {
        const int d = sc_recode_pop<CBFT_WB>(kB);
        ge_add_mem<true>(t, P, sB + (d < 0 ? -d : d) * NIELS_WORDS, d < 0);
      }
      // the next op needs T only if it is an addition
      const bool needT = (op == 0 && (addA || addB)) || (op == 1 && addB);
      if (needT) fe_mul(P.T, t.X, t.Y);
      fe_mul(P.X, t.X, t.T);
      fe_mul(P.Y, t.Y, t.Z);
      fe_mul(P.Z, t.Z, t.T);
    }
  }
  fe_store_soa(xyz_soa, b.n, i, P.X);
  fe_store_soa(xyz_soa + 9 * b.n, b.n, i, P.Y);
  fe_store_soa(xyz_soa + 18 * b.n, b.n, i, P.Z);
}

// ---------------------------------------------------------------------------------------
// K4: encode R' = (X : Y : Z) and compare it with R; verdict ballot per wave.
//
// One field inversion per block of 64 lanes x K signatures (Montgomery's trick; R' is public, so
// the inversion is the variable-time safegcd), on TWO waves so that one product follows it.  Lane t
// of each wave sees the same K signatures (i = base + j 64 + t) and forms the same leaf
// L_t = prod_j Z_j (signatures already rejected -- S >= L, A not decodable -- and Z = 0 enter as
// 1, so they cannot disturb their neighbours' inverses).
//   wave 0  root = prod_t L_t by a 6-level butterfly (__shfl_xor), inverted by the whole wave
//           (fe_invert_var<true>: safegcd30.h sg_inv30_var_wave, the divsteps on the scalar unit,
//           the limb updates lane-parallel with DPP neighbour exchanges; ~18 us of the kernel, the
//           scalar-unit chain it replaced 31 us), published in LDS;
//   wave 1  meanwhile the cofactor of every signature: E_t = prod_{s != t} L_s from inclusive
//           prefix and suffix scans over the lanes (6 levels, both scans in one fe_mul2), times
//           the lane's other Z (K = 2), times X and Y: X' = X root / Z, Y' = Y root / Z, into LDS;
//   tail    after one barrier wave j finishes slot j: x = X' root^-1, y = Y' root^-1 (one fe_mul2),
//           encode, compare with R (requested at the start), ballot.
// The critical path is the leaves, 6 products, the inversion and one product pair (the one-wave
// product tree of round 5 put 6 product pairs and the slots one after another behind the
// inversion): 35.4-35.9 us against 38.3 (same box, ladder_probe events, profiles/ab/r06/).  K = 2
// from 16K signatures (512 blocks at 64K: the finish co-runs with the other streams' ladders,
// whose 1,024 blocks of 36 KB fill a 64K batch's LDS, and a block's 9.2 KB fits beside them), K = 1
// below.
// ---------------------------------------------------------------------------------------
#define FINISH_BLOCK 128
template <int K>
__global__ void __launch_bounds__(FINISH_BLOCK) ed25519_finish_kernel(const Ed25519Batch b, const uint32_t* xyz_soa,
                                                                      const uint8_t* flags, const uint8_t* aok,
                                                                      uint64_t* verdict_words) {
  static_assert(K == 1 || K == 2, "one or two signatures per lane");
  constexpr uint32_t T = 64;
  __shared__ uint32_t xy[K][2][FE_LIMBS][T];  // X' | Y' per slot, [limb][lane]
  __shared__ uint32_t rinv[FE_LIMBS];         // root^-1
  const uint32_t t = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const size_t base = (size_t)blockIdx.x * T * K;
  fe Z[K];
  uint32_t okmask = 0;
#pragma unroll
  for (int j = 0; j < K; j++) {
    const size_t i = base + (size_t)j * T + t;
    fe_1(Z[j]);
    bool ok = false;
    if (i < b.n) {
      fe_load_soa(Z[j], xyz_soa + 18 * b.n, b.n, i);
      ok = flags[i] && unit_aok(b, aok, batch_unit(b, i)) && !fe_iszero(Z[j]);
      if (!ok) fe_1(Z[j]);
    }
    okmask |= (ok ? 1u : 0u) << j;
  }
  const uint32_t jt = wave;  // the slot this wave finishes (wave < K)
  const size_t it = base + (size_t)jt * T + t;
  uint32_t Rw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (jt < (uint32_t)K && it < b.n) load_words8(Rw, b.sig + it * 64);  // needed after the barrier
  fe leaf;
  if (K == 2)
    fe_mul(leaf, Z[0], Z[K - 1]);
  else
    fe_copy(leaf, Z[0]);
  if (wave == 0) {
    fe r = leaf;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      fe o;
#pragma unroll
      for (int k = 0; k < FE_LIMBS; k++) o.v[k] = (uint32_t)__shfl_xor((int)r.v[k], d);
      fe_mul(r, r, o);
    }
    fe_invert_var<true>(r, r);  // every leaf is non-zero, so is the root
    if (t == 0) {
#pragma unroll
      for (int k = 0; k < FE_LIMBS; k++) rinv[k] = r.v[k];
    }
  } else {
    fe P = leaf, S = leaf;  // inclusive prefix / suffix products over the lanes
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      fe p, q;
#pragma unroll
      for (int k = 0; k < FE_LIMBS; k++) {
        p.v[k] = (uint32_t)__shfl_up((int)P.v[k], d);
        q.v[k] = (uint32_t)__shfl_down((int)S.v[k], d);
      }
      if (t < (uint32_t)d) fe_1(p);
      if (t + d >= 64u) fe_1(q);
      fe_mul2_oneasm(P, P, p, S, S, q);
    }
    fe pe, se, E;  // P_(t-1), S_(t+1): E_t = the product of every other lane's leaf
#pragma unroll
    for (int k = 0; k < FE_LIMBS; k++) {
      pe.v[k] = (uint32_t)__shfl_up((int)P.v[k], 1);
      se.v[k] = (uint32_t)__shfl_down((int)S.v[k], 1);
    }
    if (t == 0) fe_1(pe);
    if (t == 63) fe_1(se);
    fe_mul(E, pe, se);
    fe c[K];  // 1 / Z_j * root: E times the lane's other signature's Z
    if (K == 2)
      fe_mul2_oneasm(c[0], E, Z[K - 1], c[K - 1], E, Z[0]);
    else
      fe_copy(c[0], E);
#pragma unroll
    for (int j = 0; j < K; j++) {
      if (!((okmask >> j) & 1u)) continue;
      const size_t i = base + (size_t)j * T + t;
      fe X, Y;
      fe_load_soa(X, xyz_soa, b.n, i);
      fe_load_soa(Y, xyz_soa + 9 * b.n, b.n, i);
      fe_mul2_oneasm(X, X, c[j], Y, Y, c[j]);
#pragma unroll
      for (int k = 0; k < FE_LIMBS; k++) {
        xy[j][0][k][t] = X.v[k];
        xy[j][1][k][t] = Y.v[k];
      }
    }
  }
  __syncthreads();
  if (jt >= (uint32_t)K) return;
  bool verdict = false;
  if ((okmask >> jt) & 1u) {
    fe inv, X, Y, x, y;
#pragma unroll
    for (int k = 0; k < FE_LIMBS; k++) {
      inv.v[k] = rinv[k];
      X.v[k] = xy[jt][0][k][t];
      Y.v[k] = xy[jt][1][k][t];
    }
    fe_mul2_oneasm(x, X, inv, y, Y, inv);
    uint32_t Rp[8];
    fe_to_words(Rp, y);
    Rp[7] ^= fe_isnegative(x) << 31;
    uint32_t diff = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) diff |= Rp[k] ^ Rw[k];
    verdict = diff == 0;
  }
  const uint64_t ballot = __ballot(verdict);
  const size_t w0 = base + (size_t)jt * T;
  if (t == 0 && w0 < b.n) verdict_words[w0 >> 6] = ballot;
}

// ---------------------------------------------------------------------------------------
// Wide fixed-base combs, four lanes per signature (key-table mode).
//
// For a point P known before the signatures arrive (B, or a loaded key's -A) the table
//   C_P[j][e] = e * 2^(w j) * P,   j = 0..npos-1, e = 0..2^(w-1)   (affine niels, 128-B entries,
//   e = 0 = identity)
// turns [s]P into sum_j sign(d_j) C_P[j][|d_j|] with signed radix-2^w digits: s' = s + offset,
// offset = 2^(w-1) sum_{j < npos-1} 2^(w j); d_j = chunk_j(s') - 2^(w-1) below the top position,
// d_top = chunk_top(s') in [0, 2^(w-1)] (CombGeom in ed25519_verify.h; tests/test_comb_recode.py
// checks the recoding exhaustively at the range edges).  One mixed addition per position and no
// doublings: B's table is radix 2^22 (12 positions, 3.2 GB in HBM), a key's
// table radix 2^w_A (default 2^13 while the tables fit the budget: 20 positions, 10.5 MB per key,
// 43 GB for 4,096 keys -- HBM is 288 GB and keys are long-lived, SigManager.cpp:139-150), so a
// verify is 12 + 20 = 32 mixed additions (the radix-256 comb of the first round: 64).
//
// The additions are dealt to the 4 lanes of a quad in order (lane q takes additions
// q*nper .. q*nper+nper-1, the A positions first), then two DPP butterfly levels (quad_perm
// xor 1, xor 2) add the four partial sums: every lane of the quad ends with
// R' = [S]B + [h](-A).  4,096 waves at 64K signatures: 4 waves per SIMD.
// ---------------------------------------------------------------------------------------
#define COMB_STRIDE 32  // words per entry: one 128-B line (y+x | y-x | 2dxy, 9 limbs each, + pad)
#define COMB_CHUNK 128  // multiples built per table-build lane
#define COMB_TMP_WORDS_PER_LANE (COMB_CHUNK * CACHED_WORDS)
#define COMB_TABLE_BLOCK 64
#define COMB_MAX_STEPS 12  // additions per lane (nper) the ladder supports

// One lane per unit: decode (aok), negate, then along ONE doubling chain P_j = 2^(w j) P and
// S_j = 2^(w - 8) P_j (the stride of a build lane's multiples, on the way to P_(j+1)) for every
// position j, stored in the cached form (YpX | YmX | Z | T2d) to pos[unit][j][P_j, S_j].  The
// table lanes of a position start from these instead of each redoing its w j doublings.
#define COMB_POS_WORDS (2 * CACHED_WORDS)
__device__ __forceinline__ void cached_store(uint32_t* e, const ge_p3& P) {
  ge_cached cj;
  ge_p3_to_cached(cj, P);
  fe_store(e, cj.YpX);
  fe_store(e + 9, cj.YmX);
  fe_store(e + 18, cj.Z);
  fe_store(e + 27, cj.T2d);
}
__device__ __forceinline__ void cached_load(ge_cached& cj, const uint32_t* e) {
  fe_load(cj.YpX, e);
  fe_load(cj.YmX, e + 9);
  fe_load(cj.Z, e + 18);
  fe_load(cj.T2d, e + 27);
}

__global__ void __launch_bounds__(COMB_TABLE_BLOCK) ed25519_comb_pos_kernel(const uint8_t* pk, size_t nunits,
                                                                           int negate, CombGeom geo, uint32_t* pos,
                                                                           uint8_t* aok) {
  const size_t u = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nunits) return;
  uint32_t Aw[8];
  load_words8(Aw, pk + u * 32);
  ge_p3 P;
  const bool ok = ge_frombytes(P, Aw);
  if (aok) aok[u] = ok ? 1 : 0;
  if (negate) {
    fe_neg(P.X, P.X);
    fe_neg(P.T, P.T);
  }
  const int cb = geo.w - 8;  // build lanes per position = 2^cb
  uint32_t* o = pos + u * (size_t)geo.npos * COMB_POS_WORDS;
#pragma nounroll
  for (int j = 0; j < geo.npos; j++) {
    uint32_t* e = o + (size_t)j * COMB_POS_WORDS;
    cached_store(e, P);
#pragma nounroll
    for (int d = 0; d < geo.w; d++) {
      if (d == cb) cached_store(e + CACHED_WORDS, P);
      if (j + 1 == geo.npos && d == cb) break;
      ge_p1p1 r;
      ge_dbl(r, P.X, P.Y, P.Z);
      ge_p1p1_to_p3(P, r);
    }
  }
}

// One lane per (unit, position j, chunk c) builds the multiples e = c + 1 + 2^cb k, k = 0..127,
// of P_j (cb = w - 8: 2^cb lanes per position, stride S_j = 2^cb P_j from
// ed25519_comb_pos_kernel): projective points and prefix Z products into tmp (lane-interleaved,
// so every tmp access is one contiguous 256-B wave access), Montgomery batch inversion, affine
// niels entries (y+x | y-x | 2dxy, 128-B lines) staged through LDS and written by the whole wave
// in 16-B pieces: the lanes of a position hold consecutive entries, so each store instruction
// writes 1 KB runs.  The c = 0 lane also writes the identity entry 0.  Units are contiguous from
// tbl, or (key_chunks != nullptr) keys a0 + u of a chunked key table, so one launch spans key
// chunks.
__global__ void __launch_bounds__(COMB_TABLE_BLOCK) ed25519_comb_table_kernel(const uint32_t* pos, size_t nunits,
                                                                             CombGeom geo, uint32_t* tbl,
                                                                             void* const* key_chunks, uint32_t a0,
                                                                             uint32_t* tmp, size_t lane0,
                                                                             size_t nlanes) {
  static_assert(COMB_TABLE_BLOCK == 64, "one wave per block: the LDS staging is per wave");
  __shared__ uint4 ent[64][COMB_STRIDE / 4];
  __shared__ uint32_t* dst[64];
  const int ln = threadIdx.x;
  const size_t gl = (size_t)blockIdx.x * blockDim.x + ln;  // lane of this launch (tmp column)
  const size_t g = lane0 + gl;
  const int cb = geo.w - 8;
  const int chunks = 1 << cb;
  const size_t u = g / ((size_t)geo.npos * chunks);
  const int j = (int)((g / chunks) % geo.npos);
  const int c = (int)(g % chunks);
  const bool live = gl < nlanes && u < nunits;
  const size_t nl = nlanes;  // tmp row stride
  const size_t estride = (size_t)chunks * COMB_STRIDE;  // words between a lane's consecutive entries
  fe inv;
  if (live) {
    const size_t wpk = geo.words_per_unit();
    uint32_t* unit_tbl = tbl + u * wpk;
    if (key_chunks) {
      const uint32_t ka = a0 + (uint32_t)u;
      unit_tbl = static_cast<uint32_t*>(key_chunks[ka >> CBFT_KEY_CHUNK_SHIFT]) + (size_t)(ka & (CBFT_KEY_CHUNK - 1)) * wpk;
    }
    uint32_t* out = unit_tbl + (size_t)j * geo.entries() * COMB_STRIDE;
    dst[ln] = out + (size_t)(c + 1) * COMB_STRIDE;
    if (c == 0) {
#pragma unroll
      for (int w = 0; w < COMB_STRIDE; w++) out[w] = (w == 0 || w == 9) ? 1u : 0u;  // identity (1, 1, 0)
    }
    ge_cached cj, cs;
    const uint32_t* pe = pos + (u * (size_t)geo.npos + j) * COMB_POS_WORDS;
    cached_load(cj, pe);
    cached_load(cs, pe + CACHED_WORDS);
    // Q = (c + 1) P_j, MSB first over the cb + 1 bits c + 1 can have
    ge_p3 Q;
    ge_p3_0(Q);
    const uint32_t k0 = (uint32_t)c + 1u;
#pragma nounroll
    for (int bit = cb; bit >= 0; bit--) {
      ge_p1p1 r;
      ge_dbl(r, Q.X, Q.Y, Q.Z);
      ge_p1p1_to_p3(Q, r);
      if ((k0 >> bit) & 1u) {
        ge_add(r, Q, cj, false);
        ge_p1p1_to_p3(Q, r);
      }
    }
    fe acc;
    fe_1(acc);
#pragma nounroll
    for (int k = 0; k < COMB_CHUNK; k++) {
      uint32_t* e = tmp + (size_t)k * CACHED_WORDS * nl;
      fe_store_soa(e, nl, gl, Q.X);
      fe_store_soa(e + 9 * nl, nl, gl, Q.Y);
      fe_store_soa(e + 18 * nl, nl, gl, Q.Z);
      fe_mul(acc, acc, Q.Z);
      fe_store_soa(e + 27 * nl, nl, gl, acc);  // prefix product Z_0 .. Z_k
      if (k + 1 < COMB_CHUNK) {
        ge_p1p1 r;
        ge_add(r, Q, cs, false);
        ge_p1p1_to_p3(Q, r);
      }
    }
    fe_invert(inv, acc);
  } else {
    dst[ln] = nullptr;
  }
  fe d2;
  fe_load_const(d2, kFeD2);
#pragma nounroll
  for (int k = COMB_CHUNK - 1; k >= 0; k--) {
    if (live) {
      const uint32_t* e = tmp + (size_t)k * CACHED_WORDS * nl;
      fe zi, x, y, z, xy, ypx, ymx, t2d;
      if (k > 0) {
        fe pre;
        fe_load_soa(pre, e - CACHED_WORDS * nl + 27 * nl, nl, gl);
        fe_mul(zi, inv, pre);
      } else {
        fe_copy(zi, inv);
      }
      fe_load_soa(z, e + 18 * nl, nl, gl);
      fe_mul(inv, inv, z);
      fe_load_soa(x, e, nl, gl);
      fe_load_soa(y, e + 9 * nl, nl, gl);
      fe_mul(x, x, zi);
      fe_mul(y, y, zi);
      fe_mul(xy, x, y);
      fe_add(ypx, y, x);
      fe_carry(ypx);
      fe_sub(ymx, y, x);
      fe_mul(t2d, xy, d2);
      uint32_t* o = reinterpret_cast<uint32_t*>(&ent[ln][0]);
      fe_store(o, ypx);
      fe_store(o + 9, ymx);
      fe_store(o + 18, t2d);
#pragma unroll
      for (int w = 27; w < COMB_STRIDE; w++) o[w] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < COMB_STRIDE / 4; it++) {  // 64 entries x 8 pieces, 64 pieces per instruction
      const int p = it * 64 + ln, L = p >> 3, piece = p & 7;
      uint32_t* d = dst[L];
      if (d) reinterpret_cast<uint4*>(d + (size_t)k * estride)[piece] = ent[L][piece];
    }
    __syncthreads();
  }
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ void fe_dpp(fe& r, const fe& a) {
#pragma unroll
  for (int k = 0; k < FE_LIMBS; k++) r.v[k] = dpp_u32<CTRL>(a.v[k]);
}

// P += (partner lane's P): quad_perm CTRL = 0xB1 (lane ^ 1) or 0x4E (lane ^ 2).  9M.
template <int CTRL>
__device__ __forceinline__ void quad_combine(ge_p3& P, bool needT) {
  ge_p3 Q;
  fe_dpp<CTRL>(Q.X, P.X);
  fe_dpp<CTRL>(Q.Y, P.Y);
  fe_dpp<CTRL>(Q.Z, P.Z);
  fe_dpp<CTRL>(Q.T, P.T);
  ge_cached c;
  ge_p3_to_cached(c, Q);
  ge_p1p1 t;
  ge_add(t, P, c, false);
  if (needT) fe_mul(P.T, t.X, t.Y);
  fe_mul(P.X, t.X, t.T);
  fe_mul(P.Y, t.Y, t.Z);
  fe_mul(P.Z, t.Z, t.T);
}

// w-bit chunk of a 256-bit little-endian word array at a runtime bit offset (bits >= 256 read
// as 0); the word selects are cndmask chains, so no scratch indexing.
__device__ __forceinline__ uint32_t chunk_at(const uint32_t* s, uint32_t off, uint32_t w) {
  const uint32_t wi = off >> 5, sh = off & 31u;
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (uint32_t t = 0; t < 8; t++) {
    lo = wi == t ? s[t] : lo;
    hi = wi + 1 == t ? s[t] : hi;
  }
  const uint64_t v = (((uint64_t)hi << 32) | lo) >> sh;
  return (uint32_t)v & ((1u << w) - 1u);
}

// s + off (mod 2^256) in place
__device__ __forceinline__ void add256(uint32_t* s, const uint32_t* off) {
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint64_t t = (uint64_t)s[k] + off[k] + c;
    s[k] = (uint32_t)t;
    c = t >> 32;
  }
}

#define COMB_MIN_WAVES 4  // waves per SIMD the quad ladder is register-allocated for

// Lane q's quarter of the comb sum [h](-A) + [S]B of signature i (h = h_in, 8 LE words): its
// nper mixed additions from the key's and B's comb tables, entries staged through LDS one
// addition ahead (sdig: COMB_MAX_STEPS x BLOCK ints, stage: BLOCK / 64 x 7 x 64 uint4 of LDS).
// The caller combines the quad's four partial sums.
template <int BLOCK, int DEPTH = 1>
__device__ __forceinline__ void comb_quad_sum(const Ed25519Batch& b, size_t i, uint32_t q, const uint32_t* h_in,
                                              const uint32_t* btbl, const CombLadder& cl, int32_t* sdig, uint4* stage,
                                              ge_p3& P, uint32_t kbase = 0, uint32_t kend = 0, int nper = 0) {
  // the quad's positions [kbase, kend) (default: all of them), nper per lane
  if (kend == 0) {
    kend = cl.a.npos + cl.b.npos;
    nper = cl.nper;
  }
  const uint32_t first = kbase + q * (uint32_t)nper;
  // thread index within the BLOCK-thread group the caller's sdig / stage belong to (a caller may
  // hand each wave of a bigger block its own arrays with BLOCK = 64)
  const uint32_t tid = threadIdx.x & (BLOCK - 1);
  // Digits of this lane's additions (signed, up to +-2^25), kept in LDS ([step][thread]:
  // conflict-free) so the addition loop holds no digit registers.
  {
    uint32_t hs[8], ss[8];
#pragma unroll
    for (int k = 0; k < 8; k++) hs[k] = h_in[k];
    load_words8(ss, b.sig + i * 64 + 32);
    add256(hs, cl.offA);
    add256(ss, cl.offB);
#pragma unroll
    for (int jj = 0; jj < COMB_MAX_STEPS; jj++) {
      const uint32_t k = first + jj;
      const bool isA = k < (uint32_t)cl.a.npos;
      const uint32_t pos = isA ? k : k - cl.a.npos;
      const uint32_t w = isA ? cl.a.w : cl.b.w;
      const uint32_t top = (isA ? cl.a.npos : cl.b.npos) - 1;
      uint32_t s[8];
#pragma unroll
      for (int t = 0; t < 8; t++) s[t] = isA ? hs[t] : ss[t];
      const uint32_t ch = chunk_at(s, pos * w, w);
      const uint32_t half = 1u << (w - 1);
      // top digit in [0, 2^(w-1)]; only S >= L (flagged, rejected in K4) can exceed it
      int d = pos == top ? (int)(ch < half ? ch : half) : (int)ch - (int)half;
      if (jj >= nper || k >= kend) d = 0;
      sdig[jj * BLOCK + tid] = d;
    }
  }
  const uint32_t* akey = b.keys.comb(batch_unit(b, i));
  auto entry = [&](uint32_t jj, int d) {
    const uint32_t k = first + jj;
    const uint32_t ad = (uint32_t)(d < 0 ? -d : d);
    if (k < (uint32_t)cl.a.npos) return akey + ((size_t)k * cl.a.entries() + ad) * COMB_STRIDE;
    const uint32_t pos = k < kend ? k - cl.a.npos : 0u;  // past the range: identity (entry 0)
    return btbl + ((size_t)pos * cl.b.entries() + ad) * COMB_STRIDE;
  };
  auto digit = [&](int jj) { return sdig[jj * BLOCK + tid]; };
  ge_p3_0(P);
  // Table entries are staged through LDS with global_load_lds (no VGPR destination), DEPTH entries
  // in flight: entry jj + DEPTH's 7 x 16 B are requested as soon as entry jj has been read out of
  // its LDS slot, so the HBM / Infinity-Cache latency (random reads over tens of GB: TLB misses)
  // overlaps DEPTH additions.  LDS image per wave and slot: [chunk 0..6][lane][16 B] (lane-linear,
  // as one global_load_lds_dwordx4 writes it), 7 KB; the caller's stage holds DEPTH slots per wave.
  uint4(*st0)[64] = reinterpret_cast<uint4(*)[64]>(stage + (tid >> 6) * DEPTH * 7 * 64);
  const uint32_t ln = tid & 63u;
  auto request = [&](const uint32_t* e, int slot) {
    uint4(*st)[64] = st0 + slot * 7;
#pragma unroll
    for (int c = 0; c < 7; c++)
      __builtin_amdgcn_global_load_lds(e + 4 * c, (__attribute__((address_space(3))) void*)&st[c][0], 16, 0, 0);
  };
  int d = digit(0);
  int dq[DEPTH];  // digits of the entries in flight, by slot
#pragma unroll
  for (int s = 0; s < DEPTH; s++) {
    dq[s] = s == 0 ? d : digit(s);
    if (s < nper) request(entry(s, dq[s]), s);
  }
#pragma nounroll
  for (int jj = 0; jj < nper; jj++) {
    const int slot = jj % DEPTH;
    // entry jj has arrived once at most DEPTH - 1 later requests (7 loads each) are outstanding;
    // in the last DEPTH - 1 iterations fewer are, so wait for all
    if (DEPTH > 1 && jj + DEPTH <= nper)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(7 * (DEPTH - 1)) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t ew[28];
    uint4(*st)[64] = st0 + slot * 7;
#pragma unroll
    for (int c = 0; c < 7; c++) {
      const uint4 v = st[c][ln];
      ew[4 * c] = v.x;
      ew[4 * c + 1] = v.y;
      ew[4 * c + 2] = v.z;
      ew[4 * c + 3] = v.w;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // entry jj is in VGPRs: the slot is free
    int dcur = dq[0];
#pragma unroll
    for (int s = 1; s < DEPTH; s++)
      if (slot == s) dcur = dq[s];
    const bool neg = dcur < 0;
    if (jj + DEPTH < nper) {
      const int dn = digit(jj + DEPTH);
#pragma unroll
      for (int s = 0; s < DEPTH; s++)
        if (slot == s) dq[s] = dn;
      request(entry(jj + DEPTH, dn), slot);
    }
    if (jj == 0) {  // the lane's first addition starts from the identity: a point set (see the pair ladder), 1 M
      fe ypx, ymx, E, H;
#pragma unroll
      for (int k = 0; k < FE_LIMBS; k++) {
        ypx.v[k] = neg ? ew[9 + k] : ew[k];
        ymx.v[k] = neg ? ew[k] : ew[9 + k];
      }
      fe_sub(E, ypx, ymx);
      fe_add(H, ypx, ymx);
      fe_carry(H);
      fe_mul(P.T, E, H);
      fe_add(P.X, E, E);
      fe_carry(P.X);
      fe_add(P.Y, H, H);
      fe_carry(P.Y);
      fe_0(P.Z);
      P.Z.v[0] = 4;
      continue;
    }
    ge_p1p1 t;
    {
      // niels (y+x, y-x, 2dxy), negated by swapping y+x <-> y-x and C <-> -C (ge_add_mem)
      fe A, B, C, D, s, e;
#pragma unroll
      for (int k = 0; k < FE_LIMBS; k++) e.v[k] = neg ? ew[9 + k] : ew[k];
      fe_add(s, P.Y, P.X);
      fe_mul(A, s, e);
#pragma unroll
      for (int k = 0; k < FE_LIMBS; k++) e.v[k] = neg ? ew[k] : ew[9 + k];
      fe_sub(s, P.Y, P.X);
      fe_mul(B, s, e);
#pragma unroll
      for (int k = 0; k < FE_LIMBS; k++) e.v[k] = ew[18 + k];
      fe_mul(C, e, P.T);
      fe_add(D, P.Z, P.Z);
      fe_sub(t.X, A, B);
      fe_add(t.Y, A, B);
      fe_add(s, D, C);
      fe_carry(s);
      fe_sub(e, D, C);
#pragma unroll
      for (int k = 0; k < FE_LIMBS; k++) {
        t.Z.v[k] = neg ? e.v[k] : s.v[k];
        t.T.v[k] = neg ? s.v[k] : e.v[k];
      }
    }
    fe_mul(P.T, t.X, t.Y);
    fe_mul(P.X, t.X, t.T);
    fe_mul(P.Y, t.Y, t.Z);
    fe_mul(P.Z, t.Z, t.T);
  }
}

__global__ void __launch_bounds__(CBFT_VERIFY_BLOCK, COMB_MIN_WAVES)
    ed25519_comb_ladder_kernel(const Ed25519Batch b, const uint32_t* h_soa, const uint32_t* btbl,
                               const CombLadder cl, uint32_t* xyz_soa) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t q = threadIdx.x & 3u;
  size_t i = g >> 2;
  const bool live = i < b.n;
  if (!live) i = b.n - 1;  // tail quads compute a copy (all lanes stay active for the DPP)
  // Digits of this lane's additions (signed, up to +-2^25), kept in LDS ([step][thread]:
  // conflict-free) so the addition loop holds no digit registers.
  __shared__ int32_t sdig[COMB_MAX_STEPS * CBFT_VERIFY_BLOCK];
  // Table entries are staged through LDS with global_load_lds (no VGPR destination): entry
  // jj+1's 7 x 16 B are requested as soon as entry jj has been read out of LDS, so its HBM /
  // Infinity-Cache latency overlaps the rest of addition jj.  LDS image per wave:
  // [chunk 0..6][lane][16 B] (lane-linear, as one global_load_lds_dwordx4 writes it), 7 KB.
  __shared__ uint4 stage[CBFT_VERIFY_BLOCK / 64 * 7 * 64];
  uint32_t hs[8];
#pragma unroll
  for (int k = 0; k < 8; k++) hs[k] = h_soa[k * b.n + i];
  ge_p3 P;
  comb_quad_sum<CBFT_VERIFY_BLOCK>(b, i, q, hs, btbl, cl, sdig, stage, P);
  quad_combine<0xB1>(P, true);
  quad_combine<0x4E>(P, false);
  if (live && q == 0) {
    fe_store_soa(xyz_soa, b.n, i, P.X);
    fe_store_soa(xyz_soa + 9 * b.n, b.n, i, P.Y);
    fe_store_soa(xyz_soa + 18 * b.n, b.n, i, P.Z);
  }
}

// ---------------------------------------------------------------------------------------
// Small batches in ONE launch (the per-request path: a few coalesced verify() calls): a block of
// four waves (four SIMDs) per 8 signatures.  Wave 0 hashes (a lane quad per signature, every lane
// of the quad the same digest), then sums [h](-A) over its quads (the key comb's positions only)
// and adds the [S]B half; wave 1 sums [S]B (B's comb positions: S is known before the hash) and
// hands it over in LDS; waves 2 and 3 decode R (each signature's square-root chain on a 16-lane DPP
// row, ge_frombytes_row; a fifth wave would share a SIMD: measured on gfx950, a decode wave that
// shares wave 0's SIMD takes 80 us against 42 us, and slows the hash).  The verdict then needs no
// inversion: encode(R') == R (OpenSSL's memcmp of the encodings) holds exactly when R's y is
// canonical, R decodes, R is not "x = 0 with the sign bit set", and R' = (X : Y : Z) equals
// (x_R, y_R) projectively (X = x_R Z, Y = y_R Z): the encoding is a bijection between points and
// canonical encodings, and the decoder picks x by the sign bit.
// ---------------------------------------------------------------------------------------
#define SMALL_SIGS 8
// comb-table entries in flight per lane (LDS: 7 KB per entry and comb wave).  PMC of the one-entry
// form: 44 % of the kernel's wave cycles in s_waitcnt (the key table's random reads over tens of
// GB), but p50 @ 1K and the lone verify measured the same at 1, 2 and 4 in flight (A/B on one
// box): the waits are off the critical path (wave 0's SHA-512)
#define SMALL_DEPTH 2
// the [S]B wave writes the SHA-512 message schedules (K[t] + W[t]) of messages up to
// SMALL_KW_BLOCKS blocks (64 + len + 17 <= 1,024 B) to LDS first, so wave 0's hash is rounds only
#define SMALL_KW_BLOCKS 8
#define SMALL_DEC_WAVES 2

// The block's verdict bits (bit s = signature blk * SMALL_SIGS + s) as SMALL_SIGS / 8 bytes; the
// last block also zeroes the bytes of its 64-bit verdict word that no block covers, so the call
// writes whole ceil(n/64) words (bits past n = 0) like the ballot kernels.
__device__ __forceinline__ void small_store_bits(uint8_t* vb, uint32_t bits) {
  constexpr uint32_t BYTES = SMALL_SIGS / 8;
#pragma unroll
  for (uint32_t k = 0; k < BYTES; k++) vb[blockIdx.x * BYTES + k] = (uint8_t)(bits >> (8 * k));
  if (blockIdx.x == gridDim.x - 1)
    for (uint32_t p = (blockIdx.x + 1) * BYTES; (p & 7u) != 0u; p++) vb[p] = 0;
}

// Decode wave dw of a small-kernel block: x_R | y_R | (R decodes && y canonical && not (x = 0
// with the sign bit set)) of its signatures into rdec.
template <bool SYNC = false>  // SYNC: the wave joins one extra __syncthreads() (see ge_frombytes_row)
__device__ __forceinline__ void small_decode_r(const Ed25519Batch& b, uint32_t blk, uint32_t dw, uint32_t ln,
                                               uint32_t (*rdec)[2 * FE_LIMBS + 1]) {
  const uint32_t sl = dw * 4 + (ln >> 4);
  const bool writer = (ln & 15u) == 0;
  size_t i = (size_t)blk * SMALL_SIGS + sl;
  if (i >= b.n) i = b.n - 1;
  uint32_t Rw[8];
  load_words8(Rw, b.sig + i * 64);
  fe X, Y;
  bool ok = ge_frombytes_row<SYNC>(X, Y, Rw);
  // y < p: the 255-bit y is not one of 2^255 - 19 .. 2^255 - 1
  bool top = (Rw[7] & 0x7fffffffu) == 0x7fffffffu && Rw[0] >= 0xffffffedu;
#pragma unroll
  for (int k = 1; k < 7; k++) top = top && Rw[k] == 0xffffffffu;
  ok = ok && !top && !(fe_iszero(X) && (Rw[7] >> 31));
  if (writer) {
#pragma unroll
    for (int k = 0; k < FE_LIMBS; k++) {
      rdec[sl][k] = X.v[k];
      rdec[sl][FE_LIMBS + k] = Y.v[k];
    }
    rdec[sl][2 * FE_LIMBS] = ok ? 1u : 0u;
  }
}
#define SMALL3_BLOCK (64 * (2 + SMALL_DEC_WAVES))
__global__ void __launch_bounds__(SMALL3_BLOCK) ed25519_small3_kernel(const Ed25519Batch b, const uint32_t* btbl,
                                                                      const CombLadder cl, uint8_t* verdict_bytes) {
  __shared__ int32_t sdig[2][COMB_MAX_STEPS * 64];
  __shared__ uint4 stage[2][SMALL_DEPTH * 7 * 64];
  __shared__ uint32_t rdec[SMALL_SIGS][2 * FE_LIMBS + 1];  // x_R | y_R | decodes
  __shared__ uint32_t sbp[SMALL_SIGS][4 * FE_LIMBS];       // [S]B as X | Y | Z | T
  __shared__ uint64_t kw[SMALL_SIGS][SMALL_KW_BLOCKS * KW_STRIDE];  // SHA-512 K[t] + W[t] per block
  const uint32_t ln = threadIdx.x & 63u, wave = threadIdx.x >> 6, q = ln & 3u, sl = (ln >> 2) & (SMALL_SIGS - 1);
  size_t i = (size_t)blockIdx.x * SMALL_SIGS + sl;
  const bool live = i < b.n && (ln >> 2) < SMALL_SIGS;
  if (i >= b.n) i = b.n - 1;
  const uint32_t na = (uint32_t)cl.a.npos, ntot = na + (uint32_t)cl.b.npos;
  // Every wave joins two barriers: "schedules written" (wave 1 -> wave 0, which compresses block 0
  // meanwhile; the decode waves join it ~12 us into their square-root chain) and "sums and
  // decodes done".  The split hash runs when
  // every signature of the block fits SMALL_KW_BLOCKS SHA-512 blocks (a wave-uniform ballot that
  // waves 0 and 1 compute alike); otherwise wave 0 hashes on its own as before.
  const bool split = __ballot(sig_sha_blocks(b, i) > SMALL_KW_BLOCKS) == 0;
  if (wave >= 2) {  // (without the split every wave passes the first barrier at its start)
    if (split) {
      small_decode_r<true>(b, blockIdx.x, wave - 2, ln, rdec);
    } else {
      __syncthreads();
      small_decode_r<false>(b, blockIdx.x, wave - 2, ln, rdec);
    }
    __syncthreads();
    return;
  }
  if (wave == 1) {  // [S]B: B's positions [na, ntot) over the quad; the digits need no hash
    if (split && (ln >> 2) < SMALL_SIGS) ed25519_sched_sig(b, i, q, kw[sl]);
    __syncthreads();
    const uint32_t zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    ge_p3 P;
    comb_quad_sum<64, SMALL_DEPTH>(b, i, q, zero, btbl, cl, sdig[1], stage[1], P, na, ntot, (int)((ntot - na + 3) / 4));
    quad_combine<0xB1>(P, true);
    quad_combine<0x4E>(P, true);
    if (q == 0 && (ln >> 2) < SMALL_SIGS) {
#pragma unroll
      for (int k = 0; k < FE_LIMBS; k++) {
        sbp[sl][k] = P.X.v[k];
        sbp[sl][FE_LIMBS + k] = P.Y.v[k];
        sbp[sl][2 * FE_LIMBS + k] = P.Z.v[k];
        sbp[sl][3 * FE_LIMBS + k] = P.T.v[k];
      }
    }
    __syncthreads();
    return;
  }
  uint32_t hs[8];
  bool flag;
  if (split) {
    ed25519_hash_sig_kw(b, i, kw[sl], hs, flag, [&] {
      __syncthreads();  // wave 1's message schedules (block 0 is done meanwhile)
    });
  } else {
    __syncthreads();
    ed25519_hash_sig(b, i, hs, flag);
  }
  ge_p3 P;
  comb_quad_sum<64, SMALL_DEPTH>(b, i, q, hs, btbl, cl, sdig[0], stage[0], P, 0, na, (int)((na + 3) / 4));
  quad_combine<0xB1>(P, true);
  quad_combine<0x4E>(P, true);
  __syncthreads();  // wave 1's [S]B, wave 2's R
  {
    ge_p3 Q;
#pragma unroll
    for (int k = 0; k < FE_LIMBS; k++) {
      Q.X.v[k] = sbp[sl][k];
      Q.Y.v[k] = sbp[sl][FE_LIMBS + k];
      Q.Z.v[k] = sbp[sl][2 * FE_LIMBS + k];
      Q.T.v[k] = sbp[sl][3 * FE_LIMBS + k];
    }
    ge_cached c;
    ge_p3_to_cached(c, Q);
    ge_p1p1 t;
    ge_add(t, P, c, false);
    fe_mul(P.X, t.X, t.T);
    fe_mul(P.Y, t.Y, t.Z);
    fe_mul(P.Z, t.Z, t.T);
  }
  fe xr, yr, t;
#pragma unroll
  for (int k = 0; k < FE_LIMBS; k++) {
    xr.v[k] = rdec[sl][k];
    yr.v[k] = rdec[sl][FE_LIMBS + k];
  }
  bool same = rdec[sl][2 * FE_LIMBS] != 0;
  fe_mul<false>(t, xr, P.Z);
  fe_sub(t, P.X, t);
  same = same && fe_iszero(t);
  fe_mul<false>(t, yr, P.Z);
  fe_sub(t, P.Y, t);
  same = same && fe_iszero(t);
  const bool verdict = live && same && flag && b.keys.aok(batch_unit(b, i));
  const uint64_t bal = __ballot(verdict);
  uint32_t bits = 0;
#pragma unroll
  for (int s2 = 0; s2 < SMALL_SIGS; s2++) bits |= (uint32_t)((bal >> (4 * s2)) & 1u) << s2;
  if (ln == 0) small_store_bits(verdict_bytes, bits);
}

// ---------------------------------------------------------------------------------------
// The same comb sum on TWO lanes per signature (lane q of a pair takes additions q*nper ..
// q*nper + nper - 1, nper = ceil(positions / 2)), one DPP combine.  Per signature that is
// 2 x (16 x 7M + 8M) = 240 lane-M at the default geometry against 4 x (8 x 7M + 17M) = 292 for
// the quad form (whose two combine levels are a quarter of a lane's work), at 2 waves per SIMD
// for a 64K batch instead of 4 (256 VGPRs per lane; gfx950 issues the mad / 64-bit mix ~9 %
// slower per instruction at 2 waves than at 4: tools/microbench/intrate2.hip).  The lower
// occupancy buys LDS for a second entry stage: entries jj+1 and jj+2 are in flight while
// addition jj runs, so the key-table / B-table reads (random over tens of GB) stay hidden.
// The two recoded scalars sit in LDS ([word][lane]) and each digit is extracted right before
// its entry is requested.
// ---------------------------------------------------------------------------------------
#define COMB2_BLOCK 128
#define COMB2_MAX_STEPS 24  // additions per lane: radix-2^8 keys + radix-2^16 B = 48 positions
#define COMB2_MIN_WAVES 2
__global__ void __launch_bounds__(COMB2_BLOCK, COMB2_MIN_WAVES)
    ed25519_comb2_ladder_kernel(const Ed25519Batch b, const uint32_t* h_soa, const uint32_t* btbl,
                                const CombLadder cl, uint32_t* xyz_soa) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t q = threadIdx.x & 1u;
  size_t i = g >> 1;
  const bool live = i < b.n;
  if (!live) i = b.n - 1;  // tail pairs compute a copy (both lanes stay active for the DPP)
  const uint32_t na = (uint32_t)cl.a.npos, nb = (uint32_t)cl.b.npos;
  // Phased split: each lane takes half of the key positions, then half of B's, so at every step
  // both lanes of every pair read the same table (the step's table, radix and scalar are
  // wave-uniform: scalar branches, no per-lane selects).  ceil(na/2) + ceil(nb/2) steps: the same
  // 16 as ceil(32/2) at the default 20 + 12 positions.
  const uint32_t naper = (na + 1u) >> 1, nbper = (nb + 1u) >> 1;
  const uint32_t nper = naper + nbper;
  __shared__ uint4 stage[COMB2_BLOCK / 64][2][7][64];  // per wave: two lane-linear 7 KB entry images
  __shared__ uint32_t sc[16][COMB2_BLOCK];              // h + offA (words 0..7), S + offB (8..15)
  {
    uint32_t hs[8], ss[8];
#pragma unroll
    for (int k = 0; k < 8; k++) hs[k] = h_soa[k * b.n + i];
    load_words8(ss, b.sig + i * 64 + 32);
    add256(hs, cl.offA);
    add256(ss, cl.offB);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      sc[k][threadIdx.x] = hs[k];
      sc[8 + k][threadIdx.x] = ss[k];
    }
  }
  // chunk of w bits at bit offset `off` of the recoded scalar in sc[base..base+7]
  auto chunk = [&](uint32_t base, uint32_t off, uint32_t w) -> uint32_t {
    const uint32_t wi = off >> 5;
    const uint32_t lo = sc[base + wi][threadIdx.x];
    const uint32_t hi = wi < 7u ? sc[base + wi + 1u][threadIdx.x] : 0u;  // bits >= 256 read as 0
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (off & 31u)) & ((1u << w) - 1u);
  };
  // signed digit of this lane's step jj (0 = the identity entry past the last position)
  auto digit = [&](uint32_t jj) -> int {
    if (jj >= nper) return 0;
    const bool isA = jj < naper;  // uniform
    const uint32_t pos = isA ? q * naper + jj : q * nbper + (jj - naper);
    const uint32_t np = isA ? na : nb;
    if (pos >= np) return 0;
    const uint32_t w = isA ? (uint32_t)cl.a.w : (uint32_t)cl.b.w;
    const uint32_t ch = chunk(isA ? 0u : 8u, pos * w, w);
    const uint32_t half = 1u << (w - 1u);
    // top digit in [0, 2^(w-1)]; only S >= L (flagged, rejected in K4) can exceed it
    return pos == np - 1u ? (int)(ch < half ? ch : half) : (int)ch - (int)half;
  };
  const uint32_t* akey = b.keys.comb(batch_unit(b, i));
  auto entry = [&](uint32_t jj, int d) {
    const uint32_t ad = (uint32_t)(d < 0 ? -d : d);
    if (jj < naper) {
      const uint32_t pos = q * naper + jj;
      return akey + ((size_t)(pos < na ? pos : 0u) * cl.a.entries() + ad) * COMB_STRIDE;
    }
    const uint32_t pos = jj < nper ? q * nbper + (jj - naper) : 0u;
    return btbl + ((size_t)(pos < nb ? pos : 0u) * cl.b.entries() + ad) * COMB_STRIDE;
  };
  const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
  auto request = [&](uint32_t slot, const uint32_t* e) {
#pragma unroll
    for (int c = 0; c < 7; c++)
      __builtin_amdgcn_global_load_lds(e + 4 * c, (__attribute__((address_space(3))) void*)&stage[wv][slot][c][0], 16,
                                       0, 0);
  };
  ge_p3 P;
  ge_p3_0(P);
  int dcur = digit(0), dnext = digit(1);
  request(0, entry(0, dcur));
  if (nper > 1u) request(1, entry(1, dnext));
#pragma nounroll
  for (uint32_t jj = 0; jj < nper; jj++) {
    const uint32_t slot = jj & 1u;
    if (jj + 1u < nper)
      asm volatile("s_waitcnt vmcnt(7)" ::: "memory");  // entry jj landed; jj + 1 may still fly
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // The stage is read with asm ds_reads: the compiler would otherwise see LDS reads after
    // global_load_lds writes and wait for ALL of them (vmcnt(0)), serialising the two stages.
    uint32_t ew[28];
    {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const uint32_t addr = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint4*)&stage[wv][slot][0][ln]);
      u32x4 v[7];
#define COMB2_DS_READ(c) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v[c]) : "v"(addr), "i"((c) * 1024))
      COMB2_DS_READ(0);
      COMB2_DS_READ(1);
      COMB2_DS_READ(2);
      COMB2_DS_READ(3);
      COMB2_DS_READ(4);
      COMB2_DS_READ(5);
      COMB2_DS_READ(6);
#undef COMB2_DS_READ
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // entry jj is in VGPRs: its stage is free
#pragma unroll
      for (int c = 0; c < 7; c++) {
        ew[4 * c] = v[c].x;
        ew[4 * c + 1] = v[c].y;
        ew[4 * c + 2] = v[c].z;
        ew[4 * c + 3] = v[c].w;
      }
    }
    const bool neg = dcur < 0;
    dcur = dnext;
    if (jj + 2u < nper) {
      dnext = digit(jj + 2u);
      request(slot, entry(jj + 2u, dnext));
    }
    if (jj == 0) {
      // The lane's first addition starts from the identity: O + (x, y) needs no product but T.
      // With E = (y+x) - (y-x) = 2x and H = (y+x) + (y-x) = 2y (swapped for a negative digit,
      // giving -x), P = (2E : 2H : 4 : E H) = (x : y : 1 : xy) scaled by 4 (XY = ZT holds):
      // 1 M instead of the addition's 7 M.  The identity entry (1, 1, 0) gives (0 : 4 : 4 : 0).
      fe ypx, ymx, E, H;
#pragma unroll
      for (int k = 0; k < FE_LIMBS; k++) {
        ypx.v[k] = neg ? ew[9 + k] : ew[k];
        ymx.v[k] = neg ? ew[k] : ew[9 + k];
      }
      fe_sub(E, ypx, ymx);  // reduced
      fe_add(H, ypx, ymx);
      fe_carry(H);
      fe_mul(P.T, E, H);
      fe_add(P.X, E, E);
      fe_carry(P.X);
      fe_add(P.Y, H, H);
      fe_carry(P.Y);
      fe_0(P.Z);
      P.Z.v[0] = 4;
      continue;
    }
    ge_p1p1 t;
    // the addition's independent products as interleaved pairs (fe_mul2_oneasm: two mad chains in
    // one asm statement, each instruction followed by the other product's independent one): (A, B),
    // then C alone, then (T, X) and (Y, Z).  Isolated ladder -2.3 %, 200-step headline -2 % against
    // seven single products (tools/probes/r06_ab2.sh); three- and four-way groups measured slower.
    {
      fe A, B, C, D, s1, s2, e1, e2, e3, s, e;
#pragma unroll
      for (int k = 0; k < FE_LIMBS; k++) {
        e1.v[k] = neg ? ew[9 + k] : ew[k];  // niels (y+x, y-x, 2dxy), negated by swapping y+x <-> y-x
        e2.v[k] = neg ? ew[k] : ew[9 + k];  // and C <-> -C (ge_add_mem)
        e3.v[k] = ew[18 + k];
      }
      fe_add(s1, P.Y, P.X);
      fe_sub(s2, P.Y, P.X);
      fe_mul2_oneasm(A, s1, e1, B, s2, e2);
      fe_mul(C, e3, P.T);
      fe_add(D, P.Z, P.Z);
      fe_sub(t.X, A, B);
      fe_add(t.Y, A, B);
      fe_add(s, D, C);
      fe_carry(s);
      fe_sub(e, D, C);
#pragma unroll
      for (int k = 0; k < FE_LIMBS; k++) {
        t.Z.v[k] = neg ? e.v[k] : s.v[k];
        t.T.v[k] = neg ? s.v[k] : e.v[k];
      }
    }
    fe_mul2_oneasm(P.T, t.X, t.Y, P.X, t.X, t.T);
    fe_mul2_oneasm(P.Y, t.Y, t.Z, P.Z, t.Z, t.T);
  }
  quad_combine<0xB1>(P, false);  // P += partner lane's P
  if (live && q == 0) {
    fe_store_soa(xyz_soa, b.n, i, P.X);
    fe_store_soa(xyz_soa + 9 * b.n, b.n, i, P.Y);
    fe_store_soa(xyz_soa + 18 * b.n, b.n, i, P.Z);
  }
}

// ---------------------------------------------------------------------------------------
// host-side launch helpers (used by cbft_hipcrypto.cpp)
// ---------------------------------------------------------------------------------------
size_t cbft_ed25519_comb_tmp_words(size_t lanes) { return lanes * COMB_TMP_WORDS_PER_LANE; }

size_t cbft_ed25519_comb_pos_words(size_t nunits, const CombGeom& g) {
  return nunits * (size_t)g.npos * COMB_POS_WORDS;
}

hipError_t cbft_ed25519_launch_comb_pos(const uint8_t* d_pk, size_t nunits, int negate, const CombGeom& g,
                                        uint32_t* d_pos, uint8_t* d_aok, hipStream_t stream) {
  if (nunits == 0) return hipSuccess;
  if (g.w < 8 || g.w > CBFT_COMB_MAX_RADIX || g.npos < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ed25519_comb_pos_kernel, dim3((unsigned)((nunits + COMB_TABLE_BLOCK - 1) / COMB_TABLE_BLOCK)),
                     dim3(COMB_TABLE_BLOCK), 0, stream, d_pk, nunits, negate, g, d_pos, d_aok);
  return hipGetLastError();
}

hipError_t cbft_ed25519_launch_comb_tables(const uint32_t* d_pos, size_t nunits, const CombGeom& g, uint32_t* d_tbl,
                                           void* const* d_chunks, uint32_t a0, uint32_t* d_tmp, size_t lane0,
                                           size_t nlanes, hipStream_t stream) {
  if (nunits == 0 || nlanes == 0) return hipSuccess;
  if (g.w < 8 || g.w > CBFT_COMB_MAX_RADIX || g.npos < 1) return hipErrorInvalidValue;
  if (lane0 + nlanes > nunits * g.npos * g.chunks()) return hipErrorInvalidValue;
  if (!d_chunks == !d_tbl) return hipErrorInvalidValue;  // exactly one destination form
  hipLaunchKernelGGL(ed25519_comb_table_kernel, dim3((unsigned)((nlanes + COMB_TABLE_BLOCK - 1) / COMB_TABLE_BLOCK)),
                     dim3(COMB_TABLE_BLOCK), 0, stream, d_pos, nunits, g, d_tbl, d_chunks, a0, d_tmp, lane0, nlanes);
  return hipGetLastError();
}
size_t cbft_ed25519_table_words_per_unit() { return (size_t)Shape::TA * CACHED_WORDS; }
size_t cbft_ed25519_base_table_words() { return (size_t)Shape::TB * NIELS_WORDS; }

static inline unsigned grid_for(size_t n) { return (unsigned)((n + CBFT_VERIFY_BLOCK - 1) / CBFT_VERIFY_BLOCK); }

hipError_t cbft_ed25519_build_base_table(uint32_t* d_tbl, hipStream_t stream) {
  hipLaunchKernelGGL(ed25519_base_table_kernel, dim3(1), dim3(64), 0, stream, d_tbl, Shape::TB);
  return hipGetLastError();
}

hipError_t cbft_ed25519_launch_prep(const uint8_t* d_pk, size_t nunits, uint32_t* d_tbl, uint8_t* d_aok,
                                    hipStream_t stream) {
  if (nunits == 0) return hipSuccess;
  hipLaunchKernelGGL(ed25519_prep_kernel, dim3(grid_for(nunits)), dim3(CBFT_VERIFY_BLOCK), 0, stream, d_pk, nunits,
                     d_tbl, d_aok);
  return hipGetLastError();
}

hipError_t cbft_ed25519_launch_verify(const Ed25519Batch& b, const Ed25519Work& w, hipStream_t stream,
                                      hipEvent_t* ev, const StageOrder* order) {
  if (b.n == 0) return hipSuccess;
  const bool comb = b.keys.chunk && w.base_comb && b.key_idx;
  if (comb && (w.comb.nper < 1 || w.comb.nper > COMB_MAX_STEPS || 4 * w.comb.nper < w.comb.a.npos + w.comb.b.npos))
    return hipErrorInvalidValue;
  if (comb && w.comb_lanes == 2 && w.comb.a.npos + w.comb.b.npos > 2 * COMB2_MAX_STEPS) return hipErrorInvalidValue;
  const dim3 grid(grid_for(b.n)), block(CBFT_VERIFY_BLOCK);
  hipError_t e;
  if (comb && w.small) {  // the per-request path: hash + quad comb + finish in one launch, unordered
    if (w.comb.nper > COMB_MAX_STEPS) return hipErrorInvalidValue;
    if (ev)
      for (int k = 0; k < 3; k++) (void)hipEventRecord(ev[k], stream);
    hipLaunchKernelGGL(ed25519_small3_kernel, dim3((unsigned)((b.n + SMALL_SIGS - 1) / SMALL_SIGS)), dim3(SMALL3_BLOCK), 0,
                       stream, b, w.base_comb, w.comb, reinterpret_cast<uint8_t*>(w.verdict_words));
    if (ev) (void)hipEventRecord(ev[3], stream);
    return hipGetLastError();
  }
  if (order && order->wait && order->hash && (e = hipStreamWaitEvent(stream, order->done[0], 0)) != hipSuccess)
    return e;
  if (ev) (void)hipEventRecord(ev[0], stream);
  const bool sorted = w.perm && w.buckets && b.msg_off;
  if (sorted) {
    const dim3 g256((unsigned)((b.n + 255) / 256)), b256(256);
    hipLaunchKernelGGL(ed25519_bucket_count_kernel, g256, b256, 0, stream, b, w.buckets);
    hipLaunchKernelGGL(ed25519_bucket_scan_kernel, dim3(1), b256, 0, stream, w.buckets, w.buckets + CBFT_SHA_BUCKETS,
                       (uint32_t)CBFT_SHA_LONG_GROUPS);
    hipLaunchKernelGGL(ed25519_bucket_scatter_kernel, g256, b256, 0, stream, b, w.buckets + CBFT_SHA_BUCKETS, w.perm);
  }
  const uint32_t* uniform_w = sorted ? (const uint32_t*)(w.buckets + 2 * CBFT_SHA_BUCKETS) : nullptr;
  const uint32_t* nshort_w = sorted && w.aux ? (const uint32_t*)(w.buckets + 2 * CBFT_SHA_BUCKETS + 1) : nullptr;
  if (nshort_w) {  // the long messages on the second stream, beside the short ones
    if ((e = hipEventRecord(w.fork_ev, stream)) != hipSuccess || (e = hipStreamWaitEvent(w.aux, w.fork_ev, 0)) != hipSuccess)
      return e;
    hipLaunchKernelGGL(ed25519_hash_long_kernel, dim3((unsigned)((b.n + 63) / 64)), dim3(HASH_LONG_BLOCK), 0, w.aux, b,
                       (const uint32_t*)w.perm, uniform_w, nshort_w, w.h_soa, w.flags);
    if ((e = hipEventRecord(w.join_ev, w.aux)) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(ed25519_hash_kernel, grid, block, 0, stream, b, sorted ? (const uint32_t*)w.perm : nullptr,
                     uniform_w, nshort_w, w.h_soa, w.flags);
  // the next batch's hash may start behind this batch's short hashes while the long tail still
  // runs on the aux stream (hash_early), or only after the whole hash stage
  if (order && order->hash_early && (e = hipEventRecord(order->done[0], stream)) != hipSuccess) return e;
  if (nshort_w && (e = hipStreamWaitEvent(stream, w.join_ev, 0)) != hipSuccess) return e;
  if (order && !order->hash_early && (e = hipEventRecord(order->done[0], stream)) != hipSuccess) return e;
  if (order && order->wait && order->ladder && (e = hipStreamWaitEvent(stream, order->done[1], 0)) != hipSuccess)
    return e;
  if (ev) (void)hipEventRecord(ev[1], stream);
  if (comb && w.comb_lanes == 2) {
    hipLaunchKernelGGL(ed25519_comb2_ladder_kernel, dim3((unsigned)((2 * b.n + COMB2_BLOCK - 1) / COMB2_BLOCK)),
                       dim3(COMB2_BLOCK), 0, stream, b, w.h_soa, w.base_comb, w.comb, w.xyz_soa);
  } else if (comb) {
    hipLaunchKernelGGL(ed25519_comb_ladder_kernel, dim3((unsigned)((4 * b.n + CBFT_VERIFY_BLOCK - 1) / CBFT_VERIFY_BLOCK)),
                       block, 0, stream, b, w.h_soa, w.base_comb, w.comb, w.xyz_soa);
  } else {
    hipLaunchKernelGGL(ed25519_ladder_kernel, grid, block, 0, stream, b, w.h_soa, w.tbl, w.base_table, w.xyz_soa);
  }
  if (order && (e = hipEventRecord(order->done[1], stream)) != hipSuccess) return e;
  if (ev) (void)hipEventRecord(ev[2], stream);
  if (w.finish_k == 2)
    hipLaunchKernelGGL(ed25519_finish_kernel<2>, dim3((unsigned)((b.n + 127) / 128)), dim3(FINISH_BLOCK), 0, stream, b,
                       w.xyz_soa, w.flags, w.aok, w.verdict_words);
  else
    hipLaunchKernelGGL(ed25519_finish_kernel<1>, dim3((unsigned)((b.n + 63) / 64)), dim3(FINISH_BLOCK), 0, stream, b,
                       w.xyz_soa, w.flags, w.aok, w.verdict_words);
  if (ev) (void)hipEventRecord(ev[3], stream);
  return hipGetLastError();
}
