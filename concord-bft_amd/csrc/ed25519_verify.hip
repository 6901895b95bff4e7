// Batched Ed25519 signature verification for gfx950 (MI355X): one signature per lane.
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

// NW big-endian 64-bit words of (M || 0x80 || 0 ...) starting at M-relative offset base.
// Only dwords that overlap [m, m+len) are loaded (an aligned dword holding >= 1 message byte
// never faults), so callers need no padding after the blob.
//
// Branch-free: dword k is read from index min(k, kmax) (kmax = last dword holding a byte of
// M), or from `safe` (any readable dword) when no dword of this window holds one; bytes at or
// past len are then masked off arithmetically, so a wave never splits on message length.
template <int NW>
__device__ __forceinline__ void load_msg_words(uint64_t* W, const uint8_t* m, uint32_t len, uint32_t base,
                                               const uint32_t* safe) {
  const uintptr_t a = (uintptr_t)(m + base);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  const int kmax = ((int)len - 1 - (int)base + (int)sh) >> 2;  // < 0: window is past M
  uint32_t d[2 * NW + 1];
#pragma unroll
  for (int k = 0; k < 2 * NW + 1; k++) {
    const uint32_t* src = kmax >= 0 ? q + (k < kmax ? k : kmax) : safe;
    d[k] = *src;
  }
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

__global__ void __launch_bounds__(CBFT_VERIFY_BLOCK) ed25519_hash_kernel(const Ed25519Batch b, uint32_t* h_soa,
                                                                          uint8_t* flags) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b.n) return;
  const uint32_t key = b.key_idx ? b.key_idx[i] : (uint32_t)i;
  uint32_t Aw[8], Rw[8], Sw[8];
  load_words8(Aw, b.pk + (size_t)key * 32);
  load_words8(Rw, b.sig + i * 64);
  load_words8(Sw, b.sig + i * 64 + 32);
  const uint8_t* m = b.msg + b.msg_off[i];
  const uint32_t len = b.msg_len[i];
  const uint32_t* safe = reinterpret_cast<const uint32_t*>(b.sig + i * 64);  // readable dword

  uint64_t H[8], W[16];
  sha512_init(H);
  const uint32_t total = 64u + len;
  const uint32_t nblocks = (total + 17u + 127u) / 128u;
  for (uint32_t blk = 0; blk < nblocks; blk++) {
    if (blk == 0) {  // R || A || M[0..63]
#pragma unroll
      for (int j = 0; j < 4; j++) W[j] = ((uint64_t)bswap32(Rw[2 * j]) << 32) | bswap32(Rw[2 * j + 1]);
#pragma unroll
      for (int j = 0; j < 4; j++) W[4 + j] = ((uint64_t)bswap32(Aw[2 * j]) << 32) | bswap32(Aw[2 * j + 1]);
      load_msg_words<8>(W + 8, m, len, 0u, safe);
    } else {
      load_msg_words<16>(W, m, len, 128u * blk - 64u, safe);
    }
    if (blk == nblocks - 1) {
      W[14] = 0;
      W[15] = (uint64_t)total << 3;
    }
    sha512_compress(H, W);
  }
  uint32_t dig[16], hw[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    dig[2 * k] = bswap32((uint32_t)(H[k] >> 32));
    dig[2 * k + 1] = bswap32((uint32_t)H[k]);
  }
  sc_reduce512(hw, dig);
#pragma unroll
  for (int k = 0; k < 8; k++) h_soa[k * b.n + i] = hw[k];
  flags[i] = sc_is_canonical(Sw) ? 1 : 0;
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

  const uint32_t unit = b.key_idx ? b.key_idx[i] : (uint32_t)i;
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
// K4: encode R' and compare with R; verdict ballot per wave
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(CBFT_VERIFY_BLOCK) ed25519_finish_kernel(const Ed25519Batch b, const uint32_t* xyz_soa,
                                                                            const uint8_t* flags, const uint8_t* aok,
                                                                            uint64_t* verdict_words) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool verdict = false;
  if (i < b.n) {
    fe X, Y, Z;
    fe_load_soa(X, xyz_soa, b.n, i);
    fe_load_soa(Y, xyz_soa + 9 * b.n, b.n, i);
    fe_load_soa(Z, xyz_soa + 18 * b.n, b.n, i);
    uint32_t Rp[8], Rw[8];
    ge_tobytes(Rp, X, Y, Z);
    load_words8(Rw, b.sig + i * 64);
    uint32_t diff = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) diff |= Rp[k] ^ Rw[k];
    const uint32_t unit = b.key_idx ? b.key_idx[i] : (uint32_t)i;
    verdict = (diff == 0) && flags[i] && aok[unit];
  }
  const uint64_t ballot = __ballot(verdict);
  if ((threadIdx.x & 63) == 0 && i < b.n) verdict_words[i >> 6] = ballot;
}

// ---------------------------------------------------------------------------------------
// Radix-256 fixed-base comb ("comb8"), four lanes per signature (key-table mode).
//
// At the headline batch (64K signatures) one lane per signature gives 1,024 waves: one wave per
// SIMD, and a lone wave issues VALU at half the SIMD's rate (MI355X_MICROARCH.md, constants
// table).  The comb sum is split instead:
//   C8_P[j][e] = e * 256^j * P,  j = 0..31, e = 0..128 (affine niels, 128-B entries, e = 0 =
//   identity);  s + 0x8080..80 has bytes b_j, digit d_j = b_j - 128 in [-128, 127], and
//   [s]P = sum_j sign(d_j) C8_P[j][|d_j|]   (32 mixed additions, no doublings).
// Lane q of each quad (4 adjacent lanes) sums 16 positions of one scalar:
//   q = 0: h positions 0..15 on -A,  q = 1: h positions 16..31,  q = 2, 3: S on B likewise,
// then two DPP butterfly levels (xor 1, xor 2) add the partial sums: every lane of the quad ends
// with R' = [S]B + [h](-A).  4,096 waves at 64K: 4 waves per SIMD.
// The per-key table (32 x 129 x 128 B = 528,384 B) lives in HBM; B's table (same size) is read
// through L2 by every lane.
// ---------------------------------------------------------------------------------------
#define C8_POS 32
#define C8_ENT 129
#define C8_STRIDE 32  // words per entry: one 128-B line
#define C8_WORDS_PER_UNIT (C8_POS * C8_ENT * C8_STRIDE)
#define C8_TMP_WORDS_PER_LANE (128 * CACHED_WORDS)
#define C8_TABLE_BLOCK 64

// One lane per (unit, position j): P_j = 256^j P (8j doublings), multiples 1..128 of P_j
// projectively into tmp, Montgomery batch inversion, affine niels into tbl[unit][j][1..128].
__global__ void __launch_bounds__(C8_TABLE_BLOCK) ed25519_comb8_table_kernel(const uint8_t* pk, size_t nunits,
                                                                             int negate, uint32_t* tbl,
                                                                             uint32_t* tmp, uint8_t* aok) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t u = g / C8_POS;
  const int j = (int)(g % C8_POS);
  if (u >= nunits) return;
  uint32_t Aw[8];
  load_words8(Aw, pk + u * 32);
  ge_p3 Pj;
  const bool ok = ge_frombytes(Pj, Aw);
  if (aok && j == 0) aok[u] = ok ? 1 : 0;
  if (negate) {
    fe_neg(Pj.X, Pj.X);
    fe_neg(Pj.T, Pj.T);
  }
#pragma nounroll
  for (int d = 0; d < 8 * j; d++) {
    ge_p1p1 r;
    ge_dbl(r, Pj.X, Pj.Y, Pj.Z);
    ge_p1p1_to_p3(Pj, r);
  }
  uint32_t* t = tmp + g * (size_t)C8_TMP_WORDS_PER_LANE;
  uint32_t* out = tbl + (u * C8_POS + j) * (size_t)(C8_ENT * C8_STRIDE);
  ge_cached cj;
  ge_p3_to_cached(cj, Pj);
  ge_p3 Q = Pj;
  fe acc;
  fe_1(acc);
#pragma nounroll
  for (int k = 1; k <= 128; k++) {
    uint32_t* e = t + (size_t)(k - 1) * CACHED_WORDS;
    fe_store(e, Q.X);
    fe_store(e + 9, Q.Y);
    fe_store(e + 18, Q.Z);
    fe_mul(acc, acc, Q.Z);
    fe_store(e + 27, acc);  // prefix product Z_1 .. Z_k
    if (k < 128) {
      ge_p1p1 r;
      ge_add(r, Q, cj, false);
      ge_p1p1_to_p3(Q, r);
    }
  }
  fe inv;
  fe_invert(inv, acc);
  fe d2;
  fe_load_const(d2, kFeD2);
#pragma nounroll
  for (int k = 128; k >= 1; k--) {
    uint32_t* e = t + (size_t)(k - 1) * CACHED_WORDS;
    fe zi, x, y, z, xy, ypx, ymx, t2d;
    if (k > 1) {
      fe pre;
      fe_load(pre, e - CACHED_WORDS + 27);
      fe_mul(zi, inv, pre);
    } else {
      fe_copy(zi, inv);
    }
    fe_load(z, e + 18);
    fe_mul(inv, inv, z);
    fe_load(x, e);
    fe_load(y, e + 9);
    fe_mul(x, x, zi);
    fe_mul(y, y, zi);
    fe_mul(xy, x, y);
    fe_add(ypx, y, x);
    fe_carry(ypx);
    fe_sub(ymx, y, x);
    fe_mul(t2d, xy, d2);
    uint32_t* o = out + (size_t)k * C8_STRIDE;
    fe_store(o, ypx);
    fe_store(o + 9, ymx);
    fe_store(o + 18, t2d);
#pragma unroll
    for (int w = 27; w < C8_STRIDE; w++) o[w] = 0;
  }
#pragma unroll
  for (int w = 0; w < C8_STRIDE; w++) out[w] = (w == 0 || w == 9) ? 1u : 0u;  // identity (1, 1, 0)
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

#ifndef CBFT_COMB8_MIN_WAVES
#define CBFT_COMB8_MIN_WAVES 4
#endif

__global__ void __launch_bounds__(CBFT_VERIFY_BLOCK, CBFT_COMB8_MIN_WAVES)
    ed25519_comb8_ladder_kernel(const Ed25519Batch b, const uint32_t* h_soa, const uint32_t* tbl,
                                const uint32_t* base8, uint32_t* xyz_soa) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t q = threadIdx.x & 3u;
  size_t i = g >> 2;
  const bool live = i < b.n;
  if (!live) i = b.n - 1;  // tail quads compute a copy (all lanes stay active for the DPP)
  const bool onB = (q & 2u) != 0;
  const uint32_t half = q & 1u;
  uint32_t w[8];
  if (onB) {
    load_words8(w, b.sig + i * 64 + 32);
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = h_soa[k * b.n + i];
  }
  // s' = s + 0x8080..80; this lane's 16 bytes (words 4*half .. 4*half+3)
  uint32_t dw[4];
  {
    uint64_t c = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint64_t s = (uint64_t)w[k] + 0x80808080u + c;
      w[k] = (uint32_t)s;
      c = s >> 32;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) dw[k] = half ? w[4 + k] : w[k];
  }
  const uint32_t* base = onB ? base8 : tbl + (size_t)b.key_idx[i] * C8_WORDS_PER_UNIT;
  base += (size_t)half * 16 * (C8_ENT * C8_STRIDE);
  ge_p3 P;
  ge_p3_0(P);
#if CBFT_COMB8_LDS
  // Table entries are staged through LDS with global_load_lds (no VGPR destination): entry
  // jj+1's 7 x 16 B are requested as soon as entry jj has been read out of LDS, so its HBM /
  // L2 latency overlaps the rest of addition jj (the key tables, 2 GB at 4,096 keys, are read
  // at random; B's table is L2-resident).  LDS image per wave: [chunk 0..6][lane][16 B]
  // (lane-linear, as one global_load_lds_dwordx4 writes it), 7 KB per wave.
  __shared__ uint4 stage[CBFT_VERIFY_BLOCK / 64][7][64];
  uint4(*st)[64] = stage[threadIdx.x >> 6];
  const uint32_t ln = threadIdx.x & 63u;
  auto pop = [&]() {
    const int d = (int)(dw[0] & 0xffu) - 128;
    dw[0] = (dw[0] >> 8) | (dw[1] << 24);
    dw[1] = (dw[1] >> 8) | (dw[2] << 24);
    dw[2] = (dw[2] >> 8) | (dw[3] << 24);
    dw[3] >>= 8;
    return d;
  };
  auto request = [&](const uint32_t* e) {
#pragma unroll
    for (int c = 0; c < 7; c++)
      __builtin_amdgcn_global_load_lds(e + 4 * c, (__attribute__((address_space(3))) void*)&st[c][0], 16, 0, 0);
  };
  int d = pop();
  request(base + (d < 0 ? -d : d) * C8_STRIDE);
#pragma nounroll
  for (int jj = 0; jj < 16; jj++) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t ew[28];
#pragma unroll
    for (int c = 0; c < 7; c++) {
      const uint4 v = st[c][ln];
      ew[4 * c] = v.x;
      ew[4 * c + 1] = v.y;
      ew[4 * c + 2] = v.z;
      ew[4 * c + 3] = v.w;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // entry jj is in VGPRs: the slot is free
    const bool neg = d < 0;
    if (jj < 15) {
      d = pop();
      request(base + ((jj + 1) * C8_ENT + (d < 0 ? -d : d)) * C8_STRIDE);
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
#else
#pragma nounroll
  for (int jj = 0; jj < 16; jj++) {
    const int d = (int)(dw[0] & 0xffu) - 128;
    dw[0] = (dw[0] >> 8) | (dw[1] << 24);
    dw[1] = (dw[1] >> 8) | (dw[2] << 24);
    dw[2] = (dw[2] >> 8) | (dw[3] << 24);
    dw[3] >>= 8;
    const uint32_t* e = base + (jj * C8_ENT + (d < 0 ? -d : d)) * C8_STRIDE;
    ge_p1p1 t;
    ge_add_mem<true>(t, P, e, d < 0);
    fe_mul(P.T, t.X, t.Y);
    fe_mul(P.X, t.X, t.T);
    fe_mul(P.Y, t.Y, t.Z);
    fe_mul(P.Z, t.Z, t.T);
  }
#endif
  quad_combine<0xB1>(P, true);
  quad_combine<0x4E>(P, false);
  if (live && q == 0) {
    fe_store_soa(xyz_soa, b.n, i, P.X);
    fe_store_soa(xyz_soa + 9 * b.n, b.n, i, P.Y);
    fe_store_soa(xyz_soa + 18 * b.n, b.n, i, P.Z);
  }
}

// ---------------------------------------------------------------------------------------
// host-side launch helpers (used by cbft_hipcrypto.cpp)
// ---------------------------------------------------------------------------------------
size_t cbft_ed25519_comb8_words_per_unit() { return (size_t)C8_WORDS_PER_UNIT; }
size_t cbft_ed25519_comb8_tmp_words_per_unit() { return (size_t)C8_POS * C8_TMP_WORDS_PER_LANE; }

hipError_t cbft_ed25519_launch_comb8_tables(const uint8_t* d_pk, size_t nunits, int negate, uint32_t* d_tbl,
                                            uint32_t* d_tmp, uint8_t* d_aok, hipStream_t stream) {
  if (nunits == 0) return hipSuccess;
  const size_t lanes = nunits * C8_POS;
  hipLaunchKernelGGL(ed25519_comb8_table_kernel, dim3((unsigned)((lanes + C8_TABLE_BLOCK - 1) / C8_TABLE_BLOCK)),
                     dim3(C8_TABLE_BLOCK), 0, stream, d_pk, nunits, negate, d_tbl, d_tmp, d_aok);
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
                                      hipEvent_t* ev) {
  if (b.n == 0) return hipSuccess;
  const dim3 grid(grid_for(b.n)), block(CBFT_VERIFY_BLOCK);
  if (ev) (void)hipEventRecord(ev[0], stream);
  hipLaunchKernelGGL(ed25519_hash_kernel, grid, block, 0, stream, b, w.h_soa, w.flags);
  if (ev) (void)hipEventRecord(ev[1], stream);
  if (w.comb_tbl && w.base_comb && b.key_idx)
    hipLaunchKernelGGL(ed25519_comb8_ladder_kernel, dim3((unsigned)((4 * b.n + CBFT_VERIFY_BLOCK - 1) / CBFT_VERIFY_BLOCK)),
                       block, 0, stream, b, w.h_soa, w.comb_tbl, w.base_comb, w.xyz_soa);
  else
    hipLaunchKernelGGL(ed25519_ladder_kernel, grid, block, 0, stream, b, w.h_soa, w.tbl, w.base_table, w.xyz_soa);
  if (ev) (void)hipEventRecord(ev[2], stream);
  hipLaunchKernelGGL(ed25519_finish_kernel, grid, block, 0, stream, b, w.xyz_soa, w.flags, w.aok, w.verdict_words);
  if (ev) (void)hipEventRecord(ev[3], stream);
  return hipGetLastError();
}
