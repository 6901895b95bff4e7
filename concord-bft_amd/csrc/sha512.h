// SHA-512 (FIPS 180-4) for one message per lane, specialised to the Ed25519 challenge
// input R || A || M (RFC 8032 §5.1.7 step 2).  64-bit words are pairs of 32-bit VGPRs;
// rotations lower to v_alignbit_b32 pairs; every 3-input xor, Ch and Maj is one v_bitop3_b32 per half.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __constant__ const uint64_t kSha512K[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull, 0x3956c25bf348b538ull,
    0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull, 0xd807aa98a3030242ull, 0x12835b0145706fbeull,
    0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull, 0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull,
    0xc19bf174cf692694ull, 0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull, 0x983e5152ee66dfabull,
    0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull, 0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull,
    0x06ca6351e003826full, 0x142929670a0e6e70ull, 0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull,
    0x53380d139d95b3dfull, 0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull, 0xd192e819d6ef5218ull,
    0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull, 0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull,
    0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull, 0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull,
    0x682e6ff3d6b2b8a3ull, 0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull, 0xca273eceea26619cull,
    0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull, 0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull,
    0x113f9804bef90daeull, 0x1b710b35131c471bull, 0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull,
    0x431d67c49c100d4cull, 0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// 64-bit rotate as two v_alignbit_b32 on the 32-bit halves (N is a compile-time constant)
template <int N>
__device__ __forceinline__ uint64_t rotr64(uint64_t x) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  uint32_t rl, rh;
  if (N < 32) {
    rl = __builtin_amdgcn_alignbit(hi, lo, N);
    rh = __builtin_amdgcn_alignbit(lo, hi, N);
  } else {
    rl = __builtin_amdgcn_alignbit(lo, hi, N - 32);
    rh = __builtin_amdgcn_alignbit(hi, lo, N - 32);
  }
  return ((uint64_t)rh << 32) | rl;
}

// gfx950 v_bitop3_b32: any 3-input boolean function in one instruction; the truth table is
// indexed by (S0, S1, S2) with S0 <-> 0xf0, S1 <-> 0xcc, S2 <-> 0xaa (0x96 = xor3, 0xe8 = majority,
// 0xca = S0 ? S1 : S2).  The compiler does not form it from a ^ b ^ c by itself.
template <uint32_t T>
__device__ __forceinline__ uint64_t bitop3_64(uint64_t a, uint64_t b, uint64_t c) {
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, T);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), T);
  uint64_t r = ((uint64_t)hi << 32) | lo;
#if defined(__HIP_DEVICE_COMPILE__)
  // one 64-bit value in a register pair: otherwise LLVM splits the following 64-bit adds into
  // zero-extended halves (~6 v_mov + 4 extra v_lshl_add_u64 per 16 rounds' schedule words)
  asm("" : "+v"(r));
#endif
  return r;
}
// x >> N (64-bit, N < 32) as v_alignbit_b32 + v_lshrrev_b32
template <int N>
__device__ __forceinline__ uint64_t shr64(uint64_t x) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return ((uint64_t)(hi >> N) << 32) | __builtin_amdgcn_alignbit(hi, lo, N);
}

#define SHA512_ROUND(a, b, c, d, e, f, g, h, kw)                                          \
  do {                                                                                    \
    const uint64_t S1_ = bitop3_64<0x96>(rotr64<14>(e), rotr64<18>(e), rotr64<41>(e));    \
    const uint64_t ch_ = bitop3_64<0xca>(e, f, g);                                        \
    const uint64_t t1_ = h + S1_ + ch_ + (kw);                                            \
    const uint64_t S0_ = bitop3_64<0x96>(rotr64<28>(a), rotr64<34>(a), rotr64<39>(a));    \
    const uint64_t mj_ = bitop3_64<0xe8>(a, b, c);                                        \
    d += t1_;                                                                             \
    h = t1_ + S0_ + mj_;                                                                  \
  } while (0)


// Rounds 0-15 straight from the block, then 4 x 16 rounds with the message schedule in a
// 16-word ring (no data-dependent control flow: an `if (r > 0)` inside the unrolled window
// made the compiler copy the whole ring every round).  The 8 working variables rotate by
// renaming (8 divides 16), so the window loop has no moves at its back edge.
__device__ __forceinline__ void sha512_compress(uint64_t* H, uint64_t* W) {
  uint64_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma unroll
  for (int j = 0; j < 16; j += 8) {
    SHA512_ROUND(a, b, c, d, e, f, g, h, kSha512K[j + 0] + W[j + 0]);
    SHA512_ROUND(h, a, b, c, d, e, f, g, kSha512K[j + 1] + W[j + 1]);
    SHA512_ROUND(g, h, a, b, c, d, e, f, kSha512K[j + 2] + W[j + 2]);
    SHA512_ROUND(f, g, h, a, b, c, d, e, kSha512K[j + 3] + W[j + 3]);
    SHA512_ROUND(e, f, g, h, a, b, c, d, kSha512K[j + 4] + W[j + 4]);
    SHA512_ROUND(d, e, f, g, h, a, b, c, kSha512K[j + 5] + W[j + 5]);
    SHA512_ROUND(c, d, e, f, g, h, a, b, kSha512K[j + 6] + W[j + 6]);
    SHA512_ROUND(b, c, d, e, f, g, h, a, kSha512K[j + 7] + W[j + 7]);
  }
#pragma nounroll
  for (int r = 16; r < 80; r += 16) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint64_t w15 = W[(j + 1) & 15], w2 = W[(j + 14) & 15];
      const uint64_t s0 = bitop3_64<0x96>(rotr64<1>(w15), rotr64<8>(w15), shr64<7>(w15));
      const uint64_t s1 = bitop3_64<0x96>(rotr64<19>(w2), rotr64<61>(w2), shr64<6>(w2));
      W[j] = W[j] + s0 + W[(j + 9) & 15] + s1;
    }
#pragma unroll
    for (int j = 0; j < 16; j += 8) {
      SHA512_ROUND(a, b, c, d, e, f, g, h, kSha512K[r + j + 0] + W[j + 0]);
      SHA512_ROUND(h, a, b, c, d, e, f, g, kSha512K[r + j + 1] + W[j + 1]);
      SHA512_ROUND(g, h, a, b, c, d, e, f, kSha512K[r + j + 2] + W[j + 2]);
      SHA512_ROUND(f, g, h, a, b, c, d, e, kSha512K[r + j + 3] + W[j + 3]);
      SHA512_ROUND(e, f, g, h, a, b, c, d, kSha512K[r + j + 4] + W[j + 4]);
      SHA512_ROUND(d, e, f, g, h, a, b, c, kSha512K[r + j + 5] + W[j + 5]);
      SHA512_ROUND(c, d, e, f, g, h, a, b, kSha512K[r + j + 6] + W[j + 6]);
      SHA512_ROUND(b, c, d, e, f, g, h, a, kSha512K[r + j + 7] + W[j + 7]);
    }
  }
  H[0] += a;
  H[1] += b;
  H[2] += c;
  H[3] += d;
  H[4] += e;
  H[5] += f;
  H[6] += g;
  H[7] += h;
}

// The compression function in two halves that two waves can run: sha512_schedule_kw expands a
// block's 16 words into kw[t] = K[t] + W[t], t = 0..79 (one wave writes them to LDS), and
// sha512_rounds_kw runs the 80 rounds from kw (another wave, reading LDS): the rounds' wave skips
// the schedule's ~1,400 instructions per block, a third of the compression.
__device__ __forceinline__ void sha512_schedule_kw(uint64_t* kw, uint64_t* W) {
#pragma unroll
  for (int j = 0; j < 16; j++) kw[j] = kSha512K[j] + W[j];
#pragma nounroll
  for (int r = 16; r < 80; r += 16) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint64_t w15 = W[(j + 1) & 15], w2 = W[(j + 14) & 15];
      const uint64_t s0 = bitop3_64<0x96>(rotr64<1>(w15), rotr64<8>(w15), shr64<7>(w15));
      const uint64_t s1 = bitop3_64<0x96>(rotr64<19>(w2), rotr64<61>(w2), shr64<6>(w2));
      W[j] = W[j] + s0 + W[(j + 9) & 15] + s1;
      kw[r + j] = kSha512K[r + j] + W[j];
    }
  }
}
__device__ __forceinline__ void sha512_rounds_kw(uint64_t* H, const uint64_t* kw) {
  uint64_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma nounroll
  for (int r = 0; r < 80; r += 16) {
    uint64_t k[16];
#pragma unroll
    for (int j = 0; j < 16; j++) k[j] = kw[r + j];
#pragma unroll
    for (int j = 0; j < 16; j += 8) {
      SHA512_ROUND(a, b, c, d, e, f, g, h, k[j + 0]);
      SHA512_ROUND(h, a, b, c, d, e, f, g, k[j + 1]);
      SHA512_ROUND(g, h, a, b, c, d, e, f, k[j + 2]);
      SHA512_ROUND(f, g, h, a, b, c, d, e, k[j + 3]);
      SHA512_ROUND(e, f, g, h, a, b, c, d, k[j + 4]);
      SHA512_ROUND(d, e, f, g, h, a, b, c, k[j + 5]);
      SHA512_ROUND(c, d, e, f, g, h, a, b, k[j + 6]);
      SHA512_ROUND(b, c, d, e, f, g, h, a, k[j + 7]);
    }
  }
  H[0] += a;
  H[1] += b;
  H[2] += c;
  H[3] += d;
  H[4] += e;
  H[5] += f;
  H[6] += g;
  H[7] += h;
}

__device__ __forceinline__ void sha512_init(uint64_t* H) {
  H[0] = 0x6a09e667f3bcc908ull;
  H[1] = 0xbb67ae8584caa73bull;
  H[2] = 0x3c6ef372fe94f82bull;
  H[3] = 0xa54ff53a5f1d36f1ull;
  H[4] = 0x510e527fade682d1ull;
  H[5] = 0x9b05688c2b3e6c1full;
  H[6] = 0x1f83d9abfb41bd6bull;
  H[7] = 0x5be0cd19137e2179ull;
}

// Byte q of (M || 0x80 || 0...), q relative to the start of M.
__device__ __forceinline__ uint32_t msg_pad_byte(const uint8_t* m, uint32_t len, uint32_t q) {
  return q < len ? (uint32_t)m[q] : (q == len ? 0x80u : 0u);
}

// Big-endian 64-bit word of (M || 0x80 || 0...) at M-relative byte offset q.
__device__ __forceinline__ uint64_t msg_word(const uint8_t* m, uint32_t len, uint32_t q) {
  uint64_t w = 0;
  if (q + 8 <= len) {
#pragma unroll
    for (int k = 0; k < 8; k++) w = (w << 8) | m[q + k];
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++) w = (w << 8) | msg_pad_byte(m, len, q + k);
  }
  return w;
}

// h = SHA-512(R || A || M) as a 512-bit little-endian integer in 16 words.
//   R, A: 8 little-endian 32-bit words each (the raw wire bytes).
__device__ __forceinline__ void sha512_ram(uint32_t* out16, const uint32_t* R, const uint32_t* A, const uint8_t* m,
                                           uint32_t len) {
  uint64_t H[8], W[16];
  sha512_init(H);
  const uint32_t total = 64u + len;                 // bytes hashed
  const uint32_t nblocks = (total + 17u + 127u) / 128u;
  for (uint32_t b = 0; b < nblocks; b++) {
    if (b == 0) {  // block 0: R || A || M[0..63]
#pragma unroll
      for (int j = 0; j < 4; j++) W[j] = ((uint64_t)bswap32(R[2 * j]) << 32) | bswap32(R[2 * j + 1]);
#pragma unroll
      for (int j = 0; j < 4; j++) W[4 + j] = ((uint64_t)bswap32(A[2 * j]) << 32) | bswap32(A[2 * j + 1]);
#pragma unroll
      for (int j = 8; j < 16; j++) W[j] = msg_word(m, len, (uint32_t)(8 * j - 64));
    } else {
      const uint32_t base = 128u * b - 64u;  // M-relative offset of this block
#pragma unroll
      for (int j = 0; j < 16; j++) W[j] = msg_word(m, len, base + 8u * j);
    }
    if (b == nblocks - 1) {
      W[14] = 0;
      W[15] = (uint64_t)total << 3;
    }
    sha512_compress(H, W);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    out16[2 * i] = bswap32((uint32_t)(H[i] >> 32));
    out16[2 * i + 1] = bswap32((uint32_t)H[i]);
  }
}
