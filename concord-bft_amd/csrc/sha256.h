// SHA-256 (FIPS 180-4), host + device, for RELIC's g1_map (md_map = SHA-256 in the reference
// build, thirdparty/relic.cmake:6-35).  Short messages only (the reference hashes 32-byte
// digests); one message per call.
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifndef BN_HD  // same definition as bn254_field.h (identical redefinition is allowed)
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BN_HD __host__ __device__ __forceinline__
#else
#define BN_HD inline
#endif
#endif

BN_HD uint32_t sha256_rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

BN_HD void sha256_block(uint32_t* h, const uint32_t* blk) {
  const uint32_t K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
  uint32_t w[64];
  for (int t = 0; t < 16; t++) w[t] = blk[t];
  for (int t = 16; t < 64; t++) {
    uint32_t s0 = sha256_rotr(w[t - 15], 7) ^ sha256_rotr(w[t - 15], 18) ^ (w[t - 15] >> 3);
    uint32_t s1 = sha256_rotr(w[t - 2], 17) ^ sha256_rotr(w[t - 2], 19) ^ (w[t - 2] >> 10);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int t = 0; t < 64; t++) {
    uint32_t S1 = sha256_rotr(e, 6) ^ sha256_rotr(e, 11) ^ sha256_rotr(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = hh + S1 + ch + K[t] + w[t];
    uint32_t S0 = sha256_rotr(a, 2) ^ sha256_rotr(a, 13) ^ sha256_rotr(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + S0 + mj;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
  h[5] += f;
  h[6] += g;
  h[7] += hh;
}

// out = SHA-256(msg[0..len)), len < 2^29
BN_HD void sha256(uint8_t* out, const uint8_t* msg, uint32_t len) {
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  const uint32_t nblk = (len + 9 + 63) / 64;
  for (uint32_t b = 0; b < nblk; b++) {
    uint32_t blk[16];
    for (int j = 0; j < 16; j++) {
      uint32_t w = 0;
      for (int k = 0; k < 4; k++) {
        const uint32_t pos = 64 * b + 4 * j + k;
        uint32_t byte = pos < len ? msg[pos] : (pos == len ? 0x80u : 0u);
        w = (w << 8) | byte;
      }
      blk[j] = w;
    }
    if (b == nblk - 1) {
      blk[14] = len >> 29;
      blk[15] = len << 3;
    }
    sha256_block(h, blk);
  }
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)(h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(h[i] >> 8);
    out[4 * i + 3] = (uint8_t)h[i];
  }
}

BN_HD uint32_t sha256_bswap(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

// h = SHA-256 state after hashing K || msg[0 .. m), m <= 64, where K is the 32 little-endian bytes
// of key[0..8) each xored with x.  Every block word is built at a compile-time index, so the
// padded message stays in registers (sha256() over a byte-indexed local buffer of run-time length
// lives in scratch memory on the GPU: ~2,200 instructions of byte addressing per block).  The
// digest bytes are the big-endian bytes of h[0..8).
BN_HD void sha256_key_msg(uint32_t* h, const uint32_t* key, uint8_t x, const uint8_t* msg, uint32_t m) {
  const uint32_t h0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                          0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  for (int i = 0; i < 8; i++) h[i] = h0[i];
  const uint32_t xx = 0x01010101u * x, total = 32u + m, nblk = (total + 9u + 63u) / 64u;
  uint32_t blk[32];
#pragma unroll
  for (int j = 0; j < 32; j++) {
    uint32_t w = 0;
    if (j < 8) {
      w = sha256_bswap(key[j] ^ xx);
    } else {
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t pos = (uint32_t)(4 * j + q - 32);
        const uint32_t byte = pos < m ? msg[pos] : (pos == m ? 0x80u : 0u);
        w = (w << 8) | byte;
      }
    }
    blk[j] = w;
  }
  if (nblk == 1) {
    blk[14] = 0;
    blk[15] = total << 3;
  } else {
    blk[30] = 0;
    blk[31] = total << 3;
  }
  sha256_block(h, blk);
  if (nblk == 2) sha256_block(h, blk + 16);
}
