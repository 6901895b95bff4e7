// BLS operations on BN-P254 shared by the GPU kernels and the host build (hash-to-G1, share
// parsing).  Semantics as restated in oracle/bn254_ref.py (RELIC conventions: parity unpinned).
#pragma once
#include "bn254_pairing.h"
#include "sha256.h"

// RELIC 2019-era ep_map: x = SHA-256(msg) (big-endian) mod p, try-and-increment until
// x^3 + 2 is a square, y = (x^3 + 2)^((p+1)/4).  (BlsAccumulatorBase.cpp:59, BlsThresholdVerifier.cpp:72)
BN_HDN void g1_map(g1a& r, const uint8_t* msg, uint32_t len) {
  uint8_t d[32];
  sha256(d, msg, len);
  uint32_t w[8];
  be32_to_words(w, d);
  fp x, one, two, rhs;
  f_from_words(x, w);  // any 256-bit value: Montgomery of (w mod p)
  uint32_t t[8] = {2, 0, 0, 0, 0, 0, 0, 0};
  f_from_words(two, t);
  f_one(one);
  for (;;) {
    f_sqr(rhs, x);
    f_mul(rhs, rhs, x);
    f_add(rhs, rhs, two);
    if (fp_sqrt(r.y, rhs)) break;
    f_add(x, x, one);
  }
  r.x = x;
  r.inf = false;
}

// 37-byte share: 4-byte big-endian id || 33-byte compressed G1 (BlsSigshareParser,
// BlsAccumulatorBase.cpp:33-43; BlsThresholdSigner.cpp:32-47)
BN_HD bool bls_parse_share(uint32_t& id, g1a& s, const uint8_t* b) {
  id = ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
  return g1_decompress(s, b + 4);
}
