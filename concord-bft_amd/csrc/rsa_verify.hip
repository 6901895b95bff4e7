// RSA-2048 PKCS#1 v1.5 / SHA-256 batch verification on gfx950.
//
// What it replaces: concord::util::crypto::RSAVerifier::verify (util/src/crypto_utils.cpp:
// 101-117,166) — Crypto++ 8.2.0 RSASS<PKCS1v15, SHA256>::Verifier::VerifyMessage, which
// SigManager instantiates for every replica and client key today (SigManager.cpp:138,146,255).
// Verdict = ((s mod n)^e mod n == 00 01 FF.. 00 || DigestInfo(SHA-256) || SHA-256(m)), exactly as
// oracle/rsa_ref.py restates it (s is not range-checked against n, as in Crypto++).
//
// Design: big-integer work with a 32-bit multiply at its core — no MFMA.  One lane
// per signature; the 2048-bit operand b and the modulus stay in VGPRs for the whole
// exponentiation (64 + 64 + 65 accumulator registers, two waves per SIMD), the row operand a_i is
// read from LDS (this lane's own column, conflict-free) or, for the multiply by s, from a
// coalesced [limb][signature] scratch array.  Montgomery products use the two-carry FIOS form:
// per (i, j) two v_mad_u64_u32 with independent carry chains c1 (a*b) and c2 (m*n), so a row's
// two chains interleave and a wave carries no cross-lane traffic at all.  Lanes of one wave may
// hold different exponents (e = 17 replica keys next to e = 65537 client keys): the
// square-and-multiply schedule runs over the wave's highest exponent bit and masks the
// multiplies per lane.
#include <hip/hip_runtime.h>

#include "rsa_verify.h"
#include "sha256.h"

namespace {

constexpr int L = RSA_LIMBS;

// EMSA-PKCS1-v1_5 representative for SHA-256 at 2048 bits, bytes 0..223 (the last 32 are the
// digest): 00 01 FF*202 00 || 3031300d060960864801650304020105000420.
__device__ __forceinline__ uint32_t em_byte(int p) {
  const uint8_t di[19] = {0x30, 0x31, 0x30, 0x0d, 0x06, 0x09, 0x60, 0x86, 0x48, 0x01,
                          0x65, 0x03, 0x04, 0x02, 0x01, 0x05, 0x00, 0x04, 0x20};
  if (p == 0) return 0x00;
  if (p == 1) return 0x01;
  if (p < 204) return 0xff;
  if (p == 204) return 0x00;
  return di[p - 205];
}
// limb k (little-endian 32-bit) of the representative, 8 <= k < 64
__device__ __forceinline__ uint32_t em_limb(int k) {
  const int p = 252 - 4 * k;
  return (em_byte(p) << 24) | (em_byte(p + 1) << 16) | (em_byte(p + 2) << 8) | em_byte(p + 3);
}

// a * b + c on v_mad_u64_u32.  Inline asm keeps the compiler from hoisting zero-extended 64-bit
// copies of the loop-invariant modulus limbs out of the row loop (they would need 64 more
// registers and spill).
__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r, carry_mask;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(carry_mask) : "v"(a), "v"(b), "v"(c));
  return r;
}

// a + b as a 64-bit value (carry in the high word).  The carry is materialised with
// v_addc_co_u32 (VCC read as carry-in, no wait states) instead of the compiler's v_cndmask
// (VCC read as a lane mask after a VALU write needs two wait states: 2 s_nop per product).
__device__ __forceinline__ uint64_t add32x2(uint32_t a, uint32_t b) {
  uint32_t lo, hi;
  asm("v_add_co_u32 %0, vcc, %2, %3\n\tv_addc_co_u32 %1, vcc, 0, 0, vcc" : "=&v"(lo), "=v"(hi) : "v"(a), "v"(b) : "vcc");
  return ((uint64_t)hi << 32) | lo;
}

// Montgomery product t = a * x * 2^-2048 mod n (fully reduced), written back into x for the lanes
// with `take` set.  x lives in LDS in this lane's own column (xl[q][lane] holds limbs 4q..4q+3);
// a(i) returns limb i of the row operand; the modulus stays in registers.
template <class ARow>
__device__ __forceinline__ void mont_mul(uint4 (*xl)[CBFT_RSA_BLOCK], uint32_t lane, const uint32_t (&nn)[L],
                                         uint32_t n0inv, ARow a, bool take) {
  uint32_t t[L + 1];
#pragma unroll
  for (int j = 0; j <= L; j++) t[j] = 0;
  uint32_t a_next = a(0);
#pragma unroll 1
  for (int i = 0; i < L; i++) {
    // keep the x limbs streaming from LDS row by row (hoisting them out of the loop would need
    // 64 more VGPRs than a two-wave-per-SIMD budget has)
    asm volatile("" ::: "memory");
    const uint32_t ai = a_next;
    if (i + 1 < L) a_next = a(i + 1);  // the next row operand (maybe a global load) overlaps this row
    uint64_t c1 = 0, c2 = 0;
    uint32_t m = 0;
#if CBFT_RSA_PREFETCH
    uint4 nxt = xl[0][lane];
#endif
#pragma unroll
    for (int q = 0; q < L / 4; q++) {
#if CBFT_RSA_PREFETCH
      const uint4 b4 = nxt;  // x limbs 4q..4q+3; the next group's LDS read is in flight meanwhile
      if (q + 1 < L / 4) nxt = xl[q + 1][lane];
#else
      const uint4 b4 = xl[q][lane];
#endif
      const uint32_t bv[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int j = 4 * q + r;
        if (j == 0) {
          const uint64_t X = mad64(ai, bv[0], add32x2(t[0], 0u));
          m = (uint32_t)X * n0inv;
          const uint64_t Y = mad64(m, nn[0], add32x2((uint32_t)X, 0u));  // low word is 0
          c1 = X >> 32;
          c2 = Y >> 32;
        } else {
          // X = ai b_j + t_j + c1 <= (2^32-1)^2 + 2 (2^32-1) = 2^64 - 1; two independent carry
          // chains (a*b and m*n) per row
          const uint64_t X = mad64(ai, bv[r], add32x2(t[j], (uint32_t)c1));
          const uint64_t Y = mad64(m, nn[j], add32x2((uint32_t)X, (uint32_t)c2));
          c1 = X >> 32;
          c2 = Y >> 32;
          t[j - 1] = (uint32_t)Y;
        }
      }
    }
    unsigned int k1, k2;
    const uint32_t s1 = __builtin_addc(t[L], (uint32_t)c1, 0u, &k1);
    t[L - 1] = __builtin_addc(s1, (uint32_t)c2, 0u, &k2);
    t[L] = k1 + k2;
  }
  // t < 2n: subtract n once if t >= n.  First pass: the borrow only; second pass: select.
  unsigned int br = 0;
#pragma unroll
  for (int j = 0; j < L; j++) (void)__builtin_subc(t[j], nn[j], br, &br);
  const bool ge = t[L] != 0 || br == 0;
  if (!take) return;
  br = 0;
#pragma unroll
  for (int q = 0; q < L / 4; q++) {
    uint32_t r[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t d = __builtin_subc(t[4 * q + k], nn[4 * q + k], br, &br);
      r[k] = ge ? d : t[4 * q + k];
    }
    xl[q][lane] = make_uint4(r[0], r[1], r[2], r[3]);
  }
}

__device__ __forceinline__ uint32_t load_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

// SHA-256 of msg[0..len) into eight big-endian state words (FIPS 180-4; compression from sha256.h)
__device__ __forceinline__ void sha256_words(uint32_t (&h)[8], const uint8_t* msg, uint32_t len) {
  h[0] = 0x6a09e667u, h[1] = 0xbb67ae85u, h[2] = 0x3c6ef372u, h[3] = 0xa54ff53au;
  h[4] = 0x510e527fu, h[5] = 0x9b05688cu, h[6] = 0x1f83d9abu, h[7] = 0x5be0cd19u;
  const uint32_t nblk = (len + 9 + 63) / 64;
  for (uint32_t bk = 0; bk < nblk; bk++) {
    uint32_t blk[16];
    const uint32_t base = 64 * bk;
    if (base + 64 <= len) {
#pragma unroll
      for (int j = 0; j < 16; j++) blk[j] = load_be32(msg + base + 4 * j);
    } else {
#pragma unroll
      for (int j = 0; j < 16; j++) {
        uint32_t w = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint32_t pos = base + 4 * j + q;
          const uint32_t byte = pos < len ? msg[pos] : (pos == len ? 0x80u : 0u);
          w = (w << 8) | byte;
        }
        blk[j] = w;
      }
      if (bk == nblk - 1) {
        blk[14] = len >> 29;
        blk[15] = len << 3;
      }
    }
    sha256_block(h, blk);
  }
}

// ---------------------------------------------------------------- key records ----------------
// One lane per key: n from big-endian bytes, n0inv = -n^-1 mod 2^32 (Newton), R^2 mod n by 2048
// modular doublings of R mod n = 2^2048 - n (n has its top bit set), validity flag.
__global__ void __launch_bounds__(64) rsa_keys_kernel(const uint8_t* mod, const uint32_t* exps, uint32_t nkeys,
                                                      uint32_t* keys) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nkeys) return;
  const uint8_t* m = mod + (size_t)k * RSA_MOD_BYTES;
  uint32_t* rec = keys + (size_t)k * RSA_KEY_WORDS;
  uint32_t n[L], x[L];
  for (int i = 0; i < L; i++) n[i] = load_be32(m + RSA_MOD_BYTES - 4 * (i + 1));
  const uint32_t e = exps[k];
  const bool ok = (n[0] & 1u) && (n[L - 1] >> 31) && (e & 1u) && e >= 3u;
  uint32_t inv = n[0];  // n0 * inv == 1 mod 2^3 for odd n0; 4 Newton steps reach 2^48
  for (int it = 0; it < 4; it++) inv *= 2u - n[0] * inv;
  // x = 2^2048 - n
  uint32_t br = 0;
  for (int i = 0; i < L; i++) {
    const uint64_t d = 0ull - n[i] - br;
    x[i] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
  for (int it = 0; it < 2048; it++) {  // x = 2 x mod n
    uint32_t top = x[L - 1] >> 31;
    for (int i = L - 1; i > 0; i--) x[i] = (x[i] << 1) | (x[i - 1] >> 31);
    x[0] <<= 1;
    uint32_t b2 = 0;
    for (int i = 0; i < L; i++) {
      const uint64_t d = (uint64_t)x[i] - n[i] - b2;
      b2 = (uint32_t)(d >> 63);
    }
    const bool ge = top || b2 == 0;
    b2 = 0;
    for (int i = 0; i < L; i++) {
      const uint64_t d = (uint64_t)x[i] - n[i] - b2;
      b2 = (uint32_t)(d >> 63);
      x[i] = ge ? (uint32_t)d : x[i];
    }
  }
  for (int i = 0; i < L; i++) {
    rec[RSA_KEY_N + i] = n[i];
    rec[RSA_KEY_R2 + i] = ok ? x[i] : 0u;
  }
  rec[RSA_KEY_N0INV] = 0u - inv;
  rec[RSA_KEY_E] = e;
  rec[RSA_KEY_OK] = ok ? 1u : 0u;
  for (int i = RSA_KEY_OK + 1; i < RSA_KEY_WORDS; i++) rec[i] = 0;
}

// ---------------------------------------------------------------- verify ---------------------
__global__ void __launch_bounds__(CBFT_RSA_BLOCK, CBFT_RSA_MIN_WAVES) rsa_verify_kernel(const RsaBatch b, uint32_t* scratch,
                                                                    uint64_t* verdicts) {
  __shared__ uint4 xl[L / 4][CBFT_RSA_BLOCK];  // the running operand x, [limb/4][lane] (conflict-free)
  const uint32_t tid = threadIdx.x;
  const size_t idx = (size_t)blockIdx.x * CBFT_RSA_BLOCK + tid;
  const size_t stride = (size_t)gridDim.x * CBFT_RSA_BLOCK;  // scratch row pitch
  const bool live = idx < b.n;
  const size_t si = live ? idx : 0;
  uint32_t kidx = b.key_idx[si];
  bool ok = live && kidx < b.nkeys;
  if (kidx >= b.nkeys) kidx = 0;
  const uint32_t* rec = b.keys + (size_t)kidx * RSA_KEY_WORDS;

  uint32_t nn[L];
#pragma unroll
  for (int q = 0; q < L / 4; q++) {
    const uint4 v = *reinterpret_cast<const uint4*>(rec + RSA_KEY_N + 4 * q);
    nn[4 * q] = v.x, nn[4 * q + 1] = v.y, nn[4 * q + 2] = v.z, nn[4 * q + 3] = v.w;
    xl[q][tid] = *reinterpret_cast<const uint4*>(rec + RSA_KEY_R2 + 4 * q);  // x = R^2 mod n
  }
  const uint32_t n0inv = rec[RSA_KEY_N0INV];
  const uint32_t e = ok ? rec[RSA_KEY_E] : 0u;
  ok = ok && rec[RSA_KEY_OK];
  const uint8_t* sg = b.sig + si * RSA_MOD_BYTES;

  // The wave's highest exponent bit (lanes may hold different e).
  int top = -1;
  if (__ballot(e != 0)) {
    for (int bit = 31; bit >= 0; bit--)
      if (__ballot((e >> bit) & 1u)) {
        top = bit;
        break;
      }
  }
  // One Montgomery-product call site drives the whole schedule (a single inlined copy):
  //   CONV  sm = s * R^2 * R^-1 = s R        a = s (signature bytes), then sm -> scratch, x = R mod n
  //   MUL   x = x * sm  (lanes with bit set)  a = sm (scratch, coalesced [limb][signature])
  //   SQR   x = x * x                         a = x (LDS)
  //   REDC  x = x * 1 * R^-1                  a = 1
  enum { CONV, MUL, SQR, REDC };
  int op = CONV, bit = top;
  for (;;) {
    const bool take = op != MUL || ((e >> bit) & 1u);
    mont_mul(
        xl, tid, nn, n0inv,
        [&](int i) -> uint32_t {
          if (op == MUL) return scratch[(size_t)i * stride + idx];
          if (op == REDC) return i == 0 ? 1u : 0u;
          if (op == CONV)  // limb i of s: big-endian word 63 - i of the (4-byte aligned) signature
            return __builtin_bswap32(*reinterpret_cast<const uint32_t*>(sg + RSA_MOD_BYTES - 4 * (i + 1)));
          const uint4 v = xl[i >> 2][tid];
          const int r = i & 3;
          return r == 0 ? v.x : r == 1 ? v.y : r == 2 ? v.z : v.w;
        },
        take);
    if (op == REDC) break;
    if (op == CONV) {
      unsigned int br = 0;  // sm -> scratch; x = R mod n = 2^2048 - n (Montgomery 1)
#pragma unroll
      for (int q = 0; q < L / 4; q++) {
        const uint4 v = xl[q][tid];
        scratch[(size_t)(4 * q) * stride + idx] = v.x;
        scratch[(size_t)(4 * q + 1) * stride + idx] = v.y;
        scratch[(size_t)(4 * q + 2) * stride + idx] = v.z;
        scratch[(size_t)(4 * q + 3) * stride + idx] = v.w;
        uint32_t r[4];
#pragma unroll
        for (int k = 0; k < 4; k++) r[k] = __builtin_subc(0u, nn[4 * q + k], br, &br);
        xl[q][tid] = make_uint4(r[0], r[1], r[2], r[3]);
      }
      op = top >= 0 ? MUL : REDC;  // the top bit is set in some lane: x = 1 * sm there
      continue;
    }
    // after MUL or SQR at `bit`: square for the next bit, multiplying where it is set
    if (op == SQR && __ballot((e >> bit) & 1u)) {
      op = MUL;
      continue;
    }
    if (bit == 0) {
      op = REDC;
      continue;
    }
    bit--;
    op = SQR;
  }

  // SHA-256 of the message (PKCS1v15 encodes the digest; crypto_utils.cpp:103 SHA256)
  uint32_t hw[8];
  sha256_words(hw, b.msg + (live ? b.msg_off[si] : 0), live ? b.msg_len[si] : 0);

  // compare x with the encoded digest
  bool eq = true;
#pragma unroll
  for (int q = 0; q < L / 4; q++) {
    const uint4 v = xl[q][tid];
    const uint32_t xv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int j = 4 * q + k;
      eq = eq && xv[k] == (j < 8 ? hw[7 - j] : em_limb(j));
    }
  }
  const uint64_t word = __ballot(ok && eq);
  if ((tid & 63) == 0 && idx < b.n) verdicts[idx >> 6] = word;
}

}  // namespace

size_t cbft_rsa_scratch_words(size_t n) {
  const size_t blocks = (n + CBFT_RSA_BLOCK - 1) / CBFT_RSA_BLOCK;
  return (size_t)RSA_LIMBS * blocks * CBFT_RSA_BLOCK;
}

hipError_t cbft_rsa_launch_keys(const uint8_t* d_mod, const uint32_t* d_exp, uint32_t nkeys, uint32_t* d_keys,
                                hipStream_t stream) {
  if (!nkeys) return hipSuccess;
  hipLaunchKernelGGL(rsa_keys_kernel, dim3((nkeys + 63) / 64), dim3(64), 0, stream, d_mod, d_exp, nkeys, d_keys);
  return hipGetLastError();
}

hipError_t cbft_rsa_launch_verify(const RsaBatch& b, uint32_t* d_scratch, uint64_t* d_verdicts, hipStream_t stream) {
  if (!b.n) return hipSuccess;
  const unsigned blocks = (unsigned)((b.n + CBFT_RSA_BLOCK - 1) / CBFT_RSA_BLOCK);
  hipLaunchKernelGGL(rsa_verify_kernel, dim3(blocks), dim3(CBFT_RSA_BLOCK), 0, stream, b, d_scratch, d_verdicts);
  return hipGetLastError();
}
