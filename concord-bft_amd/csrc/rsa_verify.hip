// RSA-2048 PKCS#1 v1.5 / SHA-256 batch verification on gfx950.
//
// What it replaces: concord::util::crypto::RSAVerifier::verify (util/src/crypto_utils.cpp:
// 101-117,166) — Crypto++ 8.2.0 RSASS<PKCS1v15, SHA256>::Verifier::VerifyMessage, which
// SigManager instantiates for every replica and client key today (SigManager.cpp:138,146,255).
// Verdict = ((s mod n)^e mod n == 00 01 FF.. 00 || DigestInfo(SHA-256) || SHA-256(m)), exactly as
// oracle/rsa_ref.py restates it (s is not range-checked against n, as in Crypto++).
//
// Design: big-integer work with a 32-bit multiply at its core — no MFMA.  Two lanes
// per signature, radix 2^28 (rsa_verify_pair_kernel below): each Montgomery row is one
// v_mad_u64_u32 per column for a*x and one for m*n with no per-column carry instructions.  Lanes
// of one wave may hold different exponents (e = 17 replica keys next to e = 65537 client keys):
// the square-and-multiply schedule runs over the wave's highest exponent bit and masks the
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
__device__ void mod_double(uint32_t (&x)[L], const uint32_t (&n)[L]) {  // x = 2 x mod n, x < n
  const uint32_t top = x[L - 1] >> 31;
  for (int i = L - 1; i > 0; i--) x[i] = (x[i] << 1) | (x[i - 1] >> 31);
  x[0] <<= 1;
  unsigned int b2 = 0;
  for (int i = 0; i < L; i++) (void)__builtin_subc(x[i], n[i], b2, &b2);
  const bool ge = top || b2 == 0;
  b2 = 0;
  for (int i = 0; i < L; i++) {
    const uint32_t d = __builtin_subc(x[i], n[i], b2, &b2);
    x[i] = ge ? d : x[i];
  }
}

// 28-bit limb i of a number given as 32-bit little-endian words
__device__ __forceinline__ uint32_t limb28(const uint32_t (&w)[L], int i) {
  const int o = 28 * i, k = o >> 5, sh = o & 31;
  const uint64_t lo = k < L ? w[k] : 0u, hi = k + 1 < L ? w[k + 1] : 0u;
  return (uint32_t)(((hi << 32) | lo) >> sh) & ((1u << 28) - 1);
}

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
  // x = 2^2048 mod n; 24 doublings -> R' mod n (R' = 2^2072); 2024 more -> R^2 = 2^4096 mod n;
  // 48 more -> R'^2 = 2^4144 mod n
  uint32_t* p = rec + RSA_KEY_P_N;
  for (int i = 0; i < RSA_PL; i++) p[i] = i < RSA_NL ? limb28(n, i) : 0u;
  for (int it = 0; it < 2096; it++) {
    mod_double(x, n);
    if (it == 23)
      for (int i = 0; i < RSA_PL; i++) rec[RSA_KEY_P_R1 + i] = (ok && i < RSA_NL) ? limb28(x, i) : 0u;
    if (it == 2047)
      for (int i = 0; i < L; i++) rec[RSA_KEY_R2 + i] = ok ? x[i] : 0u;
  }
  for (int i = 0; i < RSA_PL; i++) rec[RSA_KEY_P_R2 + i] = (ok && i < RSA_NL) ? limb28(x, i) : 0u;
  for (int i = 0; i < L; i++) rec[RSA_KEY_N + i] = n[i];
  rec[RSA_KEY_N0INV] = 0u - inv;
  rec[RSA_KEY_E] = e;
  rec[RSA_KEY_OK] = ok ? 1u : 0u;
  for (int i = RSA_KEY_OK + 1; i < RSA_KEY_P_N; i++) rec[i] = 0;
  rec[RSA_KEY_P_N0INV] = (0u - inv) & ((1u << 28) - 1);
  for (int i = RSA_KEY_P_N0INV + 1; i < RSA_KEY_WORDS; i++) rec[i] = 0;
}


// ---------------------------------------------------------------- lane-pair verify -----------
// Two lanes per signature, radix 2^28 (74 limbs, R' = 2^2072 > 4n), lazy Montgomery (operands
// stay in [0, 2n)).  The running product is 76 column accumulators (64-bit) split over the pair:
// the even lane ("L") holds positions 0..37, the odd lane ("H") 38..75, each with the modulus
// limbs its columns meet.  A product of two limbs is < 2^56, so a column absorbs every one of its
// <= 148 products without overflow: a row is exactly one v_mad_u64_u32 per column for a*x and one
// for m*n — no per-column carry instructions (a 32-bit-limb FIOS form needs four).  Two rows
// per iteration, then a two-column shift (the two columns crossing from H to L move with DPP);
// m is computed in L and broadcast to H with DPP.  x (80 slots: slot 1 + j = limb j, slot 0 = 0)
// lives in LDS per signature and is read once per row pair; the multiply-by-s operand streams
// from a coalesced [limb][signature] scratch array.
constexpr uint32_t M28 = (1u << 28) - 1;
// plain C multiply-add: the compiler sees v_mad_u64_u32 and schedules / resolves hazards itself
__device__ __forceinline__ uint64_t madc(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }
constexpr int PC = 38;               // columns per lane
constexpr int PSIG = 32;             // signatures per 64-lane block

__device__ __forceinline__ uint32_t dpp_from_odd(uint32_t v) {   // lane 2k <- lane 2k+1
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xF5, 0xF, 0xF, false);  // quad_perm [1,1,3,3]
}
__device__ __forceinline__ uint32_t dpp_from_even(uint32_t v) {  // lane 2k+1 <- lane 2k
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xA0, 0xF, 0xF, false);  // quad_perm [0,0,2,2]
}
__device__ __forceinline__ uint64_t dpp_from_odd64(uint64_t v) {
  return ((uint64_t)dpp_from_odd((uint32_t)(v >> 32)) << 32) | dpp_from_odd((uint32_t)v);
}
__device__ __forceinline__ uint64_t dpp_from_even64(uint64_t v) {
  return ((uint64_t)dpp_from_even((uint32_t)(v >> 32)) << 32) | dpp_from_even((uint32_t)v);
}

// t = a * x * R'^-1 mod n (< 2n) into x's LDS column for signatures with `take`.
// xs[slot][sig]: slot 1 + j holds limb j of x; nreg[k] = n limb (P0 + k - 1) (0 outside 0..73).
template <class ARow>
__device__ __forceinline__ void mont_mul_pair(uint32_t (*xs)[PSIG], uint32_t sl, bool hi, uint32_t (&nreg)[PC + 1],
                                              uint32_t n0inv, ARow a, bool take) {
  const int P0 = hi ? PC : 0;
  const uint32_t* xcol = &xs[P0][sl];  // this lane's slots, immediate LDS offsets from here
  uint64_t A[PC];
#pragma unroll
  for (int c = 0; c < PC; c++) A[c] = 0;
#pragma unroll 1
  for (int i = 0; i < RSA_NL; i += 2) {
    asm volatile("" ::: "memory");  // x is re-read from LDS every row pair (not hoisted: 39 VGPRs)
    // the modulus limbs are opaque to loop-invariant code motion: otherwise their zero-extended
    // 64-bit copies are hoisted out of the loop (78 VGPRs) and spill
#pragma unroll
    for (int k = 0; k <= PC; k++) asm volatile("" : "+v"(nreg[k]));
    const uint32_t a0 = a(i), a1 = a(i + 1);
    uint32_t xv[PC + 1];  // x limbs P0 - 1 .. P0 + 37 (slots P0 .. P0 + 38)
#pragma unroll
    for (int k = 0; k <= PC; k++) xv[k] = xcol[k * PSIG];
    // row i: position c (global P0 + c) += a0 x[P0 + c] + m0 n[P0 + c]
#pragma unroll
    for (int c = 0; c < PC; c++) A[c] = madc(a0, xv[c + 1], A[c]);
    const uint32_t m0 = dpp_from_even(((uint32_t)A[0] * n0inv) & M28);
#pragma unroll
    for (int c = 0; c < PC; c++) A[c] = madc(m0, nreg[c + 1], A[c]);
    A[1] += hi ? 0ull : (A[0] >> 28);
    // row i + 1: one column up: position c += a1 x[P0 + c - 1] + m1 n[P0 + c - 1]
#pragma unroll
    for (int c = 0; c < PC; c++) A[c] = madc(a1, xv[c], A[c]);
    const uint32_t m1 = dpp_from_even(((uint32_t)A[1] * n0inv) & M28);
#pragma unroll
    for (int c = 0; c < PC; c++) A[c] = madc(m1, nreg[c], A[c]);
    A[2] += hi ? 0ull : (A[1] >> 28);
    // drop positions 0, 1 (both now multiples of 2^28 with their carries moved up): shift by two
    const uint64_t u0 = dpp_from_odd64(A[0]), u1 = dpp_from_odd64(A[1]);
#pragma unroll
    for (int c = 0; c + 2 < PC; c++) A[c] = A[c + 2];
    A[PC - 2] = hi ? 0ull : u0;
    A[PC - 1] = hi ? 0ull : u1;
  }
  // carries: L resolves positions 0..37, H continues from L's carry (value < 2n < 2^2049)
  uint32_t t[PC];
  uint64_t acc = 0;
#pragma unroll
  for (int c = 0; c < PC; c++) {
    acc += A[c];
    t[c] = (uint32_t)acc & M28;
    acc >>= 28;
  }
  uint64_t cin = dpp_from_even64(acc);
  if (!hi) cin = 0;
#pragma unroll
  for (int c = 0; c < PC; c++) {
    cin += t[c];
    t[c] = (uint32_t)cin & M28;
    cin >>= 28;
  }
  __syncthreads();  // every lane has read its x slots of the last row pair
  if (take) {
#pragma unroll
    for (int c = 0; c < PC; c++) xs[1 + P0 + c][sl] = t[c];
  }
  __syncthreads();
}

__global__ void __launch_bounds__(64, 2) rsa_verify_pair_kernel(const RsaBatch b, uint32_t* scratch,
                                                                 uint32_t* verdict32) {
  __shared__ uint32_t xs[RSA_PL][PSIG];
  const uint32_t tid = threadIdx.x;
  const bool hi = tid & 1;
  const uint32_t sl = tid >> 1;
  const size_t sig = (size_t)blockIdx.x * PSIG + sl;
  const size_t stride = (size_t)gridDim.x * PSIG;  // scratch row pitch
  const bool live = sig < b.n;
  const size_t si = live ? sig : 0;
  uint32_t kidx = b.key_idx[si];
  bool ok = live && kidx < b.nkeys;
  if (kidx >= b.nkeys) kidx = 0;
  const uint32_t* rec = b.keys + (size_t)kidx * RSA_KEY_WORDS;
  const int P0 = hi ? PC : 0;

  uint32_t nreg[PC + 1];
#pragma unroll
  for (int k = 0; k <= PC; k++) {
    const int j = P0 + k - 1;
    nreg[k] = (j >= 0 && j < RSA_NL) ? rec[RSA_KEY_P_N + j] : 0u;
  }
  const uint32_t n0inv = rec[RSA_KEY_P_N0INV];
  const uint32_t e = ok ? rec[RSA_KEY_E] : 0u;
  ok = ok && rec[RSA_KEY_OK];
  const uint8_t* sg = b.sig + si * RSA_MOD_BYTES;

  // x = R'^2 mod n: L writes slots 0..39, H slots 40..79 (slot 0 and slots past limb 73 are 0)
#pragma unroll
  for (int k = 0; k < RSA_PL / 2; k++) {
    const int slot = (hi ? RSA_PL / 2 : 0) + k;
    xs[slot][sl] = slot >= 1 ? rec[RSA_KEY_P_R2 + slot - 1] : 0u;
  }
  __syncthreads();

  int top = -1;
  if (__ballot(e != 0)) {
    for (int bit = 31; bit >= 0; bit--)
      if (__ballot((e >> bit) & 1u)) {
        top = bit;
        break;
      }
  }
  // schedule: CONV (s R'), MUL / SQR over the wave's top exponent bit, REDC
  enum { CONV, MUL, SQR, REDC };
  int op = CONV, bit = top;
  for (;;) {
    const bool take = op != MUL || ((e >> bit) & 1u);
    mont_mul_pair(
        xs, sl, hi, nreg, n0inv,
        [&](int i) -> uint32_t {
          if (i >= RSA_NL) return 0u;
          if (op == MUL) return scratch[(size_t)i * stride + sig];
          if (op == REDC) return i == 0 ? 1u : 0u;
          if (op == CONV) {  // 28-bit limb i of s (big-endian, 4-byte aligned signature)
            const int o = 28 * i, k = o >> 5, sh = o & 31;
            const uint64_t lo = __builtin_bswap32(*reinterpret_cast<const uint32_t*>(sg + RSA_MOD_BYTES - 4 * (k + 1)));
            const uint64_t hw =
                k + 1 < L ? __builtin_bswap32(*reinterpret_cast<const uint32_t*>(sg + RSA_MOD_BYTES - 4 * (k + 2))) : 0u;
            return (uint32_t)(((hw << 32) | lo) >> sh) & M28;
          }
          return xs[1 + i][sl];
        },
        take);
    if (op == REDC) break;
    if (op == CONV) {  // sm -> scratch (each lane its half of the limbs); x = R' mod n
#pragma unroll
      for (int k = 0; k < RSA_PL / 2; k++) {
        const int limb = (hi ? RSA_PL / 2 : 0) + k;
        if (limb < RSA_NL) scratch[(size_t)limb * stride + sig] = xs[1 + limb][sl];
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < RSA_PL / 2; k++) {
        const int slot = (hi ? RSA_PL / 2 : 0) + k;
        xs[slot][sl] = slot >= 1 ? rec[RSA_KEY_P_R1 + slot - 1] : 0u;
      }
      __syncthreads();
      op = top >= 0 ? MUL : REDC;
      continue;
    }
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

  // x = REDC(x) <= n: reduce fully (both lanes hold the whole value), back to 32-bit words
  uint32_t t[RSA_NL];
#pragma unroll
  for (int j = 0; j < RSA_NL; j++) t[j] = xs[1 + j][sl];
  {
    int32_t br = 0;
    uint32_t d[RSA_NL];
#pragma unroll
    for (int j = 0; j < RSA_NL; j++) {
      const int32_t v = (int32_t)t[j] - (int32_t)rec[RSA_KEY_P_N + j] + br;
      d[j] = (uint32_t)v & M28;
      br = v >> 28;  // 0 or -1
    }
#pragma unroll
    for (int j = 0; j < RSA_NL; j++) t[j] = br == 0 ? d[j] : t[j];
  }
  uint32_t hw8[8];
  sha256_words(hw8, b.msg + (live ? b.msg_off[si] : 0), live ? b.msg_len[si] : 0);
  bool eq = true;
#pragma unroll
  for (int k = 0; k < L; k++) {
    const int o = 32 * k, i = o / 28, sh = o % 28;
    const uint64_t v = (uint64_t)t[i] | (i + 1 < RSA_NL ? (uint64_t)t[i + 1] << 28 : 0ull);
    eq = eq && (uint32_t)(v >> sh) == (k < 8 ? hw8[7 - k] : em_limb(k));
  }
  // even lanes carry the verdicts of this block's 32 signatures
  uint64_t w = __ballot(ok && eq && !hi);
  w &= 0x5555555555555555ull;  // compress the even bits
  w = (w | (w >> 1)) & 0x3333333333333333ull;
  w = (w | (w >> 2)) & 0x0f0f0f0f0f0f0f0full;
  w = (w | (w >> 4)) & 0x00ff00ff00ff00ffull;
  w = (w | (w >> 8)) & 0x0000ffff0000ffffull;
  w = (w | (w >> 16)) & 0x00000000ffffffffull;
  if (tid == 0) {
    verdict32[blockIdx.x] = (uint32_t)w;
    if ((blockIdx.x & 1) == 0 && blockIdx.x + 1 == gridDim.x) verdict32[blockIdx.x + 1] = 0;  // pad the u64 word
  }
}

}  // namespace

size_t cbft_rsa_scratch_words(size_t n) { return ((n + PSIG - 1) / PSIG) * PSIG * RSA_NL; }

hipError_t cbft_rsa_launch_keys(const uint8_t* d_mod, const uint32_t* d_exp, uint32_t nkeys, uint32_t* d_keys,
                                hipStream_t stream) {
  if (!nkeys) return hipSuccess;
  hipLaunchKernelGGL(rsa_keys_kernel, dim3((nkeys + 63) / 64), dim3(64), 0, stream, d_mod, d_exp, nkeys, d_keys);
  return hipGetLastError();
}

hipError_t cbft_rsa_launch_verify(const RsaBatch& b, uint32_t* d_scratch, uint64_t* d_verdicts, hipStream_t stream) {
  if (!b.n) return hipSuccess;
  const unsigned blocks = (unsigned)((b.n + PSIG - 1) / PSIG);
  hipLaunchKernelGGL(rsa_verify_pair_kernel, dim3(blocks), dim3(64), 0, stream, b, d_scratch,
                     reinterpret_cast<uint32_t*>(d_verdicts));
  return hipGetLastError();
}
