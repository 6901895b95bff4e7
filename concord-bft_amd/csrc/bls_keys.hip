// BLS BN-P254 G2 kernels for gfx950: key decoding + Miller-loop line precomputation, the multisig
// key sum, the signer's public key (threshsign path).
//
//   bls_keys_row_kernel      per G2 key, one block of two waves: decompress + subgroup check
//                            (wave 0) beside the 70 Miller-loop lines (wave 1), on row-parallel
//                            Fp (bn254_g2row.h: limbs across 16-lane rows, four products per
//                            pass); also the generator's lines (BlsThresholdVerifier ctor; lines make per-share work G2-free)
//   bls_g2_sum_row_kernel    multisig PK = sum vk_i over the signer bitmap (Jacobian partial, or
//                            compressed for cbft_bls_sum_keys), row-parallel Fp
//   bls_pubkey_row_kernel    vk = sk * g2 by a fixed-base comb of g2
#include <cstdlib>
#include <cstring>

#include "bls_common.h"
#include "bn254_g2wave.h"
#include "bn254_g2row.h"

// Normalised lines (lambda, mu: BN_LINE_WORDS words each, g2_precompute_lines_batch's values)
// from the wave's unnormalised (A, B, C) records in LDS, lambda_k = -B_k / A_k, mu_k = C_k / A_k,
// by Montgomery's trick over the A_k on row-parallel Fp: prefix products (one Fp2 product per
// step: one pass), one variable-time Fp2 inversion on every lane (public key material), the
// back-substitution (two Fp2 products per step: two passes), then the 140 lambda / mu products
// row-locally, four lines' coefficients at a time.  pre: BN_ATE_LINES x 18 words of LDS.
__device__ __noinline__ void g2r_normalise_lines(uint32_t* out, const uint32_t* abc, uint32_t* pre) {
  using R2 = F2R<uint32_t>;
  const G2RowCtx<uint32_t, uint64_t> c(0u);
  uint32_t A[6], B[6], P[6];
  R2 acc = f2r_red(f2r_ld(abc), c);  // the records' coefficients are unreduced (< 50q)
  f2r_st_row0(pre, acc);
#pragma nounroll
  for (int k = 1; k < BN_ATE_LINES; k++) {
    const R2 a = f2r_red(f2r_ld(abc + k * BN_ABC_WORDS), c);
    f2r_mul_ops(A, B, 0, acc, a);
    r_prods<3>(P, A, B, c);
    f2r_mul_res(acc, P, 0, c);
    f2r_st_row0(pre + 18 * k, acc);
  }
  fp2 n;
  rf_to_fe(n.a, acc.a);
  rf_to_fe(n.b, acc.b);
  fp2_inv<true>(n, n);
  R2 inv = f2r_from(n);
#pragma nounroll
  for (int k = BN_ATE_LINES - 1; k >= 1; k--) {
    const R2 pk = f2r_ld(pre + 18 * (k - 1)), a = f2r_red(f2r_ld(abc + k * BN_ABC_WORDS), c);
    f2r_mul_ops(A, B, 0, inv, pk);  // 1 / A_k
    f2r_mul_ops(A, B, 3, inv, a);   // 1 / (A_0 .. A_{k-1})
    r_prods<6>(P, A, B, c);
    R2 ai;
    f2r_mul_res(ai, P, 0, c);
    f2r_mul_res(inv, P, 3, c);
    f2r_st_row0(pre + 18 * k, ai);
  }
  f2r_st_row0(pre, inv);
  const int row = (threadIdx.x & 63) >> 4;
#pragma nounroll
  for (int base = 0; base < 2 * BN_ATE_LINES; base += 4) {  // 140 = 35 x 4
    const int i = base + row, k = i >> 1, mu = i & 1;
    const R2 x = f2r_red(f2r_ld(abc + k * BN_ABC_WORDS + (mu ? 36 : 18)), c), y = f2r_ld(pre + 18 * k);
    const uint32_t p0 = c.mul(x.a, y.a), p1 = c.mul(x.b, y.b), p2 = c.mul(rf_add(x.a, x.b), rf_add(y.a, y.b));
    R2 r{c.red(c.sub(p0, p1)), c.red(c.sub(c.sub(p2, p0), p1))};
    const R2 nr = f2r_red(f2r_sub(R2{c.zero, c.zero}, r, c), c);
    r.a = mu ? r.a : nr.a;  // lambda = -B / A
    r.b = mu ? r.b : nr.b;
    f2r_st(out + (size_t)k * BN_LINE_WORDS + 18 * mu, r);
  }
}

// keys65 = nullptr: the generator g2's lines only (gen_lines, one block).  Else two one-wave blocks
// per key k: block k checks r Q == O on rows (g2r_in_subgroup) and writes ok[k] (decodes && not
// infinity && in G2, g2_decompress's verdict) and aff[k]; block nkeys + k builds the 70 lines
// (g2r_lines_abc into LDS) and normalises them into lines[k] (written for every decodable key;
// only ok keys are ever read); both decode the key (one lane's work).  The chip holds 2 x 1,024
// of these waves at once (VGPR-bound), so of the n + 1 = 1,025 keys' 2,050 blocks the last two
// start when the first finish: they are lines blocks (0.63 ms alone), not subgroup checks
// (1.7 ms alone).  Measured on 1,025 keys: 4.0 ms; two-wave blocks 4.5 ms (the group key's block
// ran in a second round); one wave per key doing both tasks 4.2 ms.
#define KEYS_ROW_BLOCK 64
__global__ void __launch_bounds__(KEYS_ROW_BLOCK) bls_keys_row_kernel(const uint8_t* keys65, uint32_t nkeys,
                                                                      uint32_t* lines, uint8_t* ok, uint32_t* aff) {
  __shared__ uint32_t abc[BN_ATE_LINES * BN_ABC_WORDS];
  __shared__ uint32_t pre[BN_ATE_LINES * 18];
  const int task = keys65 ? (blockIdx.x >= nkeys) : 1;
  const uint32_t k = keys65 ? blockIdx.x - (task ? nkeys : 0) : 0;
  if (k >= nkeys) return;
  const int lane = threadIdx.x & 63;
  g2a q;
  bool dec;
  if (keys65) {
    dec = g2_decode_on_curve(q, keys65 + 65 * (size_t)k) && !q.inf;
  } else {
    fp2_load(q.x, Bn254Consts::G2X);
    fp2_load(q.y, Bn254Consts::G2Y);
    q.inf = false;
    dec = true;
  }
  if (task == 0) {
    const G2RowCtx<uint32_t, uint64_t> c(0u);
    const bool good = dec && g2r_in_subgroup(f2r_from(q.x), f2r_from(q.y), c);
    if (lane == 0) {
      ok[k] = good ? 1 : 0;
      g2a qs = q;
      if (!good) qs.inf = true;
      g2a_store(aff + (size_t)k * BLS_G2A_WORDS, qs);
    }
    return;
  }
  if (!dec) return;
  g2r_lines_abc(abc, q);
  g2r_normalise_lines(lines + (size_t)k * LINES_PER_KEY, abc, pre);
}

// multisig public key = sum of vk_i for set bits (bit id-1, LSB first) of the 256-byte bitmap
// (BlsMultisigVerifier.cpp:33-38, 89-95).  One block: each of the SUM_THREADS lanes adds its
// strided share of the (already decoded, at load) keys in Jacobian form, then an LDS tree halves
// the partial sums.  A selected key that did not decode makes the result invalid (ok = 0).
#define SUM_THREADS 256
// normalise and compress (out65) a summed key; bad = a selected key did not decode
__device__ void g2_sum_tail(const g2j& acc, bool bad, uint8_t* ok, uint8_t* out65) {
  g2a s;
  g2_to_affine(s, acc);
  const bool good = !bad;
  if (good) {
    g2_compress(out65, s);
  } else {
    for (int q = 0; q < 65; q++) out65[q] = 0;
  }
  ok[0] = good && !s.inf ? 1 : 0;
}

// The multisig key sum on row-parallel Fp (bn254_g2row.h): a block of G2S_WAVES waves.  Level 0
// (parts == nullptr): wave w of block b adds the selected keys among ids
// [lo + G2S_IDS (b G2S_WAVES + w), +G2S_IDS) within [lo, hi) by mixed additions (a selected key
// that did not decode marks the sum bad); level > 0: partials [G2S_PARTS (b G2S_WAVES + w),
// +G2S_PARTS) of count.  The block's waves then meet in an LDS tree and wave 0 writes the block's
// partial (54 words < 2q + bad flag: g2j_load form) to out_parts[b], or, with out65 (a one-block
// launch), the compressed sum and ok (g2_sum_tail).  The group law is exact in every case
// (g2r_accum).
#define G2S_WAVES 8
#define G2S_IDS 8
#define G2S_PARTS 2
#define G2S_MAX_PARTS 64  // level-0 blocks for ids up to 4,096
using G2RCtx = G2RowCtx<uint32_t, uint64_t>;
// rows -> 54 one-lane words (< 2q: each coordinate through one Montgomery product with 1) + bad
__device__ __forceinline__ void g2r_part_store(uint32_t* o, const G2R<uint32_t>& p, bool inf, bool bad,
                                               const G2RCtx& c) {
  uint32_t A[6] = {p.X.a, p.X.b, p.Y.a, p.Y.b, p.Z.a, p.Z.b}, B[6], P[6];
  for (int i = 0; i < 6; i++) B[i] = c.one;
  r_prods<6>(P, A, B, c);
  for (int i = 0; i < 6; i++) rf_st9_row0(o + 9 * i, inf ? (i < 4 ? c.one : c.zero) : P[i]);
  if (__lane_id() == 0) o[54] = bad ? 1u : 0u;
}
__device__ __forceinline__ bool g2r_part_load(G2R<uint32_t>& p, const uint32_t* o, const G2RCtx& c) {
  p.X = f2r_ld(o);
  p.Y = f2r_ld(o + 18);
  p.Z = f2r_ld(o + 36);
  return c.zero4(p.Z);  // infinity
}
__global__ void __launch_bounds__(64 * G2S_WAVES) bls_g2_sum_row_kernel(const uint32_t* aff, const uint8_t* key_ok,
                                                                      const uint8_t* bitmap, uint32_t lo, uint32_t hi,
                                                                      const uint32_t* parts, uint32_t count,
                                                                      uint32_t* out_parts, uint8_t* ok,
                                                                      uint8_t* out65) {
  __shared__ uint32_t xp[G2S_WAVES][BLS_G2_PART_WORDS + 1];
  const int wave = threadIdx.x >> 6;
  const uint32_t wid = blockIdx.x * G2S_WAVES + wave;
  const G2RCtx c(0u);
  G2R<uint32_t> acc{{c.one, c.zero}, {c.one, c.zero}, {c.zero, c.zero}};
  bool inf = true, bad = false;
  if (!parts) {
    const uint32_t s0 = lo + wid * G2S_IDS;
#pragma nounroll
    for (uint32_t id = s0; id < s0 + G2S_IDS && id < hi; id++) {
      if (!((bitmap[(id - 1) >> 3] >> ((id - 1) & 7)) & 1)) continue;
      if (!key_ok[id - 1]) {
        bad = true;
        continue;
      }
      const uint32_t* a = aff + (size_t)(id - 1) * BLS_G2A_WORDS;  // x.a x.b y.a y.b (g2a_store)
      g2r_accum_aff(acc, inf, f2r_ld(a), f2r_ld(a + 18), c);
    }
  } else {
#pragma nounroll
    for (uint32_t i = wid * G2S_PARTS; i < (wid + 1) * G2S_PARTS && i < count; i++) {
      const uint32_t* o = parts + (size_t)BLS_G2_PART_WORDS * i;
      G2R<uint32_t> q;
      const bool qinf = g2r_part_load(q, o, c);
      bad |= o[54] != 0;
      g2r_accum(acc, inf, q, qinf, c);
    }
  }
#pragma unroll 1
  for (int stride = G2S_WAVES / 2; stride >= 1; stride >>= 1) {
    if (wave >= stride && wave < 2 * stride) {
      uint32_t* o = xp[wave - stride];
      f2r_st_row0(o, acc.X);
      f2r_st_row0(o + 18, acc.Y);
      f2r_st_row0(o + 36, inf ? F2R<uint32_t>{c.zero, c.zero} : acc.Z);
      if (__lane_id() == 0) o[54] = bad ? 1u : 0u;
    }
    __syncthreads();
    if (wave < stride) {
      G2R<uint32_t> q;
      const bool qinf = g2r_part_load(q, xp[wave], c);
      bad |= xp[wave][54] != 0;
      g2r_accum(acc, inf, q, qinf, c);
    }
    __syncthreads();
  }
  if (wave != 0) return;
  if (out65) {
    __shared__ uint32_t fin[BLS_G2_PART_WORDS];
    g2r_part_store(fin, acc, inf, bad, c);
    if (__lane_id() == 0) {
      g2j s;
      g2j_load(s, fin);
      g2_sum_tail(s, bad, ok, out65);
    }
    return;
  }
  g2r_part_store(out_parts + (size_t)BLS_G2_PART_WORDS * blockIdx.x, acc, inf, bad, c);
}

// ------------------------------------------------------------------------------ launchers
size_t cbft_bls_lines_words_per_key() { return (size_t)LINES_PER_KEY; }
hipError_t cbft_bls_launch_keys(const uint8_t* d_keys65, uint32_t nkeys, uint32_t* d_lines, uint8_t* d_ok,
                                uint32_t* d_aff, hipStream_t s) {
  if (!nkeys) return hipSuccess;
  hipLaunchKernelGGL(bls_keys_row_kernel, dim3(2 * nkeys), dim3(KEYS_ROW_BLOCK), 0, s, d_keys65, nkeys, d_lines, d_ok,
                     d_aff);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_gen_lines(uint32_t* d_lines, hipStream_t s) {
  hipLaunchKernelGGL(bls_keys_row_kernel, dim3(1), dim3(KEYS_ROW_BLOCK), 0, s, nullptr, 1u, d_lines, nullptr, nullptr);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_g2_sum(const uint32_t* d_aff, const uint8_t* d_key_ok, uint32_t n, const uint8_t* d_bitmap,
                                  uint32_t lo_id, uint32_t hi_id, uint8_t* d_ok, uint8_t* d_out65, uint32_t* d_out_part,
                                  uint32_t* d_tmp, hipStream_t s) {
  if (!d_tmp) return hipErrorInvalidValue;
  const uint32_t lo = lo_id < 1 ? 1 : lo_id, hi = hi_id > n + 1 ? n + 1 : hi_id;
  const uint32_t span = hi > lo ? hi - lo : 0;
  uint32_t nb = (span + G2S_WAVES * G2S_IDS - 1) / (G2S_WAVES * G2S_IDS);
  if (nb == 0) nb = 1;
  // level 0: the keys -> nb partials; then G2S_WAVES * G2S_PARTS : 1 levels until one remains
  uint32_t* cur = d_tmp;
  uint32_t* nxt = d_tmp + (size_t)BLS_G2_PART_WORDS * G2S_MAX_PARTS;
  const bool one = nb == 1;
  hipLaunchKernelGGL(bls_g2_sum_row_kernel, dim3(nb), dim3(64 * G2S_WAVES), 0, s, d_aff, d_key_ok, d_bitmap, lo, hi,
                     (const uint32_t*)nullptr, 0u, one && d_out_part ? d_out_part : cur, d_ok,
                     one ? d_out65 : (uint8_t*)nullptr);
  while (nb > 1) {
    const uint32_t nb2 = (nb + G2S_WAVES * G2S_PARTS - 1) / (G2S_WAVES * G2S_PARTS);
    const bool last = nb2 == 1;
    hipLaunchKernelGGL(bls_g2_sum_row_kernel, dim3(nb2), dim3(64 * G2S_WAVES), 0, s, d_aff, d_key_ok, d_bitmap, lo,
                       hi, (const uint32_t*)cur, nb, last && d_out_part ? d_out_part : nxt, d_ok,
                       last ? d_out65 : (uint8_t*)nullptr);
    uint32_t* t = cur;
    cur = nxt;
    nxt = t;
    nb = nb2;
  }
  return hipGetLastError();
}
size_t cbft_bls_g2_sum_tmp_words() { return (size_t)2 * BLS_G2_PART_WORDS * G2S_MAX_PARTS; }

// ------------------------------------------------------------------------------ public key
// vk = sk * g2 (IThresholdSigner::getShareVerificationKey, BlsThresholdSigner's publicKey_) as a
// fixed-base comb: g2 is fixed, so its radix-16 multiples are precomputed once per context,
//   PUB_T[j][e] = (2e + 1) 16^j g2,  j = 0..63, e = 0..7   (affine, normalised Montgomery limbs)
// and sk = sum_j d_j 16^j with ODD digits d_j = 2 u_j - 15, u = (sk + 16^64 - 1) / 2 (an even sk is
// replaced by the odd r - sk and the result negated, both by selects), so the key is 63 mixed additions of
// +-PUB_T[j][(|d_j| - 1) / 2]: every entry read and chosen by selects, every sign by a select,
// the same instruction stream for every key.  Going up from position 0, the partial sum is an odd
// multiple below 16^j g2 in magnitude, so no addition meets +-its addend (never exceptional).
// Z is inverted blinded (Z b, variable time, times b; b from SHA-256 of the key).
#define PUB_POS 64
#define PUB_ENT 8
#define PUB_WORDS 36  // x.a | x.b | y.a | y.b, 9 limbs each

__device__ __forceinline__ void f_canon_limbs(uint32_t* o, fp x) {  // canonical Montgomery limbs
  f_canon(x);
#pragma unroll
  for (int i = 0; i < BN_LIMBS; i++) o[i] = x.v[i];
}

// one lane per position j: 16^j g2 by 4 j doublings, then its odd multiples, affine (public)
__global__ void __launch_bounds__(64) bls_pub_table_kernel(uint32_t* tbl) {
  const int j = threadIdx.x;
  if (j >= PUB_POS || blockIdx.x != 0) return;
  g2j P;
  fp2_load(P.X, Bn254Consts::G2X);
  fp2_load(P.Y, Bn254Consts::G2Y);
  fp2_one(P.Z);
#pragma nounroll
  for (int d = 0; d < 4 * j; d++) {
    g2j t;
    g2_dbl_j(t, P);
    P = t;
  }
  g2j P2, E = P;
  g2_dbl_j(P2, P);
#pragma nounroll
  for (int e = 0; e < PUB_ENT; e++) {
    if (e) {
      g2j t;
      g2_add_j(t, E, P2);
      E = t;
    }
    g2a a;
    g2_to_affine<true>(a, E);
    uint32_t* o = tbl + ((size_t)j * PUB_ENT + e) * PUB_WORDS;
    f_canon_limbs(o, a.x.a);
    f_canon_limbs(o + 9, a.x.b);
    f_canon_limbs(o + 18, a.y.a);
    f_canon_limbs(o + 27, a.y.b);
  }
}

__global__ void __launch_bounds__(64) bls_pubkey_row_kernel(const uint32_t* tbl, const uint32_t* sk, uint8_t* out65) {
  using Ctx = G2RowCtx<uint32_t, uint64_t>;
  const Ctx c(0u);
  uint32_t k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = sk[i];
  // an even sk is replaced by the odd r - sk (selected, not branched) and the point negated at the
  // end: k' in [1, r - 1], so no partial sum of the comb ever meets +-its addend mod r
  const uint32_t even = (k[0] & 1u) ^ 1u, emask = 0u - even;
  {
    const uint32_t rw[8] = {0x0000000du, 0xa1000000u, 0x00000010u, 0xff9f8000u,
                            0x00000007u, 0xba344d80u, 0x40000001u, 0x25236482u};
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int64_t d = (int64_t)rw[i] - k[i] + br;
      k[i] = ((uint32_t)d & emask) | (k[i] & ~emask);
      br = d >> 32;
    }
  }
  uint32_t u[8];
  {  // u = (k' + 2^256 - 1) / 2 = 2^255 + (k' - 1) / 2
    uint64_t cy = 0;
    uint32_t t[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      cy += (uint64_t)k[i] + 0xffffffffu;
      t[i] = (uint32_t)cy;
      cy >>= 32;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) u[i] = (t[i] >> 1) | (i < 7 ? (t[i + 1] << 31) : ((uint32_t)cy << 31));
  }
  auto pick = [&](int j, F2R<uint32_t>& qx, F2R<uint32_t>& qy) {
    const uint32_t nib = (u[j >> 3] >> (4 * (j & 7))) & 15u;  // d = 2 nib - 15
    const uint32_t dn = nib < 8u ? 1u : 0u;
    const uint32_t m = dn ? 7u - nib : nib - 8u;
    const uint32_t* base = tbl + (size_t)j * PUB_ENT * PUB_WORDS;
    qx = f2r_ld(base);
    qy = f2r_ld(base + 18);
#pragma unroll
    for (int e = 1; e < PUB_ENT; e++) {
      const F2R<uint32_t> ex = f2r_ld(base + e * PUB_WORDS), ey = f2r_ld(base + e * PUB_WORDS + 18);
      const bool hit = m == (uint32_t)e;
      qx.a = rf_sel(hit, ex.a, qx.a);
      qx.b = rf_sel(hit, ex.b, qx.b);
      qy.a = rf_sel(hit, ey.a, qy.a);
      qy.b = rf_sel(hit, ey.b, qy.b);
    }
    const F2R<uint32_t> ny{c.sub(c.zero, qy.a), c.sub(c.zero, qy.b)};  // -y + 8q (< 9q)
    qy.a = c.red(rf_sel(dn != 0u, ny.a, qy.a));
    qy.b = c.red(rf_sel(dn != 0u, ny.b, qy.b));
  };
  G2R<uint32_t> acc;
  {
    F2R<uint32_t> qx, qy;
    pick(0, qx, qy);
    acc.X = qx;
    acc.Y = qy;
    acc.Z = F2R<uint32_t>{c.one, c.zero};
  }
#pragma nounroll
  for (int j = 1; j < PUB_POS; j++) {
    F2R<uint32_t> qx, qy;
    pick(j, qx, qy);
    bool same_y;
    g2r_madd<false>((F2R<uint32_t>*)nullptr, acc, qx, qy, c, same_y);
  }
  {  // sk even: sk g2 = -(r - sk) g2 (the negation selected)
    const F2R<uint32_t> ny{c.red(c.sub(c.zero, acc.Y.a)), c.red(c.sub(c.zero, acc.Y.b))};
    acc.Y.a = rf_sel(even != 0u, ny.a, acc.Y.a);
    acc.Y.b = rf_sel(even != 0u, ny.b, acc.Y.b);
  }
  const bool inf = false;  // k' in [1, r - 1]: never the point at infinity
  g2j J;
  rf_to_fe(J.X.a, acc.X.a);
  rf_to_fe(J.X.b, acc.X.b);
  rf_to_fe(J.Y.a, acc.Y.a);
  rf_to_fe(J.Y.b, acc.Y.b);
  rf_to_fe(J.Z.a, acc.Z.a);
  rf_to_fe(J.Z.b, acc.Z.b);
  g2a a;
  if (inf) {
    a.inf = true;
    fp2_zero(a.x);
    fp2_zero(a.y);
  } else {
    uint32_t bw[8];
    {
      uint32_t hs[8];  // SHA-256 of the key's bytes xored with 0x5c
      sha256_key_msg(hs, k, 0x5c, nullptr, 0);
      for (int i = 0; i < 8; i++) bw[i] = sha256_bswap(hs[i]);
      bw[7] &= 0x1fffffffu;  // < 2^253 < q
      bw[0] |= (bw[0] | bw[1] | bw[2] | bw[3] | bw[4] | bw[5] | bw[6] | bw[7]) == 0u ? 1u : 0u;
    }
    fp b;
    f_from_words(b, bw);
    fp2 zb, zi, zi2;
    fp2_mul_fp(zb, J.Z, b);
    fp2_inv<true>(zi, zb);  // (Z b)^-1, variable time on a blinded value
    fp2_mul_fp(zi, zi, b);
    fp2_sqr(zi2, zi);
    fp2_mul(a.x, J.X, zi2);
    fp2_mul(zi2, zi2, zi);
    fp2_mul(a.y, J.Y, zi2);
    a.inf = false;
    for (int i = 0; i < 8; i++) bw[i] = 0;
  }
  if (__lane_id() == 0) g2_compress(out65, a);
}

size_t cbft_bls_pub_table_words() { return (size_t)PUB_POS * PUB_ENT * PUB_WORDS; }
hipError_t cbft_bls_launch_pub_table(uint32_t* d_tbl, hipStream_t s) {
  hipLaunchKernelGGL(bls_pub_table_kernel, dim3(1), dim3(64), 0, s, d_tbl);
  return hipGetLastError();
}
hipError_t cbft_bls_launch_pubkey_row(const uint32_t* d_tbl, const uint32_t* d_sk, uint8_t* d_out65, hipStream_t s) {
  hipLaunchKernelGGL(bls_pubkey_row_kernel, dim3(1), dim3(64), 0, s, d_tbl, d_sk, d_out65);
  return hipGetLastError();
}
