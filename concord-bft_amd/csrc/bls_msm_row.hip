// Lagrange MSM (fastMultExp, FastMultExp.cpp:26-59; BlsThresholdAccumulator.cpp:46-55) and the
// multisig share sum (BlsMultisigAccumulator.cpp:57-65) on row-parallel Fp (bn254_row.h,
// bn254_g1row.h): one WAVE per point chain, the chain's products four per round, each product's
// limbs across a 16-lane row.
//
//   bls_msm_row_kernel   one block of two waves per share j: lambda_j sigma_j = k1 sigma_j +
//                        k2 phi(sigma_j) (GLV, the constants of bls_kernels.hip): wave 0 runs the
//                        k1 half, wave 1 the k2 half and applies phi (X -> beta X) to its result;
//                        33 signed radix-16 windows (4 doublings + at most one addition from the
//                        wave's table {1..8} sigma_j) each; the halves meet in LDS.  683 shares =
//                        1,366 waves.
//   bls_g1_sum_row_kernel sum of m points, 16 waves per block: each wave loads one point (a
//                        Jacobian partial, or an affine share for the multisig sum), then an LDS
//                        tree of additions; one partial per block.  The host launches it until
//                        one partial remains, then bls_msm_finish_kernel compresses it.
//
// Points cross kernels as BLS_JAC_WORDS Jacobian words (X | Y | Z limbs, values < 2q, normalised);
// infinity is Z = 0.
#include "bls_common.h"
#include "bls_glv.h"
#include "bn254_g1row.h"

using RCtx = RowCtx<uint32_t, uint64_t>;

using RPt = G1R<uint32_t>;

// row point <- 9-limb words (one-lane limbs at p[0..8]: lane i of every row takes p[i])
__device__ __forceinline__ uint32_t rf_load_limbs(const uint32_t* p) {
  const uint32_t rl = __lane_id() & 15u;
  return rl < 9 ? p[rl] : 0u;
}

// store a point < 4q as normalised limbs < 2q (x * R mod q through one Montgomery product with 1)
__device__ __forceinline__ void rpt_store(uint32_t* o, const RPt& p, bool inf, const RCtx& c) {
  const uint32_t a[3] = {p.X, p.Y, p.Z}, b[3] = {c.one, c.one, c.one};
  uint32_t r[3];
  g1r_round<3>(r, a, b, c);
  const uint32_t rl = __lane_id() & 15u, row = __lane_id() >> 4;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint32_t n = rf_normalize(r[k]);
    if (row == 0 && rl < 9) o[9 * k + rl] = (inf && k == 2) ? 0u : n;
  }
}

__device__ __forceinline__ bool rpt_load(RPt& p, const uint32_t* o) {
  p.X = rf_load_limbs(o);
  p.Y = rf_load_limbs(o + 9);
  p.Z = rf_load_limbs(o + 18);
  return __ballot(p.Z != 0) == 0;  // Z == 0: infinity (uniform)
}

// acc += e, with the flags (wave-uniform)
__device__ __forceinline__ void rpt_accum(RPt& acc, bool& inf, const RPt& e, bool einf, const RCtx& c) {
  if (einf) return;
  if (inf) {
    acc = e;
    inf = false;
    return;
  }
  RPt r;
  if (g1r_add(r, acc, e, c) == G1R_INF)
    inf = true;
  else
    acc = r;
}

#define MSM_ROW_BLOCK 128
__global__ void __launch_bounds__(MSM_ROW_BLOCK) bls_msm_row_kernel(const uint32_t* sig, const uint32_t* lambda,
                                                                    const uint8_t* use, uint32_t k, uint32_t* out) {
  __shared__ uint32_t xch[3 * 16];
  __shared__ int xinf;
  const uint32_t j = blockIdx.x;
  if (j >= k) return;
  const int wave = threadIdx.x >> 6;
  const uint32_t tag = 0;
  const RCtx c(tag);
  RPt acc;
  bool inf = true;
  g1a s;
  g1a_load(s, sig + BLS_SIG_WORDS * (size_t)j);
  const bool live = use[j] != 0 && !s.inf;
  if (live) {
    uint32_t lw[8];
    for (int w = 0; w < 8; w++) lw[w] = lambda[8 * (size_t)j + w];
    uint32_t k1[5], k2[5];
    bool n1, n2;
    glv_split(lw, k1, k2, n1, n2);
    glv_offset(k1);
    glv_offset(k2);
    const uint32_t* kk = wave ? k2 : k1;
    const bool neg = wave ? n2 : n1;
    // table T[m] = (m + 1) sigma, m = 0..7
    RPt T[8];
    T[0].X = rf_from_fe(s.x, tag);
    T[0].Y = rf_from_fe(s.y, tag);
    T[0].Z = c.one;
    g1r_dbl(T[1], T[0], c);
    g1r_add(T[2], T[1], T[0], c);
    g1r_dbl(T[3], T[1], c);
    g1r_add(T[4], T[3], T[0], c);
    g1r_dbl(T[5], T[2], c);
    g1r_add(T[6], T[5], T[0], c);
    g1r_dbl(T[7], T[3], c);
#pragma nounroll
    for (int w = 32; w >= 0; w--) {
      if (!inf) {
        RPt t;
#pragma unroll 1
        for (int d = 0; d < 4; d++) {
          g1r_dbl(t, acc, c);
          acc = t;
        }
      }
      const int dg = glv_digit(kk, w);
      if (dg != 0) {  // wave-uniform
        const int m = (dg < 0 ? -dg : dg) - 1;
        RPt e = T[0];
#pragma unroll
        for (int i = 1; i < 8; i++)
          if (m == i) e = T[i];
        if ((dg < 0) != neg) g1r_neg(e, e, c);
        rpt_accum(acc, inf, e, false, c);
      }
    }
    if (wave == 1 && !inf) {  // phi(P) = (beta X, Y): the k2 half was run on sigma itself
      fp beta;
      uint32_t bw[8];
      for (int w = 0; w < 8; w++) bw[w] = kGlvBeta[w];
      f_from_words(beta, bw);
      acc.X = c.mul(acc.X, rf_from_fe(beta, tag));
    }
  }
  // wave 1 hands its half to wave 0
  if (wave == 1) {
    const uint32_t l = __lane_id();
    if (l < 16) {
      xch[l] = acc.X;
      xch[16 + l] = acc.Y;
      xch[32 + l] = acc.Z;
    }
    if (l == 0) xinf = inf ? 1 : 0;
  }
  __syncthreads();
  if (wave != 0) return;
  RPt h;
  const uint32_t rl = __lane_id() & 15u;
  h.X = xch[rl];
  h.Y = xch[16 + rl];
  h.Z = xch[32 + rl];
  rpt_accum(acc, inf, h, xinf != 0, c);
  rpt_store(out + BLS_JAC_WORDS * (size_t)j, acc, inf, c);
}

// sum of m points -> one Jacobian partial per block of 16 waves.  affine: points are parsed shares
// (BLS_SIG_WORDS, use[]), else Jacobian partials.
#define SUM_ROW_WAVES 16
__global__ void __launch_bounds__(64 * SUM_ROW_WAVES) bls_g1_sum_row_kernel(const uint32_t* in, const uint8_t* use,
                                                                           uint32_t m, int affine, uint32_t* out) {
  __shared__ uint32_t xp[SUM_ROW_WAVES / 2][3 * 16];
  __shared__ int xinf[SUM_ROW_WAVES / 2];
  const int wave = threadIdx.x >> 6;
  const uint32_t i = blockIdx.x * SUM_ROW_WAVES + wave;
  const uint32_t tag = 0;
  const RCtx c(tag);
  RPt acc;
  bool inf = true;
  if (i < m) {
    if (affine) {
      g1a s;
      g1a_load(s, in + BLS_SIG_WORDS * (size_t)i);
      if (use[i] && !s.inf) {
        acc.X = rf_from_fe(s.x, tag);
        acc.Y = rf_from_fe(s.y, tag);
        acc.Z = c.one;
        inf = false;
      }
    } else {
      inf = rpt_load(acc, in + BLS_JAC_WORDS * (size_t)i);
    }
  }
  const uint32_t l = __lane_id(), rl = l & 15u;
#pragma unroll 1
  for (int stride = SUM_ROW_WAVES / 2; stride >= 1; stride >>= 1) {
    if (wave >= stride && wave < 2 * stride) {
      if (l < 16) {
        xp[wave - stride][l] = acc.X;
        xp[wave - stride][16 + l] = acc.Y;
        xp[wave - stride][32 + l] = acc.Z;
      }
      if (l == 0) xinf[wave - stride] = inf ? 1 : 0;
    }
    __syncthreads();
    if (wave < stride) {
      RPt o;
      o.X = xp[wave][rl];
      o.Y = xp[wave][16 + rl];
      o.Z = xp[wave][32 + rl];
      rpt_accum(acc, inf, o, xinf[wave] != 0, c);
    }
    __syncthreads();
  }
  if (wave == 0) rpt_store(out + BLS_JAC_WORDS * (size_t)blockIdx.x, acc, inf, c);
}

// ------------------------------------------------------------------------------ launcher
// The row-parallel combine: lambda_j sigma_j per share into d_work, then sum levels (16:1 per
// block) until one partial remains; d_work holds m + ceil(m/16) + ... Jacobian points.  Returns
// the device pointer of the final partial (one point).
hipError_t cbft_bls_launch_msm_row(const uint32_t* d_sig, const uint32_t* d_lambda, const uint8_t* d_use, uint32_t m,
                                   int multisig, uint32_t* d_work, uint32_t** d_final, hipStream_t s) {
  uint32_t* cur = d_work;
  uint32_t n = m;
  int affine = 0;
  if (!multisig) {
    if (m) hipLaunchKernelGGL(bls_msm_row_kernel, dim3(m), dim3(MSM_ROW_BLOCK), 0, s, d_sig, d_lambda, d_use, m, cur);
  } else {
    affine = 1;  // the shares themselves are the points
  }
  const uint32_t* src = multisig ? d_sig : cur;
  uint32_t* dst = multisig ? d_work : cur + BLS_JAC_WORDS * (size_t)n;
  do {
    const uint32_t nb = n ? (n + SUM_ROW_WAVES - 1) / SUM_ROW_WAVES : 1;  // m = 0: one block of infinity
    hipLaunchKernelGGL(bls_g1_sum_row_kernel, dim3(nb), dim3(64 * SUM_ROW_WAVES), 0, s, src, d_use, n, affine, dst);
    affine = 0;
    src = dst;
    dst = dst + BLS_JAC_WORDS * (size_t)nb;
    n = nb;
  } while (n > 1);
  *d_final = const_cast<uint32_t*>(src);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------ signing
// sigma = sk * H, H = g1_map(msg) (BlsThresholdSigner::signData, BlsThresholdSigner.cpp:32-47),
// on row-parallel Fp with a secret-independent operation sequence.  One block of two waves:
//   GLV: sk = k1 + k2 lam (mod r), |k1|, |k2| < 2^128, signs taken branch-free (glv_split_ct);
//   wave 0 runs |k1| on +-H, wave 1 |k2| on +-H and maps its result by phi (X -> beta X);
//   each half is made odd (k + 1 when even, the extra H subtracted at the end by a select) and
//   recoded into 33 odd signed radix-16 digits d_i = 2 u_i - 15, u = (k + 16^33 - 1) / 2, so
//   every window is 4 doublings and exactly one addition of +-T[(|d| - 1) / 2], T = {1, 3, .., 15} H,
//   the entry picked by a select over all eight and its sign by a select: the same instruction
//   stream for every key.  The partial sums stay odd multiples (16 s + d with s odd never equals
//   +-d), so no addition meets an exceptional case.
//   The halves meet in LDS; the affine conversion inverts Z * b with the variable-time safegcd and
//   multiplies b back in: the blind b = SHA-256(sk || msg) mod 2^253 (< q) is secret and fresh
//   per message, so the inversion's timing says nothing about Z.
__device__ __forceinline__ void mp_neg_ct(uint32_t* a, uint32_t m /* 0 or ~0 */) {
  uint64_t c = m & 1u;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c += (uint32_t)(a[i] ^ m);
    a[i] = (uint32_t)c;
    c >>= 32;
  }
}

// glv_split with the sign handling as selects
__device__ __forceinline__ void glv_split_ct(const uint32_t* k, uint32_t* k1, uint32_t* k2, uint32_t& n1,
                                             uint32_t& n2) {
  uint32_t c1[3], c2[5], g1[3], g2[5], a1[2], a2[4], b1[4], b2[2];
#pragma unroll
  for (int i = 0; i < 3; i++) g1[i] = kGlvG1[i];
#pragma unroll
  for (int i = 0; i < 5; i++) g2[i] = kGlvG2[i];
#pragma unroll
  for (int i = 0; i < 2; i++) {
    a1[i] = kGlvA1[i];
    b2[i] = kGlvB2[i];
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    a2[i] = kGlvA2[i];
    b1[i] = kGlvB1[i];
  }
  mp_mul<8, 3, 3>(c1, k, g1, 8);
  mp_mul<8, 5, 5>(c2, k, g2, 8);
  uint32_t t[8], p[8];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = k[i];
  mp_mul<3, 2, 8>(p, c1, a1, 0);
  mp_sub8(t, p);
  mp_mul<5, 4, 8>(p, c2, a2, 0);
  mp_sub8(t, p);  // k1 = k - c1 a1 - c2 a2
  n1 = 0u - (t[7] >> 31);
  mp_neg_ct(t, n1);
#pragma unroll
  for (int i = 0; i < 5; i++) k1[i] = t[i];
  mp_mul<3, 4, 8>(t, c1, b1, 0);  // -c1 b1 = c1 |b1|
  mp_mul<5, 2, 8>(p, c2, b2, 0);
  mp_sub8(t, p);  // k2 = c1 |b1| - c2 b2
  n2 = 0u - (t[7] >> 31);
  mp_neg_ct(t, n2);
#pragma unroll
  for (int i = 0; i < 5; i++) k2[i] = t[i];
}

#define SIGN_WINDOWS 33
__global__ void __launch_bounds__(128) bls_sign_row_kernel(const uint32_t* H, const uint32_t* sk, const uint8_t* msg,
                                                           uint32_t len, uint32_t id, uint8_t* out37) {
  __shared__ uint32_t xch[3 * 16];
  const int wave = threadIdx.x >> 6;
  const uint32_t tag = 0;
  const RCtx c(tag);
  g1a h;
  // H = g1_map(msg): precomputed (H != nullptr), or computed here by each wave (both waves need
  // it; the same deterministic result), which saves the hash kernel's launch and H's round trip
  if (H)
    g1a_load(h, H);  // g1_map never returns infinity
  else
    g1_map_row(h, msg, len);
  uint32_t k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = sk[i];
  uint32_t k1[5], k2[5], n1, n2;
  glv_split_ct(k, k1, k2, n1, n2);
  uint32_t kk[5];
#pragma unroll
  for (int i = 0; i < 5; i++) kk[i] = wave ? k2[i] : k1[i];  // the wave index is public
  const uint32_t neg = wave ? n2 : n1;
  // odd: k + 1 when even (undone at the end)
  const uint32_t even = (kk[0] & 1u) ^ 1u;
  {
    uint64_t cy = even;
#pragma unroll
    for (int i = 0; i < 5; i++) {
      cy += kk[i];
      kk[i] = (uint32_t)cy;
      cy >>= 32;
    }
  }
  // u = (k + 2^132 - 1) / 2: nibble i of u gives d_i = 2 u_i - 15
  uint32_t u[5];
  {
    uint64_t cy = 0;
#pragma unroll
    for (int i = 0; i < 5; i++) {
      cy += (uint64_t)kk[i] + (i < 4 ? 0xffffffffu : 0xfu);
      u[i] = (uint32_t)cy;
      cy >>= 32;
    }
#pragma unroll
    for (int i = 0; i < 5; i++) u[i] = (u[i] >> 1) | (i < 4 ? (u[i + 1] << 31) : 0u);
  }
  // base +-H (sign by select), table T[m] = (2m + 1) base
  RPt P;
  P.X = rf_from_fe(h.x, tag);
  P.Y = rf_from_fe(h.y, tag);
  P.Z = c.one;
  {
    RPt Pn;
    g1r_neg(Pn, P, c);
    P.Y = rf_sel(neg != 0u, Pn.Y, P.Y);
  }
  RPt T[8], P2;
  T[0] = P;
  g1r_dbl(P2, P, c);
#pragma unroll
  for (int m = 1; m < 8; m++) g1r_add(T[m], T[m - 1], P2, c);  // unrolled: T stays in registers
  auto pick = [&](int w, RPt& e) {  // +-T[(|d_w| - 1) / 2] by selects over all entries
    const uint32_t nib = (u[w >> 3] >> (4 * (w & 7))) & 15u;  // d = 2 nib - 15
    const uint32_t dn = nib < 8u ? 1u : 0u;                    // d < 0
    const uint32_t m = dn ? 7u - nib : nib - 8u;               // (|d| - 1) / 2
    e = T[0];
#pragma unroll
    for (int i = 1; i < 8; i++) {
      const bool hit = m == (uint32_t)i;
      e.X = rf_sel(hit, T[i].X, e.X);
      e.Y = rf_sel(hit, T[i].Y, e.Y);
      e.Z = rf_sel(hit, T[i].Z, e.Z);
    }
    RPt en;
    g1r_neg(en, e, c);
    e.Y = rf_sel(dn != 0u, en.Y, e.Y);
  };
  RPt acc;
  pick(SIGN_WINDOWS - 1, acc);
#pragma nounroll
  for (int w = SIGN_WINDOWS - 2; w >= 0; w--) {
    RPt t;
#pragma unroll 1
    for (int d = 0; d < 4; d++) {
      g1r_dbl(t, acc, c);
      acc = t;
    }
    RPt e;
    pick(w, e);
    g1r_add(t, acc, e, c);
    acc = t;
  }
  bool inf = false;
  {  // undo the odd fix: acc - base when k was even (computed always, kept by a select)
    RPt nb, t;
    g1r_neg(nb, P, c);
    const bool zero = g1r_add(t, acc, nb, c) == G1R_INF;  // only when the half-scalar is 0
    const bool take = even != 0u;
    acc.X = rf_sel(take, t.X, acc.X);
    acc.Y = rf_sel(take, t.Y, acc.Y);
    acc.Z = rf_sel(take, t.Z, acc.Z);
    inf = take && zero;
  }
  if (wave == 1 && !inf) {  // phi(P) = (beta X, Y)
    fp beta;
    uint32_t bw[8];
    for (int w = 0; w < 8; w++) bw[w] = kGlvBeta[w];
    f_from_words(beta, bw);
    acc.X = c.mul(acc.X, rf_from_fe(beta, tag));
  }
  __shared__ int xinf;
  if (wave == 1) {
    const uint32_t l = __lane_id();
    if (l < 16) {
      xch[l] = acc.X;
      xch[16 + l] = acc.Y;
      xch[32 + l] = acc.Z;
    }
    if (l == 0) xinf = inf ? 1 : 0;
  }
  __syncthreads();
  if (wave != 0) return;
  {
    RPt o;
    const uint32_t rl = __lane_id() & 15u;
    o.X = xch[rl];
    o.Y = xch[16 + rl];
    o.Z = xch[32 + rl];
    rpt_accum(acc, inf, o, xinf != 0, c);
  }
  // affine through a blinded variable-time inversion, every lane the same one-lane values
  g1j J;
  rf_to_fe(J.X, acc.X);
  rf_to_fe(J.Y, acc.Y);
  rf_to_fe(J.Z, acc.Z);
  g1a a;
  if (inf) {
    a.inf = true;
    f_zero(a.x);
    f_zero(a.y);
  } else {
    uint32_t bw[8];
    {
      uint32_t hs[8];  // SHA-256(sk || msg[0 .. 64)) is the blind's seed
      sha256_key_msg(hs, k, 0, msg, len < 64u ? len : 64u);
      for (int i = 0; i < 8; i++) bw[i] = sha256_bswap(hs[i]);  // digest bytes as little-endian words
      bw[7] &= 0x1fffffffu;  // < 2^253 < q
      bw[0] |= (bw[0] | bw[1] | bw[2] | bw[3] | bw[4] | bw[5] | bw[6] | bw[7]) == 0u ? 1u : 0u;
    }
    fp b, zb, zi, zi2;
    f_from_words(b, bw);
    f_mul(zb, J.Z, b);
    fp_inv_var(zi, zb);
    f_mul(zi, zi, b);  // 1 / Z
    f_sqr(zi2, zi);
    f_mul(a.x, J.X, zi2);
    f_mul(zi2, zi2, zi);
    f_mul(a.y, J.Y, zi2);
    a.inf = false;
    for (int i = 0; i < 8; i++) bw[i] = 0;
  }
  if (__lane_id() == 0) {
    out37[0] = (uint8_t)(id >> 24);
    out37[1] = (uint8_t)(id >> 16);
    out37[2] = (uint8_t)(id >> 8);
    out37[3] = (uint8_t)id;
    g1_compress(out37 + 4, a);
  }
}

// H = g1_map(msg) into d_H (bls_hash_kernel), then the row-parallel signature
hipError_t cbft_bls_launch_sign_row(const uint32_t* d_H, const uint32_t* d_sk, const uint8_t* d_msg, uint32_t len,
                                    uint32_t id, uint8_t* d_out37, hipStream_t s) {
  hipLaunchKernelGGL(bls_sign_row_kernel, dim3(1), dim3(128), 0, s, d_H, d_sk, d_msg, len, id, d_out37);
  return hipGetLastError();
}
