// GF(2^255 - 19) arithmetic for gfx950, one field element per lane.
//
// Representation ("fe"): 9 unsigned 32-bit limbs in radix 2^29 (261 bits, redundant).
//   value = sum_i v[i] * 2^(29 i)   (mod p),   2^261 == 64*19 = 1216 (mod p)
//
// Why radix 2^29 x 9: the only wide multiplier on the CDNA4 VALU is v_mad_u64_u32
// (32x32+64 -> 64), measured on MI355X at half the v_add_u32 issue rate
// (tools/microbench/intrate.hip; 24-bit mads and FP64 FMA are no faster).  With 29-bit
// limbs a whole product column (<= 9 products of <= 2^60.003) plus carry-in fits in one
// 64-bit accumulator, so every partial product is exactly ONE v_mad_u64_u32 with no carry
// chain; 81 mads + 9 fold mads per multiply, 45 + 9 per square.  Two bits of headroom let
// a lazy sum of two reduced elements feed a multiply directly.
//
// Bounds (checked in DESIGN.md §fe):
//   "reduced"  : every limb < 2^29 + 2^17        (outputs of mul/sq/carry/sub)
//   "lazy"     : every limb < 2^30 + 2^18        (sum of two reduced)
//   mul/sq inputs: each operand reduced or lazy.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fe25519_asm.h"
#include "safegcd30.h"

#define FE_LIMBS 9
#define FE_MASK 0x1fffffffu

struct fe {
  uint32_t v[FE_LIMBS];
};

#define FE_INLINE __device__ __forceinline__

FE_INLINE uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  return (uint64_t)a * (uint64_t)b + c;  // -> v_mad_u64_u32
}

FE_INLINE void fe_0(fe& r) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) r.v[i] = 0;
}
FE_INLINE void fe_1(fe& r) {
  fe_0(r);
  r.v[0] = 1;
}
FE_INLINE void fe_copy(fe& r, const fe& a) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) r.v[i] = a.v[i];
}

// lazy add: reduced + reduced -> lazy
FE_INLINE void fe_add(fe& r, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) r.v[i] = a.v[i] + b.v[i];
}

// carry pass on 32-bit limbs (< 2^32 - 8) -> reduced
FE_INLINE void fe_carry(fe& r) {
  uint32_t c;
#pragma unroll
  for (int i = 0; i < FE_LIMBS - 1; i++) {
    c = r.v[i] >> 29;
    r.v[i] &= FE_MASK;
    r.v[i + 1] += c;
  }
  c = r.v[8] >> 29;
  r.v[8] &= FE_MASK;
  r.v[0] += c * 1216u;
}

// r = a - b (mod p), b reduced or lazy, a reduced or lazy -> reduced.
// Adds 256p = 2^263 - 4864, whose radix-2^29 digits are (2^31-4864, 2^31-4, ..., 2^31-4),
// every one >= any lazy limb, so no limb underflows.
FE_INLINE void fe_sub(fe& r, const fe& a, const fe& b) {
  r.v[0] = a.v[0] + (0x80000000u - 4864u) - b.v[0];
#pragma unroll
  for (int i = 1; i < FE_LIMBS; i++) r.v[i] = a.v[i] + (0x80000000u - 4u) - b.v[i];
  fe_carry(r);
}

// r = -a
FE_INLINE void fe_neg(fe& r, const fe& a) {
  r.v[0] = (0x80000000u - 4864u) - a.v[0];
#pragma unroll
  for (int i = 1; i < FE_LIMBS; i++) r.v[i] = (0x80000000u - 4u) - a.v[i];
  fe_carry(r);
}

// Column-sum multiply core.  col(k) = sum_{i+j=k} a_i b_j (as mads into a 64-bit acc).
//   High columns k = 9..16 are computed first and carried into 29-bit digits h0..h7 and an
//   unbounded top h8 (weight 2^261 * 2^(29(k-9)) == 1216 * 2^(29(k-9))); then the low
//   columns start their mad chains from (carry + 1216 h_k); the final carry (weight 2^261)
//   wraps with *1216 into limb 0.  Live state: operands + h[9] + one accumulator.
//
// The whole product is ONE dependent chain of v_mad_u64_u32 (each column's chain starts from the
// previous column's carry).  The mads are written as (non-volatile) inline asm so that LLVM cannot
// reassociate the chain into per-column partial sums: that costs a v_lshl_add_u64 per column to
// merge the carry back in (4.7 cycles per wave-instruction at 4 waves/SIMD), while the chain's
// latency is free -- on gfx950 a dependent mad chain issues at the same rate as eight independent
// ones from 1 to 16 waves per SIMD (tools/microbench/intrate2.hip, profiles/r02_intrate2.txt).
#define FE_COLUMN(acc, k, TERM)                                  \
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; i++) {         \
    int j = (k) - i;                                             \
    if (j >= 0 && j < FE_LIMBS) { TERM }                         \
  }

// CBFT_FE_CHAIN: default for the template argument C of the multiply family; kernels whose
// waves run alone on a SIMD (the inversion chains of K4) pass C = false: there the hazard nops
// between dependent asm mads cost issue slots no other wave can use.
#ifndef CBFT_FE_CHAIN
#define CBFT_FE_CHAIN 1
#endif

// acc += a * b (CHAIN: one v_mad_u64_u32, not reassociable)
template <bool CHAIN>
FE_INLINE void mac(uint64_t& acc, uint32_t a, uint32_t b) {
  if (CHAIN) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(a), "v"(b));
  } else {
    acc = mad64(a, b, acc);
  }
}
// acc += a * 1216 (the 2^261 fold; the constant rides in an SGPR)
template <bool CHAIN>
FE_INLINE void mac1216(uint64_t& acc, uint32_t a) {
  if (CHAIN) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(a), "s"(1216u));
  } else {
    acc = mad64(a, 1216u, acc);
  }
}

// CBFT_FE_ASMCOL: each column's whole mad chain is ONE inline-asm block.  The compiler puts an
// s_nop after every inline-asm statement (it cannot see the hazard state inside the text), so
// the one-asm-per-mad chain paid ~90 s_nop per multiply (480 per comb addition, ISA of the pair
// ladder); with one block per column it is 17.  Same instructions otherwise, same order.
#ifndef CBFT_FE_ASMCOL
#define CBFT_FE_ASMCOL 1
#endif
// Repetition helpers: CBFT_RL_n(M) = M(0) M(1) .. M(n-1) (asm text), CBFT_RC_n(M) the same
// comma-separated (asm operands).
#define CBFT_RL_1(M) M(0)
#define CBFT_RL_2(M) CBFT_RL_1(M) M(1)
#define CBFT_RL_3(M) CBFT_RL_2(M) M(2)
#define CBFT_RL_4(M) CBFT_RL_3(M) M(3)
#define CBFT_RL_5(M) CBFT_RL_4(M) M(4)
#define CBFT_RL_6(M) CBFT_RL_5(M) M(5)
#define CBFT_RL_7(M) CBFT_RL_6(M) M(6)
#define CBFT_RL_8(M) CBFT_RL_7(M) M(7)
#define CBFT_RL_9(M) CBFT_RL_8(M) M(8)
#define CBFT_RL_10(M) CBFT_RL_9(M) M(9)
#define CBFT_RC_1(M) M(0)
#define CBFT_RC_2(M) CBFT_RC_1(M), M(1)
#define CBFT_RC_3(M) CBFT_RC_2(M), M(2)
#define CBFT_RC_4(M) CBFT_RC_3(M), M(3)
#define CBFT_RC_5(M) CBFT_RC_4(M), M(4)
#define CBFT_RC_6(M) CBFT_RC_5(M), M(5)
#define CBFT_RC_7(M) CBFT_RC_6(M), M(6)
#define CBFT_RC_8(M) CBFT_RC_7(M), M(7)
#define CBFT_RC_9(M) CBFT_RC_8(M), M(8)
#define CBFT_RC_10(M) CBFT_RC_9(M), M(9)

#define CBFT_MC_LINE(p) "v_mad_u64_u32 %[acc], %[cc], %[x" #p "], %[y" #p "], %[acc]\n\t"
#define CBFT_MC_IN(p) [x##p] "v"(x[p]), [y##p] "v"(y[p])
#define CBFT_MC_CASE(n) \
  else if constexpr (N == n) asm(CBFT_RL_##n(CBFT_MC_LINE) : [acc] "+v"(acc), [cc] "=s"(cc) : CBFT_RC_##n(CBFT_MC_IN));
// acc += sum_{p < N} x[p] * y[p] as one dependent v_mad_u64_u32 chain (one asm statement)
template <int N>
FE_INLINE void mad_chain(uint64_t& acc, const uint32_t* x, const uint32_t* y) {
  uint64_t cc;
  static_assert(N >= 1 && N <= 10, "mad_chain: 1..10 products");
  if constexpr (N == 0) {
  }
  CBFT_MC_CASE(1) CBFT_MC_CASE(2) CBFT_MC_CASE(3) CBFT_MC_CASE(4) CBFT_MC_CASE(5)
  CBFT_MC_CASE(6) CBFT_MC_CASE(7) CBFT_MC_CASE(8) CBFT_MC_CASE(9) CBFT_MC_CASE(10)
}

// Two independent chains in one asm statement, their mads alternating: a1 += sum x y,
// a2 += sum u w (a wave then always has an independent mad ready behind a dependent one).
#define CBFT_MC2_LINE(p)                                                  \
  "v_mad_u64_u32 %[a1], %[c1], %[x" #p "], %[y" #p "], %[a1]\n\t"       \
  "v_mad_u64_u32 %[a2], %[c2], %[u" #p "], %[w" #p "], %[a2]\n\t"
#define CBFT_MC2_IN(p) [x##p] "v"(x[p]), [y##p] "v"(y[p]), [u##p] "v"(u[p]), [w##p] "v"(w[p])
#define CBFT_MC2_CASE(n)                                                                                  \
  else if constexpr (N == n) asm(CBFT_RL_##n(CBFT_MC2_LINE)                                               \
                                 : [a1] "+v"(a1), [a2] "+v"(a2), [c1] "=s"(c1), [c2] "=s"(c2)               \
                                 : CBFT_RC_##n(CBFT_MC2_IN));
template <int N>
FE_INLINE void mad_chain2(uint64_t& a1, const uint32_t* x, const uint32_t* y, uint64_t& a2, const uint32_t* u,
                          const uint32_t* w) {
  uint64_t c1, c2;
  static_assert(N >= 1 && N <= 10, "mad_chain2: 1..10 products");
  if constexpr (N == 0) {
  }
  CBFT_MC2_CASE(1) CBFT_MC2_CASE(2) CBFT_MC2_CASE(3) CBFT_MC2_CASE(4) CBFT_MC2_CASE(5)
  CBFT_MC2_CASE(6) CBFT_MC2_CASE(7) CBFT_MC2_CASE(8) CBFT_MC2_CASE(9) CBFT_MC2_CASE(10)
}

// Column k of a x b (products a_i b_{k-i}) plus, when F, a leading fold term f * 1216, as one chain
template <int K, bool F>
FE_INLINE void fe_column(uint64_t& acc, const fe& a, const fe& b, uint32_t f) {
  constexpr int LO = K < FE_LIMBS ? 0 : K - FE_LIMBS + 1;
  constexpr int HI = K < FE_LIMBS ? K : FE_LIMBS - 1;
  constexpr int N = HI - LO + 1 + (F ? 1 : 0);
  uint32_t x[N], y[N];
  int p = 0;
  if (F) {
    x[0] = f;
    y[0] = 1216u;
    p = 1;
  }
#pragma unroll
  for (int i = LO; i <= HI; i++, p++) {
    x[p] = a.v[i];
    y[p] = b.v[K - i];
  }
  mad_chain<N>(acc, x, y);
}
// Column k of a^2 (a2 = 2a): a2_i a_j for i < j plus a_{k/2}^2, and the optional fold term
template <int K, bool F>
FE_INLINE void fe_sq_column(uint64_t& acc, const fe& a, const uint32_t* a2, uint32_t f) {
  constexpr int LO = K < FE_LIMBS ? 0 : K - FE_LIMBS + 1;
  constexpr int NP = (K - LO + 1) / 2 - ((K - LO + 1) % 2 == 0 ? 0 : 0);  // pairs i < j with i >= LO
  constexpr int NPAIRS = ((K & 1) ? (K + 1) / 2 : K / 2) - LO;
  constexpr int N = NPAIRS + ((K & 1) ? 0 : 1) + (F ? 1 : 0);
  (void)NP;
  uint32_t x[N], y[N];
  int p = 0;
  if (F) {
    x[0] = f;
    y[0] = 1216u;
    p = 1;
  }
#pragma unroll
  for (int i = LO; 2 * i < K; i++, p++) {
    x[p] = a2[i];
    y[p] = a.v[K - i];
  }
  if ((K & 1) == 0) {
    x[p] = a.v[K >> 1];
    y[p] = a.v[K >> 1];
  }
  mad_chain<N>(acc, x, y);
}

template <int K>
FE_INLINE void fe_mul_hi_cols(uint64_t& t, uint32_t* h, const fe& a, const fe& b) {
  if constexpr (K < 17) {
    fe_column<K, false>(t, a, b, 0u);
    h[K - 9] = (uint32_t)t & FE_MASK;
    t >>= 29;
    fe_mul_hi_cols<K + 1>(t, h, a, b);
  }
}
template <int K>
FE_INLINE void fe_mul_lo_cols(uint64_t& acc, uint32_t* o, const uint32_t* h, const fe& a, const fe& b) {
  if constexpr (K < 9) {
    fe_column<K, true>(acc, a, b, h[K]);
    o[K] = (uint32_t)acc & FE_MASK;
    acc >>= 29;
    fe_mul_lo_cols<K + 1>(acc, o, h, a, b);
  }
}
template <int K>
FE_INLINE void fe_sq_hi_cols(uint64_t& t, uint32_t* h, const fe& a, const uint32_t* a2) {
  if constexpr (K < 17) {
    fe_sq_column<K, false>(t, a, a2, 0u);
    h[K - 9] = (uint32_t)t & FE_MASK;
    t >>= 29;
    fe_sq_hi_cols<K + 1>(t, h, a, a2);
  }
}
template <int K>
FE_INLINE void fe_sq_lo_cols(uint64_t& acc, uint32_t* o, const uint32_t* h, const fe& a, const uint32_t* a2) {
  if constexpr (K < 9) {
    fe_sq_column<K, true>(acc, a, a2, h[K]);
    o[K] = (uint32_t)acc & FE_MASK;
    acc >>= 29;
    fe_sq_lo_cols<K + 1>(acc, o, h, a, a2);
  }
}

// Two independent products, r1 = a1 b1 and r2 = a2 b2, column by column with the two mad chains
// interleaved in one asm statement per column (same arithmetic as fe_mul for each).
template <int K, bool F>
FE_INLINE void fe_column2(uint64_t& acc1, const fe& a1, const fe& b1, uint32_t f1, uint64_t& acc2, const fe& a2,
                          const fe& b2, uint32_t f2) {
  constexpr int LO = K < FE_LIMBS ? 0 : K - FE_LIMBS + 1;
  constexpr int HI = K < FE_LIMBS ? K : FE_LIMBS - 1;
  constexpr int N = HI - LO + 1 + (F ? 1 : 0);
  uint32_t x[N], y[N], u[N], w[N];
  int p = 0;
  if (F) {
    x[0] = f1;
    y[0] = 1216u;
    u[0] = f2;
    w[0] = 1216u;
    p = 1;
  }
#pragma unroll
  for (int i = LO; i <= HI; i++, p++) {
    x[p] = a1.v[i];
    y[p] = b1.v[K - i];
    u[p] = a2.v[i];
    w[p] = b2.v[K - i];
  }
  mad_chain2<N>(acc1, x, y, acc2, u, w);
}
template <int K>
FE_INLINE void fe_mul2_hi_cols(uint64_t& t1, uint32_t* h1, const fe& a1, const fe& b1, uint64_t& t2, uint32_t* h2,
                               const fe& a2, const fe& b2) {
  if constexpr (K < 17) {
    fe_column2<K, false>(t1, a1, b1, 0u, t2, a2, b2, 0u);
    h1[K - 9] = (uint32_t)t1 & FE_MASK;
    t1 >>= 29;
    h2[K - 9] = (uint32_t)t2 & FE_MASK;
    t2 >>= 29;
    fe_mul2_hi_cols<K + 1>(t1, h1, a1, b1, t2, h2, a2, b2);
  }
}
template <int K>
FE_INLINE void fe_mul2_lo_cols(uint64_t& c1, uint32_t* o1, const uint32_t* h1, const fe& a1, const fe& b1,
                               uint64_t& c2, uint32_t* o2, const uint32_t* h2, const fe& a2, const fe& b2) {
  if constexpr (K < 9) {
    fe_column2<K, true>(c1, a1, b1, h1[K], c2, a2, b2, h2[K]);
    o1[K] = (uint32_t)c1 & FE_MASK;
    c1 >>= 29;
    o2[K] = (uint32_t)c2 & FE_MASK;
    c2 >>= 29;
    fe_mul2_lo_cols<K + 1>(c1, o1, h1, a1, b1, c2, o2, h2, a2, b2);
  }
}
FE_INLINE void fe_mul_final(fe& o, uint64_t acc) {
  uint64_t w = acc * 1216ull + (uint64_t)o.v[0];
  o.v[0] = (uint32_t)w & FE_MASK;
  o.v[1] += (uint32_t)(w >> 29);
}
// r1 = a1 * b1, r2 = a2 * b2 (either output may alias any input)
FE_INLINE void fe_mul2(fe& r1, const fe& a1, const fe& b1, fe& r2, const fe& a2, const fe& b2) {
  fe o1, o2;
  uint32_t h1[9], h2[9];
  uint64_t t1 = 0, t2 = 0;
  fe_mul2_hi_cols<9>(t1, h1, a1, b1, t2, h2, a2, b2);
  h1[8] = (uint32_t)t1;
  h2[8] = (uint32_t)t2;
  uint64_t c1 = 0, c2 = 0;
  fe_mul2_lo_cols<0>(c1, o1.v, h1, a1, b1, c2, o2.v, h2, a2, b2);
  fe_mul_final(o1, c1);
  fe_mul_final(o2, c2);
  r1 = o1;
  r2 = o2;
}

// CBFT_FE_ONEASM: a whole multiply / square (fe25519_asm.h, generated by tools/gen/fe25519_asm.py:
// the same mads in the same order as the column-per-statement form) as ONE asm statement.  The
// compiler puts an s_nop between an asm statement and an instruction right after it that reads
// its results, since it cannot see inside the text: 17 per multiply with a statement per column,
// 1 with one statement.  The accumulator is pinned to v[20:21] so the text can split its digits.
#ifndef CBFT_FE_ONEASM
#define CBFT_FE_ONEASM 1
#endif
#define CBFT_FE_ASM_OUT                                                                                \
  [acc] "=&{v[20:21]}"(acc), [cc] "=s"(cc), [o0] "=&v"(o.v[0]), [o1] "=&v"(o.v[1]), [o2] "=&v"(o.v[2]), \
      [o3] "=&v"(o.v[3]), [o4] "=&v"(o.v[4]), [o5] "=&v"(o.v[5]), [o6] "=&v"(o.v[6]), [o7] "=&v"(o.v[7]), \
      [o8] "=&v"(o.v[8]), [h0] "=&v"(h[0]), [h1] "=&v"(h[1]), [h2] "=&v"(h[2]), [h3] "=&v"(h[3]),      \
      [h4] "=&v"(h[4]), [h5] "=&v"(h[5]), [h6] "=&v"(h[6]), [h7] "=&v"(h[7]), [h8] "=&v"(h[8])
#define CBFT_FE_ASM_IN9(N, X)                                                                     \
  [N##0] "v"(X[0]), [N##1] "v"(X[1]), [N##2] "v"(X[2]), [N##3] "v"(X[3]), [N##4] "v"(X[4]),    \
      [N##5] "v"(X[5]), [N##6] "v"(X[6]), [N##7] "v"(X[7]), [N##8] "v"(X[8])
FE_INLINE void fe_oneasm_final(fe& r, fe& o, uint64_t acc) {
  // acc < 2^34.2: carry of weight 2^261 == 1216
  uint64_t w = acc * 1216ull + (uint64_t)o.v[0];
  o.v[0] = (uint32_t)w & FE_MASK;
  o.v[1] += (uint32_t)(w >> 29);
  r = o;
}
FE_INLINE void fe_mul_oneasm(fe& r, const fe& a, const fe& b) {
  fe o;
  uint32_t h[9];
  uint64_t acc, cc;
  asm(CBFT_FE_MUL_ASM : CBFT_FE_ASM_OUT : CBFT_FE_ASM_IN9(a, a.v), CBFT_FE_ASM_IN9(b, b.v), [k1216] "v"(1216u));
  fe_oneasm_final(r, o, acc);
}
FE_INLINE void fe_sq_oneasm(fe& r, const fe& a, const uint32_t* a2) {
  fe o;
  uint32_t h[9];
  uint64_t acc, cc;
  asm(CBFT_FE_SQ_ASM : CBFT_FE_ASM_OUT : CBFT_FE_ASM_IN9(a, a.v), CBFT_FE_ASM_IN9(d, a2), [k1216] "v"(1216u));
  fe_oneasm_final(r, o, acc);
}

template <bool C = CBFT_FE_CHAIN>
FE_INLINE void fe_mul(fe& r, const fe& a, const fe& b) {
#if CBFT_FE_ASMCOL
  if (C && CBFT_FE_ONEASM) {
    fe_mul_oneasm(r, a, b);
    return;
  }
  if (C) {
    fe o;
    uint32_t h[9];
    uint64_t t = 0;
    fe_mul_hi_cols<9>(t, h, a, b);
    h[8] = (uint32_t)t;
    uint64_t acc = 0;
    fe_mul_lo_cols<0>(acc, o.v, h, a, b);
    uint64_t w = acc * 1216ull + (uint64_t)o.v[0];
    o.v[0] = (uint32_t)w & FE_MASK;
    o.v[1] += (uint32_t)(w >> 29);
    r = o;
    return;
  }
#endif
  fe o;  // r may alias a or b
  uint32_t h[9];
  uint64_t t = 0;
#pragma unroll
  for (int k = 9; k < 17; k++) {
    FE_COLUMN(t, k, mac<C>(t, a.v[i], b.v[j]);)
    h[k - 9] = (uint32_t)t & FE_MASK;
    t >>= 29;
  }
  h[8] = (uint32_t)t;  // < 2^32 (c16 <= 2^60.003 + carry)
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    mac1216<C>(acc, h[k]);
    FE_COLUMN(acc, k, mac<C>(acc, a.v[i], b.v[j]);)
    o.v[k] = (uint32_t)acc & FE_MASK;
    acc >>= 29;
  }
  // acc < 2^34.2: carry of weight 2^261 == 1216
  uint64_t w = acc * 1216ull + (uint64_t)o.v[0];
  o.v[0] = (uint32_t)w & FE_MASK;
  o.v[1] += (uint32_t)(w >> 29);
  r = o;
}

template <bool C = CBFT_FE_CHAIN>
FE_INLINE void fe_sq(fe& r, const fe& a) {
  fe o;  // r may alias a or b
  uint32_t a2[FE_LIMBS];
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) a2[i] = a.v[i] << 1;
#if CBFT_FE_ASMCOL
  if (C && CBFT_FE_ONEASM) {
    fe_sq_oneasm(r, a, a2);
    return;
  }
  if (C) {
    uint32_t h[9];
    uint64_t t = 0;
    fe_sq_hi_cols<9>(t, h, a, a2);
    h[8] = (uint32_t)t;
    uint64_t acc = 0;
    fe_sq_lo_cols<0>(acc, o.v, h, a, a2);
    uint64_t w = acc * 1216ull + (uint64_t)o.v[0];
    o.v[0] = (uint32_t)w & FE_MASK;
    o.v[1] += (uint32_t)(w >> 29);
    r = o;
    return;
  }
#endif
  uint32_t h[9];
  uint64_t t = 0;
#pragma unroll
  for (int k = 9; k < 17; k++) {
    FE_COLUMN(t, k, if (j > i) mac<C>(t, a2[i], a.v[j]);)
    if ((k & 1) == 0) mac<C>(t, a.v[k >> 1], a.v[k >> 1]);
    h[k - 9] = (uint32_t)t & FE_MASK;
    t >>= 29;
  }
  h[8] = (uint32_t)t;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    mac1216<C>(acc, h[k]);
    FE_COLUMN(acc, k, if (j > i) mac<C>(acc, a2[i], a.v[j]);)
    if ((k & 1) == 0) mac<C>(acc, a.v[k >> 1], a.v[k >> 1]);
    o.v[k] = (uint32_t)acc & FE_MASK;
    acc >>= 29;
  }
  uint64_t w = acc * 1216ull + (uint64_t)o.v[0];
  o.v[0] = (uint32_t)w & FE_MASK;
  o.v[1] += (uint32_t)(w >> 29);
  r = o;
}

// r = a * small (small < 2^16), a reduced/lazy
FE_INLINE void fe_mul_small(fe& r, const fe& a, uint32_t s) {
  uint64_t acc = 0;
  uint32_t t[FE_LIMBS];
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) {
    acc = mad64(a.v[i], s, acc);
    t[i] = (uint32_t)acc & FE_MASK;
    acc >>= 29;
  }
  uint64_t w = mad64((uint32_t)acc, 1216u, (uint64_t)t[0]);
  t[0] = (uint32_t)w & FE_MASK;
  t[1] += (uint32_t)(w >> 29);
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) r.v[i] = t[i];
}

// r = a^(2^n) (n >= 1); a runtime (not unrolled) loop keeps code size to one square body
template <bool C = CBFT_FE_CHAIN>
FE_INLINE void fe_sqn(fe& r, const fe& a, int n) {
  fe_sq<C>(r, a);
#pragma nounroll
  for (int i = 1; i < n; i++) fe_sq<C>(r, r);
}

// Canonical 8x32-bit little-endian words of a (fully reduced into [0, p)).
FE_INLINE void fe_to_words(uint32_t* w, const fe& a) {
  fe t;
  fe_copy(t, a);
  fe_carry(t);
  fe_carry(t);  // every limb < 2^29 now (limb0 < 2^29 + 2^14 after 1st, < 2^29 after 2nd w.h.p.)
  // fold bits >= 255 (limb 8 bits >= 23) twice
#pragma unroll
  for (int rep = 0; rep < 2; rep++) {
    uint32_t c = t.v[8] >> 23;
    t.v[8] &= 0x7fffffu;
    t.v[0] += 19u * c;
#pragma unroll
    for (int i = 0; i < FE_LIMBS - 1; i++) {
      uint32_t cc = t.v[i] >> 29;
      t.v[i] &= FE_MASK;
      t.v[i + 1] += cc;
    }
  }
  // now 0 <= t < 2^255 + tiny, t < 2p.  If t + 19 >= 2^255 then t >= p: t = t + 19 - 2^255.
  uint32_t u[FE_LIMBS];
  uint32_t c = 19;
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) {
    uint32_t s = t.v[i] + c;
    u[i] = s & FE_MASK;
    c = s >> 29;
  }
  bool ge = (u[8] >> 23) & 1u;
  u[8] &= 0x7fffffu;
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) t.v[i] = ge ? u[i] : t.v[i];
  // pack radix 2^29 -> 2^32
  w[0] = t.v[0] | (t.v[1] << 29);
  w[1] = (t.v[1] >> 3) | (t.v[2] << 26);
  w[2] = (t.v[2] >> 6) | (t.v[3] << 23);
  w[3] = (t.v[3] >> 9) | (t.v[4] << 20);
  w[4] = (t.v[4] >> 12) | (t.v[5] << 17);
  w[5] = (t.v[5] >> 15) | (t.v[6] << 14);
  w[6] = (t.v[6] >> 18) | (t.v[7] << 11);
  w[7] = (t.v[7] >> 21) | (t.v[8] << 8);
}

// Load 255 low bits of a little-endian 8-word integer (bit 255 ignored, value NOT reduced
// mod p: a non-canonical y >= p is accepted exactly as OpenSSL's fe_frombytes does).
FE_INLINE void fe_from_words(fe& r, const uint32_t* w) {
  r.v[0] = w[0] & FE_MASK;
  r.v[1] = ((w[0] >> 29) | (w[1] << 3)) & FE_MASK;
  r.v[2] = ((w[1] >> 26) | (w[2] << 6)) & FE_MASK;
  r.v[3] = ((w[2] >> 23) | (w[3] << 9)) & FE_MASK;
  r.v[4] = ((w[3] >> 20) | (w[4] << 12)) & FE_MASK;
  r.v[5] = ((w[4] >> 17) | (w[5] << 15)) & FE_MASK;
  r.v[6] = ((w[5] >> 14) | (w[6] << 18)) & FE_MASK;
  r.v[7] = ((w[6] >> 11) | (w[7] << 21)) & FE_MASK;
  r.v[8] = (w[7] >> 8) & 0x7fffffu;
}

FE_INLINE bool fe_iszero(const fe& a) {
  uint32_t w[8];
  fe_to_words(w, a);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= w[i];
  return o == 0;
}

FE_INLINE uint32_t fe_isnegative(const fe& a) {
  uint32_t w[8];
  fe_to_words(w, a);
  return w[0] & 1u;
}

FE_INLINE void fe_cmov(fe& r, const fe& a, bool c) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) r.v[i] = c ? a.v[i] : r.v[i];
}

// z^(2^250 - 1) and z^11: the shared prefix of inversion (p-2 = 2^255 - 21) and of the
// square-root power (p-5)/8 = 2^252 - 3.  Chain: 11 multiplies + 254 squarings in total.
template <bool C = CBFT_FE_CHAIN>
FE_INLINE void fe_pow_2_250_1(fe& z250, fe& z11, const fe& z) {
  fe z2, z9, t0, t1, t2;
  fe_sq<C>(z2, z);             // 2
  fe_sqn<C>(t0, z2, 2);        // 8
  fe_mul<C>(z9, t0, z);        // 9
  fe_mul<C>(z11, z9, z2);      // 11
  fe_sq<C>(t0, z11);           // 22
  fe_mul<C>(t0, t0, z9);       // 31 = 2^5 - 1
  fe_sqn<C>(t1, t0, 5);
  fe_mul<C>(t0, t1, t0);       // 2^10 - 1
  fe_sqn<C>(t1, t0, 10);
  fe_mul<C>(t1, t1, t0);       // 2^20 - 1
  fe_sqn<C>(t2, t1, 20);
  fe_mul<C>(t1, t2, t1);       // 2^40 - 1
  fe_sqn<C>(t1, t1, 10);
  fe_mul<C>(t0, t1, t0);       // 2^50 - 1
  fe_sqn<C>(t1, t0, 50);
  fe_mul<C>(t1, t1, t0);       // 2^100 - 1
  fe_sqn<C>(t2, t1, 100);
  fe_mul<C>(t1, t2, t1);       // 2^200 - 1
  fe_sqn<C>(t1, t1, 50);
  fe_mul<C>(z250, t1, t0);     // 2^250 - 1
}

// r = z^(p-2) = z^(2^255 - 21)
template <bool C = CBFT_FE_CHAIN>
FE_INLINE void fe_invert(fe& r, const fe& z) {
  fe z250, z11;
  fe_pow_2_250_1<C>(z250, z11, z);
  fe_sqn<C>(z250, z250, 5);    // 2^255 - 32
  fe_mul<C>(r, z250, z11);     // 2^255 - 21
}

// r = z^-1 for PUBLIC z (verification: R' of a signature, keys): safegcd30.h, variable time;
// 0 -> 0 like fe_invert.  One lane per inversion; ~6x fewer instructions than the Fermat chain,
// which is what the finish kernels' lone waves (batch-shared inversions, small batches) wait on.
struct Fe25519S30 {
  static constexpr int32_t P[9] = {0x3fffffed, 0x3fffffff, 0x3fffffff, 0x3fffffff, 0x3fffffff,
                                   0x3fffffff, 0x3fffffff, 0x3fffffff, 0x00007fff};
  static constexpr uint32_t PINV30 = 0x179435e5u;
};
// UNIFORM: z is the same in every lane of the wave (a finish block's tree root): the chain runs on
// the scalar unit (safegcd30.h sg_inv30_var_uniform), every lane receives the inverse.
template <bool UNIFORM = false>
FE_INLINE void fe_invert_var(fe& r, const fe& z0) {
  fe z = z0;
  if (UNIFORM) {
#pragma unroll
    for (int k = 0; k < FE_LIMBS; k++) z.v[k] = __builtin_amdgcn_readfirstlane(z0.v[k]);
  }
  uint32_t w[8];
  fe_to_words(w, z);  // canonical, [0, p)
  Sg30 x;
#pragma unroll
  for (int j = 0; j < 9; j++) {  // 8 x 32-bit words -> 9 x 30-bit limbs
    const int b = 30 * j, i = b >> 5, sh = b & 31;
    const uint64_t v = ((uint64_t)(i + 1 < 8 ? w[i + 1] : 0u) << 32) | (i < 8 ? w[i] : 0u);
    x.v[j] = (int32_t)((v >> sh) & SG_M30);
  }
  sg_inv30_var<Fe25519S30>(x);
#pragma unroll
  for (int i = 0; i < 8; i++) {  // back to words
    const int b = 32 * i, j = b / 30, sh = b % 30;
    const uint64_t v = ((uint64_t)(uint32_t)(j + 2 < 9 ? x.v[j + 2] : 0) << 60) |
                       ((uint64_t)(uint32_t)(j + 1 < 9 ? x.v[j + 1] : 0) << 30) | (uint32_t)x.v[j];
    w[i] = (uint32_t)(v >> sh);
  }
  fe_from_words(r, w);
}

// r = z^((p-5)/8) = z^(2^252 - 3)
template <bool C = CBFT_FE_CHAIN>
FE_INLINE void fe_pow22523(fe& r, const fe& z) {
  fe z250, z11;
  fe_pow_2_250_1<C>(z250, z11, z);
  fe_sqn<C>(z250, z250, 2);    // 2^252 - 4
  fe_mul<C>(r, z250, z);       // 2^252 - 3
}
