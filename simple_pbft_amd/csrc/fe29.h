// fe29.h -- P-256 field (mod p) and scalar (mod n) arithmetic for gfx950.
//
// Representation: 9 limbs of 29 bits (value = sum v[i] * 2^(29 i)), Montgomery
// form with R = 2^261.  Why 29-bit limbs on CDNA4 (DESIGN.md "Field arithmetic"):
// v_mad_u64_u32 issues at the same rate as a carry-propagating add
// (profiles/r01_valu_microbench.txt), so the cheapest multiply is one that
// never handles a carry while accumulating.  With limbs < 2^30 every partial
// product is < 2^60 and a column of 9 of them fits a 64-bit accumulator, so
// the 81 products are 81 v_mad_u64_u32 into 17 independent column
// accumulators and nothing else.
//
// Reduction mod p exploits p = 2^256 - 2^224 + 2^192 + 2^96 - 1 == -1 (mod 2^29):
// the Montgomery quotient digit is m = t_i mod 2^29 (p' = 1) and m*p lands on
// columns i+3, i+6, i+7, i+8 as m<<9, m<<18, -(m<<21), m<<24.  The negative
// term is folded into its neighbour: -m 2^224 + m 2^256 = m (2^29 - 2^21) in
// column i+7 + m (2^24 - 1) in column i+8, so the digit step is four MADs by
// positive SGPR constants (2^9, 2^18, kC21, kC24), no negation, no bias.
//
// Value/limb invariants (checked by tests/test_algo_cpu.py on CPU).  A Montgomery
// product satisfies out < a*b/2^261 + p + 2^225, whose fixed point gives:
//   M-type (fe_mul/fe_sqr output): limbs < 2^29, value < 1.172 * 2^256
//   N-type (fe_sub/fe_norm/fe_mul_small output): limbs < 2^29, value < 2^256 + 2^237
//   L-type (fe_add of two M/N values): limbs < 2^30, value < 2.344 * 2^256
//   fe_mul/fe_sqr inputs: any two of M/N/L (limbs < 2^30 keep every column < 2^64)
//   fe_sub inputs: any of M/N/L (a - b + 4p > 0 since b < 2.344 * 2^256 < 4p)
//
// Compiled by hipcc for the device and by g++ for the CPU test harness only
// (tests/cpp); the product library runs it on the GPU exclusively.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define PBFTV_HD __host__ __device__ __forceinline__
#define PBFTV_HDM __host__ __device__  // member functions
#define PBFTV_UNROLL _Pragma("unroll")
#else
#define PBFTV_HD static inline
#define PBFTV_HDM
#define PBFTV_UNROLL
#endif

#include "p256_consts.h"

namespace pbftv {

constexpr uint32_t kMask29 = (1u << 29) - 1;

struct fe {
  uint32_t v[9];
};

PBFTV_HD void fe_set(fe& r, const uint32_t c[9]) {
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) r.v[i] = c[i];
}

// 8 little-endian 32-bit words (value < 2^256) -> 9 limbs
PBFTV_HD void fe_from_words(fe& r, const uint32_t w[8]) {
  r.v[0] = w[0] & kMask29;
  PBFTV_UNROLL for (int i = 1; i < 8; ++i) {
    const int bit = 29 * i, wi = bit >> 5, sh = bit & 31;
    uint32_t lo = w[wi] >> sh;
    uint32_t hi = (sh && wi + 1 < 8) ? (w[wi + 1] << (32 - sh)) : 0u;
    r.v[i] = (lo | hi) & kMask29;
  }
  r.v[8] = w[7] >> 8;  // bits 232..255
}

// 9 normalised limbs (value < 2^256) -> 8 little-endian 32-bit words
PBFTV_HD void fe_to_words(uint32_t w[8], const fe& a) {
  PBFTV_UNROLL for (int k = 0; k < 8; ++k) {
    const int bit = 32 * k, li = bit / 29, sh = bit % 29;
    uint32_t x = a.v[li] >> sh;
    if (li + 1 < 9) x |= a.v[li + 1] << (29 - sh);
    if (sh > 26 && li + 2 < 9) x |= a.v[li + 2] << (58 - sh);
    w[k] = x;
  }
}

// ---------------------------------------------------------------------------
// signed carry normalisation + fold of bits >= 2^256 (2^256 == 2^224 - 2^192 - 2^96 + 1)
PBFTV_HD void fe_carry_signed(int32_t d[9]) {
  PBFTV_UNROLL for (int i = 0; i < 8; ++i) {
    d[i + 1] += d[i] >> 29;  // arithmetic shift
    d[i] &= (int32_t)kMask29;
  }
}

PBFTV_HD void fe_fold_signed(fe& r, int32_t d[9]) {
  // d: limbs 0..7 in [0,2^29), d[8] >= 0 holds bits 232.. (value < 2^259)
  const int32_t top = d[8] >> 24;
  d[8] &= 0xFFFFFF;
  d[0] += top;
  d[3] -= top << 9;
  d[6] -= top << 18;
  d[7] += top << 21;
  fe_carry_signed(d);
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) r.v[i] = (uint32_t)d[i];
}

// Single-pass normalise + fold of signed limbs d (|d_i| < 2^31 - 2^26).  The
// part of limb 8 at and above bit 24 (value bits >= 256) is folded in BEFORE
// the carry pass via 2^256 == 2^224 - 2^192 - 2^96 + 1 (mod p), with the
// quotient taken 4 low (floor((d_8 - 4) / 2^24)) so limb 8 ends in
// [4, 2^24 + 4) before carries and, since the carry arriving from limb 7 is in
// [-4, 4], >= 0 after.  The result is therefore a non-negative N-type
// representative for ANY sign of the input value: no multiple of p needs to
// be added for subtraction.
PBFTV_HD void fe_fold_carry(fe& r, int32_t d[9]) {
  const int32_t top = (d[8] - 4) >> 24;
  d[8] -= top << 24;
  d[0] += top;
  d[3] -= top << 9;
  d[6] -= top << 18;
  d[7] += top << 21;
  fe_carry_signed(d);
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) r.v[i] = (uint32_t)d[i];
}

// r = a - b (mod p) as N-type (a, b any of M/N/L: |a_i - b_i| < 2^30).
PBFTV_HD void fe_sub(fe& r, const fe& a, const fe& b) {
  int32_t d[9];
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) d[i] = (int32_t)a.v[i] - (int32_t)b.v[i];
  fe_fold_carry(r, d);
}

// lazy r = a + b (L-type: only as fe_mul/fe_sqr/fe_sub input)
PBFTV_HD void fe_add(fe& r, const fe& a, const fe& b) {
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] + b.v[i];
}

// r = k * a mod p (1 <= k <= 3, a limbs < 2^29) as N-type
PBFTV_HD void fe_mul_small(fe& r, const fe& a, uint32_t k) {
  int32_t d[9];
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) d[i] = (int32_t)(a.v[i] * k);
  fe_fold_carry(r, d);
}

// normalise an L-type value to N-type
PBFTV_HD void fe_norm(fe& r, const fe& a) {
  int32_t d[9];
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) d[i] = (int32_t)a.v[i];
  fe_fold_carry(r, d);
}

// r = 2p - a, lazily (a canonical or N-type with limbs < 2^29): limbs < 2^30, value < 2^257
PBFTV_HD void fe_neg_lazy(fe& r, const fe& a) {
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) r.v[i] = kP2Borrow[i] - a.v[i];
}

// digit-step multipliers for columns i+7 and i+8 (see the header)
constexpr uint32_t kC21 = (1u << 29) - (1u << 21);
constexpr uint32_t kC24 = (1u << 24) - 1u;

// A power of two the compiler cannot see: on the device, m * opaque(2^k) + t
// becomes ONE v_mad_u64_u32 (multiplier in an SGPR) instead of a 64-bit
// shift plus v_lshl_add_u64 (whose shift field only reaches 4).
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ uint32_t opaque_u32(uint32_t c) {
  uint32_t r;
  asm("s_mov_b32 %0, %1" : "=s"(r) : "i"(c));
  return r;
}
#else
static inline uint32_t opaque_u32(uint32_t c) { return c; }
#endif

// Montgomery reduction of the 17 column accumulators (t[17] is scratch).
PBFTV_HD void fe_mont_reduce_p(fe& r, uint64_t t[18]) {
  const uint32_t c9 = opaque_u32(1u << 9), c18 = opaque_u32(1u << 18), c21 = opaque_u32(kC21),
                 c24 = opaque_u32(kC24);
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    const uint32_t m = (uint32_t)t[i] & kMask29;
    t[i + 1] += t[i] >> 29;
    t[i + 3] += (uint64_t)m * c9;
    t[i + 6] += (uint64_t)m * c18;
    t[i + 7] += (uint64_t)m * c21;
    t[i + 8] += (uint64_t)m * c24;
  }
  PBFTV_UNROLL for (int j = 9; j < 16; ++j) {
    r.v[j - 9] = (uint32_t)t[j] & kMask29;
    t[j + 1] += t[j] >> 29;
  }
  r.v[7] = (uint32_t)t[16] & kMask29;
  r.v[8] = (uint32_t)(t[16] >> 29);
}

// One Montgomery digit step at column i (the body of fe_mont_reduce_p's loop).
PBFTV_HD void fe_mont_digit_p(uint64_t t[18], int i, uint32_t c9, uint32_t c18, uint32_t c21, uint32_t c24) {
  const uint32_t m = (uint32_t)t[i] & kMask29;
  t[i + 1] += t[i] >> 29;
  t[i + 3] += (uint64_t)m * c9;
  t[i + 6] += (uint64_t)m * c18;
  t[i + 7] += (uint64_t)m * c21;
  t[i + 8] += (uint64_t)m * c24;
}

PBFTV_HD void fe_mont_out_p(fe& r, uint64_t t[18]) {
  PBFTV_UNROLL for (int j = 9; j < 16; ++j) {
    r.v[j - 9] = (uint32_t)t[j] & kMask29;
    t[j + 1] += t[j] >> 29;
  }
  r.v[7] = (uint32_t)t[16] & kMask29;
  r.v[8] = (uint32_t)(t[16] >> 29);
}

// r = a * b * 2^-261 mod p (M-type).  The reduction is interleaved with the
// products: column i is final once product row i is in, so digit step i is
// issued right after that row and its serial carry overlaps the next row's
// independent multiply-adds (tools/fmul_bench.hip: 772 vs 856 SIMD-cycles per
// wave at 2 waves/SIMD).  Same sums in the same columns as
// fe_mul_rows_then_reduce -- identical results.
PBFTV_HD void fe_mul(fe& r, const fe& a, const fe& b) {
  const uint32_t c9 = opaque_u32(1u << 9), c18 = opaque_u32(1u << 18), c21 = opaque_u32(kC21),
                 c24 = opaque_u32(kC24);
  uint64_t t[18];
  PBFTV_UNROLL for (int k = 0; k < 9; ++k) t[k] = 0;
  PBFTV_UNROLL for (int k = 9; k < 18; ++k) t[k] = 0;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    PBFTV_UNROLL for (int j = 0; j < 9; ++j) t[i + j] += (uint64_t)a.v[i] * b.v[j];
    fe_mont_digit_p(t, i, c9, c18, c21, c24);
  }
  fe_mont_out_p(r, t);
}

// r = (a b + c d) * 2^-261 mod p (M-type): two products summed in the columns,
// ONE Montgomery reduction.  Column bound: a, b limbs < 2^29 and c < 2^30,
// d < 2^29 give < 9 (2^58 + 2^59) < 2^62.8 before the reduction's additions.
PBFTV_HD void fe_mul2_add(fe& r, const fe& a, const fe& b, const fe& c, const fe& d) {
  const uint32_t c9 = opaque_u32(1u << 9), c18 = opaque_u32(1u << 18), c21 = opaque_u32(kC21),
                 c24 = opaque_u32(kC24);
  uint64_t t[18];
  PBFTV_UNROLL for (int k = 0; k < 9; ++k) t[k] = 0;
  PBFTV_UNROLL for (int k = 9; k < 18; ++k) t[k] = 0;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    PBFTV_UNROLL for (int j = 0; j < 9; ++j) t[i + j] += (uint64_t)a.v[i] * b.v[j];
    PBFTV_UNROLL for (int j = 0; j < 9; ++j) t[i + j] += (uint64_t)c.v[i] * d.v[j];
    fe_mont_digit_p(t, i, c9, c18, c21, c24);
  }
  fe_mont_out_p(r, t);
}

// fe_sqr with the reduction interleaved (after square row i columns <= 2i+1
// are final); measured no faster than fe_sqr, kept for tools/fmul_bench.hip.
PBFTV_HD void fe_sqr_il(fe& r, const fe& a) {
  const uint32_t c9 = opaque_u32(1u << 9), c18 = opaque_u32(1u << 18), c21 = opaque_u32(kC21),
                 c24 = opaque_u32(kC24);
  uint64_t t[18];
  uint32_t a2[9];
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) a2[i] = a.v[i] << 1;
  PBFTV_UNROLL for (int k = 0; k < 9; ++k) t[k] = 0;
  PBFTV_UNROLL for (int k = 9; k < 18; ++k) t[k] = 0;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    t[2 * i] += (uint64_t)a.v[i] * a.v[i];
    PBFTV_UNROLL for (int j = i + 1; j < 9; ++j) t[i + j] += (uint64_t)a.v[i] * a2[j];
    if (2 * i < 9) fe_mont_digit_p(t, 2 * i, c9, c18, c21, c24);
    if (2 * i + 1 < 9) fe_mont_digit_p(t, 2 * i + 1, c9, c18, c21, c24);
  }
  fe_mont_out_p(r, t);
}

// r = a * b * 2^-261 mod p (M-type), all products first, then the reduction
// (kept as the reference schedule for tools/fmul_bench.hip; fe_mul below
// interleaves the two and is ~10 % faster on gfx950)
PBFTV_HD void fe_mul_rows_then_reduce(fe& r, const fe& a, const fe& b) {
  uint64_t t[18];
  PBFTV_UNROLL for (int k = 0; k < 9; ++k) t[k] = 0;
  PBFTV_UNROLL for (int k = 9; k < 18; ++k) t[k] = 0;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    PBFTV_UNROLL for (int j = 0; j < 9; ++j) t[i + j] += (uint64_t)a.v[i] * b.v[j];
  }
  fe_mont_reduce_p(r, t);
}

// r = a^2 * 2^-261 mod p (M-type): 45 products, cross terms doubled
PBFTV_HD void fe_sqr(fe& r, const fe& a) {
  uint64_t t[18];
  uint32_t a2[9];
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) a2[i] = a.v[i] << 1;
  PBFTV_UNROLL for (int k = 0; k < 9; ++k) t[k] = 0;
  PBFTV_UNROLL for (int k = 9; k < 18; ++k) t[k] = 0;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    t[2 * i] += (uint64_t)a.v[i] * a.v[i];
    PBFTV_UNROLL for (int j = i + 1; j < 9; ++j) t[i + j] += (uint64_t)a.v[i] * a2[j];
  }
  fe_mont_reduce_p(r, t);
}

// canonical representative in [0, p) of an M/N-type value (limbs < 2^29)
PBFTV_HD void fe_canon(fe& r, const fe& a) {
  int32_t d[9];
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) d[i] = (int32_t)a.v[i];
  fe n;
  fe_fold_signed(n, d);  // now < 2^256 + 2^231 < 2p
  int32_t s[9];
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) s[i] = (int32_t)n.v[i] - (int32_t)kP[i];
  fe_carry_signed(s);
  const bool ge = s[8] >= 0;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) r.v[i] = ge ? (uint32_t)s[i] : n.v[i];
}

PBFTV_HD bool fe_is_zero(const fe& a) {
  fe c;
  fe_canon(c, a);
  uint32_t o = 0;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) o |= c.v[i];
  return o == 0;
}

PBFTV_HD bool fe_equal(const fe& a, const fe& b) {
  fe d;
  fe_sub(d, a, b);
  return fe_is_zero(d);
}

// ---------------------------------------------------------------------------
// scalar field mod n: Montgomery (R = 2^261), generic quotient digit.
// Values kept < 2^257 (limbs < 2^29 after each multiply); inputs limbs < 2^30.
// Digit step i is interleaved right after product row i (column i is final
// then), as in fe_mul.
PBFTV_HD void fn_mul(fe& r, const fe& a, const fe& b) {
  uint64_t t[18];
  PBFTV_UNROLL for (int k = 0; k < 18; ++k) t[k] = 0;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    PBFTV_UNROLL for (int j = 0; j < 9; ++j) t[i + j] += (uint64_t)a.v[i] * b.v[j];
    const uint32_t m = ((uint32_t)t[i] * kNPrime) & kMask29;
    PBFTV_UNROLL for (int j = 0; j < 9; ++j) t[i + j] += (uint64_t)m * kN[j];
    t[i + 1] += t[i] >> 29;
  }
  PBFTV_UNROLL for (int j = 9; j < 16; ++j) {
    r.v[j - 9] = (uint32_t)t[j] & kMask29;
    t[j + 1] += t[j] >> 29;
  }
  r.v[7] = (uint32_t)t[16] & kMask29;
  r.v[8] = (uint32_t)(t[16] >> 29);
}

PBFTV_HD void fn_sqr(fe& r, const fe& a) { fn_mul(r, a, a); }

// canonical [0, n) of a value < 2n with limbs < 2^29
PBFTV_HD void fn_canon(fe& r, const fe& a) {
  int32_t s[9];
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) s[i] = (int32_t)a.v[i] - (int32_t)kN[i];
  fe_carry_signed(s);
  const bool ge = s[8] >= 0;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) r.v[i] = ge ? (uint32_t)s[i] : a.v[i];
}

// compare canonical-limb values: -1, 0, 1
PBFTV_HD int fe_cmp_words(const uint32_t a[8], const uint32_t b[8]) {
  for (int i = 7; i >= 0; --i) {
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  }
  return 0;
}

PBFTV_HD bool words_is_zero(const uint32_t a[8]) {
  uint32_t o = 0;
  PBFTV_UNROLL for (int i = 0; i < 8; ++i) o |= a[i];
  return o == 0;
}

}  // namespace pbftv
