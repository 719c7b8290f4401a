// fes.h -- signed-limb P-256 field arithmetic for the comb's hot loop (gfx950).
//
// Same numbers as fe29.h (9 limbs of 29 bits, value = sum v[i] 2^(29 i),
// Montgomery R = 2^261), but limbs are SIGNED 32-bit and products accumulate
// through v_mad_i64_i32 into signed 64-bit columns.  What that buys
// (DESIGN.md "Signed limbs"):
//   * a subtraction is 9 v_sub_u32 -- no carry chain, no fold of bits >= 2^256
//     (fe_sub: ~40 VALU instructions);
//   * the Montgomery digit of column i is its low 32 bits as they stand
//     (m = lo32(t_i) == t_i mod 2^29) and the column's carry is
//     hi32(t_i) * 8, ONE v_mad_i64_i32 -- no mask, no 64-bit shift + add
//     (fe29.h: and + v_lshrrev_b64 + v_lshl_add_u64).  The top digit is kept at
//     29 bits so the output stays below T / 2^261 + 1.0001 p;
//   * the -m 2^224 + m 2^256 terms of m p are added as m (2^29 - 2^21) into
//     column i+7 and m (2^24 - 1) into column i+8 (the same integer:
//     2^232 - 2^224 + 2^256 - 2^232): two MADs by positive constants, no
//     negation of m and no bias in the columns.
//
// Types (checked by tests/test_algo_cpu.py, CPU harness):
//   S (product output, fs_norm output): limbs 0..7 in [0, 2^29), limb 8 signed,
//       |value| < 2^257.5;
//   D (difference of two S): |limbs| < 2^29, |value| < 2^258.5;
//   canonical table coordinates and their negatives are D-type.
// Products need max|a_i| * max|b_j| <= 2^59 (columns stay below 2^62.3 in
// magnitude): S x S, S x D, D x D, and fs_mul2_add of two such pairs.
//
// Compiled by hipcc for the device and by g++ for the CPU test harness only.
#pragma once
#include "fe29.h"

namespace pbftv {

// a * b with both limbs taken as signed 32-bit (v_mad_i64_i32 on the device)
PBFTV_HD uint64_t smul(uint32_t a, uint32_t b) { return (uint64_t)((int64_t)(int32_t)a * (int64_t)(int32_t)b); }

// Column bound with the digit terms: products (<= 18 of |x| <= 2^58, or 9 of
// 2^59) reach 2^62.2 in magnitude and the positive digit terms add < 2^61.1,
// so every column stays inside int64 when its digit is taken.
PBFTV_HD void fs_cols_init(uint64_t t[17]) {
  PBFTV_UNROLL for (int k = 0; k < 17; ++k) t[k] = 0;
}

// Montgomery digit step of column i < 8 (32-bit digit, carry by one signed MAD)
// (c21 = 2^29 - 2^21, c24 = 2^24 - 1: see the header)
PBFTV_HD void fs_digit(uint64_t t[17], int i, uint32_t c8, uint32_t c9, uint32_t c18, uint32_t c21, uint32_t c24) {
  const uint32_t m = (uint32_t)t[i];
  const uint32_t h = (uint32_t)(t[i] >> 32);
  t[i + 1] += smul(h, c8);
  t[i + 3] += (uint64_t)m * c9;
  t[i + 6] += (uint64_t)m * c18;
  t[i + 7] += (uint64_t)m * c21;
  t[i + 8] += (uint64_t)m * c24;
}

// top digit (column 8): 29 bits, arithmetic carry
PBFTV_HD void fs_digit_top(uint64_t t[17], uint32_t c9, uint32_t c18, uint32_t c21, uint32_t c24) {
  const uint32_t m = (uint32_t)t[8] & kMask29;
  t[9] += (uint64_t)((int64_t)t[8] >> 29);
  t[11] += (uint64_t)m * c9;
  t[14] += (uint64_t)m * c18;
  t[15] += (uint64_t)m * c21;
  t[16] += (uint64_t)m * c24;
}

// A limb whose bits the compiler must not know.  The masked limbs of fs_out
// are provably non-negative; LLVM then rewrites a later smul's sign extension
// as a zero extension and, seeing a signed x unsigned product, expands each
// v_mad_i64_i32 into two v_mad_u64_u32, a sign shift and moves (the table
// builder's loops were ~3x the MADs).  An empty asm hides the range.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ uint32_t opaque_limb(uint32_t x) {
  asm("" : "+v"(x));
  return x;
}
#else
static inline uint32_t opaque_limb(uint32_t x) { return x; }
#endif

// columns 9..16 -> S-type limbs (signed carries)
PBFTV_HD void fs_out(fe& r, uint64_t t[17]) {
  PBFTV_UNROLL for (int j = 9; j < 16; ++j) {
    r.v[j - 9] = opaque_limb((uint32_t)t[j] & kMask29);
    t[j + 1] += (uint64_t)((int64_t)t[j] >> 29);
  }
  r.v[7] = opaque_limb((uint32_t)t[16] & kMask29);
  r.v[8] = (uint32_t)((int64_t)t[16] >> 29);
}

#define PBFTV_FS_CONSTS                                                                                   \
  const uint32_t c8 = opaque_u32(8u), c9 = opaque_u32(1u << 9), c18 = opaque_u32(1u << 18),               \
                 c21 = opaque_u32(kC21), c24 = opaque_u32(kC24)

// r = a b 2^-261 (mod p), S-type.  Digit step i right after product row i
// (column i is final then), as in fe_mul.
PBFTV_HD void fs_mul(fe& r, const fe& a, const fe& b) {
  PBFTV_FS_CONSTS;
  uint64_t t[17];
  fs_cols_init(t);
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    PBFTV_UNROLL for (int j = 0; j < 9; ++j) t[i + j] += smul(a.v[i], b.v[j]);
    if (i < 8) fs_digit(t, i, c8, c9, c18, c21, c24);
    else fs_digit_top(t, c9, c18, c21, c24);
  }
  fs_out(r, t);
}

// r = (a b + c d) 2^-261 (mod p): one reduction for two products
PBFTV_HD void fs_mul2_add(fe& r, const fe& a, const fe& b, const fe& c, const fe& d) {
  PBFTV_FS_CONSTS;
  uint64_t t[17];
  fs_cols_init(t);
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    PBFTV_UNROLL for (int j = 0; j < 9; ++j) t[i + j] += smul(a.v[i], b.v[j]);
    PBFTV_UNROLL for (int j = 0; j < 9; ++j) t[i + j] += smul(c.v[i], d.v[j]);
    if (i < 8) fs_digit(t, i, c8, c9, c18, c21, c24);
    else fs_digit_top(t, c9, c18, c21, c24);
  }
  fs_out(r, t);
}

// r = a^2 2^-261 (mod p): 45 products, cross terms by the doubled limb
// (|2 a_j| < 2^30: cross products < 2^59)
PBFTV_HD void fs_sqr(fe& r, const fe& a) {
  PBFTV_FS_CONSTS;
  uint64_t t[17];
  uint32_t a2[9];
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) a2[i] = a.v[i] << 1;
  fs_cols_init(t);
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    t[2 * i] += smul(a.v[i], a.v[i]);
    PBFTV_UNROLL for (int j = i + 1; j < 9; ++j) t[i + j] += smul(a.v[i], a2[j]);
  }
  PBFTV_UNROLL for (int i = 0; i < 8; ++i) fs_digit(t, i, c8, c9, c18, c21, c24);
  fs_digit_top(t, c9, c18, c21, c24);
  fs_out(r, t);
}

// r = a^2 2^-261 - b - 2 c (mod p): X3 = R^2 - PPP - 2Q with the subtraction
// folded into the product's columns 9..16 (and its top limb) before the output
// carry pass -- the value of fs_sqr, then the limb-wise combination and fs_norm,
// without that combination and its separate carry pass.  b, c S-type.
PBFTV_HD void fs_sqr_sub2(fe& r, const fe& a, const fe& b, const fe& c) {
  PBFTV_FS_CONSTS;
  const uint32_t cm1 = opaque_u32(0xFFFFFFFFu);  // -1 (a signed MAD subtracts a limb from a column)
  uint64_t t[17];
  uint32_t a2[9];
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) a2[i] = a.v[i] << 1;
  fs_cols_init(t);
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    t[2 * i] += smul(a.v[i], a.v[i]);
    PBFTV_UNROLL for (int j = i + 1; j < 9; ++j) t[i + j] += smul(a.v[i], a2[j]);
  }
  // - (b + 2c) 2^261: limb k lands on column 9 + k (k < 8); b_k + 2 c_k < 2^31
  PBFTV_UNROLL for (int k = 0; k < 8; ++k) t[9 + k] += smul(b.v[k] + (c.v[k] << 1), cm1);
  PBFTV_UNROLL for (int i = 0; i < 8; ++i) fs_digit(t, i, c8, c9, c18, c21, c24);
  fs_digit_top(t, c9, c18, c21, c24);
  fs_out(r, t);
  r.v[8] = r.v[8] - b.v[8] - (c.v[8] << 1);  // limb 8 of b and c: column 17, the output's top limb
}

// r = (a^2 + b c) 2^-261 (mod p): a squaring and a product under ONE
// reduction.  a D-type (cross terms by the doubled limb: < 2^59, at most 4 per
// column plus the square), b and c S-type (9 products < 2^58 per column): the
// columns stay below 2^62.2 before the digit terms, as in fs_mul2_add.  Digit
// step i follows row i: column i then holds every term of both parts.
PBFTV_HD void fs_sqr_mul_add(fe& r, const fe& a, const fe& b, const fe& c) {
  PBFTV_FS_CONSTS;
  uint64_t t[17];
  uint32_t a2[9];
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) a2[i] = a.v[i] << 1;
  fs_cols_init(t);
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    t[2 * i] += smul(a.v[i], a.v[i]);
    PBFTV_UNROLL for (int j = i + 1; j < 9; ++j) t[i + j] += smul(a.v[i], a2[j]);
    PBFTV_UNROLL for (int j = 0; j < 9; ++j) t[i + j] += smul(b.v[i], c.v[j]);
    if (i < 8) fs_digit(t, i, c8, c9, c18, c21, c24);
    else fs_digit_top(t, c9, c18, c21, c24);
  }
  fs_out(r, t);
}

// r = a - b limb-wise (D-type for S-type inputs)
PBFTV_HD void fs_sub(fe& r, const fe& a, const fe& b) {
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] - b.v[i];
}

PBFTV_HD void fs_neg(fe& r, const fe& a) {
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) r.v[i] = 0u - a.v[i];
}

// r = neg ? -a : a  (mask select: (a ^ m) - m)
PBFTV_HD void fs_cneg(fe& r, const fe& a, bool neg) {
  const uint32_t m = 0u - (uint32_t)neg;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) r.v[i] = (a.v[i] ^ m) - m;
}

// signed limbs (|l_i| < 2^31 - 2^3) -> S-type: one signed carry pass, no fold
PBFTV_HD void fs_norm(fe& r, const fe& a) {
  int32_t d[9];
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) d[i] = (int32_t)a.v[i];
  PBFTV_UNROLL for (int i = 0; i < 8; ++i) {
    d[i + 1] += d[i] >> 29;
    d[i] &= (int32_t)kMask29;
  }
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) r.v[i] = (uint32_t)d[i];
}

// canonical [0, p) of an S- or D-type value (via fe29.h's fold + conditional subtract)
PBFTV_HD void fs_canon(fe& r, const fe& a) {
  int32_t d[9];
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) d[i] = (int32_t)a.v[i];
  fe n;
  fe_fold_carry(n, d);
  fe_canon(r, n);
}

// a == 0 (mod p) for an S- or D-type value, without the canonical subtract:
// fe_fold_carry subtracts top p (top = (limb 8 - 4) >> 24, |top| <= 5) and
// leaves limb 8 in [4, 2^24 + 4), so the folded value lies in (2^233, 2^256 +
// 2^235) -- strictly inside (0, 2p) -- and its only multiple of p is p itself:
// zero iff the folded digits are p's (tests/test_algo_cpu.py checks the range
// and every multiple k p, |k| <= 5, in S- and D-type form).
PBFTV_HD bool fs_is_zero(const fe& a) {
  int32_t d[9];
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) d[i] = (int32_t)a.v[i];
  fe n;
  fe_fold_carry(n, d);
  uint32_t o = 0;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) o |= n.v[i] ^ kP[i];
  return o == 0;
}

// ---- XYZZ mixed addition on signed limbs (madd-2008-s, 8M + 2S) -------------
// acc: X, Y, ZZ, ZZZ S-type; (x2, y2) D-type (a canonical table point, y2
// possibly negated).  Unchecked, as xyzz_madd: a doubling or cancellation
// leaves ZZ = ZZZ = 0, which later additions preserve.
struct xyzz_s {
  fe x, y, zz, zzz;
};

PBFTV_HD void xyzz_madd_s(xyzz_s& acc, const fe& x2, const fe& y2) {
  fe u2, s2, p, r, pp, ppp, q, t, ny;
  fs_mul(u2, x2, acc.zz);
  fs_mul(s2, y2, acc.zzz);
  fs_sub(p, u2, acc.x);                // P = U2 - X1            D
  fs_sub(r, s2, acc.y);                // R = S2 - Y1            D
  fs_sqr(pp, p);
  fs_mul(ppp, p, pp);
  fs_mul(q, acc.x, pp);
  fe x3;
  fs_sqr_sub2(x3, r, ppp, q);          // X3 = R^2 - PPP - 2Q    S
  fs_sub(t, q, x3);                    // Q - X3                 D
  fs_neg(ny, acc.y);                   // -Y1                    D
  fs_mul2_add(acc.y, r, t, ny, ppp);   // Y3 = R (Q - X3) - Y1 PPP, one reduction
  fs_mul(acc.zz, acc.zz, pp);          // ZZ3 = ZZ1 PP
  fs_mul(acc.zzz, acc.zzz, ppp);       // ZZZ3 = ZZZ1 PPP
  acc.x = x3;
}

// The same addition with the accumulator's Y kept as W = sigma Y (sigma = +-1,
// a per-lane sign the caller tracks) and the result returned with the OTHER
// sign: for W1 = sigma Y1 and y2 given as sigma y2,
//   R' = sigma y2 ZZZ1 - W1 = sigma R            (R'^2 = R^2: X3 unchanged)
//   -sigma Y3 = -sigma R (Q - X3) + sigma Y1 PPP = R' (X3 - Q) + W1 PPP,
// so Y3 needs no negation of Y1 (xyzz_madd_s's fs_neg: 9 VALU per addition).
// Callers flip sigma after every addition; X, ZZ and ZZZ are sign-free, and the
// comb's x-coordinate check never reads Y.
PBFTV_HD void xyzz_madd_s_flip(xyzz_s& acc, const fe& x2, const fe& y2) {
  fe u2, s2, p, r, pp, ppp, q, t;
  fs_mul(u2, x2, acc.zz);
  fs_mul(s2, y2, acc.zzz);
  fs_sub(p, u2, acc.x);                // P = U2 - X1            D
  fs_sub(r, s2, acc.y);                // R' = sigma R           D
  fs_sqr(pp, p);
  fs_mul(ppp, p, pp);
  fs_mul(q, acc.x, pp);
  fe x3;
  fs_sqr_sub2(x3, r, ppp, q);          // X3 = R^2 - PPP - 2Q    S
  fs_sub(t, x3, q);                    // X3 - Q                 D
  fs_mul2_add(acc.y, r, t, acc.y, ppp);  // -sigma Y3 = R' (X3 - Q) + W1 PPP, one reduction
  fs_mul(acc.zz, acc.zz, pp);          // ZZ3 = ZZ1 PP
  fs_mul(acc.zzz, acc.zzz, ppp);       // ZZZ3 = ZZZ1 PPP
  acc.x = x3;
}

// ---- the comb's first and last additions (k_ecdsa_comb, comb2_verify) -------
// First: the first two table points are both affine (ZZ1 = ZZZ1 = 1), so
// U2 = x1, S2 = s1 y1, ZZ3 = PP and ZZZ3 = PPP: 4 products fewer than
// xyzz_madd_s_flip.  (x0, s0 y0) + (x1, s1 y1) for canonical table coordinates
// x0, y0, x1, y1 and flip = (s0 != s1).  With e = s0 s1 y0 and d = y1 - e
// (R = s1 d), the result holds W = -s1 Y3 = d (X3 - Q) + e PPP: the caller's
// sigma is -s1.  P = 0 (the two points equal or opposite) leaves ZZ = ZZZ = 0,
// which later additions keep (the caller's exceptional-step test).
PBFTV_HD void xyzz_aff_aff_s(xyzz_s& acc, const fe& x0, const fe& y0, const fe& x1, const fe& y1, bool flip) {
  fe e, dy, d, p, pp, ppp, q, x3, t;
  fs_cneg(e, y0, flip);                // e = s0 s1 y0            D
  fs_sub(dy, y1, e);                   // |limbs| < 2^30
  fs_norm(d, dy);                      // d                       S
  fs_sub(p, x1, x0);                   // P = x1 - x0             D
  fs_sqr(pp, p);
  fs_mul(ppp, p, pp);
  fs_mul(q, x0, pp);
  fs_sqr_sub2(x3, d, ppp, q);          // X3 = d^2 - PPP - 2Q     S
  fs_sub(t, x3, q);                    // X3 - Q                  D
  fs_mul2_add(acc.y, d, t, e, ppp);    // W = d (X3 - Q) + e PPP  S
  acc.x = x3;
  acc.zz = pp;
  acc.zzz = ppp;
}

// Last: the last addition is never formed.  Its x check X3 == r ZZ3 is
//   R^2 - PPP - 2Q == r ZZ1 PP  <=>  R^2 - PP (P + 2 X1 + r ZZ1) == 0,
// and P + 2 X1 = U2 + X1, so one squaring and one product under one reduction
// (fs_sqr_mul_add) replace PPP, Q, X3, Y3, ZZ3, ZZZ3 and the check's r ZZ3.
// xyzz_last_prep_s keeps what both candidates r and r + n share.
struct xyzz_last_s {
  fe p, rr, pp, base;  // P (D), R' = sigma R (D), PP (S), U2 + X1 (limbs < 2^30)
};

PBFTV_HD void xyzz_last_prep_s(xyzz_last_s& L, const xyzz_s& acc, const fe& x2, const fe& y2) {
  fe u2, s2;
  fs_mul(u2, x2, acc.zz);
  fs_mul(s2, y2, acc.zzz);
  fs_sub(L.p, u2, acc.x);
  fs_sub(L.rr, s2, acc.y);
  fs_sqr(L.pp, L.p);
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) L.base.v[i] = u2.v[i] + acc.x.v[i];
}

// d = (R^2 - PP (U2 + X1 + rz)) 2^-261 for rz = r ZZ1 (S-type): zero (mod p)
// iff the sum's x coordinate is r, given ZZ1 != 0 and P != 0
PBFTV_HD void xyzz_last_d_s(fe& d, const xyzz_last_s& L, const fe& rz) {
  fe w, wn;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) w.v[i] = 0u - L.base.v[i] - rz.v[i];  // (-3 2^29, 0]
  fs_norm(wn, w);                                                                // S
  fs_sqr_mul_add(d, L.rr, L.pp, wn);
}

}  // namespace pbftv
