// rows.h -- the latency path's ROW schedule (round 5), gfx950 device code.
//
// One field element is ONE VGPR: limb j (29 bits, signed, the fes.h value
// convention: value = sum v_j 2^(29 j), Montgomery R = 2^261) sits in lane j of
// a 16-lane row; lanes 9..15 hold 0.  A wave's four rows multiply four
// different pairs at once, and a product is nine CIOS rounds, each a DPP
// broadcast of a_i (row_newbcast:i) and of the column-0 digit, two
// v_mad_i64_i32 and a split carry (t_j <- (t_j >> 29) + (t_{j+1} mod 2^29)):
// ~624 cycles on a lone wave against ~812 for fs_mul done by one lane, and a
// value moves between rows as ONE register (three v_permlane swaps give every
// row all four rows' products) where the quad schedule moves nine limbs per
// value and picks operands with nine selects per limb.  An add-2008-s XYZZ
// addition is 4 steps = 945 ns on a lone wave, vs ~2.6 µs for a quad
// schedule level (tools/lpl_probe.hip, profiles/r05_lpl_probe.txt).
//
// Types as fes.h: a product output has limbs 0..7 in [-2^5, 2^29 + 2^5) (the
// last round's columns are < 2^33.1, so the final carry is < 2^4.1) and a
// signed top limb, |value| < |a| |b| / 2^261 + p.  Inputs need
// max|a_i| max|b_j| < 2^61 (each column then stays below 2^61.2).  Every limb
// must also fit int32: X3 = R^2 - PPP - 2Q is renormalised (row_norm) before
// Q - X3, and the fused check sums U1 + U2 + r ZZ12 instead of P + 2 U1 +
// r ZZ12 (same value, limbs < 3 2^29 + 2^6).
#pragma once
#include "fes.h"

namespace pbftv {

// (mov_dpp, not update_dpp with an old value of 0: every lane of these DPP
// moves has a source lane or bound_ctrl's zero, so the old value is never
// read, and without it the compiler drops the v_mov that materialised it --
// two per product round, 324 instructions of the row kernel; QC p50 -0.5 µs,
// profiles/r06_ab_mov_dpp)
template <int K>
__device__ __forceinline__ uint32_t row_bcast(uint32_t x) {  // lane K of the row to the whole row
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150 + K, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t row_next(uint32_t x) {  // lane j <- lane j + 1 of its row (0 past it)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x101, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t row_prev(uint32_t x) {  // lane j <- lane j - 1 of its row (0 before it)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x111, 0xF, 0xF, true);
}

// per-lane constants of the row layout
struct RowCtx {
  uint32_t pl;      // p's limb of this lane (0 past limb 8)
  uint32_t lomask;  // the final carry pass: lane 8 keeps its whole limb ...
  uint32_t himask;  // ... and carries nothing up
  uint32_t one;     // Montgomery one (R mod p)'s limb
  int L, row;       // limb index (lane & 15), row (lane >> 4)
};

__device__ __forceinline__ uint32_t limb_of(const uint32_t c[9], int L) {
  uint32_t r = 0;
  PBFTV_UNROLL for (int k = 0; k < 9; ++k) r = L == k ? c[k] : r;
  return r;
}

__device__ __forceinline__ RowCtx row_ctx() {
  RowCtx c;
  const int lane = (int)(threadIdx.x & 63u);
  c.L = lane & 15;
  c.row = lane >> 4;
  c.pl = limb_of(kP, c.L);
  c.one = limb_of(kOneP, c.L);
  c.lomask = c.L == 8 ? 0xFFFFFFFFu : kMask29;
  c.himask = c.L == 8 ? 0u : 0xFFFFFFFFu;
  return c;
}

template <int I>
__device__ __forceinline__ void row_round(int64_t& t, uint32_t a, uint32_t b, uint32_t pl) {
  const uint32_t ai = row_bcast<I>(a);
  t += (int64_t)(int32_t)ai * (int64_t)(int32_t)b;
  const uint32_t q = row_bcast<0>((uint32_t)t) & kMask29;  // -p^-1 = 1 (mod 2^29)
  t += (int64_t)(int32_t)q * (int64_t)(int32_t)pl;
  const uint32_t lo = (uint32_t)t & kMask29;  // lane 0: 0 -- the column is divisible now
  t = (t >> 29) + (int64_t)row_next(lo);
}

// a b 2^-261 (mod p), every row its own pair
__device__ __forceinline__ uint32_t row_mul(const RowCtx& c, uint32_t a, uint32_t b) {
  int64_t t = 0;
  row_round<0>(t, a, b, c.pl);
  row_round<1>(t, a, b, c.pl);
  row_round<2>(t, a, b, c.pl);
  row_round<3>(t, a, b, c.pl);
  row_round<4>(t, a, b, c.pl);
  row_round<5>(t, a, b, c.pl);
  row_round<6>(t, a, b, c.pl);
  row_round<7>(t, a, b, c.pl);
  row_round<8>(t, a, b, c.pl);
  const uint32_t lo = (uint32_t)t & c.lomask;
  const uint32_t hi = (uint32_t)(t >> 29) & c.himask;
  return lo + row_prev(hi);
}

// one signed carry pass (lane 8 keeps its whole limb): limbs 0..7 into
// [-2^2, 2^29 + 2^2) for |limbs| < 2^31.  Same value.
__device__ __forceinline__ uint32_t row_norm(const RowCtx& c, uint32_t x) {
  const uint32_t lo = x & c.lomask, hi = (uint32_t)((int32_t)x >> 29) & c.himask;
  return lo + row_prev(hi);
}

// g[r] = row r's x, in every row (v_permlane16_swap: rows 0 <-> 1, 2 <-> 3;
// v_permlane32_swap: rows 0,1 <-> 2,3)
__device__ __forceinline__ void gather4(uint32_t g[4], uint32_t x) {
  const auto ab = __builtin_amdgcn_permlane16_swap(x, x, false, false);  // [x0 x0 x2 x2], [x1 x1 x3 x3]
  const auto c = __builtin_amdgcn_permlane32_swap(ab[0], ab[0], false, false);
  const auto d = __builtin_amdgcn_permlane32_swap(ab[1], ab[1], false, false);
  g[0] = c[0];
  g[1] = d[0];
  g[2] = c[1];
  g[3] = d[1];
}

// row r takes v_r
__device__ __forceinline__ uint32_t sel4(const RowCtx& c, uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3) {
  const uint32_t lo = (c.row & 1) ? v1 : v0, hi = (c.row & 1) ? v3 : v2;
  return (c.row & 2) ? hi : lo;
}

struct xyzz_r {
  uint32_t x, y, zz, zzz;
};

// ---- XYZZ + XYZZ, add-2008-s: 4 steps, one product per row per step --------
// Both operands and the sum are the same in every row.  Row 3 of step 4
// computes rz = rm ZZ3 (r ZZ of the sum, Montgomery form: the fused last
// level's input).  A doubling or cancellation (P == 0) leaves ZZ3 = 0, which
// every later product keeps (the caller tests it once, at the top).
__device__ __forceinline__ void xyzz_add_rows(const RowCtx& c, xyzz_r& r, uint32_t& rz, const xyzz_r& A,
                                              const xyzz_r& B, uint32_t rm) {
  uint32_t g[4];
  uint32_t m = row_mul(c, sel4(c, A.x, B.x, A.y, B.y), sel4(c, B.zz, A.zz, B.zzz, A.zzz));
  gather4(g, m);  // U1, U2, S1, S2
  const uint32_t U1 = g[0], S1 = g[2], P = g[1] - g[0], R = g[3] - g[2];
  m = row_mul(c, sel4(c, P, R, A.zz, A.zzz), sel4(c, P, R, B.zz, B.zzz));
  gather4(g, m);  // PP, R^2, ZZ1 ZZ2, ZZZ1 ZZZ2
  const uint32_t PP = g[0], RR = g[1], Z12 = g[2], ZZZ12 = g[3];
  m = row_mul(c, sel4(c, P, U1, Z12, 0u), PP);
  gather4(g, m);  // PPP, Q = U1 PP, ZZ3
  const uint32_t PPP = g[0], Q = g[1], ZZ3 = g[2];
  const uint32_t X3 = row_norm(c, RR - PPP - (Q << 1));  // (Q - X3 must stay inside 32-bit limbs)
  m = row_mul(c, sel4(c, R, S1, ZZZ12, rm), sel4(c, Q - X3, PPP, PPP, ZZ3));
  gather4(g, m);  // R (Q - X3), S1 PPP, ZZZ3, r ZZ3
  r.x = X3;
  r.y = g[0] - g[1];
  r.zz = ZZ3;
  r.zzz = g[2];
  rz = g[3];
}

// ---- affine + affine into XYZZ (mmadd-2008-s), TWO additions per wave ------
// Rows 0, 1 hold window A's values, rows 2, 3 window B's (the "pair layout");
// each step the pair's two rows take one product each.  3 steps.
__device__ __forceinline__ void mmadd_pairs(const RowCtx& c, xyzz_r& S, uint32_t gx, uint32_t gy, uint32_t qx,
                                            uint32_t qy) {
  const bool odd = (c.row & 1) != 0, pb = c.row >= 2;
  uint32_t g[4];
  const uint32_t p = qx - gx, rr = qy - gy;
  uint32_t m = row_mul(c, odd ? rr : p, odd ? rr : p);
  gather4(g, m);  // PP, R^2 of each pair
  const uint32_t PP = pb ? g[2] : g[0], R2 = pb ? g[3] : g[1];
  m = row_mul(c, odd ? gx : p, PP);
  gather4(g, m);  // PPP, Q = X1 PP
  const uint32_t PPP = pb ? g[2] : g[0], Q = pb ? g[3] : g[1];
  const uint32_t X3 = row_norm(c, R2 - PPP - (Q << 1));
  m = row_mul(c, odd ? gy : rr, odd ? PPP : Q - X3);
  gather4(g, m);  // R (Q - X3), Y1 PPP
  S.x = X3;
  S.y = pb ? g[2] - g[3] : g[0] - g[1];
  S.zz = PP;
  S.zzz = PPP;
}

// the value of row 0 as a uniform fe (9 readlanes)
__device__ __forceinline__ void row_to_fe(fe& d, uint32_t x) {
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) d.v[l] = (uint32_t)__builtin_amdgcn_readlane((int)x, l);
}

// x == 0 (mod p) for an output / difference of outputs (the fes.h types after
// one signed carry pass)
__device__ __forceinline__ bool row_is_zero(uint32_t x) {
  fe d;
  row_to_fe(d, x);
  fs_norm(d, d);
  return fs_is_zero(d);
}

// The last level fused with Go's x-coordinate check against r (as
// quad_xyzz_add_check): with rz = r ZZ1,
//   X3 == r ZZ3  <=>  R^2 == PP (P + 2 U1 + rz ZZ2).
// exc: P == 0 or rz ZZ2 == 0 (a zero ZZ anywhere below), tested as one
// product P rz ZZ2 in the last step's second row.  3 steps.
__device__ __forceinline__ bool xyzz_add_check_rows(const RowCtx& c, bool& exc, const xyzz_r& A, const xyzz_r& B,
                                                    uint32_t rz) {
  uint32_t g[4];
  uint32_t m = row_mul(c, sel4(c, A.x, B.x, A.y, B.y), sel4(c, B.zz, A.zz, B.zzz, A.zzz));
  gather4(g, m);  // U1, U2, S1, S2
  const uint32_t U1 = g[0], U2 = g[1], P = g[1] - g[0], R = g[3] - g[2];
  m = row_mul(c, sel4(c, P, R, rz, 0u), sel4(c, P, R, B.zz, 0u));
  gather4(g, m);  // PP, R^2, r ZZ1 ZZ2
  const uint32_t PP = g[0], R2 = g[1], rz12 = g[2];
  const uint32_t w = U1 + U2 + rz12;  // = P + 2 U1 + r ZZ1 ZZ2; limbs < 3 (2^29 + 2^5)
  m = row_mul(c, c.row & 1 ? P : PP, c.row & 1 ? rz12 : w);
  gather4(g, m);  // PP (P + 2 U1 + r ZZ12); P r ZZ1 ZZ2, zero iff either factor is (p prime)
  // both zero tests at once, half a wave each: lanes 0-31 the check's
  // difference, lanes 32-63 the exceptional product
  fe a, b, x;
  row_to_fe(a, R2 - g[0]);
  row_to_fe(b, g[1]);
  const bool hi = (threadIdx.x & 63u) >= 32u;
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) x.v[l] = hi ? b.v[l] : a.v[l];
  fs_norm(x, x);
  const uint64_t z = __ballot(fs_is_zero(x));
  exc = ((z >> 32) & 1u) != 0;
  return (z & 1u) != 0;
}

}  // namespace pbftv
