// p256_algo.h -- ECDSA-P256 verification pipeline, one signature per lane.
//
// Semantics: Go 1.19 crypto/ecdsa.Verify (restated in
// oracle/p256_ref.c): reject unless 0 < r,s < n; e = int(hash); w = s^-1;
// u1 = e*w, u2 = r*w (mod n); R = u1*G + u2*Q; reject if R = infinity;
// accept iff R.x mod n == r.  Invalid keys are rejected at registration.
//
// Algorithm (DESIGN.md "Verify kernel"): the PBFT key set is registered once,
// so BOTH scalar multiplications are fixed-base combs over precomputed
// tables -- u*B = sum_i d_i * 2^(8i) * B with signed 8-bit digits
// d_i in [-127, 128] and table T_B[i][|d|-1] = |d| * 2^(8i) * B (affine,
// Montgomery form).  That is 33 + 33 mixed additions and zero doublings per
// verify, against ~256 doublings + ~75 additions for Shamir/wNAF.  The two
// partial sums are kept apart and added once at the end (as Go's
// CombinedMult does), so the only place the doubling / inverse cases of the
// group law can arise is that final complete addition; the comb steps still
// detect them and fall back to a correct slow path.
//
// Compiled by hipcc for the GPU kernels, and by g++ for the CPU test harness
// (tests/cpp) only.
#pragma once
#include "fe29.h"

namespace pbftv {

constexpr int kWinBits = 8;
constexpr int kWindows = 33;          // 256/8 + 1 (signed recoding carry)
constexpr int kEntries = 128;         // |d| in [1, 128]
constexpr int kEntryWords = 16;       // x[8], y[8] canonical Montgomery-form words
constexpr uint64_t kTableWords = (uint64_t)kWindows * kEntries * kEntryWords;  // per base point
constexpr uint64_t kTableBytes = kTableWords * 4;                               // 270,336 B

struct jac {
  fe x, y, z;
};

// ---- affine/Jacobian helpers (Montgomery domain) --------------------------

// dbl-2001-b, a = -3.  Input z != 0 assumed (caller tracks infinity); y == 0 impossible on P-256.
PBFTV_HD void jac_double(jac& r, const jac& p) {
  fe delta, gamma, beta, alpha, t1, t2, t3, b4;
  fe_sqr(delta, p.z);
  fe_sqr(gamma, p.y);
  fe_mul(beta, p.x, gamma);
  fe_sub(t1, p.x, delta);
  fe_add(t2, p.x, delta);
  fe_mul(t3, t1, t2);
  fe_mul_small(alpha, t3, 3);          // 3 (X - d)(X + d)
  fe_sqr(t1, alpha);
  fe_mul_small(t2, beta, 2);
  fe_mul_small(b4, t2, 2);             // 4 beta
  fe_add(t3, b4, b4);                  // 8 beta (lazy)
  fe r_x;
  fe_sub(r_x, t1, t3);
  fe_add(t1, p.y, p.z);
  fe_sqr(t3, t1);
  fe_sub(t3, t3, gamma);
  fe_sub(r.z, t3, delta);
  fe_sub(t2, b4, r_x);                 // 4beta - X3
  fe_mul(t1, alpha, t2);
  fe_sqr(t3, gamma);
  fe_mul_small(t3, t3, 2);
  fe_mul_small(t3, t3, 2);
  fe_add(t3, t3, t3);                  // 8 gamma^2 (lazy)
  fe_sub(r.y, t1, t3);
  r.x = r_x;
}

// Mixed addition acc += (x2, y2) (madd-2007-bl), acc.z != 0.
// kCheck: returns 0 normal; 1 if the points are equal (caller must double);
// 2 if the sum is the point at infinity (accumulator unchanged on 1/2).
// !kCheck: no test; in both exceptional cases H == 0 and the result has
// Z3 = 2 Z1 H == 0, which every later addition preserves -- so a single
// Z == 0 test after a whole comb detects that some step was exceptional.
template <bool kCheck = true>
PBFTV_HD int jac_madd(jac& acc, const fe& x2, const fe& y2) {
  fe z1z1, u2, s2, h, hh, i4, j, rr, v, t, t2;
  fe_sqr(z1z1, acc.z);
  fe_mul(u2, x2, z1z1);
  fe_mul(t, acc.z, z1z1);
  fe_mul(s2, y2, t);
  fe_sub(h, u2, acc.x);
  fe_sub(t, s2, acc.y);
  if (kCheck && fe_is_zero(h)) return fe_is_zero(t) ? 1 : 2;
  fe_add(rr, t, t);                    // r = 2 (S2 - Y1), lazy
  fe_sqr(hh, h);
  fe_mul_small(t, hh, 2);
  fe_add(i4, t, t);                    // I = 4 HH (lazy)
  fe_mul(j, h, i4);                    // J = H * I
  fe_mul(v, acc.x, i4);                // V = X1 * I
  fe_sqr(t, rr);                       // r^2
  fe_sub(t, t, j);
  fe_add(t2, v, v);
  fe x3;
  fe_sub(x3, t, t2);                   // X3 = r^2 - J - 2V
  fe_sub(t, v, x3);
  fe_mul(t2, rr, t);                   // r (V - X3)
  fe_mul(t, acc.y, j);
  fe y3;
  fe_add(t, t, t);
  fe_sub(y3, t2, t);                   // Y3 = r (V - X3) - 2 Y1 J
  fe_add(t, acc.z, h);
  fe_sqr(t2, t);
  fe_sub(t2, t2, z1z1);
  fe_sub(acc.z, t2, hh);               // Z3 = (Z1 + H)^2 - Z1Z1 - HH
  acc.x = x3;
  acc.y = y3;
  return 0;
}

// General Jacobian addition r = p + q (both finite).  Same return codes as jac_madd.
PBFTV_HD int jac_add(jac& r, const jac& p, const jac& q) {
  fe z1z1, z2z2, u1, u2, s1, s2, h, rr, t, hh, hhh, v;
  fe_sqr(z1z1, p.z);
  fe_sqr(z2z2, q.z);
  fe_mul(u1, p.x, z2z2);
  fe_mul(u2, q.x, z1z1);
  fe_mul(t, q.z, z2z2);
  fe_mul(s1, p.y, t);
  fe_mul(t, p.z, z1z1);
  fe_mul(s2, q.y, t);
  fe_sub(h, u2, u1);
  fe_sub(rr, s2, s1);
  if (fe_is_zero(h)) return fe_is_zero(rr) ? 1 : 2;
  fe_sqr(hh, h);
  fe_mul(hhh, hh, h);
  fe_mul(v, u1, hh);
  fe_sqr(t, rr);
  fe_sub(t, t, hhh);
  fe x3, t2;
  fe_add(t2, v, v);
  fe_sub(x3, t, t2);
  fe_sub(t, v, x3);
  fe y3;
  fe_mul(y3, rr, t);
  fe_mul(t, s1, hhh);
  fe_sub(y3, y3, t);
  fe_mul(t, p.z, q.z);
  fe_mul(r.z, t, h);
  r.x = x3;
  r.y = y3;
  return 0;
}

// ---- exponentiation helpers ------------------------------------------------

// a^e mod p (Montgomery in/out), e as 8 LE words; plain left-to-right binary.
PBFTV_HD void fe_pow(fe& r, const fe& a, const uint32_t e[8]) {
  fe acc;
  fe_set(acc, kOneP);
  for (int i = 255; i >= 0; --i) {
    fe_sqr(acc, acc);
    if ((e[i >> 5] >> (i & 31)) & 1u) fe_mul(acc, acc, a);
  }
  r = acc;
}

PBFTV_HD void fe_inv(fe& r, const fe& a) { fe_pow(r, a, kPMinus2); }

// n repeated Montgomery squarings mod n (a real loop: keeps code size small)
PBFTV_HD void fn_sqr_n(fe& a, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll 1
#endif
  for (int i = 0; i < n; ++i) fn_sqr(a, a);
}

// x^v for odd v in [1, 15] from the precomputed odd powers (v is a
// compile-time constant once the step loop below is unrolled).
PBFTV_HD const fe& fn_pick(int v, const fe& p1, const fe& p3, const fe& p5, const fe& p7, const fe& p9,
                           const fe& p11, const fe& p13, const fe& p15) {
  return v == 1 ? p1 : v == 3 ? p3 : v == 5 ? p5 : v == 7 ? p7 : v == 9 ? p9 : v == 11 ? p11 : v == 13 ? p13 : p15;
}

// s^-1 * R mod n for s = sm in Montgomery form: Fermat x^(n-2) by an addition
// chain -- the top half FFFFFFFF00000000FFFFFFFFFFFFFFFF from x^(2^32-1)
// blocks, the low half by a 4-bit sliding window (kInvNSteps, generated and
// self-checked by tools/gen_p256_consts.py): 253 squarings + 39 multiplies.
PBFTV_HD void fn_inv_mont(fe& r, const fe& x) {
  fe x2, p3, p5, p7, p9, p11, p13, p15;
  fn_sqr(x2, x);
  fn_mul(p3, x2, x);
  fn_mul(p5, p3, x2);
  fn_mul(p7, p5, x2);
  fn_mul(p9, p7, x2);
  fn_mul(p11, p9, x2);
  fn_mul(p13, p11, x2);
  fn_mul(p15, p13, x2);      // x^(2^4 - 1)
  fe t8 = p15, t16, t32, acc;
  fn_sqr_n(t8, 4);
  fn_mul(t8, t8, p15);       // x^(2^8 - 1)
  t16 = t8;
  fn_sqr_n(t16, 8);
  fn_mul(t16, t16, t8);      // x^(2^16 - 1)
  t32 = t16;
  fn_sqr_n(t32, 16);
  fn_mul(t32, t32, t16);     // x^(2^32 - 1)
  acc = t32;
  fn_sqr_n(acc, 64);
  fn_mul(acc, acc, t32);
  fn_sqr_n(acc, 32);
  fn_mul(acc, acc, t32);     // x^FFFFFFFF00000000FFFFFFFFFFFFFFFF
  PBFTV_UNROLL for (int i = 0; i < (int)(sizeof(kInvNSteps) / sizeof(kInvNSteps[0])); ++i) {
    fn_sqr_n(acc, kInvNSteps[i][0]);
    fn_mul(acc, acc, fn_pick(kInvNSteps[i][1], x, p3, p5, p7, p9, p11, p13, p15));
  }
  fn_sqr_n(acc, kInvNTail);
  r = acc;
}

// ---- byte/word helpers -----------------------------------------------------

// 32 big-endian bytes given as 8 big-endian-loaded u32 (w_be[0] = bytes 0..3) -> LE words
PBFTV_HD void be_words_to_le(uint32_t out[8], const uint32_t in_be[8]) {
  PBFTV_UNROLL for (int i = 0; i < 8; ++i) {
    uint32_t x = in_be[7 - i];
    out[i] = (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
  }
}

PBFTV_HD bool words_lt(const uint32_t a[8], const uint32_t b[8]) { return fe_cmp_words(a, b) < 0; }

// ---- stage 1: scalars --------------------------------------------------------
// Inputs as LE words.  Returns false if (r, s) fail Go's range checks.
// On success u1 = e*s^-1 mod n, u2 = r*s^-1 mod n as canonical LE words.
PBFTV_HD bool ecdsa_scalars(const uint32_t e_w[8], const uint32_t r_w[8], const uint32_t s_w[8], uint32_t u1_w[8],
                            uint32_t u2_w[8]) {
  if (words_is_zero(r_w) || words_is_zero(s_w)) return false;
  if (!words_lt(r_w, kN32) || !words_lt(s_w, kN32)) return false;
  fe e, r, s, r2n, sm, w, t;
  fe_from_words(e, e_w);
  fe_from_words(r, r_w);
  fe_from_words(s, s_w);
  fe_set(r2n, kR2N);
  fn_mul(sm, s, r2n);         // s * R
  fn_inv_mont(w, sm);         // s^-1 * R
  fn_mul(t, e, w);            // e * s^-1   (e < 2^256 < 2n: Montgomery handles it)
  fn_canon(t, t);
  fe_to_words(u1_w, t);
  fn_mul(t, r, w);
  fn_canon(t, t);
  fe_to_words(u2_w, t);
  return true;
}

// ---- signed 8-bit digits ----------------------------------------------------
// digit i of u (LE words), carry-in c (0/1); returns d in [-127, 128], updates c.
PBFTV_HD int signed_digit(const uint32_t u_w[8], int i, int& c) {
  int b = i < 32 ? (int)((u_w[i >> 2] >> (8 * (i & 3))) & 0xFFu) : 0;
  int d = b + c;
  c = d > 128 ? 1 : 0;
  return d - (c << 8);
}

// unpack a table entry (16 words: x[8], y[8]) into field elements
PBFTV_HD void entry_to_fe(fe& x, fe& y, const uint32_t e[16]) {
  fe_from_words(x, e);
  fe_from_words(y, e + 8);
}

// ---- stage 2: comb ------------------------------------------------------------
// acc = u * B using table tab (kWindows x kEntries x 16 words).  Returns false
// if the result is the point at infinity (u == 0).  TableLoad is a functor
// load(tab, window, idx, words[16]) so device code can use wide loads.
template <bool kCheck, class Load>
PBFTV_HD bool comb_pass(jac& acc, const uint32_t u_w[8], Load load) {
  bool inf = true;
  int c = 0;
  for (int i = 0; i < kWindows; ++i) {
    const int d = signed_digit(u_w, i, c);
    if (d == 0) continue;
    uint32_t ew[16];
    load(i, (d < 0 ? -d : d) - 1, ew);
    fe x, y;
    entry_to_fe(x, y, ew);
    if (d < 0) {
      fe ny;
      fe_neg_lazy(ny, y);
      fe_norm(y, ny);
    }
    if (inf) {
      acc.x = x;
      acc.y = y;
      fe_set(acc.z, kOneP);
      inf = false;
      continue;
    }
    const int st = jac_madd<kCheck>(acc, x, y);
    if (st == 1) jac_double(acc, acc);
    else if (st == 2) inf = true;
  }
  return !inf;
}

// acc = u * B using table tab (kWindows x kEntries x 16 words).  Returns false
// if the result is the point at infinity (u == 0).  Load is a functor
// load(window, idx, words[16]).  Fast unchecked pass; if it ended with Z == 0
// some step hit the doubling / inverse case (impossible for a proper comb,
// DESIGN.md) and the comb is recomputed with complete additions.
template <class Load>
PBFTV_HD bool comb_mult(jac& acc, const uint32_t u_w[8], Load load) {
  const bool ok = comb_pass<false>(acc, u_w, load);
  if (ok && fe_is_zero(acc.z)) return comb_pass<true>(acc, u_w, load);
  return ok;
}

// ---- final check --------------------------------------------------------------
// R = A + B with A, B possibly infinite; accept iff R finite and R.x mod n == r.
PBFTV_HD bool ecdsa_final(const jac& A, bool a_ok, const jac& B, bool b_ok, const uint32_t r_w[8]) {
  jac R;
  bool ok;
  if (!a_ok && !b_ok) return false;
  if (!a_ok) {
    R = B; ok = true;
  } else if (!b_ok) {
    R = A; ok = true;
  } else {
    const int st = jac_add(R, A, B);
    if (st == 1) { jac_double(R, A); ok = true; }
    else ok = (st == 0);
  }
  if (!ok) return false;
  // X == r * Z^2 (mod p), or X == (r + n) Z^2 when r + n < p
  fe z2, rr, r2p, lhs, x;
  fe_sqr(z2, R.z);
  fe_from_words(rr, r_w);
  fe_set(r2p, kR2P);
  fe_mul(rr, rr, r2p);        // r in Montgomery form
  fe_mul(lhs, rr, z2);
  if (fe_equal(lhs, R.x)) return true;
  // r + n < p  <=>  r < p - n
  if (words_lt(r_w, kPMinusN32)) {
    uint32_t rn[8];
    uint64_t cy = 0;
    for (int i = 0; i < 8; ++i) {
      cy += (uint64_t)r_w[i] + kN32[i];
      rn[i] = (uint32_t)cy;
      cy >>= 32;
    }
    fe_from_words(rr, rn);
    fe_mul(rr, rr, r2p);
    fe_mul(lhs, rr, z2);
    (void)x;
    if (fe_equal(lhs, R.x)) return true;
  }
  return false;
}

// ---- key validation + table construction -------------------------------------

// (x, y) LE words -> valid P-256 point?  On success xm, ym are Montgomery form.
PBFTV_HD bool key_check(const uint32_t x_w[8], const uint32_t y_w[8], fe& xm, fe& ym) {
  if (!words_lt(x_w, kP32) || !words_lt(y_w, kP32)) return false;
  fe x, y, r2p, t, rhs, lhs, b;
  fe_from_words(x, x_w);
  fe_from_words(y, y_w);
  fe_set(r2p, kR2P);
  fe_mul(xm, x, r2p);
  fe_mul(ym, y, r2p);
  fe_sqr(lhs, ym);
  fe_sqr(t, xm);
  fe_mul(t, t, xm);           // x^3
  fe_mul_small(rhs, xm, 3);
  fe_sub(t, t, rhs);          // x^3 - 3x
  fe_set(b, kBMont);
  fe_add(t, t, b);
  return fe_equal(lhs, t);
}

// Jacobian -> canonical affine words (Montgomery form); p finite.
PBFTV_HD void jac_to_affine_words(uint32_t out[16], const jac& p, const fe& zinv) {
  fe z2, z3, x, y;
  fe_sqr(z2, zinv);
  fe_mul(z3, z2, zinv);
  fe_mul(x, p.x, z2);
  fe_mul(y, p.y, z3);
  fe_canon(x, x);
  fe_canon(y, y);
  fe_to_words(out, x);
  fe_to_words(out + 8, y);
}

// Build one window of a comb table: out[e*16..] = (e+1) * 2^(8*win) * B, e = 0..127.
// Scratch is a flat array of field elements reached through st(slot, fe) /
// ld(slot, fe): point e uses slots 3e..3e+2 (x, y, z), the running product of
// the z's uses slot 3*kEntries + e (Montgomery's batch-inversion trick).
constexpr int kScratchSlots = 4 * kEntries;

template <class StoreF, class LoadF>
PBFTV_HD void build_window(uint32_t* out, int win, const fe& bx, const fe& by, StoreF st, LoadF ld) {
  jac cur;
  cur.x = bx;
  cur.y = by;
  fe_set(cur.z, kOneP);
  for (int k = 0; k < kWinBits * win; ++k) jac_double(cur, cur);
  fe zi;
  fe_inv(zi, cur.z);
  uint32_t bw[16];
  jac_to_affine_words(bw, cur, zi);     // B_w = 2^(8 win) B, affine
  fe ax, ay;
  entry_to_fe(ax, ay, bw);
  cur.x = ax;
  cur.y = ay;
  fe_set(cur.z, kOneP);
  for (int e = 0; e < kEntries; ++e) {
    if (e == 1) jac_double(cur, cur);
    else if (e >= 2) jac_madd(cur, ax, ay);   // (e+1) B_w; never exceptional for e+1 <= 128
    st(3 * e, cur.x);
    st(3 * e + 1, cur.y);
    st(3 * e + 2, cur.z);
  }
  fe pre, z;
  ld(2, pre);
  st(3 * kEntries, pre);
  for (int e = 1; e < kEntries; ++e) {
    ld(3 * e + 2, z);
    fe_mul(pre, pre, z);
    st(3 * kEntries + e, pre);
  }
  fe inv;
  fe_inv(inv, pre);                     // 1 / (z_0 ... z_127)
  for (int e = kEntries - 1; e >= 0; --e) {
    jac pt;
    ld(3 * e, pt.x);
    ld(3 * e + 1, pt.y);
    ld(3 * e + 2, pt.z);
    fe zinv;
    if (e > 0) {
      fe prev;
      ld(3 * kEntries + e - 1, prev);
      fe_mul(zinv, inv, prev);          // 1/z_e = 1/prefix_e * prefix_{e-1}
      fe_mul(inv, inv, pt.z);           // 1/prefix_{e-1}
    } else {
      zinv = inv;
    }
    jac_to_affine_words(out + (uint64_t)e * kEntryWords, pt, zinv);
  }
}

}  // namespace pbftv
