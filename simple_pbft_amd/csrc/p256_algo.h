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
#include <type_traits>

#include "fe29.h"
#include "fes.h"
#include "safegcd.h"

namespace pbftv {

// Comb table geometry for W-bit signed windows: digits d_i in
// [-(2^(W-1) - 1), 2^(W-1)], u = sum d_i 2^(W i); entry (i, |d|-1) holds
// |d| * 2^(W i) * B as affine (x, y), canonical Montgomery-form, 8+8 LE words.
//
// Geometry codes: W <= 26 is W-bit windows throughout.  The MIXED codes split
// exactly 257 bits (the least that absorbs the last recoding carry) into kWin
// windows, the bottom kWin - kLow of kW bits and the top kLow of kW - 1 bits:
//   11: 15 x 12 + 7 x 11  (22 windows; CPU harness)
//   21:  5 x 22 + 7 x 21  (12 windows, 1.14 GB per key instead of 1.61 at W = 22)
//   29:  5 x 29 + 4 x 28  ( 9 windows, 120 GB -- one window fewer than W = 26)
// A narrower top window holds 2^(kW-2) entries; its digit still fits, since
// the bits left for it number its width - 1.
constexpr bool comb_mixed(int c) { return c == 11 || c == 21 || c == 29; }
constexpr int comb_kw(int c) { return c == 11 ? 12 : c == 21 ? 22 : c; }
constexpr int comb_win(int c) { return c == 11 ? 22 : c == 21 ? 12 : c == 29 ? 9 : 256 / c + 1; }

template <int W>
struct CombGeom {
  static constexpr int kCode = W;
  static constexpr int kW = comb_kw(W);
  static constexpr int kWin = comb_win(W);  // 33 (W=8), 22 (12), 17 (16), 13 (20), 12 (22), 11 (24), 10 (26), 9 (29)
  static constexpr int kLow = comb_mixed(W) ? kWin * kW - 257 : 0;
  static constexpr int kHi = kWin - kLow;
  static_assert(kW >= 8 && kW <= 29, "window width");
  static_assert(comb_mixed(W) ? kLow > 0 && kLow < kWin : 256 % W <= W - 2,
                "top window must absorb the recoding carry");
  static constexpr int kEnt = 1 << (kW - 1);  // entries of a full-width window
  static constexpr uint64_t kWords = ((uint64_t)kHi * kEnt + (uint64_t)kLow * (kEnt / 2)) * 16;
  static constexpr uint64_t kBytes = kWords * 4;
  PBFTV_HDM static constexpr int width(int i) { return i < kHi ? kW : kW - 1; }
  PBFTV_HDM static constexpr int bit(int i) { return i < kHi ? i * kW : kHi * kW + (i - kHi) * (kW - 1); }
  PBFTV_HDM static constexpr int ent(int i) { return i < kHi ? kEnt : kEnt / 2; }
  // first entry of window i
  PBFTV_HDM static constexpr uint64_t base(int i) {
    return i < kHi ? (uint64_t)i * kEnt : (uint64_t)kHi * kEnt + (uint64_t)(i - kHi) * (kEnt / 2);
  }
};

// legacy names for the W = 8 geometry
constexpr int kWinBits = 8;
constexpr int kWindows = CombGeom<8>::kWin;
constexpr int kEntries = CombGeom<8>::kEnt;
constexpr int kEntryWords = 16;
constexpr uint64_t kTableWords = CombGeom<8>::kWords;
constexpr uint64_t kTableBytes = CombGeom<8>::kBytes;

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

// ---- extended Jacobian "XYZZ" coordinates: (X, Y, ZZ, ZZZ) represents the
// affine point (X / ZZ, Y / ZZZ) with ZZ^3 = ZZZ^2.  Mixed addition
// madd-2008-s costs 8M + 2S (Jacobian madd-2007-bl: 7M + 4S) and the final
// x-check needs X == r ZZ only.
struct xyzz {
  fe x, y, zz, zzz;
};

// acc += (x2, y2), acc finite (acc.x N-type, acc.y M- or N-type, y2 may be
// lazy with limbs < 2^30).  Unchecked: when the x-coordinates meet
// (doubling or cancellation) P == 0, so ZZ3 = ZZZ3 = 0, which every later
// addition preserves -- one ZZ == 0 test after a whole comb detects it.
PBFTV_HD void xyzz_madd(xyzz& acc, const fe& x2, const fe& y2) {
  fe u2, s2, p, r, pp, ppp, q, t, t2;
  fe_mul(u2, x2, acc.zz);
  fe_mul(s2, y2, acc.zzz);
  fe_sub(p, u2, acc.x);                // P = U2 - X1
  fe_sub(r, s2, acc.y);                // R = S2 - Y1
  fe_sqr(pp, p);
  fe_mul(ppp, p, pp);
  fe_mul(q, acc.x, pp);
  fe_sqr(t, r);                        // R^2
  fe_add(t2, ppp, q);
  fe_add(t2, t2, q);                   // PPP + 2Q (lazy, limbs < 2^30 + 2^29)
  fe x3;
  fe_sub(x3, t, t2);                   // X3 = R^2 - PPP - 2Q
  fe_sub(t, q, x3);
  fe_neg_lazy(t2, acc.y);              // 2p - Y1 (limbs < 2^30)
  fe_mul2_add(acc.y, r, t, t2, ppp);   // Y3 = R (Q - X3) - Y1 PPP, one reduction
  fe_mul(acc.zz, acc.zz, pp);          // ZZ3 = ZZ1 PP
  fe_mul(acc.zzz, acc.zzz, ppp);       // ZZZ3 = ZZZ1 PPP
  acc.x = x3;
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

// acc *= x^v for odd v in [1, 15] from the precomputed odd powers.  A switch
// (wave-uniform branch) rather than a reference pick, so the powers stay in
// registers instead of being spilled to addressable scratch.
PBFTV_HD void fn_mul_pow(fe& acc, int v, const fe& p1, const fe& p3, const fe& p5, const fe& p7, const fe& p9,
                         const fe& p11, const fe& p13, const fe& p15) {
  switch (v) {
    case 1: fn_mul(acc, acc, p1); break;
    case 3: fn_mul(acc, acc, p3); break;
    case 5: fn_mul(acc, acc, p5); break;
    case 7: fn_mul(acc, acc, p7); break;
    case 9: fn_mul(acc, acc, p9); break;
    case 11: fn_mul(acc, acc, p11); break;
    case 13: fn_mul(acc, acc, p13); break;
    default: fn_mul(acc, acc, p15); break;
  }
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
  for (int i = 0; i < (int)(sizeof(kInvNSteps) / sizeof(kInvNSteps[0])); ++i) {
    fn_sqr_n(acc, kInvNSteps[i][0]);
    fn_mul_pow(acc, kInvNSteps[i][1], x, p3, p5, p7, p9, p11, p13, p15);
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
  fn_inv_mont_gcd(w, sm);     // s^-1 * R
  fn_mul(t, e, w);            // e * s^-1   (e < 2^256 < 2n: Montgomery handles it)
  fn_canon(t, t);
  fe_to_words(u1_w, t);
  fn_mul(t, r, w);
  fn_canon(t, t);
  fe_to_words(u2_w, t);
  return true;
}

// ---- signed W-bit digits --------------------------------------------------------
// digit i of u (LE words), carry-in c (0/1); returns d in [-(2^(W-1)-1), 2^(W-1)], updates c.
template <int W>
PBFTV_HD int signed_digit_w(const uint32_t u_w[8], int i, int& c) {
  const int bit = CombGeom<W>::bit(i), wd = CombGeom<W>::width(i);
  uint32_t b = 0;
  if (bit < 256) {
    const int wi = bit >> 5, sh = bit & 31;
    uint64_t two = u_w[wi];
    if (wi + 1 < 8) two |= (uint64_t)u_w[wi + 1] << 32;
    b = (uint32_t)(two >> sh) & ((1u << wd) - 1u);
  }
  const int d = (int)b + c;
  c = d > (1 << (wd - 1)) ? 1 : 0;
  return d - (c << wd);
}

PBFTV_HD int signed_digit(const uint32_t u_w[8], int i, int& c) { return signed_digit_w<8>(u_w, i, c); }

// unpack a table entry (16 words: x[8], y[8]) into field elements
PBFTV_HD void entry_to_fe(fe& x, fe& y, const uint32_t e[16]) {
  fe_from_words(x, e);
  fe_from_words(y, e + 8);
}

// ---- stage 2: joint comb -------------------------------------------------------
// R = u1*G + u2*Q accumulated in ONE Jacobian point: for every window i the G
// entry of digit d1_i and the Q entry of digit d2_i are added (mixed
// additions).  For honest inputs no step is exceptional; an adversarial
// (r, s, e) can force a partial sum to meet the next table point (doubling)
// or its negative (cancellation), and in both cases the unchecked addition
// yields Z == 0, which later additions preserve.  So a single Z == 0 test at
// the end decides whether to recompute the lane with complete additions
// (kCheck), which handle doubling and the point at infinity exactly.

// Add table entry (|d|-1) of window i with sign(d) to acc.
template <bool kCheck>
PBFTV_HD void comb_add_entry(jac& acc, bool& inf, int d, const uint32_t ew[16]) {
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
    return;
  }
  const int st = jac_madd<kCheck>(acc, x, y);
  if (kCheck) {
    if (st == 1) {
      jac p;
      p.x = x;
      p.y = y;
      fe_set(p.z, kOneP);
      jac_double(acc, p);
    } else if (st == 2) {
      inf = true;
    }
  }
}

template <bool kCheck, int WG, int WQ, class LoadG, class LoadQ>
PBFTV_HD bool comb2_pass(jac& acc, const uint32_t u1[8], const uint32_t u2[8], LoadG load_g, LoadQ load_q) {
  constexpr int nG = CombGeom<WG>::kWin, nQ = CombGeom<WQ>::kWin;
  constexpr int nW = nG > nQ ? nG : nQ;
  bool inf = true;
  int c1 = 0, c2 = 0;
  for (int i = 0; i < nW; ++i) {
    uint32_t ew[16];
    if (i < nG) {
      const int d1 = signed_digit_w<WG>(u1, i, c1);
      if (d1 != 0) {
        load_g(i, (d1 < 0 ? -d1 : d1) - 1, ew);
        comb_add_entry<kCheck>(acc, inf, d1, ew);
      }
    }
    if (i < nQ) {
      const int d2 = signed_digit_w<WQ>(u2, i, c2);
      if (d2 != 0) {
        load_q(i, (d2 < 0 ? -d2 : d2) - 1, ew);
        comb_add_entry<kCheck>(acc, inf, d2, ew);
      }
    }
  }
  return !inf;
}

// u1*G + u2*Q; false if the result is the point at infinity.  load_*(window,
// idx, words[16]) fetch table entries of the WG- / WQ-bit tables.
template <int WG = 8, int WQ = 8, class LoadG, class LoadQ>
PBFTV_HD bool comb2_mult(jac& acc, const uint32_t u1[8], const uint32_t u2[8], LoadG load_g, LoadQ load_q) {
  const bool ok = comb2_pass<false, WG, WQ>(acc, u1, u2, load_g, load_q);
  if (ok && fe_is_zero(acc.z)) return comb2_pass<true, WG, WQ>(acc, u1, u2, load_g, load_q);
  return ok;
}

// ---- final check --------------------------------------------------------------
// Accept iff R is finite and R.x mod n == r, where R.x = X / D (Jacobian:
// D = Z^2; XYZZ: D = ZZ):  X == r D (mod p), or X == (r + n) D when r + n < p.
// No field inversion.
PBFTV_HD bool ecdsa_check_xd(const fe& X, const fe& z2, bool finite, const uint32_t r_w[8]) {
  if (!finite) return false;
  fe rr, r2p, lhs;
  fe_from_words(rr, r_w);
  fe_set(r2p, kR2P);
  fe_mul(rr, rr, r2p);        // r in Montgomery form
  fe_mul(lhs, rr, z2);
  if (fe_equal(lhs, X)) return true;
  if (words_lt(r_w, kPMinusN32)) {  // r + n < p
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
    if (fe_equal(lhs, X)) return true;
  }
  return false;
}

PBFTV_HD bool ecdsa_check(const jac& R, bool finite, const uint32_t r_w[8]) {
  if (!finite) return false;
  fe z2;
  fe_sqr(z2, R.z);
  return ecdsa_check_xd(R.x, z2, true, r_w);
}

PBFTV_HD bool ecdsa_check(const xyzz& R, bool finite, const uint32_t r_w[8]) {
  return ecdsa_check_xd(R.x, R.zz, finite, r_w);
}

// The same test on the signed-limb accumulator (fes.h): X == r ZZ, or
// X == (r + n) ZZ when r + n < p.
PBFTV_HD bool ecdsa_check(const xyzz_s& R, bool finite, const uint32_t r_w[8]) {
  if (!finite) return false;
  fe rr, r2p, lhs, d;
  fe_from_words(rr, r_w);
  fe_set(r2p, kR2P);
  fs_mul(rr, rr, r2p);        // r in Montgomery form
  fs_mul(lhs, rr, R.zz);
  fs_sub(d, lhs, R.x);
  if (fs_is_zero(d)) return true;
  if (words_lt(r_w, kPMinusN32)) {  // r + n < p
    uint32_t rn[8];
    uint64_t cy = 0;
    for (int i = 0; i < 8; ++i) {
      cy += (uint64_t)r_w[i] + kN32[i];
      rn[i] = (uint32_t)cy;
      cy >>= 32;
    }
    fe_from_words(rr, rn);
    fs_mul(rr, rr, r2p);
    fs_mul(lhs, rr, R.zz);
    fs_sub(d, lhs, R.x);
    if (fs_is_zero(d)) return true;
  }
  return false;
}

// ---- the throughput comb's schedule (k_ecdsa_comb; comb2_verify restates it) ---
// Joint step order: step j of the nG + nQ additions takes the G entry of
// window j/2 (j even) and the Q entry (j odd) while both tables have windows
// left, then the longer table's remaining windows.  Steps 0 and 1 are G window
// 0 and Q window 0.
template <int WG, int WQ>
struct CombSteps {
  static constexpr int nG = CombGeom<WG>::kWin, nQ = CombGeom<WQ>::kWin;
  static constexpr int nMin = nG < nQ ? nG : nQ;
  static constexpr int nD = nG + nQ;
  // LDS digit storage: d - 1 fits int16 for W <= 16 (d in [-(2^15 - 1), 2^15])
  using Digit = std::conditional_t<(CombGeom<WG>::kW > 16 || CombGeom<WQ>::kW > 16), int, short>;
  PBFTV_HDM static constexpr bool is_q(int j) { return j < 2 * nMin ? (j & 1) != 0 : nQ > nG; }
  PBFTV_HDM static constexpr int win(int j) { return j < 2 * nMin ? j >> 1 : j - nMin; }
};

// (a & b) ^ c: ONE v_bitop3_b32 on the device (truth table 0x6A: bit
// 4 a + 2 b + c of the table is the result)
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ uint32_t and_xor(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x6A);
}
#else
static inline uint32_t and_xor(uint32_t a, uint32_t b, uint32_t c) { return (a & b) ^ c; }
#endif

// entry_to_fe, then y = neg ? -y : y (D-type), with the negation folded into
// the unpacking: a limb of y is (bits & mask ^ m) - m, two instructions
// instead of entry_to_fe's mask plus fs_cneg's negate and select
PBFTV_HD void entry_to_fe_cneg(fe& x, fe& y, const uint32_t e[16], bool neg) {
  fe_from_words(x, e);
  const uint32_t* w = e + 8;
  const uint32_t m = 0u - (uint32_t)neg;
  y.v[0] = and_xor(w[0], kMask29, m) - m;
  PBFTV_UNROLL for (int i = 1; i < 8; ++i) {
    const int bit = 29 * i, wi = bit >> 5, sh = bit & 31;
    const uint32_t lo = w[wi] >> sh;
    const uint32_t hi = (sh && wi + 1 < 8) ? (w[wi + 1] << (32 - sh)) : 0u;
    y.v[i] = and_xor(lo | hi, kMask29, m) - m;
  }
  y.v[8] = ((w[7] >> 8) ^ m) - m;
}

// The accumulator is XYZZ on signed limbs with W = sigma Y (neg_y: sigma = -1;
// xyzz_madd_s_flip).  Per signature:
//   * the first two digits both non-zero (all but ~2^-20 of signatures): the
//     accumulator starts as the affine sum of their points (comb_first2_s);
//   * every further step adds its point (comb_step_s: the generic step, which
//     also starts the accumulator when digits are zero);
//   * the last digit non-zero: the last addition is fused with the x check
//     (comb_last_check_s); otherwise the plain check of the accumulator.
// A result of -1 means an exceptional step (a doubling or cancellation met by
// the unchecked additions): the signature is redone with complete additions.
PBFTV_HD void comb_first2_s(xyzz_s& acc, bool& neg_y, int d0, const uint32_t w0[16], int d1, const uint32_t w1[16]) {
  fe x0, y0, x1, y1;
  entry_to_fe(x0, y0, w0);
  entry_to_fe(x1, y1, w1);
  xyzz_aff_aff_s(acc, x0, y0, x1, y1, (d0 < 0) != (d1 < 0));
  neg_y = d1 > 0;  // sigma = -s1
}

PBFTV_HD void comb_step_s(xyzz_s& acc, bool& inf, bool& neg_y, int d, const uint32_t w[16]) {
  if (d == 0) return;
  fe x, y;
  entry_to_fe_cneg(x, y, w, (d < 0) != neg_y);  // sigma * (+-y): D-type (no carry chain)
  if (inf) {
    acc.x = x;
    fs_norm(acc.y, y);
    fe_set(acc.zz, kOneP);
    fe_set(acc.zzz, kOneP);
    inf = false;
  } else {
    xyzz_madd_s_flip(acc, x, y);  // Y3 comes back with the other sign
    neg_y = !neg_y;
  }
}

// acc finite, d != 0: 1 / 0 = accept / reject, -1 = exceptional (ZZ1 == 0 from
// an earlier step, or P == 0: the last point equals the sum or its negative)
PBFTV_HD int comb_last_check_s(const xyzz_s& acc, bool neg_y, int d, const uint32_t w[16], const uint32_t r_w[8]) {
  fe x, y, rr, r2p, rz, dd;
  entry_to_fe(x, y, w);
  fs_cneg(y, y, (d < 0) != neg_y);
  xyzz_last_s L;
  xyzz_last_prep_s(L, acc, x, y);
  if (fs_is_zero(acc.zz) || fs_is_zero(L.p)) return -1;
  fe_from_words(rr, r_w);
  fe_set(r2p, kR2P);
  fs_mul(rr, rr, r2p);  // r in Montgomery form
  fs_mul(rz, rr, acc.zz);
  xyzz_last_d_s(dd, L, rz);
  if (fs_is_zero(dd)) return 1;
  if (words_lt(r_w, kPMinusN32)) {  // r + n < p
    uint32_t rn[8];
    uint64_t cy = 0;
    for (int i = 0; i < 8; ++i) {
      cy += (uint64_t)r_w[i] + kN32[i];
      rn[i] = (uint32_t)cy;
      cy >>= 32;
    }
    fe_from_words(rr, rn);
    fs_mul(rr, rr, r2p);
    fs_mul(rz, rr, acc.zz);
    xyzz_last_d_s(dd, L, rz);
    if (fs_is_zero(dd)) return 1;
  }
  return 0;
}

// Whole comb + check for one signature, in k_ecdsa_comb's schedule (the kernel
// makes the first-pair and last-step choices per wave, which changes no
// result: the generic step is exact for every digit pattern); complete-addition
// Jacobian rerun when a step was exceptional.  out_path (optional): bit 0 first
// pair, bit 1 fused last step, bit 2 rerun.
template <int WG = 8, int WQ = 8, class LoadG, class LoadQ>
PBFTV_HD bool comb2_verify(const uint32_t u1[8], const uint32_t u2[8], const uint32_t r_w[8], LoadG load_g,
                           LoadQ load_q, int* out_path = nullptr) {
  using S = CombSteps<WG, WQ>;
  int dg[S::nD];
  int c1 = 0, c2 = 0;
  for (int j = 0; j < S::nD; ++j)
    dg[j] = S::is_q(j) ? signed_digit_w<WQ>(u2, S::win(j), c2) : signed_digit_w<WG>(u1, S::win(j), c1);
  auto load = [&](int j, uint32_t w[16]) {
    const int idx = (dg[j] < 0 ? -dg[j] : dg[j]) - 1;
    if (S::is_q(j)) load_q(S::win(j), idx, w);
    else load_g(S::win(j), idx, w);
  };
  xyzz_s A;
  bool inf = true, neg_y = false;
  uint32_t w0[16], w1[16];
  int j0 = 0, path = 0;
  if (dg[0] != 0 && dg[1] != 0) {
    load(0, w0);
    load(1, w1);
    comb_first2_s(A, neg_y, dg[0], w0, dg[1], w1);
    inf = false;
    j0 = 2;
    path |= 1;
  }
  const bool fuse = j0 == 2 && dg[S::nD - 1] != 0;
  for (int j = j0; j < (fuse ? S::nD - 1 : S::nD); ++j) {
    if (dg[j] == 0) continue;
    load(j, w0);
    comb_step_s(A, inf, neg_y, dg[j], w0);
  }
  int res;
  if (fuse) {
    load(S::nD - 1, w0);
    res = comb_last_check_s(A, neg_y, dg[S::nD - 1], w0, r_w);
    path |= 2;
  } else {
    res = (!inf && fs_is_zero(A.zz)) ? -1 : (ecdsa_check(A, !inf, r_w) ? 1 : 0);
  }
  if (res < 0) {
    path |= 4;
    jac R;
    const bool f2 = comb2_pass<true, WG, WQ>(R, u1, u2, load_g, load_q);
    res = ecdsa_check(R, f2, r_w) ? 1 : 0;
  }
  if (out_path) *out_path = path;
  return res == 1;
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

// ---- generic (W-bit) table construction, three parallel phases --------------
// For base B and window i let B_i = 2^(W i) B, E = 2^(W-1) entries, CL =
// min(E, 256).  Entry idx (multiple m = idx + 1 = hi*CL + lo + 1) is
//     m * B_i = H_hi + L_lo,  L_lo = (lo + 1) B_i,  H_hi = hi * (CL B_i),
// so every entry is ONE addition of two precomputed affine points (hi = 0:
// a copy of L).  Phase 1 (lane per window) finds B_i, phase 2 (lane per
// window) the L and H tables, phase 3 (lane per 64-entry chunk) the sums;
// each phase normalises its points to affine with one inversion per lane
// (Montgomery's batch trick).  Scratch is a flat array of field elements
// reached through st(slot, fe) / ld(slot, fe): point j uses slots 3j..3j+2,
// the running Z product slot 3*cnt + j.

// Montgomery-trick batch conversion of cnt Jacobian points (in scratch) to
// canonical affine words out[16 j ...].
template <class StoreF, class LoadF>
PBFTV_HD void batch_to_affine(uint32_t* out, int cnt, StoreF st, LoadF ld) {
  fe pre, z;
  ld(2, pre);
  st(3 * cnt, pre);
  for (int j = 1; j < cnt; ++j) {
    ld(3 * j + 2, z);
    fe_mul(pre, pre, z);
    st(3 * cnt + j, pre);
  }
  fe inv;
  fe_inv(inv, pre);
  for (int j = cnt - 1; j >= 0; --j) {
    jac pt;
    ld(3 * j, pt.x);
    ld(3 * j + 1, pt.y);
    ld(3 * j + 2, pt.z);
    fe zinv;
    if (j > 0) {
      fe prev;
      ld(3 * cnt + j - 1, prev);
      fe_mul(zinv, inv, prev);
      fe_mul(inv, inv, pt.z);
    } else {
      zinv = inv;
    }
    jac_to_affine_words(out + (uint64_t)j * 16, pt, zinv);
  }
}

// Phase 1: out = affine words of 2^(W win) * (bx, by).
PBFTV_HD void window_base(uint32_t out[16], int shift_bits, const fe& bx, const fe& by) {
  jac cur;
  cur.x = bx;
  cur.y = by;
  fe_set(cur.z, kOneP);
  for (int k = 0; k < shift_bits; ++k) jac_double(cur, cur);
  fe zi;
  fe_inv(zi, cur.z);
  jac_to_affine_words(out, cur, zi);
}

// Phase 2 helper: out[16 (k-1)] = k * P for k = 1..cnt (P affine words).
template <class StoreF, class LoadF>
PBFTV_HD void multiples(uint32_t* out, int cnt, const uint32_t pw[16], StoreF st, LoadF ld) {
  fe px, py;
  entry_to_fe(px, py, pw);
  jac cur;
  cur.x = px;
  cur.y = py;
  fe_set(cur.z, kOneP);
  for (int k = 0; k < cnt; ++k) {
    if (k == 1) jac_double(cur, cur);
    else if (k >= 2) jac_madd<false>(cur, px, py);  // (k+1) P with k+1 <= 2^15 << n: never exceptional
    st(3 * k, cur.x);
    st(3 * k + 1, cur.y);
    st(3 * k + 2, cur.z);
  }
  batch_to_affine(out, cnt, st, ld);
}

// Phase 3: out[16 j] = H + L[j] for j < cnt (H affine words; has_h = false: copy L).
// H = hi*CL*B_i and L[j] = (lo+1) B_i meet only for hi = 1, lo + 1 = CL (a doubling).
template <class StoreF, class LoadF>
PBFTV_HD void sums_chunk(uint32_t* out, int cnt, bool has_h, const uint32_t hw[16], const uint32_t* L, StoreF st,
                         LoadF ld) {
  if (!has_h) {
    for (int j = 0; j < cnt * 16; ++j) out[j] = L[j];
    return;
  }
  fe hx, hy;
  entry_to_fe(hx, hy, hw);
  for (int j = 0; j < cnt; ++j) {
    fe lx, ly;
    entry_to_fe(lx, ly, L + (uint64_t)j * 16);
    jac cur;
    cur.x = hx;
    cur.y = hy;
    fe_set(cur.z, kOneP);
    if (jac_madd<true>(cur, lx, ly) == 1) jac_double(cur, cur);
    st(3 * j, cur.x);
    st(3 * j + 1, cur.y);
    st(3 * j + 2, cur.z);
  }
  batch_to_affine(out, cnt, st, ld);
}

// Whole table of one base on the CPU harness (tests) -- the device runs the
// same phases as separate kernels (p256_kernels.hip).
template <int W, class StoreF, class LoadF>
PBFTV_HD void build_table_serial(uint32_t* table, const fe& bx, const fe& by, uint32_t* lbuf, uint32_t* hbuf,
                                 StoreF st, LoadF ld) {
  using G = CombGeom<W>;
  constexpr int CL = G::kEnt < 256 ? G::kEnt : 256;
  constexpr int NH = G::kEnt / CL;
  for (int win = 0; win < G::kWin; ++win) {
    uint32_t bw[16];
    window_base(bw, G::bit(win), bx, by);
    multiples(lbuf, CL, bw, st, ld);
    if (NH > 1) multiples(hbuf, NH - 1, lbuf + (uint64_t)(CL - 1) * 16, st, ld);
    uint32_t* tw = table + G::base(win) * 16;
    for (int hi = 0; hi < G::ent(win) / CL; ++hi)
      sums_chunk(tw + (uint64_t)hi * CL * 16, CL, hi > 0, hbuf + (uint64_t)(hi > 0 ? hi - 1 : 0) * 16, lbuf, st, ld);
  }
}

}  // namespace pbftv
