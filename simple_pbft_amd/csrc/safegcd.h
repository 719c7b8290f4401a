// safegcd.h -- x^-1 mod n (P-256 group order) by Bernstein-Yang divsteps.
//
// Replaces the Fermat chain x^(n-2) (253 squarings + 39 multiplies, ~24k
// v_mad_u64_u32 in one dependent chain) where the latency of ONE inversion
// matters -- the quorum-certificate path -- and cuts the per-lane inversion
// in the throughput scalar kernel.  Variable time: every input is public
// signature data.
//
// Algorithm (Bernstein & Yang, "Fast constant-time gcd computation and
// modular inversion", 2019), restated for 30-bit signed limbs:
//   f = n, g = x, d = 0, e = 1, eta = -1 (= -delta of the paper's divstep)
//   repeat: 30 divsteps on the low 30 bits of (f, g) give a 2x2 matrix t with
//           2^30 (f', g') = t (f, g); apply it to (f, g) exactly and to
//           (d, e) mod n (adding multiples of n so the division by 2^30 is
//           exact), keeping the invariants f == d x, g == e x (mod n)
//   until g == 0; then f = +-1 and x^-1 = +-d.
// At most 741 divsteps for 256-bit inputs (the paper's bound), i.e. 25
// batches of 30.  Inside a batch the divsteps run several at a time: a run
// of zero low bits of g is one shift, and while eta >= 0 up to min(eta+1, 6)
// low bits of g are cancelled at once with w = -g/f mod 2^k (f^-1 mod 64 by
// one Newton step from f*f == 1 mod 8).
#pragma once
#include "fe29.h"

namespace pbftv {

constexpr uint32_t kM30 = (1u << 30) - 1;

struct s30 {
  int32_t v[9];  // value = sum v[i] 2^(30 i); v[0..7] in [0, 2^30), v[8] signed
};

struct trans30 {
  int32_t u, v, q, r;
};

// 30 divsteps on the low bits of f (odd) and g; returns the new eta.
PBFTV_HD int32_t divsteps30_var(int32_t eta, uint32_t f, uint32_t g, trans30& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  int i = 30;
  for (;;) {
    const int zeros = __builtin_ctz(g | (0xFFFFFFFFu << i));
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    // g is odd here
    if (eta < 0) {  // delta > 0: (f, g) <- (g, -f)
      eta = -eta;
      uint32_t x = f;
      f = g;
      g = 0u - x;
      x = u;
      u = q;
      q = 0u - x;
      x = v;
      v = r;
      r = 0u - x;
    }
    const int lim = (eta + 1) > i ? i : (eta + 1);
    const uint32_t m = (0xFFFFFFFFu >> (32 - lim)) & 63u;
    const uint32_t w = (f * g * (f * f - 2u)) & m;  // -g / f mod 2^lim
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return eta;
}

// 30 divsteps in constant time (branch-free masks; Bernstein-Yang with
// zeta = -(delta + 1/2), as libsecp256k1's modinv32 divsteps_30): a straight
// dependent chain with no data-dependent branches -- for the latency path,
// where one wave runs one inversion and divergence-free straight-line code
// lets the compiler overlap it with the previous batch's matrix update.
PBFTV_HD int32_t divsteps30_ct(int32_t zeta, uint32_t f, uint32_t g, trans30& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  PBFTV_UNROLL for (int i = 0; i < 30; ++i) {
    uint32_t c1 = (uint32_t)(zeta >> 31);  // zeta < 0
    const uint32_t c2 = 0u - (g & 1u);     // g odd
    const uint32_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2;
    q += y & c2;
    r += z & c2;
    c1 &= c2;
    zeta = (int32_t)(((uint32_t)zeta ^ c1) - 1u);
    f += g & c1;
    u += q & c1;
    v += r & c1;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return zeta;
}

// (f, g) <- t (f, g) / 2^30 (exact)
PBFTV_HD void update_fg30(s30& f, s30& g, const trans30& t) {
  int64_t cf = (int64_t)t.u * f.v[0] + (int64_t)t.v * g.v[0];
  int64_t cg = (int64_t)t.q * f.v[0] + (int64_t)t.r * g.v[0];
  cf >>= 30;
  cg >>= 30;
  PBFTV_UNROLL for (int i = 1; i < 9; ++i) {
    cf += (int64_t)t.u * f.v[i] + (int64_t)t.v * g.v[i];
    cg += (int64_t)t.q * f.v[i] + (int64_t)t.r * g.v[i];
    f.v[i - 1] = (int32_t)((uint32_t)cf & kM30);
    g.v[i - 1] = (int32_t)((uint32_t)cg & kM30);
    cf >>= 30;
    cg >>= 30;
  }
  f.v[8] = (int32_t)cf;
  g.v[8] = (int32_t)cg;
}

// (d, e) <- t (d, e) / 2^30 mod n, inputs and outputs in (-2n, n).  The
// multiples md, me of n make the low 30 bits vanish; their sign-dependent
// start keeps the result in range.
PBFTV_HD void update_de30(s30& d, s30& e, const trans30& t) {
  const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
  int32_t md = (t.u & sd) + (t.v & se);
  int32_t me = (t.q & sd) + (t.r & se);
  int64_t cd = (int64_t)t.u * d.v[0] + (int64_t)t.v * e.v[0];
  int64_t ce = (int64_t)t.q * d.v[0] + (int64_t)t.r * e.v[0];
  md -= (int32_t)((kNInv30 * (uint32_t)cd + (uint32_t)md) & kM30);
  me -= (int32_t)((kNInv30 * (uint32_t)ce + (uint32_t)me) & kM30);
  cd += (int64_t)kN30[0] * md;
  ce += (int64_t)kN30[0] * me;
  cd >>= 30;
  ce >>= 30;
  PBFTV_UNROLL for (int i = 1; i < 9; ++i) {
    cd += (int64_t)t.u * d.v[i] + (int64_t)t.v * e.v[i] + (int64_t)kN30[i] * md;
    ce += (int64_t)t.q * d.v[i] + (int64_t)t.r * e.v[i] + (int64_t)kN30[i] * me;
    d.v[i - 1] = (int32_t)((uint32_t)cd & kM30);
    e.v[i - 1] = (int32_t)((uint32_t)ce & kM30);
    cd >>= 30;
    ce >>= 30;
  }
  d.v[8] = (int32_t)cd;
  e.v[8] = (int32_t)ce;
}

PBFTV_HD bool s30_is_zero(const s30& a) {
  int32_t o = 0;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) o |= a.v[i];
  return o == 0;
}

// a <- a + sign * n, limbs re-normalised (sign in {-1, 0, 1})
PBFTV_HD void s30_add_n(s30& a, int32_t sign) {
  int32_t c = 0;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    const int32_t x = a.v[i] + sign * (int32_t)kN30[i] + c;
    if (i < 8) {
      a.v[i] = x & (int32_t)kM30;
      c = x >> 30;
    } else {
      a.v[i] = x;
    }
  }
}

PBFTV_HD void s30_neg(s30& a) {
  int32_t c = 0;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    const int32_t x = -a.v[i] + c;
    if (i < 8) {
      a.v[i] = x & (int32_t)kM30;
      c = x >> 30;
    } else {
      a.v[i] = x;
    }
  }
}

// a - n >= 0 for normalised a >= 0
PBFTV_HD bool s30_ge_n(const s30& a) {
  int32_t c = 0;
  PBFTV_UNROLL for (int i = 0; i < 8; ++i) c = (a.v[i] - (int32_t)kN30[i] + c) >> 30;
  return a.v[8] - (int32_t)kN30[8] + c >= 0;
}

PBFTV_HD void words_to_s30(s30& a, const uint32_t w[8]) {
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    const int bit = 30 * i, wi = bit >> 5, sh = bit & 31;
    uint32_t x = w[wi] >> sh;
    if (sh > 2 && wi + 1 < 8) x |= w[wi + 1] << (32 - sh);
    a.v[i] = (int32_t)(x & kM30);
  }
}

PBFTV_HD void s30_to_words(uint32_t w[8], const s30& a) {
  PBFTV_UNROLL for (int k = 0; k < 8; ++k) {
    const int bit = 32 * k, li = bit / 30, sh = bit % 30;
    uint32_t x = (uint32_t)a.v[li] >> sh;
    if (li + 1 < 9) x |= (uint32_t)a.v[li + 1] << (30 - sh);
    if (sh > 28 && li + 2 < 9) x |= (uint32_t)a.v[li + 2] << (60 - sh);
    w[k] = x;
  }
}

// out = x^-1 mod n (canonical LE words) for 0 < x < n; 0 for x == 0.
PBFTV_HD void inv_mod_n_words(uint32_t out[8], const uint32_t x[8]) {
  s30 f, g, d, e;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    f.v[i] = (int32_t)kN30[i];
    d.v[i] = 0;
    e.v[i] = 0;
  }
  e.v[0] = 1;
  words_to_s30(g, x);
  int32_t eta = -1;
  for (int it = 0; it < 25; ++it) {
    trans30 t;
    eta = divsteps30_var(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    update_de30(d, e, t);
    update_fg30(f, g, t);
    if (s30_is_zero(g)) break;
  }
  // f = +-1; d in (-2n, n)
  if (f.v[8] < 0) s30_neg(d);  // now in (-n, 2n)
  if (d.v[8] < 0) s30_add_n(d, 1);
  if (d.v[8] < 0) s30_add_n(d, 1);
  if (s30_ge_n(d)) s30_add_n(d, -1);
  s30_to_words(out, d);
}

// inv_mod_n_words with constant-time divsteps (all 25 batches; same result).
PBFTV_HD void inv_mod_n_words_ct(uint32_t out[8], const uint32_t x[8]) {
  s30 f, g, d, e;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    f.v[i] = (int32_t)kN30[i];
    d.v[i] = 0;
    e.v[i] = 0;
  }
  e.v[0] = 1;
  words_to_s30(g, x);
  int32_t zeta = -1;
  for (int it = 0; it < 25; ++it) {
    trans30 t;
    zeta = divsteps30_ct(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    update_de30(d, e, t);
    update_fg30(f, g, t);
  }
  if (f.v[8] < 0) s30_neg(d);
  if (d.v[8] < 0) s30_add_n(d, 1);
  if (d.v[8] < 0) s30_add_n(d, 1);
  if (s30_ge_n(d)) s30_add_n(d, -1);
  s30_to_words(out, d);
}

// r = x^-1 * R mod n for x in Montgomery form (x = X R): the plain inverse
// of x is X^-1 R^-1; one Montgomery product with R^3 gives X^-1 R.
PBFTV_HD void fn_inv_mont_gcd(fe& r, const fe& x) {
  fe c;
  fn_canon(c, x);
  uint32_t w[8], iw[8];
  fe_to_words(w, c);
  inv_mod_n_words(iw, w);
  fe inv, r3;
  fe_from_words(inv, iw);
  fe_set(r3, kR3N);
  fn_mul(r, inv, r3);
}

}  // namespace pbftv
