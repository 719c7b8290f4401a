// algo_harness.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Compiles the GPU kernels' arithmetic headers (simple_pbft_amd/csrc/fe29.h,
// p256_algo.h) with g++ so that tests/test_algo_cpu.py can check, on the
// CPU of this container, the exact limb arithmetic, bounds and verify
// pipeline that the HIP kernels run.  It is never linked into or loaded by
// the product library (simple_pbft_amd/libpbftv.so), which runs this code on
// the GPU only.
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../simple_pbft_amd/csrc/p256_algo.h"
#include "../../simple_pbft_amd/csrc/fes.h"

using namespace pbftv;

extern "C" {

void h_fe_mul(const uint32_t* a, const uint32_t* b, uint32_t* r) {
  fe x, y, z;
  memcpy(x.v, a, 36); memcpy(y.v, b, 36);
  fe_mul(z, x, y);
  memcpy(r, z.v, 36);
}
void h_fe_sqr(const uint32_t* a, uint32_t* r) {
  fe x, z;
  memcpy(x.v, a, 36);
  fe_sqr(z, x);
  memcpy(r, z.v, 36);
}
void h_fe_sub(const uint32_t* a, const uint32_t* b, uint32_t* r) {
  fe x, y, z;
  memcpy(x.v, a, 36); memcpy(y.v, b, 36);
  fe_sub(z, x, y);
  memcpy(r, z.v, 36);
}
void h_fe_mul_small(const uint32_t* a, uint32_t k, uint32_t* r) {
  fe x, z;
  memcpy(x.v, a, 36);
  fe_mul_small(z, x, k);
  memcpy(r, z.v, 36);
}
void h_fe_canon(const uint32_t* a, uint32_t* r) {
  fe x, z;
  memcpy(x.v, a, 36);
  fe_canon(z, x);
  memcpy(r, z.v, 36);
}
void h_fn_mul(const uint32_t* a, const uint32_t* b, uint32_t* r) {
  fe x, y, z;
  memcpy(x.v, a, 36); memcpy(y.v, b, 36);
  fn_mul(z, x, y);
  memcpy(r, z.v, 36);
}
void h_fe_from_words(const uint32_t* w, uint32_t* r) {
  fe z;
  fe_from_words(z, w);
  memcpy(r, z.v, 36);
}
void h_fe_to_words(const uint32_t* a, uint32_t* w) {
  fe x;
  memcpy(x.v, a, 36);
  fe_to_words(w, x);
}
void h_inv_n_words(const uint32_t* x, uint32_t* out) { inv_mod_n_words(out, x); }
void h_inv_n_words_ct(const uint32_t* x, uint32_t* out) { inv_mod_n_words_ct(out, x); }

void h_fn_inv_mont(const uint32_t* a, int use_gcd, uint32_t* r) {
  fe x, y;
  fe_set(x, a);
  if (use_gcd) fn_inv_mont_gcd(y, x);
  else fn_inv_mont(y, x);
  std::memcpy(r, y.v, 36);
}

int h_scalars(const uint32_t* e, const uint32_t* r, const uint32_t* s, uint32_t* u1, uint32_t* u2) {
  return ecdsa_scalars(e, r, s, u1, u2) ? 1 : 0;
}

static void be32_to_le_words(const uint8_t* b, uint32_t* w) {
  for (int i = 0; i < 8; ++i) {
    const uint8_t* p = b + 4 * (7 - i);
    w[i] = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
  }
}

// Build the comb table of base (x, y) [big-endian 64 B]; returns key validity.
int h_build_table(const uint8_t* pub_xy, uint32_t* table) {
  uint32_t xw[8], yw[8];
  be32_to_le_words(pub_xy, xw);
  be32_to_le_words(pub_xy + 32, yw);
  fe xm, ym;
  if (!key_check(xw, yw, xm, ym)) {
    memset(table, 0, kTableBytes);
    return 0;
  }
  std::vector<fe> scratch(kScratchSlots);
  for (int w = 0; w < kWindows; ++w) {
    build_window(table + (uint64_t)w * kEntries * kEntryWords, w, xm, ym,
                 [&](int slot, const fe& v) { scratch[slot] = v; },
                 [&](int slot, fe& v) { v = scratch[slot]; });
  }
  return 1;
}

void h_build_g_table(uint32_t* table) {
  fe gx, gy;
  fe_set(gx, kGxMont);
  fe_set(gy, kGyMont);
  std::vector<fe> scratch(kScratchSlots);
  for (int w = 0; w < kWindows; ++w) {
    build_window(table + (uint64_t)w * kEntries * kEntryWords, w, gx, gy,
                 [&](int slot, const fe& v) { scratch[slot] = v; },
                 [&](int slot, fe& v) { v = scratch[slot]; });
  }
}

}  // extern "C"

// Table of width W (8, 10, 12) via the generic three-phase builder;
// base = pub (64 B BE) or G when pub is null.  Returns key validity.
template <int W>
static int build_w(const uint8_t* pub_xy, uint32_t* table) {
  fe xm, ym;
  if (pub_xy) {
    uint32_t xw[8], yw[8];
    be32_to_le_words(pub_xy, xw);
    be32_to_le_words(pub_xy + 32, yw);
    if (!key_check(xw, yw, xm, ym)) return 0;
  } else {
    fe_set(xm, kGxMont);
    fe_set(ym, kGyMont);
  }
  std::vector<fe> scratch(4 * 256);
  std::vector<uint32_t> lbuf(256 * 16), hbuf(256 * 16);
  build_table_serial<W>(table, xm, ym, lbuf.data(), hbuf.data(), [&](int slot, const fe& v) { scratch[slot] = v; },
                        [&](int slot, fe& v) { v = scratch[slot]; });
  return 1;
}

extern "C" {

int h_build_table_w(const uint8_t* pub_xy, int w, uint32_t* table) {
  switch (w) {
    case 8: return build_w<8>(pub_xy, table);
    case 10: return build_w<10>(pub_xy, table);
    case 12: return build_w<12>(pub_xy, table);
    case 11: return build_w<11>(pub_xy, table);  // mixed: 15 x 12 + 7 x 11 bits
    default: return -1;
  }
}

// Full pipeline with (WG, WQ) = (w, w) tables built by h_build_table_w.
int h_verify_w(int w, const uint8_t* hash, const uint8_t* rs, const uint32_t* gtab, const uint32_t* qtab, int key_valid) {
  if (!key_valid) return 0;
  uint32_t e[8], r[8], s[8], u1[8], u2[8];
  be32_to_le_words(hash, e);
  be32_to_le_words(rs, r);
  be32_to_le_words(rs + 32, s);
  if (!ecdsa_scalars(e, r, s, u1, u2)) return 0;
  bool ok = false;
  auto run = [&](auto geom) {
    constexpr int W = decltype(geom)::kCode;
    auto lg = [&](int win, int idx, uint32_t* out) { memcpy(out, gtab + (CombGeom<W>::base(win) + idx) * 16, 64); };
    auto lq = [&](int win, int idx, uint32_t* out) { memcpy(out, qtab + (CombGeom<W>::base(win) + idx) * 16, 64); };
    ok = comb2_verify<W, W>(u1, u2, r, lg, lq);
  };
  if (w == 8) run(CombGeom<8>());
  else if (w == 10) run(CombGeom<10>());
  else if (w == 12) run(CombGeom<12>());
  else if (w == 11) run(CombGeom<11>());
  else return -1;
  return ok ? 1 : 0;
}

// comb2_verify (k_ecdsa_comb's schedule) on chosen scalars u1, u2 and r (LE
// words) with (w, w) tables; *path: bit 0 first pair, 1 fused last step, 2 rerun
int h_comb_verify_u(int w, const uint32_t* u1, const uint32_t* u2, const uint32_t* r, const uint32_t* gtab,
                    const uint32_t* qtab, int* path) {
  bool ok = false;
  auto run = [&](auto geom) {
    constexpr int W = decltype(geom)::kCode;
    auto lg = [&](int win, int idx, uint32_t* out) { memcpy(out, gtab + (CombGeom<W>::base(win) + idx) * 16, 64); };
    auto lq = [&](int win, int idx, uint32_t* out) { memcpy(out, qtab + (CombGeom<W>::base(win) + idx) * 16, 64); };
    ok = comb2_verify<W, W>(u1, u2, r, lg, lq, path);
  };
  if (w == 8) run(CombGeom<8>());
  else if (w == 11) run(CombGeom<11>());
  else return -1;
  return ok ? 1 : 0;
}

// ---- signed-limb arithmetic (fes.h) ----
void h_fs_mul(const uint32_t* a, const uint32_t* b, uint32_t* r) {
  fe x, y, z;
  memcpy(x.v, a, 36); memcpy(y.v, b, 36);
  fs_mul(z, x, y);
  memcpy(r, z.v, 36);
}
void h_fs_sqr(const uint32_t* a, uint32_t* r) {
  fe x, z;
  memcpy(x.v, a, 36);
  fs_sqr(z, x);
  memcpy(r, z.v, 36);
}
void h_fs_mul2_add(const uint32_t* a, const uint32_t* b, const uint32_t* c, const uint32_t* d, uint32_t* r) {
  fe x, y, u, v, z;
  memcpy(x.v, a, 36); memcpy(y.v, b, 36); memcpy(u.v, c, 36); memcpy(v.v, d, 36);
  fs_mul2_add(z, x, y, u, v);
  memcpy(r, z.v, 36);
}
void h_fs_sqr_sub2(const uint32_t* a, const uint32_t* b, const uint32_t* c, uint32_t* r) {
  fe x, y, u, z;
  memcpy(x.v, a, 36); memcpy(y.v, b, 36); memcpy(u.v, c, 36);
  fs_sqr_sub2(z, x, y, u);
  memcpy(r, z.v, 36);
}
void h_fs_sqr_mul_add(const uint32_t* a, const uint32_t* b, const uint32_t* c, uint32_t* r) {
  fe x, y, u, z;
  memcpy(x.v, a, 36); memcpy(y.v, b, 36); memcpy(u.v, c, 36);
  fs_sqr_mul_add(z, x, y, u);
  memcpy(r, z.v, 36);
}
// pts = x0 || y0 || x1 || y1 (canonical limbs, 36 words); acc out as in h_xyzz_madd_s
void h_xyzz_aff_aff_s(const uint32_t* pts, int flip, uint32_t* acc) {
  fe x0, y0, x1, y1;
  memcpy(x0.v, pts, 36); memcpy(y0.v, pts + 9, 36); memcpy(x1.v, pts + 18, 36); memcpy(y1.v, pts + 27, 36);
  xyzz_s A;
  xyzz_aff_aff_s(A, x0, y0, x1, y1, flip != 0);
  memcpy(acc, A.x.v, 36); memcpy(acc + 9, A.y.v, 36); memcpy(acc + 18, A.zz.v, 36); memcpy(acc + 27, A.zzz.v, 36);
}
// the fused last step: acc (36 words), the entry's canonical words (16), digit d, r (LE words)
int h_comb_last_check_s(const uint32_t* acc, int neg_y, int d, const uint32_t* w16, const uint32_t* r) {
  xyzz_s A;
  memcpy(A.x.v, acc, 36); memcpy(A.y.v, acc + 9, 36); memcpy(A.zz.v, acc + 18, 36); memcpy(A.zzz.v, acc + 27, 36);
  return comb_last_check_s(A, neg_y != 0, d, w16, r);
}
int h_fs_is_zero(const uint32_t* a) {
  fe x;
  memcpy(x.v, a, 36);
  return fs_is_zero(x) ? 1 : 0;
}
// the fold of fs_is_zero (fe_fold_carry) on S/D-type limbs
void h_fs_fold(const uint32_t* a, uint32_t* r) {
  int32_t d[9];
  memcpy(d, a, 36);
  fe n;
  fe_fold_carry(n, d);
  memcpy(r, n.v, 36);
}
void h_fs_norm(const uint32_t* a, uint32_t* r) {
  fe x, z;
  memcpy(x.v, a, 36);
  fs_norm(z, x);
  memcpy(r, z.v, 36);
}
void h_fs_canon(const uint32_t* a, uint32_t* r) {
  fe x, z;
  memcpy(x.v, a, 36);
  fs_canon(z, x);
  memcpy(r, z.v, 36);
}
void h_xyzz_madd_s(uint32_t* acc, const uint32_t* pt) {
  xyzz_s A;
  fe x, y;
  memcpy(A.x.v, acc, 36); memcpy(A.y.v, acc + 9, 36); memcpy(A.zz.v, acc + 18, 36); memcpy(A.zzz.v, acc + 27, 36);
  memcpy(x.v, pt, 36); memcpy(y.v, pt + 9, 36);
  xyzz_madd_s(A, x, y);
  memcpy(acc, A.x.v, 36); memcpy(acc + 9, A.y.v, 36); memcpy(acc + 18, A.zz.v, 36); memcpy(acc + 27, A.zzz.v, 36);
}

void h_xyzz_madd_s_flip(uint32_t* acc, const uint32_t* pt) {
  xyzz_s A;
  fe x, y;
  memcpy(A.x.v, acc, 36); memcpy(A.y.v, acc + 9, 36); memcpy(A.zz.v, acc + 18, 36); memcpy(A.zzz.v, acc + 27, 36);
  memcpy(x.v, pt, 36); memcpy(y.v, pt + 9, 36);
  xyzz_madd_s_flip(A, x, y);
  memcpy(acc, A.x.v, 36); memcpy(acc + 9, A.y.v, 36); memcpy(acc + 18, A.zz.v, 36); memcpy(acc + 27, A.zzz.v, 36);
}

// XYZZ mixed addition on raw limbs: acc = x||y||zz||zzz (36 words), pt = x||y (18 words).
void h_xyzz_madd(uint32_t* acc, const uint32_t* pt) {
  xyzz A;
  fe x, y;
  memcpy(A.x.v, acc, 36); memcpy(A.y.v, acc + 9, 36); memcpy(A.zz.v, acc + 18, 36); memcpy(A.zzz.v, acc + 27, 36);
  memcpy(x.v, pt, 36); memcpy(y.v, pt + 9, 36);
  xyzz_madd(A, x, y);
  memcpy(acc, A.x.v, 36); memcpy(acc + 9, A.y.v, 36); memcpy(acc + 18, A.zz.v, 36); memcpy(acc + 27, A.zzz.v, 36);
}

// u * G via the joint comb (u2 = 0), unchecked (0) or complete-addition (1)
// path; affine canonical plain (non-Montgomery) x||y as LE words.  Returns 0
// for the point at infinity.
int h_comb(const uint32_t* u, const uint32_t* tab, int checked, uint32_t* out_xy) {
  jac A;
  const uint32_t zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto load = [&](int win, int idx, uint32_t* o) {
    memcpy(o, tab + ((uint64_t)win * kEntries + idx) * kEntryWords, 64);
  };
  bool ok = checked ? comb2_pass<true, 8, 8>(A, u, zero, load, load) : comb2_mult(A, u, zero, load, load);
  if (!ok) return 0;
  fe zi, x, y, plain1;
  fe_inv(zi, A.z);
  uint32_t w[16];
  jac_to_affine_words(w, A, zi);
  entry_to_fe(x, y, w);
  const uint32_t p1[9] = {1, 0, 0, 0, 0, 0, 0, 0, 0};
  fe_set(plain1, p1);
  fe_mul(x, x, plain1);  // out of Montgomery form
  fe_mul(y, y, plain1);
  fe_canon(x, x);
  fe_canon(y, y);
  fe_to_words(out_xy, x);
  fe_to_words(out_xy + 8, y);
  return 1;
}

// Full pipeline on one signature given prebuilt tables.
int h_verify(const uint8_t* hash, const uint8_t* rs, const uint32_t* gtab, const uint32_t* qtab, int key_valid) {
  if (!key_valid) return 0;
  uint32_t e[8], r[8], s[8], u1[8], u2[8];
  be32_to_le_words(hash, e);
  be32_to_le_words(rs, r);
  be32_to_le_words(rs + 32, s);
  if (!ecdsa_scalars(e, r, s, u1, u2)) return 0;
  return comb2_verify(
             u1, u2, r,
             [&](int win, int idx, uint32_t* out) { memcpy(out, gtab + ((uint64_t)win * kEntries + idx) * kEntryWords, 64); },
             [&](int win, int idx, uint32_t* out) { memcpy(out, qtab + ((uint64_t)win * kEntries + idx) * kEntryWords, 64); })
             ? 1
             : 0;
}

}  // extern "C"
