// p256_kernels.hip -- ECDSA-P256 batch verification kernels for gfx950.
//
// Throughput path: one signature per lane (64 per wave).
//   k_tab_*          key validation + fixed-base comb tables for G and every
//                    registered key (three-phase parallel build).
//   k_ecdsa_scalars  Go's range checks on (r, s), w = s^-1 mod n (K signatures
//                    per lane share one safegcd inversion), u1 = e w, u2 = r w
//                    -> 64 B of scalars per signature.
//   k_ecdsa_comb     u1*G + u2*Q as one joint signed-digit comb over the W-bit
//                    tables (XYZZ mixed additions only) and the x-coordinate check
//                    X == r ZZ (or (r+n) ZZ) -- no field inversion.  Writes
//                    the LSB-first accept bitmap via a wave ballot.
// Latency path (small batches, e.g. one quorum certificate): one WAVE per
// signature, k_ecdsa_wave (see there).
// Semantics: Go 1.19 crypto/ecdsa.Verify (see p256_algo.h); parity with the
// oracle is tested in tests/test_gpu_parity.py.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "kernels.h"
#include "p256_algo.h"

namespace pbftv {

#ifndef PBFTV_COMB_WAVES
#define PBFTV_COMB_WAVES 4  // min waves per SIMD for k_ecdsa_comb: 128 VGPRs; +1.2 % over 2 (tools/ab.sh)
#endif

// key-order sort (k_key_*): blocks of the histogram/scatter passes, largest key count sorted
constexpr uint32_t kSortBlocks = 256;
constexpr uint32_t kSortMaxKeys = 1024;

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// 32 big-endian bytes at p (16-B aligned) -> 8 LE words
__device__ __forceinline__ void load_be256(const uint8_t* __restrict__ p, uint32_t w[8]) {
  const uint4 a = *reinterpret_cast<const uint4*>(p);
  const uint4 b = *reinterpret_cast<const uint4*>(p + 16);
  w[7] = bswap32(a.x); w[6] = bswap32(a.y); w[5] = bswap32(a.z); w[4] = bswap32(a.w);
  w[3] = bswap32(b.x); w[2] = bswap32(b.y); w[1] = bswap32(b.z); w[0] = bswap32(b.w);
}

// ---------------------------------------------------------------------------
// Table construction (p256_algo.h, "generic (W-bit) table construction"):
// three kernels over all bases of a registration.  Base b of a launch is G
// when with_g && b == 0, else key key0 + b - with_g.
template <int W>
struct TabGeom {
  using G = CombGeom<W>;
  // L table: (lo+1) B_i, lo < CL; H table: hi (CL B_i), 1 <= hi < NH.  Up to
  // W = 16 CL = 256; wider windows split E = CL * NH near sqrt(E) so neither
  // phase-2 walk gets long (W = 20: 1024 x 512, W = 24: 4096 x 2048,
  // W = 26: 8192 x 4096).
  static constexpr int CL = G::kEnt < 256 ? G::kEnt : (G::kW <= 16 ? 256 : 1 << (G::kW / 2));
  static constexpr int NH = G::kEnt / CL;
  static constexpr int PC = CL < 64 ? CL : 64;              // entries per phase-3 lane
  static constexpr int SS = 4 * (CL > NH - 1 ? CL : NH - 1);  // phase-2 scratch slots per lane
};

__device__ __forceinline__ bool load_base(const uint32_t* __restrict__ keys_le, uint32_t key0, uint32_t b, int with_g,
                                          fe& bx, fe& by) {
  if (with_g && b == 0) {
    fe_set(bx, kGxMont);
    fe_set(by, kGyMont);
    return true;
  }
  const uint32_t* k = keys_le + (uint64_t)(key0 + b - with_g) * 16;
  uint32_t xw[8], yw[8];
  for (int i = 0; i < 8; ++i) { xw[i] = k[i]; yw[i] = k[8 + i]; }
  if (key_check(xw, yw, bx, by)) return true;
  fe_set(bx, kGxMont);  // invalid key: build a harmless table (never used: valid[] = 0)
  fe_set(by, kGyMont);
  return false;
}

// phase 1: lane (b, win) -> bases[(b*nwin + win)*16] = 2^(W win) B affine; valid flags for keys
template <int W>
__global__ void __launch_bounds__(64) k_tab_bases(const uint32_t* __restrict__ keys_le, uint32_t key0, uint32_t nb,
                                                  int with_g, uint32_t* __restrict__ valid,
                                                  uint32_t* __restrict__ bases) {
  constexpr int nwin = CombGeom<W>::kWin;
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= nb * nwin) return;
  const uint32_t b = lane / nwin, win = lane % nwin;
  fe bx, by;
  const bool ok = load_base(keys_le, key0, b, with_g, bx, by);
  if (win == 0 && !(with_g && b == 0)) valid[key0 + b - with_g] = ok ? 1u : 0u;
  window_base(bases + (uint64_t)lane * 16, CombGeom<W>::bit((int)win), bx, by);
}

// phase 2: lane (b, win) -> L = (lo+1) B_i (CL points) and H = hi (CL B_i) (NH-1 points)
template <int W>
__global__ void __launch_bounds__(64) k_tab_small(const uint32_t* __restrict__ bases, uint32_t nb,
                                                  uint32_t* __restrict__ lbuf, uint32_t* __restrict__ hbuf,
                                                  fe* __restrict__ scratch) {
  using T = TabGeom<W>;
  constexpr int nwin = CombGeom<W>::kWin;
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= nb * nwin) return;
  fe* sc = scratch + (uint64_t)lane * T::SS;
  auto st = [&](int slot, const fe& v) { sc[slot] = v; };
  auto ld = [&](int slot, fe& v) { v = sc[slot]; };
  uint32_t bw[16];
  for (int i = 0; i < 16; ++i) bw[i] = bases[(uint64_t)lane * 16 + i];
  uint32_t* L = lbuf + (uint64_t)lane * T::CL * 16;
  multiples(L, T::CL, bw, st, ld);
  if (T::NH > 1) {
    uint32_t mw[16];
    for (int i = 0; i < 16; ++i) mw[i] = L[(uint64_t)(T::CL - 1) * 16 + i];
    multiples(hbuf + (uint64_t)lane * (T::NH - 1) * 16, T::NH - 1, mw, st, ld);
  }
}

// phase 3: lane (b, win, hi, part) -> PC entries idx = hi*CL + part*PC + j of base b's table.
// A launch covers global lanes [lane0, lane1); scratch is indexed by lane - lane0.
template <int W>
__global__ void __launch_bounds__(64) k_tab_entries(const uint32_t* __restrict__ lbuf,
                                                    const uint32_t* __restrict__ hbuf, uint64_t lane0,
                                                    uint64_t lane1, uint32_t* __restrict__ tables,
                                                    fe* __restrict__ scratch) {
  using T = TabGeom<W>;
  using G = CombGeom<W>;
  constexpr int parts = T::CL / T::PC;
  const uint64_t local = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t lane = lane0 + local;
  const uint64_t per_base = (uint64_t)G::kWin * T::NH * parts;
  if (lane >= lane1) return;
  const uint32_t b = (uint32_t)(lane / per_base);
  uint32_t rem = (uint32_t)(lane % per_base);
  const uint32_t win = rem / (T::NH * parts);
  rem %= T::NH * parts;
  const uint32_t hi = rem / parts, part = rem % parts;
  if ((uint64_t)hi * T::CL >= (uint64_t)G::ent((int)win)) return;  // narrow top window: half the entries
  const uint64_t bw = (uint64_t)b * G::kWin + win;  // (base, window) index into lbuf/hbuf
  const uint32_t* L = lbuf + (bw * T::CL + (uint64_t)part * T::PC) * 16;
  uint32_t hw[16] = {0};
  if (hi > 0)
    for (int i = 0; i < 16; ++i) hw[i] = hbuf[(bw * (T::NH - 1) + hi - 1) * 16 + i];
  uint32_t* out = tables + (uint64_t)b * G::kWords + (G::base((int)win) + (uint64_t)hi * T::CL +
                                                      (uint64_t)part * T::PC) * 16;
  fe* sc = scratch + local * 4 * T::PC;
  sums_chunk(out, T::PC, hi > 0, hw, L, [&](int slot, const fe& v) { sc[slot] = v; },
             [&](int slot, fe& v) { v = sc[slot]; });
}

template <int W>
hipError_t build_tables_w(const uint32_t* keys_le, uint32_t key0, uint32_t nb, int with_g, uint32_t* valid,
                          uint32_t* tables, TableScratch& sc, hipStream_t st) {
  using T = TabGeom<W>;
  using G = CombGeom<W>;
  if (nb == 0) return hipSuccess;
  const uint32_t lanes12 = nb * G::kWin;
  hipLaunchKernelGGL(k_tab_bases<W>, dim3((lanes12 + 63) / 64), dim3(64), 0, st, keys_le, key0, nb, with_g, valid,
                     reinterpret_cast<uint32_t*>(sc.bases));
  hipLaunchKernelGGL(k_tab_small<W>, dim3((lanes12 + 63) / 64), dim3(64), 0, st,
                     reinterpret_cast<const uint32_t*>(sc.bases), nb, reinterpret_cast<uint32_t*>(sc.lbuf),
                     reinterpret_cast<uint32_t*>(sc.hbuf), reinterpret_cast<fe*>(sc.small_scratch));
  // phase 3 in slices of sc.entry_lanes lanes (its scratch is per lane)
  constexpr uint64_t per_base = (uint64_t)G::kWin * T::NH * (T::CL / T::PC);
  const uint64_t total = (uint64_t)nb * per_base;
  for (uint64_t l0 = 0; l0 < total; l0 += sc.entry_lanes) {
    const uint64_t l1 = total - l0 < sc.entry_lanes ? total : l0 + sc.entry_lanes;
    hipLaunchKernelGGL(k_tab_entries<W>, dim3((uint32_t)((l1 - l0 + 63) / 64)), dim3(64), 0, st,
                       reinterpret_cast<const uint32_t*>(sc.lbuf), reinterpret_cast<const uint32_t*>(sc.hbuf), l0, l1,
                       tables, reinterpret_cast<fe*>(sc.entry_scratch));
  }
  return hipGetLastError();
}

TableScratchSizes table_scratch_sizes(int w, uint32_t nb) {
  TableScratchSizes z{};
  auto fill = [&](auto geom) {
    using G = decltype(geom);
    using T = TabGeom<G::kCode>;
    z.bases = (size_t)nb * G::kWin * 64;
    z.lbuf = (size_t)nb * G::kWin * T::CL * 64;
    z.hbuf = (size_t)nb * G::kWin * (T::NH > 1 ? T::NH - 1 : 1) * 64;
    z.small_scratch = (size_t)nb * G::kWin * T::SS * sizeof(fe);
    const uint64_t total = (uint64_t)G::kWin * T::NH * (T::CL / T::PC) * nb;
    const uint64_t cap = 1ull << 17;  // 128 Ki lanes x 9 KiB of scratch
    z.entry_lanes = total < cap ? total : cap;
    z.entry_scratch = (size_t)z.entry_lanes * 4 * T::PC * sizeof(fe);
  };
  switch (w) {
#define PBFTV_W(W) \
  case W: fill(CombGeom<W>()); break;
    PBFTV_TABLE_WIDTHS(PBFTV_W)
#undef PBFTV_W
    default: fill(CombGeom<24>()); break;
  }
  return z;
}

size_t table_bytes(int w) {
  switch (w) {
#define PBFTV_W(W) \
  case W: return CombGeom<W>::kBytes;
    PBFTV_TABLE_WIDTHS(PBFTV_W)
#undef PBFTV_W
    default: return 0;
  }
}

int table_windows(int w) {
  switch (w) {
#define PBFTV_W(W) \
  case W: return CombGeom<W>::kWin;
    PBFTV_TABLE_WIDTHS(PBFTV_W)
#undef PBFTV_W
    default: return 0;
  }
}

hipError_t launch_build_tables(int w, const uint32_t* keys_le, uint32_t key0, uint32_t nb, int with_g,
                               uint32_t* valid, uint32_t* tables, TableScratch& sc, hipStream_t st) {
  switch (w) {
#define PBFTV_W(W) \
  case W: return build_tables_w<W>(keys_le, key0, nb, with_g, valid, tables, sc, st);
    PBFTV_TABLE_WIDTHS(PBFTV_W)
#undef PBFTV_W
    default: return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------
// stage 1: scalars.  scal[i] = {u1[8], u2[8]} (LE words); flag[i] = 1 if the
// signature passes Go's range checks and names a valid registered key.
//
// Each lane owns K signatures i = lane + j*L (j < K, L = lanes in the grid, so
// every load/store is coalesced across the wave) and inverts all K values of s
// with ONE Fermat inversion (Montgomery's trick): prefix products
// c_j = s_0 ... s_j go to a limb-major scratch, inv = c_{K-1}^-1, then walking
// back w_j = inv * c_{j-1}, inv *= s_j.  Per signature that is 7 Montgomery
// multiplies + 292/K for the inversion instead of 292 + 4.
__device__ __forceinline__ bool sig_ok(const uint8_t* __restrict__ sigs, const uint32_t* __restrict__ key_idx,
                                       const uint32_t* __restrict__ key_valid, uint32_t nkeys, uint64_t i,
                                       uint32_t r[8], uint32_t s[8]) {
  const uint32_t k = key_idx[i];
  load_be256(sigs + 64 * i, r);
  load_be256(sigs + 64 * i + 32, s);
  if (!(k < nkeys && key_valid[k] != 0)) return false;
  if (words_is_zero(r) || words_is_zero(s)) return false;
  return words_lt(r, kN32) && words_lt(s, kN32);
}

template <int K>
__global__ void __launch_bounds__(256) k_ecdsa_scalars(const uint8_t* __restrict__ hashes,
                                                       const uint8_t* __restrict__ sigs,
                                                       const uint32_t* __restrict__ key_idx, uint64_t n,
                                                       const uint32_t* __restrict__ key_valid, uint32_t nkeys,
                                                       uint4* __restrict__ scal, uint8_t* __restrict__ flag,
                                                       uint32_t* __restrict__ prefix,
                                                       const uint32_t* __restrict__ perm) {
  // outputs at position i; inputs of signature src(i) = perm[i] in key order (k_key_*)
  auto src = [&](uint64_t i) -> uint64_t { return perm != nullptr ? (uint64_t)perm[i] : i; };
  const uint64_t L = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  fe r2n, acc;
  fe_set(r2n, kR2N);
  fe_set(acc, kOneN);
  uint32_t okm = 0;
  for (int j = 0; j < K; ++j) {
    const uint64_t i = lane + (uint64_t)j * L;
    uint32_t r[8], sw[8] = {1, 0, 0, 0, 0, 0, 0, 0};
    bool ok = false;
    if (i < n) {
      uint32_t s[8];
      ok = sig_ok(sigs, key_idx, key_valid, nkeys, src(i), r, s);
      if (ok) PBFTV_UNROLL for (int t = 0; t < 8; ++t) sw[t] = s[t];
    }
    fe sv, sm;
    fe_from_words(sv, sw);
    fn_mul(sm, sv, r2n);
    fn_mul(acc, acc, sm);
    if (K > 1)
      PBFTV_UNROLL for (int l = 0; l < 9; ++l) prefix[((uint64_t)j * 9 + l) * L + lane] = acc.v[l];
    okm |= (ok ? 1u : 0u) << j;
  }
  fe inv;
  fn_inv_mont_gcd(inv, acc);
  for (int j = K - 1; j >= 0; --j) {
    const uint64_t i = lane + (uint64_t)j * L;
    const bool ok = (okm >> j) & 1u;
    uint32_t r[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s[8] = {1, 0, 0, 0, 0, 0, 0, 0};
    const uint64_t si = ok ? src(i) : 0;
    if (ok) {
      load_be256(sigs + 64 * si, r);
      load_be256(sigs + 64 * si + 32, s);
    }
    fe w;
    if (K > 1 && j > 0) {
      fe pre;
      PBFTV_UNROLL for (int l = 0; l < 9; ++l) pre.v[l] = prefix[((uint64_t)(j - 1) * 9 + l) * L + lane];
      fn_mul(w, inv, pre);
      fe sv, sm;
      fe_from_words(sv, s);
      fn_mul(sm, sv, r2n);
      fn_mul(inv, inv, sm);
    } else {
      w = inv;
    }
    if (i < n) {
      uint32_t u1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, u2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (ok) {
        uint32_t e[8];
        load_be256(hashes + 32 * si, e);
        fe ev, rv, t;
        fe_from_words(ev, e);
        fe_from_words(rv, r);
        fn_mul(t, ev, w);  // e * s^-1 (e < 2^256 < 2n: the Montgomery product is < 2n)
        fn_canon(t, t);
        fe_to_words(u1, t);
        fn_mul(t, rv, w);
        fn_canon(t, t);
        fe_to_words(u2, t);
      }
      uint4* o = scal + 4 * i;
      o[0] = make_uint4(u1[0], u1[1], u1[2], u1[3]);
      o[1] = make_uint4(u1[4], u1[5], u1[6], u1[7]);
      o[2] = make_uint4(u2[0], u2[1], u2[2], u2[3]);
      o[3] = make_uint4(u2[4], u2[5], u2[6], u2[7]);
      flag[i] = ok ? 1 : 0;
    }
  }
}

// ---------------------------------------------------------------------------
// stage 2: joint comb.  Signed W-bit digits are peeled off a 256-bit register
// shift (no runtime-indexed register arrays -> no scratch), and the two table
// entries of window i+1 are loaded while window i is being added.
template <int W>
struct digit_stream {
  uint32_t w[8];
  int carry;
  int k = 0;  // next window (its width differs only in the mixed geometries)
  __device__ __forceinline__ int next() {
    const int wd = CombGeom<W>::width(k++);
    const int b = (int)(w[0] & ((1u << wd) - 1u));
    PBFTV_UNROLL for (int j = 0; j < 7; ++j) w[j] = __builtin_amdgcn_alignbit(w[j + 1], w[j], wd);
    w[7] >>= wd;
    const int d = b + carry;
    carry = d > (1 << (wd - 1)) ? 1 : 0;
    return d - (carry << wd);
  }
};

template <int W>
__device__ __forceinline__ void load_entry(const uint4* __restrict__ tab, int win, int d, uint4 e[4]) {
  const int idx = (d < 0 ? -d : d) - 1;
#ifdef PBFTV_EXP_L2TAB  // timing experiment only: lookups confined to 4 MiB per window (results wrong)
  const uint4* p = tab + (CombGeom<W>::base(win) + (idx < 0 ? 0 : idx & 0xFFFF)) * 4;
#else
  const uint4* p = tab + (CombGeom<W>::base(win) + (idx < 0 ? 0 : idx)) * 4;
#endif
  e[0] = p[0]; e[1] = p[1]; e[2] = p[2]; e[3] = p[3];
}

__device__ __forceinline__ void entry_words(const uint4 e[4], uint32_t ew[16]) {
  PBFTV_UNROLL for (int q = 0; q < 4; ++q) {
    ew[4 * q] = e[q].x; ew[4 * q + 1] = e[q].y; ew[4 * q + 2] = e[q].z; ew[4 * q + 3] = e[q].w;
  }
}

// Acc = xyzz: the unchecked fast pass (comb_add_entry_xyzz); Acc = jac with
// kCheck: the complete-addition rerun (comb_add_entry<true>).
template <bool kCheck, class Acc>
__device__ __forceinline__ void comb_dev_add(Acc& acc, bool& inf, int d, const uint32_t ew[16]) {
  if constexpr (kCheck) comb_add_entry<true>(acc, inf, d, ew);
  else comb_add_entry_xyzz(acc, inf, d, ew);
}

template <bool kCheck, int WG, int WQ, class Acc>
__device__ bool comb2_dev_pass(Acc& acc, const uint32_t u1[8], const uint32_t u2[8],
                               const uint4* __restrict__ gtab, const uint4* __restrict__ qtab) {
  constexpr int nG = CombGeom<WG>::kWin, nQ = CombGeom<WQ>::kWin;
  constexpr int nW = nG > nQ ? nG : nQ;
  digit_stream<WG> s1;
  digit_stream<WQ> s2;
  PBFTV_UNROLL for (int j = 0; j < 8; ++j) { s1.w[j] = u1[j]; s2.w[j] = u2[j]; }
  s1.carry = s2.carry = 0;
  int d1 = s1.next(), d2 = s2.next();
  uint4 eg[4], eq[4];
  load_entry<WG>(gtab, 0, d1, eg);
  load_entry<WQ>(qtab, 0, d2, eq);
  bool inf = true;
  for (int i = 0; i < nW; ++i) {
    const int c1 = i < nG ? d1 : 0, c2 = i < nQ ? d2 : 0;
    uint32_t wg[16], wq[16];
    entry_words(eg, wg);
    entry_words(eq, wq);
    if (i + 1 < nG) {
      d1 = s1.next();
      load_entry<WG>(gtab, i + 1, d1, eg);
    }
    if (i + 1 < nQ) {
      d2 = s2.next();
      load_entry<WQ>(qtab, i + 1, d2, eq);
    }
    if (c1 != 0) comb_dev_add<kCheck>(acc, inf, c1, wg);
    if (c2 != 0) comb_dev_add<kCheck>(acc, inf, c2, wq);
  }
  return !inf;
}

// The complete-addition rerun is a real call so its registers do not
// inflate the fast path's allocation (it runs only for exceptional lanes).
// It re-reads its inputs from memory and returns only the accept bit: no
// local object's address crosses the call, so the fast path's accumulator
// stays in registers (a jac passed by reference would live in scratch and
// cost a 108-byte store + load per addition).
template <int WG, int WQ>
__device__ __noinline__ bool comb2_checked_verify(const uint4* __restrict__ sp, const uint8_t* __restrict__ sig,
                                                  const uint4* __restrict__ gtab, const uint4* __restrict__ qtab) {
  const uint4 a = sp[0], b = sp[1], c = sp[2], dd = sp[3];
  const uint32_t u1[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  const uint32_t u2[8] = {c.x, c.y, c.z, c.w, dd.x, dd.y, dd.z, dd.w};
  jac R;
  const bool fin = comb2_dev_pass<true, WG, WQ>(R, u1, u2, gtab, qtab);
  uint32_t r[8];
  load_be256(sig, r);
  return ecdsa_check(R, fin, r);
}

// Joint comb schedule: step j of the nG + nQ additions takes the G entry of
// window j/2 (j even) and the Q entry (j odd) while both tables have windows
// left, then the longer table's remaining windows.
template <int WG, int WQ>
struct CombSteps {
  static constexpr int nG = CombGeom<WG>::kWin, nQ = CombGeom<WQ>::kWin;
  static constexpr int nMin = nG < nQ ? nG : nQ;
  static constexpr int nD = nG + nQ;
  // LDS digit storage: d - 1 fits int16 for W <= 16 (d in [-(2^15 - 1), 2^15])
  using Digit = std::conditional_t<(CombGeom<WG>::kW > 16 || CombGeom<WQ>::kW > 16), int, short>;
  __host__ __device__ static constexpr bool is_q(int j) { return j < 2 * nMin ? (j & 1) != 0 : nQ > nG; }
  __host__ __device__ static constexpr int win(int j) { return j < 2 * nMin ? j >> 1 : j - nMin; }
};

// y = d < 0 ? 2p - y : y, lazily (limbs < 2^30: a valid fe_mul input) -- a
// per-lane mask select, no carry chain and no divergence.
__device__ __forceinline__ void fe_cneg_lazy(fe& y, bool neg) {
  const uint32_t m = 0u - (uint32_t)neg;
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) y.v[l] = y.v[l] ^ ((y.v[l] ^ (kP2Borrow[l] - y.v[l])) & m);
}

template <int W>
__device__ __forceinline__ const uint4* entry_ptr(const uint4* __restrict__ tab, int win, int d) {
  const int idx = (d < 0 ? -d : d) - 1;
#ifdef PBFTV_EXP_SMALLTAB  // timing experiment only: 256 KiB footprint per table (results wrong)
  return tab + (uint64_t)(idx < 0 ? 0 : idx & 0xFFF) * 4;
#else
  return tab + (CombGeom<W>::base(win) + (idx < 0 ? 0 : idx)) * 4;
#endif
}

// Async copy of this lane's 64-B entry into sent[.][t]: four 16-B
// global_load_lds, each writing the wave's 64 lanes contiguously at the
// wave-uniform base &sent[k][t & ~63].
__device__ __forceinline__ void issue_entry_lds(uint4 (*sent)[256], uint32_t t, const uint4* p) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this lane's reads of the slot are done
  const uint32_t wb = t & ~63u;
  __builtin_amdgcn_global_load_lds(p + 0, &sent[0][wb], 16, 0, 0);
  __builtin_amdgcn_global_load_lds(p + 1, &sent[1][wb], 16, 0, 0);
  __builtin_amdgcn_global_load_lds(p + 2, &sent[2][wb], 16, 0, 0);
  __builtin_amdgcn_global_load_lds(p + 3, &sent[3][wb], 16, 0, 0);
}

__device__ __forceinline__ void read_entry_lds(uint4 (*sent)[256], uint32_t t, uint32_t ew[16]) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's copies have landed
  uint4 e[4];
  PBFTV_UNROLL for (int k = 0; k < 4; ++k) e[k] = sent[k][t];
  entry_words(e, ew);
}

template <int WG, int WQ>
__global__ void __launch_bounds__(256, PBFTV_COMB_WAVES) k_ecdsa_comb(const uint4* __restrict__ scal, const uint8_t* __restrict__ flag,
                                                       const uint8_t* __restrict__ sigs,
                                                       const uint32_t* __restrict__ key_idx, uint64_t n,
                                                       const uint4* __restrict__ gtab,
                                                       const uint4* __restrict__ qtabs,
                                                       uint8_t* __restrict__ bitmap,
                                                       const uint32_t* __restrict__ perm,
                                                       uint8_t* __restrict__ okb) {
  using S = CombSteps<WG, WQ>;
  // signed digits of u1 / u2 in step order, one column per thread: recoded once
  // in the prologue so the main loop holds no 256-bit digit shift registers
  __shared__ typename S::Digit sdig[S::nD][256];
  // the table entry of the next step, streamed global -> LDS (no VGPRs held
  // while it is in flight): piece k of thread t at sent[k][t]
  __shared__ uint4 sent[4][256];
  const uint32_t t = threadIdx.x;
  // lane position p; with a key order (k_key_*), p is the p-th signature by key
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + t;
  const uint64_t i = perm != nullptr && p < n ? (uint64_t)perm[p] : p;
  const bool active = p < n && flag[p];  // stage 1 wrote scal/flag in the same (key) order
  bool ok = false;
  if (active) {
    const uint4* sp = scal + 4 * p;
    {
      const uint4 a = sp[0], b = sp[1], c = sp[2], dd = sp[3];
      digit_stream<WG> s1;
      digit_stream<WQ> s2;
      s1.w[0] = a.x; s1.w[1] = a.y; s1.w[2] = a.z; s1.w[3] = a.w;
      s1.w[4] = b.x; s1.w[5] = b.y; s1.w[6] = b.z; s1.w[7] = b.w;
      s2.w[0] = c.x; s2.w[1] = c.y; s2.w[2] = c.z; s2.w[3] = c.w;
      s2.w[4] = dd.x; s2.w[5] = dd.y; s2.w[6] = dd.z; s2.w[7] = dd.w;
      s1.carry = s2.carry = 0;
      PBFTV_UNROLL for (int j = 0; j < S::nD; ++j)
        sdig[j][t] = (typename S::Digit)((S::is_q(j) ? s2.next() : s1.next()) - 1);
    }
#ifdef PBFTV_EXP_SMALLTAB
    const uint4* qtab = qtabs;
#else
    const uint4* qtab = qtabs + (uint64_t)key_idx[i] * (CombGeom<WQ>::kWords / 4);
#endif
    xyzz R;
    bool inf = true;
    int d = (int)sdig[0][t] + 1;
    issue_entry_lds(sent, t, entry_ptr<WG>(gtab, 0, d));
#pragma unroll 1
#ifdef PBFTV_EXP_NOLOOP  // timing experiment only: prologue + epilogue without the comb (results wrong)
    for (int j = 0; j < 1; ++j) {
#else
    for (int j = 0; j < S::nD; ++j) {
#endif
      uint32_t w16[16];
      read_entry_lds(sent, t, w16);
      const int dc = d;
      if (j + 1 < S::nD) {  // next step's entry streams into LDS during this addition
        d = (int)sdig[j + 1][t] + 1;
        issue_entry_lds(sent, t, S::is_q(j + 1) ? entry_ptr<WQ>(qtab, S::win(j + 1), d)
                                                : entry_ptr<WG>(gtab, S::win(j + 1), d));
      }
      if (dc != 0) {
        fe x, y;
        entry_to_fe(x, y, w16);
        fe_cneg_lazy(y, dc < 0);
        if (inf) {
          R.x = x;
          fe_norm(R.y, y);
          fe_set(R.zz, kOneP);
          fe_set(R.zzz, kOneP);
          inf = false;
        } else {
#ifdef PBFTV_EXP_NOMADD  // timing experiment only: memory path without the additions (results wrong)
          PBFTV_UNROLL for (int l = 0; l < 9; ++l) { R.x.v[l] ^= x.v[l]; R.y.v[l] += y.v[l]; }
#else
          xyzz_madd(R, x, y);
#endif
        }
      }
    }
    if (!inf && fe_is_zero(R.zz)) {
      ok = comb2_checked_verify<WG, WQ>(sp, sigs + 64 * i, gtab, qtab);  // exceptional step: redo
    } else {
      uint32_t r[8];
      load_be256(sigs + 64 * i, r);
      ok = ecdsa_check(R, !inf, r);
    }
  }
  if (perm != nullptr) {  // key order: one byte per signature, k_pack_bits builds the bitmap
    if (p < n) okb[i] = ok ? 1 : 0;
    return;
  }
  // LSB-first bitmap: wave ballot, lanes 0..7 store one byte each
  const unsigned long long m = __ballot(ok);
  const uint32_t lane = t & 63u;
  const uint64_t wave_base = p - lane;
  if (lane < 8 && wave_base + 8 * lane < n) bitmap[(wave_base >> 3) + lane] = (uint8_t)(m >> (8 * lane));
}

// ---------------------------------------------------------------------------
// Key order for the comb (stage 0).  The key tables are looked up at random
// entries; when the 64 lanes of a wave name ~50 different keys (a random
// 100-key batch) every wave-wide table load touches ~50 tables, when they
// share a key the lookups fall in one table window like the G lookups do.
// Same-box A/B at 1M signatures / 100 keys (bench.py PBFTV_EXP_SORT_KEYS): comb
// 1.345 ms in arrival order, 1.237 ms key-sorted.  A counting sort in three
// small launches: per-block key histograms in LDS added into per-key totals ->
// exclusive scan of the totals -> each block claims its range of every key
// with one atomic per (block, key) and scatters through LDS cursors.  Not
// stable (the order inside a key does not matter: results go back to the
// signature's own index).
__device__ __forceinline__ void block_key_hist(uint32_t* h, const uint32_t* __restrict__ key_idx, uint64_t n,
                                               uint32_t nkeys) {
  const uint32_t nb = nkeys + 1;  // bin nkeys: out-of-range key indices (rejected later)
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const uint64_t chunk = (n + gridDim.x - 1) / gridDim.x, lo = (uint64_t)blockIdx.x * chunk;
  const uint64_t hi = lo + chunk < n ? lo + chunk : n;
  for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const uint32_t k = key_idx[i];
    atomicAdd(&h[k < nkeys ? k : nkeys], 1u);
  }
  __syncthreads();
}

__global__ void __launch_bounds__(256) k_key_hist(const uint32_t* __restrict__ key_idx, uint64_t n, uint32_t nkeys,
                                                  uint32_t* __restrict__ total) {
  __shared__ uint32_t h[kSortMaxKeys + 1];
  block_key_hist(h, key_idx, n, nkeys);
  for (uint32_t b = threadIdx.x; b <= nkeys; b += blockDim.x)
    if (h[b]) atomicAdd(&total[b], h[b]);
}

// exclusive scan of the m <= 2048 totals in place: one block, two per thread
__global__ void __launch_bounds__(1024) k_key_scan(uint32_t* __restrict__ total, uint32_t m) {
  __shared__ uint32_t s[1024];
  const uint32_t t = threadIdx.x;
  const uint32_t a = 2 * t < m ? total[2 * t] : 0u, b = 2 * t + 1 < m ? total[2 * t + 1] : 0u;
  s[t] = a + b;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {
    const uint32_t v = t >= off ? s[t - off] : 0u;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  const uint32_t excl = s[t] - a - b;
  if (2 * t < m) total[2 * t] = excl;
  if (2 * t + 1 < m) total[2 * t + 1] = excl + a;
}

__global__ void __launch_bounds__(256) k_key_scatter(const uint32_t* __restrict__ key_idx, uint64_t n, uint32_t nkeys,
                                                     uint32_t* __restrict__ start, uint32_t* __restrict__ perm) {
  __shared__ uint32_t h[kSortMaxKeys + 1];
  block_key_hist(h, key_idx, n, nkeys);
  for (uint32_t b = threadIdx.x; b <= nkeys; b += blockDim.x)
    if (h[b]) h[b] = atomicAdd(&start[b], h[b]);  // this block's range of key b
  __syncthreads();
  const uint64_t chunk = (n + gridDim.x - 1) / gridDim.x, lo = (uint64_t)blockIdx.x * chunk;
  const uint64_t hi = lo + chunk < n ? lo + chunk : n;
  for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const uint32_t k = key_idx[i];
    perm[atomicAdd(&h[k < nkeys ? k : nkeys], 1u)] = (uint32_t)i;
  }
}

// LSB-first bitmap from one byte per signature
__global__ void __launch_bounds__(256) k_pack_bits(const uint8_t* __restrict__ okb, uint64_t n,
                                                   uint8_t* __restrict__ bitmap) {
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (8 * b >= n) return;
  uint32_t v = 0;
  if (8 * b + 8 <= n) {
    const uint2 w = *reinterpret_cast<const uint2*>(okb + 8 * b);
    PBFTV_UNROLL for (int k = 0; k < 4; ++k) v |= ((w.x >> (8 * k)) & 1u) << k;
    PBFTV_UNROLL for (int k = 0; k < 4; ++k) v |= ((w.y >> (8 * k)) & 1u) << (4 + k);
  } else {
    for (uint64_t k = 0; 8 * b + k < n; ++k) v |= (okb[8 * b + k] ? 1u : 0u) << k;
  }
  bitmap[b] = (uint8_t)v;
}

bool key_sort_wanted(uint64_t n, uint32_t nkeys) {
  if (const char* e = getenv("PBFTV_KEY_SORT")) {
    if (e[0] == '0') return false;
    if (e[0] == '1') return nkeys <= kSortMaxKeys && n < (1ull << 32);
  }
  return nkeys > 8 && nkeys <= kSortMaxKeys && n >= 32768 && n < (1ull << 32);
}

size_t key_sort_scratch_bytes(uint64_t n, uint32_t nkeys) { return (size_t)n * 4 + (size_t)(nkeys + 1) * 4; }

hipError_t launch_key_sort(const uint32_t* key_idx, uint64_t n, uint32_t nkeys, void* scratch, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (nkeys > kSortMaxKeys) return hipErrorInvalidValue;
  uint32_t* perm = reinterpret_cast<uint32_t*>(scratch);
  uint32_t* total = perm + n;
  hipError_t e = hipMemsetAsync(total, 0, (size_t)(nkeys + 1) * 4, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_key_hist, dim3(kSortBlocks), dim3(256), 0, st, key_idx, n, nkeys, total);
  hipLaunchKernelGGL(k_key_scan, dim3(1), dim3(1024), 0, st, total, nkeys + 1);
  hipLaunchKernelGGL(k_key_scatter, dim3(kSortBlocks), dim3(256), 0, st, key_idx, n, nkeys, total, perm);
  return hipGetLastError();
}

hipError_t launch_pack_bits(const uint8_t* okb, uint64_t n, uint8_t* bitmap, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const uint64_t bytes = (n + 7) / 8;
  hipLaunchKernelGGL(k_pack_bits, dim3((uint32_t)((bytes + 255) / 256)), dim3(256), 0, st, okb, n, bitmap);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Latency path (small batches: a quorum certificate): ONE WAVE PER SIGNATURE.
// The throughput kernels above run one signature per lane, so a lone
// certificate is a single wave walking a 292-multiply inversion chain and 34
// dependent mixed additions -- the whole latency is one wave's serial
// instruction stream.  Here the wave splits that stream:
//   * every lane computes the scalars redundantly (Go's range checks, then
//     w = s^-1 by safegcd divsteps -- ~5x fewer dependent multiplies than
//     Fermat -- u1 = e w, u2 = r w);
//   * quad q (lanes 4q..4q+3) takes window q: the G entry of digit q of u1
//     plus the Q entry of digit q of u2, then a butterfly over the quads
//     sums the windows (ceil(log2(windows)) Jacobian additions); the four
//     lanes of a quad split each addition's multiplications (wave_sum_quads);
//   * every lane does the x-coordinate check; lane 0 reports it.
// One 64-thread block per signature, so the waves spread over every SIMD.
__device__ __forceinline__ void shfl_xor_fe(fe& dst, const fe& src, int m) {
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) dst.v[l] = (uint32_t)__shfl_xor((int)src.v[l], m, 64);
}

// r = p + q, complete: infinity flags, doubling and cancellation handled.
__device__ __forceinline__ void jac_add_complete(jac& r, bool& rinf, const jac& p, bool pinf, const jac& q,
                                                 bool qinf) {
  if (pinf || qinf) {
    r = pinf ? q : p;
    rinf = pinf && qinf;
    return;
  }
  jac s;
  const int st = jac_add(s, p, q);
  if (st == 1) {
    jac_double(r, p);
    rinf = false;
  } else {
    r = s;
    rinf = st == 2;
  }
}

// lane-per-window schedule (any window count): lane j adds its two entries
// with complete formulas, then a butterfly of complete additions.  Used when
// the windows outnumber the quads, and as the exact fallback of the quad
// schedule below.
template <int WG, int WQ>
__device__ __forceinline__ void wave_sum_lanes(jac& P, bool& inf, const uint32_t u1[8], const uint32_t u2[8],
                                               const uint4* __restrict__ gtab, const uint4* __restrict__ qtab) {
  constexpr int nG = CombGeom<WG>::kWin, nQ = CombGeom<WQ>::kWin;
  constexpr int nW = nG > nQ ? nG : nQ;
  const int j = threadIdx.x;
  digit_stream<WG> s1;
  digit_stream<WQ> s2;
  PBFTV_UNROLL for (int k = 0; k < 8; ++k) { s1.w[k] = u1[k]; s2.w[k] = u2[k]; }
  s1.carry = s2.carry = 0;
  int d1 = 0, d2 = 0;
  for (int k = 0; k < nW; ++k) {
    const int a = k < nG ? s1.next() : 0, b = k < nQ ? s2.next() : 0;
    if (k == j) { d1 = a; d2 = b; }
  }
  inf = true;
  if (d1 != 0) {
    uint4 eg[4];
    uint32_t w16[16];
    load_entry<WG>(gtab, j, d1, eg);
    entry_words(eg, w16);
    comb_add_entry<true>(P, inf, d1, w16);
  }
  if (d2 != 0) {
    uint4 eq[4];
    uint32_t w16[16];
    load_entry<WQ>(qtab, j, d2, eq);
    entry_words(eq, w16);
    comb_add_entry<true>(P, inf, d2, w16);
  }
#pragma unroll 1
  for (int m = 1; m < nW; m <<= 1) {
    jac Q;
    shfl_xor_fe(Q.x, P.x, m);
    shfl_xor_fe(Q.y, P.y, m);
    shfl_xor_fe(Q.z, P.z, m);
    const bool qinf = __shfl_xor((int)inf, m, 64) != 0;
    jac S;
    bool sinf;
    jac_add_complete(S, sinf, P, inf, Q, qinf);
    P = S;
    inf = sinf;
  }
}

// ---- quad schedule: the four lanes of a quad share one point addition ------
// Each step every lane of the quad does ONE field multiplication on operands
// picked by its role (lane & 3), and the products are broadcast inside the
// quad with DPP quad_perm moves (plain VALU, no LDS).  A Jacobian addition
// (add-2008-s: 12M + 2S) becomes 4 multiplication steps, the affine + affine
// first level 3 steps.
template <int K>
__device__ __forceinline__ void quad_bcast(fe& d, const fe& s) {
  PBFTV_UNROLL for (int l = 0; l < 9; ++l)
    d.v[l] = (uint32_t)__builtin_amdgcn_mov_dpp((int)s.v[l], K * 0x55, 0xF, 0xF, false);
}

// Value selects by masks: a ?: between loads of two objects is turned into a
// load through a selected pointer, which forces the objects into scratch.
__device__ __forceinline__ uint32_t mask_of(bool c) { return 0u - (uint32_t)c; }

__device__ __forceinline__ void quad_sel(fe& d, int role, const fe& a0, const fe& a1, const fe& a2, const fe& a3) {
  const uint32_t m0 = mask_of(role == 0), m1 = mask_of(role == 1), m2 = mask_of(role == 2), m3 = mask_of(role == 3);
  PBFTV_UNROLL for (int l = 0; l < 9; ++l)
    d.v[l] = (a0.v[l] & m0) | (a1.v[l] & m1) | (a2.v[l] & m2) | (a3.v[l] & m3);
}

// d = c0 ? a : c1 ? b : c   (masks, see above)
__device__ __forceinline__ void fe_sel3(fe& d, bool c0, const fe& a, bool c1, const fe& b, const fe& c) {
  const uint32_t ma = mask_of(c0), mb = mask_of(!c0 && c1), mc = mask_of(!c0 && !c1);
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) d.v[l] = (a.v[l] & ma) | (b.v[l] & mb) | (c.v[l] & mc);
}

// product of the role's operand pair
__device__ __forceinline__ void quad_mul(fe& p, int role, const fe& a0, const fe& b0, const fe& a1, const fe& b1,
                                         const fe& a2, const fe& b2, const fe& a3, const fe& b3) {
  fe a, b;
  quad_sel(a, role, a0, a1, a2, a3);
  quad_sel(b, role, b0, b1, b2, b3);
  fe_mul(p, a, b);
}

// (gx, gy) + (qx, qy), both affine, into XYZZ (mmadd-2008-s, 3 steps); exc if
// the x-coordinates meet.
__device__ __forceinline__ void quad_mmadd_xyzz(xyzz& r, bool& exc, int role, const fe& gx, const fe& gy,
                                                const fe& qx, const fe& qy) {
  fe p, rr, pp, r2, ppp, qq, x3, t, a, b, prod;
  fe_sub(p, qx, gx);
  fe_sub(rr, qy, gy);
  exc = fe_is_zero(p);
  quad_mul(prod, role, p, p, rr, rr, p, p, rr, rr);          // PP, R^2
  quad_bcast<0>(pp, prod);
  quad_bcast<1>(r2, prod);
  quad_mul(prod, role, p, pp, gx, pp, p, pp, gx, pp);        // PPP, Q = X1 PP
  quad_bcast<0>(ppp, prod);
  quad_bcast<1>(qq, prod);
  fe_add(t, ppp, qq);
  fe_add(t, t, qq);
  fe_sub(x3, r2, t);                                         // X3 = R^2 - PPP - 2Q
  fe_sub(t, qq, x3);
  quad_mul(prod, role, rr, t, gy, ppp, rr, t, gy, ppp);      // R (Q - X3), Y1 PPP
  quad_bcast<0>(a, prod);
  quad_bcast<1>(b, prod);
  fe_sub(r.y, a, b);
  r.x = x3;
  r.zz = pp;
  r.zzz = ppp;
}

// r = P + Q (both finite XYZZ), add-2008-s in 4 steps of <= 4 products (the
// Jacobian quad_jadd needs 5); exc if the x-coordinates meet (P == 0).
__device__ __forceinline__ void quad_xyzz_add(xyzz& r, bool& exc, int role, const xyzz& P, const xyzz& Q) {
  fe prod, u1, u2, s1, s2, p, rr, pp, r2, zz12, zzz12, ppp, qq, x3, t, a, b;
  quad_mul(prod, role, P.x, Q.zz, Q.x, P.zz, P.y, Q.zzz, Q.y, P.zzz);      // U1, U2, S1, S2
  quad_bcast<0>(u1, prod);
  quad_bcast<1>(u2, prod);
  quad_bcast<2>(s1, prod);
  quad_bcast<3>(s2, prod);
  fe_sub(p, u2, u1);
  fe_sub(rr, s2, s1);
  exc = fe_is_zero(p);
  quad_mul(prod, role, p, p, rr, rr, P.zz, Q.zz, P.zzz, Q.zzz);             // PP, R^2, ZZ1 ZZ2, ZZZ1 ZZZ2
  quad_bcast<0>(pp, prod);
  quad_bcast<1>(r2, prod);
  quad_bcast<2>(zz12, prod);
  quad_bcast<3>(zzz12, prod);
  quad_mul(prod, role, p, pp, u1, pp, zz12, pp, zz12, pp);                  // PPP, Q = U1 PP, ZZ3
  quad_bcast<0>(ppp, prod);
  quad_bcast<1>(qq, prod);
  quad_bcast<2>(r.zz, prod);
  fe_add(t, ppp, qq);
  fe_add(t, t, qq);
  fe_sub(x3, r2, t);                                                        // X3 = R^2 - PPP - 2Q
  fe_sub(t, qq, x3);
  quad_mul(prod, role, rr, t, s1, ppp, zzz12, ppp, zzz12, ppp);             // R (Q - X3), S1 PPP, ZZZ3
  quad_bcast<0>(a, prod);
  quad_bcast<1>(b, prod);
  quad_bcast<2>(r.zzz, prod);
  fe_sub(r.y, a, b);                                                        // Y3 = R (Q - X3) - S1 PPP
  r.x = x3;
}

// quad q = window q: G entry + Q entry, then a butterfly over the quads.
// exc reports a doubling / cancellation anywhere (the caller reruns the
// signature with wave_sum_lanes).
template <int WG, int WQ>
__device__ __forceinline__ void wave_sum_quads(xyzz& P, bool& inf, bool& exc, const uint32_t u1[8],
                                               const uint32_t u2[8], const uint4* __restrict__ gtab,
                                               const uint4* __restrict__ qtab) {
  constexpr int nG = CombGeom<WG>::kWin, nQ = CombGeom<WQ>::kWin;
  constexpr int nW = nG > nQ ? nG : nQ;
  static_assert(nW <= 16, "one quad per window");
  const int role = threadIdx.x & 3, q = threadIdx.x >> 2;
  digit_stream<WG> s1;
  digit_stream<WQ> s2;
  PBFTV_UNROLL for (int k = 0; k < 8; ++k) { s1.w[k] = u1[k]; s2.w[k] = u2[k]; }
  s1.carry = s2.carry = 0;
  int d1 = 0, d2 = 0;
  for (int k = 0; k < nW; ++k) {
    const int a = k < nG ? s1.next() : 0, b = k < nQ ? s2.next() : 0;
    if (k == q) { d1 = a; d2 = b; }
  }
  uint4 eg[4], eq[4];
  uint32_t w16[16];
  load_entry<WG>(gtab, q < nG ? q : 0, d1, eg);
  load_entry<WQ>(qtab, q < nQ ? q : 0, d2, eq);
  fe gx, gy, qx, qy, ny;
  entry_words(eg, w16);
  entry_to_fe(gx, gy, w16);
  if (d1 < 0) {
    fe_neg_lazy(ny, gy);
    fe_norm(gy, ny);
  }
  entry_words(eq, w16);
  entry_to_fe(qx, qy, w16);
  if (d2 < 0) {
    fe_neg_lazy(ny, qy);
    fe_norm(qy, ny);
  }
  xyzz S;
  bool e0;
  quad_mmadd_xyzz(S, e0, role, gx, gy, qx, qy);       // every quad runs it; selected below
  exc = d1 != 0 && d2 != 0 && e0;
  inf = d1 == 0 && d2 == 0;
  const bool both = d1 != 0 && d2 != 0, g_only = d1 != 0;
  fe one;
  fe_set(one, kOneP);
  fe_sel3(P.x, both, S.x, g_only, gx, qx);
  fe_sel3(P.y, both, S.y, g_only, gy, qy);
  fe_sel3(P.zz, both, S.zz, true, one, one);
  fe_sel3(P.zzz, both, S.zzz, true, one, one);
#pragma unroll 1
  for (int m = 1; m < nW; m <<= 1) {
    xyzz Q;
    shfl_xor_fe(Q.x, P.x, 4 * m);
    shfl_xor_fe(Q.y, P.y, 4 * m);
    shfl_xor_fe(Q.zz, P.zz, 4 * m);
    shfl_xor_fe(Q.zzz, P.zzz, 4 * m);
    const bool qinf = __shfl_xor((int)inf, 4 * m, 64) != 0;
    bool e;
    quad_xyzz_add(S, e, role, P, Q);
    exc = exc || (e && !inf && !qinf);
    fe_sel3(P.x, inf, Q.x, qinf, P.x, S.x);
    fe_sel3(P.y, inf, Q.y, qinf, P.y, S.y);
    fe_sel3(P.zz, inf, Q.zz, qinf, P.zz, S.zz);
    fe_sel3(P.zzz, inf, Q.zzz, qinf, P.zzz, S.zzz);
    inf = inf && qinf;
  }
}

// ecdsa_scalars with the inversion fed the plain s (no Montgomery round trip
// in front of it): w = s^-1 -> w R -> u1 = e w, u2 = r w (two independent
// products) -- one dependent Montgomery product fewer on the latency path.
__device__ __forceinline__ void ecdsa_scalars_plain_inv(const uint32_t e[8], const uint32_t r[8], const uint32_t s[8],
                                                        uint32_t u1[8], uint32_t u2[8]) {
  uint32_t iw[8];
  inv_mod_n_words(iw, s);  // 0 < s < n checked by sig_ok
  fe inv, r2n, w, ev, rv, t1, t2;
  fe_from_words(inv, iw);
  fe_set(r2n, kR2N);
  fn_mul(w, inv, r2n);     // s^-1 R
  fe_from_words(ev, e);
  fe_from_words(rv, r);
  fn_mul(t1, ev, w);       // e s^-1 (e < 2^256 < 2n)
  fn_mul(t2, rv, w);
  fn_canon(t1, t1);
  fn_canon(t2, t2);
  fe_to_words(u1, t1);
  fe_to_words(u2, t2);
}

template <int WG, int WQ>
__global__ void __launch_bounds__(64) k_ecdsa_wave(const uint8_t* __restrict__ hashes,
                                                   const uint8_t* __restrict__ sigs,
                                                   const uint32_t* __restrict__ key_idx, uint64_t n,
                                                   const uint32_t* __restrict__ key_valid, uint32_t nkeys,
                                                   const uint4* __restrict__ gtab, const uint4* __restrict__ qtabs,
                                                   uint8_t* __restrict__ bitmap, uint8_t* __restrict__ okbytes) {
  constexpr int nG = CombGeom<WG>::kWin, nQ = CombGeom<WQ>::kWin;
  constexpr int nW = nG > nQ ? nG : nQ;
  static_assert(nW <= 64, "one lane per window");
  const int j = threadIdx.x;
  const uint64_t i = blockIdx.x;
  bool ok = false;
  uint32_t r[8], s[8], e[8];
  load_be256(hashes + 32 * i, e);  // issued with sig_ok's loads: one round trip to the (host) inputs
  if (sig_ok(sigs, key_idx, key_valid, nkeys, i, r, s)) {  // wave-uniform branch
    uint32_t u1[8], u2[8];
    ecdsa_scalars_plain_inv(e, r, s, u1, u2);
    const uint4* qtab = qtabs + (uint64_t)key_idx[i] * (CombGeom<WQ>::kWords / 4);
    bool inf;
    bool exc = true;
    if constexpr (nW <= 16) {
      xyzz P;
      wave_sum_quads<WG, WQ>(P, inf, exc, u1, u2, gtab, qtab);
      exc = __any(exc);
      if (!exc) ok = ecdsa_check(P, !inf, r);
    }
    if (exc) {  // windows outnumber the quads, or a doubling somewhere: exact lane-per-window rerun
      jac P;
      wave_sum_lanes<WG, WQ>(P, inf, u1, u2, gtab, qtab);
      ok = ecdsa_check(P, !inf, r);
    }
  }
  if (j != 0) return;
  if (okbytes) {
    okbytes[i] = ok ? 1 : 0;
    return;
  }
  // one bit of the LSB-first bitmap: set or clear it with a word atomic
  // (other signatures' waves share the byte; no pre-zeroing needed)
  uint8_t* byte = bitmap + (i >> 3);
  const uintptr_t a = reinterpret_cast<uintptr_t>(byte);
  unsigned int* word = reinterpret_cast<unsigned int*>(a & ~(uintptr_t)3);
  const unsigned int bit = 1u << (((unsigned)(a & 3) << 3) + (unsigned)(i & 7));
  if (ok) atomicOr(word, bit);
  else atomicAnd(word, ~bit);
}

template <int WG, int WQ>
static void launch_wave_w(const uint8_t* hashes, const uint8_t* sigs, const uint32_t* key_idx, uint64_t n,
                          const uint32_t* key_valid, uint32_t nkeys, const uint32_t* gtab, const uint32_t* qtabs,
                          uint8_t* bitmap, uint8_t* okbytes, hipStream_t st) {
  hipLaunchKernelGGL((k_ecdsa_wave<WG, WQ>), dim3((uint32_t)n), dim3(64), 0, st, hashes, sigs, key_idx, n, key_valid,
                     nkeys, reinterpret_cast<const uint4*>(gtab), reinterpret_cast<const uint4*>(qtabs), bitmap,
                     okbytes);
}

hipError_t launch_ecdsa_wave(int wg, int wq, const uint8_t* hashes, const uint8_t* sigs, const uint32_t* key_idx,
                             uint64_t n, const uint32_t* key_valid, uint32_t nkeys, const uint32_t* gtab,
                             const uint32_t* qtabs, uint8_t* bitmap, uint8_t* okbytes, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (n > 0xFFFFFFFFull) return hipErrorInvalidValue;
#define PBFTV_WAVE(G, Q)                                                                                    \
  if (wg == G && wq == Q) {                                                                                   \
    launch_wave_w<G, Q>(hashes, sigs, key_idx, n, key_valid, nkeys, gtab, qtabs, bitmap, okbytes, st);        \
    return hipGetLastError();                                                                                 \
  }
  PBFTV_COMBOS(PBFTV_WAVE)
#undef PBFTV_WAVE
  return hipErrorInvalidValue;
}

uint64_t wave_path_max() {
  if (const char* e = getenv("PBFTV_WAVE_MAX")) return strtoull(e, nullptr, 10);
  return 2048;
}

// signatures per lane in the scalar stage: enough lanes for ~2 waves per SIMD
// (256 CUs x 4 SIMDs x 64 lanes x 2), the rest batched into the inversion.
int scalar_batch(uint64_t n) {
  if (const char* e = getenv("PBFTV_SCALAR_BATCH")) {
    const int k = atoi(e);
    if (k == 1 || k == 2 || k == 4 || k == 8 || k == 16) return k;
  }
  const uint64_t lanes = 256ull * 4 * 64 * 2;
  int k = 1;
  while (k < 16 && n >= (uint64_t)(2 * k) * lanes) k *= 2;
  return k;
}

size_t scalar_prefix_bytes(uint64_t n) {
  const int k = scalar_batch(n);
  const uint64_t L = ((n + k - 1) / k + 255) / 256 * 256;
  return (size_t)k * 9 * L * 4;
}

template <int K>
static void launch_scalars_k(const uint8_t* hashes, const uint8_t* sigs, const uint32_t* key_idx, uint64_t n,
                             const uint32_t* key_valid, uint32_t nkeys, void* scal, uint8_t* flag, uint32_t* prefix,
                             const uint32_t* perm, hipStream_t st) {
  const uint64_t lanes = (n + K - 1) / K;
  const uint64_t blocks = (lanes + 255) / 256;
  hipLaunchKernelGGL(k_ecdsa_scalars<K>, dim3((uint32_t)blocks), dim3(256), 0, st, hashes, sigs, key_idx, n,
                     key_valid, nkeys, reinterpret_cast<uint4*>(scal), flag, prefix, perm);
}

hipError_t launch_ecdsa_scalars(const uint8_t* hashes, const uint8_t* sigs, const uint32_t* key_idx, uint64_t n,
                                const uint32_t* key_valid, uint32_t nkeys, void* scal, uint8_t* flag, void* prefix,
                                const uint32_t* perm, hipStream_t st) {
  if (n == 0) return hipSuccess;
  uint32_t* pf = reinterpret_cast<uint32_t*>(prefix);
  switch (scalar_batch(n)) {
    case 1: launch_scalars_k<1>(hashes, sigs, key_idx, n, key_valid, nkeys, scal, flag, pf, perm, st); break;
    case 2: launch_scalars_k<2>(hashes, sigs, key_idx, n, key_valid, nkeys, scal, flag, pf, perm, st); break;
    case 4: launch_scalars_k<4>(hashes, sigs, key_idx, n, key_valid, nkeys, scal, flag, pf, perm, st); break;
    case 8: launch_scalars_k<8>(hashes, sigs, key_idx, n, key_valid, nkeys, scal, flag, pf, perm, st); break;
    default: launch_scalars_k<16>(hashes, sigs, key_idx, n, key_valid, nkeys, scal, flag, pf, perm, st); break;
  }
  return hipGetLastError();
}

template <int WG, int WQ>
static void launch_comb_w(const void* scal, const uint8_t* flag, const uint8_t* sigs, const uint32_t* key_idx,
                          uint64_t n, const uint32_t* gtab, const uint32_t* qtabs, uint8_t* bitmap,
                          const uint32_t* perm, uint8_t* okb, hipStream_t st) {
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL((k_ecdsa_comb<WG, WQ>), dim3((uint32_t)blocks), dim3(256), 0, st,
                     reinterpret_cast<const uint4*>(scal), flag, sigs, key_idx, n,
                     reinterpret_cast<const uint4*>(gtab), reinterpret_cast<const uint4*>(qtabs), bitmap, perm, okb);
}

hipError_t launch_ecdsa_comb(int wg, int wq, const void* scal, const uint8_t* flag, const uint8_t* sigs,
                             const uint32_t* key_idx, uint64_t n, const uint32_t* gtab, const uint32_t* qtabs,
                             uint8_t* bitmap, const uint32_t* perm, uint8_t* okb, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (perm != nullptr && okb == nullptr) return hipErrorInvalidValue;
#define PBFTV_COMB(G, Q)                                                                       \
  if (wg == G && wq == Q) {                                                                    \
    launch_comb_w<G, Q>(scal, flag, sigs, key_idx, n, gtab, qtabs, bitmap, perm, okb, st);     \
    return hipGetLastError();                                                                  \
  }
  PBFTV_COMBOS(PBFTV_COMB)
#undef PBFTV_COMB
  return hipErrorInvalidValue;
}

size_t ecdsa_scratch_bytes(uint64_t n) { return (size_t)n * 64 + (size_t)n; }

}  // namespace pbftv
