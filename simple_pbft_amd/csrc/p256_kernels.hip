// p256_kernels.hip -- ECDSA-P256 batch verification for gfx950: table
// construction, stage 1 (scalars), key order, and the dispatch of the verify
// kernels (verify_kernels.h, instantiated per G width in p256_verify_g*.hip).
//   k_tab_*          key validation + fixed-base comb tables for G and every
//                    registered key (three-phase parallel build).
//   k_ecdsa_scalars  Go's range checks on (r, s), w = s^-1 mod n (K signatures
//                    per lane share one safegcd inversion), u1 = e w, u2 = r w
//                    -> 64 B of scalars per signature.
//   k_key_*          stage 0: key order of the lanes (counting sort by key).
// Semantics: Go 1.19 crypto/ecdsa.Verify (see p256_algo.h); parity with the
// oracle is tested in tests/test_gpu_parity.py.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "kernels.h"
#include "verify_kernels.h"

namespace pbftv {

// key-order sort (k_key_*): blocks of the histogram/scatter passes, largest key count sorted
#ifndef PBFTV_SCAL_BLOCK_INV_MIN_K
#define PBFTV_SCAL_BLOCK_INV_MIN_K 4  // K from which stage 1 inverts once per block (block_batch_inv_n)
#endif

#ifndef PBFTV_SCAL_WAVES
#define PBFTV_SCAL_WAVES 1  // min waves per SIMD for k_ecdsa_scalars (the compiler settles at 124 VGPRs: 4)
#endif

constexpr uint32_t kSortBlocks = 256;
constexpr uint32_t kSortMaxKeys = 1024;
constexpr uint32_t kSortHdr = kSortMaxKeys + 64;  // key-sort header: 2 x (totals | claims), words each

// ---------------------------------------------------------------------------
// Table construction (p256_algo.h, "generic (W-bit) table construction"):
// three kernels over all bases of a registration, every phase spread over
// enough lanes to fill the chip (a registration of G alone is 9 windows).
// Base b of a launch is G when with_g && b == 0, else key key0 + b - with_g;
// its table is written at tabs[b] (a device array of per-base pointers: every
// key table is its own allocation, so keys can be added or replaced one at a
// time).
template <int W>
struct TabGeom {
  using G = CombGeom<W>;
  // L table: (lo+1) B_i, lo < CL; H table: hi (CL B_i), 1 <= hi < NH.  Up to
  // W = 16 CL = 256; wider windows split E = CL * NH near sqrt(E).
  static constexpr int CL = G::kEnt < 256 ? G::kEnt : (G::kW <= 16 ? 256 : 1 << (G::kW / 2));
  static constexpr int NH = G::kEnt / CL;
  static constexpr int LOG_CL = __builtin_ctz(CL);
  // phase 2: lanes of SEG consecutive multiples (L: SL segments, H: SH)
  static constexpr int SEG = CL < 64 ? CL : 64;
  static constexpr int SL = CL / SEG;
  static constexpr int SH = NH > 1 ? (NH - 1 + SEG - 1) / SEG : 0;
  static constexpr int SS = 4 * SEG;  // phase-2 scratch slots per lane
  // phase 3: lanes of PC entries sharing one H (one batched inversion each)
  static constexpr int PC = CL < 256 ? CL : 256;
};

__device__ __forceinline__ bool load_base(const uint32_t* __restrict__ keys_le, uint32_t b, int with_g, fe& bx,
                                          fe& by) {
  if (with_g && b == 0) {
    fe_set(bx, kGxMont);
    fe_set(by, kGyMont);
    return true;
  }
  const uint32_t* k = keys_le + (uint64_t)(b - with_g) * 16;  // this launch's keys
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
  const bool ok = load_base(keys_le, b, with_g, bx, by);
  if (win == 0 && !(with_g && b == 0)) valid[key0 + b - with_g] = ok ? 1u : 0u;
  window_base(bases + (uint64_t)lane * 16, CombGeom<W>::bit((int)win), bx, by);
}

// t P (Jacobian) for 1 <= t < 2^31 and affine P: left-to-right binary method
// (never exceptional: the running multiple is >= 2 before every addition)
__device__ __forceinline__ void jac_mul_small(jac& r, uint32_t t, const fe& px, const fe& py) {
  r.x = px;
  r.y = py;
  fe_set(r.z, kOneP);
  for (int k = 30 - __builtin_clz(t); k >= 0; --k) {
    jac_double(r, r);
    if ((t >> k) & 1u) jac_madd<false>(r, px, py);
  }
}

// phase 2: lane (bw, seg) with bw = b*nwin + win.  seg < SL: L entries
// seg*SEG .. +SEG-1, i.e. (k + 1) B_i; seg >= SL: H entries (hi - 1 for hi =
// 1 + (seg-SL)*SEG ..), i.e. hi (CL B_i).  Each lane starts from its first
// multiple (binary method) and walks the rest by mixed additions, then one
// batched inversion to affine.
template <int W>
__global__ void __launch_bounds__(64) k_tab_small(const uint32_t* __restrict__ bases, uint32_t nb,
                                                  uint32_t* __restrict__ lbuf, uint32_t* __restrict__ hbuf,
                                                  fe* __restrict__ scratch) {
  using T = TabGeom<W>;
  constexpr int nwin = CombGeom<W>::kWin;
  constexpr uint32_t segs = T::SL + T::SH;
  const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= (uint64_t)nb * nwin * segs) return;
  const uint64_t bw = lane / segs;
  const uint32_t seg = (uint32_t)(lane % segs);
  fe* sc = scratch + lane * T::SS;
  auto st = [&](int slot, const fe& v) { sc[slot] = v; };
  auto ld = [&](int slot, fe& v) { v = sc[slot]; };
  uint32_t bw16[16];
  for (int i = 0; i < 16; ++i) bw16[i] = bases[bw * 16 + i];
  fe px, py;
  entry_to_fe(px, py, bw16);
  const bool is_h = seg >= (uint32_t)T::SL;
  uint32_t first, cnt;
  uint32_t* out;
  if (!is_h) {
    first = seg * T::SEG + 1;
    cnt = T::SEG;
    out = lbuf + (bw * T::CL + (uint64_t)seg * T::SEG) * 16;
  } else {  // H walks multiples of Q = CL B_i: 2^LOG_CL doublings, then affine
    const uint32_t h0 = (seg - T::SL) * T::SEG;
    first = h0 + 1;
    cnt = (uint32_t)(T::NH - 1) - h0 < (uint32_t)T::SEG ? (uint32_t)(T::NH - 1) - h0 : (uint32_t)T::SEG;
    out = hbuf + (bw * (T::NH - 1) + h0) * 16;
    jac q;
    q.x = px;
    q.y = py;
    fe_set(q.z, kOneP);
    for (int k = 0; k < T::LOG_CL; ++k) jac_double(q, q);
    fe zi;
    fe_inv(zi, q.z);
    uint32_t qw[16];
    jac_to_affine_words(qw, q, zi);
    entry_to_fe(px, py, qw);
  }
  jac cur;
  jac_mul_small(cur, first, px, py);
  for (uint32_t k = 0; k < cnt; ++k) {
    if (k > 0) {
      if (first + k - 1 == 1) jac_double(cur, cur);  // 1 P + P
      else jac_madd<false>(cur, px, py);             // (m + 1) P, 2 <= m << n: never exceptional
    }
    st(3 * (int)k, cur.x);
    st(3 * (int)k + 1, cur.y);
    st(3 * (int)k + 2, cur.z);
  }
  batch_to_affine(out, (int)cnt, st, ld);
}

// phase 3: lane (b, win, hi, part) -> PC entries idx = hi*CL + part*PC + j of
// base b's table, entry = H_hi + L_lo by AFFINE addition with the PC
// denominators inverted together: lambda = (ly - hy) / (lx - hx),
// x3 = lambda^2 - hx - lx, y3 = lambda (hx - x3) - hy -- 6 products per entry
// plus 1/PC of an inversion.  The one doubling (hi = 1, lo + 1 = CL: L = H)
// is done in Jacobian form with its own inversion.
// A launch covers global lanes [lane0, lane1); scratch is indexed by lane - lane0.
// (2 waves per SIMD at 189 VGPRs: 3 measured the same, 4 spills and is 15 % slower; tools/reg_ab.sh)
template <int W>
__global__ void __launch_bounds__(64) k_tab_entries(const uint32_t* __restrict__ lbuf,
                                                    const uint32_t* __restrict__ hbuf, uint64_t lane0,
                                                    uint64_t lane1, uint32_t* const* __restrict__ tabs,
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
  uint32_t* out = tabs[b] + (G::base((int)win) + (uint64_t)hi * T::CL + (uint64_t)part * T::PC) * 16;
  if (hi == 0) {  // H_0 = 0: a copy of L
    for (int j = 0; j < T::PC * 16; ++j) out[j] = L[j];
    return;
  }
  uint32_t hw[16];
  for (int i = 0; i < 16; ++i) hw[i] = hbuf[(bw * (T::NH - 1) + hi - 1) * 16 + i];
  fe hx, hy;
  entry_to_fe(hx, hy, hw);
  // the doubling entry of this chunk, if any: lo + 1 = CL with hi = 1
  const int dbl = (hi == 1 && part == parts - 1) ? T::PC - 1 : -1;
  // signed-limb arithmetic (fes.h): differences are 9 subtractions, products
  // S-type.  Only the prefix products go to scratch, limb-major across the
  // launch's lanes (coalesced); d_j is recomputed from L (cache-resident: one
  // L row serves every hi of its window) on the way back.
  const uint64_t nl = lane1 - lane0;
  uint32_t* pre = reinterpret_cast<uint32_t*>(scratch) + local;
  auto st_pre = [&](int j, const fe& v) {
    PBFTV_UNROLL for (int l = 0; l < 9; ++l) pre[((uint64_t)j * 9 + l) * nl] = v.v[l];
  };
  auto ld_pre = [&](int j, fe& v) {
    PBFTV_UNROLL for (int l = 0; l < 9; ++l) v.v[l] = pre[((uint64_t)j * 9 + l) * nl];
  };
  auto den = [&](int j, fe& lx, fe& ly, fe& d) {
    entry_to_fe(lx, ly, L + (uint64_t)j * 16);
    fs_sub(d, lx, hx);
    if (j == dbl) fe_set(d, kOneP);
  };
  fe acc, lx, ly, d;
  fe_set(acc, kOneP);
  for (int j = 0; j < T::PC; ++j) {
    den(j, lx, ly, d);
    fs_mul(acc, acc, d);
    st_pre(j, acc);  // d_0 ... d_j
  }
  fe inv;
  fs_canon(acc, acc);
  fe_inv(inv, acc);
  for (int j = T::PC - 1; j >= 0; --j) {
    den(j, lx, ly, d);
    fe dinv;
    if (j > 0) {
      fe p;
      ld_pre(j - 1, p);
      fs_mul(dinv, inv, p);  // 1/d_j
      fs_mul(inv, inv, d);   // 1/(d_0 ... d_{j-1})
    } else {
      dinv = inv;
    }
    uint32_t* o = out + (uint64_t)j * 16;
    if (j == dbl) {  // 2 H
      jac p;
      p.x = hx;
      p.y = hy;
      fe_set(p.z, kOneP);
      jac_double(p, p);
      fe zi;
      fe_inv(zi, p.z);
      jac_to_affine_words(o, p, zi);
      continue;
    }
    fe dy, lam, l2, x3, t, y3;
    fs_sub(dy, ly, hy);
    fs_mul(lam, dy, dinv);        // S
    fs_sqr(l2, lam);
    PBFTV_UNROLL for (int i = 0; i < 9; ++i) x3.v[i] = l2.v[i] - hx.v[i] - lx.v[i];
    fs_norm(x3, x3);              // lambda^2 - hx - lx (S)
    fs_sub(t, hx, x3);            // D
    fs_mul(y3, lam, t);
    fs_sub(y3, y3, hy);           // lambda (hx - x3) - hy (D)
    fs_canon(x3, x3);
    fs_canon(y3, y3);
    fe_to_words(o, x3);
    fe_to_words(o + 8, y3);
  }
}

template <int W>
hipError_t build_tables_w(const uint32_t* keys_le, uint32_t key0, uint32_t nb, int with_g, uint32_t* valid,
                          uint32_t* const* tabs, TableScratch& sc, hipStream_t st) {
  using T = TabGeom<W>;
  using G = CombGeom<W>;
  if (nb == 0) return hipSuccess;
  const uint32_t lanes1 = nb * G::kWin;
  hipLaunchKernelGGL(k_tab_bases<W>, dim3((lanes1 + 63) / 64), dim3(64), 0, st, keys_le, key0, nb, with_g, valid,
                     reinterpret_cast<uint32_t*>(sc.bases));
  const uint64_t lanes2 = (uint64_t)lanes1 * (T::SL + T::SH);
  hipLaunchKernelGGL(k_tab_small<W>, dim3((uint32_t)((lanes2 + 63) / 64)), dim3(64), 0, st,
                     reinterpret_cast<const uint32_t*>(sc.bases), nb, reinterpret_cast<uint32_t*>(sc.lbuf),
                     reinterpret_cast<uint32_t*>(sc.hbuf), reinterpret_cast<fe*>(sc.small_scratch));
  // phase 3 in slices of sc.entry_lanes lanes (its scratch is per lane)
  constexpr uint64_t per_base = (uint64_t)G::kWin * T::NH * (T::CL / T::PC);
  const uint64_t total = (uint64_t)nb * per_base;
  for (uint64_t l0 = 0; l0 < total; l0 += sc.entry_lanes) {
    const uint64_t l1 = total - l0 < sc.entry_lanes ? total : l0 + sc.entry_lanes;
    hipLaunchKernelGGL(k_tab_entries<W>, dim3((uint32_t)((l1 - l0 + 63) / 64)), dim3(64), 0, st,
                       reinterpret_cast<const uint32_t*>(sc.lbuf), reinterpret_cast<const uint32_t*>(sc.hbuf), l0, l1,
                       tabs, reinterpret_cast<fe*>(sc.entry_scratch));
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
    z.small_scratch = (size_t)nb * G::kWin * (T::SL + T::SH) * T::SS * sizeof(fe);
    const uint64_t total = (uint64_t)G::kWin * T::NH * (T::CL / T::PC) * nb;
    const uint64_t cap = 1ull << 18;  // 256 Ki lanes x 9 KiB of prefix products
    z.entry_lanes = total < cap ? total : cap;
    z.entry_scratch = (size_t)z.entry_lanes * T::PC * sizeof(fe);
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
                               uint32_t* valid, uint32_t* const* tabs, TableScratch& sc, hipStream_t st) {
  switch (w) {
#define PBFTV_W(W) \
  case W: return build_tables_w<W>(keys_le, key0, nb, with_g, valid, tabs, sc, st);
    PBFTV_TABLE_WIDTHS(PBFTV_W)
#undef PBFTV_W
    default: return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------
// Key order for the comb (stage 0).  The key tables are looked up at random
// entries; when the 64 lanes of a wave name ~50 different keys (a random
// 100-key batch) every wave-wide table load touches ~50 tables, when they
// share a key the lookups fall in one table window like the G lookups do.
// Same-box A/B at 1M signatures / 100 keys (round-1 bench with the batch pre-sorted on the host): comb
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

// One launch (k_key_hist: per-block histograms in LDS added into per-key
// totals) and the scatter inside stage 1: every stage-1 block counts its own
// signatures by key in LDS during its forward pass, scans the <= 1025 totals
// itself (the key starts), claims its range of each key with one atomic on a
// claim counter, and places each record through LDS cursors in its backward
// pass.  No memset, no scan launch, no fence, no position array.  The header
// holds two sets of per-key counters (totals, claims); batch j counts into set
// j % 2 while k_key_hist's block 0 clears set (j + 1) % 2 for the next batch
// (that set's last reader, batch j - 1's stage 1, finished before this launch
// began).  Both sets start zeroed when the scratch is allocated.  Round 2
// began with memset + hist + scan + scatter: 4 launches and two 5-us fills.
__global__ void __launch_bounds__(256) k_key_hist(const uint32_t* __restrict__ key_idx, uint64_t n, uint32_t nkeys,
                                                  uint32_t* __restrict__ cur, uint32_t* __restrict__ other) {
  __shared__ uint32_t h[kSortMaxKeys + 1];
  if (blockIdx.x == 0)
    for (uint32_t b = threadIdx.x; b < 2 * kSortHdr; b += blockDim.x) other[b] = 0;
  block_key_hist(h, key_idx, n, nkeys);
  for (uint32_t b = threadIdx.x; b <= nkeys; b += blockDim.x)
    if (h[b]) atomicAdd(&cur[b], h[b]);
}

// start[b] = exclusive prefix of total[0..nkeys] (<= 1025 entries), every
// thread of the 256-thread block; start[] is complete after the call's last
// __syncthreads.
__device__ __forceinline__ void block_key_starts(const uint32_t* __restrict__ total, uint32_t nkeys, uint32_t* start,
                                                 uint32_t* part) {
  constexpr uint32_t kPer = (kSortMaxKeys + 1 + 255) / 256;
  const uint32_t t = threadIdx.x, m = nkeys + 1;
  uint32_t v[kPer], sum = 0;
  PBFTV_UNROLL for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t b = kPer * t + k;
    v[k] = b < m ? total[b] : 0u;
    sum += v[k];
  }
  part[t] = sum;
  __syncthreads();
  for (uint32_t off = 1; off < 256; off <<= 1) {
    const uint32_t x = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  PBFTV_UNROLL for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t b = kPer * t + k;
    if (b < m) start[b] = run;
    run += v[k];
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// stage 1: scalars.  One 128-B record per signature (SigRec, verify_kernels.h):
// u1 = e w, u2 = r w (LE words), r, the key index, the signature's batch
// index and ok = Go's range checks passed and the key is registered and valid.
//
// Inputs are read in ARRIVAL order -- each lane owns K signatures i = lane +
// j*L (j < K, L = lanes in the grid), so every input load is coalesced across
// the wave -- and each record is written to the signature's position in key
// order (placed through the block's LDS cursors, see block_key_starts above;
// the batch index without a key order): one full
// 128-B line per lane, so the comb reads its lane's record coalesced and never
// gathers through a permutation.  The 64 K values of s of a wave share ONE
// inversion (Montgomery's trick twice: per lane, prefix products c_j = s_0 ...
// s_j in a limb-major scratch; across the lanes, wave_batch_inv_n gives every
// lane c_{K-1}^-1 from one lane-parallel safegcd; then walking back w_j = inv
// * c_{j-1}, inv *= s_j).
//
// The lane multiplies PLAIN s values (no conversion to Montgomery form per
// signature) and fixes the powers of R once per lane.  With fn_mul(a, b) =
// a b R^-1 mod n:
//   forward   c_0 = s_0, c_j = fn_mul(c_{j-1}, s_j) = (s_0 .. s_j) R^-j;
//             the lane total c_{K-1} = P R^(1-K) -> P R by one fn_mul with R^(K+1);
//   wave      wave_batch_inv_n: P^-1 R, then one fn_mul with R^K: inv = P^-1 R^K;
//   backward  invariant inv = (s_0 .. s_j)^-1 R^(j+1):
//             w_j = fn_mul(inv, c_{j-1}) = s_j^-1 R (Montgomery form of s_j^-1),
//             inv = fn_mul(inv, s_j); w_0 = inv.
// Per signature 4 Montgomery multiplies (c_j, w_j, inv, and u1 / u2: 2) + 16/K
// for the lane fixes and the wave scans + 1/(64 K) of an inversion (round 2
// converted every s: 6 + 14/K); from K = 4 the scan and the inversion are
// shared by the block (block_batch_inv_n): 2/K + 9.75/K and 1/(256 K).
template <int K>
__global__ void __launch_bounds__(256, PBFTV_SCAL_WAVES) k_ecdsa_scalars(const uint8_t* __restrict__ hashes,
                                                       const uint8_t* __restrict__ sigs,
                                                       const uint32_t* __restrict__ key_idx, uint64_t n,
                                                       const uint32_t* __restrict__ key_valid, uint32_t nkeys,
                                                       SigRec* __restrict__ rec, uint32_t* __restrict__ prefix,
                                                       KeyOrder ko) {
  static_assert(K >= 1 && K <= 16, "kRPowN covers R^0 .. R^17");
  const uint64_t L = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // key order: this block's signatures counted per key (then its cursors)
  __shared__ uint32_t kh[kSortMaxKeys + 1], kstart[kSortMaxKeys + 1], kpart[256];
  // the lane's prefix products c_0 .. c_{K-2}: in LDS for K <= 4 (27.6 KB per
  // block at K = 4, no HBM round trip: 57 MB per launch at 1M), else in the
  // global scratch (each thread reads back only what it wrote)
  constexpr bool kPrefixLds = K <= 4;
  __shared__ uint32_t spre[kPrefixLds ? (K > 1 ? K - 1 : 1) : 1][9][256];
  const bool sorted = ko.total != nullptr;  // block-uniform
  const uint32_t nk = ko.nkeys;
  PBFTV_SPROBE(0, nk);
  if (sorted) {
    for (uint32_t b = threadIdx.x; b <= nk; b += blockDim.x) kh[b] = 0;
    block_key_starts(ko.total, nk, kstart, kpart);  // (ends with a barrier: kh[] is clear)
  }
  PBFTV_SPROBE(1, kstart[0]);
  // The forward pass reads s only (32 B): an s outside (0, n) joins the
  // products as 1.  r, the key and the hash are read once, in the backward
  // pass, where Go's remaining checks decide the record's ok.
  fe acc, rk;
  uint32_t okm = 0;  // bit j: 0 < s_j < n
  // K <= 2 (the small strong-scaling shards, one wave round): every input of
  // the lane's signatures is loaded here, so its HBM latency hides behind the
  // forward products and the inversion instead of sitting on the backward
  // pass's chain (~52 more VGPRs at K = 2, still 2 waves per SIMD)
  constexpr bool kPre = K <= 2;
  constexpr int KP = kPre ? K : 1;
  uint32_t pr[KP][8], ps[KP][8], pe[KP][8], pk[KP];
  bool pv[KP];
  constexpr int KU = kPre ? K : 1;  // fully unrolled with the prefetch (register arrays, no scratch)
#pragma unroll KU
  for (int j = 0; j < K; ++j) {
    const uint64_t i = lane + (uint64_t)j * L;
    uint32_t sw[8] = {1, 0, 0, 0, 0, 0, 0, 0};
    bool oks = false;
    if (i < n) {
      uint32_t s[8];
      load_be256(sigs + 64 * i + 32, s);
      uint32_t k;
      if constexpr (kPre) {
        load_be256(sigs + 64 * i, pr[j]);
        load_be256(hashes + 32 * i, pe[j]);
        k = pk[j] = key_idx[i];
        pv[j] = k < nkeys && key_valid[k] != 0;
        PBFTV_UNROLL for (int t = 0; t < 8; ++t) ps[j][t] = s[t];
      }
      oks = !words_is_zero(s) && words_lt(s, kN32);
      if (oks) PBFTV_UNROLL for (int t = 0; t < 8; ++t) sw[t] = s[t];
      if (sorted) {
        if constexpr (!kPre) k = key_idx[i];
        atomicAdd(&kh[k < nk ? k : nk], 1u);  // bin nk: out-of-range key indices (rejected below)
      }
    }
    fe sv;
    fe_from_words(sv, sw);
    if (j == 0) acc = sv;
    else fn_mul(acc, acc, sv);
    if (j + 1 < K) {  // c_j is read back for w_{j+1}
      if constexpr (kPrefixLds) {
        PBFTV_UNROLL for (int l = 0; l < 9; ++l) spre[j][l][threadIdx.x] = acc.v[l];
      } else {
        PBFTV_UNROLL for (int l = 0; l < 9; ++l) prefix[((uint64_t)j * 9 + l) * L + lane] = acc.v[l];
      }
    }
    okm |= (oks ? 1u : 0u) << j;
  }
  PBFTV_SPROBE(2, acc.v[0]);
  fe_set(rk, kRPowN[K + 1]);
  fn_mul(acc, acc, rk);        // P R: the lane total in Montgomery form
  if (sorted) {  // claim this block's range of every key: kh[] becomes its cursors
    __syncthreads();
    for (uint32_t b = threadIdx.x; b <= nk; b += blockDim.x)
      if (kh[b]) kh[b] = kstart[b] + atomicAdd(&ko.claim[b], kh[b]);
    __syncthreads();
  }
  PBFTV_SPROBE(3, acc.v[0]);
  fe inv;
  if constexpr (K >= PBFTV_SCAL_BLOCK_INV_MIN_K) {
    // P^-1 R: one inversion and one cross-lane scan per 256-thread block, 6
    // products per lane instead of 15 (kstart is free once the claims above
    // are made; 64 x 9 words of it hold the quad products).  Same box, two
    // streams: 1M step -0.3 %, 262k -1 %; at K <= 2 (131k, one wave round) the
    // barriers lengthen the lone kernel (0.051 vs 0.046 ms), so K <= 2 keep
    // one inversion per wave (profiles/r03_ab_block_inversion.txt)
    static_assert(kSortMaxKeys + 1 >= 64 * 9, "kstart holds the block inversion's slots");
    block_batch_inv_n(inv, acc, kstart);
  } else {
    wave_batch_inv_n(inv, acc);  // P^-1 R: one inversion per wave (64 K signatures)
  }
  PBFTV_SPROBE(4, inv.v[0]);
  if (K > 1) {
    fe_set(rk, kRPowN[K]);
    fn_mul(inv, inv, rk);      // P^-1 R^K
  }
#pragma unroll KU
  for (int j = K - 1; j >= 0; --j) {
    const uint64_t i = lane + (uint64_t)j * L;
    const bool oks = (okm >> j) & 1u;
    uint32_t r[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s[8] = {1, 0, 0, 0, 0, 0, 0, 0};
    bool ok = false;
    if (i < n) {
      uint32_t sl[8];
      if constexpr (kPre) {  // Go's range checks + a valid key on the prefetched inputs
        PBFTV_UNROLL for (int t = 0; t < 8; ++t) {
          r[t] = pr[j][t];
          sl[t] = ps[j][t];
        }
        ok = oks && pv[j] && !words_is_zero(r) && words_lt(r, kN32);
      } else {
        ok = oks && sig_ok(sigs, key_idx, key_valid, nkeys, i, r, sl);  // Go's range checks + a valid key
      }
      if (oks) PBFTV_UNROLL for (int t = 0; t < 8; ++t) s[t] = sl[t];
    }
    if (!ok) PBFTV_UNROLL for (int t = 0; t < 8; ++t) r[t] = 0;
    fe w;
    if (K > 1 && j > 0) {
      fe pre;
      if constexpr (kPrefixLds) {
        PBFTV_UNROLL for (int l = 0; l < 9; ++l) pre.v[l] = spre[j - 1][l][threadIdx.x];
      } else {
        PBFTV_UNROLL for (int l = 0; l < 9; ++l) pre.v[l] = prefix[((uint64_t)(j - 1) * 9 + l) * L + lane];
      }
      fn_mul(w, inv, pre);     // s_j^-1 R
      fe sv;
      fe_from_words(sv, s);
      fn_mul(inv, inv, sv);    // (s_0 .. s_{j-1})^-1 R^j
    } else {
      w = inv;
    }
    if (i < n) {
      uint32_t u1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, u2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (ok) {
        uint32_t e[8];
        if constexpr (kPre) {
          PBFTV_UNROLL for (int t = 0; t < 8; ++t) e[t] = pe[j][t];
        } else {
          load_be256(hashes + 32 * i, e);
        }
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
      uint64_t at = i;
      uint32_t kj;
      if constexpr (kPre) kj = pk[j];
      else kj = key_idx[i];
      if (sorted) at = atomicAdd(&kh[kj < nk ? kj : nk], 1u);  // the signature's place in key order
      SigRec* o = rec + at;
      o->q[0] = make_uint4(u1[0], u1[1], u1[2], u1[3]);
      o->q[1] = make_uint4(u1[4], u1[5], u1[6], u1[7]);
      o->q[2] = make_uint4(u2[0], u2[1], u2[2], u2[3]);
      o->q[3] = make_uint4(u2[4], u2[5], u2[6], u2[7]);
      o->q[4] = make_uint4(r[0], r[1], r[2], r[3]);
      o->q[5] = make_uint4(r[4], r[5], r[6], r[7]);
      o->q[6] = make_uint4(ok ? kj : 0u, (uint32_t)i, ok ? 1u : 0u, 0u);
    }
  }
  PBFTV_SPROBE(5, okm);
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

size_t key_sort_header_bytes() { return (size_t)(4 * kSortHdr) * 4; }
size_t key_sort_scratch_bytes(uint64_t, uint32_t) { return key_sort_header_bytes(); }

hipError_t launch_key_count(const uint32_t* key_idx, uint64_t n, uint32_t nkeys, void* scratch, uint32_t parity,
                            KeyOrder* out, hipStream_t st) {
  if (nkeys > kSortMaxKeys) return hipErrorInvalidValue;
  uint32_t* hdr = reinterpret_cast<uint32_t*>(scratch);
  uint32_t* cur = hdr + (parity & 1u) * 2 * kSortHdr;  // totals | claims of this batch
  uint32_t* other = hdr + (~parity & 1u) * 2 * kSortHdr;
  *out = KeyOrder{cur, cur + kSortHdr, nkeys};
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_key_hist, dim3(kSortBlocks), dim3(256), 0, st, key_idx, n, nkeys, cur, other);
  return hipGetLastError();
}

hipError_t launch_pack_bits(const uint8_t* okb, uint64_t n, uint8_t* bitmap, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const uint64_t bytes = (n + 7) / 8;
  hipLaunchKernelGGL(k_pack_bits, dim3((uint32_t)((bytes + 255) / 256)), dim3(256), 0, st, okb, n, bitmap);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// dispatch over the instantiation units (p256_verify_g*.hip)
bool launch_comb_part_g29(int wg, int wq, const CombArgs& a, hipStream_t st);
bool launch_comb_part_g26(int wg, int wq, const CombArgs& a, hipStream_t st);
bool launch_comb_part_g24(int wg, int wq, const CombArgs& a, hipStream_t st);
bool launch_comb_part_small(int wg, int wq, const CombArgs& a, hipStream_t st);
bool launch_wave_part_g29(int wg, int wq, const WaveArgs& a, hipStream_t st);
bool launch_wave_part_g26(int wg, int wq, const WaveArgs& a, hipStream_t st);
bool launch_wave_part_g24(int wg, int wq, const WaveArgs& a, hipStream_t st);
bool launch_wave_part_small(int wg, int wq, const WaveArgs& a, hipStream_t st);

hipError_t launch_ecdsa_wave(int wg, int wq, const uint8_t* hashes, const uint8_t* sigs, const uint32_t* key_idx,
                             uint64_t n, const uint32_t* key_valid, uint32_t nkeys, const uint32_t* gtab,
                             const uint32_t* const* qtabs, uint8_t* bitmap, uint8_t* okbytes, hipStream_t st,
                             bool one_wave) {
  if (n == 0) return hipSuccess;
  if (n > 0xFFFFFFFFull) return hipErrorInvalidValue;
  const WaveArgs a{hashes, sigs, key_idx, n, key_valid, nkeys, gtab, qtabs, bitmap, okbytes, one_wave};
  if (launch_wave_part_g29(wg, wq, a, st) || launch_wave_part_g26(wg, wq, a, st) ||
      launch_wave_part_g24(wg, wq, a, st) || launch_wave_part_small(wg, wq, a, st))
    return hipGetLastError();
  return hipErrorInvalidValue;
}

bool launch_armed_part_g29(int wg, int wq, const ArmArgs& a, hipStream_t st);
bool launch_armed_part_g26(int wg, int wq, const ArmArgs& a, hipStream_t st);
bool launch_armed_part_g24(int wg, int wq, const ArmArgs& a, hipStream_t st);
bool launch_armed_part_small(int wg, int wq, const ArmArgs& a, hipStream_t st);

hipError_t launch_ecdsa_wave_armed(int wg, int wq, const ArmArgs& a, hipStream_t st) {
  if (launch_armed_part_g29(wg, wq, a, st) || launch_armed_part_g26(wg, wq, a, st) ||
      launch_armed_part_g24(wg, wq, a, st) || launch_armed_part_small(wg, wq, a, st))
    return hipGetLastError();
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
  // with the inversion shared by the wave (wave_batch_inv_n), K only trades
  // per-lane scan products against occupancy: K = 4 at 1M (0.134 ms; K = 2 /
  // 8 / 16: 0.158 / 0.143 / 0.169 ms, tools/ab.sh same box)
  // K = 2 from 131072 (1M / 8, a strong-scaling shard: 0.046 vs 0.051 ms at
  // K = 1, K = 4 0.056), K = 4 from 262144
  const uint64_t lanes = 65536;
  int k = 1;
  while (k < 4 && n >= (uint64_t)(2 * k) * lanes) k *= 2;
  return k;
}

size_t scalar_prefix_bytes(uint64_t n) {
  const int k = scalar_batch(n);
  const uint64_t L = ((n + k - 1) / k + 255) / 256 * 256;
  return (size_t)k * 9 * L * 4;
}

template <int K>
static void launch_scalars_k(const uint8_t* hashes, const uint8_t* sigs, const uint32_t* key_idx, uint64_t n,
                             const uint32_t* key_valid, uint32_t nkeys, void* rec, uint32_t* prefix,
                             const KeyOrder& ko, hipStream_t st) {
  const uint64_t lanes = (n + K - 1) / K;
  const uint64_t blocks = (lanes + 255) / 256;
  hipLaunchKernelGGL(k_ecdsa_scalars<K>, dim3((uint32_t)blocks), dim3(256), 0, st, hashes, sigs, key_idx, n,
                     key_valid, nkeys, reinterpret_cast<SigRec*>(rec), prefix, ko);
}

hipError_t launch_ecdsa_scalars(const uint8_t* hashes, const uint8_t* sigs, const uint32_t* key_idx, uint64_t n,
                                const uint32_t* key_valid, uint32_t nkeys, void* rec, void* prefix,
                                const KeyOrder& ko, hipStream_t st) {
  if (n == 0) return hipSuccess;
  uint32_t* pf = reinterpret_cast<uint32_t*>(prefix);
  switch (scalar_batch(n)) {
    case 1: launch_scalars_k<1>(hashes, sigs, key_idx, n, key_valid, nkeys, rec, pf, ko, st); break;
    case 2: launch_scalars_k<2>(hashes, sigs, key_idx, n, key_valid, nkeys, rec, pf, ko, st); break;
    case 4: launch_scalars_k<4>(hashes, sigs, key_idx, n, key_valid, nkeys, rec, pf, ko, st); break;
    case 8: launch_scalars_k<8>(hashes, sigs, key_idx, n, key_valid, nkeys, rec, pf, ko, st); break;
    default: launch_scalars_k<16>(hashes, sigs, key_idx, n, key_valid, nkeys, rec, pf, ko, st); break;
  }
  return hipGetLastError();
}

hipError_t launch_ecdsa_comb(int wg, int wq, const void* rec, uint64_t n, const uint32_t* gtab,
                             const uint32_t* const* qtabs,
                             uint8_t* bitmap, uint8_t* okb, const uint32_t* cuflag, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const CombArgs a{rec, n, gtab, qtabs, bitmap, okb, cuflag};
  if (launch_comb_part_g29(wg, wq, a, st) || launch_comb_part_g26(wg, wq, a, st) ||
      launch_comb_part_g24(wg, wq, a, st) || launch_comb_part_small(wg, wq, a, st))
    return hipGetLastError();
  return hipErrorInvalidValue;
}

size_t ecdsa_record_bytes(uint64_t n) { return (size_t)n * sizeof(SigRec); }

}  // namespace pbftv

#ifdef PBFTV_SCAL_PROBE
extern "C" int pbftv_debug_scal_probe(uint64_t* out, size_t n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pbftv::g_scal_probe), n * sizeof(uint64_t), 0,
                                  hipMemcpyDeviceToHost);
}
#endif
