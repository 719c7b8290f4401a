// p256_kernels.hip -- ECDSA-P256 batch verification kernels for gfx950.
//
// One signature per lane (64 per wave).  Three kernels:
//   k_build_tables   key validation + fixed-base comb tables for G and every
//                    registered key (one lane per (base, 8-bit window)).
//   k_ecdsa_scalars  Go's range checks on (r, s), w = s^-1 mod n (Fermat),
//                    u1 = e w, u2 = r w  -> 64 B of scalars per signature.
//   k_ecdsa_comb     u1*G + u2*Q as two 33-step signed-digit combs (mixed
//                    additions only), one complete addition, and the x-coordinate
//                    check  X == r Z^2 (or (r+n) Z^2) -- no field inversion.
//                    Writes the LSB-first accept bitmap via a wave ballot.
// Semantics: Go 1.19 crypto/ecdsa.Verify (see p256_algo.h); parity with the
// oracle is tested in tests/test_gpu_parity.py.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "kernels.h"
#include "p256_algo.h"

namespace pbftv {

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// 32 big-endian bytes at p (16-B aligned) -> 8 LE words
__device__ __forceinline__ void load_be256(const uint8_t* __restrict__ p, uint32_t w[8]) {
  const uint4 a = *reinterpret_cast<const uint4*>(p);
  const uint4 b = *reinterpret_cast<const uint4*>(p + 16);
  w[7] = bswap32(a.x); w[6] = bswap32(a.y); w[5] = bswap32(a.z); w[4] = bswap32(a.w);
  w[3] = bswap32(b.x); w[2] = bswap32(b.y); w[1] = bswap32(b.z); w[0] = bswap32(b.w);
}

// ---------------------------------------------------------------------------
// table construction: lane = base * kWindows + window.  base 0 = G, base b>0 = key b-1.
__global__ void __launch_bounds__(64) k_build_tables(const uint32_t* __restrict__ keys_le, uint32_t nkeys,
                                                     uint32_t* __restrict__ tables, uint32_t* __restrict__ valid,
                                                     fe* __restrict__ scratch) {
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nbases = nkeys + 1;
  if (lane >= nbases * kWindows) return;
  const uint32_t base = lane / kWindows, win = lane % kWindows;
  fe bx, by;
  bool ok = true;
  if (base == 0) {
    fe_set(bx, kGxMont);
    fe_set(by, kGyMont);
  } else {
    uint32_t xw[8], yw[8];
    const uint32_t* k = keys_le + (uint64_t)(base - 1) * 16;
    for (int i = 0; i < 8; ++i) { xw[i] = k[i]; yw[i] = k[8 + i]; }
    ok = key_check(xw, yw, bx, by);
  }
  uint32_t* out = tables + (uint64_t)base * kTableWords + (uint64_t)win * kEntries * kEntryWords;
  if (win == 0 && base > 0) valid[base - 1] = ok ? 1u : 0u;
  if (!ok) {
    for (int i = 0; i < kEntries * kEntryWords; ++i) out[i] = 0;
    return;
  }
  fe* sc = scratch + (uint64_t)lane * kScratchSlots;
  build_window(out, (int)win, bx, by, [&](int s, const fe& v) { sc[s] = v; }, [&](int s, fe& v) { v = sc[s]; });
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
                                                       uint32_t* __restrict__ prefix) {
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
      ok = sig_ok(sigs, key_idx, key_valid, nkeys, i, r, s);
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
  fn_inv_mont(inv, acc);
  for (int j = K - 1; j >= 0; --j) {
    const uint64_t i = lane + (uint64_t)j * L;
    const bool ok = (okm >> j) & 1u;
    uint32_t r[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s[8] = {1, 0, 0, 0, 0, 0, 0, 0};
    if (ok) {
      load_be256(sigs + 64 * i, r);
      load_be256(sigs + 64 * i + 32, s);
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
        load_be256(hashes + 32 * i, e);
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
// stage 2: comb.  Signed 8-bit digits are peeled off a 256-bit register
// shift (no runtime-indexed register arrays -> no scratch), and the table
// entry for window i+1 is loaded while window i is being added.
struct digit_stream {
  uint32_t w[8];
  int carry;
  __device__ __forceinline__ int next() {
    const int b = (int)(w[0] & 0xFFu);
    PBFTV_UNROLL for (int j = 0; j < 7; ++j) w[j] = __builtin_amdgcn_alignbit(w[j + 1], w[j], 8);
    w[7] >>= 8;
    const int d = b + carry;
    carry = d > 128 ? 1 : 0;
    return d - (carry << 8);
  }
};

__device__ __forceinline__ void load_entry(const uint4* __restrict__ tab, int win, int d, uint4 e[4]) {
  const int idx = (d < 0 ? -d : d) - 1;
  const uint4* p = tab + ((uint64_t)win * kEntries + (idx < 0 ? 0 : idx)) * 4;
  e[0] = p[0]; e[1] = p[1]; e[2] = p[2]; e[3] = p[3];
}

template <bool kCheck>
__device__ bool comb_dev_pass(jac& acc, const uint32_t u[8], const uint4* __restrict__ tab) {
  digit_stream ds;
  PBFTV_UNROLL for (int j = 0; j < 8; ++j) ds.w[j] = u[j];
  ds.carry = 0;
  int d = ds.next();
  uint4 e[4];
  load_entry(tab, 0, d, e);
  bool inf = true;
  for (int i = 0; i < kWindows; ++i) {
    const int dc = d;
    uint32_t ew[16] = {e[0].x, e[0].y, e[0].z, e[0].w, e[1].x, e[1].y, e[1].z, e[1].w,
                       e[2].x, e[2].y, e[2].z, e[2].w, e[3].x, e[3].y, e[3].z, e[3].w};
    if (i + 1 < kWindows) {
      d = ds.next();
      load_entry(tab, i + 1, d, e);
    }
    if (dc == 0) continue;
    fe x, y;
    entry_to_fe(x, y, ew);
    if (dc < 0) {
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
    if (kCheck) {
      if (st == 1) jac_double(acc, acc);
      else if (st == 2) inf = true;
    }
  }
  return !inf;
}

// unchecked fast pass; a Z == 0 result means some step was exceptional -> rerun checked
__device__ bool comb_dev(jac& acc, const uint32_t u[8], const uint4* __restrict__ tab) {
  const bool ok = comb_dev_pass<false>(acc, u, tab);
  if (ok && fe_is_zero(acc.z)) return comb_dev_pass<true>(acc, u, tab);
  return ok;
}

__global__ void __launch_bounds__(256) k_ecdsa_comb(const uint4* __restrict__ scal, const uint8_t* __restrict__ flag,
                                                    const uint8_t* __restrict__ sigs,
                                                    const uint32_t* __restrict__ key_idx, uint64_t n,
                                                    const uint4* __restrict__ tables, uint8_t* __restrict__ bitmap) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool ok = false;
  if (i < n && flag[i]) {
    const uint4* sp = scal + 4 * i;
    const uint4 a = sp[0], b = sp[1], c = sp[2], dd = sp[3];
    const uint32_t u1[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const uint32_t u2[8] = {c.x, c.y, c.z, c.w, dd.x, dd.y, dd.z, dd.w};
    const uint4* gtab = tables;
    const uint4* qtab = tables + (uint64_t)(key_idx[i] + 1) * (kTableWords / 4);
    jac A, B;
    const bool aok = comb_dev(A, u1, gtab);
    const bool bok = comb_dev(B, u2, qtab);
    uint32_t r[8];
    load_be256(sigs + 64 * i, r);
    ok = ecdsa_final(A, aok, B, bok, r);
  }
  // LSB-first bitmap: wave ballot, lanes 0..7 store one byte each
  const unsigned long long m = __ballot(ok);
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave_base = i - lane;
  if (lane < 8 && wave_base + 8 * lane < n) bitmap[(wave_base >> 3) + lane] = (uint8_t)(m >> (8 * lane));
}

// ---------------------------------------------------------------------------
hipError_t launch_build_tables(const uint32_t* keys_le, uint32_t nkeys, uint32_t* tables, uint32_t* valid,
                               void* scratch, hipStream_t st) {
  const uint32_t lanes = (nkeys + 1) * kWindows;
  hipLaunchKernelGGL(k_build_tables, dim3((lanes + 63) / 64), dim3(64), 0, st, keys_le, nkeys, tables, valid,
                     reinterpret_cast<fe*>(scratch));
  return hipGetLastError();
}

size_t build_tables_scratch_bytes(uint32_t nkeys) {
  return (size_t)(nkeys + 1) * kWindows * kScratchSlots * sizeof(fe);
}

size_t table_bytes_per_base() { return kTableBytes; }

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
                             hipStream_t st) {
  const uint64_t lanes = (n + K - 1) / K;
  const uint64_t blocks = (lanes + 255) / 256;
  hipLaunchKernelGGL(k_ecdsa_scalars<K>, dim3((uint32_t)blocks), dim3(256), 0, st, hashes, sigs, key_idx, n,
                     key_valid, nkeys, reinterpret_cast<uint4*>(scal), flag, prefix);
}

hipError_t launch_ecdsa_scalars(const uint8_t* hashes, const uint8_t* sigs, const uint32_t* key_idx, uint64_t n,
                                const uint32_t* key_valid, uint32_t nkeys, void* scal, uint8_t* flag, void* prefix,
                                hipStream_t st) {
  if (n == 0) return hipSuccess;
  uint32_t* pf = reinterpret_cast<uint32_t*>(prefix);
  switch (scalar_batch(n)) {
    case 1: launch_scalars_k<1>(hashes, sigs, key_idx, n, key_valid, nkeys, scal, flag, pf, st); break;
    case 2: launch_scalars_k<2>(hashes, sigs, key_idx, n, key_valid, nkeys, scal, flag, pf, st); break;
    case 4: launch_scalars_k<4>(hashes, sigs, key_idx, n, key_valid, nkeys, scal, flag, pf, st); break;
    case 8: launch_scalars_k<8>(hashes, sigs, key_idx, n, key_valid, nkeys, scal, flag, pf, st); break;
    default: launch_scalars_k<16>(hashes, sigs, key_idx, n, key_valid, nkeys, scal, flag, pf, st); break;
  }
  return hipGetLastError();
}

hipError_t launch_ecdsa_comb(const void* scal, const uint8_t* flag, const uint8_t* sigs, const uint32_t* key_idx,
                             uint64_t n, const uint32_t* tables, uint8_t* bitmap, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_ecdsa_comb, dim3((uint32_t)blocks), dim3(256), 0, st, reinterpret_cast<const uint4*>(scal),
                     flag, sigs, key_idx, n, reinterpret_cast<const uint4*>(tables), bitmap);
  return hipGetLastError();
}

size_t ecdsa_scratch_bytes(uint64_t n) { return (size_t)n * 64 + (size_t)n; }

}  // namespace pbftv
