// verify_kernels.h -- the per-signature verify kernels (gfx950), shared by the
// instantiation units p256_verify_g*.hip (one per G-table width, so the
// (G, key) geometry pairs of kernels.h PBFTV_COMBOS compile in parallel).
//   k_ecdsa_comb  throughput path: one signature per lane, joint signed-digit
//                 comb over the W-bit tables in signed-limb XYZZ coordinates
//                 (fes.h), x-coordinate check X == r ZZ -- no field inversion.
//   k_ecdsa_wave  latency path (small batches, one quorum certificate): one
//                 WAVE per signature.
// Semantics: Go 1.19 crypto/ecdsa.Verify (p256_algo.h); parity with the oracle
// in tests/test_gpu_parity.py.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "kernels.h"
#include "p256_algo.h"
#include "rows.h"

namespace pbftv {

#ifndef PBFTV_COMB_BLOCK
#define PBFTV_COMB_BLOCK 256  // threads per k_ecdsa_comb block
#endif

#ifndef PBFTV_COMB_WAVES
#define PBFTV_COMB_WAVES 4  // min waves per SIMD for k_ecdsa_comb: 128 VGPRs; +1.2 % over 2 (tools/ab.sh)
#endif

// Stage timing probe (experiment builds only: make EXTRA=-DPBFTV_SCAL_PROBE,
// read by tools/scal_probe.py): lane 0 of each wave stamps wall_clock64() at
// the stage boundaries of k_ecdsa_scalars (slots 0..5) and of
// wave_batch_inv_n (6: scans, 7: safegcd); the asm ties a stamp to the value
// the stage produced.
#ifdef PBFTV_SCAL_PROBE
static __device__ uint64_t g_scal_probe[8192 * 8];
#define PBFTV_SPROBE(k, dep)                                                            \
  do {                                                                                  \
    asm volatile("" ::"v"(dep));                                                        \
    const uint64_t t_ = wall_clock64();                                                 \
    const uint64_t w_ = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;         \
    if ((threadIdx.x & 63u) == 0 && w_ < 8192) g_scal_probe[w_ * 8 + (k)] = t_;         \
  } while (0)
#else
#define PBFTV_SPROBE(k, dep) \
  do {                       \
  } while (0)
#endif

// The row schedule's stage stamps (tools/rows_probe.hip defines
// PBFTV_ROWS_PROBE before including this header): lane 0 of every wave of the
// first 128 workgroups, 16 slots per wave.
#ifdef PBFTV_ROWS_PROBE
static __device__ uint64_t g_rows_probe[128 * 8 * 16];
#define PBFTV_RPROBE(k, dep)                                                                  \
  do {                                                                                        \
    asm volatile("" ::"v"(dep));                                                              \
    const uint64_t t_ = wall_clock64();                                                       \
    if ((threadIdx.x & 63u) == 0 && blockIdx.x < 128)                                         \
      g_rows_probe[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 16 + (k)] = t_;                    \
  } while (0)
#else
#define PBFTV_RPROBE(k, dep) \
  do {                       \
  } while (0)
#endif

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// 32 big-endian bytes at p (16-B aligned) -> 8 LE words
__device__ __forceinline__ void load_be256(const uint8_t* __restrict__ p, uint32_t w[8]) {
  const uint4 a = *reinterpret_cast<const uint4*>(p);
  const uint4 b = *reinterpret_cast<const uint4*>(p + 16);
  w[7] = bswap32(a.x); w[6] = bswap32(a.y); w[5] = bswap32(a.z); w[4] = bswap32(a.w);
  w[3] = bswap32(b.x); w[2] = bswap32(b.y); w[1] = bswap32(b.z); w[0] = bswap32(b.w);
}

// Stage 1 -> stage 2 handoff, one per signature at its position in key order:
// q[0..1] u1, q[2..3] u2, q[4..5] r (LE words), q[6] = {key index, batch
// index, ok, 0}, q[7] unused (a full 128-B line per record).
struct alignas(128) SigRec {
  uint4 q[8];
};

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

// The same digits cut out of an unshifted scalar: with the window index a
// compile-time constant (fully unrolled callers), window i's raw bits are one
// funnel shift of the two words it spans (~6 instructions per window instead
// of stepping the 8-word shift, ~12).
template <int W>
struct digit_cut {
  int carry = 0;
  __device__ __forceinline__ int at(const uint32_t w[8], int i) {
    const int wd = CombGeom<W>::width(i), b = CombGeom<W>::bit(i);
    const int lo = b >> 5, sh = b & 31;
    const uint32_t wlo = lo < 8 ? w[lo] : 0u, whi = lo + 1 < 8 ? w[lo + 1] : 0u;
    const int d = (int)(__builtin_amdgcn_alignbit(whi, wlo, (uint32_t)sh) & ((1u << wd) - 1u)) + carry;
    carry = d > (1 << (wd - 1)) ? 1 : 0;
    return d - (carry << wd);
  }
};

template <int W>
__device__ __forceinline__ void load_entry(const uint4* __restrict__ tab, int win, int d, uint4 e[4]) {
  const int idx = (d < 0 ? -d : d) - 1;
  const uint4* p = tab + (CombGeom<W>::base(win) + (idx < 0 ? 0 : idx)) * 4;
  e[0] = p[0]; e[1] = p[1]; e[2] = p[2]; e[3] = p[3];
}

__device__ __forceinline__ void entry_words(const uint4 e[4], uint32_t ew[16]) {
  PBFTV_UNROLL for (int q = 0; q < 4; ++q) {
    ew[4 * q] = e[q].x; ew[4 * q + 1] = e[q].y; ew[4 * q + 2] = e[q].z; ew[4 * q + 3] = e[q].w;
  }
}

// the complete-addition rerun's step (comb_add_entry<true>)
template <bool kCheck, class Acc>
__device__ __forceinline__ void comb_dev_add(Acc& acc, bool& inf, int d, const uint32_t ew[16]) {
  static_assert(kCheck, "only the complete-addition pass reads entries this way");
  comb_add_entry<true>(acc, inf, d, ew);
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
__device__ __noinline__ bool comb2_checked_verify(const SigRec* __restrict__ rp, const uint4* __restrict__ gtab,
                                                  const uint4* __restrict__ qtab) {
  const uint4 a = rp->q[0], b = rp->q[1], c = rp->q[2], dd = rp->q[3], e = rp->q[4], f = rp->q[5];
  const uint32_t u1[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  const uint32_t u2[8] = {c.x, c.y, c.z, c.w, dd.x, dd.y, dd.z, dd.w};
  const uint32_t r[8] = {e.x, e.y, e.z, e.w, f.x, f.y, f.z, f.w};
  jac R;
  const bool fin = comb2_dev_pass<true, WG, WQ>(R, u1, u2, gtab, qtab);
  return ecdsa_check(R, fin, r);
}

// y = d < 0 ? 2p - y : y, lazily (limbs < 2^30: a valid fe_mul input) -- a
// per-lane mask select, no carry chain and no divergence.
__device__ __forceinline__ void fe_cneg_lazy(fe& y, bool neg) {
  const uint32_t m = 0u - (uint32_t)neg;
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) y.v[l] = y.v[l] ^ ((y.v[l] ^ (kP2Borrow[l] - y.v[l])) & m);
}

template <int W>
__device__ __forceinline__ const uint4* entry_ptr(const uint4* __restrict__ tab, int win, int d) {
  const int idx = (d < 0 ? -d : d) - 1;
  return tab + (CombGeom<W>::base(win) + (idx < 0 ? 0 : idx)) * 4;
}

// Async copy of this lane's 64-B entry into sent[.][t]: four 16-B
// global_load_lds, each writing the wave's 64 lanes contiguously at the
// wave-uniform base &sent[k][t & ~63].
// PBFTV_GATHER_AUX: the loads' cache-policy bits (experiment builds; 2 = nt)
#ifndef PBFTV_GATHER_AUX
#define PBFTV_GATHER_AUX 0
#endif
__device__ __forceinline__ void issue_entry_lds(uint4 (*sent)[PBFTV_COMB_BLOCK], uint32_t t, const uint4* p) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this lane's reads of the slot are done
  const uint32_t wb = t & ~63u;
  __builtin_amdgcn_global_load_lds(p + 0, &sent[0][wb], 16, 0, PBFTV_GATHER_AUX);
  __builtin_amdgcn_global_load_lds(p + 1, &sent[1][wb], 16, 0, PBFTV_GATHER_AUX);
  __builtin_amdgcn_global_load_lds(p + 2, &sent[2][wb], 16, 0, PBFTV_GATHER_AUX);
  __builtin_amdgcn_global_load_lds(p + 3, &sent[3][wb], 16, 0, PBFTV_GATHER_AUX);
}

__device__ __forceinline__ void read_entry_lds(uint4 (*sent)[PBFTV_COMB_BLOCK], uint32_t t, uint32_t ew[16]) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's copies have landed
  uint4 e[4];
  PBFTV_UNROLL for (int k = 0; k < 4; ++k) e[k] = sent[k][t];
  entry_words(e, ew);
}


// ---- a certificate's CU, yielded by the batch waves beside it (round 6) ----
// An armed workgroup shares its CU with comb waves of any batch in flight:
// its issue priority (s_setprio 3) wins the arbitration but not the VALU
// cycles a comb wave's 64-bit MADs already hold, nor the instruction cache.
// While it serves, the armed workgroup raises its CU's word in a per-device
// flag array (kernels.h kCuFlagWords; index from the hardware IDs: XCC, SE,
// SH, CU), and a comb wave on that CU parks (s_sleep) at its next step
// boundary until the word drops -- at most kCuParkTicks, so a word left set
// cannot hold a batch.  Only the CUs that serve pay: ~20 µs of their comb
// waves per certificate.
constexpr uint64_t kCuParkTicks = 5000;  // wall clock (100 MHz): 50 µs
__device__ __forceinline__ uint32_t cu_flag_index() {
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  return ((xcc & 15u) << 8) | ((hw >> 8) & 0xFFu);  // CU_ID, SH_ID, SE_ID of this XCC
}
// the armed side: wave 0 raises its CU's word (and the partner's) as soon as
// it has a signature to serve, and drops it after the verdict
__device__ __forceinline__ void raise_cu_flags(uint32_t* f, uint32_t* f2) {
  if (f && (threadIdx.x & 63u) == 0) {
    __hip_atomic_fetch_add(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (f2) __hip_atomic_fetch_add(f2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ void comb_park(const uint32_t* f) {
  const uint64_t t0 = wall_clock64();
  do {
    __builtin_amdgcn_s_sleep(4);
  } while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0 &&
           wall_clock64() - t0 < kCuParkTicks);
}

template <int WG, int WQ>
__global__ void __launch_bounds__(PBFTV_COMB_BLOCK, PBFTV_COMB_WAVES) k_ecdsa_comb(const SigRec* __restrict__ rec, uint64_t n,
                                                                    const uint4* __restrict__ gtab,
                                                                    const uint4* const* __restrict__ qtabs,
                                                                    uint8_t* __restrict__ bitmap,
                                                                    uint8_t* __restrict__ okb,
                                                                    const uint32_t* __restrict__ cuflag) {
  using S = CombSteps<WG, WQ>;
  // signed digits of u1 / u2 in step order, one column per thread: recoded once
  // in the prologue so the main loop holds no 256-bit digit shift registers
  __shared__ typename S::Digit sdig[S::nD][PBFTV_COMB_BLOCK];
  // the table entry of the next step, streamed global -> LDS (no VGPRs held
  // while it is in flight): piece k of thread t at sent[k][t]
  __shared__ uint4 sent[4][PBFTV_COMB_BLOCK];
  const uint32_t t = threadIdx.x;
  // lane p reads record p: with a key order (k_key_*) the p-th signature by key,
  // written there by stage 1 (coalesced: no gather through a permutation)
  // XCD-aware record ranges: the dispatcher deals blocks round-robin over the
  // 8 XCDs (block b -> XCD b % 8), so XCD x is given the x-th eighth of the
  // key-ordered records and its L2 and TLBs see ~1/8 of the keys (blocks past
  // the last multiple of 8 keep their index).  Same box, 3 rounds: comb
  // 0.9447 -> 0.9377 ms, step 1.0985 -> 1.0845 ms at 1M.
  const uint32_t nb = gridDim.x, b = blockIdx.x, per = nb / 8;
  const uint32_t blk = b < 8 * per ? (b % 8) * per + b / 8 : b;
  const uint64_t p = (uint64_t)blk * blockDim.x + t;
  const SigRec* rp = rec + p;
  uint4 meta = make_uint4(0, 0, 0, 0);  // key, batch index, ok
  if (p < n) meta = rp->q[6];
  bool ok = false;
  // Every lane runs the step loop (no divergence around the wave-wide entry
  // loads; comb -0.8 % same box); a lane without a valid signature has
  // all-zero digits, reads entry 0 of the G table and adds nothing.
  const bool act = meta.z != 0;
  {
    uint4 a = make_uint4(0, 0, 0, 0), b = a, c = a, dd = a;
    if (act) {
      a = rp->q[0];
      b = rp->q[1];
      c = rp->q[2];
      dd = rp->q[3];
    }
    const uint32_t w1[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const uint32_t w2[8] = {c.x, c.y, c.z, c.w, dd.x, dd.y, dd.z, dd.w};
    digit_cut<WG> s1;
    digit_cut<WQ> s2;
    PBFTV_UNROLL for (int j = 0; j < S::nD; ++j)
      sdig[j][t] = (typename S::Digit)((S::is_q(j) ? s2.at(w2, S::win(j)) : s1.at(w1, S::win(j))) - 1);
  }
  const uint4* qtab = act ? qtabs[meta.x] : gtab;  // the key's own table allocation
  xyzz_s R;  // signed-limb accumulator (fes.h); R.y holds sigma Y (xyzz_madd_s_flip)
  bool inf = true, neg_y = false;  // neg_y: sigma = -1
  // The schedule of p256_algo.h comb2_verify, chosen per WAVE: the first two
  // points are added affine + affine and the last addition is fused with the
  // x check unless a lane with a signature has a zero digit there (~2^-20 per
  // signature: then the whole wave takes the generic steps, which are exact
  // for every digit pattern).  Lanes without a signature have zero digits and
  // compute on entry 0, unread.
  const int d0 = (int)sdig[0][t] + 1, d1 = (int)sdig[1][t] + 1;
  const bool first2 = __ballot(act && (d0 == 0 || d1 == 0)) == 0;
  const bool fuse = first2 && __ballot(act && sdig[S::nD - 1][t] == -1) == 0;
  int d, j0;
  if (first2) {
    // both entries straight into registers (one memory round trip for the two),
    // step 2's entry into LDS behind them
    const uint4* p0 = entry_ptr<WG>(gtab, 0, d0);
    const uint4* p1 = entry_ptr<WQ>(qtab, 0, d1);
    uint4 e0[4], e1[4];
    PBFTV_UNROLL for (int k = 0; k < 4; ++k) {
      e0[k] = p0[k];
      e1[k] = p1[k];
    }
    d = (int)sdig[2][t] + 1;
    issue_entry_lds(sent, t, S::is_q(2) ? entry_ptr<WQ>(qtab, S::win(2), d) : entry_ptr<WG>(gtab, S::win(2), d));
    uint32_t w0[16], w1[16];
    entry_words(e0, w0);
    entry_words(e1, w1);
    comb_first2_s(R, neg_y, d0, w0, d1, w1);
    inf = false;
    j0 = 2;
  } else {
    d = d0;
    issue_entry_lds(sent, t, entry_ptr<WG>(gtab, 0, d));
    j0 = 0;
  }
  const int jend = fuse ? S::nD - 1 : S::nD;
#ifndef PBFTV_COMB_UNROLL
#define PBFTV_COMB_UNROLL 1
#endif
  const uint32_t* cuf = cuflag ? cuflag + cu_flag_index() : nullptr;  // (uniform)
#pragma unroll PBFTV_COMB_UNROLL
  for (int j = j0; j < jend; ++j) {
    uint32_t w16[16];
    read_entry_lds(sent, t, w16);
    const int dc = d;
    // this CU's certificate word, read behind the step (issued before the
    // entry loads, so its wait does not wait for them)
    const uint32_t cf = cuf ? __hip_atomic_load(cuf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    if (j + 1 < S::nD) {  // next step's entry streams into LDS during this addition
      d = (int)sdig[j + 1][t] + 1;
      issue_entry_lds(sent, t, S::is_q(j + 1) ? entry_ptr<WQ>(qtab, S::win(j + 1), d)
                                              : entry_ptr<WG>(gtab, S::win(j + 1), d));
    }
    comb_step_s(R, inf, neg_y, dc, w16);
    if (cuf && __builtin_amdgcn_readfirstlane(cf) != 0) comb_park(cuf);
  }
  if (act) {
    const uint4 e = rp->q[4], f = rp->q[5];
    const uint32_t r[8] = {e.x, e.y, e.z, e.w, f.x, f.y, f.z, f.w};
    int res;
    if (fuse) {
      uint32_t w16[16];
      read_entry_lds(sent, t, w16);  // the last step's entry
      res = comb_last_check_s(R, neg_y, d, w16, r);
    } else {
      res = (!inf && fs_is_zero(R.zz)) ? -1 : (ecdsa_check(R, !inf, r) ? 1 : 0);
    }
    // exceptional step: redo with complete additions
    ok = res < 0 ? comb2_checked_verify<WG, WQ>(rp, gtab, qtab) : res == 1;
  }
  if (okb != nullptr) {  // key order: one byte at the signature's own index, k_pack_bits builds the bitmap
    if (p < n) okb[meta.y] = ok ? 1 : 0;
    return;
  }
  // arrival order: LSB-first bitmap by wave ballot, lanes 0..7 store one byte each
  const unsigned long long m = __ballot(ok);
  const uint32_t lane = t & 63u;
  const uint64_t wave_base = p - lane;
  if (lane < 8 && wave_base + 8 * lane < n) bitmap[(wave_base >> 3) + lane] = (uint8_t)(m >> (8 * lane));
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
  const int j = (int)(threadIdx.x & 63u);  // (the armed kernel runs four waves per workgroup)
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
  const bool b0 = (role & 1) != 0, b1 = (role & 2) != 0;  // three v_cndmask per limb
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) {
    const uint32_t lo = b0 ? a1.v[l] : a0.v[l], hi = b0 ? a3.v[l] : a2.v[l];
    d.v[l] = b1 ? hi : lo;
  }
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
  fs_mul(p, a, b);  // signed-limb product (fes.h): operands S- or D-type
}

// (gx, gy) + (qx, qy), both affine S-type, into XYZZ (mmadd-2008-s, 3 steps).  Signed-limb arithmetic (fes.h): differences
// are D-type, X3 is renormalised (S), Y3 stays D-type (only multiplied later).
// The idle lane of step 3 computes rz = rm ZZ3 (r ZZ in Montgomery form, for
// the fused check of the last level).
__device__ __forceinline__ void quad_mmadd_xyzz(xyzz_s& r, fe& rz, int role, const fe& gx, const fe& gy,
                                                const fe& qx, const fe& qy, const fe& rm) {
  fe p, rr, pp, r2, ppp, qq, x3, t, a, b, prod;
  fs_sub(p, qx, gx);
  fs_sub(rr, qy, gy);
  // (x-coordinates meeting: PP = 0 = ZZ3, tested at the top of the tree)
  quad_mul(prod, role, p, p, rr, rr, p, p, rr, rr);          // PP, R^2
  quad_bcast<0>(pp, prod);
  quad_bcast<1>(r2, prod);
  quad_mul(prod, role, p, pp, gx, pp, p, pp, gx, pp);        // PPP, Q = X1 PP
  quad_bcast<0>(ppp, prod);
  quad_bcast<1>(qq, prod);
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) x3.v[i] = r2.v[i] - ppp.v[i] - (qq.v[i] << 1);
  fs_norm(x3, x3);                                           // X3 = R^2 - PPP - 2Q
  fs_sub(t, qq, x3);
  quad_mul(prod, role, rr, t, gy, ppp, rm, pp, rm, pp);      // R (Q - X3), Y1 PPP, r ZZ3
  quad_bcast<0>(a, prod);
  quad_bcast<1>(b, prod);
  quad_bcast<2>(rz, prod);
  fs_sub(r.y, a, b);
  r.x = x3;
  r.zz = pp;
  r.zzz = ppp;
}

// r = P + Q (both finite XYZZ: X, ZZ, ZZZ S-type, Y S- or D-type), add-2008-s
// in 4 steps of <= 4 products (the Jacobian quad_jadd needs 5); exc if the
// x-coordinates meet (P == 0).  The idle lane of step 4 computes rz = rm ZZ
// of the level's result: of r, or of Q / P when the other side is infinity
// (pinf / qinf), so r ZZ needs no shuffle of its own.
__device__ __forceinline__ void quad_xyzz_add(xyzz_s& r, fe& rz, int role, const xyzz_s& P, const xyzz_s& Q,
                                              const fe& rm, bool qinf) {
  fe prod, u1, u2, s1, s2, p, rr, pp, r2, zz12, zzz12, ppp, qq, x3, t, a, b;
  quad_mul(prod, role, P.x, Q.zz, Q.x, P.zz, P.y, Q.zzz, Q.y, P.zzz);      // U1, U2, S1, S2
  quad_bcast<0>(u1, prod);
  quad_bcast<1>(u2, prod);
  quad_bcast<2>(s1, prod);
  quad_bcast<3>(s2, prod);
  fs_sub(p, u2, u1);
  fs_sub(rr, s2, s1);  // (P == 0 -- a doubling or cancellation -- leaves ZZ3 = 0: the caller tests ZZ once)
  quad_mul(prod, role, p, p, rr, rr, P.zz, Q.zz, P.zzz, Q.zzz);             // PP, R^2, ZZ1 ZZ2, ZZZ1 ZZZ2
  quad_bcast<0>(pp, prod);
  quad_bcast<1>(r2, prod);
  quad_bcast<2>(zz12, prod);
  quad_bcast<3>(zzz12, prod);
  quad_mul(prod, role, p, pp, u1, pp, zz12, pp, zz12, pp);                  // PPP, Q = U1 PP, ZZ3
  quad_bcast<0>(ppp, prod);
  quad_bcast<1>(qq, prod);
  quad_bcast<2>(r.zz, prod);
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) x3.v[i] = r2.v[i] - ppp.v[i] - (qq.v[i] << 1);
  fs_norm(x3, x3);                                                          // X3 = R^2 - PPP - 2Q
  fs_sub(t, qq, x3);
  fe zsel;
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) zsel.v[l] = qinf ? P.zz.v[l] : r.zz.v[l];  // the ZZ the quad keeps
  quad_mul(prod, role, rr, t, s1, ppp, zzz12, ppp, rm, zsel);               // R (Q - X3), S1 PPP, ZZZ3, r ZZ
  quad_bcast<0>(a, prod);
  quad_bcast<1>(b, prod);
  quad_bcast<2>(r.zzz, prod);
  quad_bcast<3>(rz, prod);
  fs_sub(r.y, a, b);                                                        // Y3 = R (Q - X3) - S1 PPP
  r.x = x3;
}

// The last level fused with Go's x-coordinate check (no Y3, ZZZ3, or product
// with r afterwards): with rz = r ZZ1 from the previous level,
//   X3 == r ZZ3  <=>  R^2 - PP (P + 2 U1) == (r ZZ1) ZZ2 PP  <=>  R^2 == PP (P + 2 U1 + rz ZZ2),
// three steps instead of four plus one.  Only for the test against r (the
// caller takes the full path when r + n < p also has to be tried).  exc: this
// level's P == 0, or r ZZ1 ZZ2 == 0 -- i.e. ZZ1 ZZ2 == 0 (0 < r < n < p): an
// exceptional addition anywhere below left a zero ZZ, which every later
// product keeps (one test for the whole tree).
__device__ __forceinline__ bool quad_xyzz_add_check(bool& exc, int role, const xyzz_s& P, const xyzz_s& Q,
                                                    const fe& rz) {
  fe prod, u1, u2, s1, s2, p, rr, pp, r2, rz12, w, t, d;
  quad_mul(prod, role, P.x, Q.zz, Q.x, P.zz, P.y, Q.zzz, Q.y, P.zzz);      // U1, U2, S1, S2
  quad_bcast<0>(u1, prod);
  quad_bcast<1>(u2, prod);
  quad_bcast<2>(s1, prod);
  quad_bcast<3>(s2, prod);
  fs_sub(p, u2, u1);
  fs_sub(rr, s2, s1);
  exc = fs_is_zero(p);
  quad_mul(prod, role, p, p, rr, rr, rz, Q.zz, rz, Q.zz);                   // PP, R^2, r ZZ1 ZZ2
  quad_bcast<0>(pp, prod);
  quad_bcast<1>(r2, prod);
  quad_bcast<2>(rz12, prod);
  exc = exc || fs_is_zero(rz12);
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) w.v[i] = (u1.v[i] << 1) + rz12.v[i];
  fs_norm(w, w);
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) w.v[i] += p.v[i];                // P + 2 U1 + r ZZ12: |limbs| < 2^30
  fs_mul(t, pp, w);
  fs_sub(d, r2, t);
  return fs_is_zero(d);
}

__device__ __forceinline__ bool wave_check(const xyzz_s& P, bool finite, const fe& rm, const fe& rnm, bool rn_ok);

// Signed digit of window q (this lane's quad) of a uniform 256-bit scalar u,
// equal to the q-th digit_stream<W>::next() -- without walking the lower
// windows: the lane cuts its window's raw bits out of u (a funnel shift of the
// two words it spans), and the recoding carries come from one wave-wide
// carry-lookahead on ballots: window k generates a carry when raw_k > 2^(w-1)
// and propagates the incoming one when raw_k == 2^(w-1), so with G / P those
// masks at bit 4k (lane 4k of each quad) and bits 4k+1..4k+3 set to
// "propagate", the carries into every window are (G + (G|P)) ^ G ^ (G|P), one
// 64-bit add (~30 instructions per scalar instead of the ~130 of stepping the
// 256-bit shift through the lower windows).  Every lane of the wave must call it.
template <int W>
__device__ __forceinline__ int lane_window_digit(const uint32_t u[8], int q) {
  using Gm = CombGeom<W>;
  const bool valid = q < Gm::kWin;
  const int qq = valid ? q : 0;
  const int bit = Gm::bit(qq), wd = Gm::width(qq);
  const int wi = bit >> 5, sh = bit & 31;
  uint32_t lo = 0, hi = 0;
  PBFTV_UNROLL for (int k = 0; k < 8; ++k) {
    lo = wi == k ? u[k] : lo;
    hi = wi + 1 == k ? u[k] : hi;
  }
  uint32_t raw = __builtin_amdgcn_alignbit(hi, lo, (uint32_t)sh) & ((1u << wd) - 1u);
  if (!valid) raw = 0;
  const uint32_t half = 1u << (wd - 1);
  constexpr uint64_t kQuad0 = 0x1111111111111111ull;
  const uint64_t G = __ballot(raw > half) & kQuad0;
  const uint64_t B = G | (__ballot(raw == half) & kQuad0) | ~kQuad0;
  const uint64_t C = (G + B) ^ G ^ B;  // carry into every bit
  const int d = (int)raw + (int)((C >> (4 * q)) & 1u);
  return d - ((d > (int)half ? 1 : 0) << wd);
}

// quad q = window q: G entry + Q entry, then a butterfly over the quads; the
// last level fused with the check against r (quad_xyzz_add_check) unless
// r + n < p (then the full sum and wave_check).  exc reports a doubling /
// cancellation anywhere (the caller reruns the signature with wave_sum_lanes).
// Every lane returns the verdict.
template <int WG, int WQ>
__device__ __forceinline__ bool wave_verify_quads(bool& exc, const uint32_t u1[8], const uint32_t u2[8],
                                                  const uint4* __restrict__ gtab, const uint4* __restrict__ qtab,
                                                  const fe& rm, const fe& rnm, bool rn_ok) {
  constexpr int nG = CombGeom<WG>::kWin, nQ = CombGeom<WQ>::kWin;
  constexpr int nW = nG > nQ ? nG : nQ;
  static_assert(nW > 8 && nW <= 16, "one quad per window, four butterfly levels");
  const int role = (int)(threadIdx.x & 3u), q = (int)((threadIdx.x & 63u) >> 2);
  const int d1 = lane_window_digit<WG>(u1, q), d2 = lane_window_digit<WQ>(u2, q);
  uint4 eg[4], eq[4];
  uint32_t w16[16];
  load_entry<WG>(gtab, q < nG ? q : 0, d1, eg);
  load_entry<WQ>(qtab, q < nQ ? q : 0, d2, eq);
  fe gx, gy, qx, qy;
  entry_words(eg, w16);
  entry_to_fe(gx, gy, w16);
  fs_cneg(gy, gy, d1 < 0);
  fs_norm(gy, gy);  // S-type: R = qy - gy must stay D-type
  entry_words(eq, w16);
  entry_to_fe(qx, qy, w16);
  fs_cneg(qy, qy, d2 < 0);
  fs_norm(qy, qy);
  xyzz_s S, P;
  fe rz, rzS;
  quad_mmadd_xyzz(S, rzS, role, gx, gy, qx, qy, rm);  // every quad runs it; selected below
  // A window with two zero digits (probability ~2^-50) would be an infinite
  // partial sum inside the tree: left to the exact rerun.  (A level-0 meeting,
  // P == 0, leaves S.zz = PP = 0 and is caught by the ZZ test at the top.)
  const bool live = q < nW;  // quads past the last window hold no point
  bool rare = live && d1 == 0 && d2 == 0;
  const bool both = d1 != 0 && d2 != 0, g_only = d1 != 0;
  fe one;
  fe_set(one, kOneP);
  fe_sel3(P.x, both, S.x, g_only, gx, qx);
  fe_sel3(P.y, both, S.y, g_only, gy, qy);
  fe_sel3(P.zz, both, S.zz, true, one, one);
  fe_sel3(P.zzz, both, S.zzz, true, one, one);
  fe_sel3(rz, both, rzS, true, rm, rm);  // a lone table point: ZZ = 1, r ZZ = rm
  // Butterfly over the quads.  Only quad 0's result is read (its lanes report
  // the verdict), and the partial sums it depends on are those of the quads
  // that are multiples of 2m at level m, each adding quad q + m.  For those a
  // partner past the last window (q + m >= nW) is the point at infinity --
  // known statically -- and the quad keeps its sum; the partner of a live
  // quad is never live-but-infinite (rare windows go to the rerun), so no
  // infinity flags travel and the only select is "keep or take the sum".
  // The other quads compute don't-care values.
#pragma unroll 1
  for (int m = 1; m < 16; m <<= 1) {
    xyzz_s Q;
    shfl_xor_fe(Q.x, P.x, 4 * m);
    shfl_xor_fe(Q.y, P.y, 4 * m);
    shfl_xor_fe(Q.zz, P.zz, 4 * m);
    shfl_xor_fe(Q.zzz, P.zzz, 4 * m);
    const bool qinf = (q ^ m) >= nW;
    if (m == 8 && !rn_ok) {  // last level, fused with the check (rn_ok is wave-uniform); quad 8 < nW is live
      bool e = false;
      const bool ok = quad_xyzz_add_check(e, role, P, Q, rz);
      exc = __any(rare || (q == 0 && e));
      return ok;
    }
    quad_xyzz_add(S, rz, role, P, Q, rm, qinf);
    PBFTV_UNROLL for (int l = 0; l < 9; ++l) {
      P.x.v[l] = qinf ? P.x.v[l] : S.x.v[l];
      P.y.v[l] = qinf ? P.y.v[l] : S.y.v[l];
      P.zz.v[l] = qinf ? P.zz.v[l] : S.zz.v[l];
      P.zzz.v[l] = qinf ? P.zzz.v[l] : S.zzz.v[l];
    }
  }
  exc = __any(rare || (q == 0 && fs_is_zero(P.zz)));  // r + n < p: the full sum, its ZZ tested once
  return wave_check(P, true, rm, rnm, rn_ok);
}

// ---- latency-path scalars: the inversion spread over the wave --------------
// Bernstein-Yang safegcd (safegcd.h) with the work split by kind: the 30
// divsteps of a batch are a short serial chain on the low 30 bits of (f, g)
// and run on the SCALAR unit (uniform operands from v_readlane), while the
// 2x2 matrix update of the 270-bit (f, g) and (d, e) is one LANE PER LIMB:
//   lanes 0..8   limb L of f (A) and g (B)       (row 0 of the DPP rows)
//   lanes 16..24 limb L of d (A) and e (B) mod n (row 1)
// Limbs are 30-bit signed, kept centered (|limb| <= 2^29 + 2; the top limb is
// free), so u A + v B + md n_L stays below 2^60 in magnitude and the shifted
// limbs fit int32; the division by 2^30 moves each limb's low part one lane
// down (DPP row_shl:1) and a centered carry pass moves carries one lane up
// (row_shr:1).  md is the centered multiple of n that makes (d, e)'s low limb
// vanish; without the sign-dependent range keeping of update_de30, |d| grows by
// at most n/2 per batch (< 13.5 n after 25 batches; tests/test_algo_cpu.py
// emulates the scheme and checks every bound).  e starts at R mod n, so the
// result is R s^-1 (Montgomery form for the u1 / u2 products, no extra one).
__device__ __forceinline__ int32_t lane_from_next(int32_t x) {  // lane j <- lane j + 1 of its row (0 past the row)
  return __builtin_amdgcn_mov_dpp(x, 0x101, 0xF, 0xF, true);
}
__device__ __forceinline__ int32_t lane_from_prev(int32_t x) {  // lane j <- lane j - 1 of its row (0 before it)
  return __builtin_amdgcn_mov_dpp(x, 0x111, 0xF, 0xF, true);
}

__device__ __forceinline__ int32_t center30(uint32_t x) { return (int32_t)(x << 2) >> 2; }

// divsteps30_var (safegcd.h) shaped for the scalar unit, where every
// instruction of the one wave costs an issue slot: a lone wave issues one
// scalar instruction per ~4.2 cycles and a conditional branch, taken or not,
// costs ~24 (tools/divstep_lat.hip, profiles/r06_divstep_lat.json), so the
// inversion's latency is its instruction count plus its branches.
//
// Hand-scheduled SALU (PBFTV_DIVSTEP_ASM, the default; the C++ form below is
// the reference and the fallback), per common elimination step (a swap: 134
// of ~141 per inversion) 24 instructions and ONE branch:
//   STEP  z = min(ctz(g), i) (s_ff1 gives -1 for g == 0); the s_min's SCC is
//         "ctz(g) < i" (the batch goes on), an s_cselect keeps e1 = eta + 1
//         then and 0xFFFFFFFF otherwise, and after the shifts SCC = (that <= z)
//         is "goes on AND swaps" -- the only branch.  Anything else (the
//         batch's end, a step without a swap, a batch's first step with
//         e1 < 0) takes the rare path, which tests exactly.
//   SWAP  no register moves and no negations: the registers hold the f row
//         (f, u, v) times s_f and the g row (g, q, r) times s_g, and the swap
//         (f, g, u, v, q, r) <- (g, -f, q, r, -u, -v) exchanges the register
//         roles (copy A <-> B) and turns (s_f, s_g) into (s_g, -s_f).  Four
//         states S0 = A(+,+), S1 = B(+,-), S2 = A(-,-), S3 = B(-,+), one copy
//         of the step each, fall through S0 -> S1 -> S2 -> S3, back edge to
//         S0's swap.  What a swap still does: e1 <- 2 - e1 and nfi.
//   ELIM  w = (g nfi) & bfm(min(e1, i, 6)), g += s w, q += s u w, r += s v w
//         with s = s_f s_g (s_add or s_sub by state) and nfi = s (-f^-1 mod
//         64) from the Newton step f (f f - 2) (or f (2 - f f)).
// The exit block of each state restores the signs and the registers.
// 141 steps: 22.4k cycles -> ~19.2k; the whole inversion 30.5k -> 25.4k with
// inv_mod_n_wave's leaner batch below (bit-identical D over 256 inputs).
// Scalar ALU only: no scalar memory access of any kind.
#ifndef PBFTV_DIVSTEP_ASM
#define PBFTV_DIVSTEP_ASM 1
#endif
#if PBFTV_DIVSTEP_ASM
#define PBFTV_DS_STEP(G, U, V)                    \
  "s_ff1_i32_b32 %[z], " G "\n"                   \
  "s_min_u32 %[z], %[z], %[i]\n"                  \
  "s_cselect_b32 %[k], %[e1], -1\n"               \
  "s_lshr_b32 " G ", " G ", %[z]\n"               \
  "s_lshl_b32 " U ", " U ", %[z]\n"               \
  "s_lshl_b32 " V ", " V ", %[z]\n"               \
  "s_sub_i32 %[e1], %[e1], %[z]\n"                \
  "s_sub_u32 %[i], %[i], %[z]\n"                  \
  "s_cmp_le_u32 %[k], %[z]\n"
#define PBFTV_DS_SWAPIN(F, NFI)                   \
  "s_sub_i32 %[e1], 2, %[e1]\n"                   \
  "s_mul_i32 %[w], " F ", " F "\n"                \
  NFI                                             \
  "s_mul_i32 %[nfi], %[w], " F "\n"
#define PBFTV_DS_NFI_POS "s_add_i32 %[w], %[w], -2\n"
#define PBFTV_DS_NFI_NEG "s_sub_i32 %[w], 2, %[w]\n"
#define PBFTV_DS_ELIM(F, G, U, V, Q, R, OP)       \
  "s_mul_i32 %[w], " G ", %[nfi]\n"               \
  "s_min_u32 %[m], %[e1], %[i]\n"                 \
  "s_min_u32 %[m], %[m], 6\n"                     \
  "s_bfm_b32 %[m], %[m], 0\n"                     \
  "s_and_b32 %[w], %[w], %[m]\n"                  \
  "s_mul_i32 %[m], " F ", %[w]\n"                 \
  "s_mul_i32 %[t2], " U ", %[w]\n"                \
  "s_mul_i32 %[t3], " V ", %[w]\n"                \
  OP " " G ", " G ", %[m]\n"                      \
  OP " " Q ", " Q ", %[t2]\n"                     \
  OP " " R ", " R ", %[t3]\n"
#define PBFTV_DS_ELIM_(...) PBFTV_DS_ELIM(__VA_ARGS__)
// register roles: copy A = (f, g, u, v, q, r), copy B = (g, f, q, r, u, v)
#define PBFTV_DS_A "%[f]", "%[g]", "%[u]", "%[v]", "%[q]", "%[r]"
#define PBFTV_DS_B "%[g]", "%[f]", "%[q]", "%[r]", "%[u]", "%[v]"
#define PBFTV_DS_RARE(K, NEXT, ELIM)              \
  ".Lr" K "_%=:\n"                                \
  "s_cmp_eq_u32 %[i], 0\n"                        \
  "s_cbranch_scc1 .Lx" K "_%=\n"                  \
  "s_cmp_lt_i32 %[e1], 1\n"                       \
  "s_cbranch_scc1 .Ll" NEXT "_%=\n"               \
  ELIM                                            \
  "s_branch .Le" K "_%=\n"

__device__ __forceinline__ int32_t divsteps30_scalar(int32_t eta, uint32_t f, uint32_t g, trans30& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1, i = 30, z, w, m, t2, t3, k;
  uint32_t e1 = (uint32_t)(eta + 1);
  uint32_t nfi = f * (f * f - 2u);  // -f^-1 mod 64 (Newton step from f f = 1 mod 8)
  asm volatile(
      PBFTV_DS_STEP("%[g]", "%[u]", "%[v]")  // entry: a step in S0
      "s_cbranch_scc0 .Lr0_%=\n"
      ".Ll1_%=:\n" PBFTV_DS_SWAPIN("%[g]", PBFTV_DS_NFI_NEG) PBFTV_DS_ELIM_(PBFTV_DS_B, "s_sub_u32")
      ".Le1_%=:\n" PBFTV_DS_STEP("%[f]", "%[q]", "%[r]")
      "s_cbranch_scc0 .Lr1_%=\n"
      ".Ll2_%=:\n" PBFTV_DS_SWAPIN("%[f]", PBFTV_DS_NFI_POS) PBFTV_DS_ELIM_(PBFTV_DS_A, "s_add_u32")
      ".Le2_%=:\n" PBFTV_DS_STEP("%[g]", "%[u]", "%[v]")
      "s_cbranch_scc0 .Lr2_%=\n"
      ".Ll3_%=:\n" PBFTV_DS_SWAPIN("%[g]", PBFTV_DS_NFI_NEG) PBFTV_DS_ELIM_(PBFTV_DS_B, "s_sub_u32")
      ".Le3_%=:\n" PBFTV_DS_STEP("%[f]", "%[q]", "%[r]")
      "s_cbranch_scc0 .Lr3_%=\n"
      ".Ll0_%=:\n" PBFTV_DS_SWAPIN("%[f]", PBFTV_DS_NFI_POS) PBFTV_DS_ELIM_(PBFTV_DS_A, "s_add_u32")
      ".Le0_%=:\n" PBFTV_DS_STEP("%[g]", "%[u]", "%[v]")
      "s_cbranch_scc1 .Ll1_%=\n"
      PBFTV_DS_RARE("0", "1", PBFTV_DS_ELIM_(PBFTV_DS_A, "s_add_u32"))
      PBFTV_DS_RARE("1", "2", PBFTV_DS_ELIM_(PBFTV_DS_B, "s_sub_u32"))
      PBFTV_DS_RARE("2", "3", PBFTV_DS_ELIM_(PBFTV_DS_A, "s_add_u32"))
      PBFTV_DS_RARE("3", "0", PBFTV_DS_ELIM_(PBFTV_DS_B, "s_sub_u32"))
      ".Lx1_%=:\n"  // ended in S1 = B(+,-): u = q', v = r', q = -u', r = -v'
      "s_mov_b32 %[w], %[u]\n"
      "s_mov_b32 %[u], %[q]\n"
      "s_sub_u32 %[q], 0, %[w]\n"
      "s_mov_b32 %[w], %[v]\n"
      "s_mov_b32 %[v], %[r]\n"
      "s_sub_u32 %[r], 0, %[w]\n"
      "s_branch .Lx0_%=\n"
      ".Lx2_%=:\n"  // S2 = A(-,-)
      "s_sub_u32 %[u], 0, %[u]\n"
      "s_sub_u32 %[v], 0, %[v]\n"
      "s_sub_u32 %[q], 0, %[q]\n"
      "s_sub_u32 %[r], 0, %[r]\n"
      "s_branch .Lx0_%=\n"
      ".Lx3_%=:\n"  // S3 = B(-,+): u = -q', v = -r', q = u', r = v'
      "s_mov_b32 %[w], %[u]\n"
      "s_sub_u32 %[u], 0, %[q]\n"
      "s_mov_b32 %[q], %[w]\n"
      "s_mov_b32 %[w], %[v]\n"
      "s_sub_u32 %[v], 0, %[r]\n"
      "s_mov_b32 %[r], %[w]\n"
      ".Lx0_%=:\n"
      : [f] "+s"(f), [g] "+s"(g), [u] "+s"(u), [v] "+s"(v), [q] "+s"(q), [r] "+s"(r), [e1] "+s"(e1),
        [i] "+s"(i), [nfi] "+s"(nfi), [z] "=&s"(z), [w] "=&s"(w), [m] "=&s"(m), [t2] "=&s"(t2), [t3] "=&s"(t3),
        [k] "=&s"(k)
      :
      : "scc");
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return (int32_t)e1 - 1;
}
#undef PBFTV_DS_STEP
#undef PBFTV_DS_SWAPIN
#undef PBFTV_DS_NFI_POS
#undef PBFTV_DS_NFI_NEG
#undef PBFTV_DS_ELIM
#undef PBFTV_DS_ELIM_
#undef PBFTV_DS_A
#undef PBFTV_DS_B
#undef PBFTV_DS_RARE
#else
__device__ __forceinline__ int32_t divsteps30_scalar(int32_t eta, uint32_t f, uint32_t g, trans30& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  uint32_t nfi = f * (f * f - 2u);  // -f^-1 mod 64 (Newton step from f f = 1 mod 8)
  int i = 30;
  int z = __builtin_ctz(g | (0xFFFFFFFFu << i));
  for (;;) {
    g >>= z;
    u <<= z;
    v <<= z;
    eta -= z;
    i -= z;
    if (i == 0) break;
    if (eta < 0) {  // delta > 0: (f, g) <- (g, -f)
      eta = -eta;
      const uint32_t x = f, y = u, w = v;
      f = g;
      g = 0u - x;
      u = q;
      q = 0u - y;
      v = r;
      r = 0u - w;
      nfi = f * (f * f - 2u);
    }
    const int lim = min(eta + 1, i);  // the 6-bit cap is the & 63 (nfi is exact mod 64)
    const uint32_t w = (g * nfi) & ((1u << lim) - 1u) & 63u;  // -g / f mod 2^min(lim, 6)
    g += f * w;
    q += u * w;
    r += v * w;
    z = __builtin_ctz(g | (0xFFFFFFFFu << i));
  }
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return eta;
}
#endif

// limb re-centering: carry (x + 2^29) >> 30 one lane up (not out of the top limb)
__device__ __forceinline__ int32_t limbs_center(int32_t x, bool top) {
  const int32_t c = top ? 0 : (x + (1 << 29)) >> 30;
  return x - (int32_t)((uint32_t)c << 30) + lane_from_prev(c);
}

// (sum over lanes) / 2^30 of a 64-bit column whose low 30 bits vanish
__device__ __forceinline__ int32_t limbs_shift30(int64_t p) {
  const uint32_t lo32 = (uint32_t)p;
  const int32_t lo = center30(lo32);
  const int32_t hi = (int32_t)__builtin_amdgcn_alignbit((uint32_t)((uint64_t)p >> 32), lo32, 30) +
                     (int32_t)((lo32 >> 29) & 1u);  // floor(p / 2^30) + (lo < 0)
  return hi + lane_from_next(lo);
}

// per-lane limb L (< 9) of a uniform 9-limb value
__device__ __forceinline__ uint32_t lane_limb(const uint32_t v[9], int L) {
  uint32_t r = 0;
  PBFTV_UNROLL for (int k = 0; k < 9; ++k) r = L == k ? v[k] : r;
  return r;
}

// One batch: 30 divsteps on the scalar unit, then the matrix update of
// (f, g) and (d, e) one lane per limb; TEST: returns g != 0.  md n_L is one
// signed 64-bit MAD (nl's sign hidden from the compiler, which would otherwise
// split it into unsigned multiplies and a sign fix).
template <bool TEST>
__device__ __forceinline__ bool inv_batch(int32_t& A, int32_t& B, int32_t& eta, int32_t nl, bool top, int row) {
  const uint32_t f0 = (uint32_t)__builtin_amdgcn_readlane(A, 0), g0 = (uint32_t)__builtin_amdgcn_readlane(B, 0);
  const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane(A, 16), e0 = (uint32_t)__builtin_amdgcn_readlane(B, 16);
  trans30 t;
  eta = divsteps30_scalar(eta, f0, g0, t);
  const int32_t md = center30(0u - ((uint32_t)t.u * d0 + (uint32_t)t.v * e0) * kNInv30);
  const int32_t me = center30(0u - ((uint32_t)t.q * d0 + (uint32_t)t.r * e0) * kNInv30);
  const int64_t P = (int64_t)t.u * A + (int64_t)t.v * B + (int64_t)md * nl;
  const int64_t Q = (int64_t)t.q * A + (int64_t)t.r * B + (int64_t)me * nl;
  A = limbs_center(limbs_shift30(P), top);
  B = limbs_center(limbs_shift30(Q), top);
  return TEST ? __ballot(row == 0 && B != 0) != 0 : true;
}

// D = R x^-1 mod n + k n for some k >= 0 (D < 2^261, 29-bit limbs, uniform),
// for 0 < x < n (uniform LE words).  Every lane of the wave must call it.
__device__ __forceinline__ void inv_mod_n_wave(fe& D, const uint32_t x[8]) {
  const int lane = (int)(threadIdx.x & 63u), L = lane & 15, row = lane >> 4;
  const bool act = L < 9 && row < 2, top = L == 8;
  s30 xs;
  words_to_s30(xs, x);
  int32_t nl = act && row == 1 ? (int32_t)lane_limb(kN30, L) : 0;
  asm volatile("" : "+v"(nl));
  int32_t A = act && row == 0 ? (int32_t)lane_limb(kN30, L) : 0;                         // f = n, d = 0
  const uint32_t xl = lane_limb(reinterpret_cast<const uint32_t*>(xs.v), L);
  const uint32_t rl = lane_limb(kRN30, L);  // R mod n = 2^261 mod n
  int32_t B = act ? (int32_t)(row == 0 ? xl : rl) : 0;  // g = x, e = R mod n
  A = limbs_center(A, top);
  B = limbs_center(B, top);
  int32_t eta = -1;
  // every input takes >= 17 batches since f starts at n: the first 14 skip the
  // g == 0 test (a batch with g = 0 leaves f and d unchanged), so each batch
  // ends in one branch
#pragma unroll 1
  for (int it = 0; it < 14; ++it) inv_batch<false>(A, B, eta, nl, top, row);
#pragma unroll 1
  for (int it = 14; it < 25; ++it)
    if (!inv_batch<true>(A, B, eta, nl, top, row)) break;  // g == 0: f = +-1, d = +-R x^-1
  uint32_t fl0 = (uint32_t)__builtin_amdgcn_readlane(A, 0), fl1 = (uint32_t)__builtin_amdgcn_readlane(A, 1);
  const bool pos = fl0 + (fl1 << 30) == 1u;  // f = +-1: its value mod 2^32
  // D = +-d + 16 n > 0 (|d| < 13.5 n), normalised 30-bit limbs, then 29-bit limbs
  uint32_t w30[9];
  int64_t c = 0;
  PBFTV_UNROLL for (int k = 0; k < 9; ++k) {
    const int32_t dk = __builtin_amdgcn_readlane(A, 16 + k);
    c += (int64_t)(pos ? dk : -dk) + 16 * (int64_t)kN30[k];
    if (k < 8) {
      w30[k] = (uint32_t)c & kM30;
      c >>= 30;
    } else {
      w30[k] = (uint32_t)c;
    }
  }
  PBFTV_UNROLL for (int j = 0; j < 9; ++j) {
    const int bit = 29 * j, li = bit / 30, sh = bit % 30;
    uint32_t v = w30[li] >> sh;
    if (li + 1 < 9) v |= w30[li + 1] << (30 - sh);
    D.v[j] = v & kMask29;
  }
}

// Montgomery's trick across the wave: inv = acc^-1 (Montgomery form mod n,
// acc in Montgomery form and nonzero) for every lane with ONE inversion per
// wave.  Prefix and suffix products over the lanes by shuffle scans (12
// products per lane), inv_mod_n_wave of the total on the scalar unit, then
// acc_l^-1 = (prefix_{l-1} suffix_{l+1}) total^-1 (2 products).  Every lane of
// the wave must call it.
__device__ __forceinline__ void shfl_fe(fe& d, const fe& s, int src_lane) {
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) d.v[l] = (uint32_t)__shfl((int)s.v[l], src_lane, 64);
}

__device__ __forceinline__ void wave_batch_inv_n(fe& inv, const fe& acc) {
  const int lane = (int)(threadIdx.x & 63u);
  fe one, pre = acc, suf = acc, a, b;
  fe_set(one, kOneN);
  PBFTV_UNROLL for (int k = 1; k < 64; k <<= 1) {
    shfl_fe(a, pre, lane - k);
    shfl_fe(b, suf, lane + k);
    PBFTV_UNROLL for (int l = 0; l < 9; ++l) {
      a.v[l] = lane >= k ? a.v[l] : one.v[l];
      b.v[l] = lane + k < 64 ? b.v[l] : one.v[l];
    }
    fn_mul(pre, pre, a);  // inclusive prefix product
    fn_mul(suf, suf, b);  // inclusive suffix product
  }
  PBFTV_SPROBE(6, suf.v[0] ^ pre.v[0]);
  fe tot;
  fn_canon(tot, pre);
  uint32_t w[8];
  fe_to_words(w, tot);
  PBFTV_UNROLL for (int k = 0; k < 8; ++k) w[k] = (uint32_t)__builtin_amdgcn_readlane((int)w[k], 63);
  fe D, r2n, invt;
  inv_mod_n_wave(D, w);  // R / total: the plain inverse of the product of the (plain) values
  PBFTV_SPROBE(7, D.v[0]);
  fe_set(r2n, kR2N);
  fn_mul(invt, D, r2n);  // its Montgomery form
  shfl_fe(a, pre, lane - 1);
  shfl_fe(b, suf, lane + 1);
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) {
    a.v[l] = lane >= 1 ? a.v[l] : one.v[l];
    b.v[l] = lane < 63 ? b.v[l] : one.v[l];
  }
  fn_mul(a, a, b);
  fn_mul(inv, a, invt);
}

// The same for a 256-thread block: the 4 waves' values are multiplied within
// quads (lanes 4q .. 4q+3: inclusive prefix and suffix by two shuffle steps),
// the 64 quad products go through LDS to wave 0, which alone runs
// wave_batch_inv_n over them (one inversion and one cross-lane scan per BLOCK),
// and each lane takes its inverse as quad^-1 * (prefix before it) * (suffix
// after it).  Per lane 6 products (wave 0: + 15 and the inversion) instead of
// 15 and an inversion per wave.  slots: >= 64 * 9 words of LDS; every thread
// of the block calls this (two barriers).
__device__ __forceinline__ void block_batch_inv_n(fe& inv, const fe& acc, uint32_t* slots) {
  const int lane = (int)(threadIdx.x & 63u), q = lane & 3, wv = (int)(threadIdx.x >> 6);
  const int slot = wv * 16 + (lane >> 2);
  fe one, pre = acc, suf = acc, a, b;
  fe_set(one, kOneN);
  PBFTV_UNROLL for (int k = 1; k < 4; k <<= 1) {
    shfl_fe(a, pre, lane - k);
    shfl_fe(b, suf, lane + k);
    PBFTV_UNROLL for (int l = 0; l < 9; ++l) {
      a.v[l] = q >= k ? a.v[l] : one.v[l];
      b.v[l] = q + k < 4 ? b.v[l] : one.v[l];
    }
    fn_mul(pre, pre, a);  // inclusive prefix product within the quad
    fn_mul(suf, suf, b);  // inclusive suffix product within the quad
  }
  if (q == 3) PBFTV_UNROLL for (int l = 0; l < 9; ++l) slots[l * 64 + slot] = pre.v[l];
  __syncthreads();
  if (wv == 0) {
    fe x, y;
    PBFTV_UNROLL for (int l = 0; l < 9; ++l) x.v[l] = slots[l * 64 + lane];
    wave_batch_inv_n(y, x);  // the quad products' inverses (Montgomery form)
    PBFTV_UNROLL for (int l = 0; l < 9; ++l) slots[l * 64 + lane] = y.v[l];
  }
  __syncthreads();
  fe qi;
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) qi.v[l] = slots[l * 64 + slot];
  shfl_fe(a, pre, lane - 1);
  shfl_fe(b, suf, lane + 1);
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) {
    a.v[l] = q >= 1 ? a.v[l] : one.v[l];
    b.v[l] = q < 3 ? b.v[l] : one.v[l];
  }
  fn_mul(a, a, b);
  fn_mul(inv, a, qi);
}

// a b 2^-261 mod m with a per-lane modulus m (29-bit limbs) and mp = -m^-1 mod
// 2^29: one step of the latency path runs mod-n and mod-p products side by
// side on different lanes.  Inputs limbs < 2^29, a < 2^257, b < 2^261;
// output < a b / 2^261 + m, limbs < 2^29.
__device__ __forceinline__ void fmont_lane(fe& r, const fe& a, const fe& b, const fe& m, uint32_t mp) {
  uint64_t t[18];
  PBFTV_UNROLL for (int k = 0; k < 18; ++k) t[k] = 0;
  PBFTV_UNROLL for (int i = 0; i < 9; ++i) {
    PBFTV_UNROLL for (int j = 0; j < 9; ++j) t[i + j] += (uint64_t)a.v[i] * b.v[j];
    const uint32_t q = ((uint32_t)t[i] * mp) & kMask29;
    PBFTV_UNROLL for (int j = 0; j < 9; ++j) t[i + j] += (uint64_t)q * m.v[j];
    t[i + 1] += t[i] >> 29;
  }
  PBFTV_UNROLL for (int j = 9; j < 16; ++j) {
    r.v[j - 9] = (uint32_t)t[j] & kMask29;
    t[j + 1] += t[j] >> 29;
  }
  r.v[7] = (uint32_t)t[16] & kMask29;
  r.v[8] = (uint32_t)(t[16] >> 29);
}

__device__ __forceinline__ void fe_readlane(fe& d, const fe& s, int lane) {
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) d.v[l] = (uint32_t)__builtin_amdgcn_readlane((int)s.v[l], lane);
}

// Go's scalars for the latency path (0 < r, s < n checked by the caller), all
// uniform: u1 = e s^-1, u2 = r s^-1 mod n (LE words), and r, r + n in
// Montgomery form mod p for the final check (rn_ok: r + n < p).  One
// inversion (inv_mod_n_wave), then ONE product step: lanes 4k..4k+3 compute
// e D, r D (mod n) and r R^2, (r + n) R^2 (mod p) at once.
__device__ __forceinline__ void wave_scalars(const uint32_t e[8], const uint32_t r[8], const uint32_t s[8],
                                             uint32_t u1[8], uint32_t u2[8], fe& rm, fe& rnm, bool& rn_ok) {
  fe D;
  PBFTV_RPROBE(15, s[0]);
  inv_mod_n_wave(D, s);
  PBFTV_RPROBE(14, D.v[0]);
  uint32_t rn[8];
  uint64_t cy = 0;
  PBFTV_UNROLL for (int i = 0; i < 8; ++i) {
    cy += (uint64_t)r[i] + kN32[i];
    rn[i] = (uint32_t)cy;
    cy >>= 32;
  }
  rn_ok = words_lt(r, kPMinusN32);  // r + n < p
  const int role = (int)(threadIdx.x & 3u);
  fe ev, rv, rnv, a, b, m, r2p, nmod, pmod, prod;
  fe_from_words(ev, e);
  fe_from_words(rv, r);
  fe_from_words(rnv, rn);
  fe_set(r2p, kR2P);
  fe_set(nmod, kN);
  fe_set(pmod, kP);
  const bool modn = role < 2;
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) {
    a.v[l] = role == 0 ? ev.v[l] : (role == 3 ? rnv.v[l] : rv.v[l]);
    b.v[l] = modn ? D.v[l] : r2p.v[l];
    m.v[l] = modn ? nmod.v[l] : pmod.v[l];
  }
  fmont_lane(prod, a, b, m, modn ? kNPrime : 1u);  // p = -1 mod 2^29: -p^-1 = 1
  fn_canon(a, prod);  // lanes 0, 1: < 2^256 + n  ->  [0, n) in two steps
  fn_canon(a, a);
  uint32_t w[8];
  fe_to_words(w, a);
  PBFTV_UNROLL for (int k = 0; k < 8; ++k) {
    u1[k] = (uint32_t)__builtin_amdgcn_readlane((int)w[k], 0);
    u2[k] = (uint32_t)__builtin_amdgcn_readlane((int)w[k], 1);
  }
  fe_readlane(rm, prod, 2);
  fe_readlane(rnm, prod, 3);
}

// The same scalars for the row schedule, written by the lanes that computed
// them straight into the workgroup's LDS (lane 0: u1, lane 1: u2, lane 2:
// r R mod p as 29-bit limbs) -- no readlane of the 25 words and no per-lane
// select, ~1 µs of a lone wave's issue.  u1, u2 get one reduction step, to
// [0, 2^256): u and u - n give the same comb sum.
__device__ __forceinline__ void wave_scalars_lds(const uint32_t e[8], const uint32_t r[8], const uint32_t s[8],
                                                 uint32_t* u1, uint32_t* u2, uint32_t* rm) {
  fe D;
  PBFTV_RPROBE(15, s[0]);
  inv_mod_n_wave(D, s);
  PBFTV_RPROBE(14, D.v[0]);
  const int role = (int)(threadIdx.x & 3u);
  fe ev, rv, a, b, m, r2p, nmod, pmod, prod;
  fe_from_words(ev, e);
  fe_from_words(rv, r);
  fe_set(r2p, kR2P);
  fe_set(nmod, kN);
  fe_set(pmod, kP);
  const bool modn = role < 2;
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) {
    a.v[l] = role == 0 ? ev.v[l] : rv.v[l];
    b.v[l] = modn ? D.v[l] : r2p.v[l];
    m.v[l] = modn ? nmod.v[l] : pmod.v[l];
  }
  fmont_lane(prod, a, b, m, modn ? kNPrime : 1u);  // lanes 0, 1: e D, r D mod n; lane 2: r R mod p
  const int lane = (int)(threadIdx.x & 63u);
  if (lane < 2) {
    fn_canon(a, prod);  // < 2^256 + n  ->  < 2^256
    uint32_t w[8];
    fe_to_words(w, a);
    uint32_t* dst = lane == 0 ? u1 : u2;
    PBFTV_UNROLL for (int k = 0; k < 8; ++k) dst[k] = w[k];
  } else if (lane == 2) {
    PBFTV_UNROLL for (int l = 0; l < 9; ++l) rm[l] = prod.v[l];
  }
}

// x(P) == r or r + n (mod n) for the all-reduced XYZZ sum: lanes 0 and 1 test
// X == r ZZ and X == (r + n) ZZ with one product step.
__device__ __forceinline__ bool wave_check(const xyzz_s& P, bool finite, const fe& rm, const fe& rnm, bool rn_ok) {
  const int role = (int)(threadIdx.x & 1u);
  fe a, lhs, d;
  PBFTV_UNROLL for (int l = 0; l < 9; ++l) a.v[l] = role ? rnm.v[l] : rm.v[l];
  fs_mul(lhs, a, P.zz);
  fs_sub(d, lhs, P.x);
  const bool z = fs_is_zero(d);
  const unsigned long long bz = __ballot(z);
  return finite && ((bz & 1ull) != 0 || (rn_ok && (bz & 2ull) != 0));
}

// Go's verdict from uniform LE words e (hash), r, s, the key's table and
// whether the key is registered and valid, computed by the whole wave (every
// lane must call it; wave-uniform result).
template <int WG, int WQ>
__device__ __forceinline__ bool wave_verify_words(uint32_t e[8], uint32_t r[8], uint32_t s[8], bool key_ok,
                                                  const uint4* __restrict__ gtab, const uint4* __restrict__ qtab) {
  constexpr int nG = CombGeom<WG>::kWin, nQ = CombGeom<WQ>::kWin;
  constexpr int nW = nG > nQ ? nG : nQ;
  static_assert(nW <= 64, "one lane per window");
  if (!key_ok || words_is_zero(r) || words_is_zero(s) || !words_lt(r, kN32) || !words_lt(s, kN32)) return false;
  uint32_t u1[8], u2[8];
  fe rm, rnm;
  bool rn_ok;
  wave_scalars(e, r, s, u1, u2, rm, rnm, rn_ok);
  bool inf, ok = false;
  bool exc = true;
  if constexpr (nW > 8 && nW <= 16) {
    const bool okq = wave_verify_quads<WG, WQ>(exc, u1, u2, gtab, qtab, rm, rnm, rn_ok);
    exc = __any(exc);
    ok = __builtin_amdgcn_readfirstlane((int)okq) != 0;  // lane 0 = quad 0: the all-reduced verdict
  }
  if (exc) {  // windows outnumber the quads, or a doubling somewhere: exact lane-per-window rerun
    jac P;
    wave_sum_lanes<WG, WQ>(P, inf, u1, u2, gtab, qtab);
    ok = ecdsa_check(P, !inf, r);
  }
  return ok;
}

// ---- the row schedule (round 5): EIGHT waves per signature ----------------
// rows.h holds one field element per VGPR (limb j in lane j of a 16-lane row),
// so a wave does four products at once and an XYZZ addition costs ~0.95 µs
// instead of a quad-schedule level's ~2.6 µs.  A workgroup of eight waves
// verifies one signature:
//   * wave 0 runs Go's range checks and the scalars (the s^-1 chain, as
//     wave_verify_words) and hands u1, u2 and r R to the others through LDS;
//   * wave w takes windows 2w (rows 0, 1) and 2w + 1 (rows 2, 3): the G entry
//     of digit w of u1 plus the Q entry of digit w of u2 (mmadd_pairs: the
//     two windows side by side), then their sum (xyzz_add_rows);
//   * a tree over the waves through LDS: levels 1 and 2 add wave w + m into
//     wave w; the last (wave 4 into wave 0) is fused with the x check
//     against r (xyzz_add_check_rows).
// As in the quad schedule, a doubling or cancellation anywhere leaves a zero
// ZZ that every later product keeps (one test at the top), a live window with
// two zero digits and r + n < p (adversarial r only) go to wave 0's exact
// lane-per-window rerun.  Every thread of the workgroup calls it; the
// arguments are read from wave 0 only; wave 0 returns the verdict.
constexpr int kRowWaves = 8;

struct RowsShared {
  uint32_t ctl;  // bit 0: verify (range checks passed), bit 1: exact path (r + n < p), bit 2: a rare window
  uint32_t ready[kRowWaves];  // wave w's partial sum is in pts[w]
  uint32_t u1[8], u2[8], rm[9];
  uint64_t qtab;
  uint32_t pts[kRowWaves][4][16];  // a wave's partial sum: row 0's lanes of X, Y, ZZ, ZZZ
};

template <int WG, int WQ>
struct RowsGeom {
  static constexpr int nW = CombGeom<WG>::kWin > CombGeom<WQ>::kWin ? CombGeom<WG>::kWin : CombGeom<WQ>::kWin;
  static constexpr bool ok = nW > 8 && nW <= 2 * kRowWaves;
  static constexpr int waves = (nW + 1) / 2;  // launched: waves past the windows would have nothing to do
};

// window `win`'s entry of digit d as row-layout x, y (lane L < 9: limb L; the
// lane reads the two words of each coordinate its limb spans, one 64-B line)
template <int W>
__device__ __forceinline__ void row_entry(const uint4* __restrict__ tab, int win, int d, int L, uint32_t& x,
                                          uint32_t& y) {
  const int idx = (d < 0 ? -d : d) - 1;
  const uint32_t* p = reinterpret_cast<const uint32_t*>(tab + (CombGeom<W>::base(win) + (idx < 0 ? 0 : idx)) * 4);
  const int Lc = L < 9 ? L : 0, bit = 29 * Lc, wi = bit >> 5, sh = bit & 31;
  const int wj = wi < 7 ? wi + 1 : wi;
  const uint32_t x0 = p[wi], x1 = p[wj], y0 = p[8 + wi], y1 = p[8 + wj];
  const uint32_t m = L < 9 ? kMask29 : 0u;
  x = __builtin_amdgcn_alignbit(wi < 7 ? x1 : 0u, x0, (uint32_t)sh) & m;
  y = __builtin_amdgcn_alignbit(wi < 7 ? y1 : 0u, y0, (uint32_t)sh) & m;
}

// kExact: the exceptional cases run wave 0's exact rerun here (the launched
// kernel) and the verdict carries kRowsExact; without it (the armed kernel,
// which then needs far fewer registers while it stays resident) they return 2
// and the host serves the certificate with the launched kernel.  Returns
// 1 / 0 (valid / not), | kRowsExact (kernels.h) after the exact path, or 2.
template <int WG, int WQ, bool kExact>
__device__ __forceinline__ int block_verify_rows(const uint32_t e[8], const uint32_t r[8], const uint32_t s[8],
                                                 bool key_ok, const uint4* __restrict__ gtab,
                                                 const uint4* qtab, RowsShared* sh) {
  constexpr int nG = CombGeom<WG>::kWin, nQ = CombGeom<WQ>::kWin, nW = RowsGeom<WG, WQ>::nW;
  static_assert(RowsGeom<WG, WQ>::ok, "two windows per wave, eight waves");
  const int wv = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63u);
  PBFTV_RPROBE(0, e[0]);
  if (wv == 0) {
    uint32_t ctl = 0;
    if (key_ok && !words_is_zero(r) && !words_is_zero(s) && words_lt(r, kN32) && words_lt(s, kN32)) {
      wave_scalars_lds(e, r, s, sh->u1, sh->u2, sh->rm);
      ctl = words_lt(r, kPMinusN32) ? 3u : 1u;  // r + n < p: the exact path
      if (lane == 0) sh->qtab = (uint64_t)(uintptr_t)qtab;
    }
    if (lane == 0) sh->ctl = ctl;
    if (lane < kRowWaves) sh->ready[lane] = 0u;
    PBFTV_RPROBE(1, ctl);
  }
  __syncthreads();
  const uint32_t ctl = (uint32_t)__builtin_amdgcn_readfirstlane((int)sh->ctl);
  if (!(ctl & 1u)) return 0;  // (every wave: the same LDS word)
  uint32_t u1[8], u2[8];
  PBFTV_UNROLL for (int k = 0; k < 8; ++k) {
    u1[k] = (uint32_t)__builtin_amdgcn_readfirstlane((int)sh->u1[k]);
    u2[k] = (uint32_t)__builtin_amdgcn_readfirstlane((int)sh->u2[k]);
  }
  const uint64_t qv = sh->qtab;
  const uint4* qt = reinterpret_cast<const uint4*>(
      (uintptr_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(qv >> 32)) << 32) |
                  (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)qv)));
  if (ctl & 2u) {  // r + n < p: the exact path, wave 0 alone (no barrier follows)
    if (wv != 0) return 0;
    if constexpr (kExact) {
      jac P;
      bool inf;
      wave_sum_lanes<WG, WQ>(P, inf, u1, u2, gtab, qt);
      return (ecdsa_check(P, !inf, r) ? 1 : 0) | kRowsExact;
    } else {
      return 2;
    }
  }
  // Tree position t of this wave.  Waves w and w + 4 share a SIMD, and the
  // older one takes its issue slots first: the younger runs when the older
  // waits.  With six waves (11 or 12 windows) positions 4 and 5 are swapped,
  // so the root (the longest chain: its pair, two levels, the fused check)
  // shares SIMD 0 with the lightest position (5: one window for 11) and
  // position 4 (a pair and one level) gets SIMD 1 once position 1 has handed
  // its pair over.  With seven (13 or 14 windows) position 4 (a pair and two
  // levels) takes wave 3, the one alone on its SIMD, the root shares SIMD 0
  // with position 6 (one window for 13) and position 2 shares SIMD 2 with
  // position 3, its own first partner.
  constexpr int kWaves = RowsGeom<WG, WQ>::waves;
  int t = kWaves == 6   ? (wv == 4 ? 5 : wv == 5 ? 4 : wv)
                : kWaves == 7 ? (wv == 3 ? 4 : wv == 4 ? 6 : wv == 6 ? 3 : wv)
                              : wv;
#ifdef PBFTV_ROWS_IDENTITY  // (A/B only)
  t = wv;
#endif
  if (2 * t >= nW) return 0;  // no window (its partners know that statically)
  const RowCtx c = row_ctx();
  const uint32_t rml = c.L < 9 ? sh->rm[c.L] : 0u;
  PBFTV_RPROBE(2, rml);
  // digits of every window (quad q = window q), each row pair keeps its own
  const int q = lane >> 2;
  const int d1 = lane_window_digit<WG>(u1, q), d2 = lane_window_digit<WQ>(u2, q);
  const int wA = 2 * t, wB = 2 * t + 1;
  const int a1 = __builtin_amdgcn_readlane(d1, 4 * wA), a2 = __builtin_amdgcn_readlane(d2, 4 * wA);
  const int b1 = __builtin_amdgcn_readlane(d1, 4 * wB), b2 = __builtin_amdgcn_readlane(d2, 4 * wB);
  const bool pb = c.row >= 2;
  const int win = pb ? wB : wA, g1 = pb ? b1 : a1, g2 = pb ? b2 : a2;
  uint32_t gx, gy, qx, qy;
  row_entry<WG>(gtab, win < nG ? win : 0, g1, c.L, gx, gy);
  row_entry<WQ>(qt, win < nQ ? win : 0, g2, c.L, qx, qy);
  gy = g1 < 0 ? 0u - gy : gy;
  qy = g2 < 0 ? 0u - qy : qy;
  PBFTV_RPROBE(3, gx ^ gy ^ qx ^ qy);
  xyzz_r S;
  mmadd_pairs(c, S, gx, gy, qx, qy);  // (x-coordinates meeting: PP = 0 = ZZ, tested at the top)
  const bool both = g1 != 0 && g2 != 0, gonly = g1 != 0;
  PBFTV_RPROBE(4, S.y);
  xyzz_r Pw;  // a lone table point: ZZ = ZZZ = 1
  Pw.x = both ? S.x : (gonly ? gx : qx);
  Pw.y = both ? S.y : (gonly ? gy : qy);
  Pw.zz = both ? S.zz : c.one;
  Pw.zzz = both ? S.zzz : c.one;
  // a live window with two zero digits (probability ~2^-50): the exact rerun
  if (__any(win < nW && g1 == 0 && g2 == 0) && lane == 0) atomicOr(&sh->ctl, 4u);
  xyzz_r P, B;
  uint32_t rz = 0, g[4];
  gather4(g, Pw.x);
  P.x = g[0];
  B.x = g[2];
  gather4(g, Pw.y);
  P.y = g[0];
  B.y = g[2];
  gather4(g, Pw.zz);
  P.zz = g[0];
  B.zz = g[2];
  gather4(g, Pw.zzz);
  P.zzz = g[0];
  B.zzz = g[2];
  if (wB < nW) xyzz_add_rows(c, P, rz, P, B, rml);
  PBFTV_RPROBE(5, P.y);
  // The tree: at level m a wave w with w mod 2m == m hands its sum to wave
  // w - m and leaves; the holder waits for that one partner only (an LDS flag,
  // release / acquire at workgroup scope), not for the whole workgroup, so a
  // wave whose subtree is ready early goes on while slower ones still add.
  bool ok = false, exc = false;
  PBFTV_UNROLL for (int m = 1; m < kRowWaves; m <<= 1) {
    if ((t & (2 * m - 1)) == m) {
      if (c.row == 0) {
        sh->pts[t][0][c.L] = P.x;
        sh->pts[t][1][c.L] = P.y;
        sh->pts[t][2][c.L] = P.zz;
        sh->pts[t][3][c.L] = P.zzz;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_store(&sh->ready[t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return 0;
    }
    if (2 * (t + m) < nW) {  // add the partner's
      while (__hip_atomic_load(&sh->ready[t + m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
        __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      PBFTV_RPROBE(5 + 2 * m - (m == 4 ? 1 : 0), m);
      xyzz_r Q;
      Q.x = sh->pts[t + m][0][c.L];
      Q.y = sh->pts[t + m][1][c.L];
      Q.zz = sh->pts[t + m][2][c.L];
      Q.zzz = sh->pts[t + m][3][c.L];
      if (m == kRowWaves / 2) {  // wave 0: the last level, fused with the check
        ok = xyzz_add_check_rows(c, exc, P, Q, rz);
      } else {
        xyzz_add_rows(c, P, rz, P, Q, rml);
      }
    }
    PBFTV_RPROBE(6 + 2 * m - (m == 4 ? 1 : 0), P.y ^ (uint32_t)ok);
  }
  if (t != 0) return 0;
  exc = exc || (sh->ctl & 4u) != 0;
  if (exc) {  // a doubling / cancellation somewhere, or a rare window: exact rerun
    if constexpr (kExact) {
      jac R;
      bool inf;
      wave_sum_lanes<WG, WQ>(R, inf, u1, u2, gtab, qt);
      return (ecdsa_check(R, !inf, r) ? 1 : 0) | kRowsExact;
    } else {
      return 2;
    }
  }
  return ok ? 1 : 0;
}

// ... from memory: signature i of the (host or device) input arrays.
__device__ __forceinline__ void wave_load_sig(const uint8_t* __restrict__ hashes, const uint8_t* __restrict__ sigs,
                                              const uint32_t* __restrict__ key_idx, uint64_t i,
                                              const uint32_t* __restrict__ key_valid, uint32_t nkeys,
                                              const uint4* const* __restrict__ qtabs, uint32_t e[8], uint32_t r[8],
                                              uint32_t s[8], bool& key_ok, const uint4*& qtab) {
  load_be256(hashes + 32 * i, e);  // one round trip to the (host) inputs
  load_be256(sigs + 64 * i, r);
  load_be256(sigs + 64 * i + 32, s);
  const uint32_t k = (uint32_t)__builtin_amdgcn_readfirstlane((int)key_idx[i]);
  key_ok = k < nkeys && key_valid[k] != 0;
  qtab = qtabs[k < nkeys ? k : 0];  // (loaded now: ready when the scalars are)
  PBFTV_UNROLL for (int t = 0; t < 8; ++t) {  // one copy per wave (the loads are per lane)
    e[t] = (uint32_t)__builtin_amdgcn_readfirstlane((int)e[t]);
    r[t] = (uint32_t)__builtin_amdgcn_readfirstlane((int)r[t]);
    s[t] = (uint32_t)__builtin_amdgcn_readfirstlane((int)s[t]);
  }
}

template <int WG, int WQ>
__device__ __forceinline__ bool wave_verify_sig(const uint8_t* __restrict__ hashes, const uint8_t* __restrict__ sigs,
                                                const uint32_t* __restrict__ key_idx, uint64_t i,
                                                const uint32_t* __restrict__ key_valid, uint32_t nkeys,
                                                const uint4* __restrict__ gtab, const uint4* const* __restrict__ qtabs) {
  uint32_t r[8], s[8], e[8];
  bool key_ok;
  const uint4* qtab;
  wave_load_sig(hashes, sigs, key_idx, i, key_valid, nkeys, qtabs, e, r, s, key_ok, qtab);
  return wave_verify_words<WG, WQ>(e, r, s, key_ok, gtab, qtab);
}

__device__ __forceinline__ void wave_store_verdict(bool ok, uint64_t i, uint64_t n, uint8_t* __restrict__ bitmap,
                                                   uint8_t* __restrict__ okbytes, uint8_t flags = 0) {
  if (okbytes) {  // (the latency path's result bytes: bit 0 the verdict, kRowsExact the exact path)
    okbytes[i] = (uint8_t)((ok ? 1 : 0) | flags);
    return;
  }
  // one bit of the LSB-first bitmap: set or clear it with a word atomic
  // (other signatures' waves share the byte; no pre-zeroing needed).  The last
  // signature also clears the padding bits above it in its byte, so the tail
  // of the bitmap is deterministic (as the lane path's ballot bytes are).
  uint8_t* byte = bitmap + (i >> 3);
  const uintptr_t a = reinterpret_cast<uintptr_t>(byte);
  unsigned int* word = reinterpret_cast<unsigned int*>(a & ~(uintptr_t)3);
  const unsigned int sh = (unsigned)(a & 3) << 3;
  const unsigned int bit = 1u << (sh + (unsigned)(i & 7));
  unsigned int clear = ok ? 0u : bit;
  if (i + 1 == n) clear |= ((0xFEu << (unsigned)(i & 7)) & 0xFFu) << sh;
  if (clear) atomicAnd(word, ~clear);
  if (ok) atomicOr(word, bit);
}

template <int WG, int WQ>
__global__ void __launch_bounds__(64) k_ecdsa_wave(const uint8_t* __restrict__ hashes,
                                                   const uint8_t* __restrict__ sigs,
                                                   const uint32_t* __restrict__ key_idx, uint64_t n,
                                                   const uint32_t* __restrict__ key_valid, uint32_t nkeys,
                                                   const uint4* __restrict__ gtab, const uint4* const* __restrict__ qtabs,
                                                   uint8_t* __restrict__ bitmap, uint8_t* __restrict__ okbytes) {
  __builtin_amdgcn_s_setprio(3);  // a latency-path kernel: its waves issue ahead of a concurrent batch's
  const uint64_t i = blockIdx.x;
  const bool ok = wave_verify_sig<WG, WQ>(hashes, sigs, key_idx, i, key_valid, nkeys, gtab, qtabs);
  if (threadIdx.x == 0) wave_store_verdict(ok, i, n, bitmap, okbytes);
}

// The same, compiled to at most 128 VGPRs (4 waves per SIMD, the comb's
// budget): launched beside a lane batch (launch_wave_w one_wave), one such wave
// fits the slot ONE finished comb wave frees, where a 175-VGPR wave needs two
// on one SIMD -- and the batch's own blocks refill freed slots first.
template <int WG, int WQ>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 8)))
k_ecdsa_wave_lean(const uint8_t* __restrict__ hashes, const uint8_t* __restrict__ sigs,
                  const uint32_t* __restrict__ key_idx, uint64_t n, const uint32_t* __restrict__ key_valid,
                  uint32_t nkeys, const uint4* __restrict__ gtab, const uint4* const* __restrict__ qtabs,
                  uint8_t* __restrict__ bitmap, uint8_t* __restrict__ okbytes) {
  __builtin_amdgcn_s_setprio(3);  // (as k_ecdsa_wave: ahead of the batch it runs beside)
  const uint64_t i = blockIdx.x;
  const bool ok = wave_verify_sig<WG, WQ>(hashes, sigs, key_idx, i, key_valid, nkeys, gtab, qtabs);
  if (threadIdx.x == 0) wave_store_verdict(ok, i, n, bitmap, okbytes);
}

// the row schedule, launched: one 512-thread workgroup per signature
template <int WG, int WQ>
__global__ void __launch_bounds__(64 * kRowWaves) k_ecdsa_rows(const uint8_t* __restrict__ hashes,
                                                               const uint8_t* __restrict__ sigs,
                                                               const uint32_t* __restrict__ key_idx, uint64_t n,
                                                               const uint32_t* __restrict__ key_valid, uint32_t nkeys,
                                                               const uint4* __restrict__ gtab,
                                                               const uint4* const* __restrict__ qtabs,
                                                               uint8_t* __restrict__ bitmap, uint8_t* __restrict__ okbytes) {
  __shared__ RowsShared sh;
  __builtin_amdgcn_s_setprio(3);  // (as k_ecdsa_wave)
  const uint64_t i = blockIdx.x;
  uint32_t e[8] = {}, r[8] = {}, s[8] = {};
  bool key_ok = false;
  const uint4* qtab = nullptr;
  if (threadIdx.x < 64) wave_load_sig(hashes, sigs, key_idx, i, key_valid, nkeys, qtabs, e, r, s, key_ok, qtab);
  const int v = block_verify_rows<WG, WQ, true>(e, r, s, key_ok, gtab, qtab, &sh);
  if (threadIdx.x == 0) wave_store_verdict((v & 1) != 0, i, n, bitmap, okbytes, (uint8_t)(v & kRowsExact));
}

// ---- the armed latency kernel ------------------------------------------------
// A persistent server, launched AHEAD of the requests it serves (pbftv_api.cpp
// keeps one armed per device), so neither a launch nor a re-arm is on a
// certificate's critical path: after request `want` it waits for want + 1.
// One wave per signature slot (QcMail::kQcSlots = 8: a certificate of
// n = 3f+1 <= 9 replicas).  Each wave polls, in ONE wave-wide load (lane l
// reads dword l % 16 of line l / 16), the three 64-B lines of its slot and the
// mailbox header: every slot line carries the request number in its first and
// last dword, written by the host after the line's data (one line is read as
// one snapshot of the host's cache line, and x86 stores become visible in
// order; requiring both tags also covers a read that tore a line in two), so
// three matching lines mean n, the key and the hash / r / s are already in
// registers -- no second PCIe round trip.  Waves with slots >= n need only
// line 0 (n) and go straight back to waiting.  Every wave reaches an exit: a cancel (header stop == the
// request number it waits for, or a change of the header's halt word) or the
// budget (wall-clock ticks since launch); a wave that leaves writes
// expired = that number, and the host serves a request that raced the exit
// with a launch instead.  Waits are s_sleep between polls (spin: see
// ArmArgs); host words are read with system-scope loads; nothing is written
// through the scalar cache.  The key tables' pointers and validity flags of
// the first 128 keys are loaded once, at launch (a key change cancels first).
// key data of key k: from the per-lane prefetch for k < 128, else from memory
__device__ __forceinline__ void armed_key(uint32_t k, uint32_t nkeys, const uint4* qt_lo, const uint4* qt_hi,
                                          uint32_t kv_lo, uint32_t kv_hi, const uint32_t* __restrict__ key_valid,
                                          const uint4* const* __restrict__ qtabs, bool& key_ok, const uint4*& qtab) {
  if (k < 128 && k < nkeys) {  // prefetched
    const int kl = (int)(k & 63);
    const uint64_t ql = (uint64_t)(uintptr_t)(k < 64 ? qt_lo : qt_hi);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)ql, kl),
                   hi = __builtin_amdgcn_readlane((uint32_t)(ql >> 32), kl);
    qtab = reinterpret_cast<const uint4*>((uintptr_t)(((uint64_t)hi << 32) | lo));
    key_ok = __builtin_amdgcn_readlane(k < 64 ? kv_lo : kv_hi, kl) != 0;
  } else {
    key_ok = k < nkeys && key_valid[k] != 0;
    qtab = qtabs[k < nkeys ? k : 0];
  }
}

// Launched with kQcSlots waves (narrow) or kQcCap waves (wide: certificates
// of up to 128 signatures, e.g. a 67-vote QC of an n = 100 committee).  Waves
// past the slots are HELPERS: they never poll host memory; wave 0 relays each
// request's number and n to them through a word of uncached device memory
// (`relay`: {number, n}, n = ~0 when wave 0 leaves), and a helper whose index is below n
// reads its signature from the mailbox arrays (one PCIe round trip; the host
// writes them before the slot tags) and writes its verdict byte.
template <int WG, int WQ>
__global__ void __launch_bounds__(256) k_ecdsa_wave_armed(ArmArgs a) {
  // four waves per workgroup: one CU takes a workgroup's waves on its four
  // SIMDs, so no two armed waves of a workgroup share a SIMD's issue slots
  const uint32_t b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  QcMail* const mail = a.mail;
  uint8_t* const base = reinterpret_cast<uint8_t*>(mail);
  uint32_t want = a.want;
  const uint64_t t0 = wall_clock64();
  // live: this wave is resident (a rotation retires the old kernel after all are)
  if (lane == 0) reinterpret_cast<volatile uint32_t*>(base + QcMail::live_off(a.slot))[b] = want;
  // key data for keys < 128, two per lane (lane l: keys l and l + 64)
  const uint32_t nkeys = a.nkeys;
  const uint4* qt_lo = lane < nkeys ? reinterpret_cast<const uint4* const*>(a.qtabs)[lane] : nullptr;
  const uint4* qt_hi = lane + 64 < nkeys ? reinterpret_cast<const uint4* const*>(a.qtabs)[lane + 64] : nullptr;
  const uint32_t kv_lo = lane < nkeys ? a.key_valid[lane] : 0u, kv_hi = lane + 64 < nkeys ? a.key_valid[lane + 64] : 0u;
  const uint4* gtab = reinterpret_cast<const uint4*>(a.gtab);
  const uint4* const* qtabs = reinterpret_cast<const uint4* const*>(a.qtabs);
  uint64_t* const relay = a.relay;
  if (b >= QcMail::kQcSlots) {
    // ---- helper wave ----
    uint32_t last = 0;  // the relay starts at {0, 0}; request numbers are never 0
    for (;;) {
      uint64_t r = 0;
      for (;;) {
        // (uncached memory: a relaxed system-scope load sees wave 0's store
        // with no cache maintenance; the host inputs read next were written
        // before the slot tags wave 0 saw, and host memory is not cached here)
        r = __hip_atomic_load(relay, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((uint32_t)r != last || wall_clock64() - t0 > a.budget) break;
        __builtin_amdgcn_s_sleep(2);
      }
      const uint32_t seq = (uint32_t)r, n = (uint32_t)(r >> 32);
      if (seq == last || n == 0xFFFFFFFFu) return;  // budget, or wave 0 left
      last = seq;
      if (b >= n) continue;
      const uint64_t seen_wall = wall_clock64(), seen_clk = clock64();
      __builtin_amdgcn_s_setprio(3);
      constexpr uint32_t cap = QcMail::kQcCap;  // the armed path's layout (the host relays it out only after a disarm)
      // lanes 0-7 the hash, 8-23 r || s, 24 the key index: one round trip
      const uint32_t* src = lane < 8    ? reinterpret_cast<const uint32_t*>(base + QcMail::hashes_off(cap) + 32 * b) + lane
                            : lane < 24 ? reinterpret_cast<const uint32_t*>(base + QcMail::sigs_off(cap) + 64 * b) + (lane - 8)
                                        : reinterpret_cast<const uint32_t*>(base + QcMail::keys_off(cap) + 4 * b);
      const uint32_t v = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      uint32_t e[8], rr[8], ss[8];
      PBFTV_UNROLL for (int t = 0; t < 8; ++t) {
        e[7 - t] = bswap32(__builtin_amdgcn_readlane(v, t));
        rr[7 - t] = bswap32(__builtin_amdgcn_readlane(v, 8 + t));
        ss[7 - t] = bswap32(__builtin_amdgcn_readlane(v, 16 + t));
      }
      bool key_ok;
      const uint4* qtab;
      armed_key(__builtin_amdgcn_readlane(v, 24), nkeys, qt_lo, qt_hi, kv_lo, kv_hi, a.key_valid, qtabs, key_ok, qtab);
      const bool ok = wave_verify_words<WG, WQ>(e, rr, ss, key_ok, gtab, qtab);
      if (lane == 0) {
        if (a.stamps) {
          volatile uint64_t* st = reinterpret_cast<volatile uint64_t*>(base + QcMail::stamps_off(cap)) + 4 * b;
          st[0] = seen_wall;  // diagnostics (pbftv_qc_stamps_all), before the verdict
          st[1] = seen_clk;
          st[2] = wall_clock64();
          st[3] = clock64();
        }
        reinterpret_cast<volatile uint8_t*>(base)[QcMail::res_off(cap) + b] = ok ? 1 : 0;
      }
      __builtin_amdgcn_s_setprio(0);
    }
  }
  // ---- slot wave ----
  const uint32_t* slot = reinterpret_cast<const uint32_t*>(base + QcMail::slot_off(b));
  const uint32_t* word = lane < 48 ? slot + lane : reinterpret_cast<const uint32_t*>(base) + (lane - 48);
  for (;; ++want) {
    uint32_t v = 0;
    bool serve = false;
    for (;;) {
      v = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      // line 0 carries n; a slot past n needs only that line (the host writes
      // no inputs there), a slot below n all three
      if (__builtin_amdgcn_readlane(v, 0) == want && __builtin_amdgcn_readlane(v, 15) == want &&
          (b >= __builtin_amdgcn_readlane(v, 1) ||
           (__builtin_amdgcn_readlane(v, 16) == want && __builtin_amdgcn_readlane(v, 31) == want &&
            __builtin_amdgcn_readlane(v, 32) == want && __builtin_amdgcn_readlane(v, 47) == want))) {
        serve = true;
        break;
      }
      if (__builtin_amdgcn_readlane(v, 48 + 2) == want || __builtin_amdgcn_readlane(v, 48 + 5) != a.halt ||
          wall_clock64() - t0 > a.budget)
        break;  // header stop / halt, or the budget
      if (a.spin == 0) {
        __builtin_amdgcn_s_sleep(2);
      } else if (a.spin >= 1000) {  // (experiments) (spin - 1000) x s_sleep(8) between polls
        for (uint32_t j = 1000; j < a.spin; ++j) __builtin_amdgcn_s_sleep(8);
      } else if (a.spin > 1) {
        uint32_t x = lane;
        for (uint32_t j = 0; j < a.spin; ++j) asm volatile("v_mad_u32_u24 %0, %0, %0, %0" : "+v"(x));
      }
    }
    if (!serve) {
      if (b == 0 && relay && lane == 0)  // the helpers leave with wave 0
        __hip_atomic_store(relay, ((uint64_t)0xFFFFFFFFu << 32) | want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (lane == 0) __hip_atomic_store(mail->expired(a.slot), want, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    const uint64_t seen_wall = wall_clock64(), seen_clk = clock64();
    const uint32_t n = __builtin_amdgcn_readlane(v, 1);
    if (b == 0 && relay && n > QcMail::kQcSlots && lane == 0)
      __hip_atomic_store(relay, ((uint64_t)n << 32) | want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (b >= n) continue;
    // a certificate's waves go ahead of whatever else shares their SIMDs (the
    // waves of a large batch: issue priority only, nothing is preempted)
    __builtin_amdgcn_s_setprio(3);
    uint32_t e[8], r[8], s[8];
    const uint32_t k = __builtin_amdgcn_readlane(v, 2);
    PBFTV_UNROLL for (int t = 0; t < 8; ++t) {  // slot line j, dword 4 + t = LE dword t of the hash / r / s
      e[7 - t] = bswap32(__builtin_amdgcn_readlane(v, 4 + t));
      r[7 - t] = bswap32(__builtin_amdgcn_readlane(v, 20 + t));
      s[7 - t] = bswap32(__builtin_amdgcn_readlane(v, 36 + t));
    }
    bool key_ok;
    const uint4* qtab;
    armed_key(k, nkeys, qt_lo, qt_hi, kv_lo, kv_hi, a.key_valid, qtabs, key_ok, qtab);
    const bool ok = wave_verify_words<WG, WQ>(e, r, s, key_ok, gtab, qtab);
    if (lane == 0) {
      // the armed path's layout is always cap = kQcCap (no PCIe round trip for
      // the header's cap between the verdict and its store)
      constexpr uint32_t cap = QcMail::kQcCap;
      if (a.stamps) {
        volatile uint64_t* st = reinterpret_cast<volatile uint64_t*>(base + QcMail::stamps_off(cap)) + 4 * b;
        st[0] = seen_wall;  // diagnostics (pbftv_qc_stamps), before the verdict
        st[1] = seen_clk;
        st[2] = wall_clock64();
        st[3] = clock64();
      }
      // (coherent host memory is not cached on the GPU: the stores leave in
      // order; a system-scope release here would write back the L2 first)
      reinterpret_cast<volatile uint8_t*>(base)[QcMail::res_off(cap) + b] = ok ? 1 : 0;
    }
    __builtin_amdgcn_s_setprio(0);
  }
}

// The armed server on the row schedule: one workgroup (RowsGeom::waves waves)
// per signature slot.  Wave 0 is the slot wave of k_ecdsa_wave_armed (the same
// polls, exits, live / expired words and verdict store) -- or, in the wide
// kernel (kQcCap workgroups, a relay), a helper wave for slots >= kQcSlots; the
// other waves wait at the workgroup barrier -- they issue nothing while they
// wait -- and join block_verify_rows when wave 0 has a signature for the slot.
template <int WG, int WQ>
__global__ void __launch_bounds__(64 * kRowWaves) k_ecdsa_rows_armed(ArmArgs a) {
  __shared__ RowsShared sh;
  __shared__ uint32_t cmd;  // 0: leave, 1: serve the slot, 2: request without this slot
  const uint32_t b = blockIdx.x, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  QcMail* const mail = a.mail;
  uint8_t* const base = reinterpret_cast<uint8_t*>(mail);
  uint32_t want = a.want;
  const uint64_t t0 = wall_clock64();
  if (wv == 0 && lane == 0) reinterpret_cast<volatile uint32_t*>(base + QcMail::live_off(a.slot))[b] = want;
  const uint32_t nkeys = a.nkeys;
  const uint4* qt_lo = nullptr;
  const uint4* qt_hi = nullptr;
  uint32_t kv_lo = 0, kv_hi = 0;
  if (wv == 0) {  // key data for keys < 128, two per lane
    qt_lo = lane < nkeys ? reinterpret_cast<const uint4* const*>(a.qtabs)[lane] : nullptr;
    qt_hi = lane + 64 < nkeys ? reinterpret_cast<const uint4* const*>(a.qtabs)[lane + 64] : nullptr;
    kv_lo = lane < nkeys ? a.key_valid[lane] : 0u;
    kv_hi = lane + 64 < nkeys ? a.key_valid[lane + 64] : 0u;
  }
  const uint4* gtab = reinterpret_cast<const uint4*>(a.gtab);
  const uint4* const* qtabs = reinterpret_cast<const uint4* const*>(a.qtabs);
  const bool helper = b >= QcMail::kQcSlots;  // (wide kernel only)
  uint64_t* const relay = a.relay;
  uint32_t last = 0;  // a helper's last relayed request (the relay starts at {0, 0}; numbers are never 0)
  const uint32_t* slot = reinterpret_cast<const uint32_t*>(base + QcMail::slot_off(helper ? 0 : b));
  const uint32_t* word = lane < 48 ? slot + lane : reinterpret_cast<const uint32_t*>(base) + (lane - 48);
  // this CU's word in the yield flags (and its instruction-cache partner's: cuyield 2)
  uint32_t* const cuf = a.cuflag ? a.cuflag + cu_flag_index() : nullptr;
  uint32_t* const cuf2 = cuf && a.cuyield == 2 ? a.cuflag + (cu_flag_index() ^ 1u) : nullptr;
  for (;; ++want) {
    uint32_t e[8] = {}, r[8] = {}, s[8] = {};
    bool key_ok = false;
    const uint4* qtab = nullptr;
    uint64_t seen_wall = 0, seen_clk = 0;
    if (wv == 0 && helper) {
      // ---- a helper workgroup's wave 0: wave 0 of workgroup 0 relays each
      // request's number and n through uncached device memory (see
      // k_ecdsa_wave_armed); a slot below n reads its signature from the
      // mailbox arrays in one round trip
      uint64_t rv = 0;
      for (;;) {
        rv = __hip_atomic_load(relay, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((uint32_t)rv != last || wall_clock64() - t0 > a.budget) break;
        __builtin_amdgcn_s_sleep(2);
      }
      const uint32_t seq = (uint32_t)rv, n = (uint32_t)(rv >> 32);
      uint32_t c = 0;
      if (seq != last && n != 0xFFFFFFFFu) {
        last = seq;
        c = b < n ? 1u : 2u;
        if (c == 1u) {
          seen_wall = wall_clock64();
          seen_clk = clock64();
          constexpr uint32_t cap = QcMail::kQcCap;
          const uint32_t* src = lane < 8    ? reinterpret_cast<const uint32_t*>(base + QcMail::hashes_off(cap) + 32 * b) + lane
                                : lane < 24 ? reinterpret_cast<const uint32_t*>(base + QcMail::sigs_off(cap) + 64 * b) + (lane - 8)
                                            : reinterpret_cast<const uint32_t*>(base + QcMail::keys_off(cap) + 4 * b);
          const uint32_t v = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          PBFTV_UNROLL for (int t = 0; t < 8; ++t) {
            e[7 - t] = bswap32(__builtin_amdgcn_readlane(v, t));
            r[7 - t] = bswap32(__builtin_amdgcn_readlane(v, 8 + t));
            s[7 - t] = bswap32(__builtin_amdgcn_readlane(v, 16 + t));
          }
          armed_key(__builtin_amdgcn_readlane(v, 24), nkeys, qt_lo, qt_hi, kv_lo, kv_hi, a.key_valid, qtabs, key_ok, qtab);
        }
      }
      if (c == 1u) raise_cu_flags(cuf, cuf2);
      if (lane == 0) cmd = c;
    } else if (wv == 0) {
      uint32_t v = 0;
      bool serve = false;
      for (;;) {
        v = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (__builtin_amdgcn_readlane(v, 0) == want && __builtin_amdgcn_readlane(v, 15) == want &&
            (b >= __builtin_amdgcn_readlane(v, 1) ||
             (__builtin_amdgcn_readlane(v, 16) == want && __builtin_amdgcn_readlane(v, 31) == want &&
              __builtin_amdgcn_readlane(v, 32) == want && __builtin_amdgcn_readlane(v, 47) == want))) {
          serve = true;
          break;
        }
        if (__builtin_amdgcn_readlane(v, 48 + 2) == want || __builtin_amdgcn_readlane(v, 48 + 5) != a.halt ||
            wall_clock64() - t0 > a.budget)
          break;  // header stop / halt, or the budget
        if (a.spin == 0) {
          __builtin_amdgcn_s_sleep(2);
        } else if (a.spin >= 1000) {  // (experiments) (spin - 1000) x s_sleep(8) between polls
          for (uint32_t j = 1000; j < a.spin; ++j) __builtin_amdgcn_s_sleep(8);
        } else if (a.spin > 1) {
          uint32_t x = lane;
          for (uint32_t j = 0; j < a.spin; ++j) asm volatile("v_mad_u32_u24 %0, %0, %0, %0" : "+v"(x));
        }
      }
      uint32_t c = 0;
      if (!serve) {
        if (b == 0 && relay && lane == 0)  // the helpers leave with workgroup 0
          __hip_atomic_store(relay, ((uint64_t)0xFFFFFFFFu << 32) | want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (lane == 0) __hip_atomic_store(mail->expired(a.slot), want, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        seen_wall = wall_clock64();
        seen_clk = clock64();
        const uint32_t n = __builtin_amdgcn_readlane(v, 1);
        if (b == 0 && relay && n > QcMail::kQcSlots && lane == 0)
          __hip_atomic_store(relay, ((uint64_t)n << 32) | want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        c = b < n ? 1u : 2u;
        if (c == 1u) {
          const uint32_t k = __builtin_amdgcn_readlane(v, 2);
          PBFTV_UNROLL for (int t = 0; t < 8; ++t) {  // slot line j, dword 4 + t = LE dword t of the hash / r / s
            e[7 - t] = bswap32(__builtin_amdgcn_readlane(v, 4 + t));
            r[7 - t] = bswap32(__builtin_amdgcn_readlane(v, 20 + t));
            s[7 - t] = bswap32(__builtin_amdgcn_readlane(v, 36 + t));
          }
          armed_key(k, nkeys, qt_lo, qt_hi, kv_lo, kv_hi, a.key_valid, qtabs, key_ok, qtab);
        }
      }
      if (c == 1u) raise_cu_flags(cuf, cuf2);
      if (lane == 0) cmd = c;
    }
    __syncthreads();
    const uint32_t c = (uint32_t)__builtin_amdgcn_readfirstlane((int)cmd);
    __syncthreads();  // (cmd is rewritten only after every wave has read it)
    if (c == 0u) return;
    if (c == 2u) continue;
    __builtin_amdgcn_s_setprio(3);
    const int ok = block_verify_rows<WG, WQ, false>(e, r, s, key_ok, gtab, qtab, &sh);  // 2: the host reruns it
    if (cuf && threadIdx.x == 0) {
      __hip_atomic_fetch_sub(cuf, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cuf2) __hip_atomic_fetch_sub(cuf2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (wv == 0 && lane == 0) {
      constexpr uint32_t cap = QcMail::kQcCap;
      if (a.stamps) {
        volatile uint64_t* st = reinterpret_cast<volatile uint64_t*>(base + QcMail::stamps_off(cap)) + 4 * b;
        st[0] = seen_wall;  // diagnostics (pbftv_qc_stamps), before the verdict
        st[1] = seen_clk;
        st[2] = wall_clock64();
        st[3] = clock64();
      }
      reinterpret_cast<volatile uint8_t*>(base)[QcMail::res_off(cap) + b] = (uint8_t)ok;
    }
    __builtin_amdgcn_s_setprio(0);
  }
}

// the row schedule (PBFTV_QC_ROWS=0: the quad schedule, for A/B), read at every launch
inline bool rows_enabled() {
  const char* e = getenv("PBFTV_QC_ROWS");
  return !(e && e[0] == '0');
}
inline uint64_t rows_max_batch() {  // launched: the row schedule up to this many signatures
  const char* e = getenv("PBFTV_QC_ROWS_MAX");
  return e ? strtoull(e, nullptr, 10) : 128;
}

template <int WG, int WQ>
void launch_armed_w(const ArmArgs& a, hipStream_t st) {
  // Whole CUs for the armed waves (opt-in, PBFTV_QC_EXCLUSIVE_CU, read at
  // every arming): an armed workgroup that takes its CU's whole LDS shares no
  // CU -- and no SIMD issue slots -- with a concurrent batch's blocks.
  // "narrow": the narrow kernel only (one CU per armed slot, up to 8); "1":
  // the wide kernel too (one CU per workgroup, up to 128 CUs).  Off by
  // default, as is PBFTV_QC_YIELD: a whole CU taken from a concurrent batch
  // costs it 3-7 % (each XCD's share waits for its slowest CU).
  // (experiments) a number k >= 2: the narrow row kernel's workgroups take k
  // KiB of LDS, so a concurrent batch fits fewer blocks (39 KiB each) on
  // their CUs -- a partial exclusivity
  const char* e = getenv("PBFTV_QC_EXCLUSIVE_CU");
  const bool wide = a.relay != nullptr;
  const bool excl = e && (e[0] == '1' || (!wide && e[0] == 'n'));
  const uint32_t part_kb = e && !wide && e[0] >= '2' && e[0] <= '9' ? (uint32_t)atoi(e) : 0u;
  if constexpr (RowsGeom<WG, WQ>::ok) {
    if (rows_enabled()) {
      const uint32_t rl = excl ? 160u * 1024u - 4096u : part_kb ? std::min(part_kb, 156u) * 1024u : 0u;  // (+ static LDS)
      if (rl) {
        static bool rattr = false;
        if (!rattr) {
          (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ecdsa_rows_armed<WG, WQ>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)(160u * 1024u - 4096u));
          rattr = true;
        }
      }
      const uint32_t cap = wide ? QcMail::kQcCap : QcMail::kQcSlots;
      const uint32_t slots = a.slots >= (wide ? QcMail::kQcSlots + 1 : 1) && a.slots <= cap ? a.slots : cap;
      hipLaunchKernelGGL((k_ecdsa_rows_armed<WG, WQ>), dim3(slots), dim3(64 * RowsGeom<WG, WQ>::waves), rl, st, a);
      return;
    }
  }
  const uint32_t lds = excl ? 160u * 1024u : 0u;
  if (lds) {
    static bool attr = false;  // (per instantiation)
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ecdsa_wave_armed<WG, WQ>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr = true;
    }
  }
  hipLaunchKernelGGL((k_ecdsa_wave_armed<WG, WQ>), dim3((a.relay ? QcMail::kQcCap : QcMail::kQcSlots) / 4), dim3(256), lds,
                     st, a);
}

template <int WG, int WQ>
void launch_wave_w(const uint8_t* hashes, const uint8_t* sigs, const uint32_t* key_idx, uint64_t n,
                          const uint32_t* key_valid, uint32_t nkeys, const uint32_t* gtab,
                          const uint32_t* const* qtabs,
                          uint8_t* bitmap, uint8_t* okbytes, hipStream_t st, bool one_wave = false) {
  if constexpr (RowsGeom<WG, WQ>::ok) {
    if (n <= rows_max_batch() && rows_enabled() && !one_wave) {
      hipLaunchKernelGGL((k_ecdsa_rows<WG, WQ>), dim3((uint32_t)n), dim3(64 * RowsGeom<WG, WQ>::waves), 0, st, hashes, sigs, key_idx,
                         n, key_valid, nkeys, reinterpret_cast<const uint4*>(gtab),
                         reinterpret_cast<const uint4* const*>(qtabs), bitmap, okbytes);
      return;
    }
  }
  if (one_wave) {
    hipLaunchKernelGGL((k_ecdsa_wave_lean<WG, WQ>), dim3((uint32_t)n), dim3(64), 0, st, hashes, sigs, key_idx, n,
                       key_valid, nkeys, reinterpret_cast<const uint4*>(gtab),
                       reinterpret_cast<const uint4* const*>(qtabs), bitmap, okbytes);
    return;
  }
  hipLaunchKernelGGL((k_ecdsa_wave<WG, WQ>), dim3((uint32_t)n), dim3(64), 0, st, hashes, sigs, key_idx, n, key_valid,
                     nkeys, reinterpret_cast<const uint4*>(gtab), reinterpret_cast<const uint4* const*>(qtabs), bitmap,
                     okbytes);
}

template <int WG, int WQ>
void launch_comb_w(const void* rec, uint64_t n, const uint32_t* gtab, const uint32_t* const* qtabs, uint8_t* bitmap,
                   uint8_t* okb, const uint32_t* cuflag, hipStream_t st) {
  const uint64_t blocks = (n + PBFTV_COMB_BLOCK - 1) / PBFTV_COMB_BLOCK;
  hipLaunchKernelGGL((k_ecdsa_comb<WG, WQ>), dim3((uint32_t)blocks), dim3(PBFTV_COMB_BLOCK), 0, st,
                     reinterpret_cast<const SigRec*>(rec), n, reinterpret_cast<const uint4*>(gtab),
                     reinterpret_cast<const uint4* const*>(qtabs), bitmap, okb, cuflag);
}

// One instantiation unit: the dispatchers for the geometry pairs COMBOS(X).
#define PBFTV_VERIFY_PART(NAME, COMBOS)                                                                       \
  bool launch_comb_part_##NAME(int wg, int wq, const CombArgs& a, hipStream_t st) {                           \
    COMBOS(PBFTV_PART_COMB_CASE)                                                                              \
    return false;                                                                                             \
  }                                                                                                           \
  bool launch_wave_part_##NAME(int wg, int wq, const WaveArgs& a, hipStream_t st) {                           \
    COMBOS(PBFTV_PART_WAVE_CASE)                                                                              \
    return false;                                                                                             \
  }                                                                                                           \
  bool launch_armed_part_##NAME(int wg, int wq, const ArmArgs& a, hipStream_t st) {                           \
    COMBOS(PBFTV_PART_ARMED_CASE)                                                                             \
    return false;                                                                                             \
  }
#define PBFTV_PART_COMB_CASE(G, Q)                                                                            \
  if (wg == G && wq == Q) {                                                                                   \
    launch_comb_w<G, Q>(a.rec, a.n, a.gtab, a.qtabs, a.bitmap, a.okb, a.cuflag, st);                                    \
    return true;                                                                                              \
  }
#define PBFTV_PART_ARMED_CASE(G, Q)                                                                           \
  if (wg == G && wq == Q) {                                                                                   \
    launch_armed_w<G, Q>(a, st);                                                                              \
    return true;                                                                                              \
  }
#define PBFTV_PART_WAVE_CASE(G, Q)                                                                            \
  if (wg == G && wq == Q) {                                                                                   \
    launch_wave_w<G, Q>(a.hashes, a.sigs, a.key_idx, a.n, a.key_valid, a.nkeys, a.gtab, a.qtabs, a.bitmap,    \
                        a.okbytes, st, a.one_wave);                                                           \
    return true;                                                                                              \
  }

}  // namespace pbftv
