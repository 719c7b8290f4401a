// Field-multiplication alternatives for the comb's hot loop, measured against
// the product the comb uses: SIMD-cycles per wave per
// multiplication at 4 waves/SIMD with K independent chains per lane, and the
// XYZZ mixed addition built on each (the comb step of tools/madd_bench.hip).
//   V0 fs_mul       9 x 29-bit signed limbs, 81 v_mad_i64_i32 into 17 columns,
//                   Montgomery digits by p = -1 mod 2^29 (fes.h, the product);
//   V1 fs_mul_kara  the same columns by a 3 x 3-block Karatsuba (6 block
//                   products = 54 MADs, + the limb sums and the cross-term
//                   subtractions), same reduction;
//   V2 sol_mul      8 x 32-bit unsigned limbs, product scanning into a 96-bit
//                   accumulator, then the NIST special-form reduction of
//                   p = 2^256 - 2^224 + 2^192 + 2^96 - 1 (FIPS 186-4 D.2.3:
//                   T + 2 S1 + 2 S2 + S3 + S4 - D1 - D2 - D3 - D4, one signed
//                   carry pass, the top carry folded once; output < 2^256,
//                   not canonical -- the cheapest form a chain can use).
// Correctness: V1 against V0 limb for limb (same columns, same reduction) on
// 4096 random S/D-type pairs; V2's outputs for fixed inputs are printed for a
// big-integer check (tools/fmul_alt_check.py).  Measurement tool, not product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I simple_pbft_amd/csrc tools/fmul_alt_bench.hip -o tools/fmul_alt_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "p256_algo.h"
#include "fes.h"

using namespace pbftv;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

// ---- V1: 3 x 3-block Karatsuba columns, fes.h reduction ----
PBFTV_HD void mul3(uint64_t c[5], const uint32_t* a, const uint32_t* b) {
  c[0] = smul(a[0], b[0]);
  c[1] = smul(a[0], b[1]) + smul(a[1], b[0]);
  c[2] = smul(a[0], b[2]) + smul(a[1], b[1]) + smul(a[2], b[0]);
  c[3] = smul(a[1], b[2]) + smul(a[2], b[1]);
  c[4] = smul(a[2], b[2]);
}

PBFTV_HD void fs_mul_kara(fe& r, const fe& a, const fe& b) {
  PBFTV_FS_CONSTS;
  uint64_t P00[5], P11[5], P22[5], X01[5], X02[5], X12[5], t[17];
  uint32_t sa[3], sb[3];
  mul3(P00, a.v, b.v);
  mul3(P11, a.v + 3, b.v + 3);
  mul3(P22, a.v + 6, b.v + 6);
  PBFTV_UNROLL for (int k = 0; k < 3; ++k) { sa[k] = a.v[k] + a.v[3 + k]; sb[k] = b.v[k] + b.v[3 + k]; }
  mul3(X01, sa, sb);
  PBFTV_UNROLL for (int k = 0; k < 3; ++k) { sa[k] = a.v[k] + a.v[6 + k]; sb[k] = b.v[k] + b.v[6 + k]; }
  mul3(X02, sa, sb);
  PBFTV_UNROLL for (int k = 0; k < 3; ++k) { sa[k] = a.v[3 + k] + a.v[6 + k]; sb[k] = b.v[3 + k] + b.v[6 + k]; }
  mul3(X12, sa, sb);
  fs_cols_init(t);
  PBFTV_UNROLL for (int k = 0; k < 5; ++k) {
    t[k] += P00[k];
    t[6 + k] += P11[k];
    t[12 + k] += P22[k];
    t[3 + k] += X01[k] - P00[k] - P11[k];
    t[6 + k] += X02[k] - P00[k] - P22[k];
    t[9 + k] += X12[k] - P11[k] - P22[k];
  }
  PBFTV_UNROLL for (int i = 0; i < 8; ++i) fs_digit(t, i, c8, c9, c18, c21, c24);
  fs_digit_top(t, c9, c18, c21, c24);
  fs_out(r, t);
}

// ---- V2: 8 x 32-bit limbs, NIST special-form reduction ----
struct f32x8 {
  uint32_t v[8];
};

PBFTV_HD void sol_mul(f32x8& r, const f32x8& a, const f32x8& b) {
  uint32_t c[16];
  uint64_t acc = 0;
  uint32_t hi = 0;
  PBFTV_UNROLL for (int k = 0; k < 15; ++k) {
    PBFTV_UNROLL for (int i = 0; i < 8; ++i) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      const uint64_t p = (uint64_t)a.v[i] * b.v[j];
      acc += p;
      hi += acc < p ? 1u : 0u;
    }
    c[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  c[15] = (uint32_t)acc;
  // r = T + 2 S1 + 2 S2 + S3 + S4 - D1 - D2 - D3 - D4, word by word (signed)
  int64_t w[8];
  auto C = [&](int i) { return (int64_t)c[i]; };
  w[0] = C(0) + C(8) + C(9) - C(11) - C(12) - C(13) - C(14);
  w[1] = C(1) + C(9) + C(10) - C(12) - C(13) - C(14) - C(15);
  w[2] = C(2) + C(10) + C(11) - C(13) - C(14) - C(15);
  w[3] = C(3) + 2 * C(11) + 2 * C(12) + C(13) - C(15) - C(8) - C(9);
  w[4] = C(4) + 2 * C(12) + 2 * C(13) + C(14) - C(9) - C(10);
  w[5] = C(5) + 2 * C(13) + 2 * C(14) + C(15) - C(10) - C(11);
  w[6] = C(6) + 2 * C(14) + 2 * C(15) + C(14) + C(13) - C(8) - C(9);
  w[7] = C(7) + 2 * C(15) + C(15) + C(8) - C(10) - C(11) - C(12) - C(13);
  // carry pass, then fold the top carry k 2^256 = k (2^224 - 2^192 - 2^96 + 1)
  PBFTV_UNROLL for (int i = 0; i < 7; ++i) {
    w[i + 1] += w[i] >> 32;
    w[i] &= 0xFFFFFFFFll;
  }
  const int64_t k = w[7] >> 32;
  w[7] &= 0xFFFFFFFFll;
  w[0] += k;
  w[3] -= k;
  w[6] -= k;
  w[7] += k;
  PBFTV_UNROLL for (int i = 0; i < 7; ++i) {
    w[i + 1] += w[i] >> 32;
    w[i] &= 0xFFFFFFFFll;
  }
  PBFTV_UNROLL for (int i = 0; i < 8; ++i) r.v[i] = (uint32_t)w[i];
}

// ---- multiplication chains ----
template <int V, int K>
__global__ void __launch_bounds__(256) kmul(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int iters) {
  extern __shared__ uint32_t pad[];
  const int lane = blockIdx.x * 256 + threadIdx.x;
  uint32_t x = 0;
  if constexpr (V == 2) {
    f32x8 a[K], b;
    for (int l = 0; l < 8; ++l) b.v[l] = in[(lane * 7 + l) & 1023];
    for (int k = 0; k < K; ++k)
      for (int l = 0; l < 8; ++l) a[k].v[l] = in[(lane * 3 + 11 * k + l) & 1023] & 0x7FFFFFFFu;
    for (int i = 0; i < iters; ++i) {
      PBFTV_UNROLL for (int k = 0; k < K; ++k) sol_mul(a[k], a[k], b);
    }
    for (int k = 0; k < K; ++k)
      for (int l = 0; l < 8; ++l) x ^= a[k].v[l];
  } else {
    fe a[K], b;
    for (int l = 0; l < 9; ++l) b.v[l] = in[(lane * 7 + l) & 1023] & kMask29;
    for (int k = 0; k < K; ++k)
      for (int l = 0; l < 9; ++l) a[k].v[l] = in[(lane * 3 + 11 * k + l) & 1023] & kMask29;
    for (int i = 0; i < iters; ++i) {
      PBFTV_UNROLL for (int k = 0; k < K; ++k) {
        if constexpr (V == 0) fs_mul(a[k], a[k], b);
        else fs_mul_kara(a[k], a[k], b);
      }
    }
    for (int k = 0; k < K; ++k)
      for (int l = 0; l < 9; ++l) x ^= a[k].v[l];
  }
  if (threadIdx.x == 0) pad[0] = x;
  __syncthreads();
  out[lane] = x ^ pad[0];
}

// ---- the comb step (madd_bench V3) on fs_mul or on fs_mul_kara ----
template <bool KARA>
__device__ __forceinline__ void mulv(fe& r, const fe& a, const fe& b) {
  if constexpr (KARA) fs_mul_kara(r, a, b);
  else fs_mul(r, a, b);
}

template <bool KARA>
__device__ __forceinline__ void step(xyzz_s& acc, const fe& x2, const fe& y2) {
  fe u2, s2, p, r, pp, ppp, q, t;
  mulv<KARA>(u2, x2, acc.zz);
  mulv<KARA>(s2, y2, acc.zzz);
  fs_sub(p, u2, acc.x);
  fs_sub(r, s2, acc.y);
  fs_sqr(pp, p);
  mulv<KARA>(ppp, p, pp);
  mulv<KARA>(q, acc.x, pp);
  fe x3;
  fs_sqr_sub2(x3, r, ppp, q);
  fs_sub(t, x3, q);
  fs_mul2_add(acc.y, r, t, acc.y, ppp);
  mulv<KARA>(acc.zz, acc.zz, pp);
  mulv<KARA>(acc.zzz, acc.zzz, ppp);
  acc.x = x3;
}

template <bool KARA>
__global__ void __launch_bounds__(256, 4) kstep(const uint4* __restrict__ tab, uint32_t* __restrict__ out, int iters) {
  const int lane = blockIdx.x * 256 + threadIdx.x;
  auto ld = [&](int k, fe& x, fe& y, bool neg) {
    const uint4* p = tab + (k & 63) * 4;
    uint4 e0 = p[0], e1 = p[1], e2 = p[2], e3 = p[3];
    uint32_t w[16] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w, e2.x, e2.y, e2.z, e2.w, e3.x, e3.y, e3.z, e3.w};
    entry_to_fe_cneg(x, y, w, neg);
  };
  xyzz_s acc;
  ld(lane, acc.x, acc.y, false);
  fe_set(acc.zz, kOneP);
  fe_set(acc.zzz, kOneP);
  bool neg = false;
  for (int i = 0; i < iters; ++i) {
    fe ex, ey;
    ld(lane + 7 * i + 1, ex, ey, ((lane + i) & 1) != neg);
    step<KARA>(acc, ex, ey);
    neg = !neg;
  }
  for (int l = 0; l < 9; ++l) out[lane * 9 + l] = acc.x.v[l] ^ acc.zz.v[l] ^ acc.y.v[l] ^ acc.zzz.v[l];
}

template <int V, int K>
static void run_mul(const char* name, const uint32_t* in, uint32_t* out, int iters) {
  const int blocks = 256 * 8 * 2;
  const size_t lds = 160 * 1024 / 4 - 256;  // 4 waves/SIMD
  CHECK(hipFuncSetAttribute((const void*)kmul<V, K>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((kmul<V, K>), dim3(blocks), dim3(256), lds, 0, in, out, 2);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL((kmul<V, K>), dim3(blocks), dim3(256), lds, 0, in, out, iters);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  const double cyc = best * 1e-3 * 2.4e9 * 1024.0 / (blocks * 4.0 * iters * K);
  printf("mul  %-12s K=%d waves/SIMD=4: %8.3f ms  %6.0f SIMD-cycles per wave-mul (2.4 GHz nominal)\n", name, K, best, cyc);
}

template <bool KARA>
static void run_step(const char* name, const uint4* tab, uint32_t* out, int iters) {
  const int blocks = 256 * 4 * 4;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((kstep<KARA>), dim3(blocks), dim3(256), 0, 0, tab, out, 4);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL((kstep<KARA>), dim3(blocks), dim3(256), 0, 0, tab, out, iters);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  const double cyc = best * 1e-3 * 2.4e9 * 1024.0 / (blocks * 4.0 * iters);
  printf("step %-12s waves/SIMD>=4: %8.3f ms  %6.0f SIMD-cycles per wave-addition  %.1f M adds/s\n", name, best, cyc,
         blocks * 256.0 * iters / (best * 1e-3) / 1e6);
}

// V1 == V0 limb for limb on random S/D-type inputs (device), and V2 on fixed inputs (printed)
__global__ void kcheck(const uint32_t* __restrict__ in, uint32_t* __restrict__ bad, uint32_t* __restrict__ sol_out) {
  const int lane = blockIdx.x * 256 + threadIdx.x;
  fe a, b, r0, r1;
  for (int l = 0; l < 9; ++l) {
    a.v[l] = in[(lane * 5 + l) & 1023] & kMask29;
    b.v[l] = (in[(lane * 13 + 3 * l) & 1023] & kMask29) - (in[(lane * 17 + l) & 1023] & kMask29);  // D-type
  }
  a.v[8] = (uint32_t)((int32_t)in[(lane * 5 + 8) & 1023] >> 4);  // signed top limb (|.| < 2^27), S-type
  b.v[8] = (uint32_t)((int32_t)b.v[8] >> 4);
  fs_mul(r0, a, b);
  fs_mul_kara(r1, a, b);
  uint32_t d = 0;
  for (int l = 0; l < 9; ++l) d |= r0.v[l] ^ r1.v[l];
  if (d) atomicAdd(bad, 1u);
  if (lane < 4) {
    f32x8 x, y, z;
    for (int l = 0; l < 8; ++l) {
      x.v[l] = in[(lane * 16 + l) & 1023];
      y.v[l] = in[(lane * 16 + 8 + l) & 1023];
    }
    sol_mul(z, x, y);
    for (int l = 0; l < 8; ++l) sol_out[lane * 24 + l] = x.v[l];
    for (int l = 0; l < 8; ++l) sol_out[lane * 24 + 8 + l] = y.v[l];
    for (int l = 0; l < 8; ++l) sol_out[lane * 24 + 16 + l] = z.v[l];
  }
}

int main() {
  uint32_t h[1024];
  uint32_t s = 12345;
  for (int i = 0; i < 1024; ++i) { s = s * 1664525u + 1013904223u; h[i] = s; }
  uint32_t *in, *out, *bad, *sol;
  CHECK(hipMalloc(&in, sizeof(h)));
  CHECK(hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice));
  CHECK(hipMalloc(&out, (size_t)256 * 8 * 2 * 256 * 4 * 9));
  CHECK(hipMalloc(&bad, 4));
  CHECK(hipMalloc(&sol, 4 * 24 * 4));
  CHECK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL(kcheck, dim3(16), dim3(256), 0, 0, in, bad, sol);
  uint32_t nbad = 0, hs[96];
  CHECK(hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hs, sol, sizeof(hs), hipMemcpyDeviceToHost));
  printf("check fs_mul_kara vs fs_mul: %u of 4096 differ\n", nbad);
  for (int i = 0; i < 4; ++i) {
    printf("sol_mul");
    for (int j = 0; j < 24; ++j) printf(" %08x", hs[i * 24 + j]);
    printf("\n");
  }
  run_mul<0, 1>("fs_mul", in, out, 256);
  run_mul<0, 2>("fs_mul", in, out, 128);
  run_mul<1, 1>("fs_mul_kara", in, out, 256);
  run_mul<1, 2>("fs_mul_kara", in, out, 128);
  run_mul<2, 1>("sol_mul", in, out, 256);
  run_mul<2, 2>("sol_mul", in, out, 128);
  // the step: entries from a 64-entry table (madd_bench's)
  uint32_t t[64 * 16];
  s = 12345;
  for (int i = 0; i < 64 * 16; ++i) { s = s * 1664525u + 1013904223u; t[i] = s; }
  for (int i = 0; i < 64; ++i) { t[i * 16 + 7] &= 0x7fffffff; t[i * 16 + 15] &= 0x7fffffff; }
  uint4* tab;
  CHECK(hipMalloc(&tab, sizeof(t)));
  CHECK(hipMemcpy(tab, t, sizeof(t), hipMemcpyHostToDevice));
  run_step<false>("fs_mul", tab, out, 64);
  run_step<true>("fs_mul_kara", tab, out, 64);
  return nbad != 0;
}
