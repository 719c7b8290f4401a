// Mixed-addition throughput microbenchmark for gfx950: cycles per wave per
// point addition for the comb kernel's addition formulas at 1..4 waves/SIMD,
// table entries streamed from a small L1/L2-resident table.  Measurement tool
// for DESIGN.md §3 (not part of the product).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I simple_pbft_amd/csrc tools/madd_bench.hip -o tools/madd_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "p256_algo.h"
#include "fes.h"

using namespace pbftv;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

__device__ __forceinline__ void ld_entry(const uint4* __restrict__ tab, int k, fe& x, fe& y) {
  const uint4* p = tab + (k & 63) * 4;
  uint4 e0 = p[0], e1 = p[1], e2 = p[2], e3 = p[3];
  uint32_t w[16] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w, e2.x, e2.y, e2.z, e2.w, e3.x, e3.y, e3.z, e3.w};
  entry_to_fe(x, y, w);
}

template <int V, int WAVES>
__global__ void __launch_bounds__(256, WAVES) kbench(const uint4* __restrict__ tab, uint32_t* __restrict__ out, int iters) {
  const int lane = blockIdx.x * 256 + threadIdx.x;
  fe x, y;
  ld_entry(tab, lane, x, y);
  if constexpr (V == 0) {
    jac acc;
    acc.x = x; acc.y = y; fe_set(acc.z, kOneP);
    for (int i = 0; i < iters; ++i) {
      fe ex, ey;
      ld_entry(tab, lane + 7 * i + 1, ex, ey);
      jac_madd<false>(acc, ex, ey);
    }
    for (int l = 0; l < 9; ++l) out[lane * 9 + l] = acc.x.v[l] ^ acc.z.v[l] ^ acc.y.v[l];
  } else if constexpr (V == 2) {
    xyzz_s acc;
    acc.x = x; acc.y = y; fe_set(acc.zz, kOneP); fe_set(acc.zzz, kOneP);
    for (int i = 0; i < iters; ++i) {
      fe ex, ey;
      ld_entry(tab, lane + 7 * i + 1, ex, ey);
      xyzz_madd_s(acc, ex, ey);
    }
    for (int l = 0; l < 9; ++l) out[lane * 9 + l] = acc.x.v[l] ^ acc.zz.v[l] ^ acc.y.v[l] ^ acc.zzz.v[l];
  } else if constexpr (V == 3) {
    // the comb's own step (comb_step_s's body): the y negation folded into
    // the entry unpacking, the W = sigma Y accumulator
    xyzz_s acc;
    acc.x = x; acc.y = y; fe_set(acc.zz, kOneP); fe_set(acc.zzz, kOneP);
    bool neg = false;
    for (int i = 0; i < iters; ++i) {
      const uint4* p = tab + ((lane + 7 * i + 1) & 63) * 4;
      uint4 e0 = p[0], e1 = p[1], e2 = p[2], e3 = p[3];
      uint32_t w[16] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w, e2.x, e2.y, e2.z, e2.w, e3.x, e3.y, e3.z, e3.w};
      fe ex, ey;
      entry_to_fe_cneg(ex, ey, w, ((lane + i) & 1) != neg);
      xyzz_madd_s_flip(acc, ex, ey);
      neg = !neg;
    }
    for (int l = 0; l < 9; ++l) out[lane * 9 + l] = acc.x.v[l] ^ acc.zz.v[l] ^ acc.y.v[l] ^ acc.zzz.v[l];
  } else {
    xyzz acc;
    acc.x = x; acc.y = y; fe_set(acc.zz, kOneP); fe_set(acc.zzz, kOneP);
    for (int i = 0; i < iters; ++i) {
      fe ex, ey;
      ld_entry(tab, lane + 7 * i + 1, ex, ey);
      xyzz_madd(acc, ex, ey);
    }
    for (int l = 0; l < 9; ++l) out[lane * 9 + l] = acc.x.v[l] ^ acc.zz.v[l] ^ acc.y.v[l] ^ acc.zzz.v[l];
  }
}

template <int V, int WAVES>
static void run(const char* name, const uint4* tab, uint32_t* out, int blocks, int iters) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((kbench<V, WAVES>), dim3(blocks), dim3(256), 0, 0, tab, out, 4);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL((kbench<V, WAVES>), dim3(blocks), dim3(256), 0, 0, tab, out, iters);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double waves = blocks * 4.0;
  const double cyc = ms * 1e-3 * 2.4e9 * 1024.0 / (waves * iters);
  printf("%-24s waves/SIMD>=%d blocks %6d: %8.3f ms  %7.0f SIMD-cycles per wave-addition  %.1f M adds/s\n", name,
         WAVES, blocks, ms, cyc, blocks * 256.0 * iters / (ms * 1e-3) / 1e6);
}

int main() {
  // 64 random-looking affine points: k*G for k = 1..64 would need the curve;
  // any canonical limbs will do for timing (formulas do not branch).
  uint32_t h[64 * 16];
  uint32_t s = 12345;
  for (int i = 0; i < 64 * 16; ++i) { s = s * 1664525u + 1013904223u; h[i] = s; }
  for (int i = 0; i < 64; ++i) { h[i * 16 + 7] &= 0x7fffffff; h[i * 16 + 15] &= 0x7fffffff; }
  uint4* tab;
  uint32_t* out;
  CHECK(hipMalloc(&tab, sizeof(h)));
  CHECK(hipMemcpy(tab, h, sizeof(h), hipMemcpyHostToDevice));
  const int blocks = 256 * 4 * 4;  // enough waves for 4/SIMD x 4 rounds
  CHECK(hipMalloc(&out, (size_t)blocks * 256 * 9 * 4));
  const int iters = 64;
  run<0, 1>("madd-2007-bl jacobian", tab, out, blocks, iters);
  run<0, 2>("madd-2007-bl jacobian", tab, out, blocks, iters);
  run<0, 3>("madd-2007-bl jacobian", tab, out, blocks, iters);
  run<0, 4>("madd-2007-bl jacobian", tab, out, blocks, iters);
  run<1, 1>("madd-2008-s xyzz", tab, out, blocks, iters);
  run<1, 2>("madd-2008-s xyzz", tab, out, blocks, iters);
  run<1, 3>("madd-2008-s xyzz", tab, out, blocks, iters);
  run<1, 4>("madd-2008-s xyzz", tab, out, blocks, iters);
  run<2, 1>("madd-2008-s xyzz signed", tab, out, blocks, iters);
  run<2, 2>("madd-2008-s xyzz signed", tab, out, blocks, iters);
  run<2, 3>("madd-2008-s xyzz signed", tab, out, blocks, iters);
  run<2, 4>("madd-2008-s xyzz signed", tab, out, blocks, iters);
  run<3, 2>("comb step (flip, cneg)", tab, out, blocks, iters);
  run<3, 4>("comb step (flip, cneg)", tab, out, blocks, iters);
  return 0;
}
