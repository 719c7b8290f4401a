// Field-multiplication throughput microbenchmark for gfx950: cycles per wave
// per fe_mul for the product/reduction schedules in fe29.h, with K
// independent dependency chains per lane (ILP) and LDS-limited occupancy.
// Measurement tool for DESIGN.md §3 (not part of the product).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I simple_pbft_amd/csrc tools/fmul_bench.hip -o tools/fmul_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "fe29.h"

using namespace pbftv;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

template <int V>
__device__ __forceinline__ void mul_v(fe& r, const fe& a, const fe& b) {
  if constexpr (V == 0) fe_mul(r, a, b);
  else if constexpr (V == 1) fe_mul_rows_then_reduce(r, a, b);
  else if constexpr (V == 2) fe_sqr(r, a);
  else fe_sqr_il(r, a);
}

// occupancy limited by dynamic LDS: lds_bytes per 256-thread block
template <int V, int K>
__global__ void __launch_bounds__(256) kbench(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int iters) {
  extern __shared__ uint32_t pad[];
  const int lane = blockIdx.x * 256 + threadIdx.x;
  fe a[K], b;
  for (int l = 0; l < 9; ++l) b.v[l] = in[(lane * 7 + l) & 1023] & kMask29;
  for (int k = 0; k < K; ++k)
    for (int l = 0; l < 9; ++l) a[k].v[l] = in[(lane * 3 + 11 * k + l) & 1023] & kMask29;
  for (int i = 0; i < iters; ++i) {
    PBFTV_UNROLL for (int k = 0; k < K; ++k) mul_v<V>(a[k], a[k], b);
  }
  uint32_t x = 0;
  for (int k = 0; k < K; ++k)
    for (int l = 0; l < 9; ++l) x ^= a[k].v[l];
  if (threadIdx.x == 0) pad[0] = x;
  __syncthreads();
  out[lane] = x ^ pad[0];
}

template <int V, int K>
static void run(const char* name, const uint32_t* in, uint32_t* out, int waves_per_simd, int iters) {
  const int blocks = 256 * 8 * 2;
  const size_t lds = 160 * 1024 / waves_per_simd - 256;
  CHECK(hipFuncSetAttribute((const void*)kbench<V, K>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((kbench<V, K>), dim3(blocks), dim3(256), lds, 0, in, out, 2);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL((kbench<V, K>), dim3(blocks), dim3(256), lds, 0, in, out, iters);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double waves = blocks * 4.0;
  const double cyc = ms * 1e-3 * 2.4e9 * 1024.0 / (waves * iters * K);
  printf("%-12s K=%d waves/SIMD=%d: %8.3f ms  %6.0f SIMD-cycles per wave-op\n", name, K, waves_per_simd, ms, cyc);
}

template <int V>
static void sweep(const char* name, const uint32_t* in, uint32_t* out) {
  for (int w : {1, 2, 4}) {
    run<V, 1>(name, in, out, w, 256);
    run<V, 2>(name, in, out, w, 128);
    run<V, 4>(name, in, out, w, 64);
  }
}

int main() {
  uint32_t h[1024];
  uint32_t s = 12345;
  for (int i = 0; i < 1024; ++i) { s = s * 1664525u + 1013904223u; h[i] = s; }
  uint32_t *in, *out;
  CHECK(hipMalloc(&in, sizeof(h)));
  CHECK(hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice));
  CHECK(hipMalloc(&out, 256 * 8 * 2 * 256 * 4));
  sweep<0>("fe_mul", in, out);
  sweep<1>("fe_mul_rows_then_reduce", in, out);
  sweep<2>("fe_sqr", in, out);
  sweep<3>("fe_sqr_il", in, out);
  return 0;
}
