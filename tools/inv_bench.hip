// Throughput of the per-lane mod-n inversions (every lane a different value,
// as in k_ecdsa_scalars): variable-time safegcd (divergent loop) vs the
// constant-time divstep batches, SIMD-cycles per wave-inversion at full
// occupancy.  Measurement tool for DESIGN.md §3 (not part of the product).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I simple_pbft_amd/csrc tools/inv_bench.hip -o tools/inv_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "safegcd.h"

using namespace pbftv;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

template <int V>
__global__ void __launch_bounds__(256) kinv(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int iters) {
  const uint32_t lane = blockIdx.x * 256 + threadIdx.x;
  uint32_t x[8];
  for (int k = 0; k < 8; ++k) x[k] = in[(lane * 8 + k) & 4095];
  x[7] &= 0x7FFFFFFF;  // < n
  x[0] |= 1;
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t w[8];
    if constexpr (V == 0) inv_mod_n_words(w, x);
    else inv_mod_n_words_ct(w, x);
    acc ^= w[3];
    x[1] ^= w[0] & 0xFF;  // keep values changing (and < n)
  }
  out[lane] = acc;
}

template <int V>
static void run(const char* name, const uint32_t* in, uint32_t* out) {
  const int blocks = 256 * 8, iters = 4;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(kinv<V>, dim3(blocks), dim3(256), 0, 0, in, out, 1);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(kinv<V>, dim3(blocks), dim3(256), 0, 0, in, out, iters);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double waves = blocks * 4.0;
  printf("%-28s %8.3f ms  %8.0f SIMD-cycles per wave-inversion\n", name, ms,
         ms * 1e-3 * 2.4e9 * 1024.0 / (waves * iters));
}

int main() {
  uint32_t h[4096];
  uint32_t s = 777;
  for (int i = 0; i < 4096; ++i) { s = s * 1664525u + 1013904223u; h[i] = s; }
  uint32_t *in, *out;
  CHECK(hipMalloc(&in, sizeof(h)));
  CHECK(hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice));
  CHECK(hipMalloc(&out, 256 * 8 * 256 * 4));
  run<0>("safegcd variable-time", in, out);
  run<1>("safegcd constant-time", in, out);
  run<0>("safegcd variable-time", in, out);
  run<1>("safegcd constant-time", in, out);
  return 0;
}
