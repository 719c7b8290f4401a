// gather_calib.hip -- calibrates rocprofv3 FETCH_SIZE for the comb's access
// shape (MI355X_MICROARCH.md: "calibrate on a known byte count in your own
// access pattern"): every lane fetches S random S-byte-aligned entries of a
// 64 GiB table by global_load_lds (16 B per instruction, S / 16 instructions
// per entry) into LDS, as k_ecdsa_comb streams its 64-B table entries.  Known
// algorithmic bytes = lanes x steps x S; the kernel's time gives the gather
// rate.  S = 64 (the comb) and S = 128 (two neighbouring entries: does a 64-B
// gather cost a whole 128-B line?).
//   hipcc -O3 --offload-arch=gfx950 -o tools/gather_calib tools/gather_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./tools/gather_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int kSteps = 21;

// M independent entries in flight per lane per step (memory-level parallelism)
template <int S, int M = 1, int AUX = 0>
__device__ __forceinline__ void gather(const uint4* __restrict__ tab, uint64_t entries, uint32_t seed,
                                       uint32_t* __restrict__ sink) {
  __shared__ uint4 buf[M * S / 16][256];
  const uint32_t t = threadIdx.x, wb = t & ~63u;
  uint64_t x = (uint64_t)(blockIdx.x * 256u + t) * 0x9E3779B97F4A7C15ull + seed;
  uint32_t acc = 0;
  for (int s = 0; s < kSteps; s += M) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      x ^= x >> 33;
      x *= 0xff51afd7ed558ccdull;
      x ^= x >> 29;
      const uint4* p = tab + (x % entries) * (S / 16);
#pragma unroll
      for (int k = 0; k < S / 16; ++k) __builtin_amdgcn_global_load_lds(p + k, &buf[m * (S / 16) + k][wb], 16, 0, AUX);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < M * S / 16; ++k) acc += buf[k][t].x;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (acc == 0x12345678u) sink[0] = acc;  // keeps the loads
}

__global__ void __launch_bounds__(256) k_gather64(const uint4* tab, uint64_t entries, uint32_t seed, uint32_t* sink) {
  gather<64>(tab, entries, seed, sink);
}
__global__ void __launch_bounds__(256) k_gather128(const uint4* tab, uint64_t entries, uint32_t seed, uint32_t* sink) {
  gather<128>(tab, entries, seed, sink);
}
__global__ void __launch_bounds__(256) k_gather64x3(const uint4* tab, uint64_t entries, uint32_t seed, uint32_t* sink) {
  gather<64, 3>(tab, entries, seed, sink);
}
__global__ void __launch_bounds__(256) k_gather64nt(const uint4* tab, uint64_t entries, uint32_t seed, uint32_t* sink) {
  gather<64, 1, 2>(tab, entries, seed, sink);  // nt (aux = 2)
}
__global__ void __launch_bounds__(256) k_gather64sc(const uint4* tab, uint64_t entries, uint32_t seed, uint32_t* sink) {
  gather<64, 1, 3>(tab, entries, seed, sink);  // sc0 | nt
}

int main() {
  const size_t bytes = 64ull << 30;
  uint4* tab = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(&tab, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(tab, 1, bytes);
  const uint32_t lanes = 1u << 20, blocks = lanes / 256;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep) {
    float ms64 = 0, ms128 = 0;
    hipEventRecord(a);
    hipLaunchKernelGGL(k_gather64, dim3(blocks), dim3(256), 0, 0, tab, bytes / 64, 17u + rep, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms64, a, b);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_gather128, dim3(blocks), dim3(256), 0, 0, tab, bytes / 128, 91u + rep, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms128, a, b);
    float ms64x3 = 0;
    hipEventRecord(a);
    hipLaunchKernelGGL(k_gather64x3, dim3(blocks), dim3(256), 0, 0, tab, bytes / 64, 53u + rep, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms64x3, a, b);
    float msnt = 0, mssc = 0;
    hipEventRecord(a);
    hipLaunchKernelGGL(k_gather64nt, dim3(blocks), dim3(256), 0, 0, tab, bytes / 64, 71u + rep, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&msnt, a, b);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_gather64sc, dim3(blocks), dim3(256), 0, 0, tab, bytes / 64, 73u + rep, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&mssc, a, b);
    printf("{\"rep\": %d, \"gather64_nt\": {\"ms\": %.4f}, \"gather64_aux3\": {\"ms\": %.4f}}\n", rep, msnt, mssc);
    const double g64 = (double)lanes * kSteps * 64, g128 = (double)lanes * kSteps * 128;
    printf("{\"rep\": %d, \"gather64\": {\"bytes\": %.0f, \"ms\": %.4f, \"GBps\": %.1f}, "
           "\"gather128\": {\"bytes\": %.0f, \"ms\": %.4f, \"GBps\": %.1f}, "
           "\"gather64_3_in_flight\": {\"bytes\": %.0f, \"ms\": %.4f, \"GBps\": %.1f}}\n",
           rep, g64, ms64, g64 / ms64 / 1e6, g128, ms128, g128 / ms128 / 1e6, g64, ms64x3, g64 / ms64x3 / 1e6);
  }
  hipFree(tab);
  hipFree(sink);
  return 0;
}
