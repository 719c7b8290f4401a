// gather_comb.hip -- the comb's table reads with no arithmetic, in the comb's
// own access pattern: does k_ecdsa_comb sit on a
// random-gather ceiling?  Everything but the field arithmetic is reproduced:
//   * footprint: one 120 GB G-table allocation (CombGeom<29>) + one block of
//     100 key tables (CombGeom<21>, 1.14 GB each) = 234 GB, as registration
//     allocates them (pbftv_api.cpp build_key_tables);
//   * lanes in KEY ORDER (lane p holds key p * keys / n), blocks remapped
//     XCD-aware exactly as k_ecdsa_comb does (block b -> range (b % 8) nb / 8
//     + b / 8);
//   * the joint step order of CombSteps<29, 21> (G / key windows alternating,
//     then the key table's last three), one uniformly random entry of the
//     step's window per lane (a uniform signed digit);
//   * one 64-B entry per step streamed into LDS by four 16-B global_load_lds,
//     one step ahead (issue next, then wait for and read the current);
//   * 256-thread blocks at the comb's occupancy (--waves 4: 39 KB of LDS per
//     block as the comb holds) or free (--waves 0).
// Reports ms and the gather rate over the 21 x 64 B x n algorithmic bytes.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o tools/gather_comb tools/gather_comb.hip
//   ./tools/gather_comb [n=1048576] [reps=5]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../simple_pbft_amd/csrc/p256_algo.h"

using namespace pbftv;

constexpr int WG = 29, WQ = 21;
using GG = CombGeom<WG>;
using GQ = CombGeom<WQ>;
constexpr int nG = GG::kWin, nQ = GQ::kWin, nMin = nG < nQ ? nG : nQ, nD = nG + nQ;

__host__ __device__ constexpr bool is_q(int j) { return j < 2 * nMin ? (j & 1) != 0 : nQ > nG; }
__host__ __device__ constexpr int win(int j) { return j < 2 * nMin ? j >> 1 : j - nMin; }

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 29;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 32);
}

template <int PAD>
__global__ void __launch_bounds__(256) k_gather_comb(const uint4* __restrict__ gtab, const uint4* __restrict__ qblock,
                                                     uint64_t qtab_entries, uint32_t nkeys, uint64_t n, uint32_t seed,
                                                     uint32_t* __restrict__ sink) {
  __shared__ uint4 sent[4][256];
  __shared__ uint4 pad[PAD > 0 ? PAD : 1];  // the comb's other LDS (digits): same blocks per CU
  const uint32_t t = threadIdx.x, wb = t & ~63u;
  const uint32_t nb = gridDim.x, b = blockIdx.x, per = nb / 8;
  const uint32_t blk = b < 8 * per ? (b % 8) * per + b / 8 : b;
  const uint64_t p = (uint64_t)blk * blockDim.x + t;
  const uint32_t key = (uint32_t)(p * nkeys / n);
  const uint4* qtab = qblock + (uint64_t)key * qtab_entries * 4;
  uint32_t acc = PAD > 0 ? pad[t % (PAD > 0 ? PAD : 1)].x : 0u;
  auto ptr = [&](int j) {
    const uint64_t r = mix(p * 0x9E3779B97F4A7C15ull + (uint64_t)j * 0x632BE59BD9B4E019ull + seed);
    if (is_q(j)) return qtab + (GQ::base(win(j)) + r % GQ::ent(win(j))) * 4;
    return gtab + (GG::base(win(j)) + r % GG::ent(win(j))) * 4;
  };
  auto issue = [&](const uint4* e) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < 4; ++k) __builtin_amdgcn_global_load_lds(e + k, &sent[k][wb], 16, 0, 0);
  };
  issue(ptr(0));
#pragma unroll 1
  for (int j = 0; j < nD; ++j) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint4 e[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = sent[k][t];
    if (j + 1 < nD) issue(ptr(j + 1));
    acc += e[0].x ^ e[1].y ^ e[2].z ^ e[3].w;
  }
  if (acc == 0x12345678u && p < n) sink[0] = acc;  // keeps the loads
}

#define CHECK(x)                                                                                  \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
      exit(1);                                                                                    \
    }                                                                                             \
  } while (0)

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 20);
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const uint32_t nkeys = 100;
  const uint64_t qent = GQ::kWords / 16;  // entries (64 B) per key table
  uint4 *gtab = nullptr, *qblock = nullptr;
  uint32_t* sink = nullptr;
  CHECK(hipMalloc(&gtab, GG::kBytes));
  CHECK(hipMalloc(&qblock, GQ::kBytes * nkeys));
  CHECK(hipMalloc(&sink, 64));
  const uint64_t blocks = (n + 255) / 256;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const double bytes = (double)n * nD * 64;
  printf("{\"footprint_GB\": %.1f, \"n\": %llu, \"steps\": %d, \"algorithmic_bytes\": %.0f}\n",
         (GG::kBytes + GQ::kBytes * nkeys) / 1e9, (unsigned long long)n, nD, bytes);
  for (int rep = 0; rep < reps; ++rep) {
    float ms[2];
    for (int v = 0; v < 2; ++v) {
      // warm the clocks / TLB paths with one untimed launch per variant
      for (int w = 0; w < 2; ++w) {
        CHECK(hipEventRecord(a));
        if (v == 0)
          hipLaunchKernelGGL(k_gather_comb<0>, dim3((uint32_t)blocks), dim3(256), 0, 0, gtab, qblock, qent, nkeys, n,
                             1000u * rep + 17u * w, sink);
        else  // the comb's LDS per block (digits: 21 x 256 x 4 B + entries 16 KB = ~39 KB) -> its blocks per CU
          hipLaunchKernelGGL(k_gather_comb<1344>, dim3((uint32_t)blocks), dim3(256), 0, 0, gtab, qblock, qent, nkeys,
                             n, 1000u * rep + 17u * w + 5u, sink);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms[v], a, b));
      }
    }
    printf("{\"rep\": %d, \"free_occupancy\": {\"ms\": %.4f, \"TBps\": %.3f}, \"comb_lds\": {\"ms\": %.4f, \"TBps\": %.3f}}\n",
           rep, ms[0], bytes / ms[0] / 1e9, ms[1], bytes / ms[1] / 1e9);
  }
  CHECK(hipFree(gtab));
  CHECK(hipFree(qblock));
  CHECK(hipFree(sink));
  return 0;
}
