// rows_probe.hip -- stage stamps of the row schedule (k_ecdsa_rows, the
// launched latency kernel: eight waves per signature, verify_kernels.h
// block_verify_rows), built with PBFTV_ROWS_PROBE: wall_clock64() of wave 0
// at each stage boundary.  Tables: the n = 4 geometry (29-bit G, one 24-bit
// key table with Q = G), built with the product's table kernels.  Measurement
// tool for DESIGN.md (not the product).
//   make -C simple_pbft_amd && hipcc --offload-arch=gfx950 -O3 -std=c++17 -c tools/rows_probe.hip -o /tmp/rp.o \
//   && hipcc --offload-arch=gfx950 /tmp/rp.o simple_pbft_amd/build/p256_*.o -o tools/rows_probe
#define PBFTV_ROWS_PROBE 1
#include "../simple_pbft_amd/csrc/verify_kernels.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>
#include <unistd.h>

using namespace pbftv;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

#ifndef PROBE_WQ
#define PROBE_WQ 24
#endif
constexpr int WG = 29, WQ = PROBE_WQ;  // (-DPROBE_WQ=20: 13 windows, seven waves)

// k_ecdsa_rows' body in a kernel of this unit (the library's objects carry
// their own, unstamped, instantiation of the template)
__global__ void __launch_bounds__(64 * kRowWaves) rows_probe_k(const uint8_t* __restrict__ hashes,
                                                               const uint8_t* __restrict__ sigs,
                                                               const uint32_t* __restrict__ key_idx, uint64_t n,
                                                               const uint32_t* __restrict__ key_valid, uint32_t nkeys,
                                                               const uint4* __restrict__ gtab,
                                                               const uint4* const* __restrict__ qtabs,
                                                               uint8_t* __restrict__ bitmap) {
  __shared__ RowsShared sh;
  const uint64_t i = blockIdx.x;
  uint32_t e[8] = {}, r[8] = {}, s[8] = {};
  bool key_ok = false;
  const uint4* qtab = nullptr;
  if (threadIdx.x < 64) wave_load_sig(hashes, sigs, key_idx, i, key_valid, nkeys, qtabs, e, r, s, key_ok, qtab);
  const bool ok = block_verify_rows<WG, WQ, true>(e, r, s, key_ok, gtab, qtab, &sh) & 1;
  if (threadIdx.x == 0) wave_store_verdict(ok, i, n, bitmap, nullptr);
}

// Background load for the stage stamps (argv[1]): "gather" -- random 64-B
// loads over a 4-GB buffer at about the rate the comb's table gathers stream
// through L2 and HBM (~1.2 TB/s); "valu" -- 64-bit MAD chains, no memory; "both"; "none".  Two waves per
// SIMD on every CU (room is left for the probe's eight waves), until the host
// raises *stop (or a 3-s budget).
__global__ void __launch_bounds__(256) load_k(const uint4* __restrict__ buf, uint64_t nlines, int mode,
                                              const uint32_t* stop, uint32_t* __restrict__ sink, uint64_t budget) {
  const uint64_t t0 = wall_clock64();
  uint64_t x = 0x9E3779B97F4A7C15ull * (blockIdx.x * 256 + threadIdx.x + 1), acc = x;
  for (int it = 0;; ++it) {
    if ((it & 15) == 0 &&
        (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0 || wall_clock64() - t0 > budget))
      break;
    if (mode & 1) {  // one random 64-B line per thread per ~7 us: ~1.2 TB/s over the chip, the comb's gather rate
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      const uint4 v = buf[(x >> 20) % nlines];
      acc ^= (uint64_t)v.x + v.y + v.z + v.w;
      __builtin_amdgcn_s_sleep(127);
      __builtin_amdgcn_s_sleep(127);
    }
    if (mode & 2) {
#pragma unroll
      for (int k = 0; k < 256; ++k) acc = ((uint64_t)(uint32_t)acc * ((uint32_t)(acc >> 29) | 1u) + acc) ^ (uint64_t)k;
    }
  }
  if (acc == 0x123456789ull) sink[0] = (uint32_t)acc;
}

int main(int argc, char** argv) {
  const char* lmode = argc > 1 ? argv[1] : "none";
  const int mode = !strcmp(lmode, "gather") ? 1 : !strcmp(lmode, "valu") ? 2 : !strcmp(lmode, "both") ? 3 : 0;
  const uint32_t n = 64;
  // key = G (valid), random in-range r, s, e: the stages run in full whatever the verdict
  std::vector<uint8_t> h(32 * n), sg(64 * n), key(64);
  uint32_t x = 12345;
  auto rnd = [&]() { x = x * 1664525u + 1013904223u; return (uint8_t)(x >> 24); };
  for (auto& b : h) b = rnd();
  for (uint32_t i = 0; i < n; ++i)
    for (int k = 0; k < 64; ++k) sg[64 * i + k] = (k % 32 == 0) ? 0x7F : rnd();  // r, s < n
  const uint32_t gx[8] = {0xd898c296, 0xf4a13945, 0x2deb33a0, 0x77037d81, 0x63a440f2, 0xf8bce6e5, 0xe12c4247, 0x6b17d1f2};
  const uint32_t gy[8] = {0x37bf51f5, 0xcbb64068, 0x6b315ece, 0x2bce3357, 0x7c0f9e16, 0x8ee7eb4a, 0xfe1a7f9b, 0x4fe342e2};
  std::vector<uint32_t> keys_le(16);
  for (int k = 0; k < 8; ++k) { keys_le[k] = gx[k]; keys_le[8 + k] = gy[k]; }
  uint8_t *dh, *ds;
  uint32_t *dk, *dkeys, *dvalid, *dsink;
  uint64_t* dst;
  CHECK(hipMalloc(&dh, h.size()));
  CHECK(hipMalloc(&ds, sg.size()));
  CHECK(hipMalloc(&dk, 4 * n));
  CHECK(hipMalloc(&dkeys, 64));
  CHECK(hipMalloc(&dvalid, 64));
  CHECK(hipMalloc(&dsink, 4 * n));
  CHECK(hipMalloc(&dst, 8 * 5 * n));
  CHECK(hipMemcpy(dh, h.data(), h.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(ds, sg.data(), sg.size(), hipMemcpyHostToDevice));
  CHECK(hipMemset(dk, 0, 4 * n));
  CHECK(hipMemcpy(dkeys, keys_le.data(), 64, hipMemcpyHostToDevice));
  uint32_t *gt, *qt;
  CHECK(hipMalloc(&gt, table_bytes(WG)));
  CHECK(hipMalloc(&qt, table_bytes(WQ)));
  for (int w : {WG, WQ}) {
    const TableScratchSizes z = table_scratch_sizes(w, 1);
    void *b, *l, *hb, *ss, *es;
    CHECK(hipMalloc(&b, z.bases)); CHECK(hipMalloc(&l, z.lbuf)); CHECK(hipMalloc(&hb, z.hbuf));
    CHECK(hipMalloc(&ss, z.small_scratch)); CHECK(hipMalloc(&es, z.entry_scratch));
    TableScratch sc{b, l, hb, ss, es, z.entry_lanes};
    uint32_t** dtab;
    uint32_t* tab = w == WG ? gt : qt;
    CHECK(hipMalloc(&dtab, sizeof(void*)));
    CHECK(hipMemcpy(dtab, &tab, sizeof(void*), hipMemcpyHostToDevice));
    CHECK(launch_build_tables(w, dkeys, 0, 1, w == WG ? 1 : 0, dvalid, dtab, sc, 0));
    CHECK(hipDeviceSynchronize());
    CHECK(hipFree(b)); CHECK(hipFree(l)); CHECK(hipFree(hb)); CHECK(hipFree(ss)); CHECK(hipFree(es));
  }
  int rate_khz = 0;
  CHECK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
  const uint32_t** dq;
  CHECK(hipMalloc(&dq, sizeof(void*)));
  CHECK(hipMemcpy(dq, &qt, sizeof(void*), hipMemcpyHostToDevice));
  uint8_t* dbm;
  CHECK(hipMalloc(&dbm, n / 8 + 8));
  const int kS = 16;
  const int stages[] = {1, 2, 3, 4, 5, 7, 8, 9, 10, 12, 13};
  const char* names[] = {"scalars", "handoff", "digits_entries", "level0_mmadd", "wave_pair_add", "l1_barrier",
                         "l1_add", "l2_barrier", "l2_add", "l3_barrier", "l3_check"};
  printf("{\"geometry\": [%d, %d], \"load\": \"%s\"", WG, WQ, lmode);
  const uint64_t kLines = (4ull << 30) / 16;
  uint4* lbuf = nullptr;
  uint32_t* lstop = nullptr;
  hipStream_t ls = nullptr;
  if (mode) {
    CHECK(hipMalloc(&lbuf, kLines * 16));
    CHECK(hipMemset(lbuf, 0x5A, kLines * 16));
    CHECK(hipHostMalloc(&lstop, 64, hipHostMallocCoherent | hipHostMallocMapped));
    CHECK(hipStreamCreateWithFlags(&ls, hipStreamNonBlocking));
    CHECK(hipDeviceSynchronize());
  }
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  for (uint32_t nb : {1u, 3u, 64u}) {
    if (mode) {  // the load runs for the whole rep loop, then stops
      *(volatile uint32_t*)lstop = 0;
      hipLaunchKernelGGL(load_k, dim3(2 * ncu), dim3(256), 0, ls, lbuf, kLines, mode, lstop, dsink,
                         (uint64_t)rate_khz * 3000);
      CHECK(hipGetLastError());
      usleep(20000);
    }
    for (int rep = 0; rep < 4; ++rep) {
      hipLaunchKernelGGL(rows_probe_k, dim3(nb), dim3(64 * RowsGeom<WG, WQ>::waves), 0, 0, dh, ds, dk, (uint64_t)nb, dvalid, 1u,
                         reinterpret_cast<const uint4*>(gt), reinterpret_cast<const uint4* const*>(dq), dbm);
      CHECK(hipStreamSynchronize(0));  // (not the device: the load kernel runs on)
    }
    if (mode) {
      *(volatile uint32_t*)lstop = 1;
      CHECK(hipStreamSynchronize(ls));
    }
    std::vector<uint64_t> st(128 * 8 * kS);
    CHECK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_rows_probe), 8 * 128 * 8 * kS));
    printf(", \"n%u\": {", nb);
    // wave 0's timeline: median over the workgroups of each stage
    for (size_t k = 0; k < sizeof(stages) / sizeof(int); ++k) {
      std::vector<double> d;
      for (uint32_t b = 0; b < nb && b < 128; ++b) {
        const uint64_t* s = &st[b * 8 * kS];
        const uint64_t pv = k == 0 ? s[0] : s[stages[k - 1]];
        d.push_back((double)(s[stages[k]] - pv) * 1e3 / rate_khz);
      }
      std::sort(d.begin(), d.end());
      printf("%s\"%s_us\": %.2f", k ? ", " : "", names[k], d[d.size() / 2]);
    }
    std::vector<double> tot;
    for (uint32_t b = 0; b < nb && b < 128; ++b) tot.push_back((double)(st[b * 8 * kS + 13] - st[b * 8 * kS]) * 1e3 / rate_khz);
    std::sort(tot.begin(), tot.end());
    printf(", \"total_us\": %.2f", tot[tot.size() / 2]);
    {  // wave 0 inside the scalars: entry -> inversion start (15) -> inversion end (14) -> scalars done (1)
      std::vector<double> a, b, c;
      for (uint32_t k = 0; k < nb && k < 128; ++k) {
        const uint64_t* s = &st[k * 8 * kS];
        a.push_back((double)(s[15] - s[0]) * 1e3 / rate_khz);
        b.push_back((double)(s[14] - s[15]) * 1e3 / rate_khz);
        c.push_back((double)(s[1] - s[14]) * 1e3 / rate_khz);
      }
      std::sort(a.begin(), a.end());
      std::sort(b.begin(), b.end());
      std::sort(c.begin(), c.end());
      printf(", \"scalars_split_us\": [%.2f, %.2f, %.2f]", a[a.size() / 2], b[b.size() / 2], c[c.size() / 2]);
    }
    // workgroup 0, every wave: handoff end (2) -> entries (3) -> level 0 (4) -> pair add (5), from wave 0's stamp 2
    printf(", \"wg0_waves_us_since_handoff\": [");
    for (int w = 0; w < 8; ++w) {
      const uint64_t* s = &st[w * kS];
      const uint64_t t2 = st[2];
      printf("%s[%.2f, %.2f, %.2f, %.2f]", w ? ", " : "", (double)(s[2] - t2) * 1e3 / rate_khz,
             (double)(s[3] - t2) * 1e3 / rate_khz, (double)(s[4] - t2) * 1e3 / rate_khz, (double)(s[5] - t2) * 1e3 / rate_khz);
    }
    printf("]}");

  }
  printf("}\n");
  return 0;
}
