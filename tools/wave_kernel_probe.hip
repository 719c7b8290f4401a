// wave_kernel_probe.hip -- stage timestamps of the one-wave-per-signature
// latency kernel (k_ecdsa_wave's body, verify_kernels.h, replicated with
// wall_clock64() stamps): input loads, scalars (lane-parallel safegcd + one
// product step), quad comb with the fused check; plus the inversion alone.  Tables: the
// n = 4 geometry (29-bit G, one 24-bit key table with Q = G), built with the
// product's table kernels.  Measurement tool for DESIGN.md (not the product).
//   make -C simple_pbft_amd && hipcc --offload-arch=gfx950 -O3 -std=c++17 -c tools/wave_kernel_probe.hip -o p.o \
//   && hipcc --offload-arch=gfx950 p.o simple_pbft_amd/build/p256_*.o -o tools/wave_kernel_probe
#include "../simple_pbft_amd/csrc/verify_kernels.h"

#include <cstdio>
#include <vector>

using namespace pbftv;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int WG = 29, WQ = 24;

__global__ void __launch_bounds__(64) probe(const uint8_t* hashes, const uint8_t* sigs, const uint32_t* key_idx,
                                            const uint32_t* key_valid, const uint4* gtab, const uint4* qtabs,
                                            uint64_t* stamps, uint32_t* sink) {
  const uint64_t i = blockIdx.x;
  uint64_t t[6];
  t[0] = wall_clock64();
  uint32_t r[8], s[8], e[8];
  load_be256(hashes + 32 * i, e);
  const bool okin = sig_ok(sigs, key_idx, key_valid, 1, i, r, s);
  uint32_t acc = okin;
  for (int k = 0; k < 8; ++k) {
    e[k] = (uint32_t)__builtin_amdgcn_readfirstlane((int)e[k]);
    r[k] = (uint32_t)__builtin_amdgcn_readfirstlane((int)r[k]);
    s[k] = (uint32_t)__builtin_amdgcn_readfirstlane((int)s[k]);
    acc += e[k] ^ r[k] ^ s[k];
  }
  t[1] = wall_clock64();
  uint32_t u1[8], u2[8];
  fe rm, rnm;
  bool rn_ok;
  wave_scalars(e, r, s, u1, u2, rm, rnm, rn_ok);
  acc += u1[0] ^ u2[0] ^ rm.v[0];
  t[2] = wall_clock64();
  const uint4* qtab = qtabs + (uint64_t)key_idx[i] * (CombGeom<WQ>::kWords / 4);
  bool exc;
  const bool okq = wave_verify_quads<WG, WQ>(exc, u1, u2, gtab, qtab, rm, rnm, rn_ok);
  acc += (uint32_t)okq ^ (uint32_t)exc;
  t[3] = wall_clock64();
  acc += __builtin_amdgcn_readfirstlane((int)okq);
  t[4] = wall_clock64();
  fe D;
  inv_mod_n_wave(D, s);
  acc += D.v[3];
  t[5] = wall_clock64();
  if (threadIdx.x == 0) {
    for (int k = 0; k < 5; ++k) stamps[i * 5 + k] = t[k + 1] - t[k];
    sink[i] = acc;
  }
}

int main() {
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
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(probe, dim3(rep == 2 ? n : 1), dim3(64), 0, 0, dh, ds, dk, dvalid,
                       reinterpret_cast<const uint4*>(gt), reinterpret_cast<const uint4*>(qt), dst, dsink);
    CHECK(hipDeviceSynchronize());
  }
  std::vector<uint64_t> st(5 * n);
  CHECK(hipMemcpy(st.data(), dst, 8 * 5 * n, hipMemcpyDeviceToHost));
  const char* names[5] = {"inputs", "scalars", "quad_comb_and_check", "verdict", "inversion_alone"};
  double sum[5] = {0, 0, 0, 0, 0};
  for (uint32_t i = 0; i < n; ++i)
    for (int k = 0; k < 5; ++k) sum[k] += st[5 * i + k];
  printf("{\"geometry\": [%d, %d]", WG, WQ);
  for (int k = 0; k < 5; ++k) printf(", \"%s_us\": %.2f", names[k], sum[k] / n * 1e3 / rate_khz);
  printf("}\n");
  return 0;
}
