// launch_rt.hip -- what does the latency path pay outside its kernel?  Round
// trips with an EMPTY verify (one wave writes one byte to pinned coherent host
// memory, as k_ecdsa_wave reports its verdict):
//   launch:  host stores the sentinel, hipLaunchKernelGGL, polls the byte;
//   armed:   a one-wave kernel launched in advance spins on a host-memory
//            doorbell (bounded: it gives up after ~50 ms), the host rings it
//            and polls the reply -- the launch is off the critical path.
// p50 / p99 over N round trips each.  Measurement tool (not the product).
//   hipcc -O3 --offload-arch=gfx950 -o tools/launch_rt tools/launch_rt.hip && ./tools/launch_rt 5000
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                              \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                                \
    }                                                                                         \
  } while (0)

__global__ void __launch_bounds__(64) k_reply(uint8_t* out) {
  if (threadIdx.x == 0) out[0] = 1;
}

// spins on bell[0] (host memory) until it equals want or ~budget cycles pass;
// replies with out[0] = 1 (served) or 2 (gave up).  Loads bypass the caches.
__global__ void __launch_bounds__(64) k_armed(const uint32_t* bell, uint32_t want, uint8_t* out, uint64_t budget,
                                             int sleep) {
  const uint64_t t0 = wall_clock64();
  uint32_t v = 0;
  bool served = false;
  for (;;) {
    v = __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v == want) {
      served = true;
      break;
    }
    if (wall_clock64() - t0 > budget) break;
    if (sleep) __builtin_amdgcn_s_sleep(2);
  }
  if (threadIdx.x == 0) out[0] = served ? 1 : 2;
}

static double pct(std::vector<double>& v, double p) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(p * (v.size() - 1))];
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 5000;
  uint8_t* out = nullptr;
  uint32_t* bell = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&out), 64, hipHostMallocCoherent | hipHostMallocMapped));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&bell), 64, hipHostMallocCoherent | hipHostMallocMapped));
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int clk_khz = 100000;
  CHECK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, 0));
  const uint64_t budget = (uint64_t)clk_khz * 50;  // ~50 ms of the constant wall clock
  volatile uint8_t* vo = out;
  volatile uint32_t* vb = bell;
  using clk = std::chrono::steady_clock;
  std::vector<double> tl, ta[2];
  for (int i = 0; i < N + 100; ++i) {  // plain launch
    *vo = 0;
    const auto t0 = clk::now();
    hipLaunchKernelGGL(k_reply, dim3(1), dim3(64), 0, st, out);
    while (*vo == 0) {
    }
    const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
    if (i >= 100) tl.push_back(us);
  }
  CHECK(hipStreamSynchronize(st));
  for (int sl = 0; sl < 2; ++sl) {
    uint32_t seq = 1;
    *vb = 0;
    for (int i = 0; i < N + 100; ++i, ++seq) {
      *vo = 0;
      hipLaunchKernelGGL(k_armed, dim3(1), dim3(64), 0, st, bell, seq, out, budget, sl);
      // let it start spinning (a caller's next certificate arrives later)
      const auto tw = clk::now();
      while (std::chrono::duration<double, std::micro>(clk::now() - tw).count() < 30.0) {
      }
      const auto t0 = clk::now();
      __atomic_store_n(bell, seq, __ATOMIC_RELEASE);
      while (*vo == 0) {
      }
      const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
      if (*vo != 1) {
        fprintf(stderr, "armed kernel gave up\n");
        return 1;
      }
      if (i >= 100) ta[sl].push_back(us);
    }
    CHECK(hipStreamSynchronize(st));
  }
  printf("{\"launch_us\": {\"p50\": %.2f, \"p99\": %.2f}, \"armed_us\": {\"p50\": %.2f, \"p99\": %.2f}, "
         "\"armed_sleep_us\": {\"p50\": %.2f, \"p99\": %.2f}, \"n\": %d}\n",
         pct(tl, 0.5), pct(tl, 0.99), pct(ta[0], 0.5), pct(ta[0], 0.99), pct(ta[1], 0.5), pct(ta[1], 0.99), N);
  CHECK(hipStreamDestroy(st));
  CHECK(hipHostFree(out));
  CHECK(hipHostFree(bell));
  return 0;
}
