// What a resident, mostly sleeping kernel on another stream costs a busy
// stream (the armed latency kernel's side effect on lane-path batches,
// DESIGN 3.8.1).  Stream A runs a VALU-bound kernel (4096 blocks x 256
// threads of dependent v_mad chains, about the comb's shape) back to back;
// its time per launch is measured alone, then with a persistent kernel on
// stream B: W waves in 4-wave workgroups that poll a flag with s_sleep
// between polls until the host sets it -- the flag in device memory or in
// pinned host memory (as the armed kernel's mailbox).
//   hipcc -O3 --offload-arch=gfx950 -o tools/persist_cost tools/persist_cost.hip
//   tools/persist_cost [ITERS]   -> one JSON line (ITERS: the work kernel's loop, default 2000)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

__global__ void __launch_bounds__(256) k_work(uint32_t* out, int iters) {
  uint64_t a = threadIdx.x + 1, b = blockIdx.x * 7 + 3;
  for (int i = 0; i < iters; ++i) {
    a = (uint64_t)(uint32_t)a * (uint32_t)b + (a >> 32);
    b = (uint64_t)(uint32_t)b * (uint32_t)a + (b >> 32);
  }
  if ((a ^ b) == 0x12345) out[blockIdx.x] = 1;  // never: keeps the chain alive
}

__global__ void __launch_bounds__(256) k_persist(const uint32_t* flag, uint64_t budget) {
  const uint64_t t0 = wall_clock64();
  for (;;) {
    const uint32_t v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v != 0 || wall_clock64() - t0 > budget) break;
    __builtin_amdgcn_s_sleep(2);
  }
}

static int g_iters = 2000;
static double time_work(hipStream_t s, uint32_t* out, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k_work, dim3(4096), dim3(256), 0, s, out, g_iters);
  (void)hipEventRecord(a, s);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_work, dim3(4096), dim3(256), 0, s, out, g_iters);
  (void)hipEventRecord(b, s);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms / reps;
}

int main(int argc, char** argv) {
  if (argc > 1) g_iters = atoi(argv[1]);
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  uint32_t *out, *dflag, *hflag;
  CK(hipMalloc(&out, 4096 * 4));
  CK(hipMalloc(&dflag, 64));
  CK(hipHostMalloc(&hflag, 64, hipHostMallocCoherent | hipHostMallocMapped));
  int khz = 100000;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  const uint64_t budget = (uint64_t)khz * 5000;  // 5 s safety exit
  printf("{");
  const char* sep = "";
  for (int rep = 0; rep < 3; ++rep) {
    for (int mode = 0; mode < 4; ++mode) {  // 0 alone, 1 device flag 8 waves, 2 host flag 8 waves, 3 host flag 128 waves
      const uint32_t* flag = mode == 1 ? dflag : hflag;
      const int waves = mode == 3 ? 128 : 8;
      if (mode) {
        CK(hipMemset(dflag, 0, 64));
        *(volatile uint32_t*)hflag = 0;
        hipLaunchKernelGGL(k_persist, dim3(waves / 4), dim3(256), 0, sb, flag, budget);
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
      }
      const double ms = time_work(sa, out, 100);
      if (mode) {
        *(volatile uint32_t*)hflag = 1;
        CK(hipMemsetAsync(dflag, 1, 4, sa));
        CK(hipStreamSynchronize(sa));
        CK(hipStreamSynchronize(sb));
      }
      static const char* names[] = {"alone", "device_flag_8w", "host_flag_8w", "host_flag_128w"};
      printf("%s\"%s_%d\": %.5f", sep, names[mode], rep, ms);
      sep = ", ";
    }
  }
  printf("}\n");
  return 0;
}
