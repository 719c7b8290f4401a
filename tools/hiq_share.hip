// How many resident (persistent) kernels can sit on high-priority streams
// before a new high-priority stream shares a hardware queue with one of them?
// The armed latency kernels live on high-priority streams (pbftv_api.cpp
// qc_streams_ready), two per context; a process with several contexts on one
// GPU may hold more such streams than the runtime has high-priority hardware
// queues, and a kernel launched on a stream sharing a queue with a resident
// kernel waits for that kernel's budget.  For M = 1..10 this makes M streams
// of one kind, keeps a persistent kernel (polls a host flag, 300-ms budget) on
// the first M-1, and times one short kernel on the last: ~300 ms = shared.
//   hipcc -O3 --offload-arch=gfx950 -o tools/hiq_share tools/hiq_share.hip
//   tools/hiq_share            -> one JSON line per stream kind
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void k_persist(const uint32_t* flag, uint64_t budget) {
  const uint64_t t0 = wall_clock64();
  for (;;) {
    if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0 || wall_clock64() - t0 > budget) break;
    __builtin_amdgcn_s_sleep(2);
  }
}

__global__ void k_short(uint32_t* p) {
  if (threadIdx.x == 0) p[blockIdx.x] += 1;
}

int main() {
  int khz = 100000, ncu = 0, lo = 0, hi = 0;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  uint32_t *flag, *buf;
  CK(hipHostMalloc(&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipMalloc(&buf, 4096));
  const char* kinds[] = {"priority_high", "plain", "cu_mask_full"};
  for (int kind = 0; kind < 3; ++kind) {
    printf("{\"kind\": \"%s\", \"short_kernel_ms_by_streams\": [", kinds[kind]);
    for (int m = 1; m <= 10; ++m) {
      std::vector<hipStream_t> s(m);
      for (auto& q : s) {
        if (kind == 0) {
          CK(hipStreamCreateWithPriority(&q, hipStreamNonBlocking, hi));
        } else if (kind == 1) {
          CK(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
        } else {
          std::vector<uint32_t> mk((ncu + 31) / 32, 0xFFFFFFFFu);
          CK(hipExtStreamCreateWithCUMask(&q, (uint32_t)mk.size(), mk.data()));
        }
      }
      *(volatile uint32_t*)flag = 0;
      for (int i = 0; i + 1 < m; ++i) hipLaunchKernelGGL(k_persist, dim3(1), dim3(64), 0, s[i], flag, (uint64_t)khz * 300);
      CK(hipGetLastError());
      const auto t = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(k_short, dim3(1), dim3(64), 0, s[m - 1], buf);
      CK(hipStreamSynchronize(s[m - 1]));
      printf("%s%.2f", m > 1 ? ", " : "", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count());
      fflush(stdout);
      *(volatile uint32_t*)flag = 1;
      for (auto& q : s) CK(hipStreamSynchronize(q));
      for (auto& q : s) CK(hipStreamDestroy(q));
    }
    printf("]}\n");
  }
  return 0;
}
