// Which streams can a resident (persistent) kernel block?  HIP maps streams
// onto a small pool of hardware queues (GPU_MAX_HW_QUEUES, 4 here), and a
// queue runs its packets in order, so a kernel that never ends blocks every
// stream that shares its queue.  The armed latency kernel is such a kernel
// (pbftv_api.cpp qc_arm).  For each way of creating the persistent kernel's
// stream, this launches it (it polls a host flag, 300 ms budget), then times
// a short kernel on each of N other ordinary streams and a synchronous
// hipMemcpy: anything that waits ~300 ms shared the queue (or synchronised
// with the stream).
//   hipcc -O3 --offload-arch=gfx950 -o tools/queue_share tools/queue_share.hip
//   tools/queue_share            -> one JSON line per creation mode
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

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main(int argc, char** argv) {
  const int nother = argc > 1 ? atoi(argv[1]) : 6;
  int khz = 100000, ncu = 0;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t *flag, *buf, *hbuf;
  CK(hipHostMalloc(&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipMalloc(&buf, 4096));
  CK(hipHostMalloc(&hbuf, 4096, 0));
  const char* modes[] = {"plain_first", "plain_last", "priority_high_first", "priority_high_last", "cu_mask_first",
                         "cu_mask_last"};
  for (int mode = 0; mode < 6; ++mode) {
    const bool last = mode & 1;
    std::vector<hipStream_t> other(nother);
    hipStream_t ps = nullptr;
    auto make_p = [&] {
      if (mode < 2) {
        CK(hipStreamCreateWithFlags(&ps, hipStreamNonBlocking));
      } else if (mode < 4) {
        int lo = 0, hi = 0;
        CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        CK(hipStreamCreateWithPriority(&ps, hipStreamNonBlocking, hi));
      } else {
        std::vector<uint32_t> m((ncu + 31) / 32, 0xFFFFFFFFu);
        CK(hipExtStreamCreateWithCUMask(&ps, (uint32_t)m.size(), m.data()));
      }
    };
    if (!last) make_p();
    for (auto& s : other) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    if (last) make_p();
    *(volatile uint32_t*)flag = 0;
    hipLaunchKernelGGL(k_persist, dim3(2), dim3(256), 0, ps, flag, (uint64_t)khz * 300);
    CK(hipGetLastError());
    printf("{\"mode\": \"%s\", \"other_streams_ms\": [", modes[mode]);
    for (int i = 0; i < nother; ++i) {
      auto t = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(k_short, dim3(1), dim3(64), 0, other[i], buf);
      CK(hipStreamSynchronize(other[i]));
      printf("%s%.2f", i ? ", " : "", ms_since(t));
    }
    auto t = std::chrono::steady_clock::now();
    CK(hipMemcpy(hbuf, buf, 256, hipMemcpyDeviceToHost));
    printf("], \"sync_memcpy_ms\": %.2f", ms_since(t));
    *(volatile uint32_t*)flag = 1;
    t = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(ps));
    printf(", \"persistent_exit_ms\": %.2f}\n", ms_since(t));
    fflush(stdout);
    for (auto& s : other) CK(hipStreamDestroy(s));
    CK(hipStreamDestroy(ps));
  }
  return 0;
}
