// VALU issue-rate microbenchmark for gfx950 (MI355X).
//
// Measures the sustained lane-op throughput of the integer instructions the
// P-256 / SHA-256 kernels are built from, so that the roofline denominator in
// bench.py is a measured number rather than a datasheet guess (SURVEY.md §8(d):
// "measure the v_mad_u64_u32 rate").  Each kernel runs 8 independent chains of
// one instruction in inline asm (so the compiler cannot fold or reorder them),
// at full occupancy, and reports lane-ops/s.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_microbench.hip -o tools/valu_microbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

enum Op {
  OP_ADD_U32, OP_ADD_CO, OP_ADDC_CO, OP_MAD_U64_U32, OP_MUL_LO_U32, OP_MUL_HI_U32,
  OP_MUL_U32_U24, OP_MUL_HI_U32_U24, OP_MAD_U32_U24, OP_FMA_F64, OP_FMA_F32,
  OP_LSHL_ADD_U64, OP_BITOP3, OP_ADD3_U32, OP_ALIGNBIT, OP_CNDMASK, OP_SUB_CO_CHAIN, OP_N
};
static const char* kNames[OP_N] = {
  "v_add_u32", "v_add_co_u32", "v_add_co+v_addc_co pair(2 ops)", "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32",
  "v_mul_u32_u24", "v_mul_hi_u32_u24", "v_mad_u32_u24", "v_fma_f64", "v_fma_f32",
  "v_lshl_add_u64", "v_bitop3_b32", "v_add3_u32", "v_alignbit_b32", "v_cndmask_b32",
  "v_sub_co+v_subb_co pair(2 ops)"
};

template <int OP>
__device__ __forceinline__ void step(unsigned& x, unsigned long long& X, double& d, float& f, unsigned a, unsigned b) {
  if constexpr (OP == OP_ADD_U32) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(a));
  if constexpr (OP == OP_ADD_CO) { unsigned long long c; asm volatile("v_add_co_u32 %0, %1, %0, %2" : "+v"(x), "=s"(c) : "v"(a)); }
  if constexpr (OP == OP_ADDC_CO) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %2, vcc" : "+v"(x) : "v"(a), "v"(b) : "vcc");
  if constexpr (OP == OP_MAD_U64_U32) { unsigned long long c; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(X), "=s"(c) : "v"(a), "v"(b)); }
  if constexpr (OP == OP_MUL_LO_U32) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(a));
  if constexpr (OP == OP_MUL_HI_U32) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(a));
  if constexpr (OP == OP_MUL_U32_U24) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(a));
  if constexpr (OP == OP_MUL_HI_U32_U24) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x) : "v"(a));
  if constexpr (OP == OP_MAD_U32_U24) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(x) : "v"(a), "v"(b));
  if constexpr (OP == OP_FMA_F64) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(d));
  if constexpr (OP == OP_FMA_F32) asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(f));
  if constexpr (OP == OP_LSHL_ADD_U64) asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(X));
  if constexpr (OP == OP_BITOP3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(a), "v"(b));
  if constexpr (OP == OP_ADD3_U32) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
  if constexpr (OP == OP_ALIGNBIT) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(x));
  if constexpr (OP == OP_CNDMASK) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(a) : "vcc");
  if constexpr (OP == OP_SUB_CO_CHAIN) asm volatile("v_sub_co_u32 %0, vcc, %0, %1\n\tv_subb_co_u32 %0, vcc, %0, %2, vcc" : "+v"(x) : "v"(a), "v"(b) : "vcc");
}

template <int OP>
__global__ void __launch_bounds__(256) kern(unsigned* out, int iters, unsigned seed) {
  unsigned t = threadIdx.x + blockIdx.x * 256u + seed;
  unsigned x[8]; unsigned long long X[8]; double d[8]; float f[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { x[j] = t * (j + 3); X[j] = (unsigned long long)t * (j + 5); d[j] = 1e-3 * (t & 255) * j; f[j] = 1e-3f * (t & 255) * j; }
  unsigned a = t ^ 0x9e3779b9u, b = t * 7u;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int j = 0; j < 8; ++j) step<OP>(x[j], X[j], d[j], f[j], a, b);
    }
  }
  unsigned r = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r ^= x[j] ^ (unsigned)X[j] ^ (unsigned)(X[j] >> 32) ^ (unsigned)(long long)d[j] ^ (unsigned)f[j];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int OP>
static double run(unsigned* dout, int blocks, int iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, dout, 16, 1u);  // warm
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, dout, iters, 2u);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  double instr = (double)blocks * 256.0 * iters * 32.0;   // lane-instructions
  if (OP == OP_ADDC_CO || OP == OP_SUB_CO_CHAIN) instr *= 2.0;
  return instr / (ms * 1e-3);
}

template <int OP>
static void one(unsigned* dout, int blocks, int iters, double peak) {
  double r = run<OP>(dout, blocks, iters);
  printf("%-34s %9.2f T lane-ops/s  (%.3f of %.1f T full-rate)\n", kNames[OP], r / 1e12, r / peak, peak / 1e12);
}

int main(int argc, char** argv) {
  int blocks = argc > 1 ? atoi(argv[1]) : 256 * 8;
  int iters = argc > 2 ? atoi(argv[2]) : 4096;
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  double clk = p.clockRate * 1e3;
  double peak = (double)p.multiProcessorCount * 128.0 * clk;   // 4 SIMD x 32 lanes per clock
  printf("device %s CUs %d clock %.0f MHz blocks %d iters %d\n", p.gcnArchName, p.multiProcessorCount, clk / 1e6, blocks, iters);
  unsigned* dout; CHECK(hipMalloc(&dout, (size_t)blocks * 256 * 4));
  one<OP_ADD_U32>(dout, blocks, iters, peak);
  one<OP_ADD_CO>(dout, blocks, iters, peak);
  one<OP_ADDC_CO>(dout, blocks, iters, peak);
  one<OP_SUB_CO_CHAIN>(dout, blocks, iters, peak);
  one<OP_MAD_U64_U32>(dout, blocks, iters, peak);
  one<OP_MUL_LO_U32>(dout, blocks, iters, peak);
  one<OP_MUL_HI_U32>(dout, blocks, iters, peak);
  one<OP_MUL_U32_U24>(dout, blocks, iters, peak);
  one<OP_MUL_HI_U32_U24>(dout, blocks, iters, peak);
  one<OP_MAD_U32_U24>(dout, blocks, iters, peak);
  one<OP_FMA_F64>(dout, blocks, iters, peak);
  one<OP_FMA_F32>(dout, blocks, iters, peak);
  one<OP_LSHL_ADD_U64>(dout, blocks, iters, peak);
  one<OP_BITOP3>(dout, blocks, iters, peak);
  one<OP_ADD3_U32>(dout, blocks, iters, peak);
  one<OP_ALIGNBIT>(dout, blocks, iters, peak);
  one<OP_CNDMASK>(dout, blocks, iters, peak);
  CHECK(hipFree(dout));
  return 0;
}
