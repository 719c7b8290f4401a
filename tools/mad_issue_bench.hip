// v_mad_u64_u32 issue-cost microbenchmark for gfx950: does the (unused) SGPR
// carry-out of VOP3b v_mad_u64_u32 serialise back-to-back issue?  Blocks of
// 16 independent multiply-adds with one shared carry-out pair vs 8 rotated
// pairs, plus a dependent chain and plain 32-bit adds, at 1..8 waves/SIMD
// (occupancy limited by dynamic LDS).  Measurement tool for DESIGN.md §3.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mad_issue_bench.hip -o tools/mad_issue_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

#define M1(i, S) "v_mad_u64_u32 %[x" #i "], " S ", %[a], %[b], %[x" #i "]\n\t"
#define SAME "s[40:41]"
#define BODY_SAME M1(0, SAME) M1(1, SAME) M1(2, SAME) M1(3, SAME) M1(4, SAME) M1(5, SAME) M1(6, SAME) M1(7, SAME) \
                  M1(8, SAME) M1(9, SAME) M1(10, SAME) M1(11, SAME) M1(12, SAME) M1(13, SAME) M1(14, SAME) M1(15, SAME)
#define BODY_ROT M1(0, "s[40:41]") M1(1, "s[42:43]") M1(2, "s[44:45]") M1(3, "s[46:47]") M1(4, "s[48:49]") \
                 M1(5, "s[50:51]") M1(6, "s[52:53]") M1(7, "s[54:55]") M1(8, "s[40:41]") M1(9, "s[42:43]") \
                 M1(10, "s[44:45]") M1(11, "s[46:47]") M1(12, "s[48:49]") M1(13, "s[50:51]") M1(14, "s[52:53]") \
                 M1(15, "s[54:55]")
#define C1 "v_mad_u64_u32 %[x0], s[40:41], %[a], %[b], %[x0]\n\t"
#define BODY_CHAIN C1 C1 C1 C1 C1 C1 C1 C1 C1 C1 C1 C1 C1 C1 C1 C1
#define L1(i) "v_lshl_add_u64 %[x" #i "], %[x" #i "], 0, %[x15]\n\t"
#define BODY_LSHL L1(0) L1(1) L1(2) L1(3) L1(4) L1(5) L1(6) L1(7) L1(8) L1(9) L1(10) L1(11) L1(12) L1(13) L1(14) L1(0)
#define A1(i) "v_add_u32 %[y" #i "], %[y" #i "], %[a]\n\t"
#define BODY_ADD A1(0) A1(1) A1(2) A1(3) A1(4) A1(5) A1(6) A1(7) A1(0) A1(1) A1(2) A1(3) A1(4) A1(5) A1(6) A1(7)
#define P1(i) "v_add_co_u32 %[y" #i "], vcc, %[y" #i "], %[a]\n\tv_addc_co_u32 %[z" #i "], vcc, %[z" #i "], 0, vcc\n\t"
#define BODY_ADDC P1(0) P1(1) P1(2) P1(3) P1(4) P1(5) P1(6) P1(7)
#define X1(i) "v_mad_u64_u32 %[x" #i "], s[40:41], %[a], %[b], %[x" #i "]\n\tv_add_u32 %[y" #i "], %[y" #i "], %[a]\n\t"
#define BODY_MIX X1(0) X1(1) X1(2) X1(3) X1(4) X1(5) X1(6) X1(7)

#define I1(i) "v_mad_i64_i32 %[x" #i "], s[40:41], %[a], %[b], %[x" #i "]\n\t"
#define BODY_SIGNED I1(0) I1(1) I1(2) I1(3) I1(4) I1(5) I1(6) I1(7) I1(8) I1(9) I1(10) I1(11) I1(12) I1(13) I1(14) I1(15)
#define N1(i) "v_not_b32 %[y" #i "], %[y" #i "]\n\t"
#define BODY_NOT N1(0) N1(1) N1(2) N1(3) N1(4) N1(5) N1(6) N1(7) N1(0) N1(1) N1(2) N1(3) N1(4) N1(5) N1(6) N1(7)

#define AB1(i) "v_alignbit_b32 %[y" #i "], %[y" #i "], %[a], 7\n\t"
#define BODY_ALIGNBIT AB1(0) AB1(1) AB1(2) AB1(3) AB1(4) AB1(5) AB1(6) AB1(7) AB1(0) AB1(1) AB1(2) AB1(3) AB1(4) AB1(5) AB1(6) AB1(7)
#define B31(i) "v_bitop3_b32 %[y" #i "], %[y" #i "], %[a], %[b] bitop3:0x96\n\t"
#define BODY_BITOP3 B31(0) B31(1) B31(2) B31(3) B31(4) B31(5) B31(6) B31(7) B31(0) B31(1) B31(2) B31(3) B31(4) B31(5) B31(6) B31(7)
#define AD3(i) "v_add3_u32 %[y" #i "], %[y" #i "], %[a], %[b]\n\t"
#define BODY_ADD3 AD3(0) AD3(1) AD3(2) AD3(3) AD3(4) AD3(5) AD3(6) AD3(7) AD3(0) AD3(1) AD3(2) AD3(3) AD3(4) AD3(5) AD3(6) AD3(7)
#define AND1(i) "v_and_b32 %[y" #i "], %[y" #i "], %[a]\n\t"
#define BODY_AND AND1(0) AND1(1) AND1(2) AND1(3) AND1(4) AND1(5) AND1(6) AND1(7) AND1(0) AND1(1) AND1(2) AND1(3) AND1(4) AND1(5) AND1(6) AND1(7)
#define ASH(i) "v_ashrrev_i64 %[x" #i "], 29, %[x" #i "]\n\t"
#define BODY_ASHR64 ASH(0) ASH(1) ASH(2) ASH(3) ASH(4) ASH(5) ASH(6) ASH(7) ASH(8) ASH(9) ASH(10) ASH(11) ASH(12) ASH(13) ASH(14) ASH(15)

#define OPS_X [x0] "+v"(x[0]), [x1] "+v"(x[1]), [x2] "+v"(x[2]), [x3] "+v"(x[3]), [x4] "+v"(x[4]), [x5] "+v"(x[5]), \
  [x6] "+v"(x[6]), [x7] "+v"(x[7]), [x8] "+v"(x[8]), [x9] "+v"(x[9]), [x10] "+v"(x[10]), [x11] "+v"(x[11]), \
  [x12] "+v"(x[12]), [x13] "+v"(x[13]), [x14] "+v"(x[14]), [x15] "+v"(x[15])
#define OPS_Y [y0] "+v"(y[0]), [y1] "+v"(y[1]), [y2] "+v"(y[2]), [y3] "+v"(y[3]), [y4] "+v"(y[4]), [y5] "+v"(y[5]), \
  [y6] "+v"(y[6]), [y7] "+v"(y[7]), [z0] "+v"(z[0]), [z1] "+v"(z[1]), [z2] "+v"(z[2]), [z3] "+v"(z[3]), \
  [z4] "+v"(z[4]), [z5] "+v"(z[5]), [z6] "+v"(z[6]), [z7] "+v"(z[7])
#define CLOB "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "vcc"

enum { SAMEC, ROTC, CHAIN, LSHL, ADD, ADDC, MIX, SIGNED, NOT, ALIGNBIT, BITOP3, ADD3, AND, ASHR64, NV };
static const char* kName[NV] = {"mad_u64 16 indep, one sdst", "mad_u64 16 indep, 8 sdst rot", "mad_u64 dep chain",
                                "lshl_add_u64 indep", "add_u32 indep", "add_co+addc pairs", "mad_u64 + add_u32 alt", "mad_i64_i32 16 indep", "not_b32 indep", "alignbit_b32 (VOP3)", "bitop3_b32 (VOP3)",
                                "add3_u32 (VOP3)", "and_b32 (VOP2)", "ashrrev_i64"};

template <int V>
__global__ void __launch_bounds__(256) kb(uint32_t* out, int iters, uint32_t seed) {
  extern __shared__ uint32_t pad[];
  const uint32_t t = blockIdx.x * 256 + threadIdx.x + seed;
  uint64_t x[16];
  uint32_t y[8], z[8];
  for (int j = 0; j < 16; ++j) x[j] = (uint64_t)t * (j + 3);
  for (int j = 0; j < 8; ++j) { y[j] = t * (j + 5); z[j] = t ^ j; }
  const uint32_t a = t ^ 0x9e3779b9u, b = t * 7u;
  for (int i = 0; i < iters; ++i) {
    if constexpr (V == SAMEC) asm volatile(BODY_SAME : OPS_X : [a] "v"(a), [b] "v"(b) : CLOB);
    if constexpr (V == ROTC) asm volatile(BODY_ROT : OPS_X : [a] "v"(a), [b] "v"(b) : CLOB);
    if constexpr (V == CHAIN) asm volatile(BODY_CHAIN : OPS_X : [a] "v"(a), [b] "v"(b) : CLOB);
    if constexpr (V == LSHL) asm volatile(BODY_LSHL : OPS_X : [a] "v"(a), [b] "v"(b) : CLOB);
    if constexpr (V == ADD) asm volatile(BODY_ADD : OPS_Y : [a] "v"(a), [b] "v"(b) : CLOB);
    if constexpr (V == ADDC) asm volatile(BODY_ADDC : OPS_Y : [a] "v"(a), [b] "v"(b) : CLOB);
    if constexpr (V == MIX) asm volatile(BODY_MIX : OPS_X, OPS_Y : [a] "v"(a), [b] "v"(b) : CLOB);
    if constexpr (V == SIGNED) asm volatile(BODY_SIGNED : OPS_X : [a] "v"(a), [b] "v"(b) : CLOB);
    if constexpr (V == NOT) asm volatile(BODY_NOT : OPS_Y : [a] "v"(a), [b] "v"(b) : CLOB);
    if constexpr (V == ALIGNBIT) asm volatile(BODY_ALIGNBIT : OPS_Y : [a] "v"(a), [b] "v"(b) : CLOB);
    if constexpr (V == BITOP3) asm volatile(BODY_BITOP3 : OPS_Y : [a] "v"(a), [b] "v"(b) : CLOB);
    if constexpr (V == ADD3) asm volatile(BODY_ADD3 : OPS_Y : [a] "v"(a), [b] "v"(b) : CLOB);
    if constexpr (V == AND) asm volatile(BODY_AND : OPS_Y : [a] "v"(a), [b] "v"(b) : CLOB);
    if constexpr (V == ASHR64) asm volatile(BODY_ASHR64 : OPS_X : [a] "v"(a), [b] "v"(b) : CLOB);
  }
  uint32_t r = 0;
  for (int j = 0; j < 16; ++j) r ^= (uint32_t)x[j] ^ (uint32_t)(x[j] >> 32);
  for (int j = 0; j < 8; ++j) r ^= y[j] ^ z[j];
  if (threadIdx.x == 0) pad[0] = r;
  __syncthreads();
  out[blockIdx.x * 256 + threadIdx.x] = r ^ pad[0];
}

template <int V>
static void run(uint32_t* out, int wps) {
  const int blocks = 256 * 8 * 2, iters = 2048;
  const size_t lds = 160 * 1024 / wps - 512;
  CHECK(hipFuncSetAttribute((const void*)kb<V>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kb<V>, dim3(blocks), dim3(256), lds, 0, out, 8, 1u);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(kb<V>, dim3(blocks), dim3(256), lds, 0, out, iters, 2u);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double waves = blocks * 4.0, instr = waves * iters * 16.0;
  printf("%-30s waves/SIMD=%d  %6.2f SIMD-cycles per wave-instruction\n", kName[V], wps,
         ms * 1e-3 * 2.4e9 * 1024.0 / instr);
}

int main() {
  uint32_t* out;
  CHECK(hipMalloc(&out, 256 * 8 * 2 * 256 * 4));
  for (int w : {1, 2, 4, 8}) {
    run<SAMEC>(out, w);
    run<ROTC>(out, w);
    run<CHAIN>(out, w);
    run<LSHL>(out, w);
    run<ADD>(out, w);
    run<ADDC>(out, w);
    run<MIX>(out, w);
    run<SIGNED>(out, w);
    run<NOT>(out, w);
    run<ALIGNBIT>(out, w);
    run<BITOP3>(out, w);
    run<ADD3>(out, w);
    run<AND>(out, w);
    run<ASHR64>(out, w);
  }
  return 0;
}
