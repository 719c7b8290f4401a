// Latency of ONE P-256 Montgomery product (a b 2^-261 mod p) on a lone wave,
// in two layouts -- the question behind the latency path's comb stage
// (DESIGN.md §7.3): is a value spread one 29-bit limb per lane over a 16-lane
// row ("limb per lane") faster per product than a value held whole by one
// lane (fs_mul, the quad schedule's product)?
//   lane:  each lane a whole 9-limb value, x = fs_mul(x, y) chained;
//   row:   lane j of a row holds limb j; 9 CIOS rounds, each a DPP broadcast of
//          a_i and of the column-0 digit, two 64-bit MADs and a split carry
//          (t_j <- t_j >> 29 + (t_{j+1} mod 2^29)); mp = 1 for P-256;
//   row2:  two independent row chains interleaved.
// Measurement tool (not part of the product):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I simple_pbft_amd/csrc tools/lpl_probe.hip -o tools/lpl_probe
//   tools/lpl_probe [iters]  ->  one JSON line; values checked by tools/lpl_check.py
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "fes.h"

using namespace pbftv;

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

template <int K>
__device__ __forceinline__ uint32_t row_bcast(uint32_t x) {  // lane K of the row to every lane of it
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x150 + K, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t row_next(uint32_t x) {  // lane j <- lane j + 1 (0 past the row)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x101, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t row_prev(uint32_t x) {  // lane j <- lane j - 1 (0 before the row)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
}

template <int I>
__device__ __forceinline__ void cios_round(uint64_t& t, uint32_t a, uint32_t b, uint32_t pl) {
  const uint32_t ai = row_bcast<I>(a);
  t += (uint64_t)ai * b;
  const uint32_t q = row_bcast<0>((uint32_t)t) & kMask29;  // -p^-1 = 1 mod 2^29
  t += (uint64_t)q * pl;
  const uint32_t lo = (uint32_t)t & kMask29;  // lane 0: 0
  t = (t >> 29) + (uint64_t)row_next(lo);
}

// a b 2^-261 mod p, value < a b / 2^261 + p; limbs 0..7 < 2^29 + 2^5 after the
// carry pass; lane 8 the top limb; lanes 9..15 zero.  pl = p's limb of the lane.
__device__ __forceinline__ uint32_t row_mul(uint32_t a, uint32_t b, uint32_t pl, uint32_t lomask, uint32_t himask) {
  uint64_t t = 0;
  cios_round<0>(t, a, b, pl);
  cios_round<1>(t, a, b, pl);
  cios_round<2>(t, a, b, pl);
  cios_round<3>(t, a, b, pl);
  cios_round<4>(t, a, b, pl);
  cios_round<5>(t, a, b, pl);
  cios_round<6>(t, a, b, pl);
  cios_round<7>(t, a, b, pl);
  cios_round<8>(t, a, b, pl);
  const uint32_t lo = (uint32_t)t & lomask;                  // lane 8 keeps its whole limb
  const uint32_t hi = (uint32_t)(t >> 29) & himask;          // lane 8 carries nothing up
  return lo + row_prev(hi);
}


// ---- signed limbs (as fes.h): v_mad_i64_i32, a difference is one v_sub per value
template <int I>
__device__ __forceinline__ void scios_round(int64_t& t, uint32_t a, uint32_t b, uint32_t pl) {
  const uint32_t ai = row_bcast<I>(a);
  t += (int64_t)(int32_t)ai * (int64_t)(int32_t)b;
  const uint32_t q = row_bcast<0>((uint32_t)t) & kMask29;
  t += (int64_t)(int32_t)q * (int64_t)(int32_t)pl;
  const uint32_t lo = (uint32_t)t & kMask29;
  t = (t >> 29) + (int64_t)row_next(lo);
}
__device__ __forceinline__ uint32_t srow_mul(uint32_t a, uint32_t b, uint32_t pl, uint32_t lomask, uint32_t himask) {
  int64_t t = 0;
  scios_round<0>(t, a, b, pl);
  scios_round<1>(t, a, b, pl);
  scios_round<2>(t, a, b, pl);
  scios_round<3>(t, a, b, pl);
  scios_round<4>(t, a, b, pl);
  scios_round<5>(t, a, b, pl);
  scios_round<6>(t, a, b, pl);
  scios_round<7>(t, a, b, pl);
  scios_round<8>(t, a, b, pl);
  const uint32_t lo = (uint32_t)t & lomask;
  const uint32_t hi = (uint32_t)(t >> 29) & himask;
  return lo + row_prev(hi);
}
// every row gets the values of all four rows: g[r] = row r's x
__device__ __forceinline__ void gather4(uint32_t g[4], uint32_t x) {
  const auto ab = __builtin_amdgcn_permlane16_swap(x, x, false, false);  // [x0 x0 x2 x2], [x1 x1 x3 x3]
  const auto c = __builtin_amdgcn_permlane32_swap(ab[0], ab[0], false, false);
  const auto d = __builtin_amdgcn_permlane32_swap(ab[1], ab[1], false, false);
  g[0] = c[0];
  g[1] = d[0];
  g[2] = c[1];
  g[3] = d[1];
}
struct RowCtx {
  uint32_t pl, lomask, himask;
  bool r0, r1, r2;  // row == 0, 1, 2
};
__device__ __forceinline__ uint32_t sel4(const RowCtx& c, uint32_t a, uint32_t b, uint32_t d, uint32_t e) {
  return c.r0 ? a : (c.r1 ? b : (c.r2 ? d : e));
}
// (X1,Y1,ZZ1,ZZZ1) += (X2,Y2,ZZ2,ZZZ2), add-2008-s, every value one VGPR, the
// same in every row; each step one product per row, then a gather.
__device__ __forceinline__ void xyzz_add_rows(const RowCtx& c, uint32_t P1[4], const uint32_t P2[4]) {
  uint32_t g[4];
  uint32_t m = srow_mul(sel4(c, P1[0], P2[0], P1[1], P2[1]), sel4(c, P2[2], P1[2], P2[3], P1[3]), c.pl, c.lomask, c.himask);
  gather4(g, m);
  const uint32_t U1 = g[0], S1 = g[2], P = g[1] - g[0], R = g[3] - g[2];
  m = srow_mul(sel4(c, P, R, P1[2], P1[3]), sel4(c, P, R, P2[2], P2[3]), c.pl, c.lomask, c.himask);
  gather4(g, m);
  const uint32_t PP = g[0], RR = g[1], Z12 = g[2], ZZZ12 = g[3];
  m = srow_mul(sel4(c, P, U1, Z12, 0u), PP, c.pl, c.lomask, c.himask);
  gather4(g, m);
  const uint32_t PPP = g[0], Q = g[1], ZZ3 = g[2];
  const uint32_t X3 = RR - PPP - (Q << 1);
  m = srow_mul(sel4(c, R, S1, ZZZ12, 0u), sel4(c, Q - X3, PPP, PPP, 0u), c.pl, c.lomask, c.himask);
  gather4(g, m);
  P1[0] = X3;
  P1[1] = g[0] - g[1];
  P1[2] = ZZ3;
  P1[3] = g[2];
}

__global__ void __launch_bounds__(64) k_probe(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                              unsigned long long* __restrict__ clk, int iters, int mode) {
  const int lane = (int)threadIdx.x, L = lane & 15;
  uint32_t pl = 0;
  for (int k = 0; k < 9; ++k) pl = L == k ? kP[k] : pl;
  const uint32_t lomask = L == 8 ? 0xFFFFFFFFu : kMask29, himask = L == 8 ? 0u : 0xFFFFFFFFu;
  unsigned long long c0 = 0, c1 = 0, w0 = 0, w1 = 0;
  if (mode == 0) {  // per-lane fs_mul chain
    fe x, y;
    for (int l = 0; l < 9; ++l) {
      x.v[l] = in[l];
      y.v[l] = in[9 + l];
    }
    __syncthreads();
    c0 = clock64();
    w0 = wall_clock64();
    for (int i = 0; i < iters; ++i) fs_mul(x, x, y);
    c1 = clock64();
    w1 = wall_clock64();
    for (int l = 0; l < 9; ++l) out[lane * 9 + l] = x.v[l];
  } else if (mode == 3) {  // chained XYZZ additions P += Q in the row layout
    RowCtx c;
    c.pl = pl;
    c.lomask = lomask;
    c.himask = himask;
    const int row = lane >> 4;
    c.r0 = row == 0;
    c.r1 = row == 1;
    c.r2 = row == 2;
    uint32_t P1[4], P2[4];
    for (int k = 0; k < 4; ++k) {
      P1[k] = L < 9 ? in[18 + 9 * k + L] : 0u;
      P2[k] = L < 9 ? in[54 + 9 * k + L] : 0u;
    }
    __syncthreads();
    c0 = clock64();
    w0 = wall_clock64();
    for (int i = 0; i < iters; ++i) xyzz_add_rows(c, P1, P2);
    c1 = clock64();
    w1 = wall_clock64();
    for (int k = 0; k < 4; ++k) out[64 * k + lane] = P1[k];
  } else {
    uint32_t x = L < 9 ? in[L] : 0u, y = L < 9 ? in[9 + L] : 0u, x2 = x;
    __syncthreads();
    c0 = clock64();
    w0 = wall_clock64();
    if (mode == 1) {
      for (int i = 0; i < iters; ++i) x = row_mul(x, y, pl, lomask, himask);
    } else {
      for (int i = 0; i < iters; i += 2) {
        x = row_mul(x, y, pl, lomask, himask);
        x2 = row_mul(x2, y, pl, lomask, himask);
      }
    }
    c1 = clock64();
    w1 = wall_clock64();
    out[lane] = x;
    out[64 + lane] = x2;
  }
  if (lane == 0) {
    clk[0] = c1 - c0;
    clk[1] = w1 - w0;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  // x0, y: two arbitrary values < p in 29-bit limbs (checked on the host side)
  uint32_t h_in[90];
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (int l = 0; l < 90; ++l) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    h_in[l] = (uint32_t)(s >> 35) & kMask29;
  }
  h_in[8] &= 0x7FFFFF;  // < 2^255
  h_in[17] &= 0x7FFFFF;
  for (int k = 0; k < 8; ++k) h_in[18 + 9 * k + 8] &= 0x7FFFFF;
  uint32_t *d_in, *d_out;
  unsigned long long* d_clk;
  CHECK(hipMalloc(&d_in, sizeof(h_in)));
  CHECK(hipMalloc(&d_out, 64 * 9 * 4 * 4));
  CHECK(hipMalloc(&d_clk, 16));
  CHECK(hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice));
  int clk_khz = 0;
  CHECK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, 0));
  printf("{\"iters\": %d, \"x0\": [", iters);
  for (int l = 0; l < 9; ++l) printf("%s%u", l ? ", " : "", h_in[l]);
  printf("], \"y\": [");
  for (int l = 0; l < 9; ++l) printf("%s%u", l ? ", " : "", h_in[9 + l]);
  printf("]");
  printf(", \"pts\": [");
  for (int l = 18; l < 90; ++l) printf("%s%u", l > 18 ? ", " : "", h_in[l]);
  printf("]");
  const char* names[4] = {"lane", "row", "row2", "add"};
  for (int mode = 0; mode < 4; ++mode) {
    unsigned long long clk[2];
    static uint32_t h_out[64 * 9 * 4];
    const int it = mode == 3 ? iters / 16 : iters;
    for (int rep = 0; rep < 2; ++rep) {  // first launch warms the code
      hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, d_in, d_out, d_clk, it, mode);
      CHECK(hipDeviceSynchronize());
    }
    CHECK(hipMemcpy(clk, d_clk, 16, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(h_out, d_out, sizeof(h_out), hipMemcpyDeviceToHost));
    const double ns = (double)clk[1] * 1e6 / clk_khz;
    printf(", \"%s\": {\"iters\": %d, \"cycles_per_op\": %.1f, \"ns_per_op\": %.2f, \"out\": [", names[mode], it,
           (double)clk[0] / it, ns / it);
    if (mode == 3) {
      for (int k = 0; k < 4; ++k)
        for (int r = 0; r < 4; ++r)  // every row's copy of every coordinate
          for (int l = 0; l < 9; ++l) printf("%s%d", k + r + l ? ", " : "", (int)h_out[64 * k + 16 * r + l]);
    } else {
      for (int l = 0; l < 9; ++l) printf("%s%d", l ? ", " : "", (int)h_out[l]);
    }
    printf("]");
    if (mode == 2) {
      printf(", \"out2\": [");
      for (int l = 0; l < 9; ++l) printf("%s%d", l ? ", " : "", (int)h_out[64 + l]);
      printf("]");
    }
    printf("}");
  }
  printf("}\n");
  return 0;
}
