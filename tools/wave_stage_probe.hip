// wave_stage_probe.hip -- single-wave latency of the building blocks of the
// small-batch (one wave per signature) path, measured with the constant-rate
// wall clock inside one wave.  Build: hipcc -O3 --offload-arch=gfx950 -o
// tools/wave_stage_probe tools/wave_stage_probe.hip ; run on the GPU box.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../simple_pbft_amd/csrc/p256_algo.h"

using namespace pbftv;

constexpr int kStages = 11;

__global__ void probe(const uint32_t* in, uint64_t* ticks, uint32_t* sink, int reps, uint32_t lane_mask) {
  uint32_t e[8], r[8], s[8];
  for (int i = 0; i < 8; ++i) {
    e[i] = in[i];
    r[i] = in[8 + i];
    s[i] = in[16 + i] & 0x7FFFFFFF;
  }
  uint32_t acc = 0;
  uint64_t t[kStages + 1];
  fe a, b;
  fe_from_words(a, e);
  fe_from_words(b, r);
  jac P, Q;
  P.x = a; P.y = b; P.z = a;
  Q.x = b; Q.y = a; Q.z = b;
  t[0] = wall_clock64();
  for (int k = 0; k < reps; ++k) {  // 0: full scalars (range checks, safegcd, u1, u2)
    uint32_t u1[8], u2[8];
    s[0] ^= k;
    ecdsa_scalars(e, r, s, u1, u2);
    acc += u1[0] ^ u2[3];
  }
  t[1] = wall_clock64();
  for (int k = 0; k < reps; ++k) {  // 1: safegcd inversion alone
    uint32_t w[8];
    s[1] ^= k;
    inv_mod_n_words(w, s);
    acc += w[2];
  }
  t[2] = wall_clock64();
  for (int k = 0; k < reps; ++k) {  // 2: Fermat inversion (the chain it replaces)
    fe x;
    fn_inv_mont(x, a);
    a.v[0] ^= x.v[1] & 1;
  }
  t[3] = wall_clock64();
  for (int k = 0; k < reps * 100; ++k) fe_mul(a, a, b);  // 3: 100 dependent fe_mul
  t[4] = wall_clock64();
  for (int k = 0; k < reps; ++k) {  // 4: jac_add
    jac R;
    jac_add(R, P, Q);
    P = R;
  }
  t[5] = wall_clock64();
  for (int k = 0; k < reps; ++k) jac_madd<true>(P, a, b);  // 5: checked madd
  t[6] = wall_clock64();
  for (int k = 0; k < reps; ++k) {  // 6: jac_double
    jac R;
    jac_double(R, P);
    P = R;
  }
  t[7] = wall_clock64();
  for (int k = 0; k < reps; ++k) {  // 7: safegcd on per-lane (VALU) operands
    uint32_t w[8], sv[8];
    for (int q = 0; q < 8; ++q) sv[q] = s[q] ^ (threadIdx.x & lane_mask);
    sv[1] ^= k;
    inv_mod_n_words(w, sv);
    acc += w[2];
  }
  t[8] = wall_clock64();
  for (int k = 0; k < reps; ++k) {  // 8: safegcd on readfirstlane'd (SALU) operands
    uint32_t w[8], sv[8];
    for (int q = 0; q < 8; ++q) sv[q] = __builtin_amdgcn_readfirstlane(s[q] ^ (threadIdx.x & lane_mask));
    sv[1] ^= k;
    inv_mod_n_words(w, sv);
    acc += w[2];
  }
  t[9] = wall_clock64();
  for (int k = 0; k < reps; ++k) {  // 9: constant-time divsteps, VALU operands
    uint32_t w[8], sv[8];
    for (int q = 0; q < 8; ++q) sv[q] = s[q] ^ (threadIdx.x & lane_mask);
    sv[1] ^= k;
    inv_mod_n_words_ct(w, sv);
    acc += w[2];
  }
  t[10] = wall_clock64();
  for (int k = 0; k < reps; ++k) {  // 10: constant-time divsteps, SALU operands
    uint32_t w[8], sv[8];
    for (int q = 0; q < 8; ++q) sv[q] = __builtin_amdgcn_readfirstlane(s[q] ^ (threadIdx.x & lane_mask));
    sv[1] ^= k;
    inv_mod_n_words_ct(w, sv);
    acc += w[2];
  }
  t[11] = wall_clock64();
  if (threadIdx.x == 0) {
    for (int i = 0; i < kStages; ++i) ticks[i] = t[i + 1] - t[i];
  }
  sink[threadIdx.x] = acc ^ a.v[0] ^ P.x.v[1] ^ P.z.v[2];
}

int main() {
  int rate_khz = 0;
  hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0);
  uint32_t h_in[24];
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < 24; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    h_in[i] = (uint32_t)x;
  }
  uint32_t *d_in, *d_sink;
  uint64_t* d_t;
  hipMalloc(&d_in, sizeof(h_in));
  hipMalloc(&d_t, 8 * kStages);
  hipMalloc(&d_sink, 4 * 64);
  hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice);
  const int reps = 20;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d_in, d_t, d_sink, 2, 0u);  // warm
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d_in, d_t, d_sink, reps, 0u);
  uint64_t t[kStages];
  hipMemcpy(t, d_t, sizeof(t), hipMemcpyDeviceToHost);
  const char* names[kStages] = {"ecdsa_scalars (safegcd)", "inv_mod_n safegcd", "fn_inv_mont Fermat",
                                "fe_mul", "jac_add", "jac_madd<true>", "jac_double", "inv_mod_n VALU operands",
                                "inv_mod_n SALU operands", "inv ct VALU", "inv ct SALU"};
  const double per[kStages] = {1.0 * reps, 1.0 * reps, 1.0 * reps, 100.0 * reps, 1.0 * reps, 1.0 * reps, 1.0 * reps,
                                1.0 * reps, 1.0 * reps, 1.0 * reps, 1.0 * reps};
  printf("{\"wall_clock_khz\": %d", rate_khz);
  for (int i = 0; i < kStages; ++i) printf(", \"%s_us\": %.3f", names[i], t[i] / per[i] * 1e3 / rate_khz);
  printf("}\n");
  return 0;
}
