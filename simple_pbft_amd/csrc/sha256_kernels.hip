// sha256_kernels.hip -- lane-per-message SHA-256 for gfx950.
//
// utils.Hash (utils/utils.go:13-17) = hex(SHA-256(content)); digest()
// (pbft/consensus/pbft_impl.go:235-243) hashes the Go-JSON preimage.  Here one
// lane owns one message: it streams the message's 64-B blocks from HBM with
// dword loads re-aligned by v_alignbyte_b32 (messages sit at arbitrary byte
// offsets), byte-swaps to big-endian and runs the fully unrolled 64-round
// compression with v_alignbit_b32 rotates and v_bitop3_b32 for Ch / Maj /
// three-way XORs.  Messages of mixed length are bucketed by block count
// (k_len_hist / k_len_scan / k_len_scatter, a device counting sort) so the 64
// lanes of a wave run the same number of blocks.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "kernels.h"

namespace pbftv {

#ifndef PBFTV_SHA_WAVES
#define PBFTV_SHA_WAVES 1  // min waves per SIMD for k_sha256
#endif

__device__ __constant__ static const uint32_t kK256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
// three-way XOR as ONE v_bitop3_b32 (truth table 0x96); the compiler leaves
// a ^ b ^ c as two v_xor_b32 (~220 extra instructions per block)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// majority as ONE v_bitop3_b32 (0xE8: set when two or more inputs are set;
// symmetric, so operand order is free); the compiler's xor + v_bfi_b32 form is
// two instructions (64 per block)
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

__device__ __forceinline__ void compress(uint32_t st[8], uint32_t w[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int r = 0; r < 64; ++r) {
    uint32_t wr;
    if (r < 16) {
      wr = w[r];
    } else {
      const uint32_t x = w[(r + 1) & 15], y = w[(r + 14) & 15];
      const uint32_t s0 = xor3(rotr(x, 7), rotr(x, 18), x >> 3);
      const uint32_t s1 = xor3(rotr(y, 17), rotr(y, 19), y >> 10);
      w[r & 15] += s0 + w[(r + 9) & 15] + s1;
      wr = w[r & 15];
    }
    const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = h + S1 + ch + kK256[r] + wr;
    const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
    const uint32_t mj = maj(a, b, c);
    const uint32_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// 16 dwords of one 64-B block from a 4-B aligned address as four 16-B loads
// (global_load_dwordx4 needs only dword alignment): a quarter of the memory
// instructions -- and of the 64-lane cache-line fan-out -- of dword loads.
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ void load_block16(const uint32_t* __restrict__ q, uint32_t d[16]) {
  const u32x4_a4* v = reinterpret_cast<const u32x4_a4*>(q);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const u32x4_a4 x = v[k];
    d[4 * k] = x.x; d[4 * k + 1] = x.y; d[4 * k + 2] = x.z; d[4 * k + 3] = x.w;
  }
}

__global__ void __launch_bounds__(256, PBFTV_SHA_WAVES) k_sha256(const uint8_t* __restrict__ data, const uint64_t* __restrict__ offsets,
                                                const uint32_t* __restrict__ lengths,
                                                const uint32_t* __restrict__ order, uint64_t n,
                                                uint8_t* __restrict__ digests, const uint8_t* __restrict__ expected,
                                                uint32_t* __restrict__ bitmap32) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t m = order ? order[i] : i;
  const uint8_t* base = data + offsets[m];  // pointer arithmetic (not an int round trip) keeps global loads
  const uint32_t len = lengths[m];
  const uint32_t sh = (uint32_t)((uintptr_t)base & 3u);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(base - sh);
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  const uint32_t nfull = len >> 6;
  uint32_t w[16];
  // block b's 17 dwords (the 17th only for a misaligned message) are loaded
  // while block b - 1 is compressed
  uint32_t d[17];
  if (nfull) {
    load_block16(q, d);
    d[16] = sh ? q[16] : 0u;
  }
  for (uint32_t blk = 0; blk < nfull; ++blk) {
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = __builtin_bswap32(__builtin_amdgcn_alignbyte(d[j + 1], d[j], sh));
    if (blk + 1 < nfull) {
      const uint32_t* qb = q + 16ull * (blk + 1);
      load_block16(qb, d);
      d[16] = sh ? qb[16] : 0u;
    }
    compress(st, w);
  }
  // tail: rem bytes (0..63) + 0x80 + zeros + 64-bit bit length, in one or two blocks
  const uint32_t rem = len - (nfull << 6);
  const uint32_t* qt = q + 16ull * nfull;
#pragma unroll
  for (int j = 0; j < 17; ++j) d[j] = (4u * j < rem + sh) ? qt[j] : 0u;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint32_t x = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);  // tail bytes 4j..4j+3, little-endian
    const int v = (int)rem - 4 * j;                                  // message bytes remaining at this word
    const uint32_t keep = v >= 4 ? 0xFFFFFFFFu : (v <= 0 ? 0u : ((1u << (8 * v)) - 1u));
    x &= keep;
    if (v >= 0 && v < 4) x |= 0x80u << (8 * v);
    w[j] = __builtin_bswap32(x);
  }
  const uint64_t bits = (uint64_t)len << 3;
  if (rem + 9 <= 64) {
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
    compress(st, w);
  } else {
    compress(st, w);
#pragma unroll
    for (int j = 0; j < 14; ++j) w[j] = 0;
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
    compress(st, w);
  }
  uint4* out = reinterpret_cast<uint4*>(digests + 32 * m);
  const uint4 o0 = make_uint4(__builtin_bswap32(st[0]), __builtin_bswap32(st[1]), __builtin_bswap32(st[2]),
                              __builtin_bswap32(st[3]));
  const uint4 o1 = make_uint4(__builtin_bswap32(st[4]), __builtin_bswap32(st[5]), __builtin_bswap32(st[6]),
                              __builtin_bswap32(st[7]));
  out[0] = o0;
  out[1] = o1;
  if (expected) {
    const uint4* ex = reinterpret_cast<const uint4*>(expected + 32 * m);
    const uint4 e0 = ex[0], e1 = ex[1];
    const bool eq = e0.x == o0.x && e0.y == o0.y && e0.z == o0.z && e0.w == o0.w && e1.x == o1.x && e1.y == o1.y &&
                    e1.z == o1.z && e1.w == o1.w;
    if (eq) atomicOr(bitmap32 + (m >> 5), 1u << (m & 31));
  }
}

// ---- line-aligned staging (k_sha256_ring) ----------------------------------
// k_sha256 reads each block as 17 dword-aligned dwords starting at the
// message's own alignment, so every 128-B line of a message is fetched by two
// consecutive block loads one compression apart, and ~20 % of the second
// fetches miss the L2 (config 5: 24.5M 128-B requests for 2.18 GB of messages,
// 1.44x, profiles/r04_sha_fetch_calibration.json).  Here each lane fetches its
// message's ALIGNED 128-B lines, each exactly once (8 dwordx4 loads, issued a
// compression ahead), and keeps the last two in LDS; a block's 17 dwords are
// read back at the lane's own dword position.  LDS is ring[pos][thread]
// (pos = dword of the two-line ring, 0..63, plus a 16-dword mirror of line
// slot 0 at 64..79 so a 17-dword window never wraps): the address of every
// access is pos * 1024 + 4 * thread, so a wave's lanes always hit 64 distinct
// banks whatever their positions.  80 KiB per 256-thread block: two blocks per
// CU (2 waves/SIMD -- k_sha256 runs no faster at 4, r04_sha_fetch_calibration).
// A line is 128-B aligned, so it lies in the page of a message byte: reading a
// whole line never faults where the message is mapped.
constexpr uint32_t kRingPos = 80;  // 2 x 32 line dwords + the 16-dword mirror

__device__ __forceinline__ void ring_store(uint32_t* ring, uint32_t t, uint32_t line, const uint32_t L[32]) {
  uint32_t* r = ring + (32u * (line & 1u)) * 256u + t;
#pragma unroll
  for (int k = 0; k < 32; ++k) r[k * 256] = L[k];
  if ((line & 1u) == 0) {
    uint32_t* mr = ring + 64u * 256u + t;
#pragma unroll
    for (int k = 0; k < 16; ++k) mr[k * 256] = L[k];
  }
}

__device__ __forceinline__ void line_load(const uint32_t* __restrict__ p, uint32_t L[32]) {
  const uint4* v = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint4 x = v[k];
    L[4 * k] = x.x; L[4 * k + 1] = x.y; L[4 * k + 2] = x.z; L[4 * k + 3] = x.w;
  }
}

__global__ void __launch_bounds__(256, 2) k_sha256_ring(const uint8_t* __restrict__ data, const uint64_t* __restrict__ offsets,
                                                         const uint32_t* __restrict__ lengths,
                                                         const uint32_t* __restrict__ order, uint64_t n,
                                                         uint8_t* __restrict__ digests, const uint8_t* __restrict__ expected,
                                                         uint32_t* __restrict__ bitmap32) {
  __shared__ uint32_t ring[kRingPos * 256];  // [pos][thread], 80 KiB (static: gfx950 allows up to 160 KiB)
  const uint32_t t = threadIdx.x;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + t;
  if (i >= n) return;  // (no barriers: every lane owns its ring column)
  const uint64_t m = order ? order[i] : i;
  const uint8_t* base = data + offsets[m];
  const uint32_t len = lengths[m];
  const uintptr_t a = reinterpret_cast<uintptr_t>(base);
  const uint32_t* L0 = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)127);
  const uint32_t lob = (uint32_t)(a & 127u), sh = (uint32_t)(a & 3u);
  const uint32_t D0 = lob >> 2;                  // the message's first dword in line 0
  const uint32_t nlines = (uint32_t)(((uint64_t)lob + len + 127u) >> 7);  // lines holding message bytes (>= 1 for len >= 1)
  uint32_t L[32];
  // lines 0 and 1 (blocks 0 and 1 need nothing past line 1).  An empty message
  // on a line boundary has no line (it may sit at the very end of a mapping):
  // nothing is read, and the tail masks every ring byte.
  uint32_t R = 0;  // next line to store
  if (nlines > 0) {
    line_load(L0, L);
    ring_store(ring, t, 0, L);
    R = 1;
  }
  if (nlines > 1) {
    line_load(L0 + 32, L);
    ring_store(ring, t, 1, L);
    R = 2;
  }
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  const uint32_t nfull = len >> 6;
  uint32_t w[16], x[17];
  for (uint32_t blk = 0; blk < nfull; ++blk) {
    const uint32_t D = D0 + 16u * blk;  // this block's first dword (line-0 relative)
    const uint32_t* rp = ring + (D & 63u) * 256u + t;
#pragma unroll
    for (int j = 0; j < 17; ++j) x[j] = rp[j * 256];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = __builtin_bswap32(__builtin_amdgcn_alignbyte(x[j + 1], x[j], sh));
    // the next block's first line f: lines below f are dead; line R goes into
    // the slot of line R - 2 once that is dead, loaded now and stored after
    // this compression (one compression of latency hiding)
    const uint32_t f = (D + 16u) >> 5;
    const bool fetch = R < nlines && R - 2u < f;
    if (fetch) line_load(L0 + 32u * R, L);
    compress(st, w);
    if (fetch) {
      ring_store(ring, t, R, L);
      ++R;
    }
  }
  // tail: rem bytes (0..63) + 0x80 + zeros + 64-bit bit length, in one or two
  // blocks; ring bytes past the message end are masked off
  const uint32_t rem = len - (nfull << 6);
  {
    const uint32_t D = D0 + 16u * nfull;
    const uint32_t* rp = ring + (D & 63u) * 256u + t;
#pragma unroll
    for (int j = 0; j < 17; ++j) x[j] = rp[j * 256];
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint32_t y = __builtin_amdgcn_alignbyte(x[j + 1], x[j], sh);  // tail bytes 4j..4j+3, little-endian
    const int v = (int)rem - 4 * j;                                  // message bytes remaining at this word
    const uint32_t keep = v >= 4 ? 0xFFFFFFFFu : (v <= 0 ? 0u : ((1u << (8 * v)) - 1u));
    y &= keep;
    if (v >= 0 && v < 4) y |= 0x80u << (8 * v);
    w[j] = __builtin_bswap32(y);
  }
  const uint64_t bits = (uint64_t)len << 3;
  if (rem + 9 <= 64) {
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
    compress(st, w);
  } else {
    compress(st, w);
#pragma unroll
    for (int j = 0; j < 14; ++j) w[j] = 0;
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
    compress(st, w);
  }
  uint4* out = reinterpret_cast<uint4*>(digests + 32 * m);
  const uint4 o0 = make_uint4(__builtin_bswap32(st[0]), __builtin_bswap32(st[1]), __builtin_bswap32(st[2]),
                              __builtin_bswap32(st[3]));
  const uint4 o1 = make_uint4(__builtin_bswap32(st[4]), __builtin_bswap32(st[5]), __builtin_bswap32(st[6]),
                              __builtin_bswap32(st[7]));
  out[0] = o0;
  out[1] = o1;
  if (expected) {
    const uint4* ex = reinterpret_cast<const uint4*>(expected + 32 * m);
    const uint4 e0 = ex[0], e1 = ex[1];
    const bool eq = e0.x == o0.x && e0.y == o0.y && e0.z == o0.z && e0.w == o0.w && e1.x == o1.x && e1.y == o1.y &&
                    e1.z == o1.z && e1.w == o1.w;
    if (eq) atomicOr(bitmap32 + (m >> 5), 1u << (m & 31));
  }
}

// ---- block-count bucketing (device counting sort) ----
constexpr uint32_t kBuckets = 1024;

__device__ __forceinline__ uint32_t bucket_of(uint32_t len) {
  const uint32_t nb = (len + 8u) / 64u + 1u;  // compression calls for this message
  return nb >= kBuckets ? kBuckets - 1 : nb;
}

__global__ void __launch_bounds__(256) k_len_hist(const uint32_t* __restrict__ lengths, uint64_t n,
                                                  uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[kBuckets];
  for (uint32_t b = threadIdx.x; b < kBuckets; b += blockDim.x) h[b] = 0;
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    atomicAdd(&h[bucket_of(lengths[i])], 1u);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < kBuckets; b += blockDim.x)
    if (h[b]) atomicAdd(&hist[b], h[b]);
}

// exclusive scan in descending bucket order (longest messages first), one block of kBuckets threads
__global__ void __launch_bounds__(1024) k_len_scan(uint32_t* __restrict__ hist) {
  __shared__ uint32_t s[kBuckets];
  const uint32_t t = threadIdx.x;
  s[t] = hist[kBuckets - 1 - t];
  __syncthreads();
  for (uint32_t off = 1; off < kBuckets; off <<= 1) {
    const uint32_t v = t >= off ? s[t - off] : 0u;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  const uint32_t incl = s[t];
  hist[kBuckets - 1 - t] = incl - hist[kBuckets - 1 - t];  // exclusive start of bucket
}

__global__ void __launch_bounds__(256) k_len_scatter(const uint32_t* __restrict__ lengths, uint64_t n,
                                                     uint32_t* __restrict__ cursor, uint32_t* __restrict__ order) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t pos = atomicAdd(&cursor[bucket_of(lengths[i])], 1u);
  order[pos] = (uint32_t)i;
}

size_t sha256_order_scratch_bytes(uint64_t) { return kBuckets * sizeof(uint32_t); }

hipError_t launch_sha256_order(const uint32_t* lengths, uint64_t n, uint32_t* order, void* scratch, hipStream_t st) {
  if (n == 0) return hipSuccess;
  uint32_t* hist = reinterpret_cast<uint32_t*>(scratch);
  hipError_t e = hipMemsetAsync(hist, 0, kBuckets * sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  uint64_t blocks = (n + 255) / 256;
  const uint32_t hb = (uint32_t)(blocks < 2048 ? blocks : 2048);
  hipLaunchKernelGGL(k_len_hist, dim3(hb), dim3(256), 0, st, lengths, n, hist);
  hipLaunchKernelGGL(k_len_scan, dim3(1), dim3(kBuckets), 0, st, hist);
  hipLaunchKernelGGL(k_len_scatter, dim3((uint32_t)blocks), dim3(256), 0, st, lengths, n, hist, order);
  return hipGetLastError();
}

hipError_t launch_sha256(const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths, const uint32_t* order,
                         uint64_t n, uint8_t* digests, const uint8_t* expected, uint8_t* bitmap, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (expected) {
    hipError_t e = hipMemsetAsync(bitmap, 0, ((n + 31) / 32) * 4, st);
    if (e != hipSuccess) return e;
  }
  const uint64_t blocks = (n + 255) / 256;
  // experiment knob: dynamic LDS per block caps the blocks per CU (occupancy
  // A/B of the L2 footprint: lanes x the 128-B line each one has open)
  static const uint32_t pad = [] {
    const char* e = getenv("PBFTV_SHA_LDS_PAD");
    return e ? (uint32_t)atoi(e) : 0u;
  }();
  static const bool ring = [] {  // PBFTV_SHA_RING=0: the dword-window kernel (A/B)
    const char* e = getenv("PBFTV_SHA_RING");
    return !(e && e[0] == '0');
  }();
  if (ring) {
    hipLaunchKernelGGL(k_sha256_ring, dim3((uint32_t)blocks), dim3(256), 0, st, data, offsets, lengths, order, n,
                       digests, expected, reinterpret_cast<uint32_t*>(bitmap));
  } else {
    hipLaunchKernelGGL(k_sha256, dim3((uint32_t)blocks), dim3(256), pad, st, data, offsets, lengths, order, n,
                       digests, expected, reinterpret_cast<uint32_t*>(bitmap));
  }
  return hipGetLastError();
}

}  // namespace pbftv
