// kernels.h -- host-side launch wrappers for the gfx950 kernels (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace pbftv {

// ---- ECDSA-P256 (p256_kernels.hip) ----
size_t table_bytes_per_base();
size_t build_tables_scratch_bytes(uint32_t nkeys);
// tables: (nkeys + 1) comb tables, base 0 = G.  keys_le: nkeys x {x[8], y[8]} LE words.
hipError_t launch_build_tables(const uint32_t* keys_le, uint32_t nkeys, uint32_t* tables, uint32_t* valid,
                               void* scratch, hipStream_t st);
size_t ecdsa_scratch_bytes(uint64_t n);
// stage 1: scal (n * 64 B) + flag (n B) + prefix (scalar_prefix_bytes(n)) device scratch
int scalar_batch(uint64_t n);
size_t scalar_prefix_bytes(uint64_t n);
hipError_t launch_ecdsa_scalars(const uint8_t* hashes, const uint8_t* sigs, const uint32_t* key_idx, uint64_t n,
                                const uint32_t* key_valid, uint32_t nkeys, void* scal, uint8_t* flag, void* prefix,
                                hipStream_t st);
// stage 2: bitmap ceil(n/8) B
hipError_t launch_ecdsa_comb(const void* scal, const uint8_t* flag, const uint8_t* sigs, const uint32_t* key_idx,
                             uint64_t n, const uint32_t* tables, uint8_t* bitmap, hipStream_t st);

// ---- SHA-256 (sha256_kernels.hip) ----
// data must stay readable 4 bytes past every message end (device allocations are padded).
// order: optional permutation (lane -> message), used for block-count bucketing.
// If expected != nullptr, also writes the LSB-first match bitmap (ceil(n/8) B).
hipError_t launch_sha256(const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths, const uint32_t* order,
                         uint64_t n, uint8_t* digests, const uint8_t* expected, uint8_t* bitmap, hipStream_t st);
// Sort messages by block count on the device (counting sort): order[n] out.
size_t sha256_order_scratch_bytes(uint64_t n);
hipError_t launch_sha256_order(const uint32_t* lengths, uint64_t n, uint32_t* order, void* scratch, hipStream_t st);

}  // namespace pbftv
