// kernels.h -- host-side launch wrappers for the gfx950 kernels (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace pbftv {

// ---- ECDSA-P256 (p256_kernels.hip) ----
// Comb tables: geometry code w (p256_algo.h CombGeom: W-bit windows, or the
// mixed 21 / 29); table_bytes(w) per base (8: 264 KiB, 16: 34 MiB, 21:
// 1.14 GB, 22: 1.61 GB, 24: 5.9 GB, 26: 21.5 GB, 29: 120 GB).
size_t table_bytes(int w);
int table_windows(int w);  // windows = table entries added per scalar
// (G, key) geometry pairs with instantiated verify kernels
// (split by G width into the instantiation units p256_verify_g*.hip)
#define PBFTV_COMBOS_G29(X) X(29, 24) X(29, 22) X(29, 21) X(29, 20) X(29, 16)
#define PBFTV_COMBOS_G26(X) X(26, 24) X(26, 22) X(26, 21) X(26, 20) X(26, 16)
#define PBFTV_COMBOS_G24(X) X(24, 24) X(24, 22) X(24, 20) X(24, 16)
#define PBFTV_COMBOS_SMALL(X) X(20, 20) X(16, 16) X(16, 12) X(16, 8) X(8, 8)
#define PBFTV_COMBOS(X) PBFTV_COMBOS_G29(X) PBFTV_COMBOS_G26(X) PBFTV_COMBOS_G24(X) PBFTV_COMBOS_SMALL(X)
#define PBFTV_TABLE_WIDTHS(X) X(8) X(12) X(16) X(20) X(21) X(22) X(24) X(26) X(29)
struct TableScratch {
  void* bases;
  void* lbuf;
  void* hbuf;
  void* small_scratch;
  void* entry_scratch;
  uint64_t entry_lanes;
};
struct TableScratchSizes {
  size_t bases, lbuf, hbuf, small_scratch, entry_scratch;
  uint64_t entry_lanes;
};
TableScratchSizes table_scratch_sizes(int w, uint32_t nbases);
// Build nb tables (G first when with_g) of width w; table b is written at
// tabs[b] (a device array of nb pointers to table_bytes(w) each); keys_le:
// {x[8], y[8]} LE words per key, key0 = first key of this launch; valid[key]
// written for every key built.
hipError_t launch_build_tables(int w, const uint32_t* keys_le, uint32_t key0, uint32_t nb, int with_g,
                               uint32_t* valid, uint32_t* const* tabs, TableScratch& sc, hipStream_t st);
// stage 1 -> stage 2 records (verify_kernels.h SigRec: 128 B per signature) and
// the prefix-product scratch of stage 1's batched inversion
size_t ecdsa_record_bytes(uint64_t n);
int scalar_batch(uint64_t n);
size_t scalar_prefix_bytes(uint64_t n);
// key order of a batch (stage 0 -> stage 1): per-key totals and claim
// counters in the key-sort header; total == nullptr: arrival order
struct KeyOrder {
  const uint32_t* total;
  uint32_t* claim;
  uint32_t nkeys;
};
// stage 1: inputs in arrival order; record of signature i written at its
// place in key order (placed by stage 1 itself from ko) or at i
hipError_t launch_ecdsa_scalars(const uint8_t* hashes, const uint8_t* sigs, const uint32_t* key_idx, uint64_t n,
                                const uint32_t* key_valid, uint32_t nkeys, void* rec, void* prefix,
                                const KeyOrder& ko, hipStream_t st);
// stage 2: (wg, wq) one of PBFTV_COMBOS; qtabs = device array of the nkeys
// key tables' addresses (width wq each, one allocation per key).
// okb == nullptr: records in arrival order, LSB-first bitmap (ceil(n/8) B)
// written directly; else one byte per signature at its batch index (okb, n B)
// and launch_pack_bits builds the bitmap.
// cuflag: the device's certificate flags (kCuFlagWords, zeroed; null: the
// comb never yields to an armed certificate on its CU, verify_kernels.h)
hipError_t launch_ecdsa_comb(int wg, int wq, const void* rec, uint64_t n, const uint32_t* gtab,
                             const uint32_t* const* qtabs,
                             uint8_t* bitmap, uint8_t* okb, const uint32_t* cuflag, hipStream_t st);
constexpr uint32_t kCuFlagWords = 4096;  // one word per (XCC, SE, SH, CU)
// stage 0 (optional): per-key totals for the key order (scratch:
// key_sort_scratch_bytes = a header of key_sort_header_bytes, which must be
// ZERO when the scratch is first used and is left zero by every batch).
// parity: the caller's batch counter for this scratch (alternates the header's
// two counter sets; any sequence of values that alternates is fine).  *out is
// what stage 1 needs.
bool key_sort_wanted(uint64_t n, uint32_t nkeys);
size_t key_sort_header_bytes();
size_t key_sort_scratch_bytes(uint64_t n, uint32_t nkeys);
hipError_t launch_key_count(const uint32_t* key_idx, uint64_t n, uint32_t nkeys, void* scratch, uint32_t parity,
                            KeyOrder* out, hipStream_t st);
hipError_t launch_pack_bits(const uint8_t* okb, uint64_t n, uint8_t* bitmap, hipStream_t st);
// latency path for small batches: one wave per signature (scalars, per-window
// points, butterfly sum, check) in one launch.  Output: okbytes[i] (one byte per
// signature) when okbytes != nullptr, else bit i of bitmap set/cleared by word
// atomics (bitmap need not be zeroed; its word-aligned 4-byte span is touched).
// argument packs of the per-geometry launchers (verify_kernels.h)
struct CombArgs {
  const void* rec;
  uint64_t n;
  const uint32_t* gtab;
  const uint32_t* const* qtabs;
  uint8_t* bitmap;
  uint8_t* okb;
  const uint32_t* cuflag;
};
struct WaveArgs {
  const uint8_t* hashes;
  const uint8_t* sigs;
  const uint32_t* key_idx;
  uint64_t n;
  const uint32_t* key_valid;
  uint32_t nkeys;
  const uint32_t* gtab;
  const uint32_t* const* qtabs;
  uint8_t* bitmap;
  uint8_t* okbytes;
  bool one_wave;  // the quad schedule (one 64-thread workgroup per signature) even where rows would serve
};
// one_wave: a workgroup of one wave per signature -- beside a batch that
// holds every wave slot, such a workgroup starts in the first slot a finished
// batch block frees, where a row-schedule workgroup (5-8 waves) waits for
// several on one CU (pbftv_api.cpp launch_range)
hipError_t launch_ecdsa_wave(int wg, int wq, const uint8_t* hashes, const uint8_t* sigs, const uint32_t* key_idx,
                             uint64_t n, const uint32_t* key_valid, uint32_t nkeys, const uint32_t* gtab,
                             const uint32_t* const* qtabs, uint8_t* bitmap, uint8_t* okbytes, hipStream_t st,
                             bool one_wave = false);
// batches up to this size take the latency path (env PBFTV_WAVE_MAX overrides; 0 disables)
uint64_t wave_path_max();
// The latency path's result bytes (okbytes): bit 0 = the verdict; the
// launched row kernel (k_ecdsa_rows) sets kRowsExact when the signature took
// its exact rerun (a doubling or cancellation in the row tree, a live window
// with two zero digits, r + n < p); the armed row kernel writes 2 instead
// (the host reruns the certificate with a launch).  Counted by pbftv_qc_counters.
constexpr int kRowsExact = 4;

// The latency path's mailbox in pinned coherent host memory: a 64-B header,
// then the inputs of up to cap signatures (hashes cap*32, r||s cap*64, key
// indices cap*4) and one result byte per signature.  The host writes the
// inputs, n and then bell = the request's sequence number; an armed kernel
// (k_ecdsa_wave_armed) waiting for that number serves it; stop = seq cancels
// the armed kernel, which then reports expired = seq (verify_kernels.h); so
// does any change of halt (a disarm, or the process-wide quiesce of a GPU,
// pbftv_api.cpp).  Two armed kernels can be resident at once (a rotation's
// successor beside its predecessor, one per armed stream), so each armed
// stream slot has its OWN expired word and its own live words (each wave's
// first request number once it is resident): two kernels leaving at once
// (a halt bump) cannot overwrite each other's report.
// The first kQcSlots signatures are also written to their own 3-line slot
// (slot_off): line 0 = {tag, n, key, 0, hash[32], 0, 0, 0, tag}, line 1 =
// {tag, 0, 0, 0, r[32], 0, 0, 0, tag}, line 2 likewise with s; the tags (the
// request number) are written after their line's data, the last dword first.
struct QcMail {
  uint32_t bell, n, stop, expired_s0, cap, halt, expired_s1, pad[9];  // (stop at dword 2, halt at 5: read by the kernel)
  static constexpr uint32_t kQcSlots = 8;
  static constexpr uint32_t kQcCap = 128;  // signatures per call up to which the mailbox is laid out at cap = 128
  static constexpr int kArmSlots = 2;      // armed stream slots (pbftv_api.cpp Device::qstream)
  // the expired word of armed stream slot s
  __host__ __device__ uint32_t* expired(int s) { return s ? &expired_s1 : &expired_s0; }
  static constexpr size_t slot_off(uint32_t i) { return 64 + 192 * (size_t)i; }
  // each armed wave's first request number once it is resident (4 B per
  // wave), per armed stream slot
  static constexpr size_t live_off(int s = 0) { return 64 + 192 * (size_t)kQcSlots + 4 * (size_t)kQcCap * s; }
  // one verdict byte per signature, right after the live words: with the
  // header and the slot lines in the mailbox's FIRST 4-KiB page, so a
  // certificate of <= kQcSlots touches one page of it (one TLB entry on the
  // host, one translation on the GPU, both warm from the polling)
  static constexpr size_t res_off(uint32_t = kQcCap) { return live_off(kArmSlots); }
  // the input arrays of signatures kQcSlots.. (and of every signature on the
  // launched path), after cap verdict bytes
  static constexpr size_t arrays_off(uint32_t cap = kQcCap) {
    return (res_off() + (cap > kQcCap ? cap : kQcCap) + 63) & ~(size_t)63;
  }
  static constexpr size_t hashes_off(uint32_t cap = kQcCap) { return arrays_off(cap); }
  static constexpr size_t sigs_off(uint32_t cap) { return arrays_off(cap) + 32 * (size_t)cap; }
  static constexpr size_t keys_off(uint32_t cap) { return arrays_off(cap) + 96 * (size_t)cap; }
  // diagnostics: per armed wave (slots and helpers), its {wall clock, shader
  // clock} when it saw its request and when it wrote its verdict (pbftv_qc_stamps)
  static constexpr size_t stamps_off(uint32_t cap) { return (keys_off(cap) + 4 * (size_t)cap + 63) & ~(size_t)63; }
  static constexpr size_t bytes(uint32_t cap) { return stamps_off(cap) + 32 * (size_t)kQcCap + 64; }
};
struct ArmArgs {
  QcMail* mail;
  uint32_t want;       // the request sequence number this launch serves
  uint64_t budget;     // wall-clock ticks before it gives up
  const uint32_t* key_valid;
  uint32_t nkeys;
  const uint32_t* gtab;
  const uint32_t* const* qtabs;
  uint32_t spin;       // between polls: 0 = s_sleep, 1 = none, k >= 2 = k dependent VALU ops
  uint32_t halt;       // the mailbox's halt word at arming: any other value cancels
  uint64_t* relay;     // wide kernel (kQcCap waves): device word {number, n}, zeroed before launch; null: narrow
  uint32_t stamps;     // 1: each serving wave writes its GPU timestamps (pbftv_qc_stamps*; PBFTV_QC_STAMPS=1)
  int slot;            // its armed stream slot: the expired word and live words it writes (QcMail)
  uint32_t slots;      // narrow row-schedule kernel: signature slots armed (<= kQcSlots; one workgroup each)
  uint32_t* cuflag;    // the device's certificate flags (null: none); a serving workgroup raises its CU's word
  uint32_t cuyield;    // 2: also the word of the CU sharing its instruction cache
};
hipError_t launch_ecdsa_wave_armed(int wg, int wq, const ArmArgs& a, hipStream_t st);

// ---- SHA-256 (sha256_kernels.hip) ----
// data must stay readable 4 bytes past every message end (device allocations are padded).
// order: optional permutation (lane -> message), used for block-count bucketing.
// If expected != nullptr, also writes the LSB-first match bitmap (ceil(n/8) B).
hipError_t launch_sha256(const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths, const uint32_t* order,
                         uint64_t n, uint8_t* digests, const uint8_t* expected, uint8_t* bitmap, hipStream_t st);
// Sort messages by block count on the device (counting sort): order[n] out.
size_t sha256_order_scratch_bytes(uint64_t n);
hipError_t launch_sha256_order(const uint32_t* lengths, uint64_t n, uint32_t* order, void* scratch, hipStream_t st);

// ---- Go-JSON preimages on the device (gojson_kernels.hip) ----
// Column-wise message fields (device pointers, n entries each); a string
// column is a byte blob with per-message offset and length.
struct StrCol {
  const uint8_t* data;
  const uint64_t* off;
  const uint32_t* len;
};
struct RequestCols {
  const int64_t* ts;
  StrCol cid, op;
  const int64_t* seq;
};
struct VoteCols {
  const int64_t* view;
  const int64_t* seq;
  StrCol digest, node;
  const int64_t* type;
};
struct ReplyCols {
  const int64_t* view;
  const int64_t* ts;
  StrCol cid, node, result;
};
struct PrePrepareCols {
  const int64_t* view;
  const int64_t* seq;
  StrCol digest;
  const uint8_t* has_req;  // 0: requestMsg is nil (request columns still hold n entries)
  RequestCols req;
};
// consensus states a vote batch is checked against (State.verifyMsg)
struct StateCols {
  const int64_t* view;
  const int64_t* last_seq;
  const uint8_t* req_digest;  // 32 B per state
  const uint32_t* idx;        // per vote: its state
  uint32_t n;
};
// Message i's preimage is written at out + slot[i] (slot sized by the
// gojson_enc.h bound), its length to out_len[i].  launch_gojson_vote also
// writes msg_ok[i] = verifyMsg result when msg_ok != nullptr.
hipError_t launch_gojson_request(const RequestCols& c, uint64_t n, const uint64_t* slot, uint8_t* out,
                                 uint32_t* out_len, hipStream_t st);
hipError_t launch_gojson_vote(const VoteCols& c, uint64_t n, const uint64_t* slot, uint8_t* out, uint32_t* out_len,
                              const StateCols& s, uint8_t* msg_ok, hipStream_t st);
hipError_t launch_gojson_reply(const ReplyCols& c, uint64_t n, const uint64_t* slot, uint8_t* out, uint32_t* out_len,
                               hipStream_t st);
hipError_t launch_gojson_preprepare(const PrePrepareCols& c, uint64_t n, const uint64_t* slot, uint8_t* out,
                                    uint32_t* out_len, hipStream_t st);
// pre-prepare flush: preimage i at slot[i], its embedded request's ("null" if
// nil) at slot[n + i]; lengths likewise (out_len has 2n entries)
hipError_t launch_gojson_preprepare_pair(const PrePrepareCols& c, uint64_t n, const uint64_t* slot, uint8_t* out,
                                         uint32_t* out_len, hipStream_t st);
// verifyMsg of pre-prepares against their states, the digest field compared
// with the digest of the message's own request (req_digests, 32 B per message)
hipError_t launch_preprepare_verify(const int64_t* view, const int64_t* seq, const StrCol& digest,
                                   const uint8_t* req_digests, const StateCols& s, uint64_t n, uint8_t* msg_ok,
                                   hipStream_t st);

}  // namespace pbftv
