/* pbftv.h -- C ABI of the MI355X batch verifier for simple_pbft's crypto hot path.
 *
 * Drop-in boundary.  The reference (1556174776/simple_pbft,
 * Go) has no FFI; the functions below are what a thin cgo shim binds so the
 * Go call sites keep their signatures (INTEGRATION.md shows the binding):
 *
 *   pbftv_hash_hex            <- utils.Hash(content []byte) string          utils/utils.go:13-17
 *   pbftv_sha256_batch        <- batched utils.Hash over a pool snapshot   utils/utils.go:13-17
 *   pbftv_gojson_*            <- json.Marshal preimages hashed by digest() pbft/consensus/pbft_impl.go:235-243,
 *                                                                          pbft/consensus/pbft_msg_types.go:3-38
 *   pbftv_digest_request_batch<- digest(*RequestMsg) for many requests     pbft/consensus/pbft_impl.go:73,235-243
 *   pbftv_digest_check_batch  <- digest recompute + compare per message    pbft/consensus/pbft_impl.go:190-199
 *   pbftv_verify_msg_batch    <- State.verifyMsg over a vote snapshot      pbft/consensus/pbft_impl.go:176-202
 *   pbftv_register_keys       <- per-node public-key table (planned by the author next to
 *                                NodeTable, 需要改进的地方.md:17 / pbft/network/node.go:60-65)
 *   pbftv_ecdsa_p256_verify_batch <- Go crypto/ecdsa.Verify per signed pool message
 *                                (absent in the reference)
 *   pbftv_qc_verify           <- quorum count of prepared()/committed()    pbft/consensus/pbft_impl.go:207-232
 *
 * Conventions
 *   - The caller owns every buffer; the library never keeps a pointer after a
 *     call returns (cgo rule: no Go pointers retained by C).
 *   - Host-buffer calls are synchronous.  *_dev calls take device pointers on
 *     one of the context's devices and enqueue on `stream` (a hipStream_t, or
 *     NULL for the context's stream of that device) without synchronising.
 *   - Return 0 on success, negative PBFTV_E* on API / device errors.  A failed
 *     signature or digest is never an error: it is a 0 bit.
 *   - Bitmaps are LSB-first: bit i of the batch is (bitmap[i/8] >> (i%8)) & 1.
 *   - Big-endian 32-byte integers (hash, r, s, X, Y) exactly as Go's
 *     big.Int.FillBytes / elliptic.Marshal would lay them out.
 *   - A context is safe to share across threads (one lock per device).
 *   - There is no CPU fallback: with no usable gfx950 device pbftv_open fails
 *     with PBFTV_ENODEV.
 */
#ifndef PBFTV_H
#define PBFTV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBFTV_OK 0
#define PBFTV_EINVAL (-1)   /* bad argument (null pointer, bad device index, ...) */
#define PBFTV_ENODEV (-2)   /* no usable GPU in device_mask */
#define PBFTV_EDEVICE (-3)  /* HIP runtime / kernel error; see pbftv_last_error() */
#define PBFTV_ENOMEM (-4)   /* device or pinned host allocation failed */
#define PBFTV_ENOKEYS (-5)  /* verify called before pbftv_register_keys */

typedef struct pbftv_ctx pbftv_ctx;

/* Open a context on the GPUs in device_mask (bit d = HIP device d; 0 = all
 * visible).  Batches passed to the host-buffer calls are split into
 * contiguous shards, one per device (no collective: the shards are
 * independent and the bitmaps are concatenated). */
int pbftv_open(pbftv_ctx** out, uint32_t device_mask);
void pbftv_close(pbftv_ctx* ctx);
int pbftv_device_count(const pbftv_ctx* ctx);
/* HIP device id of the context's i-th device, or -1. */
int pbftv_device_id(const pbftv_ctx* ctx, int i);
const char* pbftv_strerror(int code);
/* Last error message of the calling thread ("" if none). */
const char* pbftv_last_error(void);
/* Pre-size per-device scratch for batches of up to n items (optional). */
int pbftv_reserve(pbftv_ctx* ctx, uint64_t n);

/* ---- device memory / stream plumbing ---------------------------------- */
/* For callers that keep pool snapshots resident in HBM (and for bench.py):
 * allocations on the context's device index dev, copies on that device's
 * stream (synchronous), and a stream synchronise.  pbftv_dev_alloc memory
 * comes from a stream-ordered pool of the context; pbftv_dev_free returns it
 * once the work queued so far on the context's streams (its own and those
 * from pbftv_stream_create) has passed, without a device-wide
 * synchronisation, and waits on the host for the context's work on other
 * caller streams -- so a free does not stop the armed latency kernels. */
int pbftv_dev_alloc(pbftv_ctx* ctx, int dev, uint64_t bytes, void** out_ptr);
int pbftv_dev_free(pbftv_ctx* ctx, int dev, void* ptr);
/* Pinned host memory (hipHostMalloc, portable): batches placed in it skip the
 * staging copy of the host-buffer verify path (e.g. a cgo shim's pool-flush
 * buffers).  A freed block is kept for the next pbftv_host_alloc of a similar
 * size (up to 1 GiB per context; released at pbftv_close), so a free does
 * not synchronise the GPU either. */
int pbftv_host_alloc(pbftv_ctx* ctx, uint64_t bytes, void** out_ptr);
int pbftv_host_free(pbftv_ctx* ctx, void* ptr);
int pbftv_memcpy_h2d(pbftv_ctx* ctx, int dev, void* dst, const void* src, uint64_t bytes);
int pbftv_memcpy_d2h(pbftv_ctx* ctx, int dev, void* dst, const void* src, uint64_t bytes);
int pbftv_memset_dev(pbftv_ctx* ctx, int dev, void* dst, int value, uint64_t bytes);
/* The context's stream of device dev as a hipStream_t (for *_dev calls). */
void* pbftv_stream(pbftv_ctx* ctx, int dev);
int pbftv_stream_sync(pbftv_ctx* ctx, int dev);
/* Caller streams on device dev for *_dev calls (non-blocking HIP streams).  A
 * stream made here owns its ECDSA verify scratch (stage-1 records, key order,
 * result bytes; freed by pbftv_stream_destroy), so verifies enqueued on two
 * such streams run concurrently on the GPU: a caller that alternates batches
 * between two streams overlaps batch j + 1's scalar stage with batch j's comb.
 * Other device scratch shared by calls on different streams (d.stream and any
 * foreign hipStream_t) is ordered by the library (an event per device), so
 * concurrent *_dev calls on several streams are safe. */
int pbftv_stream_create(pbftv_ctx* ctx, int dev, void** out_stream);
int pbftv_stream_destroy(pbftv_ctx* ctx, int dev, void* stream);
int pbftv_stream_wait(pbftv_ctx* ctx, int dev, void* stream);

/* Batches of up to n signatures take the latency path (one wave per
 * signature); larger ones the lane path (scalar + comb kernels).  Default
 * 2048, or PBFTV_WAVE_MAX at pbftv_open; 0 disables the latency path.  Read
 * once per call from the context, never from the environment on the call
 * path.
 *
 * Up to 128 signatures of a latency-path call are served by a resident
 * "armed" kernel polling a doorbell in pinned host memory (a workgroup per
 * signature slot: as many as the largest recent certificate, at least 4;
 * up to 128 once calls of 9..128 signatures have been seen), so no launch is
 * on the call's path.  A keeper thread per device replaces it
 * before its budget runs out for as long as calls keep coming.  Environment,
 * read at every arming:
 *   PBFTV_QC_ARM=0            never arm (every call launches);
 *   PBFTV_QC_ARM_MS=100       one armed kernel's budget (ms);
 *   PBFTV_QC_KEEP_MS=10000    keep one armed this long after the last call
 *                             (0: no keeper; the kernel runs out);
 *   PBFTV_QC_WIDE=0           never arm the 128-wave form;
 *   PBFTV_QC_YIELD            whether a lane-path batch halts the armed
 *                             kernel (certificates meanwhile are launched,
 *                             ~0.1 ms beside the batch instead of ~0.04 ms;
 *                             the keeper re-arms after it): "1" always, "0"
 *                             never; unset (default) when no certificate
 *                             came for PBFTV_QC_YIELD_IDLE_MS (50 ms).  A
 *                             resident server costs a busy stream ~3 %
 *                             (narrow) to 6-9 % (wide, 67 votes);
 *   PBFTV_QC_CU_YIELD         while an armed workgroup serves, the lane-path
 *                             comb waves on its CU park at their next step
 *                             (a per-CU flag word; at most 50 µs): "1" the
 *                             default, "0" never, "2" also on the CU that
 *                             shares its instruction cache.  3 signatures
 *                             beside a 1M stream 40.0 -> 33.5 µs p50 at the
 *                             same stream rate;
 *   PBFTV_QC_EXCLUSIVE_CU     armed workgroups take whole CUs, so a
 *                             concurrent batch does not share their SIMDs
 *                             (with PBFTV_QC_YIELD=0): "narrow" the narrow
 *                             kernel (one CU per armed slot), "1" the wide
 *                             one too (128 CUs); off by default;
 *   PBFTV_QC_ROWS=0           the quad schedule (one wave per signature)
 *                             instead of the row schedule (a workgroup per
 *                             signature), for A/B;
 *   PBFTV_QC_ROWS_MAX         launched batches up to this many signatures
 *                             take the row schedule (default 128);
 *   PBFTV_QC_SLOTS=k          arm k narrow slots (1..8) instead of the
 *                             largest recent certificate (at least 4);
 *   PBFTV_QC_STAMPS=1         the kernel records GPU timestamps
 *                             (pbftv_qc_stamps*);
 *   PBFTV_TRACE_QC=1          why a call was launched, on stderr.
 * The library's own device frees (scratch growth, re-registration) stop every
 * armed kernel on the GPU first (hipFree waits for every kernel); the
 * caller's pbftv_dev_free / pbftv_host_free do not. */
int pbftv_set_latency_path_max(pbftv_ctx* ctx, uint64_t n);

/* Per-kernel timing with HIP events recorded on the launch stream around every
 * kernel launch while enabled.  kernel: 0 = ecdsa scalars, 1 = ecdsa comb,
 * 2 = sha256, 3 = ecdsa wave-per-signature (small batches), 4 = Go-JSON message
 * encoder (digest / flush batches).  pbftv_kernel_time_ms synchronises the device's stream and
 * returns the summed milliseconds and the launch count since the last reset. */
#define PBFTV_K_ECDSA_SCALARS 0
#define PBFTV_K_ECDSA_COMB 1
#define PBFTV_K_SHA256 2
#define PBFTV_K_ECDSA_WAVE 3
#define PBFTV_K_GOJSON 4
int pbftv_set_kernel_timing(pbftv_ctx* ctx, int enable);
int pbftv_kernel_time_ms(pbftv_ctx* ctx, int dev, int kernel, double* out_ms, uint64_t* out_launches);
int pbftv_reset_kernel_times(pbftv_ctx* ctx);
/* Diagnostics of the last latency-path call (n <= 2048) on device dev:
 * out[0] = host ns from entry to the request being handed over (bell rung or
 * kernel launched), out[1] = host ns from entry to return, out[2] bit 0 = 1
 * if an armed kernel served it, 0 if a launch did, bits 1..31 = host ns from
 * entry to the verdicts of the first 8 signatures all in, bits 32..63 = host
 * ns from entry to holding the device lock, out[3..6] = the armed kernel's
 * slot-0 wave: GPU wall clock and shader clock when it saw the request, and
 * when it wrote its verdict (0 after a launch; written only while
 * PBFTV_QC_STAMPS=1 was set when the kernel was armed), out[7] = the
 * wall-clock rate in kHz. */
int pbftv_qc_stamps(pbftv_ctx* ctx, int dev, uint64_t out[8]);
/* The same GPU stamps for every armed wave of the last call (up to `waves`
 * entries of {seen wall, seen shader clock, done wall, done shader clock};
 * helper waves past the 8 slots included): returns the number written, 0 if a
 * launch served the call.  Stamps of waves that had no signature are stale. */
int pbftv_qc_stamps_all(pbftv_ctx* ctx, int dev, uint64_t* out, uint32_t waves);
/* Counters of the latency path on device dev since pbftv_open (diagnostics;
 * tests assert which path served what): out[0] calls, out[1] calls served by
 * an armed kernel, out[2] armed calls handed to a launched rerun (the armed
 * row kernel met an exceptional signature: a doubling or cancellation in its
 * tree, a live window with two zero digits, r + n < p), out[3] signatures that
 * took a launched row kernel's exact path, out[4] launched latency kernels,
 * out[5] armings, out[6] keeper rotations, out[7] the armed kernel now: its
 * workgroups (0: none armed) | 1 << 32 if it is the wide one. */
int pbftv_qc_counters(pbftv_ctx* ctx, int dev, uint64_t out[8]);

/* ---- SHA-256 digests (utils.Hash) ------------------------------------ */

/* utils.Hash(content): lowercase hex SHA-256, 64 chars + NUL into out_hex. */
int pbftv_hash_hex(pbftv_ctx* ctx, const uint8_t* content, uint64_t len, char out_hex[65]);

/* n messages at data+offsets[i], lengths[i] bytes -> out_digests (n*32 raw bytes). */
int pbftv_sha256_batch(pbftv_ctx* ctx, const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths,
                       uint64_t n, uint8_t* out_digests);

/* As above, plus compare against expected (n*32): bit i = digest matches. */
int pbftv_digest_check_batch(pbftv_ctx* ctx, const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths,
                             const uint8_t* expected, uint64_t n, uint8_t* out_bitmap);

/* Device-resident form on device index dev (0..pbftv_device_count-1).  The
 * data buffer must be readable 4 bytes past the end of every message
 * (pbftv_dev_alloc / hipMalloc allocations are).  order (may be NULL) is a lane ->
 * message permutation; pbftv_sha256_order_dev builds one that groups messages
 * by block count.  d_expected/d_bitmap may be NULL (digests only); d_bitmap
 * must be ceil(n/32)*4 bytes when used. */
int pbftv_sha256_batch_dev(pbftv_ctx* ctx, int dev, const uint8_t* d_data, const uint64_t* d_offsets,
                           const uint32_t* d_lengths, const uint32_t* d_order, uint64_t n, uint8_t* d_digests,
                           const uint8_t* d_expected, uint8_t* d_bitmap, void* stream);
int pbftv_sha256_order_dev(pbftv_ctx* ctx, int dev, const uint32_t* d_lengths, uint64_t n, uint32_t* d_order,
                           void* stream);

/* ---- Go-JSON digest preimages (json.Marshal of pbft_msg_types.go) ----- */
/* Each writes at most cap bytes to out and returns the full encoded length
 * (call with cap = 0 to size).  Strings are byte strings (ptr, len) and may
 * hold arbitrary bytes; encoding follows Go 1.19 encoding/json exactly. */
uint64_t pbftv_gojson_request(int64_t timestamp, const char* client_id, uint64_t client_id_len, const char* operation,
                              uint64_t operation_len, int64_t sequence_id, uint8_t* out, uint64_t cap);
uint64_t pbftv_gojson_vote(int64_t view_id, int64_t sequence_id, const char* digest, uint64_t digest_len,
                           const char* node_id, uint64_t node_id_len, int64_t msg_type, uint8_t* out, uint64_t cap);
/* Signed VoteMsg on the wire (build-added; no reference
 * counterpart): the VoteMsg fields of pbft_msg_types.go:25-31 followed by
 * Signature []byte `json:"signature"` -- base64.StdEncoding, or null when
 * sig_nil != 0 (Go's nil slice).  The signing preimage is pbftv_gojson_vote. */
uint64_t pbftv_gojson_vote_signed(int64_t view_id, int64_t sequence_id, const char* digest, uint64_t digest_len,
                                  const char* node_id, uint64_t node_id_len, int64_t msg_type, const uint8_t* sig,
                                  uint64_t sig_len, int sig_nil, uint8_t* out, uint64_t cap);
/* Signed RequestMsg / ReplyMsg / PrePrepareMsg on the wire:
 * the struct of pbft_msg_types.go:3-23 followed by "signature" as above.  Each
 * signing preimage is the unsigned encoding (pbftv_gojson_request / _reply /
 * _preprepare).  A client signs its request with the sequenceID it sent (the
 * reference's clients leave it 0; StartConsensus assigns it, pbft_impl.go:67);
 * a pre-prepare's embedded request carries the client's signature on the wire
 * (req_sig*), while the primary's preimage embeds the unsigned request. */
uint64_t pbftv_gojson_request_signed(int64_t timestamp, const char* client_id, uint64_t client_id_len,
                                     const char* operation, uint64_t operation_len, int64_t sequence_id,
                                     const uint8_t* sig, uint64_t sig_len, int sig_nil, uint8_t* out, uint64_t cap);
uint64_t pbftv_gojson_reply_signed(int64_t view_id, int64_t timestamp, const char* client_id, uint64_t client_id_len,
                                   const char* node_id, uint64_t node_id_len, const char* result, uint64_t result_len,
                                   const uint8_t* sig, uint64_t sig_len, int sig_nil, uint8_t* out, uint64_t cap);
uint64_t pbftv_gojson_preprepare_signed(int64_t view_id, int64_t sequence_id, const char* digest, uint64_t digest_len,
                                        int has_request, int64_t req_timestamp, const char* req_client_id,
                                        uint64_t req_client_id_len, const char* req_operation,
                                        uint64_t req_operation_len, int64_t req_sequence_id, const uint8_t* req_sig,
                                        uint64_t req_sig_len, int req_sig_nil, const uint8_t* sig, uint64_t sig_len,
                                        int sig_nil, uint8_t* out, uint64_t cap);
uint64_t pbftv_gojson_reply(int64_t view_id, int64_t timestamp, const char* client_id, uint64_t client_id_len,
                            const char* node_id, uint64_t node_id_len, const char* result, uint64_t result_len,
                            uint8_t* out, uint64_t cap);
uint64_t pbftv_gojson_preprepare(int64_t view_id, int64_t sequence_id, const char* digest, uint64_t digest_len,
                                 int has_request, int64_t req_timestamp, const char* req_client_id,
                                 uint64_t req_client_id_len, const char* req_operation, uint64_t req_operation_len,
                                 int64_t req_sequence_id, uint8_t* out, uint64_t cap);

/* ---- DER signatures (go1.19 crypto/ecdsa.VerifyASN1's cryptobyte parse) ---
 * SEQUENCE { INTEGER r, INTEGER s } with Go's DER strictness -> r||s (64 B
 * big-endian, the sig_rs layout of pbftv_ecdsa_p256_verify_batch).  Returns 1
 * when parsed with 0 <= r, s < 2^256, 0 when Go would reject it at the parse
 * or range check (out_rs zeroed, so the verify yields a 0 bit), PBFTV_EINVAL
 * on null pointers.  The batch form returns the number parsed (or < 0). */
int pbftv_ecdsa_der_to_rs(const uint8_t* der, uint64_t der_len, uint8_t* out_rs);
int64_t pbftv_ecdsa_der_to_rs_batch(const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths,
                                    uint64_t n, uint8_t* out_rs);

/* digest(*RequestMsg) for n requests (pbft_impl.go:235-243, called from
 * StartConsensus :73 and verifyMsg :190): the struct fields are shipped
 * column-wise, the Go-JSON preimages are built on the GPU (one lane per
 * message, same encoder as pbftv_gojson_*) and hashed there.  client_ids /
 * operations are concatenated byte strings with per-item offsets/lengths.
 * out_digests: n*32 raw bytes. */
int pbftv_digest_request_batch(pbftv_ctx* ctx, uint64_t n, const int64_t* timestamps, const uint8_t* client_ids,
                               const uint64_t* client_id_off, const uint32_t* client_id_len, const uint8_t* operations,
                               const uint64_t* operation_off, const uint32_t* operation_len,
                               const int64_t* sequence_ids, uint8_t* out_digests);

/* digest(*VoteMsg) / digest(*ReplyMsg) / digest(*PrePrepareMsg) for n
 * messages (the signed preimages of votes, replies and pre-prepares): Go-JSON
 * built on the GPU, hashed there.  For pre-prepares, has_request[i] = 0 encodes
 * requestMsg as null (the req_* columns must still hold n entries). */
int pbftv_digest_vote_batch(pbftv_ctx* ctx, uint64_t n, const int64_t* view_ids, const int64_t* sequence_ids,
                            const uint8_t* digests, const uint64_t* digest_off, const uint32_t* digest_len,
                            const uint8_t* node_ids, const uint64_t* node_id_off, const uint32_t* node_id_len,
                            const int64_t* msg_types, uint8_t* out_digests);
int pbftv_digest_reply_batch(pbftv_ctx* ctx, uint64_t n, const int64_t* view_ids, const int64_t* timestamps,
                             const uint8_t* client_ids, const uint64_t* client_id_off, const uint32_t* client_id_len,
                             const uint8_t* node_ids, const uint64_t* node_id_off, const uint32_t* node_id_len,
                             const uint8_t* results, const uint64_t* result_off, const uint32_t* result_len,
                             uint8_t* out_digests);
int pbftv_digest_preprepare_batch(pbftv_ctx* ctx, uint64_t n, const int64_t* view_ids, const int64_t* sequence_ids,
                                  const uint8_t* digests, const uint64_t* digest_off, const uint32_t* digest_len,
                                  const uint8_t* has_request, const int64_t* req_timestamps,
                                  const uint8_t* req_client_ids, const uint64_t* req_client_id_off,
                                  const uint32_t* req_client_id_len, const uint8_t* req_operations,
                                  const uint64_t* req_operation_off, const uint32_t* req_operation_len,
                                  const int64_t* req_sequence_ids, uint8_t* out_digests);

/* Pool flush of a snapshot of prepare/commit votes (GetAllPrepareMsg /
 * GetAllCommitMsg, pool/preparePool.go:56-67, pool/commitPool.go:57-68, as
 * drained by resolvePrepareMsg / resolveCommitMsg, pbft/network/node.go:559-598)
 * across any number of consensus states, in one GPU round trip per device:
 *   h_i        = SHA-256(Go-JSON(VoteMsg i))                 -> out_digests (n*32, optional)
 *   sig bit i  = crypto/ecdsa.Verify(key[key_idx[i]], h_i, r_i, s_i)
 *                                                            -> out_sig_bitmap (optional;
 *                                                               needs sig_rs n*64 BE, key_idx)
 *   msg bit i  = State.verifyMsg(view_ids[i], sequence_ids[i], digest_i) against the
 *                state state_idx[i] < n_states = (state_view_ids, state_last_seqs,
 *                32-B request digest)                        -> out_msg_bitmap (optional)
 * (pbft_impl.go:176-202; a state_idx out of range gives 0).  Bitmaps are
 * ceil(n/8) bytes, LSB-first.  A vote counts toward its state's quorum iff both
 * bits are set. */
int pbftv_flush_votes(pbftv_ctx* ctx, uint64_t n, const int64_t* view_ids, const int64_t* sequence_ids,
                      const uint8_t* digests, const uint64_t* digest_off, const uint32_t* digest_len,
                      const uint8_t* node_ids, const uint64_t* node_id_off, const uint32_t* node_id_len,
                      const int64_t* msg_types, const uint8_t* sig_rs, const uint32_t* key_idx, uint32_t n_states,
                      const int64_t* state_view_ids, const int64_t* state_last_seqs,
                      const uint8_t* state_req_digests, const uint32_t* state_idx, uint8_t* out_digests,
                      uint8_t* out_sig_bitmap, uint8_t* out_msg_bitmap);

/* Flushes of the other three signed messages, one GPU round
 * trip per device like pbftv_flush_votes; every output is optional (NULL = not
 * wanted; a signature bitmap needs sig_rs n*64 BE and key_idx).
 *
 * Requests (GetReq / resolveRequestMsg, pbft/network/node.go:150-177, 521-538):
 *   h_i = SHA-256(Go-JSON(RequestMsg i with sequence_ids[i]))  -> out_digests
 *   sig bit i = ecdsa.Verify(key[key_idx[i]], h_i, r_i, s_i)  -> out_sig_bitmap
 *   c_i = digest(RequestMsg i with SequenceID = assigned_seqs[i]), the
 *         StartConsensus digest (pbft_impl.go:67-73)          -> out_consensus_digests
 *                                                                (needs assigned_seqs) */
int pbftv_flush_requests(pbftv_ctx* ctx, uint64_t n, const int64_t* timestamps, const uint8_t* client_ids,
                         const uint64_t* client_id_off, const uint32_t* client_id_len, const uint8_t* operations,
                         const uint64_t* operation_off, const uint32_t* operation_len, const int64_t* sequence_ids,
                         const uint8_t* sig_rs, const uint32_t* key_idx, const int64_t* assigned_seqs,
                         uint8_t* out_digests, uint8_t* out_sig_bitmap, uint8_t* out_consensus_digests);
/* Replies (the client's reply collection, node.go:182-197 / client):
 *   h_i = SHA-256(Go-JSON(ReplyMsg i)) -> out_digests; sig bit i as above. */
int pbftv_flush_replies(pbftv_ctx* ctx, uint64_t n, const int64_t* view_ids, const int64_t* timestamps,
                        const uint8_t* client_ids, const uint64_t* client_id_off, const uint32_t* client_id_len,
                        const uint8_t* node_ids, const uint64_t* node_id_off, const uint32_t* node_id_len,
                        const uint8_t* results, const uint64_t* result_off, const uint32_t* result_len,
                        const uint8_t* sig_rs, const uint32_t* key_idx, uint8_t* out_digests,
                        uint8_t* out_sig_bitmap);
/* Pre-prepares (replicas, State.PrePrepare pbft_impl.go:91-109):
 *   h_i = SHA-256(Go-JSON(PrePrepareMsg i))                     -> out_digests; sig bit i
 *   q_i = digest(embedded RequestMsg i) (Hash("null") if nil)   -> out_req_digests
 *   msg bit i = verifyMsg(view_ids[i], sequence_ids[i], digest_i) with the state's
 *               ReqMsg = the embedded request: view == state_view_ids[state_idx[i]]
 *               && (last == -1 || last < sequence_ids[i]) && digest_i == hex(q_i)
 *                                                               -> out_msg_bitmap
 * (state_idx out of range -> 0). */
int pbftv_flush_preprepares(pbftv_ctx* ctx, uint64_t n, const int64_t* view_ids, const int64_t* sequence_ids,
                            const uint8_t* digests, const uint64_t* digest_off, const uint32_t* digest_len,
                            const uint8_t* has_request, const int64_t* req_timestamps, const uint8_t* req_client_ids,
                            const uint64_t* req_client_id_off, const uint32_t* req_client_id_len,
                            const uint8_t* req_operations, const uint64_t* req_operation_off,
                            const uint32_t* req_operation_len, const int64_t* req_sequence_ids, const uint8_t* sig_rs,
                            const uint32_t* key_idx, uint32_t n_states, const int64_t* state_view_ids,
                            const int64_t* state_last_seqs, const uint32_t* state_idx, uint8_t* out_digests,
                            uint8_t* out_req_digests, uint8_t* out_sig_bitmap, uint8_t* out_msg_bitmap);

/* State.verifyMsg (pbft_impl.go:176-202) over n votes against one state:
 * bit i = view_ids[i] == state_view_id
 *         && (state_last_seq == -1 || state_last_seq < sequence_ids[i])
 *         && digest_got[i] (digest_got_len[i] bytes at digest_got + digest_got_off[i])
 *            is exactly the lowercase hex of req_digest (Go string compare). */
int pbftv_verify_msg_batch(int64_t state_view_id, int64_t state_last_seq, const uint8_t req_digest[32], uint64_t n,
                           const int64_t* view_ids, const int64_t* sequence_ids, const char* digest_got,
                           const uint64_t* digest_got_off, const uint32_t* digest_got_len, uint8_t* out_bitmap);

/* ---- ECDSA-P256 signatures (Go crypto/ecdsa.Verify semantics) --------- */

/* Register the replica public keys (k * 64 B, X||Y big-endian); replaces any
 * previous set.  out_valid[j] = 1 if key j is a valid P-256 point (0 <= X,Y < p
 * and on the curve); signatures naming an invalid key always fail.  Builds the
 * fixed-base comb tables on every device (one host thread per GPU).  The G
 * table is built once per GPU and width and shared by every context of the
 * process on that GPU; the key tables of one call share one allocation, and a
 * re-registration at the same width reuses it (no VRAM re-allocation).
 * Geometry: see pbftv_table_config. */
int pbftv_register_keys(pbftv_ctx* ctx, const uint8_t* pub_xy, uint32_t k, uint8_t* out_valid);

/* Incremental key changes (membership changes without a rebuild of every
 * table): pbftv_add_keys appends k keys as indices nkeys .. nkeys + k - 1 at the
 * registered geometry (PBFTV_ENOMEM if their tables do not fit);
 * pbftv_set_key replaces key `index` (< nkeys) in place.  Both need a prior
 * pbftv_register_keys.  They, and pbftv_register_keys, first wait for every
 * verify of THIS context still in flight -- on the library's streams, on
 * streams from pbftv_stream_create and on any other caller stream a *_dev
 * call was given -- so no verify reads a table, validity flag or table
 * pointer while it is rewritten.  Other contexts on the GPU are not waited
 * for (they read their own key tables).  If any device
 * fails, every device of the context drops its key set (PBFTV_ENOKEYS until
 * the next successful pbftv_register_keys), so shards never disagree on the
 * keys. */
int pbftv_add_keys(pbftv_ctx* ctx, const uint8_t* pub_xy, uint32_t k, uint8_t* out_valid);
int pbftv_set_key(pbftv_ctx* ctx, uint32_t index, const uint8_t* pub_xy, uint8_t* out_valid);

/* Comb-table geometry chosen at registration and the HBM its tables take per
 * device.  Window codes: plain W-bit windows (8, 12, 16, 20, 22, 24, 26: 256/W + 1
 * windows, 2^(W-1) entries of 64 B each) or the mixed codes 21 (5 x 22-bit +
 * 7 x 21-bit windows: 1.14 GB per key) and 29 (5 x 29 + 4 x 28: 120 GB).  The
 * pair (G, keys) is the one with the fewest windows in total (= table
 * additions per verify) whose tables fit the device's free HBM minus a 16 GiB
 * reserve for batch scratch: on a 288 GB MI355X, 100 keys -> G 29 + keys 21
 * (9 + 12 windows, 234 GB), 4 keys -> G 29 + keys 24 (5.9 GB each), 1000 keys
 * -> keys 16 (34 MiB each).  PBFTV_TABLE_BUDGET_MB caps the key tables,
 * PBFTV_GBITS / PBFTV_QBITS force a width. */
int pbftv_table_config(const pbftv_ctx* ctx, int* out_gbits, int* out_qbits, uint64_t* out_table_bytes);

/* Verify n signatures: hashes (n*32), sig_rs (n*64: r||s big-endian),
 * key_idx (n, index into the registered table).  out_bitmap: ceil(n/8) B.
 * Batches up to 2048 signatures take the one-launch latency path (inputs read
 * by the kernel straight from pinned memory).  Larger batches are split into
 * one shard per device and each shard is pipelined in chunks: DMA of the
 * caller's buffers as they are (pinned memory, e.g. from pbftv_host_alloc,
 * directly; pageable memory through the runtime's staging) on one copy
 * stream -- every key index first, then each chunk's hashes and signatures
 * back to back into up to PBFTV_HOST_SLOTS = 16 device slots -- and each chunk
 * verified as it lands, even and odd chunks on two streams so the last two
 * overlap (PBFTV_HOST_CHUNK, default 262144 signatures; the last chunk
 * PBFTV_HOST_LAST, default 131072, takes the ragged remainder). */
int pbftv_ecdsa_p256_verify_batch(pbftv_ctx* ctx, const uint8_t* hashes, const uint8_t* sig_rs,
                                  const uint32_t* key_idx, uint64_t n, uint8_t* out_bitmap);

/* Device-resident form (device index dev); hashes/sigs 16-B aligned;
 * d_bitmap: ceil(n/8) B.  Enqueued on stream, not synchronised. */
int pbftv_ecdsa_p256_verify_batch_dev(pbftv_ctx* ctx, int dev, const uint8_t* d_hashes, const uint8_t* d_sig_rs,
                                      const uint32_t* d_key_idx, uint64_t n, uint8_t* d_bitmap, void* stream);

/* Quorum certificate: verify n signatures and count acceptances.
 * *out_accepted = popcount; *out_quorum = (*out_accepted >= quorum).  With
 * quorum = 2f this is the reference's prepared()/committed() count
 * (pbft_impl.go:212,227); with 2f+1 it is a PBFT certificate. */
int pbftv_qc_verify(pbftv_ctx* ctx, const uint8_t* hashes, const uint8_t* sig_rs, const uint32_t* key_idx, uint64_t n,
                    uint32_t quorum, uint8_t* out_bitmap, uint64_t* out_accepted, int* out_quorum);

#ifdef __cplusplus
}
#endif
#endif /* PBFTV_H */
