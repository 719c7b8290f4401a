// gojson_kernels.hip -- Go-JSON preimages of the reference's messages, built on
// the device.
//
// digest() (pbft/consensus/pbft_impl.go:235-243) hashes json.Marshal(msg); the
// signature preimages of the build-added signatures are the same encodings.
// Instead of marshalling every message on the host, the host ships the struct
// fields column-wise (int64 arrays, string blobs + offsets + lengths) and one
// lane per message writes its exact Go-JSON bytes (gojson_enc.h, the encoder
// the host path uses too) into its own slot of a preimage buffer; k_sha256
// then hashes the slots.  Slot i is at slot[i] and holds at most the encoder's
// bound for the message's field lengths (computed on the host, which has them).
//
// The vote encoder also evaluates State.verifyMsg (pbft_impl.go:176-202) for
// the state each vote is addressed to -- the digest string is already in the
// lane's hands -- so a pool flush needs no second pass over the votes.
#include <hip/hip_runtime.h>

#include "gojson_enc.h"
#include "kernels.h"

namespace pbftv {

namespace {

// byte sink into global memory (the lane's own slot)
struct DevSink {
  uint8_t* p;
  uint32_t n;
  __device__ void put(uint8_t b) { p[n++] = b; }
  __device__ uint8_t* grow(uint32_t k) {
    uint8_t* r = p + n;
    n += k;
    return r;
  }
};

__device__ __forceinline__ const uint8_t* str(const StrCol& c, uint64_t i) { return c.data + c.off[i]; }

// Go string compare of digestGot with the lowercase hex of the 32-byte request
// digest (pbft_impl.go:197): equal length 64 and equal bytes
__device__ bool hex_equals(const uint8_t* got, uint32_t got_len, const uint8_t* want32) {
  if (got_len != 64) return false;
  bool eq = true;
  for (int k = 0; k < 32; ++k) {
    const uint8_t w = want32[k];
    eq &= got[2 * k] == (uint8_t)gojson::hex_lower(w >> 4);
    eq &= got[2 * k + 1] == (uint8_t)gojson::hex_lower(w & 15);
  }
  return eq;
}

}  // namespace

__global__ void __launch_bounds__(256) k_gojson_request(RequestCols c, uint64_t n, const uint64_t* __restrict__ slot,
                                                        uint8_t* __restrict__ out, uint32_t* __restrict__ out_len) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DevSink o{out + slot[i], 0};
  gojson::request(o, c.ts[i], str(c.cid, i), c.cid.len[i], str(c.op, i), c.op.len[i], c.seq[i]);
  out_len[i] = o.n;
}

__global__ void __launch_bounds__(256) k_gojson_vote(VoteCols c, uint64_t n, const uint64_t* __restrict__ slot,
                                                     uint8_t* __restrict__ out, uint32_t* __restrict__ out_len,
                                                     StateCols s, uint8_t* __restrict__ msg_ok) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t view = c.view[i], seq = c.seq[i];
  const uint8_t* dg = str(c.digest, i);
  const uint32_t dgn = c.digest.len[i];
  DevSink o{out + slot[i], 0};
  gojson::vote(o, view, seq, dg, dgn, str(c.node, i), c.node.len[i], c.type[i]);
  out_len[i] = o.n;
  if (msg_ok) {
    const uint32_t st = s.idx[i];
    bool ok = st < s.n;
    if (ok) {
      const int64_t last = s.last_seq[st];
      ok = view == s.view[st]                   // pbft_impl.go:178
           && (last == -1 || last < seq)        // pbft_impl.go:184-188
           && hex_equals(dg, dgn, s.req_digest + 32ull * st);  // pbft_impl.go:190-199
    }
    msg_ok[i] = ok ? 1 : 0;
  }
}

__global__ void __launch_bounds__(256) k_gojson_reply(ReplyCols c, uint64_t n, const uint64_t* __restrict__ slot,
                                                      uint8_t* __restrict__ out, uint32_t* __restrict__ out_len) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DevSink o{out + slot[i], 0};
  gojson::reply(o, c.view[i], c.ts[i], str(c.cid, i), c.cid.len[i], str(c.node, i), c.node.len[i],
                str(c.result, i), c.result.len[i]);
  out_len[i] = o.n;
}

__global__ void __launch_bounds__(256) k_gojson_preprepare(PrePrepareCols c, uint64_t n,
                                                           const uint64_t* __restrict__ slot, uint8_t* __restrict__ out,
                                                           uint32_t* __restrict__ out_len) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DevSink o{out + slot[i], 0};
  const bool has = c.has_req[i] != 0;
  gojson::preprepare(o, c.view[i], c.seq[i], str(c.digest, i), c.digest.len[i], has, has ? c.req.ts[i] : 0,
                     str(c.req.cid, i), has ? c.req.cid.len[i] : 0, str(c.req.op, i), has ? c.req.op.len[i] : 0,
                     has ? c.req.seq[i] : 0);
  out_len[i] = o.n;
}

// Pre-prepare flush: message i's preimage at slot[i] (signed by the primary)
// and its embedded request's digest preimage at slot[n + i] ("null" for a nil
// request, pbft_impl.go:93,190).
__global__ void __launch_bounds__(256) k_gojson_preprepare_pair(PrePrepareCols c, uint64_t n,
                                                                const uint64_t* __restrict__ slot,
                                                                uint8_t* __restrict__ out,
                                                                uint32_t* __restrict__ out_len) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool has = c.has_req[i] != 0;
  const int64_t rts = has ? c.req.ts[i] : 0, rseq = has ? c.req.seq[i] : 0;
  const uint32_t rcn = has ? c.req.cid.len[i] : 0, ron = has ? c.req.op.len[i] : 0;
  DevSink o{out + slot[i], 0};
  gojson::preprepare(o, c.view[i], c.seq[i], str(c.digest, i), c.digest.len[i], has, rts, str(c.req.cid, i), rcn,
                     str(c.req.op, i), ron, rseq);
  out_len[i] = o.n;
  DevSink q{out + slot[n + i], 0};
  gojson::request_or_null(q, has, rts, str(c.req.cid, i), rcn, str(c.req.op, i), ron, rseq);
  out_len[n + i] = q.n;
}

// State.verifyMsg of pre-prepare i (PrePrepare, pbft_impl.go:91-97): the
// replica's state takes the embedded request as its ReqMsg, so the digest
// field is compared with the digest of that request (req_digests, 32 B each).
__global__ void __launch_bounds__(256) k_preprepare_verify(const int64_t* __restrict__ view,
                                                           const int64_t* __restrict__ seq, StrCol digest,
                                                           const uint8_t* __restrict__ req_digests, StateCols s,
                                                           uint64_t n, uint8_t* __restrict__ msg_ok) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t st = s.idx[i];
  bool ok = st < s.n;
  if (ok) {
    const int64_t last = s.last_seq[st];
    ok = view[i] == s.view[st] && (last == -1 || last < seq[i]) &&
         hex_equals(str(digest, i), digest.len[i], req_digests + 32 * i);
  }
  msg_ok[i] = ok ? 1 : 0;
}

static inline dim3 grid_for(uint64_t n) { return dim3((uint32_t)((n + 255) / 256)); }

hipError_t launch_gojson_request(const RequestCols& c, uint64_t n, const uint64_t* slot, uint8_t* out,
                                 uint32_t* out_len, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gojson_request, grid_for(n), dim3(256), 0, st, c, n, slot, out, out_len);
  return hipGetLastError();
}

hipError_t launch_gojson_vote(const VoteCols& c, uint64_t n, const uint64_t* slot, uint8_t* out, uint32_t* out_len,
                              const StateCols& s, uint8_t* msg_ok, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gojson_vote, grid_for(n), dim3(256), 0, st, c, n, slot, out, out_len, s, msg_ok);
  return hipGetLastError();
}

hipError_t launch_gojson_reply(const ReplyCols& c, uint64_t n, const uint64_t* slot, uint8_t* out, uint32_t* out_len,
                               hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gojson_reply, grid_for(n), dim3(256), 0, st, c, n, slot, out, out_len);
  return hipGetLastError();
}

hipError_t launch_gojson_preprepare(const PrePrepareCols& c, uint64_t n, const uint64_t* slot, uint8_t* out,
                                    uint32_t* out_len, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gojson_preprepare, grid_for(n), dim3(256), 0, st, c, n, slot, out, out_len);
  return hipGetLastError();
}

hipError_t launch_gojson_preprepare_pair(const PrePrepareCols& c, uint64_t n, const uint64_t* slot, uint8_t* out,
                                         uint32_t* out_len, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gojson_preprepare_pair, grid_for(n), dim3(256), 0, st, c, n, slot, out, out_len);
  return hipGetLastError();
}

hipError_t launch_preprepare_verify(const int64_t* view, const int64_t* seq, const StrCol& digest,
                                   const uint8_t* req_digests, const StateCols& s, uint64_t n, uint8_t* msg_ok,
                                   hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_preprepare_verify, grid_for(n), dim3(256), 0, st, view, seq, digest, req_digests, s, n,
                     msg_ok);
  return hipGetLastError();
}

}  // namespace pbftv
