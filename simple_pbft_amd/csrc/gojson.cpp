// gojson.cpp -- see gojson.h.  The encoding itself is gojson_enc.h, shared with
// the device encoder kernels (gojson_kernels.hip); here its Sink appends to a
// std::vector.
#include "gojson.h"

#include "gojson_enc.h"

namespace pbftv {
namespace gojson {
namespace {

struct VecSink {
  std::vector<uint8_t>& v;
  void put(uint8_t b) { v.push_back(b); }
  uint8_t* grow(uint32_t k) {
    v.resize(v.size() + k);
    return v.data() + v.size() - k;
  }
};

}  // namespace

void append_string(std::vector<uint8_t>& o, const uint8_t* s, uint64_t n) {
  VecSink k{o};
  put_string(k, s, n);
}

void append_int(std::vector<uint8_t>& o, int64_t v) {
  VecSink k{o};
  put_int(k, v);
}

void append_request(std::vector<uint8_t>& o, int64_t ts, const uint8_t* cid, uint64_t cidn, const uint8_t* op,
                    uint64_t opn, int64_t seq) {
  VecSink k{o};
  request(k, ts, cid, cidn, op, opn, seq);
}

void append_vote(std::vector<uint8_t>& o, int64_t view, int64_t seq, const uint8_t* dg, uint64_t dgn,
                 const uint8_t* nid, uint64_t nidn, int64_t mt) {
  VecSink k{o};
  vote(k, view, seq, dg, dgn, nid, nidn, mt);
}

void append_vote_signed(std::vector<uint8_t>& o, int64_t view, int64_t seq, const uint8_t* dg, uint64_t dgn,
                        const uint8_t* nid, uint64_t nidn, int64_t mt, const uint8_t* sig, uint64_t sign,
                        bool sig_nil) {
  VecSink k{o};
  vote_signed(k, view, seq, dg, dgn, nid, nidn, mt, sig, sign, sig_nil);
}

void append_reply(std::vector<uint8_t>& o, int64_t view, int64_t ts, const uint8_t* cid, uint64_t cidn,
                  const uint8_t* nid, uint64_t nidn, const uint8_t* res, uint64_t resn) {
  VecSink k{o};
  reply(k, view, ts, cid, cidn, nid, nidn, res, resn);
}

void append_preprepare(std::vector<uint8_t>& o, int64_t view, int64_t seq, const uint8_t* dg, uint64_t dgn,
                       bool has_req, int64_t rts, const uint8_t* rcid, uint64_t rcidn, const uint8_t* rop,
                       uint64_t ropn, int64_t rseq) {
  VecSink k{o};
  preprepare(k, view, seq, dg, dgn, has_req, rts, rcid, rcidn, rop, ropn, rseq);
}

void append_request_signed(std::vector<uint8_t>& o, int64_t ts, const uint8_t* cid, uint64_t cidn, const uint8_t* op,
                           uint64_t opn, int64_t seq, const SigField& sig) {
  VecSink k{o};
  request_signed(k, ts, cid, cidn, op, opn, seq, sig);
}

void append_reply_signed(std::vector<uint8_t>& o, int64_t view, int64_t ts, const uint8_t* cid, uint64_t cidn,
                         const uint8_t* nid, uint64_t nidn, const uint8_t* res, uint64_t resn, const SigField& sig) {
  VecSink k{o};
  reply_signed(k, view, ts, cid, cidn, nid, nidn, res, resn, sig);
}

void append_preprepare_signed(std::vector<uint8_t>& o, int64_t view, int64_t seq, const uint8_t* dg, uint64_t dgn,
                              bool has_req, int64_t rts, const uint8_t* rcid, uint64_t rcidn, const uint8_t* rop,
                              uint64_t ropn, int64_t rseq, const SigField& req_sig, const SigField& sig) {
  VecSink k{o};
  preprepare_signed(k, view, seq, dg, dgn, has_req, rts, rcid, rcidn, rop, ropn, rseq, req_sig, sig);
}

}  // namespace gojson
}  // namespace pbftv
