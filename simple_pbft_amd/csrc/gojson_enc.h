// gojson_enc.h -- Go 1.19 encoding/json.Marshal of the reference's message
// structs, written once for the host (gojson.cpp) and the gfx950 encoder
// kernels (gojson_kernels.hip).
//
// Restates, byte for byte:
//   pbft/consensus/pbft_msg_types.go:3-38  field order and tags; the embedded
//                                          MsgType encodes as "msgType":<int>
//   encoding/json (go1.19) encodeState.string(escapeHTML=true):
//     '"' '\\' -> \" \\ ; '\n' '\r' '\t' -> \n \r \t ; other bytes < 0x20 and
//     '<' '>' '&' -> \u00XX (lowercase hex); each byte of an invalid UTF-8
//     sequence -> \ufffd (utf8.DecodeRuneInString rules: no overlongs, no
//     surrogates, nothing above U+10FFFF); U+2028 / U+2029 -> \u2028 / \u2029;
//     every other byte is copied
//   strconv.AppendInt(.., 10) for int64 fields; compact output, no newline.
//
// A Sink is anything with  void put(uint8_t)  and  uint8_t* grow(uint32_t k)
// (append k bytes, return where they start).  Output bound (used by the
// device encoder to place each message in its own slot): a string of n bytes
// encodes to at most 6n + 2 bytes, an int64 to at most 20.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define PBFTV_GJ __host__ __device__ __forceinline__
#else
#define PBFTV_GJ inline
#endif

namespace pbftv {
namespace gojson {

PBFTV_GJ char hex_lower(uint32_t v) { return (char)(v < 10 ? '0' + v : 'a' + (v - 10)); }

template <class S>
PBFTV_GJ void lit(S& o, const char* s) {
  while (*s) o.put((uint8_t)*s++);
}

template <class S>
PBFTV_GJ void put_int(S& o, int64_t v) {
  uint64_t u = v < 0 ? 0 - (uint64_t)v : (uint64_t)v;
  uint32_t nd = 1;
  for (uint64_t p = 10; nd < 20 && u >= p; p *= 10) ++nd;  // 10^19 < 2^64: nd reaches 20 only past it
  uint8_t* w = o.grow(nd + (v < 0 ? 1u : 0u));
  if (v < 0) *w++ = '-';
  for (uint32_t k = nd; k-- > 0;) {
    w[k] = (uint8_t)('0' + (uint32_t)(u % 10));
    u /= 10;
  }
}

PBFTV_GJ bool utf8_cont(uint8_t b) { return (b & 0xC0) == 0x80; }

// length of the valid UTF-8 sequence starting at s[0] (b0 >= 0x80), 0 if
// invalid; *rune set for 2- and 3-byte sequences (4-byte ones are never U+2028/9)
PBFTV_GJ uint32_t utf8_len(const uint8_t* s, uint64_t rem, uint32_t* rune) {
  const uint8_t b0 = s[0];
  if (b0 >= 0xC2 && b0 <= 0xDF) {
    if (rem < 2 || !utf8_cont(s[1])) return 0;
    *rune = ((uint32_t)(b0 & 0x1F) << 6) | (s[1] & 0x3F);
    return 2;
  }
  if (b0 >= 0xE0 && b0 <= 0xEF) {
    const uint8_t lo = b0 == 0xE0 ? 0xA0 : 0x80, hi = b0 == 0xED ? 0x9F : 0xBF;
    if (rem < 3 || s[1] < lo || s[1] > hi || !utf8_cont(s[2])) return 0;
    *rune = ((uint32_t)(b0 & 0x0F) << 12) | ((uint32_t)(s[1] & 0x3F) << 6) | (s[2] & 0x3F);
    return 3;
  }
  if (b0 >= 0xF0 && b0 <= 0xF4) {
    const uint8_t lo = b0 == 0xF0 ? 0x90 : 0x80, hi = b0 == 0xF4 ? 0x8F : 0xBF;
    if (rem < 4 || s[1] < lo || s[1] > hi || !utf8_cont(s[2]) || !utf8_cont(s[3])) return 0;
    *rune = 0x10000;
    return 4;
  }
  return 0;  // continuation byte, C0/C1, F5..FF
}

template <class S>
PBFTV_GJ void put_string(S& o, const uint8_t* s, uint64_t n) {
  o.put('"');
  uint64_t i = 0;
  while (i < n) {
    const uint8_t b = s[i];
    if (b < 0x80) {
      ++i;
      if (b >= 0x20 && b != '"' && b != '\\' && b != '<' && b != '>' && b != '&') {
        o.put(b);
      } else if (b == '"' || b == '\\') {
        o.put('\\');
        o.put(b);
      } else if (b == '\n' || b == '\r' || b == '\t') {
        o.put('\\');
        o.put(b == '\n' ? 'n' : (b == '\r' ? 'r' : 't'));
      } else {
        uint8_t* w = o.grow(6);
        w[0] = '\\'; w[1] = 'u'; w[2] = '0'; w[3] = '0';
        w[4] = (uint8_t)hex_lower(b >> 4);
        w[5] = (uint8_t)hex_lower(b & 15);
      }
      continue;
    }
    uint32_t rune = 0;
    const uint32_t len = utf8_len(s + i, n - i, &rune);
    if (len == 0) {  // utf8.RuneError, width 1
      lit(o, "\\ufffd");
      ++i;
    } else if (rune == 0x2028 || rune == 0x2029) {
      lit(o, "\\u202");
      o.put((uint8_t)hex_lower(rune & 15));
      i += len;
    } else {
      for (uint32_t k = 0; k < len; ++k) o.put(s[i + k]);
      i += len;
    }
  }
  o.put('"');
}

// RequestMsg (pbft_msg_types.go:3-8)
template <class S>
PBFTV_GJ void request(S& o, int64_t ts, const uint8_t* cid, uint64_t cidn, const uint8_t* op, uint64_t opn,
                      int64_t seq) {
  lit(o, "{\"timestamp\":");
  put_int(o, ts);
  lit(o, ",\"clientID\":");
  put_string(o, cid, cidn);
  lit(o, ",\"operation\":");
  put_string(o, op, opn);
  lit(o, ",\"sequenceID\":");
  put_int(o, seq);
  o.put('}');
}
PBFTV_GJ uint64_t request_bound(uint64_t cidn, uint64_t opn) { return 97 + 6 * (cidn + opn); }

// VoteMsg (pbft_msg_types.go:25-31)
template <class S>
PBFTV_GJ void vote(S& o, int64_t view, int64_t seq, const uint8_t* dg, uint64_t dgn, const uint8_t* nid,
                   uint64_t nidn, int64_t mt) {
  lit(o, "{\"viewID\":");
  put_int(o, view);
  lit(o, ",\"sequenceID\":");
  put_int(o, seq);
  lit(o, ",\"digest\":");
  put_string(o, dg, dgn);
  lit(o, ",\"nodeID\":");
  put_string(o, nid, nidn);
  lit(o, ",\"msgType\":");
  put_int(o, mt);
  o.put('}');
}
PBFTV_GJ uint64_t vote_bound(uint64_t dgn, uint64_t nidn) { return 120 + 6 * (dgn + nidn); }

// []byte field (encoding/json encodeByteSlice, go1.19): nil -> null, otherwise
// a quoted base64.StdEncoding string (padded, no line breaks)
template <class S>
PBFTV_GJ void put_bytes(S& o, const uint8_t* b, uint64_t n, bool is_nil) {
  if (is_nil) {
    lit(o, "null");
    return;
  }
  const char* A = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  o.put('"');
  uint64_t i = 0;
  for (; i + 3 <= n; i += 3) {
    const uint32_t v = ((uint32_t)b[i] << 16) | ((uint32_t)b[i + 1] << 8) | b[i + 2];
    uint8_t* w = o.grow(4);
    w[0] = (uint8_t)A[v >> 18]; w[1] = (uint8_t)A[(v >> 12) & 63]; w[2] = (uint8_t)A[(v >> 6) & 63]; w[3] = (uint8_t)A[v & 63];
  }
  if (n - i == 1) {
    const uint32_t v = (uint32_t)b[i] << 16;
    uint8_t* w = o.grow(4);
    w[0] = (uint8_t)A[v >> 18]; w[1] = (uint8_t)A[(v >> 12) & 63]; w[2] = '='; w[3] = '=';
  } else if (n - i == 2) {
    const uint32_t v = ((uint32_t)b[i] << 16) | ((uint32_t)b[i + 1] << 8);
    uint8_t* w = o.grow(4);
    w[0] = (uint8_t)A[v >> 18]; w[1] = (uint8_t)A[(v >> 12) & 63]; w[2] = (uint8_t)A[(v >> 6) & 63]; w[3] = '=';
  }
  o.put('"');
}

// Signed messages on the wire (build-added): each struct of
// pbft_msg_types.go:3-31 followed by  Signature []byte `json:"signature"`.  The
// signing preimage of every message is its unsigned encoding (vote(),
// request(), reply(), preprepare() here), i.e. the wire form up to the
// signature field.
struct SigField {
  const uint8_t* p;
  uint64_t n;
  bool nil;
};

template <class S>
PBFTV_GJ void put_sig_field(S& o, const SigField& s) {
  lit(o, ",\"signature\":");
  put_bytes(o, s.p, s.n, s.nil);
  o.put('}');
}

template <class S>
PBFTV_GJ void vote_signed(S& o, int64_t view, int64_t seq, const uint8_t* dg, uint64_t dgn, const uint8_t* nid,
                          uint64_t nidn, int64_t mt, const uint8_t* sig, uint64_t sign, bool sig_nil) {
  lit(o, "{\"viewID\":");
  put_int(o, view);
  lit(o, ",\"sequenceID\":");
  put_int(o, seq);
  lit(o, ",\"digest\":");
  put_string(o, dg, dgn);
  lit(o, ",\"nodeID\":");
  put_string(o, nid, nidn);
  lit(o, ",\"msgType\":");
  put_int(o, mt);
  put_sig_field(o, SigField{sig, sign, sig_nil});
}

// ReplyMsg (pbft_msg_types.go:10-16)
template <class S>
PBFTV_GJ void reply(S& o, int64_t view, int64_t ts, const uint8_t* cid, uint64_t cidn, const uint8_t* nid,
                    uint64_t nidn, const uint8_t* res, uint64_t resn) {
  lit(o, "{\"viewID\":");
  put_int(o, view);
  lit(o, ",\"timestamp\":");
  put_int(o, ts);
  lit(o, ",\"clientID\":");
  put_string(o, cid, cidn);
  lit(o, ",\"nodeID\":");
  put_string(o, nid, nidn);
  lit(o, ",\"result\":");
  put_string(o, res, resn);
  o.put('}');
}
PBFTV_GJ uint64_t reply_bound(uint64_t cidn, uint64_t nidn, uint64_t resn) { return 102 + 6 * (cidn + nidn + resn); }

// PrePrepareMsg (pbft_msg_types.go:18-23); a nil *RequestMsg encodes as null
template <class S>
PBFTV_GJ void preprepare(S& o, int64_t view, int64_t seq, const uint8_t* dg, uint64_t dgn, bool has_req,
                         int64_t rts, const uint8_t* rcid, uint64_t rcidn, const uint8_t* rop, uint64_t ropn,
                         int64_t rseq) {
  lit(o, "{\"viewID\":");
  put_int(o, view);
  lit(o, ",\"sequenceID\":");
  put_int(o, seq);
  lit(o, ",\"digest\":");
  put_string(o, dg, dgn);
  lit(o, ",\"requestMsg\":");
  if (has_req) request(o, rts, rcid, rcidn, rop, ropn, rseq);
  else lit(o, "null");
  o.put('}');
}
PBFTV_GJ uint64_t preprepare_bound(uint64_t dgn, uint64_t rcidn, uint64_t ropn) {
  return 92 + 6 * dgn + request_bound(rcidn, ropn);
}

// digest(*RequestMsg) preimage for a possibly nil request: json.Marshal of a
// nil pointer is "null" (pbft_impl.go:190 hashes state.MsgLogs.ReqMsg, which a
// pre-prepare with requestMsg null leaves nil)
template <class S>
PBFTV_GJ void request_or_null(S& o, bool has, int64_t ts, const uint8_t* cid, uint64_t cidn, const uint8_t* op,
                              uint64_t opn, int64_t seq) {
  if (has) request(o, ts, cid, cidn, op, opn, seq);
  else lit(o, "null");
}

// signed RequestMsg: the client's signature over request() as the client sent
// it (sequenceID as given; the reference's clients leave it 0,
// pbft_msg_types.go:7 and StartConsensus pbft_impl.go:67 assigns it later)
template <class S>
PBFTV_GJ void request_signed(S& o, int64_t ts, const uint8_t* cid, uint64_t cidn, const uint8_t* op, uint64_t opn,
                             int64_t seq, const SigField& sig) {
  lit(o, "{\"timestamp\":");
  put_int(o, ts);
  lit(o, ",\"clientID\":");
  put_string(o, cid, cidn);
  lit(o, ",\"operation\":");
  put_string(o, op, opn);
  lit(o, ",\"sequenceID\":");
  put_int(o, seq);
  put_sig_field(o, sig);
}

// signed ReplyMsg (the replying node's signature over reply())
template <class S>
PBFTV_GJ void reply_signed(S& o, int64_t view, int64_t ts, const uint8_t* cid, uint64_t cidn, const uint8_t* nid,
                           uint64_t nidn, const uint8_t* res, uint64_t resn, const SigField& sig) {
  lit(o, "{\"viewID\":");
  put_int(o, view);
  lit(o, ",\"timestamp\":");
  put_int(o, ts);
  lit(o, ",\"clientID\":");
  put_string(o, cid, cidn);
  lit(o, ",\"nodeID\":");
  put_string(o, nid, nidn);
  lit(o, ",\"result\":");
  put_string(o, res, resn);
  put_sig_field(o, sig);
}

// signed PrePrepareMsg: the primary's signature over preprepare() (the
// embedded request unsigned: the digest field already commits to it); on the
// wire the embedded request carries the client's signature (request_signed)
template <class S>
PBFTV_GJ void preprepare_signed(S& o, int64_t view, int64_t seq, const uint8_t* dg, uint64_t dgn, bool has_req,
                                int64_t rts, const uint8_t* rcid, uint64_t rcidn, const uint8_t* rop, uint64_t ropn,
                                int64_t rseq, const SigField& req_sig, const SigField& sig) {
  lit(o, "{\"viewID\":");
  put_int(o, view);
  lit(o, ",\"sequenceID\":");
  put_int(o, seq);
  lit(o, ",\"digest\":");
  put_string(o, dg, dgn);
  lit(o, ",\"requestMsg\":");
  if (has_req) request_signed(o, rts, rcid, rcidn, rop, ropn, rseq, req_sig);
  else lit(o, "null");
  put_sig_field(o, sig);
}

}  // namespace gojson
}  // namespace pbftv
