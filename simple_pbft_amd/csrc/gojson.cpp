// gojson.cpp -- see gojson.h.  Table-driven: one 256-entry class table decides
// per byte whether it is copied, short-escaped, \u00XX-escaped, or starts a
// multi-byte UTF-8 sequence that must be validated like Go's
// utf8.DecodeRuneInString (invalid -> \\ufffd escape, U+2028/9 -> \\u2028 / \\u2029).
#include "gojson.h"

#include <cstring>

namespace pbftv {
namespace gojson {
namespace {

enum : uint8_t { kCopy = 0, kShort = 1, kU00 = 2, kLead2 = 3, kLead3 = 4, kLead4 = 5, kBad = 6 };

struct ClassTable {
  uint8_t c[256];
  char short_esc[128];
  constexpr ClassTable() : c(), short_esc() {
    for (int b = 0; b < 256; ++b) {
      uint8_t k = kCopy;
      if (b < 0x20) k = kU00;
      if (b == '<' || b == '>' || b == '&') k = kU00;          // escapeHTML
      if (b == '"' || b == '\\' || b == '\n' || b == '\r' || b == '\t') k = kShort;
      if (b >= 0x80) k = kBad;                                   // continuation / C0 / C1 / F5..FF
      if (b >= 0xC2 && b <= 0xDF) k = kLead2;
      if (b >= 0xE0 && b <= 0xEF) k = kLead3;
      if (b >= 0xF0 && b <= 0xF4) k = kLead4;
      c[b] = k;
    }
    short_esc['"'] = '"';
    short_esc['\\'] = '\\';
    short_esc['\n'] = 'n';
    short_esc['\r'] = 'r';
    short_esc['\t'] = 't';
  }
};

constexpr ClassTable kTab;
constexpr char kHex[] = "0123456789abcdef";

inline bool cont(uint8_t b) { return (b & 0xC0) == 0x80; }

// length of a valid UTF-8 sequence starting at s[i] (lead class given), 0 if invalid
inline int seq_len(const uint8_t* s, uint64_t n, uint64_t i, uint8_t cls, uint32_t* rune) {
  const uint64_t rem = n - i;
  const uint8_t b0 = s[i];
  if (cls == kLead2) {
    if (rem < 2 || !cont(s[i + 1])) return 0;
    *rune = ((uint32_t)(b0 & 0x1F) << 6) | (s[i + 1] & 0x3F);
    return 2;
  }
  if (cls == kLead3) {
    const uint8_t lo = b0 == 0xE0 ? 0xA0 : 0x80, hi = b0 == 0xED ? 0x9F : 0xBF;
    if (rem < 3 || s[i + 1] < lo || s[i + 1] > hi || !cont(s[i + 2])) return 0;
    *rune = ((uint32_t)(b0 & 0x0F) << 12) | ((uint32_t)(s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
    return 3;
  }
  // kLead4
  const uint8_t lo = b0 == 0xF0 ? 0x90 : 0x80, hi = b0 == 0xF4 ? 0x8F : 0xBF;
  if (rem < 4 || s[i + 1] < lo || s[i + 1] > hi || !cont(s[i + 2]) || !cont(s[i + 3])) return 0;
  *rune = 0x10000;  // never U+2028/9
  return 4;
}

inline void put(std::vector<uint8_t>& o, const char* lit) {
  o.insert(o.end(), lit, lit + std::strlen(lit));
}

}  // namespace

void append_string(std::vector<uint8_t>& o, const uint8_t* s, uint64_t n) {
  o.push_back('"');
  uint64_t i = 0, start = 0;
  auto flush = [&](uint64_t upto) {
    if (upto > start) o.insert(o.end(), s + start, s + upto);
  };
  while (i < n) {
    const uint8_t b = s[i];
    const uint8_t cls = kTab.c[b];
    if (cls == kCopy) {
      ++i;
      continue;
    }
    if (cls == kShort || cls == kU00) {
      flush(i);
      if (cls == kShort) {
        o.push_back('\\');
        o.push_back((uint8_t)kTab.short_esc[b]);
      } else {
        const char e[6] = {'\\', 'u', '0', '0', kHex[b >> 4], kHex[b & 15]};
        o.insert(o.end(), e, e + 6);
      }
      start = ++i;
      continue;
    }
    uint32_t rune = 0;
    const int len = cls == kBad ? 0 : seq_len(s, n, i, cls, &rune);
    if (len == 0) {  // utf8.RuneError, size 1
      flush(i);
      put(o, "\\ufffd");
      start = ++i;
      continue;
    }
    if (rune == 0x2028 || rune == 0x2029) {
      flush(i);
      put(o, "\\u202");
      o.push_back((uint8_t)kHex[rune & 15]);
      i += len;
      start = i;
      continue;
    }
    i += len;  // valid rune: stays in the raw copy run
  }
  flush(n);
  o.push_back('"');
}

void append_int(std::vector<uint8_t>& o, int64_t v) {
  char tmp[24];
  int k = 0;
  uint64_t u = v < 0 ? 0 - (uint64_t)v : (uint64_t)v;
  do {
    tmp[k++] = (char)('0' + u % 10);
    u /= 10;
  } while (u);
  if (v < 0) o.push_back('-');
  while (k) o.push_back((uint8_t)tmp[--k]);
}

void append_request(std::vector<uint8_t>& o, int64_t ts, const uint8_t* cid, uint64_t cidn, const uint8_t* op,
                    uint64_t opn, int64_t seq) {
  put(o, "{\"timestamp\":");
  append_int(o, ts);
  put(o, ",\"clientID\":");
  append_string(o, cid, cidn);
  put(o, ",\"operation\":");
  append_string(o, op, opn);
  put(o, ",\"sequenceID\":");
  append_int(o, seq);
  o.push_back('}');
}

void append_vote(std::vector<uint8_t>& o, int64_t view, int64_t seq, const uint8_t* dg, uint64_t dgn,
                 const uint8_t* nid, uint64_t nidn, int64_t mt) {
  put(o, "{\"viewID\":");
  append_int(o, view);
  put(o, ",\"sequenceID\":");
  append_int(o, seq);
  put(o, ",\"digest\":");
  append_string(o, dg, dgn);
  put(o, ",\"nodeID\":");
  append_string(o, nid, nidn);
  put(o, ",\"msgType\":");
  append_int(o, mt);
  o.push_back('}');
}

void append_reply(std::vector<uint8_t>& o, int64_t view, int64_t ts, const uint8_t* cid, uint64_t cidn,
                  const uint8_t* nid, uint64_t nidn, const uint8_t* res, uint64_t resn) {
  put(o, "{\"viewID\":");
  append_int(o, view);
  put(o, ",\"timestamp\":");
  append_int(o, ts);
  put(o, ",\"clientID\":");
  append_string(o, cid, cidn);
  put(o, ",\"nodeID\":");
  append_string(o, nid, nidn);
  put(o, ",\"result\":");
  append_string(o, res, resn);
  o.push_back('}');
}

void append_preprepare(std::vector<uint8_t>& o, int64_t view, int64_t seq, const uint8_t* dg, uint64_t dgn,
                       bool has_req, int64_t rts, const uint8_t* rcid, uint64_t rcidn, const uint8_t* rop,
                       uint64_t ropn, int64_t rseq) {
  put(o, "{\"viewID\":");
  append_int(o, view);
  put(o, ",\"sequenceID\":");
  append_int(o, seq);
  put(o, ",\"digest\":");
  append_string(o, dg, dgn);
  put(o, ",\"requestMsg\":");
  if (has_req) append_request(o, rts, rcid, rcidn, rop, ropn, rseq);
  else put(o, "null");
  o.push_back('}');
}

}  // namespace gojson
}  // namespace pbftv
