/* gojson_ref.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restates Go 1.19 encoding/json.Marshal for the reference's message structs
 * (pbft/consensus/pbft_msg_types.go:3-38), i.e. the exact preimage bytes that
 * digest() hashes (pbft/consensus/pbft_impl.go:235-243).  Rules (go1.19
 * encoding/json/encode.go):
 *   - compact output, struct field order, tag names as keys, no trailing newline;
 *   - int64 in decimal (strconv.AppendInt);
 *   - embedded `MsgType `json:"msgType"`` (pbft_msg_types.go:30) is a named int field;
 *   - nil *RequestMsg encodes as null;
 *   - string(): escapeHTML=true; '"' and '\\' backslash-escaped; \n \r \t short
 *     escapes; other bytes < 0x20 and '<' '>' '&' as \u00XX (lowercase hex);
 *     invalid UTF-8 (utf8.DecodeRuneInString -> RuneError,1) as the 6-byte escape "\\ufffd";
 *     U+2028 / U+2029 as "\\u2028" / "\\u2029"; everything else raw.
 * Also restates State.verifyMsg (pbft_impl.go:176-202).
 */
#include "oracle.h"

#include <string.h>

typedef struct { uint8_t* out; uint64_t cap, len; } buf;

static void put(buf* b, uint8_t c) { if (b->len < b->cap) b->out[b->len] = c; b->len++; }
static void puts_(buf* b, const char* s) { while (*s) put(b, (uint8_t)*s++); }

static void put_int(buf* b, int64_t v) {
  char tmp[24]; int n = 0;
  uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
  do { tmp[n++] = (char)('0' + u % 10); u /= 10; } while (u);
  if (v < 0) put(b, '-');
  while (n) put(b, (uint8_t)tmp[--n]);
}

/* utf8.DecodeRuneInString size for a valid sequence at s[i:], or 0 if invalid (RuneError,1) */
static int utf8_len(const uint8_t* s, uint64_t n, uint64_t i, uint32_t* rune) {
  uint8_t c = s[i];
  uint64_t rem = n - i;
  if (c >= 0xC2 && c <= 0xDF) {
    if (rem < 2 || (s[i + 1] & 0xC0) != 0x80) return 0;
    *rune = ((uint32_t)(c & 0x1F) << 6) | (s[i + 1] & 0x3F);
    return 2;
  }
  if (c >= 0xE0 && c <= 0xEF) {
    uint8_t lo = 0x80, hi = 0xBF;
    if (c == 0xE0) lo = 0xA0;
    if (c == 0xED) hi = 0x9F;
    if (rem < 2 || s[i + 1] < lo || s[i + 1] > hi) return 0;
    if (rem < 3 || (s[i + 2] & 0xC0) != 0x80) return 0;
    *rune = ((uint32_t)(c & 0x0F) << 12) | ((uint32_t)(s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
    return 3;
  }
  if (c >= 0xF0 && c <= 0xF4) {
    uint8_t lo = 0x80, hi = 0xBF;
    if (c == 0xF0) lo = 0x90;
    if (c == 0xF4) hi = 0x8F;
    if (rem < 2 || s[i + 1] < lo || s[i + 1] > hi) return 0;
    if (rem < 3 || (s[i + 2] & 0xC0) != 0x80) return 0;
    if (rem < 4 || (s[i + 3] & 0xC0) != 0x80) return 0;
    *rune = ((uint32_t)(c & 0x07) << 18) | ((uint32_t)(s[i + 1] & 0x3F) << 12) | ((uint32_t)(s[i + 2] & 0x3F) << 6) |
            (s[i + 3] & 0x3F);
    return 4;
  }
  return 0;
}

static void put_string(buf* b, const char* str, uint64_t n) {
  static const char hx[] = "0123456789abcdef";
  const uint8_t* s = (const uint8_t*)str;
  put(b, '"');
  for (uint64_t i = 0; i < n;) {
    uint8_t c = s[i];
    if (c < 0x80) {
      int safe = c >= 0x20 && c != '"' && c != '\\' && c != '<' && c != '>' && c != '&';
      if (safe) { put(b, c); i++; continue; }
      put(b, '\\');
      if (c == '\\' || c == '"') put(b, c);
      else if (c == '\n') put(b, 'n');
      else if (c == '\r') put(b, 'r');
      else if (c == '\t') put(b, 't');
      else { puts_(b, "u00"); put(b, (uint8_t)hx[c >> 4]); put(b, (uint8_t)hx[c & 15]); }
      i++;
      continue;
    }
    uint32_t rune = 0;
    int sz = utf8_len(s, n, i, &rune);
    if (sz == 0) { puts_(b, "\\ufffd"); i++; continue; }
    if (rune == 0x2028 || rune == 0x2029) { puts_(b, "\\u202"); put(b, (uint8_t)hx[rune & 15]); i += sz; continue; }
    for (int k = 0; k < sz; ++k) put(b, s[i + k]);
    i += sz;
  }
  put(b, '"');
}

static void put_request(buf* b, int64_t ts, const char* cid, uint64_t cidn, const char* op, uint64_t opn, int64_t seq) {
  puts_(b, "{\"timestamp\":"); put_int(b, ts);
  puts_(b, ",\"clientID\":"); put_string(b, cid, cidn);
  puts_(b, ",\"operation\":"); put_string(b, op, opn);
  puts_(b, ",\"sequenceID\":"); put_int(b, seq);
  put(b, '}');
}

uint64_t oracle_gojson_request(int64_t ts, const char* cid, uint64_t cidn, const char* op, uint64_t opn, int64_t seq,
                               uint8_t* out, uint64_t cap) {
  buf b = {out, cap, 0};
  put_request(&b, ts, cid, cidn, op, opn, seq);
  return b.len;
}

uint64_t oracle_gojson_vote(int64_t view, int64_t seq, const char* dg, uint64_t dgn, const char* nid, uint64_t nidn,
                            int64_t mt, uint8_t* out, uint64_t cap) {
  buf b = {out, cap, 0};
  puts_(&b, "{\"viewID\":"); put_int(&b, view);
  puts_(&b, ",\"sequenceID\":"); put_int(&b, seq);
  puts_(&b, ",\"digest\":"); put_string(&b, dg, dgn);
  puts_(&b, ",\"nodeID\":"); put_string(&b, nid, nidn);
  puts_(&b, ",\"msgType\":"); put_int(&b, mt);
  put(&b, '}');
  return b.len;
}

uint64_t oracle_gojson_reply(int64_t view, int64_t ts, const char* cid, uint64_t cidn, const char* nid, uint64_t nidn,
                             const char* res, uint64_t resn, uint8_t* out, uint64_t cap) {
  buf b = {out, cap, 0};
  puts_(&b, "{\"viewID\":"); put_int(&b, view);
  puts_(&b, ",\"timestamp\":"); put_int(&b, ts);
  puts_(&b, ",\"clientID\":"); put_string(&b, cid, cidn);
  puts_(&b, ",\"nodeID\":"); put_string(&b, nid, nidn);
  puts_(&b, ",\"result\":"); put_string(&b, res, resn);
  put(&b, '}');
  return b.len;
}

uint64_t oracle_gojson_preprepare(int64_t view, int64_t seq, const char* dg, uint64_t dgn, int has_req, int64_t rts,
                                  const char* rcid, uint64_t rcidn, const char* rop, uint64_t ropn, int64_t rseq,
                                  uint8_t* out, uint64_t cap) {
  buf b = {out, cap, 0};
  puts_(&b, "{\"viewID\":"); put_int(&b, view);
  puts_(&b, ",\"sequenceID\":"); put_int(&b, seq);
  puts_(&b, ",\"digest\":"); put_string(&b, dg, dgn);
  puts_(&b, ",\"requestMsg\":");
  if (has_req) put_request(&b, rts, rcid, rcidn, rop, ropn, rseq); else puts_(&b, "null");
  put(&b, '}');
  return b.len;
}

int oracle_verify_msg(int64_t sview, int64_t slast, const uint8_t d[32], int64_t view, int64_t seq, const char* got,
                      uint64_t gotn) {
  static const char hx[] = "0123456789abcdef";
  if (sview != view) return 0;                          /* pbft_impl.go:178 */
  if (slast != -1 && slast >= seq) return 0;            /* pbft_impl.go:184-188 */
  if (gotn != 64) return 0;                             /* Go string compare (pbft_impl.go:197) */
  for (int i = 0; i < 32; ++i)
    if (got[2 * i] != hx[d[i] >> 4] || got[2 * i + 1] != hx[d[i] & 15]) return 0;
  return 1;
}
