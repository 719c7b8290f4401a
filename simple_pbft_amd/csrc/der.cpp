// der.cpp -- ASN.1 DER ECDSA signatures -> the (r, s) layout of
// pbftv_ecdsa_p256_verify_batch (DER parsing stays on the
// host, with Go's strictness).
//
// Restates go1.19 crypto/ecdsa.VerifyASN1's parse over
// golang.org/x/crypto/cryptobyte (vendored in the Go tree):
//   input.ReadASN1(&inner, SEQUENCE) && input.Empty() &&
//   inner.ReadASN1Integer(r) && inner.ReadASN1Integer(s) && inner.Empty()
// readASN1: single-byte tags only (low 5 bits != 0x1f); short-form length, or
// long form with 1..4 length bytes, value >= 128 and no leading zero byte.
// checkASN1Integer: non-empty, minimal two's complement (no redundant 0x00 /
// 0xff lead byte).  A negative integer or one >= 2^256 can never pass
// Verify's 1 <= r, s < n test, so it is rejected here (rs zeroed -> 0 bit).
// A zero integer parses (as in Go: ReadASN1Integer accepts 0) and is rejected
// by the verify kernels' range check, like any r or s >= n.
#include <cstdint>
#include <cstring>

namespace {

struct Cur {
  const uint8_t* p;
  uint64_t n;
};

// cryptobyte.String.ReadASN1 with an expected tag
bool read_asn1(Cur& c, uint8_t tag, Cur& out) {
  if (c.n < 2) return false;
  const uint8_t t = c.p[0], lb = c.p[1];
  if ((t & 0x1f) == 0x1f) return false;
  uint64_t hdr = 2, len;
  if ((lb & 0x80) == 0) {
    len = lb;
  } else {
    const uint32_t ll = lb & 0x7f;
    if (ll == 0 || ll > 4 || c.n < 2 + (uint64_t)ll) return false;
    uint32_t v = 0;
    for (uint32_t k = 0; k < ll; ++k) v = (v << 8) | c.p[2 + k];
    if (v < 128) return false;
    if ((v >> ((ll - 1) * 8)) == 0) return false;
    hdr = 2 + ll;
    len = v;
  }
  if (c.n - hdr < len || c.n < hdr) return false;
  if (t != tag) return false;
  out.p = c.p + hdr;
  out.n = len;
  c.p += hdr + len;
  c.n -= hdr + len;
  return true;
}

// ReadASN1Integer + range: value in [1, 2^256) -> 32 B big-endian
bool read_uint256(Cur& c, uint8_t* be32, bool& in_range) {
  Cur v;
  if (!read_asn1(c, 0x02, v)) return false;
  if (v.n == 0) return false;
  if (v.n > 1 && ((v.p[0] == 0 && (v.p[1] & 0x80) == 0) || (v.p[0] == 0xff && (v.p[1] & 0x80) == 0x80))) return false;
  in_range = (v.p[0] & 0x80) == 0;  // negative values fail Verify
  const uint8_t* b = v.p;
  uint64_t n = v.n;
  if (n > 1 && b[0] == 0) ++b, --n;
  if (n > 32) in_range = false;
  if (in_range) {
    std::memset(be32, 0, 32);
    std::memcpy(be32 + 32 - n, b, n);
  }
  return true;
}

}  // namespace

extern "C" {

int pbftv_ecdsa_der_to_rs(const uint8_t* der, uint64_t der_len, uint8_t* out_rs) {
  if (out_rs == nullptr || (der == nullptr && der_len != 0)) return -1;  // PBFTV_EINVAL
  uint8_t rs[64];
  Cur in{der, der_len}, inner{nullptr, 0};
  bool r_ok = false, s_ok = false;
  const bool ok = read_asn1(in, 0x30, inner) && in.n == 0 && read_uint256(inner, rs, r_ok) &&
                  read_uint256(inner, rs + 32, s_ok) && inner.n == 0 && r_ok && s_ok;
  if (ok) std::memcpy(out_rs, rs, 64);
  else std::memset(out_rs, 0, 64);
  return ok ? 1 : 0;
}

int64_t pbftv_ecdsa_der_to_rs_batch(const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths,
                                    uint64_t n, uint8_t* out_rs) {
  if (n == 0) return 0;
  if (offsets == nullptr || lengths == nullptr || out_rs == nullptr) return -1;
  if (data == nullptr)
    for (uint64_t i = 0; i < n; ++i)
      if (lengths[i] != 0) return -1;  // PBFTV_EINVAL: encodings promised but no bytes
  int64_t parsed = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const int r = pbftv_ecdsa_der_to_rs(data ? data + offsets[i] : nullptr, data ? lengths[i] : 0, out_rs + 64 * i);
    if (r < 0) return r;
    parsed += r;
  }
  return parsed;
}

}  // extern "C"
