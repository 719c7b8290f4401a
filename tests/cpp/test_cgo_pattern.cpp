// test_cgo_pattern.cpp -- TEST PROGRAM: the C ABI driven the way a cgo shim
// drives it (Go itself is not in this image).
//
//   * one context shared by several caller threads (goroutines on OS threads),
//   * every input and output buffer owned by the caller, allocated per call
//     (a Go heap slice), and overwritten the moment the call returns -- the
//     library must not keep a pointer past its return (cgo pointer rules);
//   * mixed batch sizes on the one context: the one-wave-per-signature path
//     (3, 67), the lane path (700, 5000) and the pipelined host path (40000),
//     plus SHA-256 batches and utils.Hash;
//   * every bitmap and digest checked against the oracle (test infrastructure).
// Exit status 0 and "0 failed" on success.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../../include/pbftv.h"
#include "../../oracle/oracle.h"

static std::atomic<int> g_fail{0}, g_pass{0};
#define CHECK(c)                                                        \
  do {                                                                  \
    if (c) {                                                            \
      ++g_pass;                                                         \
    } else {                                                            \
      ++g_fail;                                                         \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);      \
    }                                                                   \
  } while (0)

struct Pool {
  std::vector<uint8_t> keys, H, S, want;
  std::vector<uint32_t> K;
  size_t n = 0;
};

// n signatures over n_keys keys, 1 in 9 corrupted, expected bits from the oracle
static Pool make_pool(size_t n, uint32_t n_keys, uint32_t seed) {
  std::mt19937_64 rng(seed);
  Pool p;
  p.n = n;
  p.keys.resize(64 * n_keys);
  std::vector<std::array<uint8_t, 32>> priv(n_keys);
  for (uint32_t k = 0; k < n_keys; ++k) {
    for (auto& b : priv[k]) b = (uint8_t)rng();
    priv[k][0] &= 0x7F;
    priv[k][31] |= 1;
    oracle_p256_pubkey(priv[k].data(), &p.keys[64 * k]);
  }
  const size_t distinct = n < 512 ? n : 512;  // signing is slow: tile 512 distinct signatures
  p.H.resize(32 * n);
  p.S.resize(64 * n);
  p.K.resize(n);
  for (size_t i = 0; i < distinct; ++i) {
    for (int b = 0; b < 32; ++b) p.H[32 * i + b] = (uint8_t)rng();
    p.K[i] = (uint32_t)(i % n_keys);
    uint8_t kn[32];
    do {
      for (auto& b : kn) b = (uint8_t)rng();
    } while (!oracle_ecdsa_p256_sign(&p.H[32 * i], priv[p.K[i]].data(), kn, &p.S[64 * i]));
  }
  for (size_t i = distinct; i < n; ++i) {
    std::memcpy(&p.H[32 * i], &p.H[32 * (i % distinct)], 32);
    std::memcpy(&p.S[64 * i], &p.S[64 * (i % distinct)], 64);
    p.K[i] = p.K[i % distinct];
  }
  for (size_t i = 0; i < n; i += 9) p.S[64 * i + (i % 64)] ^= 0x20;
  p.want.assign((n + 7) / 8, 0);
  oracle_ecdsa_p256_verify_batch(p.H.data(), p.S.data(), p.K.data(), n, p.keys.data(), n_keys, p.want.data(), 4);
  return p;
}

int main() {
  pbftv_ctx* ctx = nullptr;
  int rc = pbftv_open(&ctx, 0);
  if (rc != PBFTV_OK) {
    fprintf(stderr, "pbftv_open: %s (%s)\n", pbftv_strerror(rc), pbftv_last_error());
    return 3;
  }
  const uint32_t n_keys = 7;
  const size_t sizes[] = {3, 67, 700, 5000, 40000};
  std::vector<Pool> pools;
  for (size_t s = 0; s < sizeof(sizes) / sizeof(sizes[0]); ++s) pools.push_back(make_pool(sizes[s], n_keys, 11));
  {
    std::vector<uint8_t> keys = pools[0].keys, valid(n_keys);  // a caller-owned copy, poisoned after the call
    CHECK(pbftv_register_keys(ctx, keys.data(), n_keys, valid.data()) == PBFTV_OK);
    std::memset(keys.data(), 0xA5, keys.size());
    for (auto v : valid) CHECK(v == 1);
  }
  const int kThreads = 6, kIters = 12;
  std::vector<std::thread> th;
  for (int t = 0; t < kThreads; ++t) {
    th.emplace_back([&, t] {
      std::mt19937 rng(100 + t);
      for (int it = 0; it < kIters; ++it) {
        const Pool& p = pools[(t + it) % pools.size()];
        // a fresh "Go slice" per call, poisoned as soon as the call returns
        std::vector<uint8_t> H(p.H), S(p.S), bm((p.n + 7) / 8 + 1, 0xEE);
        std::vector<uint32_t> K(p.K);
        const int r = pbftv_ecdsa_p256_verify_batch(ctx, H.data(), S.data(), K.data(), p.n, bm.data());
        std::memset(H.data(), 0x5A, H.size());
        std::memset(S.data(), 0x5A, S.size());
        std::fill(K.begin(), K.end(), 0xFFFFFFFFu);
        CHECK(r == PBFTV_OK);
        bool same = true;
        for (size_t i = 0; i < p.n; ++i) same &= ((bm[i / 8] >> (i % 8)) & 1) == ((p.want[i / 8] >> (i % 8)) & 1);
        CHECK(same);
        // SHA-256 batch + utils.Hash on caller-owned messages
        const int nm = 1 + (int)(rng() % 200);
        std::vector<uint8_t> blob;
        std::vector<uint64_t> off(nm);
        std::vector<uint32_t> len(nm);
        for (int m = 0; m < nm; ++m) {
          off[m] = blob.size();
          len[m] = (uint32_t)(rng() % 300);
          for (uint32_t b = 0; b < len[m]; ++b) blob.push_back((uint8_t)rng());
        }
        blob.push_back(0);
        std::vector<uint8_t> dg(32 * nm);
        CHECK(pbftv_sha256_batch(ctx, blob.data(), off.data(), len.data(), nm, dg.data()) == PBFTV_OK);
        bool dok = true;
        for (int m = 0; m < nm; ++m) {
          uint8_t w[32];
          oracle_sha256(blob.data() + off[m], len[m], w);
          dok &= std::memcmp(w, &dg[32 * m], 32) == 0;
        }
        CHECK(dok);
        char hex[65];
        CHECK(pbftv_hash_hex(ctx, blob.data(), len[0], hex) == PBFTV_OK);
        char want_hex[65];
        oracle_hash_hex(blob.data(), len[0], want_hex);
        CHECK(std::strcmp(hex, want_hex) == 0);
        std::memset(blob.data(), 0x33, blob.size());
      }
    });
  }
  for (auto& x : th) x.join();
  // the context is still healthy after the concurrent use
  {
    const Pool& p = pools[2];
    std::vector<uint8_t> bm((p.n + 7) / 8, 0);
    CHECK(pbftv_ecdsa_p256_verify_batch(ctx, p.H.data(), p.S.data(), p.K.data(), p.n, bm.data()) == PBFTV_OK);
    CHECK(std::memcmp(bm.data(), p.want.data(), bm.size()) == 0);
  }
  pbftv_close(ctx);
  printf("cgo pattern: %d passed, %d failed\n", g_pass.load(), g_fail.load());
  return g_fail.load() == 0 ? 0 : 1;
}
