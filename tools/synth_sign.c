// synth_sign.c -- synthetic-input generator for bench.py / tests (tools/synth.py):
// n ECDSA-P256 signatures with OpenSSL 3 libcrypto (ECDSA_do_sign, random
// nonces) on a pool of host threads, so a 1M-signature config-4 batch is made
// of distinct signatures without a Python loop (a tiled 65,536-signature pool
// repeated the same signature 16 times, which the key order can place in
// neighbouring lanes and serve from cache -- not a real workload).
//
// Not part of the product and not the oracle: it only makes inputs.
//   cc -O2 -shared -fPIC -o tools/libsynth_sign.so tools/synth_sign.c -lcrypto -lpthread
#define OPENSSL_SUPPRESS_DEPRECATED 1
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/obj_mac.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

typedef struct {
  const uint8_t* priv;  // nkeys x 32 B big-endian private scalars
  uint32_t nkeys;
  const uint8_t* hashes;
  const uint32_t* kidx;
  uint8_t* out;  // n x 64 B: r || s big-endian
  uint64_t lo, hi;
  int rc;
} job_t;

static void* run(void* arg) {
  job_t* j = (job_t*)arg;
  EC_KEY** keys = (EC_KEY**)calloc(j->nkeys, sizeof(EC_KEY*));
  j->rc = keys ? 0 : -1;
  for (uint32_t k = 0; k < j->nkeys && j->rc == 0; ++k) {
    EC_KEY* key = EC_KEY_new_by_curve_name(NID_X9_62_prime256v1);
    BIGNUM* d = BN_bin2bn(j->priv + 32 * (size_t)k, 32, NULL);
    const EC_GROUP* g = key ? EC_KEY_get0_group(key) : NULL;
    EC_POINT* q = g ? EC_POINT_new(g) : NULL;
    if (!key || !d || !q || !EC_KEY_set_private_key(key, d) || !EC_POINT_mul(g, q, d, NULL, NULL, NULL) ||
        !EC_KEY_set_public_key(key, q))
      j->rc = -2;
    keys[k] = key;
    BN_free(d);
    EC_POINT_free(q);
  }
  for (uint64_t i = j->lo; i < j->hi && j->rc == 0; ++i) {
    const uint32_t k = j->kidx[i];
    if (k >= j->nkeys) {
      j->rc = -3;
      break;
    }
    ECDSA_SIG* sig = ECDSA_do_sign(j->hashes + 32 * i, 32, keys[k]);
    if (!sig) {
      j->rc = -4;
      break;
    }
    BN_bn2binpad(ECDSA_SIG_get0_r(sig), j->out + 64 * i, 32);
    BN_bn2binpad(ECDSA_SIG_get0_s(sig), j->out + 64 * i + 32, 32);
    ECDSA_SIG_free(sig);
  }
  if (keys)
    for (uint32_t k = 0; k < j->nkeys; ++k) EC_KEY_free(keys[k]);
  free(keys);
  return NULL;
}

// 0 on success, negative on an OpenSSL failure or a key index out of range
int synth_sign_batch(const uint8_t* priv, uint32_t nkeys, const uint8_t* hashes, const uint32_t* kidx, uint64_t n,
                     uint8_t* out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  pthread_t tid[64];
  int live[64] = {0};
  job_t jobs[64];
  const uint64_t per = (n + (uint64_t)threads - 1) / (uint64_t)threads;
  for (int t = 0; t < threads; ++t) {
    const uint64_t lo = per * (uint64_t)t < n ? per * (uint64_t)t : n;
    const uint64_t hi = lo + per < n ? lo + per : n;
    jobs[t] = (job_t){priv, nkeys, hashes, kidx, out, lo, hi, 0};
    if (pthread_create(&tid[t], NULL, run, &jobs[t]) == 0) live[t] = 1;
    else run(&jobs[t]);  // no thread: this slice on the caller's
  }
  int rc = 0;
  for (int t = 0; t < threads; ++t) {
    if (live[t]) pthread_join(tid[t], NULL);
    if (jobs[t].rc) rc = jobs[t].rc;
  }
  return rc;
}
