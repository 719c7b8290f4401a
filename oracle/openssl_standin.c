/* openssl_standin.c -- CPU BASELINE / CROSS-CHECK ONLY (never part of the product).
 *
 * "a C++ std::thread x nproc OpenSSL libcrypto baseline
 * (ECDSA_do_verify), labelled OpenSSL stand-in".  The reference's own verify
 * path would be Go crypto/ecdsa, which cannot run here (no Go toolchain); this
 * is the closest native CPU implementation in the image: OpenSSL 3 libcrypto's
 * P-256 (nistz256 assembly on x86-64) timed on host threads, each thread with
 * its own EC_KEY objects.  bench.py times it beside the GPU on the same
 * signatures and checks that the accept bits agree.
 *
 * standin_sha256_batch is the same for utils.Hash (SURVEY.md §8(d)(ii):
 * EVP_Digest SHA-256, SHA-NI on x86-64 like Go's crypto/sha256 assembly).
 *
 * Semantics match Go crypto/ecdsa.Verify for 32-byte hashes: r, s outside
 * [1, n-1] are rejected by OpenSSL; keys that OpenSSL refuses to load
 * (off-curve, coordinate >= p) reject every signature naming them.
 */
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/obj_mac.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  const uint8_t* hashes;
  const uint8_t* sigs;
  const uint32_t* kidx;
  uint64_t lo, hi;
  const uint8_t* keys;
  uint32_t nkeys;
  uint8_t* ok;
} job_t;

static EC_KEY* load_key(const uint8_t xy[64]) {
  EC_KEY* k = EC_KEY_new_by_curve_name(NID_X9_62_prime256v1);
  BIGNUM* x = BN_bin2bn(xy, 32, NULL);
  BIGNUM* y = BN_bin2bn(xy + 32, 32, NULL);
  const int good = k && x && y && EC_KEY_set_public_key_affine_coordinates(k, x, y) == 1;
  BN_free(x);
  BN_free(y);
  if (!good) {
    EC_KEY_free(k);
    ERR_clear_error();
    return NULL;
  }
  return k;
}

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  EC_KEY** ks = (EC_KEY**)calloc(j->nkeys ? j->nkeys : 1, sizeof(EC_KEY*));
  for (uint32_t k = 0; k < j->nkeys; ++k) ks[k] = load_key(j->keys + 64ull * k);
  for (uint64_t i = j->lo; i < j->hi; ++i) {
    const uint32_t k = j->kidx[i];
    uint8_t ok = 0;
    if (k < j->nkeys && ks[k]) {
      ECDSA_SIG* s = ECDSA_SIG_new();
      BIGNUM* r = BN_bin2bn(j->sigs + 64 * i, 32, NULL);
      BIGNUM* ss = BN_bin2bn(j->sigs + 64 * i + 32, 32, NULL);
      ECDSA_SIG_set0(s, r, ss);
      ok = ECDSA_do_verify(j->hashes + 32 * i, 32, s, ks[k]) == 1;
      ECDSA_SIG_free(s);
      ERR_clear_error();
    }
    j->ok[i] = ok;
  }
  for (uint32_t k = 0; k < j->nkeys; ++k) EC_KEY_free(ks[k]);
  free(ks);
  return NULL;
}

/* Verify n signatures on `threads` host threads; out_bitmap LSB-first,
 * ceil(n/8) bytes.  Returns the number accepted, or -1 on allocation failure. */
int64_t standin_ecdsa_p256_verify_batch(const uint8_t* hashes, const uint8_t* sigs, const uint32_t* kidx, uint64_t n,
                                        const uint8_t* keys, uint32_t nkeys, uint8_t* out_bitmap, int threads) {
  if (threads < 1) threads = 1;
  uint8_t* ok = (uint8_t*)calloc(n ? n : 1, 1);
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  job_t* jobs = (job_t*)calloc((size_t)threads, sizeof(job_t));
  if (!ok || !th || !jobs) return -1;
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (job_t){hashes, sigs, kidx, n * t / threads, n * (t + 1) / threads, keys, nkeys, ok};
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  int64_t acc = 0;
  memset(out_bitmap, 0, (n + 7) / 8);
  for (uint64_t i = 0; i < n; ++i) {
    out_bitmap[i >> 3] |= (uint8_t)(ok[i] << (i & 7));
    acc += ok[i];
  }
  free(ok);
  free(th);
  free(jobs);
  return acc;
}

/* ---- QC latency on the CPU ("p50 QC verify latency ...
 * single-threaded per QC") ----
 * One certificate of per_cert signatures at a time, as the reference's replica
 * would check the votes it has collected (pbft_impl.go:115-173, one
 * ecdsa.Verify per vote), on `threads` host threads: the calling thread plus
 * threads-1 persistent workers that spin on a generation counter, so a
 * certificate costs its verifies plus one cache-line hand-off, not a thread
 * start.  Keys are parsed once per thread beforehand (a replica holds its
 * peers' *ecdsa.PublicKey).  Signature i of a certificate goes to thread
 * i % threads.  out_us[c] = wall time of certificate c from the post to the
 * last verdict; gap_us of idle time (spin-free sleep) before each. */
#include <stdatomic.h>
#include <time.h>

typedef struct {
  const uint8_t* keys;
  uint32_t nkeys;
  EC_KEY** ks;
} keyset_t;

typedef struct {
  /* the certificate being verified (written by the caller before gen++) */
  const uint8_t* h;
  const uint8_t* s;
  const uint32_t* k;
  uint8_t* ok;
  uint32_t m;
  int threads;
  keyset_t* sets; /* one per thread */
  _Alignas(64) atomic_uint gen;
  _Alignas(64) atomic_uint done;
  _Alignas(64) atomic_int stop;
} qc_pool_t;

typedef struct {
  qc_pool_t* p;
  int tid;
} qc_arg_t;

static void qc_slice(qc_pool_t* p, int tid) {
  EC_KEY** ks = p->sets[tid].ks;
  for (uint32_t i = (uint32_t)tid; i < p->m; i += (uint32_t)p->threads) {
    const uint32_t k = p->k[i];
    uint8_t ok = 0;
    if (k < p->sets[tid].nkeys && ks[k]) {
      ECDSA_SIG* s = ECDSA_SIG_new();
      BIGNUM* r = BN_bin2bn(p->s + 64 * i, 32, NULL);
      BIGNUM* ss = BN_bin2bn(p->s + 64 * i + 32, 32, NULL);
      ECDSA_SIG_set0(s, r, ss);
      ok = ECDSA_do_verify(p->h + 32 * i, 32, s, ks[k]) == 1;
      ECDSA_SIG_free(s);
      ERR_clear_error();
    }
    p->ok[i] = ok;
  }
}

static void keyset_load(keyset_t* ks, const uint8_t* keys, uint32_t nkeys) {
  ks->keys = keys;
  ks->nkeys = nkeys;
  ks->ks = (EC_KEY**)calloc(nkeys ? nkeys : 1, sizeof(EC_KEY*));
  for (uint32_t k = 0; k < nkeys; ++k) ks->ks[k] = load_key(keys + 64ull * k);
}

static void keyset_free(keyset_t* ks) {
  for (uint32_t k = 0; k < ks->nkeys; ++k) EC_KEY_free(ks->ks[k]);
  free(ks->ks);
}

static void* qc_worker(void* arg) {
  qc_arg_t* a = (qc_arg_t*)arg;
  qc_pool_t* p = a->p;
  keyset_load(&p->sets[a->tid], p->sets[0].keys, p->sets[0].nkeys);
  atomic_fetch_add_explicit(&p->done, 1, memory_order_release); /* keys loaded */
  unsigned seen = 0;
  for (;;) {
    unsigned g;
    while ((g = atomic_load_explicit(&p->gen, memory_order_acquire)) == seen) {
      if (atomic_load_explicit(&p->stop, memory_order_acquire)) goto out;
      __builtin_ia32_pause();
    }
    seen = g;
    qc_slice(p, a->tid);
    atomic_fetch_add_explicit(&p->done, 1, memory_order_release);
  }
out:
  keyset_free(&p->sets[a->tid]);
  return NULL;
}

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec * 1e6 + (double)t.tv_nsec * 1e-3;
}

/* n_certs certificates of per_cert signatures each (certificate c = entries
 * [c * per_cert, (c + 1) * per_cert) of the arrays).  out_bitmap: LSB-first
 * verdicts of all n_certs * per_cert signatures.  Returns the number accepted,
 * or -1 on a bad argument / allocation failure. */
int64_t standin_qc_latency(const uint8_t* hashes, const uint8_t* sigs, const uint32_t* kidx, uint64_t n_certs,
                           uint32_t per_cert, const uint8_t* keys, uint32_t nkeys, int threads, double gap_us,
                           double* out_us, uint8_t* out_bitmap) {
  if (threads < 1) threads = 1;
  if (!per_cert) return -1;
  const uint64_t n = n_certs * per_cert;
  qc_pool_t* p = (qc_pool_t*)aligned_alloc(64, (sizeof(qc_pool_t) + 63) / 64 * 64);
  uint8_t* ok = (uint8_t*)calloc(n ? n : 1, 1);
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  qc_arg_t* args = (qc_arg_t*)calloc((size_t)threads, sizeof(qc_arg_t));
  if (!p || !ok || !th || !args) return -1;
  memset(p, 0, sizeof(*p));
  p->threads = threads;
  p->sets = (keyset_t*)calloc((size_t)threads, sizeof(keyset_t));
  keyset_load(&p->sets[0], keys, nkeys);
  atomic_store(&p->gen, 0);
  atomic_store(&p->done, 0);
  atomic_store(&p->stop, 0);
  for (int t = 1; t < threads; ++t) {
    args[t] = (qc_arg_t){p, t};
    pthread_create(&th[t], NULL, qc_worker, &args[t]);
  }
  while (atomic_load_explicit(&p->done, memory_order_acquire) != (unsigned)(threads - 1)) __builtin_ia32_pause();
  for (uint64_t c = 0; c < n_certs; ++c) {
    if (gap_us > 0) {
      struct timespec ts = {(time_t)(gap_us / 1e6), (long)(((uint64_t)gap_us % 1000000ull) * 1000ull)};
      nanosleep(&ts, NULL);
    }
    const double t0 = now_us();
    p->h = hashes + 32 * c * per_cert;
    p->s = sigs + 64 * c * per_cert;
    p->k = kidx + c * per_cert;
    p->ok = ok + c * per_cert;
    p->m = per_cert;
    atomic_store_explicit(&p->done, 0, memory_order_relaxed);
    atomic_fetch_add_explicit(&p->gen, 1, memory_order_release);
    qc_slice(p, 0);
    while (atomic_load_explicit(&p->done, memory_order_acquire) != (unsigned)(threads - 1)) __builtin_ia32_pause();
    out_us[c] = now_us() - t0;
  }
  atomic_store_explicit(&p->stop, 1, memory_order_release);
  for (int t = 1; t < threads; ++t) pthread_join(th[t], NULL);
  keyset_free(&p->sets[0]);
  int64_t acc = 0;
  memset(out_bitmap, 0, (n + 7) / 8);
  for (uint64_t i = 0; i < n; ++i) {
    out_bitmap[i >> 3] |= (uint8_t)(ok[i] << (i & 7));
    acc += ok[i];
  }
  free(p->sets);
  free(p);
  free(ok);
  free(th);
  free(args);
  return acc;
}

typedef struct {
  const uint8_t* data;
  const uint64_t* offsets;
  const uint32_t* lengths;
  uint64_t lo, hi;
  uint8_t* out;
} sha_job_t;

/* One explicitly fetched SHA-256 and one digest context per thread: EVP_Digest
 * with EVP_sha256() re-resolves the provider algorithm on every call under a
 * process-wide lock (OpenSSL 3), which serialises the threads. */
static void* sha_worker(void* arg) {
  sha_job_t* j = (sha_job_t*)arg;
  EVP_MD* md = EVP_MD_fetch(NULL, "SHA256", NULL);
  EVP_MD_CTX* c = EVP_MD_CTX_new();
  unsigned int len = 32;
  for (uint64_t i = j->lo; i < j->hi; ++i) {
    EVP_DigestInit_ex(c, md, NULL);
    EVP_DigestUpdate(c, j->data + j->offsets[i], j->lengths[i]);
    EVP_DigestFinal_ex(c, j->out + 32 * i, &len);
  }
  EVP_MD_CTX_free(c);
  EVP_MD_free(md);
  return NULL;
}

/* SHA-256 of n messages (data + offsets[i], lengths[i] bytes) on `threads`
 * host threads into out (n * 32 B).  Returns 0, or -1 on allocation failure. */
int standin_sha256_batch(const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths, uint64_t n,
                         uint8_t* out, int threads) {
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  sha_job_t* jobs = (sha_job_t*)calloc((size_t)threads, sizeof(sha_job_t));
  if (!th || !jobs) return -1;
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (sha_job_t){data, offsets, lengths, n * t / threads, n * (t + 1) / threads, out};
    pthread_create(&th[t], NULL, sha_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  return 0;
}

/* utils.Hash of ONE message on the caller's thread (EVP_Digest SHA-256 +
 * lowercase hex), reps calls, out_us[i] each call's wall time: the CPU side
 * of bench.py single_calls_us. */
int standin_hash_hex_drive(const uint8_t* msg, uint64_t len, uint32_t reps, double* out_us, char out_hex[65]) {
  static const char hx[] = "0123456789abcdef";
  unsigned char d[32];
  unsigned int dl = 0;
  int bad = 0;
  for (uint32_t i = 0; i < reps; ++i) {
    const double t0 = now_us();
    bad += EVP_Digest(msg, len, d, &dl, EVP_sha256(), NULL) != 1;
    for (int k = 0; k < 32; ++k) {
      out_hex[2 * k] = hx[d[k] >> 4];
      out_hex[2 * k + 1] = hx[d[k] & 15];
    }
    out_hex[64] = 0;
    out_us[i] = now_us() - t0;
  }
  return bad;
}
