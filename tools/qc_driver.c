/* qc_driver.c -- the QC-latency caller loop in C (bench.py / tools/qc_cadence.py).
 *
 * A replica calls pbftv_qc_verify once per certificate from compiled code (the
 * cgo binding of INTEGRATION.md: ~0.1 us per call).  Timing that loop from
 * Python adds the interpreter and ctypes to every sample, and after an idle
 * gap their cold caches cost more than the verify itself (round 4: ~45 us of
 * a 1-s-gap sample).  This loop makes the calls the way compiled code would:
 * nanosleep(gap) before each certificate, CLOCK_MONOTONIC around the call.
 * The library is called through the function pointers the caller passes in
 * (ctypes gives them), so this file needs no link against libpbftv.so.
 */
#include <stdint.h>
#include <string.h>
#include <time.h>

typedef int (*qc_verify_fn)(void* ctx, const uint8_t* hashes, const uint8_t* sig_rs, const uint32_t* key_idx,
                            uint64_t n, uint32_t quorum, uint8_t* out_bitmap, uint64_t* out_accepted, int* out_quorum);
typedef int (*qc_stamps_fn)(void* ctx, int dev, uint64_t out[8]);

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec * 1e6 + (double)t.tv_nsec * 1e-3;
}

/* n_certs certificates of per_cert signatures (certificate c = entries
 * [c * per_cert, (c + 1) * per_cert)); out_us[c] = wall time of call c,
 * out_acc[c] = its accepted count (UINT64_MAX if the call failed); when
 * stamps != NULL, out_stamps[8c .. 8c + 7] = pbftv_qc_stamps after call c.
 * Returns the number of failed calls. */
int qc_drive(void* verify, void* stamps, void* ctx, const uint8_t* hashes, const uint8_t* sigs, const uint32_t* kidx,
             uint64_t n_certs, uint32_t per_cert, uint32_t quorum, double gap_us, double* out_us, uint64_t* out_acc,
             uint64_t* out_stamps) {
  qc_verify_fn fn = (qc_verify_fn)verify;
  qc_stamps_fn st = (qc_stamps_fn)stamps;
  uint8_t bm[1024];
  int failed = 0;
  if (per_cert > 8 * sizeof(bm)) return -1;
  for (uint64_t c = 0; c < n_certs; ++c) {
    if (gap_us > 0) {
      struct timespec ts;
      ts.tv_sec = (time_t)(gap_us / 1e6);
      ts.tv_nsec = (long)((gap_us - (double)ts.tv_sec * 1e6) * 1e3);
      nanosleep(&ts, NULL);
    }
    uint64_t acc = 0;
    int q = 0;
    const double t0 = now_us();
    const int rc = fn(ctx, hashes + 32 * c * per_cert, sigs + 64 * c * per_cert, kidx + c * per_cert, per_cert, quorum,
                      bm, &acc, &q);
    out_us[c] = now_us() - t0;
    out_acc[c] = rc == 0 ? acc : UINT64_MAX;
    failed += rc != 0;
    if (st && out_stamps) {
      if (st(ctx, 0, out_stamps + 8 * c) != 0) memset(out_stamps + 8 * c, 0, 8 * sizeof(uint64_t));
    }
  }
  return failed;
}

/* The single-call drop-ins, timed the same way (bench.py single_calls_us):
 * pbftv_hash_hex (utils.Hash, utils/utils.go:13-17, called once per request
 * at pbft_impl.go:73) on one message, reps calls, out_us[i] each call's wall
 * time; out_hex = the last digest.  Returns the number of failed calls. */
typedef int (*hash_hex_fn)(void* ctx, const uint8_t* content, uint64_t len, char out_hex[65]);
int hash_drive(void* fn, void* ctx, const uint8_t* msg, uint64_t len, uint32_t reps, double* out_us, char* out_hex) {
  hash_hex_fn h = (hash_hex_fn)fn;
  int failed = 0;
  for (uint32_t i = 0; i < reps; ++i) {
    const double t0 = now_us();
    failed += h(ctx, msg, len, out_hex) != 0;
    out_us[i] = now_us() - t0;
  }
  return failed;
}

/* pbftv_verify_msg_batch at n = 1 (State.verifyMsg, pbft_impl.go:176-202, for
 * one vote): host code, no device. */
typedef int (*vmsg_fn)(int64_t view, int64_t last, const uint8_t* req_digest, uint64_t n, const int64_t* views,
                       const int64_t* seqs, const char* got, const uint64_t* got_off, const uint32_t* got_len,
                       uint8_t* out_bitmap);
int vmsg_drive(void* fn, const uint8_t* req_digest, const char* hex64, uint32_t reps, double* out_us) {
  vmsg_fn v = (vmsg_fn)fn;
  int64_t view = 0, seq = 7;
  uint64_t off = 0;
  uint32_t len = 64;
  uint8_t bm[8];
  int bad = 0;
  for (uint32_t i = 0; i < reps; ++i) {
    const double t0 = now_us();
    bad += v(0, 6, req_digest, 1, &view, &seq, hex64, &off, &len, bm) != 0 || (bm[0] & 1) != 1;
    out_us[i] = now_us() - t0;
  }
  return bad;
}
