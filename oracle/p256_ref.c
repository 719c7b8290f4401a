/* p256_ref.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * ECDSA-P256 verification restating Go 1.19 crypto/ecdsa.Verify (the parity
 * target; the reference itself has no signature code -- 需要改进的地方.md:17,
 * SURVEY.md §8 a10).  go1.19 ecdsa.go:
 *     Verify:        r,s must satisfy 0 < r,s < N, else false
 *     verifyGeneric: e = hashToInt(hash); w = s^-1 mod N; u1 = e*w mod N;
 *                    u2 = r*w mod N; (x,y) = u1*G + u2*Q;
 *                    (x,y) == (0,0) (infinity) -> false; return x mod N == r
 * Key validity is checked at registration (go1.19 panics on off-curve points).
 *
 * Deliberately a DIFFERENT algorithm from the GPU kernel so that the two are
 * independent: 4 x 64-bit limbs, generic Montgomery (CIOS) for both p and n,
 * Jacobian coordinates, bit-serial Shamir double-and-add with a complete
 * addition (doubling / inverse / infinity all handled), Fermat inversion.
 */
#include "oracle.h"

#include <pthread.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[4]; } u256;
typedef struct { u256 m; uint64_t minv; u256 r2; } mont_t;  /* minv = -m^-1 mod 2^64 */

static const u256 P_ = {{0xFFFFFFFFFFFFFFFFull, 0x00000000FFFFFFFFull, 0x0000000000000000ull, 0xFFFFFFFF00000001ull}};
static const u256 N_ = {{0xF3B9CAC2FC632551ull, 0xBCE6FAADA7179E84ull, 0xFFFFFFFFFFFFFFFFull, 0xFFFFFFFF00000000ull}};
static const u256 B_ = {{0x3BCE3C3E27D2604Bull, 0x651D06B0CC53B0F6ull, 0xB3EBBD55769886BCull, 0x5AC635D8AA3A93E7ull}};
static const u256 GX_ = {{0xF4A13945D898C296ull, 0x77037D812DEB33A0ull, 0xF8BCE6E563A440F2ull, 0x6B17D1F2E12C4247ull}};
static const u256 GY_ = {{0xCBB6406837BF51F5ull, 0x2BCE33576B315ECEull, 0x8EE7EB4A7C0F9E16ull, 0x4FE342E2FE1A7F9Bull}};

static int cmp(const u256* a, const u256* b) {
  for (int i = 3; i >= 0; --i) { if (a->v[i] != b->v[i]) return a->v[i] < b->v[i] ? -1 : 1; }
  return 0;
}
static int is_zero(const u256* a) { return !(a->v[0] | a->v[1] | a->v[2] | a->v[3]); }
static uint64_t add_raw(u256* r, const u256* a, const u256* b) {
  u128 c = 0;
  for (int i = 0; i < 4; ++i) { c += (u128)a->v[i] + b->v[i]; r->v[i] = (uint64_t)c; c >>= 64; }
  return (uint64_t)c;
}
static uint64_t sub_raw(u256* r, const u256* a, const u256* b) {
  uint64_t br = 0;
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)a->v[i] - b->v[i] - br;
    r->v[i] = (uint64_t)d;
    br = (uint64_t)(d >> 127);  /* 1 if borrowed */
  }
  return br;
}
/* r = a + b mod m (a, b < m) */
static void addm(u256* r, const u256* a, const u256* b, const u256* m) {
  u256 t; uint64_t c = add_raw(&t, a, b);
  if (c || cmp(&t, m) >= 0) sub_raw(&t, &t, m);
  *r = t;
}
static void subm(u256* r, const u256* a, const u256* b, const u256* m) {
  u256 t; uint64_t br = sub_raw(&t, a, b);
  if (br) add_raw(&t, &t, m);
  *r = t;
}
/* CIOS Montgomery multiplication: r = a*b*2^-256 mod m */
static void mulm(u256* r, const u256* a, const u256* b, const mont_t* M) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) { c += (u128)a->v[j] * b->v[i] + t[j]; t[j] = (uint64_t)c; c >>= 64; }
    c += t[4]; t[4] = (uint64_t)c; t[5] = (uint64_t)(c >> 64);
    uint64_t q = t[0] * M->minv;
    c = (u128)q * M->m.v[0] + t[0]; c >>= 64;
    for (int j = 1; j < 4; ++j) { c += (u128)q * M->m.v[j] + t[j]; t[j - 1] = (uint64_t)c; c >>= 64; }
    c += t[4]; t[3] = (uint64_t)c; t[4] = t[5] + (uint64_t)(c >> 64);
  }
  u256 res = {{t[0], t[1], t[2], t[3]}};
  if (t[4] || cmp(&res, &M->m) >= 0) sub_raw(&res, &res, &M->m);
  *r = res;
}
static void to_mont(u256* r, const u256* a, const mont_t* M) { mulm(r, a, &M->r2, M); }
static void from_mont(u256* r, const u256* a, const mont_t* M) { u256 one = {{1, 0, 0, 0}}; mulm(r, a, &one, M); }

static void mont_init(mont_t* M, const u256* m) {
  M->m = *m;
  uint64_t inv = 1;  /* Newton: inv = m0^-1 mod 2^64 */
  for (int i = 0; i < 7; ++i) inv *= 2 - m->v[0] * inv;
  M->minv = (uint64_t)0 - inv;
  /* r2 = 2^512 mod m by doubling 1 512 times */
  u256 x = {{1, 0, 0, 0}};
  for (int i = 0; i < 512; ++i) addm(&x, &x, &x, m);
  M->r2 = x;
}

static mont_t MP, MN;
static u256 P_B, P_A, P_GX, P_GY, P_ONE;  /* Montgomery-domain constants */
static pthread_once_t once = PTHREAD_ONCE_INIT;

static void init_consts(void) {
  mont_init(&MP, &P_);
  mont_init(&MN, &N_);
  u256 one = {{1, 0, 0, 0}}, three = {{3, 0, 0, 0}}, a;
  subm(&a, &P_, &three, &P_);  /* a = -3 mod p (p - 3) */
  to_mont(&P_ONE, &one, &MP);
  to_mont(&P_A, &a, &MP);
  to_mont(&P_B, &B_, &MP);
  to_mont(&P_GX, &GX_, &MP);
  to_mont(&P_GY, &GY_, &MP);
}

/* a^e mod m (Montgomery domain in/out), e plain big integer */
static void powm(u256* r, const u256* a, const u256* e, const mont_t* M, const u256* one_m) {
  u256 acc = *one_m;
  for (int i = 255; i >= 0; --i) {
    mulm(&acc, &acc, &acc, M);
    if ((e->v[i / 64] >> (i % 64)) & 1) mulm(&acc, &acc, a, M);
  }
  *r = acc;
}

static void load_be(u256* r, const uint8_t b[32]) {
  for (int i = 0; i < 4; ++i) {
    uint64_t w = 0;
    for (int j = 0; j < 8; ++j) w = (w << 8) | b[(3 - i) * 8 + j];
    r->v[i] = w;
  }
}
static void store_be(uint8_t b[32], const u256* a) {
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) b[(3 - i) * 8 + j] = (uint8_t)(a->v[i] >> (56 - 8 * j));
}

/* ---- Jacobian points over p (Montgomery domain); Z == 0 is infinity ---- */
typedef struct { u256 x, y, z; } jac;

static void jdouble(jac* r, const jac* p) {
  if (is_zero(&p->z) || is_zero(&p->y)) { memset(r, 0, sizeof *r); return; }
  /* dbl-2001-b (a = -3): delta=Z^2, gamma=Y^2, beta=X*gamma, alpha=3(X-delta)(X+delta) */
  u256 delta, gamma, beta, alpha, t1, t2, x3, y3, z3;
  mulm(&delta, &p->z, &p->z, &MP);
  mulm(&gamma, &p->y, &p->y, &MP);
  mulm(&beta, &p->x, &gamma, &MP);
  subm(&t1, &p->x, &delta, &P_);
  addm(&t2, &p->x, &delta, &P_);
  mulm(&alpha, &t1, &t2, &MP);
  addm(&t1, &alpha, &alpha, &P_);
  addm(&alpha, &t1, &alpha, &P_);
  mulm(&x3, &alpha, &alpha, &MP);                  /* alpha^2 */
  addm(&t1, &beta, &beta, &P_);                    /* 2beta */
  addm(&t1, &t1, &t1, &P_);                        /* 4beta */
  addm(&t2, &t1, &t1, &P_);                        /* 8beta */
  subm(&x3, &x3, &t2, &P_);
  addm(&t2, &p->y, &p->z, &P_);
  mulm(&z3, &t2, &t2, &MP);
  subm(&z3, &z3, &gamma, &P_);
  subm(&z3, &z3, &delta, &P_);
  subm(&t1, &t1, &x3, &P_);                        /* 4beta - X3 */
  mulm(&y3, &alpha, &t1, &MP);
  mulm(&t2, &gamma, &gamma, &MP);
  addm(&t2, &t2, &t2, &P_); addm(&t2, &t2, &t2, &P_); addm(&t2, &t2, &t2, &P_);  /* 8gamma^2 */
  subm(&y3, &y3, &t2, &P_);
  r->x = x3; r->y = y3; r->z = z3;
}

/* complete Jacobian addition */
static void jadd(jac* r, const jac* p, const jac* q) {
  if (is_zero(&p->z)) { *r = *q; return; }
  if (is_zero(&q->z)) { *r = *p; return; }
  u256 z1z1, z2z2, u1, u2, s1, s2, h, rr, t;
  mulm(&z1z1, &p->z, &p->z, &MP);
  mulm(&z2z2, &q->z, &q->z, &MP);
  mulm(&u1, &p->x, &z2z2, &MP);
  mulm(&u2, &q->x, &z1z1, &MP);
  mulm(&t, &q->z, &z2z2, &MP); mulm(&s1, &p->y, &t, &MP);
  mulm(&t, &p->z, &z1z1, &MP); mulm(&s2, &q->y, &t, &MP);
  subm(&h, &u2, &u1, &P_);
  subm(&rr, &s2, &s1, &P_);
  if (is_zero(&h)) {
    if (is_zero(&rr)) { jdouble(r, p); return; }
    memset(r, 0, sizeof *r); return;  /* P + (-P) = infinity */
  }
  u256 hh, hhh, v, x3, y3, z3;
  mulm(&hh, &h, &h, &MP);
  mulm(&hhh, &hh, &h, &MP);
  mulm(&v, &u1, &hh, &MP);
  mulm(&x3, &rr, &rr, &MP);
  subm(&x3, &x3, &hhh, &P_);
  subm(&x3, &x3, &v, &P_);
  subm(&x3, &x3, &v, &P_);
  subm(&t, &v, &x3, &P_);
  mulm(&y3, &rr, &t, &MP);
  mulm(&t, &s1, &hhh, &MP);
  subm(&y3, &y3, &t, &P_);
  mulm(&z3, &p->z, &q->z, &MP);
  mulm(&z3, &z3, &h, &MP);
  r->x = x3; r->y = y3; r->z = z3;
}

static int to_affine(const jac* p, u256* x, u256* y) {
  if (is_zero(&p->z)) return 0;
  u256 e, zi, zi2, zi3, t;
  sub_raw(&e, &P_, &(u256){{2, 0, 0, 0}});
  powm(&zi, &p->z, &e, &MP, &P_ONE);
  mulm(&zi2, &zi, &zi, &MP);
  mulm(&zi3, &zi2, &zi, &MP);
  mulm(&t, &p->x, &zi2, &MP); from_mont(x, &t, &MP);
  mulm(&t, &p->y, &zi3, &MP); from_mont(y, &t, &MP);
  return 1;
}

static int on_curve_mont(const u256* x, const u256* y) {
  u256 lhs, rhs, t;
  mulm(&lhs, y, y, &MP);
  mulm(&t, x, x, &MP);
  addm(&t, &t, &P_A, &P_);
  mulm(&rhs, &t, x, &MP);       /* x^3 + a x */
  addm(&rhs, &rhs, &P_B, &P_);
  return cmp(&lhs, &rhs) == 0;
}

int oracle_p256_key_valid(const uint8_t pub[64]) {
  pthread_once(&once, init_consts);
  u256 x, y, xm, ym;
  load_be(&x, pub); load_be(&y, pub + 32);
  if (cmp(&x, &P_) >= 0 || cmp(&y, &P_) >= 0) return 0;
  to_mont(&xm, &x, &MP); to_mont(&ym, &y, &MP);
  return on_curve_mont(&xm, &ym);
}

/* u1*G + u2*Q by joint bit-serial double-and-add (Shamir's trick) */
static void shamir(jac* r, const u256* u1, const u256* u2, const jac* g, const jac* q) {
  jac gq, acc;
  jadd(&gq, g, q);
  memset(&acc, 0, sizeof acc);
  for (int i = 255; i >= 0; --i) {
    jdouble(&acc, &acc);
    int b1 = (u1->v[i / 64] >> (i % 64)) & 1, b2 = (u2->v[i / 64] >> (i % 64)) & 1;
    if (b1 && b2) jadd(&acc, &acc, &gq);
    else if (b1) jadd(&acc, &acc, g);
    else if (b2) jadd(&acc, &acc, q);
  }
  *r = acc;
}

int oracle_ecdsa_p256_verify(const uint8_t hash[32], const uint8_t sig[64], const uint8_t pub[64]) {
  pthread_once(&once, init_consts);
  if (!oracle_p256_key_valid(pub)) return 0;
  u256 r, s, e;
  load_be(&r, sig); load_be(&s, sig + 32);
  if (is_zero(&r) || is_zero(&s) || cmp(&r, &N_) >= 0 || cmp(&s, &N_) >= 0) return 0;  /* Verify range checks */
  load_be(&e, hash);                                       /* hashToInt: 32-byte hash, no truncation */
  u256 one_n, sm, w, em, rm, u1m, u2m, u1, u2, nm2, two = {{2, 0, 0, 0}}, one = {{1, 0, 0, 0}};
  to_mont(&one_n, &one, &MN);
  to_mont(&sm, &s, &MN);
  sub_raw(&nm2, &N_, &two);
  powm(&w, &sm, &nm2, &MN, &one_n);                        /* w = s^(n-2) = s^-1 */
  /* e may be >= n: to_mont reduces (Montgomery mult by R^2 handles e < 2^256 < 2n) */
  u256 ered = e;
  if (cmp(&ered, &N_) >= 0) sub_raw(&ered, &ered, &N_);
  to_mont(&em, &ered, &MN);
  to_mont(&rm, &r, &MN);
  mulm(&u1m, &em, &w, &MN); from_mont(&u1, &u1m, &MN);
  mulm(&u2m, &rm, &w, &MN); from_mont(&u2, &u2m, &MN);
  jac g = {P_GX, P_GY, P_ONE}, q, R;
  u256 qx, qy;
  load_be(&qx, pub); load_be(&qy, pub + 32);
  to_mont(&q.x, &qx, &MP); to_mont(&q.y, &qy, &MP); q.z = P_ONE;
  shamir(&R, &u1, &u2, &g, &q);
  u256 x, y;
  if (!to_affine(&R, &x, &y)) return 0;                    /* infinity -> false */
  if (cmp(&x, &N_) >= 0) sub_raw(&x, &x, &N_);             /* x mod N (x < p < 2N) */
  return cmp(&x, &r) == 0;
}

int oracle_p256_pubkey(const uint8_t d[32], uint8_t out[64]) {
  pthread_once(&once, init_consts);
  u256 k, zero = {{0, 0, 0, 0}};
  load_be(&k, d);
  if (cmp(&k, &N_) >= 0) sub_raw(&k, &k, &N_);
  if (is_zero(&k)) return 0;
  jac g = {P_GX, P_GY, P_ONE}, R, dummy = {zero, zero, zero};
  shamir(&R, &k, &zero, &g, &dummy);
  u256 x, y;
  if (!to_affine(&R, &x, &y)) return 0;
  store_be(out, &x); store_be(out + 32, &y);
  return 1;
}

int oracle_ecdsa_p256_sign(const uint8_t hash[32], const uint8_t d[32], const uint8_t kb[32], uint8_t out[64]) {
  pthread_once(&once, init_consts);
  uint8_t rxy[64];
  if (!oracle_p256_pubkey(kb, rxy)) return 0;
  u256 r, k, dd, e, one = {{1, 0, 0, 0}}, two = {{2, 0, 0, 0}};
  load_be(&r, rxy);
  if (cmp(&r, &N_) >= 0) sub_raw(&r, &r, &N_);
  if (is_zero(&r)) return 0;
  load_be(&k, kb); load_be(&dd, d); load_be(&e, hash);
  if (cmp(&k, &N_) >= 0) sub_raw(&k, &k, &N_);
  if (cmp(&dd, &N_) >= 0) sub_raw(&dd, &dd, &N_);
  if (cmp(&e, &N_) >= 0) sub_raw(&e, &e, &N_);
  u256 one_n, km, kinv, nm2, rm, dm, em, t, s;
  to_mont(&one_n, &one, &MN);
  to_mont(&km, &k, &MN);
  sub_raw(&nm2, &N_, &two);
  powm(&kinv, &km, &nm2, &MN, &one_n);
  to_mont(&rm, &r, &MN); to_mont(&dm, &dd, &MN); to_mont(&em, &e, &MN);
  mulm(&t, &rm, &dm, &MN);
  addm(&t, &t, &em, &N_);
  mulm(&t, &t, &kinv, &MN);
  from_mont(&s, &t, &MN);
  if (is_zero(&s)) return 0;
  store_be(out, &r); store_be(out + 32, &s);
  return 1;
}

typedef struct {
  const uint8_t *hashes, *sigs, *keys; const uint32_t* key_idx; uint32_t nkeys;
  uint8_t* bits; uint64_t lo, hi;
} ec_job;

static void* ec_worker(void* arg) {
  ec_job* j = (ec_job*)arg;
  for (uint64_t i = j->lo; i < j->hi; ++i) {
    uint32_t k = j->key_idx[i];
    int ok = (k < j->nkeys) && oracle_ecdsa_p256_verify(j->hashes + 32 * i, j->sigs + 64 * i, j->keys + 64 * (uint64_t)k);
    if (ok) j->bits[i / 8] |= (uint8_t)(1u << (i % 8));
  }
  return NULL;
}

void oracle_ecdsa_p256_verify_batch(const uint8_t* hashes, const uint8_t* sigs, const uint32_t* key_idx, uint64_t n,
                                    const uint8_t* keys, uint32_t nkeys, uint8_t* bits, int nthreads) {
  pthread_once(&once, init_consts);
  memset(bits, 0, (n + 7) / 8);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  ec_job jobs[256];
  for (int t = 0; t < nthreads; ++t) {
    /* split on byte boundaries so threads never share a bitmap byte */
    uint64_t nb = (n + 7) / 8;
    uint64_t lo = 8 * (nb * t / nthreads), hi = 8 * (nb * (t + 1) / nthreads);
    if (hi > n) hi = n;
    if (lo > n) lo = n;
    jobs[t] = (ec_job){hashes, sigs, keys, key_idx, nkeys, bits, lo, hi};
    if (nthreads == 1) ec_worker(&jobs[t]); else pthread_create(&th[t], NULL, ec_worker, &jobs[t]);
  }
  if (nthreads > 1) for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}
