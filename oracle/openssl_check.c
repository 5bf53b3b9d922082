/*
 * openssl_check.c — independent third-party checker (TEST INFRASTRUCTURE ONLY).
 *
 * OpenSSL 3 `ECDSA_do_verify` on secp256k1 (NID 714) behind a semantic
 * adapter that maps OpenSSL's rules onto the reference's (SURVEY.md §8(c)
 * "Secondary cross-check"):
 *   - compact parse (secp256k1_ecdsa_signature_parse_compact, a5): r or
 *     s >= n rejects before OpenSSL sees it;
 *   - high-S (a3 step 1 / a1 normalizeSig): OpenSSL accepts high S, so
 *     HKV_LIBSECP pre-rejects s > n/2 and HKV_HASKOIN replaces s by n - s;
 *   - pubkey (secp256k1_ec_pubkey_parse, a4): only lengths 33 (02/03) and 65
 *     (04/06/07) reach EC_POINT_oct2point, which then does the range,
 *     on-curve, square-root and hybrid-parity checks itself (OpenSSL would
 *     otherwise also accept the 1-byte 0x00 infinity encoding);
 *   - ECDSA_do_verify returns 1 / 0 / -1; anything but 1 is a reject (it
 *     returns -1 where libsecp256k1 returns 0 for u1*G + u2*Q = infinity).
 *
 * Used (1) by tests/ as an implementation-independent pin of the GPU verdicts
 * at scale and of the Python/C restatements on the golden KATs, and (2) by
 * bench.py's cpu_baseline leg as the labelled NON-reference CPU fallback the
 * survey prescribes when libsecp256k1 is absent on the GPU box (§8(d)).
 * The product path (haskoin-node_amd/) never links or loads it.
 */
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/obj_mac.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>

#define REC 168

static const uint8_t N_BE[32] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                 0xFF, 0xFF, 0xFF, 0xFF, 0xFE, 0xBA, 0xAE, 0xDC, 0xE6, 0xAF, 0x48,
                                 0xA0, 0x3B, 0xBF, 0xD2, 0x5E, 0x8C, 0xD0, 0x36, 0x41, 0x41};
static const uint8_t HALF_N_BE[32] = {0x7F, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                      0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0x5D, 0x57, 0x6E, 0x73, 0x57, 0xA4,
                                      0x50, 0x1D, 0xDF, 0xE9, 0x2F, 0x46, 0x68, 0x1B, 0x20, 0xA0};

/* big-endian 256-bit compare */
static int cmp_be(const uint8_t* a, const uint8_t* b) { return memcmp(a, b, 32); }
static int is_zero_be(const uint8_t* a) {
  uint8_t o = 0;
  for (int i = 0; i < 32; ++i) o |= a[i];
  return o == 0;
}
/* r = n - a (0 < a < n), big-endian */
static void neg_mod_n_be(uint8_t* r, const uint8_t* a) {
  int borrow = 0;
  for (int i = 31; i >= 0; --i) {
    int d = (int)N_BE[i] - (int)a[i] - borrow;
    borrow = d < 0;
    r[i] = (uint8_t)(d + (borrow ? 256 : 0));
  }
}

typedef struct {
  EC_KEY* key;
  const EC_GROUP* grp;
  EC_POINT* pt;
  ECDSA_SIG* sig;
  BN_CTX* bn;
} ossl_state;

static int state_init(ossl_state* st) {
  st->key = EC_KEY_new_by_curve_name(NID_secp256k1);
  if (!st->key) return 0;
  st->grp = EC_KEY_get0_group(st->key);
  st->pt = EC_POINT_new(st->grp);
  st->sig = ECDSA_SIG_new();
  st->bn = BN_CTX_new();
  return st->pt && st->sig && st->bn;
}
static void state_free(ossl_state* st) {
  if (st->sig) ECDSA_SIG_free(st->sig);
  if (st->pt) EC_POINT_free(st->pt);
  if (st->key) EC_KEY_free(st->key);
  if (st->bn) BN_CTX_free(st->bn);
}

static int verify_one(ossl_state* st, const uint8_t* rec, int mode) {
  const uint8_t* msg = rec;
  const uint8_t* r = rec + 32;
  uint8_t s[32];
  memcpy(s, rec + 64, 32);
  if (cmp_be(r, N_BE) >= 0 || cmp_be(s, N_BE) >= 0) return 0; /* compact parse overflow */
  if (is_zero_be(r) || is_zero_be(s)) return 0;
  if (cmp_be(s, HALF_N_BE) > 0) {
    if (mode == 0) return 0; /* secp256k1_ecdsa_verify rejects high S */
    neg_mod_n_be(s, s);      /* verifyHashSig: normalizeSig first */
  }
  const unsigned len = rec[96];
  const uint8_t pre = rec[97];
  if (!((len == 33 && (pre == 2 || pre == 3)) || (len == 65 && (pre == 4 || pre == 6 || pre == 7)))) return 0;
  if (EC_POINT_oct2point(st->grp, st->pt, rec + 97, len, st->bn) != 1) return 0;
  if (EC_KEY_set_public_key(st->key, st->pt) != 1) return 0;
  BIGNUM* br = BN_bin2bn(r, 32, NULL);
  BIGNUM* bs = BN_bin2bn(s, 32, NULL);
  if (!br || !bs || ECDSA_SIG_set0(st->sig, br, bs) != 1) {
    BN_free(br);
    BN_free(bs);
    return 0;
  }
  return ECDSA_do_verify(msg, 32, st->sig, st->key) == 1;
}

int hkvo_openssl_verify_record(const uint8_t* rec, int mode) {
  ossl_state st = {0};
  int ok = state_init(&st) ? verify_one(&st, rec, mode) : -1;
  state_free(&st);
  return ok;
}

typedef struct {
  const uint8_t* recs;
  size_t lo, hi;
  int mode;
  uint8_t* out;
  int err;
} job;

static void* worker(void* arg) {
  job* j = (job*)arg;
  ossl_state st = {0};
  if (!state_init(&st)) {
    j->err = 1;
  } else {
    for (size_t i = j->lo; i < j->hi; ++i) j->out[i] = (uint8_t)verify_one(&st, j->recs + i * REC, j->mode);
  }
  state_free(&st);
  return NULL;
}

/* Verdicts of n records (include/hkv.h layout) on `threads` pthreads.
 * Returns 0, or -1 if OpenSSL could not build a secp256k1 key. */
int hkvo_openssl_verify_batch(const uint8_t* recs, size_t n, int mode, uint8_t* out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  job jobs[256];
  const size_t per = (n + (size_t)threads - 1) / (size_t)threads;
  int started[256] = {0}, err = 0;
  for (int t = 0; t < threads; ++t) {
    size_t lo = (size_t)t * per, hi = lo + per;
    if (lo > n) lo = n;
    if (hi > n) hi = n;
    jobs[t] = (job){recs, lo, hi, mode, out, 0};
    if (pthread_create(&tid[t], NULL, worker, &jobs[t]) == 0) {
      started[t] = 1;
    } else {
      worker(&jobs[t]); /* run inline when no thread is available */
      err |= jobs[t].err;
    }
  }
  for (int t = 0; t < threads; ++t)
    if (started[t] && pthread_join(tid[t], NULL) == 0) err |= jobs[t].err;
  return err ? -1 : 0;
}
