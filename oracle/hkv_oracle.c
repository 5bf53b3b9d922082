/*
 * hkv_oracle.c — CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * Plain-C restatement of the reference hot path's verify semantics, used by
 * tests/ as the checker for large batches and by bench.py's cpu_baseline leg
 * (kind "port"). The product path (haskoin-node_amd/) never links or loads it.
 *
 * Semantics restated (all [dep] — un-vendored, pinned at
 * /root/reference/stack.yaml:8-10 and stack.yaml.lock:7-20):
 *   hkvo_pubkey_parse  <- libsecp256k1 secp256k1_ec_pubkey_parse (a4)
 *   sig compact parse  <- secp256k1_ecdsa_signature_parse_compact (a5)
 *   normalize          <- secp256k1_ecdsa_signature_normalize (a6)
 *   verify             <- secp256k1_ecdsa_verify / secp256k1_ecdsa_sig_verify (a3)
 *   HASKOIN mode       <- haskoin-core Haskoin.Crypto.Signature.verifyHashSig (a1)
 *
 * Deliberately a DIFFERENT algorithm from the GPU kernels so that it checks
 * them independently: no GLV split, no fixed windows, no isomorphic-curve
 * table, no inversion-free x compare. u1*G + u2*Q is a Strauss-Shamir
 * double-scalar multiply over full 256-bit wNAF(w=5) digits with complete
 * (degenerate-case-handling) Jacobian additions; the result is converted to
 * affine by a field inversion and its x compared with r and r+n.
 * Field and scalar elements are kept fully reduced after every operation.
 *
 * Parity status: unpinned by the reference (its fixtures hold no
 * signatures); cross-checked against the Python restatement and against
 * OpenSSL 3.0.2 in tests/test_oracle.py.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[4]; } fe;   /* little-endian 64-bit limbs, < p */
typedef struct { uint64_t v[4]; } sc;   /* little-endian 64-bit limbs, < n */

static const fe FE_P = {{0xFFFFFFFEFFFFFC2FULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL}};
static const sc SC_N = {{0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL}};
static const sc SC_HALF_N = {{0xDFE92F46681B20A0ULL, 0x5D576E7357A4501DULL, 0xFFFFFFFFFFFFFFFFULL, 0x7FFFFFFFFFFFFFFFULL}};
/* 2^256 - n */
static const uint64_t SC_C[3] = {0x402DA1732FC9BEBFULL, 0x4551231950B75FC4ULL, 0x1ULL};
static const fe FE_GX = {{0x59F2815B16F81798ULL, 0x029BFCDB2DCE28D9ULL, 0x55A06295CE870B07ULL, 0x79BE667EF9DCBBACULL}};
static const fe FE_GY = {{0x9C47D08FFB10D4B8ULL, 0xFD17B448A6855419ULL, 0x5DA4FBFC0E1108A8ULL, 0x483ADA7726A3C465ULL}};

/* ---------------- 256-bit helpers ---------------- */
static int u256_cmp(const uint64_t* a, const uint64_t* b) {
  for (int i = 3; i >= 0; --i) { if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1; }
  return 0;
}
static uint64_t u256_add(uint64_t* r, const uint64_t* a, const uint64_t* b) {
  u128 c = 0;
  for (int i = 0; i < 4; ++i) { c += (u128)a[i] + b[i]; r[i] = (uint64_t)c; c >>= 64; }
  return (uint64_t)c;
}
static uint64_t u256_sub(uint64_t* r, const uint64_t* a, const uint64_t* b) {
  uint64_t borrow = 0;
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)a[i] - b[i] - borrow;
    r[i] = (uint64_t)d;
    borrow = (uint64_t)(d >> 64) ? 1 : 0;
  }
  return borrow;
}
static int u256_is_zero(const uint64_t* a) { return (a[0] | a[1] | a[2] | a[3]) == 0; }
static void u256_from_be(uint64_t* r, const uint8_t* b) {
  for (int i = 0; i < 4; ++i) {
    uint64_t w = 0;
    for (int j = 0; j < 8; ++j) w = (w << 8) | b[(3 - i) * 8 + j];
    r[i] = w;
  }
}

/* ---------------- field mod p ---------------- */
static void fe_add(fe* r, const fe* a, const fe* b) {
  uint64_t c = u256_add(r->v, a->v, b->v);
  if (c || u256_cmp(r->v, FE_P.v) >= 0) u256_sub(r->v, r->v, FE_P.v);
}
static void fe_sub(fe* r, const fe* a, const fe* b) {
  if (u256_sub(r->v, a->v, b->v)) u256_add(r->v, r->v, FE_P.v);
}
static void fe_neg(fe* r, const fe* a) {
  fe z = {{0, 0, 0, 0}};
  fe_sub(r, &z, a);
}
/* reduce an 8-limb product: 2^256 = 0x1000003D1 (mod p) */
static void fe_reduce512(fe* r, const uint64_t t[8]) {
  const uint64_t C = 0x1000003D1ULL;
  uint64_t s[5];
  u128 acc = 0;
  for (int i = 0; i < 4; ++i) { acc += (u128)t[4 + i] * C + t[i]; s[i] = (uint64_t)acc; acc >>= 64; }
  s[4] = (uint64_t)acc;                       /* < 2^34 */
  acc = (u128)s[4] * C + s[0];
  r->v[0] = (uint64_t)acc; acc >>= 64;
  for (int i = 1; i < 4; ++i) { acc += s[i]; r->v[i] = (uint64_t)acc; acc >>= 64; }
  if (acc) { /* wrapped past 2^256: add C once more (cannot wrap again) */
    u128 c2 = (u128)r->v[0] + C; r->v[0] = (uint64_t)c2; c2 >>= 64;
    for (int i = 1; i < 4 && c2; ++i) { c2 += r->v[i]; r->v[i] = (uint64_t)c2; c2 >>= 64; }
  }
  if (u256_cmp(r->v, FE_P.v) >= 0) u256_sub(r->v, r->v, FE_P.v);
}
static void mul256(uint64_t t[8], const uint64_t* a, const uint64_t* b) {
  memset(t, 0, 8 * sizeof(uint64_t));
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) { c += (u128)a[i] * b[j] + t[i + j]; t[i + j] = (uint64_t)c; c >>= 64; }
    t[i + 4] = (uint64_t)c;
  }
}
static void fe_mul(fe* r, const fe* a, const fe* b) { uint64_t t[8]; mul256(t, a->v, b->v); fe_reduce512(r, t); }
static void fe_sqr(fe* r, const fe* a) { fe_mul(r, a, a); }
static int fe_is_zero(const fe* a) { return u256_is_zero(a->v); }
static int fe_eq(const fe* a, const fe* b) { return u256_cmp(a->v, b->v) == 0; }
/* generic 4-bit fixed-window exponentiation */
static void fe_pow(fe* r, const fe* a, const uint64_t e[4]) {
  fe tab[16];
  tab[0] = (fe){{1, 0, 0, 0}};
  tab[1] = *a;
  for (int i = 2; i < 16; ++i) fe_mul(&tab[i], &tab[i - 1], a);
  fe acc = tab[0];
  for (int w = 63; w >= 0; --w) {
    for (int k = 0; k < 4; ++k) fe_sqr(&acc, &acc);
    int d = (int)((e[w / 16] >> ((w % 16) * 4)) & 15);
    if (d) fe_mul(&acc, &acc, &tab[d]);
  }
  *r = acc;
}
static void fe_inv(fe* r, const fe* a) {
  static const uint64_t E[4] = {0xFFFFFFFEFFFFFC2DULL, ~0ULL, ~0ULL, ~0ULL};
  fe_pow(r, a, E);
}
static void fe_sqrt_cand(fe* r, const fe* a) {   /* a^((p+1)/4) */
  static const uint64_t E[4] = {0xFFFFFFFFBFFFFF0CULL, ~0ULL, ~0ULL, 0x3FFFFFFFFFFFFFFFULL};
  fe_pow(r, a, E);
}

/* ---------------- scalar mod n ---------------- */
static void sc_reduce512(sc* r, const uint64_t tin[8]) {
  uint64_t t[9]; memcpy(t, tin, 8 * sizeof(uint64_t)); t[8] = 0;
  /* fold high part: t = lo + hi * C  until hi == 0 */
  for (;;) {
    uint64_t hi[5] = {t[4], t[5], t[6], t[7], t[8]};
    if ((hi[0] | hi[1] | hi[2] | hi[3] | hi[4]) == 0) break;
    uint64_t prod[9] = {0};
    for (int i = 0; i < 5; ++i) {
      u128 c = 0;
      for (int j = 0; j < 3; ++j) { c += (u128)hi[i] * SC_C[j] + prod[i + j]; prod[i + j] = (uint64_t)c; c >>= 64; }
      for (int k = i + 3; k < 9 && c; ++k) { c += prod[k]; prod[k] = (uint64_t)c; c >>= 64; }
    }
    u128 c = 0;
    for (int i = 0; i < 9; ++i) { c += (u128)prod[i] + (i < 4 ? t[i] : 0); t[i] = (uint64_t)c; c >>= 64; }
  }
  memcpy(r->v, t, 32);
  while (u256_cmp(r->v, SC_N.v) >= 0) u256_sub(r->v, r->v, SC_N.v);
}
static void sc_mul(sc* r, const sc* a, const sc* b) { uint64_t t[8]; mul256(t, a->v, b->v); sc_reduce512(r, t); }
static void sc_inv(sc* r, const sc* a) {
  static const uint64_t E[4] = {0xBFD25E8CD036413FULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL};
  sc tab[16];
  tab[0] = (sc){{1, 0, 0, 0}};
  tab[1] = *a;
  for (int i = 2; i < 16; ++i) sc_mul(&tab[i], &tab[i - 1], a);
  sc acc = tab[0];
  for (int w = 63; w >= 0; --w) {
    for (int k = 0; k < 4; ++k) sc_mul(&acc, &acc, &acc);
    int d = (int)((E[w / 16] >> ((w % 16) * 4)) & 15);
    if (d) sc_mul(&acc, &acc, &tab[d]);
  }
  *r = acc;
}

/* ---------------- group ---------------- */
typedef struct { fe x, y; int inf; } ge;
typedef struct { fe x, y, z; int inf; } gej;

static void gej_set_ge(gej* r, const ge* a) {
  r->x = a->x; r->y = a->y; r->z = (fe){{1, 0, 0, 0}}; r->inf = a->inf;
}
static void gej_double(gej* r, const gej* a) {
  if (a->inf || fe_is_zero(&a->y)) { r->inf = 1; return; }
  fe A, B, C, D, E, F, t;
  fe_sqr(&A, &a->x);
  fe_sqr(&B, &a->y);
  fe_sqr(&C, &B);
  fe_add(&t, &a->x, &B); fe_sqr(&t, &t); fe_sub(&t, &t, &A); fe_sub(&t, &t, &C); fe_add(&D, &t, &t);
  fe_add(&E, &A, &A); fe_add(&E, &E, &A);
  fe_sqr(&F, &E);
  gej o;
  fe_sub(&o.x, &F, &D); fe_sub(&o.x, &o.x, &D);
  fe_mul(&o.z, &a->y, &a->z); fe_add(&o.z, &o.z, &o.z);
  fe C8; fe_add(&C8, &C, &C); fe_add(&C8, &C8, &C8); fe_add(&C8, &C8, &C8);
  fe_sub(&t, &D, &o.x); fe_mul(&o.y, &E, &t); fe_sub(&o.y, &o.y, &C8);
  o.inf = 0;
  *r = o;
}
/* complete Jacobian + Jacobian */
static void gej_add(gej* r, const gej* a, const gej* b) {
  if (a->inf) { *r = *b; return; }
  if (b->inf) { *r = *a; return; }
  fe z1z1, z2z2, u1, u2, s1, s2, h, rr, t;
  fe_sqr(&z1z1, &a->z); fe_sqr(&z2z2, &b->z);
  fe_mul(&u1, &a->x, &z2z2); fe_mul(&u2, &b->x, &z1z1);
  fe_mul(&t, &b->z, &z2z2); fe_mul(&s1, &a->y, &t);
  fe_mul(&t, &a->z, &z1z1); fe_mul(&s2, &b->y, &t);
  fe_sub(&h, &u2, &u1); fe_sub(&rr, &s2, &s1);
  if (fe_is_zero(&h)) {
    if (fe_is_zero(&rr)) { gej_double(r, a); return; }
    r->inf = 1; return;
  }
  fe hh, hhh, v;
  fe_sqr(&hh, &h); fe_mul(&hhh, &h, &hh); fe_mul(&v, &u1, &hh);
  gej o;
  fe_sqr(&o.x, &rr); fe_sub(&o.x, &o.x, &hhh); fe_sub(&o.x, &o.x, &v); fe_sub(&o.x, &o.x, &v);
  fe_sub(&t, &v, &o.x); fe_mul(&o.y, &rr, &t); fe_mul(&t, &s1, &hhh); fe_sub(&o.y, &o.y, &t);
  fe_mul(&o.z, &a->z, &b->z); fe_mul(&o.z, &o.z, &h);
  o.inf = 0;
  *r = o;
}
static void gej_neg(gej* r, const gej* a) { *r = *a; fe_neg(&r->y, &a->y); }
static int gej_to_ge(ge* r, const gej* a) {
  if (a->inf) { r->inf = 1; return 0; }
  fe zi, zi2, zi3;
  fe_inv(&zi, &a->z); fe_sqr(&zi2, &zi); fe_mul(&zi3, &zi2, &zi);
  fe_mul(&r->x, &a->x, &zi2); fe_mul(&r->y, &a->y, &zi3); r->inf = 0;
  return 1;
}

/* wNAF(w) of a 256-bit scalar; returns length (<= 257) */
static int wnaf(int* out, const sc* k, int w) {
  uint64_t v[5] = {k->v[0], k->v[1], k->v[2], k->v[3], 0};
  int len = 0;
  memset(out, 0, 258 * sizeof(int));
  int pos = 0;
  while (pos < 258) {
    int any = (v[0] | v[1] | v[2] | v[3] | v[4]) != 0;
    if (!any) break;
    if (v[0] & 1) {
      int d = (int)(v[0] & ((1u << w) - 1));
      if (d >= (1 << (w - 1))) d -= (1 << w);
      out[pos] = d;
      /* v -= d */
      if (d > 0) { u128 b = (u128)v[0] - (uint64_t)d; v[0] = (uint64_t)b; int borrow = (int)((b >> 64) != 0);
        for (int i = 1; i < 5 && borrow; ++i) { borrow = v[i] == 0; v[i] -= 1; } }
      else { u128 c = (u128)v[0] + (uint64_t)(-d); v[0] = (uint64_t)c; uint64_t carry = (uint64_t)(c >> 64);
        for (int i = 1; i < 5 && carry; ++i) { v[i] += 1; carry = v[i] == 0; } }
      len = pos + 1;
    }
    /* v >>= 1 */
    for (int i = 0; i < 4; ++i) v[i] = (v[i] >> 1) | (v[i + 1] << 63);
    v[4] >>= 1;
    ++pos;
  }
  return len;
}

#define WQ 5
#define WG 8
static ge G_TAB[1 << (WG - 2)];     /* odd multiples 1G, 3G, ..., (2^(WG-1)-1)G */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void init_g_table(void) {
  gej g, g2, acc;
  ge G = {FE_GX, FE_GY, 0};
  gej_set_ge(&g, &G);
  gej_double(&g2, &g);
  acc = g;
  for (int i = 0; i < (1 << (WG - 2)); ++i) {
    gej_to_ge(&G_TAB[i], &acc);
    gej_add(&acc, &acc, &g2);
  }
}

/* R = u1*G + u2*Q */
static void ecmult(gej* r, const sc* u1, const sc* u2, const ge* q) {
  pthread_once(&g_once, init_g_table);
  int n1[258], n2[258];
  int l1 = wnaf(n1, u1, WG), l2 = wnaf(n2, u2, WQ);
  gej qt[1 << (WQ - 2)], q1, q2;
  gej_set_ge(&q1, q);
  gej_double(&q2, &q1);
  qt[0] = q1;
  for (int i = 1; i < (1 << (WQ - 2)); ++i) gej_add(&qt[i], &qt[i - 1], &q2);
  int len = l1 > l2 ? l1 : l2;
  gej acc; acc.inf = 1;
  for (int i = len - 1; i >= 0; --i) {
    gej_double(&acc, &acc);
    if (i < l2 && n2[i]) {
      gej t; int d = n2[i];
      if (d > 0) t = qt[(d - 1) / 2]; else gej_neg(&t, &qt[(-d - 1) / 2]);
      gej_add(&acc, &acc, &t);
    }
    if (i < l1 && n1[i]) {
      gej t; int d = n1[i];
      gej_set_ge(&t, &G_TAB[((d > 0 ? d : -d) - 1) / 2]);
      if (d < 0) fe_neg(&t.y, &t.y);
      gej_add(&acc, &acc, &t);
    }
  }
  *r = acc;
}

/* ---------------- exported API ---------------- */

/* secp256k1_ec_pubkey_parse semantics; out_xy = x||y big-endian. 1 = ok */
int hkvo_pubkey_parse(const uint8_t* pk, size_t len, uint8_t out_xy[64]);
static int pubkey_parse(ge* q, const uint8_t* pk, size_t len) {
  fe seven = {{7, 0, 0, 0}};
  if (len == 33 && (pk[0] == 2 || pk[0] == 3)) {
    u256_from_be(q->x.v, pk + 1);
    if (u256_cmp(q->x.v, FE_P.v) >= 0) return 0;
    fe x3, rhs, y, y2;
    fe_sqr(&x3, &q->x); fe_mul(&x3, &x3, &q->x); fe_add(&rhs, &x3, &seven);
    fe_sqrt_cand(&y, &rhs); fe_sqr(&y2, &y);
    if (!fe_eq(&y2, &rhs)) return 0;
    if ((int)(y.v[0] & 1) != (pk[0] & 1)) fe_neg(&y, &y);
    q->y = y; q->inf = 0;
    return 1;
  }
  if (len == 65 && (pk[0] == 4 || pk[0] == 6 || pk[0] == 7)) {
    u256_from_be(q->x.v, pk + 1);
    u256_from_be(q->y.v, pk + 33);
    if (u256_cmp(q->x.v, FE_P.v) >= 0 || u256_cmp(q->y.v, FE_P.v) >= 0) return 0;
    if (pk[0] != 4 && (int)(q->y.v[0] & 1) != (pk[0] & 1)) return 0;
    fe x3, rhs, y2;
    fe_sqr(&x3, &q->x); fe_mul(&x3, &x3, &q->x); fe_add(&rhs, &x3, &seven);
    fe_sqr(&y2, &q->y);
    if (!fe_eq(&y2, &rhs)) return 0;
    q->inf = 0;
    return 1;
  }
  return 0;
}
int hkvo_pubkey_parse(const uint8_t* pk, size_t len, uint8_t out_xy[64]) {
  ge q;
  if (!pubkey_parse(&q, pk, len)) return 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) {
      out_xy[(3 - i) * 8 + j] = (uint8_t)(q.x.v[i] >> (56 - 8 * j));
      out_xy[32 + (3 - i) * 8 + j] = (uint8_t)(q.y.v[i] >> (56 - 8 * j));
    }
  return 1;
}

/* One 168-byte record (include/hkv.h layout). mode 0 = LIBSECP, 1 = HASKOIN. */
int hkvo_verify_record(const uint8_t* rec, int mode) {
  sc r, s, m;
  u256_from_be(r.v, rec + 32);
  u256_from_be(s.v, rec + 64);
  /* compact parse: overflow fails */
  if (u256_cmp(r.v, SC_N.v) >= 0 || u256_cmp(s.v, SC_N.v) >= 0) return 0;
  unsigned pklen = rec[96];
  ge q;
  if (pklen > 65 || !pubkey_parse(&q, rec + 97, pklen)) return 0;
  if (u256_cmp(s.v, SC_HALF_N.v) > 0) {
    if (mode == 1) u256_sub(s.v, SC_N.v, s.v);   /* verifyHashSig: normalize */
    else return 0;                                /* secp256k1_ecdsa_verify: reject high-S */
  }
  if (u256_is_zero(r.v) || u256_is_zero(s.v)) return 0;
  u256_from_be(m.v, rec);
  if (u256_cmp(m.v, SC_N.v) >= 0) u256_sub(m.v, m.v, SC_N.v);
  sc sinv, u1, u2;
  sc_inv(&sinv, &s);
  sc_mul(&u1, &m, &sinv);
  sc_mul(&u2, &r, &sinv);
  gej R;
  ecmult(&R, &u1, &u2, &q);
  ge Ra;
  if (!gej_to_ge(&Ra, &R)) return 0;
  if (u256_cmp(Ra.x.v, r.v) == 0) return 1;
  /* r + n < p ?  then compare with r + n */
  uint64_t rn[4];
  uint64_t c = u256_add(rn, r.v, SC_N.v);
  if (!c && u256_cmp(rn, FE_P.v) < 0 && u256_cmp(Ra.x.v, rn) == 0) return 1;
  return 0;
}

struct job { const uint8_t* recs; size_t lo, hi; int mode; uint8_t* verdicts; };
static void* worker(void* arg) {
  struct job* j = (struct job*)arg;
  for (size_t i = j->lo; i < j->hi; ++i) j->verdicts[i] = (uint8_t)hkvo_verify_record(j->recs + i * 168, j->mode);
  return NULL;
}

/* Verify n records on nthreads pthreads; verdicts[i] = 0/1. */
int hkvo_verify_batch(const uint8_t* recs, size_t n, int mode, uint8_t* verdicts, int nthreads) {
  pthread_once(&g_once, init_g_table);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  int created[256] = {0};
  struct job jobs[256];
  size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
  for (int t = 0; t < nthreads; ++t) {
    size_t lo = (size_t)t * per, hi = lo + per;
    if (lo >= n) break;
    if (hi > n) hi = n;
    jobs[t] = (struct job){recs, lo, hi, mode, verdicts};
    if (pthread_create(&th[t], NULL, worker, &jobs[t]) == 0) created[t] = 1;
    else worker(&jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t)
    if (created[t]) pthread_join(th[t], NULL);
  return 0;
}

/* ---------------- synthetic batch generator (restatement) ----------------
 * The generator contract of hkv_gen_batch_device (include/hkv.h;
 * haskoin-node_amd/csrc/hkv_kernels.hip hkv_gen_pool_kernel /
 * hkv_gen_records_kernel), restated on the CPU so the sharded-batch tests can
 * build the same records without a GPU: record k of batch `seed` depends on
 * (seed, k) only, the key pool on seed only. The keyless construction is
 * R = aG + bQ, r = R.x mod n, s = r/b, msg = a s, s low. */
static uint64_t splitmix64(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
static void rand_scalar(sc* r, uint64_t* st) {
  for (int k = 0; k < 4; ++k) r->v[k] = splitmix64(st);
  if (u256_cmp(r->v, SC_N.v) >= 0) u256_sub(r->v, r->v, SC_N.v);
  if (u256_is_zero(r->v)) r->v[0] = 1;
}
static void u256_to_be(uint8_t* b, const uint64_t* v) {
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) b[(3 - i) * 8 + j] = (uint8_t)(v[i] >> (56 - 8 * j));
}
/* a*G + b*P, affine; 0 if infinity */
static int ecmult_affine(ge* out, const sc* a, const sc* b, const ge* p) {
  gej R;
  ecmult(&R, a, b, p);
  return gej_to_ge(out, &R);
}
/* pool key j: d = rand_scalar(seed * C + j * phi + K), Q = d G */
static void gen_pool(ge* pool, uint64_t seed, uint32_t npool) {
  static const sc ZERO = {{0, 0, 0, 0}};
  for (uint32_t j = 0; j < npool; ++j) {
    uint64_t st = seed * 0x2545F4914F6CDD1DULL + (uint64_t)j * 0x9E3779B97F4A7C15ULL + 0x5851F42D4C957F2DULL;
    sc d;
    rand_scalar(&d, &st);
    ge g = {FE_GX, FE_GY, 0};
    ecmult_affine(&pool[j], &ZERO, &d, &g);
  }
}
/* mutation classes (hkv_gen_records_kernel GEN_CLS_*): all reject in both modes */
enum { CLS_MSG = 0, CLS_R = 1, CLS_S = 2, CLS_KEY = 3, CLS_NEGKEY = 4, NCLS = 5 };

/* Records [index0, index0 + n) of batch `seed` into recs (n * 168 bytes);
 * labels[i] = 1 when record index0 + i is valid by construction (may be
 * NULL); classes[i] = the mutation class or -1 (may be NULL). The pool
 * (npool keys) is built from seed ^ "pool" as the device does. */
int hkvo_gen_batch(uint64_t seed, uint64_t index0, size_t n, uint32_t npool, uint32_t unc_permille,
                   uint32_t invalid_permille, uint8_t* recs, uint8_t* labels, int8_t* classes) {
  pthread_once(&g_once, init_g_table);
  if (npool == 0) return -1;
  ge* pool = (ge*)calloc(npool, sizeof(ge));
  if (!pool) return -1;
  gen_pool(pool, seed ^ 0x706F6F6CULL, npool);
  for (size_t i = 0; i < n; ++i) {
    const uint64_t g = index0 + i;
    uint64_t st = seed * 0xD1B54A32D192ED03ULL + g * 0x9E3779B97F4A7C15ULL + 0x8CB92BA72F3D8DD7ULL;
    sc a, b;
    rand_scalar(&a, &st);
    rand_scalar(&b, &st);
    const uint64_t pick = splitmix64(&st);
    const uint32_t j = (uint32_t)(pick % npool);
    const int unc = ((pick >> 40) % 1000u) < unc_permille;
    ge q = pool[j], R;
    ecmult_affine(&R, &a, &b, &q);
    sc r, s, bi, m;
    memcpy(r.v, R.x.v, 32);
    if (u256_cmp(r.v, SC_N.v) >= 0) u256_sub(r.v, r.v, SC_N.v);
    sc_inv(&bi, &b);
    sc_mul(&s, &r, &bi);
    sc_mul(&m, &a, &s);
    if (u256_cmp(s.v, SC_HALF_N.v) > 0) u256_sub(s.v, SC_N.v, s.v);
    int bad = 0, cls = -1;
    unsigned bit = 0;
    if (invalid_permille) {
      const uint64_t mut = splitmix64(&st);
      bad = (mut % 1000u) < invalid_permille;
      cls = (int)((mut >> 16) % NCLS);
      bit = (unsigned)(mut >> 32) & 255u;
      if (bad && cls == CLS_KEY && npool > 1) q = pool[(j + 1u + (uint32_t)((mut >> 40) % (npool - 1u))) % npool];
      if (bad && cls == CLS_KEY && npool <= 1) cls = CLS_MSG;
      if (bad && cls == CLS_NEGKEY) fe_neg(&q.y, &q.y);
      if (!bad) cls = -1;
    }
    uint8_t* o = recs + i * 168;
    memset(o, 0, 168);
    u256_to_be(o, m.v);
    u256_to_be(o + 32, r.v);
    u256_to_be(o + 64, s.v);
    o[96] = unc ? 65 : 33;
    if (unc) {
      o[97] = 4;
      u256_to_be(o + 98, q.x.v);
      u256_to_be(o + 130, q.y.v);
    } else {
      o[97] = (uint8_t)(2u | (q.y.v[0] & 1u));
      u256_to_be(o + 98, q.x.v);
    }
    if (bad && cls <= CLS_S) o[32u * (unsigned)cls + (bit >> 3)] ^= (uint8_t)(1u << (bit & 7u));
    if (labels) labels[i] = (uint8_t)!bad;
    if (classes) classes[i] = (int8_t)cls;
  }
  free(pool);
  return 0;
}

/* helpers exposed for tests: modular ops on big-endian 32-byte values */
void hkvo_fe_mul(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
  fe x, y, z; u256_from_be(x.v, a); u256_from_be(y.v, b); fe_mul(&z, &x, &y);
  for (int i = 0; i < 4; ++i) for (int j = 0; j < 8; ++j) out[(3 - i) * 8 + j] = (uint8_t)(z.v[i] >> (56 - 8 * j));
}
