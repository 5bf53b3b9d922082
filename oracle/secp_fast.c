/*
 * secp_fast.c — libsecp256k1-class CPU verifier (TEST / BASELINE INFRASTRUCTURE
 * ONLY: bench.py's cpu_baseline leg times it, tests/ check it; the product
 * path never links or loads it).
 *
 * Why it exists: BASELINE.json north_star asks for the GPU rate against "the
 * all-core host libsecp256k1 verify rate". libsecp256k1 (pinned through
 * secp256k1-haskell 1.2.0, /root/reference/stack.yaml:2-10; nix, version
 * unpinned) is neither vendored in /root/reference nor installed here or on
 * the GPU box. The port (hkv_oracle.c) is deliberately simple (no GLV, generic
 * Fermat inversions) and OpenSSL's generic-curve ECDSA is slower still, so
 * both understate a libsecp256k1 host by 3-4x (Missing 4). This
 * file restates the published algorithm of libsecp256k1's verify path so the
 * baseline is of the reference's class:
 *
 *   field     5 x 52-bit limbs, 64 x 64 -> 128-bit products, lazy (magnitude)
 *             reduction with 2^260 == 0x1000003D10 (mod p)     [field_5x52]
 *   scalar    4 x 64-bit limbs mod n; s^-1 by Bernstein-Yang safegcd with
 *             variable-time 62-bit divsteps                     [modinv64_var]
 *   u2*Q      GLV split u2 = k1 + k2*lambda (|k1|, |k2| < 2^128), wNAF w = 5,
 *             the odd multiples 1Q..15Q on one isomorphic curve ("global Z"),
 *             lambda(jQ) = (beta x, y)                          [ecmult_strauss]
 *   u1*G      u1 split in 128-bit halves, wNAF w = 15 against precomputed
 *             affine tables of the odd multiples of G and 2^128 G (8,192
 *             entries each, built once), added with the z-inverse mixed add
 *   doubling  a = 0 Jacobian, 2M + 5S                              [gej_double]
 *   compare   r * Z^2 == X in Jacobian, then r + n when r + n < p [sig_verify]
 *   parse     SEC1 keys incl. the 253S + 13M square root, hybrid parity,
 *             compact (r, s) overflow, high-S per mode (the port's semantics)
 *
 * Verdict semantics are the port's (hkvo_verify_record): tests/test_secp_fast.py
 * checks every golden KAT, the special pool and generated adversarial batches
 * against hkv_oracle.c in both modes; bench.py compares its verdicts with the
 * GPU's on every timed sample.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef __int128 i128;

/* ------------------------------------------------------------------------ */
/* field: value = sum n[i] 2^(52 i); "magnitude m" = every limb <= m (2^52-1) */
/* (limb 4 <= m (2^48 - 1) at m = 1, up to m 2^52 above)                    */
typedef struct { uint64_t n[5]; } fe;

#define M52 0xFFFFFFFFFFFFFULL
#define M48 0xFFFFFFFFFFFFULL
static const uint64_t P52[5] = {0xFFFFEFFFFFC2FULL, M52, M52, M52, M48};
#define FOLD256 0x1000003D1ULL  /* 2^256 mod p */
#define FOLD260 0x1000003D10ULL /* 2^260 mod p */

/* final carry pass of a product: c[0..4] (u128) -> limbs, magnitude 1 */
static inline void fe_carry5(fe* r, u128 c0, u128 c1, u128 c2, u128 c3, u128 c4) {
  c1 += c0 >> 52;
  c2 += c1 >> 52;
  c3 += c2 >> 52;
  c4 += c3 >> 52;
  const u128 t = c4 >> 48;
  u128 x = (u128)((uint64_t)c0 & M52) + t * FOLD256;
  r->n[0] = (uint64_t)x & M52;
  uint64_t n1 = ((uint64_t)c1 & M52) + (uint64_t)(x >> 52);
  r->n[1] = n1 & M52;
  r->n[2] = ((uint64_t)c2 & M52) + (n1 >> 52);
  r->n[3] = (uint64_t)c3 & M52;
  r->n[4] = (uint64_t)c4 & M48;
}

/* the columns 5..8 of a 5x5 limb product, carried into 52-bit pieces and
 * folded into columns 0..4 with 2^260 == FOLD260 */
static inline void fe_fold_high(u128* c0, u128* c1, u128* c2, u128* c3, u128* c4, u128 c5, u128 c6, u128 c7,
                                u128 c8) {
  c6 += c5 >> 52;
  c7 += c6 >> 52;
  c8 += c7 >> 52;
  const uint64_t h5 = (uint64_t)c5 & M52, h6 = (uint64_t)c6 & M52, h7 = (uint64_t)c7 & M52,
                 h8 = (uint64_t)c8 & M52, h9 = (uint64_t)(c8 >> 52);
  *c0 += (u128)h5 * FOLD260;
  *c1 += (u128)h6 * FOLD260;
  *c2 += (u128)h7 * FOLD260;
  *c3 += (u128)h8 * FOLD260;
  *c4 += (u128)h9 * FOLD260;
}

static inline void fe_mul(fe* r, const fe* a, const fe* b) {
  const uint64_t a0 = a->n[0], a1 = a->n[1], a2 = a->n[2], a3 = a->n[3], a4 = a->n[4];
  const uint64_t b0 = b->n[0], b1 = b->n[1], b2 = b->n[2], b3 = b->n[3], b4 = b->n[4];
  u128 c0 = (u128)a0 * b0;
  u128 c1 = (u128)a0 * b1 + (u128)a1 * b0;
  u128 c2 = (u128)a0 * b2 + (u128)a1 * b1 + (u128)a2 * b0;
  u128 c3 = (u128)a0 * b3 + (u128)a1 * b2 + (u128)a2 * b1 + (u128)a3 * b0;
  u128 c4 = (u128)a0 * b4 + (u128)a1 * b3 + (u128)a2 * b2 + (u128)a3 * b1 + (u128)a4 * b0;
  u128 c5 = (u128)a1 * b4 + (u128)a2 * b3 + (u128)a3 * b2 + (u128)a4 * b1;
  u128 c6 = (u128)a2 * b4 + (u128)a3 * b3 + (u128)a4 * b2;
  u128 c7 = (u128)a3 * b4 + (u128)a4 * b3;
  u128 c8 = (u128)a4 * b4;
  fe_fold_high(&c0, &c1, &c2, &c3, &c4, c5, c6, c7, c8);
  fe_carry5(r, c0, c1, c2, c3, c4);
}

static inline void fe_sqr(fe* r, const fe* a) {
  const uint64_t a0 = a->n[0], a1 = a->n[1], a2 = a->n[2], a3 = a->n[3], a4 = a->n[4];
  const uint64_t d0 = a0 * 2, d1 = a1 * 2, d2 = a2 * 2, d3 = a3 * 2;
  u128 c0 = (u128)a0 * a0;
  u128 c1 = (u128)d0 * a1;
  u128 c2 = (u128)d0 * a2 + (u128)a1 * a1;
  u128 c3 = (u128)d0 * a3 + (u128)d1 * a2;
  u128 c4 = (u128)d0 * a4 + (u128)d1 * a3 + (u128)a2 * a2;
  u128 c5 = (u128)d1 * a4 + (u128)d2 * a3;
  u128 c6 = (u128)d2 * a4 + (u128)a3 * a3;
  u128 c7 = (u128)d3 * a4;
  u128 c8 = (u128)a4 * a4;
  fe_fold_high(&c0, &c1, &c2, &c3, &c4, c5, c6, c7, c8);
  fe_carry5(r, c0, c1, c2, c3, c4);
}

static inline void fe_add(fe* r, const fe* a, const fe* b) {
  for (int i = 0; i < 5; ++i) r->n[i] = a->n[i] + b->n[i];
}
static inline void fe_mul_int(fe* r, uint64_t k) {
  for (int i = 0; i < 5; ++i) r->n[i] *= k;
}
/* r = 2 (m + 1) p - a for a of magnitude <= m: magnitude 2 (m + 1) */
static inline void fe_negate(fe* r, const fe* a, uint64_t m) {
  const uint64_t k = 2 * (m + 1);
  for (int i = 0; i < 5; ++i) r->n[i] = k * P52[i] - a->n[i];
}
/* carry pass + one top fold: magnitude 1, value < 2^256 (possibly >= p) */
static inline void fe_normalize_weak(fe* r) {
  uint64_t t0 = r->n[0], t1 = r->n[1], t2 = r->n[2], t3 = r->n[3], t4 = r->n[4];
  const uint64_t x = t4 >> 48;
  t4 &= M48;
  t0 += x * FOLD256;
  t1 += t0 >> 52; t0 &= M52;
  t2 += t1 >> 52; t1 &= M52;
  t3 += t2 >> 52; t2 &= M52;
  t4 += t3 >> 52; t3 &= M52;
  /* t4 may now be 2^48 exactly only if the value was >= 2^256 - small: one more fold */
  const uint64_t y = t4 >> 48;
  t4 &= M48;
  t0 += y * FOLD256;
  t1 += t0 >> 52; t0 &= M52;
  t2 += t1 >> 52; t1 &= M52;
  t3 += t2 >> 52; t2 &= M52;
  t4 += t3 >> 52; t3 &= M52;
  r->n[0] = t0; r->n[1] = t1; r->n[2] = t2; r->n[3] = t3; r->n[4] = t4;
}
/* fully reduced, < p */
static inline void fe_normalize(fe* r) {
  fe_normalize_weak(r);
  /* r >= p  <=>  r + FOLD256 >= 2^256 */
  uint64_t t0 = r->n[0] + FOLD256, t1 = r->n[1] + (t0 >> 52), t2, t3, t4;
  t0 &= M52;
  t2 = r->n[2] + (t1 >> 52); t1 &= M52;
  t3 = r->n[3] + (t2 >> 52); t2 &= M52;
  t4 = r->n[4] + (t3 >> 52); t3 &= M52;
  if (t4 >> 48) {
    r->n[0] = t0; r->n[1] = t1; r->n[2] = t2; r->n[3] = t3; r->n[4] = t4 & M48;
  }
}
static inline int fe_normalizes_to_zero(const fe* a) {
  fe t = *a;
  fe_normalize(&t);
  return (t.n[0] | t.n[1] | t.n[2] | t.n[3] | t.n[4]) == 0;
}
static inline int fe_equal_norm(const fe* a, const fe* b) {  /* both normalized */
  return ((a->n[0] ^ b->n[0]) | (a->n[1] ^ b->n[1]) | (a->n[2] ^ b->n[2]) | (a->n[3] ^ b->n[3]) |
          (a->n[4] ^ b->n[4])) == 0;
}
static void fe_from_u256(fe* r, const uint64_t v[4]) {
  r->n[0] = v[0] & M52;
  r->n[1] = (v[0] >> 52 | v[1] << 12) & M52;
  r->n[2] = (v[1] >> 40 | v[2] << 24) & M52;
  r->n[3] = (v[2] >> 28 | v[3] << 36) & M52;
  r->n[4] = v[3] >> 16;
}
static void fe_set_int(fe* r, uint64_t x) {
  r->n[0] = x; r->n[1] = r->n[2] = r->n[3] = r->n[4] = 0;
}

static void fe_sqr_n(fe* r, const fe* a, int k) {
  fe_sqr(r, a);
  for (int i = 1; i < k; ++i) fe_sqr(r, r);
}
/* a^((p+1)/4) and a^(p-2) by the standard 1-2-3-6-9-11-22-44-88-176-220-223
 * addition chain (255 squarings) */
static void fe_chain223(const fe* a, fe* x2, fe* x22, fe* x223) {
  fe x3, x6, x9, x11, x44, x88, x176, x220, t;
  fe_sqr(x2, a); fe_mul(x2, x2, a);
  fe_sqr(&x3, x2); fe_mul(&x3, &x3, a);
  fe_sqr_n(&t, &x3, 3); fe_mul(&x6, &t, &x3);
  fe_sqr_n(&t, &x6, 3); fe_mul(&x9, &t, &x3);
  fe_sqr_n(&t, &x9, 2); fe_mul(&x11, &t, x2);
  fe_sqr_n(&t, &x11, 11); fe_mul(x22, &t, &x11);
  fe_sqr_n(&t, x22, 22); fe_mul(&x44, &t, x22);
  fe_sqr_n(&t, &x44, 44); fe_mul(&x88, &t, &x44);
  fe_sqr_n(&t, &x88, 88); fe_mul(&x176, &t, &x88);
  fe_sqr_n(&t, &x176, 44); fe_mul(&x220, &t, &x44);
  fe_sqr_n(&t, &x220, 3); fe_mul(x223, &t, &x3);
}
static void fe_sqrt_cand(fe* r, const fe* a) {
  fe x2, x22, x223, t;
  fe_chain223(a, &x2, &x22, &x223);
  fe_sqr_n(&t, &x223, 23); fe_mul(&t, &t, &x22);
  fe_sqr_n(&t, &t, 6); fe_mul(&t, &t, &x2);
  fe_sqr_n(r, &t, 2);
}
static void fe_inv(fe* r, const fe* a) {  /* a^(p-2); only at table build */
  fe x2, x22, x223, t;
  fe_chain223(a, &x2, &x22, &x223);
  fe_sqr_n(&t, &x223, 23); fe_mul(&t, &t, &x22);
  fe_sqr_n(&t, &t, 5); fe_mul(&t, &t, a);
  fe_sqr_n(&t, &t, 3); fe_mul(&t, &t, &x2);
  fe_sqr_n(&t, &t, 2); fe_mul(r, &t, a);
}

/* ------------------------------------------------------------------------ */
/* scalars mod n: 4 x 64-bit limbs, < n                                     */
typedef struct { uint64_t d[4]; } sc;
static const uint64_t SN[4] = {0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL,
                               0xFFFFFFFFFFFFFFFFULL};
static const uint64_t SNH[4] = {0xDFE92F46681B20A0ULL, 0x5D576E7357A4501DULL, 0xFFFFFFFFFFFFFFFFULL,
                                0x7FFFFFFFFFFFFFFFULL};
static const uint64_t SNC[3] = {0x402DA1732FC9BEBFULL, 0x4551231950B75FC4ULL, 1ULL}; /* 2^256 - n */

static int u256_lt(const uint64_t* a, const uint64_t* b) {
  for (int i = 3; i >= 0; --i)
    if (a[i] != b[i]) return a[i] < b[i];
  return 0;
}
static void u256_from_be(uint64_t* r, const uint8_t* b) {
  for (int i = 0; i < 4; ++i) {
    uint64_t w = 0;
    for (int j = 0; j < 8; ++j) w = (w << 8) | b[(3 - i) * 8 + j];
    r[i] = w;
  }
}
static uint64_t u256_sub(uint64_t* r, const uint64_t* a, const uint64_t* b) {
  uint64_t br = 0;
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)a[i] - b[i] - br;
    r[i] = (uint64_t)d;
    br = (uint64_t)(d >> 127);
  }
  return br;
}
static uint64_t u256_add(uint64_t* r, const uint64_t* a, const uint64_t* b) {
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (u128)a[i] + b[i];
    r[i] = (uint64_t)c;
    c >>= 64;
  }
  return (uint64_t)c;
}
static int sc_is_zero(const sc* a) { return (a->d[0] | a->d[1] | a->d[2] | a->d[3]) == 0; }
static int sc_is_high(const sc* a) { return u256_lt(SNH, a->d); }
static void sc_negate(sc* r, const sc* a) {
  if (sc_is_zero(a)) { *r = *a; return; }
  u256_sub(r->d, SN, a->d);
}
static void sc_add(sc* r, const sc* a, const sc* b) {
  const uint64_t c = u256_add(r->d, a->d, b->d);
  if (c || !u256_lt(r->d, SN)) u256_sub(r->d, r->d, SN);
}
/* 512-bit product */
static void mul256(uint64_t t[8], const uint64_t* a, const uint64_t* b) {
  memset(t, 0, 64);
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) {
      c += (u128)a[i] * b[j] + t[i + j];
      t[i + j] = (uint64_t)c;
      c >>= 64;
    }
    t[i + 4] = (uint64_t)c;
  }
}
/* t (512 bits) mod n: fold the part above 2^256 with 2^256 == NC (129 bits)
 * three times (385 -> 258 -> 256 bits), then one conditional subtraction */
static void sc_reduce512(sc* r, const uint64_t t[8]) {
  uint64_t a[7];  /* t[0..3] + t[4..7] * NC : < 2^386 */
  {
    u128 c = 0;
    uint64_t p[7] = {0};
    for (int i = 0; i < 4; ++i) {
      u128 k = 0;
      for (int j = 0; j < 3; ++j) {
        k += (u128)t[4 + i] * SNC[j] + p[i + j];
        p[i + j] = (uint64_t)k;
        k >>= 64;
      }
      p[i + 3] = (uint64_t)k;
    }
    for (int i = 0; i < 7; ++i) {
      c += (u128)p[i] + (i < 4 ? t[i] : 0);
      a[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  uint64_t b[5];  /* a[0..3] + a[4..6] * NC : < 2^259 */
  {
    uint64_t p[6] = {0};
    for (int i = 0; i < 3; ++i) {
      u128 k = 0;
      for (int j = 0; j < 3; ++j) {
        k += (u128)a[4 + i] * SNC[j] + p[i + j];
        p[i + j] = (uint64_t)k;
        k >>= 64;
      }
      p[i + 3] = (uint64_t)k;
    }
    u128 c = 0;
    for (int i = 0; i < 5; ++i) {
      c += (u128)p[i] + (i < 4 ? a[i] : 0);
      b[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  /* b[4] < 8: one more fold */
  u128 c = (u128)b[4] * SNC[0] + b[0];
  r->d[0] = (uint64_t)c; c >>= 64;
  c += (u128)b[4] * SNC[1] + b[1];
  r->d[1] = (uint64_t)c; c >>= 64;
  c += (u128)b[4] * SNC[2] + b[2];
  r->d[2] = (uint64_t)c; c >>= 64;
  c += b[3];
  r->d[3] = (uint64_t)c; c >>= 64;
  if ((uint64_t)c || !u256_lt(r->d, SN)) u256_sub(r->d, r->d, SN);
}
static void sc_mul(sc* r, const sc* a, const sc* b) {
  uint64_t t[8];
  mul256(t, a->d, b->d);
  sc_reduce512(r, t);
}

/* ---- s^-1 mod n: safegcd (Bernstein-Yang) with variable-time divsteps in
 * batches of 62 (libsecp256k1 modinv64_var's algorithm) ---- */
typedef struct { int64_t v[5]; } s62;  /* value = sum v[i] 2^(62 i), limbs signed */
#define M62 0x3FFFFFFFFFFFFFFFULL
static const s62 N62 = {{0x3FD25E8CD0364141LL, 0x2ABB739ABD2280EELL, 0x3FFFFFFFFFFFFFEBLL, 0x3FFFFFFFFFFFFFFFLL,
                         0xFFLL}};
#define NINV62 0x34F20099AA774EC1ULL /* n^-1 mod 2^62 */

typedef struct { int64_t u, v, q, r; } trans2x2;

/* up to 62 divsteps on the low bits of (f, g); returns the new eta. Skips
 * runs of zeros in g at once and cancels up to 6 (or 4) low bits of g per
 * odd step with w = -g / f mod 2^k. */
static int64_t divsteps_62_var(int64_t eta, uint64_t f0, uint64_t g0, trans2x2* t) {
  uint64_t u = 1, v = 0, q = 0, r = 1;
  uint64_t f = f0, g = g0, m;
  uint32_t w;
  int i = 62, limit, zeros;
  for (;;) {
    zeros = __builtin_ctzll(g | (~0ULL << i));
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    if (eta < 0) {
      uint64_t tmp;
      eta = -eta;
      tmp = f; f = g; g = -tmp;
      tmp = u; u = q; q = -tmp;
      tmp = v; v = r; r = -tmp;
      limit = ((int)eta + 1) > i ? i : ((int)eta + 1);
      m = (~0ULL >> (64 - limit)) & 63U;
      w = (uint32_t)((f * g * (f * f - 2)) & m);  /* -g / f mod 2^limit */
    } else {
      limit = ((int)eta + 1) > i ? i : ((int)eta + 1);
      m = (~0ULL >> (64 - limit)) & 15U;
      w = (uint32_t)(f + (((f + 1) & 4) << 1));  /* f^-1 mod 16 */
      w = (uint32_t)((-(uint64_t)w * g) & m);
    }
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t->u = (int64_t)u; t->v = (int64_t)v; t->q = (int64_t)q; t->r = (int64_t)r;
  return eta;
}
/* (d, e) <- (t [d, e]) / 2^62 mod n, kept in (-2n, n) */
static void update_de(s62* d, s62* e, const trans2x2* t) {
  const int64_t u = t->u, v = t->v, q = t->q, r = t->r;
  const int64_t d0 = d->v[0], e0 = e->v[0];
  const int64_t sd = d->v[4] >> 63, se = e->v[4] >> 63;
  int64_t md = (u & sd) + (v & se), me = (q & sd) + (r & se);
  i128 cd = (i128)u * d0 + (i128)v * e0;
  i128 ce = (i128)q * d0 + (i128)r * e0;
  md -= (int64_t)((NINV62 * (uint64_t)cd + (uint64_t)md) & M62);
  me -= (int64_t)((NINV62 * (uint64_t)ce + (uint64_t)me) & M62);
  cd += (i128)N62.v[0] * md;
  ce += (i128)N62.v[0] * me;
  cd >>= 62;
  ce >>= 62;
  for (int i = 1; i < 5; ++i) {
    cd += (i128)u * d->v[i] + (i128)v * e->v[i] + (i128)N62.v[i] * md;
    ce += (i128)q * d->v[i] + (i128)r * e->v[i] + (i128)N62.v[i] * me;
    d->v[i - 1] = (int64_t)((uint64_t)cd & M62);
    e->v[i - 1] = (int64_t)((uint64_t)ce & M62);
    cd >>= 62;
    ce >>= 62;
  }
  d->v[4] = (int64_t)cd;
  e->v[4] = (int64_t)ce;
}
/* (f, g) <- (t [f, g]) / 2^62 (exact) */
static void update_fg(s62* f, s62* g, const trans2x2* t) {
  const int64_t u = t->u, v = t->v, q = t->q, r = t->r;
  i128 cf = (i128)u * f->v[0] + (i128)v * g->v[0];
  i128 cg = (i128)q * f->v[0] + (i128)r * g->v[0];
  cf >>= 62;
  cg >>= 62;
  for (int i = 1; i < 5; ++i) {
    cf += (i128)u * f->v[i] + (i128)v * g->v[i];
    cg += (i128)q * f->v[i] + (i128)r * g->v[i];
    f->v[i - 1] = (int64_t)((uint64_t)cf & M62);
    g->v[i - 1] = (int64_t)((uint64_t)cg & M62);
    cf >>= 62;
    cg >>= 62;
  }
  f->v[4] = (int64_t)cf;
  g->v[4] = (int64_t)cg;
}
static void sc_to_s62(s62* r, const sc* a) {
  const uint64_t* d = a->d;
  r->v[0] = (int64_t)(d[0] & M62);
  r->v[1] = (int64_t)((d[0] >> 62 | d[1] << 2) & M62);
  r->v[2] = (int64_t)((d[1] >> 60 | d[2] << 4) & M62);
  r->v[3] = (int64_t)((d[2] >> 58 | d[3] << 6) & M62);
  r->v[4] = (int64_t)(d[3] >> 56);
}
/* signed s62 (|value| < 2^257) -> [0, n), negated when neg */
static void s62_to_sc(sc* r, const s62* a, int neg) {
  int64_t l[5];
  i128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += a->v[i];
    l[i] = (int64_t)((uint64_t)c & M62);
    c >>= 62;  /* arithmetic */
  }
  c += a->v[4];
  l[4] = (int64_t)c;
  uint64_t w[4];
  w[0] = (uint64_t)l[0] | (uint64_t)l[1] << 62;
  w[1] = (uint64_t)l[1] >> 2 | (uint64_t)l[2] << 60;
  w[2] = (uint64_t)l[2] >> 4 | (uint64_t)l[3] << 58;
  w[3] = (uint64_t)l[3] >> 6 | (uint64_t)l[4] << 56;
  int64_t top = l[4] >> 8;  /* bits 256 and up, signed */
  while (top < 0) top += (int64_t)u256_add(w, w, SN);
  while (top > 0 || !u256_lt(w, SN)) top -= (int64_t)u256_sub(w, w, SN);
  memcpy(r->d, w, 32);
  if (neg) sc_negate(r, r);
}
static void sc_inverse(sc* r, const sc* x) {
  s62 d = {{0, 0, 0, 0, 0}}, e = {{1, 0, 0, 0, 0}}, f = N62, g;
  sc_to_s62(&g, x);
  int64_t eta = -1;
  for (int it = 0; it < 40; ++it) {
    trans2x2 t;
    eta = divsteps_62_var(eta, (uint64_t)f.v[0], (uint64_t)g.v[0], &t);
    update_de(&d, &e, &t);
    update_fg(&f, &g, &t);
    if (g.v[0] == 0 && (g.v[1] | g.v[2] | g.v[3] | g.v[4]) == 0) break;
  }
  /* f = +-1 */
  s62_to_sc(r, &d, f.v[4] < 0);
}

/* ------------------------------------------------------------------------ */
/* group                                                                    */
typedef struct { fe x, y; } ge;            /* affine (on some isomorphic curve) */
typedef struct { fe x, y, z; int inf; } gej;

static const uint64_t GX[4] = {0x59F2815B16F81798ULL, 0x029BFCDB2DCE28D9ULL, 0x55A06295CE870B07ULL,
                               0x79BE667EF9DCBBACULL};
static const uint64_t GY[4] = {0x9C47D08FFB10D4B8ULL, 0xFD17B448A6855419ULL, 0x5DA4FBFC0E1108A8ULL,
                               0x483ADA7726A3C465ULL};
static const uint64_t BETA[4] = {0xC1396C28719501EEULL, 0x9CF0497512F58995ULL, 0x6E64479EAC3434E9ULL,
                                 0x7AE96A2B657C0710ULL};

/* 2a (a = 0 curves), 2M + 5S: A = X^2, B = Y^2, C = B^2, D = 2((X + B)^2 - A - C),
 * E = 3A, X3 = E^2 - 2D, Y3 = E (D - X3) - 8C, Z3 = 2 Y Z. Inputs magnitude 1. */
static void gej_double(gej* r, const gej* a) {
  if (a->inf) { r->inf = 1; return; }
  fe A, B, C, D, E, F, t, u;
  fe_sqr(&A, &a->x);
  fe_sqr(&B, &a->y);
  fe_sqr(&C, &B);
  fe_add(&t, &a->x, &B);          /* 2 */
  fe_sqr(&t, &t);
  fe_negate(&u, &A, 1);
  fe_add(&t, &t, &u);
  fe_negate(&u, &C, 1);
  fe_add(&D, &t, &u);             /* 9 */
  fe_mul_int(&D, 2);              /* 18 */
  E = A;
  fe_mul_int(&E, 3);              /* 3 */
  fe_sqr(&F, &E);
  fe_mul(&r->z, &a->y, &a->z);
  fe_mul_int(&r->z, 2);           /* 2 */
  fe_normalize_weak(&r->z);
  t = D;
  fe_mul_int(&t, 2);              /* 36 */
  fe_negate(&u, &t, 36);
  fe_add(&r->x, &F, &u);          /* 75 */
  fe_normalize_weak(&r->x);
  fe_negate(&u, &r->x, 1);
  fe_add(&t, &D, &u);             /* 22 */
  fe_mul(&t, &E, &t);
  fe_mul_int(&C, 8);              /* 8 */
  fe_negate(&u, &C, 8);
  fe_add(&r->y, &t, &u);          /* 19 */
  fe_normalize_weak(&r->y);
  r->inf = 0;
}


/* a + (bx, by), (bx, by) affine on the curve of a's Jacobian scale, or with
 * bzinv: the point (bx, by) of a curve whose points a's curve holds as
 * (bx, by, 1 / bzinv) (the z-inverse mixed add of libsecp256k1's G terms).
 * 8M + 3S (+1M with bzinv). Exact: a == b doubles, a == -b gives infinity.
 * zr (optional): the z-ratio H (r.z = a.z H) when a is finite. */
static void gej_add_ge(gej* r, const gej* a, const ge* b, const fe* bzinv, fe* zr) {
  if (a->inf) {
    if (!bzinv) {
      r->x = b->x;
      r->y = b->y;
      fe_set_int(&r->z, 1);
    } else {  /* (bx bzinv^2, by bzinv^3, 1) */
      fe z2, z3;
      fe_sqr(&z2, bzinv);
      fe_mul(&z3, &z2, bzinv);
      fe_mul(&r->x, &b->x, &z2);
      fe_mul(&r->y, &b->y, &z3);
      fe_set_int(&r->z, 1);
    }
    r->inf = 0;
    return;
  }
  fe az, z12, u2, s2, h, rr, hh, hhh, v, t, w, v2;
  if (bzinv) fe_mul(&az, &a->z, bzinv);
  else az = a->z;
  fe_sqr(&z12, &az);
  fe_mul(&u2, &b->x, &z12);
  fe_mul(&t, &az, &z12);
  fe_mul(&s2, &b->y, &t);
  fe_negate(&w, &a->x, 1);
  fe_add(&h, &u2, &w);            /* 5 */
  fe_negate(&w, &a->y, 1);
  fe_add(&rr, &s2, &w);           /* 5 */
  if (fe_normalizes_to_zero(&h)) {
    if (fe_normalizes_to_zero(&rr)) {
      gej_double(r, a);
      return;
    }
    r->inf = 1;
    return;
  }
  if (zr) *zr = h;
  fe_sqr(&hh, &h);
  fe_mul(&hhh, &h, &hh);
  fe_mul(&v, &a->x, &hh);         /* V = X1 H^2 */
  fe_mul(&r->z, &a->z, &h);
  fe_sqr(&t, &rr);
  fe_negate(&w, &hhh, 1);
  fe_add(&t, &t, &w);             /* 5 */
  v2 = v;
  fe_mul_int(&v2, 2);
  fe_negate(&w, &v2, 2);
  fe_add(&t, &t, &w);             /* 11: X3 = R^2 - H^3 - 2V */
  fe_normalize_weak(&t);
  fe_negate(&w, &t, 1);
  fe_add(&v, &v, &w);             /* 5: V - X3 */
  fe_mul(&v, &rr, &v);
  fe_mul(&hhh, &a->y, &hhh);
  fe_negate(&w, &hhh, 1);
  fe_add(&r->y, &v, &w);          /* 5: Y3 = R (V - X3) - Y1 H^3 */
  fe_normalize_weak(&r->y);
  r->x = t;
  r->inf = 0;
}

/* ------------------------------------------------------------------------ */
/* precomputed odd multiples of G and 2^128 G (w = 15), affine on E          */
#define WINDOW_G 15
#define TABLE_G (1 << (WINDOW_G - 2))
#define WINDOW_A 5
#define TABLE_A (1 << (WINDOW_A - 2))
static ge* g_pre;      /* [TABLE_G]: (2i + 1) G */
static ge* g_pre128;   /* [TABLE_G]: (2i + 1) 2^128 G */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void odd_multiples_affine(ge* out, const gej* base, int count) {
  /* base (finite), 2 base affine, then base + k (2 base) in Jacobian, then one
   * batch inversion (Montgomery's trick) to affine */
  gej* e = (gej*)malloc(sizeof(gej) * (size_t)count);
  fe* pre = (fe*)malloc(sizeof(fe) * (size_t)count);
  gej d;
  gej_double(&d, base);
  ge da;
  {
    fe zi, zi2, zi3;
    fe_inv(&zi, &d.z);
    fe_sqr(&zi2, &zi);
    fe_mul(&zi3, &zi2, &zi);
    fe_mul(&da.x, &d.x, &zi2);
    fe_mul(&da.y, &d.y, &zi3);
  }
  e[0] = *base;
  for (int i = 1; i < count; ++i) gej_add_ge(&e[i], &e[i - 1], &da, NULL, NULL);
  pre[0] = e[0].z;
  for (int i = 1; i < count; ++i) fe_mul(&pre[i], &pre[i - 1], &e[i].z);
  fe inv;
  fe_inv(&inv, &pre[count - 1]);
  for (int i = count - 1; i >= 0; --i) {
    fe zi, zi2, zi3;
    if (i > 0) {
      fe_mul(&zi, &inv, &pre[i - 1]);
      fe_mul(&inv, &inv, &e[i].z);
    } else {
      zi = inv;
    }
    fe_sqr(&zi2, &zi);
    fe_mul(&zi3, &zi2, &zi);
    fe_mul(&out[i].x, &e[i].x, &zi2);
    fe_mul(&out[i].y, &e[i].y, &zi3);
    fe_normalize(&out[i].x);
    fe_normalize(&out[i].y);
  }
  free(e);
  free(pre);
}
static void init_tables(void) {
  g_pre = (ge*)malloc(sizeof(ge) * TABLE_G);
  g_pre128 = (ge*)malloc(sizeof(ge) * TABLE_G);
  gej g;
  fe_from_u256(&g.x, GX);
  fe_from_u256(&g.y, GY);
  fe_set_int(&g.z, 1);
  g.inf = 0;
  odd_multiples_affine(g_pre, &g, TABLE_G);
  gej g128 = g;
  for (int i = 0; i < 128; ++i) gej_double(&g128, &g128);
  odd_multiples_affine(g_pre128, &g128, TABLE_G);
}

/* ------------------------------------------------------------------------ */
/* wNAF of a non-negative value of <= len bits (3 x 64-bit limbs): digits 0 or
 * odd in (-2^(w-1), 2^(w-1)), at most one non-zero per w positions; returns
 * the number of positions used */
static inline uint32_t get_bits(const uint64_t* s, int bit, int count) {
  const int li = bit >> 6, bi = bit & 63;
  uint64_t v = s[li] >> bi;
  if (bi + count > 64 && li < 2) v |= s[li + 1] << (64 - bi);
  return (uint32_t)(v & ((1ULL << count) - 1));
}
static int wnaf_var(int* wnaf, int len, const uint64_t s[3], int w, int sign) {
  memset(wnaf, 0, sizeof(int) * (size_t)len);
  int bit = 0, carry = 0, last = -1;
  while (bit < len) {
    if ((int)get_bits(s, bit, 1) == carry) {
      ++bit;
      continue;
    }
    int now = w;
    if (now > len - bit) now = len - bit;
    int word = (int)get_bits(s, bit, now) + carry;
    carry = (word >> (w - 1)) & 1;
    word -= carry << w;
    wnaf[bit] = sign * word;
    last = bit;
    bit += now;
  }
  return last + 1;
}

/* ------------------------------------------------------------------------ */
/* GLV split: k = k1 + k2 lambda (mod n), |k1|, |k2| < 2^129               */
static const uint64_t GLV_G1[4] = {0xE893209A45DBB031ULL, 0x3DAA8A1471E8CA7FULL, 0xE86C90E49284EB15ULL,
                                   0x3086D221A7D46BCDULL};
static const uint64_t GLV_G2[4] = {0x1571B4AE8AC47F71ULL, 0x221208AC9DF506C6ULL, 0x6F547FA90ABFE4C4ULL,
                                   0xE4437ED6010E8828ULL};
static const sc GLV_MB1 = {{0x6F547FA90ABFE4C3ULL, 0xE4437ED6010E8828ULL, 0, 0}};
static const sc GLV_MB2 = {{0xD765CDA83DB1562CULL, 0x8A280AC50774346DULL, 0xFFFFFFFFFFFFFFFEULL,
                            0xFFFFFFFFFFFFFFFFULL}};
static const sc GLV_LAMBDA = {{0xDF02967C1B23BD72ULL, 0x122E22EA20816678ULL, 0xA5261C028812645AULL,
                               0x5363AD4CC05C30E0ULL}};
/* c = round(k g / 2^384) */
static void mul_shift_384(sc* c, const sc* k, const uint64_t g[4]) {
  uint64_t t[8];
  mul256(t, k->d, g);
  u128 x = (u128)t[6] + (t[5] >> 63);
  c->d[0] = (uint64_t)x;
  x >>= 64;
  x += t[7];
  c->d[1] = (uint64_t)x;
  c->d[2] = (uint64_t)(x >> 64);
  c->d[3] = 0;
}
/* magnitudes (3 limbs) and signs of the two halves */
static void glv_split(const sc* k, uint64_t m1[3], int* s1, uint64_t m2[3], int* s2) {
  sc c1, c2, t1, t2, k1, k2;
  mul_shift_384(&c1, k, GLV_G1);
  mul_shift_384(&c2, k, GLV_G2);
  sc_mul(&t1, &c1, &GLV_MB1);
  sc_mul(&t2, &c2, &GLV_MB2);
  sc_add(&k2, &t1, &t2);
  sc_mul(&t1, &k2, &GLV_LAMBDA);
  sc_negate(&t1, &t1);
  sc_add(&k1, k, &t1);
  *s1 = 1;
  *s2 = 1;
  if (sc_is_high(&k1)) { sc_negate(&k1, &k1); *s1 = -1; }
  if (sc_is_high(&k2)) { sc_negate(&k2, &k2); *s2 = -1; }
  memcpy(m1, k1.d, 24);
  memcpy(m2, k2.d, 24);
}

/* ------------------------------------------------------------------------ */
/* R = u1 G + u2 Q (Strauss: one doubling chain, four wNAF streams). R is left
 * on the isomorphic curve of the Q table: its Z on E is R.z * zg. */
#define WNAF_LEN 130
static void ecmult(gej* r, fe* zg, const ge* q, const sc* u1, const sc* u2) {
  /* the odd multiples 1Q .. 15Q with one global Z (libsecp256k1's
   * "effective affine" table): 2Q = D (Jacobian, z dz); on the curve of scale
   * dz, Q' = (qx dz^2, qy dz^3) and D is affine, so Q' + k D are mixed adds;
   * the z-ratios then rescale every entry onto the last entry's curve */
  ge pre[TABLE_A], prel[TABLE_A];
  {
    gej qj, d, e[TABLE_A];
    fe zr[TABLE_A];
    qj.x = q->x; qj.y = q->y; fe_set_int(&qj.z, 1); qj.inf = 0;
    gej_double(&d, &qj);
    ge da = {d.x, d.y};
    fe z2, z3;
    fe_sqr(&z2, &d.z);
    fe_mul(&z3, &z2, &d.z);
    fe_mul(&e[0].x, &q->x, &z2);
    fe_mul(&e[0].y, &q->y, &z3);
    fe_set_int(&e[0].z, 1);
    e[0].inf = 0;
    for (int k = 1; k < TABLE_A; ++k) gej_add_ge(&e[k], &e[k - 1], &da, NULL, &zr[k]);
    fe zs;
    fe_set_int(&zs, 1);
    for (int k = TABLE_A - 1; k >= 0; --k) {
      fe s2, s3;
      fe_sqr(&s2, &zs);
      fe_mul(&s3, &s2, &zs);
      fe_mul(&pre[k].x, &e[k].x, &s2);
      fe_mul(&pre[k].y, &e[k].y, &s3);
      if (k > 0) fe_mul(&zs, &zs, &zr[k]);
    }
    fe_mul(zg, &d.z, &e[TABLE_A - 1].z);
    fe beta;
    fe_from_u256(&beta, BETA);
    for (int k = 0; k < TABLE_A; ++k) {
      fe_mul(&prel[k].x, &pre[k].x, &beta);
      prel[k].y = pre[k].y;
    }
  }
  uint64_t m1[3], m2[3], g1[3] = {u1->d[0], u1->d[1], 0}, g2[3] = {u1->d[2], u1->d[3], 0};
  int s1, s2;
  glv_split(u2, m1, &s1, m2, &s2);
  int w1[WNAF_LEN], w2[WNAF_LEN], wg1[WNAF_LEN], wg2[WNAF_LEN];
  const int l1 = wnaf_var(w1, WNAF_LEN, m1, WINDOW_A, s1);
  const int l2 = wnaf_var(w2, WNAF_LEN, m2, WINDOW_A, s2);
  const int lg1 = wnaf_var(wg1, WNAF_LEN, g1, WINDOW_G, 1);
  const int lg2 = wnaf_var(wg2, WNAF_LEN, g2, WINDOW_G, 1);
  int bits = l1;
  if (l2 > bits) bits = l2;
  if (lg1 > bits) bits = lg1;
  if (lg2 > bits) bits = lg2;
  r->inf = 1;
  for (int i = bits - 1; i >= 0; --i) {
    gej_double(r, r);
    int d;
    ge t;
    if (i < l1 && (d = w1[i]) != 0) {
      t = pre[(d > 0 ? d : -d) >> 1];
      if (d < 0) fe_negate(&t.y, &t.y, 1);
      gej_add_ge(r, r, &t, NULL, NULL);
    }
    if (i < l2 && (d = w2[i]) != 0) {
      t = prel[(d > 0 ? d : -d) >> 1];
      if (d < 0) fe_negate(&t.y, &t.y, 1);
      gej_add_ge(r, r, &t, NULL, NULL);
    }
    if (i < lg1 && (d = wg1[i]) != 0) {
      t = g_pre[(d > 0 ? d : -d) >> 1];
      if (d < 0) fe_negate(&t.y, &t.y, 1);
      gej_add_ge(r, r, &t, zg, NULL);
    }
    if (i < lg2 && (d = wg2[i]) != 0) {
      t = g_pre128[(d > 0 ? d : -d) >> 1];
      if (d < 0) fe_negate(&t.y, &t.y, 1);
      gej_add_ge(r, r, &t, zg, NULL);
    }
  }
}

/* ------------------------------------------------------------------------ */
/* secp256k1_ec_pubkey_parse semantics (the port's pubkey_parse)            */
static const uint64_t FE_P64[4] = {0xFFFFFFFEFFFFFC2FULL, ~0ULL, ~0ULL, ~0ULL};
static int pubkey_parse(ge* q, const uint8_t* pk, size_t len) {
  uint64_t xv[4], yv[4];
  fe seven, x3, rhs, y, y2;
  fe_set_int(&seven, 7);
  if (len == 33 && (pk[0] == 2 || pk[0] == 3)) {
    u256_from_be(xv, pk + 1);
    if (!u256_lt(xv, FE_P64)) return 0;
    fe_from_u256(&q->x, xv);
    fe_sqr(&x3, &q->x);
    fe_mul(&x3, &x3, &q->x);
    fe_add(&rhs, &x3, &seven);
    fe_normalize(&rhs);
    fe_sqrt_cand(&y, &rhs);
    fe_sqr(&y2, &y);
    fe_normalize(&y2);
    if (!fe_equal_norm(&y2, &rhs)) return 0;
    fe_normalize(&y);
    if ((int)(y.n[0] & 1) != (pk[0] & 1)) {
      fe_negate(&y, &y, 1);
      fe_normalize(&y);
    }
    q->y = y;
    return 1;
  }
  if (len == 65 && (pk[0] == 4 || pk[0] == 6 || pk[0] == 7)) {
    u256_from_be(xv, pk + 1);
    u256_from_be(yv, pk + 33);
    if (!u256_lt(xv, FE_P64) || !u256_lt(yv, FE_P64)) return 0;
    if (pk[0] != 4 && (int)(yv[0] & 1) != (pk[0] & 1)) return 0;
    fe_from_u256(&q->x, xv);
    fe_from_u256(&q->y, yv);
    fe_sqr(&x3, &q->x);
    fe_mul(&x3, &x3, &q->x);
    fe_add(&rhs, &x3, &seven);
    fe_normalize(&rhs);
    fe_sqr(&y2, &q->y);
    fe_normalize(&y2);
    return fe_equal_norm(&y2, &rhs);
  }
  return 0;
}

/* One 168-byte record (include/hkv.h layout). mode 0 = LIBSECP, 1 = HASKOIN. */
int hkvo_fast_verify_record(const uint8_t* rec, int mode) {
  pthread_once(&g_once, init_tables);
  sc r, s, m;
  u256_from_be(r.d, rec + 32);
  u256_from_be(s.d, rec + 64);
  if (!u256_lt(r.d, SN) || !u256_lt(s.d, SN)) return 0;  /* compact parse: overflow fails */
  const unsigned pklen = rec[96];
  ge q;
  if (pklen > 65 || !pubkey_parse(&q, rec + 97, pklen)) return 0;
  if (sc_is_high(&s)) {
    if (mode == 1) sc_negate(&s, &s);  /* verifyHashSig: normalize */
    else return 0;                      /* secp256k1_ecdsa_verify: reject high-S */
  }
  if (sc_is_zero(&r) || sc_is_zero(&s)) return 0;
  u256_from_be(m.d, rec);
  if (!u256_lt(m.d, SN)) u256_sub(m.d, m.d, SN);
  sc sinv, u1, u2;
  sc_inverse(&sinv, &s);
  sc_mul(&u1, &m, &sinv);
  sc_mul(&u2, &r, &sinv);
  gej R;
  fe zg;
  ecmult(&R, &zg, &q, &u1, &u2);
  if (R.inf) return 0;
  /* x(R) == r  <=>  r Z^2 == X (Z on E = R.z zg) */
  fe z, z2, xr, t, X = R.x;
  fe_mul(&z, &R.z, &zg);
  fe_sqr(&z2, &z);
  fe_normalize(&X);
  fe_from_u256(&xr, r.d);
  fe_mul(&t, &xr, &z2);
  fe_normalize(&t);
  if (fe_equal_norm(&t, &X)) return 1;
  uint64_t rn[4];
  const uint64_t c = u256_add(rn, r.d, SN);
  if (c || !u256_lt(rn, FE_P64)) return 0;
  fe_from_u256(&xr, rn);
  fe_mul(&t, &xr, &z2);
  fe_normalize(&t);
  return fe_equal_norm(&t, &X);
}

struct fjob { const uint8_t* recs; size_t lo, hi; int mode; uint8_t* verdicts; };
static void* fworker(void* arg) {
  struct fjob* j = (struct fjob*)arg;
  for (size_t i = j->lo; i < j->hi; ++i) j->verdicts[i] = (uint8_t)hkvo_fast_verify_record(j->recs + i * 168, j->mode);
  return NULL;
}
/* Verify n records on nthreads pthreads; verdicts[i] = 0/1 (hkvo_verify_batch's contract). */
int hkvo_fast_verify_batch(const uint8_t* recs, size_t n, int mode, uint8_t* verdicts, int nthreads) {
  pthread_once(&g_once, init_tables);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  int created[256] = {0};
  struct fjob jobs[256];
  const size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
  for (int t = 0; t < nthreads; ++t) {
    size_t lo = (size_t)t * per, hi = lo + per;
    if (lo >= n) break;
    if (hi > n) hi = n;
    jobs[t] = (struct fjob){recs, lo, hi, mode, verdicts};
    if (pthread_create(&th[t], NULL, fworker, &jobs[t]) == 0) created[t] = 1;
    else fworker(&jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t)
    if (created[t]) pthread_join(th[t], NULL);
  return 0;
}

/* test hooks: s^-1 mod n and the GLV split on big-endian 32-byte values */
void hkvo_fast_sc_inverse(const uint8_t a[32], uint8_t out[32]) {
  sc x, r;
  u256_from_be(x.d, a);
  sc_inverse(&r, &x);
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) out[(3 - i) * 8 + j] = (uint8_t)(r.d[i] >> (56 - 8 * j));
}
/* k1, k2 magnitudes as 24-byte little-endian limb arrays, signs +-1 */
void hkvo_fast_glv_split(const uint8_t k[32], uint64_t m1[3], int* s1, uint64_t m2[3], int* s2) {
  sc x;
  u256_from_be(x.d, k);
  glv_split(&x, m1, s1, m2, s2);
}
