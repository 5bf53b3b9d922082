// hkv_scalar.h — secp256k1 scalar arithmetic mod the group order n, one
// scalar per lane, 8 little-endian 32-bit limbs, always fully reduced (< n).
//
// n = 2^256 - NC with NC = 0x1_45512319_50B75FC4_402DA173_2FC9BEBF (129 bits),
// so a 512-bit product folds as L + H*NC in three shrinking passes.
// Replaces (semantically) libsecp256k1's secp256k1_scalar_* used by
// secp256k1_ecdsa_sig_verify [dep; SURVEY.md §8(a) a3, a5, a6].
#pragma once
#include "hkv_field.h"
#include "hkv_safegcd.h"

namespace hkv {

struct sc { uint32_t v[8]; };

__constant__ static const uint32_t SC_N[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                                              0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
__constant__ static const uint32_t SC_HALF_N[8] = {0x681B20A0u, 0xDFE92F46u, 0x57A4501Du, 0x5D576E73u,
                                                   0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};
// NC = 2^256 - n, low 4 limbs (the fifth limb is 1)
constexpr uint32_t NC0 = 0x2FC9BEBFu, NC1 = 0x402DA173u, NC2 = 0x50B75FC4u, NC3 = 0x45512319u;

HKV_DEV void sc_set_u32(sc& r, uint32_t x) {
  r.v[0] = x;
#pragma unroll
  for (int i = 1; i < 8; ++i) r.v[i] = 0;
}
HKV_DEV bool u256_lt(const uint32_t* a, const uint32_t* b) {
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) (void)subb(a[i], b[i], bw);
  return bw != 0;
}
HKV_DEV bool u256_is_zero(const uint32_t* a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a[i];
  return o == 0;
}
// r = a - n if a >= n (a < 2^256 < 2n)
HKV_DEV void sc_cond_sub_n(uint32_t* a) {
  uint32_t t[8], bw = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) t[i] = subb(a[i], SC_N[i], bw);
  const bool ge = (bw == 0);
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = ge ? t[i] : a[i];
}

// acc[0..len) += h[0..hl) * NC  (acc must be wide enough for the result)
template <int LEN, int HL>
HKV_DEV void mul_add_nc(uint32_t* acc, const uint32_t* h) {
  const uint32_t nc[4] = {NC0, NC1, NC2, NC3};
  // h * NC_low (4 limbs)
#pragma unroll
  for (int i = 0; i < HL; ++i) {
    uint64_t q = 0;
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      q = (uint64_t)h[i] * nc[j] + (q >> 32);
      acc[i + j] = addc(acc[i + j], (uint32_t)q, c);
    }
    acc[i + 4] = addc(acc[i + 4], (uint32_t)(q >> 32), c);
#pragma unroll
    for (int k = i + 5; k < LEN; ++k) acc[k] = addc(acc[k], 0u, c);
  }
  // h << 128 (NC limb 4 == 1)
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < HL; ++i) acc[i + 4] = addc(acc[i + 4], h[i], c);
#pragma unroll
  for (int k = HL + 4; k < LEN; ++k) acc[k] = addc(acc[k], 0u, c);
}

HKV_DEV void sc_reduce512(sc& r, const uint32_t t[16]) {
  // pass 1: 13 limbs = L + H*NC   (H*NC < 2^385)
  uint32_t a[14];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = t[i];
#pragma unroll
  for (int i = 8; i < 14; ++i) a[i] = 0;
  mul_add_nc<14, 8>(a, t + 8);
  // pass 2: a[8..13) (< 2^131) * NC + a[0..8)  (< 2^261)
  uint32_t b[10];
#pragma unroll
  for (int i = 0; i < 8; ++i) b[i] = a[i];
  b[8] = 0;
  b[9] = 0;
  mul_add_nc<10, 5>(b, a + 8);
  // pass 3: b[8..10) (< 2^6) * NC + b[0..8)
  uint32_t c8[9];
#pragma unroll
  for (int i = 0; i < 8; ++i) c8[i] = b[i];
  c8[8] = 0;
  {
    uint32_t h = b[8];  // b[9] is 0 here
    uint64_t q = 0;
    uint32_t c = 0;
    const uint32_t nc[4] = {NC0, NC1, NC2, NC3};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      q = (uint64_t)h * nc[j] + (q >> 32);
      c8[j] = addc(c8[j], (uint32_t)q, c);
    }
    c8[4] = addc(c8[4], (uint32_t)(q >> 32) + h, c);  // + h<<128; (q>>32)+h < 2^32
#pragma unroll
    for (int k = 5; k < 9; ++k) c8[k] = addc(c8[k], 0u, c);
  }
  // c8[8] in {0,1}: fold once more (value then < 2^256)
  {
    uint32_t h = c8[8];
    uint32_t c = 0;
    c8[0] = addc(c8[0], h * NC0, c);
    c8[1] = addc(c8[1], h * NC1, c);
    c8[2] = addc(c8[2], h * NC2, c);
    c8[3] = addc(c8[3], h * NC3, c);
    c8[4] = addc(c8[4], h, c);
#pragma unroll
    for (int k = 5; k < 8; ++k) c8[k] = addc(c8[k], 0u, c);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = c8[i];
  sc_cond_sub_n(r.v);
}

HKV_DEV void sc_mul(sc& r, const sc& a, const sc& b) {
  uint32_t t[16];
  mul512(t, a.v, b.v);
  sc_reduce512(r, t);
}
HKV_DEV void sc_sqr(sc& r, const sc& a) {
  uint32_t t[16];
  sqr512(t, a.v);
  sc_reduce512(r, t);
}
HKV_DEV void sc_add(sc& r, const sc& a, const sc& b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = addc(a.v[i], b.v[i], c);
  // a + b < 2n; if carry, (a+b-2^256) + NC = a + b - n (< n)
  uint32_t k = 0;
  r.v[0] = addc(r.v[0], c ? NC0 : 0u, k);
  r.v[1] = addc(r.v[1], c ? NC1 : 0u, k);
  r.v[2] = addc(r.v[2], c ? NC2 : 0u, k);
  r.v[3] = addc(r.v[3], c ? NC3 : 0u, k);
  r.v[4] = addc(r.v[4], c, k);
#pragma unroll
  for (int i = 5; i < 8; ++i) r.v[i] = addc(r.v[i], 0u, k);
  sc_cond_sub_n(r.v);
}
HKV_DEV void sc_neg(sc& r, const sc& a) {  // n - a, with 0 -> 0
  const bool z = u256_is_zero(a.v);
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = z ? 0u : subb(SC_N[i], a.v[i], bw);
}
HKV_DEV void sc_sub(sc& r, const sc& a, const sc& b) {
  sc nb;
  sc_neg(nb, b);
  sc_add(r, a, nb);
}
HKV_DEV bool sc_is_high(const sc& a) { return u256_lt(SC_HALF_N, a.v); }

HKV_DEV void sc_sqr_n(sc& r, const sc& a, int n) {
  sc_sqr(r, a);
  for (int i = 1; i < n; ++i) sc_sqr(r, r);
}

// r = a^-1 mod n (0 < a < n; a = 0 gives 0): constant-time safegcd
// (hkv_safegcd.h), ≈ 10x fewer VALU instructions than the Fermat chain
// a^(n-2) it replaced (255 squarings + 75 multiplications mod n).
HKV_DEV void sc_inv(sc& r, const sc& a) { sgcd::inv_mod_n(r.v, a.v); }

HKV_DEV void sc_from_be_words(sc& r, const uint32_t w[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = __builtin_bswap32(w[7 - i]);
}

// GLV split constants (oracle/secp256k1_oracle.py derives the basis).
// g1 = round(2^384 * b2 / n), g2 = round(2^384 * (-b1) / n)
__constant__ static const uint32_t GLV_G1[8] = {0x45DBB031u, 0xE893209Au, 0x71E8CA7Fu, 0x3DAA8A14u,
                                                0x9284EB15u, 0xE86C90E4u, 0xA7D46BCDu, 0x3086D221u};
__constant__ static const uint32_t GLV_G2[8] = {0x8AC47F71u, 0x1571B4AEu, 0x9DF506C6u, 0x221208ACu,
                                                0x0ABFE4C4u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u};
// -b1 (128 bits) and -b2 mod n
__constant__ static const uint32_t GLV_MB1[8] = {0x0ABFE4C3u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u, 0, 0, 0, 0};
__constant__ static const uint32_t GLV_MB2[8] = {0x3DB1562Cu, 0xD765CDA8u, 0x0774346Du, 0x8A280AC5u,
                                                 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
__constant__ static const uint32_t GLV_LAMBDA[8] = {0x1B23BD72u, 0xDF02967Cu, 0x20816678u, 0x122E22EAu,
                                                    0x8812645Au, 0xA5261C02u, 0xC05C30E0u, 0x5363AD4Cu};

// c = round(k * g / 2^384): bits 384..511 of the product plus bit 383.
HKV_DEV void glv_round(sc& c, const sc& k, const uint32_t* g) {
  uint32_t t[16];
  mul512(t, k.v, g);
  uint32_t rnd = t[11] >> 31;
  uint32_t cy = rnd;
  c.v[0] = addc(t[12], 0u, cy);
  c.v[1] = addc(t[13], 0u, cy);
  c.v[2] = addc(t[14], 0u, cy);
  c.v[3] = addc(t[15], 0u, cy);
#pragma unroll
  for (int i = 4; i < 8; ++i) c.v[i] = 0;
}

// k = k1 + k2*lambda (mod n); outputs magnitudes (< 2^129, 5 limbs) and signs.
// Returns false if a magnitude does not fit (never for a correct basis).
HKV_DEV bool glv_split(const sc& k, uint32_t k1m[5], bool& neg1, uint32_t k2m[5], bool& neg2) {
  sc c1, c2, t1, t2, k2, k1;
  glv_round(c1, k, GLV_G1);
  glv_round(c2, k, GLV_G2);
  sc mb1, mb2, lam;
#pragma unroll
  for (int i = 0; i < 8; ++i) { mb1.v[i] = GLV_MB1[i]; mb2.v[i] = GLV_MB2[i]; lam.v[i] = GLV_LAMBDA[i]; }
  sc_mul(t1, c1, mb1);
  sc_mul(t2, c2, mb2);
  sc_add(k2, t1, t2);
  sc_mul(t1, k2, lam);
  sc_sub(k1, k, t1);
  neg1 = sc_is_high(k1);
  neg2 = sc_is_high(k2);
  sc a1, a2;
  sc_neg(a1, k1);
  sc_neg(a2, k2);
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    k1m[i] = neg1 ? a1.v[i] : k1.v[i];
    k2m[i] = neg2 ? a2.v[i] : k2.v[i];
  }
#pragma unroll
  for (int i = 5; i < 8; ++i) ok = ok && ((neg1 ? a1.v[i] : k1.v[i]) == 0) && ((neg2 ? a2.v[i] : k2.v[i]) == 0);
  ok = ok && (k1m[4] < 2u) && (k2m[4] < 2u);  // < 2^129
  return ok;
}

}  // namespace hkv
