// hkv_field.h — secp256k1 base-field arithmetic (mod p = 2^256 - 2^32 - 977)
// for gfx950, one field element per lane.
//
// Representation: 8 little-endian 32-bit limbs, value < 2^256 and congruent
// to the element mod p ("weak" form; may exceed p by < 2^32+977). Full
// normalisation (< p) happens only where bits are observed: comparisons,
// parity, serialisation.
//
// Instruction mapping (measured, profiles/r01_ubench_int.json): the limb
// product v_mad_u64_u32 issues at half rate (64 lane-ops/clk/CU), add-with-
// carry at full rate. A product row a_i * B is a v_mad_u64_u32 chain whose
// 64-bit addend is the previous product's high word (no carry flags needed);
// rows are accumulated with v_add_co/v_addc chains (__builtin_addc).
// Reduction uses 2^256 = 2^32 + 977 (mod p): one 8-product mad chain by 977
// plus a limb shift, then a 64-bit top fold.
//
// Replaces (semantically) libsecp256k1's secp256k1_fe_* used inside
// secp256k1_ecdsa_verify [dep; SURVEY.md §8(a) a3].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HKV_DEV __device__ __forceinline__

namespace hkv {

struct fe { uint32_t v[8]; };

HKV_DEV uint32_t addc(uint32_t a, uint32_t b, uint32_t& c) {
  uint32_t co;
  uint32_t r = __builtin_addc(a, b, c, &co);
  c = co;
  return r;
}
HKV_DEV uint32_t subb(uint32_t a, uint32_t b, uint32_t& bw) {
  uint32_t bo;
  uint32_t r = __builtin_subc(a, b, bw, &bo);
  bw = bo;
  return r;
}

// p = 2^256 - C, C = 2^32 + 977
constexpr uint32_t FE_C0 = 977u;

HKV_DEV void fe_set_zero(fe& r) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = 0;
}
HKV_DEV void fe_set_u32(fe& r, uint32_t x) {
  r.v[0] = x;
#pragma unroll
  for (int i = 1; i < 8; ++i) r.v[i] = 0;
}
HKV_DEV void fe_cmov(fe& r, const fe& a, bool f) {  // r = f ? a : r
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = f ? a.v[i] : r.v[i];
}

// r (< 2^256) += c * (2^32 + 977) where c in {0,1} came out of a 2^256 wrap.
// After a wrap the value is < C, so the second fold cannot carry past limb 2.
HKV_DEV void fe_fold_carry(fe& r, uint32_t c) {
  uint32_t k = 0;
  r.v[0] = addc(r.v[0], c * FE_C0, k);
  r.v[1] = addc(r.v[1], c, k);
  uint32_t c2 = 0;
#pragma unroll
  for (int i = 2; i < 8; ++i) r.v[i] = addc(r.v[i], (i == 2) ? k : 0u, c2);
  // c2: wrapped again (value was in [2^256 - C, 2^256)); fold once more —
  // the result is then < 2C and cannot wrap.
  uint32_t k2 = 0;
  r.v[0] = addc(r.v[0], c2 * FE_C0, k2);
  r.v[1] = addc(r.v[1], c2, k2);
  r.v[2] += k2;
}

HKV_DEV void fe_add(fe& r, const fe& a, const fe& b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = addc(a.v[i], b.v[i], c);
  fe_fold_carry(r, c);
}

// r = a - b (mod p): on borrow add p back, i.e. subtract C (mod 2^256);
// a second borrow (only when b > p + a) subtracts C once more.
HKV_DEV void fe_sub(fe& r, const fe& a, const fe& b) {
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = subb(a.v[i], b.v[i], bw);
  uint32_t b2 = 0;
  r.v[0] = subb(r.v[0], bw * FE_C0, b2);
  r.v[1] = subb(r.v[1], bw, b2);
#pragma unroll
  for (int i = 2; i < 8; ++i) r.v[i] = subb(r.v[i], 0u, b2);
  uint32_t b3 = 0;
  r.v[0] = subb(r.v[0], b2 * FE_C0, b3);
  r.v[1] = subb(r.v[1], b2, b3);
  r.v[2] -= b3;
}

HKV_DEV void fe_neg(fe& r, const fe& a) {
  fe z;
  fe_set_zero(z);
  fe_sub(r, z, a);
}

// Fold a 288-bit value (8 limbs + 64-bit top < 2^35) to 8 limbs.
HKV_DEV void fe_fold_top(fe& r, uint64_t top) {
  // top * C = top*977 + top*2^32 ; top < 2^35 -> top*977 < 2^45
  uint64_t y = top * (uint64_t)FE_C0;
  uint64_t z12 = (y >> 32) + top;  // < 2^36
  uint32_t c = 0;
  r.v[0] = addc(r.v[0], (uint32_t)y, c);
  r.v[1] = addc(r.v[1], (uint32_t)z12, c);
  r.v[2] = addc(r.v[2], (uint32_t)(z12 >> 32), c);
#pragma unroll
  for (int i = 3; i < 8; ++i) r.v[i] = addc(r.v[i], 0u, c);
  // wrapped: value now < 2^36ish, adding C cannot wrap again
  uint32_t k = 0;
  r.v[0] = addc(r.v[0], c * FE_C0, k);
  r.v[1] = addc(r.v[1], c, k);
  r.v[2] += k;
}

// Reduce the 512-bit product t[16] mod p into r (weak form).
HKV_DEV void fe_reduce512(fe& r, const uint32_t t[16]) {
  // m = H * 977 (9 limbs, m[8] < 977)
  uint32_t m[8];
  uint64_t q = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    q = (uint64_t)t[8 + j] * FE_C0 + (q >> 32);
    m[j] = (uint32_t)q;
  }
  uint32_t m8 = (uint32_t)(q >> 32);
  // r = L + m + (H << 32)
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r.v[j] = addc(t[j], m[j], c);
  uint64_t top = (uint64_t)m8 + c;
  uint32_t c2 = 0;
#pragma unroll
  for (int j = 1; j < 8; ++j) r.v[j] = addc(r.v[j], t[8 + j - 1], c2);
  top += (uint64_t)t[15] + c2;  // < 2^33 + 2^10
  fe_fold_top(r, top);
}

// 256x256 -> 512 bit product, row-wise mad chains.
HKV_DEV void mul256(uint32_t t[16], const uint32_t* a, const uint32_t* b) {
  {
    uint64_t q = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      q = (uint64_t)a[0] * b[j] + (q >> 32);
      t[j] = (uint32_t)q;
    }
    t[8] = (uint32_t)(q >> 32);
  }
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    uint64_t q = 0;
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      q = (uint64_t)a[i] * b[j] + (q >> 32);
      t[i + j] = addc(t[i + j], (uint32_t)q, c);
    }
    t[i + 8] = (uint32_t)(q >> 32) + c;  // cannot overflow (row + partial < 2^(32(i+9)))
  }
}

// 256-bit square: 28 off-diagonal products doubled + 8 diagonal squares.
HKV_DEV void sqr256(uint32_t t[16], const uint32_t* a) {
#pragma unroll
  for (int k = 0; k < 16; ++k) t[k] = 0;
  // off-diagonal rows: a_i * a_j, j > i
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    uint64_t q = 0;
    uint32_t c = 0;
#pragma unroll
    for (int j = i + 1; j < 8; ++j) {
      q = (uint64_t)a[i] * a[j] + (q >> 32);
      t[i + j] = addc(t[i + j], (uint32_t)q, c);
    }
    t[i + 8] = addc(t[i + 8], (uint32_t)(q >> 32), c);  // t[i+8] is 0 here except via carries... keep generic
    // propagate remaining carry (only possible into t[i+9] which is still 0)
    if (i + 9 < 16) t[i + 9] += c;
  }
  // double
  t[15] = (t[15] << 1) | (t[14] >> 31);
#pragma unroll
  for (int k = 14; k > 0; --k) t[k] = (t[k] << 1) | (t[k - 1] >> 31);
  t[0] <<= 1;
  // add diagonal squares
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t d = (uint64_t)a[i] * a[i];
    t[2 * i] = addc(t[2 * i], (uint32_t)d, c);
    t[2 * i + 1] = addc(t[2 * i + 1], (uint32_t)(d >> 32), c);
  }
}

HKV_DEV void fe_mul(fe& r, const fe& a, const fe& b) {
  uint32_t t[16];
  mul256(t, a.v, b.v);
  fe_reduce512(r, t);
}
HKV_DEV void fe_sqr(fe& r, const fe& a) {
  uint32_t t[16];
  sqr256(t, a.v);
  fe_reduce512(r, t);
}

// r = a * k for small k (< 2^16)
HKV_DEV void fe_mul_small(fe& r, const fe& a, uint32_t k) {
  uint64_t q = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    q = (uint64_t)a.v[j] * k + (q >> 32);
    r.v[j] = (uint32_t)q;
  }
  fe_fold_top(r, q >> 32);
}

// Full normalisation to [0, p).
HKV_DEV void fe_normalize(fe& r) {
  // t = r + C ; carry out <=> r >= p ; then r - p = t mod 2^256
  fe t;
  uint32_t c = 0;
  t.v[0] = addc(r.v[0], FE_C0, c);
  t.v[1] = addc(r.v[1], 1u, c);
#pragma unroll
  for (int i = 2; i < 8; ++i) t.v[i] = addc(r.v[i], 0u, c);
  fe_cmov(r, t, c != 0);
}

HKV_DEV bool fe_is_zero(const fe& a) {  // a in weak form
  fe t = a;
  fe_normalize(t);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= t.v[i];
  return o == 0;
}
HKV_DEV bool fe_equal(const fe& a, const fe& b) {
  fe d;
  fe_sub(d, a, b);
  return fe_is_zero(d);
}
// Compare normalised values; a, b must already be < p.
HKV_DEV bool fe_eq_norm(const fe& a, const fe& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.v[i] ^ b.v[i];
  return o == 0;
}

HKV_DEV void fe_sqr_n(fe& r, const fe& a, int n) {
  fe_sqr(r, a);
  for (int i = 1; i < n; ++i) fe_sqr(r, r);
}

// x_k = a^(2^k - 1) chain pieces shared by sqrt and inverse.
// Returns x2, x22, x223 (and x1 = a).
HKV_DEV void fe_pow_chain223(const fe& a, fe& x2, fe& x22, fe& x223) {
  fe x3, x6, x9, x11, x44, x88, x176, x220, t;
  fe_sqr(x2, a);
  fe_mul(x2, x2, a);
  fe_sqr(x3, x2);
  fe_mul(x3, x3, a);
  fe_sqr_n(t, x3, 3);
  fe_mul(x6, t, x3);
  fe_sqr_n(t, x6, 3);
  fe_mul(x9, t, x3);
  fe_sqr_n(t, x9, 2);
  fe_mul(x11, t, x2);
  fe_sqr_n(t, x11, 11);
  fe_mul(x22, t, x11);
  fe_sqr_n(t, x22, 22);
  fe_mul(x44, t, x22);
  fe_sqr_n(t, x44, 44);
  fe_mul(x88, t, x44);
  fe_sqr_n(t, x88, 88);
  fe_mul(x176, t, x88);
  fe_sqr_n(t, x176, 44);
  fe_mul(x220, t, x44);
  fe_sqr_n(t, x220, 3);
  fe_mul(x223, t, x3);
}

// r = a^((p+1)/4): a square root candidate of a. (p+1)/4 = 223 ones, 0,
// 22 ones, 0000, 11, 00.
HKV_DEV void fe_sqrt_cand(fe& r, const fe& a) {
  fe x2, x22, x223, t;
  fe_pow_chain223(a, x2, x22, x223);
  fe_sqr_n(t, x223, 23);
  fe_mul(t, t, x22);
  fe_sqr_n(t, t, 6);
  fe_mul(t, t, x2);
  fe_sqr_n(r, t, 2);
}

// r = a^(p-2) = a^-1 (a != 0). p-2 = 223 ones, 0, 22 ones, 00001, 011, 01.
HKV_DEV void fe_inv(fe& r, const fe& a) {
  fe x2, x22, x223, t;
  fe_pow_chain223(a, x2, x22, x223);
  fe_sqr_n(t, x223, 23);
  fe_mul(t, t, x22);
  fe_sqr_n(t, t, 5);
  fe_mul(t, t, a);
  fe_sqr_n(t, t, 3);
  fe_mul(t, t, x2);
  fe_sqr_n(t, t, 2);
  fe_mul(r, t, a);
}

// big-endian 32 bytes -> limbs (no reduction)
HKV_DEV void fe_from_be_words(fe& r, const uint32_t w[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = __builtin_bswap32(w[7 - i]);
}

// a < p as a 256-bit integer (a given as raw limbs)
HKV_DEV bool u256_lt_p(const uint32_t* a) {
  // a < p  <=>  a + C < 2^256 (no carry)
  uint32_t c = 0;
  (void)addc(a[0], FE_C0, c);
  (void)addc(a[1], 1u, c);
#pragma unroll
  for (int i = 2; i < 8; ++i) (void)addc(a[i], 0u, c);
  return c == 0;
}

}  // namespace hkv
