// hkv_safegcd.h — constant-time modular inversion mod the group order n by
// Bernstein–Yang "safegcd" divsteps (Bernstein, Yang: "Fast constant-time
// gcd computation and modular inversion", TCHES 2019), 30 divsteps per
// matrix over signed radix-2^30 limbs.
//
// Replaces the Fermat chain a^(n-2) (≈ 255 squarings + 75 multiplications
// mod n) used for s^-1 in secp256k1_ecdsa_sig_verify step (5) [dep; SURVEY.md
// §8(a) a3]. The result is the same field element; only the cost changes:
// 25 outer iterations × (30 divsteps on the low word, in libsecp256k1's
// variable-time form, one 2×2 matrix applied to (f, g) and, mod n, to (d, e)).
//
// Bound: for odd f < 2^256 and 0 <= g < f, ⌊(49·256 + 80)/17⌋ = 742
// divsteps (delta starting at 1) reach g = 0 (paper, Theorem 11.2); at most
// 25 × 30 = 750 are run, fewer with HKV_SGCD_EARLY (random inputs reach g = 0
// after 19 iterations in the worst lane of a wave). At that point f = ±1 and
// d·f ≡ g0^-1 (mod n). Inputs are public (signatures, keys), so the
// data-dependent stop leaks nothing.
//
// Limb form ("signed30"): limbs 0..7 hold 30 bits each in [0, 2^30), limb 8
// is signed, value = Σ l_i 2^(30 i). d and e stay in (-2n, n).
//
// Written __host__ __device__ so the host build (tests/test_safegcd.py)
// checks the same code the kernels run.
//
// Attribution: the signed-30 divstep / matrix-update structure (in
// particular update_de's sign masks and the "md -= (m^-1 * cd + md) mod 2^30"
// correction that makes the division by 2^30 exact) follows libsecp256k1's
// src/modinv32_impl.h (MIT License, Copyright (c) 2020 Peter Dettman and the
// libsecp256k1 contributors), itself an implementation of the paper above.
#pragma once
#include <stdint.h>

// HKV_SGCD_EARLY: stop once g = 0 (about 20 of the 25 iterations for random
// inputs) instead of always running the constant-time bound
#ifndef HKV_SGCD_EARLY
#define HKV_SGCD_EARLY 1
#endif
// HKV_SGCD_FLAT: the device's divstep loop without branches (divsteps30)
#ifndef HKV_SGCD_FLAT
#define HKV_SGCD_FLAT 1
#endif
#if defined(__HIPCC__)
#define HKV_HD __host__ __device__ __forceinline__
#else
#define HKV_HD static inline
#endif

namespace hkv {
namespace sgcd {

constexpr uint32_t M30 = 0x3FFFFFFFu;
// moduli in signed30 limbs with their inverse mod 2^30: the group order n
// (s^-1 in hkv_inv_kernel) and the field prime p (den^-1 in hkv_yverdict_kernel)
struct ModN {
  static constexpr int32_t L[9] = {0x10364141, 0x3F497A33, 0x348A03BB, 0x2BB739AB, 0x3FFFFEBA,
                                   0x3FFFFFFF, 0x3FFFFFFF, 0x3FFFFFFF, 0xFFFF};
  static constexpr uint32_t INV30 = 0x2A774EC1u;
};
struct ModP {
  static constexpr int32_t L[9] = {0x3FFFFC2F, 0x3FFFFFFB, 0x3FFFFFFF, 0x3FFFFFFF, 0x3FFFFFFF,
                                   0x3FFFFFFF, 0x3FFFFFFF, 0x3FFFFFFF, 0xFFFF};
  static constexpr uint32_t INV30 = 0x2DDACACFu;
};

// u256 (8 little-endian words) -> signed30
HKV_HD void to30(int32_t r[9], const uint32_t a[8]) {
  r[0] = (int32_t)(a[0] & M30);
  r[1] = (int32_t)(((a[0] >> 30) | (a[1] << 2)) & M30);
  r[2] = (int32_t)(((a[1] >> 28) | (a[2] << 4)) & M30);
  r[3] = (int32_t)(((a[2] >> 26) | (a[3] << 6)) & M30);
  r[4] = (int32_t)(((a[3] >> 24) | (a[4] << 8)) & M30);
  r[5] = (int32_t)(((a[4] >> 22) | (a[5] << 10)) & M30);
  r[6] = (int32_t)(((a[5] >> 20) | (a[6] << 12)) & M30);
  r[7] = (int32_t)(((a[6] >> 18) | (a[7] << 14)) & M30);
  r[8] = (int32_t)(a[7] >> 16);
}

HKV_HD int ctz32(uint32_t x) { return __builtin_ctz(x); }  // x != 0

// 30 divsteps on the low words of f and g, in libsecp256k1's variable-time
// form (secp256k1_modinv32_divsteps_30_var; eta = -delta): a run of even g
// is one shift (count trailing zeros), and each odd g cancels up to
// min(eta + 1, i, 8) low bits at once by adding w f, w = -g / f mod 2^8.
// It is the same divstep sequence as the constant-time form, so the 742-step
// bound holds; the inputs (signatures, keys) are public. Returns the
// transition matrix (u, v, q, r) scaled by 2^30 and the updated eta.
HKV_HD int32_t divsteps30(int32_t eta, uint32_t f, uint32_t g, int32_t t[4]) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  int i = 30;
#if (defined(__HIP_DEVICE_COMPILE__) && HKV_SGCD_FLAT) || defined(HKV_SGCD_FLAT_HOST)
  // Branch-free on the device (HKV_SGCD_FLAT_HOST: the same form in the host
  // test build, one lane): the lanes of a wave run different numbers of
  // iterations, so each step is written with selects and a lane that is done
  // (i = 0) steps with zeros = 0 and w = 0, which changes nothing; the loop
  // ends once no lane has steps left. The branchy form spends each iteration
  // on exec-mask bookkeeping for the swap and the exit.
  for (;;) {
    const int zeros = ctz32(g | (0xFFFFFFFFu << i));  // i = 0: all ones, zeros = 0
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
#if defined(__HIP_DEVICE_COMPILE__)
    if (!__any(i != 0)) break;
#else
    if (i == 0) break;
#endif
    const bool live = i != 0;
    const bool sw = live && eta < 0;  // g odd and delta > 0: (f, g, u, v, q, r) <- (g, -f, q, r, -u, -v)
    const uint32_t f0 = f, u0 = u, v0 = v;
    f = sw ? g : f;
    g = sw ? 0u - f0 : g;
    u = sw ? q : u;
    q = sw ? 0u - u0 : q;
    v = sw ? r : v;
    r = sw ? 0u - v0 : r;
    eta = sw ? -eta : eta;
    const int limit = (eta + 1) > i ? i : (eta + 1);
    const uint32_t m = live ? ((0xFFFFFFFFu >> (32 - limit)) & 255u) : 0u;
    uint32_t x = (3u * f) ^ 2u;  // f^-1 mod 2^5 (f odd)
    x *= 2u - f * x;             // mod 2^10
    const uint32_t w = (0u - g * x) & m;
    g += f * w;
    q += u * w;
    r += v * w;
  }
#else
  for (;;) {
    const int zeros = ctz32(g | (0xFFFFFFFFu << i));  // the sentinel bit i stops the count
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    if (eta < 0) {  // g odd and delta > 0: (f, g, u, v, q, r) <- (g, -f, q, r, -u, -v)
      uint32_t tmp;
      eta = -eta;
      tmp = f; f = g; g = 0u - tmp;
      tmp = u; u = q; q = 0u - tmp;
      tmp = v; v = r; r = 0u - tmp;
    }
    const int limit = (eta + 1) > i ? i : (eta + 1);
    const uint32_t m = (0xFFFFFFFFu >> (32 - limit)) & 255u;
    uint32_t x = (3u * f) ^ 2u;  // f^-1 mod 2^5 (f odd)
    x *= 2u - f * x;             // mod 2^10
    const uint32_t w = (0u - g * x) & m;
    g += f * w;
    q += u * w;
    r += v * w;
  }
#endif
  t[0] = (int32_t)u;
  t[1] = (int32_t)v;
  t[2] = (int32_t)q;
  t[3] = (int32_t)r;
  return eta;
}

// (f, g) <- t (f, g) / 2^30 (exact)
HKV_HD void update_fg(int32_t f[9], int32_t g[9], const int32_t t[4]) {
  const int64_t u = t[0], v = t[1], q = t[2], r = t[3];
  int64_t cf = u * f[0] + v * g[0];
  int64_t cg = q * f[0] + r * g[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; ++i) {
    cf += u * f[i] + v * g[i];
    cg += q * f[i] + r * g[i];
    f[i - 1] = (int32_t)((uint32_t)cf & M30);
    g[i - 1] = (int32_t)((uint32_t)cg & M30);
    cf >>= 30;
    cg >>= 30;
  }
  f[8] = (int32_t)cf;
  g[8] = (int32_t)cg;
}

// (d, e) <- t (d, e) / 2^30 (mod m), adding multiples of m to make the
// division exact; keeps d, e in (-2m, m).
template <class M>
HKV_HD void update_de(int32_t d[9], int32_t e[9], const int32_t t[4]) {
  const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
  const int32_t sd = d[8] >> 31, se = e[8] >> 31;
  int32_t md = (u & sd) + (v & se);
  int32_t me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d[0] + (int64_t)v * e[0];
  int64_t ce = (int64_t)q * d[0] + (int64_t)r * e[0];
  md -= (int32_t)((M::INV30 * (uint32_t)cd + (uint32_t)md) & M30);
  me -= (int32_t)((M::INV30 * (uint32_t)ce + (uint32_t)me) & M30);
  cd += (int64_t)M::L[0] * md;
  ce += (int64_t)M::L[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; ++i) {
    cd += (int64_t)u * d[i] + (int64_t)v * e[i] + (int64_t)M::L[i] * md;
    ce += (int64_t)q * d[i] + (int64_t)r * e[i] + (int64_t)M::L[i] * me;
    d[i - 1] = (int32_t)((uint32_t)cd & M30);
    e[i - 1] = (int32_t)((uint32_t)ce & M30);
    cd >>= 30;
    ce >>= 30;
  }
  d[8] = (int32_t)cd;
  e[8] = (int32_t)ce;
}

// r = a^-1 mod m for 0 < a < m (a = 0 gives 0).
template <class M>
HKV_HD void inv_mod(uint32_t out[8], const uint32_t a[8]) {
  int32_t f[9], g[9], d[9], e[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    f[i] = M::L[i];
    d[i] = 0;
    e[i] = 0;
  }
  e[0] = 1;
  to30(g, a);
  int32_t eta = -1;  // -delta
#pragma unroll 1
  for (int it = 0; it < 25; ++it) {
    int32_t t[4];
    eta = divsteps30(eta, (uint32_t)f[0] | ((uint32_t)f[1] << 30), (uint32_t)g[0] | ((uint32_t)g[1] << 30), t);
    update_fg(f, g, t);
    update_de<M>(d, e, t);
#if HKV_SGCD_EARLY
    // g = 0: every further divstep leaves f unchanged and d unchanged mod m
    // (matrix [[2^30, 0], [q, r]] / 2^30; update_de may add m to a negative
    // d, which the final normalisation folds away), so the loop may stop; on
    // the device when every lane of the wave has reached it
    const bool gz = (g[0] | g[1] | g[2] | g[3] | g[4] | g[5] | g[6] | g[7] | g[8]) == 0;
#if defined(__HIP_DEVICE_COMPILE__)
    if (__all(gz)) break;
#else
    if (gz) break;
#endif
#endif
  }
  // f = ±1: result = d * f, then into [0, n): d in (-2n, 2n)
  const int32_t fneg = f[8] >> 31;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // d = fneg ? -d : d  (limb-wise, then renormalise)
    c += (int64_t)((d[i] ^ fneg) - fneg);
    d[i] = (int32_t)((uint32_t)c & M30);
    c >>= 30;
  }
  d[8] = (int32_t)(c + ((d[8] ^ fneg) - fneg));
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {  // add n while negative
    const int32_t neg = d[8] >> 31;
    c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      c += (int64_t)d[i] + (M::L[i] & neg);
      d[i] = (int32_t)((uint32_t)c & M30);
      c >>= 30;
    }
    d[8] = (int32_t)(c + d[8] + (M::L[8] & neg));
  }
  {  // subtract n once if d >= n: compute d - n, keep it when non-negative
    int32_t s[9];
    c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      c += (int64_t)d[i] - M::L[i];
      s[i] = (int32_t)((uint32_t)c & M30);
      c >>= 30;
    }
    s[8] = (int32_t)(c + d[8] - M::L[8]);
    const int32_t keep = ~(s[8] >> 31);  // all ones when d - n >= 0
#pragma unroll
    for (int i = 0; i < 9; ++i) d[i] = (s[i] & keep) | (d[i] & ~keep);
  }
  // signed30 (now in [0, n)) -> 8 words
  out[0] = (uint32_t)d[0] | ((uint32_t)d[1] << 30);
  out[1] = ((uint32_t)d[1] >> 2) | ((uint32_t)d[2] << 28);
  out[2] = ((uint32_t)d[2] >> 4) | ((uint32_t)d[3] << 26);
  out[3] = ((uint32_t)d[3] >> 6) | ((uint32_t)d[4] << 24);
  out[4] = ((uint32_t)d[4] >> 8) | ((uint32_t)d[5] << 22);
  out[5] = ((uint32_t)d[5] >> 10) | ((uint32_t)d[6] << 20);
  out[6] = ((uint32_t)d[6] >> 12) | ((uint32_t)d[7] << 18);
  out[7] = ((uint32_t)d[7] >> 14) | ((uint32_t)d[8] << 16);
}

HKV_HD void inv_mod_n(uint32_t out[8], const uint32_t a[8]) { inv_mod<ModN>(out, a); }
HKV_HD void inv_mod_p(uint32_t out[8], const uint32_t a[8]) { inv_mod<ModP>(out, a); }

}  // namespace sgcd
}  // namespace hkv
