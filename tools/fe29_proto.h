// fe29_proto.h — PROTOTYPE (tools only, not the product): secp256k1 field
// elements as 9 x 29-bit limbs in 32-bit registers, for the representation
// study VERDICT r01 asked for (tools/ubench_field.hip).
//
// value = sum l_i 2^(29 i); limbs of an operand may be up to 2^30 (one lazy
// add of two normalised values), so a product column of <= 9 products
// (< 2^60 each) plus its carry stays below 2^64: the column is a plain
// v_mad_u64_u32 chain with no carry flags. Reduction: 2^261 = 2^5 * 2^256 ==
// 2^37 + 31264 (mod p), i.e. high limb h_k folds in as 31264 * h_k at limb k
// and 256 * h_k at limb k + 1; the bits of limb 8 above 2^256 fold as
// x * (2^32 + 977) = 977 x at limb 0 and 8 x at limb 1.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fe29 {

constexpr uint32_t M29 = (1u << 29) - 1;
struct fe { uint32_t v[9]; };

__device__ __forceinline__ uint64_t mad(uint32_t a, uint32_t b, uint64_t c) {
  return (uint64_t)a * b + c;
}

// t[0..17]: normalised 29-bit column limbs of the 522-bit product (t[17] < 2^21)
__device__ __forceinline__ void reduce(fe& r, const uint32_t t[18]) {
  uint64_t acc = mad(t[9], 31264u, t[0]);
  r.v[0] = (uint32_t)acc & M29;
  acc >>= 29;
#pragma unroll
  for (int k = 1; k < 9; ++k) {
    acc += t[k];
    acc = mad(t[9 + k], 31264u, acc);
    acc = mad(t[8 + k], 256u, acc);
    if (k < 8) {
      r.v[k] = (uint32_t)acc & M29;
      acc >>= 29;
    }
  }
  // limb 8 holds bits 232..; bits >= 256 fold as x * (2^32 + 977), and
  // 256 * t[17] at weight 2^261 as t[17] * (2^45 + 8003584)
  const uint32_t x = (uint32_t)(acc >> 24);
  r.v[8] = (uint32_t)acc & ((1u << 24) - 1);
  uint64_t c0 = mad(t[17], 8003584u, mad(x, 977u, r.v[0]));
  r.v[0] = (uint32_t)c0 & M29;
  uint64_t c1 = mad(t[17], 65536u, mad(x, 8u, (c0 >> 29) + r.v[1]));
  r.v[1] = (uint32_t)c1 & M29;
  r.v[2] += (uint32_t)(c1 >> 29);
}

__device__ __forceinline__ void mul(fe& r, const fe& a, const fe& b) {
  uint32_t t[18];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; ++k) {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 9) acc = mad(a.v[i], b.v[j], acc);
    }
    t[k] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  t[17] = (uint32_t)acc;
  reduce(r, t);
}

__device__ __forceinline__ void sqr(fe& r, const fe& a) {
  uint32_t a2[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) a2[i] = a.v[i] << 1;  // limbs <= 2^30 -> 2^31
  uint32_t t[18];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; ++k) {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int j = k - i;
      if (j > i && j < 9) acc = mad(a2[i], a.v[j], acc);  // off-diagonal, doubled operand
    }
    if ((k & 1) == 0) acc = mad(a.v[k >> 1], a.v[k >> 1], acc);
    t[k] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  t[17] = (uint32_t)acc;
  reduce(r, t);
}

// lazy add: limbs grow by one bit, no carries
__device__ __forceinline__ void add(fe& r, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] + b.v[i];
}

// a - b + 4p, 4p spread so limbs 0..7 lie in [2^30, 2^31) (every limb of a
// normalised b fits under them); the result needs a carry pass before it
// may feed a multiply (limbs up to ~2^31)
__device__ __forceinline__ void sub(fe& r, const fe& a, const fe& b) {
  constexpr uint32_t K[9] = {0x5FFFF0BCu, 0x5FFFFFDDu, 0x5FFFFFFDu, 0x5FFFFFFDu, 0x5FFFFFFDu,
                             0x5FFFFFFDu, 0x5FFFFFFDu, 0x5FFFFFFDu, 0x03FFFFFDu};
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] + K[i] - b.v[i];
}

// carry pass: limbs back under 2^29 (+ the top fold), for sub results
__device__ __forceinline__ void carry(fe& r) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t v = r.v[i] + c;
    r.v[i] = v & M29;
    c = v >> 29;
  }
  const uint32_t v8 = r.v[8] + c;
  const uint32_t x = v8 >> 24;
  r.v[8] = v8 & ((1u << 24) - 1);
  const uint32_t c0 = r.v[0] + x * 977u;
  r.v[0] = c0 & M29;
  r.v[1] += (c0 >> 29) + x * 8u;
}

}  // namespace fe29
