// hkv_layout.h — buffer layouts shared by the HIP kernels and the host API.
#pragma once
#include <stdint.h>

namespace hkv {

// Input record (AoS, include/hkv.h): msg32 | r32 | s32 | pklen u8 | pubkey[65] | pad[6]
constexpr int REC_SIZE = 168;
constexpr int REC_WORDS = REC_SIZE / 4;

// Prologue -> ecmult intermediate, SoA: word w of signature i at [w * n_pad + i].
enum : int {
  IM_FLAGS = 0,   // bit0 valid, bit1 k1 negative, bit2 k2 negative, bit3 glv overflow
  IM_QX = 1,      // 8 limbs, affine pubkey x (normalised)
  IM_QY = 9,      // 8 limbs, affine pubkey y (normalised)
  IM_K1 = 17,     // 5 limbs, |k1| < 2^129   (u2 = k1 + k2*lambda)
  IM_K2 = 22,     // 5 limbs, |k2| < 2^129
  IM_U1L = 27,    // 4 limbs, u1 bits 0..127
  IM_U1H = 31,    // 4 limbs, u1 bits 128..255
  IM_R = 35,      // 8 limbs, r (< n)
  IM_WORDS = 43,
};
constexpr uint32_t FLAG_VALID = 1u, FLAG_NEG1 = 2u, FLAG_NEG2 = 4u, FLAG_GLV_OVF = 8u;

// Fixed-base tables: odd/even multiples j*B for j = 1..128, B in {G, 2^128 G},
// affine, 16 dwords per entry [x(8) | y(8)], table t at entry offset t*128.
constexpr int GTAB_W = 8;              // Booth radix 2^8
constexpr int GTAB_ENTRIES = 128;
constexpr int GTAB_DWORDS = 2 * GTAB_ENTRIES * 16;

// Per-lane Q table: multiples j*Q, j = 1..8, affine on the lane's isomorphic
// curve; per entry 6 quads (16 B): x(2) | y(2) | beta*x(2). Quad q of lane L
// at [(q * n_lanes + L) * 4] dwords (lane-contiguous, coalesced stores).
constexpr int QTAB_ENTRIES = 8;
constexpr int QTAB_QUADS_PER_ENTRY = 6;
constexpr int QTAB_QUADS = QTAB_ENTRIES * QTAB_QUADS_PER_ENTRY;

constexpr int WG = 256;                // threads per workgroup (4 waves)

}  // namespace hkv
