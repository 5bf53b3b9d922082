// hkv_hash.h — SHA-256 (FIPS 180-4) and RIPEMD-160 for gfx950, one message
// per lane.
//
// The compression functions are fully unrolled straight-line VALU code
// (rotations are v_alignbit, the message schedule lives in 16 VGPRs). The
// streaming driver (sha256_stream in hkv_sighash.hip) is block-synchronous:
// every live lane of a wave fills and compresses its next 64-byte block in
// the same loop iteration, so lanes never diverge around a compression.
//
// Replaces (semantically) haskoin-core Haskoin.Crypto.Hash doubleSHA256 and
// addressHash (RIPEMD160 . SHA256) [dep; SURVEY.md §8(a) a9, §8(f) row 2].
#pragma once
#include "hkv_field.h"

namespace hkv {

HKV_DEV uint32_t rotr32(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
HKV_DEV uint32_t rotl32(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
// gfx950 v_bitop3_b32: any 3-input bitwise function in one instruction, the
// immediate its truth table over (a, b, c) = (0xF0, 0xCC, 0xAA). The compiler
// forms it for Ch / Maj but leaves the Sigma functions' XOR of three
// rotations as two v_xor_b32.
HKV_DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
HKV_DEV uint32_t sha_ch(uint32_t e, uint32_t f, uint32_t g) { return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA); }
HKV_DEV uint32_t sha_maj(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8); }

HKV_DEV void sha256_init(uint32_t h[8]) {
  h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
  h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
}

// One compression of the big-endian message words w[16] (clobbered) into h.
HKV_DEV void sha256_compress(uint32_t h[8], uint32_t w[16]) {
  constexpr uint32_t K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
      const uint32_t s0 = xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
      wt = w[t & 15] = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
    }
    const uint32_t S1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
    const uint32_t ch = sha_ch(e, f, g);
    const uint32_t t1 = hh + S1 + ch + K[t] + wt;
    const uint32_t S0 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
    const uint32_t mj = sha_maj(a, b, c);
    hh = g; g = f; f = e; e = d + t1;
    d = c; c = b; b = a; a = t1 + S0 + mj;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d;
  h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// SHA-256 of a 32-byte message given as 8 big-endian words (the outer hash
// of SHA-256d, or the input of RIPEMD-160 in HASH160).
HKV_DEV void sha256_of_digest(uint32_t out[8], const uint32_t in[8]) {
  uint32_t w[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = in[k];
  w[8] = 0x80000000u;
#pragma unroll
  for (int k = 9; k < 15; ++k) w[k] = 0;
  w[15] = 256;
  sha256_init(out);
  sha256_compress(out, w);
}

// RIPEMD-160 of the 32 bytes whose big-endian words are in_be[8] (a SHA-256
// digest). Output: the five little-endian state words (digest byte k is byte
// k%4 of out[k/4]).
HKV_DEV void ripemd160_of_digest(uint32_t out[5], const uint32_t in_be[8]) {
  constexpr int RL[80] = {0, 1, 2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 7,  4,  13, 1,
                          10, 6, 15, 3,  12, 0,  9,  5,  2,  14, 11, 8,  3,  10, 14, 4,  9,  15, 8,  1,
                          2,  7, 0,  6,  13, 11, 5,  12, 1,  9,  11, 10, 0,  8,  12, 4,  13, 3,  7,  15,
                          14, 5, 6,  2,  4,  0,  5,  9,  7,  12, 2,  10, 14, 1,  3,  8,  11, 6,  15, 13};
  constexpr int RR[80] = {5,  14, 7,  0, 9, 2,  11, 4,  13, 6,  15, 8,  1,  10, 3,  12, 6,  11, 3,  7,
                          0,  13, 5,  10, 14, 15, 8, 12, 4, 9,  1,  2,  15, 5,  1,  3,  7,  14, 6,  9,
                          11, 8,  12, 2,  10, 0,  4,  13, 8,  6,  4,  1,  3,  11, 15, 0,  5,  12, 2,  13,
                          9,  7,  10, 14, 12, 15, 10, 4,  1,  5,  8,  7,  6,  2,  13, 14, 0,  3,  9,  11};
  constexpr int SL[80] = {11, 14, 15, 12, 5,  8,  7,  9,  11, 13, 14, 15, 6,  7,  9,  8,  7,  6,  8,  13,
                          11, 9,  7,  15, 7,  12, 15, 9,  11, 7,  13, 12, 11, 13, 6,  7,  14, 9,  13, 15,
                          14, 8,  13, 6,  5,  12, 7,  5,  11, 12, 14, 15, 14, 15, 9,  8,  9,  14, 5,  6,
                          8,  6,  5,  12, 9,  15, 5,  11, 6,  8,  13, 12, 5,  12, 13, 14, 11, 8,  5,  6};
  constexpr int SR[80] = {8,  9,  9,  11, 13, 15, 15, 5,  7,  7,  8,  11, 14, 14, 12, 6,  9,  13, 15, 7,
                          12, 8,  9,  11, 7,  7,  12, 7,  6,  15, 13, 11, 9,  7,  15, 11, 8,  6,  6,  14,
                          12, 13, 5,  14, 13, 13, 7,  5,  15, 5,  8,  11, 14, 14, 6,  14, 6,  9,  12, 9,
                          12, 5,  15, 8,  8,  5,  12, 9,  12, 5,  14, 6,  8,  13, 6,  5,  15, 13, 11, 11};
  constexpr uint32_t KL[5] = {0x00000000u, 0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xA953FD4Eu};
  constexpr uint32_t KR[5] = {0x50A28BE6u, 0x5C4DD124u, 0x6D703EF3u, 0x7A6D76E9u, 0x00000000u};
  uint32_t x[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = __builtin_bswap32(in_be[k]);
  x[8] = 0x80u;
#pragma unroll
  for (int k = 9; k < 14; ++k) x[k] = 0;
  x[14] = 256;
  x[15] = 0;
  const uint32_t h0 = 0x67452301u, h1 = 0xEFCDAB89u, h2 = 0x98BADCFEu, h3 = 0x10325476u, h4 = 0xC3D2E1F0u;
  uint32_t al = h0, bl = h1, cl = h2, dl = h3, el = h4;
  uint32_t ar = h0, br = h1, cr = h2, dr = h3, er = h4;
#pragma unroll
  for (int t = 0; t < 80; ++t) {
    const int rnd = t >> 4;
    uint32_t fl, fr;
    switch (rnd) {  // left line f1..f5, right line f5..f1
      case 0: fl = bl ^ cl ^ dl; fr = br ^ (cr | ~dr); break;
      case 1: fl = (bl & cl) | (~bl & dl); fr = (br & dr) | (cr & ~dr); break;
      case 2: fl = (bl | ~cl) ^ dl; fr = (br | ~cr) ^ dr; break;
      case 3: fl = (bl & dl) | (cl & ~dl); fr = (br & cr) | (~br & dr); break;
      default: fl = bl ^ (cl | ~dl); fr = br ^ cr ^ dr; break;
    }
    uint32_t tt = rotl32(al + fl + x[RL[t]] + KL[rnd], SL[t]) + el;
    al = el; el = dl; dl = rotl32(cl, 10); cl = bl; bl = tt;
    tt = rotl32(ar + fr + x[RR[t]] + KR[rnd], SR[t]) + er;
    ar = er; er = dr; dr = rotl32(cr, 10); cr = br; br = tt;
  }
  out[0] = h1 + cl + dr;
  out[1] = h2 + dl + er;
  out[2] = h3 + el + ar;
  out[3] = h4 + al + br;
  out[4] = h0 + bl + cr;
}

}  // namespace hkv
