// hkv_group.h — secp256k1 group operations (y^2 = x^3 + 7) in Jacobian
// coordinates for gfx950, one point per lane.
//
// Formulas are the a = 0 Jacobian ones; they do not involve b, so they run
// unchanged on any isomorphic curve y^2 = x^3 + 7*Z^6 — which is what lets the
// verify kernel keep its per-signature table "affine" on an isomorphic curve
// (hkv_kernels.hip, table build) and correct the final Z once.
// Replaces (semantically) libsecp256k1 secp256k1_gej_double /
// secp256k1_gej_add_ge_var / secp256k1_gej_add_zinv_var [dep; SURVEY §8(a) a3].
#pragma once
#include "hkv_scalar.h"

namespace hkv {

struct ge { fe x, y; };
struct gej { fe x, y, z; };

__constant__ static const uint32_t FE_GX[8] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu,
                                               0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu};
__constant__ static const uint32_t FE_GY[8] = {0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u,
                                               0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};
// beta: lambda*(x, y) = (beta*x, y)
__constant__ static const uint32_t FE_BETA[8] = {0x719501EEu, 0xC1396C28u, 0x12F58995u, 0x9CF04975u,
                                                 0xAC3434E9u, 0x6E64479Eu, 0x657C0710u, 0x7AE96A2Bu};

HKV_DEV void ge_set_g(ge& r) {
#pragma unroll
  for (int i = 0; i < 8; ++i) { r.x.v[i] = FE_GX[i]; r.y.v[i] = FE_GY[i]; }
}
HKV_DEV void gej_set_ge(gej& r, const ge& a) {
  r.x = a.x;
  r.y = a.y;
  fe_set_u32(r.z, 1);
}
HKV_DEV void gej_cmov(gej& r, const gej& a, bool f) {
  fe_cmov(r.x, a.x, f);
  fe_cmov(r.y, a.y, f);
  fe_cmov(r.z, a.z, f);
}

// r = 2a for a = 0 (3M + 4S), returned as the same point scaled by 1/2:
// with A = X^2, B = Y^2, C = B^2, M = X*B, E' = 3A/2,
//   X3' = E'^2 - 2M, Y3' = E'(M - X3') - C, Z3' = Y*Z,
// i.e. (X3/4, Y3/8, Z3/2) of the textbook X3 = E^2 - 8M, Y3 = E(4M - X3) - 8C,
// Z3 = 2YZ: one halving and one shift instead of four power-of-two scalings
// (-1.4% ecmult, profiles/r02_variants.log). On this ISA a product costs
// about a square, so X*B beats the square-and-subtract form. a must not be
// infinity; y != 0 on secp256k1. r may alias a.
HKV_DEV void gej_double(gej& r, const gej& a) {
  fe A, B, C, M, E, t;
  fe_sqr(A, a.x);
  fe_sqr(B, a.y);
  fe_mul(M, a.x, B);
  fe_sqr(C, B);
  fe_mul_small(E, A, 3);
  fe_half(E, E);            // E' = 3A/2
  fe_mul(r.z, a.y, a.z);    // Z3' = YZ
  fe_sqr(t, E);
  fe_shl(B, M, 1);
  fe_sub(r.x, t, B);        // X3' = E'^2 - 2M
  fe_sub(t, M, r.x);
  fe_mul(t, E, t);
  fe_sub(r.y, t, C);        // Y3' = E'(M - X3') - C
}

// Mixed addition r = a + (bx, by) where (bx, by) is affine on the curve whose
// Jacobian z-scale is `az` (az = a.z for a plain mixed add; az = a.z * Zg for
// the "zinv" form that adds a point of the base curve to an accumulator that
// lives on the isomorphic curve of scale Zg). 8M + 3S.
// Outputs hz = (H == 0), rz = (R == 0); when hz the result is garbage and the
// caller must substitute 2a (rz) or infinity (!rz). Writes the z-ratio H.
HKV_DEV void gej_add_ge_core(gej& r, const gej& a, const fe& az, const fe& bx, const fe& by,
                             bool& hz, bool& rz, fe* zr) {
  fe z2, u2, s2, h, rr, t, hh, hhh, v;
  fe_sqr(z2, az);
  fe_mul(u2, bx, z2);
  fe_mul(t, az, z2);
  fe_mul(s2, by, t);
  fe_sub(h, u2, a.x);
  fe_sub(rr, s2, a.y);
  hz = fe_is_zero(h);
  rz = fe_is_zero(rr);
  fe_sqr(hh, h);
  fe_mul(hhh, h, hh);
  fe_mul(v, a.x, hh);
  fe_mul(r.z, a.z, h);
  if (zr) *zr = h;
  fe_sqr(t, rr);
  fe_sub(t, t, hhh);
  fe_shl(u2, v, 1);
  fe_sub(t, t, u2);         // X3 = R^2 - H^3 - 2V
  fe_sub(v, v, t);
  fe_mul(v, rr, v);
  fe_mul(hhh, a.y, hhh);
  fe_sub(r.y, v, hhh);      // Y3 = R(V - X3) - Y1 H^3
  r.x = t;
}

// Complete "accumulate" step used by every ecmult loop:
//   acc (+inf flag) += T  where T = (tx, ty) is affine on the curve of
//   Jacobian scale az (see gej_add_ge_core), `take` = this lane adds
//   (digit != 0). Lanes whose acc is infinity are left to the caller
//   (gej_accumulate_from_inf), so the mapped init point is only built when
//   some lane needs it.
// H = U2 - X1 is tested before anything is written, so the sum (8M + 3S) is
// computed in place under the lane mask live && H != 0: lanes that do not
// add keep their point without a copy, and acc = +-T (H == 0, rare) is then
// resolved exactly by a masked doubling or by going to infinity.
HKV_DEV void gej_accumulate(gej& acc, bool& inf, const fe& az, const fe& tx, const fe& ty, bool take) {
  fe h, rr;
  {
    fe z2, t;
    fe_sqr(z2, az);
    fe_mul(h, tx, z2);        // U2
    fe_mul(t, az, z2);
    fe_mul(rr, ty, t);        // S2
  }
  fe_sub(h, h, acc.x);        // H = U2 - X1
  fe_sub(rr, rr, acc.y);      // R = S2 - Y1
  const bool live = take && !inf;
  const bool hz = fe_is_zero(h);
  if (live && !hz) {
    fe hh, hhh, t2;
    fe_sqr(hh, h);
    fe_mul(hhh, h, hh);       // H^3
    fe_mul(hh, acc.x, hh);    // V = X1 H^2
    fe_mul(acc.z, acc.z, h);  // Z3 = Z1 H
    fe_sqr(h, rr);
    fe_sub(h, h, hhh);
    fe_shl(t2, hh, 1);
    fe_sub(acc.x, h, t2);     // X3 = R^2 - H^3 - 2V
    fe_sub(hh, hh, acc.x);
    fe_mul(hh, rr, hh);
    fe_mul(hhh, acc.y, hhh);
    fe_sub(acc.y, hh, hhh);   // Y3 = R(V - X3) - Y1 H^3
  }
  const bool degen = live && hz;
  if (__builtin_expect(__any(degen), 0)) {
    const bool rz = fe_is_zero(rr);
    if (degen && rz) gej_double(acc, acc);   // T == acc
    inf = inf || (degen && !rz);             // T == -acc
  }
}
// ---- paired-product forms for a lone wave per SIMD ----
// Same results as gej_double / gej_accumulate; independent field products
// are issued as interleaved pairs (fe_mul2 / fe_sqr2 / fe_sqrmul), so the
// dependency stalls of one product are filled by the other. The small-batch
// split kernel runs < 1 wave per SIMD, where a single product's chain leaves
// a third of the issue slots empty (tools/ubench_field.hip, blocks_per_cu 1).
HKV_DEV void gej_double_ilp(gej& r, const gej& a) {
  fe A, B, M, Z3, C, E, t;
  fe_sqr2(A, a.x, B, a.y);
  fe_mul2(M, a.x, B, Z3, a.y, a.z);  // M = XB, Z3' = YZ
  fe_mul_small(E, A, 3);
  fe_half(E, E);                     // E' = 3A/2
  fe_sqr2(C, B, t, E);               // C = B^2, E'^2
  r.z = Z3;
  fe_shl(B, M, 1);
  fe_sub(r.x, t, B);                 // X3' = E'^2 - 2M
  fe_sub(t, M, r.x);
  fe_mul(t, E, t);
  fe_sub(r.y, t, C);                 // Y3' = E'(M - X3') - C
}

HKV_DEV void gej_accumulate_ilp(gej& acc, bool& inf, const fe& az, const fe& tx, const fe& ty, bool take) {
  fe h, rr, hh;
  {
    fe z2, t;
    fe_sqr(z2, az);
    fe_mul2(h, tx, z2, t, az, z2);    // U2, az^3
    fe_sub(h, h, acc.x);              // H = U2 - X1
    fe_sqrmul(hh, h, rr, ty, t);      // H^2, S2
  }
  fe_sub(rr, rr, acc.y);              // R = S2 - Y1
  const bool live = take && !inf;
  const bool hz = fe_is_zero(h);
  if (live && !hz) {
    fe hhh, v, r2, z3, t2;
    fe_mul2(hhh, h, hh, v, acc.x, hh);  // H^3, V = X1 H^2
    fe_sqrmul(r2, rr, z3, acc.z, h);    // R^2, Z3 = Z1 H
    acc.z = z3;
    fe_sub(r2, r2, hhh);
    fe_shl(t2, v, 1);
    fe_sub(acc.x, r2, t2);              // X3 = R^2 - H^3 - 2V
    fe_sub(v, v, acc.x);
    fe_mul2(v, rr, v, hhh, acc.y, hhh);
    fe_sub(acc.y, v, hhh);              // Y3 = R(V - X3) - Y1 H^3
  }
  const bool degen = live && hz;
  if (__builtin_expect(__any(degen), 0)) {
    const bool rz = fe_is_zero(rr);
    if (degen && rz) gej_double(acc, acc);   // T == acc
    inf = inf || (degen && !rz);             // T == -acc
  }
}

// ---- pair-lane forms: one point on two lanes (2c, 2c + 1) ----
// A wave that runs alone on its SIMD is issue-bound on the field products
// (fe_mul: 880 SIMD cycles at one wave, the interleaved pair fe_mul2 1,740:
// profiles/r02_ubench_field_mulred.json), so two independent products of one
// point operation cost the same whether they sit in one lane or not — unless
// they sit in TWO lanes of the same instruction stream. The pair forms keep
// a Jacobian point as P = X (even lane) | Y (odd lane) and Z on the odd lane,
// and run each step's independent products on the two lanes at once; the
// operands move between the lanes with DPP quad permutations (fe_xch: swap
// within the pair, fe_bc1: the odd lane's value on both) and lane-parity
// selects (fe_sel, a bitfield insert with the all-ones odd-lane mask).
// A doubling is then 2S + 2M deep instead of 4S + 3M, a mixed addition
// 1S + 5M instead of 3S + 8M. Both lanes of a pair always take the same
// branches (their flags are made pair-uniform), so every DPP source lane is
// active.
HKV_DEV uint32_t dpp_xch(uint32_t v) {  // quad_perm [1, 0, 3, 2]
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}
HKV_DEV uint32_t dpp_bc1(uint32_t v) {  // quad_perm [1, 1, 3, 3]
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xF5, 0xF, 0xF, false);
}
HKV_DEV uint32_t dpp_bc0(uint32_t v) {  // quad_perm [0, 0, 2, 2]
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xA0, 0xF, 0xF, false);
}
HKV_DEV void fe_xch(fe& r, const fe& a) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = dpp_xch(a.v[i]);
}
HKV_DEV void fe_bc1(fe& r, const fe& a) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = dpp_bc1(a.v[i]);
}
HKV_DEV void fe_bc0(fe& r, const fe& a) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = dpp_bc0(a.v[i]);
}
// r = a on the even lane, b on the odd lane (odd: all ones on odd lanes)
HKV_DEV void fe_sel(fe& r, const fe& a, const fe& b, uint32_t odd) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = (a.v[i] & ~odd) | (b.v[i] & odd);
}
// a flag computed on one lane of the pair, made pair-uniform
HKV_DEV bool pair_even(bool f) { return dpp_bc0(f ? 1u : 0u) != 0; }
HKV_DEV bool pair_odd(bool f) { return dpp_bc1(f ? 1u : 0u) != 0; }

// 2(X, Y, Z) on a pair (P = X | Y, Z on the odd lane) in the unhalved
// form with the small multiples gathered into one lane-parallel step: with
// A = X^2, B = Y^2, M = X B, C = B^2 (dbl-2009-l: E = 3A, S = 4M)
//   X3 = 9A^2 - 8M,  Y3 = A (36M - 27A^2) - 8C,  Z3 = 2YZ.
// Products [A | B], [M | YZ], [C | A^2], then [X3 | D] as one fused pass
// (fe_lin2: both small multiples and the difference) beside [8C | 2YZ] (one
// shift), and [. | A D - 8C] as one product with an addend (fe_mul_add): 2S + 2M
// deep with no separate subtraction chain, where the halved form needed 3A,
// /2, 2M and three subtractions (tools/ubench_chain.hip).
HKV_DEV void pair_double(fe& P, fe& Z, uint32_t odd) {
  fe R1, T, O1, R2, R3, P1, P2, r, Q, t;
  fe_sqr(R1, P);              // A              | B
  fe_xch(T, R1);              // B              | A
  fe_sel(O1, T, Z, odd);      // B              | Z
  fe_mul(R2, P, O1);          // M = X B        | YZ
  fe_sqr(R3, T);              // C = B^2        | A^2
  fe_sel(P2, R2, R3, odd);    // M              | A^2
  fe_xch(P1, P2);             // A^2            | M
  fe_sel(O1, R3, R2, odd);    // C              | YZ
  fe_lin2(r, P1, odd ? 36u : 9u, P2, odd ? 27u : 8u);  // X3 | D = 36M - 27A^2
  fe_shl_var(Q, O1, odd ? 1u : 3u);   // 8C | 2YZ
  fe_xch(O1, Q);              // 2YZ            | 8C
  fe_cneg(O1, O1, odd != 0);  //                | -8C
  fe_mul_add(t, T, r, O1);    //                | Y3 = A D - 8C
  fe_sel(P, r, t, odd);
  Z = Q;                      //                | Z3
}

// The pair form of gej_accumulate: (P, Z, inf) += T with T = TXY = tx (even
// lane) | ty (odd lane), affine on the curve of Jacobian scale Z (the
// accumulator's own isomorphic curve). take must be pair-uniform; lanes at
// infinity are left to pair_accumulate_from_inf.
HKV_DEV void pair_accumulate(fe& P, fe& Z, bool& inf, const fe& TXY, bool take, uint32_t odd) {
  fe z2, O1, O2, R2, H, R3, Rr;
  fe_sqr(z2, Z);              //                | Z^2
  fe_bc1(O2, z2);             // Z^2            | Z^2
  fe_sel(O1, TXY, Z, odd);    // tx             | Z
  fe_mul(R2, O1, O2);         // U2 = tx Z^2    | Z^3
  fe_sub(H, R2, P);           // H = U2 - X1
  fe_sel(O1, H, TXY, odd);    // H              | ty
  fe_sel(O2, H, R2, odd);     // H              | Z^3
  fe_mul(R3, O1, O2);         // H^2            | S2 = ty Z^3
  fe_sub(Rr, R3, P);          //                | R = S2 - Y1
  const bool live = take && !inf;
  const bool hz = pair_even(fe_is_zero(H));
  if (live && !hz) {
    fe R5, R6, W, X3, D, R7, t;
    fe_sel(O1, H, Rr, odd);   // H              | R
    fe_sel(O2, R3, Rr, odd);  // H^2            | R
    fe_mul(R5, O1, O2);       // H^3            | R^2
    fe_xch(t, H);             //                | H
    fe_sel(O1, P, Z, odd);    // X1             | Z1
    fe_sel(O2, R3, t, odd);   // H^2            | H
    fe_mul(R6, O1, O2);       // V = X1 H^2     | Z3 = Z1 H
    fe_xch(W, R5);            // R^2            | H^3
    fe_sub(X3, W, R5);
    fe_shl(t, R6, 1);
    fe_sub(X3, X3, t);        // X3 = R^2 - H^3 - 2V
    fe_sub(D, R6, X3);        // V - X3
    fe_xch(t, D);             //                | V - X3
    fe_xch(O1, P);            // Y1             | X1
    fe_sel(O1, O1, Rr, odd);  // Y1             | R
    fe_sel(O2, R5, t, odd);   // H^3            | V - X3
    fe_mul(R7, O1, O2);       // Y1 H^3         | R (V - X3)
    fe_xch(t, R7);
    fe_sub(t, R7, t);         //                | Y3 = R (V - X3) - Y1 H^3
    fe_sel(P, X3, t, odd);
    Z = R6;                   //                | Z3
  }
  const bool degen = live && hz;
  if (__builtin_expect(__any(degen), 0)) {
    const bool rz = pair_odd(fe_is_zero(Rr));
    if (degen && rz) pair_double(P, Z, odd);   // T == acc
    inf = inf || (degen && !rz);               // T == -acc
  }
}
// ---- quad-lane form: one point on four lanes (4c .. 4c + 3) ----
// V = X | Y | Z | (unused) on quad lanes 0..3. A doubling is S + 2M deep
// against 2S + 2M in the pair form. Operands move by DPP
// quad permutations (quad_perm [s0, s1, s2, s3]: lane q reads lane s_q of
// its quad) and lane-mask selects (m0, m1, m2: all ones on quad lane 0, 1, 2).
template <int PERM>
HKV_DEV void fe_quad(fe& r, const fe& a) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.v[i], PERM, 0xF, 0xF, false);
}
constexpr int QP_0 = 0x00, QP_3 = 0xFF, QP_0112 = 0xD4;  // [0,0,0,0] [3,3,3,3] [0,1,1,3]
constexpr int QP_1100 = 0x05, QP_3021 = 0x63, QP_0333 = 0xFC;  // [1,1,0,0] [3,0,2,1] [0,3,3,3]
constexpr int QP_0331 = 0x7C;                                   // [0,3,3,1]
// 2V in the unhalved form of pair_double: [A | B | . | .], then
// [M | C | YZ | A^2] on the four lanes, [X3 | D | Z3 | -8C] by one fused
// small-multiple difference (fe_lin2), [. | Y3 = A D - 8C | . | .] by one
// product with an addend (fe_mul_add): S + 2M deep. Operands that are one
// quad permutation of a product are formed by a single DPP move per limb
// (P1, P2), and the others by two permutations and one select, not by
// broadcasts and select chains.
#ifndef HKV_QUAD_SPLIT  // 1: quad_double's lane-idle products spread over the quad (fe_mul_rows2 / 4)
#define HKV_QUAD_SPLIT 0
#endif
template <int PERM>
HKV_DEV uint32_t dpp_quad(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, PERM, 0xF, 0xF, false);
}
constexpr int QP_X2 = 0x4E, QP_X1 = 0xB1, QP_0101 = 0x44, QP_1 = 0x55;  // [2,3,0,1] [1,0,3,2] [0,1,0,1] [1,1,1,1]
// Lane-split products: the 64 limb products of one 256 x 256 product spread
// by rows of a over the lanes of a quad, the partial products summed across
// lanes by DPP, one reduction. For the products of quad_double that would
// otherwise leave lanes of the quad idle.
// r = a b on the lane with hsel = 0 of the pair {q, q ^ 2}; the partner
// (hsel = all ones) takes a's rows 4..7. Same a, b on both lanes.
HKV_DEV void fe_mul_rows2(fe& r, const fe& a, const fe& b, uint32_t hsel) {
  uint32_t ar[4], p[12], t[16];
#pragma unroll
  for (int k = 0; k < 4; ++k) ar[k] = (a.v[k] & ~hsel) | (a.v[k + 4] & hsel);
  mul4x8_ps(p, ar, b.v);
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) t[k] = p[k];
#pragma unroll
  for (int k = 0; k < 8; ++k) t[4 + k] = addc(p[4 + k], dpp_quad<QP_X2>(p[k]), c);
#pragma unroll
  for (int k = 0; k < 4; ++k) t[12 + k] = addc(0u, dpp_quad<QP_X2>(p[8 + k]), c);
  fe_reduce512(r, t);
}
// r = a b on quad lane 1: rows 0,1 of a on lane 1, 2,3 on lane 0, 4,5 on
// lane 3, 6,7 on lane 2 (m0 / m1 / m2: all ones on quad lane 0 / 1 / 2);
// the same b on every lane
HKV_DEV void fe_mul_rows4(fe& r, const fe& a, const fe& b, uint32_t m0, uint32_t m1, uint32_t m2) {
  const uint32_t m3 = ~(m0 | m1 | m2);
  uint32_t ar[2], p[10], t1[12], t[16];
#pragma unroll
  for (int k = 0; k < 2; ++k)
    ar[k] = (a.v[k] & m1) | (a.v[2 + k] & m0) | (a.v[4 + k] & m3) | (a.v[6 + k] & m2);
  mul2x8_ps(p, ar, b.v);
  uint32_t c = 0;
  t1[0] = p[0];
  t1[1] = p[1];
#pragma unroll
  for (int k = 0; k < 8; ++k) t1[2 + k] = addc(p[2 + k], dpp_quad<QP_X1>(p[k]), c);
#pragma unroll
  for (int k = 0; k < 2; ++k) t1[10 + k] = addc(0u, dpp_quad<QP_X1>(p[8 + k]), c);
  c = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) t[k] = t1[k];
#pragma unroll
  for (int k = 0; k < 8; ++k) t[4 + k] = addc(t1[4 + k], dpp_quad<QP_X2>(t1[k]), c);
#pragma unroll
  for (int k = 0; k < 4; ++k) t[12 + k] = addc(0u, dpp_quad<QP_X2>(t1[8 + k]), c);
  fe_reduce512(r, t);
}

HKV_DEV void quad_double(fe& V, uint32_t m0, uint32_t m1, uint32_t m2) {
#if HKV_QUAD_SPLIT
  // [A | B] as two 2-way row-split squares (X^2 on lanes 0, 2; Y^2 on 1, 3),
  // Y3 = A D - 8C as one 4-way row-split product landing on lane 1
  fe S, R1, Aq, RA, T, opA, opB, R2, P1, P2, r, t, C8, Dq;
  fe_quad<QP_0101>(S, V);     // X | Y | X | Y
  fe_mul_rows2(R1, S, S, ~(m0 | m1));  // A = X^2 | B = Y^2 | . | .
  fe_quad<QP_0>(Aq, R1);      // A        | A      | A  | A
  fe_quad<QP_1100>(RA, R1);   // B        | B      | A  | A
  fe_quad<QP_0112>(T, V);     // X        | .      | Y  | .
  fe_sel(opA, RA, T, m0 | m2);    // X | B | Y | A
  fe_sel(opB, RA, V, m2);         // B | B | Z | A
  fe_mul(R2, opA, opB);       // M | C | YZ | A^2
  fe_quad<QP_3021>(P1, R2);   // A^2 | M | YZ | C
  fe_quad<QP_0331>(P2, R2);   // M | A^2 | . | C
  const uint32_t k1 = m0 ? 9u : (m1 ? 36u : (m2 ? 2u : 0u));
  const uint32_t k2 = m0 ? 8u : (m1 ? 27u : (m2 ? 0u : 8u));
  fe_lin2(r, P1, k1, P2, k2); // X3 | D = 36M - 27A^2 | Z3 = 2YZ | -8C
  fe_quad<QP_3>(C8, r);       // -8C on every lane
  fe_quad<QP_1>(Dq, r);       // D on every lane
  fe_mul_rows4(t, Aq, Dq, m0, m1, m2);
  fe_add(t, t, C8);           // . | Y3 = A D - 8C | . | .
  fe_sel(V, r, t, m1);        // X3 | Y3 | Z3 | .
#else
  fe R1, Aq, RA, T, opA, opB, R2, P1, P2, r, t, C8;
  fe_sqr(R1, V);              // A = X^2 | B = Y^2 | . | .
  fe_quad<QP_0>(Aq, R1);      // A        | A      | A  | A
  fe_quad<QP_1100>(RA, R1);   // B        | B      | A  | A
  fe_quad<QP_0112>(T, V);     // X        | .      | Y  | .
  fe_sel(opA, RA, T, m0 | m2);    // X | B | Y | A
  fe_sel(opB, RA, V, m2);         // B | B | Z | A
  fe_mul(R2, opA, opB);       // M | C | YZ | A^2
  fe_quad<QP_3021>(P1, R2);   // A^2 | M | YZ | C
  fe_quad<QP_0331>(P2, R2);   // M | A^2 | . | C
  const uint32_t k1 = m0 ? 9u : (m1 ? 36u : (m2 ? 2u : 0u));
  const uint32_t k2 = m0 ? 8u : (m1 ? 27u : (m2 ? 0u : 8u));
  fe_lin2(r, P1, k1, P2, k2); // X3 | D = 36M - 27A^2 | Z3 = 2YZ | -8C
  fe_quad<QP_3>(C8, r);       // -8C on every lane
  fe_mul_add(t, Aq, r, C8);   // . | Y3 = A D - 8C | . | .
  fe_sel(V, r, t, m1);        // X3 | Y3 | Z3 | .
#endif
}

// P += TXY in place for a table build: TXY affine on the curve of the
// accumulator's Jacobian scale, P finite and never +-TXY (the multiples
// j Q, j < 9, of a point of prime order). Returns the z-ratio H = U2 - X1
// on the even lane (Z3 = Z1 H). The live branch of pair_accumulate.
HKV_DEV void pair_add_affine(fe& P, fe& Z, const fe& TXY, uint32_t odd, fe& H) {
  fe z2, O1, O2, R2, R3, Rr, R5, R6, W, X3, D, R7, t;
  fe_sqr(z2, Z);              //                | Z^2
  fe_bc1(O2, z2);             // Z^2            | Z^2
  fe_sel(O1, TXY, Z, odd);    // tx             | Z
  fe_mul(R2, O1, O2);         // U2 = tx Z^2    | Z^3
  fe_sub(H, R2, P);           // H = U2 - X1
  fe_sel(O1, H, TXY, odd);    // H              | ty
  fe_sel(O2, H, R2, odd);     // H              | Z^3
  fe_mul(R3, O1, O2);         // H^2            | S2 = ty Z^3
  fe_sub(Rr, R3, P);          //                | R = S2 - Y1
  fe_sel(O1, H, Rr, odd);     // H              | R
  fe_sel(O2, R3, Rr, odd);    // H^2            | R
  fe_mul(R5, O1, O2);         // H^3            | R^2
  fe_xch(t, H);               //                | H
  fe_sel(O1, P, Z, odd);      // X1             | Z1
  fe_sel(O2, R3, t, odd);     // H^2            | H
  fe_mul(R6, O1, O2);         // V = X1 H^2     | Z3 = Z1 H
  fe_xch(W, R5);              // R^2            | H^3
  fe_sub(X3, W, R5);
  fe_shl(t, R6, 1);
  fe_sub(X3, X3, t);          // X3 = R^2 - H^3 - 2V
  fe_sub(D, R6, X3);          // V - X3
  fe_xch(t, D);               //                | V - X3
  fe_xch(O1, P);              // Y1             | X1
  fe_sel(O1, O1, Rr, odd);    // Y1             | R
  fe_sel(O2, R5, t, odd);     // H^3            | V - X3
  fe_mul(R7, O1, O2);         // Y1 H^3         | R (V - X3)
  fe_xch(t, R7);
  fe_sub(t, R7, t);           //                | Y3 = R (V - X3) - Y1 H^3
  fe_sel(P, X3, t, odd);
  Z = R6;                     //                | Z3
}

// acc += b for two Jacobian points of one curve in pair form, exact in
// every case (gej_add_var's semantics): Pa = Xa | Ya, Pb = Xb | Yb, Za and
// Zb on both lanes, flags pair-uniform. Returns Pa = X3 | Y3 and Za = Z3 on
// both lanes. 1S + 7M deep — [Zb^2 | Za^2], [U1 = Xa Zb^2 | Za^3],
// [U2 = Xb Za^2 | Zb^3], [S2 = Yb Za^3 | S1 = Ya Zb^3], [H^2 | Za Zb],
// [H^3 | V = U1 H^2], [R^2 | Z3 = Za Zb H], [S1 H^3 | R (V - X3)] — against
// 4S + 12M one lane at a time.
HKV_DEV void pair_add_var(fe& Pa, fe& Za, bool& ainf, const fe& Pb, const fe& Zb, bool binf, uint32_t odd) {
  fe O1, O2, T, R1, R2, R3, R4, R5, R6, R7, H, Rr, X3, D, Y3, Pn, Zn;
  fe_sel(O1, Zb, Za, odd);
  fe_sqr(R1, O1);             // Zb^2           | Za^2
  fe_xch(T, R1);              // Za^2           | Zb^2
  fe_sel(O1, Pa, R1, odd);    // Xa             | Za^2
  fe_sel(O2, R1, Za, odd);    // Zb^2           | Za
  fe_mul(R2, O1, O2);         // U1 = Xa Zb^2   | Za^3
  fe_sel(O1, Pb, T, odd);     // Xb             | Zb^2
  fe_sel(O2, T, Zb, odd);     // Za^2           | Zb
  fe_mul(R3, O1, O2);         // U2 = Xb Za^2   | Zb^3
  fe_xch(T, R2);              // Za^3           | U1
  fe_xch(O1, Pb);             // Yb             | Xb
  fe_sel(O1, O1, Pa, odd);    // Yb             | Ya
  fe_sel(O2, T, R3, odd);     // Za^3           | Zb^3
  fe_mul(R4, O1, O2);         // S2 = Yb Za^3   | S1 = Ya Zb^3
  fe_sub(H, R3, R2);          // H = U2 - U1
  fe_xch(T, R4);              // S1             | S2
  fe_sub(Rr, R4, T);          // R = S2 - S1
  const bool live = !ainf && !binf;
  const bool hz = pair_even(fe_is_zero(H));
  const bool rz = pair_even(fe_is_zero(Rr));
  fe_sel(O1, H, Za, odd);     // H              | Za
  fe_sel(O2, H, Zb, odd);     // H              | Zb
  fe_mul(R1, O1, O2);         // H^2            | Za Zb
  fe_xch(T, R1);              // Za Zb          | H^2
  fe_xch(O2, R2);             // Za^3           | U1
  fe_sel(O1, H, O2, odd);     // H              | U1
  fe_sel(O2, R1, T, odd);     // H^2            | H^2
  fe_mul(R5, O1, O2);         // H^3            | V = U1 H^2
  fe_xch(T, H);               //                | H
  fe_sel(O1, Rr, R1, odd);    // R              | Za Zb
  fe_sel(O2, Rr, T, odd);     // R              | H
  fe_mul(R6, O1, O2);         // R^2            | Z3 = Za Zb H
  fe_xch(T, R5);              // V              | H^3
  fe_sub(X3, R6, R5);
  fe_shl(O1, T, 1);
  fe_sub(X3, X3, O1);         // X3 = R^2 - H^3 - 2V
  fe_sub(D, T, X3);           // V - X3
  fe_xch(O1, R4);             // S1             | S2
  fe_xch(T, Rr);              //                | R
  fe_sel(O1, O1, T, odd);     // S1             | R
  fe_xch(T, D);               //                | V - X3
  fe_sel(O2, R5, T, odd);     // H^3            | V - X3
  fe_mul(R7, O1, O2);         // S1 H^3         | R (V - X3)
  fe_xch(T, R7);              // R (V - X3)     | S1 H^3
  fe_sub(Y3, T, R7);          // Y3 = R (V - X3) - S1 H^3
  fe_xch(T, Y3);
  fe_sel(Pn, X3, T, odd);     // X3             | Y3
  fe_bc1(Zn, R6);             // Z3 on both lanes
  const bool dbl = live && hz && rz, neg = live && hz && !rz;
  if (__builtin_expect(__any(dbl), 0)) {  // acc == b: 2 acc
    fe Pd = Pa, Zd = Za, Zd2;
    pair_double(Pd, Zd, odd);
    fe_bc1(Zd2, Zd);
    fe_cmov(Pn, Pd, dbl);
    fe_cmov(Zn, Zd2, dbl);
  }
  const bool take_b = ainf && !binf;
  fe_cmov(Pa, Pn, live && !neg);
  fe_cmov(Za, Zn, live && !neg);
  fe_cmov(Pa, Pb, take_b);
  fe_cmov(Za, Zb, take_b);
  ainf = binf ? ainf : (take_b ? false : (live ? neg : ainf));
}

// (P, Z) := (TXY, 1) on pairs that take a point while at infinity
HKV_DEV void pair_accumulate_from_inf(fe& P, fe& Z, bool& inf, const fe& TXY, bool take) {
  const bool f = take && inf;
  fe_cmov(P, TXY, f);
  fe one;
  fe_set_u32(one, 1);
  fe_cmov(Z, one, f);
  inf = inf && !take;
}

// acc := (itx, ity, 1) on lanes that take a point while at infinity
HKV_DEV void gej_accumulate_from_inf(gej& acc, bool& inf, const fe& itx, const fe& ity, bool take) {
  const bool f = take && inf;
  fe_cmov(acc.x, itx, f);
  fe_cmov(acc.y, ity, f);
  fe one;
  fe_set_u32(one, 1);
  fe_cmov(acc.z, one, f);
  inf = inf && !take;
}

}  // namespace hkv
