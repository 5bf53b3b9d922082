// Lone-wave latency of the block kernel's doubling forms on gfx950 (one
// workgroup of 4 waves per CU: every wave alone on its SIMD, as in
// hkv_block_kernel). Each lane runs ITERS dependent doublings; reports SIMD
// cycles per doubling, and first checks every form against gej_double
// (projective equality after 5 doublings of pseudo-random (X, Y, Z)).
//
//   quad_double  four lanes per point (S + 2M deep)
//   pair_double  two lanes per point (2S + 2M deep)
//   fe_sqr / fe_mul / fe_sub  the primitives alone, for scale
// profiles/r03n_ubench_chain.json holds the A/B that chose the unhalved
// forms (op names *_s there) over the halved ones: quad 3,487 -> 3,367
// cycles, pair 4,028 -> 4,074 (in the kernel both together took the
// configs[0] block from 305 to 295 us).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_chain.hip -o tools/ubench_chain
#include <algorithm>
#include <cstdio>
#include <vector>
#include "../haskoin-node_amd/csrc/hkv_group.h"

using namespace hkv;
constexpr int ITERS = 128;

//  the a = 0 doubling in its 2M + 5S form, M from
// (X + B)^2 - A - C instead of X * B, in gej_double's halved scaling
// (X3/4, Y3/8, Z3/2): one square for one product, at the price of an add,
// two subtractions and a halving
__device__ __forceinline__ void gej_double_2m5s(gej& r, const gej& a) {
  fe A, B, C, M2, M, E, t;
  fe_sqr(A, a.x);
  fe_sqr(B, a.y);
  fe_add(t, a.x, B);
  fe_sqr(t, t);
  fe_sqr(C, B);
  fe_sub(t, t, A);
  fe_sub(M2, t, C);         // 2 X B
  fe_half(M, M2);
  fe_mul_small(E, A, 3);
  fe_half(E, E);            // E' = 3A/2
  fe_mul(r.z, a.y, a.z);    // Z3' = YZ
  fe_sqr(t, E);
  fe_sub(r.x, t, M2);       // X3' = E'^2 - 2M
  fe_sub(t, M, r.x);
  fe_mul(t, E, t);
  fe_sub(r.y, t, C);        // Y3' = E'(M - X3') - C
}

// ---- lane-split products (prototype): the 64 limb
// products of one 256 x 256 product spread over 2 or 4 lanes of a quad by
// rows of a, the partials summed across lanes by DPP, one reduction ----
// fe_mul_rows2 / fe_mul_rows4: hkv_group.h (HKV_QUAD_SPLIT)
// quad_double with the two products that leave lanes idle spread over them:
// [A | B] as two 2-way row-split squares (X^2 on lanes 0, 2; Y^2 on 1, 3),
// Y3 = A D - 8C as a 4-way row-split product on lane 1
__device__ __forceinline__ void quad_double_split(fe& V, uint32_t m0, uint32_t m1, uint32_t m2) {
  fe S, R1, Aq, RA, T, opA, opB, R2, P1, P2, r, t, C8, Dq;
  fe_quad<QP_0101>(S, V);     // X | Y | X | Y
  fe_mul_rows2(R1, S, S, ~(m0 | m1));  // A = X^2 | B = Y^2 | . | .
  fe_quad<QP_0>(Aq, R1);
  fe_quad<QP_1100>(RA, R1);
  fe_quad<QP_0112>(T, V);
  fe_sel(opA, RA, T, m0 | m2);
  fe_sel(opB, RA, V, m2);
  fe_mul(R2, opA, opB);       // M | C | YZ | A^2
  fe_quad<QP_3021>(P1, R2);
  fe_quad<QP_0331>(P2, R2);
  const uint32_t k1 = m0 ? 9u : (m1 ? 36u : (m2 ? 2u : 0u));
  const uint32_t k2 = m0 ? 8u : (m1 ? 27u : (m2 ? 0u : 8u));
  fe_lin2(r, P1, k1, P2, k2); // X3 | D | Z3 | -8C
  fe_quad<QP_3>(C8, r);
  fe_quad<QP_1>(Dq, r);       // D on every lane
  fe_mul_rows4(t, Aq, Dq, m0, m1, m2);
  fe_add(t, t, C8);           // . | Y3 = A D - 8C | . | .
  fe_sel(V, r, t, m1);
}

struct Stamp { unsigned long long t0, t1, r0, r1; };

__device__ void seed_point(uint32_t c, gej& p) {
  uint32_t x = c * 0x9E3779B9u + 0x1234567u;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5; p.x.v[k] = x;
    x ^= x << 13; x ^= x >> 17; x ^= x << 5; p.y.v[k] = x;
    x ^= x << 13; x ^= x >> 17; x ^= x << 5; p.z.v[k] = x;
  }
}

// a == b as projective points (X / Z^2, Y / Z^3)
__device__ bool same_point(const gej& a, const gej& b) {
  fe za2, zb2, za3, zb3, l, r;
  fe_sqr(za2, a.z); fe_sqr(zb2, b.z);
  fe_mul(za3, za2, a.z); fe_mul(zb3, zb2, b.z);
  bool ok = true;
  fe_mul(l, a.x, zb2); fe_mul(r, b.x, za2);
  fe_normalize(l); fe_normalize(r);
  ok = ok && fe_eq_norm(l, r);
  fe_mul(l, a.y, zb3); fe_mul(r, b.y, za3);
  fe_normalize(l); fe_normalize(r);
  return ok && fe_eq_norm(l, r);
}

__device__ fe shfl_fe(const fe& a, int src) {
  fe r;
#pragma unroll
  for (int k = 0; k < 8; ++k) r.v[k] = (uint32_t)__shfl((int)a.v[k], src);
  return r;
}

constexpr int NDBL = 5;
__global__ void check_forms(uint32_t* bad) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t ln = threadIdx.x & 63;
  uint32_t nb = 0;
  // quad forms: point c = tid / 4 on lanes 4c'..4c'+3
  {
    const uint32_t c = tid >> 2, qd = ln & 3u;
    const uint32_t m0 = qd == 0 ? ~0u : 0u, m1 = qd == 1 ? ~0u : 0u, m2 = qd == 2 ? ~0u : 0u;
    gej p, ref;
    seed_point(c, p);
    ref = p;
    for (int d = 0; d < NDBL; ++d) gej_double(ref, ref);
    fe V = p.z;
    fe_sel(V, V, p.y, m1);
    fe_sel(V, V, p.x, m0);
    fe V2 = V;
    for (int d = 0; d < NDBL; ++d) quad_double(V, m0, m1, m2);
    const int b4 = (int)(ln & ~3u);
    gej q;
    q.x = shfl_fe(V, b4); q.y = shfl_fe(V, b4 + 1); q.z = shfl_fe(V, b4 + 2);
    if (!same_point(q, ref)) nb |= 1u;
    for (int d = 0; d < NDBL; ++d) quad_double_split(V2, m0, m1, m2);
    q.x = shfl_fe(V2, b4); q.y = shfl_fe(V2, b4 + 1); q.z = shfl_fe(V2, b4 + 2);
    if (!same_point(q, ref)) nb |= 8u;
  }
  // 2M + 5S against 3M + 4S
  {
    gej p, ref, q;
    seed_point(tid + 0x200000u, p);
    ref = p;
    q = p;
    for (int d = 0; d < NDBL; ++d) gej_double(ref, ref);
    for (int d = 0; d < NDBL; ++d) gej_double_2m5s(q, q);
    if (!same_point(q, ref)) nb |= 4u;
  }
  // pair forms: point c = tid / 2 on lanes 2c', 2c'+1
  {
    const uint32_t c = tid >> 1;
    const uint32_t odd = (ln & 1u) ? ~0u : 0u;
    gej p, ref;
    seed_point(c + 0x100000u, p);
    ref = p;
    for (int d = 0; d < NDBL; ++d) gej_double(ref, ref);
    fe P, Z = p.z;
    fe_sel(P, p.x, p.y, odd);
    for (int d = 0; d < NDBL; ++d) pair_double(P, Z, odd);
    const int b2 = (int)(ln & ~1u);
    gej q;
    q.x = shfl_fe(P, b2); q.y = shfl_fe(P, b2 + 1); q.z = shfl_fe(Z, b2 + 1);
    if (!same_point(q, ref)) nb |= 2u;
  }
  if (nb) atomicOr(bad, nb);
}

template <int OP>
__global__ void __launch_bounds__(256) kern(uint32_t* out, Stamp* st) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t ln = threadIdx.x & 63;
  const uint32_t qd = ln & 3u;
  const uint32_t m0 = qd == 0 ? ~0u : 0u, m1 = qd == 1 ? ~0u : 0u, m2 = qd == 2 ? ~0u : 0u;
  const uint32_t odd = (ln & 1u) ? ~0u : 0u;
  gej p;
  seed_point(tid, p);
  fe V = p.x, Z = p.z, b = p.y;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (OP == 0) quad_double(V, m0, m1, m2);
    else if constexpr (OP == 1) pair_double(V, Z, odd);
    else if constexpr (OP == 2) fe_sqr(V, V);
    else if constexpr (OP == 3) fe_mul(V, V, b);
    else if constexpr (OP == 4) fe_sub(V, V, b);
    else if constexpr (OP == 5 || OP == 6) {
      gej g;
      g.x = V; g.y = b; g.z = Z;
      if constexpr (OP == 5) gej_double(g, g);
      else gej_double_2m5s(g, g);
      V = g.x; b = g.y; Z = g.z;
    } else if constexpr (OP == 7) quad_double_split(V, m0, m1, m2);
    else if constexpr (OP == 8) fe_mul_rows2(V, V, V, ~(m0 | m1));
    else if constexpr (OP == 9) fe_mul_rows4(V, V, b, m0, m1, m2);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s ^= V.v[k] ^ Z.v[k];
  out[tid] = s;
  if (threadIdx.x == 0) st[blockIdx.x] = Stamp{t0, t1, r0, r1};
}

static const char* NAMES[] = {"quad_double", "pair_double", "fe_sqr", "fe_mul", "fe_sub", "gej_double (3M+4S)",
                              "gej_double_2m5s", "quad_double_split", "fe_mul_rows2 (square)", "fe_mul_rows4"};

template <int OP>
void run(int n_cu, int wps = 1) {
  const int threads = 256, blocks = n_cu * wps;  // wps waves per SIMD
  uint32_t* out;
  Stamp* st;
  hipMalloc(&out, sizeof(uint32_t) * threads * blocks);
  hipMalloc(&st, sizeof(Stamp) * blocks);
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, out, st);
  double best = 1e30, ghz = 0;
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, out, st);
    std::vector<Stamp> hs(blocks);
    hipMemcpy(hs.data(), st, sizeof(Stamp) * blocks, hipMemcpyDeviceToHost);
    // in-kernel shader cycles of the loop (s_memtime), median over workgroups
    std::vector<double> cyc;
    double clk = 0;
    for (auto& s : hs) {
      cyc.push_back((double)(s.t1 - s.t0));
      if (s.r1 > s.r0) clk += (double)(s.t1 - s.t0) / (double)(s.r1 - s.r0) * 100e6;
    }
    std::sort(cyc.begin(), cyc.end());
    const double c = cyc[cyc.size() / 2] / ITERS / wps;  // SIMD cycles per op (wps waves share a SIMD)
    if (c < best) { best = c; ghz = clk / blocks * 1e-9; }
  }
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"simd_cycles_per_op\": %.1f, \"clk_ghz\": %.3f}\n", NAMES[OP], wps,
         best, ghz);
  hipFree(out);
  hipFree(st);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int n_cu = p.multiProcessorCount;
  uint32_t* bad;
  hipMalloc(&bad, 4);
  hipMemset(bad, 0, 4);
  hipLaunchKernelGGL(check_forms, dim3(256), dim3(256), 0, 0, bad);
  uint32_t hb = 0;
  hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
  printf("{\"check\": \"quad/pair doubling forms vs gej_double, %d doublings (bit 0 quad, 1 pair, 2 the 2M + 5S form)\", "
         "\"lanes\": %d, \"fail_mask\": %u}\n", NDBL, 256 * 256, hb);  // bit 2: 2M + 5S, bit 3: quad split
  hipFree(bad);
  run<0>(n_cu); run<1>(n_cu); run<2>(n_cu); run<3>(n_cu); run<4>(n_cu);
  run<5>(n_cu); run<6>(n_cu); run<5>(n_cu, 4); run<6>(n_cu, 4);  // the ecmult kernel runs 4 waves/SIMD
  run<7>(n_cu); run<8>(n_cu); run<9>(n_cu);
  return hb ? 1 : 0;
}
