// Per-primitive throughput of the verify kernels' field / group arithmetic on
// gfx950: each lane runs ITERS dependent iterations of one primitive; the grid
// fills every SIMD with WAVES waves. Reports SIMD-cycles per wave-op, to set
// against the primitive's VALU instruction count (the issue-bound floor).
//
// Ops 7-10 are the representation study (results in
// profiles/r02_ubench_field*.json and profiles/DESIGN_history_r01_r04.md §4): a 9 x 29-bit limb field
// (tools/fe29_proto.h: carry-free v_mad_u64_u32 columns) and a lower bound
// for 52-bit limbs on v_fma_f64 (only the 5 x 5 product with the exact
// hi/lo split and integer column accumulation — no normalisation, no
// reduction), each against the 8 x 32-bit fe_mul / fe_sqr of the product.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_field.hip -o tools/ubench_field
//        (-DHKV_MUL_ASM=0: the row-wise C product instead of the asm scanner)
#include <cstdio>
#include <vector>
#include "../haskoin-node_amd/csrc/hkv_group.h"
#include "fe29_proto.h"

using namespace hkv;
constexpr int ITERS = 256;

struct Stamp { unsigned long long t0, t1, r0, r1; };

// 52-bit limbs as doubles: a_i * b_j = hi + lo exactly with
// hi = fma(a, b, C) - C (C = 1.5 * 2^104: rounds to a multiple of 2^52) and
// lo = fma(a, b, -hi); both parts go to 64-bit integer column accumulators
// through their bit patterns (the exponent bias subtracted once per column).
__device__ __forceinline__ void fp52_mul_lower_bound(double r[5], const double a[5], const double b[5]) {
  const double C = 0x1.8p104, C2 = 0x1.8p52;
  uint64_t col[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) col[k] = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const double h = __builtin_fma(a[i], b[j], C);
      const double l = __builtin_fma(a[i], b[j], C - h) + C2;
      col[i + j + 1] += (uint64_t)__double_as_longlong(h);
      col[i + j] += (uint64_t)__double_as_longlong(l);
    }
  // the result must go back to doubles for the next multiply
#pragma unroll
  for (int k = 0; k < 5; ++k)
    r[k] = __longlong_as_double((long long)((col[k] & 0xFFFFFFFFFFFFFull) | 0x4330000000000000ull)) - 0x1p52 +
           (double)(col[k + 5] & 0xFFFFF);
}

template <int OP>
__global__ void __launch_bounds__(256) kern(const uint32_t* in, uint32_t* out, Stamp* st) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  gej p;
  fe b;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    p.x.v[k] = in[k] ^ tid;
    p.y.v[k] = in[8 + k] + tid;
    p.z.v[k] = in[16 + k] * (tid | 1);
    b.v[k] = in[24 + k] ^ (tid * 7);
  }
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (OP == 0) {
      fe_mul(p.x, p.x, b);
    } else if constexpr (OP == 1) {
      fe_sqr(p.x, p.x);
    } else if constexpr (OP == 2) {
      fe_mul(p.x, p.x, b);
      fe_mul(p.y, p.y, b);
    } else if constexpr (OP == 3) {
      fe_add(p.x, p.x, b);
    } else if constexpr (OP == 4) {
      fe_sub(p.x, p.x, b);
    } else if constexpr (OP == 5) {
      gej_double(p, p);
    } else if constexpr (OP == 6) {
      bool hz, rz;
      gej_add_ge_core(p, p, p.z, b, p.y, hz, rz, nullptr);
    } else if constexpr (OP == 11) {
      fe_mul2(p.x, p.x, b, p.y, p.y, b);
    } else if constexpr (OP == 12) {
      fe_sqr2(p.x, p.x, p.y, p.y);
    } else if constexpr (OP == 13) {
      fe_sqrmul(p.x, p.x, p.y, p.y, b);
    } else if constexpr (OP == 14) {
      fe_mul_ref(p.x, p.x, b);
    } else if constexpr (OP == 15) {
      fe_sqr_ref(p.x, p.x);
    } else if constexpr (OP == 7 || OP == 8 || OP == 9) {
      fe29::fe a29, b29;
#pragma unroll
      for (int k = 0; k < 8; ++k) { a29.v[k] = p.x.v[k] & fe29::M29; b29.v[k] = b.v[k] & fe29::M29; }
      a29.v[8] = p.x.v[0] >> 8;
      b29.v[8] = b.v[1] >> 8;
      if constexpr (OP == 7) {
        fe29::mul(a29, a29, b29);
      } else if constexpr (OP == 8) {
        fe29::sqr(a29, a29);
      } else {
        fe29::sub(a29, a29, b29);
        fe29::carry(a29);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) p.x.v[k] = a29.v[k] ^ a29.v[8];
    } else if constexpr (OP == 10) {
      double a52[5], b52[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        a52[k] = (double)(((uint64_t)(p.x.v[k] & 0xFFFFF) << 32) | p.x.v[k + 1]);
        b52[k] = (double)(((uint64_t)(b.v[k] & 0xFFFFF) << 32) | b.v[k + 1]);
      }
      fp52_mul_lower_bound(a52, a52, b52);
#pragma unroll
      for (int k = 0; k < 5; ++k) p.x.v[k] = (uint32_t)__double_as_longlong(a52[k]);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s ^= p.x.v[k] ^ p.y.v[k] ^ p.z.v[k];
  out[tid] = s;
  if (threadIdx.x == 0) st[blockIdx.x] = Stamp{t0, t1, r0, r1};
}

static const char* NAMES[] = {"fe_mul", "fe_sqr", "fe_mul x2 (independent)", "fe_add", "fe_sub", "gej_double",
                              "gej_add_ge (mixed)", "fe29_mul", "fe29_sqr", "fe29_sub+carry",
                              "fp52_mul (product only, lower bound)", "fe_mul2 (interleaved pair)",
                              "fe_sqr2 (interleaved pair)", "fe_sqrmul (interleaved pair)",
                              "fe_mul_ref (512-bit product + fe_reduce512)", "fe_sqr_ref (512-bit square + fe_reduce512)"};

template <int OP>
void run(int n_cu, int blocks_per_cu) {
  const int threads = 256, blocks = n_cu * blocks_per_cu;
  uint32_t *in, *out;
  Stamp* st;
  hipMalloc(&in, 64 * 4);
  hipMalloc(&out, sizeof(uint32_t) * threads * blocks);
  hipMalloc(&st, sizeof(Stamp) * blocks);
  std::vector<uint32_t> h(64);
  for (int i = 0; i < 64; ++i) h[i] = 0x9E3779B9u * (i + 1);
  hipMemcpy(in, h.data(), 256, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, in, out, st);
  hipEventRecord(e0);
  const int reps = 3;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, in, out, st);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<Stamp> hs(blocks);
  hipMemcpy(hs.data(), st, sizeof(Stamp) * blocks, hipMemcpyDeviceToHost);
  double clk = 0;
  int nc = 0;
  for (auto& s : hs)
    if (s.r1 > s.r0) { clk += (double)(s.t1 - s.t0) / (double)(s.r1 - s.r0) * 100e6; ++nc; }
  clk /= nc;
  // wave-ops per SIMD: blocks * 4 waves * ITERS * reps / (n_cu * 4 SIMDs)
  const double wave_ops_per_simd = (double)blocks * 4 * ITERS * reps / (n_cu * 4.0);
  const double cycles = ms * 1e-3 * clk;
  printf("{\"op\": \"%s\", \"blocks_per_cu\": %d, \"simd_cycles_per_wave_op\": %.1f, \"clk_ghz\": %.3f}\n", NAMES[OP],
         blocks_per_cu, cycles / wave_ops_per_simd, clk * 1e-9);
  hipFree(in);
  hipFree(out);
  hipFree(st);
}

// fe_inv through the reference (512-bit product) ops: the same addition chain
__device__ void fe_inv_ref(fe& r, const fe& a) {
  fe x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t;
  auto sqn = [](fe& o, const fe& i, int n) { fe_sqr_ref(o, i); for (int k = 1; k < n; ++k) fe_sqr_ref(o, o); };
  fe_sqr_ref(x2, a); fe_mul_ref(x2, x2, a);
  fe_sqr_ref(x3, x2); fe_mul_ref(x3, x3, a);
  sqn(t, x3, 3); fe_mul_ref(x6, t, x3);
  sqn(t, x6, 3); fe_mul_ref(x9, t, x3);
  sqn(t, x9, 2); fe_mul_ref(x11, t, x2);
  sqn(t, x11, 11); fe_mul_ref(x22, t, x11);
  sqn(t, x22, 22); fe_mul_ref(x44, t, x22);
  sqn(t, x44, 44); fe_mul_ref(x88, t, x44);
  sqn(t, x88, 88); fe_mul_ref(x176, t, x88);
  sqn(t, x176, 44); fe_mul_ref(x220, t, x44);
  sqn(t, x220, 3); fe_mul_ref(x223, t, x3);
  sqn(t, x223, 23); fe_mul_ref(t, t, x22);
  sqn(t, t, 5); fe_mul_ref(t, t, a);
  sqn(t, t, 3); fe_mul_ref(t, t, x2);
  sqn(t, t, 2); fe_mul_ref(r, t, a);
}

// chains: fe_inv and 64 squarings with the kernels' ops against the reference ops
__global__ void check_chains(uint32_t* bad) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  fe a;
  uint32_t x = tid * 0x85EBCA6Bu + 7;
#pragma unroll
  for (int k = 0; k < 8; ++k) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; a.v[k] = x; }
  fe r, s;
  uint32_t nb = 0;
  fe_inv(r, a); fe_inv_ref(s, a);
  fe_normalize(r); fe_normalize(s);
  nb += !fe_eq_norm(r, s);
  fe_sqr_n(r, a, 64);
  s = a;
  for (int k = 0; k < 64; ++k) fe_sqr_ref(s, s);
  fe_normalize(r); fe_normalize(s);
  nb += 2 * !fe_eq_norm(r, s);
  // fe_cneg against fe_neg + select, on random, zero, p and weak-form values >= p
  for (int e = 0; e < 6; ++e) {
    fe b = a;
    if (e == 1) fe_set_zero(b);
    if (e == 2 || e == 3) { b.v[0] = 0xFFFFFC2Fu + (e == 3 ? 5u : 0u); b.v[1] = 0xFFFFFFFEu; for (int q = 2; q < 8; ++q) b.v[q] = 0xFFFFFFFFu; }
    if (e == 4) for (int q = 0; q < 8; ++q) b.v[q] = 0xFFFFFFFFu;
    if (e == 5) { fe_set_zero(b); b.v[1] = 0xFFFFFFFFu; b.v[0] = tid; }
    for (int ng = 0; ng < 2; ++ng) {
      fe x, y;
      fe_cneg(x, b, ng != 0);
      fe_neg(y, b);
      if (ng == 0) y = b;
      fe_normalize(x); fe_normalize(y);
      nb += 8 * !fe_eq_norm(x, y);
    }
  }
  fe_mul(r, a, a); fe_mul(r, r, a); fe_sqr(r, r); fe_mul(r, a, r);
  fe_mul_ref(s, a, a); fe_mul_ref(s, s, a); fe_sqr_ref(s, s); fe_mul_ref(s, a, s);
  fe_normalize(r); fe_normalize(s);
  nb += 4 * !fe_eq_norm(r, s);
  if (nb) atomicOr(bad, nb);
}

// paired forms against the single forms on pseudo-random operands (including
// values >= p, the weak form the kernels carry)
__global__ void check_pairs(uint32_t* bad) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  fe a, b, c, d;
  uint32_t x = tid * 0x9E3779B9u + 1;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5; a.v[k] = x;
    x ^= x << 13; x ^= x >> 17; x ^= x << 5; b.v[k] = x;
    x ^= x << 13; x ^= x >> 17; x ^= x << 5; c.v[k] = x;
    x ^= x << 13; x ^= x >> 17; x ^= x << 5; d.v[k] = x;
  }
  if (tid % 7 == 0) for (int k = 0; k < 8; ++k) a.v[k] = 0xFFFFFFFFu;
  if (tid % 11 == 0) for (int k = 0; k < 8; ++k) c.v[k] = 0xFFFFFFFFu;
  if (tid % 13 == 0) for (int k = 0; k < 8; ++k) b.v[k] = 0xFFFFFFFFu;
  if (tid % 17 == 0) { for (int k = 0; k < 8; ++k) a.v[k] = 0; a.v[0] = tid & 3; }
  if (tid % 19 == 0) { a.v[0] = 0xFFFFFC2Fu; a.v[1] = 0xFFFFFFFEu; for (int k = 2; k < 8; ++k) a.v[k] = 0xFFFFFFFFu; }
  if (tid % 23 == 0) for (int k = 0; k < 8; ++k) a.v[k] = (k & 1) ? 0x80000000u : 0xFFFFFFFFu;
  fe r1, r2, s1, s2;
  uint32_t nb = 0;
  // folded-reduction forms (fe_mul / fe_sqr) against the 512-bit product path
  fe_mul(r1, a, b); fe_mul_ref(s1, a, b);
  fe_sqr(r2, a); fe_sqr_ref(s2, a);
  fe_normalize(r1); fe_normalize(r2); fe_normalize(s1); fe_normalize(s2);
  nb += !fe_eq_norm(r1, s1) + !fe_eq_norm(r2, s2);
  fe_mul(r1, c, d); fe_mul_ref(s1, c, d);
  fe_sqr(r2, c); fe_sqr_ref(s2, c);
  fe_normalize(r1); fe_normalize(r2); fe_normalize(s1); fe_normalize(s2);
  nb += !fe_eq_norm(r1, s1) + !fe_eq_norm(r2, s2);
  // in place, as the kernels call them
  r1 = a; fe_mul(r1, r1, b); fe_mul_ref(s1, a, b);
  r2 = c; fe_sqr(r2, r2); fe_sqr_ref(s2, c);
  fe_normalize(r1); fe_normalize(r2); fe_normalize(s1); fe_normalize(s2);
  nb += !fe_eq_norm(r1, s1) + !fe_eq_norm(r2, s2);
  fe_mul2(r1, a, b, r2, c, d);
  fe_mul(s1, a, b); fe_mul(s2, c, d);
  fe_normalize(r1); fe_normalize(r2); fe_normalize(s1); fe_normalize(s2);
  nb += !fe_eq_norm(r1, s1) + !fe_eq_norm(r2, s2);
  fe_sqr2(r1, a, r2, c);
  fe_sqr(s1, a); fe_sqr(s2, c);
  fe_normalize(r1); fe_normalize(r2); fe_normalize(s1); fe_normalize(s2);
  nb += !fe_eq_norm(r1, s1) + !fe_eq_norm(r2, s2);
  fe_sqrmul(r1, a, r2, c, d);
  fe_sqr(s1, a); fe_mul(s2, c, d);
  fe_normalize(r1); fe_normalize(r2); fe_normalize(s1); fe_normalize(s2);
  nb += !fe_eq_norm(r1, s1) + !fe_eq_norm(r2, s2);
  if (nb) atomicAdd(bad, nb);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int n_cu = p.multiProcessorCount;
  {
    uint32_t* bad;
    hipMalloc(&bad, 4);
    hipMemset(bad, 0, 4);
    hipLaunchKernelGGL(check_pairs, dim3(1024), dim3(256), 0, 0, bad);
    uint32_t hb = 0;
    hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    printf("{\"check\": \"paired and folded-reduction field ops vs the 512-bit path\", \"lanes\": %d, \"mismatches\": %u}\n", 1024 * 256, hb);
    hipMemset(bad, 0, 4);
    hipLaunchKernelGGL(check_chains, dim3(64), dim3(256), 0, 0, bad);
    hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    printf("{\"check\": \"fe_inv / 64 squarings / cneg / mixed chain vs the reference ops (bit mask of failing checks)\", \"lanes\": %d, \"fail_mask\": %u}\n", 64 * 256, hb);
    hipFree(bad);
  }
  for (int bpc : {1, 2, 4}) {
    run<0>(n_cu, bpc); run<1>(n_cu, bpc); run<2>(n_cu, bpc); run<3>(n_cu, bpc);
    run<4>(n_cu, bpc); run<5>(n_cu, bpc); run<6>(n_cu, bpc);
    run<7>(n_cu, bpc); run<8>(n_cu, bpc); run<9>(n_cu, bpc); run<10>(n_cu, bpc);
    run<11>(n_cu, bpc); run<12>(n_cu, bpc); run<13>(n_cu, bpc);
    run<14>(n_cu, bpc); run<15>(n_cu, bpc);
  }
  return 0;
}
