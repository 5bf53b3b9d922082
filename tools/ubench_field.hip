// Per-primitive throughput of the verify kernels' field / group arithmetic on
// gfx950: each lane runs ITERS dependent iterations of one primitive; the grid
// fills every SIMD with WAVES waves. Reports SIMD-cycles per wave-op, to set
// against the primitive's VALU instruction count (the issue-bound floor).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_field.hip -o tools/ubench_field
#include <cstdio>
#include <vector>
#include "../haskoin-node_amd/csrc/hkv_group.h"

using namespace hkv;
constexpr int ITERS = 256;

struct Stamp { unsigned long long t0, t1, r0, r1; };

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
                              "gej_add_ge (mixed)"};

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

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int n_cu = p.multiProcessorCount;
  for (int bpc : {1, 2, 4}) {
    run<0>(n_cu, bpc); run<1>(n_cu, bpc); run<2>(n_cu, bpc); run<3>(n_cu, bpc);
    run<4>(n_cu, bpc); run<5>(n_cu, bpc); run<6>(n_cu, bpc);
  }
  return 0;
}
