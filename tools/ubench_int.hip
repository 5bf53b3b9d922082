// Integer / fp64 VALU issue-rate microbenchmark for gfx950.
//
// Fixes the roofline denominator for the secp256k1 verifier (SURVEY.md §7 step 1,
// §8(d)): lane-operations per clock per CU for each candidate limb-product
// instruction. Each lane runs UNROLL independent chains of one instruction in a
// loop; the grid is 8 x 256 CUs x 1024 threads so every SIMD is saturated.
// Clock is measured in-kernel (s_memtime / s_memrealtime at 100 MHz).
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_int.hip -o tools/ubench_int
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;
constexpr int CH = 8;  // independent chains per lane

struct Stamp { unsigned long long t0, t1, r0, r1; };

template <int OP>
__global__ void __launch_bounds__(256) kern(uint32_t seed, uint32_t* out, Stamp* st) {
  uint32_t a[CH], b = seed ^ threadIdx.x;
  uint64_t acc[CH];
  double d[CH];
  double dm = 1.0000001 + (double)(seed & 7) * 1e-9;
#pragma unroll
  for (int k = 0; k < CH; ++k) { a[k] = seed * (k + 3) + threadIdx.x; acc[k] = a[k]; d[k] = (double)a[k]; }
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      if constexpr (OP == 0) {  // v_mad_u64_u32
        asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(acc[k]) : "v"(a[k]), "v"(b) : "s40", "s41");
      } else if constexpr (OP == 1) {  // v_mul_lo_u32
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 2) {  // v_mul_hi_u32
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 3) {  // v_mul_u32_u24
        asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 4) {  // v_mad_u32_u24
        asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 5) {  // v_fma_f64
        asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(d[k]) : "v"(dm));
      } else if constexpr (OP == 6) {  // v_add_u32 (full-rate reference)
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 7) {  // v_lshl_add_u64
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[k]) : "v"(acc[(k + 1) % CH]));
      } else if constexpr (OP == 8) {  // v_add_co_u32 + v_addc_co_u32 (64-bit add pair)
        asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, %2, 0, vcc"
                     : "+v"(a[k]), "+v"(b) : "v"(seed) : "vcc");
      } else if constexpr (OP == 9) {  // v_mul_hi_u32_u24
        asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 10) {  // v_mad_u64_u32 with carry-out + v_addc (product+carry chain)
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0\n\tv_addc_co_u32 %3, vcc, %3, 0, vcc"
                     : "+v"(acc[k]) : "v"(a[k]), "v"(b), "v"(a[(k+1)%CH]) : "vcc");
      } else if constexpr (OP == 11) {  // v_cndmask_b32
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 12) {  // v_mul_f64
        asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[k]) : "v"(dm));
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) s ^= a[k] ^ (uint32_t)acc[k] ^ (uint32_t)(acc[k] >> 32) ^ (uint32_t)(uint64_t)d[k] ^ b;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) { st[blockIdx.x] = Stamp{t0, t1, r0, r1}; }
}

// instructions issued per inner iteration per lane for each op (OP 8, 10 issue 2)
static const char* NAMES[] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_u32_u24",
                              "v_mad_u32_u24", "v_fma_f64", "v_add_u32", "v_lshl_add_u64",
                              "v_add_co+v_addc (pair)", "v_mul_hi_u32_u24", "v_mad_u64_u32(co)+v_addc (pair)",
                              "v_cndmask_b32", "v_mul_f64"};

template <int OP>
int run(int n_cu) {
  const int threads = 256, blocks = n_cu * 8;
  uint32_t* out; Stamp* st;
  CHECK(hipMalloc(&out, sizeof(uint32_t) * threads * blocks));
  CHECK(hipMalloc(&st, sizeof(Stamp) * blocks));
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, 12345u, out, st);
  CHECK(hipEventRecord(e0));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, 12345u + r, out, st);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<Stamp> h(blocks);
  CHECK(hipMemcpy(h.data(), st, sizeof(Stamp) * blocks, hipMemcpyDeviceToHost));
  double clk = 0; int nc = 0;
  for (auto& s : h) if (s.r1 > s.r0) { clk += (double)(s.t1 - s.t0) / (double)(s.r1 - s.r0) * 100e6; ++nc; }
  clk /= nc;
  double lane_ops = (double)reps * blocks * threads * ITERS * CH;
  double sec = ms * 1e-3;
  double per_clk_cu = lane_ops / sec / clk / n_cu;
  printf("{\"op\": \"%s\", \"lane_ops_per_s\": %.4e, \"clk_ghz\": %.3f, \"lane_ops_per_clk_per_cu\": %.2f, \"ms\": %.3f}\n",
         NAMES[OP], lane_ops / sec, clk * 1e-9, per_clk_cu, ms / reps);
  CHECK(hipFree(out)); CHECK(hipFree(st));
  return 0;
}

int main() {
  hipDeviceProp_t p; if (hipGetDeviceProperties(&p, 0) != hipSuccess) { fprintf(stderr, "no device\n"); return 1; }
  int n_cu = p.multiProcessorCount;
  printf("# device %s CUs %d\n", p.gcnArchName, n_cu);
  int rc = 0;
  rc |= run<6>(n_cu); rc |= run<0>(n_cu); rc |= run<10>(n_cu); rc |= run<1>(n_cu); rc |= run<2>(n_cu);
  rc |= run<3>(n_cu); rc |= run<9>(n_cu); rc |= run<4>(n_cu); rc |= run<5>(n_cu); rc |= run<12>(n_cu);
  rc |= run<7>(n_cu); rc |= run<8>(n_cu); rc |= run<11>(n_cu);
  return rc;
}
