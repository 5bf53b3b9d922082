// Launch-overhead microbenchmark for the block kernel's shape (round 4): the
// rocprofv3 duration of hkv_block_kernel<true> on a configs[0] block is
// ~258 us while its 256 workgroups' own start / end stamps span ~242 us
// (bench split_phases_us.groups). This times, with HIP events around 40
// back-to-back launches, kernels of the same shape (256 workgroups of 256
// threads, one wave per SIMD, 96 KB of LDS) that spin a fixed time measured
// on the 100-MHz wall clock, with and without a private (scratch) segment and
// with a straight-line code body of 0 / 320 KB, and with 0 / 2 / 16 MB
// of stores before the end, so the launch + teardown
// cost outside the kernel body is event time minus the spin.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_launch.hip -o tools/ubench_launch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int WG = 256;

// SCRATCH: a dynamically indexed private array (forces a private segment).
// BODY: a long run of dependent, non-foldable VALU work executed once per
// wave (straight-line code the I-cache sees cold on every CU).
template <bool SCRATCH, int BODY, int WR_KB, bool BIGREG = false, int LDS_KW = 24>
__global__ void __launch_bounds__(WG, 1) spin_kernel(uint32_t* out, uint32_t ticks, uint32_t sel,
                                                     unsigned long long* stamps) {
  __shared__ uint32_t lds[LDS_KW * 1024];  // 96 KB by default
  const uint32_t t = threadIdx.x;
  lds[t] = t * sel;
  __syncthreads();
  const unsigned long long t0 = wall_clock64();
  if (t == 0) stamps[2 * blockIdx.x] = t0;
  uint32_t x = lds[(t + 1) & (WG - 1)] + sel;
  // BIGREG: claim every arch VGPR and AGPR (the block kernel's 256 + 256)
  if constexpr (BIGREG) asm volatile("v_mov_b32 v255, 0\n\tv_accvgpr_write_b32 a255, 0" ::: "v255", "a255");
  if constexpr (SCRATCH) {
    volatile uint32_t p[3];
    p[sel % 3] = x;
    p[(sel + 1) % 3] = x + 1;
    p[(sel + 2) % 3] = x + 2;
    x += p[(t + sel) % 3];
  }
  if constexpr (BODY > 0) {
    asm volatile(".rept %1\n\tv_alignbit_b32 %0, %0, %0, 3\n\t.endr" : "+v"(x) : "i"(BODY));
  }
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
  __syncthreads();
  if (t == 0) stamps[2 * blockIdx.x + 1] = wall_clock64();
  if (x == 0x12345678u) out[blockIdx.x * WG + t] = x;
  // WR_KB KB of ordinary stores per workgroup before the end (dirty L2 lines
  // the end-of-kernel release writes back)
  if constexpr (WR_KB > 0) {
    uint4* o = reinterpret_cast<uint4*>(out) + (size_t)blockIdx.x * (WR_KB * 64) + t;
#pragma unroll 1
    for (int k = 0; k < WR_KB / 4; ++k) o[k * WG] = make_uint4(x, x + 1, x + 2, x + k);
  }
}

template <bool SCRATCH, int BODY, int WR_KB = 0, bool BIGREG = false, int LDS_KW = 24>
int run(const char* name, uint32_t* out, unsigned long long* stamps, int n_wg, hipStream_t st) {
  const int wall_khz = 100000;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (uint32_t us : {0u, 100u, 240u}) {
    const uint32_t ticks = us * (uint32_t)(wall_khz / 1000);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((spin_kernel<SCRATCH, BODY, WR_KB, BIGREG, LDS_KW>), dim3(n_wg), dim3(WG), 0, st, out, ticks, 1u, stamps);
    CHECK(hipStreamSynchronize(st));
    const int reps = 40;
    float best = 1e30f, sum = 0;
    for (int r = 0; r < reps; ++r) {
      CHECK(hipEventRecord(e0, st));
      hipLaunchKernelGGL((spin_kernel<SCRATCH, BODY, WR_KB, BIGREG, LDS_KW>), dim3(n_wg), dim3(WG), 0, st, out, ticks, 1u, stamps);
      CHECK(hipEventRecord(e1, st));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      sum += ms;
    }
    // the last launch's group span on the wall clock
    unsigned long long h[2 * 256];
    CHECK(hipMemcpy(h, stamps, 2 * n_wg * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    unsigned long long s0 = ~0ull, s1 = 0;
    for (int b = 0; b < n_wg; ++b) {
      s0 = h[2 * b] < s0 ? h[2 * b] : s0;
      s1 = h[2 * b + 1] > s1 ? h[2 * b + 1] : s1;
    }
    const double span_us = (double)(s1 - s0) / (wall_khz / 1000.0);
    printf("{\"kernel\": \"%s\", \"spin_us\": %u, \"event_us_min\": %.2f, \"event_us_avg\": %.2f, \"group_span_us\": %.2f, "
           "\"outside_us\": %.2f}\n", name, us, best * 1e3, sum / reps * 1e3, span_us, best * 1e3 - span_us);
  }
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

int main() {
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  uint32_t* out;
  unsigned long long* stamps;
  const int n_wg = 256;
  CHECK(hipMalloc(&out, (size_t)n_wg * 64 * 1024));
  CHECK(hipMalloc(&stamps, 2 * n_wg * sizeof(unsigned long long)));
  if (run<false, 0>("plain", out, stamps, n_wg, st)) return 1;
  if (run<true, 0>("scratch", out, stamps, n_wg, st)) return 1;
  if (run<false, 40000>("code_320k", out, stamps, n_wg, st)) return 1;
  if (run<true, 40000>("scratch_code_320k", out, stamps, n_wg, st)) return 1;
  if (run<false, 0, 8>("write_2mb", out, stamps, n_wg, st)) return 1;
  if (run<true, 0, 0, true>("scratch_vgpr512", out, stamps, n_wg, st)) return 1;
  if (run<true, 0, 0, true, 32>("scratch_vgpr512_lds128k", out, stamps, n_wg, st)) return 1;
  if (run<true, 40000, 8, true, 32>("scratch_vgpr512_lds128k_code_write", out, stamps, n_wg, st)) return 1;
  if (run<false, 0, 64>("write_16mb", out, stamps, n_wg, st)) return 1;
  CHECK(hipFree(out));
  CHECK(hipFree(stamps));
  return 0;
}
