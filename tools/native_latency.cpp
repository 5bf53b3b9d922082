// The tip block as a native caller sees it: one block's
// txs and input jobs in HBM, verified by hkv_verify_std_inputs_device from C++
// through the C ABI only (no Python, no ctypes in front of the call), the way
// a Haskell node's `foreign import ccall safe` would call it.
//
//   python3 tools/native_latency.py dump gpurun_out/blk0      (BASELINE configs[0])
//   tools/native_latency gpurun_out/blk0 > gpurun_out/native_latency.json
//
// Reported (microseconds, medians): back to back (32 calls between two HIP
// events, three times), one call alone right after a synchronize, one call
// alone after 5 ms of GPU idle; per call alone the HIP-event latency on the
// call's stream, the host time inside the call (enqueue) and the host wall
// clock from before the call to its verdict words being readable.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "../include/hkv.h"

static std::vector<uint8_t> slurp(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) {
    std::fprintf(stderr, "native_latency: cannot read %s\n", path.c_str());
    std::exit(2);
  }
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

#define HIP_OK(x)                                                                  \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "native_latency: %s: %s\n", #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: native_latency <block dir> [calls]\n");
    return 2;
  }
  const std::string dir = argv[1];
  const int calls = argc > 2 ? std::atoi(argv[2]) : 40;
  const std::vector<uint8_t> txs = slurp(dir + "/txs.bin"), offs = slurp(dir + "/offsets.bin"),
                             pool = slurp(dir + "/scripts.bin"), jobs = slurp(dir + "/jobs.bin");
  if (offs.size() < 8 || offs.size() % 4 || jobs.size() % sizeof(hkv_input_job)) {
    std::fprintf(stderr, "native_latency: malformed block files in %s\n", dir.c_str());
    return 2;
  }
  const uint32_t n_tx = (uint32_t)(offs.size() / 4 - 1);
  const size_t n = jobs.size() / sizeof(hkv_input_job);

  const int dev_id = 0;
  hkv_ctx* ctx = nullptr;
  int rc = hkv_open_devices(&dev_id, 1, HKV_OPEN_NO_SELFCHECK, &ctx);
  if (rc != HKV_OK) {
    std::fprintf(stderr, "native_latency: hkv_open_devices: %s\n", hkv_strerror(rc));
    return 1;
  }
  HIP_OK(hipSetDevice(0));
  uint8_t *d_txs, *d_pool, *d_recs;
  uint32_t *d_offs, *d_bits;
  void* d_jobs;
  const size_t n_words = (n + 63) / 64 * 2;
  HIP_OK(hipMalloc(&d_txs, txs.size()));
  HIP_OK(hipMalloc(&d_offs, offs.size()));
  HIP_OK(hipMalloc(&d_pool, std::max<size_t>(pool.size(), 1)));
  HIP_OK(hipMalloc(&d_jobs, jobs.size()));
  HIP_OK(hipMalloc(&d_recs, n * 168));
  HIP_OK(hipMalloc(&d_bits, n_words * 4));
  HIP_OK(hipMemcpy(d_txs, txs.data(), txs.size(), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_offs, offs.data(), offs.size(), hipMemcpyHostToDevice));
  if (!pool.empty()) HIP_OK(hipMemcpy(d_pool, pool.data(), pool.size(), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_jobs, jobs.data(), jobs.size(), hipMemcpyHostToDevice));
  const hkv_txs t{d_txs, d_offs, n_tx, d_pool, (uint32_t)pool.size()};
  hipStream_t st;
  HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  auto call = [&]() {
    const int r = hkv_verify_std_inputs_device(ctx, 0, &t, static_cast<const hkv_input_job*>(d_jobs), n, -1, d_recs,
                                               d_bits, st);
    if (r != HKV_OK) {
      std::fprintf(stderr, "native_latency: hkv_verify_std_inputs_device: %s\n", hkv_strerror(r));
      std::exit(1);
    }
  };
  using clk = std::chrono::steady_clock;
  auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };

  // warm-up: >= 100 ms of calls back to back (the shader clock ramps over tens of ms)
  const auto w0 = clk::now();
  do {
    for (int k = 0; k < 16; ++k) call();
    HIP_OK(hipStreamSynchronize(st));
  } while (us(w0, clk::now()) < 100e3);

  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  std::vector<double> b2b;
  for (int rep = 0; rep < 3; ++rep) {
    HIP_OK(hipStreamSynchronize(st));
    HIP_OK(hipEventRecord(e0, st));
    for (int k = 0; k < 32; ++k) call();
    HIP_OK(hipEventRecord(e1, st));
    HIP_OK(hipEventSynchronize(e1));
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    b2b.push_back(ms * 1e3 / 32);
  }

  struct Alone {
    std::vector<double> event, enqueue, wall;
  };
  auto alone = [&](double idle_ms) {
    Alone a;
    for (int k = 0; k < calls; ++k) {
      HIP_OK(hipStreamSynchronize(st));
      if (idle_ms > 0) std::this_thread::sleep_for(std::chrono::microseconds((long)(idle_ms * 1e3)));
      const auto t0 = clk::now();
      HIP_OK(hipEventRecord(e0, st));
      const auto t1 = clk::now();
      call();
      const auto t2 = clk::now();
      HIP_OK(hipEventRecord(e1, st));
      HIP_OK(hipEventSynchronize(e1));
      const auto t3 = clk::now();
      float ms = 0;
      HIP_OK(hipEventElapsedTime(&ms, e0, e1));
      a.event.push_back(ms * 1e3);
      a.enqueue.push_back(us(t1, t2));
      a.wall.push_back(us(t0, t3));
    }
    return a;
  };
  const Alone hot = alone(0.0), idle = alone(5.0);

  std::vector<uint32_t> bits(n_words);
  HIP_OK(hipMemcpy(bits.data(), d_bits, n_words * 4, hipMemcpyDeviceToHost));
  size_t accepted = 0;
  for (size_t i = 0; i < n; ++i) accepted += (bits[i / 32] >> (i % 32)) & 1u;

  std::printf(
      "{\"caller\": \"C++ through the C ABI (tools/native_latency.cpp)\", \"txs\": %u, \"inputs\": %zu, "
      "\"accepted\": %zu, \"back_to_back_us\": %.1f, \"back_to_back_reps\": [%.1f, %.1f, %.1f], "
      "\"alone\": {\"event_latency_us\": %.1f, \"host_enqueue_us\": %.1f, \"host_wall_us\": %.1f}, "
      "\"alone_after_5ms_idle\": {\"event_latency_us\": %.1f, \"host_enqueue_us\": %.1f, \"host_wall_us\": %.1f}, "
      "\"calls\": %d, \"note\": \"medians; event latency = HIP events on the call's stream around one call; host "
      "wall = before the first event to the second event's completion seen on the host\"}\n",
      n_tx, n, accepted, median(b2b), b2b[0], b2b[1], b2b[2], median(hot.event), median(hot.enqueue), median(hot.wall),
      median(idle.event), median(idle.enqueue), median(idle.wall), calls);
  HIP_OK(hipEventDestroy(e0));
  HIP_OK(hipEventDestroy(e1));
  HIP_OK(hipStreamDestroy(st));
  (void)hipFree(d_txs);
  (void)hipFree(d_offs);
  (void)hipFree(d_pool);
  (void)hipFree(d_jobs);
  (void)hipFree(d_recs);
  (void)hipFree(d_bits);
  hkv_close(ctx);
  return accepted == n ? 0 : 3;
}
