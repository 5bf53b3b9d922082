// Overlapping callers on one context from C++ threads, through the C ABI only
// (the host runtime's lock and stream logic, hkv_api.cpp), built three ways by
// haskoin-node_amd/csrc/Makefile: plain, and with the host code of libhkv and
// of this driver under AddressSanitizer (+ UBSan) or ThreadSanitizer
// (`-Xarch_host -fsanitize=...`; the GPU code is not instrumented).
//
//   python3 tools/native_latency.py dump gpurun_out/blk0 config0
//   python3 tools/native_latency.py dump gpurun_out/blk2 config2
//   python3 tools/native_latency.py dump gpurun_out/blkm multisig
//   tools/native_concurrency gpurun_out/blk0 gpurun_out/blk2 gpurun_out/blkm [threads] [rounds]
//
// Each block's verdict words are first taken from one call of the host form
// (hkv_verify_std_inputs) with nothing else running, and a generated record
// batch's from hkv_verify_host. Then `threads` threads each run `rounds`
// calls, choosing per call among: the host form of a block, the device form
// of a block on the thread's own stream (hkv_verify_std_inputs_device_status,
// its own record / verdict / status buffers), hkv_verify_host on the records,
// hkv_verify_device on the records in HBM on its own stream, and
// hkv_device_fault. Every call's verdict words must equal the reference's and
// no status word may report a fault. Prints one JSON line; exit 0 iff clean.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "../include/hkv.h"

static std::vector<uint8_t> slurp(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) {
    std::fprintf(stderr, "native_concurrency: cannot read %s\n", path.c_str());
    std::exit(2);
  }
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

#define HIP_OK(x)                                                                      \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "native_concurrency: %s: %s\n", #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

struct Block {
  std::vector<uint8_t> txs, offs, pool, jobs;
  uint32_t n_tx = 0;
  size_t n = 0;
  hkv_txs host{};                // host pointers (the host form)
  uint8_t *d_txs = nullptr, *d_pool = nullptr;
  uint32_t* d_offs = nullptr;
  hkv_input_job* d_jobs = nullptr;
  hkv_txs dev{};                 // device pointers (the device form)
  std::vector<uint32_t> want;    // reference verdict words
  size_t words() const { return (n + 63) / 64 * 2; }
};

static void load(Block& b, const std::string& dir) {
  b.txs = slurp(dir + "/txs.bin");
  b.offs = slurp(dir + "/offsets.bin");
  b.pool = slurp(dir + "/scripts.bin");
  b.jobs = slurp(dir + "/jobs.bin");
  if (b.offs.size() < 8 || b.offs.size() % 4 || b.jobs.size() % sizeof(hkv_input_job)) {
    std::fprintf(stderr, "native_concurrency: malformed block files in %s\n", dir.c_str());
    std::exit(2);
  }
  b.n_tx = (uint32_t)(b.offs.size() / 4 - 1);
  b.n = b.jobs.size() / sizeof(hkv_input_job);
  b.host = hkv_txs{b.txs.data(), reinterpret_cast<const uint32_t*>(b.offs.data()), b.n_tx, b.pool.data(),
                   (uint32_t)b.pool.size()};
  HIP_OK(hipMalloc(&b.d_txs, b.txs.size()));
  HIP_OK(hipMalloc(&b.d_offs, b.offs.size()));
  HIP_OK(hipMalloc(&b.d_pool, std::max<size_t>(b.pool.size(), 1)));
  HIP_OK(hipMalloc(&b.d_jobs, b.jobs.size()));
  HIP_OK(hipMemcpy(b.d_txs, b.txs.data(), b.txs.size(), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(b.d_offs, b.offs.data(), b.offs.size(), hipMemcpyHostToDevice));
  if (!b.pool.empty()) HIP_OK(hipMemcpy(b.d_pool, b.pool.data(), b.pool.size(), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(b.d_jobs, b.jobs.data(), b.jobs.size(), hipMemcpyHostToDevice));
  b.dev = hkv_txs{b.d_txs, b.d_offs, b.n_tx, b.d_pool, (uint32_t)b.pool.size()};
}

static bool same(const std::vector<uint32_t>& got, const std::vector<uint32_t>& want, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (((got[i / 32] ^ want[i / 32]) >> (i % 32)) & 1u) return false;
  return true;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: native_concurrency <blk0> <blk2> <blkm> [threads] [rounds]\n");
    return 2;
  }
  const int threads = argc > 4 ? std::atoi(argv[4]) : 6;
  const int rounds = argc > 5 ? std::atoi(argv[5]) : 40;
  const int dev_id = 0;
  hkv_ctx* ctx = nullptr;
  int rc = hkv_open_devices(&dev_id, 1, HKV_OPEN_NO_SELFCHECK, &ctx);
  if (rc != HKV_OK) {
    std::fprintf(stderr, "native_concurrency: hkv_open_devices: %s\n", hkv_strerror(rc));
    return 1;
  }
  HIP_OK(hipSetDevice(0));
  std::vector<Block> blocks(3);
  for (int k = 0; k < 3; ++k) load(blocks[k], argv[1 + k]);
  for (Block& b : blocks) {
    b.want.assign(b.words(), 0);
    rc = hkv_verify_std_inputs(ctx, &b.host, reinterpret_cast<const hkv_input_job*>(b.jobs.data()), b.n, -1,
                               b.want.data());
    if (rc != HKV_OK) {
      std::fprintf(stderr, "native_concurrency: reference hkv_verify_std_inputs: %s\n", hkv_strerror(rc));
      return 1;
    }
  }
  // a generated record batch (5 % invalid) for the record entry points
  const size_t nr = 20000;
  uint8_t* d_recs0;
  uint32_t* d_lab;
  HIP_OK(hipMalloc(&d_recs0, nr * 168));
  HIP_OK(hipMalloc(&d_lab, (nr + 63) / 64 * 8));
  rc = hkv_gen_batch_device(ctx, 0, 0x484B5646ull, 0, nr, 4096, 100, 50, d_recs0, d_lab, nullptr);
  HIP_OK(hipDeviceSynchronize());
  if (rc != HKV_OK) {
    std::fprintf(stderr, "native_concurrency: hkv_gen_batch_device: %s\n", hkv_strerror(rc));
    return 1;
  }
  std::vector<uint8_t> recs(nr * 168);
  HIP_OK(hipMemcpy(recs.data(), d_recs0, recs.size(), hipMemcpyDeviceToHost));
  std::vector<uint32_t> want_r((nr + 31) / 32, 0);
  rc = hkv_verify_host(ctx, recs.data(), nr, 1, want_r.data());
  if (rc != HKV_OK) return 1;

  std::atomic<long> calls{0}, mismatches{0}, errors{0}, faults{0};
  auto worker = [&](int tid) {
    HIP_OK(hipSetDevice(0));
    hipStream_t st;
    HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    size_t most = 0;
    for (const Block& b : blocks) most = std::max(most, b.n);
    uint8_t* d_recs;
    uint32_t *d_bits, *d_status;
    HIP_OK(hipMalloc(&d_recs, std::max(most, nr) * 168));
    HIP_OK(hipMalloc(&d_bits, (std::max(most, nr) + 63) / 64 * 8));
    HIP_OK(hipMalloc(&d_status, 4));
    std::vector<uint32_t> got;
    uint64_t s = 0x9E3779B97F4A7C15ull * (uint64_t)(tid + 1);
    for (int r = 0; r < rounds; ++r) {
      s ^= s << 13;
      s ^= s >> 7;
      s ^= s << 17;
      const int op = (int)(s % 5), bk = (int)((s >> 8) % 3);
      const Block& b = blocks[bk];
      int e = HKV_OK;
      bool ok = true;
      switch (op) {
        case 0: {  // host form of a block
          got.assign(b.words(), 0);
          e = hkv_verify_std_inputs(ctx, &b.host, reinterpret_cast<const hkv_input_job*>(b.jobs.data()), b.n, -1,
                                    got.data());
          ok = e == HKV_OK && same(got, b.want, b.n);
          break;
        }
        case 1: {  // device form of a block on this thread's stream, with a status word
          HIP_OK(hipMemsetAsync(d_bits, 0, b.words() * 4, st));
          HIP_OK(hipMemsetAsync(d_status, 0, 4, st));
          e = hkv_verify_std_inputs_device_status(ctx, 0, &b.dev, b.d_jobs, b.n, -1, d_recs, d_bits, d_status, st);
          got.assign(b.words(), 0);
          uint32_t status = 0;
          HIP_OK(hipMemcpyAsync(got.data(), d_bits, b.words() * 4, hipMemcpyDeviceToHost, st));
          HIP_OK(hipMemcpyAsync(&status, d_status, 4, hipMemcpyDeviceToHost, st));
          HIP_OK(hipStreamSynchronize(st));
          if (status) faults++;
          ok = e == HKV_OK && status == 0 && same(got, b.want, b.n);
          break;
        }
        case 2: {  // host records
          got.assign(want_r.size(), 0);
          e = hkv_verify_host(ctx, recs.data(), nr, 1, got.data());
          ok = e == HKV_OK && same(got, want_r, nr);
          break;
        }
        case 3: {  // device records on this thread's stream
          HIP_OK(hipMemcpyAsync(d_recs, d_recs0, nr * 168, hipMemcpyDeviceToDevice, st));
          e = hkv_verify_device(ctx, 0, d_recs, nr, 1, d_bits, st);
          got.assign((nr + 63) / 64 * 2, 0);
          HIP_OK(hipMemcpyAsync(got.data(), d_bits, got.size() * 4, hipMemcpyDeviceToHost, st));
          HIP_OK(hipStreamSynchronize(st));
          ok = e == HKV_OK && same(got, want_r, nr);
          break;
        }
        default: {  // the fault latch (read and clear; must stay clean)
          uint32_t f = 0;
          e = hkv_device_fault(ctx, 0, &f);
          if (f) faults++;
          ok = e == HKV_OK && f == 0;
          break;
        }
      }
      calls++;
      if (e != HKV_OK) errors++;
      else if (!ok) mismatches++;
    }
    HIP_OK(hipStreamSynchronize(st));
    HIP_OK(hipStreamDestroy(st));
    (void)hipFree(d_recs);
    (void)hipFree(d_bits);
    (void)hipFree(d_status);
  };
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) pool.emplace_back(worker, t);
  for (auto& t : pool) t.join();
  for (Block& b : blocks) {
    (void)hipFree(b.d_txs);
    (void)hipFree(b.d_offs);
    (void)hipFree(b.d_pool);
    (void)hipFree(b.d_jobs);
  }
  (void)hipFree(d_recs0);
  (void)hipFree(d_lab);
  hkv_close(ctx);
  size_t acc[3] = {0, 0, 0};
  for (int k = 0; k < 3; ++k)
    for (size_t i = 0; i < blocks[k].n; ++i) acc[k] += (blocks[k].want[i / 32] >> (i % 32)) & 1u;
  std::printf(
      "{\"driver\": \"tools/native_concurrency.cpp\", \"threads\": %d, \"rounds\": %d, \"calls\": %ld, "
      "\"mismatches\": %ld, \"errors\": %ld, \"faults\": %ld, \"block_inputs\": [%zu, %zu, %zu], "
      "\"block_accepts\": [%zu, %zu, %zu], \"records\": %zu}\n",
      threads, rounds, calls.load(), mismatches.load(), errors.load(), faults.load(), blocks[0].n, blocks[1].n,
      blocks[2].n, acc[0], acc[1], acc[2], nr);
  return (mismatches.load() || errors.load() || faults.load()) ? 3 : 0;
}
