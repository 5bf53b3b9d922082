// hkv_api.cpp — the C ABI (include/hkv.h) over the HIP kernels.
//
// One hkv_ctx per process; per device: a stream, the fixed-base G tables,
// the per-lane Q-table scratch sized for one full-occupancy ecmult grid, and
// growable intermediate / bitmap / record-staging buffers. hkv_verify shards
// contiguous 64-aligned index ranges over the devices, overlaps their H2D /
// kernels / D2H on per-device streams and joins. No exceptions cross the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/hkv.h"
#include "hkv_internal.h"
#include "hkv_layout.h"
#include "hkv_plan.h"

#ifndef HKV_BLOCK_ROWS  // the block kernel builds its inputs' tx index rows (0: an index launch first)
#define HKV_BLOCK_ROWS 1
#endif
#ifndef HKV_STD_OVERLAP
#define HKV_STD_OVERLAP 1
#endif

namespace {

thread_local std::string g_last_hip;

// the clock probe: 4 clock counters, 12 phase stamps, then a (start, end)
// stamp pair per workgroup of the block kernel (hkv_profile_group_stamps)
constexpr size_t CLK_GROUPS = 4096, CLK_WORDS = 16 + 2 * CLK_GROUPS;

struct DevCtx {
  int device = -1;
  int n_cu = 0;
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;  // H2D of host batches, overlapped with verify
  // the hash half of a large standard-input batch runs here beside the
  // ECDSA kernels (enqueue_std_chunk), forked from and joined back into the
  // caller's stream by these two events
  hipStream_t hash_stream = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  uint32_t* gtab = nullptr;
  uint32_t* qs = nullptr;
  uint32_t grid_max = 0;  // ecmult blocks (qs is sized for grid_max * WG lanes)
  uint32_t* im = nullptr;
  size_t im_cap = 0;      // n_pad capacity
  uint32_t* bits = nullptr;
  size_t bits_cap = 0;    // words
  uint8_t* recs = nullptr;
  size_t recs_cap = 0;    // records
  uint32_t* hbits = nullptr;  // pinned D2H staging
  size_t hbits_cap = 0;
  uint32_t* pool = nullptr;
  uint32_t pool_n = 0;
  uint64_t pool_seed = ~0ull;
  // tx index rows (hkv_sighash.hip) and host-API staging buffers
  uint32_t* txt = nullptr;
  size_t txt_cap = 0;  // bytes
  // [0..3] tx batch, [4] sighash out, [5] header batch, [6] spare
  void* stage[7] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  size_t stage_cap[7] = {0, 0, 0, 0, 0, 0, 0};
  // multisig inputs (hkv_sighash.hip section 4, hkv_kernels.hip 2e): [0] desc
  // words, [2] offsets, [3] candidate verdict words, [4] candidate + key
  // records, [5] key-check verdict words, [6] host-form verdict words
  void* ms[7] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  size_t ms_cap[7] = {0, 0, 0, 0, 0, 0, 0};
  uint32_t ms_win_cand = 0, ms_win_keys = 0;  // record-window overrides (hkv_debug_ms_window; 0 = default)
  size_t std_chunk = 0;  // verify-std-inputs chunk past one resident grid (init_device; enqueue_verify_std_inputs)
  void* ms_ctr = nullptr;            // scan sums: [epoch & 1] this call's (its tail launch zeroes the other)
  // the tail's words: [0..7] and [8..15] the two work-queue slots (claim,
  // completed items; launch `tail_epoch` uses slot tail_epoch & 1 and zeroes
  // the other), [16] the sticky fault latch (hkv_device_fault), [17] the host
  // form's per-call status word
  unsigned int* ms_bar = nullptr;
  uint32_t tail_epoch = 0;
  bool inject_tail = false;          // hkv_debug_fail_device(HKV_FAIL_TAIL): the next tail's phase waits give up
  uint32_t* call_status = nullptr;   // the current call's status word (device; HKV_STATUS_* ORed in), or null
  bool ms_dirty = false;             // a call failed after its scan launch: zero ms_ctr before the next scan
  uint32_t* rare_ctr = nullptr;      // y-free rare-lane count (hkv_finish_kernel appends, hkv_yverdict_kernel re-arms)
  bool rare_dirty = false;           // a finish launch failed part-way: zero rare_ctr before the next one
  // split launches: waves 4-5's A = u1 G, y0 and flags for the in-kernel join
  uint32_t* aux = nullptr;
  size_t aux_n = 0;                  // signatures aux holds
  // optional per-kernel timing (hkv_profile_*): events on the launch stream
  bool profile = false;
  std::vector<hipEvent_t> ev;  // triples: before prologue, between, after ecmult
  unsigned long long* clk = nullptr;  // ecmult clock probe (4 counters) + split-kernel phase stamps (12)
  int wall_khz = 0;                   // constant-rate counter frequency
  // The scratch above (im, bits, qs, txt, pool, staging) is shared by every
  // call on this device whatever stream it names: each call waits for the
  // previous user's work (this event) before enqueueing and records it after,
  // so calls on different streams run in enqueue order instead of racing.
  hipEvent_t last_use = nullptr;
  uint32_t inject = 0;  // hkv_debug_fail_device: HKV_FAIL_* of this device's next host-batch shard
};

}  // namespace

struct hkv_ctx {
  std::vector<DevCtx> devs;
  // mu: every entry point's host-side state (DevCtx fields, allocations,
  // enqueue order). tx_mu[k]: the tx-index rows, the multisig scratch and
  // the tx staging of device k — held by the sighash / std-input entry
  // points for their whole call, taken BEFORE mu. No entry point waits on
  // the device while it holds either (the device forms only enqueue).
  std::mutex mu;
  std::vector<std::unique_ptr<std::mutex>> tx_mu;
  // host-batch failover (verify_from_host): devices still in use, and how
  // many shards each has failed
  std::vector<bool> healthy;
  std::vector<uint32_t> failures;
};
struct hkv_batch {
  hkv_ctx* ctx = nullptr;
  uint8_t* host = nullptr;
  size_t cap = 0;
};

namespace {

int hip_fail(hipError_t e, const char* what) {
  g_last_hip = std::string(what) + ": " + hipGetErrorString(e);
  return HKV_E_HIP;
}
// an allocation (or other resource) failure: the call's error, not a fault of
// the device (hkv_plan.h is_device_fault: it does not make failover re-shard)
int oom_fail(hipError_t e, const char* what) {
  g_last_hip = std::string(what) + ": " + hipGetErrorString(e);
  return HKV_E_OOM;
}
#define HKV_TRY(expr, what)                       \
  do {                                            \
    hipError_t e_ = (expr);                       \
    if (e_ != hipSuccess) return hip_fail(e_, what); \
  } while (0)

size_t round_up(size_t a, size_t b) { return (a + b - 1) / b * b; }

// split (small-batch) launches when n_pad <= resident grid / HKV_SPLIT_DIV
#ifndef HKV_SPLIT_DIV
#define HKV_SPLIT_DIV 8
#endif

// verify-std-inputs batches run in chunks (enqueue_verify_std_inputs). The
// multisig verdict bits of a chunk are sized by the host bound (136 candidate
// and 16 key-check records per input: 16-of-16), so the device never reports
// a count the host must read first (the scan's 32-bit candidate sum cannot
// wrap); the 168-B records themselves live in two windows capped at
// MS_WIN_CAND + MS_WIN_KEYS records (~512 MiB), through
// which the tail kernel runs the chunk's records in rounds
// A batch of at most one resident grid runs in half-grid chunks (131,072
// inputs on an MI355X: the overlapped mid-size form, hash half beside the Q
// chains); a larger batch in chunks of up to std_chunk inputs (default 2^20;
// env HKV_STD_CHUNK at open, for tests) through the full-grid instance:
// extraction, then the record verify at 4 waves per SIMD. (Round 6: 1,007,894
// inputs in 128k chunks took 15.96 ms, 63 M inputs/s, profiles/r06y/.)
#ifndef HKV_STD_CHUNK
#define HKV_STD_CHUNK (1u << 20)
#endif
constexpr size_t MS_CAND_PER_INPUT = 136, MS_KEYS_PER_INPUT = 16;
#ifndef HKV_MS_WIN_CAND
#define HKV_MS_WIN_CAND 2752512u  // 43,008 x 64 candidate records (441 MiB)
#endif
#ifndef HKV_MS_WIN_KEYS
#define HKV_MS_WIN_KEYS 442368u   // 6,912 x 64 key-check records (71 MiB)
#endif
constexpr size_t HKV_MAX_STD_INPUTS = 0xFFFFFF00ull;
constexpr size_t MS_BAR_WORDS = 32, MS_FAULT = 16, MS_HOST_STATUS = 17;  // DevCtx::ms_bar
#ifndef HKV_HOST_FIRST_DIV  // the host-batch path's first chunk: one resident grid / this
#define HKV_HOST_FIRST_DIV 4
#endif
#ifndef HKV_HOST_MAX_GRIDS  // the host-batch path's largest chunk, in resident grids
#define HKV_HOST_MAX_GRIDS 8
#endif

int ensure_dev_buffers(DevCtx& d, size_t n_pad) {
  if (d.im_cap < n_pad) {
    if (d.im) (void)hipFree(d.im);
    d.im = nullptr;
    d.im_cap = 0;
    HKV_TRY(hipMalloc(&d.im, n_pad * hkv::IM_WORDS * sizeof(uint32_t)), "hipMalloc(intermediate)");
    d.im_cap = n_pad;
  }
  const size_t words = n_pad / 32;
  if (d.bits_cap < words) {
    if (d.bits) (void)hipFree(d.bits);
    d.bits = nullptr;
    d.bits_cap = 0;
    HKV_TRY(hipMalloc(&d.bits, words * sizeof(uint32_t)), "hipMalloc(bits)");
    d.bits_cap = words;
  }
  return HKV_OK;
}

// Order a call on stream st after the previous user of the device's scratch
// (acquire) and publish st as the new last user (release). Callers hold ctx->mu.
// The wait is taken on every call, whatever stream the last release used: a
// stream handle equal to the last one does not prove the same stream
// (hipStreamPerThread maps to a different stream per thread, and a destroyed
// stream's handle can be reused), and skipping it measured within noise
// (profiles/r05c/ab_skip_wait.txt).
int scratch_acquire(DevCtx& d, hipStream_t st) {
  HKV_TRY(hipStreamWaitEvent(st, d.last_use, 0), "hipStreamWaitEvent(scratch)");
  return HKV_OK;
}
int scratch_release(DevCtx& d, hipStream_t st) {
  HKV_TRY(hipEventRecord(d.last_use, st), "hipEventRecord(scratch)");
  return HKV_OK;
}

// the split kernels' A = u1 G, y0 and flags for the join (hkv_layout.h AUX_*)
int ensure_aux(DevCtx& d, size_t n_pad, hipStream_t st) {
  if (d.aux_n >= n_pad) return HKV_OK;
  if (d.aux) {
    HKV_TRY(hipStreamSynchronize(st), "aux sync");
    (void)hipFree(d.aux);
    d.aux = nullptr;
    d.aux_n = 0;
  }
  HKV_TRY(hipMalloc(&d.aux, n_pad * hkv::AUX_WORDS * sizeof(uint32_t)), "hipMalloc(aux)");
  d.aux_n = n_pad;
  return HKV_OK;
}

// whether a batch of n runs the small-batch (split) kernels
bool split_batch(const DevCtx& d, size_t n) {
  return round_up(n, hkv::WG) <= (size_t)d.grid_max * hkv::WG / HKV_SPLIT_DIV;
}

// whether a full-grid batch of n runs the 2-wave (mid-size) instance
bool mid_batch(const DevCtx& d, size_t n) {
  return !split_batch(d, n) && round_up(n, hkv::WG) <= (size_t)d.grid_max * hkv::WG / 2;
}

// enqueue the verify of n records at d_records; verdict words in out_bits
// ((n + 31) / 32 words, device memory) or, when null, in d.bits.
// late_join (full-grid batches of standard inputs only): the event after
// which the records carry their final messages — st waits for it after the
// ecmult launch, then the finish kernel redoes u1 from them (LATE).
// std_pro (mid-size standard-input batches, enqueue_std_chunk): the signature
// and key come from the batch's txs through the lane prologue at the head of
// the ecmult kernel instead of from records
int enqueue_verify(DevCtx& d, const void* d_records, size_t n, uint32_t mode, hipStream_t st,
                   uint32_t* out_bits = nullptr, hipEvent_t late_join = nullptr,
                   const hkv::StdOps* std_pro = nullptr) {
  const size_t n_pad = round_up(n, hkv::WG);
  int rc = ensure_dev_buffers(d, n_pad);
  if (rc) return rc;
  hipEvent_t e[3] = {nullptr, nullptr, nullptr};
  if (d.profile) {
    for (auto& x : e) HKV_TRY(hipEventCreate(&x), "hipEventCreate");
    HKV_TRY(hipEventRecord(e[0], st), "hipEventRecord");
  }
  // A batch of at most half a wave per SIMD (an eighth of the resident grid)
  // runs the small-batch kernel (hkv_pair_split_kernel: k1 and k2 chains on
  // their own waves, two lanes per chain, the signature and square-root waves
  // beside them, no separate prologue): a shorter dependency chain where
  // latency, not issue, bounds the launch.
  // Above that the duplicated doublings cost more than the chain saves
  // (measured: a 115k batch at ~1.8 waves/SIMD took 2.1 ms split vs 1.5 ms
  // unsplit; the bound itself re-measured in profiles/r02_split_threshold.log).
  const bool split = split_batch(d, n);
  // at most 2 waves per SIMD (half the 4-wave resident grid): the paired-form
  // ecmult instance, every block resident at its 2-wave allocation. (Record
  // batches keep the three prologue kernels here: the lane-per-signature form
  // measured 87 against their 75 us on a 115k batch, profiles/r04f; it pays
  // only inside the overlapped standard-input path.)
  const bool mid = mid_batch(d, n);
  if (std_pro != nullptr && !mid) return HKV_E_INTERNAL;  // (the lane prologue is a mid-size form)
  if (!split && std_pro == nullptr)
    HKV_TRY(hkv::launch_prologue(d_records, (uint32_t)n, (uint32_t)n_pad, mode, d.im, st), "prologue launch");
  if (split) {
    rc = ensure_aux(d, n_pad, st);
    if (rc) return rc;
  }
  if (d.profile) HKV_TRY(hipEventRecord(e[1], st), "hipEventRecord");
  const uint32_t blocks = split ? 0u  // (the small-batch launch sizes its own grid)
                                : (uint32_t)std::min<size_t>(n_pad / hkv::WG, mid ? d.grid_max / 2 : d.grid_max);
  uint32_t* vbits = out_bits ? out_bits : d.bits;
  const uint32_t n_words = (uint32_t)(out_bits ? (n + 31) / 32 : n_pad / 32);
  if (std_pro != nullptr)
    HKV_TRY(hkv::launch_std_ecmult_mid(*std_pro, d.im, (uint32_t)n, (uint32_t)n_pad, d.qs, blocks,
                                       d.profile ? d.clk : nullptr, st),
            "ecmult launch");
  else
    HKV_TRY(hkv::launch_ecmult(d.im, (uint32_t)n, (uint32_t)n_pad, d.gtab, d.qs, blocks, vbits, n_words, split, mid,
                               d.profile ? d.clk : nullptr, d.aux, d_records, mode, (uint32_t)d.n_cu, st),
            "ecmult launch");
  // full-grid batches: the finish kernels add u1 * G and decide x(R) == r
  // through y_c = num / den (hkv_kernels.hip §2b). The rare-lane count is
  // re-armed by the verdict kernel; a call that failed between the finish
  // and verdict launches leaves it dirty, so it is zeroed on the stream first.
  if (late_join != nullptr && !split)
    HKV_TRY(hipStreamWaitEvent(st, late_join, 0), "hipStreamWaitEvent(hash join)");
  if (!split) {
    if (d.rare_dirty) {
      HKV_TRY(hipMemsetAsync(d.rare_ctr, 0, sizeof(uint32_t), st), "hipMemset(rare counter)");
      d.rare_dirty = false;
    }
    const hipError_t e2 = hkv::launch_finish(d.im, (uint32_t)n, (uint32_t)n_pad, d.gtab, d.rare_ctr, vbits, n_words, mid,
                                                 late_join != nullptr ? d_records : nullptr, st);
    if (e2 != hipSuccess) {
      d.rare_dirty = true;
      return hip_fail(e2, "finish launch");
    }
  }
  if (d.profile) {
    HKV_TRY(hipEventRecord(e[2], st), "hipEventRecord");
    d.ev.insert(d.ev.end(), e, e + 3);
  }
  return HKV_OK;
}

int init_device(DevCtx& d, int device) {
  d.device = device;
  HKV_TRY(hipSetDevice(device), "hipSetDevice");
  hipDeviceProp_t prop;
  HKV_TRY(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    g_last_hip = std::string("device is ") + prop.gcnArchName + ", libhkv is built for gfx950 only";
    return HKV_E_NODEV;
  }
  d.n_cu = prop.multiProcessorCount;
  HKV_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking), "hipStreamCreate");
  HKV_TRY(hipStreamCreateWithFlags(&d.copy_stream, hipStreamNonBlocking), "hipStreamCreate(copy)");
  HKV_TRY(hipStreamCreateWithFlags(&d.hash_stream, hipStreamNonBlocking), "hipStreamCreate(hash)");
  HKV_TRY(hipEventCreateWithFlags(&d.ev_fork, hipEventDisableTiming), "hipEventCreate(fork)");
  HKV_TRY(hipEventCreateWithFlags(&d.ev_join, hipEventDisableTiming), "hipEventCreate(join)");
  HKV_TRY(hipEventCreateWithFlags(&d.last_use, hipEventDisableTiming), "hipEventCreate(scratch)");
  HKV_TRY(hipEventRecord(d.last_use, d.stream), "hipEventRecord(scratch)");
  // the multisig scan's two parity sums; the tail's queue words
  HKV_TRY(hipMalloc(&d.ms_ctr, 4 * sizeof(uint64_t)), "hipMalloc(multisig counters)");
  HKV_TRY(hipMemsetAsync(d.ms_ctr, 0, 4 * sizeof(uint64_t), d.stream), "hipMemset(multisig counters)");
  HKV_TRY(hipMalloc(reinterpret_cast<void**>(&d.ms_bar), MS_BAR_WORDS * sizeof(unsigned int)), "hipMalloc(multisig barrier)");
  HKV_TRY(hipMemsetAsync(d.ms_bar, 0, MS_BAR_WORDS * sizeof(unsigned int), d.stream), "hipMemset(multisig barrier)");
  HKV_TRY(hipMalloc(&d.rare_ctr, sizeof(uint32_t)), "hipMalloc(rare counter)");
  HKV_TRY(hipMemsetAsync(d.rare_ctr, 0, sizeof(uint32_t), d.stream), "hipMemset(rare counter)");
  HKV_TRY(hipStreamSynchronize(d.stream), "multisig counters sync");  // callers may use other streams
  HKV_TRY(hipDeviceGetAttribute(&d.wall_khz, hipDeviceAttributeWallClockRate, device), "wall clock rate");
  HKV_TRY(hipMalloc(&d.clk, CLK_WORDS * sizeof(unsigned long long)), "hipMalloc(clock probe)");
  HKV_TRY(hipMemsetAsync(d.clk, 0, CLK_WORDS * sizeof(unsigned long long), d.stream), "hipMemset(clock probe)");
  HKV_TRY(hipMalloc(&d.gtab, hkv::GTAB_DWORDS * sizeof(uint32_t)), "hipMalloc(gtab)");  // 448 MiB at radix 2^20
  int per_cu = 0;
  HKV_TRY(hkv::ecmult_max_blocks_per_cu(&per_cu), "occupancy query");
  if (per_cu < 1) per_cu = 1;
  d.grid_max = (uint32_t)(d.n_cu * per_cu);
  // test hook: a smaller (or larger) chunk past one grid; a multiple of 64,
  // at most 2^24 (the scan's 32-bit candidate sum: 136 per input)
  d.std_chunk = HKV_STD_CHUNK;
  if (const char* e = std::getenv("HKV_STD_CHUNK")) {
    const unsigned long long c = std::strtoull(e, nullptr, 10) / 64 * 64;
    if (c >= 64 && c <= (1ull << 24)) d.std_chunk = (size_t)c;
  }
  const size_t lanes = (size_t)d.grid_max * hkv::WG;
  HKV_TRY(hipMalloc(&d.qs, lanes * hkv::QTAB_QUADS * 16), "hipMalloc(qtab scratch)");
  HKV_TRY(hkv::launch_gtable(d.gtab, d.stream), "gtable launch");
  HKV_TRY(hipStreamSynchronize(d.stream), "gtable sync");
  return HKV_OK;
}

void clear_events(DevCtx& d) {
  for (auto e : d.ev) (void)hipEventDestroy(e);
  d.ev.clear();
}

void free_device(DevCtx& d) {
  if (d.device < 0) return;
  (void)hipSetDevice(d.device);
  if (d.stream) (void)hipStreamSynchronize(d.stream);
  (void)hipDeviceSynchronize();
  clear_events(d);
  if (d.gtab) (void)hipFree(d.gtab);
  if (d.qs) (void)hipFree(d.qs);
  if (d.im) (void)hipFree(d.im);
  if (d.bits) (void)hipFree(d.bits);
  if (d.recs) (void)hipFree(d.recs);
  if (d.pool) (void)hipFree(d.pool);
  if (d.txt) (void)hipFree(d.txt);
  for (auto p : d.stage)
    if (p) (void)hipFree(p);
  for (auto p : d.ms)
    if (p) (void)hipFree(p);
  if (d.ms_ctr) (void)hipFree(d.ms_ctr);
  if (d.ms_bar) (void)hipFree(d.ms_bar);
  if (d.rare_ctr) (void)hipFree(d.rare_ctr);
  if (d.aux) (void)hipFree(d.aux);
  if (d.hbits) (void)hipHostFree(d.hbits);
  if (d.clk) (void)hipFree(d.clk);
  if (d.last_use) (void)hipEventDestroy(d.last_use);
  if (d.stream) (void)hipStreamDestroy(d.stream);
  if (d.copy_stream) (void)hipStreamDestroy(d.copy_stream);
  if (d.hash_stream) (void)hipStreamDestroy(d.hash_stream);
  if (d.ev_fork) (void)hipEventDestroy(d.ev_fork);
  if (d.ev_join) (void)hipEventDestroy(d.ev_join);
  d = DevCtx();
}

int ensure_pool(DevCtx& d, uint64_t seed, uint32_t pool_n, hipStream_t st) {
  if (d.pool && d.pool_n == pool_n && d.pool_seed == seed) return HKV_OK;
  if (d.pool) (void)hipFree(d.pool);
  d.pool = nullptr;
  HKV_TRY(hipMalloc(&d.pool, (size_t)pool_n * 16 * sizeof(uint32_t)), "hipMalloc(pool)");
  HKV_TRY(hkv::launch_gen_pool(seed, pool_n, d.pool, st), "gen pool launch");
  d.pool_n = pool_n;
  d.pool_seed = seed;
  return HKV_OK;
}

// Self-check at open: 256 generated valid records must all verify.
int self_check(DevCtx& d) {
  const size_t n = 256;
  uint8_t* recs = nullptr;
  HKV_TRY(hipMalloc(&recs, n * hkv::REC_SIZE), "hipMalloc(selfcheck)");
  int rc = scratch_acquire(d, d.stream);
  if (!rc) rc = ensure_pool(d, 0x484B5630ull, 16, d.stream);
  if (!rc) {
    hipError_t e = hkv::launch_gen_records(0x484B5630ull, 0, (uint32_t)n, d.pool, d.pool_n, 250, 0, recs, nullptr,
                                           d.stream);
    if (e != hipSuccess) rc = hip_fail(e, "selfcheck gen");
  }
  if (!rc) rc = enqueue_verify(d, recs, n, HKV_MODE_LIBSECP, d.stream);
  uint32_t words[8] = {0};
  if (!rc) {
    hipError_t e = hipMemcpyAsync(words, d.bits, sizeof(words), hipMemcpyDeviceToHost, d.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(d.stream);
    if (e != hipSuccess) rc = hip_fail(e, "selfcheck copy");
  }
  if (!rc) rc = scratch_release(d, d.stream);
  (void)hipFree(recs);
  if (rc) return rc;
  for (uint32_t w : words)
    if (w != 0xFFFFFFFFu) {
      g_last_hip = "self-check: generated valid signatures did not verify";
      return HKV_E_INTERNAL;
    }
  return HKV_OK;
}

// ---- signature hashes / standard inputs ------------------------------------

int grow(void** p, size_t* cap, size_t bytes, const char* what) {
  if (*cap >= bytes && *p) return HKV_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  HKV_TRY(hipMalloc(p, bytes ? bytes : 16), what);
  *cap = bytes;
  return HKV_OK;
}

bool txs_ok(const hkv_txs* t) {
  return t && (t->n_tx == 0 || (t->bytes && t->offsets)) && (t->scripts || t->scripts_len == 0) &&
         t->n_tx < 0xFFFFFF00u;
}

// the tx index rows, with the BIP143 per-tx hashes of the txs that may need
// them (hkv::TX_HASHES_*: none — the fused small-batch std-input launch
// computes them per input —, every tx — the sighash API, whose jobs choose
// the BIP143 form freely —, or, for standard inputs, what the network allows)
int enqueue_tx_index(DevCtx& d, const hkv_txs* dt, hipStream_t st, uint32_t hashes = hkv::TX_HASHES_ALL) {
  int rc = grow(reinterpret_cast<void**>(&d.txt), &d.txt_cap, (size_t)dt->n_tx * hkv::TXT_WORDS * 4, "hipMalloc(txt)");
  if (rc) return rc;
  HKV_TRY(hkv::launch_tx_index(dt->bytes, dt->offsets, dt->n_tx, hashes, d.txt, st), "tx index launch");
  return HKV_OK;
}
// verifyStdInput signs with BIP143 only for witness programs (then the tx
// carries witness data, or the input fails) unless a fork id is in force,
// where every FORKID-flagged signature does
uint32_t std_tx_hashes(int32_t forkid) { return forkid >= 0 ? hkv::TX_HASHES_ALL : hkv::TX_HASHES_WITNESS; }

int enqueue_std_inputs(DevCtx& d, const hkv_txs* dt, const hkv_input_job* jobs, size_t n, int32_t forkid,
                       void* recs, hipStream_t st) {
  int rc = enqueue_tx_index(d, dt, st, std_tx_hashes(forkid));
  if (rc) return rc;
  HKV_TRY(hkv::launch_std_inputs(dt->bytes, dt->n_tx, d.txt, dt->scripts, dt->scripts_len, jobs, (uint32_t)n, forkid,
                                 static_cast<uint8_t*>(recs), st),
          "std input launch");
  return HKV_OK;
}

// Small batches of standard inputs in one verify launch (hkv_pair_split_kernel
// <true>): the chains start from the parsed keys and signatures while the
// signature wave computes the sighashes and script checks beside them.
int enqueue_std_verify_split(DevCtx& d, const hkv_txs* dt, const hkv_input_job* jobs, size_t n, int32_t forkid,
                             void* recs, uint32_t* out_bits, const hkv::MsScan* ms, const uint32_t* tx_off,
                             hipStream_t st) {
  const size_t n_pad = round_up(n, hkv::WG);
  int rc = ensure_dev_buffers(d, n_pad);
  if (!rc) rc = ensure_aux(d, n_pad, st);
  if (rc) return rc;
  hipEvent_t e[3] = {nullptr, nullptr, nullptr};
  if (d.profile) {
    for (auto& x : e) HKV_TRY(hipEventCreate(&x), "hipEventCreate");
    HKV_TRY(hipEventRecord(e[0], st), "hipEventRecord");
    HKV_TRY(hipEventRecord(e[1], st), "hipEventRecord");
  }
  HKV_TRY(hkv::launch_std_verify_split(dt->bytes, dt->n_tx, d.txt, dt->scripts, dt->scripts_len, jobs, (uint32_t)n,
                                       (uint32_t)n_pad, forkid, static_cast<uint8_t*>(recs), d.im, d.gtab, d.qs,
                                       d.aux, out_bits, (uint32_t)((n + 31) / 32), d.profile ? d.clk : nullptr,
                                       (uint32_t)d.n_cu, ms, tx_off, st),
          "std-input verify launch");
  if (d.profile) {
    HKV_TRY(hipEventRecord(e[2], st), "hipEventRecord");
    d.ev.insert(d.ev.end(), e, e + 3);
  }
  return HKV_OK;
}

// Full verifyStdInput over one chunk of jobs (enqueue_verify_std_inputs), verdict bit i
// -> out_bits (device), all enqueued on st (nothing waits on the host).
// Single-signature templates: one record per input (recs) through the verify
// kernels — small batches in one fused launch (tx index, then the block or
// pair kernel with the parse, the hashes and the script checks inside),
// larger ones the extraction kernel then the record verify. Multisig (bare /
// P2SH / P2WSH / P2SH-P2WSH): the scan (inside the block kernel, or
// hkv_ms_scan_kernel) leaves the batch total on the device and the tail
// kernel (hkv_kernels.hip 2e) does the rest, or nothing when the total is 0.
int enqueue_std_rest(DevCtx& d, const hkv_txs* dt, const hkv_input_job* jobs, size_t n, int32_t forkid, void* recs,
                     uint32_t* out_bits, hipStream_t st, bool fused, bool fused_scan, bool overlap,
                     const hkv::MsScan& ms, size_t cap_cand, size_t cap_keys);
// the multisig tail's operands for this call (launch epoch d.tail_epoch)
hkv::MsTail tail_args(DevCtx& d, const hkv_txs* dt, const hkv_input_job* jobs, size_t n, int32_t forkid,
                      uint32_t* out_bits, bool fused, const hkv::MsScan& ms, size_t cap_cand, size_t cap_keys) {
  uint8_t* cand = static_cast<uint8_t*>(d.ms[4]);
  uint64_t* ctr = static_cast<uint64_t*>(d.ms_ctr);
  hkv::MsTail t;
  t.win_cand = (uint32_t)cap_cand;
  t.win_keys = (uint32_t)cap_keys;
  t.txs = dt->bytes;
  t.tx_off = dt->offsets;
  t.n_tx = dt->n_tx;
  t.txt = d.txt;
  t.scripts = dt->scripts;
  t.scripts_len = dt->scripts_len;
  t.jobs = jobs;
  t.n = (uint32_t)n;
  t.forkid = forkid;
  // the fused launch's index hashed nothing: the multisig sighashes need the
  // BIP143 per-tx hashes the network allows (the extraction path built them)
  t.hash_txs = fused ? std_tx_hashes(forkid) : hkv::TX_HASHES_NONE;
  t.desc = ms.desc;
  t.off = ms.off;
  t.total = reinterpret_cast<unsigned long long*>(ms.counters);
  t.total_next = reinterpret_cast<unsigned long long*>(ctr + ((d.tail_epoch + 1u) & 1u));
  t.cand = cand;
  t.keyrec = cand + cap_cand * hkv::REC_SIZE;
  t.cbits = static_cast<uint32_t*>(d.ms[3]);
  t.kbits = static_cast<uint32_t*>(d.ms[5]);
  t.im = d.im;
  t.aux = d.aux;
  t.gtab = d.gtab;
  t.qs = d.qs;
  t.out_bits = out_bits;
  t.bar = d.ms_bar;
  t.epoch = d.tail_epoch;
  t.fault = d.ms_bar + MS_FAULT;
  t.status = d.call_status;
  t.force_fault = d.inject_tail ? 1u : 0u;
  return t;
}
int enqueue_std_chunk(DevCtx& d, const hkv_txs* dt, const hkv_input_job* jobs, size_t n, int32_t forkid, void* recs,
                      uint32_t* out_bits, hipStream_t st) {
  const bool fused = split_batch(d, n);
  // the block kernel (at most 16 inputs per CU) runs the multisig scan on
  // its signature wave; otherwise the scan kernel follows the verify launch
  const bool fused_scan = fused && hkv::std_split_scans((uint32_t)round_up(n, hkv::WG), (uint32_t)d.n_cu);
  const size_t all_cand = n * MS_CAND_PER_INPUT, all_keys = n * MS_KEYS_PER_INPUT;
  // the record windows: the whole bound when it fits the budget (one round),
  // else the budget (hkv_debug_ms_window can shrink both for tests)
  const size_t win_c = d.ms_win_cand ? d.ms_win_cand : HKV_MS_WIN_CAND;
  const size_t win_k = d.ms_win_keys ? d.ms_win_keys : HKV_MS_WIN_KEYS;
  const size_t cap_cand = round_up(std::min(all_cand, win_c), 64), cap_keys = round_up(std::min(all_keys, win_k), 64);
  const size_t slots = hkv::ms_tail_slots((uint32_t)d.n_cu);
  int rc = grow(&d.ms[0], &d.ms_cap[0], n * 8, "hipMalloc(multisig desc)");
  if (!rc) rc = grow(&d.ms[2], &d.ms_cap[2], n * 8, "hipMalloc(multisig offsets)");
  if (!rc) rc = grow(&d.ms[3], &d.ms_cap[3], round_up(all_cand, 64) / 8, "hipMalloc(multisig candidate bits)");
  // (the key window starts right after this call's candidate window)
  if (!rc) rc = grow(&d.ms[4], &d.ms_cap[4], (cap_cand + cap_keys) * hkv::REC_SIZE, "hipMalloc(multisig records)");
  if (!rc) rc = grow(&d.ms[5], &d.ms_cap[5], round_up(all_keys, 64) / 8, "hipMalloc(multisig key bits)");
  // the tail's candidate groups use slot-relative pair-form scratch (grid * 32 signatures)
  if (!rc) rc = ensure_dev_buffers(d, std::max(round_up(n, hkv::WG), round_up(slots, hkv::WG)));
  if (!rc) rc = ensure_aux(d, std::max(round_up(n, hkv::WG), round_up(slots, hkv::WG)), st);
  if (rc) return rc;
  uint32_t* desc = static_cast<uint32_t*>(d.ms[0]);
  uint64_t* off = static_cast<uint64_t*>(d.ms[2]);
  if (d.ms_dirty) {  // an earlier call failed after its scan launch: counters may be stale
    HKV_TRY(hipMemsetAsync(d.ms_ctr, 0, 2 * sizeof(uint64_t), st), "hipMemset(multisig counters)");
    d.ms_dirty = false;
  }
  d.ms_dirty = true;  // until this call's tail is enqueued
  // this call's scan sum: the parity word of its tail epoch (the launch that
  // runs the tail zeroes the other one for the next call)
  uint64_t* ctr = static_cast<uint64_t*>(d.ms_ctr) + (d.tail_epoch & 1u);
  const hkv::MsScan ms{desc, off, ctr};
  // Larger batches (HKV_STD_OVERLAP): the index rows on st, then the hash
  // half (BIP143 per-tx hashes, the script checks and the sighashes, writing
  // each record whole; the multisig scan) on the hash stream while st runs
  // the parse half, the prologue and the Q chains, which need only r, s and
  // the key — at mid size all inside the ecmult launch (kernel 1e); st joins
  // before the finish, which takes u1 from the final records (LATE).
  // (mid size: every chunk past the pair kernel's bound on an MI355X, where
  // the 131,072-input chunk is exactly the 2-wave grid)
  const bool overlap = !fused && HKV_STD_OVERLAP && mid_batch(d, n);
  bool forked = false;
  if (fused) {
    // the block kernel (fused_scan) builds the rows of its inputs' txs itself
    // (kernel 2d txc_fill): no index launch before it
    const bool rows = fused_scan && HKV_BLOCK_ROWS;
    if (rows)
      rc = grow(reinterpret_cast<void**>(&d.txt), &d.txt_cap, (size_t)dt->n_tx * hkv::TXT_WORDS * 4, "hipMalloc(txt)");
    else
      rc = enqueue_tx_index(d, dt, st, hkv::TX_HASHES_NONE);
    if (!rc)
      rc = enqueue_std_verify_split(d, dt, jobs, n, forkid, recs, out_bits, fused_scan ? &ms : nullptr,
                                    rows ? dt->offsets : nullptr, st);
  } else if (overlap) {
    rc = enqueue_tx_index(d, dt, st, hkv::TX_HASHES_NONE);
    if (rc) return rc;
    // (the parse half runs inside the ecmult launch's lane prologue, which
    // writes no record — the hash half writes each record whole — so the
    // fork comes right after the index rows)
    HKV_TRY(hipEventRecord(d.ev_fork, st), "hipEventRecord(fork)");
    HKV_TRY(hipStreamWaitEvent(d.hash_stream, d.ev_fork, 0), "hipStreamWaitEvent(fork)");
    forked = true;
    hipError_t e = hkv::launch_tx_hashes_only(dt->bytes, dt->offsets, dt->n_tx, std_tx_hashes(forkid), d.txt,
                                              d.hash_stream);
    if (e == hipSuccess)
      e = hkv::launch_std_inputs(dt->bytes, dt->n_tx, d.txt, dt->scripts, dt->scripts_len, jobs, (uint32_t)n, forkid,
                                 static_cast<uint8_t*>(recs), d.hash_stream);
    // the multisig scan needs only the index rows: off st's path too
    if (e == hipSuccess && !fused_scan)
      e = hkv::launch_ms_scan(dt->bytes, dt->n_tx, d.txt, dt->scripts, dt->scripts_len, jobs, (uint32_t)n, forkid,
                              desc, off, ctr, d.hash_stream);
    // (recorded whatever happened: an error below still joins st to it)
    const hipError_t e2 = hipEventRecord(d.ev_join, d.hash_stream);
    if (e != hipSuccess) rc = hip_fail(e, "std hash half launch");
    else if (e2 != hipSuccess) rc = hip_fail(e2, "hipEventRecord(join)");
  } else {
    rc = enqueue_std_inputs(d, dt, jobs, n, forkid, recs, st);
  }
  if (!rc)
    rc = enqueue_std_rest(d, dt, jobs, n, forkid, recs, out_bits, st, fused, fused_scan, overlap, ms, cap_cand,
                          cap_keys);
  // a failed call still orders st after the hash half (the next call's
  // scratch acquire then waits for it too)
  if (rc && forked) (void)hipStreamWaitEvent(st, d.ev_join, 0);
  if (!rc) d.ms_dirty = false;
  return rc;
}

// the rest of enqueue_std_chunk after the extraction launches: the
// multisig scan, the record verify, the multisig tail
int enqueue_std_rest(DevCtx& d, const hkv_txs* dt, const hkv_input_job* jobs, size_t n, int32_t forkid, void* recs,
                     uint32_t* out_bits, hipStream_t st, bool fused, bool fused_scan, bool overlap,
                     const hkv::MsScan& ms, size_t cap_cand, size_t cap_keys) {
  int rc = HKV_OK;
  if (!fused_scan && !overlap)  // (the overlapped form scanned on the hash stream)
    HKV_TRY(hkv::launch_ms_scan(dt->bytes, dt->n_tx, d.txt, dt->scripts, dt->scripts_len, jobs, (uint32_t)n, forkid,
                                ms.desc, ms.off, ms.counters, st),
            "multisig scan launch");
  if (!fused) {
    const hkv::StdOps so{dt->bytes, dt->n_tx, d.txt, dt->scripts, dt->scripts_len, jobs, forkid};
    rc = enqueue_verify(d, recs, n, HKV_MODE_HASKOIN, st, out_bits, overlap ? d.ev_join : nullptr,
                        overlap ? &so : nullptr);
    if (rc) return rc;
  }
  // (operands taken after every launch before it has sized the scratch)
  // (one workgroup per CU on every path: the tail's scratch slots are sized
  // by n_cu, hkv_internal.h launch_ms_tail; a smaller grid for block-sized
  // batches measured no different, profiles/r05k/tail_grid_ab.txt)
  const uint32_t tail_grid = (uint32_t)d.n_cu;
  HKV_TRY(hkv::launch_ms_tail(tail_args(d, dt, jobs, n, forkid, out_bits, fused, ms, cap_cand, cap_keys), tail_grid,
                              st),
          "multisig tail launch");
  ++d.tail_epoch;  // (launched: it zeroes the slot and the scan sum the next call uses)
  d.inject_tail = false;
  return HKV_OK;
}

int enqueue_verify_std_inputs(DevCtx& d, const hkv_txs* dt, const hkv_input_job* jobs, size_t n, int32_t forkid,
                              void* recs, uint32_t* out_bits, hipStream_t st) {
  const size_t grid_lanes = (size_t)d.grid_max * hkv::WG;
  const size_t chunk = n > grid_lanes ? d.std_chunk : grid_lanes / 2;
  for (size_t lo = 0; lo < n; lo += chunk) {
    const size_t cn = std::min(chunk, n - lo);
    const int rc = enqueue_std_chunk(d, dt, jobs + lo, cn, forkid, static_cast<uint8_t*>(recs) + lo * hkv::REC_SIZE,
                                     out_bits + lo / 32, st);
    if (rc) return rc;
  }
  return HKV_OK;
}

// copy a host tx batch (+ jobs) into the device's staging buffers
int stage_txs(DevCtx& d, const hkv_txs* h, const void* jobs, size_t job_bytes, hkv_txs* dt, void** djobs) {
  const size_t nbytes = h->n_tx ? h->offsets[h->n_tx] : 0;
  const size_t noff = ((size_t)h->n_tx + 1) * 4;
  int rc = grow(&d.stage[0], &d.stage_cap[0], nbytes, "hipMalloc(tx bytes)");
  if (!rc) rc = grow(&d.stage[1], &d.stage_cap[1], noff, "hipMalloc(tx offsets)");
  if (!rc) rc = grow(&d.stage[2], &d.stage_cap[2], h->scripts_len, "hipMalloc(scripts)");
  if (!rc) rc = grow(&d.stage[3], &d.stage_cap[3], job_bytes, "hipMalloc(jobs)");
  if (rc) return rc;
  if (nbytes) HKV_TRY(hipMemcpyAsync(d.stage[0], h->bytes, nbytes, hipMemcpyHostToDevice, d.stream), "H2D txs");
  if (h->n_tx) HKV_TRY(hipMemcpyAsync(d.stage[1], h->offsets, noff, hipMemcpyHostToDevice, d.stream), "H2D offsets");
  if (h->scripts_len)
    HKV_TRY(hipMemcpyAsync(d.stage[2], h->scripts, h->scripts_len, hipMemcpyHostToDevice, d.stream), "H2D scripts");
  if (job_bytes) HKV_TRY(hipMemcpyAsync(d.stage[3], jobs, job_bytes, hipMemcpyHostToDevice, d.stream), "H2D jobs");
  dt->bytes = static_cast<const uint8_t*>(d.stage[0]);
  dt->offsets = static_cast<const uint32_t*>(d.stage[1]);
  dt->n_tx = h->n_tx;
  dt->scripts = static_cast<const uint8_t*>(d.stage[2]);
  dt->scripts_len = h->scripts_len;
  *djobs = d.stage[3];
  return HKV_OK;
}

}  // namespace

extern "C" {

uint32_t hkv_version(void) { return (1u << 16) | 0u; }

const char* hkv_strerror(int err) {
  switch (err) {
    case HKV_OK: return "ok";
    case HKV_E_ARG: return "invalid argument";
    case HKV_E_NODEV: return "no usable gfx950 device";
    case HKV_E_OOM: return "out of memory";
    case HKV_E_HIP: return "HIP runtime error";
    case HKV_E_INTERNAL: return "internal self-check failed";
    default: return "unknown error";
  }
}
const char* hkv_last_hip_error(void) { return g_last_hip.c_str(); }

int hkv_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int hkv_open_devices(const int* device_ids, int n_ids, uint32_t flags, hkv_ctx** out) {
  if (!out || n_ids <= 0 || !device_ids) return HKV_E_ARG;
  *out = nullptr;
  hkv_ctx* ctx = new (std::nothrow) hkv_ctx();
  if (!ctx) return HKV_E_OOM;
  ctx->devs.resize(n_ids);
  ctx->healthy.assign(n_ids, true);
  ctx->failures.assign(n_ids, 0);
  for (int k = 0; k < n_ids; ++k) ctx->tx_mu.emplace_back(new (std::nothrow) std::mutex());
  for (auto& m : ctx->tx_mu)
    if (!m) {
      delete ctx;
      return HKV_E_OOM;
    }
  for (int k = 0; k < n_ids; ++k) {
    int rc = init_device(ctx->devs[k], device_ids[k]);
    if (!rc && !(flags & HKV_OPEN_NO_SELFCHECK)) rc = self_check(ctx->devs[k]);
    if (rc) {
      for (auto& d : ctx->devs) free_device(d);
      delete ctx;
      return rc;
    }
  }
  *out = ctx;
  return HKV_OK;
}

int hkv_open(int n_gpus, uint32_t flags, hkv_ctx** out) {
  if (!out) return HKV_E_ARG;
  int avail = hkv_device_count();
  if (avail <= 0) return HKV_E_NODEV;
  if (n_gpus <= 0 || n_gpus > avail) n_gpus = avail;
  std::vector<int> ids(n_gpus);
  for (int k = 0; k < n_gpus; ++k) ids[k] = k;
  return hkv_open_devices(ids.data(), n_gpus, flags, out);
}

void hkv_close(hkv_ctx* ctx) {
  if (!ctx) return;
  for (auto& d : ctx->devs) free_device(d);
  delete ctx;
}

int hkv_ctx_num_devices(const hkv_ctx* ctx) { return ctx ? (int)ctx->devs.size() : 0; }

int hkv_device_healthy(hkv_ctx* ctx, int dev) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return HKV_E_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  return ctx->healthy[(size_t)dev] ? 1 : 0;
}

int hkv_device_reset_health(hkv_ctx* ctx, int dev) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return HKV_E_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  ctx->healthy[(size_t)dev] = true;
  return HKV_OK;
}

int hkv_device_failures(hkv_ctx* ctx, int dev) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return HKV_E_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  return (int)ctx->failures[(size_t)dev];
}

int hkv_debug_fail_device(hkv_ctx* ctx, int dev, uint32_t when) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || when > HKV_FAIL_TAIL) return HKV_E_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (when == HKV_FAIL_TAIL) ctx->devs[(size_t)dev].inject_tail = true;
  else ctx->devs[(size_t)dev].inject = when;
  return HKV_OK;
}

int hkv_debug_ms_window(hkv_ctx* ctx, int dev, uint32_t cand_records, uint32_t key_records) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || cand_records > HKV_MS_WIN_CAND ||
      key_records > HKV_MS_WIN_KEYS)
    return HKV_E_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  DevCtx& d = ctx->devs[(size_t)dev];
  d.ms_win_cand = (uint32_t)round_up(cand_records, 64);
  d.ms_win_keys = (uint32_t)round_up(key_records, 64);
  return HKV_OK;
}

int hkv_debug_ms_scratch(hkv_ctx* ctx, int dev, size_t* bytes) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !bytes) return HKV_E_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  *bytes = ctx->devs[(size_t)dev].ms_cap[4];
  return HKV_OK;
}

int hkv_device_fault(hkv_ctx* ctx, int dev, uint32_t* fault) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !fault) return HKV_E_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  DevCtx& d = ctx->devs[(size_t)dev];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  // after every call enqueued so far on this device (the scratch order), read
  // then clear the latch
  unsigned int w = 0;
  int rc = scratch_acquire(d, d.stream);
  if (rc) return rc;
  HKV_TRY(hipMemcpyAsync(&w, d.ms_bar + MS_FAULT, sizeof(w), hipMemcpyDeviceToHost, d.stream), "D2H fault latch");
  HKV_TRY(hipMemsetAsync(d.ms_bar + MS_FAULT, 0, sizeof(unsigned int), d.stream), "hipMemset(fault latch)");
  HKV_TRY(hipStreamSynchronize(d.stream), "fault latch sync");
  *fault = w ? HKV_STATUS_TAIL_FAULT : 0u;
  return scratch_release(d, d.stream);
}

int hkv_batch_alloc(hkv_ctx* ctx, size_t max_n, hkv_batch** out) {
  if (!ctx || !out || max_n == 0) return HKV_E_ARG;
  hkv_batch* b = new (std::nothrow) hkv_batch();
  if (!b) return HKV_E_OOM;
  if (hipHostMalloc(reinterpret_cast<void**>(&b->host), max_n * hkv::REC_SIZE, hipHostMallocPortable) !=
      hipSuccess) {
    delete b;
    return HKV_E_OOM;
  }
  std::memset(b->host, 0, max_n * hkv::REC_SIZE);
  b->ctx = ctx;
  b->cap = max_n;
  *out = b;
  return HKV_OK;
}
void hkv_batch_free(hkv_batch* b) {
  if (!b) return;
  if (b->host) (void)hipHostFree(b->host);
  delete b;
}
uint8_t* hkv_batch_records(hkv_batch* b) { return b ? b->host : nullptr; }
size_t hkv_batch_capacity(const hkv_batch* b) { return b ? b->cap : 0; }

// Stop using a device whose shard failed: wait (best effort) for its copy and
// verify streams, whose async H2D copies still read the caller's host records
// and whose kernels still write d.hbits.
static void quiesce(DevCtx& d) {
  (void)hipSetDevice(d.device);
  (void)hipStreamSynchronize(d.copy_stream);
  (void)hipStreamSynchronize(d.stream);
}

// One shard of a host batch on its device: H2D of the records pipelined with
// the verify in chunks of whole resident grids (the copy stream moves chunk
// c+1 over PCIe while the verify stream works on chunk c; an event orders each
// verify after its own H2D), each chunk's verdict words to the pinned staging
// right after its verify, before d.bits is reused. (One H2D then one verify
// measured 15.84 ms against 13.09 ms pipelined for 1M records:
// profiles/r01_bench_hostpath*.log.)
static int enqueue_host_shard(DevCtx& d, const uint8_t* host, const hkv::Shard& s, uint32_t mode,
                              std::vector<hipEvent_t>& evs) {
  if (d.inject == HKV_FAIL_ENQUEUE) {
    d.inject = 0;
    g_last_hip = "injected enqueue failure (hkv_debug_fail_device)";
    return HKV_E_HIP;
  }
  if (d.inject == HKV_FAIL_ALLOC) {
    d.inject = 0;
    return oom_fail(hipErrorOutOfMemory, "injected allocation failure (hkv_debug_fail_device)");
  }
  const size_t len = s.hi - s.lo;
  hipError_t e0 = hipSetDevice(d.device);
  int rc = e0 == hipSuccess ? scratch_acquire(d, d.stream) : hip_fail(e0, "hipSetDevice");
  if (!rc) rc = scratch_acquire(d, d.copy_stream);
  if (!rc && d.recs_cap < len) {
    if (d.recs) (void)hipFree(d.recs);
    d.recs = nullptr;
    d.recs_cap = 0;
    e0 = hipMalloc(&d.recs, len * hkv::REC_SIZE);
    if (e0 != hipSuccess) rc = oom_fail(e0, "hipMalloc(records)");
    else d.recs_cap = len;
  }
  const size_t words = (len + 31) / 32;
  if (!rc && d.hbits_cap < words) {
    if (d.hbits) (void)hipHostFree(d.hbits);
    d.hbits = nullptr;
    d.hbits_cap = 0;
    e0 = hipHostMalloc(reinterpret_cast<void**>(&d.hbits), words * 4, hipHostMallocPortable);
    if (e0 != hipSuccess) rc = oom_fail(e0, "hipHostMalloc(bits)");
    else d.hbits_cap = words;
  }
  if (rc) return rc;
  // Chunk schedule: the first chunk is a quarter of a resident grid (its H2D
  // is the only copy no verify hides), then one grid, then each chunk twice
  // the one before (PCIe moves ~2.8x the records per second the verify does,
  // so the copy of chunk c+1 still ends before the verify of chunk c), in
  // whole grids; a remainder under one grid joins the chunk before it.
  // (Same-box A/B, profiles/r05z/: 1M records 9.84 / 9.97 ms against 10.58
  // with a one-grid first chunk and 10.75 / 10.69 with an eighth; one
  // quarter of the shard per chunk, the earlier schedule, exposed a
  // quarter-shard H2D before the first verify: 16M 161 ms, now 146 ms.)
  // Growth stops at HKV_HOST_MAX_GRIDS grids (a chunk of 8 grids verifies
  // for ~18 ms, far above a launch's cost), and the intermediate buffers are
  // sized once for the schedule's largest chunk before the first copy: a
  // buffer grown inside the loop would hipFree (a device-wide sync) between
  // chunks and lose the overlap.
  const size_t grid_lanes = (size_t)d.grid_max * hkv::WG;
  const uint8_t* src = host + s.lo * hkv::REC_SIZE;
  const size_t first = len >= 2 * grid_lanes ? grid_lanes / HKV_HOST_FIRST_DIV : len;
  auto step = [&](size_t off, size_t& next) {
    size_t cl = std::min(next, len - off);
    if (len - off - cl < grid_lanes) cl = len - off;
    next = std::min(std::max(2 * next, grid_lanes), (size_t)HKV_HOST_MAX_GRIDS * grid_lanes);
    return cl;
  };
  size_t largest = 0;
  for (size_t off = 0, next = first, cl = 0; off < len; off += cl) largest = std::max(largest, cl = step(off, next));
  rc = ensure_dev_buffers(d, round_up(largest, hkv::WG));
  size_t next = first;
  for (size_t off = 0, cl = 0; off < len && !rc; off += cl) {
    cl = step(off, next);
    hipEvent_t ev = nullptr;
    hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) {
      rc = oom_fail(e, "hipEventCreate");
      break;
    }
    evs.push_back(ev);
    if (e == hipSuccess)
      e = hipMemcpyAsync(d.recs + off * hkv::REC_SIZE, src + off * hkv::REC_SIZE, cl * hkv::REC_SIZE,
                         hipMemcpyHostToDevice, d.copy_stream);
    if (e == hipSuccess) e = hipEventRecord(ev, d.copy_stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(d.stream, ev, 0);
    if (e != hipSuccess) {
      rc = hip_fail(e, "H2D records");
      break;
    }
    rc = enqueue_verify(d, d.recs + off * hkv::REC_SIZE, cl, mode, d.stream);
    if (!rc) {
      e = hipMemcpyAsync(d.hbits + off / 32, d.bits, (cl + 31) / 32 * 4, hipMemcpyDeviceToHost, d.stream);
      if (e != hipSuccess) rc = hip_fail(e, "D2H bits");
    }
  }
  // the copy stream must not run ahead into the next call's H2D while this
  // call's verify still reads d.recs: it is ordered through last_use
  if (!rc) rc = scratch_release(d, d.stream);
  if (!rc) rc = scratch_acquire(d, d.copy_stream);
  return rc;
}

static int join_host_shard(DevCtx& d, const hkv::Shard& s, uint32_t* out, size_t out_words) {
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  HKV_TRY(hipStreamSynchronize(d.stream), "verify sync");
  if (d.inject == HKV_FAIL_JOIN) {
    d.inject = 0;
    g_last_hip = "injected join failure (hkv_debug_fail_device)";
    return HKV_E_HIP;
  }
  if (!hkv::merge_shard_words(out, out_words, d.hbits, s)) {
    g_last_hip = "shard does not fit the verdict bitmap";
    return HKV_E_INTERNAL;
  }
  return HKV_OK;
}

// Host batch over the context's healthy devices: contiguous 64-aligned
// shards (hkv_plan.h), and on a device failure its shard is re-verified on
// the devices still healthy (the failed device is left out of every later
// call of the context: hkv_device_healthy). Blocking.
static int verify_from_host(hkv_ctx* ctx, const uint8_t* host, size_t n, uint32_t mode, uint32_t* out) {
  if (!ctx || !host || !out || mode > HKV_MODE_HASKOIN) return HKV_E_ARG;
  if (n == 0) return HKV_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);
  std::vector<std::vector<hipEvent_t>> evs(ctx->devs.size());
  struct EventGuard {  // destroyed after every join (or on an early return)
    std::vector<std::vector<hipEvent_t>>& e;
    ~EventGuard() {
      for (auto& v : e)
        for (auto ev : v) (void)hipEventDestroy(ev);
    }
  } guard{evs};
  const size_t out_words = (n + 31) / 32;
  return hkv::run_with_failover(
      n, ctx->healthy,
      [&](const hkv::Shard& s) { return enqueue_host_shard(ctx->devs[(size_t)s.dev], host, s, mode, evs[(size_t)s.dev]); },
      [&](const hkv::Shard& s) { return join_host_shard(ctx->devs[(size_t)s.dev], s, out, out_words); },
      [&](int dev, int) {
        quiesce(ctx->devs[(size_t)dev]);
        ++ctx->failures[(size_t)dev];
      });
}

int hkv_verify(hkv_ctx* ctx, hkv_batch* b, size_t n, uint32_t mode, uint32_t* verdict_bits) {
  if (!b || n > b->cap) return HKV_E_ARG;
  return verify_from_host(ctx, b->host, n, mode, verdict_bits);
}

int hkv_verify_host(hkv_ctx* ctx, const uint8_t* records, size_t n, uint32_t mode, uint32_t* verdict_bits) {
  return verify_from_host(ctx, records, n, mode, verdict_bits);
}

int hkv_verify_device(hkv_ctx* ctx, int dev, const void* d_records, size_t n, uint32_t mode, uint32_t* d_bits,
                      void* hip_stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !d_records || !d_bits || mode > HKV_MODE_HASKOIN)
    return HKV_E_ARG;
  if (n == 0) return HKV_OK;
  if (n > 0xFFFFFF00ull) return HKV_E_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  DevCtx& d = ctx->devs[dev];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  hipStream_t st = static_cast<hipStream_t>(hip_stream);  // NULL: the null (default) stream (include/hkv.h)
  int rc = scratch_acquire(d, st);
  if (!rc) rc = enqueue_verify(d, d_records, n, mode, st, d_bits);
  if (rc) return rc;
  return scratch_release(d, st);
}

int hkv_gen_batch_device(hkv_ctx* ctx, int dev, uint64_t seed, uint64_t index0, size_t n, uint32_t pool_size,
                         uint32_t uncompressed_permille, uint32_t invalid_permille, void* d_records,
                         uint32_t* d_labels, void* hip_stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !d_records || pool_size == 0 ||
      uncompressed_permille > 1000 || invalid_permille > 1000 || n > 0xFFFFFF00ull || index0 > ~0ull - n)
    return HKV_E_ARG;
  if (n == 0) return HKV_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);
  DevCtx& d = ctx->devs[dev];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  hipStream_t st = static_cast<hipStream_t>(hip_stream);  // NULL: the null (default) stream (include/hkv.h)
  int rc = scratch_acquire(d, st);
  // the key pool depends on the batch seed only: every rank of a sharded
  // batch builds the same pool
  if (!rc) rc = ensure_pool(d, seed ^ 0x706F6F6Cull, pool_size, st);
  if (rc) return rc;
  HKV_TRY(hkv::launch_gen_records(seed, index0, (uint32_t)n, d.pool, d.pool_n, uncompressed_permille,
                                  invalid_permille, d_records, d_labels, st),
          "gen records launch");
  return scratch_release(d, st);
}

int hkv_gen_records_device(hkv_ctx* ctx, int dev, uint64_t seed, size_t n, uint32_t pool_size,
                           uint32_t uncompressed_permille, void* d_records, void* hip_stream) {
  return hkv_gen_batch_device(ctx, dev, seed, 0, n, pool_size, uncompressed_permille, 0, d_records, nullptr,
                              hip_stream);
}

int hkv_debug_op(hkv_ctx* ctx, int dev, uint32_t op, size_t n, const uint32_t* d_a, const uint32_t* d_b,
                 uint32_t* d_out, void* hip_stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !d_a || !d_b || !d_out) return HKV_E_ARG;
  if (n == 0) return HKV_OK;
  DevCtx& d = ctx->devs[dev];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  hipStream_t st = static_cast<hipStream_t>(hip_stream);  // NULL: the null (default) stream (include/hkv.h)
  HKV_TRY(hkv::launch_debug(op, (uint32_t)n, d_a, d_b, d_out, st), "debug launch");
  return HKV_OK;
}

int hkv_profile_enable(hkv_ctx* ctx, int on) {
  if (!ctx) return HKV_E_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  for (auto& d : ctx->devs) {
    (void)hipSetDevice(d.device);
    (void)hipDeviceSynchronize();
    clear_events(d);
    d.profile = on != 0;
  }
  return HKV_OK;
}

int hkv_profile_read(hkv_ctx* ctx, int dev, double* prologue_ms, double* ecmult_ms, uint64_t* launches) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !prologue_ms || !ecmult_ms || !launches)
    return HKV_E_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  DevCtx& d = ctx->devs[dev];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  double p = 0, m = 0;
  for (size_t k = 0; k + 2 < d.ev.size(); k += 3) {
    HKV_TRY(hipEventSynchronize(d.ev[k + 2]), "hipEventSynchronize");
    float a = 0, b = 0;
    HKV_TRY(hipEventElapsedTime(&a, d.ev[k], d.ev[k + 1]), "hipEventElapsedTime");
    HKV_TRY(hipEventElapsedTime(&b, d.ev[k + 1], d.ev[k + 2]), "hipEventElapsedTime");
    p += a;
    m += b;
  }
  *prologue_ms = p;
  *ecmult_ms = m;
  *launches = d.ev.size() / 3;
  clear_events(d);
  return HKV_OK;
}

int hkv_profile_clock(hkv_ctx* ctx, int dev, double* sclk_mhz) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !sclk_mhz) return HKV_E_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  DevCtx& d = ctx->devs[dev];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  HKV_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
  unsigned long long c[4] = {0, 0, 0, 0};
  HKV_TRY(hipMemcpy(c, d.clk, sizeof(c), hipMemcpyDeviceToHost), "D2H clock probe");
  *sclk_mhz = 0;
  if (c[3] > c[1] && d.wall_khz > 0) *sclk_mhz = (double)(c[2] - c[0]) / ((double)(c[3] - c[1]) / (d.wall_khz * 1e-3));
  return HKV_OK;
}

int hkv_profile_phases(hkv_ctx* ctx, int dev, uint64_t* stamps, size_t n, double* tick_ns) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !stamps || !tick_ns || n > 12) return HKV_E_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  DevCtx& d = ctx->devs[dev];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  HKV_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
  if (n) HKV_TRY(hipMemcpy(stamps, d.clk + 4, n * sizeof(uint64_t), hipMemcpyDeviceToHost), "D2H phase stamps");
  *tick_ns = d.wall_khz > 0 ? 1e6 / d.wall_khz : 0.0;
  return HKV_OK;
}

int hkv_profile_group_stamps(hkv_ctx* ctx, int dev, uint64_t* stamps, size_t n_groups, double* tick_ns) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !stamps || !tick_ns || n_groups > CLK_GROUPS)
    return HKV_E_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  DevCtx& d = ctx->devs[dev];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  HKV_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
  if (n_groups)
    HKV_TRY(hipMemcpy(stamps, d.clk + 16, 2 * n_groups * sizeof(uint64_t), hipMemcpyDeviceToHost), "D2H group stamps");
  *tick_ns = d.wall_khz > 0 ? 1e6 / d.wall_khz : 0.0;
  return HKV_OK;
}

int hkv_sighash_device(hkv_ctx* ctx, int dev, const hkv_txs* d_txs, const hkv_sighash_job* d_jobs, size_t n,
                       int32_t forkid, uint8_t* d_out, size_t out_stride, uint8_t* d_status, void* hip_stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !txs_ok(d_txs) || out_stride < 32 || out_stride % 4 ||
      out_stride > 0xFFFFFFFFu || n > 0xFFFFFF00ull)
    return HKV_E_ARG;
  if (n == 0) return HKV_OK;
  if (!d_jobs || !d_out) return HKV_E_ARG;
  std::lock_guard<std::mutex> txl(*ctx->tx_mu[dev]);
  std::lock_guard<std::mutex> lock(ctx->mu);
  DevCtx& d = ctx->devs[dev];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  hipStream_t st = static_cast<hipStream_t>(hip_stream);  // NULL: the null (default) stream (include/hkv.h)
  int rc = scratch_acquire(d, st);
  if (!rc) rc = enqueue_tx_index(d, d_txs, st);
  if (rc) return rc;
  HKV_TRY(hkv::launch_sighash(d_txs->bytes, d_txs->n_tx, d.txt, d_txs->scripts, d_txs->scripts_len, d_jobs,
                              (uint32_t)n, forkid, d_out, (uint32_t)out_stride, d_status, st),
          "sighash launch");
  return scratch_release(d, st);
}

int hkv_sighash(hkv_ctx* ctx, const hkv_txs* txs, const hkv_sighash_job* jobs, size_t n, int32_t forkid,
                uint8_t* out32, uint8_t* status) {
  if (!ctx || ctx->devs.empty() || !txs_ok(txs) || n > 0xFFFFFF00ull) return HKV_E_ARG;
  if (n == 0) return HKV_OK;
  if (!jobs || !out32) return HKV_E_ARG;
  std::lock_guard<std::mutex> txl(*ctx->tx_mu[0]);
  std::lock_guard<std::mutex> lock(ctx->mu);
  DevCtx& d = ctx->devs[0];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  hkv_txs dt;
  void* djobs = nullptr;
  int rc = scratch_acquire(d, d.stream);
  if (!rc) rc = stage_txs(d, txs, jobs, n * sizeof(hkv_sighash_job), &dt, &djobs);
  if (!rc) rc = grow(&d.stage[4], &d.stage_cap[4], n * 33, "hipMalloc(sighash out)");
  if (!rc) rc = enqueue_tx_index(d, &dt, d.stream);
  if (rc) return rc;
  uint8_t* dout = static_cast<uint8_t*>(d.stage[4]);
  HKV_TRY(hkv::launch_sighash(dt.bytes, dt.n_tx, d.txt, dt.scripts, dt.scripts_len,
                              static_cast<const hkv_sighash_job*>(djobs), (uint32_t)n, forkid, dout, 32, dout + n * 32,
                              d.stream),
          "sighash launch");
  HKV_TRY(hipMemcpyAsync(out32, dout, n * 32, hipMemcpyDeviceToHost, d.stream), "D2H sighash");
  if (status) HKV_TRY(hipMemcpyAsync(status, dout + n * 32, n, hipMemcpyDeviceToHost, d.stream), "D2H status");
  HKV_TRY(hipStreamSynchronize(d.stream), "sighash sync");
  return scratch_release(d, d.stream);
}

int hkv_std_inputs_device(hkv_ctx* ctx, int dev, const hkv_txs* d_txs, const hkv_input_job* d_jobs, size_t n,
                          int32_t forkid, void* d_records, void* hip_stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !txs_ok(d_txs) || n > 0xFFFFFF00ull) return HKV_E_ARG;
  if (n == 0) return HKV_OK;
  if (!d_jobs || !d_records) return HKV_E_ARG;
  std::lock_guard<std::mutex> txl(*ctx->tx_mu[dev]);
  std::lock_guard<std::mutex> lock(ctx->mu);
  DevCtx& d = ctx->devs[dev];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  hipStream_t st = static_cast<hipStream_t>(hip_stream);  // NULL: the null (default) stream (include/hkv.h)
  int rc = scratch_acquire(d, st);
  if (!rc) rc = enqueue_std_inputs(d, d_txs, d_jobs, n, forkid, d_records, st);
  if (!rc) rc = scratch_release(d, st);
  return rc;
}

int hkv_verify_std_inputs_device_status(hkv_ctx* ctx, int dev, const hkv_txs* d_txs, const hkv_input_job* d_jobs,
                                        size_t n, int32_t forkid, void* d_records, uint32_t* d_bits,
                                        uint32_t* d_status, void* hip_stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !txs_ok(d_txs) || n > HKV_MAX_STD_INPUTS) return HKV_E_ARG;
  if (n == 0) return HKV_OK;
  if (!d_jobs || !d_records || !d_bits) return HKV_E_ARG;
  std::lock_guard<std::mutex> txl(*ctx->tx_mu[dev]);
  std::lock_guard<std::mutex> lock(ctx->mu);
  DevCtx& d = ctx->devs[dev];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  hipStream_t st = static_cast<hipStream_t>(hip_stream);  // NULL: the null (default) stream (include/hkv.h)
  int rc = scratch_acquire(d, st);
  d.call_status = d_status;
  if (!rc) rc = enqueue_verify_std_inputs(d, d_txs, d_jobs, n, forkid, d_records, d_bits, st);
  d.call_status = nullptr;
  if (rc) return rc;
  return scratch_release(d, st);
}

int hkv_verify_std_inputs_device(hkv_ctx* ctx, int dev, const hkv_txs* d_txs, const hkv_input_job* d_jobs, size_t n,
                                 int32_t forkid, void* d_records, uint32_t* d_bits, void* hip_stream) {
  return hkv_verify_std_inputs_device_status(ctx, dev, d_txs, d_jobs, n, forkid, d_records, d_bits, nullptr,
                                             hip_stream);
}

int hkv_verify_std_inputs(hkv_ctx* ctx, const hkv_txs* txs, const hkv_input_job* jobs, size_t n, int32_t forkid,
                          uint32_t* verdict_bits) {
  if (!ctx || ctx->devs.empty() || !txs_ok(txs) || n > HKV_MAX_STD_INPUTS) return HKV_E_ARG;
  if (n == 0) return HKV_OK;
  if (!jobs || !verdict_bits) return HKV_E_ARG;
  std::lock_guard<std::mutex> txl(*ctx->tx_mu[0]);
  std::lock_guard<std::mutex> lock(ctx->mu);
  DevCtx& d = ctx->devs[0];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  hkv_txs dt;
  void* djobs = nullptr;
  int rc = scratch_acquire(d, d.stream);
  if (!rc) rc = stage_txs(d, txs, jobs, n * sizeof(hkv_input_job), &dt, &djobs);
  if (!rc && d.recs_cap < n) {
    if (d.recs) (void)hipFree(d.recs);
    d.recs = nullptr;
    d.recs_cap = 0;
    HKV_TRY(hipMalloc(&d.recs, n * hkv::REC_SIZE), "hipMalloc(records)");
    d.recs_cap = n;
  }
  if (!rc) rc = grow(&d.ms[6], &d.ms_cap[6], (n + 31) / 32 * 4, "hipMalloc(verdict words)");
  if (rc) return rc;
  // this call's status word (a fault of an earlier call is not this call's)
  uint32_t* status = reinterpret_cast<uint32_t*>(d.ms_bar + MS_HOST_STATUS);
  HKV_TRY(hipMemsetAsync(status, 0, sizeof(uint32_t), d.stream), "hipMemset(call status)");
  d.call_status = status;
  rc = enqueue_verify_std_inputs(d, &dt, static_cast<const hkv_input_job*>(djobs), n, forkid, d.recs,
                                 static_cast<uint32_t*>(d.ms[6]), d.stream);
  d.call_status = nullptr;
  if (rc) return rc;
  HKV_TRY(hipMemcpyAsync(verdict_bits, d.ms[6], (n + 31) / 32 * 4, hipMemcpyDeviceToHost, d.stream), "D2H bits");
  uint32_t fault = 0;
  HKV_TRY(hipMemcpyAsync(&fault, status, sizeof(fault), hipMemcpyDeviceToHost, d.stream), "D2H call status");
  HKV_TRY(hipStreamSynchronize(d.stream), "std inputs sync");
  if (fault & HKV_STATUS_TAIL_FAULT) {  // a multisig tail queue wait gave up (its verdicts are incomplete)
    g_last_hip = "multisig tail: work-queue wait timed out";
    (void)scratch_release(d, d.stream);
    return HKV_E_INTERNAL;
  }
  return scratch_release(d, d.stream);
}

int hkv_gen_keys_device(hkv_ctx* ctx, int dev, uint64_t seed, size_t n, uint8_t* d_priv, uint8_t* d_pub,
                        uint8_t* d_h160, void* hip_stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || n > 0xFFFFFF00ull) return HKV_E_ARG;
  if (n == 0) return HKV_OK;
  if (!d_priv || !d_pub || !d_h160) return HKV_E_ARG;
  DevCtx& d = ctx->devs[dev];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  hipStream_t st = static_cast<hipStream_t>(hip_stream);  // NULL: the null (default) stream (include/hkv.h)
  HKV_TRY(hkv::launch_gen_keys(seed, (uint32_t)n, d_priv, d_pub, d_h160, st), "gen keys launch");
  return HKV_OK;
}

int hkv_gen_sign_device(hkv_ctx* ctx, int dev, uint64_t seed, size_t n, const uint8_t* d_priv,
                        const uint32_t* d_key_idx, const uint8_t* d_msg, size_t msg_stride, uint8_t* d_sig,
                        void* hip_stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || n > 0xFFFFFF00ull || msg_stride < 32 ||
      msg_stride > 0xFFFFFFFFu)
    return HKV_E_ARG;
  if (n == 0) return HKV_OK;
  if (!d_priv || !d_msg || !d_sig) return HKV_E_ARG;
  DevCtx& d = ctx->devs[dev];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  hipStream_t st = static_cast<hipStream_t>(hip_stream);  // NULL: the null (default) stream (include/hkv.h)
  HKV_TRY(hkv::launch_gen_sign(seed, (uint32_t)n, d_priv, d_key_idx, d_msg, (uint32_t)msg_stride, d_sig, st),
          "gen sign launch");
  return HKV_OK;
}

static bool aligned(const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

int hkv_check_headers_device(hkv_ctx* ctx, int dev, const uint8_t* d_headers, size_t n, const uint8_t* d_pow_limit,
                             const uint8_t* d_prev_hash, uint8_t* d_hashes, uint8_t* d_status, void* hip_stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || n > 0xFFFFFF00ull) return HKV_E_ARG;
  if (n == 0) return HKV_OK;
  if (!d_headers || !d_pow_limit || !d_hashes || !d_status || !aligned(d_headers, 4) || !aligned(d_pow_limit, 4) ||
      !aligned(d_prev_hash, 4) || !aligned(d_hashes, 16))
    return HKV_E_ARG;
  DevCtx& d = ctx->devs[dev];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  hipStream_t st = static_cast<hipStream_t>(hip_stream);  // NULL: the null (default) stream (include/hkv.h)
  HKV_TRY(hkv::launch_headers(d_headers, (uint32_t)n, d_pow_limit, d_prev_hash, d_hashes, d_status, st),
          "headers launch");
  return HKV_OK;
}

int hkv_check_headers(hkv_ctx* ctx, const uint8_t* headers, size_t n, const uint8_t* pow_limit,
                      const uint8_t* prev_hash, uint8_t* hashes_out, uint8_t* status) {
  if (!ctx || ctx->devs.empty() || n > 0xFFFFFF00ull) return HKV_E_ARG;
  if (n == 0) return HKV_OK;
  if (!headers || !pow_limit || !hashes_out || !status) return HKV_E_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  DevCtx& d = ctx->devs[0];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  // one staging buffer: limit (32) | prev (32) | headers (n*80) | hashes (n*32) | status (n)
  int rc = scratch_acquire(d, d.stream);
  if (!rc) rc = grow(&d.stage[5], &d.stage_cap[5], 64 + n * 113, "hipMalloc(header batch)");
  if (rc) return rc;
  uint8_t* b = static_cast<uint8_t*>(d.stage[5]);
  uint8_t *dlim = b, *dprev = b + 32, *dh = b + 64, *dhash = dh + n * 80, *dst = dhash + n * 32;
  HKV_TRY(hipMemcpyAsync(dlim, pow_limit, 32, hipMemcpyHostToDevice, d.stream), "H2D pow limit");
  if (prev_hash) HKV_TRY(hipMemcpyAsync(dprev, prev_hash, 32, hipMemcpyHostToDevice, d.stream), "H2D prev");
  HKV_TRY(hipMemcpyAsync(dh, headers, n * 80, hipMemcpyHostToDevice, d.stream), "H2D headers");
  HKV_TRY(hkv::launch_headers(dh, (uint32_t)n, dlim, prev_hash ? dprev : nullptr, dhash, dst, d.stream),
          "headers launch");
  HKV_TRY(hipMemcpyAsync(hashes_out, dhash, n * 32, hipMemcpyDeviceToHost, d.stream), "D2H header hashes");
  HKV_TRY(hipMemcpyAsync(status, dst, n, hipMemcpyDeviceToHost, d.stream), "D2H header status");
  HKV_TRY(hipStreamSynchronize(d.stream), "headers sync");
  return scratch_release(d, d.stream);
}

int hkv_merkle_roots_device(hkv_ctx* ctx, int dev, const uint8_t* d_txids, const uint32_t* d_offsets,
                            size_t n_blocks, uint8_t* d_scratch, uint8_t* d_roots, uint8_t* d_mutated,
                            void* hip_stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || n_blocks > 0x7FFFFFFFull) return HKV_E_ARG;
  if (n_blocks == 0) return HKV_OK;
  if (!d_txids || !d_offsets || !d_scratch || !d_roots || !d_mutated || !aligned(d_txids, 16) ||
      !aligned(d_scratch, 16) || !aligned(d_roots, 16) || !aligned(d_offsets, 4))
    return HKV_E_ARG;
  DevCtx& d = ctx->devs[dev];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  hipStream_t st = static_cast<hipStream_t>(hip_stream);  // NULL: the null (default) stream (include/hkv.h)
  HKV_TRY(hkv::launch_merkle(d_txids, d_offsets, (uint32_t)n_blocks, d_scratch, d_roots, d_mutated, (uint32_t)d.n_cu, st),
          "merkle launch");
  return HKV_OK;
}

int hkv_merkle_roots(hkv_ctx* ctx, const uint8_t* txids, const uint32_t* offsets, size_t n_blocks,
                     uint8_t* roots_out, uint8_t* mutated) {
  if (!ctx || ctx->devs.empty() || n_blocks > 0x7FFFFFFFull) return HKV_E_ARG;
  if (n_blocks == 0) return HKV_OK;
  if (!offsets || !roots_out || !mutated) return HKV_E_ARG;
  if (offsets[0] != 0) return HKV_E_ARG;
  for (size_t b = 0; b < n_blocks; ++b)
    if (offsets[b + 1] < offsets[b]) return HKV_E_ARG;
  const size_t leaves = offsets[n_blocks];
  if (leaves && !txids) return HKV_E_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  DevCtx& d = ctx->devs[0];
  HKV_TRY(hipSetDevice(d.device), "hipSetDevice");
  // one staging buffer: txids (L*32) | scratch (L*32) | roots (B*32) | offsets ((B+1)*4) | mutated (B)
  const size_t off_bytes = (n_blocks + 1) * 4;
  int rc = scratch_acquire(d, d.stream);
  if (!rc) rc = grow(&d.stage[6], &d.stage_cap[6], leaves * 64 + n_blocks * 32 + off_bytes + n_blocks,
                     "hipMalloc(merkle batch)");
  if (rc) return rc;
  uint8_t* b = static_cast<uint8_t*>(d.stage[6]);
  uint8_t *dl = b, *dsc = dl + leaves * 32, *dr = dsc + leaves * 32, *doff = dr + n_blocks * 32,
          *dm = doff + off_bytes;
  if (leaves) HKV_TRY(hipMemcpyAsync(dl, txids, leaves * 32, hipMemcpyHostToDevice, d.stream), "H2D txids");
  HKV_TRY(hipMemcpyAsync(doff, offsets, off_bytes, hipMemcpyHostToDevice, d.stream), "H2D merkle offsets");
  HKV_TRY(hkv::launch_merkle(dl, reinterpret_cast<const uint32_t*>(doff), (uint32_t)n_blocks, dsc, dr, dm,
                             (uint32_t)d.n_cu, d.stream),
          "merkle launch");
  HKV_TRY(hipMemcpyAsync(roots_out, dr, n_blocks * 32, hipMemcpyDeviceToHost, d.stream), "D2H merkle roots");
  HKV_TRY(hipMemcpyAsync(mutated, dm, n_blocks, hipMemcpyDeviceToHost, d.stream), "D2H merkle mutated");
  HKV_TRY(hipStreamSynchronize(d.stream), "merkle sync");
  return scratch_release(d, d.stream);
}

}  // extern "C"

