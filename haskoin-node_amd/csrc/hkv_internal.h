// hkv_internal.h — declarations shared between the kernel TU and the C-ABI TU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hkv.h"

#define HKV_MODE_LIBSECP 0u
#define HKV_MODE_HASKOIN 1u

// debug/known-answer ops (hkv_debug_op in include/hkv.h)
enum {
  HKV_DBG_FE_MUL = 1,
  HKV_DBG_FE_SQR = 2,
  HKV_DBG_FE_ADD = 3,
  HKV_DBG_FE_SUB = 4,
  HKV_DBG_FE_INV = 5,
  HKV_DBG_FE_SQRT = 6,
  HKV_DBG_SC_MUL = 7,
  HKV_DBG_SC_INV = 8,
  HKV_DBG_GLV = 9,
  HKV_DBG_ECMULT_G = 10,
  HKV_DBG_MUL512 = 11,
  HKV_DBG_SQR512 = 12,
};

namespace hkv {
hipError_t launch_prologue(const void* recs, uint32_t n, uint32_t n_pad, uint32_t mode, uint32_t* im,
                           hipStream_t st);
hipError_t launch_ecmult(uint32_t* im, uint32_t n, uint32_t n_pad, const uint32_t* gtab, uint32_t* qs,
                         uint32_t grid, uint32_t* bits, uint32_t n_words, bool split, bool mid,
                         unsigned long long* clk, uint32_t* aux, const void* recs, uint32_t mode, uint32_t n_cu,
                         hipStream_t st);
hipError_t launch_gtable(uint32_t* gtab, hipStream_t st);
// the multisig scan operands a fused launch may take over (hkv_ms_scan_kernel's);
// counters: this call's running sum (candidates | key checks << 32), one of
// two parity words (the call's tail epoch): the tail reads it after the scan,
// and the launch that runs the tail zeroes the other word for the next call
struct MsScan {
  uint32_t* desc;
  uint64_t* off;
  uint64_t* counters;
};
// The multisig tail (hkv_kernels.hip 2e): one launch after the scan that
// does nothing when the batch has no multisig input and otherwise
// the BIP143 per-tx hashes (hash_txs), the candidate / key-check records, the
// key checks, the candidate verifies and the countMulSig walk — read from the
// device total, so the host never waits for it.
struct MsTail {
  const uint8_t* txs;
  const uint32_t* tx_off;
  uint32_t n_tx;
  uint32_t* txt;
  const uint8_t* scripts;
  uint32_t scripts_len;
  const hkv_input_job* jobs;
  uint32_t n;
  int32_t forkid;
  uint32_t hash_txs;  // TX_HASHES_* the tail computes first (the fused path's index hashed nothing)
  const uint32_t* desc;
  const uint64_t* off;
  unsigned long long* total;        // this call's scan sum (MsScan counters: ms_ctr[epoch & 1])
  unsigned long long* total_next;   // the next call's (ms_ctr[(epoch + 1) & 1]): zeroed by this launch
  uint8_t* cand;                    // the candidate record window (win_cand records)
  uint8_t* keyrec;                  // the key-check record window (win_keys records)
  uint32_t win_cand, win_keys;      // window capacities in records (multiples of 64): the tail runs
                                    // ceil(count / window) rounds of emit + verify
  uint32_t* cbits;                  // candidate verdict words (every candidate of the chunk)
  uint32_t* kbits;                  // key-check verdict words (every key check of the chunk)
  uint32_t* im;                     // pair-form scratch: slot stride = grid * 32
  uint32_t* aux;
  const uint32_t* gtab;
  uint32_t* qs;
  uint32_t* out_bits;               // the batch's verdict words (multisig inputs are ORed in)
  unsigned int* bar;                // two work-queue slots of 8 words (claim, done): launch `epoch` uses
                                    // slot epoch & 1 and zeroes the other
  uint32_t epoch;                   // this launch's sequence number on the device
  unsigned int* fault;              // the device's sticky fault latch (hkv_device_fault)
  uint32_t* status;                 // the call's status word (HKV_STATUS_* ORed in), or null
  uint32_t force_fault;             // test hook (hkv_debug_fail_device HKV_FAIL_TAIL): every phase wait gives up
};
hipError_t launch_ms_tail(const MsTail& a, uint32_t grid, hipStream_t st);  // grid <= n_cu (its scratch slots)
uint32_t ms_tail_slots(uint32_t n_cu);  // signatures in flight (im / aux slots the tail needs)
// small batches of standard inputs in one launch; with ms, the block kernel
// (std_split_scans) also runs the multisig scan; with tx_off (the block
// kernel only), it builds the index rows of its inputs' txs into txt itself
// (no index launch before it)
hipError_t launch_std_verify_split(const uint8_t* txs, uint32_t n_tx, const uint32_t* txt, const uint8_t* scripts,
                                   uint32_t scripts_len, const hkv_input_job* jobs, uint32_t n, uint32_t n_pad,
                                   int32_t forkid, uint8_t* recs, uint32_t* im, const uint32_t* gtab, uint32_t* qs,
                                   uint32_t* aux, uint32_t* bits, uint32_t n_words, unsigned long long* clk,
                                   uint32_t n_cu, const MsScan* ms, const uint32_t* tx_off, hipStream_t st);
bool std_split_scans(uint32_t n_pad, uint32_t n_cu);
// y-free full-grid batches: u1 * G, the y0 = num / den reduction and the verdict bitmap
// the operands of a standard-input batch (txs, index rows, prevout scripts, jobs)
struct StdOps {
  const uint8_t* txs;
  uint32_t n_tx;
  const uint32_t* txt;
  const uint8_t* scripts;
  uint32_t scripts_len;
  const hkv_input_job* jobs;
  int32_t forkid;
};
// mid-size standard-input batches (the overlapped path): std_parse, prologue,
// s^-1 and GLV in one lane per input at the head of the mid-size ecmult
// kernel's lanes
hipError_t launch_std_ecmult_mid(const StdOps& o, uint32_t* im, uint32_t n, uint32_t n_pad, uint32_t* qs,
                                 uint32_t grid, unsigned long long* clk, hipStream_t st);
// (mid: the paired-product instance; late_recs: large standard-input batches,
// u1 and the validity from the final records first)
hipError_t launch_finish(uint32_t* im, uint32_t n, uint32_t n_pad, const uint32_t* gtab, uint32_t* rare_ctr,
                         uint32_t* bits, uint32_t n_words, bool mid, const void* late_recs, hipStream_t st);
hipError_t launch_gen_pool(uint64_t seed, uint32_t npool, uint32_t* pool, hipStream_t st);
hipError_t launch_gen_records(uint64_t seed, uint64_t index0, uint32_t n, const uint32_t* pool, uint32_t npool,
                              uint32_t unc_permille, uint32_t invalid_permille, void* recs, uint32_t* labels,
                              hipStream_t st);
hipError_t launch_debug(uint32_t op, uint32_t n, const uint32_t* a, const uint32_t* b, uint32_t* out,
                        hipStream_t st);
hipError_t ecmult_max_blocks_per_cu(int* out);
hipError_t launch_gen_keys(uint64_t seed, uint32_t n, uint8_t* priv, uint8_t* pub, uint8_t* h160, hipStream_t st);
hipError_t launch_gen_sign(uint64_t seed, uint32_t n, const uint8_t* priv, const uint32_t* key_idx,
                           const uint8_t* msg, uint32_t msg_stride, uint8_t* sig, hipStream_t st);
// hkv_sighash.hip
hipError_t launch_tx_index(const uint8_t* txs, const uint32_t* tx_off, uint32_t n_tx, uint32_t hashes,
                           uint32_t* txt, hipStream_t st);
hipError_t launch_sighash(const uint8_t* txs, uint32_t n_tx, const uint32_t* txt, const uint8_t* scripts,
                          uint32_t scripts_len, const hkv_sighash_job* jobs, uint32_t n, int32_t forkid, uint8_t* out,
                          uint32_t stride, uint8_t* status, hipStream_t st);
hipError_t launch_std_inputs(const uint8_t* txs, uint32_t n_tx, const uint32_t* txt, const uint8_t* scripts,
                             uint32_t scripts_len, const hkv_input_job* jobs, uint32_t n, int32_t forkid,
                             uint8_t* recs, hipStream_t st);
// the overlapped extraction of large batches: the BIP143 per-tx hashes alone
// (rows written by launch_tx_index(TX_HASHES_NONE) before)
hipError_t launch_tx_hashes_only(const uint8_t* txs, const uint32_t* tx_off, uint32_t n_tx, uint32_t hashes,
                                 uint32_t* txt, hipStream_t st);
// multisig inputs: the scan (hkv_sighash.hip section 4; the tail in hkv_kernels.hip)
hipError_t launch_ms_scan(const uint8_t* txs, uint32_t n_tx, const uint32_t* txt, const uint8_t* scripts,
                          uint32_t scripts_len, const hkv_input_job* jobs, uint32_t n, int32_t forkid,
                          uint32_t* desc, uint64_t* off, uint64_t* counters, hipStream_t st);
// hkv_headers.hip
hipError_t launch_headers(const uint8_t* hdrs, uint32_t n, const uint8_t* pow_limit, const uint8_t* prev0,
                          uint8_t* hashes, uint8_t* status, hipStream_t st);
hipError_t launch_merkle(const uint8_t* leaves, const uint32_t* offsets, uint32_t n_blocks, uint8_t* scratch,
                         uint8_t* roots, uint8_t* mutated, uint32_t n_cu, hipStream_t st);
}  // namespace hkv
