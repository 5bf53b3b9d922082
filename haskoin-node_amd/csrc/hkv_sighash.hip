// hkv_sighash.hip — on-device signature hashes and standard-input extraction
// for gfx950.
//
// A batch is a buffer of serialised transactions (wire form, with or without
// BIP144 witnesses) plus per-signature jobs. Three kernels, one lane each:
//   1. hkv_tx_index_kernel   — per tx: bounds-checked parse of the wire form
//      into a 128-byte row (input / output / locktime offsets) and, when
//      asked, the three BIP143 per-tx hashes (hashPrevouts, hashSequence,
//      hashOutputs), computed once per tx and shared by its inputs.
//   2. hkv_sighash_kernel    — per job: haskoin-core txSigHash (legacy) or
//      txSigHashForkId (BIP143) -> 32-byte msg32, written with a caller
//      stride (stride 168 writes straight into verify records).
//   3. hkv_std_input_kernel  — per input: the non-ECDSA half of
//      verifyStdInput for P2PK / P2PKH / P2WPKH / P2SH-P2WPKH prevouts (template match,
//      strict DER decode + low S + hashtype, HASH160 check, sighash) -> one
//      168-byte verify record; a failed check writes an all-zero record, which
//      the verify kernels reject (pubkey length 0).
//
// Preimages are never materialised. Each lane runs a small generator that
// emits its preimage as "pieces" (a byte range of the tx / script buffers, or
// an up-to-8-byte literal such as a re-encoded varint, a zeroed sequence or a
// stored hash), and sha256_stream absorbs them block-synchronously through a
// per-lane 64-byte LDS slot. Varints that haskoin re-serialises (input and
// output counts, script lengths) are always re-emitted canonically, so
// non-canonical encodings in the input hash exactly as the reference does.
//
// Reference semantics restated [dep; haskoin-core-1.1.0 pinned at
// /root/reference/stack.yaml:10]: Haskoin.Script.SigHash txSigHash /
// txSigHashForkId / decodeTxSig, Haskoin.Crypto.Signature decodeStrictSig
// (libsecp256k1 secp256k1_ecdsa_signature_parse_der), Haskoin.Transaction.
// Builder verifyStdInput; CPU restatement: oracle/sighash_oracle.py.
#include "hkv_hash.h"
#include "hkv_scalar.h"
#include "hkv_layout.h"
#include "hkv_internal.h"
#include "../../include/hkv.h"

#include "hkv_sighash_dev.h"

namespace hkv {

__global__ void __launch_bounds__(WG) hkv_tx_index_kernel(const uint8_t* __restrict__ txs,
                                                          const uint32_t* __restrict__ tx_off, uint32_t n_tx,
                                                          uint32_t* __restrict__ txt) {
  const uint32_t t = blockIdx.x * WG + threadIdx.x;
  if (t >= n_tx) return;
  uint32_t row[8];
  tx_index_row(txs, tx_off, t, row);
#pragma unroll
  for (int k = 0; k < 8; ++k) txt[(size_t)t * TXT_WORDS + k] = row[k];
}

// 1b. the three BIP143 per-tx hashes, one lane per (tx, hash): blockIdx.y
// selects hashPrevouts / hashSequence / hashOutputs (wave-uniform), so the
// three SHA-256d streams of a tx run side by side instead of one after the
// other (a block's index is latency-bound: one wave per 64 txs).
// Each lane parses its tx itself (the three blockIdx.y lanes of a tx repeat
// the cheap walk; y = 0 writes the row), so the index costs no launch of its own.
// witness_only: hash only the txs with witness data (the others' rows keep
// stale hash words, which no standard input on a network without a fork id reads)
__global__ void __launch_bounds__(WG) hkv_tx_hash_kernel(const uint8_t* __restrict__ txs,
                                                         const uint32_t* __restrict__ tx_off, uint32_t n_tx,
                                                         uint32_t witness_only, uint32_t write_rows,
                                                         uint32_t* __restrict__ txt) {
  __shared__ uint32_t buf[16 * WG];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t which = blockIdx.y;  // 0 prevouts, 1 sequences, 2 outputs
  uint32_t row[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (t < n_tx) {
    tx_index_row(txs, tx_off, t, row);
    if (which == 0 && write_rows) {
#pragma unroll
      for (int k = 0; k < 8; ++k) txt[(size_t)t * TXT_WORDS + k] = row[k];
    }
  }
  const bool go = t < n_tx && (row[TXT_FLAGS] & TXF_OK) && (!witness_only || (row[TXT_FLAGS] & TXF_WITNESS));
  Gen g;
  uint32_t h[8], d[8];
  gen_clear(g);
  g.T = txs;
  if (which == 2) {  // hashOutputs (each output re-serialised canonically)
    g.ooff = row[TXT_OUTS_FIRST]; g.ocnt = row[TXT_NOUT]; g.ret = PH_DONE; g.phase = PH_O_VAL;
  } else {
    g.nin = row[TXT_NIN]; g.ioff = row[TXT_INS]; g.j = 0; g.phase = which == 0 ? PH_P_IN : PH_S_IN;
  }
  sha256_stream(h, g, go, buf);
  sha256d_finish(d, h);
  if (go) {
    const int slot = which == 0 ? TXT_HP : (which == 1 ? TXT_HS : TXT_HO);
#pragma unroll
    for (int k = 0; k < 8; ++k) txt[(size_t)t * TXT_WORDS + slot + k] = d[k];
  }
}

// ---------------------------------------------------------------------------
// 2. sighash jobs
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(WG) hkv_sighash_kernel(const uint8_t* __restrict__ txs, uint32_t n_tx,
                                                         const uint32_t* __restrict__ txt,
                                                         const uint8_t* __restrict__ scripts, uint32_t scripts_len,
                                                         const hkv_sighash_job* __restrict__ jobs, uint32_t n,
                                                         int32_t forkid, uint8_t* __restrict__ out, uint32_t stride,
                                                         uint8_t* __restrict__ status) {
  __shared__ uint32_t buf[16 * WG];
  const uint32_t jx = blockIdx.x * blockDim.x + threadIdx.x;
  const bool in_range = jx < n;
  uint32_t stc = HKV_SH_BAD_REF;
  JobCtx c;
  c.forkid_form = false; c.one = false; c.single_hash = false;
  const uint32_t* row = txt;
  const uint8_t* code = scripts;
  uint32_t code_len = 0;
  uint64_t value = 0;
  uint32_t* o32 = reinterpret_cast<uint32_t*>(out + (size_t)jx * stride);
  if (in_range) {
    const hkv_sighash_job jb = jobs[jx];
    const bool ref_ok = jb.tx < n_tx && jb.script_off <= scripts_len && scripts_len - jb.script_off >= jb.script_len &&
                        jb.kind <= HKV_SIGHASH_FORKID;
    if (ref_ok) {
      row = txt + (size_t)jb.tx * TXT_WORDS;
      if (!(row[TXT_FLAGS] & TXF_OK)) stc = HKV_SH_BAD_TX;
      else if (jb.input >= row[TXT_NIN]) stc = HKV_SH_BAD_INPUT;
      else stc = HKV_SH_OK;
    }
    if (stc == HKV_SH_OK) {
      job_setup(c, txs, row, jb.input, jb.sighash, jb.kind == HKV_SIGHASH_FORKID, forkid);
      code = scripts + jb.script_off;
      code_len = jb.script_len;
      value = jb.value;
    }
  }
  const bool ok = in_range && stc == HKV_SH_OK;
  Gen g;
  uint32_t h[8], d[8];
  // BIP143 SINGLE: hashOutputs = SHA-256d(output i), parked in the job's output slot
  const bool need_single = ok && c.single_hash;
  if (__any(need_single)) {
    gen_clear(g);
    g.T = txs; g.ooff = c.single_off; g.ocnt = 1; g.ret = PH_DONE; g.phase = PH_O_VAL;
    sha256_stream(h, g, need_single, buf);
    sha256d_finish(d, h);
    if (need_single) {
#pragma unroll
      for (int k = 0; k < 8; ++k) o32[k] = d[k];
    }
  }
  const bool live = ok && !c.one;
  if (live) gen_job(g, c, txs, row, code, code_len, false, value, o32);
  else gen_clear(g);
  sha256_stream(h, g, live, buf);
  sha256d_finish(d, h);
  if (in_range) {
#pragma unroll
    for (int k = 0; k < 8; ++k) o32[k] = live ? d[k] : ((ok && c.one && k == 0) ? 1u : 0u);
    if (status) status[jx] = (uint8_t)stc;
  }
}

__global__ void __launch_bounds__(WG) hkv_std_input_kernel(const uint8_t* __restrict__ txs, uint32_t n_tx,
                                                           const uint32_t* __restrict__ txt,
                                                           const uint8_t* __restrict__ scripts, uint32_t scripts_len,
                                                           const hkv_input_job* __restrict__ jobs, uint32_t n,
                                                           int32_t forkid, uint8_t* __restrict__ recs) {
  __shared__ uint32_t buf[16 * WG];
  const uint32_t jx = blockIdx.x * blockDim.x + threadIdx.x;
  StdIn x;
  std_parse(x, txs, n_tx, txt, scripts, scripts_len, jobs, jx, n, forkid);
  uint32_t* r32 = reinterpret_cast<uint32_t*>(recs + (size_t)jx * REC_SIZE);
  uint32_t d[8];
  const bool live = std_hash(x, txs, forkid, r32, buf, d);
  if (jx >= n) return;
  std_write_record(r32, x, live, d);
}

// 4. multisig inputs: the scan (hkv_sighash_dev.h ms_scan_lane), candidate
//    records, the countMulSig walk
__global__ void __launch_bounds__(WG) hkv_ms_scan_kernel(const uint8_t* __restrict__ txs, uint32_t n_tx,
                                                         const uint32_t* __restrict__ txt,
                                                         const uint8_t* __restrict__ scripts, uint32_t scripts_len,
                                                         const hkv_input_job* __restrict__ jobs, uint32_t n,
                                                         int32_t forkid, uint32_t* __restrict__ desc,
                                                         uint64_t* __restrict__ off,
                                                         unsigned long long* __restrict__ counters) {
  __shared__ uint32_t buf[16 * WG];
  const uint32_t jx = blockIdx.x * WG + threadIdx.x;
  ms_scan_lane(txs, n_tx, txt, scripts, scripts_len, jobs, jx, jx < n, forkid, desc, off, counters, buf);
}

}  // namespace hkv

// ---------------------------------------------------------------------------
// launch wrappers (called by hkv_api.cpp)
// ---------------------------------------------------------------------------
namespace hkv {

static inline uint32_t blocks_for(size_t n) { return (uint32_t)((n + WG - 1) / WG); }

hipError_t launch_tx_index(const uint8_t* txs, const uint32_t* tx_off, uint32_t n_tx, uint32_t hashes,
                           uint32_t* txt, hipStream_t st) {
  if (n_tx == 0) return hipSuccess;
  if (hashes != TX_HASHES_NONE)
    hipLaunchKernelGGL(hkv_tx_hash_kernel, dim3((n_tx + xtpb_for(n_tx) - 1) / xtpb_for(n_tx), 3), dim3(xtpb_for(n_tx)), 0, st,
                       txs, tx_off, n_tx, hashes == TX_HASHES_WITNESS ? 1u : 0u, 1u, txt);
  else
    hipLaunchKernelGGL(hkv_tx_index_kernel, dim3(blocks_for(n_tx)), dim3(WG), 0, st, txs, tx_off, n_tx, txt);
  return hipGetLastError();
}
hipError_t launch_tx_hashes_only(const uint8_t* txs, const uint32_t* tx_off, uint32_t n_tx, uint32_t hashes,
                                 uint32_t* txt, hipStream_t st) {
  if (n_tx == 0 || hashes == TX_HASHES_NONE) return hipSuccess;
  hipLaunchKernelGGL(hkv_tx_hash_kernel, dim3((n_tx + xtpb_for(n_tx) - 1) / xtpb_for(n_tx), 3), dim3(xtpb_for(n_tx)), 0,
                     st, txs, tx_off, n_tx, hashes == TX_HASHES_WITNESS ? 1u : 0u, 0u, txt);
  return hipGetLastError();
}
hipError_t launch_sighash(const uint8_t* txs, uint32_t n_tx, const uint32_t* txt, const uint8_t* scripts,
                          uint32_t scripts_len, const hkv_sighash_job* jobs, uint32_t n, int32_t forkid, uint8_t* out,
                          uint32_t stride, uint8_t* status, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(hkv_sighash_kernel, dim3((n + xtpb_for(n) - 1) / xtpb_for(n)), dim3(xtpb_for(n)), 0, st, txs, n_tx, txt, scripts, scripts_len,
                     jobs, n, forkid, out, stride, status);
  return hipGetLastError();
}
hipError_t launch_std_inputs(const uint8_t* txs, uint32_t n_tx, const uint32_t* txt, const uint8_t* scripts,
                             uint32_t scripts_len, const hkv_input_job* jobs, uint32_t n, int32_t forkid,
                             uint8_t* recs, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(hkv_std_input_kernel, dim3((n + xtpb_for(n) - 1) / xtpb_for(n)), dim3(xtpb_for(n)), 0, st, txs, n_tx, txt, scripts,
                     scripts_len, jobs, n, forkid, recs);
  return hipGetLastError();
}

}  // namespace hkv

// ---------------------------------------------------------------------------
// multisig launch wrappers
// ---------------------------------------------------------------------------
namespace hkv {

// per-input desc words and record offsets; *counters (the call's parity
// word, zeroed by the call before) ends as the number of candidate records |
// key-check records << 32 (the tail kernel reads it, stream-ordered after the
// scan)
hipError_t launch_ms_scan(const uint8_t* txs, uint32_t n_tx, const uint32_t* txt, const uint8_t* scripts,
                          uint32_t scripts_len, const hkv_input_job* jobs, uint32_t n, int32_t forkid,
                          uint32_t* desc, uint64_t* off, uint64_t* counters, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(hkv_ms_scan_kernel, dim3(blocks_for(n)), dim3(WG), 0, st, txs, n_tx, txt, scripts, scripts_len,
                     jobs, n, forkid, desc, off, reinterpret_cast<unsigned long long*>(counters));
  return hipGetLastError();
}

}  // namespace hkv
