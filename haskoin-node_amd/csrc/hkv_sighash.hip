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
                                                         uint32_t witness_only, uint32_t* __restrict__ txt) {
  __shared__ uint32_t buf[16 * WG];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t which = blockIdx.y;  // 0 prevouts, 1 sequences, 2 outputs
  uint32_t row[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (t < n_tx) {
    tx_index_row(txs, tx_off, t, row);
    if (which == 0) {
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

// ---------------------------------------------------------------------------
// 4. multisig inputs (bare and P2SH): candidate (signature, key) records
// ---------------------------------------------------------------------------
// haskoin-core verifyStdInput's PayMulSig branch [dep; oracle/sighash_oracle.py
// std_multisig]: countMulSig walks the keys in order against the current
// signature; a match consumes both, a miss only the key, an empty signature
// (OP_0) one of each; the input verifies iff the count equals m and every
// key of the script is a point (importPubKey). Which comparisons the walk
// makes depends on earlier verdicts, so the batch checks every pair it could
// make (signature j < min(#sigs, n) against keys j..n-1) and
// hkv_ms_resolve_kernel replays the walk over the verdict bits.
//   hkv_ms_scan_kernel    per input: template + scriptSig decode (+ the P2SH
//                         redeem HASH160), desc words and candidate counts
//   (exclusive scan of the counts -> record offsets)
//   hkv_ms_emit_kernel    per input: sighash of each signature, candidate and
//                         key-check records
//   hkv_ms_resolve_kernel per input: the countMulSig walk -> verdict bit
// Keys must be direct pushes (21 / 41) with PubKeyI prefixes, the limit the
// P2PK template shares, so haskoin's canonical re-encoding (encodeOutput) of
// the script equals its bytes.
constexpr uint32_t MS_OK = 1u << 31, MS_P2SH = 1u << 30;

// OP_m <keys> OP_n OP_CHECKMULTISIG, 1 <= m <= n <= 16
HKV_DEV bool ms_template(const uint8_t* sc, uint32_t L, uint32_t& m, uint32_t& n) {
  if (L < 3 || sc[L - 1] != 0xAEu) return false;
  m = (uint32_t)sc[0] - 0x50u;
  n = (uint32_t)sc[L - 2] - 0x50u;
  if (m < 1u || m > 16u || n < 1u || n > 16u || m > n) return false;
  uint32_t off = 1, k = 0;
  while (off < L - 2 && k < 17u) {
    const uint32_t op = sc[off];
    if (op != 0x21u && op != 0x41u) return false;
    if (off + 1 + op > L - 2) return false;
    const uint32_t pre = sc[off + 1];
    if (op == 0x21u ? (pre != 2u && pre != 3u) : (pre != 4u)) return false;
    off += 1 + op;
    ++k;
  }
  return off == L - 2 && k == n;
}
// key k of a validated template
HKV_DEV const uint8_t* ms_key(const uint8_t* sc, uint32_t k, uint32_t& len) {
  uint32_t off = 1;
  for (uint32_t q = 0; q < k; ++q) off += 1 + sc[off];
  len = sc[off];
  return sc + off + 1;
}
// skip one script op (haskoin's Script parse: a push must fit)
HKV_DEV bool skip_op(const uint8_t* p, uint32_t& off, uint32_t end) {
  const uint32_t op = p[off];
  if (op == 0u || op > 0x4Eu) {
    ++off;
    return true;
  }
  uint32_t d_off, d_len;
  return read_push(p, off, end, d_off, d_len);
}

struct MsIn {
  const uint8_t* code;  // scriptCode: the prevout, redeem or witness script
  uint32_t code_len;
  // the signature items: scriptSig form — the byte range after the OP_0
  // dummy (and before a P2SH redeem push); witness form — it_off is the
  // length varint of the item after the empty dummy, n_items of them
  uint32_t it_off, it_end, n_items;
  uint32_t m, n, s_eff, mask, n_cand;
  bool p2sh, wit;            // HASH160(rd) == the P2SH hash; witness form (SHA-256 check, BIP143)
  const uint8_t* rd;         // P2SH: the pushed redeem script (a multisig script, or 00 20 <h32>)
  uint32_t rd_len;
  const uint8_t* wprog;      // witness form: the 32-byte program
};

// next item: d_len == 0 means TxSignatureEmpty; false = not a push (decode fails)
HKV_DEV bool ms_item(const uint8_t* txs, const MsIn& r, uint32_t& off, uint32_t& d_off, uint32_t& d_len) {
  if (r.wit) {
    d_len = get_varint(txs, off);
    d_off = off;
    off += d_len;
    return true;
  }
  if (txs[off] == 0u) {
    ++off;
    d_len = 0;
    return true;
  }
  return read_push(txs, off, r.it_end, d_off, d_len);
}

// decode a multisig input except the hash checks (P2SH HASH160, P2WSH SHA-256)
HKV_DEV bool ms_parse(MsIn& r, const uint8_t* txs, const uint32_t* row, uint32_t input, const uint8_t* spk,
                      uint32_t L, int32_t forkid) {
  r.p2sh = L == 23u && spk[0] == 0xA9u && spk[1] == 0x14u && spk[22] == 0x87u;
  r.wit = false;
  r.rd = txs;
  r.rd_len = 0;
  r.wprog = spk;
  uint32_t in_off, ss_off, ss_len, seq_off;
  walk_input(txs, row[TXT_INS], input, in_off, ss_off, ss_len, seq_off);
  const uint32_t end = ss_off + ss_len;
  if (L == 34u && spk[0] == 0u && spk[1] == 0x20u) {  // P2WSH: empty scriptSig
    if (ss_len != 0) return false;
    r.wit = true;
    r.wprog = spk + 2;
  } else if (r.p2sh && ss_len > 0 && txs[ss_off] != 0u) {  // P2SH-P2WSH: exactly one push of 00 20 <h32>
    uint32_t c = ss_off, d_off = 0, d_len = 0;
    if (!read_push(txs, c, end, d_off, d_len) || c != end || d_len != 34u || txs[d_off] != 0u ||
        txs[d_off + 1] != 0x20u)
      return false;
    r.wit = true;
    r.rd = txs + d_off;
    r.rd_len = 34;
    r.wprog = r.rd + 2;
  }
  if (r.wit) {  // witness = [empty dummy] ++ items ++ [witness script]
    if (!(row[TXT_FLAGS] & TXF_WITNESS)) return false;
    uint32_t w = walk_witness(txs, row[TXT_OUTS_END], input);
    const uint32_t cnt = get_varint(txs, w);
    if (cnt < 2u || get_varint(txs, w) != 0u) return false;
    r.it_off = w;
    r.n_items = cnt - 2u;
    for (uint32_t k = 0; k < r.n_items; ++k) w += get_varint(txs, w);
    r.code_len = get_varint(txs, w);
    r.code = txs + w;
    r.it_end = w;
  } else {
    if (ss_len == 0 || txs[ss_off] != 0u) return false;  // haskoin matchMulSig: OP_0 first
    r.it_off = ss_off + 1;
    if (r.p2sh) {
      uint32_t off = ss_off + 1, last = 0, n_ops = 0;
      while (off < end) {
        last = off;
        if (!skip_op(txs, off, end)) return false;
        ++n_ops;
      }
      if (n_ops == 0) return false;
      uint32_t c = last, d_off = 0, d_len = 0;
      if (!read_push(txs, c, end, d_off, d_len)) return false;  // the redeem script: OP_PUSHDATA
      r.code = r.rd = txs + d_off;
      r.code_len = r.rd_len = d_len;
      r.it_end = last;
    } else {
      r.code = spk;
      r.code_len = L;
      r.it_end = end;
    }
    r.n_items = 0xFFFFFFFFu;  // until it_end
  }
  if (!ms_template(r.code, r.code_len, r.m, r.n)) return false;
  uint32_t j = 0, mask = 0, cand = 0, off = r.it_off;
  while (r.wit ? j < r.n_items : off < r.it_end) {
    uint32_t d_off = 0, d_len = 0;
    if (!ms_item(txs, r, off, d_off, d_len)) return false;  // any other op fails the decode
    if (d_len) {
      uint32_t rr[8], ss[8], sh;
      if (!decode_tx_sig(txs, d_off, d_len, forkid, rr, ss, sh)) return false;
      if (j < r.n) {
        mask |= 1u << j;
        cand += r.n - j;
      }
    }
    ++j;
  }
  r.s_eff = j < r.n ? j : r.n;
  r.mask = mask;
  r.n_cand = cand;
  return true;
}

// job -> (row, prevout script); false for a bad reference / unparsed tx
HKV_DEV bool ms_job(const hkv_input_job& jb, uint32_t n_tx, const uint32_t* txt, const uint8_t* scripts,
                    uint32_t scripts_len, const uint32_t*& row, const uint8_t*& spk) {
  if (!(jb.tx < n_tx && jb.script_off <= scripts_len && scripts_len - jb.script_off >= jb.script_len)) return false;
  row = txt + (size_t)jb.tx * TXT_WORDS;
  if (!((row[TXT_FLAGS] & TXF_OK) && jb.input < row[TXT_NIN])) return false;
  spk = scripts + jb.script_off;
  return true;
}

__global__ void __launch_bounds__(WG) hkv_ms_scan_kernel(const uint8_t* __restrict__ txs, uint32_t n_tx,
                                                         const uint32_t* __restrict__ txt,
                                                         const uint8_t* __restrict__ scripts, uint32_t scripts_len,
                                                         const hkv_input_job* __restrict__ jobs, uint32_t n,
                                                         int32_t forkid, uint32_t* __restrict__ desc,
                                                         uint64_t* __restrict__ off,
                                                         unsigned long long* __restrict__ counters,
                                                         volatile unsigned long long* __restrict__ host_total,
                                                         unsigned long long seq) {
  unsigned long long* total = counters;                                  // candidates | keys << 32
  unsigned int* done = reinterpret_cast<unsigned int*>(counters + 1);    // finished workgroups
  __shared__ uint32_t buf[16 * WG];
  const uint32_t jx = blockIdx.x * WG + threadIdx.x;
  MsIn r;
  r.p2sh = r.wit = false;
  r.code = r.rd = r.wprog = scripts;
  r.code_len = r.rd_len = 0;
  bool ok = false;
  const uint8_t* spk = scripts;
  if (jx < n) {
    const hkv_input_job jb = jobs[jx];
    const uint32_t* row = txt;
    ok = ms_job(jb, n_tx, txt, scripts, scripts_len, row, spk);
    if (ok) {
      const uint32_t L = jb.script_len;
      const bool p2sh = L == 23u && spk[0] == 0xA9u && spk[1] == 0x14u && spk[22] == 0x87u;
      const bool p2wsh = L == 34u && spk[0] == 0u && spk[1] == 0x20u;
      const bool bare = L >= 3u && spk[L - 1] == 0xAEu;
      ok = (p2sh || p2wsh || bare) && ms_parse(r, txs, row, jb.input, spk, L, forkid);
    }
  }
  Gen g;
  uint32_t h[8];
  // P2SH: HASH160(redeem script) == the script hash
  const bool need = ok && r.p2sh;
  if (__any(need)) {
    gen_clear(g);
    g.code = r.rd;
    g.code_len = r.rd_len;
    g.phase = PH_RANGE;
    sha256_stream(h, g, need, buf);
    uint32_t rip[5];
    ripemd160_of_digest(rip, h);
    if (need) ok = ok && eq_h160(spk + 2, rip);
  }
  // P2WSH (native or nested): SHA-256(witness script) == the program
  const bool need_ws = ok && r.wit;
  if (__any(need_ws)) {
    gen_clear(g);
    g.code = r.code;
    g.code_len = r.code_len;
    g.phase = PH_RANGE;
    sha256_stream(h, g, need_ws, buf);
    if (need_ws) ok = ok && eq_sha256(r.wprog, h);
  }
  if (jx < n) {
    desc[2 * (size_t)jx] = ok ? (MS_OK | (r.p2sh ? MS_P2SH : 0u) | r.m | (r.n << 8) | (r.s_eff << 16)) : 0u;
    desc[2 * (size_t)jx + 1] = ok ? r.mask : 0u;
    // record ranges: candidates in the low 32 bits, key checks in the high 32
    // (their sums stay below 2^32); placement order is irrelevant to verdicts
    off[jx] = ok ? (uint64_t)atomicAdd(total, (unsigned long long)r.n_cand | ((unsigned long long)r.n << 32)) : 0ull;
  }
  // The last workgroup to finish publishes the sum to the caller's pinned
  // host word and re-arms both device counters, so the stream carries no
  // memset and no D2H copy (the host waits on an event after this kernel).
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(done, 1u) == gridDim.x - 1) {
    __threadfence();
    const unsigned long long t = atomicExch(total, 0ull);
    atomicExch(done, 0u);
    host_total[0] = t;
    __threadfence_system();
    host_total[1] = seq;  // the host polls this word
    __threadfence_system();
  }
}

// record: msg32 (digest byte order words) | r | s (limbs, written big-endian) |
// pklen | pubkey | zero padding
HKV_DEV void write_record(uint32_t* r32, const uint32_t msg[8], const uint32_t r[8], const uint32_t s[8],
                          const uint8_t* pub, uint32_t pub_len) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    r32[k] = msg[k];
    r32[8 + k] = __builtin_bswap32(r[7 - k]);
    r32[16 + k] = __builtin_bswap32(s[7 - k]);
  }
#pragma unroll
  for (int w = 0; w < 18; ++w) {
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int q = 4 * w + b;  // byte 96 + q of the record
      uint32_t byte = 0;
      if (q == 0) byte = pub_len;
      else if ((uint32_t)(q - 1) < pub_len && q - 1 < 65) byte = pub[q - 1];
      v |= byte << (8 * b);
    }
    r32[24 + w] = v;
  }
}

__global__ void __launch_bounds__(WG) hkv_ms_emit_kernel(const uint8_t* __restrict__ txs, uint32_t n_tx,
                                                         const uint32_t* __restrict__ txt,
                                                         const uint8_t* __restrict__ scripts, uint32_t scripts_len,
                                                         const hkv_input_job* __restrict__ jobs, uint32_t n,
                                                         int32_t forkid, const uint32_t* __restrict__ desc,
                                                         const uint64_t* __restrict__ off64,
                                                         uint8_t* __restrict__ cand, uint8_t* __restrict__ keyrec) {
  __shared__ uint32_t buf[16 * WG];
  const uint32_t jx = blockIdx.x * WG + threadIdx.x;
  bool go = jx < n && (desc[2 * (size_t)jx] & MS_OK);
  MsIn r;
  r.code = r.rd = r.wprog = scripts; r.code_len = r.rd_len = 0; r.s_eff = 0; r.mask = 0; r.n = 0;
  r.it_off = r.it_end = 0; r.p2sh = r.wit = false;
  const uint32_t* row = txt;
  const uint8_t* spk = scripts;
  uint32_t input = 0;
  uint64_t value = 0;
  uint32_t cbase = 0, kbase = 0;
  if (go) {
    const hkv_input_job jb = jobs[jx];
    input = jb.input;
    value = jb.value;
    go = ms_job(jb, n_tx, txt, scripts, scripts_len, row, spk) &&
         ms_parse(r, txs, row, jb.input, spk, jb.script_len, forkid);
    const uint64_t o = off64[jx];
    cbase = (uint32_t)o;
    kbase = (uint32_t)(o >> 32);
  }
  // key-check records (msg, r, s zero): one per key of the script
  if (go) {
    const uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t k = 0; k < r.n; ++k) {
      uint32_t kl;
      const uint8_t* kp = ms_key(r.code, k, kl);
      write_record(reinterpret_cast<uint32_t*>(keyrec + (size_t)(kbase + k) * REC_SIZE), z, z, z, kp, kl);
    }
  }
  // per signature j < s_eff: its sighash, then records (msg_j, r_j, s_j, key_k), k = j..n-1
  uint32_t off = r.it_off, idx = cbase;
  Gen g;
  uint32_t h[8], d[8];
  for (uint32_t j = 0; __any(go && j < r.s_eff); ++j) {
    const bool here = go && j < r.s_eff;
    uint32_t d_off = 0, d_len = 0;
    if (here) (void)ms_item(txs, r, off, d_off, d_len);
    const bool live = here && ((r.mask >> j) & 1u);
    uint32_t rr[8], ss[8], sh = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) rr[k] = ss[k] = 0;
    if (live) (void)decode_tx_sig(txs, d_off, d_len, forkid, rr, ss, sh);
    JobCtx c;
    c.forkid_form = false; c.one = false; c.single_hash = false;
    if (live) job_setup(c, txs, row, input, sh, r.wit, forkid);  // P2WSH: BIP143 over the witness script
    uint32_t* r32 = reinterpret_cast<uint32_t*>(cand + (size_t)idx * REC_SIZE);  // first record of sig j
    const bool need_single = live && c.single_hash;
    if (__any(need_single)) {
      gen_clear(g);
      g.T = txs; g.ooff = c.single_off; g.ocnt = 1; g.ret = PH_DONE; g.phase = PH_O_VAL;
      sha256_stream(h, g, need_single, buf);
      sha256d_finish(d, h);
      if (need_single) {
#pragma unroll
        for (int k = 0; k < 8; ++k) r32[k] = d[k];  // scratch: hashOutputs of output i
      }
    }
    const bool hashed = live && !c.one;
    if (hashed) gen_job(g, c, txs, row, r.code, r.code_len, false, value, r32);
    else gen_clear(g);
    sha256_stream(h, g, hashed, buf);
    sha256d_finish(d, h);
    if (live) {
      uint32_t msg[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) msg[k] = hashed ? d[k] : (k == 0 ? 1u : 0u);
      for (uint32_t k = j; k < r.n; ++k) {
        uint32_t kl;
        const uint8_t* kp = ms_key(r.code, k, kl);
        write_record(reinterpret_cast<uint32_t*>(cand + (size_t)(idx++) * REC_SIZE), msg, rr, ss, kp, kl);
      }
    }
  }
}

__device__ __forceinline__ bool bit_at(const uint32_t* b, uint32_t i) { return (b[i >> 5] >> (i & 31u)) & 1u; }

__global__ void __launch_bounds__(WG) hkv_ms_resolve_kernel(const uint32_t* __restrict__ desc,
                                                            const uint64_t* __restrict__ off64, uint32_t n,
                                                            const uint32_t* __restrict__ cbits,
                                                            const uint32_t* __restrict__ kbits,
                                                            uint32_t* __restrict__ out_bits) {
  const uint32_t jx = blockIdx.x * WG + threadIdx.x;
  if (jx >= n) return;
  const uint32_t d0 = desc[2 * (size_t)jx];
  if (!(d0 & MS_OK)) return;
  const uint32_t mask = desc[2 * (size_t)jx + 1];
  const uint32_t m = d0 & 0xFFu, nk = (d0 >> 8) & 0xFFu, s_eff = (d0 >> 16) & 0xFFu;
  const uint64_t o = off64[jx];
  uint32_t start = (uint32_t)o;
  const uint32_t kbase = (uint32_t)(o >> 32);
  bool keys_ok = true;
  for (uint32_t k = 0; k < nk; ++k) keys_ok = keys_ok && bit_at(kbits, kbase + k);
  // countMulSig': start = index of candidate (j, j)
  uint32_t count = 0, j = 0;
  for (uint32_t k = 0; k < nk; ++k) {
    if (j >= s_eff) break;
    if (!((mask >> j) & 1u)) {  // TxSignatureEmpty: consumes the key and the signature
      ++j;
      continue;
    }
    if (bit_at(cbits, start + (k - j))) {
      ++count;
      start += nk - j;
      ++j;
    }
  }
  if (keys_ok && count == m) atomicOr(&out_bits[jx >> 5], 1u << (jx & 31u));
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
                       txs, tx_off, n_tx, hashes == TX_HASHES_WITNESS ? 1u : 0u, txt);
  else
    hipLaunchKernelGGL(hkv_tx_index_kernel, dim3(blocks_for(n_tx)), dim3(WG), 0, st, txs, tx_off, n_tx, txt);
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

// per-input desc words and record offsets; *total (zeroed here) ends as the
// number of candidate records | key-check records << 32
hipError_t launch_ms_scan(const uint8_t* txs, uint32_t n_tx, const uint32_t* txt, const uint8_t* scripts,
                          uint32_t scripts_len, const hkv_input_job* jobs, uint32_t n, int32_t forkid,
                          uint32_t* desc, uint64_t* off, uint64_t* counters, uint64_t* host_total, uint64_t seq,
                          hipStream_t st) {
  if (n == 0) return hipSuccess;  // the caller publishes the empty sum itself
  hipLaunchKernelGGL(hkv_ms_scan_kernel, dim3(blocks_for(n)), dim3(WG), 0, st, txs, n_tx, txt, scripts, scripts_len,
                     jobs, n, forkid, desc, off, reinterpret_cast<unsigned long long*>(counters),
                     reinterpret_cast<volatile unsigned long long*>(host_total), (unsigned long long)seq);
  return hipGetLastError();
}
hipError_t launch_ms_emit(const uint8_t* txs, uint32_t n_tx, const uint32_t* txt, const uint8_t* scripts,
                          uint32_t scripts_len, const hkv_input_job* jobs, uint32_t n, int32_t forkid,
                          const uint32_t* desc, const uint64_t* off, uint8_t* cand, uint8_t* keyrec, hipStream_t st) {
  hipLaunchKernelGGL(hkv_ms_emit_kernel, dim3(blocks_for(n)), dim3(WG), 0, st, txs, n_tx, txt, scripts, scripts_len,
                     jobs, n, forkid, desc, off, cand, keyrec);
  return hipGetLastError();
}
hipError_t launch_ms_resolve(const uint32_t* desc, const uint64_t* off, uint32_t n, const uint32_t* cbits,
                             const uint32_t* kbits, uint32_t* out_bits, hipStream_t st) {
  hipLaunchKernelGGL(hkv_ms_resolve_kernel, dim3(blocks_for(n)), dim3(WG), 0, st, desc, off, n, cbits, kbits,
                     out_bits);
  return hipGetLastError();
}

}  // namespace hkv
