/*
 * hkv.h — C ABI of libhkv: MI355X batch secp256k1 ECDSA verification.
 *
 * Drop-in boundary for the signature-check hot path of a haskoin-node based
 * validator. What each entry point replaces:
 *
 *   hkv_verify / hkv_verify_device
 *       replaces N per-input calls of haskoin-core
 *       `verifyHashSig :: Ctx -> Hash256 -> Sig -> PubKey -> Bool`
 *       (Haskoin.Crypto.Signature, haskoin-core-1.1.0 pinned at
 *       /root/reference/stack.yaml:10) in mode HKV_HASKOIN, and of
 *       secp256k1-haskell `verifySig` -> FFI `secp256k1_ecdsa_verify`
 *       (secp256k1-haskell-1.2.0, /root/reference/stack.yaml:9) in mode
 *       HKV_LIBSECP. Per-record parsing replaces `importPubKey`
 *       (secp256k1_ec_pubkey_parse) and `importCompactSig`
 *       (secp256k1_ecdsa_signature_parse_compact) so raw/adversarial bytes
 *       get exact reject parity. The reference itself never verifies; the
 *       batch is fed from the node's block/tx events
 *       (/root/reference/src/Haskoin/Node.hs:151-174, Peer.hs:309-344).
 *   hkv_open / hkv_close
 *       replaces secp256k1-haskell `createContext`/`withContext` (one
 *       shared read-only context per process).
 *   hkv_sighash / hkv_sighash_device
 *       replaces N calls of haskoin-core
 *       `txSigHash :: Network -> Tx -> Script -> Word64 -> Int -> SigHash -> Hash256`
 *       and `txSigHashForkId` (Haskoin.Script.SigHash) — the producer of
 *       every msg32 verifyHashSig checks.
 *   hkv_verify_std_inputs / hkv_verify_std_inputs_device
 *       replaces N calls of haskoin-core
 *       `verifyStdInput :: Network -> Ctx -> Tx -> Int -> ScriptOutput -> Word64 -> Bool`
 *       (Haskoin.Transaction.Builder) for P2PK / P2PKH / P2WPKH / multisig
 *       prevouts, bare or behind P2SH / P2WSH / P2SH-P2WSH: decodeTxSig
 *       (strict DER, low S, hashtype), the HASH160 / SHA-256 script checks,
 *       legacy or BIP143 sighash, verifyHashSig and the countMulSig walk,
 *       all on device.
 *   hkv_check_headers / hkv_check_headers_device
 *       replaces the per-header part of haskoin-core `connectBlocks` reached
 *       from importHeaders (/root/reference/src/Haskoin/Node/Chain.hs:500-520):
 *       headerHash, isValidPOW (decodeCompact) and the prev-hash link.
 *
 * Streams: device-form calls enqueue on the caller's stream; calls on one
 * device share its scratch buffers, so each call is ordered after the
 * previous call on that device (an event wait), whatever stream either used.
 *
 * Conventions: no C++ exceptions cross this boundary; every function that
 * can fail returns 0 (HKV_OK) or a negative hkv_err. A verdict is never an
 * error: malformed records simply get bit 0. Verdict bit i of the output is
 * bit (i % 32) of word (i / 32); 1 = accept.
 *
 * Record layout (HKV_RECORD_SIZE = 168 bytes, 8-byte aligned array):
 *   [0,32)    msg32   (the Hash256 bytes as secp256k1 `msg32`, no reversal)
 *   [32,64)   r       big-endian (compact signature first half)
 *   [64,96)   s       big-endian
 *   [96]      pubkey length in bytes (33 or 65 are the only valid ones)
 *   [97,162)  pubkey  SEC1 bytes (02/03 compressed, 04 uncompressed,
 *                     06/07 hybrid), zero padded
 *   [162,168) zero padding
 */
#ifndef HKV_H
#define HKV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HKV_RECORD_SIZE 168

/* verify modes */
#define HKV_LIBSECP 0u /* secp256k1_ecdsa_verify: high-S rejected        */
#define HKV_HASKOIN 1u /* verifyHashSig: normalize to low-S, then verify */

enum hkv_err {
  HKV_OK = 0,
  HKV_E_ARG = -1,      /* bad argument (NULL, n > capacity, bad mode)   */
  HKV_E_NODEV = -2,    /* no usable gfx950 device                       */
  HKV_E_OOM = -3,      /* device or pinned host allocation failed       */
  HKV_E_HIP = -4,      /* HIP runtime error (see hkv_last_hip_error)     */
  HKV_E_INTERNAL = -5, /* self-check failed at open                      */
};

typedef struct hkv_ctx hkv_ctx;
typedef struct hkv_batch hkv_batch;

/* open flags */
#define HKV_OPEN_NO_SELFCHECK 1u /* skip the known-answer self-check at open */

/* Open a context on the first n_gpus visible devices (n_gpus <= 0: all).
 * Builds the fixed-base tables on every device and, unless flags has
 * HKV_OPEN_NO_SELFCHECK, verifies 256 generated signatures per device
 * (HKV_E_INTERNAL if any is rejected). */
int hkv_open(int n_gpus, uint32_t flags, hkv_ctx** out);
/* Open on an explicit list of HIP device ordinals (one process per GPU:
 * pass {LOCAL_RANK}). Context device index k refers to device_ids[k]. */
int hkv_open_devices(const int* device_ids, int n_ids, uint32_t flags, hkv_ctx** out);
void hkv_close(hkv_ctx* ctx);
int hkv_ctx_num_devices(const hkv_ctx* ctx);
/* Device k of the context still takes host-batch shards (1) or has failed
 * one with a device fault (0); negative on a bad argument. */
int hkv_device_healthy(hkv_ctx* ctx, int dev);
/* Give device k host-batch shards again (after the caller has decided it
 * recovered, e.g. a hipDeviceReset or a passing probe batch). */
int hkv_device_reset_health(hkv_ctx* ctx, int dev);
/* Host-batch shards device k has failed (0 or 1: a failed device gets no
 * more shards); negative on a bad argument. */
int hkv_device_failures(hkv_ctx* ctx, int dev);
/* Test hook: device k's next host-batch shard fails — HKV_FAIL_ENQUEUE
 * before anything is enqueued, HKV_FAIL_JOIN after its work completed — as a
 * HIP error would, exercising the failover of hkv_verify / hkv_verify_host;
 * HKV_FAIL_ALLOC as a staging allocation would (HKV_E_OOM: the call fails,
 * the device stays healthy). */
#define HKV_FAIL_NONE 0u
#define HKV_FAIL_ENQUEUE 1u
#define HKV_FAIL_JOIN 2u
#define HKV_FAIL_ALLOC 3u
/* HKV_FAIL_TAIL: the next multisig tail launch on device k gives up the
 * first wait of its work queue at a phase transition (the timeout branch of a
 * wait for the phase before, taken at once without looking at the count), so
 * the fault reporting below can be tested; deterministic for any batch with a
 * multisig input. */
#define HKV_FAIL_TAIL 4u
int hkv_debug_fail_device(hkv_ctx* ctx, int dev, uint32_t when);
/* Test hooks of the multisig record windows (hkv_verify_std_inputs*): the
 * tail runs a chunk's candidate and key-check records in rounds through two
 * windows of at most 2,752,512 + 442,368 records (~512 MiB); _window sets
 * smaller capacities for device dev's later calls (records, rounded up to
 * 64; 0 = the default), so tests can force many rounds on small batches;
 * _scratch reports the bytes the windows hold allocated on device dev. */
int hkv_debug_ms_window(hkv_ctx* ctx, int dev, uint32_t cand_records, uint32_t key_records);
int hkv_debug_ms_scratch(hkv_ctx* ctx, int dev, size_t* bytes);

/* Pinned host record buffer with room for max_n records. */
int hkv_batch_alloc(hkv_ctx* ctx, size_t max_n, hkv_batch** out);
void hkv_batch_free(hkv_batch* b);
uint8_t* hkv_batch_records(hkv_batch* b);
size_t hkv_batch_capacity(const hkv_batch* b);

/* Verify records [0, n) of the batch. Shards contiguous 64-aligned index
 * ranges across the context's healthy devices; writes ceil(n/32) words.
 * Blocking. Failover: when a device's shard fails with a device fault (a
 * HIP error while enqueueing or while waiting for it: HKV_E_HIP), that device
 * is marked unhealthy until hkv_device_reset_health and its shard is
 * re-verified on the devices still healthy; the call fails only when none is
 * left (the last error, or HKV_E_NODEV once every device of the context is
 * unhealthy). An allocation failure (HKV_E_OOM) is returned as is: no device
 * changes health and nothing is re-sharded. */
int hkv_verify(hkv_ctx* ctx, hkv_batch* b, size_t n, uint32_t mode, uint32_t* verdict_bits);

/* Same, from any host memory (copied through the context's staging). */
int hkv_verify_host(hkv_ctx* ctx, const uint8_t* records, size_t n, uint32_t mode, uint32_t* verdict_bits);

/* Device-resident form: d_records (n * 168 bytes) and d_bits
 * (>= ceil(n/64)*2 words) live in HBM of the context's device `dev`; work is
 * enqueued on `hip_stream` and NOT synchronised. In every *_device entry point
 * NULL means the null (default) stream, which is ordered against the
 * blocking streams of the process, e.g. PyTorch's default stream.
 * Used by one-process-per-GPU sharding (bench.py) and by zero-copy callers. */
int hkv_verify_device(hkv_ctx* ctx, int dev, const void* d_records, size_t n, uint32_t mode,
                      uint32_t* d_bits, void* hip_stream);

/* Synthetic valid records (keyless construction) written
 * to device memory: pubkeys from a pool of `pool_size` keys, a per-mille
 * share of uncompressed keys, all signatures low-S. Enqueued on hip_stream. */
int hkv_gen_records_device(hkv_ctx* ctx, int dev, uint64_t seed, size_t n, uint32_t pool_size,
                           uint32_t uncompressed_permille, void* d_records, void* hip_stream);
/* A slice of one synthetic batch: records [index0, index0 + n) of the batch
 * `seed` (record k depends on (seed, k) only, and the key pool on seed only,
 * so ranks generating contiguous slices produce exactly the one-process
 * batch; BASELINE configs[4]). invalid_permille of the records are mutated
 * into a class that rejects in both modes: a flipped bit of msg32, r or s,
 * another key of the pool, or the negated key. d_labels (NULL or
 * ceil(n/64)*2 words): bit i = record index0 + i is valid by construction.
 * hkv_gen_records_device is this call with index0 = 0, invalid_permille = 0.
 * CPU restatement (test infrastructure): oracle/hkv_oracle.c hkvo_gen_batch. */
int hkv_gen_batch_device(hkv_ctx* ctx, int dev, uint64_t seed, uint64_t index0, size_t n, uint32_t pool_size,
                         uint32_t uncompressed_permille, uint32_t invalid_permille, void* d_records,
                         uint32_t* d_labels, void* hip_stream);

/* ------------------------------------------------------------------------
 * Signature hashes and standard inputs on device (SURVEY.md §8(a) a7-a9,
 * §8(f) row 2).
 *
 * A tx batch is a buffer of serialised transactions (wire form, BIP144
 * witness form allowed) with n_tx + 1 byte offsets (tx t occupies
 * bytes[offsets[t], offsets[t+1])), plus a pool of scripts the jobs refer to
 * by (offset, length). In the *_device entry points every pointer of the
 * hkv_txs and the job / output arrays live in HBM of device `dev`.
 * ------------------------------------------------------------------------ */
typedef struct hkv_txs {
  const uint8_t* bytes;
  const uint32_t* offsets; /* n_tx + 1 entries, non-decreasing, < 2^32 */
  uint32_t n_tx;
  const uint8_t* scripts;
  uint32_t scripts_len;
} hkv_txs;

#define HKV_SIGHASH_LEGACY 0u /* haskoin-core txSigHash                  */
#define HKV_SIGHASH_FORKID 1u /* haskoin-core txSigHashForkId (BIP143)   */
#define HKV_NO_FORKID (-1)    /* network without a fork id (BTC)         */

/* One call of txSigHash / txSigHashForkId:
 *   txSigHash net tx scriptCode value input sighash
 * scriptCode = scripts[script_off, script_off + script_len). 32 bytes. */
typedef struct hkv_sighash_job {
  uint32_t tx;
  uint32_t input;
  uint32_t script_off;
  uint32_t script_len;
  uint64_t value;   /* prevout amount (BIP143 form) */
  uint32_t sighash; /* SigHash word */
  uint32_t kind;    /* HKV_SIGHASH_LEGACY / HKV_SIGHASH_FORKID */
} hkv_sighash_job;

/* per-job status (hkv_sighash*): the hash of a failed job is all zero */
#define HKV_SH_OK 0u
#define HKV_SH_BAD_TX 1u    /* the tx does not parse within its bounds   */
#define HKV_SH_BAD_INPUT 2u /* input index >= number of inputs           */
#define HKV_SH_BAD_REF 3u   /* tx index or script range out of the batch */

/* One standard input for verifyStdInput: input `input` of tx `tx` spends a
 * prevout with scriptPubKey = scripts[script_off, +script_len) and amount
 * `value`. Templates (haskoin verifyStdInput): P2PK (21 <33> ac / 41 <65> ac),
 * P2PKH, P2WPKH, multisig (OP_m <keys> OP_n OP_CHECKMULTISIG, keys as direct
 * 21 / 41 pushes), each of P2PK / P2PKH / P2WPKH / P2WSH / multisig behind
 * P2SH, and P2PK / P2PKH / multisig behind P2WSH (native or P2SH-nested);
 * any other prevout script verifies false. 24 bytes. */
typedef struct hkv_input_job {
  uint32_t tx;
  uint32_t input;
  uint32_t script_off;
  uint32_t script_len;
  uint64_t value;
} hkv_input_job;

/* Batch txSigHash / txSigHashForkId (forkid: HKV_NO_FORKID or the network's
 * fork id, e.g. 0 for BCH). out32: n * 32 bytes; status: n bytes or NULL.
 * Host memory; runs on the context's first device. Blocking. */
int hkv_sighash(hkv_ctx* ctx, const hkv_txs* txs, const hkv_sighash_job* jobs, size_t n, int32_t forkid,
                uint8_t* out32, uint8_t* status);
/* Device form: hash j goes to d_out + j * out_stride (out_stride % 4 == 0;
 * 168 writes the msg32 field of verify records in place). Enqueued on
 * hip_stream, not synchronised. */
int hkv_sighash_device(hkv_ctx* ctx, int dev, const hkv_txs* d_txs, const hkv_sighash_job* d_jobs, size_t n,
                       int32_t forkid, uint8_t* d_out, size_t out_stride, uint8_t* d_status, void* hip_stream);
/* The non-ECDSA half of verifyStdInput on device: one 168-byte verify record
 * per single-signature input (all-zero when the template / DER / HASH160
 * checks fail, and for multisig inputs, which only the verify entry points
 * below resolve). */
int hkv_std_inputs_device(hkv_ctx* ctx, int dev, const hkv_txs* d_txs, const hkv_input_job* d_jobs, size_t n,
                          int32_t forkid, void* d_records, void* hip_stream);
/* Full batch verifyStdInput: extraction + ECDSA (HKV_HASKOIN semantics).
 * d_records: scratch of n * 168 bytes; verdict bit i in d_bits
 * (>= ceil(n/64)*2 words). Multisig inputs follow haskoin-core countMulSig:
 * every (signature j, key k >= j) pair the walk could compare is verified as
 * its own record, every key of the script is parse-checked, and the walk is
 * replayed on device (count == m and all keys valid).
 * ASYNCHRONOUS: everything is enqueued on hip_stream and the call returns
 * without waiting for any of it (the batch's multisig record count stays on
 * the device: the tail, one launch after the verify on every path, reads it
 * and does nothing when it is 0), so a
 * caller may enqueue block k+1 while block k verifies, and hip_stream may be
 * gated on events recorded after the call. A batch of at most one resident
 * grid (262,144 inputs on an MI355X) runs in chunks of half a grid (131,072),
 * a larger one in chunks of up to 2^20 inputs (the environment variable
 * HKV_STD_CHUNK, read at hkv_open, overrides the 2^20: a test hook). Multisig
 * scratch per chunk: the verdict bits by the 16-of-16 bound
 * (136 candidate + 16 key-check bits per input) and the 168-B records in two
 * windows, the bound or at most 2,752,512 + 442,368 records (~512 MiB), which
 * the tail runs in rounds when a chunk's records exceed them: ~0.1 GB for a
 * 4,000-input block, ~512 MiB for any larger chunk, multisig or not,
 * allocated on first use and kept.
 * A multisig tail whose work-queue wait gave up leaves its multisig
 * verdicts at 0 and reports HKV_STATUS_TAIL_FAULT (below) — this form only
 * through hkv_device_fault; use the _status form to get it per call.
 * n <= 0xFFFFFF00. */
int hkv_verify_std_inputs_device(hkv_ctx* ctx, int dev, const hkv_txs* d_txs, const hkv_input_job* d_jobs, size_t n,
                                 int32_t forkid, void* d_records, uint32_t* d_bits, void* hip_stream);
/* Status bits a verify call reports (hkv_verify_std_inputs_device_status,
 * hkv_device_fault). HKV_STATUS_TAIL_FAULT: a wait of the multisig tail's
 * work queue gave up (seconds; the queue needs no co-residency, so only a
 * hung or preempted workgroup, or the HKV_FAIL_TAIL test hook, causes it):
 * some multisig inputs of the batch were left rejected whatever their
 * signatures. Never a false accept. */
#define HKV_STATUS_TAIL_FAULT 1u
/* hkv_verify_std_inputs_device with a status word: d_status (device memory
 * of `dev`, or NULL) gets the call's HKV_STATUS_* bits ORed in on hip_stream,
 * so an asynchronous caller learns of a fault when it reads its verdicts.
 * The caller zeroes it. */
int hkv_verify_std_inputs_device_status(hkv_ctx* ctx, int dev, const hkv_txs* d_txs, const hkv_input_job* d_jobs,
                                        size_t n, int32_t forkid, void* d_records, uint32_t* d_bits,
                                        uint32_t* d_status, void* hip_stream);
/* Read and clear device dev's sticky fault latch: HKV_STATUS_* bits of every
 * verify call on the device since the last read (any entry point). Waits for
 * the device's enqueued calls. */
int hkv_device_fault(hkv_ctx* ctx, int dev, uint32_t* fault);
/* Host-memory form of the above; writes ceil(n/32) verdict words. Blocking.
 * Same bound on n. HKV_E_INTERNAL if this call's multisig tail reported
 * HKV_STATUS_TAIL_FAULT (some multisig verdicts stayed 0). */
int hkv_verify_std_inputs(hkv_ctx* ctx, const hkv_txs* txs, const hkv_input_job* jobs, size_t n, int32_t forkid,
                          uint32_t* verdict_bits);

/* ---------------------------------------------------------------------------
 * Header batches: the data-parallel part of
 * importHeaders (/root/reference/src/Haskoin/Node/Chain.hs:500-520), which
 * hands up to 2,000 headers per peer message to haskoin-core connectBlocks
 * [dep]. Per header: headerHash (SHA-256d of the 80-byte wire form) and
 * isValidPOW net h = target > 0 && !overflow && target <= powLimit &&
 * headerPOW h <= target, with (target, overflow) = decodeCompact h.bits;
 * plus the batch linkage connectBlocks relies on (prev field of header i
 * == headerHash of header i-1). The chain-context checks (median time past,
 * retarget / nextWorkRequired, checkpoints, BIP34) stay on the host.
 * ------------------------------------------------------------------------ */
#define HKV_HDR_POW_OK 0x01u           /* isValidPOW                               */
#define HKV_HDR_LINK_OK 0x02u          /* prev == hash of the previous header      */
#define HKV_HDR_NEGATIVE 0x04u         /* decodeCompact sign bit with nonzero word */
#define HKV_HDR_OVERFLOW 0x08u         /* decodeCompact overflow                   */
#define HKV_HDR_ZERO_TARGET 0x10u      /* target == 0                              */
#define HKV_HDR_ABOVE_LIMIT 0x20u      /* target > powLimit                        */
#define HKV_HDR_HASH_ABOVE 0x40u       /* headerPOW > target                       */

/* headers: n * 80 wire bytes. pow_limit: 32 bytes, little-endian integer
 * (the network's powLimit). prev_hash: 32 bytes in internal (digest) order,
 * the hash header 0 must extend, or NULL (header 0 then counts as linked).
 * hashes_out: n * 32 bytes (digest order, i.e. headerHash's serialisation);
 * status: n bytes of HKV_HDR_* flags. Host memory, first device, blocking. */
int hkv_check_headers(hkv_ctx* ctx, const uint8_t* headers, size_t n, const uint8_t* pow_limit,
                      const uint8_t* prev_hash, uint8_t* hashes_out, uint8_t* status);
/* Device form: every pointer in HBM of device `dev`; enqueued on hip_stream,
 * not synchronised. */
int hkv_check_headers_device(hkv_ctx* ctx, int dev, const uint8_t* d_headers, size_t n, const uint8_t* d_pow_limit,
                             const uint8_t* d_prev_hash, uint8_t* d_hashes, uint8_t* d_status, void* hip_stream);

/* ---------------------------------------------------------------------------
 * Block merkle roots: haskoin-core buildMerkleRoot [dep, haskoin-core-1.1.0
 * Haskoin.Block.Merkle], as the reference's block test applies it
 * (/root/reference/test/Haskoin/NodeSpec.hs:185-193: b.header.merkle ==
 * buildMerkleRoot (txHash <$> b.txs)) to blocks from getBlocks
 * (src/Haskoin/Node/Peer.hs:309-344). Batched over many blocks.
 * txids: offsets[n_blocks] * 32 bytes, digest order (txHash serialisation);
 * block b owns txids [offsets[b], offsets[b+1]). roots_out: n_blocks * 32
 * (an empty block gets 32 zero bytes). mutated: n_blocks bytes, 1 when two
 * equal hashes are paired at some level (CVE-2012-2459 duplicate-tx form).
 * Host memory, first device, blocking. */
int hkv_merkle_roots(hkv_ctx* ctx, const uint8_t* txids, const uint32_t* offsets, size_t n_blocks,
                     uint8_t* roots_out, uint8_t* mutated);
/* Device form: every pointer in HBM of device `dev`; d_scratch holds
 * offsets[n_blocks] * 32 bytes and may alias nothing else; 16-byte aligned
 * txids / scratch / roots. Enqueued on hip_stream, not synchronised. */
int hkv_merkle_roots_device(hkv_ctx* ctx, int dev, const uint8_t* d_txids, const uint32_t* d_offsets,
                            size_t n_blocks, uint8_t* d_scratch, uint8_t* d_roots, uint8_t* d_mutated,
                            void* hip_stream);

/* Synthetic-data hooks (block-mix generator, off the verify path):
 * n random private keys -> d_priv (n*32, big-endian), compressed public keys
 * d_pub (n*33) and their HASH160 d_h160 (n*20);
 * ECDSA signatures (r||s big-endian, low S, random nonces) of msg j
 * (d_msg + j*msg_stride) with key d_key_idx[j] -> d_sig (n*64). */
int hkv_gen_keys_device(hkv_ctx* ctx, int dev, uint64_t seed, size_t n, uint8_t* d_priv, uint8_t* d_pub,
                        uint8_t* d_h160, void* hip_stream);
int hkv_gen_sign_device(hkv_ctx* ctx, int dev, uint64_t seed, size_t n, const uint8_t* d_priv,
                        const uint32_t* d_key_idx, const uint8_t* d_msg, size_t msg_stride, uint8_t* d_sig,
                        void* hip_stream);

/* Known-answer hook for the tests: applies op (see hkv_internal.h) to n
 * pairs of 8-limb little-endian operands in device memory; 16 words out. */
int hkv_debug_op(hkv_ctx* ctx, int dev, uint32_t op, size_t n, const uint32_t* d_a, const uint32_t* d_b,
                 uint32_t* d_out, void* hip_stream);

/* Per-kernel timing with HIP events recorded on the launch stream around the
 * prologue and ecmult kernels of every subsequent verify (bench.py's roofline).
 * read: synchronises, returns summed milliseconds and the launch count, resets. */
int hkv_profile_enable(hkv_ctx* ctx, int on);
int hkv_profile_read(hkv_ctx* ctx, int dev, double* prologue_ms, double* ecmult_ms, uint64_t* launches);
/* Shader clock (MHz) block 0 of the last profiled ecmult launch ran at:
 * clock64() / wall_clock64() deltas around its work (so the roofline can be
 * priced at the measured clock). Synchronises the device. */
int hkv_profile_clock(hkv_ctx* ctx, int dev, double* sclk_mhz);

/* Phase stamps of workgroup 0 of the last profiled small-batch (split)
 * launch: n <= 12 constant-rate clock values (tick_ns nanoseconds per tick)
 * at its phase boundaries — 0 start, 1 k1 table built, 2 past barrier P,
 * 3 k1 chain done, 4 past barrier A, 5 join done, 6 signature parse done,
 * 7 u1 G done, 8 key sqrt done, 9 k2 table built, 10 k2 chain done.
 * Synchronises the device. */
int hkv_profile_phases(hkv_ctx* ctx, int dev, uint64_t* stamps, size_t n, double* tick_ns);

/* Per-workgroup (start, end) constant-rate clock stamps of the last profiled
 * block-kernel launch (a block: at most 16 signatures per CU): stamps[2g] =
 * workgroup g's first instruction, stamps[2g + 1] = its last; n_groups <=
 * 4096. Where the launch's span goes beyond workgroup 0's phase stamps.
 * Synchronises the device. (Measurement only; no reference counterpart.) */
int hkv_profile_group_stamps(hkv_ctx* ctx, int dev, uint64_t* stamps, size_t n_groups, double* tick_ns);

const char* hkv_strerror(int err);
const char* hkv_last_hip_error(void);
int hkv_device_count(void);
/* ABI version: (major << 16) | minor */
uint32_t hkv_version(void);

#ifdef __cplusplus
}
#endif
#endif /* HKV_H */
