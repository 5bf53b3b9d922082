// hkv_sighash_dev.h — device helpers of the signature-hash path, shared by
// hkv_sighash.hip (the sighash / standard-input / multisig kernels) and
// hkv_kernels.hip (the small-batch kernel that computes each input's sighash
// on its signature wave, hkv_pair_split_kernel<true>): byte readers, the
// preimage generator and block-synchronous SHA-256 stream, tx index rows,
// the per-job legacy / BIP143 setup, strict DER and the template predicates.
// Reference semantics: see hkv_sighash.hip's header.
#pragma once
#include "hkv_hash.h"
#include "hkv_scalar.h"
#include "hkv_layout.h"
#include "../../include/hkv.h"

namespace hkv {
// ---------------------------------------------------------------------------
// byte-level readers
// ---------------------------------------------------------------------------
// bounds-checked varint (the tx index parse); values >= 2^32 fail (no such
// count or length fits a batch)
HKV_DEV bool rd_varint(const uint8_t* p, uint32_t& off, uint32_t end, uint32_t& v) {
  if (off >= end) return false;
  const uint32_t t = p[off];
  if (t < 0xFDu) {
    v = t;
    off += 1;
    return true;
  }
  const uint32_t w = t == 0xFDu ? 2u : (t == 0xFEu ? 4u : 8u);
  if (end - off < 1u + w) return false;
  uint32_t lo = 0, hi = 0;
  for (uint32_t k = 0; k < w; ++k) {
    const uint32_t b = p[off + 1 + k];
    if (k < 4) lo |= b << (8 * k);
    else hi |= b;
  }
  if (hi) return false;
  v = lo;
  off += 1 + w;
  return true;
}
// unchecked varint on a structure the index kernel already validated
HKV_DEV uint32_t get_varint(const uint8_t* p, uint32_t& off) {
  const uint32_t t = p[off];
  if (t < 0xFDu) {
    off += 1;
    return t;
  }
  if (t == 0xFDu) {
    const uint32_t v = p[off + 1] | (p[off + 2] << 8);
    off += 3;
    return v;
  }
  const uint32_t v = p[off + 1] | (p[off + 2] << 8) | (p[off + 3] << 16) | ((uint32_t)p[off + 4] << 24);
  off += t == 0xFEu ? 5u : 9u;
  return v;
}
HKV_DEV uint64_t varint_lit(uint32_t v, uint32_t& n) {
  if (v < 0xFDu) {
    n = 1;
    return v;
  }
  if (v <= 0xFFFFu) {
    n = 3;
    return 0xFDull | ((uint64_t)v << 8);
  }
  n = 5;
  return 0xFEull | ((uint64_t)v << 8);
}

// Script op scan (haskoin scriptOps): true if every push fits; counts
// single-byte OP_CODESEPARATOR (0xab) ops outside push data.
HKV_DEV bool script_scan(const uint8_t* s, uint32_t len, uint32_t& n_sep) {
  uint32_t off = 0;
  n_sep = 0;
  while (off < len) {
    const uint32_t op = s[off];
    uint64_t ol = 1;
    if (op >= 1u && op <= 75u) {
      ol = 1 + op;
    } else if (op == 0x4Cu) {
      if (len - off < 2) return false;
      ol = 2 + (uint64_t)s[off + 1];
    } else if (op == 0x4Du) {
      if (len - off < 3) return false;
      ol = 3 + (uint64_t)(s[off + 1] | (s[off + 2] << 8));
    } else if (op == 0x4Eu) {
      if (len - off < 5) return false;
      ol = 5 + (uint64_t)(s[off + 1] | (s[off + 2] << 8) | (s[off + 3] << 16) | ((uint32_t)s[off + 4] << 24));
    } else if (op == 0xABu) {
      ++n_sep;
    }
    if (ol > (uint64_t)(len - off)) return false;
    off += (uint32_t)ol;
  }
  return true;
}
HKV_DEV uint32_t script_op_len(const uint8_t* s, uint32_t off) {
  const uint32_t op = s[off];
  if (op >= 1u && op <= 75u) return 1 + op;
  if (op == 0x4Cu) return 2 + s[off + 1];
  if (op == 0x4Du) return 3 + (s[off + 1] | (s[off + 2] << 8));
  if (op == 0x4Eu) return 5 + (s[off + 1] | (s[off + 2] << 8) | (s[off + 3] << 16) | ((uint32_t)s[off + 4] << 24));
  return 1;
}

// ---------------------------------------------------------------------------
// preimage generator
// ---------------------------------------------------------------------------
enum : uint32_t {
  PH_DONE = 0,
  // txSigHash (legacy) preimage
  PH_L_VER, PH_L_NIN, PH_L_IN_OP, PH_L_IN_SLEN, PH_L_IN_CODE, PH_L_IN_SEQ, PH_L_OUTS, PH_L_BLANK_A,
  PH_L_BLANK_B, PH_L_LOCK, PH_L_SH,
  // output walker (value, canonical script length, script), returns to g.ret
  PH_O_VAL, PH_O_LEN, PH_O_SCRIPT,
  // txSigHashForkId (BIP143) preimage
  PH_F_VER, PH_F_HASH, PH_F_OUTPOINT, PH_F_SLEN, PH_F_CODE, PH_F_VALUE, PH_F_SEQ, PH_F_HO, PH_F_LOCK, PH_F_SH,
  // per-tx BIP143 parts
  PH_P_IN, PH_S_IN,
  // a single byte range
  PH_RANGE,
};
constexpr uint32_t GF_ACP = 1u, GF_ALL = 2u, GF_NONE = 4u, GF_SINGLE = 8u, GF_STRIP = 16u, GF_P2WPKH = 32u;

struct Gen {
  const uint8_t* src;  // current piece: byte range (src != null) or literal
  uint64_t lit;
  uint32_t rem;
  uint32_t phase, ret;
  const uint8_t* T;    // tx buffer (absolute offsets below)
  uint32_t start, nin, nout, ins, outs_first, lock;
  uint32_t i, shn, flags;
  uint32_t j, ioff, seq_at, cnt;
  uint32_t ooff, ocnt, osl, oscr;
  uint32_t in_i, in_i_seq, single_off;
  const uint8_t* code;
  uint32_t code_len, code_out, ccur;
  uint64_t value;
  const uint32_t* hp;  // 32-byte hashes in digest byte order (null = zeros)
  const uint32_t* hs;
  const uint32_t* ho;
};

HKV_DEV void gen_clear(Gen& g) {
  g.src = nullptr; g.lit = 0; g.rem = 0; g.phase = PH_DONE; g.ret = PH_DONE; g.T = nullptr;
  g.start = g.nin = g.nout = g.ins = g.outs_first = g.lock = 0;
  g.i = g.shn = g.flags = 0; g.j = g.ioff = g.seq_at = g.cnt = 0;
  g.ooff = g.ocnt = g.osl = g.oscr = 0; g.in_i = g.in_i_seq = g.single_off = 0;
  g.code = nullptr; g.code_len = g.code_out = g.ccur = 0; g.value = 0;
  g.hp = g.hs = g.ho = nullptr;
}
HKV_DEV void piece_copy(Gen& g, const uint8_t* p, uint32_t n) { g.src = p; g.rem = n; }
HKV_DEV void piece_lit(Gen& g, uint64_t v, uint32_t n) { g.src = nullptr; g.lit = v; g.rem = n; }
HKV_DEV void piece_varint(Gen& g, uint32_t v) {
  uint32_t n;
  const uint64_t l = varint_lit(v, n);
  piece_lit(g, l, n);
}
HKV_DEV void piece_hash(Gen& g, const uint32_t* h, uint32_t q) {
  piece_lit(g, h ? ((uint64_t)h[2 * q] | ((uint64_t)h[2 * q + 1] << 32)) : 0ull, 8);
}

// Set up the next non-empty piece, or reach PH_DONE.
HKV_DEV void gen_advance(Gen& g) {
  const uint8_t* T = g.T;
  switch (g.phase) {
    // ---- txSigHash: serialize (tx copy) ++ LE32 sighash ----
    case PH_L_VER: piece_copy(g, T + g.start, 4); g.phase = PH_L_NIN; break;
    case PH_L_NIN:
      piece_varint(g, (g.flags & GF_ACP) ? 1u : g.nin);
      g.j = (g.flags & GF_ACP) ? g.i : 0u;
      g.ioff = (g.flags & GF_ACP) ? g.in_i : g.ins;
      g.phase = PH_L_IN_OP;
      break;
    case PH_L_IN_OP: {
      piece_copy(g, T + g.ioff, 36);
      uint32_t o = g.ioff + 36;
      const uint32_t sl = get_varint(T, o);
      g.seq_at = o + sl;
      g.phase = PH_L_IN_SLEN;
      break;
    }
    case PH_L_IN_SLEN:
      if (g.j == g.i) {
        piece_varint(g, g.code_out);
        g.ccur = 0;
        g.phase = PH_L_IN_CODE;
      } else {
        piece_lit(g, 0, 1);
        g.phase = PH_L_IN_SEQ;
      }
      break;
    case PH_L_IN_CODE:
      if (!(g.flags & GF_STRIP)) {
        piece_copy(g, g.code, g.code_len);
        g.phase = PH_L_IN_SEQ;
        break;
      }
      while (g.ccur < g.code_len) {  // drop OP_CODESEPARATOR ops
        const uint32_t op = g.code[g.ccur];
        const uint32_t ol = script_op_len(g.code, g.ccur);
        if (op == 0xABu) {
          g.ccur += 1;
          continue;
        }
        piece_copy(g, g.code + g.ccur, ol);
        g.ccur += ol;
        return;
      }
      g.phase = PH_L_IN_SEQ;
      break;
    case PH_L_IN_SEQ:
      if ((g.flags & GF_ALL) || g.j == g.i) piece_copy(g, T + g.seq_at, 4);
      else piece_lit(g, 0, 4);
      if (g.flags & GF_ACP) {
        g.phase = PH_L_OUTS;
      } else {
        g.j += 1;
        g.ioff = g.seq_at + 4;
        g.phase = g.j < g.nin ? PH_L_IN_OP : PH_L_OUTS;
      }
      break;
    case PH_L_OUTS:
      if (g.flags & GF_ALL) {
        piece_varint(g, g.nout);
        g.ooff = g.outs_first;
        g.ocnt = g.nout;
        g.ret = PH_L_LOCK;
        g.phase = PH_O_VAL;
      } else if (g.flags & GF_NONE) {
        piece_lit(g, 0, 1);
        g.phase = PH_L_LOCK;
      } else {
        piece_varint(g, g.i + 1);
        g.cnt = 0;
        g.phase = PH_L_BLANK_A;
      }
      break;
    case PH_L_BLANK_A:  // SINGLE: i outputs (2^64-1, empty script), then output i
      if (g.cnt < g.i) {
        piece_lit(g, ~0ull, 8);
        g.phase = PH_L_BLANK_B;
      } else {
        g.ooff = g.single_off;
        g.ocnt = 1;
        g.ret = PH_L_LOCK;
        g.phase = PH_O_VAL;
      }
      break;
    case PH_L_BLANK_B: piece_lit(g, 0, 1); g.cnt += 1; g.phase = PH_L_BLANK_A; break;
    case PH_L_LOCK: piece_copy(g, T + g.lock, 4); g.phase = PH_L_SH; break;
    case PH_L_SH: piece_lit(g, g.shn, 4); g.phase = PH_DONE; break;
    // ---- outputs ----
    case PH_O_VAL: {
      if (g.ocnt == 0) {
        g.phase = g.ret;
        break;
      }
      piece_copy(g, T + g.ooff, 8);
      uint32_t o = g.ooff + 8;
      g.osl = get_varint(T, o);
      g.oscr = o;
      g.phase = PH_O_LEN;
      break;
    }
    case PH_O_LEN: piece_varint(g, g.osl); g.phase = PH_O_SCRIPT; break;
    case PH_O_SCRIPT:
      piece_copy(g, T + g.oscr, g.osl);
      g.ooff = g.oscr + g.osl;
      g.ocnt -= 1;
      g.phase = PH_O_VAL;
      break;
    // ---- txSigHashForkId ----
    case PH_F_VER: piece_copy(g, T + g.start, 4); g.cnt = 0; g.phase = PH_F_HASH; break;
    case PH_F_HASH:
      piece_hash(g, g.cnt < 4 ? g.hp : g.hs, g.cnt & 3u);
      g.cnt += 1;
      if (g.cnt == 8) g.phase = PH_F_OUTPOINT;
      break;
    case PH_F_OUTPOINT: piece_copy(g, T + g.in_i, 36); g.phase = PH_F_SLEN; break;
    case PH_F_SLEN: piece_varint(g, g.code_len); g.cnt = 0; g.phase = PH_F_CODE; break;
    case PH_F_CODE:
      if (!(g.flags & GF_P2WPKH)) {
        piece_copy(g, g.code, g.code_len);
        g.phase = PH_F_VALUE;
      } else if (g.cnt == 0) {  // scriptCode 76 a9 14 <h20> 88 ac of a P2WPKH program
        piece_lit(g, 0x14A976ull, 3);
        g.cnt = 1;
      } else if (g.cnt == 1) {
        piece_copy(g, g.code, 20);
        g.cnt = 2;
      } else {
        piece_lit(g, 0xAC88ull, 2);
        g.phase = PH_F_VALUE;
      }
      break;
    case PH_F_VALUE: piece_lit(g, g.value, 8); g.phase = PH_F_SEQ; break;
    case PH_F_SEQ: piece_copy(g, T + g.in_i_seq, 4); g.cnt = 0; g.phase = PH_F_HO; break;
    case PH_F_HO:
      piece_hash(g, g.ho, g.cnt);
      g.cnt += 1;
      if (g.cnt == 4) g.phase = PH_F_LOCK;
      break;
    case PH_F_LOCK: piece_copy(g, T + g.lock, 4); g.phase = PH_F_SH; break;
    case PH_F_SH: piece_lit(g, g.shn, 4); g.phase = PH_DONE; break;
    // ---- hashPrevouts / hashSequence inputs ----
    case PH_P_IN: {
      if (g.j == g.nin) {
        g.phase = PH_DONE;
        break;
      }
      piece_copy(g, T + g.ioff, 36);
      uint32_t o = g.ioff + 36;
      const uint32_t sl = get_varint(T, o);
      g.ioff = o + sl + 4;
      g.j += 1;
      break;
    }
    case PH_S_IN: {
      if (g.j == g.nin) {
        g.phase = PH_DONE;
        break;
      }
      uint32_t o = g.ioff + 36;
      const uint32_t sl = get_varint(T, o);
      piece_copy(g, T + o + sl, 4);
      g.ioff = o + sl + 4;
      g.j += 1;
      break;
    }
    case PH_RANGE: piece_copy(g, g.code, g.code_len); g.phase = PH_DONE; break;
    default: g.phase = PH_DONE; break;
  }
}

HKV_DEV bool gen_more(Gen& g) {
  while (g.rem == 0 && g.phase != PH_DONE) gen_advance(g);
  return g.rem != 0;
}
HKV_DEV uint32_t gen_next(Gen& g) {
  uint32_t b;
  if (g.src) {
    b = *g.src;
    g.src += 1;
  } else {
    b = (uint32_t)g.lit & 0xFFu;
    g.lit >>= 8;
  }
  g.rem -= 1;
  return b;
}

// Block-extraction kernels (hkv_tx_hash_kernel, hkv_sighash_kernel,
// hkv_std_input_kernel) take one-wave workgroups for up to HKV_XSMALL lanes
// (a block: its lanes spread over 4x the CUs; configs[0] 696 -> 687 us,
// configs[2] 736 -> 726 us) and WG-thread ones above (batches of blocks:
// 64-thread groups measured 1-3% slower there; profiles/r02_variants_xtpb.log).
// Their LDS slots keep the WG stride either way.
#ifndef HKV_XSMALL
#define HKV_XSMALL 16384
#endif
static inline uint32_t xtpb_for(size_t n) { return n <= HKV_XSMALL ? 64u : (uint32_t)WG; }

// The next up to 4 message bytes, packed big-endian from the top of w;
// returns how many (fewer than 4 only at the end of the message). Inside a
// piece the 4 bytes come from 4 independent loads (or the literal's next
// 32 bits) instead of 4 dependent load / store rounds; piece boundaries take
// the byte path.
HKV_DEV uint32_t gen_word(Gen& g, uint32_t& w) {
  if (g.rem >= 4u) {
    if (g.src) {
      const uint8_t* s = g.src;
      w = ((uint32_t)s[0] << 24) | ((uint32_t)s[1] << 16) | ((uint32_t)s[2] << 8) | (uint32_t)s[3];
      g.src += 4;
    } else {
      w = __builtin_bswap32((uint32_t)g.lit);
      g.lit >>= 32;
    }
    g.rem -= 4u;
    return 4u;
  }
  uint32_t n = 0;
  w = 0;
  for (int k = 0; k < 4; ++k) {
    if (!gen_more(g)) break;
    w |= gen_next(g) << (24 - 8 * k);
    ++n;
  }
  return n;
}

// SHA-256 of the generator's message, block-synchronous over the wave: each
// iteration every live lane writes its next 64 bytes (message, then 0x80,
// zeros and the 64-bit length) into its LDS slot buf[word * WG + tid] and all
// of them compress together. Call from wave-uniform control flow.
HKV_DEV void sha256_stream(uint32_t h[8], Gen& g, bool live, uint32_t* buf) {
  sha256_init(h);
  const uint32_t tid = threadIdx.x;
  // word at a time: 16 LDS word stores per block; 0x80 right after the last
  // message byte; the length in words 14-15 of the block that has room
  // (the byte-at-a-time form it replaced: extraction 188 -> 152 us on the
  // configs[2] block, profiles/r02_variants.log)
  uint32_t st = live ? 0u : 3u;  // 0 message, 1 padding (0x80 written), 3 done
  uint64_t len = 0;
  while (__any(st != 3u)) {
    if (st != 3u) {
      bool fits = st == 1u;  // a block after the 0x80 block always has room
#pragma unroll 1
      for (uint32_t k = 0; k < 16u; ++k) {
        uint32_t v = 0;
        if (st == 0u) {
          const uint32_t nb = gen_word(g, v);
          len += nb;
          if (nb < 4u) {
            v |= 0x80u << (24 - 8 * nb);
            st = 1u;
            fits = k < 14u;
          }
        }
        buf[k * WG + tid] = v;
      }
      uint32_t w[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = buf[k * WG + tid];
      const bool last = st == 1u && fits;
      if (last) {
        const uint64_t bits = len << 3;
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
      }
      sha256_compress(h, w);
      if (last) st = 3u;
    }
  }
}

// SHA-256d digest -> 8 words in digest byte order
HKV_DEV void sha256d_finish(uint32_t out[8], const uint32_t h[8]) {
  uint32_t d[8];
  sha256_of_digest(d, h);
#pragma unroll
  for (int k = 0; k < 8; ++k) out[k] = __builtin_bswap32(d[k]);
}

// ---------------------------------------------------------------------------
// walkers over a validated tx
// ---------------------------------------------------------------------------
HKV_DEV void walk_input(const uint8_t* T, uint32_t ins, uint32_t i, uint32_t& in_off, uint32_t& ss_off,
                        uint32_t& ss_len, uint32_t& seq_off) {
  uint32_t off = ins;
  for (uint32_t j = 0;; ++j) {
    uint32_t o = off + 36;
    const uint32_t sl = get_varint(T, o);
    if (j == i) {
      in_off = off;
      ss_off = o;
      ss_len = sl;
      seq_off = o + sl;
      return;
    }
    off = o + sl + 4;
  }
}
HKV_DEV uint32_t walk_output(const uint8_t* T, uint32_t first, uint32_t k) {
  uint32_t off = first;
  for (uint32_t j = 0; j < k; ++j) {
    uint32_t o = off + 8;
    const uint32_t sl = get_varint(T, o);
    off = o + sl;
  }
  return off;
}
HKV_DEV uint32_t walk_witness(const uint8_t* T, uint32_t wstart, uint32_t i) {
  uint32_t off = wstart;
  for (uint32_t j = 0; j < i; ++j) {
    const uint32_t cnt = get_varint(T, off);
    for (uint32_t c = 0; c < cnt; ++c) {
      const uint32_t il = get_varint(T, off);
      off += il;
    }
  }
  return off;
}

// ---------------------------------------------------------------------------
// 1. tx index
// ---------------------------------------------------------------------------
// bounds-checked parse of tx t's wire form into the first 8 words of its row
HKV_DEV void tx_index_row(const uint8_t* __restrict__ txs, const uint32_t* __restrict__ tx_off, uint32_t t,
                          uint32_t row[8]) {
  bool ok = false;
  {
    const uint32_t st = tx_off[t], end = tx_off[t + 1];
    ok = end >= st && end - st >= 10;
    uint32_t off = st + 4, nin = 0, nout = 0;
    bool seg = false;
    if (ok && txs[off] == 0 && txs[off + 1] == 1) {
      seg = true;
      off += 2;
    }
    ok = ok && rd_varint(txs, off, end, nin);
    const uint32_t ins = off;
    for (uint32_t j = 0; ok && j < nin; ++j) {
      uint32_t sl = 0;
      ok = end - off >= 36;
      off += ok ? 36 : 0;
      ok = ok && rd_varint(txs, off, end, sl) && end - off >= 4 && end - off - 4 >= sl;
      off += ok ? sl + 4 : 0;
    }
    ok = ok && rd_varint(txs, off, end, nout);
    const uint32_t outs_first = off;
    for (uint32_t k = 0; ok && k < nout; ++k) {
      uint32_t sl = 0;
      ok = end - off >= 8;
      off += ok ? 8 : 0;
      ok = ok && rd_varint(txs, off, end, sl) && end - off >= sl;
      off += ok ? sl : 0;
    }
    const uint32_t outs_end = off;
    for (uint32_t j = 0; ok && seg && j < nin; ++j) {
      uint32_t cnt = 0;
      ok = rd_varint(txs, off, end, cnt);
      for (uint32_t c = 0; ok && c < cnt; ++c) {
        uint32_t il = 0;
        ok = rd_varint(txs, off, end, il) && end - off >= il;
        off += ok ? il : 0;
      }
    }
    ok = ok && end - off == 4;
    row[TXT_FLAGS] = (ok ? TXF_OK : 0u) | (seg ? TXF_WITNESS : 0u);
    row[TXT_INS] = ins;
    row[TXT_NIN] = nin;
    row[TXT_NOUT] = nout;
    row[TXT_OUTS_FIRST] = outs_first;
    row[TXT_OUTS_END] = outs_end;
    row[TXT_LOCK] = off;
    row[TXT_START] = st;
  }
}

// ---------------------------------------------------------------------------
// shared per-job setup: everything a legacy / BIP143 preimage needs
// ---------------------------------------------------------------------------
struct JobCtx {
  uint32_t start, nin, nout, ins, outs_first, lock;
  uint32_t i, sh, shn, flags;
  uint32_t in_i, in_i_seq, single_off;
  bool forkid_form;   // BIP143 preimage
  bool one;           // legacy SINGLE with i >= #outputs: sign the integer one
  bool single_hash;   // BIP143 SINGLE with i < #outputs: per-job hashOutputs
};

HKV_DEV void job_setup(JobCtx& c, const uint8_t* T, const uint32_t* row, uint32_t i, uint32_t sh, bool forkid_form,
                       int32_t forkid) {
  c.start = row[TXT_START];
  c.nin = row[TXT_NIN];
  c.nout = row[TXT_NOUT];
  c.ins = row[TXT_INS];
  c.outs_first = row[TXT_OUTS_FIRST];
  c.lock = row[TXT_LOCK];
  c.i = i;
  c.sh = sh;
  // txSigHash on a fork-id network dispatches FORKID-flagged types to the BIP143 form
  c.forkid_form = forkid_form || (forkid >= 0 && (sh & 0x40u));
  c.shn = (c.forkid_form && forkid >= 0) ? (sh | ((uint32_t)forkid << 8)) : sh;
  const uint32_t base = sh & 0x1Fu;
  const bool none = base == 2u, single = base == 3u;
  c.flags = ((sh & 0x80u) ? GF_ACP : 0u) | ((!none && !single) ? GF_ALL : 0u) | (none ? GF_NONE : 0u) |
            (single ? GF_SINGLE : 0u);
  uint32_t ss_off, ss_len;
  walk_input(T, c.ins, i, c.in_i, ss_off, ss_len, c.in_i_seq);
  c.one = !c.forkid_form && single && i >= c.nout;
  c.single_hash = c.forkid_form && single && i < c.nout;
  c.single_off = (single && i < c.nout) ? walk_output(T, c.outs_first, i) : 0u;
}

// main-preimage generator for a job; code = scriptCode bytes (for the
// P2WPKH form: the 20-byte program, flag GF_P2WPKH); h3: the tx's BIP143
// hashPrevouts | hashSequence | hashOutputs (24 words; null: the index row's)
HKV_DEV void gen_job(Gen& g, const JobCtx& c, const uint8_t* T, const uint32_t* row, const uint8_t* code,
                     uint32_t code_len, bool p2wpkh_code, uint64_t value, const uint32_t* single_ho,
                     const uint32_t* h3 = nullptr) {
  if (h3 == nullptr) h3 = row + TXT_HP;
  gen_clear(g);
  g.T = T;
  g.start = c.start; g.nin = c.nin; g.nout = c.nout; g.ins = c.ins; g.outs_first = c.outs_first; g.lock = c.lock;
  g.i = c.i; g.shn = c.shn; g.flags = c.flags;
  g.in_i = c.in_i; g.in_i_seq = c.in_i_seq; g.single_off = c.single_off;
  g.code = code; g.code_len = code_len; g.code_out = code_len; g.value = value;
  if (c.forkid_form) {
    if (p2wpkh_code) {
      g.flags |= GF_P2WPKH;
      g.code_len = 25;
    }
    const bool acp = (c.flags & GF_ACP) != 0;
    g.hp = acp ? nullptr : h3;
    g.hs = (acp || !(c.flags & GF_ALL)) ? nullptr : h3 + 8;
    g.ho = (c.flags & GF_ALL) ? h3 + 16 : (c.single_hash ? single_ho : nullptr);
    g.phase = PH_F_VER;
  } else {
    uint32_t n_sep = 0;
    if (script_scan(code, code_len, n_sep) && n_sep) {
      g.flags |= GF_STRIP;
      g.code_out = code_len - n_sep;
    }
    g.phase = PH_L_VER;
  }
}

// ---------------------------------------------------------------------------
// 3. standard inputs -> verify records
// ---------------------------------------------------------------------------
// secp256k1_der_read_len
HKV_DEV bool der_read_len(const uint8_t* p, uint32_t& off, uint32_t end, uint32_t& len) {
  if (off >= end) return false;
  const uint32_t b1 = p[off++];
  if (b1 == 0xFFu) return false;
  if ((b1 & 0x80u) == 0) {
    len = b1;
    return true;
  }
  const uint32_t lenleft = b1 & 0x7Fu;
  if (lenleft == 0) return false;          // indefinite length
  if (lenleft > end - off) return false;
  if (p[off] == 0) return false;           // not the shortest encoding
  if (lenleft > 8) return false;
  uint64_t v = 0;
  for (uint32_t k = 0; k < lenleft; ++k) v = (v << 8) | p[off++];
  if (v > (uint64_t)(end - off)) return false;
  if (v < 128) return false;
  len = (uint32_t)v;
  return true;
}
// secp256k1_der_parse_integer: overflow (negative, > 32 bytes, >= n) -> 0
HKV_DEV bool der_parse_int(const uint8_t* p, uint32_t& off, uint32_t end, uint32_t r[8]) {
  if (off >= end || p[off] != 0x02u) return false;
  ++off;
  uint32_t rlen = 0;
  if (!der_read_len(p, off, end, rlen)) return false;
  if (rlen == 0 || rlen > end - off) return false;
  const uint32_t b0 = p[off], b1 = rlen > 1 ? p[off + 1] : 0u;
  if (b0 == 0x00u && rlen > 1 && (b1 & 0x80u) == 0) return false;
  if (b0 == 0xFFu && rlen > 1 && (b1 & 0x80u) == 0x80u) return false;
  bool overflow = (b0 & 0x80u) != 0;
  if (b0 == 0) {
    ++off;
    --rlen;
  }
  if (rlen > 32) overflow = true;
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = 0;
  if (!overflow) {
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      if ((uint32_t)q < rlen) r[q >> 2] |= (uint32_t)p[off + rlen - 1 - q] << (8 * (q & 3));
    }
    if (!u256_lt(r, SC_N)) overflow = true;
  }
  if (overflow) {
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = 0;
  }
  off += rlen;
  return true;
}
HKV_DEV bool der_parse_sig(const uint8_t* p, uint32_t off, uint32_t end, uint32_t r[8], uint32_t s[8]) {
  if (off >= end || p[off] != 0x30u) return false;
  ++off;
  uint32_t len = 0;
  if (!der_read_len(p, off, end, len)) return false;
  if (len != end - off) return false;
  if (!der_parse_int(p, off, end, r)) return false;
  if (!der_parse_int(p, off, end, s)) return false;
  return off == end;
}
// haskoin-core decodeTxSig: hashtype byte (known base type; FORKID only on a
// fork-id network), then decodeStrictSig = DER parse + r, s != 0 + low S.
HKV_DEV bool decode_tx_sig(const uint8_t* p, uint32_t off, uint32_t len, int32_t forkid, uint32_t r[8], uint32_t s[8],
                           uint32_t& sh) {
  if (len < 1) return false;
  sh = p[off + len - 1];
  const uint32_t base = sh & 0x1Fu;
  if (!(base >= 1u && base <= 3u && !(forkid < 0 && (sh & 0x40u)))) return false;
  if (!der_parse_sig(p, off, off + len - 1, r, s)) return false;
  return !u256_is_zero(r) && !u256_is_zero(s) && !u256_lt(SC_HALF_N, s);
}

// one data push (opcodes 1..78) at off within [off, end): data range
HKV_DEV bool read_push(const uint8_t* p, uint32_t& off, uint32_t end, uint32_t& d_off, uint32_t& d_len) {
  if (off >= end) return false;
  const uint32_t op = p[off];
  uint32_t hdr, len;
  if (op >= 1u && op <= 75u) {
    hdr = 1;
    len = op;
  } else if (op == 0x4Cu) {
    if (end - off < 2) return false;
    hdr = 2;
    len = p[off + 1];
  } else if (op == 0x4Du) {
    if (end - off < 3) return false;
    hdr = 3;
    len = p[off + 1] | (p[off + 2] << 8);
  } else if (op == 0x4Eu) {
    if (end - off < 5) return false;
    hdr = 5;
    len = p[off + 1] | (p[off + 2] << 8) | (p[off + 3] << 16) | ((uint32_t)p[off + 4] << 24);
  } else {
    return false;
  }
  if ((uint64_t)hdr + len > (uint64_t)(end - off)) return false;
  d_off = off + hdr;
  d_len = len;
  off += hdr + len;
  return true;
}

// haskoin PubKeyI encoding: 02/03 + 32 bytes or 04 + 64 bytes
HKV_DEV bool pubkey_bytes_ok(const uint8_t* p, uint32_t len) {
  return (len == 33u && (p[0] == 2u || p[0] == 3u)) || (len == 65u && p[0] == 4u);
}
// direct-push P2PK script (21 <33> ac / 41 <65> ac)
HKV_DEV bool is_p2pk(const uint8_t* sc, uint32_t L) {
  return ((L == 35u && sc[0] == 0x21u) || (L == 67u && sc[0] == 0x41u)) && sc[L - 1] == 0xACu;
}
HKV_DEV bool is_p2pkh(const uint8_t* sc, uint32_t L) {
  return L == 25u && sc[0] == 0x76u && sc[1] == 0xA9u && sc[2] == 0x14u && sc[23] == 0x88u && sc[24] == 0xACu;
}
// 20-byte hash in memory == RIPEMD-160 words / 32-byte hash == SHA-256 state
HKV_DEV bool eq_h160(const uint8_t* p, const uint32_t rip[5]) {
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 5; ++k)
    ok = ok && (uint32_t)(p[4 * k] | (p[4 * k + 1] << 8) | (p[4 * k + 2] << 16) | ((uint32_t)p[4 * k + 3] << 24)) == rip[k];
  return ok;
}
HKV_DEV bool eq_sha256(const uint8_t* p, const uint32_t h[8]) {
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 8; ++k)
    ok = ok && (((uint32_t)p[4 * k] << 24) | (p[4 * k + 1] << 16) | (p[4 * k + 2] << 8) | p[4 * k + 3]) == h[k];
  return ok;
}

// Single-signature templates (haskoin verifyStdInput): P2PK, P2PKH, P2WPKH;
// P2SH around P2PK / P2PKH / P2WPKH / P2WSH; P2WSH (native or P2SH-nested)
// around P2PK / P2PKH. Multisig inputs: hkv_ms_* (section 4).

// ---------------------------------------------------------------------------
// verifyStdInput's non-ECDSA half, in two parts (hkv_std_input_kernel runs
// both; the small-batch verify kernel runs std_parse on every wave of a
// workgroup and std_hash on its signature wave after the Q chains started)
// ---------------------------------------------------------------------------
struct StdIn {
  bool ok;                    // every check so far passed
  const uint32_t* row;        // the tx's index row
  const uint8_t* spk;         // prevout scriptPubKey
  uint32_t input, sh;         // input index, sighash type word
  uint64_t value;
  const uint8_t* pub;         // pubkey bytes
  uint32_t pub_len;
  const uint8_t* code;        // sighash scriptCode (P2WPKH form: the 20-byte program)
  uint32_t code_len;
  bool segwit, p2wpkh;
  const uint8_t* kh;          // HASH160(pubkey) must equal these 20 bytes (has_kh)
  const uint8_t* rd;          // P2SH: HASH160(redeem script) == spk[2..22] (has_rd)
  uint32_t rd_len;
  const uint8_t* ws;          // P2WSH: SHA-256(witness script) == wprog (has_ws)
  uint32_t ws_len;
  const uint8_t* wprog;
  bool has_kh, has_rd, has_ws;
  uint32_t r[8], s[8];        // the decoded signature (limbs)
  const uint8_t* T;           // the tx bytes the pointers above index (txs, or the input's LDS copy)
};

// Part A: template match, strict DER decode (low S, hashtype), pubkey bytes.
// No hashing: everything the ECDSA chains need (r, s, the key) is known here.
HKV_DEV void std_parse(StdIn& x, const uint8_t* __restrict__ txs, uint32_t n_tx, const uint32_t* __restrict__ txt,
                       const uint8_t* __restrict__ scripts, uint32_t scripts_len,
                       const hkv_input_job* __restrict__ jobs, uint32_t jx, uint32_t n, int32_t forkid,
                       const uint8_t* tview = nullptr, const uint8_t* sview = nullptr, bool key_only = false) {
  // tview / sview: the input's tx and prevout script copied to LDS (the block
  // kernel's TxCache): tview[off] is byte off of txs, sview[k] byte k of the
  // script; null: read from HBM. key_only: the caller needs the key and the
  // template checks, not the signature (the chain waves of the small-batch
  // kernels: the verdict takes its validity from the signature wave's full
  // parse), so the DER decode is skipped and r, s stay zero
  const uint8_t* T = tview != nullptr ? tview : txs;
  const bool in_range = jx < n;
  bool ok = false;
  const uint32_t* row = txt;
  const uint8_t* spk = scripts;
  uint32_t sig_off = 0, sig_len = 0, pub_len = 0, sh = 0, input = 0;
  const uint8_t* pub = txs;
  uint64_t value = 0;
  const uint8_t* code = scripts;
  uint32_t code_len = 0;
  bool segwit = false, p2wpkh = false;
  const uint8_t* kh = scripts;
  const uint8_t* rd = txs;
  uint32_t rd_len = 0;
  const uint8_t* ws = txs;
  uint32_t ws_len = 0;
  const uint8_t* wprog = scripts;
  bool has_kh = false, has_rd = false, has_ws = false;
  uint32_t r[8], s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = s[k] = 0;
  if (in_range) {
    const hkv_input_job jb = jobs[jx];
    input = jb.input;
    value = jb.value;
    ok = jb.tx < n_tx && jb.script_off <= scripts_len && scripts_len - jb.script_off >= jb.script_len;
    if (ok) {
      row = txt + (size_t)jb.tx * TXT_WORDS;
      ok = (row[TXT_FLAGS] & TXF_OK) && jb.input < row[TXT_NIN];
    }
    if (ok) {
      spk = sview != nullptr ? sview : scripts + jb.script_off;
      const uint32_t L = jb.script_len;
      uint32_t in_off, ss_off, ss_len, seq_off;
      walk_input(T, row[TXT_INS], jb.input, in_off, ss_off, ss_len, seq_off);
      const uint32_t ss_end = ss_off + ss_len;
      uint32_t c = ss_off, pub_off = 0;
      // witness program to open: 1 P2WPKH [sig, pub], 2 P2WSH [stack.., ws]
      uint32_t open_wit = 0;
      if (is_p2pk(spk, L)) {  // scriptSig = <sig>; pubkey from the prevout
        ok = read_push(T, c, ss_end, sig_off, sig_len) && c == ss_end;
        pub = spk + 1;
        pub_len = L - 2;
        code = spk;
        code_len = L;
      } else if (is_p2pkh(spk, L)) {  // scriptSig = <sig> <pubkey>
        ok = read_push(T, c, ss_end, sig_off, sig_len) && read_push(T, c, ss_end, pub_off, pub_len) &&
             c == ss_end;
        pub = T + pub_off;
        kh = spk + 3;
        has_kh = true;
        code = spk;
        code_len = 25;
      } else if (L == 22u && spk[0] == 0x00u && spk[1] == 0x14u) {  // P2WPKH: empty scriptSig
        ok = ss_len == 0;
        code = kh = spk + 2;
        has_kh = true;
        open_wit = 1;
      } else if (L == 34u && spk[0] == 0x00u && spk[1] == 0x20u) {  // P2WSH: empty scriptSig
        ok = ss_len == 0;
        wprog = spk + 2;
        open_wit = 2;
      } else if (L == 23u && spk[0] == 0xA9u && spk[1] == 0x14u && spk[22] == 0x87u) {
        // P2SH: every op a push; the last one is the redeem script
        uint32_t np = 0, o0 = 0, l0 = 0, o1 = 0, l1 = 0, ol = 0, ll = 0;
        while (ok && c < ss_end) {
          uint32_t d_off = 0, d_len = 0;
          ok = read_push(T, c, ss_end, d_off, d_len);
          if (np == 0) { o0 = d_off; l0 = d_len; }
          if (np == 1) { o1 = d_off; l1 = d_len; }
          ol = d_off;
          ll = d_len;
          ++np;
        }
        ok = ok && np >= 1;
        rd = T + ol;
        rd_len = ll;
        has_rd = true;
        if (ok) {
          if (ll == 22u && rd[0] == 0u && rd[1] == 0x14u) {  // P2SH-P2WPKH
            ok = np == 1;
            code = kh = rd + 2;
            has_kh = true;
            open_wit = 1;
          } else if (ll == 34u && rd[0] == 0u && rd[1] == 0x20u) {  // P2SH-P2WSH
            ok = np == 1;
            wprog = rd + 2;
            open_wit = 2;
          } else if (is_p2pk(rd, ll)) {  // P2SH-P2PK: <sig> <redeem>
            ok = np == 2;
            sig_off = o0; sig_len = l0;
            pub = rd + 1;
            pub_len = ll - 2;
            code = rd;
            code_len = ll;
          } else if (is_p2pkh(rd, ll)) {  // P2SH-P2PKH: <sig> <pubkey> <redeem>
            ok = np == 3;
            sig_off = o0; sig_len = l0;
            pub = T + o1;
            pub_len = l1;
            kh = rd + 3;
            has_kh = true;
            code = rd;
            code_len = 25;
          } else {
            ok = false;  // multisig redeem scripts: hkv_ms_*; anything else is not standard
          }
        }
      } else {
        ok = false;
      }
      if (ok && open_wit) {
        ok = (row[TXT_FLAGS] & TXF_WITNESS) != 0;
        uint32_t w = ok ? walk_witness(T, row[TXT_OUTS_END], jb.input) : 0u;
        const uint32_t cnt = ok ? get_varint(T, w) : 0u;
        if (open_wit == 1) {  // [sig, pubkey]
          ok = ok && cnt == 2u;
          if (ok) {
            sig_len = get_varint(T, w);
            sig_off = w;
            w += sig_len;
            pub_len = get_varint(T, w);
            pub = T + w;
          }
          segwit = p2wpkh = true;
        } else {  // [sig, ws] (P2PK) or [sig, pubkey, ws] (P2PKH)
          ok = ok && (cnt == 2u || cnt == 3u);
          if (ok) {
            sig_len = get_varint(T, w);
            sig_off = w;
            w += sig_len;
            uint32_t l1 = 0, o1 = 0;
            if (cnt == 3u) {
              l1 = get_varint(T, w);
              o1 = w;
              w += l1;
            }
            ws_len = get_varint(T, w);
            ws = T + w;
            has_ws = true;
            if (cnt == 2u && is_p2pk(ws, ws_len)) {
              pub = ws + 1;
              pub_len = ws_len - 2;
            } else if (cnt == 3u && is_p2pkh(ws, ws_len)) {
              pub = T + o1;
              pub_len = l1;
              kh = ws + 3;
              has_kh = true;
            } else {
              ok = false;  // P2WSH multisig: hkv_ms_*
            }
            code = ws;
            code_len = ws_len;
          }
          segwit = true;
        }
      }
    }
    if (ok && !key_only) ok = decode_tx_sig(T, sig_off, sig_len, forkid, r, s, sh);
    if (ok) ok = pubkey_bytes_ok(pub, pub_len);
  }
  x.ok = ok; x.row = row; x.spk = spk; x.input = input; x.sh = sh; x.value = value;
  x.pub = pub; x.pub_len = pub_len; x.code = code; x.code_len = code_len; x.segwit = segwit; x.p2wpkh = p2wpkh;
  x.kh = kh; x.rd = rd; x.rd_len = rd_len; x.ws = ws; x.ws_len = ws_len; x.wprog = wprog;
  x.has_kh = has_kh; x.has_rd = has_rd; x.has_ws = has_ws; x.T = T;
#pragma unroll
  for (int k = 0; k < 8; ++k) { x.r[k] = r[k]; x.s[k] = s[k]; }
}

// the three BIP143 per-tx hashes of row's tx into h3 (hashPrevouts |
// hashSequence | hashOutputs) for the lanes that need them (block-synchronous)
HKV_DEV void bip143_tx_hashes(const uint8_t* __restrict__ txs, const uint32_t* row, bool need, uint32_t* h3,
                              uint32_t* buf) {
#pragma unroll 1
  for (int which = 0; which < 3; ++which) {
    Gen g;
    uint32_t h[8], d[8];
    gen_clear(g);
    g.T = txs;
    if (need) {
      if (which == 2) {  // hashOutputs (each output re-serialised canonically)
        g.ooff = row[TXT_OUTS_FIRST]; g.ocnt = row[TXT_NOUT]; g.ret = PH_DONE; g.phase = PH_O_VAL;
      } else {
        g.nin = row[TXT_NIN]; g.ioff = row[TXT_INS]; g.j = 0; g.phase = which == 0 ? PH_P_IN : PH_S_IN;
      }
    }
    sha256_stream(h, g, need, buf);
    sha256d_finish(d, h);
    if (need) {
#pragma unroll
      for (int k = 0; k < 8; ++k) h3[8 * which + k] = d[k];
    }
  }
}

// The same three hashes for the G inputs on lanes 0..G-1 of a wave whose
// other lanes are idle (the block kernel's signature wave, G = 16): lane
// w G + c computes hash w of input c's tx, so the three streams run as one
// block-synchronous stream; the digests go to input c's h3 scratch. Call
// from wave-uniform control flow with every lane of the wave.
HKV_DEV void bip143_tx_hashes_spread(const uint8_t* __restrict__ txs, const uint32_t* row, bool need, uint32_t* h3,
                                     uint32_t* buf, uint32_t G, const uint8_t* tview = nullptr) {
  const uint32_t L = threadIdx.x & 63u, c = L % G, which = L / G;
  const uint64_t rp = reinterpret_cast<uint64_t>(row), hp = reinterpret_cast<uint64_t>(h3);
  // input c's tx bytes (its LDS copy when the caller has one)
  const uint64_t tp = reinterpret_cast<uint64_t>(tview != nullptr ? tview : txs);
  const uint64_t tc = (uint64_t)(uint32_t)__shfl((int)(uint32_t)tp, (int)c) |
                      ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(tp >> 32), (int)c) << 32);
  const uint64_t rc = (uint64_t)(uint32_t)__shfl((int)(uint32_t)rp, (int)c) |
                      ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(rp >> 32), (int)c) << 32);
  const uint64_t hc = (uint64_t)(uint32_t)__shfl((int)(uint32_t)hp, (int)c) |
                      ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(hp >> 32), (int)c) << 32);
  const bool go = __shfl(need ? 1 : 0, (int)c) != 0 && which < 3u;
  const uint32_t* rw = reinterpret_cast<const uint32_t*>(rc);
  Gen g;
  uint32_t h[8], d[8];
  gen_clear(g);
  g.T = reinterpret_cast<const uint8_t*>(tc);
  if (go) {
    if (which == 2) {  // hashOutputs (each output re-serialised canonically)
      g.ooff = rw[TXT_OUTS_FIRST]; g.ocnt = rw[TXT_NOUT]; g.ret = PH_DONE; g.phase = PH_O_VAL;
    } else {
      g.nin = rw[TXT_NIN]; g.ioff = rw[TXT_INS]; g.j = 0; g.phase = which == 0 ? PH_P_IN : PH_S_IN;
    }
  }
  sha256_stream(h, g, go, buf);
  sha256d_finish(d, h);
  if (go) {
    uint32_t* o = reinterpret_cast<uint32_t*>(hc);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[8 * which + k] = d[k];
  }
  __threadfence_block();  // the digests before the owning lanes read them
}

// Part B: the HASH160 / SHA-256 script checks and the sighash (updates x.ok).
// Call from wave-uniform control flow (block-synchronous SHA-256 streams
// through buf[16 * WG]). single_ho: 8 scratch words of the lane (BIP143
// SINGLE parks its hashOutputs there). h3: null when the index rows carry the
// BIP143 per-tx hashes (hkv_tx_hash_kernel), else 24 scratch words of the
// lane, where they are computed for this input's tx. Returns whether d holds
// the sighash; false with x.ok means the legacy SINGLE bug (the message is
// the integer 1).
HKV_DEV bool std_hash(StdIn& x, const uint8_t* __restrict__ txs, int32_t forkid, uint32_t* single_ho, uint32_t* buf,
                      uint32_t d[8], uint32_t* h3 = nullptr, bool h3_ready = false) {
  bool ok = x.ok;
  const uint32_t* row = x.row;
  const uint8_t* spk = x.spk;
  const uint8_t* pub = x.pub;
  const uint32_t pub_len = x.pub_len, input = x.input, sh = x.sh;
  const uint8_t* code = x.code;
  const uint32_t code_len = x.code_len;
  const bool segwit = x.segwit, p2wpkh = x.p2wpkh, has_kh = x.has_kh, has_rd = x.has_rd, has_ws = x.has_ws;
  const uint8_t *kh = x.kh, *rd = x.rd, *ws = x.ws, *wprog = x.wprog;
  const uint32_t rd_len = x.rd_len, ws_len = x.ws_len;
  const uint64_t value = x.value;
  const uint8_t* T = x.T != nullptr ? x.T : txs;
  uint32_t* r32 = single_ho;
  Gen g;
  uint32_t h[8];
  // HASH160(pubkey) == the key hash (P2PKH, P2WPKH and their wrapped forms)
  const bool need_h160 = ok && has_kh;
  if (__any(need_h160)) {
    gen_clear(g);
    g.code = pub; g.code_len = pub_len; g.phase = PH_RANGE;
    sha256_stream(h, g, need_h160, buf);
    uint32_t rip[5];
    ripemd160_of_digest(rip, h);
    if (need_h160) ok = ok && eq_h160(kh, rip);
  }
  // P2SH: HASH160(redeem script) == the script hash
  const bool need_rd = ok && has_rd;
  if (__any(need_rd)) {
    gen_clear(g);
    g.code = rd; g.code_len = rd_len; g.phase = PH_RANGE;
    sha256_stream(h, g, need_rd, buf);
    uint32_t rip[5];
    ripemd160_of_digest(rip, h);
    if (need_rd) ok = ok && eq_h160(spk + 2, rip);
  }
  // P2WSH: SHA-256(witness script) == the 32-byte program
  const bool need_ws = ok && has_ws;
  if (__any(need_ws)) {
    gen_clear(g);
    g.code = ws; g.code_len = ws_len; g.phase = PH_RANGE;
    sha256_stream(h, g, need_ws, buf);
    if (need_ws) ok = ok && eq_sha256(wprog, h);
  }
  // sighash: legacy txSigHash over the scriptCode (prevout or redeem script),
  // or txSigHashForkId (BIP143) over 76 a9 14 <h20> 88 ac (P2WPKH) / the
  // witness script (P2WSH)
  JobCtx c;
  c.forkid_form = false; c.one = false; c.single_hash = false;
  if (ok) job_setup(c, T, row, input, sh, segwit, forkid);
  const bool need_single = ok && c.single_hash;
  if (__any(need_single)) {
    gen_clear(g);
    g.T = T; g.ooff = c.single_off; g.ocnt = 1; g.ret = PH_DONE; g.phase = PH_O_VAL;
    sha256_stream(h, g, need_single, buf);
    sha256d_finish(d, h);
    if (need_single) {
#pragma unroll
      for (int k = 0; k < 8; ++k) r32[k] = d[k];  // scratch: record bytes 0..31
    }
  }
  const bool live = ok && !c.one;
  if (h3 != nullptr && !h3_ready) {
    const bool need_tx = live && c.forkid_form;
    if (__any(need_tx)) bip143_tx_hashes(T, row, need_tx, h3, buf);
  }
  if (!live) gen_clear(g);
  else gen_job(g, c, T, row, code, p2wpkh ? 20u : code_len, p2wpkh, value, r32, h3);
  sha256_stream(h, g, live, buf);
  sha256d_finish(d, h);
  x.ok = ok;
  return live;
}

// record: msg32 | r | s | pklen | pubkey | 0 (all zero when a check failed)
HKV_DEV void std_write_record(uint32_t* r32, const StdIn& x, bool live, const uint32_t d[8]) {
  const bool ok = x.ok;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    r32[k] = !ok ? 0u : (live ? d[k] : (k == 0 ? 1u : 0u));
    r32[8 + k] = ok ? __builtin_bswap32(x.r[7 - k]) : 0u;
    r32[16 + k] = ok ? __builtin_bswap32(x.s[7 - k]) : 0u;
  }
#pragma unroll
  for (int w = 0; w < 18; ++w) {
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int q = 4 * w + b;  // byte 96 + q of the record
      uint32_t byte = 0;
      if (q == 0) byte = x.pub_len;
      else if ((uint32_t)(q - 1) < x.pub_len && q - 1 < 65) byte = x.pub[q - 1];
      v |= byte << (8 * b);
    }
    r32[24 + w] = ok ? v : 0u;
  }
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


// The scan of one input (hkv_ms_scan_kernel, and the block kernel's
// square-root wave): template + scriptSig / witness decode, the P2SH
// HASH160 and the P2WSH SHA-256 checks (block-synchronous: call from
// wave-uniform control flow, buf = 16 * WG words indexed by threadIdx.x),
// the input's desc words and its record range, allocated from the 64-bit
// device counter total (candidates in the low 32 bits, key checks in the
// high 32; placement order is irrelevant to verdicts).
HKV_DEV void ms_scan_lane(const uint8_t* __restrict__ txs, uint32_t n_tx, const uint32_t* __restrict__ txt,
                          const uint8_t* __restrict__ scripts, uint32_t scripts_len,
                          const hkv_input_job* __restrict__ jobs, uint32_t jx, bool in_range, int32_t forkid,
                          uint32_t* __restrict__ desc, uint64_t* __restrict__ off, unsigned long long* total,
                          uint32_t* buf) {
  MsIn r;
  r.p2sh = r.wit = false;
  r.code = r.rd = r.wprog = scripts;
  r.code_len = r.rd_len = 0;
  bool ok = false;
  const uint8_t* spk = scripts;
  if (in_range) {
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
  if (in_range) {
    desc[2 * (size_t)jx] = ok ? (MS_OK | (r.p2sh ? MS_P2SH : 0u) | r.m | (r.n << 8) | (r.s_eff << 16)) : 0u;
    desc[2 * (size_t)jx + 1] = ok ? r.mask : 0u;
    off[jx] = ok ? (uint64_t)atomicAdd(total, (unsigned long long)r.n_cand | ((unsigned long long)r.n << 32)) : 0ull;
  }
}
// record: msg32 (digest byte order words) | r | s (limbs, written big-endian) |
// pklen | pubkey | zero padding
HKV_DEV void ms_write_record(uint32_t* r32, const uint32_t msg[8], const uint32_t r[8], const uint32_t s[8],
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

// The records of one scanned multisig input (the tail kernel's emit phase):
// one key-check record per key of its script (msg, r, s zero), then per
// signature j < s_eff its sighash and the candidate records (msg_j, r_j, s_j,
// key_k), k = j..n-1, at the ranges the scan allocated. Only the records that
// fall in this round's windows are written — candidate records
// [cw0, cw0 + cwn) at cand[index - cw0], key-check records [kw0, kw0 + kwn)
// at keyrec[index - kw0] — and a signature none of whose candidates falls
// in the window is not hashed (the tail runs its record windows in rounds so
// that its scratch stays within a fixed budget). Block-synchronous hashing:
// call from wave-uniform control flow with buf = 16 * blockDim words.
HKV_DEV void ms_emit_lane(const uint8_t* __restrict__ txs, uint32_t n_tx, const uint32_t* __restrict__ txt,
                          const uint8_t* __restrict__ scripts, uint32_t scripts_len,
                          const hkv_input_job* __restrict__ jobs, uint32_t jx, bool in_range, int32_t forkid,
                          const uint32_t* __restrict__ desc, const uint64_t* __restrict__ off64,
                          uint8_t* __restrict__ cand, uint8_t* __restrict__ keyrec, uint32_t cw0, uint32_t cwn,
                          uint32_t kw0, uint32_t kwn, uint32_t* buf) {
  bool go = in_range && (desc[2 * (size_t)jx] & MS_OK);
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
  if (go) {
    const uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t k = 0; k < r.n; ++k) {
      const uint32_t w = kbase + k - kw0;  // (wraps past 2^32 below the window)
      if (w >= kwn) continue;
      uint32_t kl;
      const uint8_t* kp = ms_key(r.code, k, kl);
      ms_write_record(reinterpret_cast<uint32_t*>(keyrec + (size_t)w * REC_SIZE), z, z, z, kp, kl);
    }
  }
  uint32_t off = r.it_off, idx = cbase;
  Gen g;
  uint32_t h[8], d[8];
  for (uint32_t j = 0; __any(go && j < r.s_eff); ++j) {
    const bool here = go && j < r.s_eff;
    uint32_t d_off = 0, d_len = 0;
    if (here) (void)ms_item(txs, r, off, d_off, d_len);
    // signature j's candidates [idx, idx + n - j) against the window: the
    // hash is needed only when one of them is written in this round
    const uint32_t lo = idx > cw0 ? idx : cw0, hi_w = cw0 + cwn, hi_j = idx + (r.n - j);
    const bool live = here && ((r.mask >> j) & 1u) && lo < (hi_w < hi_j ? hi_w : hi_j);
    uint32_t rr[8], ss[8], sh = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) rr[k] = ss[k] = 0;
    if (live) (void)decode_tx_sig(txs, d_off, d_len, forkid, rr, ss, sh);
    JobCtx c;
    c.forkid_form = false; c.one = false; c.single_hash = false;
    if (live) job_setup(c, txs, row, input, sh, r.wit, forkid);  // P2WSH: BIP143 over the witness script
    // (scratch for hashOutputs: the first of sig j's records in the window,
    // overwritten by that record once the hash is done)
    uint32_t* r32 = reinterpret_cast<uint32_t*>(cand + (size_t)(live ? lo - cw0 : 0u) * REC_SIZE);
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
        const uint32_t w = idx + (k - j) - cw0;  // (wraps past 2^32 below the window)
        if (w >= cwn) continue;
        uint32_t kl;
        const uint8_t* kp = ms_key(r.code, k, kl);
        ms_write_record(reinterpret_cast<uint32_t*>(cand + (size_t)w * REC_SIZE), msg, rr, ss, kp, kl);
      }
    }
    if (here && ((r.mask >> j) & 1u)) idx += r.n - j;
  }
}

HKV_DEV bool ms_bit_at(const uint32_t* b, uint32_t i) { return (b[i >> 5] >> (i & 31u)) & 1u; }

// haskoin-core countMulSig over the candidate verdicts of one input (the tail
// kernel's last phase): all keys decode and the walk's count equals m -> the
// input's verdict bit is set.
HKV_DEV void ms_resolve_lane(const uint32_t* __restrict__ desc, const uint64_t* __restrict__ off64, uint32_t jx,
                             bool in_range, const uint32_t* __restrict__ cbits, const uint32_t* __restrict__ kbits,
                             uint32_t* __restrict__ out_bits) {
  if (!in_range) return;
  const uint32_t d0 = desc[2 * (size_t)jx];
  if (!(d0 & MS_OK)) return;
  const uint32_t mask = desc[2 * (size_t)jx + 1];
  const uint32_t m = d0 & 0xFFu, nk = (d0 >> 8) & 0xFFu, s_eff = (d0 >> 16) & 0xFFu;
  const uint64_t o = off64[jx];
  uint32_t start = (uint32_t)o;
  const uint32_t kbase = (uint32_t)(o >> 32);
  bool keys_ok = true;
  for (uint32_t k = 0; k < nk; ++k) keys_ok = keys_ok && ms_bit_at(kbits, kbase + k);
  // countMulSig': start = index of candidate (j, j)
  uint32_t count = 0, j = 0;
  for (uint32_t k = 0; k < nk; ++k) {
    if (j >= s_eff) break;
    if (!((mask >> j) & 1u)) {  // TxSignatureEmpty: consumes the key and the signature
      ++j;
      continue;
    }
    if (ms_bit_at(cbits, start + (k - j))) {
      ++count;
      start += nk - j;
      ++j;
    }
  }
  if (keys_ok && count == m) atomicOr(&out_bits[jx >> 5], 1u << (jx & 31u));
}

// One BIP143 per-tx hash (which: 0 hashPrevouts, 1 hashSequence, 2
// hashOutputs) of a tx whose index row the caller has built (row), into its
// row in txt (row_out: only the hash words are written) — the tail kernel's
// first phase on the fused block path, whose index pass hashed nothing.
// Block-synchronous like ms_emit_lane.
HKV_DEV void tx_hash_word_lane(const uint8_t* __restrict__ txs, const uint32_t row[8], uint32_t* __restrict__ row_out,
                               uint32_t which, bool go, uint32_t* buf) {
  go = go && (row[TXT_FLAGS] & TXF_OK) != 0;
  Gen g;
  uint32_t h[8], d[8];
  gen_clear(g);
  g.T = txs;
  if (which == 2) {
    g.ooff = row[TXT_OUTS_FIRST]; g.ocnt = row[TXT_NOUT]; g.ret = PH_DONE; g.phase = PH_O_VAL;
  } else {
    g.nin = row[TXT_NIN]; g.ioff = row[TXT_INS]; g.j = 0; g.phase = which == 0 ? PH_P_IN : PH_S_IN;
  }
  sha256_stream(h, g, go, buf);
  sha256d_finish(d, h);
  if (go) {
    const int slot = which == 0 ? TXT_HP : (which == 1 ? TXT_HS : TXT_HO);
#pragma unroll
    for (int k = 0; k < 8; ++k) row_out[slot + k] = d[k];
  }
}

}  // namespace hkv
