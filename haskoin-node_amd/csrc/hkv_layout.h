// hkv_layout.h — buffer layouts shared by the HIP kernels and the host API.
#pragma once
#include <stdint.h>

namespace hkv {

// Input record (AoS, include/hkv.h): msg32 | r32 | s32 | pklen u8 | pubkey[65] | pad[6]
constexpr int REC_SIZE = 168;
constexpr int REC_WORDS = REC_SIZE / 4;

// Prologue -> ecmult intermediate, SoA: word w of signature i at [w * n_pad + i].
enum : int {
  IM_FLAGS = 0,   // bit0 valid, bit1 k1 negative, bit2 k2 negative, bit3 glv overflow
  IM_QX = 1,      // 8 limbs, affine pubkey x (normalised)
  IM_QY = 9,      // 8 limbs, affine pubkey y (normalised)
  IM_K1 = 17,     // 5 limbs, |k1| < 2^129   (u2 = k1 + k2*lambda)
  IM_K2 = 22,     // 5 limbs, |k2| < 2^129
  IM_U1L = 27,    // 4 limbs, u1 bits 0..127
  IM_U1H = 31,    // 4 limbs, u1 bits 128..255
  IM_R = 35,      // 8 limbs, r (< n)
  IM_C = 43,      // 8 limbs, batch-inversion prefix product, then s^-1
  IM_DIG = 51,    // NWIN (<= 33) words: window w's radix-2^QW Booth digits of k1, k2
  IM_GDIG = 84,   // 2 x GWIN words: radix-2^GTAB_W Booth digits of u1_lo, u1_hi
  // between the parse and scalar kernels: s (normalised) and m = msg mod n
  IM_S = IM_K1,   // 8 limbs over K1|K2 (10 words)
  IM_M = IM_U1L,  // 8 limbs over U1L|U1H
};
// Q digit word of window w (w = 0..NWIN-1, bit position QW*w): biased Booth
//   digits, bits 0..QW d1 + QBIAS (k1, radix 2^QW, -QBIAS..QBIAS), bits
//   QW+1..2QW+1 d2 + QBIAS (k2)
// G digit word of G window j (j = 0..GWIN-1, bit position GTAB_W*j = Q
// window GSTEP*j), one per u1 half: bits 0..GTAB_W-1 |d| (0..2^(GTAB_W-1)),
// bit GTAB_W sign. Default radix 2^20: 7 windows, every fifth Q window.
// HKV_QW = 5 (radix-32 Q windows: 52 instead of 66 Q additions, 125
// doublings, a 16-entry table) is correct (GPU suite green) but measured
// 1-1.5% slower at 1M (profiles/r02_variants.log): the 400 MB of per-lane
// tables of a full grid no longer stay in the 256 MB MALL.
#ifndef HKV_QW
#define HKV_QW 4
#endif
#ifndef HKV_GTAB_W
#define HKV_GTAB_W 20
#endif
constexpr int QW = HKV_QW;                       // Booth radix 2^QW of the k1 / k2 windows
static_assert(QW == 4 || QW == 5, "radix-16 or radix-32 Q windows");
constexpr int GTAB_W = HKV_GTAB_W;            // Booth radix of the fixed-base tables
static_assert(GTAB_W % QW == 0 && GTAB_W >= 8 && GTAB_W <= 28, "G windows sit on Q window boundaries");
constexpr int NWIN = (130 + QW - 1) / QW;        // 33 / 26: |k| < 2^129 plus the Booth carry
static_assert(IM_DIG + NWIN <= IM_GDIG, "digit words fit");
constexpr int QBIAS = 1 << (QW - 1);             // digit range -QBIAS..QBIAS
constexpr int QDIG_BITS = QW + 1;                // width of a biased digit in the digit word
constexpr uint32_t QDIG_MASK = (1u << QDIG_BITS) - 1u;
constexpr int GWIN = (128 + GTAB_W) / GTAB_W;  // covers 129 bits with the Booth carry
constexpr int GSTEP = GTAB_W / QW;             // Q windows per G window
constexpr uint32_t GD_MAG = (1u << GTAB_W) - 1u, GD_NEG = 1u << GTAB_W;
constexpr int IM_WORDS = IM_GDIG + 2 * GWIN;
constexpr uint32_t DIG_ZERO = (uint32_t)QBIAS | ((uint32_t)QBIAS << QDIG_BITS);

// signatures per thread in the scalar kernel (one s^-1 per BATCH_INV via
// Montgomery's trick: 3(B-1) multiplications + 1 inversion)
#ifndef HKV_BATCH_INV
#define HKV_BATCH_INV 16
#endif
constexpr int BATCH_INV = HKV_BATCH_INV;
constexpr uint32_t FLAG_VALID = 1u, FLAG_NEG1 = 2u, FLAG_NEG2 = 4u, FLAG_GLV_OVF = 8u;

// y-free verification (every launch shape; hkv_kernels.hip §2b): the
// prologue stores w = x^3 + 7 over IM_QY instead of solving y = sqrt(w);
// ecmult runs u2 * Q' on E_w : y^2 = x^3 + 7 w^3 with Q' = (x w, w^2) and
// leaves B' = (X, Y, Z) over the Q-digit words; the finish kernel adds the
// u1 * G sum from per-window tables and reduces "x(u1 G + u2 Q) == r" to
// y_c = num / den, accepted iff y_c^2 == w with the key's y parity. Small
// batches (hkv_pair_split_kernel, §2c) run the u1 * G sum and the key's
// square root on their own waves beside the two Q chains and join exactly in
// the kernel.
// the small-batch kernel's signature / square-root waves' output for the join (SoA, its own buffer): A = u1 G (24 words), y0 (8), flags
enum : int { AUX_AX = 0, AUX_Y0 = 24, AUX_FLAGS = 32, AUX_SQ = 33, AUX_WORDS = 34 };  // AUX_SQ: the pair kernel's sqrt wave
constexpr uint32_t AUXF_AINF = 1u, AUXF_SQ = 2u;
constexpr uint32_t FLAG_YODD = 16u;      // the key's y is odd (prefix 03/07, or the 04 key's y)
constexpr uint32_t FLAG_COMP = 32u;      // compressed key: x^3 + 7 not yet shown to be a square
constexpr uint32_t FLAG_BINF = 64u;      // B' = u2 * Q' is infinity
constexpr uint32_t FLAG_DECIDED = 128u;  // the finish kernel decided the verdict (rare cases)
constexpr uint32_t FLAG_ACCEPT = 256u;   // ... and it is accept
constexpr uint32_t FLAG_RARE = 512u;     // A or B infinity, or A = +-B: the exact slow path decides
constexpr uint32_t FLAG_AINF = 1024u;    // A = u1 * G is infinity (u1 = 0)
enum : int {
  IM_W = IM_QY,         // 8 limbs, w = x^3 + 7 (normalised)
  IM_BX = IM_DIG,       // 3 x 8 limbs: B' = (X, Y, Z) Jacobian on E_w (ecmult -> finish)
  IM_NUM = IM_DIG,      // 3 x 8 limbs: num_r, num_{r+n}, den (finish -> verdict kernel)
  IM_DEN = IM_DIG + 16,
  IM_AX = IM_QX,        // rare lanes: A = u1 * G parked over x (8) and K1..U1H (16)
  IM_AY = IM_K1,
};
constexpr int IM_RARE_LIST = IM_AY + 16;  // the finish kernel's compacted rare-lane indices
static_assert(IM_RARE_LIST < IM_R, "A and the rare list fit below r");
static_assert(IM_DIG + 24 <= IM_GDIG, "B' and num/den fit over the Q digits");

// Fixed-base tables in HBM: multiples j*B for j = 1..2^19, affine, 16 dwords
// per entry [x(8) | y(8)], table t at entry offset t*2^19: table 2j + h holds
// B = 2^(GTAB_W j + 128 h) G (j = 0..GWIN-1), so the u1 * G sum (finish
// kernel, split waves 4-5) takes one addition per table and no doublings.
constexpr int GTAB_ENTRIES = 1 << (GTAB_W - 1);
constexpr int GTAB_TABLES = 2 * GWIN;
constexpr size_t GTAB_DWORDS = (size_t)GTAB_TABLES * GTAB_ENTRIES * 16;

// Per-lane Q table: multiples j*Q, j = 1..QBIAS, affine on the lane's isomorphic
// curve; per entry 6 quads (16 B): x(2) | y(2) | beta*x(2); entry e of lane L
// at quad (e * n_lanes + L) * 6 (hkv_kernels.hip qtab_ptr).
constexpr int QTAB_ENTRIES = QBIAS;
constexpr int QTAB_QUADS_PER_ENTRY = 6;
constexpr int QTAB_QUADS = QTAB_ENTRIES * QTAB_QUADS_PER_ENTRY;

constexpr int WG = 256;                // threads per workgroup (4 waves)

// Per-transaction index (hkv_sighash.hip, tx index kernel), AoS rows of
// TXT_WORDS words so a job's gather of its tx row is one 128-byte line.
// Offsets are absolute byte offsets into the batch's tx buffer. The three
// BIP143 hashes are stored in digest byte order (word k = bytes 4k..4k+3,
// little-endian), i.e. exactly as they appear in a preimage.
enum : int {
  TXT_FLAGS = 0,        // bit0 parsed ok, bit1 witness serialisation
  TXT_INS = 1,          // first input
  TXT_NIN = 2,
  TXT_NOUT = 3,
  TXT_OUTS_FIRST = 4,   // first output (after the count varint)
  TXT_OUTS_END = 5,     // end of outputs = start of the witness section
  TXT_LOCK = 6,         // locktime
  TXT_START = 7,        // first byte of the tx (version)
  TXT_HP = 8,           // hashPrevouts
  TXT_HS = 16,          // hashSequence
  TXT_HO = 24,          // hashOutputs
  TXT_WORDS = 32,
};
constexpr uint32_t TXF_OK = 1u, TXF_WITNESS = 2u;
// which txs the index pass computes the BIP143 per-tx hashes for
enum : uint32_t { TX_HASHES_NONE = 0, TX_HASHES_ALL = 1, TX_HASHES_WITNESS = 2 };

// minimum waves per SIMD the ecmult kernel's register allocation targets
#ifndef HKV_ECMULT_PARK  // hkv_ecmult_kernel parks Zg and the GLV signs in LDS (1) or leaves them to the allocator (0)
#define HKV_ECMULT_PARK 1
#endif
#ifndef HKV_ECMULT_WAVES
#define HKV_ECMULT_WAVES 4
#endif

}  // namespace hkv
