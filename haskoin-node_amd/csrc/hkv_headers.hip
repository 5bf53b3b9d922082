// hkv_headers.hip — batch block-header checks.
//
// The data-parallel part of haskoin-node's header sync: importHeaders
// (/root/reference/src/Haskoin/Node/Chain.hs:500-520) hands each peer's
// `headers` message (up to 2,000 headers) to haskoin-core connectBlocks
// [dep, haskoin-core-1.1.0, stack.yaml:10], which for every header computes
// headerHash (SHA-256d of the 80-byte wire form) and checks isValidPOW and
// that the header extends its predecessor. Those three are independent per
// header and run here, one lane per header:
//
//   hkv_header_kernel  SHA-256d (2 + 1 compressions), decodeCompact of the
//                      bits field, isValidPOW against powLimit, and the prev
//                      field of header i == hash of header i-1 (header 0
//                      against the caller's tip hash), the predecessor's hash
//                      read from LDS.
//
// Memory: a workgroup's 256 headers (20,480 contiguous bytes: its 255 own and
// the one before them) are staged into LDS by coalesced dword loads, then each
// lane reads its own 20 words. The
// work is 3 SHA-256 compressions per 80-byte header: latency- and ALU-light,
// far below both the VALU and HBM rooflines at sync batch sizes (a 2,000-
// header message is 160 KB); DESIGN.md records the measured rate.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hkv_hash.h"
#include "hkv_layout.h"
#include "hkv_internal.h"
#include "../../include/hkv.h"

namespace hkv {

constexpr int HDR_WORDS = 20;  // 80 bytes

// haskoin-core decodeCompact (Haskoin.Block.Common) [dep]: the Bitcoin
// "compact" target. Writes the target as 8 little-endian limbs when it does
// not overflow. Returns the HKV_HDR_{NEGATIVE,OVERFLOW,ZERO_TARGET} flags.
HKV_DEV uint32_t decode_compact(uint32_t bits, uint32_t t[8]) {
  const uint32_t size = bits >> 24;
  const uint32_t w0 = bits & 0x007FFFFFu;
  const uint32_t word = size <= 3 ? (w0 >> (8 * (3 - size))) : w0;
  uint32_t fl = 0;
  if (word != 0 && (bits & 0x00800000u)) fl |= HKV_HDR_NEGATIVE;
  if (word != 0 && (size > 34 || (word > 0xFFu && size > 33) || (word > 0xFFFFu && size > 32)))
    fl |= HKV_HDR_OVERFLOW;
  if (word == 0) fl |= HKV_HDR_ZERO_TARGET;
  // value = word << 8*(size-3) (size > 3); fits 256 bits whenever !overflow
  const uint32_t s = size > 3 ? 8u * (size - 3u) : 0u;
  const uint64_t v = (uint64_t)word << (s & 31u);
  const uint32_t li = s >> 5;
#pragma unroll
  for (int j = 0; j < 8; ++j) t[j] = ((uint32_t)j == li) ? (uint32_t)v : ((uint32_t)j == li + 1) ? (uint32_t)(v >> 32) : 0u;
  return fl;
}

// a > b for 8-limb little-endian integers
HKV_DEV bool u256_gt(const uint32_t a[8], const uint32_t b[8]) {
  bool gt = false, decided = false;
#pragma unroll
  for (int j = 7; j >= 0; --j) {
    gt = decided ? gt : (a[j] > b[j]);
    decided = decided || (a[j] != b[j]);
  }
  return gt;
}

// One workgroup owns HDR_OWN = WG - 1 consecutive headers: lane t hashes
// header base - 1 + t, so lane 0 recomputes the last header of the previous
// workgroup (in workgroup 0 it idles and header 0 links against the caller's
// tip) and every prev-field check reads its predecessor's hash from LDS. One
// launch instead of a hash kernel and a link kernel that re-read the hashes,
// at 1/256 extra hashing.
constexpr uint32_t HDR_OWN = WG - 1;

__global__ void __launch_bounds__(WG) hkv_header_kernel(const uint32_t* __restrict__ hdrs, uint32_t n,
                                                        const uint32_t* __restrict__ pow_limit,
                                                        const uint32_t* __restrict__ prev0,
                                                        uint32_t* __restrict__ hashes, uint8_t* __restrict__ status) {
  __shared__ uint32_t lds[WG * HDR_WORDS];
  __shared__ uint32_t lh[WG * 8];
  const uint32_t t = threadIdx.x;
  const uint32_t base = blockIdx.x * HDR_OWN;  // the first header this workgroup owns (lane 1)
  const uint32_t s0 = blockIdx.x == 0 ? 1u : 0u;  // workgroup 0 has no predecessor slot
  const uint32_t first = base + s0 - 1;          // header in slot s0
  const uint32_t last = min(base + HDR_OWN, n);  // one past the last staged header
  const uint32_t cnt = last - first;
  const uint32_t* src = hdrs + (size_t)first * HDR_WORDS;
  uint32_t* dst = lds + s0 * HDR_WORDS;
  for (uint32_t k = t; k < cnt * HDR_WORDS; k += WG) dst[k] = src[k];
  __syncthreads();
  // slot t holds header base - 1 + t
  const bool staged = t >= s0 && t < s0 + cnt;
  const uint32_t i = base + t - 1;
  uint32_t h[HDR_WORDS], hv[8];
  uint32_t fl = 0;
  if (staged) {
#pragma unroll
    for (int k = 0; k < HDR_WORDS; ++k) h[k] = lds[t * HDR_WORDS + k];

    // SHA-256 of the 80 bytes: block 1 = words 0..15, block 2 = words 16..19 + padding
    uint32_t st[8], w[16];
    sha256_init(st);
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = __builtin_bswap32(h[k]);
    sha256_compress(st, w);
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = __builtin_bswap32(h[16 + k]);
    w[4] = 0x80000000u;
#pragma unroll
    for (int k = 5; k < 15; ++k) w[k] = 0;
    w[15] = 640;
    sha256_compress(st, w);
    uint32_t d[8];
    sha256_of_digest(d, st);

    // headerHash bytes in digest order == little-endian limbs of headerPOW
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      hv[k] = __builtin_bswap32(d[k]);
      lh[t * 8 + k] = hv[k];
    }

    // isValidPOW
    uint32_t tgt[8], lim[8];
    fl = decode_compact(h[18], tgt);
#pragma unroll
    for (int k = 0; k < 8; ++k) lim[k] = pow_limit[k];
    if (!(fl & HKV_HDR_OVERFLOW)) {
      if (u256_gt(tgt, lim)) fl |= HKV_HDR_ABOVE_LIMIT;
      if (u256_gt(hv, tgt)) fl |= HKV_HDR_HASH_ABOVE;
    }
    if (!(fl & (HKV_HDR_NEGATIVE | HKV_HDR_OVERFLOW | HKV_HDR_ZERO_TARGET | HKV_HDR_ABOVE_LIMIT | HKV_HDR_HASH_ABOVE)))
      fl |= HKV_HDR_POW_OK;
  }
  __syncthreads();
  if (!staged || t == 0) return;  // lane 0 only supplied its hash
  // prev field (words 1..8) against the hash of header i - 1 (header 0:
  // the caller's tip, or linked by definition without one)
  const uint32_t* q = i ? lh + (t - 1) * 8 : prev0;
  uint32_t diff = 0;
  if (q) {
#pragma unroll
    for (int k = 0; k < 8; ++k) diff |= h[1 + k] ^ q[k];
  }
  if (diff == 0) fl |= HKV_HDR_LINK_OK;
  uint32_t* out = hashes + (size_t)i * 8;
#pragma unroll
  for (int k = 0; k < 8; k += 4) *reinterpret_cast<uint4*>(out + k) = make_uint4(hv[k], hv[k + 1], hv[k + 2], hv[k + 3]);
  status[i] = (uint8_t)fl;
}

// ---------------------------------------------------------------------------
// Block merkle roots. The reference's own block test
// asserts b.header.merkle == buildMerkleRoot (txHash <$> b.txs)
// (/root/reference/test/Haskoin/NodeSpec.hs:185-193) on blocks fetched by
// getBlocks (src/Haskoin/Node/Peer.hs:309-344); buildMerkleRoot is
// haskoin-core-1.1.0 Haskoin.Block.Merkle [dep]: pairwise SHA-256d of
// 64-byte concatenations, an odd level's last hash paired with itself.
// `mutated` is Bitcoin Core's CVE-2012-2459 flag (two equal hashes paired
// at any level), so a caller can reject a duplicated-tx block whose root
// still matches.
//
// One workgroup per block: a 256-lane sweep per level, levels separated by
// workgroup barriers, the tree built in place in the block's own scratch
// range (chunk k writes [256k, 256k+256) after chunk k/2 has read it).
// Algorithmic work: 3 SHA-256 compressions per inner node (n - 1 nodes per
// n-leaf block), 96 B of traffic per node.

// SHA-256d of a||b, both 32-byte digests held as little-endian words of the
// digest bytes; out in the same form.
HKV_DEV void sha256d_pair(uint32_t out[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t st[8], w[16];
  sha256_init(st);
#pragma unroll
  for (int k = 0; k < 8; ++k) { w[k] = __builtin_bswap32(a[k]); w[8 + k] = __builtin_bswap32(b[k]); }
  sha256_compress(st, w);
  w[0] = 0x80000000u;
#pragma unroll
  for (int k = 1; k < 15; ++k) w[k] = 0;
  w[15] = 512;
  sha256_compress(st, w);
  uint32_t d[8];
  sha256_of_digest(d, st);
#pragma unroll
  for (int k = 0; k < 8; ++k) out[k] = __builtin_bswap32(d[k]);
}

HKV_DEV void load8(uint32_t v[8], const uint32_t* p) {
  const uint4 x = *reinterpret_cast<const uint4*>(p), y = *reinterpret_cast<const uint4*>(p + 4);
  v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
}
HKV_DEV void store8(uint32_t* p, const uint32_t v[8]) {
  *reinterpret_cast<uint4*>(p) = make_uint4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<uint4*>(p + 4) = make_uint4(v[4], v[5], v[6], v[7]);
}

__global__ void __launch_bounds__(WG) hkv_merkle_kernel(const uint32_t* __restrict__ leaves,
                                                        const uint32_t* __restrict__ offsets,
                                                        uint32_t* __restrict__ scratch, uint32_t* __restrict__ roots,
                                                        uint8_t* __restrict__ mutated) {
  const uint32_t blk = blockIdx.x;
  const uint32_t off = offsets[blk];
  uint32_t cnt = offsets[blk + 1] - off;
  const uint32_t* src = leaves + (size_t)off * 8;
  uint32_t* tree = scratch + (size_t)off * 8;
  int mut = 0;
  while (cnt > 1) {  // cnt is workgroup-uniform: every barrier below is reached by all lanes
    const uint32_t half = (cnt + 1) >> 1;
    for (uint32_t base = 0; base < half; base += WG) {
      const uint32_t i = base + threadIdx.x;
      uint32_t o[8];
      if (i < half) {
        uint32_t a[8], b[8];
        const uint32_t j = 2 * i + 1 < cnt ? 2 * i + 1 : cnt - 1;
        load8(a, src + (size_t)(2 * i) * 8);
        load8(b, src + (size_t)j * 8);
        if (j != 2 * i) {
          uint32_t diff = 0;
#pragma unroll
          for (int k = 0; k < 8; ++k) diff |= a[k] ^ b[k];
          mut |= diff == 0;
        }
        sha256d_pair(o, a, b);
      }
      __syncthreads();  // this chunk's reads precede its in-place writes
      if (i < half) store8(tree + (size_t)i * 8, o);
      __syncthreads();
    }
    src = tree;
    cnt = half;
  }
  mut = __syncthreads_or(mut);
  if (threadIdx.x == 0) {
    uint32_t r[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (cnt == 1) load8(r, src);  // cnt == 0: an empty block, all-zero root
    store8(roots + (size_t)blk * 8, r);
    mutated[blk] = (uint8_t)(mut != 0);
  }
}

// Few-block batches: each block's tree is cut into MERKLE_SPLIT aligned
// subtrees of 2^H leaves (H smallest with ceil(n / 2^H) <= MERKLE_SPLIT), one
// workgroup each, so a lone block's lower levels run on several CUs. An
// aligned subtree root is a node of the full tree; the rightmost one, when it
// collapses below height H, is paired with itself up to H exactly as the full
// tree's odd-level rule does. Subtree root -> its slot 0 in scratch, its
// mutated flag -> word 0 of slot 1 (written only when it has >= 2 leaves).
// hkv_merkle_top_kernel then joins the m <= MERKLE_SPLIT roots per block.
constexpr uint32_t MERKLE_SPLIT = 8;

HKV_DEV uint32_t merkle_split_height(uint32_t cnt) {
  uint32_t h = 0;
  while (((cnt + (1u << h) - 1) >> h) > MERKLE_SPLIT) ++h;
  return h;
}

__global__ void __launch_bounds__(WG) hkv_merkle_sub_kernel(const uint32_t* __restrict__ leaves,
                                                            const uint32_t* __restrict__ offsets,
                                                            uint32_t* __restrict__ scratch) {
  const uint32_t blk = blockIdx.x / MERKLE_SPLIT, sub = blockIdx.x % MERKLE_SPLIT;
  const uint32_t off = offsets[blk];
  const uint32_t total = offsets[blk + 1] - off;
  if (total < 2) return;
  const uint32_t H = merkle_split_height(total);
  const uint32_t m = (total + (1u << H) - 1) >> H;
  const uint32_t start = sub << H;
  if (start >= total) return;  // all three returns are workgroup-uniform
  const uint32_t c0 = min(1u << H, total - start);
  uint32_t cnt = c0;
  const uint32_t* src = leaves + (size_t)(off + start) * 8;
  uint32_t* tree = scratch + (size_t)(off + start) * 8;
  uint32_t level = 0;
  int mut = 0;
  while (cnt > 1) {
    const uint32_t half = (cnt + 1) >> 1;
    for (uint32_t base = 0; base < half; base += WG) {
      const uint32_t i = base + threadIdx.x;
      uint32_t o[8];
      if (i < half) {
        uint32_t a[8], b[8];
        const uint32_t j = 2 * i + 1 < cnt ? 2 * i + 1 : cnt - 1;
        load8(a, src + (size_t)(2 * i) * 8);
        load8(b, src + (size_t)j * 8);
        if (j != 2 * i) {
          uint32_t diff = 0;
#pragma unroll
          for (int k = 0; k < 8; ++k) diff |= a[k] ^ b[k];
          mut |= diff == 0;
        }
        sha256d_pair(o, a, b);
      }
      __syncthreads();
      if (i < half) store8(tree + (size_t)i * 8, o);
      __syncthreads();
    }
    src = tree;
    cnt = half;
    ++level;
  }
  mut = __syncthreads_or(mut);
  if (threadIdx.x == 0) {
    uint32_t x[8];
    load8(x, src);
    if (m > 1)
      for (; level < H; ++level) sha256d_pair(x, x, x);
    store8(tree, x);
    if (c0 >= 2) tree[8] = (uint32_t)(mut != 0);
  }
}

__global__ void __launch_bounds__(64) hkv_merkle_top_kernel(const uint32_t* __restrict__ leaves,
                                                            const uint32_t* __restrict__ offsets,
                                                            const uint32_t* __restrict__ scratch,
                                                            uint32_t* __restrict__ roots,
                                                            uint8_t* __restrict__ mutated) {
  __shared__ uint32_t node[MERKLE_SPLIT][8];
  const uint32_t blk = blockIdx.x;
  const uint32_t off = offsets[blk];
  const uint32_t total = offsets[blk + 1] - off;
  const uint32_t t = threadIdx.x;
  if (total < 2) {  // block-uniform
    if (t == 0) {
      uint32_t r[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (total == 1) load8(r, leaves + (size_t)off * 8);
      store8(roots + (size_t)blk * 8, r);
      mutated[blk] = 0;
    }
    return;
  }
  const uint32_t H = merkle_split_height(total);
  uint32_t cnt = (total + (1u << H) - 1) >> H;
  int mut = 0;
  if (t < cnt) {
    const uint32_t* p = scratch + (size_t)(off + (t << H)) * 8;
    load8(node[t], p);
    const uint32_t ct = min(1u << H, total - (t << H));
    if (ct >= 2) mut = p[8] != 0;
  }
  __syncthreads();
  while (cnt > 1) {  // at most 3 levels of <= 4 pairs
    const uint32_t half = (cnt + 1) >> 1;
    uint32_t o[8];
    if (t < half) {
      const uint32_t j = 2 * t + 1 < cnt ? 2 * t + 1 : cnt - 1;
      if (j != 2 * t) {
        uint32_t diff = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) diff |= node[2 * t][k] ^ node[j][k];
        mut |= diff == 0;
      }
      sha256d_pair(o, node[2 * t], node[j]);
    }
    __syncthreads();
    if (t < half)
#pragma unroll
      for (int k = 0; k < 8; ++k) node[t][k] = o[k];
    __syncthreads();
    cnt = half;
  }
  mut = __syncthreads_or(mut);
  if (t == 0) {
    store8(roots + (size_t)blk * 8, node[0]);
    mutated[blk] = (uint8_t)(mut != 0);
  }
}

hipError_t launch_merkle(const uint8_t* leaves, const uint32_t* offsets, uint32_t n_blocks, uint8_t* scratch,
                         uint8_t* roots, uint8_t* mutated, uint32_t n_cu, hipStream_t st) {
  if (n_blocks == 0) return hipSuccess;
  if (n_blocks <= n_cu) {  // no more blocks than CUs: split each tree over MERKLE_SPLIT workgroups
    hipLaunchKernelGGL(hkv_merkle_sub_kernel, dim3(n_blocks * MERKLE_SPLIT), dim3(WG), 0, st,
                       reinterpret_cast<const uint32_t*>(leaves), offsets, reinterpret_cast<uint32_t*>(scratch));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(hkv_merkle_top_kernel, dim3(n_blocks), dim3(64), 0, st,
                       reinterpret_cast<const uint32_t*>(leaves), offsets,
                       reinterpret_cast<const uint32_t*>(scratch), reinterpret_cast<uint32_t*>(roots), mutated);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(hkv_merkle_kernel, dim3(n_blocks), dim3(WG), 0, st, reinterpret_cast<const uint32_t*>(leaves),
                     offsets, reinterpret_cast<uint32_t*>(scratch), reinterpret_cast<uint32_t*>(roots), mutated);
  return hipGetLastError();
}

hipError_t launch_headers(const uint8_t* hdrs, uint32_t n, const uint8_t* pow_limit, const uint8_t* prev0,
                          uint8_t* hashes, uint8_t* status, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const uint32_t blocks = (n + HDR_OWN - 1) / HDR_OWN;
  hipLaunchKernelGGL(hkv_header_kernel, dim3(blocks), dim3(WG), 0, st, reinterpret_cast<const uint32_t*>(hdrs), n,
                     reinterpret_cast<const uint32_t*>(pow_limit), reinterpret_cast<const uint32_t*>(prev0),
                     reinterpret_cast<uint32_t*>(hashes), status);
  return hipGetLastError();
}

}  // namespace hkv
