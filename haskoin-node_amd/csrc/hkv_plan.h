// hkv_plan.h — host-side shard planning, bitmap merging and device failover
// for the multi-device entry points (hkv_api.cpp verify_from_host). Pure C++
// (no HIP), so tests/host_plan.cpp drives exactly this code under ASan and
// UBSan on the CPU.
//
// Failover follows SURVEY.md §5 ("per-GPU failure -> re-shard onto the
// remaining GPUs"), the library counterpart of the reference's supervised
// peers: a peer that dies is removed and its work goes elsewhere
// (/root/reference/src/Haskoin/Node/PeerMgr.hs:215,230,383, PeerDied).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <cstring>
#include <vector>

namespace hkv {

struct Shard {
  size_t lo = 0, hi = 0;  // records [lo, hi)
  int dev = -1;           // context device index
};

// Contiguous shards of [lo, hi) over devs (context device indices), in
// order: every start is 64-aligned relative to lo (a wave's ballot word pair
// never straddles two shards; lo itself is 64-aligned by the callers), the
// last device takes the remainder; empty shards are dropped. The same rule
// as haskoin-node_amd/hkv/shard.py shard_bounds.
inline std::vector<Shard> plan_shards(size_t lo, size_t hi, const std::vector<int>& devs) {
  std::vector<Shard> out;
  if (hi <= lo || devs.empty()) return out;
  const size_t n = hi - lo, nd = devs.size();
  size_t per = (n + nd - 1) / nd;
  per = (per + 63) / 64 * 64;
  for (size_t k = 0; k < nd; ++k) {
    Shard s;
    s.lo = lo + (k * per < n ? k * per : n);
    s.hi = lo + ((k * per + per) < n ? k * per + per : n);
    if (k + 1 == nd) s.hi = hi;
    s.dev = devs[k];
    if (s.hi > s.lo) out.push_back(s);
  }
  return out;
}

// Copy a shard's verdict words (bit 0 = record s.lo) into the caller's
// bitmap of out_words words. s.lo must be a multiple of 32; false when the
// shard does not fit (the caller's arithmetic is wrong: nothing is written).
inline bool merge_shard_words(uint32_t* out, size_t out_words, const uint32_t* words, const Shard& s) {
  if (s.lo % 32 != 0 || s.hi < s.lo) return false;
  const size_t w = (s.hi - s.lo + 31) / 32;
  if (s.lo / 32 + w > out_words) return false;
  if (w) std::memcpy(out + s.lo / 32, words, w * sizeof(uint32_t));
  return true;
}

// Only a HIP runtime error from the device's own streams, launches or
// synchronisation (HKV_E_HIP = -4) says the device is bad. Allocation
// failures (HKV_E_OOM), argument and internal errors are the call's, not the
// device's: re-sharding them onto the other devices would need even larger
// buffers there, so one out-of-memory would cascade over every device.
inline bool is_device_fault(int rc) { return rc == -4; }

// Run [0, n) over the healthy devices with failover. enqueue(shard) starts a
// shard on its device and returns 0 or an error; join(shard) waits for it
// and merges its verdicts, returning 0 or an error. A round starts at most
// one shard per device (a device's staging buffers hold one shard) and joins
// every shard it started. A device whose enqueue or join fails with a device
// fault (is_device_fault) is marked unhealthy (healthy[dev] = false), and its
// shards — the failed one and any still queued for it — are re-planned over
// the devices still healthy, round after round, until all of [0, n) is
// verified (returns 0) or no healthy device is left (returns the last error,
// or -2 = HKV_E_NODEV when none was healthy to begin with). Shards that
// completed are never re-run. on_fail(dev, rc) is told about each device's
// first failure. Any other error ends the call: no further shard is started,
// the shards already started are joined (their copies still read the
// caller's records), no device changes health, and that error is returned.
template <class Enqueue, class Join, class OnFail>
int run_with_failover(size_t n, std::vector<bool>& healthy, Enqueue enqueue, Join join, OnFail on_fail) {
  auto healthy_devs = [&]() {
    std::vector<int> devs;
    for (size_t k = 0; k < healthy.size(); ++k)
      if (healthy[k]) devs.push_back((int)k);
    return devs;
  };
  std::vector<int> devs = healthy_devs();
  if (devs.empty()) return -2;
  std::vector<Shard> todo = plan_shards(0, n, devs);
  int last_rc = 0;
  auto fail = [&](int dev, int rc) {
    last_rc = rc;
    if (healthy[(size_t)dev]) on_fail(dev, rc);
    healthy[(size_t)dev] = false;
  };
  int abort_rc = 0;  // first non-device error: the call ends after this round's joins
  while (!todo.empty()) {
    std::vector<Shard> round, rest, started, failed;
    std::vector<bool> busy(healthy.size(), false);
    for (const Shard& s : todo) {
      if (!healthy[(size_t)s.dev]) failed.push_back(s);
      else if (busy[(size_t)s.dev]) rest.push_back(s);
      else {
        busy[(size_t)s.dev] = true;
        round.push_back(s);
      }
    }
    for (const Shard& s : round) {
      if (abort_rc) break;
      const int rc = healthy[(size_t)s.dev] ? enqueue(s) : 0;
      if (!healthy[(size_t)s.dev]) failed.push_back(s);
      else if (rc && !is_device_fault(rc)) abort_rc = rc;
      else if (rc) {
        fail(s.dev, rc);
        failed.push_back(s);
      } else {
        started.push_back(s);
      }
    }
    for (const Shard& s : started) {
      const int rc = join(s);
      if (rc && !is_device_fault(rc)) {
        if (!abort_rc) abort_rc = rc;
      } else if (rc) {
        fail(s.dev, rc);
        failed.push_back(s);
      }
    }
    if (abort_rc) return abort_rc;
    todo.clear();
    for (const Shard& s : rest) (healthy[(size_t)s.dev] ? todo : failed).push_back(s);
    if (failed.empty()) continue;
    devs = healthy_devs();
    if (devs.empty()) return last_rc ? last_rc : -2;
    for (const Shard& f : failed) {
      const std::vector<Shard> sub = plan_shards(f.lo, f.hi, devs);
      todo.insert(todo.end(), sub.begin(), sub.end());
    }
  }
  return 0;
}

}  // namespace hkv
