// Host test of haskoin-node_amd/csrc/hkv_plan.h (the shard planning, bitmap
// merge and device failover of hkv_api.cpp verify_from_host), built by
// tests/test_host_plan.py with -fsanitize=address,undefined: the same header
// the library compiles, driven by mock devices whose enqueue / join fail on
// a random schedule. Prints "ok <cases>" or the first failure and exits 1.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../haskoin-node_amd/csrc/hkv_plan.h"

static uint32_t verdict(size_t i) {  // a deterministic stand-in for a verdict bit
  uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull;
  z ^= z >> 29;
  return (uint32_t)(z & 1u);
}

#define CHECK(c, ...)                    \
  do {                                   \
    if (!(c)) {                          \
      std::printf("FAIL: " __VA_ARGS__); \
      std::printf("\n");                 \
      return false;                      \
    }                                    \
  } while (0)

static bool check_plan(size_t lo, size_t hi, int nd) {
  std::vector<int> devs;
  for (int k = 0; k < nd; ++k) devs.push_back(k * 3 + 1);
  const std::vector<hkv::Shard> p = hkv::plan_shards(lo, hi, devs);
  size_t at = lo;
  for (size_t k = 0; k < p.size(); ++k) {
    CHECK(p[k].lo == at, "plan gap lo=%zu hi=%zu nd=%d", lo, hi, nd);
    CHECK(p[k].hi > p[k].lo, "empty shard");
    CHECK((p[k].lo - lo) % 64 == 0, "unaligned start");
    CHECK(k == 0 || p[k].dev > p[k - 1].dev, "device order");
    at = p[k].hi;
  }
  CHECK(at == (hi > lo ? hi : lo), "plan does not cover [%zu, %zu)", lo, hi);
  CHECK(p.size() <= (size_t)nd, "too many shards");
  return true;
}

// one failover run: nd mock devices; fail_at[d] = round in which device d
// fails (-1: never), fail_join[d] = it fails at join rather than at enqueue
static bool check_failover(std::mt19937_64& rng, size_t n, int nd) {
  std::vector<int> fail_at(nd, -1);
  std::vector<bool> fail_join(nd, false);
  int n_fail = 0;
  for (int d = 0; d < nd; ++d)
    if (rng() % 3 == 0) {
      fail_at[d] = (int)(rng() % 3);
      fail_join[d] = rng() & 1;
      ++n_fail;
    }
  std::vector<bool> healthy(nd, true);
  std::vector<std::vector<uint32_t>> staging(nd);  // per-device verdict words (d.hbits)
  std::vector<int> round_of(nd, 0), pending(nd, 0), verified(n, 0), fails(nd, 0);
  std::vector<uint32_t> out((n + 31) / 32 + 1, 0xDEADBEEFu);
  const size_t out_words = (n + 31) / 32;
  auto enqueue = [&](const hkv::Shard& s) {
    if (s.dev < 0 || s.dev >= nd || !healthy[(size_t)s.dev]) return 99;  // enqueue on an unhealthy device
    if (pending[(size_t)s.dev]) return 98;  // two shards in flight on one device
    const int r = round_of[(size_t)s.dev]++;
    if (fail_at[(size_t)s.dev] == r && !fail_join[(size_t)s.dev]) return -4;
    std::vector<uint32_t>& w = staging[(size_t)s.dev];
    w.assign((s.hi - s.lo + 31) / 32, 0);
    for (size_t i = s.lo; i < s.hi; ++i) w[(i - s.lo) / 32] |= verdict(i) << ((i - s.lo) % 32);
    pending[(size_t)s.dev] = 1;
    return 0;
  };
  auto join = [&](const hkv::Shard& s) {
    pending[(size_t)s.dev] = 0;
    if (fail_at[(size_t)s.dev] == round_of[(size_t)s.dev] - 1 && fail_join[(size_t)s.dev]) return -4;
    if (!hkv::merge_shard_words(out.data(), out_words, staging[(size_t)s.dev].data(), s)) return 97;
    for (size_t i = s.lo; i < s.hi; ++i) ++verified[i];
    return 0;
  };
  auto on_fail = [&](int dev, int) { ++fails[(size_t)dev]; };
  const int rc = hkv::run_with_failover(n, healthy, enqueue, join, on_fail);
  CHECK(rc != 97 && rc != 98 && rc != 99, "harness violation rc=%d", rc);
  bool any_left = false;
  for (int d = 0; d < nd; ++d) {
    CHECK(fails[d] <= 1, "device reported twice");
    CHECK(healthy[d] == (fails[d] == 0), "health flag vs reports");
    any_left = any_left || healthy[d];
  }
  if (rc == 0) {
    for (size_t i = 0; i < n; ++i) {
      CHECK(verified[i] == 1, "record %zu verified %d times (n=%zu nd=%d)", i, verified[i], n, nd);
      CHECK(((out[i / 32] >> (i % 32)) & 1u) == verdict(i), "verdict bit %zu", i);
    }
    CHECK(out[out_words] == 0xDEADBEEFu, "write past the bitmap");
  } else {
    CHECK(!any_left, "failed with healthy devices left (rc=%d)", rc);
    for (size_t i = 0; i < n; ++i) CHECK(verified[i] <= 1, "record %zu verified twice", i);
  }
  return true;
}

int main() {
  std::mt19937_64 rng(0x504C414E);
  size_t cases = 0;
  for (int nd = 1; nd <= 9; ++nd)
    for (size_t n : {0ul, 1ul, 31ul, 32ul, 63ul, 64ul, 65ul, 127ul, 128ul, 129ul, 1000ul, 4097ul}) {
      for (size_t lo : {0ul, 64ul, 640ul})
        if (!check_plan(lo, lo + n, nd)) return 1;
      ++cases;
    }
  for (int it = 0; it < 20000; ++it) {
    const int nd = 1 + (int)(rng() % 8);
    const size_t n = (rng() % 4) == 0 ? rng() % 70 : rng() % 6000;
    if (!check_failover(rng, n, nd)) return 1;
    ++cases;
  }
  // every device fails: an error, never a partial success
  {
    std::vector<bool> healthy(3, true);
    int fails = 0;
    const int rc = hkv::run_with_failover(
        1000, healthy, [](const hkv::Shard&) { return -4; }, [](const hkv::Shard&) { return 0; },
        [&](int, int) { ++fails; });
    if (rc != -4 || fails != 3) {
      std::printf("FAIL: all-fail rc=%d fails=%d\n", rc, fails);
      return 1;
    }
    // an allocation failure (HKV_E_OOM = -3) on one device ends the call with
    // that error but takes no device out of service: nothing is re-sharded,
    // the shards already started are joined, and the next call uses every
    // device again (one OOM must not cascade over the context)
    for (int fail_dev = 0; fail_dev < 3; ++fail_dev) {
      std::vector<bool> h3(3, true);
      int reported = 0, enq = 0, joins = 0;
      std::vector<int> in_flight(3, 0);
      const int rc2 = hkv::run_with_failover(
          5000, h3,
          [&](const hkv::Shard& s) {
            if (s.dev == fail_dev) return -3;
            ++enq;
            in_flight[(size_t)s.dev] = 1;
            return 0;
          },
          [&](const hkv::Shard& s) {
            ++joins;
            in_flight[(size_t)s.dev] = 0;
            return 0;
          },
          [&](int, int) { ++reported; });
      if (rc2 != -3 || reported != 0 || !(h3[0] && h3[1] && h3[2]) || joins != enq || in_flight[0] + in_flight[1] + in_flight[2]) {
        std::printf("FAIL: alloc failure dev=%d rc=%d reported=%d enq=%d joins=%d\n", fail_dev, rc2, reported, enq,
                    joins);
        return 1;
      }
      int used = 0;
      if (hkv::run_with_failover(5000, h3, [&](const hkv::Shard&) { ++used; return 0; },
                                 [](const hkv::Shard&) { return 0; }, [](int, int) {}) != 0 || used != 3) {
        std::printf("FAIL: devices not reused after an allocation failure\n");
        return 1;
      }
      // the same at join: the error is returned, every started shard joined
      std::vector<bool> h4(3, true);
      int joined = 0;
      const int rc3 = hkv::run_with_failover(
          5000, h4, [](const hkv::Shard&) { return 0; },
          [&](const hkv::Shard& s) { ++joined; return s.dev == fail_dev ? -3 : 0; }, [](int, int) {});
      if (rc3 != -3 || joined != 3 || !(h4[0] && h4[1] && h4[2])) {
        std::printf("FAIL: alloc failure at join dev=%d rc=%d joined=%d\n", fail_dev, rc3, joined);
        return 1;
      }
    }
    std::vector<bool> none(2, false);
    if (hkv::run_with_failover(10, none, [](const hkv::Shard&) { return 0; }, [](const hkv::Shard&) { return 0; },
                               [](int, int) {}) != -2) {
      std::printf("FAIL: no healthy device\n");
      return 1;
    }
  }
  std::printf("ok %zu\n", cases);
  return 0;
}
