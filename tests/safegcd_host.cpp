// Host build of haskoin-node_amd/csrc/hkv_safegcd.h for tests/test_safegcd.py:
// reads 64-hex-digit values (one per line) and prints their inverses mod n,
// or mod p with the argument "p".
#include <cstdio>
#include <cstring>

#include "../haskoin-node_amd/csrc/hkv_safegcd.h"

int main(int argc, char** argv) {
  const bool mod_p = argc > 1 && argv[1][0] == 'p';
  char line[128];
  while (std::fgets(line, sizeof line, stdin)) {
    if (std::strlen(line) < 64) continue;
    uint32_t a[8], r[8];
    for (int w = 0; w < 8; ++w) {
      unsigned x = 0;
      std::sscanf(line + 8 * (7 - w), "%8x", &x);
      a[w] = x;
    }
    if (mod_p)
      hkv::sgcd::inv_mod_p(r, a);
    else
      hkv::sgcd::inv_mod_n(r, a);
    for (int w = 7; w >= 0; --w) std::printf("%08x", r[w]);
    std::printf("\n");
  }
  return 0;
}
