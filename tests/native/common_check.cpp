// Host-side checks of pg_common.h arithmetic (no GPU): the chunked reverse
// complement against the digit loop, and the table hash perm / unperm pair
// (a bijection of kb-bit keys: the partitioned build bins records by h's top bits).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <random>

#include "../../pangenome_amd/csrc/pg_internal.h"

int main() {
  using namespace pg;
  std::mt19937_64 g(7);
  long bad = 0, n = 0;
  for (int k = 1; k <= 27; ++k) {
    int kb = 0;
    const TableView t = make_hash(k, kb);
    const uint64_t mx = pow5(k);
    if (mx > (kb >= 64 ? ~0ull : (1ull << kb))) ++bad;           // keys < 5^k <= 2^kb
    for (int i = 0; i < 100000; ++i) {
      const uint64_t x = i == 0 ? 0 : i == 1 ? mx - 1 : g() % mx;
      ++n;
      if (t.rc(x) != rc_key(x, k)) ++bad;
      if (t.unperm(t.perm(x)) != x) ++bad;
      if (kb < 64 && (t.perm(x) >> kb) != 0) ++bad;                // h < 2^kb: the coarse bin is h's top bits
    }
  }
  std::printf("checked %ld bad %ld\n", n, bad);
  return bad != 0;
}
