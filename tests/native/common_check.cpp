// Host-side checks of pg_common.h arithmetic (no GPU): the chunked reverse
// complement against the digit loop, and the table hash perm / unperm pair.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <random>

#include "../../pangenome_amd/csrc/pg_internal.h"

int main() {
  using namespace pg;
  std::mt19937_64 g(7);
  long bad = 0, n = 0;
  for (int k = 1; k <= 27; ++k) {
    uint64_t buckets, ovf;
    const TableView t = make_geometry(k, 1000000, buckets, ovf);
    const uint64_t mx = pow5(k);
    for (int i = 0; i < 100000; ++i) {
      const uint64_t x = i == 0 ? 0 : i == 1 ? mx - 1 : g() % mx;
      ++n;
      if (t.rc(x) != rc_key(x, k)) ++bad;
      if (t.unperm(t.perm(x)) != x) ++bad;
    }
  }
  std::printf("checked %ld bad %ld\n", n, bad);
  return bad != 0;
}
