// BVec construction on random length distributions: the begin bounds (from a length histogram)
// against a sort of the lengths, and per case a digest of every bin's contents after
// insert_finalize (tests/test_bvec_core.py).
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "../../meshclust_amd/csrc/host/bvec.hpp"
#include "../../meshclust_amd/csrc/host/common.hpp"

int main() {
  std::mt19937_64 rng(7);
  int bad = 0;
  for (int cs = 0; cs < 60; cs++) {
    const size_t n = 1 + rng() % (cs < 10 ? 50 : 20000);
    const uint64_t bin = 1 + rng() % (cs % 3 == 0 ? 7 : 1000);
    std::vector<uint64_t> len(n);
    const int kind = cs % 5;
    for (auto &l : len) {
      if (kind == 0) l = 1000;                                   // config B / D: one length
      else if (kind == 1) l = 990 + rng() % 21;                  // a few lengths
      else if (kind == 2) l = 8000 + rng() % 4001;               // config E's spread
      else if (kind == 3) l = rng() % 3 ? 500 : 1 + rng() % 5000;  // a dominant length and a tail
      else l = (rng() % 4 == 0) ? (1ull << 27) + rng() % 9 : 1 + rng() % 100;  // above the histogram
    }
    mc::BVec bv(len, bin);
    std::vector<uint64_t> s = len;
    std::sort(s.begin(), s.end());
    std::vector<uint64_t> want;
    for (size_t i = 0; i < n; i += bin) want.push_back(s[i]);
    if (want != bv.begin_bounds()) {
      printf("case %d: begin bounds differ\n", cs);
      bad++;
    }
    for (uint32_t id = 0; id < n; id++) bv.insert(id);
    bv.insert_finalize(1);
    uint64_t h = 1469598103934665603ull;
    for (const auto &b : bv.bins()) {
      h = (h ^ (b.size() + 0x9e37)) * 1099511628211ull;
      for (uint32_t p : b) h = (h ^ bv.static_order()[p]) * 1099511628211ull;
    }
    printf("case %d n %zu bin %llu digest %016llx\n", cs, n, (unsigned long long)bin, (unsigned long long)h);
  }
  printf(bad ? "BAD\n" : "OK\n");
  return bad ? 1 : 0;
}
