// Checks mc::LazyIntroSort (meshclust_amd/csrc/host/lazysort.hpp) against libstdc++'s own
// std::sort, and against libstdc++'s internal __introsort_loop + __final_insertion_sort with
// a forced small depth limit (heapsort fallback), at every position, in random query orders.
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "../../meshclust_amd/csrc/host/lazysort.hpp"

static bool cmpk(uint64_t a, uint64_t b) { return (a >> 32) < (b >> 32); }

int main() {
  std::mt19937_64 rng(12345);
  int cases = 0;
  for (int t = 0; t < 400; t++) {
    const int64_t n = t < 40 ? t : (int64_t)(rng() % (t < 300 ? 3000 : 60000)) + 1;
    const uint32_t kmax = (uint32_t)(1 + rng() % (t % 3 == 0 ? 4 : t % 3 == 1 ? 100 : 10000));
    std::vector<uint64_t> a(n);
    for (int64_t i = 0; i < n; i++) a[i] = ((uint64_t)(rng() % kmax) << 32) | (uint64_t)i;
    if (t % 7 == 0) std::sort(a.begin(), a.end());            // presorted input
    if (t % 11 == 0) std::reverse(a.begin(), a.end());        // reversed input
    const int depth = (t % 5 == 0 && n > 16) ? (int)(rng() % 4) : -1;
    std::vector<uint64_t> want = a;
    if (depth < 0) {
      std::sort(want.begin(), want.end(), cmpk);
    } else if (n > 1) {
      auto c = __gnu_cxx::__ops::__iter_comp_iter(cmpk);
      std::__introsort_loop(want.begin(), want.end(), (long)depth, c);
      std::__final_insertion_sort(want.begin(), want.end(), c);
    }
    mc::LazyIntroSort lz(a, depth);
    std::vector<int64_t> q(n);
    for (int64_t i = 0; i < n; i++) q[i] = i;
    std::shuffle(q.begin(), q.end(), rng);
    const int64_t nq = (t % 2) ? std::min<int64_t>(n, 40) : n;
    for (int64_t i = 0; i < nq; i++)
      if (lz.at(q[i]) != want[q[i]]) {
        printf("MISMATCH case %d n=%lld kmax=%u depth=%d pos=%lld\n", t, (long long)n, kmax, depth, (long long)q[i]);
        return 1;
      }
    std::vector<uint64_t> full = a;  // the whole-array form, partitions run as OpenMP tasks
#pragma omp parallel num_threads(4)
#pragma omp single
    mc::LazyIntroSort::sort_words(full.data(), n, depth, 64);
    if (full != want) {
      printf("MISMATCH sort_words case %d n=%lld kmax=%u depth=%d\n", t, (long long)n, kmax, depth);
      return 1;
    }
    // ... with every range of 17 words or more partitioned by the team (hoare_cut_par)
    full = a;
    mc::LazyIntroSort::par_min = 17;
#pragma omp parallel num_threads(4)
#pragma omp single
    mc::LazyIntroSort::sort_words(full.data(), n, depth, 64);
    mc::LazyIntroSort::par_min = 32768;
    if (full != want) {
      printf("MISMATCH sort_words (parallel cuts) case %d n=%lld kmax=%u depth=%d\n", t, (long long)n, kmax, depth);
      return 1;
    }
    cases++;
  }
  printf("OK %d cases\n", cases);
  return 0;
}
