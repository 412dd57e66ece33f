// Checks the device lazy introsort (mc_split_begin_words / mc_split_select_words, split.hip)
// against libstdc++'s std::sort -- and against std::__introsort_loop + __final_insertion_sort
// at forced small depth limits (the heapsort fallback) -- at queried positions, several arrays
// per call, queries spread over several calls (the partitions persist between them).
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "../../include/meshclust_amd.h"

static bool cmpk(uint64_t a, uint64_t b) { return (a >> 32) < (b >> 32); }

int main(int argc, char **argv) {
  mc_ctx *ctx = nullptr;
  if (mc_ctx_create(0, &ctx) != MC_OK) {
    printf("FAIL ctx: %s\n", mc_last_error());
    return 2;
  }
  std::mt19937_64 rng(777);
  const int ncase = argc > 1 ? atoi(argv[1]) : 120;
  int cases = 0;
  for (int t = 0; t < ncase; t++) {
    const int depth = (t % 6 == 5) ? (int)(rng() % 4) : -1;
    const int64_t n = t < 24 ? t + 1
                      : depth >= 0 ? (int64_t)(rng() % 2000) + 17
                      : t == ncase - 1 ? 300000
                                       : (int64_t)(rng() % (t % 4 == 0 ? 60000 : 3000)) + 1;
    const uint32_t narr = 1 + (uint32_t)(rng() % 6);
    std::vector<uint64_t> all((size_t)narr * n);
    std::vector<std::vector<uint64_t>> want(narr);
    for (uint32_t a = 0; a < narr; a++) {
      const uint32_t kmax = (uint32_t)(1 + rng() % ((t + a) % 3 == 0 ? 4 : (t + a) % 3 == 1 ? 100 : 10001));
      std::vector<uint64_t> v(n);
      for (int64_t i = 0; i < n; i++) v[i] = ((uint64_t)(rng() % kmax) << 32) | (uint64_t)i;
      if ((t + a) % 7 == 0) std::sort(v.begin(), v.end());
      if ((t + a) % 11 == 0) std::reverse(v.begin(), v.end());
      std::copy(v.begin(), v.end(), all.begin() + (size_t)a * n);
      want[a] = v;
      if (depth < 0) {
        std::sort(want[a].begin(), want[a].end(), cmpk);
      } else if (n > 1) {
        auto c = __gnu_cxx::__ops::__iter_comp_iter(cmpk);
        std::__introsort_loop(want[a].begin(), want[a].end(), (long)depth, c);
        std::__final_insertion_sort(want[a].begin(), want[a].end(), c);
      }
    }
    if (mc_split_begin_words(ctx, all.data(), narr, (uint64_t)n, depth) != MC_OK) {
      printf("FAIL begin case %d: %s\n", t, mc_last_error());
      return 1;
    }
    // queries: every position of small arrays, else ~60 per array; in 1-4 calls
    std::vector<uint32_t> qa;
    std::vector<uint64_t> qp;
    for (uint32_t a = 0; a < narr; a++) {
      const int64_t nq = n <= 64 ? n : 60;
      for (int64_t i = 0; i < nq; i++) {
        qa.push_back(a);
        qp.push_back(n <= 64 ? (uint64_t)i : rng() % (uint64_t)n);
      }
    }
    std::vector<size_t> perm(qa.size());
    for (size_t i = 0; i < perm.size(); i++) perm[i] = i;
    std::shuffle(perm.begin(), perm.end(), rng);
    const int calls = 1 + (int)(rng() % 4);
    for (int k = 0; k < calls; k++) {
      const size_t b = perm.size() * k / calls, e = perm.size() * (k + 1) / calls;
      std::vector<uint32_t> a1;
      std::vector<uint64_t> p1, out(e - b);
      for (size_t i = b; i < e; i++) {
        a1.push_back(qa[perm[i]]);
        p1.push_back(qp[perm[i]]);
      }
      if (mc_split_select_words(ctx, a1.size(), a1.data(), p1.data(), out.data()) != MC_OK) {
        printf("FAIL select case %d: %s\n", t, mc_last_error());
        return 1;
      }
      for (size_t i = 0; i < out.size(); i++)
        if (out[i] != want[a1[i]][p1[i]]) {
          printf("MISMATCH case %d n=%lld narr=%u depth=%d array %u pos %llu: got %016llx want %016llx\n", t,
                 (long long)n, narr, depth, a1[i], (unsigned long long)p1[i], (unsigned long long)out[i],
                 (unsigned long long)want[a1[i]][p1[i]]);
          return 1;
        }
    }
    cases++;
  }
  mc_split_end(ctx);
  mc_ctx_destroy(ctx);
  printf("OK %d cases\n", cases);
  return 0;
}
