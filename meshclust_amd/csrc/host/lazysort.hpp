// lazysort.hpp -- the permutation std::sort (libstdc++, GCC 11) gives, evaluated lazily.
//
// Trainer::split (Trainer.cpp:691-701) sorts all N points by their distance to each of the
// 150 pivots with std::sort -- an unstable introsort, so the order among equal keys (keys are
// integers <= 10000: ties are everywhere) is defined only by that algorithm -- and then reads
// ~35 positions of each sorted array (the alignment binary search and the 20 samples).
// This class reproduces libstdc++'s std::sort result at any queried position without sorting
// the whole array: introsort's partitions act on disjoint ranges, so only the ranges that
// contain a queried position need to be partitioned, recursively, exactly as
// std::__introsort_loop would (median-of-three to first, unguarded Hoare partition, the
// depth limit 2*floor(log2 N) with heapsort fallback).  The final insertion sort never moves
// an element across a partition boundary (every element left of a cut is <= every element
// right of it and insertion sort moves only strictly smaller elements), so it equals a
// stable insertion sort of each leaf range.
//
// Elements are 64-bit words compared by their upper 32 bits (key << 32 | payload), the
// split comparator `a->distance(*p) < b->distance(*p)` on (key, id) words.
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace mc {

class LazyIntroSort {
 public:
  // Takes the input sequence (the array std::sort would be called on).
  explicit LazyIntroSort(std::vector<uint64_t> a, int depth_override = -1) : a_(std::move(a)) {
    const int64_t n = (int64_t)a_.size();
    int lg = 0;
    while (n >> (lg + 1)) lg++;
    nodes_.push_back(Node{0, n, depth_override >= 0 ? depth_override : 2 * lg, -1, 0, false});
  }

  // Element at position pos of the sorted array.
  uint64_t at(int64_t pos) {
    int idx = 0;
    for (;;) {
      Node &nd = nodes_[idx];
      if (nd.final) return a_[pos];
      if (nd.left < 0) {
        expand(idx);
        continue;
      }
      idx = pos < nodes_[idx].cut ? nodes_[idx].left : nodes_[idx].left + 1;
    }
  }

  size_t size() const { return a_.size(); }

  // The whole array sorted exactly as std::sort sorts it (same partitions, same leaves), the
  // right part of every partition above `grain` elements handed to an OpenMP task.  Call
  // from inside a parallel region's single construct, or serially.
  static void sort_words(uint64_t *f, int64_t n, int depth = -1, int64_t grain = 8192) {
    if (depth < 0) {
      int lg = 0;
      while (n >> (lg + 1)) lg++;
      depth = 2 * lg;
    }
    while (n > 16) {
      if (depth == 0) {
        auto cmp = [](uint64_t x, uint64_t y) { return less(x, y); };
        std::make_heap(f, f + n, cmp);
        std::sort_heap(f, f + n, cmp);
        return;
      }
      depth--;
      const int64_t cut = partition_pivot(f, n);
      uint64_t *r = f + cut;
      const int64_t rn = n - cut;
      const int d = depth;
      if (rn > grain) {
#pragma omp task firstprivate(r, rn, d, grain)
        sort_words(r, rn, d, grain);
      } else {
        sort_words(r, rn, d, grain);
      }
      n = cut;
    }
    insertion_sort(f, n);
  }

 private:
  struct Node {
    int64_t lo, hi;
    int depth;
    int left;     // index of the left child (right child = left + 1), -1 if not partitioned
    int64_t cut;  // partition point
    bool final;
  };
  static bool less(uint64_t x, uint64_t y) { return (x >> 32) < (y >> 32); }

  void expand(int idx) {
    const int64_t lo = nodes_[idx].lo, hi = nodes_[idx].hi;
    const int depth = nodes_[idx].depth;
    uint64_t *f = a_.data() + lo;
    const int64_t n = hi - lo;
    if (n <= 16) {  // leaf of __introsort_loop: __final_insertion_sort restricted to it
      insertion_sort(f, n);
      nodes_[idx].final = true;
      return;
    }
    if (depth == 0) {  // std::__partial_sort(first, last, last) = make_heap + sort_heap
      auto cmp = [](uint64_t x, uint64_t y) { return less(x, y); };
      std::make_heap(f, f + n, cmp);
      std::sort_heap(f, f + n, cmp);
      nodes_[idx].final = true;
      return;
    }
    const int64_t cut = lo + partition_pivot(f, n);
    const int child = (int)nodes_.size();
    nodes_.push_back(Node{lo, cut, depth - 1, -1, 0, false});
    nodes_.push_back(Node{cut, hi, depth - 1, -1, 0, false});
    nodes_[idx].left = child;
    nodes_[idx].cut = cut;
  }

  // std::__unguarded_partition_pivot: median of (first+1, mid, last-1) moved to first, then
  // std::__unguarded_partition(first+1, last, first).  Returns the cut offset.
  static int64_t partition_pivot(uint64_t *f, int64_t n) {
    uint64_t *a = f + 1, *b = f + n / 2, *c = f + n - 1;
    if (less(*a, *b)) {
      if (less(*b, *c)) std::iter_swap(f, b);
      else if (less(*a, *c)) std::iter_swap(f, c);
      else std::iter_swap(f, a);
    } else if (less(*a, *c)) {
      std::iter_swap(f, a);
    } else if (less(*b, *c)) {
      std::iter_swap(f, c);
    } else {
      std::iter_swap(f, b);
    }
#ifdef _OPENMP
    if (n >= par_min && omp_in_parallel()) return hoare_cut_par(f, n);
#endif
    return hoare_cut(f, n);
  }

  // std::__unguarded_partition(f+1, f+n, f) computed from two stopper bitmasks.  The left
  // scan stops at keys >= pivot, the right scan at keys <= pivot; the k-th swap exchanges the
  // k-th left stopper l_k with the k-th right stopper r_k of the ORIGINAL array as long as
  // l_k < r_k (neither scan ever reads a position an earlier swap wrote before the scans
  // cross), and the returned cut is min(l_{K+1}, r_K): a left scan that runs past r_K stops
  // there, because r_K now holds a key >= pivot.  Same swaps, same cut, without a
  // data-dependent branch per element.
  static int64_t hoare_cut(uint64_t *f, int64_t n) {
    static thread_local std::vector<uint64_t> ge, le;
    const uint64_t pk = f[0] >> 32;
    const int64_t nw = (n + 63) >> 6;
    ge.assign(nw, 0);
    le.assign(nw, 0);
    for (int64_t w = 0; w < nw; w++) {
      const int64_t base = w << 6, cnt = std::min<int64_t>(64, n - base);
      uint64_t g = 0, l = 0;
      for (int64_t b = 0; b < cnt; b++) {
        const uint64_t k = f[base + b] >> 32;
        g |= (uint64_t)(k >= pk) << b;
        l |= (uint64_t)(k <= pk) << b;
      }
      ge[w] = g;
      le[w] = l;
    }
    ge[0] &= ~1ull;  // the left scan starts at f+1; the right scan may stop at the pivot, f[0]
    auto next_ge = [&](int64_t from) -> int64_t {
      if (from >= n) return n;
      int64_t w = from >> 6;
      uint64_t bits = ge[w] & (~0ull << (from & 63));
      while (!bits) {
        if (++w >= nw) return n;
        bits = ge[w];
      }
      return (w << 6) + __builtin_ctzll(bits);
    };
    auto prev_le = [&](int64_t from) -> int64_t {
      if (from < 0) return -1;
      int64_t w = from >> 6;
      uint64_t bits = le[w] & (~0ull >> (63 - (from & 63)));
      while (!bits) {
        if (--w < 0) return -1;
        bits = le[w];
      }
      return (w << 6) + 63 - __builtin_clzll(bits);
    };
    int64_t li = next_ge(1), ri = prev_le(n - 1), last_r = n;
    while (li < ri) {
      std::iter_swap(f + li, f + ri);
      last_r = ri;
      li = next_ge(li + 1);
      ri = prev_le(ri - 1);
    }
    return std::min(li, last_r);
  }

#ifdef _OPENMP
 public:
  // ranges of at least par_min words are partitioned by the team (hoare_cut_par); the checks
  // lower it to exercise the parallel form on small arrays
  static inline int64_t par_min = 32768;

 private:
  // k-th (from 1) set bit of the words m[0, nw), given the prefix popcounts c (c[w] = bits in
  // m[0, w)): its position
  static int64_t select_bit(const std::vector<uint64_t> &m, const std::vector<int64_t> &c, int64_t k) {
    const int64_t w = (int64_t)(std::upper_bound(c.begin(), c.end(), k - 1) - c.begin()) - 1;
    uint64_t bits = m[w];
    for (int64_t r = k - c[w]; r > 1; r--) bits &= bits - 1;
    return (w << 6) + __builtin_ctzll(bits);
  }
  // hoare_cut's swaps and cut with the team: the stopper masks by tasks, the k-th stoppers by
  // prefix popcounts, K (the last k with l_k < r_k, monotone) by bisection, the K independent
  // swaps by tasks, each walking its own run of k from its first pair
  static int64_t hoare_cut_par(uint64_t *f, int64_t n) {
    const uint64_t pk = f[0] >> 32;
    const int64_t nw = (n + 63) >> 6;
    std::vector<uint64_t> ge(nw), le(nw);
    constexpr int64_t G = 512;  // words per task
#pragma omp taskloop grainsize(1) shared(ge, le)
    for (int64_t c = 0; c < (nw + G - 1) / G; c++) {
      for (int64_t w = c * G; w < std::min(nw, (c + 1) * G); w++) {
        const int64_t base = w << 6, cnt = std::min<int64_t>(64, n - base);
        uint64_t g = 0, l = 0;
        for (int64_t b = 0; b < cnt; b++) {
          const uint64_t k = f[base + b] >> 32;
          g |= (uint64_t)(k >= pk) << b;
          l |= (uint64_t)(k <= pk) << b;
        }
        ge[w] = g;
        le[w] = l;
      }
    }
    ge[0] &= ~1ull;  // the left scan starts at f+1; the right scan may stop at the pivot, f[0]
    std::vector<int64_t> cg(nw + 1), cl(nw + 1);
    cg[0] = cl[0] = 0;
    for (int64_t w = 0; w < nw; w++) {
      cg[w + 1] = cg[w] + __builtin_popcountll(ge[w]);
      cl[w + 1] = cl[w] + __builtin_popcountll(le[w]);
    }
    const int64_t CL = cg[nw], TL = cl[nw];
    auto lk = [&](int64_t k) { return select_bit(ge, cg, k); };           // k-th left stopper
    auto rk = [&](int64_t k) { return select_bit(le, cl, TL - k + 1); };  // k-th from the right
    int64_t lo = 0, hi = std::min(CL, TL) + 1;  // P(lo) true, P(hi) false
    while (hi - lo > 1) {
      const int64_t k = lo + (hi - lo) / 2;
      if (lk(k) < rk(k)) lo = k;
      else hi = k;
    }
    const int64_t K = lo;
    constexpr int64_t S = 4096;  // swaps per task
#pragma omp taskloop grainsize(1) shared(ge, le, cg, cl)
    for (int64_t t = 0; t < (K + S - 1) / S; t++) {
      const int64_t k0 = 1 + t * S, k1 = std::min(K, k0 + S - 1);
      int64_t li = lk(k0), ri = rk(k0);
      for (int64_t k = k0;; k++) {
        std::iter_swap(f + li, f + ri);
        if (k == k1) break;
        int64_t w = (li + 1) >> 6;  // next left stopper after li
        uint64_t bits = ge[w] & (~0ull << ((li + 1) & 63));
        while (!bits) bits = ge[++w];
        li = (w << 6) + __builtin_ctzll(bits);
        w = (ri - 1) >> 6;  // previous right stopper before ri
        bits = le[w] & (~0ull >> (63 - ((ri - 1) & 63)));
        while (!bits) bits = le[--w];
        ri = (w << 6) + 63 - __builtin_clzll(bits);
      }
    }
    const int64_t l_next = K < CL ? lk(K + 1) : n, r_last = K >= 1 ? rk(K) : n;
    return std::min(l_next, r_last);
  }
#endif

  // stable insertion sort (std::__insertion_sort / __unguarded_linear_insert move only
  // strictly smaller elements)
  static void insertion_sort(uint64_t *f, int64_t n) {
    for (int64_t i = 1; i < n; i++) {
      const uint64_t v = f[i];
      int64_t j = i;
      while (j > 0 && less(v, f[j - 1])) {
        f[j] = f[j - 1];
        j--;
      }
      f[j] = v;
    }
  }

  std::vector<uint64_t> a_;
  std::vector<Node> nodes_;
};

}  // namespace mc
