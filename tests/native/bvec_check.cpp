// Checks the closed-form bvec window logic of meshclust_amd/csrc/gpu/bvec_core.hpp (used by
// the device-resident accumulation kernel) against the host BVec restatement
// (meshclust_amd/csrc/host/bvec.cpp, itself byte-identical to the reference end to end):
// random length distributions, get_range + window for random query lengths, interleaved
// with pop / erase / remove_available until the bvec is empty.
#include <algorithm>
#include <cstdio>
#include <random>
#include <set>
#include <vector>

#include "../../meshclust_amd/csrc/gpu/bvec_core.hpp"
#include "../../meshclust_amd/csrc/host/bvec.hpp"
#include "../../meshclust_amd/csrc/host/common.hpp"

using mc::BVec;

struct NaiveAcc {
  const BVec &bv;
  uint64_t nbins() { return bv.bins().size(); }
  uint64_t cnt(uint64_t b) { return bv.bins().at(b).size(); }
  void index_of(uint64_t point, uint64_t *lo, uint64_t *hi) {
    const auto &bb = bv.begin_bounds();
    uint64_t low = bb.size() - 1, high = 0;
    for (uint64_t i = 0; i < bb.size(); i++) {
      uint64_t prev = i ? bb[i - 1] : 0, pi = i ? i - 1 : 0;
      if (point >= prev && point <= bb[i]) {
        low = std::min(low, pi);
        high = std::max(high, pi);
      }
    }
    if (point >= bb.back()) high = std::max<uint64_t>(high, bb.size() - 1);
    *lo = low;
    *hi = high;
  }
  int64_t first_nonempty() {
    for (uint64_t i = 0; i < nbins(); i++)
      if (cnt(i)) return (int64_t)i;
    return -1;
  }
  int64_t last_nonempty() {
    for (int64_t i = (int64_t)nbins() - 1; i >= 0; i--)
      if (cnt(i)) return i;
    return -1;
  }
  uint64_t count_lt(uint64_t b, uint64_t L) {
    uint64_t n = 0;
    for (uint32_t p : bv.bins()[b]) n += bv.static_lengths()[p] < L;
    return n;
  }
  uint64_t count_le(uint64_t b, uint64_t L) {
    uint64_t n = 0;
    for (uint32_t p : bv.bins()[b]) n += bv.static_lengths()[p] <= L;
    return n;
  }
  uint64_t prefix(uint64_t b) {
    uint64_t s = 0;
    for (uint64_t i = 0; i < b && i < nbins(); i++) s += cnt(i);
    return s;
  }
  uint64_t total() { return prefix(nbins()); }
  void locate_rank(uint64_t rank, uint64_t *b, uint64_t *c) {
    for (uint64_t i = 0; i < nbins(); i++) {
      if (rank < cnt(i)) {
        *b = i;
        *c = rank;
        return;
      }
      rank -= cnt(i);
    }
    *b = nbins();
    *c = 0;
  }
  uint64_t select(uint64_t b, uint64_t c) { return bv.bins()[b][c]; }
};


// The O(log) forms the device controller uses: index_of by two binary searches over the
// sorted begin bounds, a Fenwick tree over the per-bin alive counts, and per-bin rank counts
// from a binary search over the (length-sorted) static positions of the bin.
struct FastAcc {
  const BVec &bv;
  std::vector<uint64_t> lo;
  std::vector<uint8_t> alive;
  std::vector<uint64_t> fw;
  uint64_t lg = 1;
  FastAcc(const BVec &b, const std::vector<uint64_t> &lo_) : bv(b), lo(lo_) {
    const uint64_t nb = lo.size() - 1;
    alive.assign(lo[nb], 0);
    for (const auto &bin : bv.bins())
      for (uint32_t p : bin) alive[p] = 1;
    fw.assign(nb + 1, 0);
    for (uint64_t bi = 0; bi < nb; bi++)
      for (uint64_t i = bi + 1; i <= nb; i += i & (~i + 1)) fw[i] += bv.bins()[bi].size();
    while (lg * 2 <= nb) lg *= 2;
  }
  uint64_t nbins() { return lo.size() - 1; }
  uint64_t cnt(uint64_t b) { return b < nbins() ? bv.bins().at(b).size() : 0; }
  void index_of(uint64_t point, uint64_t *l, uint64_t *h) {
    mcg::bv_index_of_sorted(bv.begin_bounds(), nbins(), point, l, h);
  }
  uint64_t prefix(uint64_t b) { return mcg::bv_fw_prefix(fw, std::min(b, nbins())); }
  uint64_t total() { return prefix(nbins()); }
  void locate_rank(uint64_t rank, uint64_t *b, uint64_t *c) { mcg::bv_fw_locate(fw, nbins(), lg, rank, b, c); }
  int64_t first_nonempty() {
    if (!total()) return -1;
    uint64_t b, c;
    locate_rank(0, &b, &c);
    return (int64_t)b;
  }
  int64_t last_nonempty() {
    const uint64_t t = total();
    if (!t) return -1;
    uint64_t b, c;
    locate_rank(t - 1, &b, &c);
    return (int64_t)b;
  }
  uint64_t alive_in(uint64_t a, uint64_t z) {
    uint64_t n = 0;
    for (uint64_t p = a; p < z; p++) n += alive[p];
    return n;
  }
  uint64_t count_lt(uint64_t b, uint64_t L) {
    const auto &sl = bv.static_lengths();
    const uint64_t k = std::lower_bound(sl.begin() + lo[b], sl.begin() + lo[b + 1], L) - sl.begin();
    return alive_in(lo[b], k);
  }
  uint64_t count_le(uint64_t b, uint64_t L) {
    const auto &sl = bv.static_lengths();
    const uint64_t k = std::upper_bound(sl.begin() + lo[b], sl.begin() + lo[b + 1], L) - sl.begin();
    return alive_in(lo[b], k);
  }
  uint64_t select(uint64_t b, uint64_t c) {
    for (uint64_t p = lo[b]; p < lo[b + 1]; p++)
      if (alive[p] && c-- == 0) return p;
    return ~0ull;
  }
};

int main() {
  std::mt19937_64 rng(777);
  long checks = 0, fast_checks = 0, empty_edge_checks = 0;
  for (int t = 0; t < 300; t++) {
    const size_t n = t < 20 ? (size_t)t + 1 : (size_t)(rng() % 6000) + 1;
    std::vector<uint64_t> len(n);
    const int kind = t % 4;
    for (auto &l : len) {
      if (kind == 0) l = 970 + rng() % 61;                     // config B-like
      else if (kind == 1) l = 1 + rng() % 5000;                // wide
      else if (kind == 2) l = 100 * (1 + rng() % 8);           // few distinct values
      else l = (rng() % 3 == 0) ? 500 + rng() % 10 : 1000 + rng() % 2000;
    }
    const uint64_t bin_size = (t % 3 == 0) ? 1000 : 1 + rng() % 300;
    BVec bv(len, bin_size);
    for (uint32_t i = 0; i < n; i++) bv.insert(i);
    bv.insert_finalize();
    std::vector<uint64_t> blo(1, 0);
    for (const auto &bin : bv.bins()) blo.push_back(blo.back() + bin.size());
    const double sims[] = {0.9, 0.55, 0.8, 0.95, 0.99};
    for (int it = 0; it < 4000 && bv.size() > 0; it++) {
      // query
      for (int q = 0; q < 3; q++) {
        uint64_t L = (rng() % 4 == 0) ? 1 + rng() % 7000 : len[rng() % n];
        double sim = sims[rng() % 5];
        uint64_t bl = (uint64_t)(L * sim), el = (uint64_t)(L / sim);
        auto want = bv.get_range(bl, el);
        NaiveAcc a{bv};
        mcg::BPos f, b;
        mcg::bv_get_range(a, bl, el, f, b);
        if (f.first != want.first.first || f.second != want.first.second || b.first != want.second.first ||
            b.second != want.second.second) {
          printf("RANGE MISMATCH t=%d it=%d L=%llu sim=%g: want (%zu,%zu)-(%zu,%zu) got (%llu,%llu)-(%llu,%llu)\n", t, it,
                 (unsigned long long)L, sim, want.first.first, want.first.second, want.second.first, want.second.second,
                 (unsigned long long)f.first, (unsigned long long)f.second, (unsigned long long)b.first,
                 (unsigned long long)b.second);
          return 1;
        }
        uint64_t S1 = 0, E1 = 0, S2 = 0, E2 = 0;
        int herr = 0, derr = 0;
        int64_t c1 = 0;
        try {
          c1 = bv.window(want.first, want.second, &S1, &E1);
        } catch (const mc::Error &e) {
          herr = std::string(e.what()).find("null") != std::string::npos ? 2 : 1;
        }
        int64_t c2 = mcg::bv_window(a, f, b, &S2, &E2, &derr);
        if (herr != derr || (!herr && (c1 != c2 || (c1 > 0 && (S1 != S2 || E1 != E2))))) {
          printf("WINDOW MISMATCH t=%d it=%d: host err %d count %lld S %llu E %llu / core err %d count %lld S %llu E %llu\n",
                 t, it, herr, (long long)c1, (unsigned long long)S1, (unsigned long long)E1, derr, (long long)c2,
                 (unsigned long long)S2, (unsigned long long)E2);
          return 1;
        }
        FastAcc fa(bv, blo);
        mcg::BPos f2, b2;
        mcg::bv_get_range(fa, bl, el, f2, b2);
        uint64_t S3 = 0, E3 = 0;
        int ferr = 0;
        int64_t c3 = mcg::bv_window(fa, f2, b2, &S3, &E3, &ferr);
        if (f2.first != f.first || f2.second != f.second || b2.first != b.first || b2.second != b.second ||
            ferr != derr || c3 != c2 || (!ferr && c3 > 0 && (S3 != S2 || E3 != E2))) {
          printf("FAST MISMATCH t=%d it=%d\n", t, it);
          return 1;
        }
        // the device controller's nearest-alive form (edge bins non-empty, or empty: then front is
        // the first alive position overall and back the first alive position of the last
        // non-empty bin, as bvec::inner_index_of's empty-bin branch makes them)
        {
          uint64_t lo_, hi_;
          mcg::bv_index_of_sorted(bv.begin_bounds(), fa.nbins(), bl, &lo_, &hi_);
          const uint64_t fb = lo_;
          mcg::bv_index_of_sorted(bv.begin_bounds(), fa.nbins(), el, &lo_, &hi_);
          const uint64_t bb = hi_;
          const bool ef = fa.cnt(fb) > 0, eb = fa.cnt(bb) > 0;
          auto bin_first_alive = [&](bool last) -> uint64_t {  // first alive of the first / last non-empty bin
            const int64_t i = last ? fa.last_nonempty() : fa.first_nonempty();
            if (i < 0) return ~0ull;
            for (uint64_t p = blo[i]; p < blo[i + 1]; p++)
              if (fa.alive[p]) return p;
            return ~0ull;
          };
          const uint64_t ovf = ef ? 0 : bin_first_alive(false), ovb = eb ? 0 : bin_first_alive(true);
          if ((ef || ovf != ~0ull) && (eb || ovb != ~0ull)) {
            const auto &sl = bv.static_lengths();
            const uint64_t pf0 = std::lower_bound(sl.begin() + blo[fb], sl.begin() + blo[fb + 1], bl) - sl.begin();
            const uint64_t plt = std::lower_bound(sl.begin() + blo[bb], sl.begin() + blo[bb + 1], el) - sl.begin();
            const uint64_t ple = std::upper_bound(sl.begin() + blo[bb], sl.begin() + blo[bb + 1], el) - sl.begin();
            auto next_alive = [&](uint64_t a, uint64_t z) -> uint64_t {
              for (uint64_t p = a; p < z; p++)
                if (fa.alive[p]) return p;
              return ~0ull;
            };
            auto prev_alive = [&](uint64_t a, uint64_t z) -> uint64_t {
              for (uint64_t p = z; p > a; p--)
                if (fa.alive[p - 1]) return p - 1;
              return ~0ull;
            };
            uint64_t S4 = 0, E4 = 0;
            mcg::bv_fast_window(ef ? next_alive(pf0, blo[fb + 1]) : ovf, ef ? prev_alive(blo[fb], pf0) : ~0ull,
                                eb ? next_alive(ple, blo[bb + 1]) : ovb, eb ? prev_alive(blo[bb], ple) : ~0ull, plt, &S4,
                                &E4);
            const bool has = E4 != ~0ull && S4 != ~0ull && E4 >= S4;
            if (derr || has != (c2 > 0) || (has && (S4 != S2 || E4 != E2))) {
              printf("NEAREST-ALIVE MISMATCH t=%d it=%d: core err %d count %lld S %llu E %llu / fast S %llu E %llu\n", t,
                     it, derr, (long long)c2, (unsigned long long)S2, (unsigned long long)E2, (unsigned long long)S4,
                     (unsigned long long)E4);
              return 1;
            }
            fast_checks++;
            if (!ef || !eb) empty_edge_checks++;
          }
        }
        checks++;
      }
      // mutate
      int op = (int)(rng() % 3);
      if (op == 0) {
        bv.pop();
      } else {
        std::vector<uint32_t> alive;
        for (const auto &bin : bv.bins()) alive.insert(alive.end(), bin.begin(), bin.end());
        if (alive.empty()) break;
        if (op == 1) {
          uint32_t p = alive[rng() % alive.size()];
          auto rc = bv.locate(p);
          bv.erase(rc.first, rc.second);
        } else {
          std::set<uint32_t> pick;
          size_t k = 1 + rng() % std::min<size_t>(alive.size(), 40);
          while (pick.size() < k) pick.insert(alive[rng() % alive.size()]);
          std::vector<uint32_t> ps(pick.begin(), pick.end()), avail;
          bv.remove_positions(ps, 0, bv.bins().size() - 1, avail);
        }
      }
    }
    // the empty bvec as well
    NaiveAcc a{bv};
    if (bv.size() == 0) {
      auto want = bv.get_range(900, 1100);
      mcg::BPos f, b;
      mcg::bv_get_range(a, 900, 1100, f, b);
      if (f.first != want.first.first || f.second != want.first.second || b.first != want.second.first ||
          b.second != want.second.second) {
        printf("EMPTY RANGE MISMATCH t=%d\n", t);
        return 1;
      }
    }
  }
  printf("OK %ld checks (%ld nearest-alive, %ld with an empty edge bin)\n", checks, fast_checks, empty_edge_checks);
  return 0;
}
