// trainer.cpp -- see trainer.hpp.  Compiled with -ffp-contract=off.
#include "trainer.hpp"

#include "lazysort.hpp"  // (the two full sorts; the per-pivot sorts are on the device)

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <memory>
#include <set>
#include <thread>

namespace mc {

namespace {

struct ExitZero : Error {
  ExitZero(const std::string &m) : Error(m, 0) {}
};

// get_bin of resize_vec / bin_data (Trainer.cpp:217-225, 493-501)
inline int get_bin(double x, double min_align, double max_align, int num_bins) {
  if (x >= max_align) return num_bins - 1;
  if (x <= min_align) return 0;
  return (int)(num_bins * (x - min_align) / (max_align - min_align));
}

using Labeled = std::pair<PairId, double>;

// resize_vec (Trainer.cpp:201-243): bins by identity, then repeatedly takes the first
// ceil(left/bins) items of every bin from the top bin down -- it can over-fill.
std::vector<Labeled> resize_vec(const std::vector<Labeled> &vec, size_t new_size, double min_align,
                                double max_align, int num_bins) {
  if (new_size == vec.size()) return vec;
  std::vector<std::vector<Labeled>> bins(num_bins);
  for (const auto &p : vec) bins.at(get_bin(p.second, min_align, max_align, num_bins)).push_back(p);
  std::vector<Labeled> data;
  while (data.size() < new_size) {
    int items_left = (int)(new_size - data.size());
    int take = (int)std::ceil((double)items_left / num_bins);
    for (int i = (int)bins.size() - 1; i >= 0; i--)
      for (int j = 0; j < (int)std::min((size_t)take, bins[i].size()); j++) data.push_back(bins[i][j]);
  }
  return data;
}

// bin_data (Trainer.cpp:490-526): 10 identity bins, alternate rows go to train / test,
// the parity flipping from bin to bin.
std::pair<std::vector<PairId>, std::vector<PairId>> bin_data(const std::vector<Labeled> &vec, double min_align,
                                                             double max_align) {
  const int n_bins = 10;
  std::vector<std::vector<Labeled>> bins(n_bins);
  for (const auto &d : vec) bins.at(get_bin(d.second, min_align, max_align, n_bins)).push_back(d);
  std::vector<PairId> train, test;
  int last = 0;
  for (const auto &bin : bins) {
    for (int i = 0; i < (int)bin.size(); i++) {
      if (i % 2 == last) train.push_back(bin[i].first);
      else test.push_back(bin[i].first);
    }
    last = !last;
  }
  return {train, test};
}

}  // namespace

bool Trainer::hdr_less(uint32_t a, uint32_t b) const { return ds_.headers[a].compare(ds_.headers[b]) < 0; }

bool Trainer::gather(const std::vector<uint64_t> &mine, std::vector<uint64_t> &all) const {
  const ShardComm *cm = cfg_.comm;
  if (!cm || cm->world <= 1) return false;
  all.assign(mine.size() * (size_t)cm->world, 0);
  if (cm->allgather(cm->user, mine.data(), mine.size() * 8, all.data()) != 0)
    throw PeerError("training all-gather across ranks failed");
  return true;
}

void Trainer::nw_batch(const std::vector<PairId> &pairs, std::vector<double> &ident) {
  std::vector<uint32_t> a(pairs.size()), b(pairs.size());
  for (size_t i = 0; i < pairs.size(); i++) {
    a[i] = pairs[i].first;
    b[i] = pairs[i].second;
  }
  ident.assign(pairs.size(), 0.0);
  if (pairs.empty()) return;
  for (const auto &p : pairs) {
    nw_pairs++;
    nw_cells += ds_.lengths[p.first] * ds_.lengths[p.second];
  }
  check(mc_nw_identity(ctx_, a.data(), b.data(), pairs.size(), ident.data(), nullptr, nullptr), "mc_nw_identity");
}

// Header order of pair ids (the reference's std::set<pair<Point*, Point*>> comparators order
// by Point::get_header, Trainer.cpp:653-667 / 264-269): each id's first 16 header bytes as two
// big-endian words, so most comparisons are integer ones; equal prefixes of headers longer than
// 16 bytes fall back to the full compare.  (string_view::compare is a memcmp: unsigned bytes,
// a prefix first -- which the zero-padded words and then the lengths reproduce.)
namespace {
struct HdrKey {
  uint64_t k0, k1;
  uint32_t len, id;
};
HdrKey hdr_key(const Dataset &ds, uint32_t id) {
  const std::string_view h = ds.headers[id];
  unsigned char b[16] = {0};
  memcpy(b, h.data(), h.size() < 16 ? h.size() : 16);
  uint64_t w0 = 0, w1 = 0;
  for (int i = 0; i < 8; i++) {
    w0 = (w0 << 8) | b[i];
    w1 = (w1 << 8) | b[8 + i];
  }
  return HdrKey{w0, w1, (uint32_t)std::min<size_t>(h.size(), 0xffffffffu), id};
}
int hdr_cmp(const Dataset &ds, const HdrKey &x, const HdrKey &y) {
  if (x.k0 != y.k0) return x.k0 < y.k0 ? -1 : 1;
  if (x.k1 != y.k1) return x.k1 < y.k1 ? -1 : 1;
  if (x.len <= 16 && y.len <= 16) return x.len < y.len ? -1 : x.len > y.len ? 1 : 0;
  const int c = ds.headers[x.id].compare(ds.headers[y.id]);
  return c < 0 ? -1 : c > 0 ? 1 : 0;
}
// std::set<pair, header order>'s contents and order from inserting v[0], v[1], ... (what
// insert keeps: the first of each run of equivalent elements): the indices of v in that order.
// Each element carries its two ids' keys, so the sort reads no header for most comparisons.
template <typename GetPair>
std::vector<uint32_t> header_set_order(const Dataset &ds, size_t n, GetPair pair_of) {
  struct E {
    HdrKey a, b;
    uint32_t idx;
  };
  std::vector<E> e(n);
  for (size_t i = 0; i < n; i++) {
    const PairId p = pair_of(i);
    e[i] = E{hdr_key(ds, p.first), hdr_key(ds, p.second), (uint32_t)i};
  }
  auto cmp = [&](const E &x, const E &y) {
    const int c = hdr_cmp(ds, x.a, y.a);
    return c != 0 ? c : hdr_cmp(ds, x.b, y.b);
  };
  std::stable_sort(e.begin(), e.end(), [&](const E &x, const E &y) { return cmp(x, y) < 0; });
  std::vector<uint32_t> out;
  out.reserve(n);
  for (size_t i = 0; i < n; i++)
    if (i == 0 || cmp(e[i - 1], e[i]) != 0) out.push_back(e[i].idx);
  return out;
}
}  // namespace

std::vector<uint32_t> Trainer::length_order(const Dataset &ds, int threads) {
  const size_t N = ds.size();
  std::vector<uint32_t> points(N);
  for (size_t i = 0; i < N; i++) points[i] = (uint32_t)i;
  bool wide = false;
  for (size_t t = 0; t < N; t++) wide |= ds.lengths[t] >> 32 != 0;
  if (wide) {
    std::sort(points.begin(), points.end(),
              [&](uint32_t a, uint32_t b) { return ds.lengths[a] < ds.lengths[b]; });  // Trainer.cpp:672-675
  } else {
    // std::sort with a key-only comparator on (key << 32 | id) words: LazyIntroSort::sort_words
    // performs the same partitions and leaves (so the same permutation, ties included)
    std::vector<uint64_t> w(N);
    for (size_t t = 0; t < N; t++) w[t] = ((uint64_t)ds.lengths[t] << 32) | t;
#pragma omp parallel num_threads(threads)
#pragma omp single
    LazyIntroSort::sort_words(w.data(), (int64_t)w.size());
    for (size_t t = 0; t < N; t++) points[t] = (uint32_t)w[t];
  }
  return points;
}

// Trainer::split (Trainer.cpp:653-783)
std::vector<PairId> Trainer::split() {
  const size_t N = ds_.size();
  std::vector<PairId> pairs;  // the reference's header-ordered std::set (set_order below)
  std::vector<uint32_t> points(N);
  for (size_t i = 0; i < N; i++) points[i] = (uint32_t)i;
  std::vector<uint32_t> all_ids = points;  // distance keys are requested in id order
  {
    Scope s(timer_, "train.sort_keys");
    Scope s2(timer_, "train.sort_keys.first");
    // Both sorts are std::sort with a key-only comparator on (key << 32 | id) words:
    // LazyIntroSort::sort_words performs the same partitions and leaves (so the same
    // permutation, ties included), with the subranges sorted as parallel tasks.
    auto exact_sort = [&](std::vector<uint64_t> &w) {
#pragma omp parallel num_threads(cfg_.threads)
#pragma omp single
      LazyIntroSort::sort_words(w.data(), (int64_t)w.size());
    };
    std::vector<uint64_t> w(N);
    if (cfg_.length_order.size() == N) points = cfg_.length_order;
    else points = length_order(ds_, cfg_.threads);
    uint32_t begin_pt = points[N / 2];
    std::vector<uint16_t> key0(N);
    check(mc_distance_keys(ctx_, &begin_pt, 1, all_ids.data(), N, key0.data()), "mc_distance_keys");
    for (size_t t = 0; t < N; t++) w[t] = ((uint64_t)key0[points[t]] << 32) | points[t];
    exact_sort(w);  // Trainer.cpp:679-684
    for (size_t t = 0; t < N; t++) points[t] = (uint32_t)w[t];
  }
  int num_iterations = (int)std::ceil(((double)cfg_.n_points) / cfg_.max_pts_from_one) - 1;
  if (num_iterations <= 0) throw Error("sample size must exceed points per pivot (integer division by zero in Trainer::split)", 1);
  std::vector<uint32_t> indices;
  for (int i = 0; i <= num_iterations; i++) indices.push_back(points[(size_t)i * (N - 1) / (size_t)num_iterations]);
  if (cfg_.verbose) printf("Point pairs: %zu\n", indices.size());
  const size_t to_add_each = cfg_.max_pts_from_one / 2;
  const size_t P = indices.size();
  // Each pivot's std::sort runs on (key << 32 | id) words with a comparator that looks only at
  // the key: the comparison outcomes -- and so the permutation -- are those of sorting ids by
  // keys[id].  Each pivot's std::sort(points, by distance to pivot i) (Trainer.cpp:691-701) is evaluated
  // on the device (mc_split_*, split.hip): the (key << 32 | id) arrays stay in HBM and only
  // the positions the binary search and the sampler read are resolved, with std::sort's exact
  // tie order.
  // reads longer than 4 kb on average (config E's genomes): every alignment is ~10^8 cells
  const bool long_reads = [&] {
    uint64_t tot = 0;
    for (size_t t = 0; t < N; t++) tot += ds_.lengths[t];
    return N > 0 && tot / N > 4096;
  }();
  // Rounds after the first align the next `look` levels of every chain's decision tree (2^look - 1
  // pairs per chain); two levels per round measured fastest at config B without the spine round
  // (9 rounds of 450 pairs in the latency form instead of 16 of 150).  With long reads a round
  // is bound by its cells, not by its fixed costs, and the branch not taken is a third of them:
  // one level per round (E9100's search 210 ms against 239, with nw.hip's 8-row chained blocks).
  // MC_NW_LOOKAHEAD = 1..4 forces it.
  const int look = [&] {
    const char *e = getenv("MC_NW_LOOKAHEAD");
    const int v = e ? atoi(e) : long_reads ? 1 : 2;
    return v < 1 ? 1 : v > 4 ? 4 : v;
  }();
  // The first round aligns each chain's whole "left spine" -- the pivots the search visits while
  // every identity stays below the cutoff (N/2, N/4, N/8, ...) -- in one batch (MC_NW_SPINE=0/1
  // forces it off / on; by default on for mean read lengths up to 4 kb, below).
  // The array is sorted by k-mer distance to the pivot, so the search walks left until it nears
  // the few points within the cutoff of the pivot (its own cluster): at config B the first ~9 of
  // ~15 levels, in one round of ~2,400 pairs (the throughput form) instead of ~5 dependent rounds.
  // A chain whose identities turn above the cutoff earlier just leaves the rest of its spine
  // unused; every decision is still taken from its own alignment, so the pivots are the same.
  // The spine pays where a round's fixed costs (a select call, the host walk, a latency-form
  // batch that fills the chip 1.8 deep) outweigh the alignments it may waste: short reads.  At
  // 8-12 kb (config E) every wasted pair is 10^8 cells, and E9100's search measured 257 ms with
  // the spine against 239 ms without, so it is off above a mean length of 4 kb.
  const bool spine = [&] {
    const char *e = getenv("MC_NW_SPINE");
    if (e) return atoi(e) != 0;
    return N > 0 && !long_reads;
  }();
  // one round's nodes of chain state (p, o): node n aligns position pos[n]; its children (identity
  // below the cutoff: p - o; above: p + o, both with offset o / 2) are kid[n][0] / kid[n][1], -1
  // when not aligned this round (the walk stops there and the next round starts from it); a node
  // whose offset is 0 is not aligned (the chain stops there, as `gather` drops it)
  struct Plan {
    std::vector<size_t> pos;
    std::vector<std::array<int, 2>> kid;
  };
  auto tree = [&](size_t p, size_t o, int d, Plan &pl) {  // the complete tree of depth d
    pl.pos.clear();
    pl.kid.clear();
    if (o == 0) return;
    std::vector<size_t> off;
    pl.pos.push_back(p);
    pl.kid.push_back({-1, -1});
    off.push_back(o);
    std::vector<int> level = {0};
    for (int l = 1; l < d; l++) {
      std::vector<int> next;
      for (int n : level) {
        const size_t oc = off[(size_t)n] / 2;
        if (oc == 0) continue;
        for (int side = 0; side < 2; side++) {
          pl.kid[(size_t)n][(size_t)side] = (int)pl.pos.size();
          next.push_back((int)pl.pos.size());
          pl.pos.push_back(side ? pl.pos[(size_t)n] + off[(size_t)n] : pl.pos[(size_t)n] - off[(size_t)n]);
          pl.kid.push_back({-1, -1});
          off.push_back(oc);
        }
      }
      level.swap(next);
    }
  };
  // Several ranks: rank r runs the chains (binary searches and samples) of its block of pivots
  // [i0, i1) -- each chain needs only its own pivot's sorted array -- and the sampled pairs are
  // all-gathered at the end (one exchange; the pairs go into a header-ordered set, so the
  // union is the same whatever rank found them).
  const int W = cfg_.comm && cfg_.comm->world > 1 ? cfg_.comm->world : 1;
  const size_t per = (P + (size_t)W - 1) / (size_t)W;
  const size_t i0 = std::min(P, per * (size_t)(W > 1 ? cfg_.comm->rank : 0)), i1 = std::min(P, i0 + per);
  // The spine round aligns the first L levels of every chain, L = 2,048 / chains: the NW
  // throughput form holds 2,048 waves at once on MI355X (256 CUs x 4 SIMDs x 2 waves of 256
  // registers), and a batch one wave larger runs a second, mostly empty generation.  Config B's
  // 150 chains: 13 of ~15 levels, 1,950 pairs; the search 4.9-5.9 -> 4.2 ms
  // (profiles/r06/ab/spine_levels.txt).  The deeper levels go to the next rounds (identical
  // pivots either way).  MC_NW_SPINE_LEVELS = L forces L.
  const int spine_levels = [&] {
    const char *e = getenv("MC_NW_SPINE_LEVELS");
    const int v = e ? atoi(e) : 0;
    if (v > 0) return v;
    const size_t chains = i1 > i0 ? i1 - i0 : 1;
    return (int)std::max<size_t>(1, 2048 / chains);
  }();
  auto left_spine = [&](size_t p, size_t o, Plan &pl) {  // every level, identity below the cutoff
    pl.pos.clear();
    pl.kid.clear();
    for (int lv = 0; o > 0 && lv < spine_levels; o /= 2, lv++) {
      if (!pl.pos.empty()) pl.kid.back()[0] = (int)pl.pos.size();
      pl.pos.push_back(p);
      pl.kid.push_back({-1, -1});
      p -= o;
    }
  };
  const uint64_t nw_pairs0 = nw_pairs, nw_cells0 = nw_cells;
  {
    Scope s(timer_, "train.sort_keys");
    Scope s3(timer_, "train.sort_keys.pivots");
    if (i1 > i0) check(mc_split_begin(ctx_, indices.data() + i0, (uint32_t)(i1 - i0), points.data(), N), "mc_split_begin");
  }
  // ids at sorted positions of the pivots' arrays
  std::vector<uint32_t> q_arr, q_ids;
  std::vector<uint64_t> q_pos;
  auto select = [&]() {
    q_ids.resize(q_arr.size());
    if (!q_arr.empty()) {  // (arrays are numbered from this rank's first pivot)
      std::vector<uint32_t> la(q_arr.size());
      for (size_t q = 0; q < q_arr.size(); q++) la[q] = q_arr[q] - (uint32_t)i0;
      check(mc_split_select(ctx_, q_arr.size(), la.data(), q_pos.data(), q_ids.data()), "mc_split_select");
    }
  };
  // binary search with alignment (:703-721): the 150 dependent chains advance together.  Each
  // round aligns, for every active chain, the next `look` levels of its decision tree at once
  // (the current pivot, both positions the next comparison can move to, ...: 2^look - 1 pairs
  // per chain), then walks the tree with the identities: the same decisions as one level per
  // round -- the same pivots -- in ceil(levels / look) dependent rounds instead of one per
  // level.  The alignments of the branches not taken are extra work (counted in nw_cells).
  std::vector<size_t> offset(P, N / 4), pivot(P, 2 * (N / 4));
  std::vector<char> active(P, 1);
  // Sampler positions of the current pivot estimate (the loops of :732-755 below).
  auto sample_positions = [&](size_t pv, std::vector<size_t> &out) {
    const size_t npts = N;
    double before_inc = (double)pv / to_add_each, after_inc = ((double)(npts - pv)) / to_add_each;
    double bs = 0, as = (double)pv;
    for (int t = 0; t < (int)to_add_each; t++, bs += before_inc) out.push_back((size_t)(int)std::round(bs));
    for (int t = 0; t < (int)to_add_each && std::round(as) < (double)npts; t++, as += after_inc)
      out.push_back((size_t)(int)std::round(as));
  };
  {
    Scope s(timer_, "train.nw_search");
    std::vector<PairId> batch;
    std::vector<size_t> who, first;  // chain of each batch entry's tree; first entry of each chain
    std::vector<Plan> plan(P);
    for (int round = 0;; round++) {
      who.clear();
      for (size_t i = i0; i < i1; i++) {
        if (active[i] && offset[i] == 0) active[i] = 0;
        if (active[i]) who.push_back(i);
      }
      {
        Scope s2(timer_, "train.nw_search.resolve");
        first.assign(who.size() + 1, 0);
        q_arr.clear();
        q_pos.clear();
        for (size_t t = 0; t < who.size(); t++) {
          const size_t i = who[t];
          if (round == 0 && spine) left_spine(pivot[i], offset[i], plan[i]);
          else tree(pivot[i], offset[i], look, plan[i]);
          for (size_t n = 0; n < plan[i].pos.size(); n++) {
            q_arr.push_back((uint32_t)i);
            q_pos.push_back(plan[i].pos[n]);
          }
          first[t + 1] = q_arr.size();
        }
        select();
        batch.resize(q_arr.size());
        for (size_t q = 0; q < q_arr.size(); q++) batch[q] = PairId(indices[q_arr[q]], q_ids[q]);
      }
      if (batch.empty()) break;
      std::vector<double> al;
      {
        Scope s3(timer_, "train.nw_search.align");
        nw_batch(batch, al);
      }
      for (size_t t = 0; t < who.size(); t++) {
        const size_t i = who[t];
        const double *val = al.data() + first[t];  // this chain's nodes, in plan order
        for (int n = 0; n >= 0 && active[i];) {
          const double algn = val[n];
          if (algn < cfg_.cutoff) {
            pivot[i] -= offset[i];
            n = plan[i].kid[(size_t)n][0];
          } else if (algn > cfg_.cutoff) {
            pivot[i] += offset[i];
            n = plan[i].kid[(size_t)n][1];
          } else {
            active[i] = 0;
            break;
          }
          offset[i] /= 2;
          if (offset[i] == 0) break;  // (the next round's gather drops the chain)
        }
      }
    }
  }
  int aerr = 0;
  std::vector<std::vector<PairId>> bufs(P);
  {
    Scope sb(timer_, "train.sample");
    q_arr.clear();
    q_pos.clear();
    std::vector<size_t> sp;
    for (size_t i = i0; i < i1; i++) {
      sp.clear();
      sample_positions(pivot[i], sp);
      for (size_t x : sp) {
        q_arr.push_back((uint32_t)i);
        q_pos.push_back(x);
      }
    }
    select();
    for (size_t q = 0; q < q_arr.size(); q++) {
      const uint32_t p = indices[q_arr[q]], x = q_ids[q];
      bufs[q_arr[q]].push_back(hdr_less(p, x) ? PairId(p, x) : PairId(x, p));
    }
    if (i1 > i0) check(mc_split_end(ctx_), "mc_split_end");
    // the ranks' pivots and samples: [nw pairs, nw cells, pairs, pivot[i0..i1), pairs (a << 32 | b)]
    const size_t cap = per * (2 * to_add_each);
    std::vector<uint64_t> mine(3 + per + cap, 0), all;
    mine[0] = nw_pairs - nw_pairs0;
    mine[1] = nw_cells - nw_cells0;
    size_t np = 0;
    for (size_t i = i0; i < i1; i++) {
      mine[3 + (i - i0)] = pivot[i];
      for (const PairId &pr : bufs[i]) mine[3 + per + np++] = ((uint64_t)pr.first << 32) | pr.second;
    }
    mine[2] = np;
    if (gather(mine, all)) {
      nw_pairs = nw_pairs0;
      nw_cells = nw_cells0;
      for (int r = 0; r < W; r++) {
        const uint64_t *b = all.data() + (size_t)r * mine.size();
        const size_t r0 = std::min(P, per * (size_t)r), r1 = std::min(P, r0 + per);
        nw_pairs += b[0];
        nw_cells += b[1];
        for (size_t i = r0; i < r1; i++) {
          pivot[i] = b[3 + (i - r0)];
          if (r != cfg_.comm->rank) bufs[i].clear();
        }
        if (r == cfg_.comm->rank) continue;
        // (another rank's pairs go to the first pivot of its block: only the union matters)
        for (uint64_t q = 0; q < b[2] && r1 > r0; q++)
          bufs[r0].push_back(PairId((uint32_t)(b[3 + per + q] >> 32), (uint32_t)b[3 + per + q]));
      }
    }
  }
  Scope sp(timer_, "train.sample.pair_set");
  for (size_t i = 0; i < P; i++) {  // the warning flag keeps the serial loop's last writer
    double before_inc = (double)pivot[i] / to_add_each;
    double after_inc = ((double)(N - pivot[i])) / to_add_each;
    if (before_inc < 1) aerr = 1;
    else if (after_inc < 1) aerr = -1;
    pairs.insert(pairs.end(), bufs[i].begin(), bufs[i].end());
  }
  {
    const std::vector<uint32_t> ord = header_set_order(ds_, pairs.size(), [&](size_t i) { return pairs[i]; });
    std::vector<PairId> set(ord.size());
    for (size_t i = 0; i < ord.size(); i++) set[i] = pairs[ord[i]];
    pairs.swap(set);
  }
  if (aerr < 0) fprintf(stderr, "Warning: Alignment may be too small for sampling\n");
  else if (aerr > 0) fprintf(stderr, "Warning: Alignment may be too large for sampling\n");
  return pairs;
}

// Trainer::get_labels (Trainer.cpp:253-333).  random_shuffle only permutes the alignment
// order; results land in header-ordered sets, so it has no effect and is skipped.
void Trainer::get_labels(const std::vector<PairId> &vec, std::vector<Labeled> &bp, std::vector<Labeled> &bn) {
  std::vector<double> al;
  {
    Scope s(timer_, "train.nw_labels");
    const int W = cfg_.comm && cfg_.comm->world > 1 ? cfg_.comm->world : 1;
    if (W == 1) {
      nw_batch(vec, al);
    } else {
      // rank r aligns pairs [r * per, (r + 1) * per); the identities are all-gathered
      const size_t m = vec.size(), per = (m + (size_t)W - 1) / (size_t)W;
      const size_t j0 = std::min(m, per * (size_t)cfg_.comm->rank), j1 = std::min(m, j0 + per);
      const uint64_t p0 = nw_pairs, c0 = nw_cells;
      std::vector<double> part;
      nw_batch(std::vector<PairId>(vec.begin() + j0, vec.begin() + j1), part);
      std::vector<uint64_t> mine(2 + per, 0), all;
      mine[0] = nw_pairs - p0;
      mine[1] = nw_cells - c0;
      for (size_t j = j0; j < j1; j++) memcpy(&mine[2 + (j - j0)], &part[j - j0], 8);
      gather(mine, all);
      nw_pairs = p0;
      nw_cells = c0;
      al.assign(m, 0.0);
      for (int r = 0; r < W; r++) {
        const uint64_t *b = all.data() + (size_t)r * mine.size();
        const size_t r0 = std::min(m, per * (size_t)r), r1 = std::min(m, r0 + per);
        nw_pairs += b[0];
        nw_cells += b[1];
        for (size_t j = r0; j < r1; j++) memcpy(&al[j], &b[2 + (j - r0)], 8);
      }
    }
  }
  Scope sl(timer_, "train.label_sets");
  // the reference's header-ordered std::set<pair<pair<Point*, Point*>, double>> per side
  std::vector<Labeled> buf_pos, buf_neg;
  for (size_t i = 0; i < vec.size(); i++) {
    if (al[i] >= cfg_.cutoff) buf_pos.push_back({vec[i], al[i]});
    else buf_neg.push_back({vec[i], al[i]});
  }
  for (std::vector<Labeled> *v : {&buf_pos, &buf_neg}) {
    const std::vector<uint32_t> ord = header_set_order(ds_, v->size(), [&](size_t i) { return (*v)[i].first; });
    std::vector<Labeled> set(ord.size());
    for (size_t i = 0; i < ord.size(); i++) set[i] = (*v)[ord[i]];
    v->swap(set);
  }
  if (cfg_.verbose) printf("positive=%zu negative=%zu\n", buf_pos.size(), buf_neg.size());
  if (buf_pos.empty() || buf_neg.empty()) {
    std::string m = "Identity value does not match sampled data: ";
    m += buf_pos.empty() ? "Too many sequences below identity" : "Too many sequences above identity";
    printf("%s\n", m.c_str());
    throw ExitZero(m);
  }
  size_t m_size = std::min(buf_pos.size(), buf_neg.size());
  std::vector<Labeled> &vpos = buf_pos, &vneg = buf_neg;
  bp = resize_vec(vpos, m_size, cfg_.cutoff, 1, 5);
  bn = resize_vec(vneg, m_size, 0.4, cfg_.cutoff, 5);
  if (cfg_.verbose) printf("positive=%zu negative=%zu\n", bp.size(), bn.size());
}

// generate_feat_mat (Trainer.cpp:367-414): column 0 is the constant 1, then the combos of
// feat->compute(first, second); labels +1 for the positive block, -1 for the negative.
Matrix Trainer::feat_matrix(const std::vector<PairId> &pos, const std::vector<PairId> &neg, int ncols,
                            Matrix &labels) {
  const size_t n = pos.size() + neg.size();
  Matrix fm((int)n, ncols);
  labels = Matrix((int)n, 1);
  std::vector<uint32_t> a(n), b(n);
  for (size_t i = 0; i < n; i++) {
    const PairId &p = i < pos.size() ? pos[i] : neg[i - pos.size()];
    a[i] = p.first;
    b[i] = p.second;
  }
  const size_t ns = feat.lookup.size();
  std::vector<double> raw(n * ns);
  if (n) check(mc_pair_features(ctx_, a.data(), b.data(), n, feat.lookup.data(), (int)ns, raw.data()), "mc_pair_features");
  for (size_t i = 0; i < n; i++) {
    double *cache = &raw[i * ns];
    feat.normalize_cache(cache);
    fm.set((int)i, 0, 1);
    for (int col = 1; col < ncols; col++) fm.set((int)i, col, feat.combo(col - 1, cache));
    labels.set((int)i, 0, i < pos.size() ? 1 : -1);
  }
  return fm;
}

void Trainer::train(double acc_cutoff) {
  std::pair<std::vector<PairId>, std::vector<PairId>> training, testing;
  if (cfg_.k != 0) {
    if (cfg_.verbose) printf("Splitting data\n");
    split_pairs = split();
    get_labels(split_pairs, label_pos, label_neg);
    auto pos = bin_data(label_pos, cfg_.cutoff, 1);
    training.first = pos.first;
    testing.first = pos.second;
    auto neg = bin_data(label_neg, 0, cfg_.cutoff);
    training.second = neg.first;
    testing.second = neg.second;
    if (cfg_.verbose)
      printf("training positive: %zu\ntraining negative: %zu\ntesting positive: %zu\ntesting negative: %zu\n",
             training.first.size(), training.second.size(), testing.first.size(), testing.second.size());
    if (testing.first.empty() || testing.second.empty()) throw Error("not enough points to sample", 1);
  }
  if (cfg_.k == 0) {  // alignment mode (Trainer.cpp:570-577)
    feat.add_feature(MC_FEAT_ALIGN, MC_COMBO_SELF);
    feat.normalize_with({}, 0);
    feat.finalize();
    weights = {-1 * cfg_.cutoff, 1};
    return;
  }
  Scope s(timer_, "train.glm");
  const std::vector<std::pair<uint16_t, int>> bit_feats = {
      {MC_FEAT_INTERSECTION | MC_FEAT_LD, MC_COMBO_SELF},
      {MC_FEAT_MANHATTAN | MC_FEAT_LD, MC_COMBO_SQUARED},
      {MC_FEAT_PEARSON, MC_COMBO_SELF},
      {MC_FEAT_KULCZYNSKI2 | MC_FEAT_LD, MC_COMBO_SQUARED}};
  double prev_acc = -10000;
  std::vector<std::vector<double>> matvec;
  std::vector<FeatureSet> features;
  GLM glm;
  const size_t min_no_features = std::max(1, (int)bit_feats.size() - 1);
  for (size_t num_features = min_no_features; num_features <= bit_feats.size(); num_features++) {
    for (size_t j = feat.size(); j < num_features && j < bit_feats.size(); j++)
      feat.add_feature(bit_feats[j].first, bit_feats[j].second);
    // feat->normalize(training.first); feat->normalize(training.second); (min/max carry over)
    {
      auto need = feat.flags_needed();
      std::vector<uint32_t> a, b;
      for (auto *v : {&training.first, &training.second})
        for (const auto &p : *v) {
          a.push_back(p.first);
          b.push_back(p.second);
        }
      std::vector<double> raw(a.size() * need.size());
      if (!need.empty() && !a.empty())
        check(mc_pair_features(ctx_, a.data(), b.data(), a.size(), need.data(), (int)need.size(), raw.data()),
              "mc_pair_features");
      feat.normalize_with(raw, a.size());
    }
    feat.finalize();
    if (cfg_.verbose) feat.print_bounds();
    Matrix ltrain, ltest;
    Matrix mtrain = feat_matrix(training.first, training.second, (int)num_features + 1, ltrain);
    Matrix mtest = feat_matrix(testing.first, testing.second, (int)num_features + 1, ltest);
    glm.train(mtrain, ltrain);
    std::vector<double> w(glm.weights.rows);
    for (int r = 0; r < glm.weights.rows; r++) w[r] = glm.weights.get(r, 0);
    weights = w;
    Matrix p = glm.predict(mtest);
    for (int row = 0; row < p.rows; row++)
      if (p.get(row, 0) == 0) p.set(row, 0, -1);
    double acc = std::get<0>(glm.accuracy(ltest, p, cfg_.verbose));
    Matrix q = glm.predict(mtrain);
    for (int row = 0; row < q.rows; row++)
      if (q.get(row, 0) == 0) q.set(row, 0, -1);
    glm.accuracy(ltrain, q, cfg_.verbose);
    if (acc - prev_acc <= 1 && acc >= 90.0) {
      weights = matvec.back();
      feat = features.back();
      if (cfg_.verbose) printf("feat size is %zu\n", feat.size());
      break;
    }
    matvec.push_back(weights);
    features.push_back(feat);
    prev_acc = acc;
    if (acc >= acc_cutoff) {
      if (cfg_.verbose) printf("breaking from acc cutoff\n");
      break;
    }
  }
  if (cfg_.verbose) printf("Final: feat size is %zu\nUsing %zu features\n", feat.size(), weights.size() - 1);
}

}  // namespace mc
