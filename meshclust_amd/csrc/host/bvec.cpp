// bvec.cpp -- see bvec.hpp.  Index arithmetic follows the reference line by line in meaning
// (size_t wrap-arounds included); storage is ids instead of (Point*, bool) pairs because the
// "similar" marks live on the device.
#include "bvec.hpp"

#include <algorithm>
#include <cstdlib>
#ifdef __AVX2__
#include <immintrin.h>
#endif
#include <limits>

#include "common.hpp"
#include "lazysort.hpp"

namespace mc {

BVec::BVec(const std::vector<uint64_t> &lengths_by_id, uint64_t bin_size) : len_(lengths_by_id) {
  // the sorted lengths at ranks 0, bin_size, 2 bin_size, ...: from a histogram of the lengths
  // when they are small (every read up to 64 Mb), else from the sort itself
  uint64_t mx = 0;
  for (uint64_t l : lengths_by_id) mx = l > mx ? l : mx;
  const size_t n = lengths_by_id.size();
  if (n && mx < (1ull << 26) && mx < 64 * (uint64_t)n + 1024) {
    std::vector<uint32_t> cnt(mx + 1, 0);
    for (uint64_t l : lengths_by_id) cnt[l]++;
    uint64_t v = 0, below = 0;  // ranks [below, below + cnt[v]) hold length v
    for (uint64_t i = 0; i < n; i += bin_size) {
      while (below + cnt[v] <= i) below += cnt[v++];
      begin_bounds_.push_back(v);
    }
  } else {
    std::vector<uint64_t> lengths = lengths_by_id;
    std::sort(lengths.begin(), lengths.end());
    for (uint64_t i = 0; i < lengths.size(); i += bin_size) begin_bounds_.push_back(lengths[i]);
  }
  data_.resize(begin_bounds_.size());
  sizes_.assign(begin_bounds_.size(), 0);
  pend_.reserve(n);
  if (n && begin_bounds_.size() < 0xffffffffull) {
    uint64_t lo = ~0ull;
    for (uint64_t l : lengths_by_id) lo = l < lo ? l : lo;
    if (mx - lo < (1ull << 22)) {
      memo_lo_ = lo;
      memo_tab_.assign(mx - lo + 1, {(uint32_t)-1, (uint32_t)-1});
    }
  }
}

bool BVec::index_of(uint64_t point, size_t *pfront, size_t *pback) const {
  size_t low = begin_bounds_.size() - 1, high = 0;
  for (size_t i = 0; i < begin_bounds_.size(); i++) {
    size_t prev = 0, prev_index = 0;
    if (i > 0) {
      prev_index = i - 1;
      prev = begin_bounds_[i - 1];
    }
    if (point >= prev && point <= begin_bounds_[i]) {
      low = std::min(low, prev_index);
      high = std::max(high, prev_index);
    }
  }
  if (point >= begin_bounds_[begin_bounds_.size() - 1]) high = std::max(high, begin_bounds_.size() - 1);
  if (pfront) *pfront = low;
  if (pback) *pback = high;
  return true;
}

bool BVec::inner_index_of(uint64_t length, size_t &idx, size_t *pfront, size_t *pback) const {
  if (data_.at(idx).empty() || idx == data_.size()) {
    if (pfront) {
      for (size_t i = 0; i < data_.size(); i++)
        if (!data_.at(i).empty()) {
          idx = i;
          *pfront = 0;
          break;
        }
    }
    if (pback) {
      for (int i = (int)data_.size() - 1; i >= 0; i--)
        if (!data_.at(i).empty()) {
          idx = i;
          *pback = 0;
          break;
        }
    }
    return true;
  }
  const auto &bin = data_[idx];
  size_t front = 0, back = 0;
  size_t low = 0, high = bin.size() - 1;
  if (length < plen_[bin[low]] && pfront != nullptr) *pfront = low;
  if (length > plen_[bin[high]] && pback != nullptr) *pback = high;
  for (; low <= high;) {
    size_t mid = (low + high) / 2;
    uint64_t d = plen_[bin[mid]];
    if (d == length) {
      front = mid;
      back = mid;
      break;
    } else if (length < d) {
      high = mid;
    } else if (length > d) {
      low = mid + 1;
    }
    if (low == high) {
      front = low;
      back = high;
      break;
    }
  }
  if (pfront) {
    for (long i = (long)front; i >= 0 && plen_[bin[i]] == length; i--) front = (size_t)i;
    *pfront = front;
  }
  if (pback) {
    for (long i = (long)back; i < (long)bin.size() && plen_[bin[i]] == length; i++) back = (size_t)i;
    *pback = back;
  }
  return true;
}

void BVec::insert(uint32_t id) {
  uint64_t len = len_[id];
  size_t front = 0, back = 0;
  // index_of depends only on the length and the (fixed) bin bounds: memoise it (a table indexed
  // by the length when the lengths span a small range -- every insert's lookup one load, not a
  // binary search with a mispredicted branch per level -- else a sorted list)
  if (len >= memo_lo_ && len - memo_lo_ < memo_tab_.size()) {
    auto &e = memo_tab_[len - memo_lo_];
    if (e.first == (uint32_t)-1) {
      index_of(len, &front, &back);
      e = {(uint32_t)front, (uint32_t)back};
    }
    front = e.first;
    back = e.second;
  } else {
    auto it = std::lower_bound(index_memo_.begin(), index_memo_.end(), len,
                               [](const std::pair<uint64_t, std::pair<size_t, size_t>> &e, uint64_t v) { return e.first < v; });
    if (it != index_memo_.end() && it->first == len) {
      front = it->second.first;
      back = it->second.second;
    } else {
      index_of(len, &front, &back);
      index_memo_.insert(it, {len, {front, back}});
    }
  }
  // the middle one of the bins front..back with the fewest entries (min_sizes[size / 2]): the
  // smallest size over the range, how many bins have it, then the (count / 2)-th of them -- two
  // passes over the contiguous bin sizes (config D: every insert's range is tens of bins wide)
  if (front > back || back >= sizes_.size()) throw Error("bvec: no bins to insert into", 1);
  const uint32_t *sz = sizes_.data();
  const size_t n = back - front + 1;
  uint32_t minimum = 0xffffffffu;
  size_t count = 0, i = 0;
#ifdef __AVX2__
  // eight bins per step: the minimum, then a mask of the bins at it (popcount), and the k-th
  // of them found eight bins at a time
  __m256i vm = _mm256_set1_epi32(-1);
  for (; i + 8 <= n; i += 8) vm = _mm256_min_epu32(vm, _mm256_loadu_si256((const __m256i *)(sz + front + i)));
  alignas(32) uint32_t lanes[8];
  _mm256_store_si256((__m256i *)lanes, vm);
  for (int l = 0; l < 8; l++) minimum = lanes[l] < minimum ? lanes[l] : minimum;
  for (; i < n; i++) minimum = sz[front + i] < minimum ? sz[front + i] : minimum;
  const __m256i vmin = _mm256_set1_epi32((int)minimum);
  auto mask8 = [&](size_t j) {
    return (uint32_t)_mm256_movemask_ps(
        _mm256_castsi256_ps(_mm256_cmpeq_epi32(_mm256_loadu_si256((const __m256i *)(sz + front + j)), vmin)));
  };
  for (i = 0; i + 8 <= n; i += 8) count += (size_t)__builtin_popcount(mask8(i));
  for (; i < n; i++) count += sz[front + i] == minimum;
  size_t k = count / 2, bin = front;
  for (i = 0; i + 8 <= n; i += 8) {
    uint32_t m = mask8(i);
    const size_t c = (size_t)__builtin_popcount(m);
    if (k >= c) {
      k -= c;
      continue;
    }
    while (k--) m &= m - 1;
    bin = front + i + (size_t)__builtin_ctz(m);
    break;
  }
  if (i + 8 > n)
    for (bin = front + i;; bin++)
      if (sz[bin] == minimum && k-- == 0) break;
#else
  for (; i < n; i++) minimum = sz[front + i] < minimum ? sz[front + i] : minimum;
  for (i = 0; i < n; i++) count += sz[front + i] == minimum;
  size_t k = count / 2, bin = front;
  for (;; bin++)
    if (sz[bin] == minimum && k-- == 0) break;
#endif
  pend_.push_back(((uint64_t)bin << 32) | id);  // (placed into the bins by insert_finalize)
  sizes_[bin]++;
}

void BVec::insert_finalize(int threads) {
  // the inserts' bins, in insertion order (the order a bin's ids had when pushed one by one)
  for (size_t b = 0; b < data_.size(); b++) data_[b].reserve(data_[b].size() + sizes_[b]);
  for (uint64_t e : pend_) data_[e >> 32].push_back((uint32_t)e);
  pend_.clear();
  pend_.shrink_to_fit();
  // std::sort of each bin by length (bvec.cpp's insert_finalize): the same permutation from
  // LazyIntroSort::sort_words on (length << 32 | id) words, bins and subranges as tasks
  bool wide = false;
  for (uint64_t l : len_) wide |= l >> 32 != 0;
  if (wide) {
    for (auto &bin : data_)
      std::sort(bin.begin(), bin.end(), [&](uint32_t a, uint32_t b) { return len_[a] < len_[b]; });
  } else {
#pragma omp parallel num_threads(threads > 0 ? threads : 1)
#pragma omp single
    for (auto &bin : data_) {
      if (bin.size() < 2) continue;
      std::vector<uint32_t> *b = &bin;
#pragma omp task firstprivate(b)
      {
        std::vector<uint64_t> w(b->size());
        for (size_t t = 0; t < w.size(); t++) w[t] = (len_[(*b)[t]] << 32) | (*b)[t];
        LazyIntroSort::sort_words(w.data(), (int64_t)w.size());
        for (size_t t = 0; t < w.size(); t++) (*b)[t] = (uint32_t)w[t];
      }
    }
  }
  // from here on bins hold static positions (ascending): bin r's entries are the positions
  // from its offset on (the bins in order), each bin filled by one thread
  std::vector<uint64_t> off(data_.size() + 1, 0);
  for (size_t r = 0; r < data_.size(); r++) off[r + 1] = off[r] + data_[r].size();
  const uint64_t tot = off.back();
  order_.assign(tot, 0);
  bin_of_.assign(tot, 0);
  plen_.assign(tot, 0);
  spos_.assign(len_.size(), std::numeric_limits<uint64_t>::max());
#pragma omp parallel for num_threads(threads > 0 ? threads : 1) schedule(dynamic, 16)
  for (int64_t r = 0; r < (int64_t)data_.size(); r++) {
    uint64_t p = off[r];
    for (uint32_t &e : data_[r]) {
      const uint32_t id = e;
      e = (uint32_t)p;
      spos_[id] = p;  // (ids are unique: no two threads write one entry)
      order_[p] = id;
      bin_of_[p] = (uint32_t)r;
      plen_[p] = len_[id];
      p++;
    }
  }
}

uint32_t BVec::pop() {
  for (auto &bin : data_)
    if (!bin.empty()) {
      uint32_t p = bin[0];
      bin.erase(bin.begin());
      return order_[p];
    }
  return NONE;
}

std::pair<BIdx, BIdx> BVec::get_range(uint64_t begin_len, uint64_t end_len) const {
  BIdx front, back;
  front.first = 0;
  front.second = 0;
  back.first = data_.size() - 1;
  back.second = data_[back.first].size() - 1;
  index_of(begin_len, &front.first, nullptr);
  index_of(end_len, nullptr, &back.first);
  inner_index_of(begin_len, front.first, &front.second, nullptr);
  inner_index_of(end_len, back.first, nullptr, &back.second);
  return {front, back};
}

void BVec::erase(size_t r, size_t c) { data_.at(r).erase(data_.at(r).begin() + c); }

int64_t BVec::window(const BIdx &b, const BIdx &e, uint64_t *S, uint64_t *E) const {
  // bvec_iterator::operator- (bvec_iterator.h:61-76), size_t arithmetic wrapping
  auto less = [](const BIdx &x, const BIdx &y) {
    return x.first < y.first || (x.first == y.first && x.second < y.second);
  };
  auto minus = [&](const BIdx &x, const BIdx &y) -> int64_t {  // x - y with x >= y
    if (x.first == y.first) return (int64_t)(x.second - y.second);
    uint64_t sum = 0;
    sum += x.second;
    sum += data_.at(y.first).size() - y.second;
    for (size_t i = y.first + 1; i < x.first; i++) sum += data_.at(i).size();
    return (int64_t)sum;
  };
  int64_t diff = less(e, b) ? -minus(b, e) : minus(e, b);
  int64_t count = diff + 1;
  if (count <= 0) return count;
  // the first visited element is istart itself; deref = col->at(r).at(c)
  size_t r = b.first, c = b.second;
  if (r >= data_.size() || c >= data_[r].size()) throw Error("bvec_iterator dereference out of range", 1);
  *S = data_[r][c];
  int64_t remaining = count - 1;
  while (remaining > 0) {  // operator++ (bvec_iterator.cpp:3-21)
    int64_t avail = (int64_t)data_[r].size() - 1 - (int64_t)c;
    if (remaining <= avail) {
      c += (size_t)remaining;
      remaining = 0;
      break;
    }
    remaining -= avail + 1;
    r++;
    c = 0;
    while (r < data_.size() && data_[r].empty()) r++;
    if (r >= data_.size()) throw Error("tried incrementing null iterator", 1);
  }
  *E = data_[r][c];
  return count;
}

void BVec::remove_positions(const std::vector<uint32_t> &pos_sorted, size_t a, size_t b,
                            std::vector<uint32_t> &available) {
  // Only the bins holding flagged candidates change; within a bin the survivors keep their
  // order and the flagged ids leave in bvec order (== ascending static position).  Bins hold
  // ascending static positions, so each bin is compacted from its first flagged entry on.
  size_t k = 0;
  while (k < pos_sorted.size()) {
    const size_t r = bin_of_[pos_sorted[k]];
    if (r < a || r > b) throw Error("remove_available: flagged candidate outside the window bins", 3);
    auto &bin = data_[r];
    size_t j = (size_t)(std::lower_bound(bin.begin(), bin.end(), pos_sorted[k]) - bin.begin());
    size_t w = j;
    for (; j < bin.size(); j++) {
      const uint32_t p = bin[j];
      if (k < pos_sorted.size() && p == pos_sorted[k]) {
        available.push_back(order_[p]);
        k++;
        continue;
      }
      if (k >= pos_sorted.size() || bin_of_[pos_sorted[k]] != r) {  // no flagged entry left in this bin
        std::copy(bin.begin() + j, bin.end(), bin.begin() + w);
        w += bin.size() - j;
        break;
      }
      bin[w++] = p;
    }
    bin.resize(w);
    if (k < pos_sorted.size() && bin_of_[pos_sorted[k]] == r)
      throw Error("remove_available: flagged candidate not alive in its bin", 3);
  }
}

std::pair<size_t, size_t> BVec::locate(uint64_t pos) const {
  const size_t r = bin_of_[pos];
  const auto &bin = data_[r];
  auto it = std::lower_bound(bin.begin(), bin.end(), (uint32_t)pos);
  if (it == bin.end() || *it != pos) throw Error("bvec: static position not alive", 3);
  return {r, (size_t)(it - bin.begin())};
}

size_t BVec::size() const {
  size_t t = 0;
  for (const auto &b : data_) t += b.size();
  return t;
}

}  // namespace mc
