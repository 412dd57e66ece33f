// bvec.hpp -- host mirror of the reference's length-binned candidate store
// (src/cluster/src/bvec.{h,cpp}, bvec_iterator.{h,cpp}).
//
// After insert_finalize the bvec is only ever shrunk (pop / erase / remove_available), so
// the device keeps one static candidate order (bin-major, length-sorted within each bin)
// plus an alive mask; this mirror keeps the bins themselves so that get_range's quirks
// (empty-bin fallbacks that widen the window, the high = mid binary search) are evaluated
// exactly, and translates bvec positions (bin, column) into static positions.
#pragma once
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

namespace mc {

struct BIdx {
  size_t first = 0, second = 0;
};

class BVec {
 public:
  BVec(const std::vector<uint64_t> &lengths_by_id, uint64_t bin_size = 1000);  // bvec.cpp:9-24
  void insert(uint32_t id);                                                   // bvec.cpp:151-177
  void insert_finalize(int threads = 1);                                                 // bvec.cpp:208-218
  uint32_t pop();                                                             // bvec.cpp:26-37
  std::pair<BIdx, BIdx> get_range(uint64_t begin_len, uint64_t end_len) const;  // bvec.cpp:245-278
  void erase(size_t r, size_t c);                                             // bvec.cpp:280-284

  // The get_close loop `for (i = istart; i <= iend; ++i)` under OpenMP runs
  // (iend - istart) + 1 iterations (bvec_iterator::operator-, bvec_iterator.h:61-76),
  // visiting istart advanced k times.  Returns that count (<= 0: no iteration) and, when
  // positive, the static positions of the first and last visited candidates.
  int64_t window(const BIdx &b, const BIdx &e, uint64_t *S, uint64_t *E) const;
  // remove_available (bvec.cpp:289-318): drop the given static positions (ascending) from
  // bins a..b, appending their ids to `available` in bvec order.
  void remove_positions(const std::vector<uint32_t> &pos_sorted, size_t a, size_t b,
                        std::vector<uint32_t> &available);
  // (r, c) of the static position pos (alive).
  std::pair<size_t, size_t> locate(uint64_t pos) const;

  const std::vector<uint32_t> &static_order() const { return order_; }
  // current bins (static positions, after insert_finalize), begin bounds, bin of a position
  const std::vector<std::vector<uint32_t>> &bins() const { return data_; }
  const std::vector<uint64_t> &begin_bounds() const { return begin_bounds_; }
  const std::vector<uint64_t> &static_lengths() const { return plen_; }
  uint64_t spos(uint32_t id) const { return spos_[id]; }
  size_t size() const;
  static const uint32_t NONE = 0xffffffffu;

 private:
  bool index_of(uint64_t len, size_t *front, size_t *back) const;
  bool inner_index_of(uint64_t len, size_t &idx, size_t *front, size_t *back) const;

  const std::vector<uint64_t> &len_;
  std::vector<std::vector<uint32_t>> data_;  // ids until insert_finalize, static positions after
  std::vector<uint64_t> begin_bounds_;
  std::vector<uint32_t> order_;   // static position -> id
  std::vector<uint64_t> spos_;    // id -> static position
  std::vector<uint32_t> bin_of_;  // static position -> bin (bins never change membership)
  std::vector<uint64_t> plen_;    // static position -> length
  std::vector<std::pair<uint64_t, std::pair<size_t, size_t>>> index_memo_;  // length -> index_of
  uint64_t memo_lo_ = 0;                                  // ... or by length - memo_lo_
  std::vector<std::pair<uint32_t, uint32_t>> memo_tab_;  // (0xffffffff: not looked up yet)
  std::vector<uint32_t> sizes_;  // entries per bin while inserting (insert's scan reads these)
  std::vector<uint64_t> pend_;   // the inserts so far, bin << 32 | id (insert_finalize places them)
};

}  // namespace mc
