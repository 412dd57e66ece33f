// feature.hpp -- host-side state of the reference's Feature<T> (src/cluster/src/Feature.h:46-134):
// which single features exist (lookup order), their min/max normalisation bounds and the
// combo products.  Raw feature values are computed on the GPU (mc_pair_features); the
// bookkeeping around them is restated here exactly.
#pragma once
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

#include "../../../include/meshclust_amd.h"

namespace mc {

struct FeatureSet {
  uint16_t flags = 0;
  std::vector<std::pair<int, std::vector<int>>> combos;
  std::vector<double> mins, maxs;
  std::vector<bool> is_sims, is_finalized;
  std::vector<uint16_t> lookup;

  void add_feature(uint16_t f_flags, int combo);   // Feature.cpp:7-31
  void finalize();                                 // Feature.cpp:34-40
  size_t size() const { return combos.size(); }
  int index_of(uint16_t f) const;
  // Feature.cpp:86-114: raw values of the not-yet-finalized singles over the pairs; the
  // caller supplies raw[pair * nflag + f] for `flags_needed()` in that order.
  std::vector<uint16_t> flags_needed() const;
  void normalize_with(const std::vector<double> &raw, size_t npairs);
  void normalize_cache(double *cache) const;       // Feature.cpp:41-52
  double combo(int col, const double *cache) const;  // Feature.h:69-88
  mc_classifier to_classifier(const std::vector<double> &weights) const;
  void print_bounds() const;
};

bool feat_is_sim(uint16_t f);  // Feature.cpp:161-204

}  // namespace mc
