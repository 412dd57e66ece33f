// feature.cpp -- see feature.hpp.  Compiled with -ffp-contract=off (no FMA in the
// reference's normalize_cache / operator(), verified by objdump of Feature.o).
#include "feature.hpp"

#include <cfloat>
#include <cstdio>
#include <cstring>

#include "common.hpp"

namespace mc {

bool feat_is_sim(uint16_t f) {
  switch (f) {
    case MC_FEAT_ALIGN: return true;
    case MC_FEAT_LD: return false;
    case MC_FEAT_MANHATTAN: return false;
    case MC_FEAT_INTERSECTION: return true;
    case MC_FEAT_PEARSON: return false;
    case MC_FEAT_KULCZYNSKI2: return true;
    default: throw Error("bad feature flag " + std::to_string(f), 1);
  }
}

int FeatureSet::index_of(uint16_t f) const {
  for (size_t i = 0; i < lookup.size(); i++)
    if (lookup[i] == f) return (int)i;
  return -1;
}

void FeatureSet::add_feature(uint16_t f_flags, int combo) {
  if (combo != MC_COMBO_SQUARED && combo != MC_COMBO_SELF) throw Error("invalid combo", 1);
  std::vector<int> indices;
  for (uint32_t f = 1; f <= f_flags; f <<= 1) {
    if ((f_flags & f) != 0) {
      if ((flags & f) == 0) {
        lookup.push_back((uint16_t)f);
        mins.push_back(DBL_MAX);
        maxs.push_back(DBL_MIN);  // std::numeric_limits<double>::min(), not -DBL_MAX
        is_sims.push_back(feat_is_sim((uint16_t)f));
        is_finalized.push_back(false);
        flags |= (uint16_t)f;
      }
      indices.push_back(index_of((uint16_t)f));
    }
  }
  combos.emplace_back(combo, indices);
}

void FeatureSet::finalize() {
  for (size_t i = 0; i < is_finalized.size(); i++) is_finalized[i] = true;
}

std::vector<uint16_t> FeatureSet::flags_needed() const {
  std::vector<uint16_t> f;
  for (size_t i = 0; i < lookup.size(); i++)
    if (lookup[i] != MC_FEAT_ALIGN && !is_finalized[i]) f.push_back(lookup[i]);
  return f;
}

void FeatureSet::normalize_with(const std::vector<double> &raw, size_t npairs) {
  size_t col = 0;
  const size_t nflag = flags_needed().size();
  for (size_t i = 0; i < lookup.size(); i++) {
    double small = mins[i], big = maxs[i];
    if (lookup[i] == MC_FEAT_ALIGN) {
      mins[i] = 0;
      maxs[i] = 1;
      continue;
    }
    if (is_finalized[i]) continue;
    for (size_t j = 0; j < npairs; j++) {
      double v = raw[j * nflag + col];
      if (v < small) small = v;
      if (v > big) big = v;
    }
    mins[i] = small;
    maxs[i] = big;
    col++;
  }
}

void FeatureSet::normalize_cache(double *cache) const {
  for (size_t i = 0; i < lookup.size(); i++) {
    double val = (cache[i] - mins[i]) / (maxs[i] - mins[i]);
    cache[i] = is_sims[i] ? val : 1 - val;
  }
}

double FeatureSet::combo(int col, const double *cache) const {
  const auto &pr = combos.at(col);
  double prod = 1;
  if (pr.first == MC_COMBO_SELF) {
    for (int idx : pr.second) prod *= cache[idx];
  } else {
    for (int idx : pr.second) prod *= cache[idx] * cache[idx];
  }
  return prod;
}

mc_classifier FeatureSet::to_classifier(const std::vector<double> &weights) const {
  mc_classifier c;
  memset(&c, 0, sizeof c);
  if (lookup.size() > MC_MAX_SINGLE || combos.size() > MC_MAX_COMBO) throw Error("too many features", 1);
  c.n_single = (int)lookup.size();
  for (size_t i = 0; i < lookup.size(); i++) {
    c.lookup[i] = lookup[i];
    c.is_sim[i] = is_sims[i] ? 1 : 0;
    c.mins[i] = mins[i];
    c.maxs[i] = maxs[i];
  }
  c.n_combo = (int)combos.size();
  for (size_t i = 0; i < combos.size(); i++) {
    c.combo_kind[i] = combos[i].first;
    c.combo_len[i] = (int)combos[i].second.size();
    if (combos[i].second.size() > MC_MAX_COMBO_LEN) throw Error("combo too long", 1);
    for (size_t j = 0; j < combos[i].second.size(); j++) c.combo_idx[i][j] = combos[i].second[j];
  }
  if (weights.size() != combos.size() + 1) throw Error("weight/combo count mismatch", 1);
  for (size_t i = 0; i < weights.size(); i++) c.weights[i] = weights[i];
  return c;
}

void FeatureSet::print_bounds() const {
  for (size_t i = 0; i < lookup.size(); i++) printf("bounds[%zu]: %g to %g\n", i, mins[i], maxs[i]);
}

}  // namespace mc
