// trainer.hpp -- restatement of Trainer<T>::train and its sampling (src/cluster/src/Trainer.cpp:
// 201-333 resize_vec/get_labels, 490-651 bin_data/train, 653-783 split).  Every data-parallel
// piece (distance sort keys, NW identities, raw features) runs on the GPU through the C-ABI;
// the sampling, the sorts (std::sort, so tie order matches the reference) and the GLM fit
// stay on the host.
#pragma once
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

#include "common.hpp"
#include "fasta.hpp"
#include "feature.hpp"
#include "glm.hpp"

namespace mc {

using PairId = std::pair<uint32_t, uint32_t>;

struct TrainerConfig {
  size_t n_points = 3000;        // --sample (Runner.cpp:35-37)
  size_t max_pts_from_one = 20;  // --pivot  (Runner.h:31)
  double cutoff = 0.90;          // --id
  int k = 4;                     // 0 => alignment mode (Runner.cpp:332)
  int threads = 1;
  bool verbose = true;
  // several ranks: each runs the sampler's binary searches of its block of pivots and its
  // share of the label alignments; the results are all-gathered (null / world 1: one rank)
  const ShardComm *comm = nullptr;
  // the ids ordered by length as split's first std::sort leaves them (Trainer.cpp:672-675),
  // computed ahead by the caller (Trainer::length_order, overlapping the upload and K1); empty:
  // split computes it
  std::vector<uint32_t> length_order;
};

class Trainer {
 public:
  Trainer(const Dataset &ds, mc_ctx *ctx, const TrainerConfig &cfg, PhaseTimer &timer)
      : ds_(ds), ctx_(ctx), cfg_(cfg), timer_(timer) {}
  void train(double acc_cutoff = 97.5);
  // split's first sort: the ids by length, exactly as std::sort leaves them
  static std::vector<uint32_t> length_order(const Dataset &ds, int threads);
  mc_classifier classifier() const { return feat.to_classifier(weights); }

  FeatureSet feat;
  std::vector<double> weights;
  // exposed for tests / diagnostics
  std::vector<PairId> split_pairs;
  std::vector<std::pair<PairId, double>> label_pos, label_neg;
  uint64_t nw_pairs = 0, nw_cells = 0;  // work counters (NW cell updates)

 private:
  std::vector<PairId> split();
  void get_labels(const std::vector<PairId> &vec, std::vector<std::pair<PairId, double>> &bp,
                  std::vector<std::pair<PairId, double>> &bn);
  Matrix feat_matrix(const std::vector<PairId> &pos, const std::vector<PairId> &neg, int ncols,
                     Matrix &labels);
  void nw_batch(const std::vector<PairId> &pairs, std::vector<double> &ident);
  // all-gather of `words` u64 per rank (every rank the same count); false: one rank
  bool gather(const std::vector<uint64_t> &mine, std::vector<uint64_t> &all) const;
  bool hdr_less(uint32_t a, uint32_t b) const;

  const Dataset &ds_;
  mc_ctx *ctx_;
  TrainerConfig cfg_;
  PhaseTimer &timer_;
};

}  // namespace mc
