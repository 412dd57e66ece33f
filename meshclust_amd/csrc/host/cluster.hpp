// cluster.hpp -- restatement of ClusterFactory<T>::MS and its helpers
// (src/cluster/src/ClusterFactory.cpp:289-380 mean_shift_update, 382-425 get_mean,
// 427-493 merge, 495-520 print_output, 637-714 accumulate, 717-761 MS).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "bvec.hpp"
#include "common.hpp"
#include "fasta.hpp"

namespace mc {

struct Center {
  uint32_t centre;               // id of the point the centre was cloned from (Center.h:14-27)
  std::vector<uint32_t> points;  // members, in the reference's order
  bool del = false;
};

// The ranks (one process per GPU) that share one clustering.  Every get_close
// step of the accumulation is split over the ranks by record (static bvec blocks), each
// mean-shift iteration by centre; the ranks exchange partial step results and new centres with
// `allgather` (equal blocks of `bytes`, rank order into `out`; returns 0 on success).

// Fault injection for the multi-rank tests: MC_FAULT=<rank>:<stage> makes that rank throw at
// that stage ("upload", "train", "accumulate", "update"), so the tests can check that every
// other rank stops with an error instead of waiting in an exchange forever.
void fault_point(const ShardComm *comm, const char *stage);

struct ClusterConfig {
  const ShardComm *comm = nullptr;  // null: one rank
  double sim = 0.90;
  int iterations = 15;
  int delta = 5;
  bool verbose = true;
  bool align = false;  // classifier feature is Feature::align (Runner.cpp:32-34, 332)
  int width = 1;       // histogram bytes per bin (Runner.cpp:75-89)
};

struct ClusterStats {
  uint64_t scan_steps = 0;
  uint64_t scan_candidates = 0;  // sum of get_close window sizes (K2 evaluations)
  uint64_t update_evals = 0;     // filter evaluations in the mean-shift updates
  uint64_t merge_evals = 0;
  uint64_t update_iters_fixed = 0;  // update iterations left out at a fixed point (counted, not run)
  uint64_t update_evals_run = 0;    // update_evals of the iterations actually run
  uint64_t nw_pairs = 0, nw_cells = 0;  // training alignments
  uint64_t align_nw_pairs = 0, align_nw_cells = 0;  // alignment mode: classifier alignments
  // which accumulation loop ran: "device" (mc_accumulate, one persistent kernel) or "steps"
  // (host-driven mc_scan per get_close step) with the reason
  std::string accum_path;
  std::string update_path;  // several ranks: the mean-shift iterations split by centre or replicated
};

// Runs accumulation + `iterations` rounds of mean-shift update and merge.
std::vector<Center> mean_shift_cluster(const Dataset &ds, mc_ctx *ctx, BVec &bv, const ClusterConfig &cfg,
                                       PhaseTimer &timer, ClusterStats &stats);

// CD-HIT style writer (ClusterFactory.cpp:495-520).
void write_clstr(const std::string &path, const Dataset &ds, const std::vector<Center> &part, int threads = 1);

}  // namespace mc
