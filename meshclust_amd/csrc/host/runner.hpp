// runner.hpp -- the meshclust driver: options (Runner::get_opts, src/cluster/src/Runner.cpp:
// 150-263), k choice (find_k :265-292), histogram width dispatch (run :41-90) and the
// do_run pipeline (:321-375), on top of the libmcgpu C-ABI.
#pragma once
#include <string>
#include <vector>

#include "cluster.hpp"
#include "common.hpp"
#include "fasta.hpp"
#include "trainer.hpp"

namespace mc {

struct Options {
  int k = -1;
  double similarity = 0.90;
  int iterations = 15;
  int delta = 5;
  bool align = false;
  int sample_size = 0;
  int pivots = 20;
  int threads = 0;  // 0 = OpenMP default
  std::string output = "output.clstr";
  std::vector<std::string> files;
  // additions of this implementation
  int device = 0;
  std::vector<int> devices;  // --devices 0,1,..: one clustering shared by these GPUs (RCCL)
  bool quiet = false;
  std::string stats_json;  // per-phase timings + work counts
};

// Parses argv like the reference; bad input throws mc::Error (OptionError in runner.cpp)
// with the reference's message and exit code.
Options parse_options(int argc, char **argv, bool require_files = true);

struct RunResult {
  std::vector<Center> part;
  PhaseTimer timer;
  ClusterStats stats;
  int k = 0;
  int width = 1;
  uint64_t largest = 0;
  size_t n = 0;
};

// Full pipeline on an already parsed dataset and an open context (bench.py reuses both).
bool tune_host_heap();  // process-global malloc settings (runner.cpp); true when applied
RunResult run_pipeline(const Dataset &ds, mc_ctx *ctx, Options opt, bool upload = true,
                       const ShardComm *comm = nullptr);

// JSON summary of a run (phase timings, work counts) for --stats-json and the C API.
std::string stats_json(const RunResult &rr, double parse_ms, double write_ms);

int meshclust_main(int argc, char **argv);

}  // namespace mc
