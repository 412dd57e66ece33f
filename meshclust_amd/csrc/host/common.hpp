// common.hpp -- shared host-side helpers for the meshclust driver.
#pragma once
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/meshclust_amd.h"

namespace mc {

// Error the reference would raise (uncaught exception / exit).  The driver prints it and
// exits non-zero, as the reference does.
struct Error : std::runtime_error {
  int code;
  explicit Error(const std::string &m, int c = 1) : std::runtime_error(m), code(c) {}
};
// A rank stopping because another rank reported a failure (or an exchange was aborted): the
// multi-rank driver reports the failing rank's own error in preference to these.
// Several ranks (GPUs) sharing one clustering: rank r of `world`, and an all-gather of a fixed
// number of bytes per rank (RCCL between processes, a shared buffer between the threads of
// one process, gloo in the CPU tests).
struct ShardComm {
  int rank = 0, world = 1;
  int (*allgather)(void *user, const void *in, uint64_t bytes, void *out) = nullptr;
  void *user = nullptr;
};

struct PeerError : Error {
  explicit PeerError(const std::string &m) : Error(m, 1) {}
};

// Labels the all-gathers that follow on `comm` (run_pipeline wraps every rank's comm with a
// timer): per phase, the time this rank waited for the last rank to arrive and the exchange
// itself, "comm.<phase>.wait" / "comm.<phase>.xfer" in ms, with ".calls" and ".kb" beside them.
void comm_phase(const ShardComm *comm, const char *phase);

// Throws mc::Error when an ABI call fails (no fallback path exists).
inline void check(int rc, const char *what) {
  if (rc != MC_OK) {
    const char *e = mc_last_error();
    throw Error(std::string(what) + " failed: " + (e ? e : "?"), 3);
  }
}

// Per-phase wall-clock accounting (printed with --timing, read by bench.py).
struct PhaseTimer {
  std::map<std::string, double> ms;
  std::vector<std::string> order;
  void add(const std::string &k, double v) {
    if (!ms.count(k)) order.push_back(k);
    ms[k] += v;
  }
};

// MC_PHASE_LOG=1: every phase's start and end on stderr as it happens (unbuffered), so a run
// that stops making progress shows where (the multi-rank tests' time limits print the tail)
inline bool phase_log_on() {
  static const bool on = getenv("MC_PHASE_LOG") && atoi(getenv("MC_PHASE_LOG")) != 0;
  return on;
}

inline double phase_clock_ms() {  // (steady clock, ms; the phase log's timestamps)
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Scope {
  PhaseTimer &t;
  std::string k;
  std::chrono::steady_clock::time_point s;
  Scope(PhaseTimer &tt, std::string kk) : t(tt), k(std::move(kk)), s(std::chrono::steady_clock::now()) {
    if (phase_log_on()) fprintf(stderr, "[phase %p %.3f] + %s\n", (void *)&tt, phase_clock_ms(), k.c_str());
  }
  ~Scope() {
    auto e = std::chrono::steady_clock::now();
    const double v = std::chrono::duration<double, std::milli>(e - s).count();
    t.add(k, v);
    if (phase_log_on()) fprintf(stderr, "[phase %p %.3f] - %s %.3f ms\n", (void *)&t, phase_clock_ms(), k.c_str(), v);
  }
};

}  // namespace mc
