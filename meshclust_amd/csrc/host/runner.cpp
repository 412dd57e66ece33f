// runner.cpp -- see runner.hpp.
#include "runner.hpp"

#include <libgen.h>
#include <malloc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <atomic>
#include <condition_variable>
#include <exception>
#include <mutex>
#include <memory>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace mc {

static void usage(const char *prog) {
  printf("Usage: %s *.fasta [--id 0.90] [--kmer 3] [--delta 5] [--output output.clstr] [--iterations 20] "
         "[--align] [--sample 3000] [--pivot 40] [--threads TMAX] [--device GPU] [--devices GPU,GPU,..] "
         "[--stats-json FILE]\n",
         prog);
  printf("MI355X-native MeShClust (meshclust_amd, C-ABI v%d)\n", MC_ABI_VERSION);
}

// Bad options end the reference with a message (Runner.cpp:150-263: usage on stdout or a
// message on stderr, then exit).  Here they throw OptionError, so a library caller (capi.cpp)
// gets an error code instead of losing its process; meshclust_main prints the same text.
struct OptionError : Error {
  bool usage;  // print the usage text (stdout) instead of the message (stderr)
  OptionError(const std::string &m, int c, bool u) : Error(m, c), usage(u) {}
};

Options parse_options(int argc, char **argv, bool require_files) {
  Options o;
  for (int i = 1; i < argc; i++) {
    std::string arg = argv[i];
    auto need_long = [&](long lo, const char *msg) -> long {
      errno = 0;
      long v = strtol(argv[i + 1], nullptr, 10);
      if (errno) throw OptionError(std::string(argv[i + 1]) + ": " + strerror(errno), EXIT_FAILURE, false);
      if (v < lo) throw OptionError(msg, EXIT_FAILURE, false);
      return v;
    };
    if (arg == "--id" && i + 1 < argc) {
      char *end = nullptr;
      double v = strtod(argv[i + 1], &end);
      if (end == argv[i + 1] || v <= 0 || v >= 1) throw OptionError("Similarity must be between 0 and 1", EXIT_FAILURE, false);
      o.similarity = v;
      i++;
    } else if ((arg == "-k" || arg == "--kmer") && i + 1 < argc) {
      o.k = (int)need_long(1, "K must be greater than 0.");
      i++;
    } else if ((arg == "-o" || arg == "--output") && i + 1 < argc) {
      o.output = argv[++i];
    } else if (arg == "-a" || arg == "--align") {
      o.align = true;
    } else if ((arg == "-s" || arg == "--sample") && i + 1 < argc) {
      o.sample_size = (int)need_long(1, "Sample size must be greater than 0.");
      i++;
    } else if ((arg == "-p" || arg == "--pivot") && i + 1 < argc) {
      o.pivots = (int)need_long(1, "Points per pivot must be greater than 0.");
      i++;
    } else if ((arg == "-t" || arg == "--threads") && i + 1 < argc) {
      int t = atoi(argv[i + 1]);
      if (t <= 0) throw OptionError("Number of threads must be greater than 0.", 1, false);
      o.threads = t;
      i++;
    } else if ((arg == "-d" || arg == "--delta") && i + 1 < argc) {
      o.delta = (int)need_long(0, "Delta must be greater than 0.");
      i++;
    } else if ((arg == "-i" || arg == "--iter" || arg == "--iterations") && i + 1 < argc) {
      o.iterations = (int)need_long(1, "Iterations must be greater than 0.");
      i++;
    } else if (arg == "--device" && i + 1 < argc) {
      o.device = atoi(argv[++i]);
    } else if (arg == "--devices" && i + 1 < argc) {
      o.devices.clear();
      for (const char *p = argv[++i]; *p;) {
        char *end = nullptr;
        long d = strtol(p, &end, 10);
        if (end == p || d < 0) throw OptionError("--devices takes a comma-separated list of GPU indices", 1, false);
        o.devices.push_back((int)d);
        p = *end == ',' ? end + 1 : end;
        if (*end && *end != ',') throw OptionError("--devices takes a comma-separated list of GPU indices", 1, false);
      }
    } else if (arg == "--stats-json" && i + 1 < argc) {
      o.stats_json = argv[++i];
    } else if (arg == "--quiet") {
      o.quiet = true;
    } else {
      struct stat st;
      if (stat(argv[i], &st) == 0 && S_ISREG(st.st_mode)) o.files.push_back(argv[i]);
      else throw OptionError(std::string("unknown option or missing file: ") + argv[i], EXIT_FAILURE, true);
    }
  }
  if (o.files.empty() && require_files) throw OptionError("no input files", EXIT_FAILURE, true);
  std::sort(o.files.begin(), o.files.end(), [](const std::string &a, const std::string &b) {
    char *as = strdup(a.c_str()), *bs = strdup(b.c_str());
    bool r = std::string(basename(as)) < std::string(basename(bs));
    free(as);
    free(bs);
    return r;
  });
  return o;
}

// Runner::find_k (Runner.cpp:265-292): integer mean length per file, mean over files.
static int find_k(const Dataset &ds, bool verbose) {
  unsigned long long length = 0;
  for (size_t f = 0; f < ds.file_count.size(); f++) length += ds.file_len_sum[f] / ds.file_count[f];
  length /= ds.file_count.size();
  int newk = (int)std::ceil(std::log((double)length) / std::log(4)) - 1;
  if (verbose) printf("avg length: %llu\nRecommended K: %d\n", length, newk);
  return newk;
}

// The parser's file buffer and the training sampler's short-lived arrays (~150 MB per
// clustering at config B: split keys, the per-pivot sort inputs) are large blocks.  This keeps
// freed blocks in the heap -- no mmap for large blocks (M_MMAP_MAX 0: glibc caps
// M_MMAP_THRESHOLD at 32 MiB, so a threshold cannot cover them), no trimming -- so repeated
// parses and clusterings in one process touch no new pages.  Process-global: the CLI calls it
// for its own process; a host embedding the library opts in with mcl_tune_host_heap.
bool tune_host_heap() {
  static int ok = -1;
  // (trim threshold at mallopt's int maximum: config D's 1 GB file buffer stays in the heap)
  if (ok < 0) ok = mallopt(M_MMAP_MAX, 0) == 1 && mallopt(M_TRIM_THRESHOLD, std::numeric_limits<int>::max()) == 1;
  return ok == 1;
}

// The ranks' all-gathers, timed.  Each block travels with its sender's entry time on the
// host's monotonic clock (one clock for every process of a node), so a rank splits each
// exchange into waiting for the last rank to arrive and the exchange after that.
struct TimedComm {
  ShardComm inner;
  PhaseTimer *timer = nullptr;
  std::string phase = "setup";
  std::vector<uint8_t> ib, ob;
};

static double mono_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int timed_allgather(void *user, const void *in, uint64_t bytes, void *out) {
  auto *t = (TimedComm *)user;
  const int W = t->inner.world;
  const uint64_t blk = 8 + bytes;
  t->ib.resize(blk);
  t->ob.resize(blk * (uint64_t)W);
  const double t0 = mono_us();
  memcpy(t->ib.data(), &t0, 8);
  if (bytes) memcpy(t->ib.data() + 8, in, bytes);
  const int rc = t->inner.allgather(t->inner.user, t->ib.data(), blk, t->ob.data());
  const double t1 = mono_us();
  if (rc) return rc;
  double last = t0;
  for (int r = 0; r < W; r++) {
    double tr;
    memcpy(&tr, t->ob.data() + blk * r, 8);
    last = std::max(last, tr);
    if (bytes) memcpy((char *)out + bytes * r, t->ob.data() + blk * r + 8, bytes);
  }
  const std::string k = "comm." + t->phase;
  t->timer->add(k + ".wait", (last - t0) / 1000.0);
  t->timer->add(k + ".xfer", (t1 - std::max(last, t0)) / 1000.0);
  t->timer->add(k + ".calls", 1.0);
  t->timer->add(k + ".kb", (double)(blk * (uint64_t)W) / 1024.0);
  return 0;
}

void comm_phase(const ShardComm *comm, const char *phase) {
  if (comm && comm->allgather == timed_allgather) ((TimedComm *)comm->user)->phase = phase;
}

// Ranks sharing one GPU (the one-GPU rehearsal, or --devices 0,0): each context takes a CU
// partition of its own (mc_ctx_partition), slot = its order among the ranks with the same PCI
// bus id.  Their kernels then never queue behind one another's persistent grids.
static void partition_shared_gpu(const ShardComm &comm, mc_ctx *ctx, PhaseTimer &timer) {
  struct Blk {
    char pci[64];
  };
  Blk mine{};
  if (mc_ctx_pci_bus_id(ctx, mine.pci, sizeof mine.pci) != MC_OK) mine.pci[0] = 0;
  std::vector<Blk> all(comm.world);
  if (comm.allgather(comm.user, &mine, sizeof mine, all.data()) != 0) throw PeerError("all-gather across ranks failed");
  int share = 0, slot = 0;
  for (int r = 0; r < comm.world; r++)
    if (mine.pci[0] && strncmp(all[r].pci, mine.pci, sizeof mine.pci) == 0) {
      if (r < comm.rank) slot++;
      share++;
    }
  if (share > 1 && !getenv("MC_NO_PARTITION")) {
    check(mc_ctx_partition(ctx, slot, share), "mc_ctx_partition");
    timer.add("gpu_share", (double)share);
  }
}

RunResult run_pipeline(const Dataset &ds, mc_ctx *ctx, Options opt, bool upload, const ShardComm *comm_in) {
  RunResult rr;
  TimedComm tcomm;
  ShardComm wrapped;
  const ShardComm *comm = comm_in;
  if (comm_in && comm_in->allgather) {
    tcomm.inner = *comm_in;
    tcomm.timer = &rr.timer;
    wrapped = *comm_in;
    wrapped.allgather = timed_allgather;
    wrapped.user = &tcomm;
    comm = &wrapped;
    if (comm->world > 1) partition_shared_gpu(*comm, ctx, rr.timer);
  }
  rr.n = ds.size();
  const bool verbose = !opt.quiet;
  int threads = opt.threads;
#ifdef _OPENMP
  if (threads <= 0) threads = omp_get_max_threads();
#else
  threads = 1;
#endif
  if (opt.k == -1) opt.k = find_k(ds, verbose);
  if (opt.similarity < 0.6) opt.align = true;
  if (opt.sample_size == 0) opt.sample_size = 3000;
  if (opt.k < 1 || opt.k > 12) throw Error("k must be in 1..12 on this engine (4^k-bin dense histograms)", 1);
  rr.k = opt.k;
  auto t0 = std::chrono::steady_clock::now();
  // split's first sort (ids by length) depends on the lengths alone: a host thread computes it
  // while the upload and K1 run (k-mer mode; joined before the trainer starts)
  std::vector<uint32_t> len_order;
  std::exception_ptr len_err;  // (rethrown after the join: an exception must not end the thread)
  std::thread len_thread;
  if (!opt.align && opt.similarity >= 0.6)
    len_thread = std::thread([&]() {
      try {
        len_order = Trainer::length_order(ds, threads);
      } catch (...) {
        len_err = std::current_exception();
      }
    });
  struct JoinLen {
    std::thread &t;
    ~JoinLen() {
      if (t.joinable()) t.join();
    }
  } join_len{len_thread};
  // The bvec (Runner.cpp:345-350: construct, insert every point, insert_finalize) depends only
  // on the lengths, so a host thread builds it while the upload, K1 and the trainer run (the
  // host mostly waits on the GPU there), with a quarter of the cores for its per-bin sorts (the
  // trainer's teams keep the rest); its time -- the constructor included -- overlaps them.
  std::unique_ptr<BVec> bvp;
  double bvec_ms = 0, bvec_lap[2] = {0, 0};  // whole build; inserts, finalize
  std::exception_ptr bvec_err;
  std::thread bvec_thread([&]() {
    try {
      using clk = std::chrono::steady_clock;
      const auto b0 = clk::now();
      bvp.reset(new BVec(ds.lengths, 1000));
      const auto b1 = clk::now();
      for (uint32_t id = 0; id < ds.size(); id++) bvp->insert(id);
      const auto b2 = clk::now();
      bvp->insert_finalize(std::max(1, threads / 4));
      const auto b3 = clk::now();
      bvec_ms = std::chrono::duration<double, std::milli>(b3 - b0).count();
      bvec_lap[0] = std::chrono::duration<double, std::milli>(b2 - b1).count();
      bvec_lap[1] = std::chrono::duration<double, std::milli>(b3 - b2).count();
    } catch (...) {
      bvec_err = std::current_exception();
    }
  });
  struct JoinBvec {
    std::thread &t;
    ~JoinBvec() {
      if (t.joinable()) t.join();
    }
  } join_bvec{bvec_thread};
  fault_point(comm, "upload");
  if (upload) {
    Scope s(rr.timer, "upload");
    check(mc_load_packed(ctx, ds.packed.data(), ds.pk_off.data(), ds.seq_off.data(), ds.size(), ds.exc_pos.data(),
                         ds.exc_val.data(), ds.exc_pos.size(), ds.seg.data(), ds.seg_off.data()),
          "mc_load_packed");
  }
  {
    Scope s(rr.timer, "kmer");
    check(mc_kmer_max(ctx, opt.k, &rr.largest), "mc_kmer_max");
    int width = rr.largest <= 0xff ? 1 : rr.largest <= 0xffff ? 2 : rr.largest <= 0xffffffffull ? 4 : 8;
    // diagnostics / tests: a wider histogram type than Runner.cpp:75-89 would pick (the
    // 32/64-bit feature paths, with their unsigned wrap-arounds, on small inputs)
    if (const char *fw = getenv("MC_FORCE_WIDTH")) width = std::max(width, atoi(fw));
    rr.width = width;
    if (verbose) printf("Using %d bit histograms\n", 8 * width);
    check(mc_kmer_build(ctx, opt.k, width), "mc_kmer_build");
  }
  comm_phase(comm, "train");
  TrainerConfig tc;
  tc.n_points = opt.sample_size;
  tc.max_pts_from_one = opt.pivots;
  tc.cutoff = opt.similarity;
  tc.k = opt.align ? 0 : opt.k;
  tc.threads = threads;
  tc.verbose = verbose;
  tc.comm = comm;
  {
    Scope s(rr.timer, "len_order.wait");
    if (len_thread.joinable()) len_thread.join();
  }
  if (len_err) std::rethrow_exception(len_err);
  tc.length_order = std::move(len_order);
  Trainer tr(ds, ctx, tc, rr.timer);
  {
    Scope s(rr.timer, "train");
    tr.train();
  }
  {
    Scope s(rr.timer, "bvec.wait");
    bvec_thread.join();
  }
  fault_point(comm, "train");
  rr.timer.add("bvec.overlapped", bvec_ms);
  rr.timer.add("bvec.overlapped.insert", bvec_lap[0]);
  rr.timer.add("bvec.overlapped.finalize", bvec_lap[1]);
  if (bvec_err) std::rethrow_exception(bvec_err);
  mc_classifier cls = tr.classifier();
  check(mc_set_classifier(ctx, &cls), "mc_set_classifier");
  ClusterConfig cc;
  cc.sim = opt.similarity;
  cc.iterations = opt.iterations;
  cc.delta = opt.delta;
  cc.verbose = verbose;
  cc.align = opt.align;
  cc.width = rr.width;
  cc.comm = comm;
  rr.part = mean_shift_cluster(ds, ctx, *bvp, cc, rr.timer, rr.stats);
  rr.stats.nw_pairs = tr.nw_pairs;
  rr.stats.nw_cells = tr.nw_cells;
  rr.timer.add("total_pipeline",
               std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  return rr;
}

std::string stats_json(const RunResult &rr, double parse_ms, double write_ms) {
  char b[512];
  std::string o;
  snprintf(b, sizeof b, "{\"n\": %zu, \"k\": %d, \"width\": %d, \"clusters\": %zu, \"parse_ms\": %.3f, \"write_ms\": %.3f",
           rr.n, rr.k, rr.width, rr.part.size(), parse_ms, write_ms);
  o += b;
  snprintf(b, sizeof b,
           ", \"scan_steps\": %llu, \"scan_candidates\": %llu, \"update_evals\": %llu, \"merge_evals\": %llu"
           ", \"nw_pairs\": %llu, \"nw_cells\": %llu, \"align_nw_pairs\": %llu, \"align_nw_cells\": %llu",
           (unsigned long long)rr.stats.scan_steps, (unsigned long long)rr.stats.scan_candidates,
           (unsigned long long)rr.stats.update_evals, (unsigned long long)rr.stats.merge_evals,
           (unsigned long long)rr.stats.nw_pairs, (unsigned long long)rr.stats.nw_cells,
           (unsigned long long)rr.stats.align_nw_pairs, (unsigned long long)rr.stats.align_nw_cells);
  o += b;
  o += ", \"accum_path\": \"" + rr.stats.accum_path + "\"";
  if (!rr.stats.update_path.empty()) o += ", \"update_path\": \"" + rr.stats.update_path + "\"";
  o += ", \"update_iters_fixed\": " + std::to_string(rr.stats.update_iters_fixed);
  o += ", \"update_evals_run\": " + std::to_string(rr.stats.update_evals_run);
  o += ", \"phases_ms\": {";
  for (size_t i = 0; i < rr.timer.order.size(); i++) {
    snprintf(b, sizeof b, "%s\"%s\": %.3f", i ? ", " : "", rr.timer.order[i].c_str(), rr.timer.ms.at(rr.timer.order[i]));
    o += b;
  }
  o += "}}";
  return o;
}

static void write_stats(const std::string &path, const RunResult &rr, double parse_ms, double write_ms) {
  FILE *f = fopen(path.c_str(), "w");
  if (!f) return;
  fprintf(f, "%s\n", stats_json(rr, parse_ms, write_ms).c_str());
  fclose(f);
}

// --devices: one host thread per GPU, each with its own context, sharing one clustering
// (cluster.cpp: the device-sharded accumulation whose kernels exchange through the mailbox,
// the centre all-gather per mean-shift iteration).  The ranks are threads of this process, so
// their host-side all-gathers are a shared buffer and a condition variable; the first thread
// that fails aborts the exchange, and every thread waiting in it returns an error.
struct ThreadComm {
  int world;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<uint8_t> buf;
  uint64_t bytes = 0, gen = 0;
  int arrived = 0, left = 0;
  bool draining = false, aborted = false;

  explicit ThreadComm(int w) : world(w) {}
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
  }
  int allgather(int rank, const void *in, uint64_t n, void *out) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return aborted || !draining; });  // the previous round fully copied out
    if (aborted) return 1;
    if (arrived == 0) {
      bytes = n;
      buf.resize(n * world);
    }
    if (n != bytes) {  // ranks disagree on the block size: a driver bug, stop every rank
      aborted = true;
      cv.notify_all();
      return 1;
    }
    if (n) memcpy(buf.data() + (size_t)rank * n, in, n);
    const uint64_t g = gen;
    if (++arrived == world) {
      arrived = 0;
      gen++;
      draining = true;
      left = world;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return aborted || gen != g; });
      if (aborted) return 1;
    }
    if (n) memcpy(out, buf.data(), n * world);
    if (--left == 0) {
      draining = false;
      cv.notify_all();
    }
    return 0;
  }
};

struct ThreadRank {
  ThreadComm *tc;
  int rank;
};

static int allgather_threads(void *user, const void *in, uint64_t bytes, void *out) {
  auto *r = (ThreadRank *)user;
  return r->tc->allgather(r->rank, in, bytes, out);
}

static RunResult run_multi_gpu(const Dataset &ds, const Options &opt) {
  const int W = (int)opt.devices.size();
  ThreadComm tc(W);
  std::atomic<int> first{-1}, first_peer{-1};  // the first own failure; the first peer-reported one
  std::vector<ThreadRank> tr(W);
  std::vector<RunResult> res(W);
  std::vector<std::exception_ptr> err(W);
  std::vector<std::thread> th;
  for (int r = 0; r < W; r++)
    th.emplace_back([&, r]() {
      mc_ctx *ctx = nullptr;
      try {
        check(mc_ctx_create(opt.devices[r], &ctx), "mc_ctx_create");
        tr[r] = ThreadRank{&tc, r};
        ShardComm sc;
        sc.rank = r;
        sc.world = W;
        sc.allgather = allgather_threads;
        sc.user = &tr[r];
        Options o = opt;
        o.quiet = opt.quiet || r != 0;
        res[r] = run_pipeline(ds, ctx, o, true, &sc);
      } catch (...) {
        err[r] = std::current_exception();
        bool peer = false;
        try {
          std::rethrow_exception(err[r]);
        } catch (const PeerError &) {
          peer = true;
        } catch (...) {
        }
        int none = -1;
        (peer ? first_peer : first).compare_exchange_strong(none, r);  // the root cause, not the aborted exchanges
        tc.abort();
      }
      if (ctx) mc_ctx_destroy(ctx);
    });
  for (auto &t : th) t.join();
  if (first >= 0) std::rethrow_exception(err[first]);
  if (first_peer >= 0) std::rethrow_exception(err[first_peer]);
  return std::move(res[0]);
}

int meshclust_main(int argc, char **argv) {
  tune_host_heap();
  Options opt;
  try {
    opt = parse_options(argc, argv);
  } catch (const OptionError &e) {
    if (e.usage) usage(argv[0]);
    else fprintf(stderr, "%s\n", e.what());
    return e.code;
  }
  int threads = opt.threads;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
  threads = omp_get_max_threads();
#endif
  mc_ctx *ctx = nullptr;
  try {
    for (const auto &f : opt.files)
      if (access(f.c_str(), F_OK) == -1) {
        fprintf(stderr, "File \"%s\" does not exist\n", f.c_str());
        exit(1);
      }
    auto t0 = std::chrono::steady_clock::now();
    Dataset ds;
    parse_fasta_files(opt.files, ds, threads);
    double parse_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    RunResult rr;
    if (opt.devices.size() > 1) {
      rr = run_multi_gpu(ds, opt);
    } else {
      check(mc_ctx_create(opt.devices.empty() ? opt.device : opt.devices[0], &ctx), "mc_ctx_create");
      rr = run_pipeline(ds, ctx, opt);
    }
    auto t1 = std::chrono::steady_clock::now();
    if (!opt.quiet) printf("Printing output\n");
    write_clstr(opt.output, ds, rr.part, threads);
    double write_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    if (!opt.stats_json.empty()) write_stats(opt.stats_json, rr, parse_ms, write_ms);
    mc_ctx_destroy(ctx);
    return 0;
  } catch (const Error &e) {
    if (e.code != 0) fprintf(stderr, "meshclust: %s\n", e.what());
    if (ctx) mc_ctx_destroy(ctx);
    return e.code;
  } catch (const std::exception &e) {
    fprintf(stderr, "meshclust: %s\n", e.what());
    if (ctx) mc_ctx_destroy(ctx);
    return 1;
  }
}

}  // namespace mc
