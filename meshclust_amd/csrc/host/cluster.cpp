// cluster.cpp -- see cluster.hpp.
#include "cluster.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>

#include <algorithm>
#include <cerrno>
#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>

namespace mc {

void fault_point(const ShardComm *comm, const char *stage) {
  const char *f = getenv("MC_FAULT");
  if (!f || !comm) return;
  const char *colon = strchr(f, ':');
  if (colon && atoi(f) == comm->rank && strcmp(colon + 1, stage) == 0)
    throw Error(std::string("injected fault (MC_FAULT) at ") + stage + " on rank " + std::to_string(comm->rank), 1);
}

namespace {

// Replay of Feature::align's memo table (Feature.cpp:221-243) for alignment mode.
//
// The reference memoises every identity by the unordered id pair, keeping the orientation of
// the first call.  Centres of `part` are Center clones, and DivergencePoint::clone
// (DivergencePoint.h:37-43) copies histogram, header, id and length but not the data string,
// so after accumulation every align() against a centre aligns against "" unless the pair is
// already memoised.  GlobAlignE(x, "") ends in its boundary column: identity 0/|x| (0, or NaN
// for two empty strings; GlobAlignE.cpp:148-160, 278-291) -- never similar for any --id in
// (0, 1).  Hence, after accumulation, a pair is similar only if accumulation memoised it:
//   (m, c) was aligned in accumulation  <=>  some get_close step t had centre c, m alive and
//   m's static position inside the step's window [S_t, E_t]   (or the same with m, c swapped).
// Both cannot hold: a centre is never alive again, so the orientation is unique, and a
// recurring pair recurs in the same orientation (identical value).  The memo is therefore
// reconstructed from the step windows and each point's removal time instead of storing
// every accumulation pair; identities are recomputed on the device on first use.
class AlignMemo {
 public:
  AlignMemo(size_t n, const BVec &bv) : kill_(n, NEVER), bv_(bv) {}
  // get_close step #steps_ starts: centre c over static window [S, E]
  void begin_step(uint32_t c, uint64_t S, uint64_t E) {
    win_.push_back({S, E});
    by_centre_[c].push_back(steps_);
    steps_++;
  }
  // point removed from the bvec now: alive for steps < steps_ (flagged ones were scanned in
  // the step that just ran, pops/erases happen between steps)
  void removed(uint32_t id) {
    if (kill_[id] == NEVER) kill_[id] = steps_;
  }
  // 1: memoised as align(m, c); 2: as align(c, m); 0: not memoised in accumulation
  int orient(uint32_t m, uint32_t c) const {
    if (scanned(m, c)) return 1;
    if (scanned(c, m)) return 2;
    return 0;
  }
  static uint64_t key(uint32_t a, uint32_t b) {
    return a < b ? ((uint64_t)a << 32) | b : ((uint64_t)b << 32) | a;
  }
  std::unordered_map<uint64_t, double> ident;  // identities computed so far (device NW)

 private:
  bool scanned(uint32_t cand, uint32_t centre) const {
    auto it = by_centre_.find(centre);
    if (it == by_centre_.end()) return false;
    const uint64_t sp = bv_.spos(cand);
    for (uint32_t t : it->second)
      if (kill_[cand] > t && win_[t].first <= sp && sp <= win_[t].second) return true;
    return false;
  }
  static constexpr uint32_t NEVER = 0xffffffffu;
  std::vector<uint32_t> kill_;
  std::vector<std::pair<uint64_t, uint64_t>> win_;
  std::unordered_map<uint32_t, std::vector<uint32_t>> by_centre_;
  uint32_t steps_ = 0;
  const BVec &bv_;
};

// Identities of the memoised pairs among (a[i], b[i]) in their memo orientation; computes the
// missing ones in one device NW batch.  val[i] = identity, hit[i] = memoised.
void memo_lookup(AlignMemo &memo, mc_ctx *ctx, const Dataset &ds, const std::vector<uint32_t> &a,
                 const std::vector<uint32_t> &b, std::vector<double> &val, std::vector<uint8_t> &hit,
                 ClusterStats &stats) {
  const size_t m = a.size();
  val.assign(m, 0.0);
  hit.assign(m, 0);
  std::vector<uint32_t> na, nb;
  std::vector<uint64_t> nkey;
  std::unordered_map<uint64_t, size_t> pending;
  std::vector<int> orient(m);
  for (size_t i = 0; i < m; i++) {
    const int o = memo.orient(a[i], b[i]);
    orient[i] = o;
    if (!o) continue;
    hit[i] = 1;
    const uint64_t k = AlignMemo::key(a[i], b[i]);
    if (memo.ident.count(k) || pending.count(k)) continue;
    pending[k] = na.size();
    na.push_back(o == 1 ? a[i] : b[i]);
    nb.push_back(o == 1 ? b[i] : a[i]);
    nkey.push_back(k);
  }
  if (!na.empty()) {
    std::vector<double> id(na.size());
    check(mc_nw_identity(ctx, na.data(), nb.data(), na.size(), id.data(), nullptr, nullptr), "mc_nw_identity");
    for (size_t q = 0; q < na.size(); q++) {
      memo.ident[nkey[q]] = id[q];
      stats.align_nw_pairs++;
      stats.align_nw_cells += ds.lengths[na[q]] * ds.lengths[nb[q]];
    }
  }
  for (size_t i = 0; i < m; i++)
    if (hit[i]) val[i] = memo.ident.at(AlignMemo::key(a[i], b[i]));
}

// One get_close step sharded by record over the ranks of `comm`: every rank
// scans its static blocks of the window (mc_scan_part), the ranks all-gather their partial
// results -- {first max of combo 0, is_min, flagged positions} -- and combine them exactly as
// the serial loop of Trainer::get_close would (Trainer.cpp:34-114: is_min is the AND over all
// candidates; the result is the FIRST maximum in bvec order, i.e. the largest value with ties
// to the lowest static position), then every rank applies remove_available + get_mean to the
// union (mc_scan_commit).  One exchange of a fixed 1 KiB block per rank per step; a second
// one only when some rank flagged more than kInline candidates.
struct ShardBlock {
  static constexpr uint32_t kInline = 248;
  double best_val;
  uint64_t best_pos;
  uint32_t has_best, is_min, n_flagged, failed;
  uint32_t flagged[kInline];
};
static_assert(sizeof(ShardBlock) == 1024, "exchange block");

void sharded_step(mc_ctx *ctx, const ShardComm &comm, uint32_t centre, uint64_t S, uint64_t E,
                  std::vector<uint32_t> &flag_buf, std::vector<uint32_t> &all_flagged, mc_scan_result *res,
                  PhaseTimer &timer) {
  mc_scan_result loc{};
  // A rank whose scan fails still takes part in the exchange, with its block marked failed, so
  // every rank throws after the same all-gather instead of its peers waiting in it forever.
  std::string scan_err;
  {
    Scope sc(timer, "accumulate.scan_part");
    try {
      check(mc_scan_part(ctx, centre, S, E, (uint32_t)comm.rank, (uint32_t)comm.world, flag_buf.data(),
                         flag_buf.size(), &loc),
            "mc_scan_part");
    } catch (const std::exception &e) {
      scan_err = e.what();
      loc = mc_scan_result{};
    }
  }
  Scope sx(timer, "accumulate.exchange");
  const int W = comm.world;
  ShardBlock mine;
  memset(&mine, 0, sizeof mine);
  mine.failed = scan_err.empty() ? 0 : 1;
  mine.best_val = loc.best_val;
  mine.best_pos = loc.best_pos;
  mine.has_best = loc.has_best ? 1 : 0;
  mine.is_min = loc.is_min ? 1 : 0;
  mine.n_flagged = (uint32_t)loc.n_flagged;
  memcpy(mine.flagged, flag_buf.data(), std::min<uint64_t>(loc.n_flagged, ShardBlock::kInline) * 4);
  std::vector<ShardBlock> all(W);
  if (comm.allgather(comm.user, &mine, sizeof mine, all.data()) != 0) {
    // (a peer that saw this rank's failure may end the exchange first: the cause is ours)
    if (!scan_err.empty()) throw Error(scan_err, 1);
    throw PeerError("get_close all-gather across ranks failed");
  }
  for (int r = 0; r < W; r++)
    if (all[r].failed) {
      if (scan_err.empty()) throw PeerError("get_close failed on rank " + std::to_string(r));
      throw Error(scan_err, 1);
    }
  memset(res, 0, sizeof *res);
  res->is_min = 1;
  res->best_val = -1.0;
  uint64_t total = 0, most = 0;
  for (const auto &b : all) {
    res->is_min &= (int32_t)b.is_min;
    if (b.has_best && (!res->has_best || b.best_val > res->best_val ||
                       (b.best_val == res->best_val && b.best_pos < res->best_pos))) {
      res->has_best = 1;
      res->best_val = b.best_val;
      res->best_pos = b.best_pos;
    }
    total += b.n_flagged;
    most = std::max<uint64_t>(most, b.n_flagged);
  }
  all_flagged.clear();
  if (most > ShardBlock::kInline) {  // long lists: one more all-gather of every full list
    std::vector<uint32_t> big(most, 0), gathered(most * W);
    std::copy(flag_buf.begin(), flag_buf.begin() + loc.n_flagged, big.begin());
    if (comm.allgather(comm.user, big.data(), most * 4, gathered.data()) != 0)
      throw PeerError("get_close all-gather across ranks failed");
    for (int r = 0; r < W; r++)
      all_flagged.insert(all_flagged.end(), gathered.begin() + most * r, gathered.begin() + most * r + all[r].n_flagged);
  } else {
    for (const auto &b : all) all_flagged.insert(all_flagged.end(), b.flagged, b.flagged + b.n_flagged);
  }
  std::sort(all_flagged.begin(), all_flagged.end());  // each part is ascending; blocks interleave
  if (all_flagged.size() != total || (total == 0) != (res->is_min != 0))
    throw Error("inconsistent sharded get_close results", 1);
  res->n_flagged = total;
}

// The ranks' step mailbox for the device-sharded accumulation (mc_set_mailbox): a POSIX
// shared-memory segment that rank 0 creates and every rank maps (one process per GPU, or the
// threads of one process), registered with each rank's context.  Collective over `comm`;
// every rank learns whether all of them attached, so they all take the same path.
struct SharedMailbox {
  void *p = nullptr;
  size_t bytes = 0;
  mc_ctx *ctx = nullptr;
  ~SharedMailbox() {
    if (ctx) mc_set_mailbox(ctx, nullptr, 0, 0, 0, 1);
    if (p) munmap(p, bytes);
  }
};

static bool attach_mailbox(const ShardComm &comm, mc_ctx *ctx, uint64_t n, uint32_t nbins, SharedMailbox &mb,
                           bool failed_before) {
  struct Blk {
    char name[52];
    int32_t failed;  // this rank's process once saw the mailbox hand-offs time out
    int32_t ok;
    uint32_t grid;  // this rank's accumulation grid (then: its plan's tile of ownership)
    char pci[64];   // this rank's GPU: ranks on one GPU split its CUs
  };
  static_assert(sizeof(Blk) == 128, "mailbox exchange block");
  const int W = comm.world;
  const size_t bytes = mc_mailbox_bytes(W, n);
  Blk mine{};
  mine.failed = failed_before ? 1 : 0;
  if (mc_ctx_pci_bus_id(ctx, mine.pci, sizeof mine.pci) != MC_OK) mine.pci[0] = 0;
  int fd = -1;
  if (comm.rank == 0) {
    snprintf(mine.name, sizeof mine.name, "/mcl_mbox_%d_%llx", (int)getpid(),
             (unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count());
    fd = shm_open(mine.name, O_CREAT | O_EXCL | O_RDWR, 0600);
    mine.ok = fd >= 0 && ftruncate(fd, (off_t)bytes) == 0;  // (zero-filled: no granule carries a tag)
  }
  std::vector<Blk> all(W);
  if (comm.allgather(comm.user, &mine, sizeof mine, all.data()) != 0)
    throw PeerError("mailbox all-gather across ranks failed");
  bool ok = all[0].ok != 0;
  for (const auto &b : all) ok &= b.failed == 0;  // (any rank's earlier timeout: none of them tries)
  if (ok && comm.rank != 0) fd = shm_open(all[0].name, O_RDWR, 0600);
  if (ok && fd >= 0) {
    void *p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (p != MAP_FAILED) {
      mb.p = p;
      mb.bytes = bytes;
    }
  }
  if (fd >= 0) close(fd);
  int share = 0;
  for (const auto &b : all) share += strncmp(b.pci, mine.pci, sizeof mine.pci) == 0;
  uint32_t info[4] = {0, 0, 0, 0};
  // (mb.ctx: the mailbox is registered with this context, whatever the plan says -- every exit
  // below that does not use it detaches it before the segment is unmapped)
  bool plan = false;
  if (ok && mb.p && mc_set_mailbox(ctx, mb.p, bytes, comm.rank, W, std::max(share, 1)) == MC_OK) {
    mb.ctx = ctx;
    plan = mc_accum_plan_info(ctx, nbins, info) == MC_OK;
  }
  mine.ok = plan;
  mine.grid = info[0];
  if (comm.allgather(comm.user, &mine, sizeof mine, all.data()) != 0)
    throw PeerError("mailbox all-gather across ranks failed");
  if (comm.rank == 0 && all[0].name[0]) shm_unlink(all[0].name);  // every rank has mapped it (or failed)
  for (const auto &b : all) ok &= b.ok != 0;
  // Tile t of the static order belongs to rank t mod W, so every rank must deal tiles of the
  // same size -- which the plan derives from the grid (the dense form needs a worker's share
  // to fit one workgroup).  Every rank takes the smallest grid among the ranks, and the ranks
  // compare the resulting tiles; any disagreement (e.g. an MC_ACCUM_* override on one rank
  // only) sends all of them to the host-driven sharded steps.
  if (ok) {
    uint32_t gmin = ~0u;
    for (const auto &b : all) gmin = std::min(gmin, b.grid);
    // every device buffer of the accumulation is allocated before this all-gather, so no rank
    // frees memory (hipFree waits for the whole device) once any rank's persistent kernel spins
    // on the mailbox: the ranks of one process share the device
    mine.grid = (mc_set_accum_grid(ctx, gmin) == MC_OK && mc_accum_plan_info(ctx, nbins, info) == MC_OK &&
                 mc_accum_reserve(ctx, nbins) == MC_OK)
                    ? info[1]
                    : 0;
    if (comm.allgather(comm.user, &mine, sizeof mine, all.data()) != 0)
      throw PeerError("mailbox all-gather across ranks failed");
    for (const auto &b : all) ok &= b.grid != 0 && b.grid == all[0].grid;
  }
  if (!ok && mb.ctx) {
    mc_set_mailbox(ctx, nullptr, 0, 0, 0, 1);
    mb.ctx = nullptr;
  }
  return ok;
}

// Alignment mode, one get_close step with its NW alignments split over the ranks: rank r aligns
// every W-th alive candidate of the window (mc_align_part), the ranks all-gather the identities
// and every rank finishes the step on the whole identity vector (mc_scan_ident) -- the same
// flags, removals and next centre everywhere, with no other exchange.  (A window of config C
// at 100k holds nearly every alive read: ~10^11 NW cells per step against ~0.8 MB of identities.)
static void align_sharded_step(mc_ctx *ctx, const ShardComm &comm, uint32_t centre, uint64_t S, uint64_t E,
                               std::vector<uint32_t> &flag_buf, mc_scan_result *res, PhaseTimer &timer,
                               ClusterStats &stats) {
  const uint64_t W = (uint64_t)comm.world, blk = (E - S + 1 + W - 1) / W;  // (a bound on any part's count)
  std::vector<double> mine(blk + 1, 0.0), all((blk + 1) * W);
  uint64_t np = 0, pairs = 0, cells = 0;
  // A rank whose NW part fails (an MC_ERR_TIMEOUT of the chained blocks, an allocation, a HIP
  // error) still joins the all-gather with its count word set to kFailed, so every rank stops
  // after the same exchange (as sharded_step) instead of its peers waiting in it.
  constexpr uint64_t kFailed = ~0ull;
  std::string part_err;
  {
    Scope s(timer, "accumulate.align_part");
    try {
      fault_point(&comm, "align_part");
      check(mc_align_part(ctx, centre, S, E, (uint32_t)comm.rank, (uint32_t)W, mine.data() + 1, blk, &np, &pairs,
                          &cells),
            "mc_align_part");
    } catch (const std::exception &e) {
      part_err = e.what();
      np = kFailed;
    }
  }
  memcpy(mine.data(), &np, 8);
  if (comm.allgather(comm.user, mine.data(), mine.size() * 8, all.data()) != 0) {
    if (!part_err.empty()) throw Error(part_err, 1);
    throw PeerError("identity all-gather across ranks failed");
  }
  for (uint64_t r = 0; r < W; r++) {
    uint64_t nr = 0;
    memcpy(&nr, all.data() + r * (blk + 1), 8);
    if (nr == kFailed) {
      if (part_err.empty()) throw PeerError("alignment part failed on rank " + std::to_string(r));
      throw Error(part_err, 1);
    }
  }
  std::vector<double> ident(pairs);
  for (uint64_t r = 0; r < W; r++) {
    uint64_t nr = 0;
    memcpy(&nr, all.data() + r * (blk + 1), 8);
    if (nr != (pairs + W - 1 - r) / W) throw PeerError("alignment shard: the ranks' windows differ");
    for (uint64_t j = 0; j < nr; j++) ident[j * W + r] = all[r * (blk + 1) + 1 + j];
  }
  Scope sc(timer, "accumulate.mc_scan");
  check(mc_scan_ident(ctx, centre, S, E, ident.data(), flag_buf.data(), flag_buf.size(), res), "mc_scan_ident");
  stats.align_nw_pairs += pairs;
  stats.align_nw_cells += cells;
}

// accumulate (ClusterFactory.cpp:637-714): grow one cluster around `last` until get_close
// finds no similar candidate; returns the next seed through *last_ptr.  With `shard`, every
// get_close step is split over the ranks (sharded_step).
void accumulate(uint32_t *last_ptr, const Dataset &ds, mc_ctx *ctx, BVec &bv, std::vector<Center> &centers,
                const ClusterConfig &cfg, ClusterStats &stats, std::vector<uint32_t> &flag_buf, PhaseTimer &timer,
                AlignMemo *memo, const ShardComm *shard, std::vector<uint32_t> &all_flagged,
                const ShardComm *ashard) {
  uint32_t last = *last_ptr;
  std::vector<uint32_t> current = {last};
  check(mc_cluster_begin(ctx, last), "mc_cluster_begin");
  bool is_min = false;
  const auto &order = bv.static_order();
  while (!is_min) {
    uint64_t len = ds.lengths[last];
    std::pair<BIdx, BIdx> bounds;
    uint64_t S = 0, E = 0;
    int64_t count;
    {
      Scope sr(timer, "accumulate.window");
      bounds = bv.get_range((uint64_t)(len * cfg.sim), (uint64_t)(len / cfg.sim));
      count = bv.window(bounds.first, bounds.second, &S, &E);
    }
    mc_scan_result res{};
    if (count > 0) {
      stats.scan_steps++;
      stats.scan_candidates += (uint64_t)count;
      if (memo) memo->begin_step(last, S, E);
      if (shard) {
        sharded_step(ctx, *shard, last, S, E, flag_buf, all_flagged, &res, timer);
      } else if (ashard) {
        align_sharded_step(ctx, *ashard, last, S, E, flag_buf, &res, timer, stats);
      } else {
        Scope sc(timer, "accumulate.mc_scan");
        check(mc_scan(ctx, last, S, E, flag_buf.data(), flag_buf.size(), &res), "mc_scan");
        stats.align_nw_pairs += res.nw_pairs;
        stats.align_nw_cells += res.nw_cells;
      }
    } else {  // the OpenMP loop runs no iteration: result NULL, is_min stays true
      res.is_min = 1;
      res.has_best = 0;
    }
    is_min = res.is_min != 0;
    if (is_min) {
      if (!res.has_best) {
        uint32_t p = bv.pop();
        if (p != BVec::NONE) {
          check(mc_kill(ctx, bv.spos(p)), "mc_kill");
          if (memo) memo->removed(p);
        }
        *last_ptr = p;
      } else {
        auto rc = bv.locate(res.best_pos);
        *last_ptr = order[res.best_pos];
        bv.erase(rc.first, rc.second);
        check(mc_kill(ctx, res.best_pos), "mc_kill");
        if (memo) memo->removed(order[res.best_pos]);
      }
    } else {
      if (shard) {
        mc_scan_result cr{};
        {
          Scope sc(timer, "accumulate.commit");
          check(mc_scan_commit(ctx, all_flagged.data(), all_flagged.size(), &cr), "mc_scan_commit");
        }
        res.new_centre = cr.new_centre;
      }
      Scope sr(timer, "accumulate.remove");
      std::vector<uint32_t> flagged = shard ? all_flagged
                                            : std::vector<uint32_t>(flag_buf.begin(), flag_buf.begin() + res.n_flagged);
      if (memo)
        for (uint32_t pos : flagged) memo->removed(order[pos]);
      bv.remove_positions(flagged, bounds.first.first, bounds.second.first, current);
      last = res.new_centre;
    }
  }
  centers.push_back(Center{last, std::move(current), false});
}

// merge's cascade (ClusterFactory.cpp:427-493 + Trainer::merge, Trainer.cpp:129-157).
// Merging only moves member lists, never centres, so every (candidate, current) centre pair is
// classified in one batch first; sim/c0 are indexed like pa/pb (poff per current centre).
void merge_cascade(std::vector<Center> &part, const std::vector<uint64_t> &poff, const std::vector<uint8_t> &sim,
                   const std::vector<double> &c0) {
  const uint32_t C = (uint32_t)part.size();
  for (uint32_t i = 0; i < C; i++) {
    long best_i = 0;
    double best_v = DBL_MIN;  // std::numeric_limits<double>::min()
    for (uint64_t q = poff[i]; q < poff[i + 1]; q++) {
      if (sim[q]) {
        long t = (long)i + 1 + (long)(q - poff[i]);
        if (!(best_v > c0[q])) {  // best = best.second > dist ? best : (i, dist): last max wins
          best_i = t;
          best_v = c0[q];
        }
      }
    }
    if (best_i > (long)i) {
      auto &to_add = part[best_i].points;
      auto &to_del = part[i].points;
      to_add.insert(to_add.end(), to_del.begin(), to_del.end());
      part[i].del = true;
    }
  }
  part.erase(std::remove_if(part.begin(), part.end(), [](const Center &c) { return c.del; }), part.end());
}

}  // namespace

std::vector<Center> mean_shift_cluster(const Dataset &ds, mc_ctx *ctx, BVec &bv, const ClusterConfig &cfg,
                                       PhaseTimer &timer, ClusterStats &stats) {
  std::vector<Center> part;
  const auto &order = bv.static_order();
  check(mc_set_order(ctx, order.data(), order.size()), "mc_set_order");
  std::vector<uint32_t> flag_buf(order.size() + 1), all_flagged;
  std::unique_ptr<AlignMemo> memo;
  if (cfg.align) memo.reset(new AlignMemo(ds.size(), bv));
  // Record-sharded accumulation (every get_close step split over the ranks) when several ranks
  // share the clustering and the device takes sharded steps (8/16-bit k-mer histograms);
  // otherwise each rank runs the whole chain (identical on every rank).
  // MC_SHARD_FORCE=1 (tests) takes the sharded code path with a single rank too.
  const bool multi = cfg.comm && (cfg.comm->world > 1 || getenv("MC_SHARD_FORCE"));
  const ShardComm *shard = (multi && !memo && cfg.width <= 2 && !getenv("MC_SHARD_REPLICATE")) ? cfg.comm : nullptr;
  // Alignment mode: every step's NW alignments (the whole cost of config C) split over the ranks
  // (align_sharded_step); MC_ALIGN_REPLICATE=1 keeps every rank aligning every window itself.
  const ShardComm *ashard = (multi && memo && !getenv("MC_ALIGN_REPLICATE")) ? cfg.comm : nullptr;
  // The accumulation is split over the ranks only when one GPU would stream its rows from HBM
  // (more reads than the dense resident form holds in the workers' LDS: ~130k on 256 CUs).
  // Below that a get_close step is bound by its latency chain -- hand-offs, fan-in, collect --
  // not by the scan the ranks would split, and the per-step mailbox exchange between GPUs would
  // lengthen the chain: every rank then runs the whole (identical) chain itself, while the
  // training and the mean-shift iterations stay sharded.  MC_SHARD_ACCUM=1 shards at any size
  // (tests); the ranks take the same decision (one all-gather).
  const char *force_acc = getenv("MC_SHARD_ACCUM");
  if (shard && cfg.comm->world > 1 && !(force_acc && *force_acc && strcmp(force_acc, "0") != 0) && !getenv("MC_SHARD_FORCE")) {
    uint32_t info[4] = {0, 0, 0, 0};
    const int32_t fits = mc_accum_plan_info(ctx, (uint32_t)bv.bins().size(), info) == MC_OK && (info[2] & 1u) ? 1 : 0;
    std::vector<int32_t> all(cfg.comm->world);
    if (cfg.comm->allgather(cfg.comm->user, &fits, sizeof fits, all.data()) != 0)
      throw PeerError("all-gather across ranks failed");
    bool every = true;
    for (int32_t f : all) every &= f != 0;
    if (every) shard = nullptr;
  }
  // Sharded ranks run ONE device-resident loop together: every rank's persistent kernel
  // scans its tiles and the kernels exchange each step through the shared mailbox
  // (mc_set_mailbox); MC_SHARD_HOST_STEPS=1, or a mailbox that cannot be attached on every
  // rank, keeps the host-driven sharded steps (mc_scan_part + all-gather + mc_scan_commit).
  comm_phase(cfg.comm, "accumulate");
  fault_point(cfg.comm, "accumulate");
  SharedMailbox mbox;
  // (a mailbox whose hand-offs once timed out in this process is not tried again: every later
  // clustering goes to the host-driven sharded steps -- the ranks agree on it in
  // attach_mailbox's first all-gather, so a group whose ranks have different histories agrees)
  static std::atomic<bool> mailbox_failed{false};
  const bool dev_shard = shard && !getenv("MC_SHARD_HOST_STEPS") && !getenv("MC_ACCUM_STEPS") &&
                         attach_mailbox(*shard, ctx, order.size(), (uint32_t)bv.bins().size(), mbox, mailbox_failed.load());
  // The device-resident loop (mc_accumulate) unless alignment mode or the configuration
  // asks for the step API; MC_ACCUM_STEPS=1 forces the host-driven loop (both are GPU paths).
  bool done = false;
  if (shard && !dev_shard) {
    stats.accum_path = "sharded steps x" + std::to_string(shard->world);
  } else if (!memo && !getenv("MC_ACCUM_STEPS")) {
    Scope s(timer, "accumulate");
    const auto &bins = bv.bins();
    std::vector<uint32_t> bin_lo(bins.size() + 1, 0);
    for (size_t b = 0; b < bins.size(); b++) bin_lo[b + 1] = bin_lo[b] + (uint32_t)bins[b].size();
    const size_t n = order.size();
    std::vector<uint32_t> centres(n), ids(n);
    std::vector<uint64_t> moff(n + 1);
    uint64_t ncl = 0, st[5] = {0, 0, 0, 0, 0};
    int rc = mc_accumulate(ctx, bin_lo.data(), bv.begin_bounds().data(), (uint32_t)bins.size(), cfg.sim,
                           centres.data(), moff.data(), ids.data(), &ncl, st);
    std::string mbox_note;
    if (dev_shard) {
      // every rank learns every rank's outcome: a mailbox the ranks' GPUs could not all see
      // (each kernel's hand-off deadline expired: MC_ERR_TIMEOUT) sends all of them to the
      // host-driven sharded steps together; any other failure stops all of them, with this
      // rank's own message where it failed itself
      const std::string own = rc == MC_OK ? std::string() : std::string(mc_last_error());
      int32_t mine[2] = {rc, 0}, all[2 * 64];
      if (shard->allgather(shard->user, mine, sizeof mine, all) != 0) throw PeerError("all-gather across ranks failed");
      int worst = MC_OK;  // MC_OK < timeouts / unsupported (fall back) < anything else (stop)
      for (int r = 0; r < shard->world; r++) {
        const int e = all[2 * r];
        if (e == MC_OK) continue;
        if (e == MC_ERR_TIMEOUT || e == MC_ERR_UNSUPPORTED) {
          if (worst == MC_OK || (worst == MC_ERR_UNSUPPORTED && e == MC_ERR_TIMEOUT)) worst = e;
        } else {
          worst = e;
          break;
        }
      }
      if (worst == MC_ERR_TIMEOUT) {
        fprintf(stderr, "meshclust: device-sharded accumulation: the ranks' mailbox hand-offs timed out; "
                        "taking the host-driven sharded steps\n");
        mbox_note = " (mailbox timed out)";
        mailbox_failed.store(true);
        rc = MC_ERR_UNSUPPORTED;
      } else if (worst != MC_OK && worst != MC_ERR_UNSUPPORTED) {
        // a real failure somewhere: this rank's own error goes to check() below with its message
        if (rc == MC_OK || rc == MC_ERR_TIMEOUT || rc == MC_ERR_UNSUPPORTED)
          throw PeerError("device-sharded accumulation failed on another rank" + (own.empty() ? "" : " (here: " + own + ")"));
      } else {
        rc = worst;
      }
    }
    if (rc == MC_OK) {
      for (uint64_t c = 0; c < ncl; c++)
        part.push_back(Center{centres[c], std::vector<uint32_t>(ids.begin() + moff[c], ids.begin() + moff[c + 1]), false});
      stats.scan_steps += st[0];
      stats.scan_candidates += st[1];
      timer.add("accumulate.dev_window", st[2] / 1000.0);
      timer.add("accumulate.dev_wait", st[3] / 1000.0);
      timer.add("accumulate.dev_collect", st[4] / 1000.0);
      done = true;
      stats.accum_path = dev_shard                              ? "device x" + std::to_string(shard->world)
                         : (multi && cfg.comm->world > 1) ? "device (replicated x" + std::to_string(cfg.comm->world) + ")"
                                                          : "device";
    } else if (rc == MC_ERR_TIMEOUT && !dev_shard) {
      // (a replicated or single-rank loop depends on no other rank: a hand-off deadline here
      // means this GPU did not run the persistent grid together -- the step loop is exact too)
      stats.accum_path = std::string("steps (") + mc_last_error() + ")";
      fprintf(stderr, "meshclust: device accumulation timed out; taking the host-driven get_close steps\n");
    } else if (rc != MC_ERR_UNSUPPORTED) {
      check(rc, "mc_accumulate");
    } else if (dev_shard) {  // (every rank: the same configuration) -> the host-driven sharded steps
      stats.accum_path = "sharded steps x" + std::to_string(shard->world) + mbox_note;
    } else {
      // both loops are GPU paths and give identical partitions; say which one ran
      stats.accum_path = std::string("steps (") + mc_last_error() + ")";
      if (cfg.verbose) fprintf(stderr, "accumulation: host-driven get_close steps: %s\n", mc_last_error());
    }
  } else {
    stats.accum_path = !memo     ? std::string("steps (MC_ACCUM_STEPS)")
                       : ashard ? "steps (alignment mode, NW sharded x" + std::to_string(ashard->world) + ")"
                                : std::string("steps (alignment mode)");
  }
  if (!done) {
    Scope s(timer, "accumulate");
    uint32_t last = bv.pop();
    if (last != BVec::NONE) {
      check(mc_kill(ctx, bv.spos(last)), "mc_kill");
      if (memo) memo->removed(last);
    }
    while (last != BVec::NONE)
      accumulate(&last, ds, ctx, bv, part, cfg, stats, flag_buf, timer, memo.get(), shard, all_flagged, ashard);
  }
  comm_phase(cfg.comm, "update");
  Scope s(timer, "update+merge");
  std::vector<uint8_t> fused_sim;
  std::vector<double> fused_c0;
  // the clusters' member lists change only when the merge pass merged something (the
  // partition shrinks): otherwise the next iteration reuses them as they are
  std::vector<uint32_t> members;
  std::vector<uint64_t> off;
  bool rebuild = true;
  // Several ranks: the iterations are split over them by centre (centre all-gather) only when
  // that pays.  Every rank runs the first iteration whole (one device round trip, identical
  // everywhere); then the ranks exchange its time and the time of one exchange, and split the
  // remaining iterations if a rank's share of an iteration saves more than the exchange and
  // the separate merge-pair call cost (MC_SHARD_UPDATE=0/1 forces the choice; MC_SHARD_FORCE,
  // the one-rank test of the sharded path, splits from the first iteration).
  int split_update = (multi && !memo) ? -1 : 0;
  if (split_update < 0 && getenv("MC_SHARD_FORCE")) split_update = 1;
  if (split_update < 0 && getenv("MC_SHARD_UPDATE")) split_update = atoi(getenv("MC_SHARD_UPDATE")) ? 1 : 0;
  bool all_iterations = getenv("MC_UPDATE_ALL_ITERATIONS") != nullptr;
  if (multi) {
    // the loop's branches that lead to an exchange (the fixed-point exit, the split decision)
    // must be the same on every rank: every rank takes rank 0's environment choices
    int32_t mine[2] = {split_update, all_iterations ? 1 : 0}, all[2 * 64];
    if (cfg.comm->world > 64 || cfg.comm->allgather(cfg.comm->user, mine, 8, all) != 0)
      throw PeerError("all-gather across ranks failed");
    split_update = all[0];
    all_iterations = all[1] != 0;
  }
  double t_first = 0;
  for (int it = 0; it < cfg.iterations; it++) {
    bool fused = false;
    uint64_t fused_np = 0;
    if (split_update < 0 && it == 1) {
      const auto t0 = std::chrono::steady_clock::now();
      double probe = 0, got[64];
      if (cfg.comm->allgather(cfg.comm->user, &probe, 8, got) != 0) throw PeerError("all-gather across ranks failed");
      const double t_ag = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      double mine2[2] = {t_first, t_ag}, all2[2 * 64];
      if (cfg.comm->allgather(cfg.comm->user, mine2, 16, all2) != 0) throw PeerError("all-gather across ranks failed");
      double it_ms = 0, ag_ms = 0;
      for (int r = 0; r < cfg.comm->world; r++) {
        it_ms = std::max(it_ms, all2[2 * r]);
        ag_ms = std::max(ag_ms, all2[2 * r + 1]);
      }
      const double W = (double)cfg.comm->world;
      split_update = it_ms * (1.0 - 1.0 / W) > 2.0 * ag_ms + 0.1 ? 1 : 0;
      timer.add("update.decision.iteration_ms", it_ms);
      timer.add("update.decision.exchange_ms", ag_ms);
    }
    if (multi && !memo && it == 0) fault_point(cfg.comm, "update");
    const auto t_it0 = std::chrono::steady_clock::now();
    // mean_shift_update for every centre, all reading the same state (ClusterFactory.cpp:744-749)
    const uint32_t C = (uint32_t)part.size();
    std::vector<uint32_t> cids(C), newc(C);
    if (rebuild) {
      members.clear();
      off.assign(C + 1, 0);
      for (uint32_t j = 0; j < C; j++) {
        members.insert(members.end(), part[j].points.begin(), part[j].points.end());
        off[j + 1] = members.size();
      }
    }
    for (uint32_t j = 0; j < C; j++) cids[j] = part[j].centre;
    uint64_t it_update_evals = 0;
    for (uint32_t j = 0; j < C; j++) {
      uint32_t b = j >= (uint32_t)cfg.delta ? j - cfg.delta : 0;
      uint32_t e = std::min<uint32_t>(j + cfg.delta, C - 1);
      it_update_evals += off[e + 1] - off[b];
    }
    stats.update_evals += it_update_evals;
    stats.update_evals_run += it_update_evals;
    if (C && !memo && multi && split_update == 1) {
      // this rank's share of the centres, then the centre-reassignment all-gather
      const uint32_t W = (uint32_t)cfg.comm->world, per = (C + W - 1) / W;
      const uint32_t j0 = std::min<uint32_t>(C, per * (uint32_t)cfg.comm->rank), j1 = std::min<uint32_t>(C, j0 + per);
      // block: [status word, this rank's `per` new centres]; a failed rank sends status 1, so
      // every rank (also one whose share is empty, C < W) stops after the same exchange
      const uint32_t blk = per + 1;
      std::vector<uint32_t> mine(blk, 0), all((size_t)blk * W, 0);
      std::string ms_err;
      try {
        fault_point(cfg.comm, "update");
        check(mc_mean_shift_range(ctx, cids.data(), C, off.data(), members.data(), cfg.delta, j0, j1, mine.data() + 1),
              "mc_mean_shift_range");
      } catch (const std::exception &e) {
        ms_err = e.what();
        mine[0] = 1;
      }
      if (cfg.comm->allgather(cfg.comm->user, mine.data(), (uint64_t)blk * 4, all.data()) != 0) {
        // (a peer that saw this rank's failure may end the exchange first: the cause is ours)
        if (!ms_err.empty()) throw Error(ms_err, 1);
        throw PeerError("centre all-gather across ranks failed");
      }
      for (uint32_t r = 0; r < W; r++)
        if (all[(size_t)r * blk]) {
          if (ms_err.empty()) throw PeerError("mean-shift update failed on rank " + std::to_string(r));
          throw Error(ms_err, 1);
        }
      for (uint32_t j = 0; j < C; j++) newc[j] = all[(size_t)(j / per) * blk + 1 + j % per];
    } else if (C && !memo) {
      // mean shift and the merge pass's classifier pairs over the new centres in one device
      // round trip (the pairs below are exactly these, in this order)
      Scope sm(timer, "update.mean_shift+merge_pairs");
      uint64_t np = 0;
      uint64_t npairs = 0;  // sum over i of min(delta, C - 1 - i)
      for (uint32_t i = 0; i < C; i++) npairs += std::min<uint64_t>((uint64_t)std::max(cfg.delta, 0), C - 1 - i);
      fused_sim.resize(npairs);
      fused_c0.resize(fused_sim.size());
      check(mc_update_iteration(ctx, cids.data(), C, off.data(), members.data(), cfg.delta, newc.data(),
                                fused_sim.data(), fused_c0.data(), &np),
            "mc_update_iteration");
      fused = true;
      fused_np = np;
    } else if (C) {
      // Trainer::filter(center clone, good): feat->compute(*member, *clone) (Trainer.cpp:334-349)
      std::vector<uint32_t> fa, fb;
      for (uint32_t j = 0; j < C; j++) {
        uint32_t b = j >= (uint32_t)cfg.delta ? j - cfg.delta : 0;
        uint32_t e = std::min<uint32_t>(j + cfg.delta, C - 1);
        for (uint64_t q = off[b]; q < off[e + 1]; q++) {
          fa.push_back(members[q]);
          fb.push_back(cids[j]);
        }
      }
      std::vector<double> val;
      std::vector<uint8_t> hit, keep(fa.size(), 0);
      memo_lookup(*memo, ctx, ds, fa, fb, val, hit, stats);
      std::vector<double> raw;
      std::vector<size_t> idx;
      for (size_t q = 0; q < fa.size(); q++)
        if (hit[q]) {
          raw.push_back(val[q]);
          idx.push_back(q);
        }
      std::vector<uint8_t> sim(raw.size());
      if (!raw.empty())
        check(mc_classify_values(ctx, raw.data(), raw.size(), sim.data(), nullptr, nullptr), "mc_classify_values");
      for (size_t r = 0; r < idx.size(); r++) keep[idx[r]] = sim[r];
      check(mc_mean_shift_select(ctx, cids.data(), C, off.data(), members.data(), cfg.delta, keep.data(), newc.data()),
            "mc_mean_shift_select");
    }
    bool moved = false;  // some centre changed in this iteration's mean shift
    for (uint32_t j = 0; j < C; j++) {
      moved |= newc[j] != part[j].centre;
      part[j].centre = newc[j];
    }
    std::vector<uint32_t> pa, pb;
    std::vector<uint64_t> poff(C + 1, 0);
    for (uint32_t i = 0; i < C; i++) {
      long last = std::min((long)C - 1, (long)i + cfg.delta);
      for (long t = (long)i + 1; t <= last; t++) {
        pa.push_back(part[t].centre);  // feat->compute(*cen, *p): candidate first
        pb.push_back(part[i].centre);
      }
      poff[i + 1] = pa.size();
    }
    stats.merge_evals += pa.size();
    std::vector<uint8_t> sim(pa.size(), 0);
    std::vector<double> c0(pa.size(), 0.0);
    if (fused) {
      if (fused_np != pa.size()) throw Error("mc_update_iteration: merge pair count mismatch", 1);
      std::copy(fused_sim.begin(), fused_sim.begin() + pa.size(), sim.begin());
      std::copy(fused_c0.begin(), fused_c0.begin() + pa.size(), c0.begin());
    } else if (!pa.empty() && !memo) {
      Scope sm(timer, "update.merge_pairs");
      check(mc_classify_pairs(ctx, pa.data(), pb.data(), pa.size(), sim.data(), c0.data(), nullptr), "mc_classify_pairs");
    } else if (!pa.empty()) {  // both centres are clones: only memoised pairs can be similar
      std::vector<double> val;
      std::vector<uint8_t> hit;
      memo_lookup(*memo, ctx, ds, pa, pb, val, hit, stats);
      std::vector<double> raw;
      std::vector<size_t> idx;
      for (size_t q = 0; q < pa.size(); q++)
        if (hit[q]) {
          raw.push_back(val[q]);
          idx.push_back(q);
        }
      std::vector<uint8_t> s2(raw.size());
      std::vector<double> c2(raw.size());
      if (!raw.empty())
        check(mc_classify_values(ctx, raw.data(), raw.size(), s2.data(), c2.data(), nullptr), "mc_classify_values");
      for (size_t r = 0; r < idx.size(); r++) {
        sim[idx[r]] = s2[r];
        c0[idx[r]] = c2[r];
      }
    }
    {
      Scope sc(timer, "update.cascade");
      merge_cascade(part, poff, sim, c0);
    }
    rebuild = part.size() != C;
    if (it == 0) t_first = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_it0).count();
    // A fixed point: no centre moved and nothing merged (a merge always deletes a cluster), so
    // the state -- every cluster's centre and members -- is what this iteration started from, and
    // each remaining iteration (a deterministic function of that state: the same mean shifts,
    // the same merge pairs, no merge) would leave it unchanged again.  Their evaluations are
    // counted as if run.  (Alignment mode: the remaining iterations would look up the same pairs
    // in the memo, every one of them aligned by now -- memo_lookup aligns only pairs it has not
    // seen, and nothing else changes the memo during the updates -- so they would add nothing.)
    if (!moved && !rebuild && !all_iterations) {
      const uint64_t rest = (uint64_t)(cfg.iterations - 1 - it);
      stats.update_evals += rest * it_update_evals;
      stats.merge_evals += rest * (uint64_t)pa.size();
      stats.update_iters_fixed = rest;
      break;
    }
  }
  if (multi && !memo)
    stats.update_path = split_update == 1 ? "split x" + std::to_string(cfg.comm->world) : "replicated";
  return part;
}


// print_output (ClusterFactory.cpp:495-520): ">Cluster c" for every non-empty cluster, then
// "i\t{len}nt, {header}... " per member with '*' after the centre.  Clusters are formatted
// into per-thread buffers in parallel and written in order.
void write_clstr(const std::string &path, const Dataset &ds, const std::vector<Center> &part, int threads) {
  const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) throw Error("cannot open output " + path, 1);
  const size_t C = part.size();
  std::vector<int> label(C, -1);
  int counter = 0;
  for (size_t c = 0; c < C; c++)
    if (!part[c].points.empty()) label[c] = counter++;
  const int T = std::max(1, std::min<int>(threads, (int)(C / 64) + 1));
  std::vector<std::string> out(T);
  std::vector<uint64_t> at(T + 1, 0);
  bool ok = true;
  auto ndig = [](unsigned long long v) {
    int n = 1;
    while (v >= 10) {
      v /= 10;
      n++;
    }
    return n;
  };
  auto put = [](char *o, unsigned long long v, int n) {  // n = ndig(v)
    for (int i = n - 1; i >= 0; i--) {
      o[i] = (char)('0' + v % 10);
      v /= 10;
    }
    return o + n;
  };
  std::vector<size_t> bytes(T, 0);
  // exact size of every thread's part first
#pragma omp parallel for schedule(static, 1) num_threads(T)
  for (int t = 0; t < T; t++) {
    const size_t c0 = C * t / T, c1 = C * (t + 1) / T;
    size_t n = 0;
    for (size_t c = c0; c < c1; c++) {
      const auto &cen = part[c];
      if (cen.points.empty()) continue;
      n += 10 + (size_t)ndig((unsigned long long)label[c]);
      unsigned long long pt = 0;
      for (uint32_t p : cen.points)
        n += (size_t)ndig(pt++) + 1 + (size_t)ndig(ds.lengths[p]) + 4 + ds.headers[p].size() + 4 +
             (p == cen.centre ? 1 : 0) + 1;
    }
    bytes[t] = n;
  }
  for (int t = 0; t < T; t++) at[t + 1] = at[t] + bytes[t];
  // every line written in place into its part
  auto format = [&](int t, char *w) {
    const size_t c0 = C * t / T, c1 = C * (t + 1) / T;
    for (size_t c = c0; c < c1; c++) {
      const auto &cen = part[c];
      if (cen.points.empty()) continue;
      memcpy(w, ">Cluster ", 9);
      w = put(w + 9, (unsigned long long)label[c], ndig((unsigned long long)label[c]));
      *w++ = '\n';
      unsigned long long pt = 0;
      for (uint32_t p : cen.points) {
        w = put(w, pt, ndig(pt));
        pt++;
        *w++ = '\t';
        w = put(w, ds.lengths[p], ndig(ds.lengths[p]));
        memcpy(w, "nt, ", 4);
        w += 4;
        const auto h = ds.headers[p];
        memcpy(w, h.data(), h.size());
        w += h.size();
        memcpy(w, "... ", 4);
        w += 4;
        if (p == cen.centre) *w++ = '*';
        *w++ = '\n';
      }
    }
  };
  // every part formatted and written at its offset by its own thread (parallel copies into the
  // page cache; measured against a shared mapping of the file, which every thread formats into
  // straight: 1.55 vs 1.40 ms for config B's 4 MB -- the mapping's page faults cost more)
#pragma omp parallel for schedule(static, 1) num_threads(T) reduction(&& : ok)
  for (int t = 0; t < T; t++) {
    out[t].resize(bytes[t]);
    if (bytes[t]) format(t, &out[t][0]);
    const char *d = out[t].data();
    size_t off = 0;
    while (off < out[t].size()) {
      const ssize_t r = pwrite(fd, d + off, out[t].size() - off, (off_t)(at[t] + off));
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) {
        ok = false;
        break;
      }
      off += (size_t)r;
    }
  }
  ok &= close(fd) == 0;
  if (!ok) throw Error("cannot write output " + path, 1);
}

}  // namespace mc
