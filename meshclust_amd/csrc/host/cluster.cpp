// cluster.cpp -- see cluster.hpp.
#include "cluster.hpp"

#include <algorithm>
#include <cfloat>
#include <cstdio>

namespace mc {

namespace {

// accumulate (ClusterFactory.cpp:637-714): grow one cluster around `last` until get_close
// finds no similar candidate; returns the next seed through *last_ptr.
void accumulate(uint32_t *last_ptr, const Dataset &ds, mc_ctx *ctx, BVec &bv, std::vector<Center> &centers,
                const ClusterConfig &cfg, ClusterStats &stats, std::vector<uint32_t> &flag_buf, PhaseTimer &timer) {
  uint32_t last = *last_ptr;
  std::vector<uint32_t> current = {last};
  check(mc_cluster_begin(ctx, last), "mc_cluster_begin");
  bool is_min = false;
  while (!is_min) {
    uint64_t len = ds.lengths[last];
    auto bounds = bv.get_range((uint64_t)(len * cfg.sim), (uint64_t)(len / cfg.sim));
    uint64_t S = 0, E = 0;
    int64_t count = bv.window(bounds.first, bounds.second, &S, &E);
    mc_scan_result res{};
    if (count > 0) {
      stats.scan_steps++;
      stats.scan_candidates += (uint64_t)count;
      Scope sc(timer, "accumulate.mc_scan");
      check(mc_scan(ctx, last, S, E, flag_buf.data(), flag_buf.size(), &res), "mc_scan");
    } else {  // the OpenMP loop runs no iteration: result NULL, is_min stays true
      res.is_min = 1;
      res.has_best = 0;
    }
    is_min = res.is_min != 0;
    if (is_min) {
      if (!res.has_best) {
        uint32_t p = bv.pop();
        if (p != BVec::NONE) check(mc_kill(ctx, bv.spos(p)), "mc_kill");
        *last_ptr = p;
      } else {
        auto rc = bv.locate(res.best_pos);
        *last_ptr = bv.static_order()[res.best_pos];
        bv.erase(rc.first, rc.second);
        check(mc_kill(ctx, res.best_pos), "mc_kill");
      }
    } else {
      std::vector<uint32_t> flagged(flag_buf.begin(), flag_buf.begin() + res.n_flagged);
      bv.remove_positions(flagged, bounds.first.first, bounds.second.first, current);
      last = res.new_centre;
    }
  }
  centers.push_back(Center{last, std::move(current), false});
}

}  // namespace

std::vector<Center> mean_shift_cluster(const Dataset &ds, mc_ctx *ctx, BVec &bv, const ClusterConfig &cfg,
                                       PhaseTimer &timer, ClusterStats &stats) {
  std::vector<Center> part;
  const auto &order = bv.static_order();
  check(mc_set_order(ctx, order.data(), order.size()), "mc_set_order");
  std::vector<uint32_t> flag_buf(order.size() + 1);
  {
    Scope s(timer, "accumulate");
    uint32_t last = bv.pop();
    if (last != BVec::NONE) check(mc_kill(ctx, bv.spos(last)), "mc_kill");
    while (last != BVec::NONE) accumulate(&last, ds, ctx, bv, part, cfg, stats, flag_buf, timer);
  }
  Scope s(timer, "update+merge");
  for (int it = 0; it < cfg.iterations; it++) {
    // mean_shift_update for every centre, all reading the same state (ClusterFactory.cpp:744-749)
    const uint32_t C = (uint32_t)part.size();
    std::vector<uint32_t> cids(C), members, newc(C);
    std::vector<uint64_t> off(C + 1, 0);
    for (uint32_t j = 0; j < C; j++) {
      cids[j] = part[j].centre;
      members.insert(members.end(), part[j].points.begin(), part[j].points.end());
      off[j + 1] = members.size();
    }
    for (uint32_t j = 0; j < C; j++) {
      uint32_t b = j >= (uint32_t)cfg.delta ? j - cfg.delta : 0;
      uint32_t e = std::min<uint32_t>(j + cfg.delta, C - 1);
      stats.update_evals += off[e + 1] - off[b];
    }
    if (C) check(mc_mean_shift(ctx, cids.data(), C, off.data(), members.data(), cfg.delta, newc.data()), "mc_mean_shift");
    for (uint32_t j = 0; j < C; j++) part[j].centre = newc[j];
    // merge (ClusterFactory.cpp:427-493 + Trainer::merge, Trainer.cpp:129-157).  Merging
    // only moves member lists, never centres, so every (candidate, current) centre pair is
    // classified in one batch and the sequential cascade is replayed on the host.
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
    std::vector<uint8_t> sim(pa.size());
    std::vector<double> c0(pa.size());
    if (!pa.empty())
      check(mc_classify_pairs(ctx, pa.data(), pb.data(), pa.size(), sim.data(), c0.data(), nullptr), "mc_classify_pairs");
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
  return part;
}

void write_clstr(const std::string &path, const Dataset &ds, const std::vector<Center> &part) {
  FILE *f = fopen(path.c_str(), "w");
  if (!f) throw Error("cannot open output " + path, 1);
  std::vector<char> buf(1 << 20);
  setvbuf(f, buf.data(), _IOFBF, buf.size());
  int counter = 0;
  for (const auto &cen : part) {
    if (cen.points.empty()) continue;
    fprintf(f, ">Cluster %d\n", counter);
    int pt = 0;
    for (uint32_t p : cen.points) {
      fprintf(f, "%d\t%llunt, %s... ", pt, (unsigned long long)ds.lengths[p], ds.headers[p].c_str());
      if (p == cen.centre) fputc('*', f);
      fputc('\n', f);
      pt++;
    }
    counter++;
  }
  fclose(f);
}

}  // namespace mc
