// mc_oracle_engine.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A sequential CPU implementation of the libmcgpu C-ABI (include/meshclust_amd.h) built
// from the oracle restatement (mc_oracle.c).  tests/ link the host driver objects against
// this library instead of libmcgpu to check, without a GPU, that the host restatement of
// the reference control flow (training sampler, bvec, accumulate, mean shift, merge,
// writer) reproduces the reference's .clstr byte for byte.  The shipped bin/meshclust
// links only libmcgpu; this file is never part of the product.
#include <cfloat>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mc_oracle.h"
#include "../meshclust_amd/csrc/host/lazysort.hpp"

struct mc_ctx {
  std::vector<uint8_t> codes;
  std::vector<uint64_t> seq_off, seg_off;
  std::vector<int32_t> seg;
  uint64_t n = 0;
  int k = 0, B = 0, width = 1;
  std::vector<uint8_t> hist;  // n * B * width
  std::vector<uint64_t> mags;
  mc_classifier cls{};
  bool has_cls = false;
  bool align = false;  // classifier = Feature::align alone (Trainer.cpp:570-577)
  std::vector<uint32_t> order;
  std::vector<uint8_t> alive;
  std::vector<uint32_t> members;  // current cluster, in `current` order
  std::vector<mc::LazyIntroSort> split;  // mc_split_*: the host's lazy introsort
};

static thread_local std::string g_err;
static int fail(int code, const std::string &m) {
  g_err = m;
  return code;
}

extern "C" {

const char *mc_last_error(void) { return g_err.c_str(); }
int mc_abi_version(void) { return MC_ABI_VERSION; }

int mc_ctx_create(int, mc_ctx **out) {
  *out = new mc_ctx();
  return MC_OK;
}
int mc_ctx_destroy(mc_ctx *c) {
  delete c;
  return MC_OK;
}

int mc_load_sequences(mc_ctx *c, const uint8_t *codes, const uint64_t *seq_off, uint64_t n, const int32_t *seg,
                      const uint64_t *seg_off) {
  c->n = n;
  c->codes.assign(codes, codes + seq_off[n]);
  c->seq_off.assign(seq_off, seq_off + n + 1);
  c->seg_off.assign(seg_off, seg_off + n + 1);
  c->seg.assign(seg, seg + 2 * seg_off[n]);
  return MC_OK;
}

// the packed form of the host parser: unpacked here to the bytes the reference holds
int mc_load_packed(mc_ctx *c, const uint32_t *packed, const uint64_t *pk_off, const uint64_t *seq_off, uint64_t n,
                   const uint64_t *exc_pos, const uint8_t *exc_val, uint64_t nexc, const int32_t *seg,
                   const uint64_t *seg_off) {
  std::vector<uint8_t> codes(seq_off[n]);
  for (uint64_t i = 0; i < n; i++)
    for (uint64_t j = 0; j < seq_off[i + 1] - seq_off[i]; j++)
      codes[seq_off[i] + j] = (uint8_t)((packed[pk_off[i] + j / 16] >> (2 * (j % 16))) & 3u);
  for (uint64_t q = 0; q < nexc; q++) codes[exc_pos[q]] = exc_val[q];
  return mc_load_sequences(c, codes.data(), seq_off, n, seg, seg_off);
}

static int hist_of(mc_ctx *c, uint64_t i, int k, std::vector<uint64_t> &h) {
  h.resize((size_t)1 << (2 * k));
  const uint8_t *s = c->codes.data() + c->seq_off[i];
  int64_t len = (int64_t)(c->seq_off[i + 1] - c->seq_off[i]);
  int nseg = (int)(c->seg_off[i + 1] - c->seg_off[i]);
  return mco_kmer_hist(s, len, c->seg.data() + 2 * c->seg_off[i], nseg, k, 1, h.data());
}

int mc_kmer_max(mc_ctx *c, int k, uint64_t *largest) {
  uint64_t mx = 0;
  std::vector<uint64_t> h;
  for (uint64_t i = 0; i < c->n; i++) {
    int rc = hist_of(c, i, k, h);
    if (rc) return fail(rc, "invalid nucleotide in k-mer");
    for (auto v : h) mx = v > mx ? v : mx;
  }
  *largest = mx;
  return MC_OK;
}

int mc_kmer_build(mc_ctx *c, int k, int width) {
  c->k = k;
  c->B = 1 << (2 * k);
  c->width = width;
  c->hist.assign(c->n * c->B * width, 0);
  c->mags.assign(c->n, 0);
  std::vector<uint64_t> h;
  for (uint64_t i = 0; i < c->n; i++) {
    int rc = hist_of(c, i, k, h);
    if (rc) return fail(rc, "invalid nucleotide in k-mer");
    uint64_t mag = 0;
    uint8_t *dst = c->hist.data() + i * c->B * width;
    for (int b = 0; b < c->B; b++) {
      uint64_t v = h[b];
      mag += v;
      switch (width) {
        case 1: ((uint8_t *)dst)[b] = (uint8_t)v; break;
        case 2: ((uint16_t *)dst)[b] = (uint16_t)v; break;
        case 4: ((uint32_t *)dst)[b] = (uint32_t)v; break;
        default: ((uint64_t *)dst)[b] = v; break;
      }
    }
    c->mags[i] = mag;
  }
  return MC_OK;
}

int mc_get_histograms(mc_ctx *c, void *hist, uint64_t *mags) {
  if (hist) memcpy(hist, c->hist.data(), c->hist.size());
  if (mags) memcpy(mags, c->mags.data(), c->mags.size() * 8);
  return MC_OK;
}

static const void *row(mc_ctx *c, uint32_t id) { return c->hist.data() + (size_t)id * c->B * c->width; }
static uint64_t len_of(mc_ctx *c, uint32_t id) { return c->seq_off[id + 1] - c->seq_off[id]; }

int mc_distance_keys(mc_ctx *c, const uint32_t *piv, uint32_t np, const uint32_t *ids, uint64_t m, uint16_t *keys) {
#pragma omp parallel for schedule(dynamic)
  for (uint32_t p = 0; p < np; p++)
    for (uint64_t i = 0; i < m; i++)
      keys[p * m + i] = (uint16_t)mco_distance(row(c, ids[i]), row(c, piv[p]), c->width, c->B, c->mags[ids[i]],
                                               c->mags[piv[p]]);
  return MC_OK;
}

int mc_split_begin(mc_ctx *c, const uint32_t *piv, uint32_t np, const uint32_t *order, uint64_t n) {
  std::vector<uint16_t> keys((size_t)np * n);
  int rc = mc_distance_keys(c, piv, np, order, n, keys.data());
  if (rc) return rc;
  c->split.clear();
  c->split.reserve(np);
  for (uint32_t p = 0; p < np; p++) {
    std::vector<uint64_t> w(n);
    for (uint64_t t = 0; t < n; t++) w[t] = ((uint64_t)keys[(size_t)p * n + t] << 32) | order[t];
    if (p == 0 && getenv("MC_DUMP_SPLIT")) {  // (diagnostics: the first pivot's array)
      FILE *fd = fopen(getenv("MC_DUMP_SPLIT"), "wb");
      if (fd) {
        fwrite(w.data(), 8, n, fd);
        fclose(fd);
      }
    }
    c->split.emplace_back(std::move(w));
  }
  return MC_OK;
}

int mc_split_begin_words(mc_ctx *c, const uint64_t *words, uint32_t narr, uint64_t n, int depth) {
  c->split.clear();
  for (uint32_t a = 0; a < narr; a++)
    c->split.emplace_back(std::vector<uint64_t>(words + (size_t)a * n, words + (size_t)(a + 1) * n), depth);
  return MC_OK;
}

int mc_split_select_words(mc_ctx *c, uint64_t nq, const uint32_t *arr, const uint64_t *pos, uint64_t *out) {
  for (uint64_t i = 0; i < nq; i++)
    if (arr[i] >= c->split.size() || pos[i] >= c->split[arr[i]].size()) return fail(MC_ERR_ARG, "split query out of range");
  // one thread per array (a LazyIntroSort is not shared between threads)
  std::vector<std::vector<uint64_t>> by(c->split.size());
  for (uint64_t i = 0; i < nq; i++) by[arr[i]].push_back(i);
#pragma omp parallel for schedule(dynamic)
  for (size_t a = 0; a < by.size(); a++)
    for (uint64_t i : by[a]) out[i] = c->split[a].at((int64_t)pos[i]);
  return MC_OK;
}

int mc_split_select(mc_ctx *c, uint64_t nq, const uint32_t *arr, const uint64_t *pos, uint32_t *ids) {
  std::vector<uint64_t> w(nq);
  int rc = mc_split_select_words(c, nq, arr, pos, w.data());
  if (rc) return rc;
  for (uint64_t i = 0; i < nq; i++) ids[i] = (uint32_t)w[i];
  return MC_OK;
}

int mc_split_end(mc_ctx *c) {
  c->split.clear();
  return MC_OK;
}

static int raw_one(mc_ctx *c, uint16_t f, uint32_t a, uint32_t b, double *out) {
  return mco_raw(f, row(c, a), row(c, b), c->width, c->B, c->mags[a], c->mags[b], len_of(c, a), len_of(c, b), out);
}

int mc_pair_features(mc_ctx *c, const uint32_t *a, const uint32_t *b, uint64_t m, const uint16_t *flags, int nflag,
                     double *raw) {
  for (uint64_t i = 0; i < m; i++)
    for (int f = 0; f < nflag; f++) {
      int rc = raw_one(c, flags[f], a[i], b[i], &raw[i * nflag + f]);
      if (rc) return fail(rc, "feature error");
    }
  return MC_OK;
}

int mc_set_classifier(mc_ctx *c, const mc_classifier *cls) {
  c->cls = *cls;
  c->has_cls = true;
  c->align = cls->n_single == 1 && cls->lookup[0] == MC_FEAT_ALIGN;
  return MC_OK;
}

// GlobAlignE(a, 0, la-1, b, 0, lb-1, 1, -1, 2, 1).getIdentity() (Feature::align, Feature.cpp:221-243)
static double nw_ident(mc_ctx *c, uint32_t a, uint32_t b) {
  int sc, l, d;
  double id;
  mco_nw(c->codes.data() + c->seq_off[a], (int)len_of(c, a), c->codes.data() + c->seq_off[b], (int)len_of(c, b), 1,
         -1, 2, 1, &sc, &l, &d, &id);
  return id;
}

int mc_classify_values(mc_ctx *c, const double *raw, uint64_t m, uint8_t *similar, double *combo0, double *sum) {
  const int ns = c->cls.n_single;
  for (uint64_t i = 0; i < m; i++) {
    double r[MC_MAX_SINGLE] = {0};
    for (int f = 0; f < ns; f++) r[f] = raw[i * ns + f];
    double s, c0;
    int d = mco_classify(&c->cls, r, &s, &c0);
    if (similar) similar[i] = (uint8_t)d;
    if (combo0) combo0[i] = c0;
    if (sum) sum[i] = s;
  }
  return MC_OK;
}

static int classify(mc_ctx *c, uint32_t a, uint32_t b, double *sum, double *c0) {
  double raw[MC_MAX_SINGLE];
  for (int f = 0; f < c->cls.n_single; f++) raw_one(c, c->cls.lookup[f], a, b, &raw[f]);
  return mco_classify(&c->cls, raw, sum, c0);
}

int mc_classify_pairs(mc_ctx *c, const uint32_t *a, const uint32_t *b, uint64_t m, uint8_t *similar, double *combo0,
                      double *sum) {
  if (c->align) return fail(MC_ERR_STATE, "mc_classify_pairs is not available in alignment mode");
  for (uint64_t i = 0; i < m; i++) {
    double s, c0;
    int d = classify(c, a[i], b[i], &s, &c0);
    if (similar) similar[i] = (uint8_t)d;
    if (combo0) combo0[i] = c0;
    if (sum) sum[i] = s;
  }
  return MC_OK;
}

int mc_nw_identity(mc_ctx *c, const uint32_t *a, const uint32_t *b, uint64_t m, double *ident, int32_t *len,
                   int32_t *ids) {
#pragma omp parallel for schedule(dynamic)
  for (uint64_t i = 0; i < m; i++) {
    int sc, l, d;
    double id;
    mco_nw(c->codes.data() + c->seq_off[a[i]], (int)len_of(c, a[i]), c->codes.data() + c->seq_off[b[i]],
           (int)len_of(c, b[i]), 1, -1, 2, 1, &sc, &l, &d, &id);
    ident[i] = id;
    if (len) len[i] = l;
    if (ids) ids[i] = d;
  }
  return MC_OK;
}

int mc_nw_identity_raw(mc_ctx *, const uint8_t *a, const uint64_t *ao, const uint8_t *b, const uint64_t *bo,
                       uint64_t m, double *ident, int32_t *len, int32_t *ids, int32_t *score) {
  for (uint64_t i = 0; i < m; i++) {
    int sc, l, d;
    double id;
    mco_nw(a + ao[i], (int)(ao[i + 1] - ao[i]), b + bo[i], (int)(bo[i + 1] - bo[i]), 1, -1, 2, 1, &sc, &l, &d, &id);
    ident[i] = id;
    if (len) len[i] = l;
    if (ids) ids[i] = d;
    if (score) score[i] = sc;
  }
  return MC_OK;
}

int mc_set_order(mc_ctx *c, const uint32_t *order, uint64_t n) {
  c->order.assign(order, order + n);
  c->alive.assign(n, 1);
  return MC_OK;
}
int mc_kill(mc_ctx *c, uint64_t pos) {
  c->alive[pos] = 0;
  return MC_OK;
}
int mc_cluster_begin(mc_ctx *c, uint32_t first) {
  c->members.assign(1, first);
  return MC_OK;
}

static uint32_t mean_closest(mc_ctx *c, const std::vector<uint32_t> &mem) {
  std::vector<double> mean(c->B, 0.0);
  for (uint32_t id : mem) {
    const void *r = row(c, id);
    for (int b = 0; b < c->B; b++) {
      double v;
      switch (c->width) {
        case 1: v = ((const uint8_t *)r)[b]; break;
        case 2: v = ((const uint16_t *)r)[b]; break;
        case 4: v = ((const uint32_t *)r)[b]; break;
        default: v = (double)((const uint64_t *)r)[b]; break;
      }
      mean[b] += v;
    }
  }
  double bottom = (double)mem.size();
  for (auto &m : mean) m /= bottom;
  uint32_t best = 0xffffffffu;
  double bd = DBL_MAX;
  for (uint32_t id : mem) {
    double d = mco_distance_d(row(c, id), c->width, c->B, mean.data());
    if (best == 0xffffffffu || d < bd) {
      bd = d;
      best = id;
    }
  }
  return best;
}

// the serial get_close loop over the window (alignment mode: `ident` per position of S..E;
// count: whether the NW pairs are counted here)
static int scan_loop(mc_ctx *c, uint32_t centre, uint64_t S, uint64_t E, const std::vector<double> &ident, bool count,
                     uint32_t *flagged, uint64_t cap, mc_scan_result *res) {
  memset(res, 0, sizeof *res);
  double best_val = -1;
  bool has = false;
  uint64_t best_pos = 0, nf = 0;
  bool is_min = true;
  for (uint64_t pos = S; pos <= E; pos++) {
    if (!c->alive[pos]) continue;
    uint32_t id = c->order[pos];
    double s, c0;
    int d;
    if (c->align) {
      double r[MC_MAX_SINGLE] = {ident[pos - S]};
      d = mco_classify(&c->cls, r, &s, &c0);
      if (count) {
        res->nw_pairs++;
        res->nw_cells += len_of(c, id) * len_of(c, centre);
      }
    } else {
      d = classify(c, id, centre, &s, &c0);
    }
    if (c0 > best_val) {
      best_val = c0;
      best_pos = pos;
      has = true;
    }
    if (d) {
      is_min = false;
      if (nf >= cap) return fail(MC_ERR_ARG, "flag buffer too small");
      flagged[nf++] = (uint32_t)pos;
      c->alive[pos] = 0;
      c->members.push_back(id);
    }
  }
  res->is_min = is_min;
  res->has_best = has;
  res->best_pos = best_pos;
  res->best_val = best_val;
  res->n_flagged = nf;
  if (!is_min) res->new_centre = mean_closest(c, c->members);
  res->n_members = (uint32_t)c->members.size();
  return MC_OK;
}

int mc_scan(mc_ctx *c, uint32_t centre, uint64_t S, uint64_t E, uint32_t *flagged, uint64_t cap, mc_scan_result *res) {
  std::vector<double> ident;
  if (c->align) {  // Feature::align(*pt, *p) for the whole window, then the serial loop
    ident.assign(E - S + 1, 0.0);
#pragma omp parallel for schedule(dynamic)
    for (uint64_t pos = S; pos <= E; pos++)
      if (c->alive[pos]) ident[pos - S] = nw_ident(c, c->order[pos], centre);
  }
  return scan_loop(c, centre, S, E, ident, true, flagged, cap, res);
}

int mc_align_part(mc_ctx *c, uint32_t centre, uint64_t S, uint64_t E, uint32_t part, uint32_t nparts, double *ident,
                  uint64_t cap, uint64_t *n_part, uint64_t *pairs, uint64_t *cells) {
  if (!c->align) return fail(MC_ERR_STATE, "mc_align_part: alignment mode only");
  if (S > E || E >= c->order.size() || nparts == 0 || part >= nparts || !n_part) return fail(MC_ERR_ARG, "bad window");
  std::vector<uint32_t> mine;
  uint64_t np = 0, cl = 0, i = 0;
  for (uint64_t pos = S; pos <= E; pos++) {
    if (!c->alive[pos]) continue;
    const uint32_t id = c->order[pos];
    np++;
    cl += len_of(c, id) * len_of(c, centre);
    if (i++ % nparts == part) mine.push_back(id);
  }
  if (pairs) *pairs = np;
  if (cells) *cells = cl;
  *n_part = mine.size();
  if (mine.size() > cap || (!ident && !mine.empty())) return fail(MC_ERR_ARG, "mc_align_part: identity buffer too small");
#pragma omp parallel for schedule(dynamic)
  for (int64_t j = 0; j < (int64_t)mine.size(); j++) ident[j] = nw_ident(c, mine[j], centre);
  return MC_OK;
}

int mc_scan_ident(mc_ctx *c, uint32_t centre, uint64_t S, uint64_t E, const double *ident, uint32_t *flagged,
                  uint64_t cap, mc_scan_result *res) {
  if (!c->align) return fail(MC_ERR_STATE, "mc_scan_ident: alignment mode only");
  if (S > E || E >= c->order.size()) return fail(MC_ERR_ARG, "bad window");
  std::vector<double> win(E - S + 1, 0.0);
  uint64_t i = 0;
  for (uint64_t pos = S; pos <= E; pos++)
    if (c->alive[pos]) win[pos - S] = ident[i++];
  return scan_loop(c, centre, S, E, win, false, flagged, cap, res);
}

int mc_scan_part(mc_ctx *c, uint32_t centre, uint64_t S, uint64_t E, uint32_t part, uint32_t nparts, uint32_t *flagged,
                 uint64_t cap, mc_scan_result *res) {
  if (c->align) return fail(MC_ERR_UNSUPPORTED, "sharded get_close steps take k-mer histograms");
  if (S > E || E >= c->order.size() || nparts == 0 || part >= nparts) return fail(MC_ERR_ARG, "bad sharded window");
  memset(res, 0, sizeof *res);
  double best_val = -1;
  bool has = false;
  uint64_t best_pos = 0, nf = 0;
  for (uint64_t pos = S; pos <= E; pos++) {
    if (!c->alive[pos] || (pos / MC_SHARD_BLOCK) % nparts != part) continue;
    double s, c0;
    const int d = classify(c, c->order[pos], centre, &s, &c0);
    if (c0 > best_val) {
      best_val = c0;
      best_pos = pos;
      has = true;
    }
    if (d) {
      if (nf >= cap) return fail(MC_ERR_ARG, "flag buffer too small");
      flagged[nf++] = (uint32_t)pos;
    }
  }
  res->is_min = nf == 0;
  res->has_best = has;
  res->best_pos = best_pos;
  res->best_val = best_val;
  res->n_flagged = nf;
  res->new_centre = 0xffffffffu;
  res->n_members = (uint32_t)c->members.size();
  return MC_OK;
}

int mc_scan_commit(mc_ctx *c, const uint32_t *flagged, uint64_t n, mc_scan_result *res) {
  if (c->align) return fail(MC_ERR_UNSUPPORTED, "sharded get_close steps take k-mer histograms");
  memset(res, 0, sizeof *res);
  for (uint64_t i = 0; i < n; i++) {
    if (flagged[i] >= c->order.size() || !c->alive[flagged[i]] || (i && flagged[i] <= flagged[i - 1]))
      return fail(MC_ERR_ARG, "mc_scan_commit: positions must be ascending, alive and in range");
    c->alive[flagged[i]] = 0;
    c->members.push_back(c->order[flagged[i]]);
  }
  res->is_min = n == 0;
  res->n_flagged = n;
  res->new_centre = n ? mean_closest(c, c->members) : 0xffffffffu;
  res->n_members = (uint32_t)c->members.size();
  return MC_OK;
}

int mc_mean_shift_select(mc_ctx *c, const uint32_t *cid, uint32_t C, const uint64_t *off, const uint32_t *members,
                         int delta, const uint8_t *keep, uint32_t *newc) {
  uint64_t k = 0;
  for (uint32_t j = 0; j < C; j++) {
    long b = (long)j - delta < 0 ? 0 : (long)j - delta;
    long e = (long)j + delta < (long)C - 1 ? (long)j + delta : (long)C - 1;
    std::vector<uint32_t> good;
    for (uint64_t q = off[b]; q < off[e + 1]; q++, k++)
      if (keep[k]) good.push_back(members[q]);
    newc[j] = good.empty() ? cid[j] : mean_closest(c, good);
  }
  return MC_OK;
}

int mc_mean_shift_range(mc_ctx *c, const uint32_t *cid, uint32_t C, const uint64_t *off, const uint32_t *members,
                        int delta, uint32_t j0, uint32_t j1, uint32_t *newc) {
  if (c->align) return fail(MC_ERR_STATE, "mc_mean_shift is not available in alignment mode");
  if (j0 > j1 || j1 > C) return fail(MC_ERR_ARG, "bad centre range");
#pragma omp parallel for schedule(dynamic)
  for (uint32_t j = j0; j < j1; j++) {
    long b = (long)j - delta < 0 ? 0 : (long)j - delta;
    long e = (long)j + delta < (long)C - 1 ? (long)j + delta : (long)C - 1;
    std::vector<uint32_t> good;
    for (uint64_t q = off[b]; q < off[e + 1]; q++) {
      double s, c0;
      if (classify(c, members[q], cid[j], &s, &c0)) good.push_back(members[q]);
    }
    newc[j - j0] = good.empty() ? cid[j] : mean_closest(c, good);
  }
  return MC_OK;
}

int mc_mean_shift(mc_ctx *c, const uint32_t *cid, uint32_t C, const uint64_t *off, const uint32_t *members, int delta,
                  uint32_t *newc) {
  return mc_mean_shift_range(c, cid, C, off, members, delta, 0, C, newc);
}

int mc_update_iteration(mc_ctx *c, const uint32_t *cid, uint32_t C, const uint64_t *off, const uint32_t *members,
                        int delta, uint32_t *newc, uint8_t *similar, double *combo0, uint64_t *npairs) {
  if (!npairs || delta < 0) return fail(MC_ERR_ARG, "bad arguments");
  if (c->align) return fail(MC_ERR_STATE, "mc_update_iteration is not available in alignment mode");
  *npairs = 0;
  if (int rc = mc_mean_shift_range(c, cid, C, off, members, delta, 0, C, newc)) return rc;
  std::vector<uint32_t> pa, pb;
  for (uint32_t i = 0; i < C; i++)
    for (uint32_t t = i + 1; t < C && t <= i + (uint32_t)delta; t++) {
      pa.push_back(newc[t]);
      pb.push_back(newc[i]);
    }
  *npairs = pa.size();
  return mc_classify_pairs(c, pa.data(), pb.data(), pa.size(), similar, combo0, nullptr);
}

int mc_accumulate(mc_ctx *, const uint32_t *, const uint64_t *, uint32_t, double, uint32_t *, uint64_t *, uint32_t *,
                  uint64_t *, uint64_t *) {
  return fail(MC_ERR_UNSUPPORTED, "the CPU oracle engine drives accumulation step by step");
}

// The device-sharded accumulation's mailbox is read by the ranks' persistent kernels; the CPU
// engine's ranks take the host-driven sharded steps instead.
uint64_t mc_mailbox_bytes(int world, uint64_t n) { return world < 1 ? 0 : 2ull * world * (8 + n / world + 513) * 8; }
int mc_ctx_pci_bus_id(mc_ctx *, char *buf, int len) {
  if (!buf || len < 16) return MC_ERR_ARG;
  snprintf(buf, len, "cpu");
  return MC_OK;
}
int mc_set_mailbox(mc_ctx *, void *, uint64_t, int, int world, int) {
  return world == 0 ? MC_OK : fail(MC_ERR_UNSUPPORTED, "no device-sharded accumulation in the CPU oracle engine");
}
int mc_accum_plan_info(mc_ctx *, uint32_t, uint32_t *) {
  return fail(MC_ERR_UNSUPPORTED, "the CPU oracle engine drives accumulation step by step");
}
int mc_set_accum_grid(mc_ctx *, uint32_t) { return MC_OK; }
int mc_accum_reserve(mc_ctx *, uint32_t) {
  return fail(MC_ERR_UNSUPPORTED, "the CPU oracle engine drives accumulation step by step");
}
// (ranks of the CPU engine share the host's cores; there is no CU mask to split)
int mc_ctx_partition(mc_ctx *, int slot, int share) {
  return share < 1 || slot < 0 || slot >= share ? MC_ERR_ARG : MC_OK;
}

// RCCL is a GPU-side transport: the CPU engine's ranks exchange through the caller's callback.
int mc_comm_unique_id(uint8_t *) { return fail(MC_ERR_UNSUPPORTED, "no RCCL in the CPU oracle engine"); }
int mc_comm_create(int, int, int, const uint8_t *, mc_comm **) {
  return fail(MC_ERR_UNSUPPORTED, "no RCCL in the CPU oracle engine");
}
int mc_comm_allgather(mc_comm *, const void *, uint64_t, void *) { return MC_ERR_UNSUPPORTED; }
int mc_comm_stats(const mc_comm *, uint64_t *, uint64_t *) { return MC_ERR_UNSUPPORTED; }
int mc_comm_destroy(mc_comm *, int) { return MC_OK; }

int mc_timers(mc_ctx *, double *ms, int n, int) {
  for (int i = 0; i < n; i++) ms[i] = 0;
  return MC_OK;
}

}  // extern "C"
