/*
 * mc_oracle.c -- TEST INFRASTRUCTURE ONLY (see mc_oracle.h).
 *
 * Plain C restatement of the reference hot-path arithmetic.  Compiled with
 * -ffp-contract=off; every place where the reference build (g++ -O3 with FMA available)
 * contracts a*b+c into a fused multiply-add is written as an explicit fma() -- verified by
 * objdump of the reference objects (vfnmadd213sd in DivergencePoint::distance/distance_d,
 * vfmadd in the Trainer::get_close/filter/merge sums; no FMA in Feature::intersection/
 * pearson/manhattan/kulczynski2, normalize_cache or operator()).
 * Integer arithmetic mirrors the reference's C++ types per histogram width T (uint8/16/32/64),
 * including its unsigned wrap-arounds.
 */
#include "mc_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- K1: k-mer counting */
/* KmerHashTable::hash(sequence, keyStart) (KmerHashTable.cpp:106-130): first base is the
 * most significant base-4 digit; any code outside 0..3 throws InvalidInputException. */
int mco_kmer_hist(const uint8_t *seq, int64_t len, const int32_t *seg, int nseg, int k,
                  uint64_t init, uint64_t *out) {
  if (k < 1 || k > 15) return MC_ERR_ARG;
  uint64_t B = 1ull << (2 * k);
  uint64_t top = 1ull << (2 * (k - 1)); /* mMinusOne[c] = c * bases[0] (:53-56) */
  for (uint64_t i = 0; i < B; i++) out[i] = init;
  for (int s = 0; s < nseg; s++) {
    int64_t first = seg[2 * s], last = (int64_t)seg[2 * s + 1] - k + 1; /* fill_table :46-50 */
    /* validation loop over k-mer START positions only (:136-148) */
    for (int64_t i = first; i <= last; i++)
      if (seq[i] > 3) return MC_ERR_INPUT;
    /* first k-mer fully checked (:150 -> :106-130) */
    if (first + k > len) return MC_ERR_INPUT;
    uint64_t h = 0;
    for (int i = 0; i < k; i++) {
      uint8_t c = seq[first + i];
      if (c > 3) return MC_ERR_INPUT;
      h = h * 4 + c;
    }
    if (h >= B) return MC_ERR_INPUT;
    out[h]++;
    /* rolling hash (:153-158), wholesaleIncrement bounds check (:203-206) */
    for (int64_t i = first + 1; i <= last; i++) {
      h = 4 * (h - (uint64_t)seq[i - 1] * top) + seq[i + k - 1];
      if (h >= B) return MC_ERR_INPUT;
      out[h]++;
    }
  }
  return MC_OK;
}

/* ---------------------------------------------------------------- typed accessors */
static inline uint64_t ld(const void *p, int width, int i) {
  switch (width) {
    case 1: return ((const uint8_t *)p)[i];
    case 2: return ((const uint16_t *)p)[i];
    case 4: return ((const uint32_t *)p)[i];
    default: return ((const uint64_t *)p)[i];
  }
}
/* value of the C++ expression `2 * std::min(p, q)` of type T promoted (int for u8/u16). */
static inline uint64_t twice_min(uint64_t a, uint64_t b, int width) {
  uint64_t m = a < b ? a : b;
  switch (width) {
    case 1:
    case 2: return 2 * m;                              /* int, exact            */
    case 4: return (uint64_t)(uint32_t)(2u * (uint32_t)m); /* unsigned int wraps */
    default: return 2 * m;                             /* uint64 wraps          */
  }
}

/* DivergencePoint<T>::distance (DivergencePoint.cpp:68-81). */
uint64_t mco_distance(const void *p, const void *q, int width, int B, uint64_t magp, uint64_t magq) {
  uint64_t dist = 0;
  const uint64_t mag = magp + magq;
  for (int i = 0; i < B; i++) {
    uint64_t a = ld(p, width, i), b = ld(q, width, i);
    dist += a < b ? a : b;
  }
  dist *= 2;
  double frac = (double)dist / (double)mag;
  return (uint64_t)(fma(-frac, frac, 1.0) * 10000.0);
}

/* DivergencePoint<T>::distance_d (DivergencePoint.cpp:53-65): (T)mean truncates, and the
 * uint64 `mag` is re-truncated after every bin. */
double mco_distance_d(const void *p, int width, int B, const double *mean) {
  uint64_t dist = 0, mag = 0;
  for (int i = 0; i < B; i++) {
    uint64_t a = ld(p, width, i);
    double m = mean[i];
    uint64_t tm;
    switch (width) {
      case 1: tm = (uint8_t)(int32_t)m; break;
      case 2: tm = (uint16_t)(int32_t)m; break;
      case 4: tm = (uint32_t)(int64_t)m; break;
      default: tm = (uint64_t)m; break;
    }
    dist += twice_min(a, tm, width);
    mag = (uint64_t)((double)mag + ((double)a + m));
  }
  double frac = (double)dist / (double)mag;
  return fma(-frac, frac, 1.0) * 10000.0;
}

/* ---------------------------------------------------------------- features */
static double f_intersection(const void *p, const void *q, int w, int B, uint64_t mp, uint64_t mq) {
  uint64_t dist = 0; /* uintmax_t dist += 2 * std::min(...) (Feature.cpp:264-269) */
  for (int i = 0; i < B; i++) dist += twice_min(ld(p, w, i), ld(q, w, i), w);
  return (double)dist / (double)(mp + mq);
}

static double f_pearson(const void *p, const void *q, int w, int B, uint64_t mp, uint64_t mq) {
  /* Feature.cpp:273-294 */
  double dap = (double)mp / B, daq = (double)mq / B;
  int ap = (int)round(dap), aq = (int)round(daq);
  uint64_t dot = 0, np = 0, nq = 0; /* intmax_t sums, computed modulo 2^64 */
  for (int i = 0; i < B; i++) {
    uint64_t a = ld(p, w, i), b = ld(q, w, i);
    int64_t dp, dq;
    if (w <= 2) {
      dp = (int64_t)a - ap;
      dq = (int64_t)b - aq;
    } else if (w == 4) { /* unsigned int arithmetic, then widened (the u32 trap) */
      dp = (int64_t)(uint64_t)(uint32_t)((uint32_t)a - (uint32_t)ap);
      dq = (int64_t)(uint64_t)(uint32_t)((uint32_t)b - (uint32_t)aq);
    } else {
      dp = (int64_t)(a - (uint64_t)(int64_t)ap);
      dq = (int64_t)(b - (uint64_t)(int64_t)aq);
    }
    np += (uint64_t)dp * (uint64_t)dp;
    nq += (uint64_t)dq * (uint64_t)dq;
    dot += (uint64_t)dp * (uint64_t)dq;
  }
  double prod = (double)(int64_t)(np * nq);
  double den = sqrt(0.5 < prod ? prod : 0.5);
  return (double)(int64_t)dot / den;
}

static double f_manhattan(const void *p, const void *q, int w, int B) {
  uint32_t sum = 0; /* `int sum` accumulating T-typed |p-q| (Feature.cpp:315-322) */
  for (int i = 0; i < B; i++) {
    uint64_t a = ld(p, w, i), b = ld(q, w, i);
    sum += (uint32_t)(a > b ? a - b : b - a);
  }
  return (double)(int32_t)sum;
}

static double f_kulczynski2(const void *p, const void *q, int w, int B, uint64_t mp, uint64_t mq) {
  /* Feature.cpp:206-220 */
  uint64_t min_sum = 0;
  double ap = (double)mp / B, aq = (double)mq / B;
  for (int i = 0; i < B; i++) {
    uint64_t a = ld(p, w, i), b = ld(q, w, i);
    min_sum += a < b ? a : b;
  }
  double coeff = ((double)B * (ap + aq)) / ((2.0 * ap) * aq);
  return coeff * (double)min_sum;
}

int mco_raw(uint16_t flag, const void *p, const void *q, int width, int B, uint64_t magp,
            uint64_t magq, uint64_t lenp, uint64_t lenq, double *out) {
  switch (flag) {
    case MC_FEAT_LD: /* Feature.cpp:325-339 */
      if (lenp == 0 || lenq == 0) return MC_ERR_INPUT;
      *out = (double)(lenp > lenq ? lenp - lenq : lenq - lenp);
      return MC_OK;
    case MC_FEAT_MANHATTAN: *out = f_manhattan(p, q, width, B); return MC_OK;
    case MC_FEAT_INTERSECTION: *out = f_intersection(p, q, width, B, magp, magq); return MC_OK;
    case MC_FEAT_PEARSON: *out = f_pearson(p, q, width, B, magp, magq); return MC_OK;
    case MC_FEAT_KULCZYNSKI2: *out = f_kulczynski2(p, q, width, B, magp, magq); return MC_OK;
    default: return MC_ERR_ARG;
  }
}

void mco_normalize(const mc_classifier *c, double *cache) {
  for (int i = 0; i < c->n_single; i++) {
    double val = (cache[i] - c->mins[i]) / (c->maxs[i] - c->mins[i]);
    cache[i] = c->is_sim[i] ? val : 1 - val;
  }
}

double mco_combo(const mc_classifier *c, int col, const double *cache) {
  double prod = 1;
  for (int j = 0; j < c->combo_len[col]; j++) {
    double v = cache[c->combo_idx[col][j]];
    if (c->combo_kind[col] == MC_COMBO_SELF) prod *= v;
    else prod *= v * v;
  }
  return prod;
}

int mco_classify(const mc_classifier *c, const double *raw, double *sum_out, double *combo0) {
  double cache[MC_MAX_SINGLE];
  memcpy(cache, raw, sizeof(double) * c->n_single);
  mco_normalize(c, cache);
  double sum = c->weights[0];
  for (int col = 0; col < c->n_combo; col++) {
    double v = mco_combo(c, col, cache);
    if (col == 0 && combo0) *combo0 = v;
    sum = fma(c->weights[col + 1], v, sum);
  }
  if (sum_out) *sum_out = sum;
  return round(1.0 / (1 + exp(-sum))) == 1.0;
}

/* ---------------------------------------------------------------- K3: GlobAlignE */
/* Restates GlobAlignE::findAlignment (GlobAlignE.cpp:123-292) with the same three state
 * rows (M = matches, Y = upperGap, X = lowerGap), each carrying (score, length, identities),
 * the same finite "-infinity" and the same tie priorities. */
void mco_nw(const uint8_t *a, int la, const uint8_t *b, int lb, int match, int mismatch,
            int gap_open, int gap_ext, int *score_out, int *len_out, int *ids_out,
            double *identity) {
  const int len1 = la + 1, len2 = lb + 1;
  int *buf = (int *)malloc(sizeof(int) * 9 * (size_t)len1);
  int *M = buf, *Y = buf + len1, *X = buf + 2 * len1;
  int *ML = buf + 3 * len1, *YL = buf + 4 * len1, *XL = buf + 5 * len1;
  int *MI = buf + 6 * len1, *YI = buf + 7 * len1, *XI = buf + 8 * len1;
  int shorter = (len2 < len1 ? len2 : len1) - 1;
  int lenDiff = abs(len2 - len1);
  int maxDiff = 0;
  if (lenDiff >= 1) maxDiff += -gap_open - (lenDiff * gap_ext);
  maxDiff += (mismatch * shorter) - 1;
  const int ninf = maxDiff;
  M[0] = 0; Y[0] = ninf; X[0] = ninf;
  ML[0] = YL[0] = XL[0] = 0;
  MI[0] = YI[0] = XI[0] = 0;
  for (int i = 1; i < len1; i++) {
    Y[i] = ninf; M[i] = ninf; X[i] = -gap_open - i * gap_ext;
    ML[i] = YL[i] = XL[i] = i;
    MI[i] = YI[i] = XI[i] = 0;
  }
  for (int j = 1; j < len2; j++) {
    int mLag = M[0], mLenLag = ML[0], mIdLag = MI[0];
    int yLag = -gap_open - (j - 1) * gap_ext, yLenLag = j - 1, yIdLag = 0;
    for (int i = 1; i < len1; i++) {
      int yBegin = M[i] - (gap_open + gap_ext);
      int yCont = Y[i] - gap_ext;
      int ans = yBegin > yCont ? yBegin : yCont;
      int s1 = Y[i], s2 = YL[i], s3 = YI[i];
      Y[i] = ans;
      if (ans == yBegin) { YL[i] = ML[i] + 1; YI[i] = MI[i]; }
      else { YL[i] = YL[i] + 1; }
      int sc = (a[i - 1] == b[j - 1]) ? match : mismatch;
      int matched = mLag + sc, xEnd = X[i - 1] + sc, yEnd = yLag + sc;
      ans = matched > xEnd ? matched : xEnd;
      ans = ans > yEnd ? ans : yEnd;
      mLag = M[i];
      M[i] = ans;
      int tLen = ML[i], tId = MI[i];
      int hit = sc == match;
      if (ans == matched) { ML[i] = mLenLag + 1; MI[i] = mIdLag + hit; }
      else if (ans == xEnd) { ML[i] = XL[i - 1] + 1; MI[i] = XI[i - 1] + hit; }
      else { ML[i] = yLenLag + 1; MI[i] = yIdLag + hit; }
      mLenLag = tLen; mIdLag = tId;
      yLag = s1; yLenLag = s2; yIdLag = s3;
    }
    M[0] = ninf; ML[0] = j; MI[0] = 0;
    X[0] = ninf; XL[0] = j; XI[0] = 0;
    for (int i = 1; i < len1; i++) {
      int xBegin = M[i - 1] - (gap_open + gap_ext);
      int xCont = X[i - 1] - gap_ext;
      int ans = xBegin > xCont ? xBegin : xCont;
      X[i] = ans;
      if (ans == xBegin) { XL[i] = ML[i - 1] + 1; XI[i] = MI[i - 1]; }
      else { XL[i] = XL[i - 1] + 1; XI[i] = XI[i - 1]; }
    }
  }
  int e = len1 - 1;
  int sc = M[e] > X[e] ? M[e] : X[e];
  sc = sc > Y[e] ? sc : Y[e];
  int L, I;
  if (sc == M[e]) { L = ML[e]; I = MI[e]; }
  else if (sc == X[e]) { L = XL[e]; I = XI[e]; }
  else { L = YL[e]; I = YI[e]; }
  if (score_out) *score_out = sc;
  if (len_out) *len_out = L;
  if (ids_out) *ids_out = I;
  if (identity) *identity = (double)I / L;
  free(buf);
}
