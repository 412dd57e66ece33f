// features.hpp -- device-side K2 math: per-pair integer statistics of two k-mer histograms,
// the raw similarity features of src/cluster/src/Feature.cpp and the GLM decision of
// Trainer::get_close/filter/merge, all bit-exact with the reference build.
//
// For 8- and 16-bit histograms every feature is a function of four integer sums, computed
// with packed byte instructions (v_sad_u8: sum |p-q| of 4 bytes, v_dot4_u32_u8: sum p*q):
//   Smin = sum min(p,q) = (mag_p + mag_q - Sabs) / 2          intersection, kulczynski2, distance
//   Sabs = sum |p-q|                                          manhattan
//   Sdot = sum p*q, with per-point sum p^2 precomputed        pearson:
//     sum (p-ap)(q-aq) = Sdot - aq*mag_p - ap*mag_q + B*ap*aq  (exact int64 identity)
// 32/64-bit histograms fall back to a per-bin loop that mirrors the reference's C++ types
// including its unsigned wrap-arounds (raw_exact).
#pragma once
#include "mcgpu.hpp"

namespace mcg {

struct PS {  // pair statistics
  uint64_t smin, sabs, sdot;
};

struct PInfo {
  uint64_t mag, sumsq, len;
};

template <typename T>
struct Acc;

template <>
struct Acc<uint8_t> {
  // four independent accumulator chains per sum (one per 32-bit word of a chunk): a row's 64
  // byte instructions of each kind are four dependent chains of 16, not one of 64
  uint32_t s4[4] = {0, 0, 0, 0}, d4[4] = {0, 0, 0, 0};
  uint32_t sad = 0, dot = 0;  // valid after fold() (finish / reduce16 fold themselves)
  __device__ __forceinline__ void add(const uint4 &a, const uint4 &b) {
    s4[0] = __builtin_amdgcn_sad_u8(a.x, b.x, s4[0]);
    s4[1] = __builtin_amdgcn_sad_u8(a.y, b.y, s4[1]);
    s4[2] = __builtin_amdgcn_sad_u8(a.z, b.z, s4[2]);
    s4[3] = __builtin_amdgcn_sad_u8(a.w, b.w, s4[3]);
    d4[0] = __builtin_amdgcn_udot4(a.x, b.x, d4[0], false);
    d4[1] = __builtin_amdgcn_udot4(a.y, b.y, d4[1], false);
    d4[2] = __builtin_amdgcn_udot4(a.z, b.z, d4[2], false);
    d4[3] = __builtin_amdgcn_udot4(a.w, b.w, d4[3], false);
  }
  __device__ __forceinline__ void add_sad(const uint4 &a, const uint4 &b) {  // (sum |p - q| only)
    s4[0] = __builtin_amdgcn_sad_u8(a.x, b.x, s4[0]);
    s4[1] = __builtin_amdgcn_sad_u8(a.y, b.y, s4[1]);
    s4[2] = __builtin_amdgcn_sad_u8(a.z, b.z, s4[2]);
    s4[3] = __builtin_amdgcn_sad_u8(a.w, b.w, s4[3]);
  }
  __device__ __forceinline__ void fold() {
    sad += (s4[0] + s4[1]) + (s4[2] + s4[3]);
    dot += (d4[0] + d4[1]) + (d4[2] + d4[3]);
    s4[0] = s4[1] = s4[2] = s4[3] = 0;
    d4[0] = d4[1] = d4[2] = d4[3] = 0;
  }
  __device__ __forceinline__ void reduce16() {
    fold();
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) {
      sad += __shfl_xor(sad, o, 64);
      dot += __shfl_xor(dot, o, 64);
    }
  }
  __device__ __forceinline__ void wave_reduce();  // the whole wave's sums in every lane
  __device__ __forceinline__ PS finish(uint64_t magp, uint64_t magq) const {
    const uint32_t sa = sad + (s4[0] + s4[1]) + (s4[2] + s4[3]);
    const uint32_t dt = dot + (d4[0] + d4[1]) + (d4[2] + d4[3]);
    PS s;
    s.sabs = sa;
    s.smin = (magp + magq - sa) >> 1;
    s.sdot = dt;
    return s;
  }
};

// ---- wave reductions on DPP (VALU lane moves, no LDS permute) -----------------------------
// quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror, then row_bcast:15 (rows 1, 3)
// and row_bcast:31 (rows 2, 3): the reduction of all 64 lanes ends in lane 63.  Lanes of rows a
// broadcast does not write keep `old`.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp_mv(uint32_t old, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROWS, 0xf, false);
}
#define MCG_DPP_STEPS(X) X(0xB1, 0xf) X(0x4E, 0xf) X(0x141, 0xf) X(0x140, 0xf) X(0x142, 0xa) X(0x143, 0xc)

// sum of v over the wave, valid in lane 63 (wave_sum32_all: in every lane, via readlane)
__device__ __forceinline__ uint32_t wave_sum32_l63(uint32_t v) {
#define MCG_SUM_STEP(C, R) v += dpp_mv<C, R>(0u, v);
  MCG_DPP_STEPS(MCG_SUM_STEP)
#undef MCG_SUM_STEP
  return v;
}
__device__ __forceinline__ uint32_t wave_sum32_all(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_sum32_l63(v), 63);
}
__device__ __forceinline__ uint64_t wave_sum64_all(uint64_t v) {
#define MCG_SUM64_STEP(C, R)                                                       \
  {                                                                                \
    const uint64_t o = ((uint64_t)dpp_mv<C, R>(0u, (uint32_t)(v >> 32)) << 32) |   \
                       dpp_mv<C, R>(0u, (uint32_t)v);                              \
    v += o;                                                                        \
  }
  MCG_DPP_STEPS(MCG_SUM64_STEP)
#undef MCG_SUM64_STEP
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
  return ((uint64_t)hi << 32) | lo;
}
// max / min of a double over the wave (DPP moves of the two halves + v_max_f64 / v_min_f64),
// in every lane; the value is one of the inputs, bit for bit
template <bool MAX>
__device__ __forceinline__ double wave_ext_f64_all(double v) {
#define MCG_EXT_STEP(C, R)                                                                            \
  {                                                                                                   \
    const uint64_t vb = __builtin_bit_cast(uint64_t, v);                                              \
    const uint64_t ov = ((uint64_t)dpp_mv<C, R>((uint32_t)(vb >> 32), (uint32_t)(vb >> 32)) << 32) |  \
                        dpp_mv<C, R>((uint32_t)vb, (uint32_t)vb);                                     \
    const double o = __builtin_bit_cast(double, ov);                                                  \
    v = MAX ? __builtin_fmax(v, o) : __builtin_fmin(v, o);                                            \
  }
  MCG_DPP_STEPS(MCG_EXT_STEP)
#undef MCG_EXT_STEP
  const uint64_t vb = __builtin_bit_cast(uint64_t, v);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(vb >> 32), 63) << 32) |
                                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)vb, 63));
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int L) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), L) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, L);
}

// the best (value, key) pair of the wave under a strict total order `better(a, ka, b, kb)`,
// returned in every lane; V is double or uint64_t, keys uint64_t
template <typename V, typename Better>
__device__ __forceinline__ void wave_best_all(V &v, uint64_t &k, Better better) {
#define MCG_BEST_STEP(C, R)                                                                          \
  {                                                                                                  \
    const uint64_t vb = __builtin_bit_cast(uint64_t, v);                                             \
    const uint64_t ov = ((uint64_t)dpp_mv<C, R>((uint32_t)(vb >> 32), (uint32_t)(vb >> 32)) << 32) | \
                        dpp_mv<C, R>((uint32_t)vb, (uint32_t)vb);                                    \
    const uint64_t ok = ((uint64_t)dpp_mv<C, R>((uint32_t)(k >> 32), (uint32_t)(k >> 32)) << 32) |   \
                        dpp_mv<C, R>((uint32_t)k, (uint32_t)k);                                      \
    const V ovv = __builtin_bit_cast(V, ov);                                                         \
    if (better(ovv, ok, v, k)) {                                                                     \
      v = ovv;                                                                                       \
      k = ok;                                                                                        \
    }                                                                                                \
  }
  MCG_DPP_STEPS(MCG_BEST_STEP)
#undef MCG_BEST_STEP
  const uint64_t vb = __builtin_bit_cast(uint64_t, v);
  const uint64_t r = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(vb >> 32), 63) << 32) |
                     (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)vb, 63);
  v = __builtin_bit_cast(V, r);
  k = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(k >> 32), 63) << 32) |
      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)k, 63);
}

__device__ __forceinline__ void Acc<uint8_t>::wave_reduce() {
  fold();
  sad = wave_sum32_all(sad);
  dot = wave_sum32_all(dot);
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int o) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  lo = __shfl_xor(lo, o, 64);
  hi = __shfl_xor(hi, o, 64);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  lo = __shfl(lo, src, 64);
  hi = __shfl(hi, src, 64);
  return ((uint64_t)hi << 32) | lo;
}

// Generic element accumulator (16/32/64-bit bins): Smin, Sabs (mod 2^32 like `int sum`), Sdot.
template <typename T>
struct Acc {
  uint64_t smin = 0, sabs = 0, sdot = 0;
  __device__ __forceinline__ void add(const uint4 &a, const uint4 &b) {
    const T *pa = reinterpret_cast<const T *>(&a);
    const T *pb = reinterpret_cast<const T *>(&b);
#pragma unroll
    for (int i = 0; i < (int)(16 / sizeof(T)); i++) {
      uint64_t x = pa[i], y = pb[i];
      smin += x < y ? x : y;
      sabs += (uint32_t)(x > y ? x - y : y - x);
      sdot += x * y;
    }
  }
  __device__ __forceinline__ void add_sad(const uint4 &a, const uint4 &b) { add(a, b); }
  __device__ __forceinline__ void reduce16() {
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) {
      smin += shfl_xor64(smin, o);
      sabs += shfl_xor64(sabs, o);
      sdot += shfl_xor64(sdot, o);
    }
  }
  __device__ __forceinline__ void wave_reduce() {
    smin = wave_sum64_all(smin);
    sabs = wave_sum64_all(sabs);
    sdot = wave_sum64_all(sdot);
  }
  __device__ __forceinline__ PS finish(uint64_t, uint64_t) const { return PS{smin, sabs, sdot}; }
};

// DivergencePoint::distance (DivergencePoint.cpp:68-81): trunc_u64(fma(-f,f,1)*1e4)
__device__ __forceinline__ uint64_t distance_key(uint64_t smin, uint64_t magp, uint64_t magq) {
  uint64_t dist = smin * 2;
  double frac = (double)dist / (double)(magp + magq);
  return (uint64_t)(__builtin_fma(-frac, frac, 1.0) * 10000.0);
}

// Feature.cpp:273-294 via the integer identity (8/16-bit bins: dp = p - ap is exact int math).
__device__ __forceinline__ double pearson_fast(const PS &s, const PInfo &p, const PInfo &q, int B) {
  double dap = (double)p.mag / B, daq = (double)q.mag / B;
  int64_t ap = (int)round(dap), aq = (int)round(daq);
  int64_t mp = (int64_t)p.mag, mq = (int64_t)q.mag, b = B;
  int64_t dot = (int64_t)s.sdot - aq * mp - ap * mq + b * ap * aq;
  int64_t np = (int64_t)p.sumsq - 2 * ap * mp + b * ap * ap;
  int64_t nq = (int64_t)q.sumsq - 2 * aq * mq + b * aq * aq;
  double prod = (double)(int64_t)((uint64_t)np * (uint64_t)nq);
  return (double)dot / sqrt(0.5 < prod ? prod : 0.5);
}

__device__ __forceinline__ double raw_fast(uint16_t f, const PS &s, const PInfo &p, const PInfo &q, int B) {
  switch (f) {
    case MC_FEAT_LD: return (double)(p.len > q.len ? p.len - q.len : q.len - p.len);
    case MC_FEAT_MANHATTAN: return (double)(int32_t)(uint32_t)s.sabs;
    case MC_FEAT_INTERSECTION: return (double)(s.smin * 2) / (double)(p.mag + q.mag);
    case MC_FEAT_PEARSON: return pearson_fast(s, p, q, B);
    case MC_FEAT_KULCZYNSKI2: {
      double ap = (double)p.mag / B, aq = (double)q.mag / B;
      double coeff = ((double)B * (ap + aq)) / ((2.0 * ap) * aq);
      return coeff * (double)s.smin;
    }
    default: return __builtin_nan("");
  }
}

// Per-bin restatement for 32/64-bit bins (mirrors oracle mco_raw / Feature.cpp exactly).
template <typename T>
__device__ double raw_exact(uint16_t f, const T *p, const T *q, int B, const PInfo &pi, const PInfo &qi) {
  if (f == MC_FEAT_LD) return (double)(pi.len > qi.len ? pi.len - qi.len : qi.len - pi.len);
  if (f == MC_FEAT_MANHATTAN) {
    uint32_t sum = 0;
    for (int i = 0; i < B; i++) sum += (uint32_t)(p[i] > q[i] ? p[i] - q[i] : q[i] - p[i]);
    return (double)(int32_t)sum;
  }
  if (f == MC_FEAT_INTERSECTION || f == MC_FEAT_KULCZYNSKI2) {
    uint64_t d = 0, ms = 0;
    for (int i = 0; i < B; i++) {
      T m = p[i] < q[i] ? p[i] : q[i];
      d += (uint64_t)(T)(m * 2);  // `2 * std::min` in T (unsigned wrap for 32/64-bit T)
      ms += m;
    }
    if (f == MC_FEAT_INTERSECTION) return (double)d / (double)(pi.mag + qi.mag);
    double ap = (double)pi.mag / B, aq = (double)qi.mag / B;
    double coeff = ((double)B * (ap + aq)) / ((2.0 * ap) * aq);
    return coeff * (double)ms;
  }
  if (f == MC_FEAT_PEARSON) {
    double dap = (double)pi.mag / B, daq = (double)qi.mag / B;
    int ap = (int)round(dap), aq = (int)round(daq);
    uint64_t dot = 0, np = 0, nq = 0;
    for (int i = 0; i < B; i++) {
      int64_t dp, dq;
      if (sizeof(T) == 4) {
        dp = (int64_t)(uint64_t)(uint32_t)((uint32_t)p[i] - (uint32_t)ap);
        dq = (int64_t)(uint64_t)(uint32_t)((uint32_t)q[i] - (uint32_t)aq);
      } else {
        dp = (int64_t)((uint64_t)p[i] - (uint64_t)(int64_t)ap);
        dq = (int64_t)((uint64_t)q[i] - (uint64_t)(int64_t)aq);
      }
      np += (uint64_t)dp * (uint64_t)dp;
      nq += (uint64_t)dq * (uint64_t)dq;
      dot += (uint64_t)dp * (uint64_t)dq;
    }
    double prod = (double)(int64_t)(np * nq);
    return (double)(int64_t)dot / sqrt(0.5 < prod ? prod : 0.5);
  }
  return __builtin_nan("");
}

__device__ __forceinline__ double pick8(const double (&v)[MC_MAX_SINGLE], int idx) {
  double r = 0;
#pragma unroll
  for (int i = 0; i < MC_MAX_SINGLE; i++) r = (idx == i) ? v[i] : r;
  return r;
}

// normalize_cache (Feature.cpp:41-52) + operator() (Feature.h:69-88) + the fma GLM sum of
// Trainer.cpp:84-95.  Returns the decision round(1/(1+exp(-sum))) == 1 as sum >= thr.
__device__ __forceinline__ int classify_raw(const DevClassifier &C, double (&raw)[MC_MAX_SINGLE], double *c0,
                                            double *sum_out) {
  const mc_classifier &c = C.c;
#pragma unroll
  for (int i = 0; i < MC_MAX_SINGLE; i++) {
    if (i < c.n_single) {
      double val = (raw[i] - c.mins[i]) / (c.maxs[i] - c.mins[i]);
      raw[i] = c.is_sim[i] ? val : 1 - val;
    }
  }
  double sum = c.weights[0];
  double first = 0;
  for (int col = 0; col < c.n_combo; col++) {
    double prod = 1;
    for (int j = 0; j < c.combo_len[col]; j++) {
      double v = pick8(raw, c.combo_idx[col][j]);
      if (c.combo_kind[col] == MC_COMBO_SELF) prod *= v;
      else prod *= v * v;
    }
    if (col == 0) first = prod;
    sum = __builtin_fma(c.weights[col + 1], prod, sum);
  }
  *c0 = first;
  if (sum_out) *sum_out = sum;
  return sum >= C.thr;
}

// Per-histogram terms of pearson / kulczynski2 (Feature.cpp:206-220, 273-294) that do not
// depend on the pair: computed once per candidate (or per centre and step) instead of per pair.
struct PTerms {
  int64_t ap;  // (int)round(mag / B)
  int64_t np;  // sum (p - ap)^2 = sumsq - 2 ap mag + B ap^2 (8/16-bit bins: exact)
  double da;   // mag / B
};
__device__ __forceinline__ PTerms pterms(uint64_t mag, uint64_t sumsq, int B) {
  const double da = (double)mag / B;
  const int64_t a = (int)round(da), m = (int64_t)mag, b = B;
  return PTerms{a, (int64_t)sumsq - 2 * a * m + b * a * a, da};
}

// classify_raw for the trainer's feature set (DevClassifier::layout 3 / 4), 8/16-bit bins:
// the same IEEE operations in the same order (raw_fast, normalize_cache, operator(), the fma
// GLM sum), with the pair-independent terms taken from PTerms -- a few divisions per pair
// instead of the generic form's selects and loops.
__device__ __forceinline__ int classify_std(const DevClassifier &C, const PS &s, const PInfo &p, const PTerms &tp,
                                            const PInfo &q, const PTerms &tq, int B, double *c0) {
  const mc_classifier &c = C.c;
  double v[5];
  v[0] = (double)(p.len > q.len ? p.len - q.len : q.len - p.len);             // LD
  v[1] = (double)(s.smin * 2) / (double)(p.mag + q.mag);                        // INTERSECTION
  v[2] = (double)(int32_t)(uint32_t)s.sabs;                                     // MANHATTAN
  {                                                                             // PEARSON
    const int64_t dot = (int64_t)s.sdot - tq.ap * (int64_t)p.mag - tp.ap * (int64_t)q.mag + (int64_t)B * tp.ap * tq.ap;
    const double prod = (double)(int64_t)((uint64_t)tp.np * (uint64_t)tq.np);
    v[3] = (double)dot / sqrt(0.5 < prod ? prod : 0.5);
  }
  const bool kul = C.layout == 4;
  if (kul) v[4] = (((double)B * (tp.da + tq.da)) / ((2.0 * tp.da) * tq.da)) * (double)s.smin;  // KULCZYNSKI2
#pragma unroll
  for (int i = 0; i < 5; i++) {
    if (i == 4 && !kul) break;
    const double val = (v[i] - c.mins[i]) / (c.maxs[i] - c.mins[i]);
    v[i] = c.is_sim[i] ? val : 1 - val;
  }
  const double a0 = v[0] * v[1];
  const double a1 = (v[0] * v[0]) * (v[2] * v[2]);
  const double a2 = v[3];
  double sum = c.weights[0];
  sum = __builtin_fma(c.weights[1], a0, sum);
  sum = __builtin_fma(c.weights[2], a1, sum);
  sum = __builtin_fma(c.weights[3], a2, sum);
  if (kul) sum = __builtin_fma(c.weights[4], (v[0] * v[0]) * (v[4] * v[4]), sum);
  *c0 = a0;
  return sum >= C.thr;
}

// Division-light decision for the accumulation workers (the same decision and combo 0 as
// classify_std, bit for bit).  Combo 0 (LD x INTERSECTION) is computed exactly: the first
// maximum of get_close compares its values.  The other GLM terms are evaluated with
// reciprocals (two Newton steps: a few ulps) and normalised by the host's RN(1/range); the
// decision is taken from that sum only when it clears the threshold by a margin that bounds
// the difference to the exact sum many times over (every approximate quotient is within
// 2^-48 relative of the exact one; the margin allows 2^-40 on every term).  Otherwise, or for
// any non-finite value, classify_std decides.
// (two Newton steps: from any hardware estimate within 2^-14 to a few ulps)
__device__ __forceinline__ double rcp_nr(double b) {
  double y = __builtin_amdgcn_rcp(b);
  y = __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
  return __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
}
__device__ __forceinline__ double rsq_nr(double a) {
  double y = __builtin_amdgcn_rsq(a);
  const double h = 0.5 * a;
  y = y * __builtin_fma(-h * y, y, 1.5);
  return y * __builtin_fma(-h * y, y, 1.5);
}
__device__ __forceinline__ int classify_fast(const DevClassifier &C, const FastCls &F, const PS &s, const PInfo &p,
                                             const PTerms &tp, const PInfo &q, const PTerms &tq, int B, double *c0) {
  const mc_classifier &c = C.c;
  const bool kul = C.layout == 4;
  // exact: LD and INTERSECTION, normalised, and combo 0
  double v0 = (double)(p.len > q.len ? p.len - q.len : q.len - p.len);
  double v1 = (double)(s.smin * 2) / (double)(p.mag + q.mag);
  {
    const double n0 = (v0 - c.mins[0]) / (c.maxs[0] - c.mins[0]), n1 = (v1 - c.mins[1]) / (c.maxs[1] - c.mins[1]);
    v0 = c.is_sim[0] ? n0 : 1 - n0;
    v1 = c.is_sim[1] ? n1 : 1 - n1;
  }
  const double a0 = v0 * v1;
  *c0 = a0;
  // approximate: MANHATTAN, PEARSON (, KULCZYNSKI2)
  double r[5], e[5], v[5];
  r[2] = (double)(int32_t)(uint32_t)s.sabs;
  {
    const int64_t dot = (int64_t)s.sdot - tq.ap * (int64_t)p.mag - tp.ap * (int64_t)q.mag + (int64_t)B * tp.ap * tq.ap;
    const double prod = (double)(int64_t)((uint64_t)tp.np * (uint64_t)tq.np);
    const double pr = 0.5 < prod ? prod : 0.5;
    r[3] = (double)dot * rsq_nr(pr);
  }
  r[4] = kul ? ((double)B * (tp.da + tq.da)) * rcp_nr((2.0 * tp.da) * tq.da) * (double)s.smin : 0.0;
  const int nf = kul ? 5 : 4;
#pragma unroll
  for (int i = 2; i < 5; i++) {
    if (i >= nf) {
      v[i] = e[i] = 0.0;
      continue;
    }
    const double n = (r[i] - c.mins[i]) * F.rinv[i];
    v[i] = F.noff[i] + F.nsgn[i] * n;
    // |approximate - exact| of v[i]: 2^-40 of (|raw| + |min|) / |range| + 2^-40 (|v| + 1)
    e[i] = 0x1p-40 * ((__builtin_fabs(r[i]) + __builtin_fabs(c.mins[i])) * __builtin_fabs(F.rinv[i]) +
                      __builtin_fabs(v[i]) + 1.0);
  }
  const double q00 = v0 * v0;
  const double a1 = q00 * (v[2] * v[2]);
  const double a2 = v[3];
  const double a3 = q00 * (v[4] * v[4]);
  double sum = c.weights[0];
  sum = __builtin_fma(c.weights[1], a0, sum);
  sum = __builtin_fma(c.weights[2], a1, sum);
  sum = __builtin_fma(c.weights[3], a2, sum);
  if (kul) sum = __builtin_fma(c.weights[4], a3, sum);
  const double d1 = q00 * (2.0 * __builtin_fabs(v[2]) + e[2]) * e[2] + 0x1p-40 * __builtin_fabs(a1);
  const double d3 = q00 * (2.0 * __builtin_fabs(v[4]) + e[4]) * e[4] + 0x1p-40 * __builtin_fabs(a3);
  const double mag = __builtin_fabs(c.weights[0]) + __builtin_fabs(c.weights[1] * a0) + __builtin_fabs(c.weights[2] * a1) +
                     __builtin_fabs(c.weights[3] * a2) + (kul ? __builtin_fabs(c.weights[4] * a3) : 0.0);
  const double margin = 2.0 * (__builtin_fabs(c.weights[2]) * d1 + __builtin_fabs(c.weights[3]) * e[3] +
                               (kul ? __builtin_fabs(c.weights[4]) * d3 : 0.0)) +
                        0x1p-40 * mag;
  if (__builtin_isfinite(sum) && __builtin_isfinite(margin) && __builtin_isfinite(a0)) {
    if (sum - margin >= C.thr) return 1;
    if (sum + margin < C.thr) return 0;
  }
  double cx;
  return classify_std(C, s, p, tp, q, tq, B, &cx);
}

// ---- the accumulation workers' short form (8-bit bins, every magnitude < 2^24) ------------
// RN(a / b) for a constant b from the host's y = RN(1 / b): q0 = RN(a y), r = a - b q0 (exact
// by fma), RN(q0 + r y) is the correctly rounded quotient (Markstein's theorem; b, y, a and the
// remainder normal: FastCls::mk and the raw features' ranges keep them so).
__device__ __forceinline__ double mk_div(double a, double b, double y) {
  const double q0 = a * y;
  return __builtin_fma(__builtin_fma(-q0, b, a), y, q0);
}
// pterms with the division by B as mk_div (the same PTerms, bit for bit)
__device__ __forceinline__ PTerms pterms_mk(uint64_t mag, uint64_t sumsq, int B, double rB) {
  const double da = mk_div((double)mag, (double)B, rB);
  const int64_t a = (int)round(da), m = (int64_t)mag, b = B;
  return PTerms{a, (int64_t)sumsq - 2 * a * m + b * a * a, da};
}
// a histogram's terms in 32 bits; ok = they bound every integer of the pair arithmetic below
// 2^53 (magnitude < 2^24, length < 2^31, sum (p - ap)^2 < 2^26), so doubles hold it exactly
struct PSm {
  uint32_t mag, len, ap, np;
  bool ok;
};
__device__ __forceinline__ PSm psmall(const PInfo &p, const PTerms &t) {
  const bool ok = p.mag < (1ull << 24) && p.len < (1ull << 31) && t.ap >= 0 && t.np >= 0 && t.np < (1ll << 26);
  return PSm{(uint32_t)p.mag, (uint32_t)p.len, (uint32_t)t.ap, (uint32_t)t.np, ok};
}
// classify_small's constants in one 208-byte block.  The accumulation workers keep a copy in LDS
// and read it with the candidate's row (one LDS wait), instead of re-loading the kernel
// arguments: the persistent kernel's loop holds too many uniform values for them all to stay in
// scalar registers, and each reload was a scalar-memory round trip on the scoring chain.
struct SmallK {
  double mins[5], range[2], rinv[5], noff[3], nsgn[3], w[5], thr;  // noff / nsgn: features 2..4
  int32_t sim0, sim1, kul, pad;
};
static_assert(sizeof(SmallK) % 16 == 0, "SmallK is copied as 16-byte words");
__host__ __device__ __forceinline__ SmallK make_smallk(const DevClassifier &C, const FastCls &F) {
  SmallK k;
  for (int i = 0; i < 5; i++) {
    k.mins[i] = C.c.mins[i];
    k.rinv[i] = F.rinv[i];
    k.w[i] = C.c.weights[i];
  }
  for (int i = 0; i < 2; i++) k.range[i] = F.range[i];
  for (int i = 0; i < 3; i++) {
    k.noff[i] = F.noff[2 + i];
    k.nsgn[i] = F.nsgn[2 + i];
  }
  k.thr = C.thr;
  k.sim0 = C.c.is_sim[0];
  k.sim1 = C.c.is_sim[1];
  k.kul = C.layout == 4;
  k.pad = 0;
  return k;
}

// classify_fast from the 8-bit sums (sad = sum |p - q|, dot = sum p q) and the PSm terms of
// both histograms (kq = mag_q - B aq): LD, INTERSECTION and combo 0 exact (the LD / INT
// normalisations as mk_div by the host's RN(1 / range)), MANHATTAN exact, PEARSON's integers
// exact in doubles (every one below 2^53), the decision by classify_fast's margin.  *undecided:
// the caller decides by classify_std.  Every value it returns or stores is classify_std's.
__device__ __forceinline__ int classify_small(const SmallK &K, uint32_t sad, uint32_t dot, const PSm &p, const PSm &q,
                                              double kq, double dap, double daq, int B, double *c0, bool *undecided) {
  const bool kul = K.kul != 0;
  const uint32_t dl = p.len > q.len ? p.len - q.len : q.len - p.len;
  const uint32_t ms = p.mag + q.mag, s2 = ms - sad;  // s2 = 2 Smin
  double v0 = mk_div((double)dl - K.mins[0], K.range[0], K.rinv[0]);
  double v1 = mk_div((double)s2 / (double)ms - K.mins[1], K.range[1], K.rinv[1]);
  v0 = K.sim0 ? v0 : 1 - v0;
  v1 = K.sim1 ? v1 : 1 - v1;
  const double a0 = v0 * v1;
  *c0 = a0;
  double r[5], e[5], v[5];
  r[2] = (double)(int32_t)sad;
  {
    const double d = __builtin_fma(-(double)p.ap, kq, __builtin_fma(-(double)q.ap, (double)p.mag, (double)dot));
    const double prod = (double)p.np * (double)q.np;
    const double pr = 0.5 < prod ? prod : 0.5;
    r[3] = d * rsq_nr(pr);
  }
  r[4] = kul ? ((double)B * (dap + daq)) * rcp_nr((2.0 * dap) * daq) * (double)(s2 >> 1) : 0.0;
  const int nf = kul ? 5 : 4;
#pragma unroll
  for (int i = 2; i < 5; i++) {
    if (i >= nf) {
      v[i] = e[i] = 0.0;
      continue;
    }
    const double n = (r[i] - K.mins[i]) * K.rinv[i];
    v[i] = K.noff[i - 2] + K.nsgn[i - 2] * n;
    e[i] = 0x1p-40 * ((__builtin_fabs(r[i]) + __builtin_fabs(K.mins[i])) * __builtin_fabs(K.rinv[i]) +
                      __builtin_fabs(v[i]) + 1.0);
  }
  const double q00 = v0 * v0;
  const double a1 = q00 * (v[2] * v[2]);
  const double a2 = v[3];
  const double a3 = q00 * (v[4] * v[4]);
  double sum = K.w[0];
  sum = __builtin_fma(K.w[1], a0, sum);
  sum = __builtin_fma(K.w[2], a1, sum);
  sum = __builtin_fma(K.w[3], a2, sum);
  if (kul) sum = __builtin_fma(K.w[4], a3, sum);
  const double d1 = q00 * (2.0 * __builtin_fabs(v[2]) + e[2]) * e[2] + 0x1p-40 * __builtin_fabs(a1);
  const double d3 = q00 * (2.0 * __builtin_fabs(v[4]) + e[4]) * e[4] + 0x1p-40 * __builtin_fabs(a3);
  const double mag = __builtin_fabs(K.w[0]) + __builtin_fabs(K.w[1] * a0) + __builtin_fabs(K.w[2] * a1) +
                     __builtin_fabs(K.w[3] * a2) + (kul ? __builtin_fabs(K.w[4] * a3) : 0.0);
  const double margin = 2.0 * (__builtin_fabs(K.w[2]) * d1 + __builtin_fabs(K.w[3]) * e[3] +
                               (kul ? __builtin_fabs(K.w[4]) * d3 : 0.0)) +
                        0x1p-40 * mag;
  *undecided = false;
  if (__builtin_isfinite(sum) && __builtin_isfinite(margin) && __builtin_isfinite(a0)) {
    if (sum - margin >= K.thr) return 1;
    if (sum + margin < K.thr) return 0;
  }
  *undecided = true;
  return 0;
}
__device__ __forceinline__ int classify_small(const DevClassifier &C, const FastCls &F, uint32_t sad, uint32_t dot,
                                              const PSm &p, const PSm &q, double kq, double dap, double daq, int B,
                                              double *c0, bool *undecided) {
  return classify_small(make_smallk(C, F), sad, dot, p, q, kq, dap, daq, B, c0, undecided);
}
// the SmallK block from LDS: volatile 16-byte reads, so they are issued where the scoring needs
// them (beside the row's reads) and never hoisted into registers across the worker's loop
__device__ __forceinline__ SmallK lds_smallk(const SmallK *p) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const volatile __attribute__((address_space(3))) v4u *q = (const volatile __attribute__((address_space(3))) v4u *)p;
  v4u w[sizeof(SmallK) / 16];
#pragma unroll
  for (int i = 0; i < (int)(sizeof(SmallK) / 16); i++) w[i] = q[i];
  SmallK k;
  __builtin_memcpy(&k, w, sizeof(SmallK));
  return k;
}

template <typename T>
__device__ __forceinline__ uint4 ld16(const uint8_t *row, int ch) {
  return reinterpret_cast<const uint4 *>(row)[ch];
}

// Integer pair statistics for the 64 candidates of one wave, 16 lanes per histogram row so
// every load instruction reads four whole 256-byte rows (1 KiB) contiguously.  Lane l ends up
// with the statistics of the pair it owns (my_a vs my_b, or my_a vs the LDS-resident centre).
// Rows of at most 16 chunks (8-bit bins up to k = 4): one chunk per lane and row, so the 16
// passes' loads are independent -- issued CEN ? 8 : 4 passes at a time (their rows and
// magnitudes in flight together, clamped addresses for the idle lanes) instead of one round
// trip per pass.
template <typename T, int BATCH, bool CEN>
__device__ __forceinline__ PS wave_pair_stats_short(const HistView &H, uint32_t my_a, uint32_t my_b, bool valid,
                                                    const uint4 *centre_lds, uint64_t centre_mag, int nch) {
  const int lane = threadIdx.x & 63, group = lane >> 4, lig = lane & 15;
  const int ch = lig < nch ? lig : 0;
  PS mine{0, 0, 0};
  for (int p0 = 0; p0 < 16; p0 += BATCH) {
    uint4 ra[BATCH], rb[BATCH];
    uint64_t ma[BATCH], mb[BATCH];
    bool vv[BATCH];
#pragma unroll
    for (int u = 0; u < BATCH; u++) {
      const int cl = (p0 + u) * 4 + group;
      const uint32_t a = __shfl(my_a, cl, 64);
      const int v = __shfl((int)valid, cl, 64);
      vv[u] = v != 0;
      const uint32_t a0 = v ? a : 0u;  // (row 0 stands in for an idle group: a valid address)
      ra[u] = ld16<T>(H.hist + (uint64_t)a0 * H.pitch, ch);
      ma[u] = H.mag[a0];
      if constexpr (CEN) {
        rb[u] = centre_lds[ch];
        mb[u] = centre_mag;
      } else {
        const uint32_t b = __shfl(my_b, cl, 64), b0 = v ? b : 0u;
        rb[u] = ld16<T>(H.hist + (uint64_t)b0 * H.pitch, ch);
        mb[u] = H.mag[b0];
      }
    }
#pragma unroll
    for (int u = 0; u < BATCH; u++) {
      Acc<T> acc;
      if (vv[u] && lig < nch) acc.add(ra[u], rb[u]);
      acc.reduce16();
      const PS s = acc.finish(vv[u] ? ma[u] : 0, CEN ? mb[u] : (vv[u] ? mb[u] : 0));
      // lane l takes the result of pass l/4 from the leader of group l%4
      const int src = (lane & 3) * 16;
      const uint64_t x0 = shfl64(s.smin, src), x1 = shfl64(s.sabs, src), x2 = shfl64(s.sdot, src);
      if (p0 + u == (lane >> 2)) mine = PS{x0, x1, x2};
    }
  }
  return mine;
}

template <typename T>
__device__ __forceinline__ PS wave_pair_stats(const HistView &H, uint32_t my_a, uint32_t my_b, bool valid,
                                              const uint4 *centre_lds, uint64_t centre_mag) {
  const int lane = threadIdx.x & 63, group = lane >> 4, lig = lane & 15;
  const int nch = (int)((H.B * (int)sizeof(T) + 15) / 16);
  if (nch <= 16) {
    if (centre_lds) return wave_pair_stats_short<T, 8, true>(H, my_a, my_b, valid, centre_lds, centre_mag, nch);
    return wave_pair_stats_short<T, 4, false>(H, my_a, my_b, valid, centre_lds, centre_mag, nch);
  }
  PS mine{0, 0, 0};
  for (int pass = 0; pass < 16; pass++) {
    const int cl = pass * 4 + group;
    uint32_t a = __shfl(my_a, cl, 64);
    uint32_t b = __shfl(my_b, cl, 64);
    int v = __shfl((int)valid, cl, 64);
    Acc<T> acc;
    if (v) {
      const uint8_t *ra = H.hist + (uint64_t)a * H.pitch;
      if (centre_lds) {
        for (int ch = lig; ch < nch; ch += 16) acc.add(ld16<T>(ra, ch), centre_lds[ch]);
      } else {
        const uint8_t *rb = H.hist + (uint64_t)b * H.pitch;
        for (int ch = lig; ch < nch; ch += 16) acc.add(ld16<T>(ra, ch), ld16<T>(rb, ch));
      }
    }
    acc.reduce16();
    uint64_t ma = v ? H.mag[a] : 0;
    uint64_t mb = centre_lds ? centre_mag : (v ? H.mag[b] : 0);
    PS s = acc.finish(ma, mb);
    // lane l takes the result of pass l/4 from the leader of group l%4
    const int src = (lane & 3) * 16;
    uint64_t x0 = shfl64(s.smin, src), x1 = shfl64(s.sabs, src), x2 = shfl64(s.sdot, src);
    if (pass == (lane >> 2)) mine = PS{x0, x1, x2};
  }
  return mine;
}

// ---------------------------------------------------------------------------------------
// get_mean / Trainer::closest for 8/16-bit bins (ClusterFactory.cpp:382-425, Trainer.cpp:351-365).
// With m_b = S_b / M, (T)m_b = floor(S_b / M) = F_b and the per-bin re-truncated magnitude of
// distance_d equals sum_b (p_b + F_b) exactly (tests/test_identities.py), so
//   distance_d(p, mean) = 1e4 * fma(-f, f, 1),  f = 2*sum min(p_b, F_b) / (mag_p + sum F_b)
// is a SAD reduction of p against the packed integer mean F.
struct RowRef {  // chunk c of row r = base[r * rstride + c * cstride]
  const uint4 *base;
  uint64_t rstride, cstride;
  __device__ __forceinline__ uint4 chunk(uint64_t r, int c) const { return base[r * rstride + (uint64_t)c * cstride]; }
};

template <typename T>
__device__ __forceinline__ uint64_t elem(const RowRef &R, uint64_t r, int b) {
  constexpr int per = 16 / (int)sizeof(T);
  uint4 v = R.chunk(r, b / per);
  return reinterpret_cast<const T *>(&v)[b % per];
}

// Adds the histograms of rows[0..M) into sum[0..B) (u64; LDS or global).  Work items are
// (row, chunk) pairs so every thread issues independent 16-byte loads, then folds its chunk
// into the sums with LDS/global atomics -- no per-thread serial walk over the rows.
template <typename T, int NTH>
__device__ __forceinline__ void add_rows(const RowRef &R, const uint32_t *rows, uint32_t M, int nch, uint64_t *sum) {
  constexpr int per = 16 / (int)sizeof(T);
  if (nch * 2 <= NTH && (uint64_t)M * (sizeof(T) == 1 ? 0xffull : 0xffffull) <= 0xffffffffull && sizeof(T) <= 2) {
    // short rows: thread (chunk c, slice sl) adds its chunk over the rows q = sl (mod nsl) in
    // 32-bit registers, four rows' loads in flight, then one atomic per bin and thread -- nsl
    // per bin instead of M (every row adding to the same bins was M-way atomic contention)
    const int nsl = NTH / nch;
    for (int t = threadIdx.x; t < nch * nsl; t += NTH) {
      const int c = t % nch, sl = t / nch;
      uint32_t acc[per];
#pragma unroll
      for (int e = 0; e < per; e++) acc[e] = 0;
      uint32_t q = (uint32_t)sl;
      for (; q + 3u * (uint32_t)nsl < M; q += 4u * (uint32_t)nsl) {
        const uint4 v0 = R.chunk(rows[q], c), v1 = R.chunk(rows[q + (uint32_t)nsl], c),
                    v2 = R.chunk(rows[q + 2u * (uint32_t)nsl], c), v3 = R.chunk(rows[q + 3u * (uint32_t)nsl], c);
        const T *p0 = reinterpret_cast<const T *>(&v0), *p1 = reinterpret_cast<const T *>(&v1),
                *p2 = reinterpret_cast<const T *>(&v2), *p3 = reinterpret_cast<const T *>(&v3);
#pragma unroll
        for (int e = 0; e < per; e++) acc[e] += (uint32_t)p0[e] + (uint32_t)p1[e] + (uint32_t)p2[e] + (uint32_t)p3[e];
      }
      for (; q < M; q += (uint32_t)nsl) {
        const uint4 v = R.chunk(rows[q], c);
        const T *pv = reinterpret_cast<const T *>(&v);
#pragma unroll
        for (int e = 0; e < per; e++) acc[e] += pv[e];
      }
#pragma unroll
      for (int e = 0; e < per; e++)
        if (acc[e]) atomicAdd((unsigned long long *)&sum[c * per + e], (unsigned long long)acc[e]);
    }
    return;
  }
  const uint64_t items = (uint64_t)M * nch;
  for (uint64_t it = threadIdx.x; it < items; it += NTH) {
    const uint32_t q = (uint32_t)(it / nch);
    const int c = (int)(it % nch);
    const uint4 v = R.chunk(rows[q], c);
    const T *pv = reinterpret_cast<const T *>(&v);
#pragma unroll
    for (int e = 0; e < per; e++)
      if (pv[e]) atomicAdd((unsigned long long *)&sum[c * per + e], (unsigned long long)pv[e]);
  }
}

// Column sums for wide rows (>= 32 chunks): thread t owns chunks t, t + NTH, ... and adds them
// up over all M rows in registers (a wave reads 64 consecutive chunks of one row: 1 KiB
// contiguous), then stores its bins -- no atomics, which at B = 4,096 bins would be M x 4,096
// per workgroup.  Overwrites sum[0..B).
template <typename T, int NTH, typename S>
__device__ __forceinline__ void add_rows_owned_as(const RowRef &R, const uint32_t *rows, uint32_t M, int nch, int B,
                                                  uint64_t *sum) {
  constexpr int per = 16 / (int)sizeof(T);
  for (int c = threadIdx.x; c < nch; c += NTH) {
    S acc[per];
#pragma unroll
    for (int e = 0; e < per; e++) acc[e] = 0;
    uint32_t q = 0;
    for (; q + 4 <= M; q += 4) {  // four rows' loads in flight
      const uint4 v0 = R.chunk(rows[q], c), v1 = R.chunk(rows[q + 1], c), v2 = R.chunk(rows[q + 2], c),
                  v3 = R.chunk(rows[q + 3], c);
      const T *p0 = reinterpret_cast<const T *>(&v0), *p1 = reinterpret_cast<const T *>(&v1),
              *p2 = reinterpret_cast<const T *>(&v2), *p3 = reinterpret_cast<const T *>(&v3);
#pragma unroll
      for (int e = 0; e < per; e++) acc[e] += (S)p0[e] + (S)p1[e] + (S)p2[e] + (S)p3[e];
    }
    for (; q < M; q++) {
      const uint4 v = R.chunk(rows[q], c);
      const T *pv = reinterpret_cast<const T *>(&v);
#pragma unroll
      for (int e = 0; e < per; e++) acc[e] += pv[e];
    }
#pragma unroll
    for (int e = 0; e < per; e++)
      if (c * per + e < B) sum[c * per + e] = acc[e];
  }
}
// 32-bit accumulators while M rows of T cannot carry a bin past 2^32 (every 8-bit input below
// 16.8M members; 16-bit rows up to 65,537 members), 64-bit beyond
template <typename T, int NTH>
__device__ __forceinline__ void add_rows_owned(const RowRef &R, const uint32_t *rows, uint32_t M, int nch, int B,
                                               uint64_t *sum) {
  constexpr uint64_t tmax = sizeof(T) == 1 ? 0xffull : sizeof(T) == 2 ? 0xffffull : 0xffffffffull;
  if ((uint64_t)M * tmax <= 0xffffffffull) add_rows_owned_as<T, NTH, uint32_t>(R, rows, M, nch, B, sum);
  else add_rows_owned_as<T, NTH, uint64_t>(R, rows, M, nch, B, sum);
}

// One workgroup.  rows[q] (q < M) are row indices into R with magnitudes mags[rows[q]];
// keys[q] (or q itself) orders ties like the reference's serial first-min scan.
// sum: B u64 holding the column sums of the M rows.  Fl: nch uint4 (LDS).  Returns the winner.
template <typename T, int NTH>
__device__ uint64_t mean_closest_fast(const RowRef &R, const uint32_t *rows, const uint64_t *keys, uint32_t M,
                                      const uint64_t *mags, int B, int nch, const uint64_t *sum, uint4 *Fl) {
  __shared__ double rd[NTH / 64];
  __shared__ uint64_t rk[NTH / 64];
  __shared__ uint64_t rr[NTH / 64];
  __shared__ uint64_t sF;
  if (threadIdx.x == 0) sF = 0;
  __syncthreads();
  constexpr int per = 16 / (int)sizeof(T);
  uint64_t part = 0;
  for (int c = threadIdx.x; c < nch; c += NTH) {
    uint4 v = make_uint4(0, 0, 0, 0);
    T *pv = reinterpret_cast<T *>(&v);
    for (int i = 0; i < per; i++) {
      const int b = c * per + i;
      const uint64_t S = b < B ? sum[b] : 0;
      const uint64_t F = (S >> 32) == 0 ? (uint64_t)((uint32_t)S / M) : S / M;  // 32-bit divide when it fits
      pv[i] = (T)F;
      part += F;
    }
    Fl[c] = v;
  }
  if (part) atomicAdd((unsigned long long *)&sF, (unsigned long long)part);
  __syncthreads();
  const uint64_t sumF = sF;
  double bd = __builtin_inf();
  uint64_t bk = ~0ull, br = 0;
  if (nch >= 32) {
    // wide rows: one row per wave, 64 lanes over its chunks; every lane ends with the wave's
    // first minimum (the reductions below then see equal values in every lane)
    const int lane = threadIdx.x & 63;
    for (uint32_t q = threadIdx.x >> 6; q < M; q += NTH / 64) {
      const uint64_t r = rows[q];
      Acc<T> acc;
      int c = lane;
      for (; c + 192 < nch; c += 256) {
        const uint4 v0 = R.chunk(r, c), v1 = R.chunk(r, c + 64), v2 = R.chunk(r, c + 128), v3 = R.chunk(r, c + 192);
        acc.add_sad(v0, Fl[c]);
        acc.add_sad(v1, Fl[c + 64]);
        acc.add_sad(v2, Fl[c + 128]);
        acc.add_sad(v3, Fl[c + 192]);
      }
      for (; c < nch; c += 64) acc.add_sad(R.chunk(r, c), Fl[c]);
      acc.wave_reduce();
      const uint64_t mp = mags[r];
      const PS s = acc.finish(mp, sumF);
      const double frac = (double)(2 * s.smin) / (double)(mp + sumF);
      const double d = __builtin_fma(-frac, frac, 1.0) * 10000.0;
      const uint64_t key = keys ? keys[q] : q;
      if (d < bd || (d == bd && key < bk)) {
        bd = d;
        bk = key;
        br = r;
      }
    }
  } else
  for (uint32_t q = threadIdx.x; q < M; q += NTH) {
    const uint64_t r = rows[q];
    Acc<T> acc;
    if (nch == 16) {  // k = 4 at 8 bits (or k = 3 at 16): all loads in flight at once
      uint4 v[16], f[16];
#pragma unroll
      for (int c = 0; c < 16; c++) {
        v[c] = R.chunk(r, c);
        f[c] = Fl[c];
      }
#pragma unroll
      for (int c = 0; c < 16; c++) acc.add_sad(v[c], f[c]);  // (distance_d needs no dot product)
    } else {
#pragma unroll 8
      for (int c = 0; c < nch; c++) acc.add_sad(R.chunk(r, c), Fl[c]);
    }
    const uint64_t mp = mags[r];
    const PS s = acc.finish(mp, sumF);
    const double frac = (double)(2 * s.smin) / (double)(mp + sumF);
    const double d = __builtin_fma(-frac, frac, 1.0) * 10000.0;
    const uint64_t key = keys ? keys[q] : q;
    if (d < bd || (d == bd && key < bk)) {
      bd = d;
      bk = key;
      br = r;
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    double od = __shfl_xor(bd, o, 64);
    uint64_t ok = shfl_xor64(bk, o), orr = shfl_xor64(br, o);
    if (od < bd || (od == bd && ok < bk)) {
      bd = od;
      bk = ok;
      br = orr;
    }
  }
  if ((threadIdx.x & 63) == 0) {
    rd[threadIdx.x >> 6] = bd;
    rk[threadIdx.x >> 6] = bk;
    rr[threadIdx.x >> 6] = br;
  }
  __syncthreads();
  uint64_t win = rr[0];
  if (threadIdx.x == 0) {
    double d = rd[0];
    uint64_t k = rk[0];
    for (int i = 1; i < NTH / 64; i++)
      if (rd[i] < d || (rd[i] == d && rk[i] < k)) {
        d = rd[i];
        k = rk[i];
        win = rr[i];
      }
  }
  __syncthreads();
  return win;
}

}  // namespace mcg
