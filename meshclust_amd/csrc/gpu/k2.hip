// k2.hip -- K2: pairwise k-mer features + GLM classification.
//
//   distance_keys_kernel  DivergencePoint::distance of every point to up to P pivots
//                         (Trainer::split's sort keys, Trainer.cpp:681-701): pivots staged in LDS,
//                         each candidate row read once from HBM.
//   pairs_kernel          raw features / classification of explicit pairs (Feature::normalize
//                         inputs, generate_feat_mat, Trainer::merge).
//   scan_kernel           Trainer::get_close (Trainer.cpp:34-114) over a bvec window: centre in
//                         LDS, candidates streamed, similar ones killed and appended to the
//                         cluster, first max of combo 0 reduced per workgroup.
//   finalize_kernel       get_close's cross-workgroup reduction + bvec::remove_available
//                         bookkeeping + get_mean (ClusterFactory.cpp:382-425).
//   mean_shift_kernel     mean_shift_update (ClusterFactory.cpp:289-380) for every centre.
#include "features.hpp"

namespace mcg {

namespace {

constexpr int NT = 256;

__device__ __forceinline__ PInfo pinfo(const HistView &H, uint32_t id) {
  return PInfo{H.mag[id], H.sumsq[id], H.len[id]};
}

// Raw features of lookup order for one pair (lane-local).
template <typename T>
__device__ __forceinline__ void raw_lookup(const HistView &H, const mc_classifier &c, const PS &s, uint32_t a,
                                           uint32_t b, const PInfo &pa, const PInfo &pb,
                                           double (&raw)[MC_MAX_SINGLE]) {
#pragma unroll
  for (int i = 0; i < MC_MAX_SINGLE; i++) {
    if (i < c.n_single) {
      if (sizeof(T) <= 2) {
        raw[i] = raw_fast(c.lookup[i], s, pa, pb, H.B);
      } else {
        raw[i] = raw_exact<T>(c.lookup[i], reinterpret_cast<const T *>(H.hist + (uint64_t)a * H.pitch),
                              reinterpret_cast<const T *>(H.hist + (uint64_t)b * H.pitch), H.B, pa, pb);
      }
    } else {
      raw[i] = 0;
    }
  }
}

// -------------------------------------------------------------------- distance keys
// grid.x covers candidates (4 per wave pass, 16 lanes per row); pivots in LDS tiles.
template <typename T>
__global__ __launch_bounds__(NT) void distance_keys_kernel(HistView H, const uint32_t *__restrict__ piv, uint32_t npiv,
                                                           const uint32_t *__restrict__ ids, uint64_t m,
                                                           uint16_t *__restrict__ keys, uint32_t ptile) {
  extern __shared__ __attribute__((aligned(16))) uint4 plds[];
  const int nch = (int)((H.B * (int)sizeof(T) + 15) / 16);
  if constexpr (sizeof(T) == 1) {
    if (nch <= 16) {
      // rows of at most 16 chunks (k <= 4): a point per lane, its row in registers, the pivot
      // tile in LDS (broadcast reads); Smin from 4 v_sad_u8 per chunk and the magnitudes, no
      // cross-lane reduction, and each pivot's 64 keys of a wave stored as one 128-byte run
      uint64_t *pmag = reinterpret_cast<uint64_t *>(plds + (size_t)ptile * nch);
      for (uint32_t p0 = 0; p0 < npiv; p0 += ptile) {
        const uint32_t pn = min(ptile, npiv - p0);
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < pn * (uint32_t)nch; t += NT) {
          const uint32_t pp = t / nch, ch = t % nch;
          plds[pp * nch + ch] = reinterpret_cast<const uint4 *>(H.hist + (uint64_t)piv[p0 + pp] * H.pitch)[ch];
        }
        for (uint32_t t = threadIdx.x; t < pn; t += NT) pmag[t] = H.mag[piv[p0 + t]];
        __syncthreads();
        for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i - threadIdx.x < m; i += (uint64_t)gridDim.x * NT) {
          const bool valid = i < m;
          const uint32_t id = valid ? ids[i] : 0;
          const uint4 *row = reinterpret_cast<const uint4 *>(H.hist + (uint64_t)id * H.pitch);
          uint4 mine[16];
#pragma unroll
          for (int c = 0; c < 16; c++) mine[c] = c < nch ? row[c] : make_uint4(0, 0, 0, 0);
          const uint64_t magi = H.mag[id];
          for (uint32_t pp = 0; pp < pn; pp++) {
            const uint4 *pr = plds + (size_t)pp * nch;
            uint32_t s4[4] = {0, 0, 0, 0};
#pragma unroll
            for (int c = 0; c < 16; c++)
              if (c < nch) {
                const uint4 q = pr[c];
                s4[0] = __builtin_amdgcn_sad_u8(mine[c].x, q.x, s4[0]);
                s4[1] = __builtin_amdgcn_sad_u8(mine[c].y, q.y, s4[1]);
                s4[2] = __builtin_amdgcn_sad_u8(mine[c].z, q.z, s4[2]);
                s4[3] = __builtin_amdgcn_sad_u8(mine[c].w, q.w, s4[3]);
              }
            const uint32_t sad = (s4[0] + s4[1]) + (s4[2] + s4[3]);
            const uint64_t magp = pmag[pp];
            const uint64_t smin = (magi + magp - sad) >> 1;
            if (valid) keys[(uint64_t)(p0 + pp) * m + i] = (uint16_t)distance_key(smin, magi, magp);
          }
        }
      }
      return;
    }
  }
  const int lane = threadIdx.x & 63, group = lane >> 4, lig = lane & 15, wave = wave_id();
  const int rows_per_block = 16;  // 4 waves x 4 groups
  for (uint32_t p0 = 0; p0 < npiv; p0 += ptile) {
    const uint32_t pn = min(ptile, npiv - p0);
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < pn * (uint32_t)nch; t += NT) {
      uint32_t pp = t / nch, ch = t % nch;
      plds[pp * nch + ch] = reinterpret_cast<const uint4 *>(H.hist + (uint64_t)piv[p0 + pp] * H.pitch)[ch];
    }
    __syncthreads();
    for (uint64_t base = (uint64_t)blockIdx.x * rows_per_block; base < m; base += (uint64_t)gridDim.x * rows_per_block) {
      const uint64_t i = base + wave * 4 + group;
      const bool valid = i < m;
      const uint32_t id = valid ? ids[i] : 0;
      const uint8_t *row = H.hist + (uint64_t)id * H.pitch;
      // (both loops over the 16 slots unrolled: a runtime-bounded loop indexed the array
      // dynamically, which put it in scratch memory -- 272 bytes per lane, a reload per pivot)
      uint4 mine[16];
      const int per = (nch + 15) / 16;
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const int ch = lig + 16 * q;
        mine[q] = (q < per && valid && ch < nch) ? reinterpret_cast<const uint4 *>(row)[ch] : make_uint4(0, 0, 0, 0);
      }
      const uint64_t magi = valid ? H.mag[id] : 0;
      for (uint32_t pp = 0; pp < pn; pp++) {
        Acc<T> acc;
#pragma unroll
        for (int q = 0; q < 16; q++) {
          const int ch = lig + 16 * q;
          if (q < per && ch < nch) acc.add(mine[q], plds[pp * nch + ch]);
        }
        // rows wider than 256 chunks are streamed from global (k >= 7 at 1 byte)
        for (int ch = lig + 256; ch < nch; ch += 16)
          if (valid) acc.add(reinterpret_cast<const uint4 *>(row)[ch], plds[pp * nch + ch]);
        acc.reduce16();
        const uint64_t magp = H.mag[piv[p0 + pp]];
        PS s = acc.finish(magi, magp);
        if (valid && lig == 0) keys[(uint64_t)(p0 + pp) * m + i] = (uint16_t)distance_key(s.smin, magi, magp);
      }
    }
  }
}

// -------------------------------------------------------------------- explicit pairs
template <typename T>
__global__ __launch_bounds__(NT) void pairs_kernel(HistView H, DevClassifier C, const uint32_t *__restrict__ A,
                                                   const uint32_t *__restrict__ Bi, uint64_t m, uint16_t f0, uint16_t f1,
                                                   uint16_t f2, uint16_t f3, uint16_t f4, int nflag, double *raw_out,
                                                   uint8_t *sim, double *c0_out, double *sum_out, int classify) {
  for (uint64_t base = (uint64_t)blockIdx.x * NT; base < m; base += (uint64_t)gridDim.x * NT) {
    const uint64_t i = base + threadIdx.x;
    const bool valid = i < m;
    const uint32_t a = valid ? A[i] : 0, b = valid ? Bi[i] : 0;
    PS s = wave_pair_stats<T>(H, a, b, valid, nullptr, 0);
    if (!valid) continue;
    const PInfo pa = pinfo(H, a), pb = pinfo(H, b);
    if (!classify) {
      const uint16_t fl[5] = {f0, f1, f2, f3, f4};
      for (int f = 0; f < nflag; f++) {
        double v;
        if (sizeof(T) <= 2) v = raw_fast(fl[f], s, pa, pb, H.B);
        else
          v = raw_exact<T>(fl[f], reinterpret_cast<const T *>(H.hist + (uint64_t)a * H.pitch),
                           reinterpret_cast<const T *>(H.hist + (uint64_t)b * H.pitch), H.B, pa, pb);
        raw_out[i * nflag + f] = v;
      }
    } else {
      double raw[MC_MAX_SINGLE];
      raw_lookup<T>(H, C.c, s, a, b, pa, pb, raw);
      double c0, sum;
      int d = classify_raw(C, raw, &c0, &sum);
      if (sim) sim[i] = (uint8_t)d;
      if (c0_out) c0_out[i] = c0;
      if (sum_out) sum_out[i] = sum;
    }
  }
}

// -------------------------------------------------------------------- precomputed values
// normalize_cache + operator() + GLM decision of pairs whose single-feature values are given
// (alignment mode: identities looked up through the host's replay of Feature::align's memo).
__global__ __launch_bounds__(NT) void values_kernel(DevClassifier C, const double *__restrict__ raw_in, uint64_t m,
                                                    uint8_t *sim, double *c0_out, double *sum_out) {
  const int ns = C.c.n_single;
  for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < m; i += (uint64_t)gridDim.x * NT) {
    double raw[MC_MAX_SINGLE];
#pragma unroll
    for (int f = 0; f < MC_MAX_SINGLE; f++) raw[f] = f < ns ? raw_in[i * ns + f] : 0.0;
    double c0, sum;
    const int d = classify_raw(C, raw, &c0, &sum);
    if (sim) sim[i] = (uint8_t)d;
    if (c0_out) c0_out[i] = c0;
    if (sum_out) sum_out[i] = sum;
  }
}

// -------------------------------------------------------------------- accumulation scan
__device__ __forceinline__ bool better(double v, uint64_t p, double bv, uint64_t bp) {
  return v > bv || (v == bv && p < bp);
}

template <typename T>
__global__ __launch_bounds__(NT) void scan_kernel(HistView H, DevClassifier C, const uint32_t *__restrict__ order,
                                                  uint8_t *__restrict__ alive, uint32_t centre, uint64_t S, uint64_t E,
                                                  ScanPartial *__restrict__ partials, ScanDev *__restrict__ sd,
                                                  uint32_t *__restrict__ flags_out, uint32_t *__restrict__ members,
                                                  uint64_t *__restrict__ mkeys, uint32_t step,
                                                  const double *__restrict__ ident) {
  extern __shared__ __attribute__((aligned(16))) uint4 clds[];
  __shared__ double rv[NT / 64];
  __shared__ uint64_t rp[NT / 64];
  const int nch = (int)((H.B * (int)sizeof(T) + 15) / 16);
  for (int t = threadIdx.x; t < nch; t += NT) clds[t] = reinterpret_cast<const uint4 *>(H.hist + (uint64_t)centre * H.pitch)[t];
  __syncthreads();
  const PInfo pc = pinfo(H, centre);
  const uint32_t mbase = sd->nmembers;
  const uint64_t W = E - S + 1;
  double best_v = -1.0;  // get_close's initializer: (NULL, -1, 0, 0), strict `>`
  uint64_t best_p = ~0ull;
  for (uint64_t base = (uint64_t)blockIdx.x * NT; base < W; base += (uint64_t)gridDim.x * NT) {
    const uint64_t pos = S + base + threadIdx.x;
    const bool valid = (base + threadIdx.x < W) && alive[pos];
    const uint32_t id = valid ? order[pos] : 0;
    PS s{0, 0, 0};
    if (!ident) s = wave_pair_stats<T>(H, id, centre, valid, clds, pc.mag);  // uniform branch
    if (valid) {
      const PInfo pi = pinfo(H, id);
      double raw[MC_MAX_SINGLE];
      if (ident) {  // alignment mode: Feature::align(*pt, *p) computed by the NW kernel
        raw[0] = ident[pos];
        for (int i = 1; i < MC_MAX_SINGLE; i++) raw[i] = 0;
      } else {
        raw_lookup<T>(H, C.c, s, id, centre, pi, pc, raw);  // feat->compute(*pt, *p): candidate first
      }
      double c0;
      int d = classify_raw(C, raw, &c0, nullptr);
      if (better(c0, pos, best_v, best_p) && c0 > -1.0) {
        best_v = c0;
        best_p = pos;
      }
      if (d) {
        alive[pos] = 0;
        uint32_t slot = atomicAdd(&sd->nflag, 1u);
        flags_out[slot] = (uint32_t)pos;
        members[mbase + slot] = id;
        mkeys[mbase + slot] = ((uint64_t)step << 32) | (uint64_t)pos;
      }
    }
  }
  // workgroup argmax (value desc, position asc); NaN never wins (comparisons are false)
  for (int o = 32; o >= 1; o >>= 1) {
    double ov = __shfl_xor(best_v, o, 64);
    uint64_t op = shfl_xor64(best_p, o);
    if (better(ov, op, best_v, best_p)) {
      best_v = ov;
      best_p = op;
    }
  }
  const int w = wave_id();
  if ((threadIdx.x & 63) == 0) {
    rv[w] = best_v;
    rp[w] = best_p;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double v = rv[0];
    uint64_t p = rp[0];
    for (int i = 1; i < NT / 64; i++)
      if (better(rv[i], rp[i], v, p)) {
        v = rv[i];
        p = rp[i];
      }
    partials[blockIdx.x] = ScanPartial{v, p, p != ~0ull ? 1 : 0, 0};
  }
}

// distance_d (DivergencePoint.cpp:53-65) of one histogram row against a double mean.
template <typename T>
__device__ __forceinline__ double distance_d(const T *row, const double *mean, int B) {
  uint64_t dist = 0, mag = 0;
  for (int i = 0; i < B; i++) {
    const uint64_t a = row[i];
    const double m = mean[i];
    uint64_t tm;
    if (sizeof(T) == 1) tm = (uint8_t)(int32_t)m;
    else if (sizeof(T) == 2) tm = (uint16_t)(int32_t)m;
    else if (sizeof(T) == 4) tm = (uint32_t)(int64_t)m;
    else tm = (uint64_t)m;
    const uint64_t mn = a < tm ? a : tm;
    dist += sizeof(T) <= 2 ? 2 * mn : (uint64_t)(T)(mn * 2);
    mag = (uint64_t)((double)mag + ((double)a + m));
  }
  const double frac = (double)dist / (double)mag;
  return __builtin_fma(-frac, frac, 1.0) * 10000.0;
}

// Mean of the given rows, then the first row (by key) closest to it.  One workgroup.
// mean_lds must hold B doubles.
template <typename T, int NTH>
__device__ void mean_closest(const HistView &H, const uint32_t *ids, const uint64_t *keys, uint32_t M, double *mean,
                             uint32_t *out_id) {
  __shared__ double rd[NTH / 64];
  __shared__ uint64_t rk[NTH / 64];
  __shared__ uint32_t ri[NTH / 64];
  const double bottom = (double)M;
  for (int b = threadIdx.x; b < H.B; b += NTH) {
    uint64_t sum = 0;
    for (uint32_t q = 0; q < M; q++) sum += reinterpret_cast<const T *>(H.hist + (uint64_t)ids[q] * H.pitch)[b];
    mean[b] = (double)sum / bottom;
  }
  __syncthreads();
  double bd = __builtin_inf();
  uint64_t bk = ~0ull;
  uint32_t bi = 0;
  for (uint32_t q = threadIdx.x; q < M; q += NTH) {
    const T *row = reinterpret_cast<const T *>(H.hist + (uint64_t)ids[q] * H.pitch);
    double d = distance_d<T>(row, mean, H.B);
    uint64_t key = keys ? keys[q] : q;
    if (d < bd || (d == bd && key < bk)) {
      bd = d;
      bk = key;
      bi = ids[q];
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    double od = __shfl_xor(bd, o, 64);
    uint64_t ok = shfl_xor64(bk, o);
    uint32_t oi = __shfl_xor(bi, o, 64);
    if (od < bd || (od == bd && ok < bk)) {
      bd = od;
      bk = ok;
      bi = oi;
    }
  }
  const int w = wave_id();
  if ((threadIdx.x & 63) == 0) {
    rd[w] = bd;
    rk[w] = bk;
    ri[w] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double d = rd[0];
    uint64_t k = rk[0];
    uint32_t i0 = ri[0];
    for (int i = 1; i < NTH / 64; i++)
      if (rd[i] < d || (rd[i] == d && rk[i] < k)) {
        d = rd[i];
        k = rk[i];
        i0 = ri[i];
      }
    *out_id = i0;
  }
  __syncthreads();
}

constexpr int FT = 1024;

template <typename T, bool GM>  // GM: the mean in global scratch (B > 4096), see mean_shift_kernel
__global__ __launch_bounds__(FT) void finalize_kernel(HistView H, const ScanPartial *__restrict__ partials, int nparts,
                                                      ScanDev *__restrict__ sd, const uint32_t *__restrict__ members,
                                                      const uint64_t *__restrict__ mkeys, double *__restrict__ gmean) {
  extern __shared__ __attribute__((aligned(16))) double mean_lds[];
  __shared__ double rv[FT / 64];
  __shared__ uint64_t rp[FT / 64];
  __shared__ uint32_t new_id;
  double bv = -1.0;
  uint64_t bp = ~0ull;
  for (int i = threadIdx.x; i < nparts; i += FT) {
    ScanPartial p = partials[i];
    if (p.has && better(p.val, p.pos, bv, bp)) {
      bv = p.val;
      bp = p.pos;
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    double ov = __shfl_xor(bv, o, 64);
    uint64_t op = shfl_xor64(bp, o);
    if (better(ov, op, bv, bp)) {
      bv = ov;
      bp = op;
    }
  }
  if ((threadIdx.x & 63) == 0) {
    rv[threadIdx.x >> 6] = bv;
    rp[threadIdx.x >> 6] = bp;
  }
  __syncthreads();
  const uint32_t nflag = sd->nflag;
  const uint32_t M = sd->nmembers + nflag;
  if (nflag > 0) {
    double *mean;
    if constexpr (GM) mean = gmean;
    else mean = mean_lds;
    mean_closest<T, FT>(H, members, mkeys, M, mean, &new_id);
  }
  if (threadIdx.x == 0) {
    double v = rv[0];
    uint64_t p = rp[0];
    for (int i = 1; i < FT / 64; i++)
      if (better(rv[i], rp[i], v, p)) {
        v = rv[i];
        p = rp[i];
      }
    mc_scan_result r;
    r.is_min = nflag == 0;
    r.has_best = p != ~0ull;
    r.best_pos = p;
    r.best_val = v;
    r.n_flagged = nflag;
    r.new_centre = nflag ? new_id : 0xffffffffu;
    r.n_members = M;
    sd->r = r;
    sd->nmembers = M;
    sd->nflag = 0;
  }
}

// -------------------------------------------------------------------- mean shift
// One workgroup per centre j: members of clusters j-delta..j+delta (cluster order) are
// classified against centre j (Trainer::filter, Trainer.cpp:334-349); the survivors' mean
// and the first survivor closest to it (Trainer::closest, :351-365) give the new centre.
// GM: the column sums / mean in global scratch (they do not fit LDS with the centre's chunks) --
// a compile-time choice: picked at run time, the buffer's accesses would be FLAT instructions.
template <typename T, bool GM>
__global__ __launch_bounds__(NT) void mean_shift_kernel(HistView H, DevClassifier C, const uint32_t *__restrict__ cid,
                                                        uint32_t Cn, const uint64_t *__restrict__ off,
                                                        const uint32_t *__restrict__ mem, int delta,
                                                        const uint64_t *__restrict__ soff, uint32_t *__restrict__ kept,
                                                        uint32_t *__restrict__ nkept, double *__restrict__ gmean,
                                                        const uint8_t *__restrict__ keep, uint32_t *__restrict__ newc,
                                                        uint32_t jbase) {
  extern __shared__ __attribute__((aligned(16))) uint4 dyn[];
  // XCD-aware order (speed only: blocks are dealt round-robin over the 8 XCDs): the blocks one
  // XCD runs take consecutive centres, so the neighbourhoods j - delta .. j + delta they read
  // overlap in that XCD's L2 instead of being fetched by eight L2s
  uint32_t jl;
  {
    const uint32_t nb = gridDim.x, x = blockIdx.x % 8, k = blockIdx.x / 8, r = nb % 8, qlo = nb / 8;
    jl = x < r ? x * (qlo + 1) + k : r * (qlo + 1) + (x - r) * qlo + k;
  }
  const uint32_t j = jbase + jl;
  const int nch = (int)((H.B * (int)sizeof(T) + 15) / 16);
  uint4 *clds = dyn;
  double *mean = reinterpret_cast<double *>(dyn + nch);
  const uint32_t centre = cid[j];
  for (int t = threadIdx.x; t < nch; t += NT) clds[t] = reinterpret_cast<const uint4 *>(H.hist + (uint64_t)centre * H.pitch)[t];
  __syncthreads();
  const PInfo pc = pinfo(H, centre);
  const uint32_t bj = j >= (uint32_t)delta ? j - (uint32_t)delta : 0;
  const uint32_t ej = min(j + (uint32_t)delta, Cn - 1);
  const uint64_t lo = off[bj], hi = off[ej + 1];
  uint32_t *mine = kept + soff[j];
  // survivors are compacted in member order: a wave ballot gives each survivor its rank
  // (the next round's member id is loaded a round ahead, and a member's magnitudes before its
  // pair statistics: their round trips overlap the row loads)
  uint32_t id_next = lo + threadIdx.x < hi ? mem[lo + threadIdx.x] : 0;
  uint32_t kept_n = 0;  // survivors so far (uniform)
  int par = 0;
  for (uint64_t base = lo; base < hi; base += NT) {
    const uint64_t q = base + threadIdx.x;
    const bool valid = q < hi;
    const uint32_t id = valid ? id_next : 0;
    id_next = q + NT < hi ? mem[q + NT] : 0;
    int d = 0;
    if (keep) {  // filter decision supplied by the caller (alignment mode)
      d = valid ? keep[soff[j] + (q - lo)] : 0;
    } else {
      const PInfo pi = valid ? pinfo(H, id) : PInfo{0, 0, 0};
      PS s = wave_pair_stats<T>(H, id, centre, valid, clds, pc.mag);
      if (valid) {
        double raw[MC_MAX_SINGLE];
        raw_lookup<T>(H, C.c, s, id, centre, pi, pc, raw);
        double c0;
        d = classify_raw(C, raw, &c0, nullptr);
      }
    }
    // ordered compaction within the workgroup: wave prefix via ballot, waves in order; the
    // running count in every thread's register and the wave counts double-buffered, so a round
    // takes one barrier (a buffer is rewritten two rounds later, after the next round's barrier)
    __shared__ uint32_t wcount[2][NT / 64];
    const uint64_t bal = __ballot(d);
    const int lane = threadIdx.x & 63, w = wave_id();
    if (lane == 0) wcount[par][w] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t before = kept_n, tot = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; i++) {
      const uint32_t x = wcount[par][i];
      if (i < w) before += x;
      tot += x;
    }
    const uint32_t rank = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
    if (d) mine[before + rank] = id;
    kept_n += tot;
    par ^= 1;
  }
  __syncthreads();  // (the survivors' ids are read back by every thread below)
  const uint32_t M = kept_n;
  if (threadIdx.x == 0) nkept[j] = M;
  if (M == 0) {
    if (threadIdx.x == 0) newc[j] = centre;
    return;
  }
  // (launch_mean_shift's LDS plan: the sums stay in LDS when the chunks and B doubles fit 64 KiB)
  double *mbuf;
  if constexpr (GM) mbuf = gmean + (uint64_t)j * H.B;
  else mbuf = mean;
  if constexpr (sizeof(T) <= 2) {
    // integer mean + SAD closest (tests/test_identities.py); sums reuse the mean buffer
    const RowRef R{reinterpret_cast<const uint4 *>(H.hist), H.pitch / 16, 1};
    uint4 *Fl = clds;  // the centre chunks are no longer needed
    uint64_t *sums = reinterpret_cast<uint64_t *>(mbuf);
    __syncthreads();
    if (nch >= 32) {
      add_rows_owned<T, NT>(R, mine, M, nch, H.B, sums);
    } else {
      for (int b = threadIdx.x; b < H.B; b += NT) sums[b] = 0;
      __syncthreads();
      add_rows<T, NT>(R, mine, M, nch, sums);
    }
    __syncthreads();
    const uint64_t win = mean_closest_fast<T, NT>(R, mine, nullptr, M, H.mag, H.B, nch, sums, Fl);
    if (threadIdx.x == 0) newc[j] = (uint32_t)win;
  } else {
    __shared__ uint32_t out_id;
    mean_closest<T, NT>(H, mine, nullptr, M, mbuf, &out_id);
    if (threadIdx.x == 0) newc[j] = out_id;
  }
}

// -------------------------------------------------------------------- accumulation output
// Each cluster's members in `current` order (the seed, then each step's flagged candidates in
// bvec order): one workgroup per cluster sorts its u64 keys -- step << 32 | static position,
// or the seed's 0 replaced by its position -- by a bitonic network in LDS and writes the ids
// (static order -> id).  Clusters of more than OM_MAX members are left to the host.  The grid is
// capped (OM_GRID) and strides over the clusters: a mostly-singleton input can have more clusters
// than a launch may hold workgroups.
constexpr int OM_MAX = 4096, OM_T = 256;
constexpr uint64_t OM_GRID = 65536;
__global__ __launch_bounds__(OM_T) void order_members_kernel(const uint64_t *__restrict__ keys,
                                                             const uint32_t *__restrict__ pos,
                                                             const uint64_t *__restrict__ cl_off,
                                                             const uint32_t *__restrict__ order,
                                                             uint32_t *__restrict__ ids, uint64_t ncl) {
  __shared__ uint64_t k[OM_MAX];
  for (uint64_t cl = blockIdx.x; cl < ncl; cl += gridDim.x) {
    const uint64_t a = cl_off[cl], b = cl_off[cl + 1];
    const uint32_t m = (uint32_t)(b - a);
    if (b - a > (uint64_t)OM_MAX) continue;  // (uniform)
    if (m == 1) {  // (a singleton: nothing to order)
      if (threadIdx.x == 0) ids[a] = order[pos[a]];
      continue;
    }
    uint32_t P = 1;
    while (P < m) P <<= 1;
    __syncthreads();  // (the previous cluster's reads of k are done)
    for (uint32_t i = threadIdx.x; i < P; i += OM_T) {
      const uint64_t x = i < m ? keys[a + i] : ~0ull;
      k[i] = i < m && x == 0 ? (uint64_t)pos[a + i] : x;
    }
    __syncthreads();
    for (uint32_t len = 2; len <= P; len <<= 1)
      for (uint32_t j = len >> 1; j > 0; j >>= 1) {
        for (uint32_t i = threadIdx.x; i < P; i += OM_T) {
          const uint32_t l = i ^ j;
          if (l > i) {
            const uint64_t x = k[i], y = k[l];
            const bool up = (i & len) == 0;
            if (up ? x > y : x < y) {
              k[i] = y;
              k[l] = x;
            }
          }
        }
        __syncthreads();
      }
    for (uint32_t i = threadIdx.x; i < m; i += OM_T) ids[a + i] = order[(uint32_t)k[i]];
  }
}

int grid_for(uint64_t work, int per_block, int cap) {
  uint64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > (uint64_t)cap) g = cap;
  return (int)g;
}

}  // namespace

#define MCG_DISPATCH_T(width, KERNEL_CALL)        \
  switch (width) {                                \
    case 1: { typedef uint8_t T; KERNEL_CALL; break; }  \
    case 2: { typedef uint16_t T; KERNEL_CALL; break; } \
    case 4: { typedef uint32_t T; KERNEL_CALL; break; } \
    default: { typedef uint64_t T; KERNEL_CALL; break; } \
  }

int launch_order_members(mc_ctx *c, const uint64_t *d_keys, const uint32_t *d_pos, const uint64_t *d_cl_off, uint64_t ncl,
                         uint32_t *d_ids) {
  if (!ncl) return MC_OK;
  const unsigned grid = (unsigned)(ncl < OM_GRID ? ncl : OM_GRID);
  order_members_kernel<<<grid, OM_T, 0, c->stream>>>(d_keys, d_pos, d_cl_off, (const uint32_t *)c->order.p, d_ids,
                                                     ncl);
  MCG_CHECK(hipGetLastError());
  return MC_OK;
}
uint64_t order_members_max() { return OM_MAX; }

int launch_distance_keys(mc_ctx *c, const uint32_t *d_piv, uint32_t npiv, const uint32_t *d_ids, uint64_t m,
                         uint16_t *d_keys) {
  if (m == 0 || npiv == 0) return MC_OK;
  const HistView H = hist_view(c);
  const int nch = (int)((H.B * H.width + 15) / 16);
  const bool lane_rows = H.width == 1 && nch <= 16;  // (distance_keys_kernel's point-per-lane form)
  uint32_t ptile = (uint32_t)std::max(1, 65536 / (nch * 16 + (lane_rows ? 8 : 0)));
  ptile = std::min(ptile, npiv);
  const size_t lds = (size_t)ptile * nch * 16 + (lane_rows ? (size_t)ptile * 8 : 0);
  const int grid = lane_rows ? grid_for(m, NT, 2048) : grid_for(m, 16, 2048);
  timed_begin(c);
  MCG_DISPATCH_T(c->width, (distance_keys_kernel<T><<<grid, NT, lds, c->stream>>>(H, d_piv, npiv, d_ids, m, d_keys, ptile)));
  MCG_CHECK(hipGetLastError());
  timed_end(c, F_KEYS);
  return MC_OK;
}

int launch_pairs(mc_ctx *c, const uint32_t *d_a, const uint32_t *d_b, uint64_t m, const uint16_t *flags, int nflag,
                 double *d_raw, uint8_t *d_sim, double *d_c0, double *d_sum, bool classify) {
  if (m == 0) return MC_OK;
  const HistView H = hist_view(c);
  uint16_t f[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < nflag && i < 5; i++) f[i] = flags[i];
  const int grid = grid_for(m, NT, 4096);
  timed_begin(c);
  MCG_DISPATCH_T(c->width, (pairs_kernel<T><<<grid, NT, 0, c->stream>>>(H, c->cls, d_a, d_b, m, f[0], f[1], f[2], f[3], f[4], nflag,
                                                                      d_raw, d_sim, d_c0, d_sum, classify ? 1 : 0)));
  MCG_CHECK(hipGetLastError());
  timed_end(c, F_PAIRS);
  return MC_OK;
}

// merge's classifier pairs over the new centres (ClusterFactory.cpp:427-493): centre i's pairs
// are (new[t], new[i]) for t = i+1 .. i + (poff[i+1] - poff[i]), at poff[i]..
__global__ __launch_bounds__(256) void merge_pairs_kernel(const uint32_t *__restrict__ d_new, uint32_t C,
                                                          const uint64_t *__restrict__ poff, uint32_t *pa, uint32_t *pb) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= C) return;
  const uint64_t q0 = poff[i], n = poff[i + 1] - q0;
  const uint32_t ci = d_new[i];
  for (uint64_t d = 0; d < n; d++) {
    pa[q0 + d] = d_new[i + 1 + d];
    pb[q0 + d] = ci;
  }
}

int launch_merge_pairs(mc_ctx *c, const uint32_t *d_new, uint32_t C, const uint64_t *d_poff, uint32_t *d_a,
                       uint32_t *d_b) {
  if (C == 0) return MC_OK;
  merge_pairs_kernel<<<(C + 255) / 256, 256, 0, c->stream>>>(d_new, C, d_poff, d_a, d_b);
  MCG_CHECK(hipGetLastError());
  return MC_OK;
}

int launch_values(mc_ctx *c, const double *d_raw, uint64_t m, uint8_t *d_sim, double *d_c0, double *d_sum) {
  if (m == 0) return MC_OK;
  const int grid = grid_for(m, NT, 4096);
  timed_begin(c);
  values_kernel<<<grid, NT, 0, c->stream>>>(c->cls, d_raw, m, d_sim, d_c0, d_sum);
  MCG_CHECK(hipGetLastError());
  timed_end(c, F_PAIRS);
  return MC_OK;
}

int launch_scan(mc_ctx *c, uint32_t centre, uint64_t S, uint64_t E, const double *d_ident, int *nblocks) {
  const HistView H = hist_view(c);
  const int nch = (int)((H.B * H.width + 15) / 16);
  const uint64_t W = E - S + 1;
  const int grid = grid_for(W, NT, 2048);
  *nblocks = grid;
  timed_begin(c);
  auto *sd = (ScanDev *)c->scan_dev.p;
  uint32_t *flags = (uint32_t *)((char *)c->scan_dev.p + sizeof(ScanDev));
  MCG_DISPATCH_T(c->width, (scan_kernel<T><<<grid, NT, (size_t)nch * 16, c->stream>>>(
                               H, c->cls, (const uint32_t *)c->order.p, (uint8_t *)c->alive.p, centre, S, E,
                               (ScanPartial *)c->partials.p, sd, flags, (uint32_t *)c->members.p,
                               (uint64_t *)c->member_keys.p, c->step, d_ident)));
  MCG_CHECK(hipGetLastError());
  timed_end(c, F_SCAN);
  return MC_OK;
}

int launch_finalize(mc_ctx *c, int nblocks) {
  const HistView H = hist_view(c);
  const size_t lds = H.B <= 4096 ? (size_t)H.B * 8 : 0;
  if (H.B > 4096 && ensure(c->s_g, (size_t)H.B * 8)) return MC_ERR_OOM;
  timed_begin(c);
  MCG_DISPATCH_T(c->width, ((H.B > 4096 ? finalize_kernel<T, true> : finalize_kernel<T, false>)<<<1, FT, lds, c->stream>>>(
                               H, (const ScanPartial *)c->partials.p, nblocks, (ScanDev *)c->scan_dev.p,
                               (const uint32_t *)c->members.p, (const uint64_t *)c->member_keys.p,
                               (double *)c->s_g.p)));
  MCG_CHECK(hipGetLastError());
  timed_end(c, F_FINAL);
  return MC_OK;
}

int launch_mean_shift(mc_ctx *c, const uint32_t *d_cid, uint32_t C, const uint64_t *d_off, const uint64_t *h_off,
                      const uint32_t *d_mem, int delta, const uint8_t *d_keep, uint32_t *d_new, uint32_t j0,
                      uint32_t j1) {
  if (C == 0 || j0 >= j1) return MC_OK;
  const HistView H = hist_view(c);
  const int nch = (int)((H.B * H.width + 15) / 16);
  // scratch: per-centre survivor lists (offsets = sizes of the neighbourhoods)
  std::vector<uint64_t> soff(C + 1, 0);
  for (uint32_t j = 0; j < C; j++) {
    uint32_t b = j >= (uint32_t)delta ? j - delta : 0;
    uint32_t e = std::min<uint32_t>(j + delta, C - 1);
    soff[j + 1] = soff[j] + (h_off[e + 1] - h_off[b]);
  }
  if (ensure(c->s_d, (C + 1) * 8) || ensure(c->s_e, std::max<uint64_t>(soff[C], 1) * 4) || ensure(c->s_f, (size_t)C * 4))
    return MC_ERR_OOM;
  const bool gm = (size_t)nch * 16 + (size_t)H.B * 8 > 65536;  // column sums / mean in LDS when they fit
  if (gm && ensure(c->s_g, (size_t)C * H.B * 8)) return MC_ERR_OOM;
  MCG_CHECK(hipMemcpyAsync(c->s_d.p, soff.data(), (C + 1) * 8, hipMemcpyHostToDevice, c->stream));
  const size_t lds = (size_t)nch * 16 + (gm ? 0 : (size_t)H.B * 8);
  timed_begin(c);
  MCG_DISPATCH_T(c->width, ((gm ? mean_shift_kernel<T, true> : mean_shift_kernel<T, false>)<<<j1 - j0, NT, lds, c->stream>>>(
                               H, c->cls, d_cid, C, d_off, d_mem, delta, (const uint64_t *)c->s_d.p,
                               (uint32_t *)c->s_e.p, (uint32_t *)c->s_f.p, (double *)c->s_g.p, d_keep, d_new, j0)));
  MCG_CHECK(hipGetLastError());
  timed_end(c, F_MSHIFT);
  return MC_OK;
}

}  // namespace mcg
