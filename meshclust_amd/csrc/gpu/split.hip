// split.hip -- Trainer::split's per-pivot std::sort (Trainer.cpp:691-701), evaluated on the
// device at exactly the positions the trainer reads.
//
// The trainer sorts all N points by their distance key to each of ~150 pivots with std::sort
// (an unstable introsort: among equal keys -- keys are integers <= 10000, ties are everywhere --
// the order is defined only by that algorithm) and then reads ~35 positions of each sorted
// array (the alignment binary search, Trainer.cpp:703-721, and the sampler, :732-755).  The
// host's mc::LazyIntroSort (csrc/host/lazysort.hpp) reproduces libstdc++'s result at a queried
// position by partitioning only the ranges that hold it; this file is the same algorithm with
// each pivot's array resident in HBM and its partitions done by one workgroup:
//   * std::__introsort_loop: median of (first+1, mid, last-1) moved to first, then the
//     unguarded Hoare partition of [first+1, last) around it; depth limit 2 floor(log2 n)
//     with std::make_heap + std::sort_heap below it; ranges of <= 16 elements are leaves,
//     finished by a stable insertion sort (what __final_insertion_sort does to them).
//   * The Hoare partition as data-parallel passes: the left scan stops at keys >= pivot
//     (positions l_1 < l_2 < ...), the right scan at keys <= pivot (r_1 > r_2 > ...); the k-th
//     swap exchanges l_k and r_k of the array as it was before the partition for every k <= K,
//     K the last k with l_k < r_k (no scan reads a position an earlier swap wrote before the
//     scans cross, so all K swaps are independent), and the cut is min(l_{K+1}, r_K).  A
//     workgroup counts the stoppers of its threads' segments, writes their positions in order
//     (exclusive scan), finds K by a two-round parallel bisection and does the K swaps at once.
// Elements are 64-bit words (key << 32 | id) compared by the key alone.  Each pivot's tree of
// partitioned ranges persists across calls (the trainer's rounds query deeper positions of
// the same arrays).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "mcgpu.hpp"

namespace mcg {

namespace {

constexpr int ST = 1024;  // threads per workgroup
constexpr int SW = ST / 64;
// A range of at most LMAX words still to be partitioned is copied into LDS and its query's
// walk finishes there (every level a few LDS passes instead of global round trips); the range
// is written back at the end.  LDS: LMAX words | left / right stopper positions (u16)
constexpr int64_t LMAX = 8192;
constexpr size_t SEL_LDS = (size_t)LMAX * 8 + 2 * (size_t)LMAX * 2;

__device__ __forceinline__ bool kless(uint64_t x, uint64_t y) { return (x >> 32) < (y >> 32); }

// (FP: a global or an LDS-typed pointer -- the two paths stay apart, no FLAT accesses)
#define SP_LDS __attribute__((address_space(3)))
template <typename FP>
__device__ void insertion_sort_1(FP f, int64_t n) {  // std::__insertion_sort (stable)
  for (int64_t i = 1; i < n; i++) {
    const uint64_t v = f[i];
    int64_t j = i;
    while (j > 0 && kless(v, f[j - 1])) {
      f[j] = f[j - 1];
      j--;
    }
    f[j] = v;
  }
}

// libstdc++'s std::__adjust_heap / std::__push_heap with the key comparator
template <typename FP>
__device__ void adjust_heap_1(FP f, int64_t hole, int64_t len, uint64_t v) {
  const int64_t top = hole;
  int64_t child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (kless(f[child], f[child - 1])) child--;
    f[hole] = f[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    f[hole] = f[child - 1];
    hole = child - 1;
  }
  int64_t parent = (hole - 1) / 2;
  while (hole > top && kless(f[parent], v)) {
    f[hole] = f[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  f[hole] = v;
}

// std::__partial_sort(first, last, last) = std::__make_heap + std::__sort_heap (one thread:
// reached only below the depth limit, i.e. on degenerate partitions)
template <typename FP>
__device__ void heap_sort_1(FP f, int64_t n) {
  if (n < 2) return;
  for (int64_t parent = (n - 2) / 2;; parent--) {
    adjust_heap_1(f, parent, n, f[parent]);
    if (parent == 0) break;
  }
  for (int64_t last = n; last > 1;) {
    last--;
    const uint64_t v = f[last];
    f[last] = f[0];
    adjust_heap_1(f, 0, last, v);
  }
}

struct SelArgs {
  uint64_t *words;   // narr arrays of n words
  uint64_t n;
  uint32_t *scr;     // narr x 2n: left stoppers | right stoppers (positions, ascending)
  SplitNode *nodes;  // narr x maxnode
  int32_t *nnodes;   // narr
  int32_t maxnode;
  int32_t depth0;    // the root's depth limit (2 floor(log2 n), or a test override)
  const uint32_t *qarr;  // per workgroup: its array
  const uint64_t *qoff;  // per workgroup: its queries [qoff[b], qoff[b + 1])
  const uint64_t *qpos;  // query positions
  uint64_t *qout;        // the word std::sort puts at each queried position
  int *err;
  unsigned long long *prof;  // MC_SPLIT_PROFILE: thread 0's realtime ticks per phase (8 counters)
  int nowave;                // MC_SPLIT_NO_WAVE: every LDS partition by the whole workgroup
};

// inclusive scan over the wave by DPP (rows of 16 by row_shr 1 / 2 / 4 / 8, then the rows'
// totals by row_bcast 15 / 31): six VALU adds, no LDS round trip (a __shfl_up scan is six
// dependent ds_bpermute round trips)
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

// Workgroup-wide exclusive scan of two counters (every thread gets its offsets and the totals).
__device__ __forceinline__ void block_scan2(uint32_t a, uint32_t b, uint32_t *ea, uint32_t *eb, uint32_t *ta,
                                            uint32_t *tb, uint32_t *s) {
  const int lane = threadIdx.x & 63, wv = wave_id();
  const uint32_t ia = wave_scan_incl(a), ib = wave_scan_incl(b);  // inclusive scans within the wave
  if (lane == 63) {
    s[wv] = ia;
    s[SW + wv] = ib;
  }
  __syncthreads();
  uint32_t pa = 0, pb = 0, sa = 0, sb = 0;
  for (int i = 0; i < SW; i++) {
    if (i < wv) {
      pa += s[i];
      pb += s[SW + i];
    }
    sa += s[i];
    sb += s[SW + i];
  }
  *ea = pa + ia - a;
  *eb = pb + ib - b;
  *ta = sa;
  *tb = sb;
  __syncthreads();  // s is reused by the caller's next scan
}

// One workgroup partitions f[0, n) (n > 16) exactly as std::__unguarded_partition_pivot;
// returns the cut.  L / R: scratch for n positions each (global u32, or LDS u16 when f is the
// LDS copy of a range of at most LMAX words).  Global ranges: `stg` (LDS, 2 ST * 8 words) stages
// the stopper positions, `scnt` (LDS, 256 words) holds the pass's counts.
template <typename PT, typename FP>
__device__ int64_t partition_wg(FP f, int64_t n, PT *L, PT *R, uint32_t *s32, uint64_t *s64,
                                unsigned long long *prof = nullptr, SP_LDS uint32_t *stg = nullptr,
                                SP_LDS uint32_t *scnt = nullptr) {
  const int t = threadIdx.x;
  // (MC_SPLIT_PROFILE, global ranges: thread 0's realtime ticks in the median, the stopper pass,
  // the bisection and the swaps, prof[8..11])
  uint64_t tp = prof && t == 0 ? __builtin_amdgcn_s_memrealtime() : 0;
  auto pmark = [&](int i) {
    if (prof && t == 0) {
      const uint64_t u = __builtin_amdgcn_s_memrealtime();
      atomicAdd(&prof[8 + i], (unsigned long long)(u - tp));
      tp = u;
    }
  };
  if (t == 0) {  // std::__move_median_to_first(first, first + 1, mid, last - 1)
    const uint64_t a = f[1], b = f[n / 2], c = f[n - 1];
    int64_t m;
    if (kless(a, b)) m = kless(b, c) ? n / 2 : kless(a, c) ? n - 1 : 1;
    else m = kless(a, c) ? 1 : kless(b, c) ? n - 1 : n / 2;
    const uint64_t x = f[0];
    f[0] = f[m];
    f[m] = x;
  }
  __syncthreads();
  pmark(0);
  const uint64_t pk = f[0] >> 32;
  uint32_t CL, TL;
  if constexpr (sizeof(PT) == 2) {
    // LDS copy: segments of S consecutive positions per thread, counted, scanned, written
    const int64_t S = (n + ST - 1) / ST;
    const int64_t i0 = (int64_t)t * S < n ? (int64_t)t * S : n, i1 = i0 + S < n ? i0 + S : n;
    uint32_t cg = 0, cl = 0;
    for (int64_t i = i0; i < i1; i++) {
      const uint64_t k = f[i] >> 32;
      cg += (i >= 1 && k >= pk) ? 1u : 0u;
      cl += k <= pk ? 1u : 0u;
    }
    uint32_t og, ol;
    block_scan2(cg, cl, &og, &ol, &CL, &TL, s32);
    for (int64_t i = i0; i < i1; i++) {
      const uint64_t k = f[i] >> 32;
      if (i >= 1 && k >= pk) L[og++] = (PT)i;
      if (k <= pk) R[ol++] = (PT)i;
    }
  } else {
    // global range: chunks of ST * CPT words, word e * ST + t of a chunk to thread t (every load
    // of a chunk in flight at once, each load instruction 512 contiguous bytes per wave).  The
    // stoppers are ranked in position order by ballots and a scan over the (e, wave) counts, staged
    // in LDS (`stg`) and written out contiguously -- one coalesced store per 64 positions instead
    // of a scattered 4-byte store per stopper.
    // (the next chunk's words are loaded before this chunk's ranking: the barriers wait for LDS
    // only, so the loads stay in flight across them)
    constexpr int CPT = 8;
    constexpr uint32_t CH = (uint32_t)ST * CPT;
    static_assert(CPT * SW == 128, "the (e, wave) counts are two per lane of one wave");
    const int wv = __builtin_amdgcn_readfirstlane(wave_id()), lane = t & 63;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;  // lanes below this one
    uint32_t bg = 0, bl = 0;  // stoppers before this chunk
    uint32_t kn[CPT];
#pragma unroll
    for (int e = 0; e < CPT; e++) {
      const int64_t i = (int64_t)e * ST + t;
      kn[e] = i < n ? (uint32_t)(f[i] >> 32) : 0u;
    }
    for (int64_t c0 = 0; c0 < n; c0 += (int64_t)CH) {
      uint32_t kk[CPT];
#pragma unroll
      for (int e = 0; e < CPT; e++) kk[e] = kn[e];
#pragma unroll
      for (int e = 0; e < CPT; e++) {
        const int64_t i = c0 + CH + (int64_t)e * ST + t;
        kn[e] = i < n ? (uint32_t)(f[i] >> 32) : 0u;
      }
      uint64_t bL[CPT], bR[CPT];
#pragma unroll
      for (int e = 0; e < CPT; e++) {
        const int64_t i = c0 + (int64_t)e * ST + t;
        bL[e] = __ballot(i < n && i >= 1 && kk[e] >= pk);
        bR[e] = __ballot(i < n && kk[e] <= pk);
        if (lane == 0) {
          scnt[e * SW + wv] = (uint32_t)__popcll(bL[e]);
          scnt[CPT * SW + e * SW + wv] = (uint32_t)__popcll(bR[e]);
        }
      }
      __syncthreads();
      // exclusive offsets of the (e, wave) groups in position order, by every wave
      const uint32_t a0 = scnt[2 * lane], a1 = scnt[2 * lane + 1];
      const uint32_t b0 = scnt[CPT * SW + 2 * lane], b1 = scnt[CPT * SW + 2 * lane + 1];
      const uint32_t ia = wave_scan_incl(a0 + a1), ib = wave_scan_incl(b0 + b1);
      const uint32_t tg = (uint32_t)__builtin_amdgcn_readlane((int)ia, 63), tl = (uint32_t)__builtin_amdgcn_readlane((int)ib, 63);
      const uint32_t ma = (wv & 1) ? ia - a1 : ia - a0 - a1, mb = (wv & 1) ? ib - b1 : ib - b0 - b1;
#pragma unroll
      for (int e = 0; e < CPT; e++) {
        const int src = (e * SW + wv) >> 1;
        const uint32_t oa = (uint32_t)__builtin_amdgcn_readlane((int)ma, src), ob = (uint32_t)__builtin_amdgcn_readlane((int)mb, src);
        const uint32_t i = (uint32_t)(c0 + (int64_t)e * ST + t);
        if ((bL[e] >> lane) & 1) stg[oa + (uint32_t)__popcll(bL[e] & lt)] = i;
        if ((bR[e] >> lane) & 1) stg[CH + ob + (uint32_t)__popcll(bR[e] & lt)] = i;
      }
      __syncthreads();
      for (uint32_t j = t; j < tg; j += ST) L[bg + j] = (PT)stg[j];
      for (uint32_t j = t; j < tl; j += ST) R[bl + j] = (PT)stg[CH + j];
      bg += tg;
      bl += tl;
    }
    CL = bg;
    TL = bl;
  }
  __syncthreads();
  pmark(1);
  // K = the last k with l_k < r_k (l_k = L[k - 1], r_k = R[TL - k]); monotone in k: bisection
  // over (lo, hi) with P(lo) true, P(hi) false, ST probes per round
  const int64_t m = CL < TL ? CL : TL;
  int64_t lo = 0, hi = m + 1;
  while (hi - lo > 1) {
    const int64_t span = hi - lo;
    const int64_t k = lo + 1 + ((span - 1) * (int64_t)t) / ST;  // in (lo, hi), nondecreasing in t
    const bool p = L[k - 1] < R[TL - k];
    const uint64_t bal = __ballot(p);
    if ((t & 63) == 0) s32[wave_id()] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t c = 0;
    for (int i = 0; i < SW; i++) c += s32[i];
    // the probes with P true are a prefix (threads 0 .. c - 1): the new bracket is between the
    // last true probe and the first false one
    if (t == (int)c - 1) s64[0] = (uint64_t)k;
    if (t == (int)c) s64[1] = (uint64_t)k;
    __syncthreads();
    const int64_t nlo = c > 0 ? (int64_t)s64[0] : lo, nhi = c < (uint32_t)ST ? (int64_t)s64[1] : hi;
    __syncthreads();
    lo = nlo;
    hi = nhi;
  }
  const int64_t K = lo;
  pmark(2);
  // the K independent swaps, four per thread in flight
  for (int64_t k0 = 1 + t; k0 <= K; k0 += 4 * ST) {
    uint32_t a[4], b[4];
    uint64_t x[4], y[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int64_t k = k0 + (int64_t)e * ST;
      a[e] = k <= K ? (uint32_t)L[k - 1] : 0u;
      b[e] = k <= K ? (uint32_t)R[TL - k] : 0u;
    }
#pragma unroll
    for (int e = 0; e < 4; e++)
      if (k0 + (int64_t)e * ST <= K) {
        x[e] = f[a[e]];
        y[e] = f[b[e]];
      }
#pragma unroll
    for (int e = 0; e < 4; e++)
      if (k0 + (int64_t)e * ST <= K) {
        f[a[e]] = y[e];
        f[b[e]] = x[e];
      }
  }
  const int64_t lk1 = K < (int64_t)CL ? (int64_t)L[K] : n, rK = K >= 1 ? (int64_t)R[TL - K] : n;
  __syncthreads();
  pmark(3);
  if (prof && t == 0) {
    atomicAdd(&prof[12], (unsigned long long)n);
    atomicAdd(&prof[13], (unsigned long long)K);
  }
  return lk1 < rK ? lk1 : rK;
}

// The array's tree of partitioned ranges is mirrored in LDS (its first NCACHE nodes): a query's
// walk down the levels earlier calls have partitioned reads one LDS node per level instead of
// a global one (a dependent memory round trip per level, ~17 levels per query at n = 100k).
constexpr int NCACHE = 512;

// partition_wg's algorithm by wave 0 alone, for an LDS range of at most WMAX words (the lower
// levels of every query's walk): the stoppers are compacted 64 positions per ballot, K is a
// 64-probe bisection by ballot, the swaps go 64 at a time -- no
// workgroup barrier inside (LDS operations of one wave are performed in order).  Returns the
// cut in every lane.  (The same stoppers, K, swaps and cut as partition_wg: the swaps are
// disjoint, so their order does not matter.)
constexpr int64_t WMAX = 2048;
__device__ int64_t partition_wave(SP_LDS uint64_t *f, int64_t n, SP_LDS uint16_t *L, SP_LDS uint16_t *R,
                                  unsigned long long *prof = nullptr) {
  const int lane = threadIdx.x & 63;
  uint64_t tp = prof && lane == 0 ? __builtin_amdgcn_s_memrealtime() : 0;
  auto pmark = [&](int i) {  // (MC_SPLIT_PROFILE: prof[17..19] stoppers, bisection, swaps; [20] swaps)
    if (prof && lane == 0) {
      const uint64_t u = __builtin_amdgcn_s_memrealtime();
      atomicAdd(&prof[17 + i], (unsigned long long)(u - tp));
      tp = u;
    }
  };
  if (lane == 0) {  // std::__move_median_to_first(first, first + 1, mid, last - 1)
    const uint64_t a = f[1], b = f[n / 2], c = f[n - 1];
    int64_t m;
    if (kless(a, b)) m = kless(b, c) ? n / 2 : kless(a, c) ? n - 1 : 1;
    else m = kless(a, c) ? 1 : kless(b, c) ? n - 1 : n / 2;
    const uint64_t x = f[0];
    f[0] = f[m];
    f[m] = x;
  }
  const uint64_t pk = f[0] >> 32;
  // the stoppers in position order: 64 consecutive positions per ballot (a lane each), four
  // such groups' LDS reads in flight
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;  // lanes below this one
  uint32_t CL = 0, TL = 0;
  for (int64_t c0 = 0; c0 < n; c0 += 256) {
    uint64_t kk[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int64_t i = c0 + u * 64 + lane;
      kk[u] = i < n ? f[i] >> 32 : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int64_t i = c0 + u * 64 + lane;
      const bool gl = i < n && i >= 1 && kk[u] >= pk, gr = i < n && kk[u] <= pk;
      const uint64_t bl = __ballot(gl), br = __ballot(gr);
      if (gl) L[CL + (uint32_t)__popcll(bl & lt)] = (uint16_t)i;
      if (gr) R[TL + (uint32_t)__popcll(br & lt)] = (uint16_t)i;
      CL += (uint32_t)__popcll(bl);
      TL += (uint32_t)__popcll(br);
    }
  }
  pmark(0);
  // K = the last k with L[k - 1] < R[TL - k]: bracket (lo, hi), 64 probes per round
  const int64_t m = CL < TL ? CL : TL;
  int64_t lo = 0, hi = m + 1;
  while (hi - lo > 1) {
    const int64_t span = hi - lo;
    const int64_t k = lo + 1 + ((span - 1) * (int64_t)lane) / 64;  // in (lo, hi), nondecreasing in lane
    const bool pr = L[k - 1] < R[TL - k];
    const int c = (int)__popcll(__ballot(pr));  // the true probes are lanes 0 .. c - 1
    const int64_t nlo = c > 0 ? (int64_t)__builtin_amdgcn_readlane((int)k, c - 1) : lo;
    const int64_t nhi = c < 64 ? (int64_t)__builtin_amdgcn_readlane((int)k, c) : hi;
    lo = nlo;
    hi = nhi;
  }
  const int64_t K = lo;
  pmark(1);
  for (int64_t k = 1 + lane; k <= K; k += 64) {
    const uint32_t pa = L[k - 1], pb = R[TL - k];
    const uint64_t x = f[pa], y = f[pb];
    f[pa] = y;
    f[pb] = x;
  }
  const int64_t lk1 = K < (int64_t)CL ? (int64_t)L[K] : n, rK = K >= 1 ? (int64_t)R[TL - K] : n;
  pmark(2);
  if (prof && lane == 0) atomicAdd(&prof[20], (unsigned long long)K);
  return lk1 < rK ? lk1 : rK;
}

__global__ __launch_bounds__(ST) void select_kernel(SelArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint64_t s_dyn[];
  __shared__ uint32_t s32[2 * SW];
  __shared__ uint64_t s64[2];
  __shared__ SplitNode s_nd;
  __shared__ int32_t s_nn, s_idx;
  __shared__ SplitNode s_cache[NCACHE];
  __shared__ uint32_t s_cnt[256];
  uint64_t *LW = s_dyn;                                       // LMAX words
  uint16_t *LL = reinterpret_cast<uint16_t *>(s_dyn + LMAX);  // LMAX + LMAX stopper positions
  uint16_t *LR = LL + LMAX;
  const int t = threadIdx.x;
  const uint32_t arr = a.qarr[blockIdx.x];
  uint64_t *W = a.words + (uint64_t)arr * a.n;
  uint32_t *L = a.scr + (uint64_t)arr * 2 * a.n, *R = L + a.n;
  SplitNode *nd = a.nodes + (uint64_t)arr * a.maxnode;
  if (t == 0) {
    s_nn = a.nnodes[arr];
    if (s_nn == 0) {  // the root: the whole array
      nd[0] = SplitNode{0, (int64_t)a.n, 0, a.depth0, -1, 0, 0};
      s_cache[0] = nd[0];
      s_nn = 1;
    }
  }
  __syncthreads();
  {
    const int32_t nc = s_nn < NCACHE ? s_nn : NCACHE;
    for (int32_t i = t; i < nc; i += ST)
      if (i > 0 || a.nnodes[arr] != 0) s_cache[i] = nd[i];
  }
  __syncthreads();
  for (uint64_t q = a.qoff[blockIdx.x]; q < a.qoff[blockIdx.x + 1]; q++) {
    const int64_t pos = (int64_t)a.qpos[q];
    int32_t idx = 0;
    bool in_lds = false;  // the walk continues on the LDS copy of [lbase, lend)
    int64_t lbase = 0, lend = 0;
    uint64_t tm = a.prof ? __builtin_amdgcn_s_memrealtime() : 0;
    auto mark = [&](int ph) {
      if (a.prof && t == 0) {
        const uint64_t u = __builtin_amdgcn_s_memrealtime();
        atomicAdd(&a.prof[ph], (unsigned long long)(u - tm));
        tm = u;
      }
    };
    // node i in every thread: a cached node straight from the LDS mirror (a uniform read, no
    // barrier: every mirrored node was written before a barrier all threads have passed), any
    // other through thread 0 -- so the levels earlier calls partitioned cost no barrier at all
    auto fetch_node = [&](int32_t i) -> SplitNode {
      if (i < NCACHE) return s_cache[i];
      if (t == 0) s_nd = nd[i];
      __syncthreads();
      const SplitNode r = s_nd;
      __syncthreads();
      return r;
    };
    SplitNode x = fetch_node(0);
    mark(0);
    for (;;) {
      if (x.fin) {
        if (t == 0) a.qout[q] = in_lds ? ((SP_LDS uint64_t *)LW)[pos - lbase] : W[pos];
        break;
      }
      if (x.left >= 0) {  // (never in LDS: the nodes visited there are fresh)
        idx = pos < x.cut ? x.left : x.left + 1;
        x = fetch_node(idx);
        mark(0);
        continue;
      }
      const int64_t n = x.hi - x.lo;
      if (!in_lds && n > 16 && n <= LMAX && x.depth > 0) {
        for (int64_t i = t; i < n; i += ST) LW[i] = W[x.lo + i];
        in_lds = true;
        lbase = x.lo;
        lend = x.hi;
        __syncthreads();
        mark(1);
      }
      SP_LDS uint64_t *fl = (SP_LDS uint64_t *)LW + (x.lo - lbase);
      uint64_t *fg = W + x.lo;
      if (n <= 16 || x.depth == 0) {  // a leaf, or the heapsort fallback below the depth limit
        if (t == 0) {
          if (in_lds) {
            if (n <= 16) insertion_sort_1(fl, n);
            else heap_sort_1(fl, n);
          } else {
            if (n <= 16) insertion_sort_1(fg, n);
            else heap_sort_1(fg, n);
          }
        }
        // the node is marked finished only after the barrier: a wave still reading this node
        // from the mirror (no barrier on that read) must see it unfinished, or it would leave
        // the walk and skip this barrier
        __syncthreads();
        if (t == 0) {
          nd[idx].fin = 1;
          if (idx < NCACHE) s_cache[idx].fin = 1;
        }
        x.fin = 1;
        mark(2);
        continue;
      }
      int64_t cut;
      const uint64_t tp0 = a.prof && t == 0 ? __builtin_amdgcn_s_memrealtime() : 0;
      if (in_lds && n <= WMAX && !a.nowave) {
        if (t < 64) {
          const int64_t c = partition_wave(fl, n, (SP_LDS uint16_t *)LL, (SP_LDS uint16_t *)LR, a.prof);
          if (t == 0) s64[0] = (uint64_t)c;
        }
        __syncthreads();
        cut = x.lo + (int64_t)s64[0];
        __syncthreads();  // (s64 is partition_wg's scratch too)
        if (a.prof && t == 0) {
          atomicAdd(&a.prof[14], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - tp0));
          atomicAdd(&a.prof[15], 1ull);
          atomicAdd(&a.prof[16], (unsigned long long)n);
        }
      } else {
        cut = x.lo + (in_lds ? partition_wg<uint16_t>(fl, n, LL, LR, s32, s64)
                             : partition_wg<uint32_t>(fg, n, L + x.lo, R + x.lo, s32, s64, a.prof,
                                                    (SP_LDS uint32_t *)LW, (SP_LDS uint32_t *)s_cnt));
      }
      if (t == 0) {
        if (s_nn + 2 > a.maxnode) {
          atomicMax(a.err, 1);
          nd[idx].fin = 1;  // (ends this query's walk; the call reports the error)
          if (idx < NCACHE) s_cache[idx].fin = 1;
          s_nd.fin = 1;
          s_idx = idx;
        } else {
          const SplitNode lc{x.lo, cut, 0, x.depth - 1, -1, 0, 0}, rc{cut, x.hi, 0, x.depth - 1, -1, 0, 0};
          nd[s_nn] = lc;
          nd[s_nn + 1] = rc;
          nd[idx].left = s_nn;
          nd[idx].cut = cut;
          if (s_nn < NCACHE) s_cache[s_nn] = lc;
          if (s_nn + 1 < NCACHE) s_cache[s_nn + 1] = rc;
          if (idx < NCACHE) {
            s_cache[idx].left = s_nn;
            s_cache[idx].cut = cut;
          }
          // (the child taken built from selects of its fields: a select of the two structs was
          // materialised in scratch memory, a store and a reload per partition)
          const bool goleft = pos < cut;
          s_idx = goleft ? s_nn : s_nn + 1;
          s_nd = SplitNode{goleft ? x.lo : cut, goleft ? cut : x.hi, 0, x.depth - 1, -1, 0, 0};
          s_nn += 2;
        }
      }
      __syncthreads();
      idx = s_idx;
      x = s_nd;
      __syncthreads();  // (s_nd is rewritten by the next uncached fetch or partition)
      mark(in_lds ? 4 : 3);
      if (a.prof && t == 0) atomicAdd(&a.prof[in_lds ? 7 : 6], 1ull);
    }
    if (in_lds) {  // the partitioned range back to the array
      __syncthreads();
      for (int64_t i = t; i < lend - lbase; i += ST) W[lbase + i] = LW[i];
    }
    __syncthreads();
    mark(5);
  }
  if (t == 0) a.nnodes[arr] = s_nn;
}

__global__ void split_words_kernel(const uint16_t *__restrict__ keys, const uint32_t *__restrict__ order, uint64_t n,
                                   uint32_t npiv, uint64_t *__restrict__ words) {
  const uint64_t total = n * npiv;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x)
    words[i] = ((uint64_t)keys[i] << 32) | order[i % n];
}

}  // namespace

int split_build_words(mc_ctx *c, const uint32_t *d_order, uint64_t n, uint32_t npiv, const uint16_t *d_keys,
                      uint64_t *d_words) {
  const uint64_t total = n * npiv;
  const int blocks = (int)std::min<uint64_t>((total + 255) / 256, 8192);
  split_words_kernel<<<blocks, 256, 0, c->stream>>>(d_keys, d_order, n, npiv, d_words);
  MCG_CHECK(hipGetLastError());
  return MC_OK;
}

int launch_select(mc_ctx *c, uint64_t *d_words, uint64_t n, uint32_t *d_scr, SplitNode *d_nodes, int32_t *d_nnodes,
                  int32_t maxnode, int32_t depth0, uint32_t ngroups, const uint32_t *d_qarr, const uint64_t *d_qoff,
                  const uint64_t *d_qpos, uint64_t *d_qout, int *d_err) {
  if (!ngroups) return MC_OK;
  static const bool prof = getenv("MC_SPLIT_PROFILE") != nullptr;
  static unsigned long long *d_prof = nullptr;
  if (prof && !d_prof) {
    MCG_CHECK(hipMalloc(&d_prof, 256));
    MCG_CHECK(hipMemset(d_prof, 0, 256));
  }
  SelArgs a;
  a.words = d_words;
  a.n = n;
  a.scr = d_scr;
  a.nodes = d_nodes;
  a.nnodes = d_nnodes;
  a.maxnode = maxnode;
  a.depth0 = depth0;
  a.qarr = d_qarr;
  a.qoff = d_qoff;
  a.qpos = d_qpos;
  a.qout = d_qout;
  a.err = d_err;
  a.prof = prof ? d_prof : nullptr;
  a.nowave = getenv("MC_SPLIT_NO_WAVE") ? 1 : 0;
  MCG_CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(&select_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)SEL_LDS));
  select_kernel<<<ngroups, ST, SEL_LDS, c->stream>>>(a);
  MCG_CHECK(hipGetLastError());
  if (prof) {  // this call, in us summed over workgroups
    unsigned long long h[32];
    MCG_CHECK(hipMemcpyAsync(h, d_prof, 256, hipMemcpyDeviceToHost, c->stream));
    MCG_CHECK(hipMemsetAsync(d_prof, 0, 256, c->stream));
    MCG_CHECK(hipStreamSynchronize(c->stream));
    fprintf(stderr, "[split] ngroups %u  sum over WGs (us): nodes %.0f lds-load %.0f leaf %.0f part-global %.0f (%llu) "
            "part-lds %.0f (%llu) writeback %.0f\n", ngroups, h[0] / 100.0, h[1] / 100.0, h[2] / 100.0, h[3] / 100.0,
            h[6], h[4] / 100.0, h[7], h[5] / 100.0);
    if (h[6])
      fprintf(stderr, "[split]   global partitions (us): median %.0f pass %.0f bisect %.0f swaps %.0f; words %llu swaps %llu\n",
              h[8] / 100.0, h[9] / 100.0, h[10] / 100.0, h[11] / 100.0, h[12], h[13]);
    if (h[15])
      fprintf(stderr, "[split]   one-wave partitions (us): %.0f (%llu, words %llu): stoppers %.0f bisect %.0f swaps %.0f (%llu)\n",
              h[14] / 100.0, h[15], h[16], h[17] / 100.0, h[18] / 100.0, h[19] / 100.0, h[20]);
  }
  return MC_OK;
}

}  // namespace mcg
