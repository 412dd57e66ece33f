// accum.hip -- the whole accumulation phase (ClusterFactory::MS's accumulate loop,
// ClusterFactory.cpp:637-714 and 717-730) as ONE persistent, cooperatively launched kernel.
//
// Every step of accumulation depends on the previous one (the next centre is the member
// closest to the cluster's mean), so the phase is a chain of ~2 steps per cluster, each a
// scan of the bvec window.  Driving that chain from the host costs a launch and a PCIe round
// trip per step; here the chain never leaves the GPU:
//
//   WG 0 (controller)   keeps the bvec in LDS -- an alive bitmap over static positions plus
//                       per-bin alive counts -- and runs bvec::get_range / the bvec_iterator
//                       window (bvec_core.hpp, the closed forms checked against the host
//                       restatement), pop / erase / remove_available, the cluster's running
//                       integer column sums, get_mean + Trainer::closest, and the cluster
//                       bookkeeping; it publishes each step's (centre, S, E) and collects the
//                       step's result.
//   all WGs             scan the window: Trainer::get_close (Trainer.cpp:34-114) on the
//                       chunk-major static layout, one lane per candidate, centre in LDS;
//                       similar candidates are killed and listed per workgroup, combo-0's
//                       first maximum is reduced per workgroup.
//
// Static chunk c (NT positions) is always scanned by workgroup c mod G, and G is a multiple
// of 8, so a chunk always lands on the same XCD and its rows stay in that XCD's L2; the alive
// flags of a workgroup's chunks live in its own LDS.
//
// Hand-offs carry only a few words, so they use sc1 stores and loads (relaxed agent-scope
// atomics: L1 bypassed, coherent across XCDs) with a drain before each signal instead of
// release/acquire fences (MI355X_MICROARCH.md hand-off table, first row).  The signal words
// carry the step number in their upper half, so a reader polls the payload itself and one
// L2 round trip per hand-off disappears:
//   controller -> workers   a step record in a ring {centre, S, E, kill-log length}, each word
//                           tagged with the step (after a drain of the kill log: pops / erases
//                           are appended to a log that owners apply before their next scan);
//                           workers poll the next step's slot; `go` = step only serves a
//                           workgroup that fell a whole ring behind
//   workers -> controller   flagged positions, drained, then a 4-word {max, position, count}
//                           partial, every word tagged with the step, polled by the controller
// Only the workgroups owning a chunk of the window take part in a step.  Every spin has a
// deadline, so a fault cannot leave a wave spinning forever (error 99).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "bvec_core.hpp"
#include "features.hpp"

namespace mcg {

namespace {

constexpr int NT = 512;
constexpr int NW = NT / 64;
constexpr uint32_t NONE = 0xffffffffu;
constexpr uint32_t MCAP = 1024;  // members of the current cluster mirrored in LDS
constexpr uint32_t RING = 64;    // step records kept for workgroups that read them late


// A workgroup's result for one step: {val high half, val low half, position, flagged count},
// each word tagged with the step in its upper 32 bits, so the controller polls the words
// themselves (no arrival counter) and accepts them when all four carry the step.
struct AccPartial {
  uint64_t w[4];
};

// Static part of a centre's bvec window (bvec::get_range, bvec.cpp:245-278), per point id:
// the window lengths, the bins index_of picks, and how many static positions of those bins
// are shorter than (or not longer than) the window lengths.  Only alive counts change during
// accumulation, so the controller turns these into inner_index_of's ranks with LDS popcounts.
struct WinTab {
  uint64_t bl, el;          // (uint64_t)(len * sim), (uint64_t)(len / sim)
  uint32_t fb, bb;          // index_of(bl).low, index_of(el).high
  uint32_t kf, kblt, kble;  // static positions of bin fb with length < bl; of bin bb < el, <= el
  uint32_t pad;
};

struct AccArgs {
  // chunk-major static layout (scan.hip build_static) and id-major rows (centre)
  const uint4 *hs;
  uint64_t npad;
  int nch, B;
  const uint64_t *mag_s, *sumsq_s, *len_s;
  // bvec structure
  uint64_t N;
  uint32_t nb;
  const uint32_t *bin_lo;    // nb + 1 static starts
  const uint64_t *bounds;    // nb begin_bounds
  double sim;
  const WinTab *wtab;        // per static position
  // hand-off (every handed-off word is stored and loaded with sc1 accesses, see below)
  uint64_t *ring;   // RING step records of 4 words
  uint32_t *klog;   // static positions killed by the controller (pop / erase), append-only
  uint32_t *go;     // latest published step (for a workgroup that fell RING steps behind)
  AccPartial *partials;
  uint32_t *flist;  // G * fcap
  uint64_t fcap;
  // output
  uint32_t *mem_pos;   // N: member static positions, cluster after cluster
  uint64_t *mkeys;     // N: (step << 32 | pos), 0 for a cluster's seed
  uint32_t *cl_centre; // N: static position of each cluster's centre
  uint64_t *cl_off;    // N + 1
  uint64_t *out;       // [0] clusters [1] steps [2] candidates [3] error [4] members
  uint64_t budget;     // longest wait for one hand-off, s_memrealtime ticks (100 MHz)
  int prof;            // controller phase timers (MC_ACCUM_PROFILE)
};

struct Red {  // LDS scratch for block-wide reductions and scans
  uint64_t a[NW], b[NW];
  double d[NW];
  uint64_t r0, r1;
};

__device__ __forceinline__ bool timed_out(const AccArgs &A, uint64_t t0) {
  return __builtin_amdgcn_s_memrealtime() - t0 > A.budget;
}

// Hand-off primitives.  Relaxed agent-scope atomics lower to global loads/stores with sc1:
// they bypass the CU's L1 and are coherent across XCDs without release/acquire fences when
// every handed-off word is written this way, each storing wave drains (vmcnt(0)) before
// the signal and every load of the words is also sc1 (MI355X_MICROARCH.md, hand-off table,
// first row).  The drain is inline asm so the compiler cannot drop it.
__device__ __forceinline__ void st64(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st32(uint32_t *p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld64(const uint64_t *p) {
  return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld32(const uint32_t *p) {
  return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// exclusive prefix of v over threads (thread order); *total = sum
__device__ uint64_t block_excl_scan(uint64_t v, uint64_t *total, Red &R) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t u = shfl64(inc, lane >= o ? lane - o : lane);
    if (lane >= o) inc += u;
  }
  __syncthreads();
  if (lane == 63) R.b[w] = inc;
  __syncthreads();
  uint64_t before = 0, tot = 0;
  for (int i = 0; i < NW; i++) {
    if (i < w) before += R.b[i];
    tot += R.b[i];
  }
  __syncthreads();
  *total = tot;
  return before + inc - v;
}

__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
  for (int o = 32; o >= 1; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
  return v;
}

// The bvec held by the controller workgroup: LDS bitmap of alive static positions, per-bin
// alive counts with a Fenwick tree over them, bin starts and begin bounds (bvec.cpp's bins
// after insert_finalize).  Every query is answered by each wave on its own from LDS (binary
// searches, Fenwick walks, one-wave popcount scans), so a query costs no workgroup barrier;
// callers keep queries uniform and put a barrier between kills and the next query.  The
// O(log) forms are checked against the host bvec in tests/native/bvec_check.cpp (FastAcc).
struct DevBvec {
  uint32_t *bits;
  uint32_t *cn;
  uint32_t *fw;          // Fenwick tree, fw[1..nb]
  const uint32_t *lo;    // LDS copy, nb + 1
  const uint64_t *bnd;   // LDS copy, nb
  const uint64_t *plen;  // global: length by static position (non-decreasing inside a bin)
  uint64_t nb, lg;       // lg: highest power of two <= nb
  WinTab h{~0ull, ~0ull, ~0u, ~0u, 0, 0, 0, 0};  // the current centre's static window data

  __device__ uint64_t nbins() const { return nb; }
  // accessor interface of bvec_core.hpp
  __device__ uint64_t cnt(uint64_t b) { return b < nb ? cn[b] : 0; }
  __device__ void index_of(uint64_t point, uint64_t *plow, uint64_t *phigh) {  // bvec.cpp:38-53
    bv_index_of_sorted(bnd, nb, point, plow, phigh);
  }
  __device__ uint64_t prefix(uint64_t b) { return bv_fw_prefix(fw, b < nb ? b : nb); }
  __device__ uint64_t total() { return prefix(nb); }
  __device__ void locate_rank(uint64_t rank, uint64_t *pb, uint64_t *pc) { bv_fw_locate(fw, nb, lg, rank, pb, pc); }
  __device__ int64_t first_nonempty() {
    if (!total()) return -1;
    uint64_t b, c;
    locate_rank(0, &b, &c);
    return (int64_t)b;
  }
  __device__ int64_t last_nonempty() {
    const uint64_t t = total();
    if (!t) return -1;
    uint64_t b, c;
    locate_rank(t - 1, &b, &c);
    return (int64_t)b;
  }
  __device__ uint32_t masked_word(uint64_t w, uint64_t p0, uint64_t p1) const {
    uint32_t word = bits[w];
    const uint64_t s = w << 5;
    if (s < p0) word &= ~0u << (p0 - s);
    if (s + 32 > p1) word &= (p1 - s) >= 32 ? ~0u : ((1u << (p1 - s)) - 1u);
    return word;
  }
  __device__ uint64_t alive_in(uint64_t p0, uint64_t p1) const {  // alive positions in [p0, p1)
    if (p0 >= p1) return 0;
    const uint64_t w0 = p0 >> 5, w1 = (p1 + 31) >> 5;
    uint32_t n = 0;
    for (uint64_t w = w0 + (threadIdx.x & 63); w < w1; w += 64) n += (uint32_t)__popc(masked_word(w, p0, p1));
    return wave_sum32(n);
  }
  // first position of [a, z) whose length is >= L (strict: > L)
  __device__ uint64_t len_bound(uint64_t a, uint64_t z, uint64_t L, bool strict) const {
    while (a < z) {
      const uint64_t m = (a + z) / 2;
      const uint64_t l = plen[m];
      if (strict ? l <= L : l < L) a = m + 1;
      else z = m;
    }
    return a;
  }
  __device__ uint64_t count_lt(uint64_t b, uint64_t L) {
    uint64_t k;
    if (b == h.fb && L == h.bl) k = lo[b] + h.kf;
    else if (b == h.bb && L == h.el) k = lo[b] + h.kblt;
    else k = len_bound(lo[b], lo[b + 1], L, false);
    return alive_in(lo[b], k);
  }
  __device__ uint64_t count_le(uint64_t b, uint64_t L) {
    const uint64_t k = b == h.bb && L == h.el ? lo[b] + h.kble : len_bound(lo[b], lo[b + 1], L, true);
    return alive_in(lo[b], k);
  }
  // static position of the c-th alive element of bin b (one wave: popcount scan over the words)
  __device__ uint64_t select(uint64_t b, uint64_t c) const {
    const int lane = threadIdx.x & 63;
    const uint64_t p0 = lo[b], p1 = lo[b + 1];
    const uint64_t w0 = p0 >> 5, w1 = (p1 + 31) >> 5;
    for (uint64_t base = w0; base < w1; base += 64) {
      const uint64_t w = base + lane;
      const uint32_t word = w < w1 ? masked_word(w, p0, p1) : 0u;
      const uint32_t pc = (uint32_t)__popc(word);
      uint32_t inc = pc;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = (uint32_t)__shfl_up((int)inc, o, 64);
        if (lane >= o) inc += u;
      }
      const uint32_t tot = (uint32_t)__shfl((int)inc, 63, 64);
      if (c < tot) {
        const uint64_t hit = __ballot(inc > c);
        const int L = __builtin_ctzll(hit);
        uint32_t x = (uint32_t)__shfl((int)word, L, 64);
        const uint32_t before = (uint32_t)__shfl((int)(inc - pc), L, 64);
        for (uint64_t k = c - before; k > 0; k--) x &= x - 1;
        return ((base + (uint64_t)L) << 5) + (uint64_t)__builtin_ctz(x);
      }
      c -= tot;
    }
    return ~0ull;
  }
  __device__ uint64_t bin_of(uint64_t p) const {  // single-thread binary search
    uint64_t a = 0, z = nb;  // lo[a] <= p < lo[z]
    while (z - a > 1) {
      const uint64_t m = (a + z) / 2;
      if (lo[m] <= p) a = m;
      else z = m;
    }
    return a;
  }
  // kill one static position (bvec::pop / erase / remove_available); any thread, atomics
  __device__ void kill_one(uint64_t p) {
    atomicAnd(&bits[p >> 5], ~(1u << (p & 31)));
    const uint64_t b = bin_of(p);
    atomicSub(&cn[b], 1u);
    for (uint64_t i = b + 1; i <= nb; i += i & (~i + 1)) atomicSub(&fw[i], 1u);
  }
  __device__ void invalidate() {}
};

// Column sums of rows[0..M) (static positions) added into sum[0..B) (LDS).  Thread (chunk c,
// row group g) accumulates chunk c of rows g, g + ng, ... in registers and adds its totals once,
// so the LDS atomics per step do not grow with the number of new members.
template <typename T>
__device__ void add_rows_acc(const RowRef &R, const uint32_t *rows, uint32_t M, int nch, uint64_t *sum) {
  constexpr int per = 16 / (int)sizeof(T);
  const int ng = nch < NT ? NT / nch : 1;
  for (int item = threadIdx.x; item < nch * ng; item += NT) {
    const int c = item % nch, grp = item / nch;
    uint64_t a[per];
#pragma unroll
    for (int e = 0; e < per; e++) a[e] = 0;
#pragma unroll 4
    for (uint32_t q = (uint32_t)grp; q < M; q += (uint32_t)ng) {
      const uint4 v = R.chunk(rows[q], c);
      const T *pv = reinterpret_cast<const T *>(&v);
#pragma unroll
      for (int e = 0; e < per; e++) a[e] += pv[e];
    }
#pragma unroll
    for (int e = 0; e < per; e++)
      if (a[e]) atomicAdd((unsigned long long *)&sum[c * per + e], (unsigned long long)a[e]);
  }
}

__device__ __forceinline__ bool better(double v, uint64_t p, double bv, uint64_t bp) {
  return v > bv || (v == bv && p < bp);
}

__device__ uint64_t lower_len(const uint64_t *len_s, uint64_t a, uint64_t z, uint64_t L, bool strict) {
  while (a < z) {
    const uint64_t m = (a + z) / 2;
    if (strict ? len_s[m] <= L : len_s[m] < L) a = m + 1;
    else z = m;
  }
  return a;
}

__global__ __launch_bounds__(256) void wintab_kernel(uint64_t n, const uint64_t *__restrict__ len_s,
                                                     const uint32_t *__restrict__ bin_lo,
                                                     const uint64_t *__restrict__ bnd, uint32_t nb, double sim,
                                                     WinTab *__restrict__ out) {
  for (uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x; id < n; id += (uint64_t)gridDim.x * 256) {
    const uint64_t L = len_s[id];  // id = static position
    WinTab w;
    w.bl = (uint64_t)((double)L * sim);  // get_range(len * sim, len / sim), ClusterFactory.cpp:650
    w.el = (uint64_t)((double)L / sim);
    uint64_t lo_, hi_;
    bv_index_of_sorted(bnd, nb, w.bl, &lo_, &hi_);
    w.fb = (uint32_t)lo_;
    bv_index_of_sorted(bnd, nb, w.el, &lo_, &hi_);
    w.bb = (uint32_t)hi_;
    w.kf = (uint32_t)(lower_len(len_s, bin_lo[w.fb], bin_lo[w.fb + 1], w.bl, false) - bin_lo[w.fb]);
    w.kblt = (uint32_t)(lower_len(len_s, bin_lo[w.bb], bin_lo[w.bb + 1], w.el, false) - bin_lo[w.bb]);
    w.kble = (uint32_t)(lower_len(len_s, bin_lo[w.bb], bin_lo[w.bb + 1], w.el, true) - bin_lo[w.bb]);
    w.pad = 0;
    out[id] = w;
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void accum_kernel(AccArgs A, DevClassifier C) {
  extern __shared__ __attribute__((aligned(16))) uint4 dyn[];
  __shared__ Red R;
  __shared__ uint32_t s_flag[NT];
  __shared__ uint32_t s_mpos[MCAP];  // current cluster: static positions and tie keys (first MCAP)
  __shared__ uint64_t s_mkey[MCAP];
  __shared__ uint32_t s_wcnt[NW];
  __shared__ double s_bv[NW];
  __shared__ uint64_t s_bp[NW];
  __shared__ uint32_t s_go;
  __shared__ uint64_t s_rec[4];
  __shared__ int s_abort;
  const uint32_t G = gridDim.x, g = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint4 *clds = dyn;  // centre chunks
  const RowRef Rs{A.hs, 1, A.npad};

  // ---------------- controller state (WG 0) ----------------------------------------------
  uint4 *Fl = dyn + A.nch;
  uint64_t *msum = reinterpret_cast<uint64_t *>(dyn + 2 * A.nch);
  uint32_t *cnt = reinterpret_cast<uint32_t *>(msum + A.B);
  uint32_t *fw = cnt + ((A.nb + 1) & ~1u);
  uint32_t *lo = fw + ((A.nb + 2) & ~1u);
  uint64_t *bnd = reinterpret_cast<uint64_t *>(lo + ((A.nb + 2) & ~1u));
  uint32_t *bits = reinterpret_cast<uint32_t *>(bnd + A.nb);
  // every workgroup: alive flags of the positions it owns (chunks g, g + G, ...), local index
  // (chunk / G) * NT + offset.  Flagged candidates are cleared by the owner; the controller's
  // pops and erases arrive through the kill log.
  uint8_t *lal = reinterpret_cast<uint8_t *>(bits + (A.N + 31) / 32);
  for (uint64_t i = threadIdx.x; i < A.fcap; i += NT) lal[i] = 1;
  uint32_t kcur = 0;  // kill-log entries applied so far
  uint64_t lg = 1;
  while (lg * 2 <= A.nb) lg *= 2;
  DevBvec bv{bits, cnt, fw, lo, bnd, A.len_s, A.nb, lg};
  const bool ctl = g == 0;
  // controller registers (uniform within WG 0)
  uint32_t last = NONE;      // current centre (static position)
  uint64_t cl_start = 0;     // first member index of the current cluster
  uint64_t M = 0;            // members of the current cluster
  uint64_t ncl = 0, nsteps = 0, ncand = 0;
  uint32_t step = 0;
  uint64_t err = 0;
  uint32_t kn = 0;                                   // kill-log length
  uint64_t t_win = 0, t_wait = 0, t_coll = 0, t_mark = 0;  // controller phase time, 100 MHz ticks
  uint64_t t_sub[4] = {0, 0, 0, 0};  // collect: reduce, gather+kill, column sums, closest

  auto finish_cluster = [&]() {
    if (threadIdx.x == 0) {
      A.cl_centre[ncl] = last;
      A.cl_off[ncl + 1] = cl_start + M;
    }
    ncl++;
    cl_start += M;
    M = 0;
  };
  auto new_cluster = [&](uint64_t pos) {  // accumulate's `current = {last}`
    if (threadIdx.x == 0) {
      A.mem_pos[cl_start] = (uint32_t)pos;
      A.mkeys[cl_start] = 0;
      s_mpos[0] = (uint32_t)pos;
      s_mkey[0] = 0;
    }
    for (int b = threadIdx.x; b < A.B; b += NT) msum[b] = elem<T>(Rs, pos, b);
    M = 1;
    __syncthreads();
  };
  auto pop = [&]() -> uint64_t {  // bvec::pop (bvec.cpp:26-37): static position or ~0
    const int64_t b = bv.first_nonempty();
    if (b < 0) return ~0ull;
    const uint64_t p = bv.select((uint64_t)b, 0);
    if (threadIdx.x == 0) {
      bv.kill_one(p);
      st32(A.klog + kn, (uint32_t)p);
    }
    kn++;
    __syncthreads();
    bv.invalidate();
    return p;
  };

  if (ctl) {
    // bvec after insert_finalize: every static position alive
    for (uint64_t i = threadIdx.x; i <= A.nb; i += NT) lo[i] = A.bin_lo[i];
    for (uint64_t i = threadIdx.x; i < A.nb; i += NT) {
      bnd[i] = A.bounds[i];
      cnt[i] = A.bin_lo[i + 1] - A.bin_lo[i];
    }
    __syncthreads();
    for (uint64_t i = threadIdx.x + 1; i <= A.nb; i += NT) {  // Fenwick node i covers bins (i - lowbit(i), i]
      uint32_t t = 0;
      for (uint64_t b = i - (i & (~i + 1)); b < i; b++) t += cnt[b];
      fw[i] = t;
    }
    const uint64_t nwords = (A.N + 31) / 32;
    for (uint64_t w = threadIdx.x; w < nwords; w += NT) {
      const uint64_t rem = A.N - w * 32;
      bits[w] = rem >= 32 ? ~0u : ((1u << rem) - 1u);
    }
    if (threadIdx.x == 0) A.cl_off[0] = 0;
    __syncthreads();
    const uint64_t p = pop();  // MS: Point<T>* last = points.pop()
    if (p != ~0ull) {
      last = (uint32_t)p;
      new_cluster(p);
    }
  }

  uint32_t seen = 0;
  for (;;) {
    // ============ controller: advance the accumulate loop to the next scan step ============
    if (ctl) {
      if (A.prof && threadIdx.x == 0) t_mark = __builtin_amdgcn_s_memrealtime();
      uint64_t S = 0, E = 0;
      bool have = false;
      while (last != NONE && !err) {
        bv.h = A.wtab[last];
        BPos f, b;
        bv_get_range(bv, bv.h.bl, bv.h.el, f, b);
        int e = 0;
        const int64_t count = bv_window(bv, f, b, &S, &E, &e);
        if (e) {
          err = 10 + e;
          break;
        }
        if (count > 0) {
          ncand += (uint64_t)count;
          have = true;
          break;
        }
        // the OpenMP loop ran no iteration: is_min with a NULL result -> pop a new seed
        const uint64_t p = pop();
        finish_cluster();
        last = p == ~0ull ? NONE : (uint32_t)p;
        if (p != ~0ull) new_cluster(p);
      }
      step++;
      if (have) nsteps++;
      if (threadIdx.x == 0) {
        // step record: every word carries the step in its upper half (positions < 2^31), so a
        // reader that finds all four tags equal to the step it was signalled holds an untorn
        // record even if the slot is being reused
        uint64_t *r = A.ring + (uint64_t)(step % RING) * 4;
        const uint64_t tag = (uint64_t)step << 32;
        drain();  // kill-log entries complete before the record that announces them
        st64(r + 0, tag | (have ? last : NONE));
        st64(r + 1, tag | S);
        st64(r + 2, tag | E);
        st64(r + 3, tag | kn);
        // `go` is only a hint for a workgroup that fell RING steps behind: it re-validates the
        // record's tags after reading it, so no drain is needed between the two
        st32(A.go, step);
        if (A.prof) {
          const uint64_t t = __builtin_amdgcn_s_memrealtime();
          t_win += t - t_mark;
          t_mark = t;
        }
      }
    }
    // ============ everyone: wait for the step ============================================
    if (threadIdx.x == 0) {
      s_abort = 0;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      // steps are published in order: poll the next step's record itself (its words carry
      // the step); a workgroup that finds the slot already rewritten for a later step fell
      // RING steps behind and catches up through `go`
      const uint32_t want = seen + 1;
      const uint64_t *rn = A.ring + (uint64_t)(want % RING) * 4;
      bool late = false;
      for (uint32_t it = 1;; it++) {
        const uint64_t w0 = ld64(rn + 0), w1 = ld64(rn + 1), w2 = ld64(rn + 2), w3 = ld64(rn + 3);
        const uint32_t t_0 = (uint32_t)(w0 >> 32), t_1 = (uint32_t)(w1 >> 32), t_2 = (uint32_t)(w2 >> 32),
                       t_3 = (uint32_t)(w3 >> 32);
        if (t_0 == want && t_1 == want && t_2 == want && t_3 == want) {
          s_rec[0] = w0;
          s_rec[1] = (uint32_t)w1;
          s_rec[2] = (uint32_t)w2;
          s_rec[3] = w3;
          s_go = want;
          break;
        }
        if ((int32_t)(t_0 - want) > 0 || (int32_t)(t_1 - want) > 0 || (int32_t)(t_2 - want) > 0 ||
            (int32_t)(t_3 - want) > 0) {
          late = true;
          break;
        }
        if ((it & 255) == 0 && timed_out(A, t0)) {
          s_abort = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      while (late) {
        uint32_t v;
        for (uint32_t it = 1; (v = ld32(A.go)) == seen; it++) {
          if ((it & 255) == 0 && timed_out(A, t0)) break;  // deadline checked every 256 polls
          __builtin_amdgcn_s_sleep(1);
        }
        if (v == seen) {
          s_abort = 1;
          break;
        }
        const uint64_t *r = A.ring + (uint64_t)(v % RING) * 4;
        const uint64_t w0 = ld64(r + 0), w1 = ld64(r + 1), w2 = ld64(r + 2), w3 = ld64(r + 3);
        if ((w0 >> 32) == v && (w1 >> 32) == v && (w2 >> 32) == v && (w3 >> 32) == v) {
          s_rec[0] = w0;
          s_rec[1] = (uint32_t)w1;
          s_rec[2] = (uint32_t)w2;
          s_rec[3] = w3;
          s_go = v;
          break;
        }
        // that slot is being rewritten for a later step: read `go` again
      }
    }
    __syncthreads();
    if (s_abort) {
      if (threadIdx.x == 0) atomicMax((unsigned long long *)&A.out[3], 99ull);
      return;
    }
    seen = s_go;
    struct {
      uint32_t centre;
      uint64_t S, E;
      uint32_t step;
    } P{(uint32_t)s_rec[0], s_rec[1], s_rec[2], seen};
    const uint32_t kend = (uint32_t)s_rec[3];
    if (P.centre == NONE) break;

    // ============ workgroups owning chunks of the window: scan them (Trainer::get_close) ===
    // Chunk c0 + i belongs to workgroup (c0 + i) mod G; only the nact workgroups owning a
    // chunk of [S, E] take part in the step (and arrive), the others wait for the next go.
    const uint64_t c0 = P.S / NT, c1 = P.E / NT;
    const uint32_t nact = (uint32_t)(c1 - c0 + 1 < (uint64_t)G ? c1 - c0 + 1 : (uint64_t)G);
    const uint32_t mine = (g + G - (uint32_t)(c0 % G)) % G;
    if (mine < nact) {
    // The centre's chunks (staged in LDS below) and magnitudes depend only on the step record:
    // loaded before the kill log is applied, so they share one round trip with the log's.
    // (Prefetching the first chunk of candidate rows too would hold 64 more VGPRs across the
    // barrier: the kernel then spills.)
    const uint64_t ch0 = c0 + mine;
    uint4 cpre = make_uint4(0, 0, 0, 0);
    if (threadIdx.x < A.nch) cpre = Rs.chunk(P.centre, threadIdx.x);
    const PInfo pc{A.mag_s[P.centre], A.sumsq_s[P.centre], A.len_s[P.centre]};
    for (uint64_t i = kcur + threadIdx.x; i < kend; i += NT) {  // controller kills since last time
      const uint32_t p = ld32(A.klog + i);
      const uint64_t ch = p / NT;
      if (ch % G == g) lal[(ch / G) * NT + p % NT] = 0;
    }
    kcur = kend;
    if (threadIdx.x < A.nch) clds[threadIdx.x] = cpre;
    for (int c = NT + threadIdx.x; c < A.nch; c += NT) clds[c] = Rs.chunk(P.centre, c);
    __syncthreads();
    double best_v = -1.0;
    uint64_t best_p = ~0ull;
    uint32_t nfl = 0;  // this workgroup's flagged count (uniform)
    for (uint64_t ch = ch0; ch <= c1; ch += G) {
      const uint64_t pos = ch * NT + threadIdx.x;
      uint8_t *la = lal + (ch / G) * NT + threadIdx.x;
      const bool valid = pos >= P.S && pos <= P.E && *la;
      int d = 0;
      if (valid) {
        Acc<T> acc;
        const uint4 *col = A.hs + pos;
        PInfo pi;
        if (A.nch == 16) {
          uint4 v[16];
#pragma unroll
          for (int k = 0; k < 16; k++) v[k] = col[(uint64_t)k * A.npad];
          pi = PInfo{A.mag_s[pos], A.sumsq_s[pos], A.len_s[pos]};
#pragma unroll
          for (int k = 0; k < 16; k++) acc.add(v[k], clds[k]);
        } else {
#pragma unroll 8
          for (int k = 0; k < A.nch; k++) acc.add(col[(uint64_t)k * A.npad], clds[k]);
          pi = PInfo{A.mag_s[pos], A.sumsq_s[pos], A.len_s[pos]};
        }
        const PS s = acc.finish(pi.mag, pc.mag);
        double raw[MC_MAX_SINGLE];
#pragma unroll
        for (int i = 0; i < MC_MAX_SINGLE; i++)
          raw[i] = i < C.c.n_single ? raw_fast(C.c.lookup[i], s, pi, pc, A.B) : 0.0;  // compute(*pt, *p)
        double cv;
        d = classify_raw(C, raw, &cv, nullptr);
        if (cv > -1.0 && better(cv, pos, best_v, best_p)) {
          best_v = cv;
          best_p = pos;
        }
        if (d) *la = 0;
      }
      // ordered compaction of this chunk's flagged positions (ascending position)
      const uint64_t bal = __ballot(d);
      if (lane == 0) s_wcnt[wv] = (uint32_t)__popcll(bal);
      __syncthreads();
      uint32_t before = nfl;
      uint32_t tot = 0;
      for (int i = 0; i < NW; i++) {
        if (i < wv) before += s_wcnt[i];
        tot += s_wcnt[i];
      }
      if (d) st32(A.flist + (uint64_t)g * A.fcap + before + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull)), (uint32_t)pos);
      nfl += tot;
      __syncthreads();
    }
    for (int o = 32; o >= 1; o >>= 1) {
      const double ov = __shfl_xor(best_v, o, 64);
      const uint64_t op = shfl_xor64(best_p, o);
      if (better(ov, op, best_v, best_p)) {
        best_v = ov;
        best_p = op;
      }
    }
    if (lane == 0) {
      s_bv[wv] = best_v;
      s_bp[wv] = best_p;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // flag / alive stores of every wave drained
    __syncthreads();
    if (threadIdx.x == 0) {
      double v = s_bv[0];
      uint64_t p = s_bp[0];
      for (int i = 1; i < NW; i++)
        if (better(s_bv[i], s_bp[i], v, p)) {
          v = s_bv[i];
          p = s_bp[i];
        }
      // every wave's list / alive stores were drained before the barrier: the tagged partial
      // words are the signal
      uint64_t *q = A.partials[g].w;
      const uint64_t tag = (uint64_t)P.step << 32, vb = (uint64_t)__double_as_longlong(v);
      st64(q + 0, tag | (vb >> 32));
      st64(q + 1, tag | (vb & 0xffffffffull));
      st64(q + 2, tag | (p == ~0ull ? (uint64_t)NONE : p));
      st64(q + 3, tag | nfl);
    }
    }  // active workgroup
    if (!ctl) continue;

    // ============ controller: collect the step (get_close's reduction + get_mean) =========
    // thread t polls the partial of the t-th active workgroup until its four words carry this
    // step (s_abort is 0 here: set only on a failed wait, which returns)
    double bv_ = -1.0;
    uint64_t bp_ = ~0ull, cnt_w = 0;
    if (threadIdx.x < nact) {
      const uint64_t *q = A.partials[(c0 + threadIdx.x) % G].w;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (uint32_t it = 1;; it++) {
        const uint64_t w0 = ld64(q + 0), w1 = ld64(q + 1), w2 = ld64(q + 2), w3 = ld64(q + 3);
        if ((uint32_t)(w0 >> 32) == P.step && (uint32_t)(w1 >> 32) == P.step && (uint32_t)(w2 >> 32) == P.step &&
            (uint32_t)(w3 >> 32) == P.step) {
          bv_ = __longlong_as_double((long long)((w0 << 32) | (w1 & 0xffffffffull)));
          const uint32_t p32 = (uint32_t)w2;
          bp_ = p32 == NONE ? ~0ull : (uint64_t)p32;
          cnt_w = (uint32_t)w3;
          break;
        }
        if ((it & 255) == 0 && timed_out(A, t0)) {
          s_abort = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (A.prof && threadIdx.x == 0) {
      const uint64_t t = __builtin_amdgcn_s_memrealtime();
      t_wait += t - t_mark;
      t_mark = t;
    }
    __syncthreads();
    if (s_abort) {
      if (threadIdx.x == 0) atomicMax((unsigned long long *)&A.out[3], 99ull);
      return;
    }
    // first maximum over workgroups, flagged counts and their offsets
    uint64_t nflag;
    const uint64_t off_w = block_excl_scan(cnt_w, &nflag, R);
    if (threadIdx.x < nact) s_flag[threadIdx.x] = (uint32_t)off_w;  // nact <= G <= NT
    for (int o = 32; o >= 1; o >>= 1) {
      const double ov = __shfl_xor(bv_, o, 64);
      const uint64_t op = shfl_xor64(bp_, o);
      if (better(ov, op, bv_, bp_)) {
        bv_ = ov;
        bp_ = op;
      }
    }
    if (lane == 0) {
      s_bv[wv] = bv_;
      s_bp[wv] = bp_;
    }
    __syncthreads();
    double best_val = s_bv[0];
    uint64_t best_pos = s_bp[0];
    for (int i = 1; i < NW; i++)
      if (better(s_bv[i], s_bp[i], best_val, best_pos)) {
        best_val = s_bv[i];
        best_pos = s_bp[i];
      }
    uint64_t tq = 0;
    if (A.prof && threadIdx.x == 0) {
      tq = __builtin_amdgcn_s_memrealtime();
      t_sub[0] += tq - t_mark;
    }
    if (nflag > 0) {
      // remove_available: the flagged positions join the cluster (keys keep bvec order)
      const uint64_t mb = cl_start + M;
      for (uint64_t i = threadIdx.x; i < nflag; i += NT) {
        uint32_t a = 0, z = nact;  // last active workgroup with offset <= i
        while (z - a > 1) {
          const uint32_t m = (a + z) / 2;
          if (s_flag[m] <= i) a = m;
          else z = m;
        }
        const uint32_t p = ld32(A.flist + (uint64_t)((c0 + a) % G) * A.fcap + (i - s_flag[a]));
        const uint64_t key = ((uint64_t)P.step << 32) | p;
        A.mem_pos[mb + i] = p;
        A.mkeys[mb + i] = key;
        if (M + i < MCAP) {
          s_mpos[M + i] = p;
          s_mkey[M + i] = key;
        }
        bv.kill_one(p);
      }
      __syncthreads();
      if (A.prof && threadIdx.x == 0) {
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        t_sub[1] += t - tq;
        tq = t;
      }
      // row indices from LDS when the cluster fits there: the chunk loads are then the only
      // global round trip
      const bool in_lds = M + nflag <= MCAP;
      add_rows_acc<T>(Rs, in_lds ? s_mpos + M : A.mem_pos + mb, (uint32_t)nflag, A.nch, msum);
      M += nflag;
      __syncthreads();
      if (A.prof && threadIdx.x == 0) {
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        t_sub[2] += t - tq;
        tq = t;
      }
      const uint64_t win0 = mean_closest_fast<T, NT>(Rs, in_lds ? s_mpos : A.mem_pos + cl_start,
                                                     in_lds ? s_mkey : A.mkeys + cl_start, (uint32_t)M,
                                                     A.mag_s, A.B, A.nch, msum, Fl);
      if (threadIdx.x == 0) R.r0 = win0;  // the winner is thread 0's; make it uniform
      __syncthreads();
      const uint64_t win = R.r0;
      __syncthreads();
      if (A.prof && threadIdx.x == 0) t_sub[3] += __builtin_amdgcn_s_memrealtime() - tq;
      last = (uint32_t)win;
      bv.invalidate();
    } else if (best_pos != ~0ull) {
      // is_min with a result: the best candidate seeds the next cluster (bvec::erase)
      if (threadIdx.x == 0) {
        bv.kill_one(best_pos);
        st32(A.klog + kn, (uint32_t)best_pos);
      }
      kn++;
      __syncthreads();
      bv.invalidate();
      finish_cluster();
      last = (uint32_t)best_pos;
      new_cluster(best_pos);
    } else {
      const uint64_t p = pop();
      finish_cluster();
      last = p == ~0ull ? NONE : (uint32_t)p;
      if (p != ~0ull) new_cluster(p);
    }
    __syncthreads();
    if (A.prof && threadIdx.x == 0) {
      const uint64_t t = __builtin_amdgcn_s_memrealtime();
      t_coll += t - t_mark;
    }
  }
  if (ctl && threadIdx.x == 0) {
    A.out[0] = ncl;
    A.out[1] = nsteps;
    A.out[2] = ncand;
    if (err) atomicMax((unsigned long long *)&A.out[3], (unsigned long long)err);
    A.out[4] = cl_start;
    A.out[5] = t_win;
    A.out[6] = t_wait;
    A.out[7] = t_coll;
    for (int i = 0; i < 4; i++) A.out[8 + i] = t_sub[i];
  }
}

}  // namespace

// Grid: one workgroup per CU, a multiple of the 8 XCDs.
static uint32_t accum_grid(const mc_ctx *c) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess) cus = 256;
  uint32_t G = (uint32_t)cus / 8 * 8;
  if (G > (uint32_t)NT) G = NT;
  if (G < 8) G = 8;
  return G;
}
// positions owned by one workgroup (its chunks g, g + G, ...)
static uint64_t accum_fcap(const mc_ctx *c, uint32_t G) {
  const uint64_t chunks = (c->norder + NT - 1) / NT;
  return ((chunks + G - 1) / G) * NT;
}

// LDS bytes: controller state + the per-workgroup alive flags (all workgroups get the same
// allocation)
static size_t accum_lds(const mc_ctx *c, uint32_t nb, uint32_t G) {
  const int nch = (int)((c->B * c->width + 15) / 16);
  return (size_t)2 * nch * 16 + (size_t)c->B * 8 + (size_t)((nb + 1) & ~1u) * 4 + (size_t)((nb + 2) & ~1u) * 8 +
         (size_t)nb * 8 + (c->norder + 31) / 32 * 4 + accum_fcap(c, G);
}

bool accum_supported(const mc_ctx *c, uint32_t nb) {
  if (c->width != 1 && c->width != 2) return false;
  if (c->cls.align) return false;
  if (c->norder >= (1ull << 31)) return false;
  // + static LDS (reductions, member mirror) and headroom
  return accum_lds(c, nb, accum_grid(c)) + 24 * 1024 <= 160 * 1024;
}

int launch_accum(mc_ctx *c, const uint32_t *d_bin_lo, const uint64_t *d_bounds, uint32_t nb, double sim,
                 uint32_t *d_mem_pos, uint64_t *d_mkeys, uint32_t *d_cl_centre, uint64_t *d_cl_off, uint64_t *d_out) {
  const uint32_t G = accum_grid(c);
  const size_t lds = accum_lds(c, nb, G);
  const void *fn = c->width == 1 ? reinterpret_cast<const void *>(&accum_kernel<uint8_t>)
                                 : reinterpret_cast<const void *>(&accum_kernel<uint16_t>);
  MCG_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int per_cu = 0;
  MCG_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, NT, lds));
  if (per_cu < 1) {
    set_error("accumulation kernel does not fit on a CU");
    return MC_ERR_HIP;
  }
  const uint64_t fcap = accum_fcap(c, G);
  const size_t hand = 256 + (size_t)RING * 32;  // go, step ring
  const size_t part_bytes = ((size_t)G * sizeof(AccPartial) + 255) / 256 * 256;
  const size_t flist_bytes = ((size_t)G * fcap * 4 + 255) / 256 * 256;
  if (ensure(c->s_a, hand) || ensure(c->s_b, part_bytes + c->n * sizeof(WinTab)) ||
      ensure(c->s_c, flist_bytes + c->norder * 4 + 16))
    return MC_ERR_OOM;
  WinTab *d_wtab = (WinTab *)((char *)c->s_b.p + part_bytes);
  timed_begin(c);
  wintab_kernel<<<(int)std::min<uint64_t>((c->n + 255) / 256, 2048), 256, 0, c->stream>>>(
      c->norder, (const uint64_t *)c->len_s.p, d_bin_lo, d_bounds, nb, sim, d_wtab);
  MCG_CHECK(hipGetLastError());
  timed_end(c, F_FINAL);
  MCG_CHECK(hipMemsetAsync(c->s_a.p, 0, hand, c->stream));
  MCG_CHECK(hipMemsetAsync(c->s_b.p, 0, part_bytes, c->stream));  // no partial carries a step tag yet
  AccArgs A;
  memset(&A, 0, sizeof A);
  A.hs = (const uint4 *)c->hs.p;
  A.npad = c->npad;
  A.nch = (int)((c->B * c->width + 15) / 16);
  A.B = c->B;
  A.mag_s = (const uint64_t *)c->mag_s.p;
  A.sumsq_s = (const uint64_t *)c->sumsq_s.p;
  A.len_s = (const uint64_t *)c->len_s.p;
  A.N = c->norder;
  A.nb = nb;
  A.bin_lo = d_bin_lo;
  A.bounds = d_bounds;
  A.sim = sim;
  A.wtab = d_wtab;
  A.go = (uint32_t *)c->s_a.p;
  A.ring = (uint64_t *)((char *)c->s_a.p + 256);
  A.partials = (AccPartial *)c->s_b.p;
  A.flist = (uint32_t *)c->s_c.p;
  A.klog = (uint32_t *)((char *)c->s_c.p + flist_bytes);
  A.fcap = fcap;
  A.mem_pos = d_mem_pos;
  A.mkeys = d_mkeys;
  A.cl_centre = d_cl_centre;
  A.cl_off = d_cl_off;
  A.out = d_out;
  A.budget = 20ull * 100000000ull;  // a single hand-off never takes 20 s: give up, report error 99
  A.prof = getenv("MC_ACCUM_PROFILE") ? 1 : 0;
  DevClassifier cls = c->cls;
  void *args[] = {&A, &cls};
  timed_begin(c);
  MCG_CHECK(hipLaunchCooperativeKernel(fn, dim3(G), dim3(NT), args, (unsigned)lds, c->stream));
  timed_end(c, F_SCAN);
  return MC_OK;
}

}  // namespace mcg
