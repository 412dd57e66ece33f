// accum_impl.hpp -- the whole accumulation phase (ClusterFactory::MS's accumulate loop,
// ClusterFactory.cpp:637-714 and 717-730) as ONE persistent, cooperatively launched kernel.
//
// Every step of accumulation depends on the previous one (the next centre is the member
// closest to the cluster's mean), so the phase is a chain of ~2 steps per cluster, each a
// scan of the bvec window.  The chain never leaves the GPU:
//
//   WG 0 (controller)   keeps the bvec -- an alive bitmap over static positions (LDS, or
//                       global memory for very large n) plus per-bin alive counts with a
//                       Fenwick tree -- and runs bvec::get_range / the bvec_iterator window
//                       (bvec_core.hpp: four nearest-alive queries when both edge bins hold
//                       alive elements, the general closed forms otherwise), pop / erase /
//                       remove_available, the cluster's integer column sums, get_mean +
//                       Trainer::closest over a member cache in LDS, and publishes each step.
//   every WG            scans the chunks of the window it owns: Trainer::get_close
//                       (Trainer.cpp:34-114), one lane per candidate, centre in LDS; similar
//                       candidates are killed and handed over with their histogram rows, the
//                       first maximum of combo 0 is reduced per workgroup.
//
// Static chunk c (NT positions) always belongs to workgroup c mod G, and G is a multiple of the
// 8 XCDs, so a chunk stays on one XCD.  When every workgroup owns at most RES chunks (n up to
// RES * G * NT: 131k reads per chunk slot on 256 CUs) the chunks' histogram rows are loaded
// into registers once and stay there for the whole phase: a step then reads no candidate
// bytes from memory at all.  Larger n streams the window's rows from HBM every step.
//
// Hand-offs are 8-byte {step tag, data} granules written with sc1 stores and read with sc1
// loads, so a reader that sees every tag equal to the step it waits for holds an untorn
// record without a fence (MI355X_MICROARCH.md, hand-off table row 1; data-tagged granules as
// in handoff-1to1):
//   controller -> workers   the step record: centre row + magnitudes, window S..E, kill-log
//                           length and its last KINL entries (pops / erases)
//   workers -> controller   an 8-granule partial {max, position, flagged, scanned, the first
//                           INL flagged positions} (further flagged positions in a list, sc1
//                           stores drained before the partial); the controller loads the
//                           flagged rows from the read-only static layout itself, while it is
//                           still waiting for the slower workers
// Every spin has a deadline (error 99: never a hang).
#pragma once
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
constexpr uint64_t NONE64 = ~0ull;
constexpr uint32_t RING = 64;          // step records kept for workgroups that read them late
constexpr uint32_t TRACE_STEPS = 4096;
constexpr int TRACE_W = 20;            // trace words per step (MC_ACCUM_PROFILE=2), see trace_mark
constexpr uint32_t TRACE2_STEPS = 256;
constexpr int T2W = 6;  // trace2 words per worker and step
constexpr int KINL = 4;                // kill-log entries carried inline in a step record
constexpr int REC_HDR = 14;            // centre, S, E, kn, KINL kills, mag / sumsq / len (2 each)
// flags in the record's kill-log word (header word 3): the span is the exact window; a thin
// record (a new seed's: no row, no magnitudes -- the dense workers load them)
constexpr uint32_t REC_EXACT = 0x80000000u, REC_THIN = 0x40000000u, REC_KMASK = 0x3fffffffu;
constexpr int PART_G = 8;              // granules per partial
constexpr int INL = 3;                 // flagged positions carried inline in a partial
constexpr uint32_t PLIST = 1024;       // flagged positions of one step listed in the controller's LDS
constexpr uint32_t GMAX = 256;         // workgroups: the controller polls the G - 1 workers' partials with one thread each
// Wide rows (B * w >= 512 bytes: k >= 5 at 8 bits, k >= 4 at 16): a wave scores one candidate
// (64 lanes over the row, read row-major from `hr`), so a tile of NW candidates is the unit of
// ownership instead of a 512-position chunk, and a few-hundred-candidate window spreads over
// dozens of workers instead of the one or two that own its chunks.
constexpr int WIDE_NCH = 32;
// Several ranks (GPUs) sharing one accumulation: global tile t belongs to rank t mod W, whose
// worker (t / W) mod GW scans it.  Each rank's controller keeps the whole (replicated) chain
// state and exchanges, per step, {first max, flagged positions} with the other ranks' kernels
// through a mailbox in host memory shared by all of them: MBOX_HDR granules per rank and step
// (the first MBOX_INL flagged positions inline, so a step with few flags per rank needs one
// read round), then its further flagged positions, every granule tagged with the step; two
// parities of slots, since a rank can be at most one step ahead of another.
constexpr int MBOX_HDR = 16;  // best value hi / lo, best position, flagged, scanned, inline flags
constexpr int MBOX_INL = MBOX_HDR - 5;

// Static part of a centre's bvec window (bvec::get_range, bvec.cpp:245-278), per static
// position: the window lengths, the bins index_of picks, and how many static positions of
// those bins are shorter than (or not longer than) the window lengths.
struct WinTab {
  uint64_t bl, el;          // (uint64_t)(len * sim), (uint64_t)(len / sim)
  uint32_t fb, bb;          // index_of(bl).low, index_of(el).high
  uint32_t kf, kblt, kble;  // static positions of bin fb with length < bl; of bin bb < el, <= el
  uint32_t pad;
};

// What the controller needs of a static position when it joins a cluster: magnitudes and
// window data, one 64-byte line (its row is in the row-major static copy `hr`)
struct MInfo {
  uint64_t mag, sumsq, len, bin;  // bin: the bvec bin holding this static position
  WinTab wt;
};
static_assert(sizeof(MInfo) % 8 == 0, "MInfo is loaded as 8-byte words");
constexpr int MINFO_W = (int)(sizeof(MInfo) / 8);

// A position's MInfo as independent 8-byte loads (issue them all, then `minfo_take`): a struct
// copy is split into field loads that the compiler places next to each use, one memory round
// trip at a time when LDS stores (generic pointers) sit in between.
__device__ __forceinline__ void minfo_issue(const MInfo *m, uint2 (&w)[MINFO_W]) {
  const uint2 *s = reinterpret_cast<const uint2 *>(m);
#pragma unroll
  for (int k = 0; k < MINFO_W; k++) w[k] = s[k];
}
__device__ __forceinline__ MInfo minfo_take(uint2 (&w)[MINFO_W]) {
#pragma unroll
  for (int k = 0; k < MINFO_W; k++) asm volatile("" : "+v"(w[k].x), "+v"(w[k].y));
  MInfo r;
  __builtin_memcpy(&r, w, sizeof(MInfo));
  return r;
}

struct AccArgs {
  int dbg;     // MC_ACCUM_DBG bits (opt-in variants, both measured slower at config B): 1 per-bin
               // aggregated bvec kills (window 3.9 -> 20.2 ms), 2 quad-per-member closest search
  FastCls fc;  // the workers' division-light decision (features.hpp classify_fast)
  // chunk-major static layout (scan.hip build_static)
  const uint4 *hs;
  uint64_t npad;
  int nch, B;
  const uint64_t *mag_s, *sumsq_s, *len_s;
  // bvec structure
  uint64_t N;
  uint32_t nb;
  const uint32_t *bin_lo;  // nb + 1 static starts
  const uint64_t *bounds;  // nb begin_bounds
  const MInfo *minfo;      // per static position
  const uint4 *hr;         // rows in static order, row-major (nch chunks each)
  uint32_t *gbits;         // alive bitmap in global memory (n too large for LDS), else null
  // hand-off
  uint64_t *ring;  // RING records of rec_g granules
  uint64_t *ringb;  // spec: RING x 2 granules, the exact window {S, E} of step s (NONE: no scan)
  int spec;         // the record carries a superset of the window; the exact one follows (dense)
  int poll1;        // the controller polls a partial's tag granule before loading it whole
  int psleep;       // s_sleep between the controller's polls of a partial (0, 1, 2, 4)
  int etake;        // a polling thread takes its worker's flagged members as soon as it has the partial
  int xfast;        // nearest-alive window also when an edge bin is empty (off: MC_ACCUM_NO_XFAST)
  int thin;         // dense (and dense streaming) workers: a new seed's record goes out without its row (the workers
                    // load it), before the controller has loaded the seed (MC_ACCUM_THIN=0: off)
  int rpoll;        // dense workers: waves polling the step record (MC_ACCUM_RPOLL, 1..4)
  int rpoll_gap;    // ... wave w starts w * rpoll_gap * 512 clocks late (MC_ACCUM_RPOLL_GAP)
  uint32_t rec_g;
  uint64_t *klog;      // static positions killed by the controller (pop / erase), append-only,
                       // entry e a granule tagged e + 1 (a reader checks the tag: no drain
                       // is needed before the step record that counts it)
  uint32_t *go;        // latest published step (for a workgroup that fell RING steps behind)
  uint64_t *partials;  // G * PART_G granules
  uint32_t *fpos;      // worker w's flagged positions beyond the INL inline ones, at w * fcap
  uint64_t fcap;
  int res;        // chunks per worker whose rows live in its LDS (0: rows stream from memory)
  uint4 *cc;      // streaming: per-chunk compacted copies of the alive rows (null: read hs)
  uint4 *srows;   // dense streaming workers: two row buffers of fcap entries per worker
  uint32_t dres;  // ... entries 0 .. dres-1 of a worker's list (each thread's first) also in its
                  // LDS, which the controller's member cache sizes the launch's LDS for anyway
  uint32_t mrow;  // member cache entries (LDS)
  // output
  uint32_t *mem_pos;    // N: member static positions, cluster after cluster
  uint64_t *mkeys;      // N: (step << 32 | pos), 0 for a cluster's seed
  uint32_t *cl_centre;  // N: static position of each cluster's centre
  uint64_t *cl_off;     // N + 1
  uint64_t *out;        // [0] clusters [1] steps [2] candidates [3] error [4] members, timers
  uint64_t budget;      // longest wait for one hand-off, s_memrealtime ticks (100 MHz)
  int prof;             // controller phase timers (MC_ACCUM_PROFILE)
  uint64_t *trace;      // MC_ACCUM_PROFILE>=2: per-step timestamps, TRACE_STEPS x TRACE_W
  int trace_all;        // MC_ACCUM_PROFILE=3: every active worker marks min/max (atomics)
  uint64_t *trace2;     // MC_ACCUM_PROFILE=4 (dense form): per step < TRACE2_STEPS and worker,
                        // {record seen, scores done, partial stored} (plain stores, no contention)
  // ranks: this one's tiles are t = lt * W + rank; mbox (host memory, device-mapped) non-null
  // when the ranks' kernels exchange every step, slot_g granules per rank slot
  uint32_t W, rank;
  uint64_t *mbox;
  uint64_t slot_g;
};

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

// 16-byte load that bypasses the CU's L1 (`nt`): the compacted row copies are rewritten by the
// same workgroup between steps, and L2 has the fresh bytes
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt16(const uint4 *p) {
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t *>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// LDS reads through LDS-typed pointers.  Where a value comes from the controller's LDS cache or
// from global memory (cached ? LDS : global), the compiler otherwise merges the two loads into
// ONE flat load through a select of the pointers -- and a flat load waits on every outstanding
// vector memory operation (s_waitcnt vmcnt(0) lgkmcnt(0)): the step record's stores included
// (0.7 us of each config-B step, the record's second word waited for its first to land).
#define MC_LDS __attribute__((address_space(3)))
#define MC_GLB __attribute__((address_space(1)))
__device__ __forceinline__ uint32_t lds_u32(const uint32_t *p) { return *(const MC_LDS uint32_t *)p; }
__device__ __forceinline__ uint64_t lds_u64(const uint64_t *p) { return *(const MC_LDS uint64_t *)p; }
__device__ __forceinline__ uint4 lds_u4(const uint4 *p) {
  const u32x4_t v = *(const MC_LDS u32x4_t *)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void glb_st16(MC_GLB u32x4_t *p, const uint4 &v) { *p = (u32x4_t){v.x, v.y, v.z, v.w}; }
__device__ __forceinline__ void lds_st16(MC_LDS u32x4_t *p, const uint4 &v) { *p = (u32x4_t){v.x, v.y, v.z, v.w}; }
__device__ __forceinline__ uint4 lds_ld16(const MC_LDS u32x4_t *p) {
  const u32x4_t v = *p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ WinTab lds_wt(const WinTab *p) {
  static_assert(sizeof(WinTab) == 40, "WinTab is read as five 8-byte words");
  const MC_LDS uint64_t *q = (const MC_LDS uint64_t *)p;
  uint64_t w[5];
#pragma unroll
  for (int i = 0; i < 5; i++) w[i] = q[i];
  WinTab r;
  __builtin_memcpy(&r, w, sizeof(WinTab));
  return r;
}

// Step trace (MC_ACCUM_PROFILE=2/3), words per step: 0 record published, 7 controller has
// every partial, 8 collect done, 9 active workers; =3: 1/2 first/last worker saw it, 3/4
// first/last scan done, 5/6 first/last partial stored (minima kept as maxima of ~t); =2: the
// middle active worker alone (plain stores) 10 saw it, 11 kill log applied, 12 wave 0 scanned,
// 13 every wave scanned + reduced, 14 partial stored.
__device__ __forceinline__ void trace_mark(const AccArgs &A, uint32_t step, int slot, uint64_t t) {
  if (!A.trace || !A.trace_all || step >= TRACE_STEPS) return;
  uint64_t *w = A.trace + (uint64_t)step * TRACE_W;
  atomicMax((unsigned long long *)&w[slot], (unsigned long long)~t);
  atomicMax((unsigned long long *)&w[slot + 1], (unsigned long long)t);
}
__device__ __forceinline__ bool timed_out(const AccArgs &A, uint64_t t0) { return now() - t0 > A.budget; }

// Hand-off primitives: relaxed agent-scope atomics lower to global loads / stores with sc1
// (L1 bypassed, coherent across XCDs); the drain is inline asm so the compiler keeps it.
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
// the mailbox: host memory shared by every rank's GPU -- system-scope granules
__device__ __forceinline__ void st64x(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld64x(const uint64_t *p) {
  return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// this rank's tiles of global tiles [c0, c1]: local tiles [*lt0, *lt1] (global = lt * W + rank)
__device__ __forceinline__ bool rank_tiles(uint64_t c0, uint64_t c1, uint32_t W, uint32_t r, uint64_t *lt0,
                                           uint64_t *lt1) {
  if (W == 1) {
    *lt0 = c0;
    *lt1 = c1;
    return true;
  }
  if (c1 < r) return false;
  const uint64_t a = c0 <= r ? 0 : (c0 - r + W - 1) / W, b = (c1 - r) / W;
  *lt0 = a;
  *lt1 = b;
  return a <= b;
}
__device__ __forceinline__ uint64_t gran(uint32_t tag, uint32_t data) { return ((uint64_t)tag << 32) | data; }

__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) { return wave_sum32_all(v); }

// n / d and n % d for a run-time divisor d (the worker count) and n < 2^22 (chunk indices):
// float reciprocal, then one correction either way (|error| < 0.5 before truncation), instead
// of the compiler's 64-bit division sequence.
struct Div32 {
  uint32_t d;
  float inv;
  __device__ __forceinline__ explicit Div32(uint32_t d_) : d(d_), inv(1.0f / (float)d_) {}
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    uint32_t q = (uint32_t)((float)n * inv);
    const int32_t r = (int32_t)(n - q * d);
    if (r < 0) q--;
    else if ((uint32_t)r >= d) q++;
    return q;
  }
  __device__ __forceinline__ uint32_t mod(uint32_t n) const { return n - div(n) * d; }
};

__device__ __forceinline__ bool better(double v, uint64_t p, double bv, uint64_t bp) {
  return v > bv || (v == bv && p < bp);
}

// The bvec held by the controller workgroup: bitmap of alive static positions (LDS or
// global), per-bin alive counts with a Fenwick tree over them, bin starts and begin bounds
// (bvec.cpp's bins after insert_finalize).  Queries are answered by each wave on its own;
// callers keep queries uniform and put a barrier between kills and the next query.  The
// closed forms are checked against the host bvec in tests/native/bvec_check.cpp.
struct DevBvec {
  uint32_t *gbits;        // the bitmap in global memory (gb), else null
  MC_LDS uint32_t *bits;  // ... in LDS (!gb)
  bool gb;  // bits in global memory: sc1 loads (the atomics that clear bits act in L2)
  uint32_t *cn;
  uint32_t *fw;
  const uint32_t *lo;
  const uint64_t *bnd;
  const uint64_t *plen;  // global: length by static position
  uint64_t nb, lg;
  WinTab h{~0ull, ~0ull, ~0u, ~0u, 0, 0, 0, 0};

  __device__ uint64_t nbins() const { return nb; }
  __device__ uint32_t word(uint64_t w) const { return gb ? ld32(gbits + w) : bits[w]; }
  __device__ __forceinline__ void clear_bit(uint64_t p) {
    if (gb) atomicAnd(&gbits[p >> 5], ~(1u << (p & 31)));
    else __hip_atomic_fetch_and(&bits[p >> 5], ~(1u << (p & 31)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __device__ uint64_t cnt(uint64_t b) { return b < nb ? cn[b] : 0; }
  __device__ void index_of(uint64_t point, uint64_t *plow, uint64_t *phigh) {
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
    uint32_t x = word(w);
    const uint64_t s = w << 5;
    if (s < p0) x &= ~0u << (p0 - s);
    if (s + 32 > p1) x &= (p1 - s) >= 32 ? ~0u : ((1u << (p1 - s)) - 1u);
    return x;
  }
  __device__ uint64_t alive_in(uint64_t p0, uint64_t p1) const {  // alive positions in [p0, p1)
    if (p0 >= p1) return 0;
    const uint64_t w0 = p0 >> 5, w1 = (p1 + 31) >> 5;
    uint32_t n = 0;
    for (uint64_t w = w0 + (threadIdx.x & 63); w < w1; w += 64) n += (uint32_t)__popc(masked_word(w, p0, p1));
    return wave_sum32(n);
  }
  // first / last alive position of [p, q) (one wave, uniform result), ~0 if none
  __device__ uint64_t next_alive(uint64_t p, uint64_t q) const {
    const int lane = threadIdx.x & 63;
    for (uint64_t base = p >> 5; p < q && (base << 5) < q; base += 64) {
      const uint64_t w = base + (uint64_t)lane;
      const uint32_t x = (w << 5) < q ? masked_word(w, p, q) : 0u;
      const uint64_t bal = __ballot(x != 0);
      if (bal) {
        const int L = __builtin_ctzll(bal);
        const uint32_t y = (uint32_t)__builtin_amdgcn_readlane((int)x, L);
        return ((base + (uint64_t)L) << 5) + (uint64_t)__builtin_ctz(y);
      }
    }
    return NONE64;
  }
  // first alive position of bin b (b < 0: none) -- with first_nonempty / last_nonempty, the
  // position bvec::inner_index_of's empty-bin branch makes the window's front / back
  __device__ uint64_t first_alive_of(int64_t b) const { return b < 0 ? NONE64 : next_alive(lo[b], lo[b + 1]); }
  __device__ uint64_t prev_alive(uint64_t p, uint64_t q) const {
    if (p >= q) return NONE64;
    const int lane = threadIdx.x & 63;
    const int64_t wfirst = (int64_t)(p >> 5);
    for (int64_t top = (int64_t)((q - 1) >> 5); top >= wfirst; top -= 64) {
      const int64_t w = top - lane;
      const uint32_t x = w >= wfirst ? masked_word((uint64_t)w, p, q) : 0u;
      const uint64_t bal = __ballot(x != 0);
      if (bal) {
        const int L = __builtin_ctzll(bal);  // lowest lane = highest word
        const uint32_t y = (uint32_t)__builtin_amdgcn_readlane((int)x, L);
        return ((uint64_t)(top - L) << 5) + (uint64_t)(31 - __builtin_clz(y));
      }
    }
    return NONE64;
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
      const uint32_t x = w < w1 ? masked_word(w, p0, p1) : 0u;
      const uint32_t pc = (uint32_t)__popc(x);
      uint32_t inc = pc;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = (uint32_t)__shfl_up((int)inc, o, 64);
        if (lane >= o) inc += u;
      }
      const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
      if (c < tot) {
        const uint64_t hit = __ballot(inc > c);
        const int L = __builtin_ctzll(hit);
        uint32_t y = (uint32_t)__builtin_amdgcn_readlane((int)x, L);
        const uint32_t before = (uint32_t)__builtin_amdgcn_readlane((int)(inc - pc), L);
        for (uint64_t k = c - before; k > 0; k--) y &= y - 1;
        return ((base + (uint64_t)L) << 5) + (uint64_t)__builtin_ctz(y);
      }
      c -= tot;
    }
    return NONE64;
  }
  __device__ uint64_t bin_of(uint64_t p) const {  // single-thread binary search
    uint64_t a = 0, z = nb;                        // lo[a] <= p < lo[z]
    while (z - a > 1) {
      const uint64_t m = (a + z) / 2;
      if (lo[m] <= p) a = m;
      else z = m;
    }
    return a;
  }
  // kill one static position (bvec::pop / erase / remove_available); any thread, atomics
  __device__ __forceinline__ void kill_one(uint64_t p) { kill_in(p, bin_of(p)); }
  __device__ __forceinline__ void kill_in(uint64_t p, uint64_t b) {  // ... when its bin b is known
    clear_bit(p);
    count_sub(b, 1u);
  }
  __device__ __forceinline__ void count_sub(uint64_t b, uint32_t n) {  // n kills in bin b: counts only
    atomicSub(&cn[b], n);
    for (uint64_t i = b + 1; i <= nb; i += i & (~i + 1)) atomicSub(&fw[i], n);
  }
  // kills of a list (every thread of the workgroup; p / b valid where `act`): the bits one
  // atomic each, the counts once per distinct bin of each wave (a step's new members share a
  // few bins: per-member Fenwick walks were same-address LDS atomics in series)
  __device__ __forceinline__ void kill_list(bool act, uint64_t p, uint64_t b) {
    if (act) clear_bit(p);
    uint64_t pending = __ballot(act);
    while (pending) {
      const int L = __builtin_ctzll(pending);
      const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, L);
      const uint64_t same = __ballot(act && (uint32_t)b == b0) & pending;
      if ((int)(threadIdx.x & 63) == L) count_sub(b0, (uint32_t)__popcll(same));
      pending &= ~same;
    }
  }
};

// The controller's cache of the current cluster's first members (LDS)
struct MemberCache {
  uint32_t *pos;
  uint64_t *key;
  uint64_t *info;  // 3 per entry: mag, sumsq, len
  WinTab *wt;
  uint4 *row;      // rp chunks per entry (nch + 1: the pad spreads rows over the LDS banks)
  int rp;
};

// One candidate against the centre held in LDS (feat->compute(*pt, *p) of get_close):
// returns the decision, *cv = combo 0.
template <typename T>
__device__ __forceinline__ int classify_cand(const Acc<T> &acc, const PInfo &pi, const PInfo &pc, int B,
                                             const DevClassifier &C, double *cv) {
  const PS s = acc.finish(pi.mag, pc.mag);
  if (C.layout) return classify_std(C, s, pi, pterms(pi.mag, pi.sumsq, B), pc, pterms(pc.mag, pc.sumsq, B), B, cv);
  double raw[MC_MAX_SINGLE];
#pragma unroll
  for (int i = 0; i < MC_MAX_SINGLE; i++) raw[i] = i < C.c.n_single ? raw_fast(C.c.lookup[i], s, pi, pc, B) : 0.0;
  return classify_raw(C, raw, cv, nullptr);
}

// ============================================================================================
// Workers (WG 1 .. G-1): chunk c of the static order belongs to worker c mod (G - 1).  With
// A.res > 0 the rows of a worker's chunks are loaded into its LDS once (chunk-major, so lane t
// reads row t's chunks conflict-free) and never read from memory again.
// LDS: record words | alive flags (fcap) | resident rows (res * nch * NT uint4)
// ============================================================================================
template <typename T, int NCH, bool WIDE, bool CPT, bool PROF>
__device__ __forceinline__ void worker(const AccArgs &A, const DevClassifier &C, uint4 *dyn) {
  // profiling state only in the PROF instantiation (MC_ACCUM_PROFILE): the production kernel
  // carries no timer registers
  [[maybe_unused]] const bool prof_on = PROF && A.prof;
  [[maybe_unused]] uint64_t *const trace = PROF ? A.trace : nullptr;
  [[maybe_unused]] uint64_t *const trace2 = PROF ? A.trace2 : nullptr;
  __shared__ double s_bv[NW];
  __shared__ uint64_t s_bp[NW];
  __shared__ uint32_t s_nfl, s_nscan, s_go, s_inl[INL], s_nfl_w[NW];
  __shared__ int s_abort;
  constexpr int NC = NCH > 0 ? NCH : 1;
  const uint32_t GW = gridDim.x - 1, w = blockIdx.x - 1;
  const Div32 dgw(GW);
  const int lane = threadIdx.x & 63, wv = wave_id();
  const int nch = NCH > 0 ? NCH : A.nch;
  const int rec_words = (int)A.rec_g;
  constexpr uint32_t TS = WIDE ? (uint32_t)NW : (uint32_t)NT;  // positions per owned tile
  uint32_t *srec = reinterpret_cast<uint32_t *>(dyn);
  // centre row: record words 0 .. 4 nch, or (wide rows) loaded from `hr` after the record
  uint4 *lcen = dyn + (rec_words + 3) / 4;
  const uint4 *clds = WIDE ? lcen : dyn;
  uint8_t *lal = reinterpret_cast<uint8_t *>(lcen + (WIDE ? nch : 0));
  uint4 *lrow = reinterpret_cast<uint4 *>(lal + (A.fcap + 15) / 16 * 16);
  // streaming with compaction (A.cc): per local chunk, its compacted entries' slots (lrow's place)
  uint16_t *clist = reinterpret_cast<uint16_t *>(lrow);
  __shared__ uint32_t s_ccnt[64], s_alive;  // (fcap / NT <= 64 chunks per worker when A.cc)
  // alive flags of the positions this worker owns (tiles w, w + GW, ...), local index
  // (tile / GW) * TS + offset: flagged candidates are cleared by their owner thread, and so
  // are the controller's pops and erases, which arrive with the step records
  for (uint64_t i = threadIdx.x; i < A.fcap; i += NT) lal[i] = 1;
  if (CPT) {
    for (uint64_t i = threadIdx.x; i < A.fcap; i += NT) clist[i] = (uint16_t)(i % NT);
    for (uint64_t i = threadIdx.x; i < A.fcap / NT; i += NT) s_ccnt[i] = NT | 0x80000000u;  // (bit 31: rows still in hs)
  }
  const int res = A.res;
  // resident chunks' per-candidate data (res <= 2 kept in registers; fixed indices only, so
  // nothing is spilled to scratch)
  PInfo rinf0{0, 0, 0}, rinf1{0, 0, 0};
  PTerms rterm0{0, 0, 0.0}, rterm1{0, 0, 0.0};
  for (int i = 0; i < res; i++) {
    const uint64_t pos = (((uint64_t)w + (uint64_t)i * GW) * A.W + A.rank) * NT + threadIdx.x;
    for (int k = 0; k < nch; k++)
      lrow[((uint64_t)i * nch + k) * NT + threadIdx.x] = pos < A.N ? A.hs[(uint64_t)k * A.npad + pos] : make_uint4(0, 0, 0, 0);
    if (i < 2 && pos < A.N) {
      const PInfo pi{A.mag_s[pos], A.sumsq_s[pos], A.len_s[pos]};
      const PTerms pt = pterms(pi.mag, pi.sumsq, A.B);
      if (i == 0) {
        rinf0 = pi;
        rterm0 = pt;
      } else {
        rinf1 = pi;
        rterm1 = pt;
      }
    }
  }
  if (threadIdx.x == 0) s_abort = 0;
  __syncthreads();
  uint32_t kcur = 0, seen = 0;
  for (;;) {
    // ---- wait for the next step's record (wave 0) --------------------------------------
    if (wv == 0) {
      const uint64_t t0 = now();
      const uint32_t want = seen + 1;
      int state = 0;  // 0 waiting, 1 got it, 2 abort
      uint32_t got = want;
      // steps are published in order: poll the next step's slot itself (its granules carry
      // the step); a worker that finds the slot rewritten for a later step fell RING steps
      // behind and catches up through `go`
      bool late = false;
      const uint64_t *rn = A.ring + (uint64_t)(want % RING) * A.rec_g;
      for (uint32_t it = 1;; it++) {
        bool ok = true, ahead = false;
        for (int j = lane; j < rec_words; j += 64) {
          const uint64_t x = ld64(rn + j);
          const uint32_t t = (uint32_t)(x >> 32);
          ok &= t == want;
          ahead |= (int32_t)(t - want) > 0;
          srec[j] = (uint32_t)x;
        }
        if (__ballot(!ok) == 0) {
          state = 1;
          break;
        }
        if (__ballot(ahead) != 0) {
          late = true;
          break;
        }
        if ((it & 255) == 0 && timed_out(A, t0)) {
          state = 2;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      while (late && state == 0) {
        uint32_t v = 0;
        if (lane == 0) {
          for (uint32_t it = 1; (v = ld32(A.go)) == seen; it++) {
            if ((it & 255) == 0 && timed_out(A, t0)) break;
            __builtin_amdgcn_s_sleep(1);
          }
        }
        v = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
        if (v == seen) {
          state = 2;
          break;
        }
        const uint64_t *r = A.ring + (uint64_t)(v % RING) * A.rec_g;
        bool ok = true;
        for (int j = lane; j < rec_words; j += 64) {
          const uint64_t x = ld64(r + j);
          ok &= (uint32_t)(x >> 32) == v;
          srec[j] = (uint32_t)x;
        }
        if (__ballot(!ok) == 0) {
          state = 1;
          got = v;
        }
        // else: that slot is being rewritten for a later step: read `go` again
      }
      if (lane == 0) {
        if (state == 2) s_abort = 1;
        s_go = got;
      }
    }
    __syncthreads();
    if (s_abort) {
      if (threadIdx.x == 0) atomicMax((unsigned long long *)&A.out[3], 99ull);
      return;
    }
    seen = s_go;
    uint64_t t_seen = 0;
    if (trace && threadIdx.x == 0) t_seen = now();  // (recorded only by active workers)
    const uint32_t *hdr = srec + (WIDE ? 0 : 4 * nch);
    if (hdr[0] == NONE) return;  // accumulation finished
    const uint64_t P_S = hdr[1], P_E = hdr[2];
    const uint32_t kend = hdr[3] & 0x7fffffffu;  // (bit 31: the dense form's exact-span flag)
    const PInfo pc{(uint64_t)hdr[4 + KINL] | ((uint64_t)hdr[5 + KINL] << 32),
                   (uint64_t)hdr[6 + KINL] | ((uint64_t)hdr[7 + KINL] << 32),
                   (uint64_t)hdr[8 + KINL] | ((uint64_t)hdr[9 + KINL] << 32)};
    const PTerms tq = pterms(pc.mag, pc.sumsq, A.B);  // the centre's pair-independent terms
    // the controller's kills since the last record applied here: each thread clears the
    // flags of the positions it owns (offset = its thread index), so no barrier is needed
    {
      const uint32_t kinl0 = kend > (uint32_t)KINL ? kend - KINL : 0;
      const uint64_t t0k = kinl0 > kcur ? now() : 0;
      for (uint32_t e = kcur; e < kend; e++) {
        uint32_t p;
        if (e >= kinl0) {
          p = hdr[4 + KINL - (kend - e)];
        } else {  // older than the record's inline entries: the tagged log entry
          uint64_t g = ld64(A.klog + e);
          for (uint32_t it = 1; (uint32_t)(g >> 32) != e + 1; it++) {
            if ((it & 255) == 0 && timed_out(A, t0k)) {
              s_abort = 1;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
            g = ld64(A.klog + e);
          }
          p = (uint32_t)g;
        }
        const uint64_t ch = p / TS;
        if ((p % TS) == (uint32_t)threadIdx.x && (A.W == 1 || ch % A.W == A.rank)) {
          const uint32_t lt = (uint32_t)(A.W == 1 ? ch : ch / A.W);
          const uint32_t cq = dgw.div(lt);
          if (lt - cq * GW == w) lal[(uint64_t)cq * TS + threadIdx.x] = 0;
        }
      }
      kcur = kend;
    }
    uint64_t t_klog = 0, t_sad = 0, t_top = 0;
    if (trace && threadIdx.x == 0) t_klog = now();
    // ---- the chunks of the window this worker owns: Trainer::get_close ----------------
    uint64_t c0, c1;  // this rank's (local) tiles of the window
    if (!rank_tiles(P_S / TS, P_E / TS, A.W, A.rank, &c0, &c1)) continue;
    const uint32_t nact = (uint32_t)(c1 - c0 + 1 < (uint64_t)GW ? c1 - c0 + 1 : (uint64_t)GW);
    const uint32_t mine = dgw.mod(w + GW - dgw.mod((uint32_t)c0));
    if (mine >= nact) continue;
    if (threadIdx.x == 0) {
      s_nfl = 0;
      s_nscan = 0;
    }
    if constexpr (WIDE)  // the centre's row (read-only static copy) for this step's tiles
      for (int c = threadIdx.x; c < nch; c += NT) lcen[c] = A.hr[(uint64_t)hdr[0] * nch + c];
    uint64_t t_w7 = 0, t_bar = 0;
    if (trace && threadIdx.x == NT - 64) t_w7 = now();  // (profile: the last wave reaches the barrier)
    __syncthreads();
    if (trace && (threadIdx.x == 0 || threadIdx.x == NT - 64)) t_bar = now();
    double best_v = -1.0;
    uint64_t best_p = NONE64;
    uint32_t nscan = 0;
    const uint64_t base = (uint64_t)w * A.fcap;
    // a flagged candidate: its position goes inline into the partial (the first INL) or to
    // this worker's list; the controller reads rows and magnitudes itself (read-only data)
    auto flag_pos = [&](uint64_t pos) {
      const uint32_t idx = atomicAdd(&s_nfl, 1u);
      if (idx < (uint32_t)INL) s_inl[idx] = (uint32_t)pos;
      else st32(A.fpos + base + idx, (uint32_t)pos);
    };
    if constexpr (WIDE) {
      // one candidate per wave: lanes take chunks lane, lane + 64, ... of its row (coalesced
      // 1 KiB loads), four loads in flight, sums reduced over the wave; every lane then holds
      // the same statistics and runs the same classifier
      for (uint64_t ch = c0 + mine; ch <= c1; ch += GW) {
        const uint64_t li = dgw.div((uint32_t)ch);
        const uint64_t pos = (ch * A.W + A.rank) * TS + (uint64_t)wv;
        uint8_t *la = lal + li * TS + wv;
        if (!(pos >= P_S && pos <= P_E && *la)) continue;
        if (lane == 0) nscan++;
        const uint4 *row = A.hr + pos * (uint64_t)nch;
        Acc<T> acc;
        int c = lane;
        for (; c + 192 < nch; c += 256) {
          const uint4 v0 = row[c], v1 = row[c + 64], v2 = row[c + 128], v3 = row[c + 192];
          acc.add(v0, clds[c]);
          acc.add(v1, clds[c + 64]);
          acc.add(v2, clds[c + 128]);
          acc.add(v3, clds[c + 192]);
        }
        for (; c < nch; c += 64) acc.add(row[c], clds[c]);
        acc.wave_reduce();
        const PInfo pi{A.mag_s[pos], A.sumsq_s[pos], A.len_s[pos]};
        double cv;
        if (classify_cand<T>(acc, pi, pc, A.B, C, &cv) && lane == 0) {
          *la = 0;
          flag_pos(pos);
        }
        if (cv > -1.0 && better(cv, pos, best_v, best_p)) {
          best_v = cv;
          best_p = pos;
        }
      }
    } else if constexpr (CPT) {
      // streaming with compaction: a chunk's rows stream from HBM every step, and once half of
      // its listed entries are dead the worker rewrites the alive rows densely (A.cc, entry
      // order = slot order) -- the loads of dead neighbours' cache lines went with them
      // (config D: 1.8x the algorithmic bytes fetched without this, profiles/r03_v4)
      for (uint64_t ch = c0 + mine; ch <= c1; ch += GW) {
        const uint32_t li = dgw.div((uint32_t)ch);
        const uint64_t cbase = (ch * A.W + A.rank) * NT;
        uint4 *creg = A.cc + ch * (uint64_t)NC * NT;  // (local chunk ch: its region of cc)
        const uint32_t cw = s_ccnt[li];
        const bool in_hs = (cw >> 31) != 0;
        const uint32_t n = cw & 0xffffu;
        const uint32_t t = threadIdx.x;
        const uint32_t slot = t < n ? (uint32_t)clist[(uint64_t)li * NT + t] : 0u;
        const bool alive = t < n && lal[(uint64_t)li * NT + slot];
        // rebuild when fewer than half of the listed entries are alive (one WG-uniform decision)
        if (t == 0) s_alive = 0;
        __syncthreads();
        {
          const uint32_t c = wave_sum32(alive ? 1u : 0u);
          if (lane == 0 && c) atomicAdd(&s_alive, c);
        }
        __syncthreads();
        const uint32_t nal = s_alive;
        uint32_t e = t;  // this lane's entry after the (possible) rebuild
        bool mine_alive = alive;
        uint32_t myslot = slot;
        if (nal * 2 < n && n > 64) {
          // rank of this alive entry among the alive ones (entry order = slot order)
          const uint64_t bal = __ballot(alive);
          const uint32_t below = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
          if (lane == 0) s_nfl_w[wv] = (uint32_t)__popcll(bal);
          uint4 row[NC];
          if (alive) {
#pragma unroll
            for (int k = 0; k < NC; k++)
              row[k] = in_hs ? A.hs[(uint64_t)k * A.npad + cbase + slot] : ld_nt16(creg + (uint64_t)k * NT + t);
          }
          __syncthreads();  // every read of the old entries before any write
          uint32_t r = below;
          for (int i = 0; i < wv; i++) r += s_nfl_w[i];
          if (alive) {
#pragma unroll
            for (int k = 0; k < NC; k++) creg[(uint64_t)k * NT + r] = row[k];
            clist[(uint64_t)li * NT + r] = (uint16_t)slot;
          }
          e = alive ? r : NT;  // (dead lanes hold no entry now)
          if (t == 0) s_ccnt[li] = nal;
          __syncthreads();
          mine_alive = alive;
          myslot = slot;
        }
        (void)e;
        const uint32_t cw2 = s_ccnt[li];
        const bool from_hs = (cw2 >> 31) != 0;
        const uint32_t n2 = cw2 & 0xffffu;
        // scan: lane t takes entry t of the (possibly rebuilt) list
        {
          const bool rebuilt = (cw2 != cw);
          const uint32_t sl = rebuilt ? (t < n2 ? (uint32_t)clist[(uint64_t)li * NT + t] : 0u) : myslot;
          const bool al = rebuilt ? (t < n2) : mine_alive;
          const uint64_t pos = cbase + sl;
          if (al && pos >= P_S && pos <= P_E && lal[(uint64_t)li * NT + sl]) {
            nscan++;
            uint4 v[NC];
#pragma unroll
            for (int k = 0; k < NC; k++)
              v[k] = from_hs ? A.hs[(uint64_t)k * A.npad + pos] : ld_nt16(creg + (uint64_t)k * NT + t);
            const PInfo pi{A.mag_s[pos], A.sumsq_s[pos], A.len_s[pos]};
            Acc<T> acc;
            double cv;
#pragma unroll
            for (int k = 0; k < NC; k++) acc.add(v[k], clds[k]);
            if (classify_cand<T>(acc, pi, pc, A.B, C, &cv)) {
              lal[(uint64_t)li * NT + sl] = 0;
              flag_pos(pos);
            }
            if (cv > -1.0 && better(cv, pos, best_v, best_p)) {
              best_v = cv;
              best_p = pos;
            }
          }
        }
      }
    } else
    for (uint64_t ch = c0 + mine; ch <= c1; ch += GW) {
      const uint64_t li = dgw.div((uint32_t)ch);  // local chunk index
      const uint64_t pos = (ch * A.W + A.rank) * NT + threadIdx.x;
      uint8_t *la = lal + li * NT + threadIdx.x;
      if (!(pos >= P_S && pos <= P_E && *la)) continue;
      nscan++;
      if (trace && threadIdx.x == 0) t_top = now();
      Acc<T> acc;
      double cv;
      if ((int64_t)li < res) {  // resident rows (LDS)
        const uint4 *rr = lrow + li * (uint64_t)nch * NT + threadIdx.x;
        if constexpr (NCH > 0) {
          // every LDS read of a half row in flight before the first use (one wait per half,
          // not one LDS round trip per chunk)
          constexpr int HB = NC >= 8 ? 8 : NC;
#pragma unroll
          for (int k0 = 0; k0 < NC; k0 += HB) {
            uint4 rv[HB], cvv[HB];
#pragma unroll
            for (int k = 0; k < HB; k++) {
              rv[k] = rr[(uint64_t)(k0 + k) * NT];
              cvv[k] = clds[k0 + k];
            }
#pragma unroll
            for (int k = 0; k < HB; k++) acc.add(rv[k], cvv[k]);
          }
        } else {
          for (int k = 0; k < nch; k++) acc.add(rr[(uint64_t)k * NT], clds[k]);
        }
        if constexpr (sizeof(T) == 1)
          if (trace && threadIdx.x == 0) {  // (profile: the byte sums are done)
            acc.fold();
            asm volatile("" ::"v"(acc.sad), "v"(acc.dot));
            t_sad = now();
          }
        int d;
        if (li < 2 && C.layout) {
          const PInfo pi = li == 0 ? rinf0 : rinf1;
          d = classify_std(C, acc.finish(pi.mag, pc.mag), pi, li == 0 ? rterm0 : rterm1, pc, tq, A.B, &cv);
#ifdef MC_EXP_DOUBLE_CLASSIFY  // timing experiment: the classifier's cost, run twice
          {
            double cv2;
            PInfo p2 = pi;
            const uint64_t z = (uint64_t)(A.budget >> 62);  // 0 at run time, unknown to the compiler
            p2.len += z;
            p2.mag += z;
            p2.sumsq += z;
            const int d2 = classify_std(C, acc.finish(p2.mag, pc.mag), p2, pterms(p2.mag, p2.sumsq, A.B), pc, tq, A.B, &cv2);
            d &= d2 | (cv2 == cv ? 1 : 0);
            cv = cv2 > cv ? cv2 : cv;
          }
#endif
        } else {
          const PInfo pi = li == 0 ? rinf0 : li == 1 ? rinf1 : PInfo{A.mag_s[pos], A.sumsq_s[pos], A.len_s[pos]};
          d = classify_cand<T>(acc, pi, pc, A.B, C, &cv);
        }
        if (d) {
          *la = 0;
          flag_pos(pos);
        }
      } else {  // streaming: the rows come from memory
        const uint4 *col = A.hs + pos;
        if constexpr (NCH > 0) {
          uint4 v[NC];
#pragma unroll
          for (int k = 0; k < NC; k++) v[k] = col[(uint64_t)k * A.npad];
          const PInfo pi{A.mag_s[pos], A.sumsq_s[pos], A.len_s[pos]};
#pragma unroll
          for (int k = 0; k < NC; k++) acc.add(v[k], clds[k]);
          if (classify_cand<T>(acc, pi, pc, A.B, C, &cv)) {
            *la = 0;
            flag_pos(pos);
          }
        } else {
#pragma unroll 8
          for (int k = 0; k < nch; k++) acc.add(col[(uint64_t)k * A.npad], clds[k]);
          const PInfo pi{A.mag_s[pos], A.sumsq_s[pos], A.len_s[pos]};
          if (classify_cand<T>(acc, pi, pc, A.B, C, &cv)) {
            *la = 0;
            flag_pos(pos);
          }
        }
      }
      if (cv > -1.0 && better(cv, pos, best_v, best_p)) {
        best_v = cv;
        best_p = pos;
      }
    }
    uint64_t t_scanned = 0;
    if (trace && threadIdx.x == 0) t_scanned = now();
    // first maximum of this worker; scanned count
    wave_best_all(best_v, best_p, better);
    nscan = wave_sum32(nscan);
    if (lane == 0) {
      s_bv[wv] = best_v;
      s_bp[wv] = best_p;
      atomicAdd(&s_nscan, nscan);
    }
    drain();  // this wave's flagged-list stores are complete before the partial announces them
    __syncthreads();
    if (trace && !A.trace_all && threadIdx.x == 0 && mine == nact / 2 && seen < TRACE_STEPS) {
      uint64_t *tr = trace + (uint64_t)seen * TRACE_W;
      tr[10] = t_seen;
      tr[11] = t_klog;
      tr[12] = t_scanned;
      tr[15] = t_sad;
      tr[16] = t_top;
      tr[18] = t_bar;
      tr[13] = now();
    }
    if (trace && !A.trace_all && threadIdx.x == NT - 64 && mine == nact / 2 && seen < TRACE_STEPS) {
      trace[(uint64_t)seen * TRACE_W + 17] = t_w7;
      trace[(uint64_t)seen * TRACE_W + 19] = t_bar;
    }
    if (threadIdx.x < PART_G) {  // lane j of wave 0 stores granule j
      double v = s_bv[0];
      uint64_t p = s_bp[0];
      for (int i = 1; i < NW; i++)
        if (better(s_bv[i], s_bp[i], v, p)) {
          v = s_bv[i];
          p = s_bp[i];
        }
      const uint64_t vb = (uint64_t)__double_as_longlong(v);
      const int j = threadIdx.x;
      const uint32_t nfl = s_nfl;
      const uint32_t data = j == 0   ? (uint32_t)(vb >> 32)
                            : j == 1 ? (uint32_t)vb
                            : j == 2 ? (p == NONE64 ? NONE : (uint32_t)p)
                            : j == 3 ? nfl
                            : j == 4 ? s_nscan
                                     : ((uint32_t)(j - 5) < nfl ? s_inl[j - 5] : NONE);
      st64(A.partials + (uint64_t)w * PART_G + j, gran(seen, data));
      if (trace && !A.trace_all && j == 0 && mine == nact / 2 && seen < TRACE_STEPS)
        trace[(uint64_t)seen * TRACE_W + 14] = now();
      if (trace && A.trace_all && j == 0) {
        const uint64_t t = now();
        trace_mark(A, seen, 1, t_seen);
        trace_mark(A, seen, 3, t_scanned);
        trace_mark(A, seen, 5, t);
      }
    }
  }
}

// ============================================================================================
// Dense resident workers (narrow rows, at most NT candidates per worker).  Tiles of DT static
// positions are dealt round-robin over the workers (tile t -> worker t mod GW), so a window
// spreads over all of them instead of the one or two hundred that own its 512-position
// chunks.  A worker keeps its alive candidates DENSE -- entry e is thread e, its row is LDS row
// e (chunk-major: lane e reads row e conflict-free), entries sorted by static position -- and
// compacts them after every step in which some died (flagged, or popped / erased by the
// controller), while the controller collects: a step runs ceil(alive / 64) waves, not eight.
// Per-entry magnitudes and pair-independent terms live in the entry's thread's registers.
// LDS: record words | rows (nch * NT uint4) | entry positions (NT u32, compaction staging)
// ============================================================================================
constexpr int DT = 64;
constexpr int DMAXCH = 16;  // chunks per row the dense form takes (a row per thread in registers while compacting)

// A thin record (the controller's publish_thin): the new seed's row and magnitudes from the
// static copies into the record's LDS copy, by the workgroup (the controller published the record
// before it had loaded them itself).  Ends with a barrier.
__device__ __forceinline__ void load_thin_record(const AccArgs &A, uint32_t *srec, int nch, uint64_t cp) {
  const uint32_t t = threadIdx.x;
  uint4 rv = make_uint4(0, 0, 0, 0);
  uint64_t mv = 0;
  if (t < (uint32_t)nch) rv = A.hr[cp * nch + t];
  else if (t >= 64 && t < 67) mv = t == 64 ? A.mag_s[cp] : t == 65 ? A.sumsq_s[cp] : A.len_s[cp];
  if (t < (uint32_t)nch) reinterpret_cast<uint4 *>(srec)[t] = rv;
  else if (t >= 64 && t < 67) {
    srec[4 * nch + 4 + KINL + 2 * (t - 64)] = (uint32_t)mv;
    srec[4 * nch + 5 + KINL + 2 * (t - 64)] = (uint32_t)(mv >> 32);
  }
  __syncthreads();
}

template <typename T, int NCH, bool PROF>
__device__ __forceinline__ void worker_dense(const AccArgs &A, const DevClassifier &C, uint4 *dyn) {
  // profiling state only in the PROF instantiation (MC_ACCUM_PROFILE): the production kernel
  // carries no timer registers
  [[maybe_unused]] const bool prof_on = PROF && A.prof;
  [[maybe_unused]] uint64_t *const trace = PROF ? A.trace : nullptr;
  [[maybe_unused]] uint64_t *const trace2 = PROF ? A.trace2 : nullptr;
  __shared__ double s_bv[NW];
  __shared__ uint64_t s_bp[NW];
  __shared__ uint32_t s_nfl, s_go, s_inl[INL], s_wc[NW];
  __shared__ int s_abort;
  __shared__ uint64_t s_b[2];  // spec: part B of the step, {tag << 32 | S}, {tag << 32 | E}
  __shared__ uint64_t s_tw[NW];  // MC_ACCUM_PROFILE=4: each wave's scores-done time
  __shared__ uint64_t s_t0[3];   // ... thread 0's record-seen, scores-done and part-B times
  __shared__ uint32_t s_arr;     // waves that have reduced this step's scores
  __shared__ uint32_t s_rgot;    // the step whose record a polling wave has written to srec
  __shared__ SmallK s_sk;        // classify_small's constants (read with each candidate's row)
  constexpr int NC = NCH > 0 ? NCH : DMAXCH;
  constexpr int RPW = (4 * NC + REC_HDR + 63) / 64;  // record words per polling lane
  const uint32_t GW = gridDim.x - 1, w = blockIdx.x - 1;
  const Div32 dgw(GW);
  const int lane = threadIdx.x & 63, wv = wave_id();
  const uint32_t t = threadIdx.x;
  const int nch = NCH > 0 ? NCH : A.nch;
  const int rec_words = (int)A.rec_g;
  uint32_t *srec = reinterpret_cast<uint32_t *>(dyn);
  const uint4 *clds = dyn;  // the centre row: record words 0 .. 4 nch
  uint4 *lrow = dyn + (rec_words + 3) / 4;
  uint32_t *lpos = reinterpret_cast<uint32_t *>(lrow + (size_t)nch * NT);
  // entry t: this worker's (t / DT)-th tile, offset t % DT -- positions increase with t, so the
  // entries below N are a prefix
  uint32_t pos_t = 0;
  bool al_t = false;
  {
    const uint64_t lt = (uint64_t)w + (uint64_t)(t / DT) * GW;
    const uint64_t pos = (lt * A.W + A.rank) * DT + (t % DT);
    al_t = t < A.fcap && pos < A.N;
    if (al_t) {
      pos_t = (uint32_t)pos;
      for (int k = 0; k < nch; k++) lrow[(uint64_t)k * NT + t] = A.hs[(uint64_t)k * A.npad + pos];
    }
  }
  uint32_t n_ent = (uint32_t)__syncthreads_count(al_t);
  PInfo pi_t{0, 0, 0};
  PTerms pt_t{0, 0, 0.0};
  PSm ps_t{0, 0, 0, 0, false};
  if (al_t) {
    pi_t = PInfo{A.mag_s[pos_t], A.sumsq_s[pos_t], A.len_s[pos_t]};
    pt_t = pterms(pi_t.mag, pi_t.sumsq, A.B);
    ps_t = psmall(pi_t, pt_t);
  }
  // classify_small: 8-bit bins and the host's mk_div conditions (per pair: both PSm ok)
  const bool small_on = sizeof(T) == 1 && A.fc.on && A.fc.mk;
  if (t == 0) {
    s_abort = 0;
    s_b[0] = s_b[1] = 0;
    s_arr = 0;
    s_rgot = 0;
    s_sk = make_smallk(C, A.fc);
  }
  __syncthreads();
  uint32_t kcur = 0, seen = 0;
  for (;;) {
    // ---- wait for the next step's record --------------------------------------------------
    // Waves 0 .. rpoll-1 poll it, wave w starting w gaps later, so the record is seen within a
    // fraction of one poll round trip after it lands; the first wave with every granule tagged
    // writes the words to LDS and marks s_rgot (the others stop at their next check).  Wave 0
    // alone takes the path of a worker that fell RING steps behind.
    if (wv < A.rpoll) {
      const uint64_t t0 = now();
      const uint32_t want = seen + 1;
      int state = 0;
      uint32_t got = want;
      bool late = false;
      const uint64_t *rn = A.ring + (uint64_t)(want % RING) * A.rec_g;
      for (int g = 0; g < wv * A.rpoll_gap; g++) __builtin_amdgcn_s_sleep(8);
      for (uint32_t it = 1;; it++) {
        if (__hip_atomic_load(&s_rgot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == want) {
          state = 1;
          break;
        }
        bool ok = true, okh = true, ahead = false;
        uint32_t xv[RPW];
#pragma unroll
        for (int u = 0; u < RPW; u++) {
          const int j = lane + 64 * u;
          const uint64_t x = j < rec_words ? ld64(rn + j) : gran(want, 0);
          const uint32_t tg = (uint32_t)(x >> 32);
          ok &= tg == want;
          if (j >= 4 * nch) okh &= tg == want;
          ahead |= (int32_t)(tg - want) > 0;
          xv[u] = (uint32_t)x;
        }
        // a thin record (every header granule tagged, bit 30 of its kill-log word) carries no row
        if (__ballot(!ok) != 0 && __ballot(!okh) == 0) {
          const int jk = 4 * nch + 3;
          uint32_t kw = 0;
#pragma unroll
          for (int u = 0; u < RPW; u++)
            if ((jk >> 6) == u) kw = (uint32_t)__builtin_amdgcn_readlane((int)xv[u], jk & 63);
          if (kw & REC_THIN) ok = true;
        }
        if (__ballot(!ok) == 0) {
#pragma unroll
          for (int u = 0; u < RPW; u++)
            if (lane + 64 * u < rec_words) srec[lane + 64 * u] = xv[u];
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          if (lane == 0) __hip_atomic_store(&s_rgot, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          state = 1;
          break;
        }
        if (__ballot(ahead) != 0) {
          late = wv == 0;
          break;
        }
        if ((it & 255) == 0 && timed_out(A, t0)) {
          state = 2;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (wv == 0) {
      while (late && state == 0) {
        uint32_t v = 0;
        if (lane == 0) {
          for (uint32_t it = 1; (v = ld32(A.go)) == seen; it++) {
            if ((it & 255) == 0 && timed_out(A, t0)) break;
            __builtin_amdgcn_s_sleep(1);
          }
        }
        v = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
        if (v == seen) {
          state = 2;
          break;
        }
        const uint64_t *r = A.ring + (uint64_t)(v % RING) * A.rec_g;
        bool ok = true, okh = true;
        for (int j = lane; j < rec_words; j += 64) {
          const uint64_t x = ld64(r + j);
          ok &= (uint32_t)(x >> 32) == v;
          if (j >= 4 * nch) okh &= (uint32_t)(x >> 32) == v;
          srec[j] = (uint32_t)x;
        }
        if (__ballot(!ok) != 0 && __ballot(!okh) == 0 && (lds_u32(srec + 4 * nch + 3) & REC_THIN)) ok = true;
        if (__ballot(!ok) == 0) {
          state = 1;
          got = v;
        }
      }
      if (lane == 0) {
        if (state == 2) s_abort = 1;
        s_go = got;
        s_nfl = 0;
      }
      } else if (state == 2 && lane == 0) {
        s_abort = 1;
      }
    }
    __syncthreads();
    if (s_abort) {
      if (t == 0) atomicMax((unsigned long long *)&A.out[3], 99ull);
      return;
    }
    seen = s_go;
    uint64_t t_seen = 0, t_klog = 0, t_scanned = 0;
    if (trace && t == 0) t_seen = now();
    const uint32_t *hdr = srec + 4 * nch;
    if (hdr[0] == NONE) return;  // accumulation finished
    if (hdr[3] & REC_THIN) load_thin_record(A, srec, nch, hdr[0]);
    const uint64_t P_S = hdr[1], P_E = hdr[2];
    // bit 31 of the kill-log word: the record's span IS the exact window (no part B follows);
    // bit 30: a thin record
    const uint32_t kend = hdr[3] & REC_KMASK;
    const bool exact = (hdr[3] >> 31) != 0;
    const PInfo pc{(uint64_t)hdr[4 + KINL] | ((uint64_t)hdr[5 + KINL] << 32),
                   (uint64_t)hdr[6 + KINL] | ((uint64_t)hdr[7 + KINL] << 32),
                   (uint64_t)hdr[8 + KINL] | ((uint64_t)hdr[9 + KINL] << 32)};
    const PTerms tq = pterms_mk(pc.mag, pc.sumsq, A.B, A.fc.rB);
    const PSm ps_q = psmall(pc, tq);
    const double kq = (double)((int64_t)pc.mag - (int64_t)A.B * tq.ap);
    // the controller's kills since the last record: every thread compares them with its own
    // entry (one or two per step; no search, no barrier)
    {
      const uint32_t kinl0 = kend > (uint32_t)KINL ? kend - KINL : 0;
      const uint64_t t0k = kinl0 > kcur ? now() : 0;
      for (uint32_t e = kcur; e < kend; e++) {
        uint32_t p;
        if (e >= kinl0) {
          p = hdr[4 + KINL - (kend - e)];
        } else {
          uint64_t g = ld64(A.klog + e);
          for (uint32_t it = 1; (uint32_t)(g >> 32) != e + 1; it++) {
            if ((it & 255) == 0 && timed_out(A, t0k)) {
              s_abort = 1;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
            g = ld64(A.klog + e);
          }
          p = (uint32_t)g;
        }
        if (p == pos_t) al_t = false;
      }
      kcur = kend;
    }
    if (trace && t == 0) t_klog = now();
    // ---- scores of the record's span: the exact window, or (spec) a superset of it --------
    const bool comp = al_t && pos_t >= P_S && pos_t <= P_E;
    int d_t = 0;
    double cv_t = -1.0;
    if (comp) {
      Acc<T> acc;
      const uint4 *rr = lrow + t;
      constexpr int HB = NC >= 8 ? 8 : NC;
      const SmallK sk = lds_smallk(&s_sk);
      if constexpr (NCH > 0) {
#pragma unroll
        for (int k0 = 0; k0 < NC; k0 += HB) {
          uint4 rv[HB], cvv[HB];
#pragma unroll
          for (int k = 0; k < HB; k++) {
            rv[k] = rr[(uint64_t)(k0 + k) * NT];
            cvv[k] = clds[k0 + k];
          }
#pragma unroll
          for (int k = 0; k < HB; k++) acc.add(rv[k], cvv[k]);
        }
      } else {
        for (int k = 0; k < nch; k++) acc.add(rr[(uint64_t)k * NT], clds[k]);
      }
      bool und = true;
      if constexpr (sizeof(T) == 1) {
        if (small_on && ps_q.ok && ps_t.ok) {
          acc.fold();
          d_t = classify_small(sk, acc.sad, acc.dot, ps_t, ps_q, kq, pt_t.da, tq.da, A.B, &cv_t, &und);
          if (und) {
            double cx;
            d_t = classify_std(C, acc.finish(pi_t.mag, pc.mag), pi_t, pt_t, pc, tq, A.B, &cx);
            und = false;
          }
        }
      }
      if (und)
        d_t = A.fc.on    ? classify_fast(C, A.fc, acc.finish(pi_t.mag, pc.mag), pi_t, pt_t, pc, tq, A.B, &cv_t)
              : C.layout ? classify_std(C, acc.finish(pi_t.mag, pc.mag), pi_t, pt_t, pc, tq, A.B, &cv_t)
                         : classify_cand<T>(acc, pi_t, pc, A.B, C, &cv_t);
    }
    if (trace && t == 0) t_scanned = now();
    if (trace2 && lane == 0) s_tw[wv] = now();
    if (trace2 && t == 0) {
      s_t0[0] = t_seen;
      s_t0[1] = t_scanned;
      s_t0[2] = 0;
    }
    uint64_t W_S = P_S, W_E = P_E;  // the exact window
    bool abandon = false;
    uint64_t t_bgot = 0, t_red = 0;
    if (A.spec && !exact) {
      // part B: from the LDS copy once a wave has it, else polled by this wave's lanes 0 / 1.
      // (A wave that gives up marks the abort and takes the step as abandoned, so every wave
      // still reaches the one barrier below.)
      const uint64_t *rb = A.ringb + (uint64_t)(seen % RING) * 2;
      const uint64_t t0 = now();
      uint64_t b0 = 0, b1 = 0;
      for (uint32_t it = 1;; it++) {
        b0 = __hip_atomic_load(&s_b[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        b1 = __hip_atomic_load(&s_b[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if ((uint32_t)(b0 >> 32) == seen && (uint32_t)(b1 >> 32) == seen) break;
        const uint64_t g = lane < 2 ? ld64(rb + lane) : 0;
        b0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(g >> 32), 0) << 32) |
             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)g, 0);
        b1 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(g >> 32), 1) << 32) |
             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)g, 1);
        if ((uint32_t)(b0 >> 32) == seen && (uint32_t)(b1 >> 32) == seen) {
          if (lane == 0) {
            __hip_atomic_store(&s_b[0], b0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_store(&s_b[1], b1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          break;
        }
        if ((it & 255) == 0 && timed_out(A, t0)) {
          if (lane == 0) s_abort = 1;
          b0 = b1 = NONE;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (trace2 && t == 0) t_bgot = now();
      if (trace2 && t == 0) s_t0[2] = t_bgot;
      W_S = (uint32_t)b0;
      W_E = (uint32_t)b1;
      abandon = (uint32_t)W_S == NONE;
    }
    uint64_t c0 = 0, c1 = 0;
    const bool any_tile = !abandon && rank_tiles(W_S / DT, W_E / DT, A.W, A.rank, &c0, &c1);
    const uint32_t nact = any_tile ? (uint32_t)(c1 - c0 + 1 < (uint64_t)GW ? c1 - c0 + 1 : (uint64_t)GW) : 0u;
    const uint32_t mine = any_tile ? dgw.mod(w + GW - dgw.mod((uint32_t)c0)) : 0u;
    const bool active = any_tile && mine < nact;  // (uniform: every wave has the same part B)
    bool died = false;
    if (active) {
      double best_v = -1.0;
      uint64_t best_p = NONE64;
      uint32_t nscan = 0;
      bool listed = false;  // a flagged position went to this worker's list in global memory
      if (comp && pos_t >= W_S && pos_t <= W_E) {
        nscan = 1;
        if (d_t) {
          al_t = false;
          const uint32_t idx = atomicAdd(&s_nfl, 1u);
          if (idx < (uint32_t)INL) s_inl[idx] = pos_t;
          else {
            st32(A.fpos + (uint64_t)w * A.fcap + idx, pos_t);
            listed = true;
          }
        }
        if (cv_t > -1.0) {
          best_v = cv_t;
          best_p = pos_t;
        }
      }
      const uint64_t scanned = __ballot(nscan != 0);
      // the wave's first maximum: entry e is lane e % 64 of wave e / 64 and entries are in
      // static-position order, so of the lanes holding the wave's largest value the lowest one
      // holds the first maximum (a max reduction and a ballot, no (value, position) pairs moved)
      const uint64_t cands = __ballot(best_p != NONE64);
      if (cands) {  // (waves with no candidate skip it)
        const double m = wave_ext_f64_all<true>(best_v);
        const uint64_t hit = __ballot(best_p != NONE64 && best_v == m);
        const int L = __builtin_ctzll(hit);
        best_v = __builtin_bit_cast(double, readlane64(__builtin_bit_cast(uint64_t, best_v), L));
        best_p = readlane64(best_p, L);
      }
      if (lane == 0) {
        s_bv[wv] = best_v;
        s_bp[wv] = best_p;
        s_wc[wv] = (uint32_t)__popcll(scanned);
      }
      // this wave's flagged-list stores are complete before the partial announces them
      if (__ballot(listed)) drain();
      // arrival: the wave that completes the workgroup's scores combines the eight waves'
      // results and publishes the partial (no workgroup barrier on the path)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      uint32_t arr = 0;
      if (lane == 0) arr = atomicAdd(&s_arr, 1u);
      arr = (uint32_t)__builtin_amdgcn_readfirstlane((int)arr);
      if (arr == (uint32_t)NW - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (trace2 && lane == 0) t_red = now();
        if (lane < PART_G) {
          double vv[NW];
          uint64_t pp[NW];
          uint32_t ns = 0;
#pragma unroll
          for (int i = 0; i < NW; i++) {
            vv[i] = s_bv[i];
            pp[i] = s_bp[i];
            ns += s_wc[i];
          }
          double v = vv[0];
          uint64_t p = pp[0];
#pragma unroll
          for (int i = 1; i < NW; i++)
            if (better(vv[i], pp[i], v, p)) {
              v = vv[i];
              p = pp[i];
            }
          const uint64_t vb = (uint64_t)__double_as_longlong(v);
          const int j = lane;
          const uint32_t nfl = s_nfl;
          const uint32_t data = j == 0   ? (uint32_t)(vb >> 32)
                                : j == 1 ? (uint32_t)vb
                                : j == 2 ? (p == NONE64 ? NONE : (uint32_t)p)
                                : j == 3 ? nfl
                                : j == 4 ? ns
                                         : ((uint32_t)(j - 5) < nfl ? s_inl[j - 5] : NONE);
          st64(A.partials + (uint64_t)w * PART_G + j, gran(seen, data));
          if (j == 0) s_arr = 0;  // (the next step's arrivals come after the next record)
          if (trace && !A.trace_all && j == 0 && mine == nact / 2 && seen < TRACE_STEPS) {
            uint64_t *tr = trace + (uint64_t)seen * TRACE_W;
            tr[10] = t_seen;
            tr[11] = t_klog;
            tr[12] = t_scanned;
            tr[13] = t_scanned;
            tr[14] = now();
          }
          if (trace && A.trace_all && j == 0) {
            const uint64_t tn = now();
            trace_mark(A, seen, 1, t_seen);
            trace_mark(A, seen, 3, t_scanned);
            trace_mark(A, seen, 5, tn);
          }
          if (trace2 && j == 0 && seen < TRACE2_STEPS) {
            uint64_t *tr = trace2 + ((uint64_t)seen * GMAX + w) * T2W;
            tr[0] = s_t0[0];
            tr[1] = s_t0[1];
            tr[2] = now();
            uint64_t tw = 0;
            for (int i = 0; i < NW; i++) tw = s_tw[i] > tw ? s_tw[i] : tw;
            tr[3] = s_t0[2];
            tr[4] = tw;
            tr[5] = t_red;
          }
        }
      }
    }
    // ---- compaction (off the critical path: the controller is collecting) ----------------
    died = t < n_ent && !al_t;
    const int any_died = __syncthreads_or(died);
    if (s_abort) {
      if (t == 0) atomicMax((unsigned long long *)&A.out[3], 99ull);
      return;
    }
    if (any_died) {
      const bool keep = t < n_ent && al_t;
      const uint64_t bal = __ballot(keep);
      if (lane == 0) s_wc[wv] = (uint32_t)__popcll(bal);
      __syncthreads();
      uint32_t r = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull)), tot = 0;
      for (int i = 0; i < NW; i++) {
        if (i < wv) r += s_wc[i];
        tot += s_wc[i];
      }
      const bool move = keep && r != t;
      // rows move down in groups of eight chunks: every read of a group before any write
      for (int k0 = 0; k0 < nch; k0 += 8) {
        uint4 v0, v1, v2, v3, v4, v5, v6, v7;
        const int kn = nch - k0;
        uint4 *src = lrow + (uint64_t)k0 * NT + t;
        if (move) {
          v0 = src[0];
          if (kn > 1) v1 = src[NT];
          if (kn > 2) v2 = src[2 * NT];
          if (kn > 3) v3 = src[3 * NT];
          if (kn > 4) v4 = src[4 * NT];
          if (kn > 5) v5 = src[5 * NT];
          if (kn > 6) v6 = src[6 * NT];
          if (kn > 7) v7 = src[7 * NT];
        }
        __syncthreads();
        uint4 *dst = lrow + (uint64_t)k0 * NT + r;
        if (move) {
          dst[0] = v0;
          if (kn > 1) dst[NT] = v1;
          if (kn > 2) dst[2 * NT] = v2;
          if (kn > 3) dst[3 * NT] = v3;
          if (kn > 4) dst[4 * NT] = v4;
          if (kn > 5) dst[5 * NT] = v5;
          if (kn > 6) dst[6 * NT] = v6;
          if (kn > 7) dst[7 * NT] = v7;
        }
        __syncthreads();
      }
      if (keep) lpos[r] = pos_t;
      __syncthreads();
      n_ent = tot;
      al_t = t < n_ent;
      if (al_t) {
        const uint32_t np = lpos[t];
        if (np != pos_t) {
          pos_t = np;
          pi_t = PInfo{A.mag_s[pos_t], A.sumsq_s[pos_t], A.len_s[pos_t]};
          pt_t = pterms(pi_t.mag, pi_t.sumsq, A.B);
          ps_t = psmall(pi_t, pt_t);
        }
      }
    }
  }
}

// ============================================================================================
// Dense streaming workers (narrow rows, more than NT candidates per worker: config D on one to
// four GPUs).  Tiles of DT positions are dealt round-robin as in the dense form, and a worker
// keeps its alive candidates as ONE dense list in static-position order -- but the rows live in
// HBM, in a per-worker buffer laid out for the scan: entry e is lane e % 64 of group e / 64, and a
// group's chunk k is 64 consecutive 16-byte words (one coalesced 1 KiB load per wave).  Thread t
// takes entries t, t + NT, ...  A dead entry's row is simply not loaded; once a quarter of the
// list has died the worker rewrites the alive rows densely into its other buffer (off the
// critical path, after its partial), so the streamed bytes stay within 4/3 of the alive rows'
// -- the chunk-major static layout fetched every 128-byte line that held one alive row, 1.8x the
// alive bytes at config D (profiles/r03_v11/config_d_pmc.json).  The compaction's traffic is
// the alive rows once per quarter of deaths: gigabytes against the scan's terabytes.
// LDS: record words | entry positions (compaction staging)
// ============================================================================================
constexpr int SJ = 32;  // entries per thread the dense streaming form takes (fcap <= SJ * NT: bits of a mask)

// 16-byte load that bypasses this CU's vector L1 (sc1): the rows were written by other threads
// of this workgroup (compaction), whose stores reached L2 before the barrier
__device__ __forceinline__ uint4 ld_sc1_16(const __amdgpu_buffer_rsrc_t r, uint32_t off) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16);
  return make_uint4(v.x, v.y, v.z, v.w);
}

template <typename T, int NCH>
__device__ __forceinline__ void worker_dstream(const AccArgs &A, const DevClassifier &C, uint4 *dyn) {
  __shared__ double s_bv[NW];
  __shared__ uint64_t s_bp[NW];
  __shared__ uint32_t s_nfl, s_go, s_inl[INL], s_wc[NW], s_cnt;
  __shared__ int s_abort;
  __shared__ uint32_t s_arr;
  __shared__ SmallK s_sk;  // classify_small's constants (read with each candidate's row)
  constexpr int NC = NCH > 0 ? NCH : DMAXCH;
  const uint32_t GW = gridDim.x - 1, w = blockIdx.x - 1;
  const Div32 dgw(GW);
  const int lane = threadIdx.x & 63, wv = wave_id();
  const uint32_t t = threadIdx.x;
  const int nch = NCH > 0 ? NCH : A.nch;
  const int rec_words = (int)A.rec_g;
  uint32_t *srec = reinterpret_cast<uint32_t *>(dyn);
  const uint4 *clds = dyn;  // the centre row: record words 0 .. 4 nch
  // entry positions of the current list and the rebuild's target (fcap each)
  // (LDS- and global-typed: a buffer picked by index would otherwise be a flat access)
  MC_LDS uint32_t *lpos[2] = {(MC_LDS uint32_t *)reinterpret_cast<uint32_t *>(dyn + (rec_words + 3) / 4), nullptr};
  lpos[1] = lpos[0] + (A.fcap + 3) / 4 * 4;
  // this worker's two row buffers (fcap entries each), as buffer resources for sc1 loads; an
  // entry is its nch row chunks and an info chunk {mag, len, ap, np} (classify_small's PSm,
  // ap = ~0 when not ok), so the scan reads no per-position arrays
  const uint32_t CH = (uint32_t)nch + 1;
  const uint64_t wrow = A.fcap * (uint64_t)CH;  // uint4 per buffer
  MC_GLB u32x4_t *rb[2] = {(MC_GLB u32x4_t *)(A.srows + (uint64_t)w * 2 * wrow),
                           (MC_GLB u32x4_t *)(A.srows + ((uint64_t)w * 2 + 1) * wrow)};
  const __amdgpu_buffer_rsrc_t rr[2] = {__builtin_amdgcn_make_buffer_rsrc((u32x4_t *)rb[0], 0, (int)(wrow * 16), 0x00020000),
                                        __builtin_amdgcn_make_buffer_rsrc((u32x4_t *)rb[1], 0, (int)(wrow * 16), 0x00020000)};
  int cur = 0;
  const uint32_t J = (uint32_t)((A.fcap + NT - 1) / NT);  // entries per thread (<= SJ)
  auto slot = [&](uint32_t e, int k) -> uint32_t {  // uint4 index of entry e's chunk k in a buffer
    return ((e >> 6) * CH + (uint32_t)k) * 64u + (e & 63u);
  };
  // entries below dres (each thread's first, j = 0) are scanned from an LDS copy, chunk k of
  // entry e at lres[k * dres + e]: as the rebuilds shrink the list, more and more of it is
  // resident (the HBM buffers keep every row: the rebuild reads them)
  const uint32_t dres = A.dres;
  MC_LDS u32x4_t *lres = (MC_LDS u32x4_t *)(lpos[1] + (A.fcap + 3) / 4 * 4);
  const bool small_on = sizeof(T) == 1 && A.fc.on && A.fc.mk;
  // entry e = t + NT j: this worker's (e / DT)-th tile, offset e % DT (positions increase with
  // the entry, so the entries below N are a prefix)
  uint32_t alive = 0;  // bit j: entry t + NT j alive
  for (uint32_t j = 0; j < J; j++) {
    const uint32_t e = t + NT * j;
    if (e >= A.fcap) break;
    const uint64_t lt = (uint64_t)w + (uint64_t)(e / DT) * GW;
    const uint64_t p = (lt * A.W + A.rank) * DT + (e % DT);
    if (p >= A.N) break;
    lpos[0][e] = (uint32_t)p;
    alive |= 1u << j;
    for (int k = 0; k < nch; k++) {
      const uint4 x = A.hs[(uint64_t)k * A.npad + p];
      glb_st16(rb[0] + slot(e, k), x);
      if (e < dres) lds_st16(lres + (uint32_t)k * dres + e, x);
    }
    const PInfo pi{A.mag_s[p], A.sumsq_s[p], A.len_s[p]};
    const PSm ps = psmall(pi, pterms(pi.mag, pi.sumsq, A.B));
    const uint4 xi = make_uint4(ps.mag, ps.len, ps.ok ? ps.ap : ~0u, ps.np);
    glb_st16(rb[0] + slot(e, nch), xi);
    if (e < dres) lds_st16(lres + (uint32_t)nch * dres + e, xi);
  }
  drain();  // (the rows are read back with sc1 loads after the barrier below)
  if (t == 0) {
    s_cnt = 0;
    s_abort = 0;
    s_arr = 0;
    s_sk = make_smallk(C, A.fc);
  }
  __syncthreads();
  {
    const uint32_t c = wave_sum32((uint32_t)__popc(alive));
    if (lane == 0 && c) atomicAdd(&s_cnt, c);
  }
  __syncthreads();
  uint32_t n_ent = s_cnt;  // list length (alive or not since the last rebuild)
  uint32_t kcur = 0, seen = 0;
  for (;;) {
    // ---- wait for the next step's record (wave 0), as `worker` ---------------------------
    if (wv == 0) {
      const uint64_t t0 = now();
      const uint32_t want = seen + 1;
      int state = 0;
      uint32_t got = want;
      bool late = false;
      const uint64_t *rn = A.ring + (uint64_t)(want % RING) * A.rec_g;
      for (uint32_t it = 1;; it++) {
        bool ok = true, okh = true, ahead = false;
        for (int j = lane; j < rec_words; j += 64) {
          const uint64_t x = ld64(rn + j);
          const uint32_t tg = (uint32_t)(x >> 32);
          ok &= tg == want;
          if (j >= 4 * nch) okh &= tg == want;
          ahead |= (int32_t)(tg - want) > 0;
          srec[j] = (uint32_t)x;
        }
        // (a thin record: every header granule tagged, bit 30 of its kill-log word; no row)
        if (__ballot(!ok) != 0 && __ballot(!okh) == 0 && (lds_u32(srec + 4 * nch + 3) & REC_THIN)) ok = true;
        if (__ballot(!ok) == 0) {
          state = 1;
          break;
        }
        if (__ballot(ahead) != 0) {
          late = true;
          break;
        }
        if ((it & 255) == 0 && timed_out(A, t0)) {
          state = 2;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      while (late && state == 0) {
        uint32_t v = 0;
        if (lane == 0) {
          for (uint32_t it = 1; (v = ld32(A.go)) == seen; it++) {
            if ((it & 255) == 0 && timed_out(A, t0)) break;
            __builtin_amdgcn_s_sleep(1);
          }
        }
        v = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
        if (v == seen) {
          state = 2;
          break;
        }
        const uint64_t *r = A.ring + (uint64_t)(v % RING) * A.rec_g;
        bool ok = true, okh = true;
        for (int j = lane; j < rec_words; j += 64) {
          const uint64_t x = ld64(r + j);
          ok &= (uint32_t)(x >> 32) == v;
          if (j >= 4 * nch) okh &= (uint32_t)(x >> 32) == v;
          srec[j] = (uint32_t)x;
        }
        if (__ballot(!ok) != 0 && __ballot(!okh) == 0 && (lds_u32(srec + 4 * nch + 3) & REC_THIN)) ok = true;
        if (__ballot(!ok) == 0) {
          state = 1;
          got = v;
        }
      }
      if (lane == 0) {
        if (state == 2) s_abort = 1;
        s_go = got;
        s_nfl = 0;
      }
    }
    __syncthreads();
    if (s_abort) {
      if (t == 0) atomicMax((unsigned long long *)&A.out[3], 99ull);
      return;
    }
    seen = s_go;
    const uint32_t *hdr = srec + 4 * nch;
    if (hdr[0] == NONE) return;  // accumulation finished
    if (hdr[3] & REC_THIN) load_thin_record(A, srec, nch, hdr[0]);
    uint64_t W_S = hdr[1], W_E = hdr[2];
    const uint32_t kend = hdr[3] & REC_KMASK;
    const bool exact = (hdr[3] >> 31) != 0;
    const PInfo pc{(uint64_t)hdr[4 + KINL] | ((uint64_t)hdr[5 + KINL] << 32),
                   (uint64_t)hdr[6 + KINL] | ((uint64_t)hdr[7 + KINL] << 32),
                   (uint64_t)hdr[8 + KINL] | ((uint64_t)hdr[9 + KINL] << 32)};
    const PTerms tq = pterms_mk(pc.mag, pc.sumsq, A.B, A.fc.rB);
    const PSm ps_q = psmall(pc, tq);
    const double kq = (double)((int64_t)pc.mag - (int64_t)A.B * tq.ap);
    const bool small_q = small_on && ps_q.ok;
    const MC_LDS uint32_t *lp = lpos[cur];
    // the controller's kills since the last record, against each entry of this thread
    {
      const uint32_t kinl0 = kend > (uint32_t)KINL ? kend - KINL : 0;
      const uint64_t t0k = kinl0 > kcur ? now() : 0;
      for (uint32_t e = kcur; e < kend; e++) {
        uint32_t p;
        if (e >= kinl0) {
          p = hdr[4 + KINL - (kend - e)];
        } else {
          uint64_t g = ld64(A.klog + e);
          for (uint32_t it = 1; (uint32_t)(g >> 32) != e + 1; it++) {
            if ((it & 255) == 0 && timed_out(A, t0k)) {
              s_abort = 1;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
            g = ld64(A.klog + e);
          }
          p = (uint32_t)g;
        }
        for (uint32_t j = 0; j < J; j++)
          if (((alive >> j) & 1u) && lp[t + NT * j] == p) alive &= ~(1u << j);
      }
      kcur = kend;
    }
    // the exact window: the record's span, or part B (a superset span was published first)
    bool abandon = false;
    if (A.spec && !exact) {
      const uint64_t *rbp = A.ringb + (uint64_t)(seen % RING) * 2;
      const uint64_t t0 = now();
      uint64_t b0 = 0, b1 = 0;
      for (uint32_t it = 1;; it++) {
        const uint64_t g = lane < 2 ? ld64(rbp + lane) : 0;
        b0 = readlane64(g, 0);
        b1 = readlane64(g, 1);
        if ((uint32_t)(b0 >> 32) == seen && (uint32_t)(b1 >> 32) == seen) break;
        if ((it & 255) == 0 && timed_out(A, t0)) {
          if (lane == 0) s_abort = 1;
          b0 = b1 = NONE;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      W_S = (uint32_t)b0;
      W_E = (uint32_t)b1;
      abandon = (uint32_t)W_S == NONE;
    }
    uint64_t c0 = 0, c1 = 0;
    const bool any_tile = !abandon && rank_tiles(W_S / DT, W_E / DT, A.W, A.rank, &c0, &c1);
    const uint32_t nact = any_tile ? (uint32_t)(c1 - c0 + 1 < (uint64_t)GW ? c1 - c0 + 1 : (uint64_t)GW) : 0u;
    const uint32_t mine = any_tile ? dgw.mod(w + GW - dgw.mod((uint32_t)c0)) : 0u;
    const bool active = any_tile && mine < nact;  // (uniform)
    if (active) {
      double best_v = -1.0;
      uint64_t best_p = NONE64;
      uint32_t nscan = 0;
      bool listed = false;
      const __amdgpu_buffer_rsrc_t R = rr[cur];
      for (uint32_t j = 0; j < J; j++) {
        const uint32_t e = t + NT * j;
        if (!((alive >> j) & 1u)) continue;
        const uint32_t p = lp[e];
        if (p < W_S || p > W_E) continue;
        nscan++;
        uint4 v[NC], inf;
        if (e < dres) {
#pragma unroll
          for (int k = 0; k < NC; k++)
            if (k < nch) v[k] = lds_ld16(lres + (uint32_t)k * dres + e);
          inf = lds_ld16(lres + (uint32_t)nch * dres + e);
        } else {
#pragma unroll
          for (int k = 0; k < NC; k++)
            if (k < nch) v[k] = ld_sc1_16(R, slot(e, k) * 16u);
          inf = ld_sc1_16(R, slot(e, nch) * 16u);
        }
        const SmallK sk = lds_smallk(&s_sk);
        Acc<T> acc;
#pragma unroll
        for (int k = 0; k < NC; k++)
          if (k < nch) acc.add(v[k], clds[k]);
        double cv = -1.0;
        int d = 0;
        bool und = true;
        if constexpr (sizeof(T) == 1) {
          if (small_q && inf.z != ~0u) {
            const PSm ps{inf.x, inf.y, inf.z, inf.w, true};
            acc.fold();
            const double dap = C.layout == 4 ? mk_div((double)inf.x, (double)A.B, A.fc.rB) : 0.0;
            d = classify_small(sk, acc.sad, acc.dot, ps, ps_q, kq, dap, tq.da, A.B, &cv, &und);
          }
        }
        if (und) {  // (classify_small undecided or not applicable: the per-position arrays)
          const PInfo pi{A.mag_s[p], A.sumsq_s[p], A.len_s[p]};
          const PTerms pt = pterms(pi.mag, pi.sumsq, A.B);
          double cx;
          d = A.fc.on    ? classify_fast(C, A.fc, acc.finish(pi.mag, pc.mag), pi, pt, pc, tq, A.B, &cx)
              : C.layout ? classify_std(C, acc.finish(pi.mag, pc.mag), pi, pt, pc, tq, A.B, &cx)
                         : classify_cand<T>(acc, pi, pc, A.B, C, &cx);
          if (cv == -1.0) cv = cx;
        }
        if (d) {
          alive &= ~(1u << j);
          const uint32_t idx = atomicAdd(&s_nfl, 1u);
          if (idx < (uint32_t)INL) s_inl[idx] = p;
          else {
            st32(A.fpos + (uint64_t)w * A.fcap + idx, p);
            listed = true;
          }
        }
        if (cv > -1.0 && better(cv, p, best_v, best_p)) {
          best_v = cv;
          best_p = p;
        }
      }
      nscan = wave_sum32(nscan);
      // the wave's first maximum (a lane's entries are not adjacent: pairs only on ties)
      if (__ballot(best_p != NONE64)) {
        const double m = wave_ext_f64_all<true>(best_v);
        const uint64_t hit = __ballot(best_p != NONE64 && best_v == m);
        if (__popcll(hit) > 1) {
          wave_best_all(best_v, best_p, better);
        } else {
          const int L = __builtin_ctzll(hit);
          best_v = __builtin_bit_cast(double, readlane64(__builtin_bit_cast(uint64_t, best_v), L));
          best_p = readlane64(best_p, L);
        }
      }
      if (lane == 0) {
        s_bv[wv] = best_v;
        s_bp[wv] = best_p;
        s_wc[wv] = nscan;
      }
      if (__ballot(listed)) drain();
      // arrival: the wave that completes the workgroup's scores publishes the partial
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      uint32_t arr = 0;
      if (lane == 0) arr = atomicAdd(&s_arr, 1u);
      arr = (uint32_t)__builtin_amdgcn_readfirstlane((int)arr);
      if (arr == (uint32_t)NW - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (lane < PART_G) {
          double v = s_bv[0];
          uint64_t pp = s_bp[0];
          uint32_t ns = s_wc[0];
#pragma unroll
          for (int i = 1; i < NW; i++) {
            ns += s_wc[i];
            if (better(s_bv[i], s_bp[i], v, pp)) {
              v = s_bv[i];
              pp = s_bp[i];
            }
          }
          const uint64_t vb = (uint64_t)__double_as_longlong(v);
          const int jj = lane;
          const uint32_t nfl = s_nfl;
          const uint32_t data = jj == 0   ? (uint32_t)(vb >> 32)
                                : jj == 1 ? (uint32_t)vb
                                : jj == 2 ? (pp == NONE64 ? NONE : (uint32_t)pp)
                                : jj == 3 ? nfl
                                : jj == 4 ? ns
                                          : ((uint32_t)(jj - 5) < nfl ? s_inl[jj - 5] : NONE);
          st64(A.partials + (uint64_t)w * PART_G + jj, gran(seen, data));
          if (jj == 0) s_arr = 0;  // (the next step's arrivals come after the next record)
        }
      }
    }
    // ---- the list's rebuild once a quarter of it has died (off the critical path: the
    // controller is collecting) -----------------------------------------------------------
    if (t == 0) s_cnt = 0;
    __syncthreads();
    if (s_abort) {
      if (t == 0) atomicMax((unsigned long long *)&A.out[3], 99ull);
      return;
    }
    {
      const uint32_t c = wave_sum32((uint32_t)__popc(alive));
      if (lane == 0 && c) atomicAdd(&s_cnt, c);
    }
    __syncthreads();
    const uint32_t nal = s_cnt;
    if ((n_ent - nal) * 4 >= n_ent && nal < n_ent) {
      // new index of an alive entry = alive entries before it in entry order (entry
      // e = t + NT j: by j, then by t): one block scan per j
      const int nxt = cur ^ 1;
      uint32_t base = 0;
      for (uint32_t j = 0; j < J; j++) {
        const bool al = (alive >> j) & 1u;
        const uint64_t bal = __ballot(al);
        if (lane == 0) s_wc[wv] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t r = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull)), tot = 0;
        for (int i = 0; i < NW; i++) {
          if (i < wv) r += s_wc[i];
          tot += s_wc[i];
        }
        if (al) {
          const uint32_t e = t + NT * j;
          for (int k = 0; k <= nch; k++) {
            const uint4 x = ld_sc1_16(rr[cur], slot(e, k) * 16u);
            glb_st16(rb[nxt] + slot(r, k), x);
            if (r < dres) lds_st16(lres + (uint32_t)k * dres + r, x);  // (the rebuild reads only the HBM copies)
          }
          lpos[nxt][r] = lp[e];
        }
        base += tot;
        __syncthreads();  // (s_wc is rewritten by the next round)
      }
      drain();  // every row store has reached L2 before the barrier (the next reads are sc1)
      __syncthreads();
      n_ent = base;
      alive = 0;
      for (uint32_t j = 0; j < J; j++)
        if (t + NT * j < n_ent) alive |= 1u << j;
      cur = nxt;
    }
  }
}

// ============================================================================================
// Controller (WG 0).  LDS: integer mean row | column sums | bvec (counts, Fenwick tree, bin
// starts, begin bounds, bitmap unless global) | member cache
// ============================================================================================
template <typename T, int NCH, bool WIDE, int TSZ, bool PROF>
__device__ __forceinline__ void controller(const AccArgs &A, uint4 *dyn) {
  // profiling state only in the PROF instantiation (MC_ACCUM_PROFILE): the production kernel
  // carries no timer registers
  [[maybe_unused]] const bool prof_on = PROF && A.prof;
  [[maybe_unused]] uint64_t *const trace = PROF ? A.trace : nullptr;
  [[maybe_unused]] uint64_t *const trace2 = PROF ? A.trace2 : nullptr;
  __shared__ uint64_t s_red[3 * NW];
  __shared__ double s_bv[NW];
  __shared__ uint64_t s_bp[NW];
  __shared__ uint32_t s_new;  // members taken into the cluster this step
  __shared__ uint32_t s_plist[PLIST];  // ... their positions
  __shared__ uint32_t s_pbin[PLIST];   // ... their bvec bins (kills deferred to the next window)
  __shared__ uint64_t s_q[4];
  __shared__ uint32_t s_klast[KINL];
  __shared__ uint32_t s_span_all;  // spec: the last record's span was every position
  __shared__ int s_abort;
  __shared__ uint64_t s_sumF;
  __shared__ double s_xv[64];  // the ranks' step headers (mailbox)
  __shared__ uint64_t s_xp[64];
  __shared__ uint32_t s_xn[64], s_xs[64], s_xi[64][MBOX_INL];
  constexpr int NC = NCH > 0 ? NCH : 1;
  const uint32_t GW = gridDim.x - 1;
  const int lane = threadIdx.x & 63, wv = wave_id();
  const int nch = NCH > 0 ? NCH : A.nch;
  const int rec_words = (int)A.rec_g;
  uint8_t *Fl = reinterpret_cast<uint8_t *>(dyn);  // integer mean row
  uint64_t *msum = reinterpret_cast<uint64_t *>(Fl + (size_t)nch * 16);
  uint32_t *cnt = reinterpret_cast<uint32_t *>(msum + A.B);
  uint32_t *fw = cnt + ((A.nb + 1) & ~1u);
  uint32_t *lo = fw + ((A.nb + 2) & ~1u);
  uint64_t *bnd = reinterpret_cast<uint64_t *>(lo + ((A.nb + 2) & ~1u));
  uint32_t *lbits = reinterpret_cast<uint32_t *>(bnd + A.nb);
  const uint64_t nwords = (A.N + 31) / 32;
  MemberCache mc;
  {
    uint8_t *p = reinterpret_cast<uint8_t *>(lbits + (A.gbits ? 0 : (nwords + 3) / 4 * 4));
    mc.rp = WIDE ? 0 : nch + 1;  // (wide rows: member metadata only, rows read from `hr`)
    mc.row = reinterpret_cast<uint4 *>(p);
    p += (size_t)A.mrow * mc.rp * 16;
    mc.wt = reinterpret_cast<WinTab *>(p);
    p += (size_t)A.mrow * sizeof(WinTab);
    mc.info = reinterpret_cast<uint64_t *>(p);
    p += (size_t)A.mrow * 24;
    mc.key = reinterpret_cast<uint64_t *>(p);
    p += (size_t)A.mrow * 8;
    mc.pos = reinterpret_cast<uint32_t *>(p);
  }
  for (int i = threadIdx.x; i < nch * 16; i += NT) Fl[i] = 0;  // the mean row's padding stays zero
  if (threadIdx.x == 0) {
    s_abort = 0;
    s_new = 0;
  }
  uint64_t lg = 1;
  while (lg * 2 <= A.nb) lg *= 2;
  // the workers' partials as a buffer resource (16-byte sc1 polls, aux 16 = sc1)
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc(A.partials, 0, (int)(GW * PART_G * 8), 0x00020000);
  DevBvec bv{A.gbits, (MC_LDS uint32_t *)lbits, A.gbits != nullptr, cnt, fw, lo, bnd, A.len_s, A.nb, lg};
  uint32_t last = NONE;   // current centre (static position)
  uint32_t last_q = 0;    // its member index in the current cluster
  uint64_t cl_start = 0;  // first member index of the current cluster
  uint64_t M = 0;         // members of the current cluster
  uint64_t ncl = 0, nsteps = 0, ncand = 0;
  uint32_t step = 0;
  uint64_t err = 0;
  uint32_t kn = 0;      // kill-log length
  bool rec_exact = false;  // the record being published carries the exact window (no part B)
  bool thin_out = false;   // this step's record went out thin (its part B is still to come)
  uint32_t npend = 0;   // new members s_plist[0, npend) whose bvec kills are still to be done
  uint64_t t_wait = 0, t_coll = 0, t_mark = 0;
  const uint64_t clk0 = prof_on ? __builtin_amdgcn_s_memtime() : 0, rt0 = prof_on ? now() : 0;
  uint64_t t_sub[4] = {0, 0, 0, 0};  // collect: reduce (stragglers), column sums, mean, closest
  uint64_t t_ws[4] = {0, 0, 0, 0};   // window: centre window data, window, record; [3] collect's takes
  uint64_t t_cl[3] = {0, 0, 0};      // closest: members scored (wave 0), reduced + barrier, winner + barrier
  uint64_t t_pub[2] = {0, 0};        // window (spec): the record's span, the record's stores issued
  uint64_t t_wk[5] = {0, 0, 0, 0, 0};  // window: bvec kills, fast form, general form (time); fast, general (count)

  // The controller's global stores of cluster bookkeeping (cluster table, member list, kill
  // log) come from thread 64, never from wave 0: wave 0 publishes the next step record, and
  // the compiler waits for every outstanding vector-memory operation of that wave before the
  // record's first store (its words come from LDS or, for an uncached centre, global loads: one
  // merged register, one conservative vmcnt(0)) -- a write-through store still in flight there
  // held the record back by a memory round trip at every cluster change.
  constexpr uint32_t BK = 64;
  auto finish_cluster = [&]() {
    if (threadIdx.x == BK) {
      A.cl_centre[ncl] = last;
      A.cl_off[ncl + 1] = cl_start + M;
    }
    ncl++;
    cl_start += M;
    M = 0;
  };
  // accumulate's `current = {last}`: member 0 of a new cluster, its row, sums and window data
  // (kill: the seed also leaves the bvec here -- bvec::erase of get_close's best candidate --
  // with its bin from the member info, no search for it)
  auto log_kill = [&](uint64_t p) {  // a pop / erase, for the workers (thread 0: LDS, thread BK: global)
    if (threadIdx.x == BK) st64(A.klog + kn, gran(kn + 1, (uint32_t)p));
    if (threadIdx.x == 0) s_klast[kn % KINL] = (uint32_t)p;
  };
  // (thread 0's global stores come after every load of the seed: a load behind a store waits
  // for the store, see publish)
  auto new_cluster = [&](uint64_t pos, bool kill = false, bool logged = false) {
    if (A.mrow && !WIDE)
      for (int c = threadIdx.x; c < nch; c += NT) mc.row[c] = A.hr[pos * nch + c];
    for (int b = threadIdx.x; b < A.B; b += NT) msum[b] = reinterpret_cast<const T *>(A.hr + pos * nch)[b];
    if (kill && !logged) log_kill(pos);
    if (threadIdx.x == 0) {
      if (A.mrow) {
        uint2 w[MINFO_W];
        minfo_issue(A.minfo + pos, w);
        const MInfo mi = minfo_take(w);
        if (kill) bv.kill_in(pos, mi.bin);
        mc.pos[0] = (uint32_t)pos;
        mc.key[0] = 0;
        mc.info[0] = mi.mag;
        mc.info[1] = mi.sumsq;
        mc.info[2] = mi.len;
        mc.wt[0] = mi.wt;
      } else if (kill) {
        bv.kill_one(pos);
      }
    }
    if (threadIdx.x == BK) {
      st32(A.mem_pos + cl_start, (uint32_t)pos);
      st64(A.mkeys + cl_start, 0);
    }
    M = 1;
    last_q = 0;
    if (kill && !logged) kn++;
    // (no drain: the seed's member-list entries are never read back in the kernel -- member 0
    // is always in the LDS cache -- and the kill log is tagged, so the stores need not have
    // landed before the next step is published)
    __syncthreads();
  };
  auto pop = [&]() -> uint64_t {  // bvec::pop (bvec.cpp:26-37): static position or ~0
    const int64_t b = bv.first_nonempty();
    if (b < 0) return NONE64;
    const uint64_t p = bv.select((uint64_t)b, 0);
    if (threadIdx.x == 0) bv.kill_in(p, (uint64_t)b);
    log_kill(p);
    kn++;
    __syncthreads();
    return p;
  };
  // data word j of the record for the current `last` (centre row words, then the header)
  auto rec_word = [&](int j, bool have, uint64_t S, uint64_t E) -> uint32_t {
    const bool cached = last_q < A.mrow;
    if (!WIDE && j < 4 * nch) {
      if (last == NONE) return 0;
      const uint4 v = cached ? lds_u4(mc.row + (size_t)last_q * mc.rp + j / 4) : A.hr[(uint64_t)last * nch + j / 4];
      return (j & 3) == 0 ? v.x : (j & 3) == 1 ? v.y : (j & 3) == 2 ? v.z : v.w;
    }
    const int h = j - (WIDE ? 0 : 4 * nch);
    if (h == 0) return have ? last : NONE;
    if (h == 1) return (uint32_t)S;
    if (h == 2) return (uint32_t)E;
    if (h == 3) return kn | (rec_exact ? 0x80000000u : 0u);
    if (h < 4 + KINL) {  // kill-log entry kn - KINL + (h - 4)
      const int64_t e = (int64_t)kn - KINL + (h - 4);
      return e >= 0 ? s_klast[e % KINL] : NONE;
    }
    if (last == NONE) return 0;
    const int f = (h - 4 - KINL) / 2, hi = (h - 4 - KINL) & 1;
    const uint64_t v =
        cached ? lds_u64(mc.info + (size_t)last_q * 3 + f) : (f == 0 ? A.mag_s[last] : f == 1 ? A.sumsq_s[last] : A.len_s[last]);
    return hi ? (uint32_t)(v >> 32) : (uint32_t)v;
  };

  // publish the record of `step` for the current `last` (wave 0: one granule per lane, every
  // granule tagged with the step).  Kill-log entries are tagged granules: a worker that needs
  // one checks its tag, so the record is not held back until they land.  `go` is only a hint
  // for a worker that fell RING steps behind: it re-validates the record's tags after reading.
  // rec_word for a cached centre (row and magnitudes in the member cache): every word is one
  // LDS read from a per-lane address or a uniform value -- no per-word branches (the general
  // form's divergent cases cost a single wave ≈0.7 us per record)
  auto rec_word_cached = [&](int j, bool have, uint64_t S, uint64_t E) -> uint32_t {
    const int h = j - 4 * nch;
    const int64_t e = (int64_t)kn - KINL + (h - 4);
    const MC_LDS uint32_t *row = (const MC_LDS uint32_t *)(mc.row + (size_t)last_q * mc.rp);
    const MC_LDS uint32_t *inf = (const MC_LDS uint32_t *)(mc.info + (size_t)last_q * 3);
    const MC_LDS uint32_t *p = h < 0               ? row + j
                               : h < 4 + KINL      ? (const MC_LDS uint32_t *)s_klast + (e >= 0 ? (uint32_t)e % KINL : 0u)
                                                   : inf + (h - 4 - KINL);
    const uint32_t x = *p;
    if (h < 0) return x;
    if (h == 0) return have ? last : NONE;
    if (h == 1) return (uint32_t)S;
    if (h == 2) return (uint32_t)E;
    if (h == 3) return kn | (rec_exact ? 0x80000000u : 0u);
    if (h < 4 + KINL) return e >= 0 ? x : NONE;
    return x;
  };
  // (Every word of a lane is read before its first store: on gfx9 stores count in vmcnt, so a
  // load issued after a store waits for that store to complete -- a write-through round trip.)
  // rec_read / rec_store: the record's words j0 .. j0 + 64 * PW - 1 (PW per lane, held in
  // registers between the reads and the stores); publish: every word
  constexpr int PW = 4;
  auto rec_read = [&](int j0, uint64_t S, uint64_t E, bool have, uint32_t (&d)[PW]) {
    const bool fastw = !WIDE && last != NONE && last_q < A.mrow;  // (uniform)
    if (fastw) {
#pragma unroll
      for (int u = 0; u < PW; u++) {
        const int j = j0 + u * 64 + lane;
        d[u] = j < rec_words ? rec_word_cached(j, have, S, E) : 0u;
      }
    } else {
#pragma unroll
      for (int u = 0; u < PW; u++) {
        const int j = j0 + u * 64 + lane;
        d[u] = j < rec_words ? rec_word(j, have, S, E) : 0u;
      }
    }
  };
  auto rec_store = [&](int j0, const uint32_t (&d)[PW]) {
    uint64_t *r = A.ring + (uint64_t)(step % RING) * A.rec_g;
#pragma unroll
    for (int u = 0; u < PW; u++) {
      const int j = j0 + u * 64 + lane;
      if (j < rec_words) st64(r + j, gran(step, d[u]));
    }
  };
  // a thin record (dense workers): the header of a new seed's step -- span every position, no
  // row and no magnitudes (each worker loads them from the static copies) -- published as soon
  // as get_close has chosen the seed, before the controller has loaded it (wave 0)
  auto publish_thin = [&](uint32_t pos) {
    const int h = lane;
    const int64_t e = (int64_t)kn - KINL + (h - 4);
    const uint32_t kx = s_klast[e >= 0 ? (uint32_t)e % KINL : 0u];
    const uint32_t x = h == 0 ? pos : h == 1 ? 0u : h == 2 ? (uint32_t)(A.N - 1) : h == 3 ? (kn | REC_THIN)
                     : h < 4 + KINL ? (e >= 0 ? kx : NONE) : 0u;
    if (4 * nch + h < rec_words) st64(A.ring + (uint64_t)(step % RING) * A.rec_g + 4 * nch + h, gran(step, x));
    if (lane == 0) st32(A.go, step);
  };
  auto publish = [&](uint64_t S, uint64_t E, bool have) {
    for (int j0 = 0; j0 < rec_words; j0 += 64 * PW) {
      uint32_t d[PW];
      rec_read(j0, S, E, have, d);
      rec_store(j0, d);
    }
    if (lane == 0) st32(A.go, step);
  };

  // member qm of the current cluster is static position p, flagged in this step (key step << 32
  // | p orders members like the bvec walk): member list, cache entry (row, magnitudes, window
  // data from the read-only static arrays) or column sums past the cache, and the bvec kill
  // (wide rows: the row stays in `hr`; its column sums are added here only for a member past
  // the step's list, `sums`, the others by the column-sum pass over the list)
  // (defer >= 0: the bvec kill is left to the next window -- the bin goes to s_pbin[defer])
  auto take = [&](uint64_t qm, uint32_t p, bool sums, int64_t defer = -1) {
    const uint64_t key = ((uint64_t)step << 32) | p;
    const uint4 *hrow = A.hr + (uint64_t)p * nch;
    // every load of the member is issued before the first store: LDS stores go through generic
    // pointers, which the compiler does not move loads past (a load -> wait -> store per 16
    // bytes was 21 dependent memory round trips per member, ≈2.9 us of a config-B step)
    const bool cached = qm < A.mrow;
    uint2 w[MINFO_W];
    minfo_issue(A.minfo + p, w);
    if constexpr (!WIDE && NCH > 0) {
      if (cached) {
        uint4 rv[NC];
#pragma unroll
        for (int k = 0; k < NC; k++) rv[k] = hrow[k];
        // (the scheduler would otherwise sink each load to its store: hold them all here)
#pragma unroll
        for (int k = 0; k < NC; k++) asm volatile("" : "+v"(rv[k].x), "+v"(rv[k].y), "+v"(rv[k].z), "+v"(rv[k].w));
#pragma unroll
        for (int k = 0; k < NC; k++) mc.row[qm * mc.rp + k] = rv[k];
      }
    } else if (!WIDE && cached) {
      for (int k = 0; k < nch; k++) mc.row[qm * mc.rp + k] = hrow[k];
    }
    const MInfo mi = minfo_take(w);
    st32(A.mem_pos + cl_start + qm, p);
    st64(A.mkeys + cl_start + qm, key);
    if (cached) {
      mc.pos[qm] = p;
      mc.key[qm] = key;
      mc.info[qm * 3 + 0] = mi.mag;
      mc.info[qm * 3 + 1] = mi.sumsq;
      mc.info[qm * 3 + 2] = mi.len;
      mc.wt[qm] = mi.wt;
    }
    if (WIDE ? sums : qm >= A.mrow) {
      constexpr int per = 16 / (int)sizeof(T);
      for (int k = 0; k < nch; k++) {
        const uint4 v = hrow[k];
        const T *pv = reinterpret_cast<const T *>(&v);
#pragma unroll
        for (int e = 0; e < per; e++)
          if (pv[e]) atomicAdd((unsigned long long *)&msum[k * per + e], (unsigned long long)pv[e]);
      }
    }
    if (defer >= 0) s_pbin[defer] = (uint32_t)mi.bin;
    else bv.kill_in(p, mi.bin);
  };

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
  if (!A.gbits)  // (a global bitmap is initialised by the launcher)
    for (uint64_t x = threadIdx.x; x < nwords; x += NT) {
      const uint64_t rem = A.N - x * 32;
      lbits[x] = rem >= 32 ? ~0u : ((1u << rem) - 1u);
    }
  if (threadIdx.x == 0) {
    A.cl_off[0] = 0;
    s_span_all = 0;
  }
  __syncthreads();
  {
    const uint64_t p = pop();  // MS: Point<T>* last = points.pop()
    if (p != NONE64) {
      last = (uint32_t)p;
      new_cluster(p);
    }
  }

  for (;;) {
    // ============ advance the accumulate loop to the next scan step ========================
    if (prof_on && threadIdx.x == 0) t_mark = now();
    uint64_t S = 0, E = 0;
    bool have = false;
    while (last != NONE && !err) {
      const WinTab wt = last_q < A.mrow ? lds_wt(mc.wt + last_q) : A.minfo[last].wt;  // the centre's window data
      if (prof_on && threadIdx.x == 0) {
        drain();
        const uint64_t t = now();
        t_ws[0] += t - t_mark;
        t_mark = t;
      }
      if (A.spec) {
        // publish the centre now, with a superset of its window: the fast form's window lies in
        // the two edge bins' span [lo[fb], lo[bb + 1]) (bv_fast_window), the general one anywhere.
        // The workers score that span while the exact window is computed (part B, below).  (The
        // step's new members are not killed in the bvec yet: an edge bin with more alive
        // entries than that is nonempty after the kills.)
        const bool fast_after = wt.fb < A.nb && wt.bb < A.nb && cnt[wt.fb] > npend && cnt[wt.bb] > npend;
        // When the window lengths take both edge bins whole -- no static position of bin fb is
        // shorter than len * sim (kf = 0) and none of bin bb longer than len / sim (kble = its
        // size) -- the fast window is [first alive of fb, last alive of bb]: every alive
        // position of the span.  The record then says so and no part B follows (configs B and
        // D: reads within 10 % of each other's length make every window such a span).
        rec_exact = fast_after && wt.kf == 0 && (uint64_t)wt.kble == (uint64_t)(lo[wt.bb + 1] - lo[wt.bb]);
        uint64_t tp0 = 0;
        if (prof_on && threadIdx.x == 0) tp0 = now();
        // The record's words are read from LDS before the other waves start the last step's
        // bvec kills: those are LDS atomics on shared Fenwick nodes, and the record's reads
        // queued behind them held every member step's record back by ≈2 µs.
        const uint64_t S0 = fast_after ? lo[wt.fb] : 0, E0 = fast_after ? lo[wt.bb + 1] - 1 : A.N - 1;
        if (!thin_out) {  // (a thin record is out already: its exact window follows as part B)
          step++;
          if (threadIdx.x == BK) s_span_all = S0 == 0 && E0 == A.N - 1;  // (read after the collect's barriers)
          if (rec_words <= 64 * PW) {  // (uniform: every record of a dense or narrow-row launch)
            uint32_t d[PW];
            if (wv == 0) rec_read(0, S0, E0, true, d);
            if (npend) __syncthreads();
            if (wv == 0) {
              rec_store(0, d);
              if (lane == 0) st32(A.go, step);
            }
          } else if (wv == 0) {
            publish(S0, E0, true);
          }
        }
        if (prof_on && threadIdx.x == 0) {
          const uint64_t t = now();
          t_pub[0] += tp0 - t_mark;  // the record's span (edge bins' counts)
          t_pub[1] += t - tp0;       // the record's words and stores issued
        }
        if (trace2 && threadIdx.x == 0 && step < TRACE_STEPS) trace[(uint64_t)step * TRACE_W + 6] = now();
      }
      uint64_t tk0 = 0;
      if (prof_on && threadIdx.x == 0) tk0 = now();
      if (npend) {  // the last step's bvec kills, after the record is out
        if (!(A.dbg & 1)) {
          // (waves 1.. only: wave 0 is issuing the record's stores)
          if (threadIdx.x >= 64)
            for (uint32_t i = threadIdx.x - 64; i < npend; i += NT - 64) bv.kill_in(s_plist[i], s_pbin[i]);
        } else
        for (uint32_t i0 = 0; i0 < npend; i0 += NT) {
          const uint32_t i = i0 + threadIdx.x;
          const bool act = i < npend;
          bv.kill_list(act, act ? s_plist[i] : 0, act ? s_pbin[i] : 0);
        }
        npend = 0;
        __syncthreads();
      }
      if (prof_on && threadIdx.x == 0) {
        const uint64_t t = now();
        t_wk[0] += t - tk0;
        tk0 = t;
      }
      if (A.spec && rec_exact) {  // the span of the record is the window (alive after the kills)
        S = lo[wt.fb];
        E = lo[wt.bb + 1] - 1;
        rec_exact = false;
        if (thin_out && wv == 0 && lane < 2) st64(A.ringb + (uint64_t)(step % RING) * 2 + lane, gran(step, (uint32_t)(lane ? E : S)));
        thin_out = false;
        if (prof_on && threadIdx.x == 0) {
          const uint64_t t = now();
          t_ws[1] += t - t_mark;
          t_mark = t;
        }
        have = true;
        break;
      }
      const bool ef = wt.fb < A.nb && cnt[wt.fb] > 0, eb = wt.bb < A.nb && cnt[wt.bb] > 0;
      bool fast = wt.fb < A.nb && wt.bb < A.nb && ((ef && eb) || A.xfast);
      int64_t count = 0;
      if (fast) {
        // nearest-alive form (bv_fast_window): four one-wave queries side by side.  An empty
        // edge bin sends bvec::inner_index_of to the first / last non-empty bin, offset 0
        // (bvec.cpp:55-104): front is then the first alive position overall, back the first
        // alive position of the last non-empty bin (tests/native/bvec_check.cpp).
        if (wv < 4) {
          const uint64_t pf = lo[wt.fb] + wt.kf, qb = lo[wt.bb] + wt.kble;
          uint64_t r;
          if (wv == 0) r = ef ? bv.next_alive(pf, lo[wt.fb + 1]) : bv.first_alive_of(bv.first_nonempty());
          else if (wv == 1) r = ef ? bv.prev_alive(lo[wt.fb], pf) : NONE64;
          else if (wv == 2) r = eb ? bv.next_alive(qb, lo[wt.bb + 1]) : bv.first_alive_of(bv.last_nonempty());
          else r = eb ? bv.prev_alive(lo[wt.bb], qb) : NONE64;
          if (lane == 0) s_q[wv] = r;
        }
        __syncthreads();
        const uint64_t q0 = s_q[0], q1 = s_q[1], q2 = s_q[2], q3 = s_q[3];
        __syncthreads();  // s_q is reused
        // (no alive element at all: the general form, which reports the reference's errors)
        fast = (ef || q0 != NONE64) && (eb || q2 != NONE64);
        if (fast) {
          bv_fast_window(q0, q1, q2, q3, lo[wt.bb] + wt.kblt, &S, &E);
          count = (S != NONE64 && E != NONE64 && E >= S) ? 1 : 0;
        }
      }
      if (!fast) {
        bv.h = wt;
        BPos f, b;
        bv_get_range(bv, wt.bl, wt.el, f, b);
        int e = 0;
        count = bv_window(bv, f, b, &S, &E, &e);
        if (e) {
          err = 10 + e;
          if (A.spec && wv == 0 && lane < 2) st64(A.ringb + (uint64_t)(step % RING) * 2 + lane, gran(step, NONE));
          break;
        }
      }
      if (prof_on && threadIdx.x == 0) {
        const uint64_t t = now();
        t_ws[1] += t - t_mark;
        t_mark = t;
        t_wk[fast ? 1 : 2] += t - tk0;
        t_wk[fast ? 3 : 4]++;
      }
      thin_out = false;
      if (count > 0) {
        have = true;
        if (A.spec && wv == 0 && lane < 2) st64(A.ringb + (uint64_t)(step % RING) * 2 + lane, gran(step, (uint32_t)(lane ? E : S)));
        break;
      }
      // part B: no scan for this step (the workers drop their scores)
      if (A.spec && wv == 0 && lane < 2) st64(A.ringb + (uint64_t)(step % RING) * 2 + lane, gran(step, NONE));
      // the OpenMP loop ran no iteration: is_min with a NULL result -> pop a new seed
      const uint64_t p = pop();
      finish_cluster();
      last = p == NONE64 ? NONE : (uint32_t)p;
      if (p != NONE64) new_cluster(p);
    }
    if (have) nsteps++;
    if (!A.spec || !have) {
      step++;
      if (wv == 0) publish(S, E, have);
    }
    if (prof_on && threadIdx.x == 0) {
      const uint64_t t = now();
      t_ws[2] += t - t_mark;
      t_mark = t;
      if (trace && step < TRACE_STEPS) trace[(uint64_t)step * TRACE_W + 0] = t;
    }
    if (!have) break;  // the record told the workers to stop

    // ============ collect the step (get_close's reduction + get_mean) ======================
    constexpr uint64_t TS = (uint64_t)TSZ;  // positions per tile of the workers' ownership
    uint64_t c0 = 0, c1 = 0;
    const uint32_t nact = rank_tiles(S / TS, E / TS, A.W, A.rank, &c0, &c1)
                              ? (uint32_t)(c1 - c0 + 1 < (uint64_t)GW ? c1 - c0 + 1 : (uint64_t)GW)
                              : 0u;
    // mailbox: this rank's slot of the step's parity; the local flagged positions go there
    uint64_t *mslot = A.mbox ? A.mbox + ((uint64_t)(step & 1) * A.W + A.rank) * A.slot_g : nullptr;
    // thread P0 + t polls the partial of the t-th active worker until its granules carry the
    // step, then lists that worker's flagged positions (a slot from an LDS counter: member order
    // is irrelevant, the keys step << 32 | position order them like the bvec walk).  Wave 0 polls
    // nothing: it publishes the next record, and anything it leaves in flight (a mailbox store
    // to host memory) would hold that record's first store back (see BK).
    constexpr uint32_t P0 = 64;
    const uint32_t pt = threadIdx.x - P0;
    double bv_ = -1.0;
    uint64_t bp_ = NONE64;
    uint32_t cnt_w = 0, scan_w = 0;
    if (threadIdx.x >= P0 && pt < nact) {  // (nact <= G - 1 < NT - P0)
      const uint32_t wk = Div32(GW).mod((uint32_t)c0 + pt);
      const uint64_t *q = A.partials + (uint64_t)wk * PART_G;
      const uint32_t poff = wk * PART_G * 8;
      const uint64_t t0 = now();
      uint64_t g8[PART_G];
      for (uint32_t it = 1;; it++) {
        // the whole partial per poll: one round trip once it has landed (A.poll1: the tag
        // granule first, then all of them)
        bool ok = true;
        if (A.poll1) {
          ok = (uint32_t)(ld64(q + 4 + INL) >> 32) == step;
          if (ok) {
#pragma unroll
            for (int j = 0; j < 5 + INL; j++) {
              g8[j] = ld64(q + j);
              ok &= (uint32_t)(g8[j] >> 32) == step;
            }
          }
        } else {
          // 16-byte sc1 loads of granule pairs (half the requests of 8-byte loads; each 8-byte
          // granule still carries its own tag)
#pragma unroll
          for (int j = 0; j < PART_G / 2; j++) {
            const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(prs, (int)(poff + 16 * j), 0, 16);
            g8[2 * j] = ((uint64_t)v.y << 32) | v.x;
            g8[2 * j + 1] = ((uint64_t)v.w << 32) | v.z;
          }
#pragma unroll
          for (int j = 0; j < 5 + INL; j++) ok &= (uint32_t)(g8[j] >> 32) == step;
        }
        if (ok) break;
        if ((it & 255) == 0 && timed_out(A, t0)) {
          s_abort = 1;
          break;
        }
        // (MC_ACCUM_POLL_SLEEP: the pause between two polls of a partial, 64-clock units)
        if (A.psleep == 1) __builtin_amdgcn_s_sleep(1);
        else if (A.psleep == 2) __builtin_amdgcn_s_sleep(2);
        else if (A.psleep == 4) __builtin_amdgcn_s_sleep(4);
      }
      if (!s_abort) {
        bv_ = __longlong_as_double((long long)((g8[0] << 32) | (g8[1] & 0xffffffffull)));
        bp_ = (uint32_t)g8[2] == NONE ? NONE64 : (uint64_t)(uint32_t)g8[2];
        cnt_w = (uint32_t)g8[3];
        scan_w = (uint32_t)g8[4];
        // this worker's flagged positions into the step's list: cnt_w slots reserved at once
        const uint32_t slot0 = cnt_w ? atomicAdd(&s_new, cnt_w) : 0u;
        for (uint32_t j = 0; j < cnt_w; j++) {
          const uint32_t p = j < (uint32_t)INL ? (uint32_t)g8[5 + j] : ld32(A.fpos + (uint64_t)wk * A.fcap + j);
          const uint32_t slot = slot0 + j;
          if (mslot) {  // (several ranks: every rank takes the union, below)
            st64x(mslot + (slot < (uint32_t)MBOX_INL ? 5 + slot : MBOX_HDR - MBOX_INL + slot), gran(step, p));
          } else if (slot < PLIST) {
            s_plist[slot] = p;
            if (A.etake) take(M + slot, p, false, (int64_t)slot);  // (MC_ACCUM_EARLY_TAKE)
          } else {  // a list overflow: this thread takes the member itself (past the cache)
            take(M + slot, p, true);
            drain();
          }
        }
      }
    }
    if (prof_on && threadIdx.x == 0) {
      const uint64_t t = now();
      t_wait += t - t_mark;
      t_mark = t;
    }
    // block reduction: the first maximum, the flagged and scanned totals (the wave's largest
    // value by a max reduction; only equal values from several workers need the positions)
    {
      const double m = wave_ext_f64_all<true>(bv_);
      const uint64_t hit = __ballot(bp_ != NONE64 && bv_ == m);
      if (__popcll(hit) > 1) {
        wave_best_all(bv_, bp_, better);
      } else if (hit) {
        const int L = __builtin_ctzll(hit);
        bv_ = __builtin_bit_cast(double, readlane64(__builtin_bit_cast(uint64_t, bv_), L));
        bp_ = readlane64(bp_, L);
      } else {
        bv_ = -1.0;
        bp_ = NONE64;
      }
    }
    const uint32_t wscan = wave_sum32(scan_w), wflag = wave_sum32(cnt_w);
    if (lane == 0) {
      s_bv[wv] = bv_;
      s_bp[wv] = bp_;
      s_red[wv] = wflag;
      s_red[NW + wv] = wscan;
    }
    if (threadIdx.x == 0) s_sumF = 0;
    __syncthreads();
    if (trace && threadIdx.x == 0 && step < TRACE_STEPS) {
      trace[(uint64_t)step * TRACE_W + 7] = now();
      trace[(uint64_t)step * TRACE_W + 9] = nact;
    }
    if (s_abort) {
      if (threadIdx.x == 0) atomicMax((unsigned long long *)&A.out[3], 99ull);
      return;
    }
    // the eight waves' results, one per lane (every wave the same): totals by DPP sums, the
    // first maximum by a max reduction (positions only on equal values)
    uint64_t nflag, nsc;
    double best_val;
    uint64_t best_pos;
    {
      const uint32_t fl = lane < NW ? (uint32_t)s_red[lane] : 0u, sc = lane < NW ? (uint32_t)s_red[NW + lane] : 0u;
      double v = lane < NW ? s_bv[lane] : -1.0;
      uint64_t p = lane < NW ? s_bp[lane] : NONE64;
      nflag = wave_sum32(fl);
      nsc = wave_sum32(sc);
      const double m = wave_ext_f64_all<true>(v);
      const uint64_t hit = __ballot(p != NONE64 && v == m);
      if (__popcll(hit) > 1) {
        wave_best_all(v, p, better);
        best_val = v;
        best_pos = p;
      } else if (hit) {
        const int L = __builtin_ctzll(hit);
        best_val = __builtin_bit_cast(double, readlane64(__builtin_bit_cast(uint64_t, v), L));
        best_pos = readlane64(p, L);
      } else {
        best_val = -1.0;
        best_pos = NONE64;
      }
    }
    if (mslot) {
      // ---- the ranks' exchange: publish this rank's header, take every rank's ----------
      // get_close over the union is the serial loop's: is_min = nothing flagged anywhere, the
      // result the first maximum by (value, static position), every flagged candidate joins
      if (threadIdx.x >= BK && threadIdx.x < BK + MBOX_HDR) {  // (not wave 0, see BK)
        const uint64_t vb = (uint64_t)__double_as_longlong(best_val);
        const int j = threadIdx.x - BK;
        const uint32_t data = j == 0   ? (uint32_t)(vb >> 32)
                              : j == 1 ? (uint32_t)vb
                              : j == 2 ? (best_pos == NONE64 ? NONE : (uint32_t)best_pos)
                              : j == 3 ? (uint32_t)nflag
                              : j == 4 ? (uint32_t)nsc
                                       : NONE;
        // (inline slots of this rank's flagged positions were written while collecting)
        if (j < 5 || (uint64_t)(j - 5) >= nflag) st64x(mslot + j, gran(step, data));
      }
      uint64_t *mbase = A.mbox + (uint64_t)(step & 1) * A.W * A.slot_g;
      if (threadIdx.x < A.W) {  // thread r reads rank r's header (W <= 64: wave 0)
        const uint64_t *h = mbase + (uint64_t)threadIdx.x * A.slot_g;
        const uint64_t t0 = now();
        uint64_t g[MBOX_HDR];
        for (uint32_t it = 1;; it++) {
          bool ok = true;
#pragma unroll
          for (int j = 0; j < MBOX_HDR; j++) {
            g[j] = ld64x(h + j);
            ok &= (uint32_t)(g[j] >> 32) == step;
          }
          if (ok) break;
          if ((it & 63) == 0 && timed_out(A, t0)) {
            s_abort = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        s_xv[threadIdx.x] = __longlong_as_double((long long)((g[0] << 32) | (g[1] & 0xffffffffull)));
        s_xp[threadIdx.x] = (uint32_t)g[2] == NONE ? NONE64 : (uint64_t)(uint32_t)g[2];
        s_xn[threadIdx.x] = (uint32_t)g[3];
        s_xs[threadIdx.x] = (uint32_t)g[4];
#pragma unroll
        for (int j = 0; j < MBOX_INL; j++) s_xi[threadIdx.x][j] = (uint32_t)g[5 + j];
      }
      __syncthreads();
      if (s_abort) {
        if (threadIdx.x == 0) atomicMax((unsigned long long *)&A.out[3], 99ull);
        return;
      }
      nflag = 0;
      nsc = 0;
      best_val = -1.0;
      best_pos = NONE64;
      for (uint32_t r = 0; r < A.W; r++) {
        nflag += s_xn[r];
        nsc += s_xs[r];
        if (s_xp[r] != NONE64 && better(s_xv[r], s_xp[r], best_val, best_pos)) {
          best_val = s_xv[r];
          best_pos = s_xp[r];
        }
      }
      // the union of the flagged positions: list entry i is rank r's entry i - (earlier ranks')
      for (uint64_t i = threadIdx.x; i < nflag; i += NT) {
        uint32_t r = 0;
        uint64_t j = i;
        while (j >= s_xn[r]) j -= s_xn[r++];
        const uint64_t *e = mbase + (uint64_t)r * A.slot_g + MBOX_HDR - MBOX_INL + j;
        const uint64_t t0 = now();
        uint64_t g = j < (uint64_t)MBOX_INL ? gran(step, s_xi[r][j]) : ld64x(e);
        for (uint32_t it = 1; (uint32_t)(g >> 32) != step; it++) {
          if ((it & 63) == 0 && timed_out(A, t0)) {
            s_abort = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          g = ld64x(e);
        }
        if (i < PLIST) {
          s_plist[i] = (uint32_t)g;
        } else {
          take(M + i, (uint32_t)g, true);
          drain();
        }
      }
      __syncthreads();
      if (s_abort) {
        if (threadIdx.x == 0) atomicMax((unsigned long long *)&A.out[3], 99ull);
        return;
      }
    }
    ncand += nsc;
    uint64_t tq = 0;
    if (prof_on && threadIdx.x == 0) {
      tq = now();
      t_sub[0] += tq - t_mark;
    }
    if (nflag > 0) {
      // remove_available: the new members, one thread each, all their loads in flight at once
      // (member i on thread i + 64: wave 0, which publishes the next record, keeps no
      // outstanding stores for that record's drain to wait on)
      if (!A.etake || mslot)
        for (uint64_t i = (threadIdx.x + NT - 64) % NT; i < nflag && i < PLIST; i += NT)
          take(M + i, s_plist[i], false, (int64_t)i);
      npend = nflag < PLIST ? (uint32_t)nflag : PLIST;
      if (M + nflag > A.mrow) drain();  // members past the cache are read back from mem_pos / mkeys
      __syncthreads();
      if (prof_on && threadIdx.x == 0) t_ws[3] += now() - tq;  // (the takes, inside "column sums")
      // column sums of the cached new members: thread (word w of a row, member slice sl) adds
      // up its 32-bit word over the slice's members, then one LDS atomic per bin and thread
      const uint64_t q0 = M, q1 = M + nflag < A.mrow ? M + nflag : (uint64_t)A.mrow;
      const uint32_t nlist = nflag < PLIST ? (uint32_t)nflag : PLIST;
      M += nflag;
      if constexpr (WIDE) {
        // column sums of the listed new members straight from `hr`: thread (chunk c, member
        // slice sl) adds its 16-byte chunk over the slice's members (independent loads), then one
        // LDS atomic per bin and thread
        constexpr int per = 16 / (int)sizeof(T);
        const int nsl = nch >= NT ? 1 : NT / nch;
        for (int t = threadIdx.x; t < nch * nsl; t += NT) {
          const int c = t % nch, sl = t / nch;
          uint32_t sum[per];
#pragma unroll
          for (int e = 0; e < per; e++) sum[e] = 0;
          // (eight members' chunks in flight per thread: the loads are independent)
          uint32_t i = (uint32_t)sl;
          for (; i + 7u * (uint32_t)nsl < nlist; i += 8u * (uint32_t)nsl) {
            uint4 v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = A.hr[(uint64_t)s_plist[i + (uint32_t)u * (uint32_t)nsl] * nch + c];
#pragma unroll
            for (int u = 0; u < 8; u++) {
              const T *pv = reinterpret_cast<const T *>(&v[u]);
#pragma unroll
              for (int e = 0; e < per; e++) sum[e] += pv[e];
            }
          }
          for (; i < nlist; i += (uint32_t)nsl) {
            const uint4 v = A.hr[(uint64_t)s_plist[i] * nch + c];
            const T *pv = reinterpret_cast<const T *>(&v);
#pragma unroll
            for (int e = 0; e < per; e++) sum[e] += pv[e];
          }
#pragma unroll
          for (int e = 0; e < per; e++)
            if (sum[e] && c * per + e < A.B) atomicAdd((unsigned long long *)&msum[c * per + e], (unsigned long long)sum[e]);
        }
      } else {
        constexpr int per = 4 / (int)sizeof(T);  // bins per 32-bit word
        const int wpr = (A.B + per - 1) / per;
        const int nsl = wpr >= NT ? 1 : NT / wpr;
        for (int t = threadIdx.x; t < wpr * nsl; t += NT) {
          const int wd = t % wpr, sl = t / wpr;
          uint32_t sum[per];
#pragma unroll
          for (int e = 0; e < per; e++) sum[e] = 0;
          for (uint64_t q = q0 + (uint64_t)sl; q < q1; q += (uint64_t)nsl) {
            const uint32_t x = reinterpret_cast<const uint32_t *>(mc.row + q * mc.rp)[wd];
#pragma unroll
            for (int e = 0; e < per; e++) sum[e] += sizeof(T) == 1 ? (x >> (8 * e)) & 0xffu : (x >> (16 * e)) & 0xffffu;
          }
#pragma unroll
          for (int e = 0; e < per; e++)
            if (sum[e] && wd * per + e < A.B) atomicAdd((unsigned long long *)&msum[wd * per + e], (unsigned long long)sum[e]);
        }
      }
      __syncthreads();
      if (prof_on && threadIdx.x == 0) {
        const uint64_t t = now();
        t_sub[1] += t - tq;
        tq = t;
      }
      // the integer mean F_b = floor(S_b / M) and its total (features.hpp: get_mean as a SAD
      // reduction)
      uint64_t part = 0;
      for (int b = threadIdx.x; b < A.B; b += NT) {
        const uint64_t sb = msum[b];
        const uint64_t F = (sb >> 32) == 0 ? (uint64_t)((uint32_t)sb / (uint32_t)M) : sb / M;
        reinterpret_cast<T *>(Fl)[b] = (T)F;
        part += F;
      }
      part = wave_sum64_all(part);
      if (lane == 0 && part) atomicAdd((unsigned long long *)&s_sumF, (unsigned long long)part);
      __syncthreads();
      if (prof_on && threadIdx.x == 0) {
        const uint64_t t = now();
        t_sub[2] += t - tq;
        tq = t;
      }
      // Trainer::closest: first minimum of distance_d over the members (ties by key)
      const uint64_t sumF = s_sumF;
      const uint4 *F4 = reinterpret_cast<const uint4 *>(Fl);
      double bd = __builtin_inf();
      uint64_t bk = NONE64, bq = 0;
      if constexpr (WIDE) {
        // one member per wave (rows from `hr`, 64 lanes over the row): every lane ends with
        // the wave's first minimum
        auto member_row = [&](uint64_t q) -> const uint4 * {
          const uint32_t r = q < A.mrow ? lds_u32(mc.pos + q) : ld32(A.mem_pos + cl_start + q);
          return A.hr + (uint64_t)r * nch;
        };
        auto score = [&](uint64_t q, Acc<T> &acc) {
          const uint64_t mp = q < A.mrow ? lds_u64(mc.info + q * 3) : A.mag_s[ld32(A.mem_pos + cl_start + q)];
          const uint64_t key = q < A.mrow ? lds_u64(mc.key + q) : ld64(A.mkeys + cl_start + q);
          const PS s = acc.finish(mp, sumF);
          const double frac = (double)(2 * s.smin) / (double)(mp + sumF);
          const double d = __builtin_fma(-frac, frac, 1.0) * 10000.0;
          if (d < bd || (d == bd && key < bk)) {
            bd = d;
            bk = key;
            bq = q;
          }
        };
        if (nch <= 256) {
          // at most four chunks per lane: the next member's row is loaded while this one is
          // reduced (two members in flight per wave; a past-the-end load re-reads a valid row,
          // so every trip issues the same loads)
          auto load = [&](uint64_t q, uint4 (&v)[4]) {
            const uint4 *row = member_row(q < M ? q : (uint64_t)wv);
#pragma unroll
            for (int u = 0; u < 4; u++) {
              const int c = lane + 64 * u;
              v[u] = row[c < nch ? c : nch - 1];
            }
          };
          auto reduce = [&](uint64_t q, const uint4 (&v)[4]) {
            Acc<T> acc;
#pragma unroll
            for (int u = 0; u < 4; u++) {
              const int c = lane + 64 * u;
              if (c < nch) acc.add_sad(v[u], F4[c]);
            }
            acc.wave_reduce();
            score(q, acc);
          };
          uint4 va[4], vb[4];
          uint64_t q = wv;
          if (q < M) {
            load(q, va);
            for (;;) {
              load(q + NW, vb);
              reduce(q, va);
              q += NW;
              if (q >= M) break;
              load(q + NW, va);
              reduce(q, vb);
              q += NW;
              if (q >= M) break;
            }
          }
        } else {
          for (uint64_t q = wv; q < M; q += NW) {
            const uint4 *row = member_row(q);
            Acc<T> acc;
            int c = lane;
            for (; c + 192 < nch; c += 256) {
              const uint4 v0 = row[c], v1 = row[c + 64], v2 = row[c + 128], v3 = row[c + 192];
              acc.add_sad(v0, F4[c]);
              acc.add_sad(v1, F4[c + 64]);
              acc.add_sad(v2, F4[c + 128]);
              acc.add_sad(v3, F4[c + 192]);
            }
            for (; c < nch; c += 64) acc.add_sad(row[c], F4[c]);
            acc.wave_reduce();
            score(q, acc);
          }
        }
      } else if (NCH > 0 && NC % 4 == 0 && sizeof(T) == 1 && (A.dbg & 2)) {
        // a quad of lanes per member, a quarter of the row each, SAD only (distance_d needs
        // sum |p - F| and the magnitudes): a quarter of the dependent LDS reads per lane
        constexpr int CPL = NC >= 4 ? NC / 4 : 1;
        const int sub = threadIdx.x & 3;
        for (uint64_t q = threadIdx.x >> 2; q < M; q += NT / 4) {
          uint32_t s4[CPL];
          if (q < A.mrow) {
            const uint4 *row = mc.row + q * mc.rp + sub * CPL;
            uint4 rv[CPL], fv[CPL];
#pragma unroll
            for (int k = 0; k < CPL; k++) {
              rv[k] = row[k];
              fv[k] = F4[sub * CPL + k];
            }
#pragma unroll
            for (int k = 0; k < CPL; k++) {
              s4[k] = __builtin_amdgcn_sad_u8(rv[k].x, fv[k].x, 0u);
              s4[k] = __builtin_amdgcn_sad_u8(rv[k].y, fv[k].y, s4[k]);
              s4[k] = __builtin_amdgcn_sad_u8(rv[k].z, fv[k].z, s4[k]);
              s4[k] = __builtin_amdgcn_sad_u8(rv[k].w, fv[k].w, s4[k]);
            }
          } else {
            const uint64_t r = ld32(A.mem_pos + cl_start + q);
#pragma unroll
            for (int k = 0; k < CPL; k++) {
              const uint4 a = A.hr[r * nch + sub * CPL + k], f = F4[sub * CPL + k];
              s4[k] = __builtin_amdgcn_sad_u8(a.x, f.x, 0u);
              s4[k] = __builtin_amdgcn_sad_u8(a.y, f.y, s4[k]);
              s4[k] = __builtin_amdgcn_sad_u8(a.z, f.z, s4[k]);
              s4[k] = __builtin_amdgcn_sad_u8(a.w, f.w, s4[k]);
            }
          }
          uint32_t sad = 0;
#pragma unroll
          for (int k = 0; k < CPL; k++) sad += s4[k];
          sad += dpp_mv<0xB1>(0u, sad);  // quad_perm [1,0,3,2]
          sad += dpp_mv<0x4E>(0u, sad);  // quad_perm [2,3,0,1]: every lane of the quad has the sum
          if (sub == 0) {
            const uint64_t mp = q < A.mrow ? lds_u64(mc.info + q * 3) : A.mag_s[ld32(A.mem_pos + cl_start + q)];
            const uint64_t key = q < A.mrow ? lds_u64(mc.key + q) : ld64(A.mkeys + cl_start + q);
            const uint64_t smin = (mp + sumF - sad) >> 1;
            const double frac = (double)(2 * smin) / (double)(mp + sumF);
            const double d = __builtin_fma(-frac, frac, 1.0) * 10000.0;
            if (d < bd || (d == bd && key < bk)) {
              bd = d;
              bk = key;
              bq = q;
            }
          }
        }
      } else
      for (uint64_t q = threadIdx.x; q < M; q += NT) {
        Acc<T> acc;
        uint64_t mp, key;
        if (q < A.mrow) {
          const uint4 *row = mc.row + q * mc.rp;
          if constexpr (NCH > 0) {  // half a row of LDS reads in flight per wait
            constexpr int HB = NC >= 8 ? 8 : NC;
#pragma unroll
            for (int k0 = 0; k0 < NC; k0 += HB) {
              uint4 rv[HB], fv[HB];
#pragma unroll
              for (int k = 0; k < HB; k++) {
                rv[k] = row[k0 + k];
                fv[k] = F4[k0 + k];
              }
#pragma unroll
              for (int k = 0; k < HB; k++) acc.add_sad(rv[k], fv[k]);  // (distance_d needs no dot product)
            }
          } else {
            for (int k = 0; k < nch; k++) acc.add_sad(row[k], F4[k]);
          }
          mp = mc.info[q * 3];
          key = mc.key[q];
        } else {
          const uint64_t r = ld32(A.mem_pos + cl_start + q);
          for (int k = 0; k < nch; k++) acc.add_sad(A.hr[r * nch + k], F4[k]);
          mp = A.mag_s[r];
          key = ld64(A.mkeys + cl_start + q);
        }
        const PS s = acc.finish(mp, sumF);
        const double frac = (double)(2 * s.smin) / (double)(mp + sumF);
        const double d = __builtin_fma(-frac, frac, 1.0) * 10000.0;
        if (d < bd || (d == bd && key < bk)) {
          bd = d;
          bk = key;
          bq = q;
        }
      }
      uint64_t tc0 = 0;
      if (prof_on && threadIdx.x == 0) {
        tc0 = now();
        t_cl[0] += tc0 - tq;
      }
      {  // first minimum by (distance, key); keys are unique, so the lane holding it gives q.
         // The wave's smallest distance by a min reduction; only a tie between lanes needs the
         // (distance, key) pair reduction
        const double md = wave_ext_f64_all<false>(bd);
        uint64_t hit = __ballot(bk != NONE64 && bd == md);
        double rd = md;
        uint64_t rk = NONE64;
        if (__popcll(hit) > 1) {
          rd = bd;
          rk = bk;
          wave_best_all(rd, rk, [](double a, uint64_t ka, double b, uint64_t kb) { return a < b || (a == b && ka < kb); });
          hit = __ballot(bd == rd && bk == rk);
        }
        const int L = hit ? __builtin_ctzll(hit) : 0;
        if (hit) rk = readlane64(bk, L);
        bq = readlane64(bq, L);
        bd = hit ? rd : __builtin_inf();
        bk = rk;
      }
      if (lane == 0) {
        s_bv[wv] = bd;
        s_red[2 * NW + wv] = bk;
        s_bp[wv] = bq;
      }
      __syncthreads();
      uint64_t tc1 = 0;
      if (prof_on && threadIdx.x == 0) {
        tc1 = now();
        t_cl[1] += tc1 - tc0;
      }
      // the eight waves' minima, one per lane (every wave the same): the smallest distance by a
      // min reduction, the smallest key among equal distances (keys are unique)
      uint64_t win;
      {
        const double dd = lane < NW ? s_bv[lane] : __builtin_inf();
        const uint64_t kk = lane < NW ? s_red[2 * NW + lane] : NONE64;
        const uint64_t pp = lane < NW ? s_bp[lane] : 0;
        const double md = wave_ext_f64_all<false>(dd);
        uint64_t hit = __ballot(kk != NONE64 && dd == md);
        int L = hit ? __builtin_ctzll(hit) : 0;
        if (__popcll(hit) > 1) {
          uint64_t bestk = NONE64;
          for (uint64_t m = hit; m; m &= m - 1) {
            const int l = __builtin_ctzll(m);
            const uint64_t kl = readlane64(kk, l);
            if (kl < bestk) {
              bestk = kl;
              L = l;
            }
          }
        }
        win = readlane64(pp, L);
      }
      last_q = (uint32_t)win;
      if (win < A.mrow) last = lds_u32(mc.pos + win);  // (uniform branch: no global load on the cached path)
      else last = ld32(A.mem_pos + cl_start + win);
      // (no barrier: s_bv / s_bp / s_red / s_new are next written in the next step's fan-in,
      // after the barrier that ends this step's deferred bvec kills -- npend > 0 here)
      if (threadIdx.x == 0) s_new = 0;
      if (prof_on && threadIdx.x == 0) {
        const uint64_t t = now();
        t_sub[3] += t - tq;
        t_cl[2] += t - tc1;
      }
    } else if (best_pos != NONE64) {
      // is_min with a result: the best candidate seeds the next cluster (bvec::erase)
      finish_cluster();
      last = (uint32_t)best_pos;
      // (thin: its record goes out now, ahead of the seed's loads -- when the last record's span
      // was every position, so the workers score no more than they did)
      thin_out = A.thin && s_span_all;
      if (thin_out) {
        log_kill(best_pos);
        kn++;
        step++;
        if (wv == 0) publish_thin((uint32_t)best_pos);
      }
      new_cluster(best_pos, true, thin_out);
    } else {
      const uint64_t p = pop();
      finish_cluster();
      last = p == NONE64 ? NONE : (uint32_t)p;
      if (p != NONE64) new_cluster(p);
    }
    if (prof_on && threadIdx.x == 0) {
      const uint64_t t = now();
      t_coll += t - t_mark;
      if (trace && step < TRACE_STEPS) trace[(uint64_t)step * TRACE_W + 8] = t;
    }
  }
  if (threadIdx.x == 0) {
    A.out[0] = ncl;
    A.out[1] = nsteps;
    A.out[2] = ncand;
    if (err) atomicMax((unsigned long long *)&A.out[3], (unsigned long long)err);
    A.out[4] = cl_start;
    A.out[5] = t_ws[0] + t_ws[1] + t_ws[2];
    A.out[6] = t_wait;
    A.out[7] = t_coll;
    for (int i = 0; i < 4; i++) A.out[8 + i] = t_sub[i];
    for (int i = 0; i < 4; i++) A.out[12 + i] = t_ws[i];
    for (int i = 0; i < 3; i++) A.out[18 + i] = t_cl[i];
    for (int i = 0; i < 2; i++) A.out[21 + i] = t_pub[i];
    for (int i = 0; i < 5; i++) A.out[23 + i] = t_wk[i];
    if (prof_on) {
      A.out[16] = __builtin_amdgcn_s_memtime() - clk0;
      A.out[17] = now() - rt0;
    }
  }
}

// NCH: compile-time chunks per row (0: A.nch at run time).
// CPT: streaming rows with per-chunk compaction (A.cc; the resident form compiled out)
// DENSE: dense resident workers (worker_dense, DT-position tiles)
// DSTREAM: dense streaming workers (worker_dstream, DT-position tiles, rows in HBM)
template <typename T, int NCH, bool WIDE = false, bool CPT = false, bool DENSE = false, bool DSTREAM = false, bool PROF = false>
__global__ __launch_bounds__(NT) void accum_kernel(AccArgs A, DevClassifier C) {
  extern __shared__ __attribute__((aligned(16))) uint4 dyn[];
  constexpr int TSZ = (DENSE || DSTREAM) ? DT : WIDE ? NW : NT;
  if (blockIdx.x == 0) controller<T, NCH, WIDE, TSZ, PROF>(A, dyn);
  else if constexpr (DENSE) worker_dense<T, NCH, PROF>(A, C, dyn);
  else if constexpr (DSTREAM) worker_dstream<T, NCH>(A, C, dyn);
  else worker<T, NCH, WIDE, CPT, PROF>(A, C, dyn);
}

}  // namespace

}  // namespace mcg
