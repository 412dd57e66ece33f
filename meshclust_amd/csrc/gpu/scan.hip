// scan.hip -- the accumulation step (ClusterFactory::accumulate, ClusterFactory.cpp:637-714) as
// ONE launch for 8/16-bit histograms:
//
//   Trainer::get_close (Trainer.cpp:34-114)      every workgroup: one lane per candidate
//   bvec::remove_available (bvec.cpp:289-318)    similar candidates killed + appended
//   get_mean (ClusterFactory.cpp:382-425)        last workgroup (arrival ticket): integer mean
//                                                 + first-closest member via SAD
//   result hand-off                              last workgroup writes the step result and
//                                                 the flagged positions straight into pinned
//                                                 host memory and publishes a sequence number
//
// Layout: for the scan the histograms are re-laid "chunk-major" in static bvec order,
// hs[c * npad + pos] = 16-byte chunk c of the candidate at static position pos, so a
// window [S, E] is read as nch perfectly coalesced 1 KiB-per-wave streams and each lane
// accumulates its own candidate's SAD/dot in registers (no cross-lane reduction).  The
// centre row sits in LDS and is read as a broadcast.
#include <cstdio>
#include <cstring>
#include <vector>

#include "features.hpp"

namespace mcg {

namespace {

constexpr int ST = 256;
static_assert(ST == MC_SHARD_BLOCK, "a sharded step scans whole MC_SHARD_BLOCK blocks, one workgroup each");

template <typename T>
__global__ __launch_bounds__(ST) void build_static_kernel(const uint8_t *__restrict__ hist, uint64_t pitch,
                                                          const uint32_t *__restrict__ order, uint64_t n, int nch,
                                                          uint4 *__restrict__ hs, uint64_t npad,
                                                          const uint64_t *__restrict__ mag,
                                                          const uint64_t *__restrict__ sumsq,
                                                          const uint64_t *__restrict__ len, uint64_t *__restrict__ mag_s,
                                                          uint64_t *__restrict__ sumsq_s, uint64_t *__restrict__ len_s) {
  for (uint64_t pos = (uint64_t)blockIdx.x * ST + threadIdx.x; pos < n; pos += (uint64_t)gridDim.x * ST) {
    const uint32_t id = order[pos];
    const uint4 *row = reinterpret_cast<const uint4 *>(hist + (uint64_t)id * pitch);
    for (int c = 0; c < nch; c++) hs[(uint64_t)c * npad + pos] = row[c];
    mag_s[pos] = mag[id];
    sumsq_s[pos] = sumsq[id];
    len_s[pos] = len[id];
  }
}

struct FusedArgs {
  const uint4 *hs;
  uint64_t npad;
  int nch, B;
  const uint64_t *mag_s, *sumsq_s, *len_s;
  const uint32_t *order;
  uint8_t *alive;
  const uint8_t *hist;  // id-major rows (centre)
  uint64_t pitch;
  const uint64_t *mag, *sumsq, *len;
  uint32_t centre;
  uint64_t S, E;
  uint64_t kills[8];
  int nkill;
  int new_cluster;
  uint64_t first_pos;
  uint32_t step;
  ScanPartial *partials;
  uint32_t *ticket;
  ScanDev *sd;
  uint32_t *flags_dev;
  uint32_t *mem_pos;
  uint64_t *mkeys;
  uint64_t *msum;
  HostScan *hres;
  uint32_t seq;
  uint64_t *stamps;  // diagnostic build only (MC_STAMPS): s_memrealtime at phase boundaries
  const double *ident;  // alignment mode: NW identity per static position (else null)
  // workgroup w scans static positions pos0 + w * pstride + [0, ST) (clipped to [S, E]):
  // pos0 = S, pstride = ST for a whole window; one rank's blocks of a sharded window otherwise
  uint64_t pos0, pstride;
  int part;  // sharded step (mc_scan_part): find and report only, the commit kernel applies
};

// mc_scan_commit: remove_available + get_mean of a sharded step, on the union of the ranks'
// flagged positions (ascending static positions in flags_dev[0, nflag)).
struct CommitArgs {
  const uint4 *hs;
  uint64_t npad;
  int nch, B;
  const uint64_t *mag_s;
  const uint32_t *order;
  uint8_t *alive;
  const uint32_t *flags_dev;
  uint32_t nflag;
  int new_cluster;
  uint64_t first_pos;
  uint32_t step;
  ScanDev *sd;
  uint32_t *mem_pos;
  uint64_t *mkeys;
  uint64_t *msum;
  HostScan *hres;
  uint32_t seq;
};

#ifdef MC_STAMPS
#define STAMP(i)                                                                       \
  do {                                                                                 \
    if (threadIdx.x == 0) atomicMax((unsigned long long *)&A.stamps[i], __builtin_amdgcn_s_memrealtime()); \
  } while (0)
#define STAMP_MIN(i)                                                                   \
  do {                                                                                 \
    if (threadIdx.x == 0) atomicMin((unsigned long long *)&A.stamps[i], __builtin_amdgcn_s_memrealtime()); \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#define STAMP_MIN(i) \
  do {               \
  } while (0)
#endif

__device__ __forceinline__ bool better(double v, uint64_t p, double bv, uint64_t bp) {
  return v > bv || (v == bv && p < bp);
}

// GS: the cluster's column sums in global memory (B > 4096) -- a compile-time choice, so the
// LDS sums are not FLAT accesses
template <typename T, bool GS>
__global__ __launch_bounds__(ST) void fused_scan_kernel(FusedArgs A, DevClassifier C) {
  extern __shared__ __attribute__((aligned(16))) uint4 dyn[];
  uint4 *clds = dyn;          // centre chunks
  uint4 *Fl = dyn + A.nch;    // packed integer mean (last workgroup)
  __shared__ double rv[ST / 64];
  __shared__ uint64_t rp[ST / 64];
  __shared__ int s_last;
  STAMP_MIN(0);
  for (int c = threadIdx.x; c < A.nch; c += ST)
    clds[c] = reinterpret_cast<const uint4 *>(A.hist + (uint64_t)A.centre * A.pitch)[c];
  __syncthreads();
  const PInfo pc{A.mag[A.centre], A.sumsq[A.centre], A.len[A.centre]};
  const uint32_t mbase = A.new_cluster ? 1u : A.sd->nmembers;
  const uint64_t pos = A.pos0 + (uint64_t)blockIdx.x * A.pstride + threadIdx.x;
  bool valid = pos >= A.S && pos <= A.E && A.alive[pos];
  for (int i = 0; i < A.nkill; i++) valid = valid && pos != A.kills[i];
  double best_v = -1.0;  // get_close's initializer (NULL, -1, 0, 0) with a strict `>`
  uint64_t best_p = ~0ull;
  if (valid) {
    double raw[MC_MAX_SINGLE];
    if (A.ident) {  // alignment mode: Feature::align(*pt, *p) computed by the NW kernel
      raw[0] = A.ident[pos];
#pragma unroll
      for (int i = 1; i < MC_MAX_SINGLE; i++) raw[i] = 0.0;
    } else {
      Acc<T> acc;
      const uint4 *col = A.hs + pos;
      if (A.nch == 16) {
        uint4 v[16];
#pragma unroll
        for (int c = 0; c < 16; c++) v[c] = col[(uint64_t)c * A.npad];
#pragma unroll
        for (int c = 0; c < 16; c++) acc.add(v[c], clds[c]);
      } else {
#pragma unroll 8
        for (int c = 0; c < A.nch; c++) acc.add(col[(uint64_t)c * A.npad], clds[c]);
      }
      const PInfo pi{A.mag_s[pos], A.sumsq_s[pos], A.len_s[pos]};
      const PS s = acc.finish(pi.mag, pc.mag);
#pragma unroll
      for (int i = 0; i < MC_MAX_SINGLE; i++)
        raw[i] = i < C.c.n_single ? raw_fast(C.c.lookup[i], s, pi, pc, A.B) : 0.0;  // compute(*pt, *p)
    }
    double c0;
    const int d = classify_raw(C, raw, &c0, nullptr);
    if (c0 > -1.0) {  // NaN never qualifies
      best_v = c0;
      best_p = pos;
    }
    if (d) {
      const uint32_t slot = atomicAdd(&A.sd->nflag, 1u);
      A.flags_dev[slot] = (uint32_t)pos;
      if (!A.part) {
        A.alive[pos] = 0;
        A.mem_pos[mbase + slot] = (uint32_t)pos;
        A.mkeys[mbase + slot] = ((uint64_t)A.step << 32) | pos;
      }
    }
  }
  // workgroup first-max of combo 0
  for (int o = 32; o >= 1; o >>= 1) {
    double ov = __shfl_xor(best_v, o, 64);
    uint64_t op = shfl_xor64(best_p, o);
    if (better(ov, op, best_v, best_p)) {
      best_v = ov;
      best_p = op;
    }
  }
  if ((threadIdx.x & 63) == 0) {
    rv[threadIdx.x >> 6] = best_v;
    rp[threadIdx.x >> 6] = best_p;
  }
  __syncthreads();  // also drains every wave's stores before the release below
  STAMP(1);
  if (threadIdx.x == 0) {
    double v = rv[0];
    uint64_t p = rp[0];
    for (int i = 1; i < ST / 64; i++)
      if (better(rv[i], rp[i], v, p)) {
        v = rv[i];
        p = rp[i];
      }
    A.partials[blockIdx.x] = ScanPartial{v, p, p != ~0ull ? 1 : 0, 0};
    // publish this workgroup's stores, then take an arrival ticket (Guideline 16 form)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t t = __hip_atomic_fetch_add(A.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = t == gridDim.x - 1;
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!s_last) return;
  STAMP(2);

  // ---------------- last workgroup: get_close's reduction + get_mean -------------------
  double bv = -1.0;
  uint64_t bp = ~0ull;
  for (uint32_t i = threadIdx.x; i < gridDim.x; i += ST) {
    const ScanPartial q = A.partials[i];
    if (q.has && better(q.val, q.pos, bv, bp)) {
      bv = q.val;
      bp = q.pos;
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
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    rv[threadIdx.x >> 6] = bv;
    rp[threadIdx.x >> 6] = bp;
  }
  __syncthreads();
  STAMP(3);
  const uint32_t nflag = __hip_atomic_load(&A.sd->nflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t M = A.part ? A.sd->nmembers : mbase + nflag;
  uint32_t new_id = 0xffffffffu;
  if (nflag > 0 && !A.part) {
    if (A.new_cluster) {
      if (threadIdx.x == 0) {
        A.mem_pos[0] = (uint32_t)A.first_pos;
        A.mkeys[0] = 0;
      }
    }
    const RowRef R{A.hs, 1, A.npad};
    // integer column sums of the cluster: running sum from the previous step (or the new
    // cluster's first member) + this step's flagged members, folded in LDS
    uint64_t *lsum;
    if constexpr (GS) lsum = A.msum;
    else lsum = reinterpret_cast<uint64_t *>(Fl + A.nch);
    for (int b = threadIdx.x; b < A.B; b += ST) lsum[b] = A.new_cluster ? elem<T>(R, A.first_pos, b) : A.msum[b];
    __syncthreads();
    add_rows<T, ST>(R, A.flags_dev, nflag, A.nch, lsum);
    __syncthreads();
    if constexpr (!GS)
      for (int b = threadIdx.x; b < A.B; b += ST) A.msum[b] = lsum[b];
    STAMP(4);
    const uint64_t win = mean_closest_fast<T, ST>(R, A.mem_pos, A.mkeys, M, A.mag_s, A.B, A.nch, lsum, Fl);
    STAMP(5);
    new_id = A.order[win];
  }
  if (threadIdx.x == 0) {
    double v = rv[0];
    uint64_t p = rp[0];
    for (int i = 1; i < ST / 64; i++)
      if (better(rv[i], rp[i], v, p)) {
        v = rv[i];
        p = rp[i];
      }
    if (!A.part) A.sd->nmembers = M;
    A.sd->nflag = 0;
    for (int i = 0; i < A.nkill; i++) A.alive[A.kills[i]] = 0;
    HostScan *h = A.hres;
    h->r.is_min = nflag == 0;
    h->r.has_best = p != ~0ull;
    h->r.best_pos = p;
    h->r.best_val = v;
    h->r.n_flagged = nflag;
    h->r.new_centre = new_id;
    h->r.n_members = M;
    *A.ticket = 0;
  }
  for (uint32_t q = threadIdx.x; q < nflag; q += ST) A.hres->flags[q] = A.flags_dev[q];
  __syncthreads();
  STAMP(6);
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(&A.hres->seq, A.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <typename T, bool GS>
__global__ __launch_bounds__(ST) void commit_kernel(CommitArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint4 dyn[];
  uint4 *Fl = dyn;  // packed integer mean
  const uint32_t mbase = A.new_cluster ? 1u : A.sd->nmembers;
  const uint32_t M = mbase + A.nflag;
  for (uint32_t q = threadIdx.x; q < A.nflag; q += ST) {
    const uint32_t pos = A.flags_dev[q];
    A.alive[pos] = 0;
    A.mem_pos[mbase + q] = pos;
    A.mkeys[mbase + q] = ((uint64_t)A.step << 32) | pos;
  }
  if (A.new_cluster && threadIdx.x == 0) {
    A.mem_pos[0] = (uint32_t)A.first_pos;
    A.mkeys[0] = 0;
  }
  __syncthreads();
  uint32_t new_id = 0xffffffffu;
  if (A.nflag > 0) {  // the same running integer sums + closest member as fused_scan_kernel
    const RowRef R{A.hs, 1, A.npad};
    uint64_t *lsum;
    if constexpr (GS) lsum = A.msum;
    else lsum = reinterpret_cast<uint64_t *>(Fl + A.nch);
    for (int b = threadIdx.x; b < A.B; b += ST) lsum[b] = A.new_cluster ? elem<T>(R, A.first_pos, b) : A.msum[b];
    __syncthreads();
    add_rows<T, ST>(R, A.flags_dev, A.nflag, A.nch, lsum);
    __syncthreads();
    if constexpr (!GS)
      for (int b = threadIdx.x; b < A.B; b += ST) A.msum[b] = lsum[b];
    const uint64_t win = mean_closest_fast<T, ST>(R, A.mem_pos, A.mkeys, M, A.mag_s, A.B, A.nch, lsum, Fl);
    new_id = A.order[win];
  }
  if (threadIdx.x == 0) {
    A.sd->nmembers = M;
    HostScan *h = A.hres;
    h->r.is_min = A.nflag == 0;
    h->r.n_flagged = A.nflag;
    h->r.new_centre = new_id;
    h->r.n_members = M;
    __threadfence_system();
    __hip_atomic_store(&A.hres->seq, A.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace

int build_static(mc_ctx *c) {
  const int nch = (int)((c->B * c->width + 15) / 16);
  c->npad = (c->norder + 63) / 64 * 64;
  if (ensure(c->hs, (size_t)nch * c->npad * 16) || ensure(c->mag_s, c->npad * 8) || ensure(c->sumsq_s, c->npad * 8) ||
      ensure(c->len_s, c->npad * 8))
    return MC_ERR_OOM;
  const int grid = (int)std::min<uint64_t>((c->norder + ST - 1) / ST, 4096);
  timed_begin(c);
  switch (c->width) {
    case 1:
      build_static_kernel<uint8_t><<<grid, ST, 0, c->stream>>>(
          (const uint8_t *)c->hist.p, c->pitch, (const uint32_t *)c->order.p, c->norder, nch, (uint4 *)c->hs.p, c->npad,
          (const uint64_t *)c->mag.p, (const uint64_t *)c->sumsq.p, (const uint64_t *)c->len.p, (uint64_t *)c->mag_s.p,
          (uint64_t *)c->sumsq_s.p, (uint64_t *)c->len_s.p);
      break;
    default:
      build_static_kernel<uint16_t><<<grid, ST, 0, c->stream>>>(
          (const uint8_t *)c->hist.p, c->pitch, (const uint32_t *)c->order.p, c->norder, nch, (uint4 *)c->hs.p, c->npad,
          (const uint64_t *)c->mag.p, (const uint64_t *)c->sumsq.p, (const uint64_t *)c->len.p, (uint64_t *)c->mag_s.p,
          (uint64_t *)c->sumsq_s.p, (uint64_t *)c->len_s.p);
      break;
  }
  MCG_CHECK(hipGetLastError());
  timed_end(c, F_LAYOUT);
  return MC_OK;
}

int launch_fused_scan(mc_ctx *c, uint32_t centre, uint64_t S, uint64_t E, uint32_t seq, const double *d_ident,
                      uint32_t part, uint32_t nparts) {
  const int nch = (int)((c->B * c->width + 15) / 16);
  uint64_t pos0 = S, pstride = ST, nblk = (E - S + 1 + ST - 1) / ST;
  if (nparts) {  // the rank's blocks: static block b (positions [b*ST, (b+1)*ST)) with b % nparts == part
    const uint64_t b_lo = S / ST, b_hi = E / ST;
    const uint64_t f = b_lo + (part + nparts - b_lo % nparts) % nparts;
    nblk = f <= b_hi ? (b_hi - f) / nparts + 1 : 0;
    pos0 = f * ST;
    pstride = (uint64_t)nparts * ST;
    if (nblk == 0) {  // nothing of this window is ours: one empty workgroup still publishes
      pos0 = E + 1;
      nblk = 1;
    }
  }
  const int grid = (int)nblk;
  FusedArgs A;
  memset(&A, 0, sizeof A);
  A.hs = (const uint4 *)c->hs.p;
  A.npad = c->npad;
  A.nch = nch;
  A.B = c->B;
  A.mag_s = (const uint64_t *)c->mag_s.p;
  A.sumsq_s = (const uint64_t *)c->sumsq_s.p;
  A.len_s = (const uint64_t *)c->len_s.p;
  A.order = (const uint32_t *)c->order.p;
  A.alive = (uint8_t *)c->alive.p;
  A.hist = (const uint8_t *)c->hist.p;
  A.pitch = c->pitch;
  A.mag = (const uint64_t *)c->mag.p;
  A.sumsq = (const uint64_t *)c->sumsq.p;
  A.len = (const uint64_t *)c->len.p;
  A.centre = centre;
  A.S = S;
  A.E = E;
  A.nkill = (int)c->pending_kills.size();
  for (int i = 0; i < A.nkill; i++) A.kills[i] = c->pending_kills[i];
  A.new_cluster = c->pending_begin ? 1 : 0;
  A.first_pos = c->pending_first_pos;
  A.step = c->step;
  A.partials = (ScanPartial *)c->partials.p;
  A.ticket = (uint32_t *)c->ticket.p;
  A.sd = (ScanDev *)c->scan_dev.p;
  A.flags_dev = (uint32_t *)((char *)c->scan_dev.p + sizeof(ScanDev));
  A.mem_pos = (uint32_t *)c->members.p;
  A.mkeys = (uint64_t *)c->member_keys.p;
  A.msum = (uint64_t *)c->msum.p;
  A.hres = c->h_res_dev;
  A.seq = seq;
  A.ident = d_ident;
  A.pos0 = pos0;
  A.pstride = pstride;
  A.part = nparts ? 1 : 0;
#ifdef MC_STAMPS
  static uint64_t *stamps = nullptr;
  static std::vector<double> acc(8, 0.0);
  static uint64_t nacc = 0;
  if (!stamps) (void)hipMalloc(&stamps, 64);
  if (nacc) {  // fold the previous launch's stamps (it has completed: its result was consumed)
    uint64_t h[8];
    (void)hipMemcpy(h, stamps, 64, hipMemcpyDeviceToHost);
    for (int i = 1; i < 7; i++) acc[i] += (double)(h[i] - h[0]) / 100.0;  // 100 MHz -> us
    if (nacc % 500 == 0) {
      fprintf(stderr, "[stamps] n=%llu avg us from first-wg start:", (unsigned long long)nacc);
      for (int i = 1; i < 7; i++) fprintf(stderr, " %d:%.2f", i, acc[i] / nacc);
      fprintf(stderr, "\n");
    }
  }
  {
    uint64_t init[8] = {~0ull, 0, 0, 0, 0, 0, 0, 0};
    (void)hipMemcpy(stamps, init, 64, hipMemcpyHostToDevice);
  }
  nacc++;
  A.stamps = stamps;
#endif
  const size_t lds = (size_t)2 * nch * 16 + (c->B <= 4096 ? (size_t)c->B * 8 : 0);
  timed_begin(c);
  const bool gs = c->B > 4096;
  if (c->width == 1) (gs ? fused_scan_kernel<uint8_t, true> : fused_scan_kernel<uint8_t, false>)<<<grid, ST, lds, c->stream>>>(A, c->cls);
  else (gs ? fused_scan_kernel<uint16_t, true> : fused_scan_kernel<uint16_t, false>)<<<grid, ST, lds, c->stream>>>(A, c->cls);
  MCG_CHECK(hipGetLastError());
  timed_end(c, F_SCAN);
  c->pending_kills.clear();
  if (!nparts) c->pending_begin = false;  // a sharded step's cluster starts at its commit
  return MC_OK;
}

int launch_commit(mc_ctx *c, const uint32_t *d_flags, uint32_t nflag, uint32_t seq) {
  const int nch = (int)((c->B * c->width + 15) / 16);
  CommitArgs A;
  memset(&A, 0, sizeof A);
  A.hs = (const uint4 *)c->hs.p;
  A.npad = c->npad;
  A.nch = nch;
  A.B = c->B;
  A.mag_s = (const uint64_t *)c->mag_s.p;
  A.order = (const uint32_t *)c->order.p;
  A.alive = (uint8_t *)c->alive.p;
  A.flags_dev = d_flags;
  A.nflag = nflag;
  A.new_cluster = c->pending_begin ? 1 : 0;
  A.first_pos = c->pending_first_pos;
  A.step = c->step;
  A.sd = (ScanDev *)c->scan_dev.p;
  A.mem_pos = (uint32_t *)c->members.p;
  A.mkeys = (uint64_t *)c->member_keys.p;
  A.msum = (uint64_t *)c->msum.p;
  A.hres = c->h_res_dev;
  A.seq = seq;
  const size_t lds = (size_t)nch * 16 + (c->B <= 4096 ? (size_t)c->B * 8 : 0);
  timed_begin(c);
  const bool gs = c->B > 4096;
  if (c->width == 1) (gs ? commit_kernel<uint8_t, true> : commit_kernel<uint8_t, false>)<<<1, ST, lds, c->stream>>>(A);
  else (gs ? commit_kernel<uint16_t, true> : commit_kernel<uint16_t, false>)<<<1, ST, lds, c->stream>>>(A);
  MCG_CHECK(hipGetLastError());
  timed_end(c, F_SCAN);
  c->pending_begin = false;
  return MC_OK;
}

}  // namespace mcg
