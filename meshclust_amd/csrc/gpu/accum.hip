// accum.hip -- host side of the device-resident accumulation (ClusterFactory::MS's accumulate
// loop, ClusterFactory.cpp:637-714): the plan (worker form, LDS layout, grid), the per-position
// window tables, and the launch of accum_kernel (accum_impl.hpp).  The kernel's instantiations
// live in one translation unit per worker form (accum_dense.hip, accum_wide.hip,
// accum_dstream.hip, accum_chunk.hip), so they compile in parallel; each has a PROF twin
// carrying the MC_ACCUM_PROFILE timers, which the production instantiations do not.
#include "accum_impl.hpp"

namespace mcg {

namespace {

__device__ uint64_t lower_len(const uint64_t *len_s, uint64_t a, uint64_t z, uint64_t L, bool strict) {
  while (a < z) {
    const uint64_t m = (a + z) / 2;
    if (strict ? len_s[m] <= L : len_s[m] < L) a = m + 1;
    else z = m;
  }
  return a;
}

__global__ __launch_bounds__(256) void wintab_kernel(uint64_t n, const uint64_t *__restrict__ len_s,
                                                     const uint64_t *__restrict__ mag_s,
                                                     const uint64_t *__restrict__ sumsq_s,
                                                     const uint32_t *__restrict__ bin_lo,
                                                     const uint64_t *__restrict__ bnd, uint32_t nb, double sim,
                                                     const uint4 *__restrict__ hs, uint64_t npad, int nch,
                                                     MInfo *__restrict__ out, uint4 *__restrict__ hr) {
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
    MInfo m;
    m.mag = mag_s[id];
    m.sumsq = sumsq_s[id];
    m.len = L;
    {  // bin: bin_lo[b] <= id < bin_lo[b + 1]
      uint64_t a = 0, z = nb;
      while (z - a > 1) {
        const uint64_t mid = (a + z) / 2;
        if (bin_lo[mid] <= id) a = mid;
        else z = mid;
      }
      m.bin = a;
    }
    m.wt = w;
    out[id] = m;
    for (int c = 0; c < nch; c++) hr[id * nch + c] = hs[(uint64_t)c * npad + id];
  }
}

__global__ void bits_init_kernel(uint32_t *bits, uint64_t n) {
  const uint64_t nwords = (n + 31) / 32;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t rem = n - w * 32;
    bits[w] = rem >= 32 ? ~0u : ((1u << rem) - 1u);
  }
}

struct AccPlan {
  const void *fn = nullptr;
  int res = 0;         // chunks per worker resident in its LDS (0: streaming)
  bool gbits = false;  // bitmap in global memory
  bool wide = false;   // a wave per candidate (accum_kernel<T, 0, true>)
  bool compact = false;  // streaming rows with per-chunk compaction (A.cc)
  bool dense = false;    // dense resident workers (worker_dense)
  bool dstream = false;  // dense streaming workers (worker_dstream)
  uint32_t mrow = 0;   // member cache entries
  size_t lds = 0;
  uint32_t G = 0;
  uint64_t fcap = 0;
  uint32_t rec_g = 0;
};

// Grid: one workgroup per CU (a multiple of the 8 XCDs): the controller and G - 1 workers.
uint32_t accum_grid(const mc_ctx *c) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess) cus = 256;
  // MC_ACCUM_GRID (tests): fewer workgroups, e.g. two ranks' kernels sharing one GPU
  if (const char *g = getenv("MC_ACCUM_GRID")) cus = std::min(cus, atoi(g));
  // ranks sharing this GPU (tests): each takes its share of the CUs less one per XCD -- the
  // kernels are launched plainly at different times, and a workgroup the dispatcher places on
  // a busier XCD must still find a free CU there (round-robin XCD placement is observed, not
  // promised: two exactly-fitting grids once left one workgroup waiting for the other kernel)
  // (mc_ctx_partition: the context's CU mask, less one CU per XCD of slack -- the dispatcher's
  // placement of workgroups over the XCDs is observed, not promised, and every workgroup of the
  // persistent grid must find a free CU of the mask)
  if (c->part_cus > 0) cus = std::min(cus, c->part_cus - 8);
  else if (c->mb_world > 0 && c->mb_share > 1) cus = cus / c->mb_share - 8;
  // mc_set_accum_grid: ranks sharing a mailbox run the smallest grid among them, so that every
  // rank derives the same tile of ownership from it (accum_plan's dense test depends on G)
  if (c->acc_grid > 0) cus = std::min<int>(cus, (int)c->acc_grid);
  uint32_t G = (uint32_t)cus / 8 * 8;
  if (G > GMAX) G = GMAX;
  if (G < 8) G = 8;
  return G;
}

// Variant and LDS layouts for this context; false when the configuration cannot run on the
// device.  Both roles get the same dynamic LDS (one workgroup per CU either way).
bool accum_plan(const mc_ctx *c, uint32_t nb, AccPlan *pl) {
  if (c->width != 1 && c->width != 2) return false;
  if (c->cls.align) return false;
  if (c->norder >= (1ull << 31)) return false;
  const int nch = (int)((c->B * c->width + 15) / 16);
  const uint32_t G = accum_grid(c), GW = G - 1;
  const bool wide = nch >= WIDE_NCH && !getenv("MC_ACCUM_NARROW");
  const uint64_t ts = wide ? NW : NT;
  const uint64_t W = c->mb_world > 0 ? (uint64_t)c->mb_world : 1;
  const uint64_t chunks = ((c->norder + ts - 1) / ts + W - 1) / W;  // this rank's tiles
  if (chunks >= (1ull << 22)) return false;  // (Div32's range)
  const uint64_t per_w = (chunks + GW - 1) / GW;
  pl->G = G;
  pl->wide = wide;
  pl->fcap = per_w * ts;
  pl->rec_g = (uint32_t)(wide ? REC_HDR : 4 * nch + REC_HDR);
  const bool prof = getenv("MC_ACCUM_PROFILE") != nullptr;
  pl->fn = wide ? accum_fn_wide(c->width, prof) : accum_fn_chunk(c->width, nch, false);
  const size_t static_lds = 16 * 1024;  // both roles' __shared__ words (13.1 KB), with margin
  const size_t cap = 160 * 1024 - static_lds;
  // worker: record words, centre row (wide), alive flags, resident rows (not wide)
  const size_t wfix = (size_t)(pl->rec_g + 3) / 4 * 16 + (wide ? (size_t)nch * 16 : 0) + (pl->fcap + 15) / 16 * 16;
  const size_t chunk_bytes = (size_t)nch * NT * 16;
  pl->res = (!wide && !getenv("MC_ACCUM_STREAM") && wfix + per_w * chunk_bytes <= cap) ? (int)per_w : 0;
  if (wfix >= cap) return false;
  size_t wfix_dense = 0;
  // dense resident workers: DT-position tiles round-robin, at most NT entries per worker
  if (!wide && nch <= DMAXCH && !getenv("MC_ACCUM_NO_DENSE") && !getenv("MC_ACCUM_STREAM")) {
    const uint64_t dchunks = ((c->norder + DT - 1) / DT + W - 1) / W;
    const uint64_t dper = (dchunks + GW - 1) / GW;
    const size_t dfix = (size_t)(pl->rec_g + 3) / 4 * 16 + (size_t)nch * NT * 16 + (size_t)NT * 4;
    if (dper * DT <= (uint64_t)NT && dfix <= cap) {
      pl->dense = true;
      pl->res = 0;
      pl->fcap = dper * DT;
      wfix_dense = dfix;
      pl->fn = accum_fn_dense(c->width, nch, prof);
    }
  }
  // dense streaming workers (config D on one to four GPUs): DT-position tiles, one dense list of
  // at most SJ * NT entries per worker with its rows in HBM; MC_ACCUM_NO_DSTREAM keeps the
  // 512-position-chunk streaming form
  if (!pl->dense && !wide && nch <= DMAXCH && pl->res == 0 && !getenv("MC_ACCUM_NO_DSTREAM") &&
      !getenv("MC_ACCUM_STREAM") && !getenv("MC_ACCUM_COMPACT")) {
    const uint64_t dchunks = ((c->norder + DT - 1) / DT + W - 1) / W;
    const uint64_t dper = (dchunks + GW - 1) / GW;
    const size_t dfix = (size_t)(pl->rec_g + 3) / 4 * 16 + 2 * (size_t)((dper * DT + 3) / 4 * 4) * 4;
    if (dper * DT <= (uint64_t)SJ * NT && dfix <= cap) {
      pl->dstream = true;
      pl->fcap = dper * DT;
      wfix_dense = dfix;
      pl->fn = accum_fn_dstream(c->width, nch, prof);
    }
  }
  // streaming rows (config D): compacted per chunk by its worker, the slot list in LDS -- opt in
  // (MC_ACCUM_COMPACT): measured slower at D1M, accumulation 1060 -> 1424 ms (profiles/r03_v10)
  pl->compact = !pl->dense && !wide && nch == 16 && c->width == 1 && pl->res == 0 && per_w <= 64 && getenv("MC_ACCUM_COMPACT") &&
                wfix + pl->fcap * 2 <= cap;
  if (pl->compact) pl->fn = accum_fn_chunk(1, 16, true);
  // controller: mean row, column sums, bvec (+ bitmap unless global), member cache
  auto cfix = [&](bool gbits) {
    size_t s = (size_t)nch * 16 + (size_t)c->B * 8;
    s += (size_t)((nb + 1) & ~1u) * 4 + 2 * (size_t)((nb + 2) & ~1u) * 4 + (size_t)nb * 8;
    if (!gbits) s += (size_t)((c->norder + 31) / 32 + 3) / 4 * 16;
    return s;
  };
  const size_t per_entry = (wide ? 0 : (size_t)(nch + 1) * 16) + sizeof(WinTab) + 24 + 8 + 4;
  // MC_ACCUM_GBITS=1 (tests): the global-bitmap variant that N >~ 900k needs, at any N
  for (int gb = getenv("MC_ACCUM_GBITS") ? 1 : 0; gb < 2; gb++) {
    const size_t f = cfix(gb != 0);
    if (f >= cap) continue;
    const uint64_t m = std::min<uint64_t>(1024, (cap - f) / per_entry);
    if (m >= 64 || (gb == 1 && m >= 1)) {
      pl->gbits = gb != 0;
      pl->mrow = (uint32_t)m;
      pl->lds = std::max(f + m * per_entry, (pl->dense || pl->dstream) ? wfix_dense
                                                      : wfix + (size_t)pl->res * chunk_bytes + (pl->compact ? pl->fcap * 2 : 0));
      return true;
    }
  }
  return false;
}

// s_a: go word + step ring; s_b: partials (+ global bitmap); s_c: flagged positions + kill
// log; s_i: member info (MInfo per static position); s_j: row-major static rows; s_k: the
// compacted / dense streaming row copies; s_d..s_g, acc_out: mc_accumulate's own inputs and
// outputs (abi.hip)
struct AccBytes {
  size_t ring, part, bits, fpos, klog;
};
int accum_alloc(mc_ctx *c, const AccPlan &pl, uint32_t nb, AccBytes *ab) {
  const uint32_t GW = pl.G - 1;
  const int nch = (int)((c->B * c->width + 15) / 16);
  ab->ring = 256 + (size_t)RING * pl.rec_g * 8 + (size_t)RING * 16;
  ab->part = ((size_t)GW * PART_G * 8 + 255) / 256 * 256;
  ab->bits = pl.gbits ? ((c->norder + 31) / 32 * 4 + 255) / 256 * 256 : 0;
  ab->fpos = ((size_t)GW * pl.fcap * 4 + 255) / 256 * 256;
  ab->klog = (c->norder * 8 + 16 + 255) / 256 * 256;
  if (ensure(c->s_a, ab->ring) || ensure(c->s_b, ab->part + ab->bits) || ensure(c->s_c, ab->fpos + ab->klog))
    return MC_ERR_OOM;
  if (ensure(c->s_i, c->norder * sizeof(MInfo) + 64) || ensure(c->s_j, c->norder * (size_t)nch * 16 + 64))
    return MC_ERR_OOM;
  // compacted row copies: one region of NT rows per local chunk (this rank's chunks); or the
  // dense streaming workers' two row buffers each
  const size_t cc_bytes = pl.compact    ? (size_t)(pl.fcap / NT) * GW * NT * (size_t)nch * 16
                          : pl.dstream ? (size_t)2 * GW * pl.fcap * (size_t)(nch + 1) * 16
                                       : 0;
  if (cc_bytes && ensure(c->s_k, cc_bytes)) return MC_ERR_OOM;
  if (ensure(c->s_d, ((size_t)nb + 1) * 4 + 16) || ensure(c->s_e, (size_t)nb * 8 + 16) ||
      ensure(c->s_f, c->norder * 4 + 16) || ensure(c->s_g, (c->norder + 1) * 8 + 16) || ensure(c->acc_out, 256) ||
      ensure(c->ord_ids, c->norder * 4 + 16))  // (mc_accumulate's ordered member ids)
    return MC_ERR_OOM;
  return MC_OK;
}

}  // namespace

uint64_t mailbox_slot_granules(uint32_t world, uint64_t n) {
  return MBOX_HDR + (n + world - 1) / world + NT;  // header + the most positions a rank owns
}

bool accum_supported(const mc_ctx *c, uint32_t nb) {
  AccPlan pl;
  return accum_plan(c, nb, &pl);
}

bool accum_plan_info(const mc_ctx *c, uint32_t nb, uint32_t info[4]) {
  AccPlan pl;
  if (!accum_plan(c, nb, &pl)) return false;
  info[0] = pl.G;
  info[1] = (pl.dense || pl.dstream) ? (uint32_t)DT : pl.wide ? (uint32_t)NW : (uint32_t)NT;  // the kernel's TSZ
  info[2] = (pl.dense ? 1u : 0u) | (pl.wide ? 2u : 0u) | (pl.res > 0 ? 4u : 0u) |
            (!pl.dense && !pl.wide && pl.res == 0 ? 8u : 0u) | (pl.dstream ? 16u : 0u);
  info[3] = (uint32_t)pl.lds;
  return true;
}

int accum_reserve(mc_ctx *c, uint32_t nb) {
  AccPlan pl;
  if (!accum_plan(c, nb, &pl)) {
    set_error("device-resident accumulation does not take this configuration");
    return MC_ERR_UNSUPPORTED;
  }
  AccBytes ab;
  return accum_alloc(c, pl, nb, &ab);
}

int launch_accum(mc_ctx *c, const uint32_t *d_bin_lo, const uint64_t *d_bounds, uint32_t nb, double sim,
                 uint32_t *d_mem_pos, uint64_t *d_mkeys, uint32_t *d_cl_centre, uint64_t *d_cl_off, uint64_t *d_out) {
  AccPlan pl;
  if (!accum_plan(c, nb, &pl)) {
    set_error("device-resident accumulation does not take this configuration");
    return MC_ERR_UNSUPPORTED;
  }
  const uint32_t G = pl.G, GW = G - 1;
  const int nch = (int)((c->B * c->width + 15) / 16);
  {
    hipFuncAttributes fa;
    MCG_CHECK(hipFuncGetAttributes(&fa, pl.fn));
    if (fa.sharedSizeBytes + pl.lds > 160 * 1024) {  // (accum_plan's static_lds margin is too small)
      set_error("accumulation kernel: static + dynamic LDS exceed 160 KB (" + std::to_string(fa.sharedSizeBytes) +
                " + " + std::to_string(pl.lds) + ")");
      return MC_ERR_HIP;
    }
  }
  MCG_CHECK(hipFuncSetAttribute(pl.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl.lds));
  int per_cu = 0;
  MCG_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pl.fn, NT, pl.lds));
  if (per_cu < 1) {
    set_error("accumulation kernel does not fit on a CU");
    return MC_ERR_HIP;
  }
  const uint64_t fcap = pl.fcap;
  AccBytes ab;
  if (int rc = accum_alloc(c, pl, nb, &ab)) return rc;
  const size_t ring_bytes = ab.ring, part_bytes = ab.part, fpos_bytes = ab.fpos;
  MInfo *d_minfo = (MInfo *)c->s_i.p;
  uint4 *d_hr = (uint4 *)c->s_j.p;
  uint32_t *d_bits = pl.gbits ? (uint32_t *)((char *)c->s_b.p + part_bytes) : nullptr;
  timed_begin(c);
  wintab_kernel<<<(int)std::min<uint64_t>((c->n + 255) / 256, 2048), 256, 0, c->stream>>>(
      c->norder, (const uint64_t *)c->len_s.p, (const uint64_t *)c->mag_s.p, (const uint64_t *)c->sumsq_s.p, d_bin_lo,
      d_bounds, nb, sim, (const uint4 *)c->hs.p, c->npad, nch, d_minfo, d_hr);
  MCG_CHECK(hipGetLastError());
  if (d_bits) {
    bits_init_kernel<<<(int)std::min<uint64_t>(c->norder / 32 / 256 + 1, 1024), 256, 0, c->stream>>>(d_bits, c->norder);
    MCG_CHECK(hipGetLastError());
  }
  timed_end(c, F_FINAL);
  MCG_CHECK(hipMemsetAsync(c->s_a.p, 0, ring_bytes, c->stream));  // no record carries a step tag yet
  MCG_CHECK(hipMemsetAsync(c->s_b.p, 0, part_bytes, c->stream));  // ... nor a partial
  AccArgs A;
  memset(&A, 0, sizeof A);
  A.hs = (const uint4 *)c->hs.p;
  A.npad = c->npad;
  A.nch = nch;
  A.B = c->B;
  A.mag_s = (const uint64_t *)c->mag_s.p;
  A.sumsq_s = (const uint64_t *)c->sumsq_s.p;
  A.len_s = (const uint64_t *)c->len_s.p;
  A.N = c->norder;
  A.nb = nb;
  A.bin_lo = d_bin_lo;
  A.bounds = d_bounds;
  A.minfo = d_minfo;
  A.hr = d_hr;
  A.gbits = d_bits;
  A.go = (uint32_t *)c->s_a.p;
  A.ring = (uint64_t *)((char *)c->s_a.p + 256);
  A.ringb = A.ring + (size_t)RING * pl.rec_g;
  A.spec = (pl.dense || pl.dstream) && !getenv("MC_ACCUM_NO_SPEC") ? 1 : 0;
  A.thin = A.spec && (pl.dense || pl.dstream) && !(getenv("MC_ACCUM_THIN") && atoi(getenv("MC_ACCUM_THIN")) == 0) ? 1 : 0;
  A.poll1 = getenv("MC_ACCUM_POLL1") ? 1 : 0;
  A.etake = getenv("MC_ACCUM_EARLY_TAKE") && atoi(getenv("MC_ACCUM_EARLY_TAKE")) ? 1 : 0;
  A.xfast = getenv("MC_ACCUM_NO_XFAST") ? 0 : 1;
  {
    const char *e = getenv("MC_ACCUM_RPOLL"), *g = getenv("MC_ACCUM_RPOLL_GAP");
    const int v = e ? atoi(e) : 1, gv = g ? atoi(g) : 2;
    A.rpoll = v < 1 ? 1 : v > 4 ? 4 : v;
    A.rpoll_gap = gv < 0 ? 0 : gv > 16 ? 16 : gv;
  }
  A.psleep = getenv("MC_ACCUM_POLL_SLEEP") ? atoi(getenv("MC_ACCUM_POLL_SLEEP")) : 1;
  A.rec_g = pl.rec_g;
  A.partials = (uint64_t *)c->s_b.p;
  char *sc = (char *)c->s_c.p;
  A.fpos = (uint32_t *)sc;
  A.klog = (uint64_t *)(sc + fpos_bytes);
  A.fcap = fcap;
  A.res = pl.res;
  A.cc = pl.compact ? (uint4 *)c->s_k.p : nullptr;
  A.srows = pl.dstream ? (uint4 *)c->s_k.p : nullptr;
  if (pl.dstream && !(getenv("MC_ACCUM_DRES") && atoi(getenv("MC_ACCUM_DRES")) == 0)) {
    // the LDS the launch holds beyond the worker's record and two position lists (accum_plan's
    // dfix), in whole entries of nch + 1 chunks, at most one per thread
    const size_t dfix = (size_t)(pl.rec_g + 3) / 4 * 16 + 2 * (size_t)((fcap + 3) / 4 * 4) * 4;
    const size_t per = (size_t)(nch + 1) * 16;
    A.dres = pl.lds > dfix ? (uint32_t)std::min<size_t>(NT, (pl.lds - dfix) / per) : 0u;
  }
  A.mrow = pl.mrow;
  A.mem_pos = d_mem_pos;
  A.mkeys = d_mkeys;
  A.cl_centre = d_cl_centre;
  A.cl_off = d_cl_off;
  A.out = d_out;
  A.fc = c->fcls;
  A.fc.rB = 1.0 / (double)A.B;
  A.dbg = getenv("MC_ACCUM_DBG") ? atoi(getenv("MC_ACCUM_DBG")) : 0;
  A.budget = 20ull * 100000000ull;  // a single hand-off never takes 20 s: give up, report error 99
  A.W = c->mb_world > 0 ? (uint32_t)c->mb_world : 1u;
  A.rank = c->mb_world > 0 ? (uint32_t)c->mb_rank : 0u;
  A.mbox = c->mb_world > 0 ? (uint64_t *)c->mb_dev : nullptr;
  A.slot_g = mailbox_slot_granules(A.W, c->norder);
  A.prof = getenv("MC_ACCUM_PROFILE") ? 1 : 0;
  A.trace = nullptr;
  if (getenv("MC_ACCUM_PROFILE") && atoi(getenv("MC_ACCUM_PROFILE")) >= 2) {
    const size_t tb = TRACE_STEPS * TRACE_W * 8, tb2 = (size_t)TRACE2_STEPS * GMAX * T2W * 8;
    if (ensure(c->s_h, tb + tb2)) return MC_ERR_OOM;
    MCG_CHECK(hipMemsetAsync(c->s_h.p, 0, tb + tb2, c->stream));
    A.trace = (uint64_t *)c->s_h.p;
    A.trace_all = atoi(getenv("MC_ACCUM_PROFILE")) == 3;
    A.trace2 = atoi(getenv("MC_ACCUM_PROFILE")) >= 4 ? (uint64_t *)((char *)c->s_h.p + tb) : nullptr;
  }
  if (getenv("MC_ACCUM_PROFILE"))
    fprintf(stderr, "[accum] variant: width %d nch %d wide %d dense %d dstream %d resident chunks/worker %d compact %d global-bitmap %d member-cache %u lds %zu G %u rank %u/%u fcap %llu dres %u\n",
            c->width, nch, (int)pl.wide, (int)pl.dense, (int)pl.dstream, pl.res, (int)pl.compact, (int)pl.gbits, pl.mrow, pl.lds, G,
            A.rank, A.W, (unsigned long long)pl.fcap, A.dres);
  DevClassifier cls = c->cls;
  void *args[] = {&A, &cls};
  timed_begin(c);
  // One workgroup per CU (the LDS plan admits no second): a cooperative launch guarantees
  // they are all resident.  Several ranks' kernels (mailbox) may share a GPU in tests, where a
  // second cooperative launch would wait for the first; they take a plain launch (every
  // hand-off has its 20 s deadline either way).
  // A context confined to a CU mask (mc_ctx_partition) launches plainly too: the cooperative
  // check counts the whole GPU, and the grid was sized to the mask.
  if (A.mbox || c->part_cus > 0 || getenv("MC_ACCUM_PLAIN_LAUNCH"))
    MCG_CHECK(hipLaunchKernel(pl.fn, dim3(G), dim3(NT), args, (unsigned)pl.lds, c->stream));
  else
    MCG_CHECK(hipLaunchCooperativeKernel(pl.fn, dim3(G), dim3(NT), args, (unsigned)pl.lds, c->stream));
  timed_end(c, F_SCAN);
  return MC_OK;
}

}  // namespace mcg
