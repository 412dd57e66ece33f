// abi.hip -- the C-ABI of include/meshclust_amd.h on top of the gfx950 kernels.
// Every entry point is synchronous at the ABI (one HIP stream per context inside) and fails
// loudly: there is no CPU fallback anywhere in libmcgpu.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mcgpu.hpp"

namespace mcg {

static thread_local std::string g_err;

void set_error(const std::string &m) { g_err = m; }

int hip_fail(hipError_t e, const char *what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return e == hipErrorOutOfMemory ? MC_ERR_OOM : MC_ERR_HIP;
}

int ensure(Buf &b, size_t bytes) {
  if (bytes <= b.bytes) return MC_OK;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  size_t want = std::max<size_t>(bytes, 256);
  if (hipMalloc(&b.p, want) != hipSuccess) {
    g_err = "hipMalloc of " + std::to_string(want) + " bytes failed";
    b.p = nullptr;
    return MC_ERR_OOM;
  }
  b.bytes = want;
  return MC_OK;
}

static void release(Buf &b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

static hipEvent_t pool_event(mc_ctx *c, size_t i) {
  while (c->ev_pool.size() <= i) {
    hipEvent_t e;
    (void)hipEventCreate(&e);
    c->ev_pool.push_back(e);
  }
  return c->ev_pool[i];
}

void timed_begin(mc_ctx *c) {
  const int i = (int)(2 * c->ev_pending.size());
  (void)hipEventRecord(pool_event(c, i), c->stream);
  c->ev_open = i;
}

void timed_end(mc_ctx *c, Family f) {
  const int i = c->ev_open;
  (void)hipEventRecord(pool_event(c, i + 1), c->stream);
  c->ev_pending.emplace_back((int)f, i);
}

void flush_timers(mc_ctx *c) {
  for (auto &pr : c->ev_pending) {
    float ms = 0;
    (void)hipEventSynchronize(c->ev_pool[pr.second + 1]);
    (void)hipEventElapsedTime(&ms, c->ev_pool[pr.second], c->ev_pool[pr.second + 1]);
    c->fam_ms[pr.first] += ms;
    c->fam_n[pr.first] += 1;
  }
  c->ev_pending.clear();
}

HistView hist_view(const mc_ctx *c) {
  return HistView{(const uint8_t *)c->hist.p, (const uint64_t *)c->mag.p, (const uint64_t *)c->sumsq.p,
                  (const uint64_t *)c->len.p, c->pitch, c->B, c->width};
}

// round(1/(1+exp(-s))) == 1 is monotone in s; find the smallest double s with that
// outcome using the host's libm exp -- the same glibc the reference links -- so the device
// decision `sum >= thr` equals the reference's for every sum.
static double decision_threshold() {
  auto pos = [](double s) { return std::round(1.0 / (1 + std::exp(-s))) == 1.0; };
  double lo = -1e-12, hi = 0.0;  // pos(lo) false, pos(hi) true
  if (pos(lo) || !pos(hi)) return 0.0;
  for (int it = 0; it < 200; it++) {
    double mid = lo / 2 + hi / 2;
    if (mid == lo || mid == hi) break;
    if (pos(mid)) hi = mid;
    else lo = mid;
  }
  while (true) {  // hi is positive, nextafter(hi, lo) is not
    double d = std::nextafter(hi, lo);
    if (d == lo || !pos(d)) break;
    hi = d;
  }
  return hi;
}

template <typename T>
static int upload(mc_ctx *c, Buf &b, const T *h, size_t count, hipStream_t s) {
  const size_t bytes = count * sizeof(T);
  if (int rc = ensure(b, bytes + 16)) return rc;
  if (!count) return MC_OK;
  // Small inputs (the per-call id lists, offsets, member lists) go through a pinned staging
  // ring owned by the context: a copy from pinned memory is a plain DMA, a pageable one is
  // staged by the runtime.  A region is reused only after a stream synchronize that follows
  // its copy (the ring wraps behind one).
  static const bool staged = !getenv("MC_PAGEABLE_UPLOADS");
  constexpr size_t STAGE = 8u << 20, SMALL = 1u << 20;
  if (staged && bytes <= SMALL) {
    if (!c->h_stage && hipHostMalloc((void **)&c->h_stage, STAGE, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      c->h_stage = nullptr;
    }
    if (c->h_stage) {
      size_t off = (c->stage_off + 255) & ~(size_t)255;
      if (off + bytes > STAGE) {
        MCG_CHECK(hipStreamSynchronize(s));
        off = 0;
      }
      memcpy(c->h_stage + off, h, bytes);
      MCG_CHECK(hipMemcpyAsync(b.p, c->h_stage + off, bytes, hipMemcpyHostToDevice, s));
      c->stage_off = off + bytes;
      return MC_OK;
    }
  }
  MCG_CHECK(hipMemcpyAsync(b.p, h, bytes, hipMemcpyHostToDevice, s));
  return MC_OK;
}

// launch helpers' small host arrays (nw.hip's bucket lists) through the same pinned ring
int stage_h2d(mc_ctx *c, void *dst, const void *src, size_t bytes) {
  if (!bytes) return MC_OK;
  constexpr size_t STAGE = 8u << 20, SMALL = 1u << 20;
  if (bytes <= SMALL && !getenv("MC_PAGEABLE_UPLOADS")) {
    if (!c->h_stage && hipHostMalloc((void **)&c->h_stage, STAGE, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      c->h_stage = nullptr;
    }
    if (c->h_stage) {
      size_t off = (c->stage_off + 255) & ~(size_t)255;
      if (off + bytes > STAGE) {
        MCG_CHECK(hipStreamSynchronize(c->stream));
        off = 0;
      }
      memcpy(c->h_stage + off, src, bytes);
      MCG_CHECK(hipMemcpyAsync(dst, c->h_stage + off, bytes, hipMemcpyHostToDevice, c->stream));
      c->stage_off = off + bytes;
      return MC_OK;
    }
  }
  MCG_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
  MCG_CHECK(hipStreamSynchronize(c->stream));  // (a pageable source may go out of scope)
  return MC_OK;
}

template <typename T>
static int download(T *h, const void *d, size_t count, hipStream_t s) {
  if (count) MCG_CHECK(hipMemcpyAsync(h, d, count * sizeof(T), hipMemcpyDeviceToHost, s));
  return MC_OK;
}

struct DPart {  // one result of a call: `bytes` from device `d` to host `h` (h null: not wanted)
  void *h;
  const void *d;
  size_t bytes;
};
static int download_pinned(mc_ctx *c, const void *d, size_t bytes, hipStream_t s, uint8_t **h);
// A call's results through the pinned landing buffer: one DMA per part into it, one stream
// synchronize, then the host copies (every part a pageable download was a runtime-staged copy).
// Ends with the stream synchronized, as the direct downloads it replaces did.
static int download_parts(mc_ctx *c, std::initializer_list<DPart> parts, hipStream_t s) {
  size_t total = 0;
  for (const DPart &p : parts)
    if (p.h && p.bytes) total += (p.bytes + 255) / 256 * 256;
  uint8_t *stage = nullptr;  // (the buffer only: no copy, so no failure but the allocation's)
  if (total > 0 && c->h_dstage_cap < total) (void)download_pinned(c, nullptr, total, s, &stage);
  const bool pinned = total > 0 && c->h_dstage_cap >= total;
  if (pinned) {
    size_t off = 0;
    for (const DPart &p : parts)
      if (p.h && p.bytes) {
        MCG_CHECK(hipMemcpyAsync(c->h_dstage + off, p.d, p.bytes, hipMemcpyDeviceToHost, s));
        off += (p.bytes + 255) / 256 * 256;
      }
  } else {
    for (const DPart &p : parts)
      if (p.h && p.bytes) MCG_CHECK(hipMemcpyAsync(p.h, p.d, p.bytes, hipMemcpyDeviceToHost, s));
  }
  MCG_CHECK(hipStreamSynchronize(s));
  if (pinned) {
    size_t off = 0;
    for (const DPart &p : parts)
      if (p.h && p.bytes) {
        memcpy(p.h, c->h_dstage + off, p.bytes);
        off += (p.bytes + 255) / 256 * 256;
      }
  }
  return MC_OK;
}

// One device region of a call's results copied to the context's pinned landing buffer (a plain
// DMA; a pageable destination is staged by the runtime, one staged copy per download) and the
// stream synchronized: the caller then copies the parts out of *h.  *h is null only when the
// landing buffer cannot be allocated (the caller then downloads the parts directly); a failing
// copy or synchronize is reported as the error it is, with its call site.
static int download_pinned(mc_ctx *c, const void *d, size_t bytes, hipStream_t s, uint8_t **h) {
  *h = nullptr;
  if (bytes > c->h_dstage_cap) {
    if (c->h_dstage) (void)hipHostFree(c->h_dstage);
    c->h_dstage = nullptr;
    c->h_dstage_cap = 0;
    const size_t cap = std::max<size_t>(bytes, 1u << 20);
    if (hipHostMalloc((void **)&c->h_dstage, cap, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      c->h_dstage = nullptr;
      return MC_OK;
    }
    c->h_dstage_cap = cap;
  }
  if (d) {  // (download_parts passes none: the buffer only)
    MCG_CHECK(hipMemcpyAsync(c->h_dstage, d, bytes, hipMemcpyDeviceToHost, s));
    MCG_CHECK(hipStreamSynchronize(s));
  }
  *h = c->h_dstage;
  return MC_OK;
}

}  // namespace mcg

using namespace mcg;

#define TRY(x)                  \
  do {                          \
    int _rc = (x);              \
    if (_rc != MC_OK) return _rc; \
  } while (0)

extern "C" {

const char *mc_last_error(void) { return mcg::g_err.c_str(); }
int mc_abi_version(void) { return MC_ABI_VERSION; }

int mc_ctx_create(int device, mc_ctx **out) {
  if (!out) return MC_ERR_ARG;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) {
    set_error("no HIP device available (libmcgpu requires an MI355X / gfx950 GPU)");
    return MC_ERR_HIP;
  }
  if (device < 0 || device >= ndev) {
    set_error("device index out of range");
    return MC_ERR_ARG;
  }
  MCG_CHECK(hipSetDevice(device));
  hipDeviceProp_t prop;
  MCG_CHECK(hipGetDeviceProperties(&prop, device));
  if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos) {
    set_error(std::string("libmcgpu is built for gfx950, device is ") + prop.gcnArchName);
    return MC_ERR_HIP;
  }
  auto *c = new mc_ctx();
  c->device = device;
  MCG_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  MCG_CHECK(hipEventCreate(&c->ev0));
  MCG_CHECK(hipEventCreate(&c->ev1));
  c->cls.thr = decision_threshold();
  *out = c;
  return MC_OK;
}

static void mailbox_detach(mc_ctx *c);

int mc_ctx_destroy(mc_ctx *c) {
  if (!c) return MC_OK;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  mailbox_detach(c);
  for (Buf *b : {&c->codes, &c->seq_off, &c->seg, &c->seg_off, &c->packed, &c->pk_off, &c->impure, &c->hist, &c->mag, &c->sumsq, &c->len, &c->order,
                 &c->alive, &c->members, &c->member_keys, &c->partials, &c->scan_dev, &c->flags_out, &c->s_a, &c->s_b,
                 &c->s_c, &c->s_d, &c->s_e, &c->s_f, &c->s_g, &c->s_h, &c->s_i, &c->s_j, &c->s_k, &c->hs, &c->mag_s, &c->sumsq_s, &c->len_s, &c->ticket,
                 &c->msum, &c->ident_s, &c->al_a, &c->al_b, &c->al_out, &c->al_id, &c->ord_ids, &c->acc_out, &c->sp_words, &c->sp_keys,
                 &c->sp_scr, &c->sp_nodes, &c->sp_nn, &c->sp_q, &c->sp_err, &c->u_off, &c->u_mem, &c->nw_items, &c->nw_gran})
    release(*b);
  if (c->h_scan) (void)hipHostFree(c->h_scan);
  if (c->h_stage) (void)hipHostFree(c->h_stage);
  if (c->h_dstage) (void)hipHostFree(c->h_dstage);
  if (c->h_res) (void)hipHostFree(c->h_res);
  for (auto e : c->ev_pool) (void)hipEventDestroy(e);
  (void)hipEventDestroy(c->ev0);
  (void)hipEventDestroy(c->ev1);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return MC_OK;
}

// shared by both loaders: offsets, segments, buffers; the byte and packed forms follow
static int load_common(mc_ctx *c, const uint64_t *seq_off, uint64_t n, const int32_t *seg, const uint64_t *seg_off,
                       std::vector<uint64_t> &pk_off) {
  MCG_CHECK(hipSetDevice(c->device));
  for (uint64_t i = 0; i < n; i++)
    if (seq_off[i + 1] < seq_off[i] || seg_off[i + 1] < seg_off[i]) {
      set_error("offsets must be non-decreasing");
      return MC_ERR_ARG;
    }
  c->n = n;
  c->k = 0;
  c->kmer_spec_k = 0;
  c->h_seq_off.assign(seq_off, seq_off + n + 1);
  if (pk_off.empty()) {
    pk_off.resize(n + 1);
    pk_off[0] = 0;
    for (uint64_t i = 0; i < n; i++) pk_off[i + 1] = pk_off[i] + (seq_off[i + 1] - seq_off[i] + 15) / 16;
  }
  TRY(ensure(c->codes, seq_off[n] + 16));
  TRY(ensure(c->packed, pk_off[n] * 4 + 16));
  TRY(ensure(c->impure, n + 16));
  TRY(upload(c, c->pk_off, pk_off.data(), n + 1, c->stream));
  TRY(upload(c, c->seq_off, seq_off, n + 1, c->stream));
  TRY(upload(c, c->seg, seg, 2 * seg_off[n], c->stream));
  TRY(upload(c, c->seg_off, seg_off, n + 1, c->stream));
  return MC_OK;
}

int mc_load_sequences(mc_ctx *c, const uint8_t *codes, const uint64_t *seq_off, uint64_t n, const int32_t *seg,
                      const uint64_t *seg_off) {
  if (c) {
    c->h_uoff.clear();
    c->h_umem.clear();
  }
  if (!c || !seq_off || !seg_off || (n && !codes)) return MC_ERR_ARG;
  std::vector<uint64_t> pk_off;
  TRY(load_common(c, seq_off, n, seg, seg_off, pk_off));
  if (seq_off[n]) MCG_CHECK(hipMemcpyAsync(c->codes.p, codes, seq_off[n], hipMemcpyHostToDevice, c->stream));
  if (n) TRY(launch_pack(c));
  MCG_CHECK(hipStreamSynchronize(c->stream));
  flush_timers(c);
  return MC_OK;
}

int mc_load_packed(mc_ctx *c, const uint32_t *packed, const uint64_t *pk_off, const uint64_t *seq_off, uint64_t n,
                   const uint64_t *exc_pos, const uint8_t *exc_val, uint64_t nexc, const int32_t *seg,
                   const uint64_t *seg_off) {
  if (c) {
    c->h_uoff.clear();
    c->h_umem.clear();
  }
  if (!c || !pk_off || !seq_off || !seg_off || (n && !packed) || (nexc && (!exc_pos || !exc_val))) return MC_ERR_ARG;
  for (uint64_t i = 0; i < n; i++)
    if (pk_off[i + 1] - pk_off[i] != (seq_off[i + 1] - seq_off[i] + 15) / 16) {
      set_error("pk_off must give every record ceil(length / 16) words");
      return MC_ERR_ARG;
    }
  // impure sequences: those holding an exception byte (exc_pos ascending)
  std::vector<uint8_t> imp(n, 0);
  for (uint64_t q = 0, i = 0; q < nexc; q++) {
    if (exc_pos[q] >= seq_off[n] || (q && exc_pos[q] <= exc_pos[q - 1])) {
      set_error("exception positions must be ascending and inside the sequences");
      return MC_ERR_ARG;
    }
    while (seq_off[i + 1] <= exc_pos[q]) i++;
    imp[i] = 1;
  }
  std::vector<uint64_t> pko(pk_off, pk_off + n + 1);
  TRY(load_common(c, seq_off, n, seg, seg_off, pko));
  if (pk_off[n]) MCG_CHECK(hipMemcpyAsync(c->packed.p, packed, pk_off[n] * 4, hipMemcpyHostToDevice, c->stream));
  if (n) MCG_CHECK(hipMemcpyAsync(c->impure.p, imp.data(), n, hipMemcpyHostToDevice, c->stream));
  if (nexc) {
    TRY(ensure(c->s_a, nexc * 8 + 16));
    TRY(ensure(c->s_b, nexc + 16));
    MCG_CHECK(hipMemcpyAsync(c->s_a.p, exc_pos, nexc * 8, hipMemcpyHostToDevice, c->stream));
    MCG_CHECK(hipMemcpyAsync(c->s_b.p, exc_val, nexc, hipMemcpyHostToDevice, c->stream));
  }
  if (n) TRY(launch_expand(c, nexc, (const uint64_t *)c->s_a.p, (const uint8_t *)c->s_b.p));
  MCG_CHECK(hipStreamSynchronize(c->stream));
  flush_timers(c);
  return MC_OK;
}

static int kmer_common(mc_ctx *c, int k, int width, bool write, uint64_t *largest) {
  if (!c || k < 1 || k > 12) {
    set_error("k must be in 1..12 (dense 4^k-bin histograms)");
    return MC_ERR_ARG;
  }
  if (c->n == 0 || !c->codes.p) {
    set_error("no sequences loaded");
    return MC_ERR_STATE;
  }
  MCG_CHECK(hipSetDevice(c->device));
  TRY(ensure(c->s_f, 64));
  MCG_CHECK(hipMemsetAsync(c->s_f.p, 0, 64, c->stream));
  uint64_t *d_max = (uint64_t *)c->s_f.p;
  int *d_err = (int *)((char *)c->s_f.p + 8);
  c->k = 0;  // rows are being (re)written
  c->kmer_spec_k = 0;
  c->B = 1 << (2 * k);
  c->width = width;
  c->pitch = ((uint64_t)c->B * width + 15) / 16 * 16;
  TRY(ensure(c->hist, c->n * c->pitch));
  TRY(ensure(c->mag, c->n * 8));
  TRY(ensure(c->sumsq, c->n * 8));
  TRY(ensure(c->len, c->n * 8));
  TRY(launch_kmer(c, k, width, write, d_max, d_err));
  uint64_t h[2] = {0, 0};
  MCG_CHECK(hipMemcpyAsync(h, c->s_f.p, 16, hipMemcpyDeviceToHost, c->stream));
  MCG_CHECK(hipStreamSynchronize(c->stream));
  flush_timers(c);
  if ((int)h[1] != 0) {
    set_error("a k-mer contains a code outside 0..3 (KmerHashTable::hash would throw InvalidInputException)");
    return MC_ERR_INPUT;
  }
  if (largest) *largest = h[0];
  return MC_OK;
}

// The largest-count pass (Runner.cpp:57-67) writes the 8-bit rows as it goes: when the
// maximum fits 8 bits, mc_kmer_build(k, 1) then has nothing left to do (K1 runs once).
int mc_kmer_max(mc_ctx *c, int k, uint64_t *largest) {
  uint64_t mx = 0;
  TRY(kmer_common(c, k, 1, true, &mx));
  if (mx <= 0xff) {
    c->k = k;
    c->kmer_spec_k = k;
  }
  if (largest) *largest = mx;
  return MC_OK;
}

int mc_kmer_build(mc_ctx *c, int k, int width) {
  if (!c || (width != 1 && width != 2 && width != 4 && width != 8)) return MC_ERR_ARG;
  if (c->kmer_spec_k == k && width == 1 && c->k == k) return MC_OK;  // written by mc_kmer_max
  TRY(kmer_common(c, k, width, true, nullptr));
  c->k = k;
  return MC_OK;
}

int mc_get_histograms(mc_ctx *c, void *hist, uint64_t *mags) {
  if (!c || c->k == 0) return MC_ERR_STATE;
  MCG_CHECK(hipSetDevice(c->device));
  const size_t rowb = (size_t)c->B * c->width;
  if (hist) MCG_CHECK(hipMemcpy2DAsync(hist, rowb, c->hist.p, c->pitch, rowb, c->n, hipMemcpyDeviceToHost, c->stream));
  if (mags) TRY(download(mags, c->mag.p, c->n, c->stream));
  MCG_CHECK(hipStreamSynchronize(c->stream));
  flush_timers(c);
  return MC_OK;
}

static int check_ids(mc_ctx *c, const uint32_t *ids, uint64_t m) {
  for (uint64_t i = 0; i < m; i++)
    if (ids[i] >= c->n) {
      set_error("point id out of range");
      return MC_ERR_ARG;
    }
  return MC_OK;
}

int mc_distance_keys(mc_ctx *c, const uint32_t *pivots, uint32_t npiv, const uint32_t *ids, uint64_t m, uint16_t *keys) {
  if (!c || c->k == 0) return MC_ERR_STATE;
  MCG_CHECK(hipSetDevice(c->device));
  TRY(check_ids(c, pivots, npiv));
  TRY(check_ids(c, ids, m));
  TRY(upload(c, c->s_a, pivots, npiv, c->stream));
  TRY(upload(c, c->s_b, ids, m, c->stream));
  TRY(ensure(c->s_c, (size_t)npiv * m * 2 + 16));
  TRY(launch_distance_keys(c, (uint32_t *)c->s_a.p, npiv, (uint32_t *)c->s_b.p, m, (uint16_t *)c->s_c.p));
  TRY(download(keys, c->s_c.p, (size_t)npiv * m, c->stream));
  MCG_CHECK(hipStreamSynchronize(c->stream));
  flush_timers(c);
  return MC_OK;
}

// ---- Trainer::split's sorts (split.hip) -----------------------------------------------------
static int split_reset(mc_ctx *c, uint32_t narr, uint64_t n, int depth) {
  if (n >= (1ull << 32)) {
    set_error("mc_split: arrays of 2^32 elements or more");
    return MC_ERR_ARG;
  }
  TRY(ensure(c->sp_scr, (size_t)narr * 2 * n * 4 + 16));
  TRY(ensure(c->sp_nodes, (size_t)narr * SPLIT_MAXNODE * sizeof(SplitNode)));
  TRY(ensure(c->sp_nn, (size_t)narr * 4 + 16));
  TRY(ensure(c->sp_err, 16));
  MCG_CHECK(hipMemsetAsync(c->sp_nn.p, 0, (size_t)narr * 4, c->stream));
  MCG_CHECK(hipMemsetAsync(c->sp_err.p, 0, 16, c->stream));
  int lg = 0;
  while (n >> (lg + 1)) lg++;
  c->sp_n = n;
  c->sp_narr = narr;
  c->sp_depth0 = depth >= 0 ? depth : 2 * lg;
  return MC_OK;
}

int mc_split_begin(mc_ctx *c, const uint32_t *pivots, uint32_t npiv, const uint32_t *order, uint64_t n) {
  if (!c || c->k == 0) return MC_ERR_STATE;
  if (!npiv || !n) return MC_ERR_ARG;
  MCG_CHECK(hipSetDevice(c->device));
  TRY(check_ids(c, pivots, npiv));
  TRY(check_ids(c, order, n));
  TRY(upload(c, c->s_a, pivots, npiv, c->stream));
  TRY(upload(c, c->s_b, order, n, c->stream));
  TRY(ensure(c->sp_keys, (size_t)npiv * n * 2 + 16));
  TRY(ensure(c->sp_words, (size_t)npiv * n * 8 + 16));
  TRY(split_reset(c, npiv, n, -1));
  TRY(launch_distance_keys(c, (uint32_t *)c->s_a.p, npiv, (uint32_t *)c->s_b.p, n, (uint16_t *)c->sp_keys.p));
  TRY(split_build_words(c, (uint32_t *)c->s_b.p, n, npiv, (uint16_t *)c->sp_keys.p, (uint64_t *)c->sp_words.p));
  MCG_CHECK(hipStreamSynchronize(c->stream));
  flush_timers(c);
  return MC_OK;
}

int mc_split_begin_words(mc_ctx *c, const uint64_t *words, uint32_t narr, uint64_t n, int depth) {
  if (!c || !words || !narr || !n) return MC_ERR_ARG;
  MCG_CHECK(hipSetDevice(c->device));
  TRY(ensure(c->sp_words, (size_t)narr * n * 8 + 16));
  MCG_CHECK(hipMemcpyAsync(c->sp_words.p, words, (size_t)narr * n * 8, hipMemcpyHostToDevice, c->stream));
  TRY(split_reset(c, narr, n, depth));
  MCG_CHECK(hipStreamSynchronize(c->stream));
  return MC_OK;
}

int mc_split_select_words(mc_ctx *c, uint64_t nq, const uint32_t *arr, const uint64_t *pos, uint64_t *out) {
  if (!c) return MC_ERR_ARG;
  if (!c->sp_narr) return MC_ERR_STATE;
  if (!nq) return MC_OK;
  for (uint64_t i = 0; i < nq; i++)
    if (arr[i] >= c->sp_narr || pos[i] >= c->sp_n) {
      set_error("mc_split_select: array index or position out of range");
      return MC_ERR_ARG;
    }
  MCG_CHECK(hipSetDevice(c->device));
  // queries grouped by array (counting sort; one workgroup per array with queries)
  std::vector<uint64_t> cnt(c->sp_narr + 1, 0);
  for (uint64_t i = 0; i < nq; i++) cnt[arr[i] + 1]++;
  for (uint32_t a = 0; a < c->sp_narr; a++) cnt[a + 1] += cnt[a];
  std::vector<uint64_t> qpos(nq), slot(nq);
  {
    std::vector<uint64_t> fill(cnt.begin(), cnt.end() - 1);
    for (uint64_t i = 0; i < nq; i++) {
      const uint64_t j = fill[arr[i]]++;
      qpos[j] = pos[i];
      slot[i] = j;
    }
  }
  std::vector<uint32_t> qarr;
  std::vector<uint64_t> qoff;
  for (uint32_t a = 0; a < c->sp_narr; a++)
    if (cnt[a + 1] > cnt[a]) {
      qarr.push_back(a);
      qoff.push_back(cnt[a]);
    }
  qoff.push_back(nq);
  const uint32_t ng = (uint32_t)qarr.size();
  // one buffer: qarr | qoff | qpos | qout
  const size_t o_off = ((size_t)ng * 4 + 15) / 16 * 16, o_pos = o_off + (size_t)(ng + 1) * 8, o_out = o_pos + nq * 8;
  TRY(ensure(c->sp_q, o_out + nq * 8 + 16));
  std::vector<uint8_t> hq(o_out);
  memcpy(hq.data(), qarr.data(), (size_t)ng * 4);
  memcpy(hq.data() + o_off, qoff.data(), (size_t)(ng + 1) * 8);
  memcpy(hq.data() + o_pos, qpos.data(), nq * 8);
  uint8_t *dq = (uint8_t *)c->sp_q.p;
  TRY(upload(c, c->sp_q, hq.data(), hq.size(), c->stream));
  timed_begin(c);
  TRY(launch_select(c, (uint64_t *)c->sp_words.p, c->sp_n, (uint32_t *)c->sp_scr.p, (SplitNode *)c->sp_nodes.p,
                    (int32_t *)c->sp_nn.p, SPLIT_MAXNODE, c->sp_depth0, ng, (const uint32_t *)dq,
                    (const uint64_t *)(dq + o_off), (const uint64_t *)(dq + o_pos), (uint64_t *)(dq + o_out),
                    (int *)c->sp_err.p));
  timed_end(c, F_KEYS);
  std::vector<uint64_t> qout(nq);
  int err = 0;
  TRY(download_parts(c, {{qout.data(), dq + o_out, nq * 8}, {&err, c->sp_err.p, 4}}, c->stream));
  flush_timers(c);
  if (err) {
    set_error("mc_split_select: more partitioned ranges than the device tree holds");
    return MC_ERR_UNSUPPORTED;
  }
  for (uint64_t i = 0; i < nq; i++) out[i] = qout[slot[i]];
  return MC_OK;
}

int mc_split_select(mc_ctx *c, uint64_t nq, const uint32_t *arr, const uint64_t *pos, uint32_t *ids) {
  std::vector<uint64_t> w(nq);
  TRY(mc_split_select_words(c, nq, arr, pos, w.data()));
  for (uint64_t i = 0; i < nq; i++) ids[i] = (uint32_t)w[i];
  return MC_OK;
}

int mc_split_end(mc_ctx *c) {
  if (!c) return MC_ERR_ARG;
  // the buffers stay with the context (grow-only) for the next clustering: freeing and
  // re-allocating ~0.4 GB per training cost more than the sorts
  c->sp_narr = 0;
  c->sp_n = 0;
  return MC_OK;
}

int mc_pair_features(mc_ctx *c, const uint32_t *a, const uint32_t *b, uint64_t m, const uint16_t *flags, int nflag,
                     double *raw) {
  if (!c || c->k == 0) return MC_ERR_STATE;
  if (nflag < 0 || nflag > 5) return MC_ERR_ARG;
  for (int f = 0; f < nflag; f++)
    if (flags[f] == MC_FEAT_ALIGN) {
      set_error("mc_pair_features: ALIGN is not a k-mer feature (use mc_nw_identity)");
      return MC_ERR_ARG;
    }
  MCG_CHECK(hipSetDevice(c->device));
  TRY(check_ids(c, a, m));
  TRY(check_ids(c, b, m));
  TRY(upload(c, c->s_a, a, m, c->stream));
  TRY(upload(c, c->s_b, b, m, c->stream));
  TRY(ensure(c->s_c, m * nflag * 8 + 16));
  TRY(launch_pairs(c, (uint32_t *)c->s_a.p, (uint32_t *)c->s_b.p, m, flags, nflag, (double *)c->s_c.p, nullptr,
                   nullptr, nullptr, false));
  TRY(download(raw, c->s_c.p, m * nflag, c->stream));
  MCG_CHECK(hipStreamSynchronize(c->stream));
  flush_timers(c);
  return MC_OK;
}

int mc_set_classifier(mc_ctx *c, const mc_classifier *cls) {
  if (!c || !cls) return MC_ERR_ARG;
  if (cls->n_single < 1 || cls->n_single > MC_MAX_SINGLE || cls->n_combo < 1 || cls->n_combo > MC_MAX_COMBO)
    return MC_ERR_ARG;
  bool align = false;
  for (int i = 0; i < cls->n_single; i++)
    if (cls->lookup[i] == MC_FEAT_ALIGN) align = true;
  // the reference only ever uses ALIGN alone (Trainer.cpp:570-577)
  if (align && (cls->n_single != 1 || cls->n_combo != 1 || cls->combo_len[0] != 1)) {
    set_error("MC_FEAT_ALIGN must be the only feature of an alignment-mode classifier");
    return MC_ERR_ARG;
  }
  c->cls.c = *cls;
  c->cls.align = align ? 1 : 0;
  // the trainer's feature set (Feature::add_feature order: Feature.cpp:7-31) -> classify_std
  c->cls.layout = 0;
  const uint16_t want[5] = {MC_FEAT_LD, MC_FEAT_INTERSECTION, MC_FEAT_MANHATTAN, MC_FEAT_PEARSON, MC_FEAT_KULCZYNSKI2};
  const int kinds[4] = {MC_COMBO_SELF, MC_COMBO_SQUARED, MC_COMBO_SELF, MC_COMBO_SQUARED};
  const int lens[4] = {2, 2, 1, 2};
  const int idx[4][2] = {{0, 1}, {0, 2}, {3, 0}, {0, 4}};
  if (!align && (cls->n_single == 4 || cls->n_single == 5) && cls->n_combo == cls->n_single - 1) {
    bool ok = true;
    for (int i = 0; i < cls->n_single; i++) ok &= cls->lookup[i] == want[i];
    for (int j = 0; j < cls->n_combo; j++) {
      ok &= cls->combo_kind[j] == kinds[j] && cls->combo_len[j] == lens[j];
      for (int e = 0; e < lens[j]; e++) ok &= cls->combo_idx[j][e] == idx[j][e];
    }
    if (ok) c->cls.layout = cls->n_single == 4 ? 3 : 4;
  }
  if (getenv("MC_CLASSIFY_GENERIC")) c->cls.layout = 0;  // diagnostics: the generic form only
  c->fcls.on = c->cls.layout != 0 && !getenv("MC_CLASSIFY_EXACT");
  c->fcls.mk = c->fcls.on && !getenv("MC_CLASSIFY_NO_SMALL");
  c->fcls.rB = 0.0;
  for (int i = 0; i < MC_MAX_SINGLE; i++) {
    c->fcls.rinv[i] = 0.0;
    c->fcls.noff[i] = 0.0;
    c->fcls.nsgn[i] = 1.0;
    if (i >= cls->n_single) continue;
    if (!cls->is_sim[i]) {
      c->fcls.noff[i] = 1.0;
      c->fcls.nsgn[i] = -1.0;
    }
    const double r = cls->maxs[i] - cls->mins[i];
    c->fcls.range[i] = r;
    c->fcls.rinv[i] = 1.0 / r;
    if (i < 2) {  // mk_div's operands stay normal: |range|, |min| (or min = 0) within 2^-200 .. 2^200
      const auto mid = [](double x) { return std::isfinite(x) && std::fabs(x) >= 0x1p-200 && std::fabs(x) <= 0x1p200; };
      if (!(mid(r) && mid(c->fcls.rinv[i]) && (cls->mins[i] == 0.0 || mid(cls->mins[i])))) c->fcls.mk = 0;
    }
    if (i >= 2 && !(std::isfinite(r) && r != 0.0 && std::isfinite(c->fcls.rinv[i]) && c->fcls.rinv[i] != 0.0 &&
                    std::isfinite(cls->mins[i])))
      c->fcls.on = 0;
  }
  c->has_cls = true;
  return MC_OK;
}

static int no_align(mc_ctx *c, const char *what) {
  if (!c->cls.align) return MC_OK;
  set_error(std::string(what) + " is not available in alignment mode (see include/meshclust_amd.h)");
  return MC_ERR_STATE;
}

int mc_classify_pairs(mc_ctx *c, const uint32_t *a, const uint32_t *b, uint64_t m, uint8_t *similar, double *combo0,
                      double *sum) {
  if (!c || c->k == 0 || !c->has_cls) return MC_ERR_STATE;
  TRY(no_align(c, "mc_classify_pairs"));
  MCG_CHECK(hipSetDevice(c->device));
  TRY(check_ids(c, a, m));
  TRY(check_ids(c, b, m));
  TRY(upload(c, c->s_a, a, m, c->stream));
  TRY(upload(c, c->s_b, b, m, c->stream));
  TRY(ensure(c->s_c, m * 17 + 64));
  uint8_t *d_sim = (uint8_t *)c->s_c.p;
  double *d_c0 = (double *)((char *)c->s_c.p + (m + 15) / 16 * 16);
  double *d_sum = d_c0 + m;
  TRY(launch_pairs(c, (uint32_t *)c->s_a.p, (uint32_t *)c->s_b.p, m, nullptr, 0, nullptr, d_sim, d_c0, d_sum, true));
  TRY(download_parts(c, {{similar, d_sim, m}, {combo0, d_c0, m * 8}, {sum, d_sum, m * 8}}, c->stream));
  flush_timers(c);
  return MC_OK;
}

int mc_nw_identity(mc_ctx *c, const uint32_t *a, const uint32_t *b, uint64_t m, double *ident, int32_t *len,
                   int32_t *ids) {
  if (!c || !c->codes.p) return MC_ERR_STATE;
  if (m == 0) return MC_OK;
  MCG_CHECK(hipSetDevice(c->device));
  TRY(check_ids(c, a, m));
  TRY(check_ids(c, b, m));
  std::vector<uint64_t> la(m), lb(m);
  for (uint64_t i = 0; i < m; i++) {
    la[i] = c->h_seq_off[a[i] + 1] - c->h_seq_off[a[i]];
    lb[i] = c->h_seq_off[b[i] + 1] - c->h_seq_off[b[i]];
  }
  TRY(upload(c, c->s_d, a, m, c->stream));
  TRY(upload(c, c->s_e, b, m, c->stream));
  TRY(ensure(c->s_f, m * 16 + 64));
  double *d_id = (double *)c->s_f.p;
  int32_t *d_len = (int32_t *)(d_id + m), *d_ids = d_len + m;
  TRY(launch_nw(c, (uint8_t *)c->codes.p, (uint64_t *)c->seq_off.p, (uint32_t *)c->s_d.p, (uint8_t *)c->codes.p,
                (uint64_t *)c->seq_off.p, (uint32_t *)c->s_e.p, m, la, lb, d_id, d_len, d_ids, nullptr));
  TRY(download_parts(c, {{ident, d_id, m * 8}, {len, d_len, m * 4}, {ids, d_ids, m * 4}}, c->stream));
  flush_timers(c);
  return MC_OK;
}

int mc_nw_identity_raw(mc_ctx *c, const uint8_t *a, const uint64_t *a_off, const uint8_t *b, const uint64_t *b_off,
                       uint64_t m, double *ident, int32_t *len, int32_t *ids, int32_t *score) {
  if (!c) return MC_ERR_ARG;
  if (m == 0) return MC_OK;
  MCG_CHECK(hipSetDevice(c->device));
  std::vector<uint64_t> la(m), lb(m);
  std::vector<uint32_t> idx(m);
  for (uint64_t i = 0; i < m; i++) {
    la[i] = a_off[i + 1] - a_off[i];
    lb[i] = b_off[i + 1] - b_off[i];
    idx[i] = (uint32_t)i;  // empty strings are allowed (GlobAlignE with len1 or len2 == 1)
  }
  // one scratch region: A bytes | B bytes | offsets | indices | outputs
  const size_t abytes = (a_off[m] - a_off[0] + 15) / 16 * 16, bbytes = (b_off[m] - b_off[0] + 15) / 16 * 16;
  const size_t total = abytes + bbytes + 2 * (m + 1) * 8 + m * 4 + m * 16 + 64;
  TRY(ensure(c->s_g, total));
  char *base = (char *)c->s_g.p;
  uint8_t *dA = (uint8_t *)base;
  uint8_t *dB = dA + abytes;
  uint64_t *dAo = (uint64_t *)(dB + bbytes), *dBo = dAo + (m + 1);
  uint32_t *dI = (uint32_t *)(dBo + (m + 1));
  double *dId = (double *)(((uintptr_t)(dI + m) + 15) / 16 * 16);
  int32_t *dL = (int32_t *)(dId + m), *dIds = dL + m;
  int32_t *dSc = nullptr;
  TRY(ensure(c->s_f, m * 4 + 16));
  dSc = (int32_t *)c->s_f.p;
  std::vector<uint64_t> ao(a_off, a_off + m + 1), bo(b_off, b_off + m + 1);
  for (auto &v : ao) v -= a_off[0];
  for (auto &v : bo) v -= b_off[0];
  MCG_CHECK(hipMemcpyAsync(dA, a + a_off[0], ao[m], hipMemcpyHostToDevice, c->stream));
  MCG_CHECK(hipMemcpyAsync(dB, b + b_off[0], bo[m], hipMemcpyHostToDevice, c->stream));
  MCG_CHECK(hipMemcpyAsync(dAo, ao.data(), (m + 1) * 8, hipMemcpyHostToDevice, c->stream));
  MCG_CHECK(hipMemcpyAsync(dBo, bo.data(), (m + 1) * 8, hipMemcpyHostToDevice, c->stream));
  MCG_CHECK(hipMemcpyAsync(dI, idx.data(), m * 4, hipMemcpyHostToDevice, c->stream));
  TRY(launch_nw(c, dA, dAo, dI, dB, dBo, dI, m, la, lb, dId, dL, dIds, dSc));
  TRY(download_parts(c, {{ident, dId, m * 8}, {len, dL, m * 4}, {ids, dIds, m * 4}, {score, dSc, m * 4}}, c->stream));
  flush_timers(c);
  return MC_OK;
}

static const size_t kFlagPrefix = 4096;  // flagged positions copied back with the result

static bool fused(const mc_ctx *c) { return c->width == 1 || c->width == 2; }

int mc_set_order(mc_ctx *c, const uint32_t *order, uint64_t n) {
  if (!c || !order || n != c->n) return MC_ERR_ARG;
  if (c->k == 0) return MC_ERR_STATE;
  MCG_CHECK(hipSetDevice(c->device));
  TRY(check_ids(c, order, n));
  c->norder = n;
  c->h_spos.assign(n, 0);
  for (uint64_t p = 0; p < n; p++) c->h_spos[order[p]] = p;
  c->h_order.assign(order, order + n);
  c->h_alive.assign(n, 1);
  TRY(upload(c, c->order, order, n, c->stream));
  TRY(ensure(c->alive, n + 16));
  MCG_CHECK(hipMemsetAsync(c->alive.p, 1, n, c->stream));
  TRY(ensure(c->members, (n + 1) * 4));
  TRY(ensure(c->member_keys, (n + 1) * 8));
  TRY(ensure(c->partials, ((n + 255) / 256 + 4096) * sizeof(ScanPartial)));
  TRY(ensure(c->scan_dev, sizeof(ScanDev) + std::max<uint64_t>(n + 1, kFlagPrefix) * 4));
  if (!c->h_scan) {
    c->h_scan_cap = sizeof(ScanDev) + kFlagPrefix * 4;
    MCG_CHECK(hipHostMalloc((void **)&c->h_scan, c->h_scan_cap, hipHostMallocDefault));
  }
  MCG_CHECK(hipMemsetAsync(c->scan_dev.p, 0, sizeof(ScanDev), c->stream));
  c->step = 0;
  c->pending_kills.clear();
  c->pending_begin = false;
  if (fused(c)) {
    TRY(ensure(c->ticket, 64));
    MCG_CHECK(hipMemsetAsync(c->ticket.p, 0, 64, c->stream));
    TRY(ensure(c->msum, (size_t)c->B * 8));
    const size_t hbytes = sizeof(HostScan) + (n + 16) * 4;
    if (c->h_res && c->h_res_cap < hbytes) {
      (void)hipHostFree(c->h_res);
      c->h_res = nullptr;
    }
    if (!c->h_res) {
      MCG_CHECK(hipHostMalloc((void **)&c->h_res, hbytes, hipHostMallocMapped));
      MCG_CHECK(hipHostGetDevicePointer((void **)&c->h_res_dev, c->h_res, 0));
      c->h_res_cap = hbytes;
    }
    c->h_res->seq = 0;
    c->seq = 0;
    TRY(build_static(c));
  }
  MCG_CHECK(hipStreamSynchronize(c->stream));
  flush_timers(c);
  return MC_OK;
}

int mc_kill(mc_ctx *c, uint64_t pos) {
  if (!c || pos >= c->norder) return MC_ERR_ARG;
  c->h_alive[pos] = 0;
  if (fused(c)) {  // applied by the next scan launch (which also excludes it from its window)
    if (c->pending_kills.size() == 8) {
      for (uint64_t p : c->pending_kills) MCG_CHECK(hipMemsetAsync((uint8_t *)c->alive.p + p, 0, 1, c->stream));
      c->pending_kills.clear();
    }
    c->pending_kills.push_back(pos);
    return MC_OK;
  }
  MCG_CHECK(hipMemsetAsync((uint8_t *)c->alive.p + pos, 0, 1, c->stream));
  return MC_OK;
}

int mc_cluster_begin(mc_ctx *c, uint32_t first) {
  if (!c || first >= c->n || c->norder == 0) return MC_ERR_ARG;
  if (fused(c)) {  // deferred into the next scan launch
    c->pending_begin = true;
    c->pending_first_pos = c->h_spos[first];
    return MC_OK;
  }
  ScanDev sd;
  memset(&sd, 0, sizeof sd);
  sd.nmembers = 1;
  // members[0] = first with tie-break key 0 (it is `current`'s first element)
  static thread_local uint64_t zero = 0;
  MCG_CHECK(hipMemcpyAsync(c->members.p, &first, 4, hipMemcpyHostToDevice, c->stream));
  MCG_CHECK(hipMemcpyAsync(c->member_keys.p, &zero, 8, hipMemcpyHostToDevice, c->stream));
  MCG_CHECK(hipMemcpyAsync(c->scan_dev.p, &sd, sizeof sd, hipMemcpyHostToDevice, c->stream));
  MCG_CHECK(hipStreamSynchronize(c->stream));
  flush_timers(c);
  return MC_OK;
}

// Spin on the sequence number the fused scan publishes in pinned host memory.
static int wait_seq(mc_ctx *c, uint32_t seq) {
  auto t0 = std::chrono::steady_clock::now();
  for (uint64_t it = 0;; it++) {
    if (__atomic_load_n(&c->h_res->seq, __ATOMIC_ACQUIRE) == seq) return MC_OK;
    if ((it & 4095) == 4095) {
      hipError_t e = hipStreamQuery(c->stream);
      if (e != hipSuccess && e != hipErrorNotReady) return hip_fail(e, "fused scan kernel");
      if (e == hipSuccess) {
        if (__atomic_load_n(&c->h_res->seq, __ATOMIC_ACQUIRE) == seq) return MC_OK;
        set_error("fused scan finished without publishing its result");
        return MC_ERR_HIP;
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) {
        set_error("fused scan result timeout");
        return MC_ERR_HIP;
      }
    }
    __builtin_ia32_pause();
  }
}

// Alignment mode, first half of a get_close step: Feature::align(*pt, *p) (Feature.cpp:
// 221-243; GlobAlignE with the candidate as seq1 and the centre as seq2) for every alive
// candidate of the window, written to ident_s[static position].  Within accumulation the
// reference's memo never changes a value: a centre is never alive again, so a (candidate,
// centre) pair can only recur in the same orientation (see cluster.cpp, AlignMemo).
static int align_window(mc_ctx *c, uint32_t centre, uint64_t S, uint64_t E, uint64_t *pairs, uint64_t *cells) {
  std::vector<uint32_t> ai, bi, out;
  std::vector<uint64_t> la, lb;
  const uint64_t lc = c->h_seq_off[centre + 1] - c->h_seq_off[centre];
  uint64_t cl = 0;
  for (uint64_t pos = S; pos <= E; pos++) {
    if (!c->h_alive[pos]) continue;
    const uint32_t id = c->h_order[pos];
    const uint64_t l = c->h_seq_off[id + 1] - c->h_seq_off[id];
    ai.push_back(id);
    bi.push_back(centre);
    out.push_back((uint32_t)pos);
    la.push_back(l);
    lb.push_back(lc);
    cl += l * lc;
  }
  *pairs = ai.size();
  *cells = cl;
  TRY(ensure(c->ident_s, c->norder * 8 + 16));
  if (ai.empty()) return MC_OK;
  TRY(upload(c, c->al_a, ai.data(), ai.size(), c->stream));
  TRY(upload(c, c->al_b, bi.data(), bi.size(), c->stream));
  TRY(upload(c, c->al_out, out.data(), out.size(), c->stream));
  return launch_nw(c, (uint8_t *)c->codes.p, (uint64_t *)c->seq_off.p, (uint32_t *)c->al_a.p, (uint8_t *)c->codes.p,
                   (uint64_t *)c->seq_off.p, (uint32_t *)c->al_b.p, ai.size(), la, lb, (double *)c->ident_s.p, nullptr,
                   nullptr, nullptr, (uint32_t *)c->al_out.p);
}

// mc_scan's step after the identities (alignment mode: d_ident, per static position) are on
// the device
static int scan_step(mc_ctx *c, uint32_t centre, uint64_t S, uint64_t E, const double *d_ident, uint64_t nw_pairs,
                     uint64_t nw_cells, uint32_t *flagged_pos, uint64_t cap, mc_scan_result *res) {
  if (fused(c)) {
    const uint32_t seq = ++c->seq;
    TRY(launch_fused_scan(c, centre, S, E, seq, d_ident));
    TRY(wait_seq(c, seq));
    *res = c->h_res->r;
    res->nw_pairs = nw_pairs;
    res->nw_cells = nw_cells;
    const uint64_t nf = res->n_flagged;
    if (nf > cap) {
      set_error("flagged buffer too small");
      return MC_ERR_ARG;
    }
    memcpy(flagged_pos, c->h_res->flags, nf * 4);
    std::sort(flagged_pos, flagged_pos + nf);
    for (uint64_t i = 0; i < nf; i++) c->h_alive[flagged_pos[i]] = 0;
    if (c->ev_pending.size() > 512) {
      MCG_CHECK(hipStreamSynchronize(c->stream));
      flush_timers(c);
    }
    return MC_OK;
  }
  int nblocks = 0;
  TRY(launch_scan(c, centre, S, E, d_ident, &nblocks));
  TRY(launch_finalize(c, nblocks));
  MCG_CHECK(hipMemcpyAsync(c->h_scan, c->scan_dev.p, c->h_scan_cap, hipMemcpyDeviceToHost, c->stream));
  MCG_CHECK(hipStreamSynchronize(c->stream));
  flush_timers(c);
  *res = c->h_scan->r;
  res->nw_pairs = nw_pairs;
  res->nw_cells = nw_cells;
  const uint64_t nf = res->n_flagged;
  if (nf > cap) {
    set_error("flagged buffer too small");
    return MC_ERR_ARG;
  }
  const uint32_t *hf = (const uint32_t *)((char *)c->h_scan + sizeof(ScanDev));
  const uint64_t first = std::min<uint64_t>(nf, kFlagPrefix);
  memcpy(flagged_pos, hf, first * 4);
  if (nf > first) {
    MCG_CHECK(hipMemcpyAsync(flagged_pos + first, (char *)c->scan_dev.p + sizeof(ScanDev) + first * 4, (nf - first) * 4,
                             hipMemcpyDeviceToHost, c->stream));
    MCG_CHECK(hipStreamSynchronize(c->stream));
    flush_timers(c);
  }
  std::sort(flagged_pos, flagged_pos + nf);
  for (uint64_t i = 0; i < nf; i++) c->h_alive[flagged_pos[i]] = 0;
  return MC_OK;
}

int mc_scan(mc_ctx *c, uint32_t centre, uint64_t S, uint64_t E, uint32_t *flagged_pos, uint64_t cap,
            mc_scan_result *res) {
  if (!c || !res || !c->has_cls || c->norder == 0) return MC_ERR_STATE;
  if (S > E || E >= c->norder || centre >= c->n) return MC_ERR_ARG;
  c->step++;
  uint64_t nw_pairs = 0, nw_cells = 0;
  const double *d_ident = nullptr;
  if (c->cls.align) {
    TRY(align_window(c, centre, S, E, &nw_pairs, &nw_cells));
    d_ident = (const double *)c->ident_s.p;
  }
  return scan_step(c, centre, S, E, d_ident, nw_pairs, nw_cells, flagged_pos, cap, res);
}

int mc_align_part(mc_ctx *c, uint32_t centre, uint64_t S, uint64_t E, uint32_t part, uint32_t nparts, double *ident,
                  uint64_t cap, uint64_t *n_part, uint64_t *pairs, uint64_t *cells) {
  if (!c || !c->has_cls || c->norder == 0 || !c->cls.align) return MC_ERR_STATE;
  if (S > E || E >= c->norder || centre >= c->n || nparts == 0 || part >= nparts || !n_part) return MC_ERR_ARG;
  std::vector<uint32_t> ai, bi;
  std::vector<uint64_t> la, lb;
  const uint64_t lc = c->h_seq_off[centre + 1] - c->h_seq_off[centre];
  uint64_t np = 0, cl = 0, i = 0;
  for (uint64_t pos = S; pos <= E; pos++) {
    if (!c->h_alive[pos]) continue;
    const uint32_t id = c->h_order[pos];
    const uint64_t l = c->h_seq_off[id + 1] - c->h_seq_off[id];
    np++;
    cl += l * lc;
    if (i++ % nparts != part) continue;
    ai.push_back(id);
    bi.push_back(centre);
    la.push_back(l);
    lb.push_back(lc);
  }
  if (pairs) *pairs = np;
  if (cells) *cells = cl;
  *n_part = ai.size();
  if (ai.size() > cap || (!ident && !ai.empty())) {
    set_error("mc_align_part: identity buffer too small");
    return MC_ERR_ARG;
  }
  if (ai.empty()) return MC_OK;
  // identities to a compact buffer in candidate order (no result slots: pair i -> ident[i])
  TRY(ensure(c->ident_s, c->norder * 8 + 16));
  TRY(ensure(c->al_id, ai.size() * 8 + 16));
  TRY(upload(c, c->al_a, ai.data(), ai.size(), c->stream));
  TRY(upload(c, c->al_b, bi.data(), bi.size(), c->stream));
  TRY(launch_nw(c, (uint8_t *)c->codes.p, (uint64_t *)c->seq_off.p, (uint32_t *)c->al_a.p, (uint8_t *)c->codes.p,
                (uint64_t *)c->seq_off.p, (uint32_t *)c->al_b.p, ai.size(), la, lb, (double *)c->al_id.p, nullptr,
                nullptr, nullptr, nullptr));
  MCG_CHECK(hipMemcpyAsync(ident, c->al_id.p, ai.size() * 8, hipMemcpyDeviceToHost, c->stream));
  MCG_CHECK(hipStreamSynchronize(c->stream));
  flush_timers(c);
  return MC_OK;
}

int mc_scan_ident(mc_ctx *c, uint32_t centre, uint64_t S, uint64_t E, const double *ident, uint32_t *flagged_pos,
                  uint64_t cap, mc_scan_result *res) {
  if (!c || !res || !c->has_cls || c->norder == 0 || !c->cls.align) return MC_ERR_STATE;
  if (S > E || E >= c->norder || centre >= c->n) return MC_ERR_ARG;
  c->step++;
  // the window's identities at their static positions (dead positions: never read)
  std::vector<double> win(E - S + 1, 0.0);
  uint64_t i = 0;
  for (uint64_t pos = S; pos <= E; pos++)
    if (c->h_alive[pos]) win[pos - S] = ident[i++];
  TRY(ensure(c->ident_s, c->norder * 8 + 16));
  MCG_CHECK(hipMemcpyAsync((double *)c->ident_s.p + S, win.data(), win.size() * 8, hipMemcpyHostToDevice, c->stream));
  // (the pageable copy is complete when the scan's result arrives: the same stream)
  const int rc = scan_step(c, centre, S, E, (const double *)c->ident_s.p, 0, 0, flagged_pos, cap, res);
  MCG_CHECK(hipStreamSynchronize(c->stream));
  return rc;
}

int mc_scan_part(mc_ctx *c, uint32_t centre, uint64_t S, uint64_t E, uint32_t part, uint32_t nparts,
                 uint32_t *flagged_pos, uint64_t cap, mc_scan_result *res) {
  if (!c || !res || !c->has_cls || c->norder == 0) return MC_ERR_STATE;
  if (S > E || E >= c->norder || centre >= c->n || nparts == 0 || part >= nparts) return MC_ERR_ARG;
  if (!fused(c) || c->cls.align) {
    set_error("sharded get_close steps take 8/16-bit k-mer histograms");
    return MC_ERR_UNSUPPORTED;
  }
  c->step++;
  const uint32_t seq = ++c->seq;
  TRY(launch_fused_scan(c, centre, S, E, seq, nullptr, part, nparts));
  TRY(wait_seq(c, seq));
  *res = c->h_res->r;
  res->new_centre = 0xffffffffu;
  const uint64_t nf = res->n_flagged;
  if (nf > cap) {
    set_error("flagged buffer too small");
    return MC_ERR_ARG;
  }
  memcpy(flagged_pos, c->h_res->flags, nf * 4);
  std::sort(flagged_pos, flagged_pos + nf);
  return MC_OK;
}

int mc_scan_commit(mc_ctx *c, const uint32_t *flagged_pos, uint64_t n, mc_scan_result *res) {
  if (!c || !res || !c->has_cls || c->norder == 0) return MC_ERR_STATE;
  if (!fused(c) || c->cls.align) {
    set_error("sharded get_close steps take 8/16-bit k-mer histograms");
    return MC_ERR_UNSUPPORTED;
  }
  if (n > c->norder || (n && !flagged_pos)) return MC_ERR_ARG;
  for (uint64_t i = 0; i < n; i++)
    if (flagged_pos[i] >= c->norder || (i && flagged_pos[i] <= flagged_pos[i - 1]) || !c->h_alive[flagged_pos[i]]) {
      set_error("mc_scan_commit: positions must be ascending, alive and in range");
      return MC_ERR_ARG;
    }
  uint32_t *d_flags = (uint32_t *)((char *)c->scan_dev.p + sizeof(ScanDev));
  if (n) MCG_CHECK(hipMemcpyAsync(d_flags, flagged_pos, n * 4, hipMemcpyHostToDevice, c->stream));
  for (uint64_t p : c->pending_kills) MCG_CHECK(hipMemsetAsync((uint8_t *)c->alive.p + p, 0, 1, c->stream));
  c->pending_kills.clear();
  const uint32_t seq = ++c->seq;
  TRY(launch_commit(c, d_flags, (uint32_t)n, seq));
  TRY(wait_seq(c, seq));
  memset(res, 0, sizeof *res);
  res->is_min = n == 0;
  res->n_flagged = n;
  res->new_centre = c->h_res->r.new_centre;
  res->n_members = c->h_res->r.n_members;
  for (uint64_t i = 0; i < n; i++) c->h_alive[flagged_pos[i]] = 0;
  return MC_OK;
}

// ---- mailbox of several ranks sharing one accumulation -------------------------------------
// The host range is registered once per process (hipHostRegister is process-wide), counted by
// the contexts that use it: the threads of `bin/meshclust --devices` share one buffer.
static std::mutex g_mb_mu;
static std::map<void *, int> g_mb_refs;

static void mailbox_detach(mc_ctx *c) {
  if (!c->mb_host) return;
  std::lock_guard<std::mutex> lk(g_mb_mu);
  auto it = g_mb_refs.find(c->mb_host);
  if (it != g_mb_refs.end() && --it->second == 0) {
    (void)hipHostUnregister(c->mb_host);
    g_mb_refs.erase(it);
  }
  c->mb_host = c->mb_dev = nullptr;
  c->mb_bytes = 0;
  c->mb_rank = c->mb_world = 0;
  c->mb_share = 1;
  c->acc_grid = 0;
}

uint64_t mc_mailbox_bytes(int world, uint64_t n) {
  if (world < 1) return 0;
  return 2ull * (uint64_t)world * mailbox_slot_granules((uint32_t)world, n) * 8;
}

int mc_ctx_pci_bus_id(mc_ctx *c, char *buf, int len) {
  if (!c || !buf || len < 16) return MC_ERR_ARG;
  MCG_CHECK(hipDeviceGetPCIBusId(buf, len, c->device));
  return MC_OK;
}

int mc_set_mailbox(mc_ctx *c, void *host, uint64_t bytes, int rank, int world, int share) {
  if (!c) return MC_ERR_ARG;
  MCG_CHECK(hipSetDevice(c->device));
  mailbox_detach(c);
  if (world == 0) return MC_OK;
  if (!host || world < 1 || world > 64 || rank < 0 || rank >= world || share < 1 || share > world ||
      ((uintptr_t)host & 7))
    return MC_ERR_ARG;
  {
    std::lock_guard<std::mutex> lk(g_mb_mu);
    auto it = g_mb_refs.find(host);
    if (it == g_mb_refs.end()) {
      const hipError_t e = hipHostRegister(host, bytes, hipHostRegisterMapped | hipHostRegisterPortable);
      if (e != hipSuccess) return hip_fail(e, "hipHostRegister (mailbox)");
      g_mb_refs[host] = 1;
    } else {
      it->second++;
    }
  }
  void *dev = nullptr;
  const hipError_t e = hipHostGetDevicePointer(&dev, host, 0);
  if (e != hipSuccess) {
    c->mb_host = host;  // (counted above)
    mailbox_detach(c);
    return hip_fail(e, "hipHostGetDevicePointer (mailbox)");
  }
  c->mb_host = host;
  c->mb_dev = dev;
  c->mb_bytes = bytes;
  c->mb_rank = rank;
  c->mb_world = world;
  c->mb_share = share;
  return MC_OK;
}

int mc_accum_plan_info(mc_ctx *c, uint32_t nbins, uint32_t info[4]) {
  if (!c || !info || nbins == 0) return MC_ERR_ARG;
  if (!c->has_cls || c->norder == 0) return MC_ERR_STATE;
  if (!fused(c) || !accum_plan_info(c, nbins, info)) {
    set_error("device-resident accumulation does not take this configuration");
    return MC_ERR_UNSUPPORTED;
  }
  return MC_OK;
}

int mc_set_accum_grid(mc_ctx *c, uint32_t grid) {
  if (!c) return MC_ERR_ARG;
  c->acc_grid = grid;
  return MC_OK;
}

int mc_accum_reserve(mc_ctx *c, uint32_t nbins) {
  if (!c || nbins == 0) return MC_ERR_ARG;
  if (!c->has_cls || c->norder == 0) return MC_ERR_STATE;
  if (!fused(c)) {
    set_error("device-resident accumulation does not take this configuration");
    return MC_ERR_UNSUPPORTED;
  }
  MCG_CHECK(hipSetDevice(c->device));
  return accum_reserve(c, nbins);
}

int mc_ctx_partition(mc_ctx *c, int slot, int share) {
  if (!c || share < 1 || share > 32 || slot < 0 || slot >= share) return MC_ERR_ARG;
  // (a run per clustering partitions again: the same slot keeps its stream -- re-creating it
  // synchronised with the device and cost milliseconds per rehearsal step)
  if (slot == c->part_slot && share == c->part_share) return MC_OK;
  MCG_CHECK(hipSetDevice(c->device));
  MCG_CHECK(hipStreamSynchronize(c->stream));
  int cus = 0;
  MCG_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
  hipStream_t s = nullptr;
  int n = 0;
  if (share == 1) {
    MCG_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  } else {
    // CU i joins slot (i / 8) % share: groups of eight consecutive mask bits alternate between
    // the slots, so each slot holds the same number of CUs of every XCD whether the mask's bits
    // are dealt to the XCDs round-robin or in contiguous runs
    std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
    for (int i = 0; i < cus; i++)
      if ((i / 8) % share == slot) {
        mask[(size_t)i / 32] |= 1u << (i % 32);
        n++;
      }
    if (n < 16) {
      set_error("mc_ctx_partition: fewer than 16 CUs per slot");
      return MC_ERR_ARG;
    }
    MCG_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  }
  (void)hipStreamDestroy(c->stream);
  c->stream = s;
  c->part_slot = slot;
  c->part_share = share;
  c->part_cus = share == 1 ? 0 : n;
  return MC_OK;
}

int mc_accumulate(mc_ctx *c, const uint32_t *bin_lo, const uint64_t *bounds, uint32_t nbins, double sim,
                  uint32_t *centre_ids, uint64_t *member_off, uint32_t *member_ids, uint64_t *nclusters,
                  uint64_t *stats) {
  if (!c || !c->has_cls || c->norder == 0) return MC_ERR_STATE;
  if (!bin_lo || !bounds || nbins == 0 || bin_lo[nbins] != c->norder || !centre_ids || !member_off || !member_ids ||
      !nclusters)
    return MC_ERR_ARG;
  for (uint32_t b = 0; b < nbins; b++)
    if (bin_lo[b] > bin_lo[b + 1]) return MC_ERR_ARG;
  if (!fused(c) || !accum_supported(c, nbins)) {
    set_error("device-resident accumulation does not take this configuration");
    return MC_ERR_UNSUPPORTED;
  }
  if (c->mb_world > 0 && c->mb_bytes < mc_mailbox_bytes(c->mb_world, c->norder)) {
    set_error("mailbox smaller than mc_mailbox_bytes(world, n)");
    return MC_ERR_ARG;
  }
  MCG_CHECK(hipSetDevice(c->device));
  const uint64_t n = c->norder;
  TRY(upload(c, c->s_d, bin_lo, (size_t)nbins + 1, c->stream));
  TRY(upload(c, c->s_e, bounds, nbins, c->stream));
  TRY(ensure(c->s_f, n * 4 + 16));
  TRY(ensure(c->s_g, (n + 1) * 8 + 16));
  TRY(ensure(c->acc_out, 256));
  MCG_CHECK(hipMemsetAsync(c->acc_out.p, 0, 256, c->stream));
  TRY(launch_accum(c, (const uint32_t *)c->s_d.p, (const uint64_t *)c->s_e.p, nbins, sim, (uint32_t *)c->members.p,
                   (uint64_t *)c->member_keys.p, (uint32_t *)c->s_f.p, (uint64_t *)c->s_g.p,
                   (uint64_t *)c->acc_out.p));
  uint64_t out[32];
  TRY(download_parts(c, {{out, c->acc_out.p, 256}}, c->stream));
  flush_timers(c);
  if (out[3]) {
    set_error(out[3] == 99 ? "device accumulation: hand-off timed out"
              : out[3] == 11 ? "bvec_iterator dereference out of range (the reference throws here)"
                             : "tried incrementing null iterator (the reference throws here)");
    return out[3] == 99 ? MC_ERR_TIMEOUT : MC_ERR_INPUT;
  }
  const uint64_t ncl = out[0], nmem = out[4];
  if (ncl > n || nmem != n) {
    set_error("device accumulation produced an inconsistent partition");
    return MC_ERR_HIP;
  }
  // the partition: each cluster's members sorted on the device (order_members_kernel), then the
  // ids, centres and offsets copied out through the pinned landing buffer; a cluster too large
  // for the kernel is sorted here
  TRY(ensure(c->ord_ids, n * 4 + 16));
  TRY(launch_order_members(c, (const uint64_t *)c->member_keys.p, (const uint32_t *)c->members.p,
                           (const uint64_t *)c->s_g.p, ncl, (uint32_t *)c->ord_ids.p));
  TRY(download_parts(c, {{member_ids, c->ord_ids.p, n * 4}, {centre_ids, c->s_f.p, ncl * 4},
                         {member_off, c->s_g.p, (ncl + 1) * 8}}, c->stream));
  const uint64_t om = order_members_max();
  for (uint64_t k = 0; k < ncl; k++) {
    const uint64_t a = member_off[k], b = member_off[k + 1];
    if (b - a <= om) continue;
    // `current` order: a key is step << 32 | position with step >= 1, or 0 for the seed -- with
    // the seed's key replaced by its position (< 2^32, so still first) one u64 sort orders it
    std::vector<uint64_t> kk(b - a);
    std::vector<uint32_t> pp(b - a);
    TRY(download_parts(c, {{kk.data(), (const uint64_t *)c->member_keys.p + a, (b - a) * 8},
                           {pp.data(), (const uint32_t *)c->members.p + a, (b - a) * 4}}, c->stream));
    for (uint64_t i = 0; i < b - a; i++)
      if (kk[i] == 0) kk[i] = pp[i];
    std::sort(kk.begin(), kk.end());
    for (uint64_t i = a; i < b; i++) member_ids[i] = c->h_order[(uint32_t)kk[i - a]];
  }
  for (uint64_t k = 0; k < ncl; k++) centre_ids[k] = c->h_order[centre_ids[k]];  // static positions -> ids
  *nclusters = ncl;
  if (stats) {
    stats[0] = out[1];
    stats[1] = out[2];
    for (int i = 0; i < 3; i++) stats[2 + i] = out[5 + i] / 100;  // controller phases, 100 MHz ticks -> us
  }
  if (getenv("MC_ACCUM_PROFILE")) {
    fprintf(stderr, "[accum] steps %llu window %.3f (centre data %.3f window %.3f record %.3f) wait %.3f collect %.3f "
            "(stragglers+reduce %.3f column sums %.3f [takes %.3f] mean %.3f closest %.3f) ms\n",
            (unsigned long long)out[1], out[5] / 1e5, out[12] / 1e5, out[13] / 1e5, out[14] / 1e5, out[6] / 1e5,
            out[7] / 1e5, out[8] / 1e5, out[9] / 1e5, out[15] / 1e5, out[10] / 1e5, out[11] / 1e5);
    fprintf(stderr, "[accum] closest: members scored %.3f, reduced %.3f, winner %.3f ms\n", out[18] / 1e5, out[19] / 1e5,
            out[20] / 1e5);
    fprintf(stderr, "[accum] window: record span %.3f, record stores issued %.3f ms\n", out[21] / 1e5, out[22] / 1e5);
    fprintf(stderr, "[accum] window: bvec kills %.3f, fast form %.3f (%llu), general form %.3f (%llu) ms\n", out[23] / 1e5,
            out[24] / 1e5, (unsigned long long)out[26], out[25] / 1e5, (unsigned long long)out[27]);
    if (out[17])  // the controller's shader-clock ticks over its 100 MHz real-time ticks
      fprintf(stderr, "[accum] controller shader clock %.0f MHz over %.3f ms\n", (double)out[16] / ((double)out[17] / 100.0),
              out[17] / 1e5);
    if (atoi(getenv("MC_ACCUM_PROFILE")) >= 4 && c->s_h.p) {
      // dense workers, per step < 256: distribution of the active workers' times after the
      // record (exact window) was published -- seen, scores done, partial stored -- and the
      // controller's all-partials time
      const int TW = 20, S2 = 256, G2 = 256, T2 = 6;  // accum.hip TRACE_W, TRACE2_STEPS, GMAX, T2W
      std::vector<uint64_t> tr(4096 * TW), t2((size_t)S2 * G2 * T2);
      MCG_CHECK(hipMemcpyAsync(tr.data(), c->s_h.p, tr.size() * 8, hipMemcpyDeviceToHost, c->stream));
      MCG_CHECK(hipMemcpyAsync(t2.data(), (char *)c->s_h.p + tr.size() * 8, t2.size() * 8, hipMemcpyDeviceToHost, c->stream));
      MCG_CHECK(hipStreamSynchronize(c->stream));
      // columns: seen, scores (wave 0), part B (wave 0), after the B barrier, after the reduce
      // barrier, partial stored
      const int col[6] = {0, 1, 3, 4, 5, 2};
      double acc[6][3] = {{0}}, all = 0, nw = 0, apub = 0;
      uint64_t ns = 0;
      for (int st = 2; st < S2; st++) {
        const uint64_t t0 = tr[(size_t)st * TW], ta = tr[(size_t)st * TW + 7];
        if (!t0 || !ta) continue;
        std::vector<double> v[6];
        for (int w = 0; w < G2; w++) {
          const uint64_t *x = &t2[((size_t)st * G2 + w) * T2];
          if (!x[2]) continue;
          for (int i = 0; i < 6; i++) v[i].push_back(x[col[i]] ? (double)(int64_t)(x[col[i]] - t0) / 100 : 0.0);
        }
        if (v[5].empty()) continue;
        for (int i = 0; i < 6; i++) {
          std::sort(v[i].begin(), v[i].end());
          acc[i][0] += v[i][0];
          acc[i][1] += v[i][v[i].size() / 2];
          acc[i][2] += v[i].back();
        }
        all += (double)(int64_t)(ta - t0) / 100;
        apub += tr[(size_t)st * TW + 6] ? (double)(int64_t)(tr[(size_t)st * TW + 6] - t0) / 100 : 0.0;
        nw += (double)v[5].size();
        ns++;
      }
      if (ns) {
        const char *nm[6] = {"seen", "scores", "partB", "last-wave-scores", "reduced", "partial"};
        fprintf(stderr, "[accum trace4] %llu steps, %.1f workers, us after the exact window's publish (min/med/max):",
                (unsigned long long)ns, nw / ns);
        for (int i = 0; i < 6; i++) fprintf(stderr, " %s %.2f/%.2f/%.2f", nm[i], acc[i][0] / ns, acc[i][1] / ns, acc[i][2] / ns);
        fprintf(stderr, "; controller all-seen %.2f; record (centre) published %.2f\n", all / ns, apub / ns);
      }
    }
    if (atoi(getenv("MC_ACCUM_PROFILE")) >= 2 && c->s_h.p) {
      // per step (first 4096; accum.hip trace_mark): record published -> first / last active
      // worker saw it -> first / last scan done -> first / last partial stored -> controller
      // has every partial -> collect done
      const int TW = 20;  // accum.hip TRACE_W
      std::vector<uint64_t> tr(4096 * TW);
      MCG_CHECK(hipMemcpyAsync(tr.data(), c->s_h.p, tr.size() * 8, hipMemcpyDeviceToHost, c->stream));
      MCG_CHECK(hipStreamSynchronize(c->stream));
      double a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, m[7] = {0, 0, 0, 0, 0, 0, 0};
      uint64_t cnt = 0, nact = 0, mcnt = 0, scnt = 0, bcnt = 0;
      double mb[3] = {0, 0, 0};
      for (uint64_t st = 1; st < 4096; st++) {  // MC_ACCUM_PROFILE=2: the middle active worker
        const uint64_t *t = &tr[st * TW];
        if (!t[0] || !t[10] || !t[14]) continue;
        for (int i = 0; i < 5; i++) m[i] += (double)(int64_t)(t[10 + i] - t[0]);
        if (t[15]) {  // (thread 0's own candidate was scanned)
          m[5] += (double)(int64_t)(t[15] - t[0]);
          m[6] += (double)(int64_t)(t[16] - t[0]);
          scnt++;
        }
        if (t[17] && t[18] && t[19]) {
          mb[0] += (double)(int64_t)(t[17] - t[0]);
          mb[1] += (double)(int64_t)(t[18] - t[0]);
          mb[2] += (double)(int64_t)(t[19] - t[0]);
          bcnt++;
        }
        mcnt++;
      }
      if (mcnt)
        fprintf(stderr, "[accum trace] middle worker, avg us after publish: seen %.2f kill-log %.2f wave0-top %.2f "
                "wave0-sums %.2f wave0-scanned %.2f all-scanned %.2f partial %.2f\n", m[0] / mcnt / 100, m[1] / mcnt / 100,
                scnt ? m[6] / scnt / 100 : 0.0, scnt ? m[5] / scnt / 100 : 0.0, m[2] / mcnt / 100, m[3] / mcnt / 100, m[4] / mcnt / 100);
      if (bcnt)
        fprintf(stderr, "[accum trace] middle worker barrier: last wave arrives %.2f, wave 0 leaves %.2f, last wave leaves %.2f\n",
                mb[0] / bcnt / 100, mb[1] / bcnt / 100, mb[2] / bcnt / 100);
      for (uint64_t st = 1; st < 4096; st++) {
        const uint64_t *t = &tr[st * TW];
        if (!t[0] || !t[7] || !t[8]) continue;
        const uint64_t p = t[0], s0 = ~t[1], s1 = t[2], c0 = ~t[3], c1 = t[4], q0 = ~t[5], q1 = t[6];
        const double d[9] = {(double)(int64_t)(s0 - p), (double)(int64_t)(s1 - p), (double)(int64_t)(c0 - p),
                             (double)(int64_t)(c1 - p), (double)(int64_t)(q0 - p), (double)(int64_t)(q1 - p),
                             (double)(int64_t)(t[7] - p), (double)(int64_t)(t[8] - p), 0.0};
        for (int i = 0; i < 8; i++) a[i] += d[i];
        nact += t[9];
        cnt++;
      }
      if (cnt)
        fprintf(stderr, "[accum trace] %llu steps, avg us after publish: seen %.2f..%.2f scanned %.2f..%.2f "
                "partial %.2f..%.2f all-seen %.2f collect-done %.2f; active WGs %.1f\n", (unsigned long long)cnt,
                a[0] / cnt / 100, a[1] / cnt / 100, a[2] / cnt / 100, a[3] / cnt / 100, a[4] / cnt / 100,
                a[5] / cnt / 100, a[6] / cnt / 100, a[7] / cnt / 100, (double)nact / cnt);
    }
  }
  return MC_OK;
}

int mc_classify_values(mc_ctx *c, const double *raw, uint64_t m, uint8_t *similar, double *combo0, double *sum) {
  if (!c || !c->has_cls) return MC_ERR_STATE;
  if (m == 0) return MC_OK;
  if (!raw) return MC_ERR_ARG;
  MCG_CHECK(hipSetDevice(c->device));
  const int ns = c->cls.c.n_single;
  TRY(upload(c, c->s_a, raw, m * ns, c->stream));
  TRY(ensure(c->s_c, m * 17 + 64));
  uint8_t *d_sim = (uint8_t *)c->s_c.p;
  double *d_c0 = (double *)((char *)c->s_c.p + (m + 15) / 16 * 16);
  double *d_sum = d_c0 + m;
  TRY(launch_values(c, (const double *)c->s_a.p, m, d_sim, d_c0, d_sum));
  TRY(download_parts(c, {{similar, d_sim, m}, {combo0, d_c0, m * 8}, {sum, d_sum, m * 8}}, c->stream));
  flush_timers(c);
  return MC_OK;
}

static int mean_shift_common(mc_ctx *c, const uint32_t *centre_ids, uint32_t C, const uint64_t *member_off,
                             const uint32_t *members, int delta, const uint8_t *keep, uint32_t *new_centre,
                             uint32_t j0, uint32_t j1) {
  if (!c || !c->has_cls || c->k == 0 || delta < 0) return MC_ERR_STATE;
  if (j0 > j1 || j1 > C) return MC_ERR_ARG;
  if (C == 0 || j0 == j1) return MC_OK;
  MCG_CHECK(hipSetDevice(c->device));
  TRY(check_ids(c, centre_ids, C));
  const uint64_t nm = member_off[C];
  TRY(check_ids(c, members, nm));
  TRY(upload(c, c->s_a, centre_ids, C, c->stream));
  TRY(upload(c, c->s_b, member_off, C + 1, c->stream));
  TRY(upload(c, c->s_c, members, nm, c->stream));
  const uint8_t *d_keep = nullptr;
  if (keep) {
    uint64_t nk = 0;
    for (uint32_t j = 0; j < C; j++) {
      const uint32_t b = j >= (uint32_t)delta ? j - delta : 0;
      const uint32_t e = std::min<uint32_t>(j + delta, C - 1);
      nk += member_off[e + 1] - member_off[b];
    }
    TRY(upload(c, c->al_out, keep, nk, c->stream));
    d_keep = (const uint8_t *)c->al_out.p;
  }
  TRY(ensure(c->flags_out, (size_t)C * 4 + 16));
  TRY(launch_mean_shift(c, (uint32_t *)c->s_a.p, C, (uint64_t *)c->s_b.p, member_off, (uint32_t *)c->s_c.p, delta,
                        d_keep, (uint32_t *)c->flags_out.p, j0, j1));
  TRY(download(new_centre, (uint32_t *)c->flags_out.p + j0, j1 - j0, c->stream));
  MCG_CHECK(hipStreamSynchronize(c->stream));
  flush_timers(c);
  return MC_OK;
}

int mc_mean_shift(mc_ctx *c, const uint32_t *centre_ids, uint32_t C, const uint64_t *member_off, const uint32_t *members,
                  int delta, uint32_t *new_centre) {
  if (!c) return MC_ERR_ARG;
  TRY(no_align(c, "mc_mean_shift"));
  return mean_shift_common(c, centre_ids, C, member_off, members, delta, nullptr, new_centre, 0, C);
}

int mc_update_iteration(mc_ctx *c, const uint32_t *centre_ids, uint32_t C, const uint64_t *member_off,
                        const uint32_t *members, int delta, uint32_t *new_centre, uint8_t *similar, double *combo0,
                        uint64_t *npairs) {
  if (!c || !npairs || !member_off) return MC_ERR_ARG;
  TRY(no_align(c, "mc_update_iteration"));
  if (!c->has_cls || c->k == 0 || delta < 0) return MC_ERR_STATE;
  *npairs = 0;
  if (C == 0) return MC_OK;
  MCG_CHECK(hipSetDevice(c->device));
  TRY(check_ids(c, centre_ids, C));
  const uint64_t nm = member_off[C];
  std::vector<uint64_t> poff(C + 1, 0);
  for (uint32_t i = 0; i < C; i++) poff[i + 1] = poff[i] + std::min<uint64_t>((uint64_t)delta, C - 1 - i);
  const uint64_t m = poff[C];
  TRY(upload(c, c->s_a, centre_ids, C, c->stream));
  const bool same = c->h_uoff.size() == (size_t)C + 1 && c->h_umem.size() == nm &&
                    std::memcmp(c->h_uoff.data(), member_off, ((size_t)C + 1) * 8) == 0 &&
                    (nm == 0 || std::memcmp(c->h_umem.data(), members, nm * 4) == 0);
  if (!same) {
    TRY(check_ids(c, members, nm));
    c->h_uoff.clear();
    c->h_umem.clear();
    TRY(upload(c, c->u_off, member_off, C + 1, c->stream));
    TRY(upload(c, c->u_mem, members, nm, c->stream));
    c->h_uoff.assign(member_off, member_off + C + 1);
    c->h_umem.assign(members, members + nm);
  }
  TRY(upload(c, c->s_h, poff.data(), C + 1, c->stream));
  // results in one region of s_j: combo0 (m doubles) | similar (m bytes) | new centres (C words)
  const size_t o_new = (m * 9 + 15) / 16 * 16, res_bytes = o_new + (size_t)C * 4;
  TRY(ensure(c->s_i, m * 8 + 16));
  TRY(ensure(c->s_j, res_bytes + 64));
  uint32_t *d_new = (uint32_t *)((uint8_t *)c->s_j.p + o_new);
  uint32_t *d_pa = (uint32_t *)c->s_i.p, *d_pb = d_pa + m;
  double *d_c0 = (double *)c->s_j.p;
  uint8_t *d_sim = (uint8_t *)(d_c0 + m);
  TRY(launch_mean_shift(c, (uint32_t *)c->s_a.p, C, (uint64_t *)c->u_off.p, member_off, (uint32_t *)c->u_mem.p, delta,
                        nullptr, d_new, 0, C));
  if (m) {
    TRY(launch_merge_pairs(c, d_new, C, (const uint64_t *)c->s_h.p, d_pa, d_pb));
    TRY(launch_pairs(c, d_pa, d_pb, m, nullptr, 0, nullptr, d_sim, d_c0, nullptr, true));
  }
  // the whole result region in one copy to pinned memory (three pageable downloads were three
  // staged copies per iteration)
  uint8_t *h = nullptr;
  TRY(download_pinned(c, c->s_j.p, res_bytes, c->stream, &h));
  if (h) {
    if (m && combo0) memcpy(combo0, h, m * 8);
    if (m && similar) memcpy(similar, h + m * 8, m);
    memcpy(new_centre, h + o_new, (size_t)C * 4);
  } else {
    if (m && similar) TRY(download(similar, d_sim, m, c->stream));
    if (m && combo0) TRY(download(combo0, d_c0, m, c->stream));
    TRY(download(new_centre, d_new, C, c->stream));
    MCG_CHECK(hipStreamSynchronize(c->stream));
  }
  flush_timers(c);
  *npairs = m;
  return MC_OK;
}

int mc_mean_shift_range(mc_ctx *c, const uint32_t *centre_ids, uint32_t C, const uint64_t *member_off,
                        const uint32_t *members, int delta, uint32_t j0, uint32_t j1, uint32_t *new_centre) {
  TRY(no_align(c, "mc_mean_shift_range"));
  return mean_shift_common(c, centre_ids, C, member_off, members, delta, nullptr, new_centre, j0, j1);
}

int mc_mean_shift_select(mc_ctx *c, const uint32_t *centre_ids, uint32_t C, const uint64_t *member_off,
                         const uint32_t *members, int delta, const uint8_t *keep, uint32_t *new_centre) {
  if (!c || !keep) return MC_ERR_ARG;
  return mean_shift_common(c, centre_ids, C, member_off, members, delta, keep, new_centre, 0, C);
}

int mc_sync(mc_ctx *c) {
  if (!c) return MC_ERR_ARG;
  MCG_CHECK(hipSetDevice(c->device));
  MCG_CHECK(hipDeviceSynchronize());
  return MC_OK;
}

int mc_timers(mc_ctx *c, double *ms_out, int n, int reset) {
  if (!c) return MC_ERR_ARG;
  (void)hipStreamSynchronize(c->stream);
  flush_timers(c);
  for (int f = 0; f < F_NFAM && 2 * f + 1 < n; f++) {
    ms_out[2 * f] = c->fam_ms[f];
    ms_out[2 * f + 1] = c->fam_n[f];
  }
  if (reset)
    for (int f = 0; f < F_NFAM; f++) c->fam_ms[f] = c->fam_n[f] = 0;
  return MC_OK;
}

}  // extern "C"
