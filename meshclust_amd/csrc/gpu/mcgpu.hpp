// mcgpu.hpp -- internal header of libmcgpu (MI355X / gfx950 engine behind include/meshclust_amd.h).
//
// Data layout in HBM (one context = one GPU):
//   codes      n sequences' one-digit bytes, concatenated (the NW input, Point::get_data_str)
//   packed     the same as 2-bit codes, 16 bases per 32-bit word, records word-aligned (K1 input)
//   seq_off    byte offsets (n+1), seg/seg_off: k-mer segments per sequence
//   hist       n rows of B = 4^k bins of width w bytes, id order, row pitch 16-byte aligned
//   mag/sumsq  per row: sum of bins (pseudo magnitude) and sum of squared bins
//   len        per row: sequence length (incl. N) for the length-difference feature
//   order/alive  static bvec order (position -> id) and the alive mask of accumulation
//   members    the growing cluster of the current accumulation (ids + tie-break keys)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../../include/meshclust_amd.h"

namespace mcg {

// This wave's index in its workgroup, as a wave-uniform (SGPR) value: threadIdx.x >> 6 is
// uniform per wave, but the compiler's divergence analysis cannot see that, and everything
// derived from it (loop bounds, wave roles) would otherwise be computed per lane with
// exec-mask branches.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

// Kernel families for the device timers (mc_timers): ms and launch count per family.
// F_LAYOUT: the static bvec-order copies of the rows (build_static), after K1
enum Family { F_KMER = 0, F_KEYS, F_PAIRS, F_SCAN, F_FINAL, F_MSHIFT, F_NW, F_LAYOUT, F_NFAM };

// Classifier in the form the kernels consume (mc_classifier + the exact decision threshold).
struct DevClassifier {
  mc_classifier c;
  double thr;  // round(1/(1+exp(-sum))) == 1  <=>  sum >= thr   (host glibc exp, see abi.hip)
  int align;   // the only feature is MC_FEAT_ALIGN: raw[0] is an NW identity (Trainer.cpp:570-577)
  // layout 3 / 4: the feature set Trainer::train builds (feat_set = 1, Trainer.cpp:583-588):
  // lookup [LD, INT, MAN, PEARSON(, KUL)], combos [LD*INT, (LD*MAN)^2, PEARSON(, (LD*KUL)^2)]
  // with 3 or 4 combos (features.hpp classify_std); 0 = any other (classify_raw)
  int layout;
};

// The accumulation workers' division-light decision (features.hpp classify_fast), passed to
// the accumulation kernel only: rinv[i] = RN(1 / (maxs[i] - mins[i])) on the host, and
// is_sim ? n : 1 - n == noff + nsgn * n; on = 1 when the classifier has the trainer's layout
// and every range of features 2..4 is finite and nonzero.
// classify_small (8-bit bins, small magnitudes) also takes range[i] = RN(maxs[i] - mins[i]) and
// divides features 0 / 1 by it as mk_div (mk = 1 when those ranges and minima keep every operand
// of the division normal), and rB = RN(1 / B) for the centre's PTerms (set by the launcher).
struct FastCls {
  double rinv[MC_MAX_SINGLE], noff[MC_MAX_SINGLE], nsgn[MC_MAX_SINGLE], range[MC_MAX_SINGLE];
  double rB;
  int on, mk;
};

// Read-only view of the device histogram matrix passed to kernels by value.
struct HistView {
  const uint8_t *hist;
  const uint64_t *mag;
  const uint64_t *sumsq;
  const uint64_t *len;
  uint64_t pitch;  // bytes per row
  int B;           // bins
  int width;       // bytes per bin
};

struct ScanPartial {
  double val;
  uint64_t pos;
  int32_t has;
  int32_t pad;
};

// Device-side result record of one accumulation step (mirrors mc_scan_result).
struct ScanDev {
  mc_scan_result r;
  uint32_t nflag;     // atomic counter of flagged candidates this step
  uint32_t nmembers;  // members in the current cluster
};

struct Buf {
  void *p = nullptr;
  size_t bytes = 0;
};

// A range of one array of the device lazy introsort (split.hip): partitioned (left >= 0:
// children left, left + 1, cut between them) or finished (fin: a sorted leaf).
struct SplitNode {
  int64_t lo, hi, cut;
  int32_t depth, left, fin, pad;
};

// Pinned, device-mapped record the fused scan publishes (zero-copy; seq written last).
struct HostScan {
  mc_scan_result r;
  uint32_t seq;
  uint32_t pad;
  uint32_t flags[1];  // n_flagged static positions follow
};

}  // namespace mcg

struct mc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  uint8_t *h_stage = nullptr;  // pinned staging ring for small uploads (abi.hip upload)
  uint8_t *h_dstage = nullptr;  // pinned landing buffer for a call's results (abi.hip download_pinned)
  size_t h_dstage_cap = 0;
  size_t stage_off = 0;
  // sequences
  uint64_t n = 0;
  std::vector<uint64_t> h_seq_off;
  mcg::Buf codes, seq_off, seg, seg_off;
  mcg::Buf packed, pk_off, impure;  // 2-bit codes (16 bases per word, records word-aligned), impure flags
  int kmer_spec_k = 0;              // K1 rows already written at 8 bits for this k (mc_kmer_max's pass)
  // histograms
  int k = 0, B = 0, width = 0;
  uint64_t pitch = 0;
  mcg::Buf hist, mag, sumsq, len;
  // classifier
  mcg::DevClassifier cls{};
  mcg::FastCls fcls{};
  bool has_cls = false;
  // accumulation state
  uint64_t norder = 0;
  mcg::Buf order, alive, members, member_keys, partials, scan_dev, flags_out;
  uint32_t step = 0;
  mcg::ScanDev *h_scan = nullptr;  // pinned mirror of scan_dev + flagged prefix (generic path)
  size_t h_scan_cap = 0;
  // fused path (8/16-bit bins): static chunk-major layout + zero-copy result
  mcg::Buf hs, mag_s, sumsq_s, len_s, ticket, msum;
  uint64_t npad = 0;
  mcg::HostScan *h_res = nullptr, *h_res_dev = nullptr;
  size_t h_res_cap = 0;
  uint32_t seq = 0;
  std::vector<uint64_t> pending_kills;
  bool pending_begin = false;
  uint64_t pending_first_pos = 0;
  std::vector<uint64_t> h_spos;  // id -> static position
  // alignment mode: host mirror of order/alive (builds the NW pair list of a window) and the
  // per-static-position identity the scan kernels classify
  std::vector<uint32_t> h_order;
  std::vector<uint8_t> h_alive;
  mcg::Buf ident_s, al_a, al_b, al_out, al_id, ord_ids;
  mcg::Buf acc_out;  // device-resident accumulation: counters / error word
  // Trainer::split's sorted arrays (mc_split_*): words, stopper scratch, range trees, queries
  mcg::Buf sp_words, sp_keys, sp_scr, sp_nodes, sp_nn, sp_q, sp_err;
  uint64_t sp_n = 0;
  uint32_t sp_narr = 0;
  int sp_depth0 = 0;
  // several ranks sharing one accumulation (mc_set_mailbox): host-memory mailbox, mapped
  void *mb_host = nullptr, *mb_dev = nullptr;
  uint64_t mb_bytes = 0;
  int mb_rank = 0, mb_world = 0, mb_share = 1;
  uint32_t acc_grid = 0;  // mc_set_accum_grid: cap on the accumulation kernel's workgroups (0: none)
  // mc_ctx_partition: this context's stream runs on slot `part_slot` of `part_share` disjoint CU
  // sets of its GPU (ranks sharing one GPU); part_cus CUs in the mask (0: the whole GPU)
  int part_slot = 0, part_share = 1, part_cus = 0;
  // scratch
  mcg::Buf s_a, s_b, s_c, s_d, s_e, s_f, s_g, s_h, s_i, s_j, s_k;
  mcg::Buf nw_items, nw_gran;  // NW chained row blocks: work items, bottom-row granules
  // mc_update_iteration's member lists on the device and their host shadow: re-uploaded only
  // when a merge changed them (cleared when sequences are loaded: the ids were checked against n)
  mcg::Buf u_off, u_mem;
  std::vector<uint64_t> h_uoff;
  std::vector<uint32_t> h_umem;
  std::vector<void *> pinned;
  // timers: event pairs recorded around kernels, resolved lazily after the next stream sync
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<int, int>> ev_pending;  // (family, pool index of the begin event)
  int ev_open = -1;
  double fam_ms[mcg::F_NFAM] = {0};
  double fam_n[mcg::F_NFAM] = {0};
};

namespace mcg {

void set_error(const std::string &m);
int hip_fail(hipError_t e, const char *what);
int ensure(Buf &b, size_t bytes);  // grow-only device buffer
void timed_begin(mc_ctx *c);
void timed_end(mc_ctx *c, Family f);
void flush_timers(mc_ctx *c);  // after a stream synchronisation

HistView hist_view(const mc_ctx *c);

// ---- launchers (defined in kmer.hip, k2.hip, nw.hip) -------------------------------------
int launch_expand(mc_ctx *c, uint64_t nexc, const uint64_t *d_exc_pos, const uint8_t *d_exc_val);
int launch_pack(mc_ctx *c);
int launch_kmer(mc_ctx *c, int k, int width, bool write, uint64_t *d_max, int *d_err);
int launch_distance_keys(mc_ctx *c, const uint32_t *d_piv, uint32_t npiv, const uint32_t *d_ids, uint64_t m,
                         uint16_t *d_keys);
// split.hip: words[p * n + t] = keys[p * n + t] << 32 | order[t]; the lazy introsort's queries
constexpr int32_t SPLIT_MAXNODE = 32768;
int split_build_words(mc_ctx *c, const uint32_t *d_order, uint64_t n, uint32_t npiv, const uint16_t *d_keys,
                      uint64_t *d_words);
// each accumulation cluster's members sorted by key and mapped to ids (k2.hip); clusters of
// more than order_members_max() members are left untouched
int launch_order_members(mc_ctx *c, const uint64_t *d_keys, const uint32_t *d_pos, const uint64_t *d_cl_off, uint64_t ncl,
                         uint32_t *d_ids);
uint64_t order_members_max();
// a small host array to device memory through the context's pinned staging ring (abi.hip)
int stage_h2d(mc_ctx *c, void *dst, const void *src, size_t bytes);
int launch_select(mc_ctx *c, uint64_t *d_words, uint64_t n, uint32_t *d_scr, SplitNode *d_nodes, int32_t *d_nnodes,
                  int32_t maxnode, int32_t depth0, uint32_t ngroups, const uint32_t *d_qarr, const uint64_t *d_qoff,
                  const uint64_t *d_qpos, uint64_t *d_qout, int *d_err);
int launch_pairs(mc_ctx *c, const uint32_t *d_a, const uint32_t *d_b, uint64_t m, const uint16_t *flags, int nflag,
                 double *d_raw, uint8_t *d_sim, double *d_c0, double *d_sum, bool classify);
int launch_scan(mc_ctx *c, uint32_t centre, uint64_t S, uint64_t E, const double *d_ident, int *nblocks);
int launch_merge_pairs(mc_ctx *c, const uint32_t *d_new, uint32_t C, const uint64_t *d_poff, uint32_t *d_a,
                       uint32_t *d_b);
int launch_values(mc_ctx *c, const double *d_raw, uint64_t m, uint8_t *d_sim, double *d_c0, double *d_sum);
int launch_finalize(mc_ctx *c, int nblocks);
int launch_mean_shift(mc_ctx *c, const uint32_t *d_cid, uint32_t C, const uint64_t *d_off, const uint64_t *h_off,
                      const uint32_t *d_mem, int delta, const uint8_t *d_keep, uint32_t *d_new, uint32_t j0,
                      uint32_t j1);
int build_static(mc_ctx *c);
bool accum_supported(const mc_ctx *c, uint32_t nb);
bool accum_plan_info(const mc_ctx *c, uint32_t nb, uint32_t info[4]);
uint64_t mailbox_slot_granules(uint32_t world, uint64_t n);  // mailbox granules per rank slot
// accum_kernel instantiations (accum_impl.hpp), one translation unit per worker form; width 1 / 2
// bytes per bin, nch 16 selects the compile-time 16-chunk rows (8-bit k = 4), prof the twin with
// the MC_ACCUM_PROFILE timers (the chunk forms have none: their profile runs carry no timers)
const void *accum_fn_dense(int width, int nch, bool prof);
const void *accum_fn_dstream(int width, int nch, bool prof);
const void *accum_fn_wide(int width, bool prof);
const void *accum_fn_chunk(int width, int nch, bool compact);
// every device buffer launch_accum needs for `nb` bins, allocated now (mc_accum_reserve: ranks
// sharing a GPU allocate before any rank launches, so no hipFree waits on a spinning peer kernel)
int accum_reserve(mc_ctx *c, uint32_t nb);
int launch_accum(mc_ctx *c, const uint32_t *d_bin_lo, const uint64_t *d_bounds, uint32_t nb, double sim,
                 uint32_t *d_mem_pos, uint64_t *d_mkeys, uint32_t *d_cl_centre, uint64_t *d_cl_off, uint64_t *d_out);
// nparts > 0: a sharded step (mc_scan_part) over this rank's static blocks only
int launch_fused_scan(mc_ctx *c, uint32_t centre, uint64_t S, uint64_t E, uint32_t seq, const double *d_ident,
                      uint32_t part = 0, uint32_t nparts = 0);
// mc_scan_commit: d_flags[0, nflag) ascending static positions (all ranks' flagged)
int launch_commit(mc_ctx *c, const uint32_t *d_flags, uint32_t nflag, uint32_t seq);
// NW on byte strings: pair p aligns A[aoff[ai[p]] .. aoff[ai[p]+1]) against B[...] (rows = A).
// Results go to slot p, or to slot d_out[p] when d_out is given.
int launch_nw(mc_ctx *c, const uint8_t *d_A, const uint64_t *d_aoff, const uint32_t *d_ai, const uint8_t *d_B,
              const uint64_t *d_boff, const uint32_t *d_bi, uint64_t m, const std::vector<uint64_t> &h_alen,
              const std::vector<uint64_t> &h_blen, double *d_ident, int32_t *d_len, int32_t *d_ids,
              int32_t *d_score, const uint32_t *d_out = nullptr);

}  // namespace mcg

#define MCG_CHECK(expr)                                   \
  do {                                                    \
    hipError_t _e = (expr);                               \
    if (_e != hipSuccess) return mcg::hip_fail(_e, #expr); \
  } while (0)
