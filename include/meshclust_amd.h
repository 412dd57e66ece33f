/*
 * meshclust_amd.h -- C-ABI of libmcgpu, the MI355X (gfx950) engine for MeShClust's
 * data-parallel hot path.  Plain pointers and sizes only; no C++ or torch types.
 *
 * MeShClust v1 has no plugin/FFI API: its hot path is reached through C++ template
 * seams inside one binary.  Each entry point below replaces one of those
 * seams; the reference interface it stands in for is cited as file:line relative to the
 * reference tree (src/...).  The host program (bin/meshclust, meshclust_amd/csrc/host)
 * restates the reference control flow and calls only these functions for the hot path.
 *
 * Conventions
 *   - every function returns MC_OK (0) or an MC_ERR_* code; mc_last_error() gives text.
 *     Nothing throws across the ABI.  Errors are loud: there is no CPU fallback.
 *   - point ids are the reference's ids: input order over all files (Runner.cpp:345-349).
 *   - one host thread per context; calls are synchronous at the ABI (HIP streams inside).
 *   - the caller owns every host array; the library owns device memory.
 */
#ifndef MESHCLUST_AMD_H
#define MESHCLUST_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MC_ABI_VERSION 1

#define MC_OK 0
#define MC_ERR_ARG 1     /* bad argument / shape                                  */
#define MC_ERR_HIP 2     /* HIP runtime or kernel failure                         */
#define MC_ERR_STATE 3   /* call made in the wrong order (e.g. no sequences yet)  */
#define MC_ERR_OOM 4     /* device allocation failed                              */
#define MC_ERR_INPUT 5   /* input the reference would reject (bad nucleotide ...) */
#define MC_ERR_UNSUPPORTED 6 /* this device path cannot take the request; use the step API  */
#define MC_ERR_TIMEOUT 7 /* a persistent kernel's hand-off deadline expired (a peer never answered) */

/* Feature flags and combo kinds: identical values to src/cluster/src/Feature.h:9-22. */
#define MC_FEAT_ALIGN (1 << 0)
#define MC_FEAT_LD (1 << 1)
#define MC_FEAT_MANHATTAN (1 << 2)
#define MC_FEAT_INTERSECTION (1 << 4)
#define MC_FEAT_PEARSON (1 << 5)
#define MC_FEAT_KULCZYNSKI2 (1 << 10)
#define MC_COMBO_SQUARED 1
#define MC_COMBO_SELF 2

#define MC_MAX_SINGLE 8
#define MC_MAX_COMBO 8
#define MC_MAX_COMBO_LEN 4

/*
 * Trained classifier = Feature<T> state after normalize()/finalize() plus the GLM weight
 * column (Feature.h:122-130, Trainer.h:45-46).  `lookup` is the single-feature order,
 * `combo_*` the products of Feature::operator() (Feature.h:69-88), `weights[0]` the
 * intercept and `weights[1+c]` the weight of combo c (Trainer.cpp:84-95).
 */
typedef struct mc_classifier {
  int32_t n_single;
  uint16_t lookup[MC_MAX_SINGLE];
  int32_t is_sim[MC_MAX_SINGLE];
  double mins[MC_MAX_SINGLE];
  double maxs[MC_MAX_SINGLE];
  int32_t n_combo;
  int32_t combo_kind[MC_MAX_COMBO];
  int32_t combo_len[MC_MAX_COMBO];
  int32_t combo_idx[MC_MAX_COMBO][MC_MAX_COMBO_LEN];
  double weights[MC_MAX_COMBO + 1];
} mc_classifier;

/* Result of one accumulation step (Trainer::get_close + ClusterFactory get_mean). */
typedef struct mc_scan_result {
  int32_t is_min;       /* get_close's is_min_r: no candidate classified similar      */
  int32_t has_best;     /* get<0>(result) != NULL (some combo-0 value > -1)            */
  uint64_t best_pos;    /* static position of the first maximum of combo 0            */
  double best_val;      /* that maximum                                                */
  uint64_t n_flagged;   /* candidates marked similar (removed from the window)         */
  uint32_t new_centre;  /* get_mean's argmin distance_d over the cluster (if !is_min)  */
  uint32_t n_members;   /* cluster size after this step                                */
  uint64_t nw_pairs;    /* alignment mode: NW alignments run for this step (else 0)    */
  uint64_t nw_cells;    /* alignment mode: their DP cells, sum of len1 * len2          */
} mc_scan_result;

typedef struct mc_ctx mc_ctx;

const char *mc_last_error(void);
int mc_abi_version(void);

/* Context on one GPU (hipSetDevice(device)); one process per GPU. */
int mc_ctx_create(int device, mc_ctx **out);
int mc_ctx_destroy(mc_ctx *ctx);

/*
 * Upload the encoded sequences.  codes: concatenation of every sequence's one-digit
 * string as ChromosomeOneDigit leaves it (0..3 inside segments, 'N' or the raw upper-case
 * byte outside; ChromosomeOneDigit.cpp:95-144).  seq_off[n+1] byte offsets.  seg: int32
 * pairs [start,end] (inclusive) per segment (Chromosome.cpp:162-258), seg_off[n+1] pair
 * offsets.  Replaces the Chromosome objects consumed by fill_table (ClusterFactory.h:40-55)
 * and by GlobAlignE through Point::get_data_str (Trainer.cpp:18-27).
 */
int mc_load_sequences(mc_ctx *ctx, const uint8_t *codes, const uint64_t *seq_off, uint64_t n,
                      const int32_t *seg, const uint64_t *seg_off);

/*
 * The same sequences in the form the host parser produces (meshclust_amd/csrc/host/fasta.cpp):
 * 2-bit codes, 16 bases per 32-bit word (base j of a record at bits 2*(j % 16) of word
 * pk_off[i] + j / 16; pk_off[i+1] - pk_off[i] = ceil(length_i / 16)), plus the nexc bytes that
 * are not 0..3 (the 'N' ChromosomeOneDigit leaves outside segments, ChromosomeOneDigit.cpp:
 * 122-144, or the raw bytes of a record without segments) at ascending global byte positions
 * exc_pos.  seq_off/seg/seg_off as for mc_load_sequences.  A quarter of the bytes cross PCIe;
 * the device keeps both the packed form (K1 input) and the expanded bytes (NW input).
 */
int mc_load_packed(mc_ctx *ctx, const uint32_t *packed, const uint64_t *pk_off, const uint64_t *seq_off, uint64_t n,
                   const uint64_t *exc_pos, const uint8_t *exc_val, uint64_t nexc, const int32_t *seg,
                   const uint64_t *seg_off);

/*
 * Largest k-mer count of the pseudocount-1 uint64 tables (Runner.cpp:57-67).  The pass also
 * writes the 8-bit histograms, so when the count fits 8 bits the following
 * mc_kmer_build(ctx, k, 1) costs nothing (K1 reads the sequences once).  1 <= k <= 12.
 */
int mc_kmer_max(mc_ctx *ctx, int k, uint64_t *largest);

/*
 * Device-resident histograms, pseudocount 1, of width 1/2/4/8 bytes, plus their
 * magnitudes (DivergencePoint mag incl. pseudocounts).  Replaces
 * ClusterFactory::get_divergence_point (ClusterFactory.cpp:989-1010) + KmerHashTable
 * wholesaleIncrement (KmerHashTable.cpp:193-223).
 */
int mc_kmer_build(mc_ctx *ctx, int k, int width_bytes);

/* Copy histograms (n * 4^k * width bytes, id order) and magnitudes to the host. */
int mc_get_histograms(mc_ctx *ctx, void *hist, uint64_t *mags);

/*
 * keys[p * m + i] = points[ids[i]]->distance(*points[pivots[p]])
 * (DivergencePoint::distance, DivergencePoint.cpp:68-81; used by Trainer::split's sort
 * comparators, Trainer.cpp:681-701).  Keys are <= 10000.
 */
int mc_distance_keys(mc_ctx *ctx, const uint32_t *pivots, uint32_t npiv, const uint32_t *ids,
                     uint64_t m, uint16_t *keys);

/*
 * Trainer::split's per-pivot sorts on the device (Trainer.cpp:691-701: std::sort of the
 * points by distance to each pivot, then reads of ~35 positions of each sorted array by the
 * alignment binary search, :703-721, and the sampler, :732-755).
 *   mc_split_begin: for pivot p, the array std::sort is called on is (key << 32 | id) over
 *     `order` (keys as mc_distance_keys); it stays in HBM.
 *   mc_split_select: ids[i] = the id std::sort (libstdc++ introsort, ties included) puts at
 *     position pos[i] of pivot arr[i]'s array; only the ranges holding the queried positions
 *     are partitioned, and the partitions persist for later calls.
 *   mc_split_begin_words / mc_split_select_words: the same on arbitrary word arrays compared
 *     by their upper 32 bits (depth < 0: std::sort's 2 floor(log2 n) limit), returning words.
 *   mc_split_end: ends the queries (the device buffers stay with the context for reuse).
 */
int mc_split_begin(mc_ctx *ctx, const uint32_t *pivots, uint32_t npiv, const uint32_t *order, uint64_t n);
int mc_split_begin_words(mc_ctx *ctx, const uint64_t *words, uint32_t narr, uint64_t n, int depth);
int mc_split_select(mc_ctx *ctx, uint64_t nq, const uint32_t *arr, const uint64_t *pos, uint32_t *ids);
int mc_split_select_words(mc_ctx *ctx, uint64_t nq, const uint32_t *arr, const uint64_t *pos, uint64_t *words);
int mc_split_end(mc_ctx *ctx);

/*
 * raw[i * nflag + f] = Feature<T>::raw(flags[f], *points[a[i]], *points[b[i]])
 * (Feature.cpp:117-160) for the k-mer features LD/MANHATTAN/INTERSECTION/PEARSON/
 * KULCZYNSKI2.  Used by Feature::normalize (Feature.cpp:86-114).
 */
int mc_pair_features(mc_ctx *ctx, const uint32_t *a, const uint32_t *b, uint64_t m,
                     const uint16_t *flags, int nflag, double *raw);

/* Install the trained classifier used by every classify/scan/mean-shift call. */
int mc_set_classifier(mc_ctx *ctx, const mc_classifier *cls);

/*
 * For each pair i: cache = feat->compute(*points[a[i]], *points[b[i]]); sum = w0 + fma
 * chain over combos; similar = round(1/(1+exp(-sum))) == 1.  Replaces the per-pair body
 * of Trainer::merge (Trainer.cpp:129-157), filter (:334-349) and generate_feat_mat
 * (:367-414).  Any output pointer may be NULL.
 */
int mc_classify_pairs(mc_ctx *ctx, const uint32_t *a, const uint32_t *b, uint64_t m,
                      uint8_t *similar, double *combo0, double *sum);

/*
 * Batched utility::GlobAlignE(seqA,0,la-1,seqB,0,lb-1,1,-1,2,1).getIdentity() on the loaded
 * sequences (GlobAlignE.cpp:123-305; called by Trainer::align, Trainer.cpp:15-31, and
 * Feature::align, Feature.cpp:221-243).  len/ids may be NULL.
 */
int mc_nw_identity(mc_ctx *ctx, const uint32_t *a, const uint32_t *b, uint64_t m, double *ident,
                   int32_t *len, int32_t *ids);

/* The same on caller-provided byte strings (no loaded sequences needed). */
int mc_nw_identity_raw(mc_ctx *ctx, const uint8_t *a, const uint64_t *a_off, const uint8_t *b,
                       const uint64_t *b_off, uint64_t m, double *ident, int32_t *len,
                       int32_t *ids, int32_t *score);

/*
 * Accumulation (ClusterFactory::accumulate, ClusterFactory.cpp:637-714).
 * The bvec of Runner.cpp:342-350 is only ever shrunk after insert_finalize, so the device
 * holds one static candidate order (bin-major, length-sorted within bins) plus an alive
 * mask.  order[pos] = point id.
 */
int mc_set_order(mc_ctx *ctx, const uint32_t *order, uint64_t n);
/* bvec::pop / bvec::erase of one static position (bvec.cpp:95-106, 349-353). */
int mc_kill(mc_ctx *ctx, uint64_t pos);
/* Start a new cluster whose member list is {first} (accumulate's `current = {last}`). */
int mc_cluster_begin(mc_ctx *ctx, uint32_t first_id);
/*
 * One get_close step (Trainer.cpp:34-114) of centre `centre_id` over the alive static
 * positions S..E (inclusive; the bvec_iterator range of ClusterFactory.cpp:650-654), then,
 * if some candidate was similar, bvec::remove_available (bvec.cpp:289-318) + get_mean
 * (ClusterFactory.cpp:382-425).  flagged_pos receives the removed static positions in
 * ascending (bvec) order; cap is its capacity.
 */
int mc_scan(mc_ctx *ctx, uint32_t centre_id, uint64_t S, uint64_t E, uint32_t *flagged_pos,
            uint64_t cap, mc_scan_result *res);

/*
 * One get_close step sharded by record over `nparts` GPUs (Trainer.cpp:34-114
 * is an OpenMP loop over the window, ClusterFactory.cpp:650-654).  Every rank holds the same
 * bvec state; rank `part` scans only the alive positions of S..E in its static blocks: block
 * b = [b * MC_SHARD_BLOCK, (b + 1) * MC_SHARD_BLOCK) belongs to part b % nparts.  Nothing is
 * removed: flagged_pos receives this part's similar candidates (ascending); res holds this
 * part's is_min / has_best / best_pos / best_val / n_flagged.  The ranks then combine the
 * parts (is_min AND, first maximum = largest best_val, ties to the lowest best_pos, flagged
 * lists merged) and all call mc_scan_commit with the union.  8/16-bit histograms, k-mer
 * classifier (else MC_ERR_UNSUPPORTED).
 */
#define MC_SHARD_BLOCK 256
int mc_scan_part(mc_ctx *ctx, uint32_t centre_id, uint64_t S, uint64_t E, uint32_t part, uint32_t nparts,
                 uint32_t *flagged_pos, uint64_t cap, mc_scan_result *res);
/*
 * Second half of a sharded step: bvec::remove_available (bvec.cpp:289-318) of the union of
 * every part's flagged positions (ascending, n may be 0) and get_mean (ClusterFactory.cpp:
 * 382-425) over the grown cluster: res->new_centre, res->n_members, res->is_min = (n == 0).
 */
int mc_scan_commit(mc_ctx *ctx, const uint32_t *flagged_pos, uint64_t n, mc_scan_result *res);

/*
 * Alignment mode (--align, or an identity below 0.6: Runner.cpp:231-236), a get_close step's
 * Feature::align(*pt, *p) values (Feature.cpp:221-243; Trainer.cpp:34-114's OpenMP loop over
 * the window) sharded over `nparts` ranks: of the alive static positions of S..E in ascending
 * order, candidate i is aligned (GlobAlignE, the candidate as seq1, the centre as seq2) by part
 * i % nparts.  ident[0 .. *n_part) receives this part's identities in candidate order (cap: its
 * capacity); *pairs / *cells count the WHOLE window's alignments (the same on every part).
 * Nothing changes on the context.
 */
int mc_align_part(mc_ctx *ctx, uint32_t centre_id, uint64_t S, uint64_t E, uint32_t part, uint32_t nparts,
                  double *ident, uint64_t cap, uint64_t *n_part, uint64_t *pairs, uint64_t *cells);
/*
 * The rest of mc_scan's alignment-mode step with the identities given: ident[i] is
 * Feature::align of the window's i-th alive candidate (ascending static position, as the
 * parts of mc_align_part interleave back).  Flags, removes and re-centres exactly as mc_scan;
 * res->nw_pairs / nw_cells are 0 (mc_align_part counted them).
 */
int mc_scan_ident(mc_ctx *ctx, uint32_t centre_id, uint64_t S, uint64_t E, const double *ident,
                  uint32_t *flagged_pos, uint64_t cap, mc_scan_result *res);

/*
 * The whole accumulation phase on the device: ClusterFactory::MS's loop
 * `last = points.pop(); while (last) accumulate(&last, ...)` (ClusterFactory.cpp:717-730,
 * accumulate :637-714) run by one persistent kernel, bvec included -- no host round trip per
 * get_close step.  Call after mc_set_order on the fresh bvec: bin b holds the static
 * positions [bin_lo[b], bin_lo[b+1]) (bin_lo[nbins] = n) and bounds[b] is its begin bound
 * (bvec.cpp:9-24, 208-218).  sim is --id.  Output: *nclusters clusters in creation order;
 * cluster c has centre centre_ids[c] and members member_ids[member_off[c] ..
 * member_off[c+1]) in the reference's `current` order.  stats (may be NULL, else 5 entries)
 * receives {get_close steps, sum of window sizes, then the device controller's time in us:
 * bvec window + publish, waiting for the scanning workgroups, collect + get_mean}.  Returns MC_ERR_UNSUPPORTED when this bvec does not
 * fit the device controller (alignment mode, 32/64-bit histograms, very large n); the caller
 * then drives accumulation with mc_scan.
 */
int mc_accumulate(mc_ctx *ctx, const uint32_t *bin_lo, const uint64_t *bounds, uint32_t nbins, double sim,
                  uint32_t *centre_ids, uint64_t *member_off, uint32_t *member_ids, uint64_t *nclusters,
                  uint64_t *stats);

/*
 * One accumulation shared by `world` ranks, one GPU each (the loop of
 * ClusterFactory.cpp:717-730 whose get_close steps, Trainer.cpp:81-106, are split by record).
 * Every rank registers the same host-memory mailbox of mc_mailbox_bytes(world, n) zeroed bytes
 * (a POSIX shared-memory segment mapped by each rank's process, or one buffer shared by the
 * threads of one process) with mc_set_mailbox, after mc_set_order; then all ranks call
 * mc_accumulate with identical arguments.  Each rank's persistent kernel scans only its
 * interleaved tiles of every window (tile t of the static order belongs to rank t mod world);
 * per step the kernels exchange {first maximum of combo 0, flagged positions} through the
 * mailbox without the host, and every rank applies the same remove_available + get_mean, so
 * every rank returns the same partition as a single-rank run.  A rank that fails stops the
 * others after the exchange's deadline (MC_ERR_TIMEOUT).  world 0 detaches.
 */
uint64_t mc_mailbox_bytes(int world, uint64_t n);
/* share: how many ranks' kernels run on this rank's GPU (>= 1; each then takes that share of
   the CUs, so they are co-resident: tests put two ranks on one GPU) */
int mc_set_mailbox(mc_ctx *ctx, void *host, uint64_t bytes, int rank, int world, int share);
/* the PCI bus id of the context's GPU (ranks sharing a GPU find each other with it) */
int mc_ctx_pci_bus_id(mc_ctx *ctx, char *buf, int len);
/*
 * The accumulation kernel's plan for this context and bvec (call after mc_set_order and
 * mc_set_mailbox): info[0] workgroups, info[1] static positions per tile of ownership (every
 * rank sharing a mailbox must use the same tile: tile t belongs to rank t mod world), info[2]
 * flags {1 dense resident workers, 2 wide rows, 4 resident rows, 8 streaming rows}, info[3]
 * the dynamic LDS bytes.  MC_ERR_UNSUPPORTED when mc_accumulate would not take it.
 * mc_set_accum_grid caps the workgroups (0: one per CU, or the CU share of the ranks on this
 * GPU): ranks sharing a mailbox take the smallest grid among them, so each derives the same plan.
 */
int mc_accum_plan_info(mc_ctx *ctx, uint32_t nbins, uint32_t info[4]);
int mc_set_accum_grid(mc_ctx *ctx, uint32_t grid);
/*
 * Allocate now every device buffer mc_accumulate needs for this bvec (call after
 * mc_set_accum_grid): mc_accumulate then allocates and frees nothing.  Ranks that share one
 * GPU in one process call it before a common barrier, so that no rank's hipFree -- which waits
 * for the whole device -- runs while a peer's persistent kernel spins on this rank's step
 * records (the Trainer.cpp:81-106 loop split by record).
 */
int mc_accum_reserve(mc_ctx *ctx, uint32_t nbins);
/*
 * Confine the context to slot `slot` of `share` disjoint CU sets of its GPU (ranks sharing one
 * GPU: the one-GPU rehearsal of the record-sharded loops, ClusterFactory.cpp:744-749 and
 * Trainer.cpp:81-106).  The context's stream is re-created with a CU mask (a hardware queue of
 * its own), so every kernel of the rank -- the persistent accumulation grid included, sized to
 * the mask -- runs on those CUs only and never waits behind a peer rank's spinning kernel.
 * share 1 restores the whole GPU.  Call while the context is idle.
 */
int mc_ctx_partition(mc_ctx *ctx, int slot, int share);

/*
 * One mean-shift iteration over all centres (the omp parallel for of ClusterFactory.cpp:
 * 744-749 around mean_shift_update, :289-380): for centre j, the members of clusters
 * j-delta..j+delta (CSR member_off[C+1]/members, cluster order) are filtered by the
 * classifier (Trainer::filter) and the first member closest (distance_d) to their mean
 * becomes new_centre[j] (Trainer::closest, Trainer.cpp:351-365); unchanged if none pass.
 */
int mc_mean_shift(mc_ctx *ctx, const uint32_t *centre_ids, uint32_t C, const uint64_t *member_off,
                  const uint32_t *members, int delta, uint32_t *new_centre);

/*
 * One iteration of MS's update loop (ClusterFactory.cpp:740-760) in one device round trip:
 * mc_mean_shift over all centres, then the classifier pairs of merge (ClusterFactory.cpp:
 * 427-493, Trainer::merge Trainer.cpp:129-157) over the NEW centres: for i in [0, C) and t in
 * (i, min(C-1, i+delta)], pair q (i-major, t ascending) = feat->compute(new_centre[t],
 * new_centre[i]); similar[q] / combo0[q] as mc_classify_pairs.  *npairs receives the pair
 * count (sum over i of min(delta, C-1-i)); similar and combo0 need room for it.
 */
int mc_update_iteration(mc_ctx *ctx, const uint32_t *centre_ids, uint32_t C, const uint64_t *member_off,
                        const uint32_t *members, int delta, uint32_t *new_centre, uint8_t *similar,
                        double *combo0, uint64_t *npairs);

/*
 * The same for centres j0 <= j < j1 only (new_centre holds j1 - j0 entries): the per-rank
 * share of one iteration when the update is sharded over GPUs by centre; the ranks then
 * all-gather the new centres (the centre-reassignment exchange).
 */
int mc_mean_shift_range(mc_ctx *ctx, const uint32_t *centre_ids, uint32_t C, const uint64_t *member_off,
                        const uint32_t *members, int delta, uint32_t j0, uint32_t j1, uint32_t *new_centre);

/*
 * ---- alignment mode (--align, or --id < 0.6: Runner.cpp:32-34, 332) ---------------------
 * The trainer then installs a classifier whose only feature is MC_FEAT_ALIGN (identity of
 * utility::GlobAlignE, normalised with min 0 / max 1, weights {-cutoff, 1}; Trainer.cpp:
 * 570-577, Feature.cpp:90-95).  With such a classifier:
 *   - mc_scan runs the batched NW kernel of every alive window candidate (seq1) against the
 *     centre (seq2) -- Feature::align(*pt, *p) inside Trainer::get_close -- and classifies
 *     the identities; remove_available + get_mean are unchanged (k-mer histograms).
 *   - mc_classify_pairs / mc_mean_shift are not available (their pairs go through the
 *     reference's Feature::align memo, which the host replays): use mc_nw_identity +
 *     mc_classify_values + mc_mean_shift_select instead.
 */

/*
 * Classify precomputed single-feature values: raw[i * n_single + f] is feature lookup[f] of
 * pair i (Feature::compute_all_raw, Feature.cpp:54-84).  Same normalisation, combos, fma GLM
 * sum and decision as mc_classify_pairs.  Any output pointer may be NULL.
 */
int mc_classify_values(mc_ctx *ctx, const double *raw, uint64_t m, uint8_t *similar, double *combo0,
                       double *sum);

/*
 * mean_shift_update (ClusterFactory.cpp:289-380) with the Trainer::filter decision supplied
 * by the caller: for centre j the neighbourhood is members[member_off[b_j] .. member_off[e_j+1])
 * (b_j = max(0, j-delta), e_j = min(C-1, j+delta)); keep holds one byte per neighbourhood
 * entry, neighbourhoods concatenated in j order.  new_centre[j] = the first kept member
 * closest (distance_d) to the kept members' mean, or centre_ids[j] if none is kept.
 */
int mc_mean_shift_select(mc_ctx *ctx, const uint32_t *centre_ids, uint32_t C, const uint64_t *member_off,
                         const uint32_t *members, int delta, const uint8_t *keep, uint32_t *new_centre);

/*
 * ---- ranks sharing one clustering --------------------------------------
 * The reference runs on one host (OpenMP); here one process (or thread) per GPU shares a
 * clustering.  mc_comm is an RCCL communicator (librccl opened at run time) whose only
 * operation is an all-gather of equal host blocks in rank order, staged through the rank's
 * GPU and carried by RCCL over xGMI.  Rank 0 makes the id, the caller distributes it (e.g.
 * torch.distributed broadcast), every rank calls mc_comm_create (it blocks until all joined).
 * mc_comm_allgather's signature is the host driver's exchange callback
 * (mcl_run_sharded(..., allgather = mc_comm_allgather, user = comm)).
 */
typedef struct mc_comm mc_comm;
#define MC_COMM_ID_BYTES 128
int mc_comm_unique_id(uint8_t *id /* MC_COMM_ID_BYTES */);
int mc_comm_create(int device, int rank, int world, const uint8_t *id, mc_comm **out);
int mc_comm_allgather(mc_comm *comm, const void *in, uint64_t bytes, void *out /* world * bytes */);
int mc_comm_stats(const mc_comm *comm, uint64_t *calls, uint64_t *bytes);
/* abort != 0: ncclCommAbort (a peer failed), else ncclCommDestroy. */
int mc_comm_destroy(mc_comm *comm, int abort);

/* Wait for all work on the context's GPU (every stream; benchmark boundaries). */
int mc_sync(mc_ctx *ctx);

/* Device time (ms) and launches accumulated per kernel family since the last reset
   (diagnostics): ms_out[2f], ms_out[2f+1] for f = k-mer, keys, pairs, scan, finalize,
   mean shift, NW, static layout. */
int mc_timers(mc_ctx *ctx, double *ms_out, int n, int reset);

#ifdef __cplusplus
}
#endif
#endif
