// nw.hip -- K3: batched global alignment identity, bit-exact with utility::GlobAlignE
// (src/utility/GlobAlignE.cpp:123-305; Gotoh affine gaps, match 1 / mismatch -1 / open 2 /
// extend 1, each DP state carrying (score, path length, identities)).
//
// One wavefront per pair, anti-diagonal wavefront over the DP matrix: lane l owns R
// consecutive rows of seq1 and sweeps the columns of seq2 one step behind lane l-1, so at
// step t it computes column t-l+1 for its R rows.  The bottom row of lane l-1 (M, X, Y and
// their payloads) and the seq2 code travel down the wave through one DPP lane shift per value
// and step; nothing but that hand-off leaves registers.  Every move adds 1 to GlobAlignE's path
// length and a diagonal move consumes a base of each sequence, a gap move one base, so a
// path ending at (i, j) has length i + j - (diagonal moves).  A state therefore carries the
// diagonal count and the identity count packed in one payload word (diag << 16 | ids, or
// 32/32 bits for long pairs): a predecessor choice moves both with one select, a gap move
// leaves the payload unchanged, and the final length is la + lb - diag.  Sequences longer than 64*R rows are cut
// into row blocks whose boundary row is kept in global scratch.
//
// Recurrences (rows i over seq1, columns j over seq2; GlobAlignE's names in brackets):
//   Y(i,j) [upperGap] = max(M(i,j-1) - (o+e), Y(i,j-1) - e)          ties: from M
//   M(i,j) [matches]  = max(M, X, Y at (i-1,j-1)) + s(i,j)           ties: M, then X, then Y
//   X(i,j) [lowerGap] = max(M(i-1,j) - (o+e), X(i-1,j) - e)          ties: from M
// with the reference's finite "-infinity" and boundary rows/columns (:125-170, :250-256).
//
// The kernels keep every state as T = score + i + j.  Each comparison above is between values
// of one cell (the three states of (i-1,j-1), of (i,j-1) or of (i-1,j), or of (la,lb) at the
// end), so a per-cell offset changes no decision; in T the recurrences read
//   Y = max(M - (o+e-1), Y + (1-e)),  X likewise,  M = max3 + s + 2,
// and with e = 1 a gap extension adds nothing: one VALU instruction less per state and cell.
// The score is T(la,lb) - (la + lb).
#include <algorithm>

#include "mcgpu.hpp"

namespace mcg {

namespace {

constexpr int GO = 2, GE = 1, MATCH = 1, MISMATCH = -1;
// the same moves in T = score + i + j (see above)
constexpr int OPEN_T = GO + GE - 1, EXT_T = 1 - GE, MATCH_T = MATCH + 2, MISMATCH_T = MISMATCH + 2;
// M is kept as M - MOFF (T - OPEN_T): both gap recurrences then compare a stored value with a
// stored value, and only the diagonal's comparison offsets max(X, Y) -- one VALU instruction less
// per cell (see the cell loop)
constexpr int MOFF = OPEN_T;

template <typename P>
struct Pack;
template <>
struct Pack<uint32_t> {
  static constexpr int SH = 16;
};
template <>
struct Pack<uint64_t> {
  static constexpr int SH = 32;
};

// Lane l receives lane l-1's value (DPP wave_shr:1, a VALU move; lane 0's result is
// unspecified and always overwritten by the callers).
__device__ __forceinline__ int dpp_shr1(int v) { return __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, false); }
template <typename P>
__device__ __forceinline__ P dshr(P v) {
  if constexpr (sizeof(P) == 4) {
    return (P)(uint32_t)dpp_shr1((int)v);
  } else {
    const uint32_t lo = (uint32_t)dpp_shr1((int)(uint32_t)v), hi = (uint32_t)dpp_shr1((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
  }
}

struct NWPairs {
  const uint8_t *A;
  const uint64_t *aoff;
  const uint32_t *ai;
  const uint8_t *Bq;
  const uint64_t *boff;
  const uint32_t *bi;
  const uint32_t *pidx;   // pair indices handled by this launch
  uint32_t npairs;
  int *bnd;               // boundary scratch (multi-block pairs)
  const uint64_t *bnd_off;  // per launch-slot offset into bnd (in ints)
  double *ident;
  int32_t *len;
  int32_t *ids;
  int32_t *score;
  const uint32_t *out;  // optional result slot per pair (else the pair index)
  // chained row blocks (CH): one single-wave workgroup per (pair, row block); work item i is
  // pair pidx[i], block pblk[i], items of a pair consecutive in block order; a workgroup takes
  // the next item from *ctr, so every block's predecessor was dispatched before it
  const uint16_t *pblk;
  uint32_t *ctr;
  uint64_t *cbuf;        // tagged granules: column j of a block's bottom row at 6 j .. 6 j + 5,
                         // {j << 32 | value} for M, X, Y and their payloads
  const uint64_t *cin;   // per item: granule offset of the block above's bottom row (~0: none)
  const uint64_t *cout;  // per item: granule offset of this block's bottom row (~0: last block)
  int *err;              // a hand-off that never arrived (20 s)
};

// ---------------------------------------------------------------------------------------
// One kernel, two launch forms.  A pair per workgroup of W waves: wave w owns rows
// [w*64*R, (w+1)*64*R) of each row block and runs 64 + KLAG steps behind wave w-1; lane 63 of
// wave w-1 leaves its bottom row for column j in an LDS ring that lane 0 of wave w reads
// KLAG + 1 steps later.  A workgroup barrier every KLAG steps orders those writes and reads (a
// slot is rewritten RING_C columns later, with a barrier in between).  Inside a wave the
// bottom row moves down by one lane per step with DPP wave_shr:1 (a VALU move, no LDS round
// trip).
//  * throughput form (many pairs: the label batch, the --align window scans): W = 1, a wave
//    per pair, R = 4 / 8 / 16 rows per lane, no LDS;
//  * latency form (< 1,024 pairs: the sampler's dependent rounds): W = 4 / 8 / 16 waves.
// The steady-state steps (every lane inside the matrix) run unrolled by two with no per-lane
// branches, so the state registers of consecutive steps alternate instead of being copied
// back: 18 VALU instructions per cell at R = 16 against 26.5 for the earlier single-wave
// kernel, whose loop-carried state cost ~90 v_mov per step.
constexpr int KLAG = 16, RING_C = 64;
struct GenStep {  // tags of the step variants
  static constexpr bool value = true;
};
struct SteadyStep {
  static constexpr bool value = false;
};


// CH (chained row blocks): a single-wave workgroup computes ONE row block of its pair (64 R
// rows), concurrently with the pair's other blocks in other workgroups.  The block above's
// bottom row arrives as tagged granules in global memory, 64 columns per batch: lane l loads
// column 64 m + 1 + l of batch m one batch ahead, checks the tags when the batch comes due
// (spinning only if the block above is behind) and lane 0 takes column t + 1 at step t with a
// readlane -- where the seq2 codes come from too -- so the hand-in costs no LDS, no barrier and
// no per-step load.  Lane 63 leaves this block's bottom row in LDS, a column per step; every
// 64 columns the wave stores them as granules, a column per lane.
template <int R, typename P, int W, bool CH = false>
__global__ __launch_bounds__(64 * W) void nw_mw_kernel(NWPairs q) {
  static_assert(!CH || (W == 1 && sizeof(P) == 4), "chained blocks: one wave, 32-bit payloads");
  constexpr int SH = Pack<P>::SH;
  constexpr P LEN1 = (P)1 << SH;
  constexpr int ROWS = 64 * R * W;  // rows per block
  __shared__ int rM[RING_C][W], rX[RING_C][W], rY[RING_C][W];
  __shared__ P rMP[RING_C][W], rXP[RING_C][W], rYP[RING_C][W];
  __shared__ int s_out[CH ? 6 : 1][64];  // CH: this block's bottom row, the current 64 columns
  uint32_t slot = blockIdx.x;
  if constexpr (CH) {
    uint32_t v = 0;
    if (threadIdx.x == 0) v = atomicAdd(q.ctr, 1u);
    slot = (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
  }
  if (slot >= q.npairs) return;
  const uint32_t p = q.pidx[slot];
  const uint8_t *a = q.A + q.aoff[q.ai[p]];
  const int la = (int)(q.aoff[q.ai[p] + 1] - q.aoff[q.ai[p]]);
  const uint8_t *b = q.Bq + q.boff[q.bi[p]];
  const int lb = (int)(q.boff[q.bi[p] + 1] - q.boff[q.bi[p]]);
  const int lane = threadIdx.x & 63, w = wave_id(), gl = (int)threadIdx.x;
  const int len1 = la + 1, len2 = lb + 1;
  const int shorter = (len2 < len1 ? len2 : len1) - 1;
  const int lenDiff = len2 > len1 ? len2 - len1 : len1 - len2;
  int maxDiff = 0;
  if (lenDiff >= 1) maxDiff += -GO - lenDiff * GE;
  maxDiff += MISMATCH * shorter - 1;
  const int NINF = maxDiff;
  int *bnd = q.bnd ? q.bnd + q.bnd_off[slot] : nullptr;  // 6 ints per column, columns 0..lb
  const int nblk = (la + ROWS - 1) / ROWS;
  int fin_score = 0;
  P fin_pay = 0;
  const int blk_first = CH ? (int)q.pblk[slot] : 0, blk_end = CH ? blk_first + 1 : (nblk > 0 ? nblk : 1);
  for (int blk = blk_first; blk < blk_end; blk++) {
    const int itop = blk * ROWS + gl * R + 1;  // first row of this lane
    uint8_t ac[R];
    int M[R], X[R], Y[R];
    P MP[R], XP[R], YP[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int i = itop + r;
      ac[r] = i <= la ? a[i - 1] : (uint8_t)0xFF;
      M[r] = NINF + i - MOFF;  // column 0 (GlobAlignE.cpp:140-160), T = score + i
      Y[r] = NINF + i;
      X[r] = -GO - i * GE + i;
      MP[r] = XP[r] = YP[r] = 0;  // i gap moves, no diagonal
    }
    int dM, dX, dY;
    P dMP, dXP, dYP;
    {
      const int i = itop - 1;
      if (i == 0) {
        dM = -MOFF;
        dX = NINF;
        dY = -GO;
        dMP = dXP = dYP = 0;
      } else {
        dM = NINF + i - MOFF;
        dX = -GO - i * GE + i;
        dY = NINF + i;
        dMP = dXP = dYP = 0;
      }
    }
    int oM = NINF, oX = NINF, oY = NINF;
    P oMP = 0, oXP = 0, oYP = 0;
    int ob = 0;
    const int lagw = w * (64 + KLAG);
    const int steps = lb + 63 + (W - 1) * (64 + KLAG);
    int bcur = 0, bnext = lane < lb ? b[lane] : 0;  // seq2 codes for lane 0: one 64-byte block per 64 steps, lane l holding byte l, loaded a block ahead and read with a uniform readlane
    // lane 0's hand-in for its next column, loaded one step ahead so the LDS / global latency
    // hides behind a step of cell updates (the slot was written >= KLAG steps earlier, with a
    // barrier in between, see above)
    int nM = NINF, nX = NINF, nY = NINF;
    P nMP = 0, nXP = 0, nYP = 0;
    auto fetch = [&](int jn) {
      if (CH || lane != 0 || jn < 1 || jn > lb) return;
      if (w > 0) {
        const int sl = jn % RING_C;
        nM = rM[sl][w];
        nX = rX[sl][w];
        nY = rY[sl][w];
        nMP = rMP[sl][w];
        nXP = rXP[sl][w];
        nYP = rYP[sl][w];
      } else if (blk > 0) {
        const int *sb = bnd + 6 * jn;
        nM = sb[0];
        nX = sb[1];
        nY = sb[2];
        nMP = (P)(uint32_t)sb[3];
        nXP = (P)(uint32_t)sb[4];
        nYP = (P)(uint32_t)sb[5];
        if constexpr (sizeof(P) == 8) {
          const int *s2 = bnd + 6 * (lb + 1) + 6 * jn;
          nMP |= (P)(uint32_t)s2[3] << 32;
          nXP |= (P)(uint32_t)s2[4] << 32;
          nYP |= (P)(uint32_t)s2[5] << 32;
        }
      }
    };
    fetch(1 - lagw);
    // CH: the block above's bottom row in batches of 64 columns (see the kernel's comment):
    // hv = the current batch's values (lane l: column 64 m + 1 + l), gn = the next batch's
    // granules in flight
    const uint64_t *cin = nullptr;
    // (this block's bottom row out: the pointer formed once -- read from q inside the loop, the
    // atomic stores beside it, which may alias q's arrays, would make it a global load per step)
    uint64_t *cout = nullptr;
    uint32_t hv[6] = {0, 0, 0, 0, 0, 0};
    uint64_t gn[6] = {0, 0, 0, 0, 0, 0};
    bool failed = false;
    uint64_t t0 = 0;
    auto gload = [&](int c) {
#pragma unroll
      for (int v = 0; v < 6; v++)
        gn[v] = __hip_atomic_load(const_cast<uint64_t *>(cin + 6 * (uint64_t)c + v), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
    };
    if constexpr (CH) {
      if (q.cout[slot] != ~0ull) cout = q.cbuf + q.cout[slot];
      if (q.cin[slot] != ~0ull) {
        cin = q.cbuf + q.cin[slot];
        t0 = __builtin_amdgcn_s_memrealtime();
        if (1 + lane <= lb) gload(1 + lane);
      }
    }
    // batch m comes due at step 64 m: its tags checked (a lane whose column the block above has
    // not written yet reloads it, a short sleep between tries; 20 s without it: the launch's
    // error word, garbage values), then batch m + 1's loads issued
    auto take_batch = [&](int idx) {
      const int c = idx + 1 + lane;
      const bool need = c <= lb;
      for (uint32_t it = 1;; it++) {
        bool ok = true;
#pragma unroll
        for (int v = 0; v < 6; v++) ok = ok && (uint32_t)(gn[v] >> 32) == (uint32_t)c;
        ok = ok || !need;
        if (__ballot(!ok) == 0) break;
        if (failed || ((it & 255) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > 2000000000ull)) {
          if (!failed && lane == 0) atomicOr(q.err, 1);
          failed = true;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
        if (!ok) gload(c);
      }
#pragma unroll
      for (int v = 0; v < 6; v++) hv[v] = (uint32_t)gn[v];
      if (c + 64 <= lb) gload(c + 64);
    };
    const bool row0 = w == 0 && blk == 0;  // lane 0's upper neighbour is GlobAlignE's row 0
    // One step of this wave.  GEN: the general form (ramp-up / ramp-down: lanes outside
    // 1 <= j <= lb idle).  Steady state (every lane inside, lb >= 64): no per-lane branches --
    // lane 0's hand-in is a select and its prefetch a broadcast LDS read of a uniform slot.
    auto step = [&](int t, auto gen_tag) {
      constexpr bool GEN = decltype(gen_tag)::value;
      const int j = t - lane - lagw + 1;  // column of this lane at this step
      const int idx = t - lagw;           // lane 0 reads seq2[idx]
      if ((!GEN || idx >= 0) && (idx & 63) == 0) {
        bcur = bnext;
        const int nx = idx + 64 + lane;
        bnext = nx < lb ? b[nx] : 0;
      }
      const int b0 = __builtin_amdgcn_readlane(bcur, idx & 63);
      if constexpr (CH) {
        if (cin) {  // lane 0's hand-in for column idx + 1 (uniform: cin, idx)
          if ((idx & 63) == 0) take_batch(idx);
          nM = __builtin_amdgcn_readlane((int)hv[0], idx & 63);
          nX = __builtin_amdgcn_readlane((int)hv[1], idx & 63);
          nY = __builtin_amdgcn_readlane((int)hv[2], idx & 63);
          nMP = (P)(uint32_t)__builtin_amdgcn_readlane((int)hv[3], idx & 63);
          nXP = (P)(uint32_t)__builtin_amdgcn_readlane((int)hv[4], idx & 63);
          nYP = (P)(uint32_t)__builtin_amdgcn_readlane((int)hv[5], idx & 63);
        }
      }
      int uM = dpp_shr1(oM), uX = dpp_shr1(oX), uY = dpp_shr1(oY);
      P uMP = dshr<P>(oMP), uXP = dshr<P>(oXP), uYP = dshr<P>(oYP);
      int bc = dpp_shr1(ob);
      if constexpr (GEN) {
        if (lane == 0) {
          bc = (j >= 1 && j <= lb) ? b0 : 0;
          if (j >= 1 && j <= lb) {
            if (row0) {  // row 0: M = X = -inf, Y = -o - j*e, lengths j (T: + j)
              uM = NINF + j - MOFF;
              uX = NINF + j;
              uY = -GO - j * GE + j;
              uMP = uXP = uYP = 0;
            } else {  // bottom row of wave w-1 (or of the previous row block) at column j
              uM = nM;
              uX = nX;
              uY = nY;
              uMP = nMP;
              uXP = nXP;
              uYP = nYP;
            }
          }
        }
        fetch(j + 1);
      } else {
        const bool l0 = lane == 0;
        bc = l0 ? b0 : bc;
        const int hM = row0 ? NINF + j - MOFF : nM, hX = row0 ? NINF + j : nX, hY = row0 ? -GO - j * GE + j : nY;
        const P hMP = row0 ? (P)0 : nMP, hXP = row0 ? (P)0 : nXP, hYP = row0 ? (P)0 : nYP;
        uM = l0 ? hM : uM;
        uX = l0 ? hX : uX;
        uY = l0 ? hY : uY;
        uMP = l0 ? hMP : uMP;
        uXP = l0 ? hXP : uXP;
        uYP = l0 ? hYP : uYP;
        const int jn = idx + 2;  // lane 0's next column (uniform)
        if (CH) {
        } else if (w > 0) {
          const int sl = jn % RING_C;
          nM = rM[sl][w];
          nX = rX[sl][w];
          nY = rY[sl][w];
          nMP = rMP[sl][w];
          nXP = rXP[sl][w];
          nYP = rYP[sl][w];
        } else if (blk > 0 && jn <= lb) {
          const int *sb = bnd + 6 * jn;
          nM = sb[0];
          nX = sb[1];
          nY = sb[2];
          nMP = (P)(uint32_t)sb[3];
          nXP = (P)(uint32_t)sb[4];
          nYP = (P)(uint32_t)sb[5];
          if constexpr (sizeof(P) == 8) {
            const int *s2 = bnd + 6 * (lb + 1) + 6 * jn;
            nMP |= (P)(uint32_t)s2[3] << 32;
            nXP |= (P)(uint32_t)s2[4] << 32;
            nYP |= (P)(uint32_t)s2[5] << 32;
          }
        }
      }
      if (!GEN || (j >= 1 && j <= lb)) {
        int aM = uM, aX = uX;
        P aMP = uMP, aXP = uXP;
        int gM = dM, gX = dX, gY = dY;
        P gMP = dMP, gXP = dXP, gYP = dYP;
#pragma unroll
        for (int r = 0; r < R; r++) {
          const int pM = M[r], pX = X[r], pY = Y[r];
          const P pMP = MP[r], pXP = XP[r], pYP = YP[r];
          // (M values are M - MOFF: pM, gM, aM below)
          const int yb = pM, yc = pY + EXT_T;  // upperGap (GlobAlignE.cpp:233-251): M - (o+e-1) vs Y
          const bool yFromM = yb >= yc;
          Y[r] = yFromM ? yb : yc;
          YP[r] = yFromM ? pMP : pYP;
          const bool hit = ac[r] == (uint8_t)bc;  // matches (:255-299)
          const int sc = hit ? MATCH_T : MISMATCH_T;
          // M on ties, then X, then Y: M iff M >= max(X, Y), else X iff X >= Y -- with gM = M -
          // MOFF: gM >= max(X, Y) - MOFF, and the new M - MOFF = max(gM, max(X, Y) - MOFF) + sc
          const bool xy = gX >= gY;
          const int mxy = xy ? gX : gY;
          const P pxy = xy ? gXP : gYP;
          const int m2 = mxy - MOFF;
          const bool fromM = gM >= m2;
          const int best = fromM ? gM : m2;
          const P bestP = fromM ? gMP : pxy;
          M[r] = best + sc;
          MP[r] = bestP + LEN1 + (hit ? (P)1 : (P)0);
          const int xb = aM, xc = aX + EXT_T;  // lowerGap (:316-330): M - (o+e-1) vs X
          const bool xFromM = xb >= xc;
          X[r] = xFromM ? xb : xc;
          XP[r] = xFromM ? aMP : aXP;
          aM = M[r];
          aX = X[r];
          aMP = MP[r];
          aXP = XP[r];
          gM = pM;
          gX = pX;
          gY = pY;
          gMP = pMP;
          gXP = pXP;
          gYP = pYP;
        }
        dM = uM;
        dX = uX;
        dY = uY;
        dMP = uMP;
        dXP = uXP;
        dYP = uYP;
        oM = M[R - 1];
        oX = X[R - 1];
        oY = Y[R - 1];
        oMP = MP[R - 1];
        oXP = XP[R - 1];
        oYP = YP[R - 1];
        ob = bc;
        if (lane == 63) {
          if (w + 1 < W) {
            const int sl = j % RING_C;
            rM[sl][w + 1] = oM;
            rX[sl][w + 1] = oX;
            rY[sl][w + 1] = oY;
            rMP[sl][w + 1] = oMP;
            rXP[sl][w + 1] = oXP;
            rYP[sl][w + 1] = oYP;
          } else if (CH && cout) {  // staged in LDS, flushed 64 columns at a time (below)
            const int sl = (j - 1) & 63;
            s_out[0][sl] = oM;
            s_out[1][sl] = oX;
            s_out[2][sl] = oY;
            s_out[3][sl] = (int)(uint32_t)oMP;
            s_out[4][sl] = (int)(uint32_t)oXP;
            s_out[5][sl] = (int)(uint32_t)oYP;
          } else if (!CH && blk + 1 < nblk) {
            int *sb = bnd + 6 * j;
            sb[0] = oM;
            sb[1] = oX;
            sb[2] = oY;
            sb[3] = (int)(uint32_t)oMP;
            sb[4] = (int)(uint32_t)oXP;
            sb[5] = (int)(uint32_t)oYP;
            if constexpr (sizeof(P) == 8) {
              int *s2 = bnd + 6 * (lb + 1) + 6 * j;
              s2[3] = (int)(uint32_t)(oMP >> 32);
              s2[4] = (int)(uint32_t)(oXP >> 32);
              s2[5] = (int)(uint32_t)(oYP >> 32);
            }
          }
        }
      } else {
        ob = bc;
      }
      if constexpr (CH) {
        // lane 63 finished column t - 62: at the end of a 64-column batch (or the row) every
        // lane stores its column's six granules from LDS.  (Stored straight from lane 63 each
        // step, the stores' source registers -- the next step's state -- made every step wait
        // for the previous step's stores to complete.)
        const int jl = t - 62;
        if (cout && jl >= 1 && jl <= lb && ((jl & 63) == 0 || jl == lb)) {
          const int c = ((jl - 1) & ~63) + 1 + lane;
          if (c <= jl) {
            uint64_t *o = cout + 6 * (uint64_t)c;
            const uint64_t tg = (uint64_t)(uint32_t)c << 32;
#pragma unroll
            for (int v = 0; v < 6; v++)
              __hip_atomic_store(o + v, tg | (uint32_t)s_out[v][lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
      if (W > 1 && (t % KLAG) == KLAG - 1) __syncthreads();
    };
    // steady state: lane 63's column >= 1 and lane 0's <= lb, i.e. lagw + 63 <= t < lagw + lb
    const int ts0 = lb >= 64 ? lagw + 63 : steps, ts1 = lb >= 64 ? lagw + lb : steps;
    int t = 0;
    for (; t < ts0; t++) step(t, GenStep{});
    for (; t + 1 < ts1; t += 2) {  // two steps per trip: the state registers alternate, no copies
      step(t, SteadyStep{});
      step(t + 1, SteadyStep{});
    }
    for (; t < ts1; t++) step(t, SteadyStep{});
    for (; t < steps; t++) step(t, GenStep{});
    const int fl = la - blk * ROWS - 1;
    if (fl >= 0 && fl < ROWS && gl == fl / R) {
      const int r = fl % R;
      int mM = 0, mX = 0, mY = 0;
      P pM = 0, pX = 0, pY = 0;
#pragma unroll
      for (int rr = 0; rr < R; rr++)
        if (rr == r) {
          mM = M[rr] + MOFF;
          mX = X[rr];
          mY = Y[rr];
          pM = MP[rr];
          pX = XP[rr];
          pY = YP[rr];
        }
      int sc = mM > mX ? mM : mX;  // GlobAlignE.cpp:278-291
      sc = sc > mY ? sc : mY;
      fin_score = sc - (la + lb);  // (T -> score)
      fin_pay = sc == mM ? pM : (sc == mX ? pX : pY);
    }
    __threadfence_block();
    __syncthreads();
  }
  const int fl = la - (nblk - 1) * ROWS - 1;
  const int owner = la == 0 ? 0 : fl / R;
  if (gl == owner && (!CH || blk_first == nblk - 1)) {
    int L, I;
    if (la == 0) {
      // no rows (len1 == 1): only cell 0 of each state row exists.  With columns (lb > 0)
      // every j leaves matches[0] = lowerGap[0] = -inf, matchLen[0] = j and upperGap[0] = -inf
      // untouched, so the final max picks `matches` (GlobAlignE.cpp:244-251, 278-283): score
      // -inf, length lb, 0 identities.  Without columns the initial state is the answer, 0/0.
      L = lb;
      I = 0;
      fin_score = lb > 0 ? NINF : 0;
    } else {
      L = la + lb - (int)(fin_pay >> SH);
      I = (int)(fin_pay & (((P)1 << SH) - 1));
    }
    const uint32_t o = q.out ? q.out[p] : p;
    q.ident[o] = (double)I / (double)L;
    if (q.len) q.len[o] = L;
    if (q.ids) q.ids[o] = I;
    if (q.score) q.score[o] = fin_score;
  }
}

// Waves per pair in the latency form: four (one per SIMD) at every length.  Round 1 measured
// eight faster for config E's 8-12 kb genomes (profiles/r01_v7_nw_waves.txt); on the round-4
// kernels four waves are faster there too: E9100's sampler rounds 301 ms against 317-319 ms at
// eight, 369 ms at sixteen and 577 ms at two (profiles/r04/v5/nw_width.txt).  MC_NW_WAVES = 2,
// 4, 8 or 16 forces one width for every pair.
inline int mw_waves(uint64_t) {
  static const int forced = [] {
    const char *e = getenv("MC_NW_WAVES");
    const int v = e ? atoi(e) : 0;
    return v == 2 || v == 4 || v == 8 || v == 16 ? v : 0;
  }();
  return forced ? forced : 4;
}

template <int R, typename P>
int launch_bucket(mc_ctx *c, NWPairs q) {
  if (q.npairs == 0) return MC_OK;
  nw_mw_kernel<R, P, 1><<<q.npairs, 64, 0, c->stream>>>(q);
  MCG_CHECK(hipGetLastError());
  return MC_OK;
}

int launch_bucket_ch(mc_ctx *c, NWPairs q, int r) {
  if (q.npairs == 0) return MC_OK;
  if (r == 16) nw_mw_kernel<16, uint32_t, 1, true><<<q.npairs, 64, 0, c->stream>>>(q);
  else nw_mw_kernel<8, uint32_t, 1, true><<<q.npairs, 64, 0, c->stream>>>(q);
  MCG_CHECK(hipGetLastError());
  return MC_OK;
}

template <int R, typename P>
int launch_bucket_mw(mc_ctx *c, NWPairs q, int waves) {
  if (q.npairs == 0) return MC_OK;
  switch (waves) {
    case 2: nw_mw_kernel<R, P, 2><<<q.npairs, 128, 0, c->stream>>>(q); break;
    case 4: nw_mw_kernel<R, P, 4><<<q.npairs, 256, 0, c->stream>>>(q); break;
    case 16: nw_mw_kernel<R, P, 16><<<q.npairs, 1024, 0, c->stream>>>(q); break;
    default: nw_mw_kernel<R, P, 8><<<q.npairs, 512, 0, c->stream>>>(q); break;
  }
  MCG_CHECK(hipGetLastError());
  return MC_OK;
}

}  // namespace

int launch_nw(mc_ctx *c, const uint8_t *d_A, const uint64_t *d_aoff, const uint32_t *d_ai, const uint8_t *d_B,
              const uint64_t *d_boff, const uint32_t *d_bi, uint64_t m, const std::vector<uint64_t> &alen,
              const std::vector<uint64_t> &blen, double *d_ident, int32_t *d_len, int32_t *d_ids,
              int32_t *d_score, const uint32_t *d_out) {
  if (m == 0) return MC_OK;
  // bucket pairs by rows per lane and payload width; boundary scratch for multi-block pairs.
  // Few pairs (fewer than the chip's SIMDs) are latency-bound: one multi-wave workgroup per pair;
  // many pairs: one wavefront per pair.
  static const uint64_t mw_max = [] {  // MC_NW_MW_MAX: largest batch for the latency form
    const char *e = getenv("MC_NW_MW_MAX");
    return e ? (uint64_t)atoll(e) : (uint64_t)1024;
  }();
  const bool mw = m < mw_max;
  // chained row blocks (MC_NW_CHAIN=0 turns them off): a pair longer than one block of 64 x R
  // rows gets a single-wave workgroup per block, the blocks running concurrently a pipeline lag
  // (~130 steps) apart -- in the latency form, where few pairs leave SIMDs idle; MC_NW_CHAIN=2
  // chains the throughput form's long pairs too
  static const int chain_mode = [] {
    const char *e = getenv("MC_NW_CHAIN");
    return e ? atoi(e) : 1;
  }();
  // rows per lane of a chained block: 16 (the throughput form's step, 256 registers, two waves
  // per SIMD) or 8 (154 registers, three waves per SIMD, but ~10% more instructions per cell and
  // twice the blocks).  8 for long pairs (mean row length above 4 kb): E9100's search rounds of
  // 150 pairs of 8-12 kb (one tree level per round, trainer.cpp) fill the chip's SIMDs ~1.5 deep
  // at 16 and ~3 deep at 8, 210 ms against 225 (at two levels per round 8 lost, 269 against 239);
  // 16 otherwise (1 kb pairs fit one block of 16).  MC_NW_CHAIN_R=8 / 16 forces either.
  static const int chain_r_env = [] {
    const char *e = getenv("MC_NW_CHAIN_R");
    const int v = e ? atoi(e) : 0;
    return v == 8 || v == 16 ? v : 0;
  }();
  // MC_NW_TR_R = 4 / 8: the largest rows per lane of the throughput form (default 16; E9100's
  // label batch of ~3,000 8-12 kb pairs: 199 ms at 16, 232-240 at 8 -- three waves per SIMD
  // instead of two do not pay for ~10 % more instructions per cell -- and 327 at 4)
  static const int tr_rmax = [] {
    const char *e = getenv("MC_NW_TR_R");
    const int v = e ? atoi(e) : 16;
    return v == 4 ? 0 : v == 8 ? 1 : 2;
  }();
  uint64_t la_sum = 0;
  for (uint64_t i = 0; i < m; i++) la_sum += alen[i];
  const int chain_r = chain_r_env ? chain_r_env : la_sum > 4096 * m ? 8 : 16;
  std::vector<uint32_t> ch_pair;  // work items: pair, block, granule offsets in / out
  std::vector<uint16_t> ch_blk;
  std::vector<uint64_t> ch_in, ch_out;
  uint64_t ch_gran = 0;           // granules of every chained pair's block bottom rows
  enum { NB = 32 };  // latency form: (R, payload) x waves 2 / 4 / 8 / 16
  int bucket_waves[NB] = {0};
  std::vector<uint32_t> bucket[NB];
  std::vector<uint64_t> boff[NB];
  uint64_t scratch[NB] = {0};
  // longest pairs first (by DP cells): the dispatcher hands workgroups to free slots in launch
  // order, so the longest ones do not start last and leave a tail (config E: 8-12 kb genomes,
  // cells vary 2.3x).  Results go to each pair's own slot; the order changes nothing else.
  std::vector<uint32_t> order(m);
  for (uint64_t i = 0; i < m; i++) order[i] = (uint32_t)i;
  std::stable_sort(order.begin(), order.end(),
                   [&](uint32_t x, uint32_t y) { return alen[x] * blen[x] > alen[y] * blen[y]; });
  for (uint64_t oi = 0; oi < m; oi++) {
    const uint64_t i = order[oi];
    const uint64_t la = alen[i], lb = blen[i];
    const bool wide = la + lb >= 65535;
    const uint64_t rows_c = 64ull * chain_r;
    if ((chain_mode >= 2 || (chain_mode == 1 && mw)) && !wide && la > rows_c && lb >= 1) {
      const uint64_t nblk = (la + rows_c - 1) / rows_c;
      for (uint64_t b = 0; b < nblk; b++) {
        ch_pair.push_back((uint32_t)i);
        ch_blk.push_back((uint16_t)b);
        ch_in.push_back(b == 0 ? ~0ull : ch_gran + (b - 1) * 6 * (lb + 1));
        ch_out.push_back(b + 1 == nblk ? ~0ull : ch_gran + b * 6 * (lb + 1));
      }
      ch_gran += (nblk - 1) * 6 * (lb + 1);
      continue;
    }
    int r, bk;
    uint64_t rows;
    if (mw) {
      const int wv = mw_waves(la);
      const uint64_t w64 = 64ull * wv;  // rows of R = 1
      r = la <= w64 ? 0 : la <= 2 * w64 ? 1 : la <= 4 * w64 ? 2 : 3;  // R = 1, 2, 4, 8 over the waves
      bk = r + (wide ? 4 : 0) + (wv == 2 ? 24 : wv == 4 ? 0 : wv == 8 ? 8 : 16);
      bucket_waves[bk] = wv;
      rows = w64 << r;
    } else {
      r = la <= 256 ? 0 : la <= 512 ? 1 : 2;  // R = 4, 8, 16
      if (r > tr_rmax) r = tr_rmax;
      bk = r + (wide ? 3 : 0);
      rows = 64ull * (r == 0 ? 4 : r == 1 ? 8 : 16);
    }
    bucket[bk].push_back((uint32_t)i);
    boff[bk].push_back(scratch[bk]);
    if (la > rows) scratch[bk] += 12 * (lb + 1);
  }
  timed_begin(c);
  uint64_t total_idx = 0, total_scr = 0, total_ch = 0;
  for (int k = 0; k < NB; k++) {
    total_idx += bucket[k].size();
    total_scr += scratch[k];
  }
  total_ch = ch_pair.size();
  if (ensure(c->s_a, total_idx * 4 + 16) || ensure(c->s_b, total_idx * 8 + 16) ||
      ensure(c->s_c, std::max<uint64_t>(total_scr, 1) * 4))
    return MC_ERR_OOM;
  if (total_ch) {
    // items: pair (4 B) | block (2 B, padded) | in, out offsets (8 B each); 4 counters and an
    // error word; the granule buffer zeroed (no stale tag survives from an earlier launch)
    const size_t ib = (total_ch * 4 + 255) / 256 * 256, bb = (total_ch * 2 + 255) / 256 * 256,
                 ob = (total_ch * 8 + 255) / 256 * 256;
    if (ensure(c->nw_items, ib + bb + 2 * ob + 256) || ensure(c->nw_gran, ch_gran * 8 + 64)) return MC_ERR_OOM;
    MCG_CHECK(hipMemsetAsync(c->nw_gran.p, 0, ch_gran * 8 + 64, c->stream));
    char *base = (char *)c->nw_items.p;
    MCG_CHECK(hipMemsetAsync(base + ib + bb + 2 * ob, 0, 256, c->stream));
    const size_t n = total_ch;
    if (int rc = stage_h2d(c, base, ch_pair.data(), n * 4)) return rc;
    if (int rc = stage_h2d(c, base + ib, ch_blk.data(), n * 2)) return rc;
    if (int rc = stage_h2d(c, base + ib + bb, ch_in.data(), n * 8)) return rc;
    if (int rc = stage_h2d(c, base + ib + bb + ob, ch_out.data(), n * 8)) return rc;
    NWPairs q{d_A, d_aoff, d_ai, d_B, d_boff, d_bi, (uint32_t *)base, (uint32_t)n, nullptr, nullptr,
              d_ident, d_len, d_ids, d_score, d_out};
    q.pblk = (const uint16_t *)(base + ib);
    q.ctr = (uint32_t *)(base + ib + bb + 2 * ob);
    q.cbuf = (uint64_t *)c->nw_gran.p;
    q.cin = (const uint64_t *)(base + ib + bb);
    q.cout = (const uint64_t *)(base + ib + bb + ob);
    q.err = (int *)(base + ib + bb + 2 * ob + 32);
    if (int rc = launch_bucket_ch(c, q, chain_r)) return rc;
  }
  uint64_t io = 0, so = 0;
  for (int k = 0; k < NB; k++) {
    if (bucket[k].empty()) continue;
    for (auto &v : boff[k]) v += so;
    if (int rc = stage_h2d(c, (uint32_t *)c->s_a.p + io, bucket[k].data(), bucket[k].size() * 4)) return rc;
    if (int rc = stage_h2d(c, (uint64_t *)c->s_b.p + io, boff[k].data(), boff[k].size() * 8)) return rc;
    NWPairs q{d_A, d_aoff, d_ai, d_B, d_boff, d_bi, (uint32_t *)c->s_a.p + io, (uint32_t)bucket[k].size(),
              (int *)c->s_c.p, (uint64_t *)c->s_b.p + io, d_ident, d_len, d_ids, d_score, d_out};
    int rc = MC_OK;
    if (mw) {
      const int wv = bucket_waves[k];
      switch (k % 8) {
        case 0: rc = launch_bucket_mw<1, uint32_t>(c, q, wv); break;
        case 1: rc = launch_bucket_mw<2, uint32_t>(c, q, wv); break;
        case 2: rc = launch_bucket_mw<4, uint32_t>(c, q, wv); break;
        case 3: rc = launch_bucket_mw<8, uint32_t>(c, q, wv); break;
        case 4: rc = launch_bucket_mw<1, uint64_t>(c, q, wv); break;
        case 5: rc = launch_bucket_mw<2, uint64_t>(c, q, wv); break;
        case 6: rc = launch_bucket_mw<4, uint64_t>(c, q, wv); break;
        default: rc = launch_bucket_mw<8, uint64_t>(c, q, wv); break;
      }
    } else switch (k) {
      case 0: rc = launch_bucket<4, uint32_t>(c, q); break;
      case 1: rc = launch_bucket<8, uint32_t>(c, q); break;
      case 2: rc = launch_bucket<16, uint32_t>(c, q); break;
      case 3: rc = launch_bucket<4, uint64_t>(c, q); break;
      case 4: rc = launch_bucket<8, uint64_t>(c, q); break;
      default: rc = launch_bucket<16, uint64_t>(c, q); break;
    }
    if (rc) return rc;
    io += bucket[k].size();
    so += scratch[k];
  }
  // (the host arrays went through the pinned ring: nothing here waits for the copies)
  timed_end(c, F_NW);
  if (total_ch) {
    MCG_CHECK(hipStreamSynchronize(c->stream));
    const size_t ib = (total_ch * 4 + 255) / 256 * 256, bb = (total_ch * 2 + 255) / 256 * 256,
                 ob = (total_ch * 8 + 255) / 256 * 256;
    int herr = 0;
    MCG_CHECK(hipMemcpyAsync(&herr, (char *)c->nw_items.p + ib + bb + 2 * ob + 32, 4, hipMemcpyDeviceToHost, c->stream));
    MCG_CHECK(hipStreamSynchronize(c->stream));
    if (herr) {
      set_error("NW chained row blocks: a block's hand-off never arrived");
      return MC_ERR_TIMEOUT;
    }
  }
  return MC_OK;
}

}  // namespace mcg
