// kmer.hip -- sequence residency and K1, the per-sequence k-mer histograms (SURVEY.md §8(a)
// a4-a7).
//
// Residency.  Every sequence is held twice in HBM: as 2-bit codes (16 bases per 32-bit word,
// each record starting on a word: K1's input) and as one-digit bytes (the NW input,
// Point::get_data_str).  The host parser uploads the packed form plus the sparse list of bytes
// that are not 0..3 (the 'N' encodeNucleotides leaves outside segments) -- a quarter of the
// bytes over PCIe -- and expand_kernel writes the byte form; mc_load_sequences (bytes) runs
// the other way through pack_kernel.  A sequence with any byte outside 0..3 is "impure": K1
// then reads its bytes (where such a byte inside a k-mer must raise the reference's error).
//
// K1.  Reference: fill_table (src/cluster/src/ClusterFactory.h:40-55) drives
// KmerHashTable::wholesaleIncrement (src/nonltr/KmerHashTable.cpp:193-223) over every
// segment [s, e]: k-mers start at s .. e-k+1, index = sum code[i]*4^(k-1-i) (first base most
// significant), forward strand only, table initialised to the pseudocount 1.
//
// Per-wavefront LDS bins: each wave owns a 4^k u32 table in LDS.  Short sequences: one wave
// per sequence (no cross-wave traffic at all).  Long sequences (mean length >= 4 kb): the W
// waves of a workgroup share one sequence and their tables are summed at write-out.  A lane
// takes 16 consecutive k-mer starts: it loads the three packed words that cover bases
// [p, p + 16 + k - 1) (the wave's loads are consecutive words: coalesced), funnels them into a
// 64-bit window and rolls the k-mer index over it.  k >= 8 (4^k u32 > LDS) uses per-wave
// tables in global scratch with the same code.
//
// One pass: the row is written at the width the caller asks for (mc_kmer_max speculates
// 8 bits) together with its magnitude (sum of bins incl. pseudocounts = DivergencePoint::mag),
// sum of squares and length, and the row maxima are reduced; the reference's largest-count
// pass (Runner.cpp:57-67) is that maximum, so a second pass runs only when 8 bits do not hold
// it.
#include "features.hpp"

namespace mcg {

namespace {

constexpr int KT = 256;       // threads per workgroup
constexpr int KW = KT / 64;   // waves per workgroup

// ---------------------------------------------------------------- residency kernels
// packed word w of sequence s -> 16 bytes of the one-digit string (one lane per word)
__global__ __launch_bounds__(256) void expand_kernel(const uint32_t *__restrict__ pk, const uint64_t *__restrict__ pk_off,
                                                     const uint64_t *__restrict__ seq_off, uint64_t n,
                                                     uint8_t *__restrict__ codes) {
  const int lane = threadIdx.x & 63;
  for (uint64_t s = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64; s < n;
       s += (uint64_t)gridDim.x * blockDim.x / 64) {
    const uint64_t w0 = pk_off[s], w1 = pk_off[s + 1], b0 = seq_off[s], L = seq_off[s + 1] - b0;
    for (uint64_t w = w0 + lane; w < w1; w += 64) {
      const uint32_t v = pk[w];
      const uint64_t j0 = (w - w0) * 16;
      uint8_t *dst = codes + b0 + j0;
      const uint64_t m = L - j0 < 16 ? L - j0 : 16;
      for (uint64_t j = 0; j < m; j++) dst[j] = (uint8_t)((v >> (2 * j)) & 3u);
    }
  }
}

__global__ __launch_bounds__(256) void exceptions_kernel(const uint64_t *__restrict__ pos, const uint8_t *__restrict__ val,
                                                         uint64_t m, uint8_t *__restrict__ codes) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x)
    codes[pos[i]] = val[i];
}

// one-digit bytes -> packed words + impure flag (one wave per sequence)
__global__ __launch_bounds__(256) void pack_kernel(const uint8_t *__restrict__ codes, const uint64_t *__restrict__ seq_off,
                                                   const uint64_t *__restrict__ pk_off, uint64_t n,
                                                   uint32_t *__restrict__ pk, uint8_t *__restrict__ impure) {
  const int lane = threadIdx.x & 63;
  for (uint64_t s = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64; s < n;
       s += (uint64_t)gridDim.x * blockDim.x / 64) {
    const uint64_t w0 = pk_off[s], w1 = pk_off[s + 1], b0 = seq_off[s], L = seq_off[s + 1] - b0;
    bool bad = false;
    for (uint64_t w = w0 + lane; w < w1; w += 64) {
      const uint64_t j0 = (w - w0) * 16;
      const uint64_t m = L - j0 < 16 ? L - j0 : 16;
      uint32_t v = 0;
      for (uint64_t j = 0; j < m; j++) {
        const uint8_t c = codes[b0 + j0 + j];
        bad |= c > 3;
        v |= (uint32_t)(c & 3) << (2 * j);
      }
      pk[w] = v;
    }
    const bool any = __ballot(bad) != 0;
    if (lane == 0) impure[s] = any ? 1 : 0;
  }
}

// ---------------------------------------------------------------- K1
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
  for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)v, o, 64), hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_max64(uint64_t v) {
  for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)v, o, 64), hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
    const uint64_t x = ((uint64_t)hi << 32) | lo;
    v = x > v ? x : v;
  }
  return v;
}

struct KArgs {
  const uint32_t *pk;
  const uint64_t *pk_off;
  const uint8_t *codes;
  const uint64_t *seq_off;
  const uint8_t *impure;
  const int32_t *seg;
  const uint64_t *seg_off;
  uint64_t n;
  int k;
  int coop;          // 1: the waves of a workgroup share one sequence
  int shared;        // 1: ... and one table (k = 7: 4^7 u32 = 64 KiB of LDS)
  int stream8;       // the streaming form (kmer_stream8) for 8-bit rows with k = 4..6
  uint32_t *gtab;    // k >= 8: per-wave tables in global memory (gridDim * KW * B)
  uint8_t *hist;
  uint64_t pitch;
  uint64_t *mag, *sumsq, *len_out;
  unsigned long long *gmax;
  int *err;
};

// Count the k-mers of starts [p_lo, p_hi] of sequence s (segment-local start range) into
// `tab` with this wave's lanes taking 16 consecutive starts each; `part` / `nparts` split the
// 16-start groups between the waves that share the sequence.
__device__ __forceinline__ void count_range(const KArgs &A, uint64_t s, int64_t p_lo, int64_t p_hi, int64_t L,
                                            bool pure, uint32_t *tab, int part, int nparts, uint64_t pk0, uint64_t pk1) {
  const int lane = threadIdx.x & 63;
  const int k = A.k;
  const uint32_t mask = k == 16 ? 0xffffffffu : ((1u << (2 * k)) - 1u);
  const int64_t ngroups = (p_hi - p_lo) / 16 + 1;
  for (int64_t g = (int64_t)part * 64 + lane; g < ngroups; g += (int64_t)nparts * 64) {
    const int64_t p0 = p_lo + g * 16;
    const int cnt = (int)(p_hi - p0 + 1 < 16 ? p_hi - p0 + 1 : 16);
    if (p0 + cnt - 1 + k > L) {  // a k-mer past the sequence end (only a segment shorter than k)
      atomicOr(A.err, 1);
      continue;
    }
    if (pure) {
      // bases [p0, p0 + cnt + k - 1) from the 2-bit words: a 64-bit window at bit 2*(p0 % 16)
      const uint32_t *w = A.pk + pk0 + (p0 >> 4);
      const uint64_t nw = pk1 - pk0 - (uint64_t)(p0 >> 4);
      const uint64_t lo = ((uint64_t)(nw > 1 ? w[1] : 0u) << 32) | w[0];
      const uint64_t hi = nw > 2 ? w[2] : 0u;
      const int sh = (int)(p0 & 15) * 2;
      const uint64_t win = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
      uint32_t h = 0;
      for (int i = 0; i < k - 1; i++) h = (h << 2) | (uint32_t)((win >> (2 * i)) & 3u);
      for (int j = 0; j < cnt; j++) {
        h = ((h << 2) | (uint32_t)((win >> (2 * (j + k - 1))) & 3u)) & mask;
        atomicAdd(&tab[h], 1u);
      }
    } else {
      const uint8_t *b = A.codes + A.seq_off[s] + p0;
      uint32_t h = 0;
      bool bad = false;
      for (int i = 0; i < k - 1; i++) {
        const uint8_t c = b[i];
        bad |= c > 3;
        h = (h << 2) | (c & 3u);
      }
      for (int j = 0; j < cnt; j++) {
        const uint8_t c = b[j + k - 1];
        bad |= c > 3;
        h = ((h << 2) | (c & 3u)) & mask;
        if (!bad) atomicAdd(&tab[h], 1u);
      }
      if (bad) atomicOr(A.err, 1);  // KmerHashTable::hash throws InvalidInputException
    }
  }
}

__device__ __forceinline__ void count_sequence(const KArgs &A, uint64_t s, uint32_t *tab, int part, int nparts) {
  const int64_t L = (int64_t)(A.seq_off[s + 1] - A.seq_off[s]);
  const bool pure = A.impure[s] == 0;
  for (uint64_t g = A.seg_off[s]; g < A.seg_off[s + 1]; g++) {
    const int64_t first = A.seg[2 * g], last = (int64_t)A.seg[2 * g + 1] - A.k + 1;
    count_range(A, s, first, last < first ? first : last, L, pure, tab, part, nparts, A.pk_off[s], A.pk_off[s + 1]);  // a short segment still hashes at `first`
  }
}

// Table reads / zeroing: plain LDS accesses, or for the global tables relaxed agent-scope
// atomics (sc1: the L1 is bypassed, the counts live in L2 where the atomics added them).
__device__ __forceinline__ uint32_t tab_ld(const uint32_t *p, bool glob) {
  return glob ? __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
}
__device__ __forceinline__ void tab_zero(uint32_t *p, bool glob) {
  if (glob) __hip_atomic_store(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = 0;
}
// every table access of this wave complete (LDS: lgkmcnt; global: vmcnt)
__device__ __forceinline__ void tab_drain(bool glob) {
  if (glob) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// Row of sequence s from the summed tables tabs[0..ntab) (stride B): write (width T) + stats;
// the calling wave only.  Zeroes the tables for the next sequence.
// 8-bit rows from one LDS table with B a multiple of 256 (k >= 4): every lane takes 32-bit
// words of the row (four bins: one 16-byte LDS read and one zeroing write), the wave's stores
// are 256 contiguous bytes, and the magnitude / sum of squares / maximum are DPP reductions
__device__ __forceinline__ void write_row8(const KArgs &A, uint64_t s, uint32_t *tab, int B, bool write, uint64_t *wmax,
                                           uint64_t len) {
  const int lane = threadIdx.x & 63;
  uint32_t m = 0, mx = 0;  // (a magnitude is the record's k-mer count + B: 32 bits below 4 Gb)
  uint64_t sq64 = 0;
  uint8_t *row = A.hist + s * A.pitch;
  for (int q = lane; q < B / 4; q += 64) {
    uint4 c = reinterpret_cast<const uint4 *>(tab)[q];
    reinterpret_cast<uint4 *>(tab)[q] = make_uint4(0, 0, 0, 0);
    c.x += 1;  // pseudocount (ClusterFactory.cpp:995)
    c.y += 1;
    c.z += 1;
    c.w += 1;
    m += c.x + c.y + c.z + c.w;
    sq64 += (uint64_t)c.x * c.x + (uint64_t)c.y * c.y + (uint64_t)c.z * c.z + (uint64_t)c.w * c.w;
    mx = max(max(c.x, c.y), max(max(c.z, c.w), mx));
    if (write) reinterpret_cast<uint32_t *>(row)[q] = (c.x & 0xffu) | (c.y & 0xffu) << 8 | (c.z & 0xffu) << 16 | (c.w & 0xffu) << 24;
  }
  if (write)  // the row's padding up to the pitch
    for (uint64_t b = (uint64_t)B + lane; b < A.pitch; b += 64) row[b] = 0;
  const uint64_t m64 = wave_sum64_all(m), s64 = wave_sum64_all(sq64);
  uint32_t wm = mx;
#define MCG_MAX_STEP(C, R) wm = max(wm, dpp_mv<C, R>(wm, wm));
  MCG_DPP_STEPS(MCG_MAX_STEP)
#undef MCG_MAX_STEP
  wm = (uint32_t)__builtin_amdgcn_readlane((int)wm, 63);
  if (lane == 0 && write) {
    A.mag[s] = m64;
    A.sumsq[s] = s64;
    A.len_out[s] = len;
  }
  *wmax = wm > *wmax ? wm : *wmax;
}

template <typename T>
__device__ __forceinline__ void write_row(const KArgs &A, uint64_t s, uint32_t *tab0, int ntab, int B, bool write,
                                          bool glob, uint64_t *wmax, uint64_t len) {
  const int lane = threadIdx.x & 63;
  if constexpr (sizeof(T) == 1) {
    if (ntab == 1 && !glob && (B & 255) == 0) {
      write_row8(A, s, tab0, B, write, wmax, len);
      return;
    }
  }
  constexpr int per = 16 / (int)sizeof(T);  // bins per 16-byte store
  uint64_t m = 0, sq = 0, mx = 0;
  uint8_t *row = A.hist + s * A.pitch;
  const int nst = (B + per - 1) / per;
  for (int q = lane; q < nst; q += 64) {
    T out[per];
#pragma unroll
    for (int e = 0; e < per; e++) {
      const int b = q * per + e;
      uint64_t v = 0;
      if (b < B) {
        uint32_t c = 0;
        for (int t = 0; t < ntab; t++) {
          c += tab_ld(tab0 + (size_t)t * B + b, glob);
          tab_zero(tab0 + (size_t)t * B + b, glob);
        }
        v = (uint64_t)c + 1;  // pseudocount (ClusterFactory.cpp:995)
        m += v;
        sq += v * v;
        mx = v > mx ? v : mx;
      }
      out[e] = (T)v;
    }
    if (write) {
      if ((q + 1) * per <= B || B * (int)sizeof(T) >= 16) {
        *reinterpret_cast<uint4 *>(row + (size_t)q * 16) = *reinterpret_cast<const uint4 *>(out);
      } else {  // a row narrower than 16 bytes (k = 1, 8-bit): bytes, then zero the pad
        for (int e = 0; e < B - q * per; e++) reinterpret_cast<T *>(row)[q * per + e] = out[e];
      }
    }
  }
  if (write) {
    const uint64_t used = ((uint64_t)B * sizeof(T) + 15) / 16 * 16;
    for (uint64_t b = (uint64_t)B * sizeof(T) + lane; b < A.pitch; b += 64)
      if (b >= used || B * sizeof(T) < 16) row[b] = 0;
  }
  m = wave_sum64(m);
  sq = wave_sum64(sq);
  mx = wave_max64(mx);
  if (lane == 0 && write) {
    A.mag[s] = m;
    A.sumsq[s] = sq;
    A.len_out[s] = len;
  }
  *wmax = mx > *wmax ? mx : *wmax;
}

// ---- the streaming form (8-bit rows, k = 4..6, one wave per sequence): configs B and D --------
// A wave takes 64 sequences at a time (their metadata loaded lane by lane); for each one it
// holds this lane's three packed words of its first 16-start group, and issues the NEXT
// sequence's words before it counts the current one, so a sequence's load latency is covered by
// the previous one's LDS work instead of stalling the wave.  The per-sequence row statistics
// stay in registers (lane j keeps sequence j's) and go out as three coalesced 512-byte stores
// per 64 sequences; the row maximum is a per-lane running maximum, reduced once per wave.
struct Pre {
  uint32_t w0, w1, w2;
};
__device__ __forceinline__ Pre pre_load(const KArgs &A, uint64_t pk0, uint64_t pk1, int64_t p0, bool act) {
  Pre r{0u, 0u, 0u};
  if (act) {
    const uint32_t *w = A.pk + pk0 + (p0 >> 4);
    const uint64_t nw = pk1 - pk0 - (uint64_t)(p0 >> 4);
    r.w0 = w[0];
    if (nw > 1) r.w1 = w[1];
    if (nw > 2) r.w2 = w[2];
  }
  return r;
}
// the 16 (or fewer) k-mers of starts [p0, p0 + cnt) from this lane's words
__device__ __forceinline__ void count_words(const Pre &w, int64_t p0, int cnt, int k, uint32_t mask, uint32_t *tab) {
  const uint64_t lo = ((uint64_t)w.w1 << 32) | w.w0, hi = w.w2;
  const int sh = (int)(p0 & 15) * 2;
  const uint64_t win = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
  uint32_t h = 0;
  for (int i = 0; i < k - 1; i++) h = (h << 2) | (uint32_t)((win >> (2 * i)) & 3u);
  for (int j = 0; j < cnt; j++) {
    h = ((h << 2) | (uint32_t)((win >> (2 * (j + k - 1))) & 3u)) & mask;
    atomicAdd(&tab[h], 1u);
  }
}

// The same with k a compile-time constant K (k = 4, 5, 6: configs B, D, E): the 16 k-mers
// unrolled, each one a bitfield of the window with its 2-bit groups reversed once (base j of
// the window at bits [62 - 2j, 63 - 2j]: the k-mer of start j, first base most significant as
// KmerHashTable's hash, is bits [64 - 2(j + K), 64 - 2j)) instead of a rolling hash with a
// variable 64-bit shift, and the starts past `cnt` (a sequence's last group) counted into a
// trash word instead of a divergent loop: 2-4 VALU instructions per k-mer instead of 7 (the
// kernel is VALU-issue bound: 0.83 of the issue rate at D1M, LDS 0.41 busy)
template <int K>
__device__ __forceinline__ void count_words_k(const Pre &w, int64_t p0, int cnt, uint32_t *tab, uint32_t *trash) {
  const uint64_t lo = ((uint64_t)w.w1 << 32) | w.w0, hi = w.w2;
  const int sh = (int)(p0 & 15) * 2;
  const uint64_t win = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;  // base j at bits 2j (low), 2j + 1
  // bit reversal puts base j at bits 31 - 2j / 30 - 2j with its two bits swapped: swap them back
  uint32_t a = __builtin_bitreverse32((uint32_t)win), b = __builtin_bitreverse32((uint32_t)(win >> 32));
  a = ((a >> 1) & 0x55555555u) | ((a & 0x55555555u) << 1);
  b = ((b >> 1) & 0x55555555u) | ((b & 0x55555555u) << 1);
  // k-mer j is bits [lo, lo + 2K) of a:b, lo = 64 - 2(j + K): one bitfield extract from the word
  // that holds it (a compile-time choice), then the table address (one shift-add)
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const int lo = 64 - 2 * (j + K);
    // (the extract as asm: left to itself the compiler folds the table's x4 into a shift and a
    // mask and adds the base -- three instructions where bfe + lshl_add are two)
    uint32_t h;
    if (lo >= 32) asm("v_bfe_u32 %0, %1, %2, %3" : "=v"(h) : "v"(a), "i"(lo - 32), "i"(2 * K));
    else if (lo + 2 * K <= 32) asm("v_bfe_u32 %0, %1, %2, %3" : "=v"(h) : "v"(b), "i"(lo), "i"(2 * K));
    else asm("v_bfe_u32 %0, %1, 0, %2" : "=v"(h) : "v"(__builtin_amdgcn_alignbit(a, b, (uint32_t)lo)), "i"(2 * K));
    atomicAdd(j < cnt ? tab + h : trash, 1u);
  }
}

// S sub-tables per wave (lanes l*64/S .. (l+1)*64/S - 1 count into sub-table l): a k-mer
// increment is an LDS atomic, and lanes of one instruction that hit the same bin serialise;
// S tables take those collisions apart (k = 4: S = 4, 4 KiB per wave).  The row sums them.
template <int S, int K = 0>
__device__ __forceinline__ void kmer_stream8(const KArgs &A, uint32_t *tab0, int B_, bool write, uint64_t *wmax_out,
                                             uint32_t *trash) {
  const int wv = wave_id(), lane = threadIdx.x & 63;
  const int B = K ? 1 << (2 * K) : B_;
  uint32_t *tab = tab0 + (size_t)(lane / (64 / S)) * B;
  const int k = K ? K : A.k;
  const uint32_t mask = (1u << (2 * k)) - 1u;
  const uint64_t stride = (uint64_t)gridDim.x * KW;
  uint32_t lmax = 0;  // this lane's largest bin (+ pseudocount) over every row it wrote
  for (uint64_t sb = (uint64_t)blockIdx.x * KW + wv; sb < A.n; sb += 64 * stride) {
    const uint64_t si = sb + (uint64_t)lane * stride;
    const bool vi = si < A.n;
    const uint64_t s0 = vi ? si : 0;
    // (sequence lengths and packed word counts below 2^32: the loader's limits)
    const uint64_t pk0 = A.pk_off[s0];
    const uint32_t Ls = (uint32_t)(A.seq_off[s0 + 1] - A.seq_off[s0]), npk = (uint32_t)(A.pk_off[s0 + 1] - pk0);
    const uint64_t g0 = A.seg_off[s0], g1 = A.seg_off[s0 + 1];
    const bool one = vi && A.impure[s0] == 0 && g1 == g0 + 1;  // pure, one segment
    const int32_t sf = one ? A.seg[2 * g0] : 0, sl = one ? A.seg[2 * g0 + 1] : 0;
    const uint64_t left = (A.n - sb + stride - 1) / stride;
    const int nb = left < 64 ? (int)left : 64;
    uint64_t my_m = 0, my_sq = 0;  // lane j: sequence j's statistics (its length is Ls)
    // the first group's words of sequence jj (lane = group index), issued one sequence ahead
    auto issue = [&](int jj) -> Pre {
      const bool o = __builtin_amdgcn_readlane((int)one, jj) != 0;
      if (!o) return Pre{0u, 0u, 0u};
      const int64_t first = __builtin_amdgcn_readlane(sf, jj);
      const int64_t last0 = (int64_t)__builtin_amdgcn_readlane(sl, jj) - k + 1;
      const int64_t last = last0 < first ? first : last0;
      const int64_t ng = (last - first) / 16 + 1;
      const uint64_t q0 = readlane64(pk0, jj);
      return pre_load(A, q0, q0 + (uint32_t)__builtin_amdgcn_readlane((int)npk, jj), first + (int64_t)lane * 16, lane < ng);
    };
    // two sequences' words in flight ahead of the one being counted
    Pre cur = issue(0);
    Pre nx1 = nb > 1 ? issue(1) : Pre{0u, 0u, 0u};
    for (int jj = 0; jj < nb; jj++) {
      const uint64_t s = sb + (uint64_t)jj * stride;
      const uint64_t L = (uint32_t)__builtin_amdgcn_readlane((int)Ls, jj);
      const Pre nxt = jj + 2 < nb ? issue(jj + 2) : Pre{0u, 0u, 0u};
      if (__builtin_amdgcn_readlane((int)one, jj)) {
        const int64_t first = __builtin_amdgcn_readlane(sf, jj);
        const int64_t last0 = (int64_t)__builtin_amdgcn_readlane(sl, jj) - k + 1;
        const int64_t p_lo = first, p_hi = last0 < first ? first : last0;
        const uint64_t q0 = readlane64(pk0, jj), q1 = q0 + (uint32_t)__builtin_amdgcn_readlane((int)npk, jj);
        const int64_t ngroups = (p_hi - p_lo) / 16 + 1;
        for (int64_t g = lane; g < ngroups; g += 64) {
          const int64_t p0 = p_lo + g * 16;
          const int cnt = (int)(p_hi - p0 + 1 < 16 ? p_hi - p0 + 1 : 16);
          if (p0 + cnt - 1 + k > (int64_t)L) {  // a k-mer past the sequence end (a segment shorter than k)
            atomicOr(A.err, 1);
            continue;
          }
          if constexpr (K > 0) count_words_k<K>(g == lane ? cur : pre_load(A, q0, q1, p0, true), p0, cnt, tab, trash);
          else count_words(g == lane ? cur : pre_load(A, q0, q1, p0, true), p0, cnt, k, mask, tab);
        }
      } else {
        count_sequence(A, s, tab, 0, 1);
      }
      cur = nx1;
      nx1 = nxt;
      tab_drain(false);
      // the row: bins + pseudocount, written as bytes; magnitude and sum of squares reduced over
      // the wave, the maximum kept per lane
      uint32_t m = 0, sq = 0;  // (32 bits: a row of L < 2^16 - B k-mers has sum (c + 1)^2 < 2^32)
      uint64_t m64 = 0, sq64 = 0;
      const bool small = L + (uint64_t)B < 65536;
      uint8_t *row = A.hist + s * A.pitch;
      for (int q = lane; q < B / 4; q += 64) {
        uint4 c = reinterpret_cast<const uint4 *>(tab0)[q];
        reinterpret_cast<uint4 *>(tab0)[q] = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 1; u < S; u++) {
          const uint4 d = reinterpret_cast<const uint4 *>(tab0 + (size_t)u * B)[q];
          reinterpret_cast<uint4 *>(tab0 + (size_t)u * B)[q] = make_uint4(0, 0, 0, 0);
          c.x += d.x;
          c.y += d.y;
          c.z += d.z;
          c.w += d.w;
        }
        c.x += 1;  // pseudocount (ClusterFactory.cpp:995)
        c.y += 1;
        c.z += 1;
        c.w += 1;
        m += c.x + c.y + c.z + c.w;
        if (small) sq += c.x * c.x + c.y * c.y + c.z * c.z + c.w * c.w;
        else sq64 += (uint64_t)c.x * c.x + (uint64_t)c.y * c.y + (uint64_t)c.z * c.z + (uint64_t)c.w * c.w;
        lmax = max(max(c.x, c.y), max(max(c.z, c.w), lmax));
        if (write) reinterpret_cast<uint32_t *>(row)[q] = (c.x & 0xffu) | (c.y & 0xffu) << 8 | (c.z & 0xffu) << 16 | (c.w & 0xffu) << 24;
      }
      if (write)  // the row's padding up to the pitch
        for (uint64_t b = (uint64_t)B + lane; b < A.pitch; b += 64) row[b] = 0;
      // (a pure one-segment sequence counted every start of [p_lo, p_hi] once: its magnitude is
      // that count + B pseudocounts, no reduction)
      const bool one_jj = K > 0 && __builtin_amdgcn_readlane((int)one, jj) != 0;
      if (one_jj && small) {
        const int64_t first = __builtin_amdgcn_readlane(sf, jj);
        const int64_t last0 = (int64_t)__builtin_amdgcn_readlane(sl, jj) - k + 1;
        m64 = (uint64_t)((last0 < first ? first : last0) - first + 1) + (uint64_t)B;
        sq = wave_sum32_all(sq);
        sq64 = sq;
      } else if (small) {
        m = wave_sum32_all(m);
        sq = wave_sum32_all(sq);
        m64 = m;
        sq64 = sq;
      } else {
        m64 = wave_sum64_all(m);
        sq64 = wave_sum64_all(sq64);
      }
      if (lane == jj) {
        my_m = m64;
        my_sq = sq64;
      }
      tab_drain(false);
    }
    if (write && lane < nb) {
      const uint64_t s = sb + (uint64_t)lane * stride;
      A.mag[s] = my_m;
      A.sumsq[s] = my_sq;
      A.len_out[s] = Ls;
    }
  }
  uint32_t wm = lmax;
#define MCG_MAX_STEP(C, R) wm = max(wm, dpp_mv<C, R>(wm, wm));
  MCG_DPP_STEPS(MCG_MAX_STEP)
#undef MCG_MAX_STEP
  *wmax_out = (uint32_t)__builtin_amdgcn_readlane((int)wm, 63);
}

// GLOB: the tables in global scratch (k >= 8).  A compile-time choice: a table pointer picked
// at run time between LDS and global memory makes every table access a FLAT instruction.
// STREAM: kmer_stream8 alone (a kernel of its own: its register allocation, not the general
// form's, sets the occupancy).
template <typename T, bool GLOB, bool STREAM = false, int S = 1, int K = 0>
__global__ __launch_bounds__(KT) void kmer_kernel(KArgs A, bool write) {
  extern __shared__ __attribute__((aligned(16))) uint32_t ltab[];
  __shared__ uint64_t s_max[KW];
  const int B = 1 << (2 * A.k);
  const int wv = wave_id(), lane = threadIdx.x & 63;
  constexpr bool glob = GLOB;
  uint32_t *base;  // this workgroup's tables
  if constexpr (GLOB) base = A.gtab + (uint64_t)blockIdx.x * KW * (uint64_t)B;
  else base = ltab;
  uint32_t *mytab = base + (A.shared ? 0 : (size_t)wv * S * B);
  uint64_t wmax = 0;
  if (!A.shared || wv == 0)
    for (int b = lane; b < S * B; b += 64) tab_zero(mytab + b, glob);
  tab_drain(glob);
  if constexpr (STREAM) {
    // (trash: one word per wave past the tables, for the starts a last group does not have)
    kmer_stream8<S, K>(A, mytab, B, write, &wmax, ltab + (size_t)KW * S * B + wv);
  } else if (!A.coop) {
    // one wave per sequence: the wave's own table, no workgroup barrier.  The metadata of the
    // wave's next 64 sequences (offsets, purity, segment bounds) are loaded lane by lane in two
    // round trips and handed out by readlane, instead of a chain of dependent loads per sequence
    const uint64_t stride = (uint64_t)gridDim.x * KW;
    for (uint64_t sb = (uint64_t)blockIdx.x * KW + wv; sb < A.n; sb += 64 * stride) {
      const uint64_t si = sb + (uint64_t)lane * stride;
      const bool vi = si < A.n;
      const uint64_t s0 = vi ? si : 0;
      const uint64_t so0 = A.seq_off[s0], so1 = A.seq_off[s0 + 1], pk0 = A.pk_off[s0], pk1 = A.pk_off[s0 + 1];
      const uint64_t g0 = A.seg_off[s0], g1 = A.seg_off[s0 + 1];
      const bool one = vi && A.impure[s0] == 0 && g1 == g0 + 1;  // pure, one segment: the fast form
      const int32_t sf = one ? A.seg[2 * g0] : 0, sl = one ? A.seg[2 * g0 + 1] : 0;
      const uint64_t left = (A.n - sb + stride - 1) / stride;
      const int nb = left < 64 ? (int)left : 64;
      for (int jj = 0; jj < nb; jj++) {
        const uint64_t s = sb + (uint64_t)jj * stride;
        const uint64_t L = readlane64(so1, jj) - readlane64(so0, jj);
        if (__builtin_amdgcn_readlane((int)one, jj)) {
          const int64_t first = __builtin_amdgcn_readlane(sf, jj);
          const int64_t last = (int64_t)__builtin_amdgcn_readlane(sl, jj) - A.k + 1;
          count_range(A, s, first, last < first ? first : last, (int64_t)L, true, mytab, 0, 1, readlane64(pk0, jj),
                      readlane64(pk1, jj));
        } else {
          count_sequence(A, s, mytab, 0, 1);
        }
        tab_drain(glob);
        write_row<T>(A, s, mytab, 1, B, write, glob, &wmax, L);
        tab_drain(glob);
      }
    }
  } else {
    // the KW waves share a sequence (per-wave tables, or one shared table); wave 0 sums the
    // tables into the row
    __syncthreads();
    for (uint64_t s = blockIdx.x; s < A.n; s += gridDim.x) {
      count_sequence(A, s, mytab, wv, KW);
      tab_drain(glob);
      __syncthreads();
      if (wv == 0) {
        write_row<T>(A, s, base, A.shared ? 1 : KW, B, write, glob, &wmax, A.seq_off[s + 1] - A.seq_off[s]);
        tab_drain(glob);
      }
      __syncthreads();
    }
  }
  if (lane == 0) s_max[wv] = wmax;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int i = 0; i < KW; i++) t = s_max[i] > t ? s_max[i] : t;
    // (one device-scope atomic per workgroup only when it raises the maximum: thousands of
    // same-address atomics serialise at one L2 channel)
    if (t > __hip_atomic_load(A.gmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(A.gmax, (unsigned long long)t);
  }
}

}  // namespace

int launch_expand(mc_ctx *c, uint64_t nexc, const uint64_t *d_exc_pos, const uint8_t *d_exc_val) {
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((c->n + 3) / 4, 8192));
  expand_kernel<<<grid, 256, 0, c->stream>>>((const uint32_t *)c->packed.p, (const uint64_t *)c->pk_off.p,
                                            (const uint64_t *)c->seq_off.p, c->n, (uint8_t *)c->codes.p);
  MCG_CHECK(hipGetLastError());
  if (nexc) {
    exceptions_kernel<<<(int)std::min<uint64_t>((nexc + 255) / 256, 4096), 256, 0, c->stream>>>(
        d_exc_pos, d_exc_val, nexc, (uint8_t *)c->codes.p);
    MCG_CHECK(hipGetLastError());
  }
  return MC_OK;
}

int launch_pack(mc_ctx *c) {
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((c->n + 3) / 4, 8192));
  pack_kernel<<<grid, 256, 0, c->stream>>>((const uint8_t *)c->codes.p, (const uint64_t *)c->seq_off.p,
                                          (const uint64_t *)c->pk_off.p, c->n, (uint32_t *)c->packed.p,
                                          (uint8_t *)c->impure.p);
  MCG_CHECK(hipGetLastError());
  return MC_OK;
}

int launch_kmer(mc_ctx *c, int k, int width, bool write, uint64_t *d_max, int *d_err) {
  const int B = 1 << (2 * k);
  KArgs A;
  A.pk = (const uint32_t *)c->packed.p;
  A.pk_off = (const uint64_t *)c->pk_off.p;
  A.codes = (const uint8_t *)c->codes.p;
  A.seq_off = (const uint64_t *)c->seq_off.p;
  A.impure = (const uint8_t *)c->impure.p;
  A.seg = (const int32_t *)c->seg.p;
  A.seg_off = (const uint64_t *)c->seg_off.p;
  A.n = c->n;
  A.k = k;
  // long sequences: the waves of a workgroup share one (mean length >= 4 kb); k = 7: one
  // 64 KiB LDS table shared by the workgroup's waves
  const bool per_wave_lds = (size_t)KW * B * 4 <= 64 * 1024, shared_lds = !per_wave_lds && (size_t)B * 4 <= 64 * 1024;
  A.shared = shared_lds ? 1 : 0;
  A.coop = (c->n && c->h_seq_off[c->n] / c->n >= 4096) || shared_lds ? 1 : 0;
  A.stream8 = getenv("MC_KMER_NO_STREAM") ? 0 : 1;
  A.hist = (uint8_t *)c->hist.p;
  A.pitch = c->pitch;
  A.mag = (uint64_t *)c->mag.p;
  A.sumsq = (uint64_t *)c->sumsq.p;
  A.len_out = (uint64_t *)c->len.p;
  A.gmax = (unsigned long long *)d_max;
  A.err = d_err;
  const uint64_t units = A.coop ? c->n : (c->n + KW - 1) / KW;
  int grid = (int)std::min<uint64_t>(units, 8192);
  if (grid == 0) return MC_OK;
  size_t lds = 0;
  A.gtab = nullptr;
  if (per_wave_lds || shared_lds) {
    lds = shared_lds ? (size_t)B * 4 : (size_t)KW * B * 4;
  } else {
    // 4^k u32 per wave does not fit LDS: per-wave tables in global scratch, as many resident
    // workgroups as the scratch allows (<= 1 GiB)
    const uint64_t per_wg = (uint64_t)KW * B * 4;
    grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)grid, (1ull << 30) / per_wg));
    if (int rc = ensure(c->s_g, (size_t)grid * per_wg)) return rc;
    MCG_CHECK(hipMemsetAsync(c->s_g.p, 0, (size_t)grid * per_wg, c->stream));
    A.gtab = (uint32_t *)c->s_g.p;
  }
  timed_begin(c);
  const bool g = A.gtab != nullptr;
  switch (width) {
    case 1:
      if (!g && !A.coop && !A.shared && (B & 255) == 0 && A.stream8) {
        // sub-tables per wave: k = 4 four (16 KiB per workgroup), k = 5 two (32 KiB), else one
        // (S > 1 measured slower: 76 vs 68 us at config B, 531 vs 507 us at D1M -- the table
        // atomics are not what bounds the kernel; MC_KMER_SUB=1 keeps the sub-tables for tests)
        const int S = getenv("MC_KMER_SUB") ? (k == 4 ? 4 : k == 5 ? 2 : 1) : 1;
        const size_t sl = (size_t)KW * S * B * 4 + KW * 4;
        if (S == 4) kmer_kernel<uint8_t, false, true, 4><<<grid, KT, sl, c->stream>>>(A, write);
        else if (S == 2) kmer_kernel<uint8_t, false, true, 2><<<grid, KT, sl, c->stream>>>(A, write);
        else if (k == 4 && !getenv("MC_KMER_RUNTIME_K")) kmer_kernel<uint8_t, false, true, 1, 4><<<grid, KT, sl, c->stream>>>(A, write);
        else if (k == 5 && !getenv("MC_KMER_RUNTIME_K")) kmer_kernel<uint8_t, false, true, 1, 5><<<grid, KT, sl, c->stream>>>(A, write);
        else if (k == 6 && !getenv("MC_KMER_RUNTIME_K")) kmer_kernel<uint8_t, false, true, 1, 6><<<grid, KT, sl, c->stream>>>(A, write);
        else kmer_kernel<uint8_t, false, true, 1><<<grid, KT, sl, c->stream>>>(A, write);
      }
      else
        (g ? kmer_kernel<uint8_t, true> : kmer_kernel<uint8_t, false>)<<<grid, KT, lds, c->stream>>>(A, write);
      break;
    case 2: (g ? kmer_kernel<uint16_t, true> : kmer_kernel<uint16_t, false>)<<<grid, KT, lds, c->stream>>>(A, write); break;
    case 4: (g ? kmer_kernel<uint32_t, true> : kmer_kernel<uint32_t, false>)<<<grid, KT, lds, c->stream>>>(A, write); break;
    default: (g ? kmer_kernel<uint64_t, true> : kmer_kernel<uint64_t, false>)<<<grid, KT, lds, c->stream>>>(A, write); break;
  }
  MCG_CHECK(hipGetLastError());
  timed_end(c, F_KMER);
  return MC_OK;
}

}  // namespace mcg
