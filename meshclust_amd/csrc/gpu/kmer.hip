// kmer.hip -- K1: per-sequence k-mer histograms.
//
// Reference: fill_table (src/cluster/src/ClusterFactory.h:40-55) drives
// KmerHashTable::wholesaleIncrement (src/nonltr/KmerHashTable.cpp:193-223) over every
// segment [s, e]: k-mers start at s .. e-k+1, index = sum code[i]*4^(k-1-i) (first base most
// significant), forward strand only, table initialised to the pseudocount 1.
//
// One workgroup per sequence: the 4^k counters live in LDS (k <= 7: <= 64 KiB), each
// thread hashes a strided subset of k-mer start positions and increments with LDS atomics,
// then the table is written out as one histogram row of the chosen width together with its
// magnitude (sum of bins incl. pseudocounts = DivergencePoint::mag) and sum of squares.
// Pass `build == false` only reduces the largest bin (Runner.cpp:57-67 picks the width).
#include "mcgpu.hpp"

namespace mcg {

namespace {

constexpr int KT = 256;  // threads per workgroup

__device__ __forceinline__ uint64_t block_sum_u64(uint64_t v, uint64_t *red) {
  for (int o = 32; o >= 1; o >>= 1) {
    uint32_t lo = __shfl_xor((uint32_t)v, o, 64), hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
    v += ((uint64_t)hi << 32) | lo;
  }
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  uint64_t t = 0;
  for (int i = 0; i < KT / 64; i++) t += red[i];
  return t;
}

__device__ __forceinline__ uint64_t block_max_u64(uint64_t v, uint64_t *red) {
  for (int o = 32; o >= 1; o >>= 1) {
    uint32_t lo = __shfl_xor((uint32_t)v, o, 64), hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
    uint64_t x = ((uint64_t)hi << 32) | lo;
    v = x > v ? x : v;
  }
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  uint64_t t = 0;
  for (int i = 0; i < KT / 64; i++) t = red[i] > t ? red[i] : t;
  return t;
}

template <typename T>
__global__ __launch_bounds__(KT) void kmer_kernel(const uint8_t *__restrict__ codes, const uint64_t *__restrict__ seq_off,
                                                  const int32_t *__restrict__ seg, const uint64_t *__restrict__ seg_off,
                                                  uint64_t n, int k, bool build, uint8_t *__restrict__ hist,
                                                  uint64_t pitch, uint64_t *__restrict__ mag,
                                                  uint64_t *__restrict__ sumsq, uint64_t *__restrict__ len_out,
                                                  unsigned long long *__restrict__ gmax, int *__restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) uint32_t table[];
  __shared__ uint64_t red[KT / 64];
  const int B = 1 << (2 * k);
  for (uint64_t s = blockIdx.x; s < n; s += gridDim.x) {
    for (int b = threadIdx.x; b < B; b += KT) table[b] = 0;
    __syncthreads();
    const uint8_t *seq = codes + seq_off[s];
    const int64_t L = (int64_t)(seq_off[s + 1] - seq_off[s]);
    for (uint64_t g = seg_off[s]; g < seg_off[s + 1]; g++) {
      const int64_t first = seg[2 * g], last = (int64_t)seg[2 * g + 1] - k + 1;
      const int64_t lastp = last < first ? first : last;  // a short segment still hashes at `first`
      for (int64_t p = first + threadIdx.x; p <= lastp; p += KT) {
        if (p + k > L) {
          atomicOr(err, 1);
          continue;
        }
        uint32_t h = 0;
        bool bad = false;
        for (int i = 0; i < k; i++) {
          uint8_t c = seq[p + i];
          bad |= c > 3;
          h = (h << 2) | (c & 3);
        }
        if (bad) {
          atomicOr(err, 1);
          continue;
        }
        atomicAdd(&table[h], 1u);
      }
    }
    __syncthreads();
    uint64_t m = 0, sq = 0, mx = 0;
    for (int b = threadIdx.x; b < B; b += KT) {
      uint64_t v = (uint64_t)table[b] + 1;  // pseudocount (ClusterFactory.cpp:995)
      m += v;
      sq += v * v;
      mx = v > mx ? v : mx;
    }
    if (build) {
      T *row = reinterpret_cast<T *>(hist + s * pitch);
      for (int b = threadIdx.x; b < B; b += KT) row[b] = (T)(table[b] + 1);
      const int used = B * (int)sizeof(T);
      for (int b = used + threadIdx.x; b < (int)pitch; b += KT) hist[s * pitch + b] = 0;  // zero padding
      uint64_t tm = block_sum_u64(m, red);
      uint64_t tq = block_sum_u64(sq, red);
      if (threadIdx.x == 0) {
        mag[s] = tm;
        sumsq[s] = tq;
        len_out[s] = (uint64_t)L;
      }
    } else {
      uint64_t tx = block_max_u64(mx, red);
      if (threadIdx.x == 0) atomicMax(gmax, (unsigned long long)tx);
    }
    __syncthreads();
  }
}

}  // namespace

int launch_kmer(mc_ctx *c, int k, int width, bool build, uint64_t *d_max, int *d_err) {
  const int B = 1 << (2 * k);
  const size_t lds = (size_t)B * 4;
  const int grid = (int)std::min<uint64_t>(c->n, 8192);
  if (grid == 0) return MC_OK;
  timed_begin(c);
  const uint8_t *codes = (const uint8_t *)c->codes.p;
  const uint64_t *so = (const uint64_t *)c->seq_off.p;
  const int32_t *sg = (const int32_t *)c->seg.p;
  const uint64_t *sgo = (const uint64_t *)c->seg_off.p;
  uint8_t *h = (uint8_t *)c->hist.p;
  uint64_t *mg = (uint64_t *)c->mag.p, *sq = (uint64_t *)c->sumsq.p, *ln = (uint64_t *)c->len.p;
  auto *mx = (unsigned long long *)d_max;
  switch (width) {
    case 1: kmer_kernel<uint8_t><<<grid, KT, lds, c->stream>>>(codes, so, sg, sgo, c->n, k, build, h, c->pitch, mg, sq, ln, mx, d_err); break;
    case 2: kmer_kernel<uint16_t><<<grid, KT, lds, c->stream>>>(codes, so, sg, sgo, c->n, k, build, h, c->pitch, mg, sq, ln, mx, d_err); break;
    case 4: kmer_kernel<uint32_t><<<grid, KT, lds, c->stream>>>(codes, so, sg, sgo, c->n, k, build, h, c->pitch, mg, sq, ln, mx, d_err); break;
    default: kmer_kernel<uint64_t><<<grid, KT, lds, c->stream>>>(codes, so, sg, sgo, c->n, k, build, h, c->pitch, mg, sq, ln, mx, d_err); break;
  }
  MCG_CHECK(hipGetLastError());
  timed_end(c, F_KMER);
  return MC_OK;
}

}  // namespace mcg
