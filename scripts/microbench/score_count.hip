// score_count.hip -- the accumulation workers' per-candidate scoring chain in isolation, for
// counting its instructions (scripts/isa_count.py): 16 chunks of SAD / dot4 against the centre
// (accum_impl.hpp worker_dense), then classify_small on the sums.  Never launched.
#include "../../meshclust_amd/csrc/gpu/features.hpp"

using namespace mcg;

__global__ void score_one(const uint4 *__restrict__ rows, const uint4 *__restrict__ centre, const SmallK *__restrict__ k,
                          const PSm *__restrict__ ps, PSm q, double kq, double daq, int B, double *__restrict__ cv,
                          int *__restrict__ d) {
  const int t = threadIdx.x;
  Acc<uint8_t> acc;
  uint4 rv[16], cw[16];
#pragma unroll
  for (int c = 0; c < 16; c++) {
    rv[c] = rows[c * 512 + t];
    cw[c] = centre[c];
  }
#pragma unroll
  for (int c = 0; c < 16; c++) acc.add(rv[c], cw[c]);
  acc.fold();
  bool und = false;
  double c0 = 0.0;
  const int r = classify_small(*k, acc.sad, acc.dot, ps[t], q, kq, 0.0, daq, B, &c0, &und);
  cv[t] = c0;
  d[t] = und ? 2 : r;
}
