// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE against known byte counts for the load
// widths this repository's HBM kernels use (MI355X_MICROARCH.md: "On gfx950 FETCH_SIZE reports
// exactly 1/2 of the bytes of a wide coalesced streaming read (16 B/lane) ... Other access widths
// are uncalibrated").  Each kernel reads a 1 GiB buffer once (4x the 256 MiB Infinity Cache, so
// the reads reach HBM), one launch per pattern:
//   read_b32    4 B per lane, coalesced (64 lanes x 4 B = 256 B per wave load)
//   read_b128  16 B per lane, coalesced (1 KiB per wave load)
//   read_k1     kmer_kernel's pattern (kmer.hip pre_load): lane l of a wave loads dwords l, l+1
//               and l+2 of a 16-dword-per-lane group -- three overlapping 256-B wave loads per
//               64 dwords, each dword fetched from HBM once
// A one-word result per workgroup keeps the loads live.  Run each FETCH_SIZE pass on its own:
//   hipcc -O3 --offload-arch=gfx950 fetch_calib.hip -o fetch_calib
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d out -- ./fetch_calib
// The ratio FETCH_SIZE / 1 GiB per kernel is the correction for that access width.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr size_t BYTES = 1ull << 30;

__global__ __launch_bounds__(256) void read_b32(const uint32_t *__restrict__ p, size_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= p[i];
  if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;  // (practically never: keeps the loads)
}

__global__ __launch_bounds__(256) void read_b128(const uint4 *__restrict__ p, size_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;
}

// 64 dwords per wave step; lane l reads dwords base + l, l + 1, l + 2 (the last two lanes' extra
// words belong to the next step, as a read's trailing k-mers do)
__global__ __launch_bounds__(256) void read_k1(const uint32_t *__restrict__ p, size_t n, uint32_t *out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t acc = 0;
  for (size_t base = ((size_t)blockIdx.x * 4 + wv) * 64; base + 66 < n; base += (size_t)gridDim.x * 4 * 64) {
    const uint32_t *w = p + base + lane;
    acc ^= w[0] ^ (w[1] << 1) ^ (w[2] << 2);
  }
  if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;
}

int main() {
  uint32_t *buf, *out;
  CHECK(hipMalloc(&buf, BYTES));
  CHECK(hipMalloc(&out, 1 << 20));
  CHECK(hipMemset(buf, 0x5a, BYTES));
  // (evict the buffer from the Infinity Cache between patterns: write another 512 MiB)
  uint32_t *flush;
  CHECK(hipMalloc(&flush, 512ull << 20));
  const int grid = 256 * 8;
  for (int rep = 0; rep < 2; rep++) {
    CHECK(hipMemset(flush, rep, 512ull << 20));
    read_b32<<<grid, 256>>>(buf, BYTES / 4, out);
    CHECK(hipMemset(flush, rep + 1, 512ull << 20));
    read_b128<<<grid, 256>>>(reinterpret_cast<const uint4 *>(buf), BYTES / 16, out);
    CHECK(hipMemset(flush, rep + 2, 512ull << 20));
    read_k1<<<grid, 256>>>(buf, BYTES / 4, out);
  }
  CHECK(hipDeviceSynchronize());
  printf("{\"bytes_read_per_launch\": %zu}\n", BYTES);
  CHECK(hipFree(flush));
  CHECK(hipFree(out));
  CHECK(hipFree(buf));
  return 0;
}
