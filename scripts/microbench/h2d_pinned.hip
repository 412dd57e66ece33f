// Upload of a 25 MB packed dataset (config B): pageable source vs a pinned one, and the cost of
// pinning it (hipHostMalloc, first use) -- scripts/microbench, not part of the product.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
static double ms(std::chrono::steady_clock::time_point a) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
}
int main() {
  const size_t B = 25u << 20;
  void *d = nullptr;
  if (hipMalloc(&d, B) != hipSuccess) return 1;
  hipStream_t s;
  hipStreamCreate(&s);
  char *pg = (char *)malloc(B);
  memset(pg, 1, B);
  for (int r = 0; r < 3; r++) {
    auto t = std::chrono::steady_clock::now();
    hipMemcpyAsync(d, pg, B, hipMemcpyHostToDevice, s);
    hipStreamSynchronize(s);
    printf("pageable H2D 25 MB: %.3f ms\n", ms(t));
  }
  for (int r = 0; r < 3; r++) {  // a fresh pageable buffer each time (a new dataset per run)
    char *fb = (char *)malloc(B);
    memset(fb, 2, B);
    auto t = std::chrono::steady_clock::now();
    (void)hipMemcpyAsync(d, fb, B, hipMemcpyHostToDevice, s);
    (void)hipStreamSynchronize(s);
    printf("fresh pageable H2D 25 MB: %.3f ms\n", ms(t));
    free(fb);
  }
  for (int r = 0; r < 3; r++) {
    auto t = std::chrono::steady_clock::now();
    char *pn = nullptr;
    if (hipHostMalloc((void **)&pn, B, hipHostMallocDefault) != hipSuccess) return 2;
    const double ta = ms(t);
    memset(pn, 1, B);
    t = std::chrono::steady_clock::now();
    hipMemcpyAsync(d, pn, B, hipMemcpyHostToDevice, s);
    hipStreamSynchronize(s);
    const double tc = ms(t);
    t = std::chrono::steady_clock::now();
    hipHostFree(pn);
    printf("hipHostMalloc 25 MB: %.3f ms, pinned H2D: %.3f ms, hipHostFree: %.3f ms\n", ta, tc, ms(t));
  }
  return 0;
}
