// Probe: a trivial cooperative launch, then exit.  Under rocprofv3 --kernel-trace, does the
// process fault in the HSA runtime's exit handler (as bench.py does after accum_kernel)?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int *p) {
  if (threadIdx.x == 0) atomicAdd(p, 1);
}
int main() {
  int *d = nullptr;
  if (hipMalloc(&d, 4) != hipSuccess) return 2;
  (void)hipMemset(d, 0, 4);
  void *args[] = {&d};
  hipError_t e = hipLaunchCooperativeKernel((const void *)k, dim3(256), dim3(512), args, 0, nullptr);
  if (e != hipSuccess) { printf("launch: %s\n", hipGetErrorString(e)); return 3; }
  int h = 0;
  (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  printf("blocks %d\n", h);
  (void)hipFree(d);
  return 0;
}
