// valu_peak.hip -- the gfx950 VALU issue rate for the 32-bit integer instruction classes the NW
// kernel's cell update and the accumulation scan are made of: independent
// streams of one instruction (the compare + select pair counts as one "instruction" here),
// at 1, 2, 4 and 8 waves per SIMD.  Prints lane-instructions per clock per CU and per second
// (the NW roofline's peak, bench.py nw_roofline).  Each thread runs 8 independent register
// chains so no instruction waits on its predecessor's result.
//   hipcc -O3 --offload-arch=gfx950 valu_peak.hip -o valu_peak && ./valu_peak
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

constexpr int ITERS = 4096;
constexpr int UNROLL = 16;  // instructions per chain per iteration (x 8 chains)

template <int OP>
__device__ __forceinline__ void op(uint32_t &a, uint32_t b, uint32_t c) {
  if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
  else if constexpr (OP == 1) asm volatile("v_max_i32 %0, %0, %1" : "+v"(a) : "v"(b));
  else if constexpr (OP == 2) asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
  else if constexpr (OP == 3) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
  else if constexpr (OP == 4) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a) : "v"(b));
  else if constexpr (OP == 5) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a) : "v"(b));
  else if constexpr (OP == 6) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b) : "vcc");
  else if constexpr (OP == 7) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[20:21]" : "+v"(a) : "v"(b) : "s20", "s21");
  else if constexpr (OP == 8)  // the select pattern: a compare into an SGPR pair, then a select on it
    asm volatile("v_cmp_gt_i32_e64 s[22:23], %0, %1\n\tv_cndmask_b32_e64 %0, %0, %1, s[22:23]" : "+v"(a) : "v"(b) : "s22", "s23");
  else if constexpr (OP == 9) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a) : "v"(b), "v"(c));
  else if constexpr (OP == 10) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c));
  else if constexpr (OP == 11) asm volatile("v_dot4_u32_u8 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c));
  else if constexpr (OP == 12) asm volatile("v_mov_b32 %0, %1" : "=v"(a) : "v"(b));
  else if constexpr (OP == 13) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a) : "v"(b));
  else if constexpr (OP == 14) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a) : "v"(b));
  else asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
}

template <int OP>
__global__ __launch_bounds__(256) void valu_kernel(uint32_t *out, uint32_t seed) {
  uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5, r6 = r0 + 6, r7 = r0 + 7;
  const uint32_t b = seed ^ blockIdx.x, c = seed + 3u;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      op<OP>(r0, b, c);
      op<OP>(r1, b, c);
      op<OP>(r2, b, c);
      op<OP>(r3, b, c);
      op<OP>(r4, b, c);
      op<OP>(r5, b, c);
      op<OP>(r6, b, c);
      op<OP>(r7, b, c);
    }
  }
  const uint32_t s = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
  if (s == 0x9e3779b9u) out[blockIdx.x] = s;  // (keeps the chains live)
}

template <int OP>
double run(int waves_per_simd, int cus, double *clk_mhz) {
  uint32_t *d;
  CHECK(hipMalloc(&d, 1 << 20));
  const int blocks = cus * waves_per_simd;  // 256-thread blocks = one wave per SIMD each
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  valu_kernel<OP><<<blocks, 256>>>(d, 1);  // warm-up
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; rep++) {
    CHECK(hipEventRecord(e0));
    valu_kernel<OP><<<blocks, 256>>>(d, 1);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  CHECK(hipFree(d));
  const double lane_insts = (double)blocks * 256 * ITERS * UNROLL * 8;
  return lane_insts / (best * 1e-3);
  (void)clk_mhz;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const double clk = p.clockRate / 1e3;  // MHz (peak engine clock)
  constexpr int NOPS = 16;
  const char *names[NOPS] = {"v_add_u32", "v_max_i32", "v_max3_i32", "v_add3_u32", "v_pk_add_u16", "v_pk_max_i16",
                             "v_cndmask_b32 (vcc)", "v_cndmask_b32_e64 (sgpr pair)", "v_cmp_gt_i32_e64 + v_cndmask_b32_e64 (pair)",
                             "v_bfi_b32", "v_sad_u8", "v_dot4_u32_u8", "v_mov_b32", "v_sub_u32", "v_max_u32", "v_and_or_b32"};
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_mhz\": %.0f, \"results\": [\n", p.gcnArchName, cus, clk);
  bool first = true;
  for (int o = 0; o < NOPS; o++) {
    for (int w : {1, 2, 4, 8}) {
      double r = 0;
      switch (o) {
        case 0: r = run<0>(w, cus, nullptr); break;
        case 1: r = run<1>(w, cus, nullptr); break;
        case 2: r = run<2>(w, cus, nullptr); break;
        case 3: r = run<3>(w, cus, nullptr); break;
        case 4: r = run<4>(w, cus, nullptr); break;
        case 5: r = run<5>(w, cus, nullptr); break;
        case 6: r = run<6>(w, cus, nullptr); break;
        case 7: r = run<7>(w, cus, nullptr); break;
        case 8: r = run<8>(w, cus, nullptr); break;
        case 9: r = run<9>(w, cus, nullptr); break;
        case 10: r = run<10>(w, cus, nullptr); break;
        case 11: r = run<11>(w, cus, nullptr); break;
        case 12: r = run<12>(w, cus, nullptr); break;
        case 13: r = run<13>(w, cus, nullptr); break;
        case 14: r = run<14>(w, cus, nullptr); break;
        default: r = run<15>(w, cus, nullptr); break;
      }
      printf("%s {\"inst\": \"%s\", \"waves_per_simd\": %d, \"lane_insts_per_s\": %.4e, \"lane_insts_per_clk_per_cu\": %.2f}",
             first ? "" : ",\n", names[o], w, r, r / (clk * 1e6) / cus);
      first = false;
    }
  }
  printf("\n]}\n");
  return 0;
}
