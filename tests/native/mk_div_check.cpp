// The accumulation workers' division by a constant (features.hpp mk_div: q0 = RN(a y),
// RN(q0 + (a - b q0) y) with y = RN(1 / b)) equals IEEE a / b: exhaustively for the centre's
// mag / B at every magnitude below 2^24 and the histogram sizes 4^k (pterms_mk), and on random
// operands of the kinds classify_small divides (an integer or a [0, 1] value minus a minimum,
// over a range RN(max - min), both within FastCls::mk's 2^-200 .. 2^200).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

static double mk_div(double a, double b, double y) {
  const double q0 = a * y;
  return std::fma(std::fma(-q0, b, a), y, q0);
}
static uint64_t s = 0x9e3779b97f4a7c15ull;
static uint64_t xr() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double ud() { return (double)(xr() >> 11) * 0x1p-53; }
static double any(int lo, int hi) {
  const double m = 1.0 + (double)(xr() >> 12) * 0x1p-52;
  const double v = std::ldexp(m, lo + (int)(xr() % (uint64_t)(hi - lo + 1)));
  return (xr() & 1) ? -v : v;
}
static bool same(double x, double y) { return std::memcmp(&x, &y, 8) == 0 || (std::isnan(x) && std::isnan(y)); }

int main() {
  long bad = 0;
  for (int k = 1; k <= 8; k++) {
    const double B = (double)(1u << (2 * k)), y = 1.0 / B;
    for (uint32_t m = 0; m < (1u << 24); m += (k <= 4 ? 1u : 7u))
      if (!same(mk_div((double)m, B, y), (double)m / B)) bad++;
  }
  for (long it = 0; it < 20000000L; it++) {
    const double mn = (it & 3) == 0 ? 0.0 : any(-200, 40), mx = mn + any(-200, 40);
    const double b = mx - mn;
    if (!(b != 0 && std::isfinite(b) && std::fabs(b) >= 0x1p-200)) continue;
    const double y = 1.0 / b;
    const double v = (it & 1) ? (double)(xr() % 2000000) : ud();
    const double a = v - mn;
    if (!same(mk_div(a, b, y), a / b)) {
      if (bad < 5) std::printf("a=%a b=%a\n", a, b);
      bad++;
    }
  }
  if (bad) {
    std::printf("FAIL %ld\n", bad);
    return 1;
  }
  std::printf("OK\n");
  return 0;
}
