// accum_dense.hip -- accum_kernel instantiations for the dense resident workers (worker_dense:
// configs A, B, E at k <= 4 and a rank's share of D) (accum_impl.hpp); a translation unit of its
// own so the accumulation's variants compile in parallel.
#include "accum_impl.hpp"

namespace mcg {

const void *accum_fn_dense(int width, int nch, bool prof) {
  if (width == 1 && nch == 16) return prof
             ? reinterpret_cast<const void *>(&accum_kernel<uint8_t, 16, false, false, true, false, true>)
             : reinterpret_cast<const void *>(&accum_kernel<uint8_t, 16, false, false, true>);
  if (width == 1) return prof
             ? reinterpret_cast<const void *>(&accum_kernel<uint8_t, 0, false, false, true, false, true>)
             : reinterpret_cast<const void *>(&accum_kernel<uint8_t, 0, false, false, true>);
  return prof
             ? reinterpret_cast<const void *>(&accum_kernel<uint16_t, 0, false, false, true, false, true>)
             : reinterpret_cast<const void *>(&accum_kernel<uint16_t, 0, false, false, true>);
}

}  // namespace mcg
