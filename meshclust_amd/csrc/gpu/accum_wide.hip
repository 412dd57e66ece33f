// accum_wide.hip -- accum_kernel instantiations for the wide rows (a wave per candidate: config E,
// k >= 5 at 8 bits) (accum_impl.hpp); a translation unit of its own so the accumulation's variants
// compile in parallel.
#include "accum_impl.hpp"

namespace mcg {

const void *accum_fn_wide(int width, bool prof) {
  if (width == 1) return prof
             ? reinterpret_cast<const void *>(&accum_kernel<uint8_t, 0, true, false, false, false, true>)
             : reinterpret_cast<const void *>(&accum_kernel<uint8_t, 0, true>);
  return prof
             ? reinterpret_cast<const void *>(&accum_kernel<uint16_t, 0, true, false, false, false, true>)
             : reinterpret_cast<const void *>(&accum_kernel<uint16_t, 0, true>);
}

}  // namespace mcg
