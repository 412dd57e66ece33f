// accum_chunk.hip -- accum_kernel instantiations for the 512-position chunk workers (resident or
// streamed rows; MC_ACCUM_NO_DENSE / _STREAM / _COMPACT) (accum_impl.hpp); a translation unit of
// its own so the accumulation's variants compile in parallel.
#include "accum_impl.hpp"

namespace mcg {

const void *accum_fn_chunk(int width, int nch, bool compact) {
  if (compact) return reinterpret_cast<const void *>(&accum_kernel<uint8_t, 16, false, true>);
  if (width == 1 && nch == 16) return reinterpret_cast<const void *>(&accum_kernel<uint8_t, 16>);
  if (width == 1) return reinterpret_cast<const void *>(&accum_kernel<uint8_t, 0>);
  return reinterpret_cast<const void *>(&accum_kernel<uint16_t, 0>);
}

}  // namespace mcg
