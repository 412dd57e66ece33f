// accum_dstream.hip -- accum_kernel instantiations for the dense streaming workers (worker_dstream:
// config D on one to four GPUs) (accum_impl.hpp); a translation unit of its own so the
// accumulation's variants compile in parallel.
#include "accum_impl.hpp"

namespace mcg {

const void *accum_fn_dstream(int width, int nch, bool prof) {
  if (width == 1 && nch == 16) return prof
             ? reinterpret_cast<const void *>(&accum_kernel<uint8_t, 16, false, false, false, true, true>)
             : reinterpret_cast<const void *>(&accum_kernel<uint8_t, 16, false, false, false, true>);
  if (width == 1) return reinterpret_cast<const void *>(&accum_kernel<uint8_t, 0, false, false, false, true>);
  return reinterpret_cast<const void *>(&accum_kernel<uint16_t, 0, false, false, false, true>);
}

}  // namespace mcg
