// LDS-DMA conv / GEMM kernels of variant family 2 (igemm.h glds_part), compiled here and nowhere else.
#include "glds_launch.h"

namespace tony {
namespace glds {
template int run_glds_part<false, 2>(const Gather&, const void*, int64_t, void*, int64_t, int64_t, int64_t, int, float*,
                                      int64_t, int, hipStream_t, RowMap, BTaps, int, X3Planes, const MultiClass*);
}  // namespace glds
}  // namespace tony
