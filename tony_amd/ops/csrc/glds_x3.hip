// The fused-plane x3 (fp32) LDS-DMA conv kernels (igemm.h X3Planes, codes kX3First..), compiled here only.
#include "glds_launch.h"

namespace tony {
namespace glds {
template int run_glds_part<true, 0>(const Gather&, const void*, int64_t, void*, int64_t, int64_t, int64_t, int, float*,
                                    int64_t, int, hipStream_t, RowMap, BTaps, int, X3Planes, const MultiClass*);
}  // namespace glds
}  // namespace tony
