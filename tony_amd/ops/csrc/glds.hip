// The LDS-DMA conv / GEMM entry (igemm.h run_glds / run_glds_x3): argument checks, then the variant's
// family launcher (glds_p0..3.hip, glds_x3.hip -- one translation unit each, compiled in parallel).
#include "igemm.h"

namespace tony {
namespace glds {

namespace {
int checks(const Gather& g, const void* B, int64_t ldb, const void* C, int64_t ldc, X3Planes xp, BTaps bt,
           int stream_m, const MultiClass* classes, bool x3) {
  if (classes != nullptr && (x3 || stream_m > 0 || xp.atab != nullptr || classes->n < 1 || classes->n > kMaxClasses))
    return -1;
  if (x3 != (xp.btap != 0)) return -1;
  if (xp.atab != nullptr && (x3 || bt.S != 0 || (reinterpret_cast<uintptr_t>(xp.atab) & 15))) return -1;
  if ((ldc % 8) || (ldb % 8) || (reinterpret_cast<uintptr_t>(C) & 15) || (reinterpret_cast<uintptr_t>(B) & 15) ||
      (reinterpret_cast<uintptr_t>(g.src) & 15) || (g.ld % 8) || (g.K % 8))
    return -3;
  return 0;
}
}  // namespace

int run_glds(const Gather& g, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N, int epi,
             float* st, int64_t sstride, int v, hipStream_t stream, RowMap rmap, BTaps bt, int stream_m, X3Planes xp,
             const MultiClass* classes) {
  if (const int rc = checks(g, B, ldb, C, ldc, xp, bt, stream_m, classes, false)) return rc;
  if (v < kGldsFirst || v >= kGldsFirst + kNumGlds) return -3;
  switch (glds_part(v - kGldsFirst)) {
    case 0: return run_glds_part<false, 0>(g, B, ldb, C, ldc, M, N, epi, st, sstride, v, stream, rmap, bt, stream_m, xp, classes);
    case 1: return run_glds_part<false, 1>(g, B, ldb, C, ldc, M, N, epi, st, sstride, v, stream, rmap, bt, stream_m, xp, classes);
    case 2: return run_glds_part<false, 2>(g, B, ldb, C, ldc, M, N, epi, st, sstride, v, stream, rmap, bt, stream_m, xp, classes);
    case 3: return run_glds_part<false, 3>(g, B, ldb, C, ldc, M, N, epi, st, sstride, v, stream, rmap, bt, stream_m, xp, classes);
    default: return -3;
  }
}

int run_glds_x3(const Gather& g, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N, int epi,
                float* st, int64_t sstride, int v, hipStream_t stream, RowMap rmap, BTaps bt, int stream_m,
                X3Planes xp) {
  if (const int rc = checks(g, B, ldb, C, ldc, xp, bt, stream_m, nullptr, true)) return rc;
  if (v < kX3First || v >= kX3First + kNumX3 || bt.S != 0 || (xp.alo % 8) || (xp.blo % 8) || (xp.btap % 8))
    return -3;
  return run_glds_part<true, 0>(g, B, ldb, C, ldc, M, N, epi, st, sstride, v, stream, rmap, bt, stream_m, xp, nullptr);
}

}  // namespace glds
}  // namespace tony
