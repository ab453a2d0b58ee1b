// Batched conv-weight transpose [Co][R][S][Ci] -> [Ci][R][S][Co] for every conv of a model in ONE
// launch (the backward-data GEMMs read W with the output channels contiguous).
//
// Weights change only at the optimizer step, so the trainer refreshes all transposed copies once per
// step right after the PS apply (ops/wt_cache.py) instead of every dgrad transposing its own weight
// (≈70 small torch copy kernels per Inception-v3 step).  Work list: one descriptor per weight; every
// workgroup transposes one 64 x 64 (co x ci) tile of one tap through LDS (row padded by one element:
// the column read is bank-conflict free), with 16-byte row loads where the tile is full width.
#include "common.h"

using namespace tony;

namespace {

struct TDesc {
  const uint16_t* src;  // [Co][RS][Ci]
  uint16_t* dst;        // [Ci][RS][Co]
  int co, rs, ci;
  int tiles_ci, tiles_co;
  int tile_begin;       // prefix sum of tiles over the descriptors
};

constexpr int T = 64;

__global__ __launch_bounds__(256) void transpose_batch_kernel(const TDesc* __restrict__ descs, int n) {
  __shared__ uint16_t tile[T][T + 2];
  // locate this workgroup's descriptor (binary search over the tile prefix sums; n is ~100)
  const int b = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (descs[mid].tile_begin <= b) lo = mid; else hi = mid - 1;
  }
  const TDesc d = descs[lo];
  int t = b - d.tile_begin;
  const int tci = t % d.tiles_ci;
  t /= d.tiles_ci;
  const int tco = t % d.tiles_co;
  const int tap = t / d.tiles_co;
  const int co0 = tco * T, ci0 = tci * T;
  const int64_t src_row = static_cast<int64_t>(d.rs) * d.ci;  // elements between consecutive co
  const int64_t dst_row = static_cast<int64_t>(d.rs) * d.co;  // elements between consecutive ci
  // load: 64 rows (co) x 64 cols (ci); thread -> (row = tid / 4 + 64 k / 4 ..., 16 elements)
  for (int v = threadIdx.x; v < T * (T / 8); v += 256) {
    const int r = v >> 3, c8 = (v & 7) * 8;
    const int co = co0 + r, ci = ci0 + c8;
    const uint16_t* p = d.src + co * src_row + static_cast<int64_t>(tap) * d.ci + ci;
    if (co < d.co && ci + 8 <= d.ci && (reinterpret_cast<uintptr_t>(p) & 15) == 0) {
      const uint4 q = *reinterpret_cast<const uint4*>(p);
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        tile[r][c8 + 2 * e] = static_cast<uint16_t>(w[e] & 0xffff);
        tile[r][c8 + 2 * e + 1] = static_cast<uint16_t>(w[e] >> 16);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) tile[r][c8 + e] = (co < d.co && ci + e < d.ci) ? p[e] : 0;
    }
  }
  __syncthreads();
  // store: 64 rows (ci) x 64 cols (co)
  for (int v = threadIdx.x; v < T * (T / 8); v += 256) {
    const int r = v >> 3, c8 = (v & 7) * 8;
    const int ci = ci0 + r, co = co0 + c8;
    if (ci >= d.ci) continue;
    uint16_t* p = d.dst + ci * dst_row + static_cast<int64_t>(tap) * d.co + co;
    if (co + 8 <= d.co && (reinterpret_cast<uintptr_t>(p) & 15) == 0) {
      uint32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        w[e] = static_cast<uint32_t>(tile[c8 + 2 * e][r]) | (static_cast<uint32_t>(tile[c8 + 2 * e + 1][r]) << 16);
      *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      for (int e = 0; e < 8 && co + e < d.co; ++e) p[e] = tile[c8 + e][r];
    }
  }
}

}  // namespace

// Size in bytes of one descriptor (the Python side packs the work list to match).
TONY_API int tony_transpose_desc_bytes() { return static_cast<int>(sizeof(TDesc)); }

// descs: device array of n descriptors (tile_begin filled in, ascending); total_tiles = sum of tiles.
TONY_API int tony_transpose_batch(const void* descs, int n, int total_tiles, hipStream_t stream) {
  if (n <= 0 || total_tiles <= 0 || descs == nullptr) return -1;
  transpose_batch_kernel<<<total_tiles, 256, 0, stream>>>(static_cast<const TDesc*>(descs), n);
  TONY_LAUNCH_CHECK();
  return 0;
}
