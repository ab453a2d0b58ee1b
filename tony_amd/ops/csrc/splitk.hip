// Split-K combine for the weight-gradient GEMMs (conv.hip conv_wgrad_kernel, gemm.hip
// gemm_tn_splitk_kernel): dst[i] (+)= sum over s of slab[s * n + i].
//
// The wgrad kernels split the huge M = N*H*W reduction over ~2 workgroups per CU.  Adding every
// partial tile into one fp32 dW with float atomics costs splits x |dW| x 4 bytes at the chip-wide
// atomic rate (MI355X_MICROARCH.md, 'Global float atomics': ~1.3 TB/s) -- 25 MB, ~19 us, for a
// 17x17 Inception conv -- so the partials are stored plainly to a slab and summed here, and the sum
// lands directly in the parameter's (bf16 or fp32) flat-gradient slot: no zero-fill of a dW
// accumulator, no separate accumulate kernel.
#include <algorithm>

#include "common.h"

using namespace tony;

namespace {

// Block = 64 float4 columns x 4 split groups: group g sums splits g, g+4, ... (four independent
// loads in flight per thread per round), the groups combine through LDS, group 0 writes.
constexpr int kCols = 64, kGroups = 4;

// blockIdx.y = chunk of `chunk` splits (rows rstride floats apart) summed into dst + blockIdx.y * dstride:
// one chunk of all splits (the combine), or the first of two passes when the columns alone cannot
// fill the GPU -- a stem layer's ~10 K floats over 512 splits ran 34-66 us as 20-36 workgroups each
// walking all 512 rows; pass 1 sums chunks in place (chunk g's sum over its own first row, read only
// by this workgroup), pass 2 the chunk sums.
template <bool BF16>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* slab, int splits, int chunk,
                                                            int64_t n, int64_t rstride, void* dst,
                                                            int64_t dstride, int accumulate) {
  __shared__ float4 part[kGroups - 1][kCols];
  const int col = threadIdx.x % kCols, grp = threadIdx.x / kCols;
  const int64_t n4 = n >> 2;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kCols + col;
  const int s0 = blockIdx.y * chunk;
  splits = min(splits - s0, chunk);
  dst = BF16 ? static_cast<void*>(static_cast<uint16_t*>(dst) + blockIdx.y * dstride)
             : static_cast<void*>(static_cast<float*>(dst) + blockIdx.y * dstride);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) {
    const float4* base = reinterpret_cast<const float4*>(slab + s0 * rstride) + i;
    const int64_t stride = rstride >> 2;  // float4s between consecutive splits
    int k = grp;
    for (; k + 3 * kGroups < splits; k += 4 * kGroups) {
      const float4 a = base[(k)*stride], b = base[(k + kGroups) * stride];
      const float4 c = base[(k + 2 * kGroups) * stride], d = base[(k + 3 * kGroups) * stride];
      s.x += (a.x + b.x) + (c.x + d.x);
      s.y += (a.y + b.y) + (c.y + d.y);
      s.z += (a.z + b.z) + (c.z + d.z);
      s.w += (a.w + b.w) + (c.w + d.w);
    }
    for (; k < splits; k += kGroups) {
      const float4 a = base[k * stride];
      s.x += a.x;
      s.y += a.y;
      s.z += a.z;
      s.w += a.w;
    }
  }
  if (grp > 0) part[grp - 1][col] = s;
  __syncthreads();
  if (grp > 0 || i >= n4) return;
#pragma unroll
  for (int g = 0; g < kGroups - 1; ++g) {
    const float4 v = part[g][col];
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  if (BF16) {
    uint2* p = reinterpret_cast<uint2*>(dst) + i;
    float a0 = s.x, a1 = s.y, a2 = s.z, a3 = s.w;
    if (accumulate) {
      const uint2 o = *p;
      a0 += __uint_as_float(o.x << 16);
      a1 += __uint_as_float(o.x & 0xffff0000u);
      a2 += __uint_as_float(o.y << 16);
      a3 += __uint_as_float(o.y & 0xffff0000u);
    }
    *p = make_uint2(static_cast<uint32_t>(f2bf(a0)) | (static_cast<uint32_t>(f2bf(a1)) << 16),
                    static_cast<uint32_t>(f2bf(a2)) | (static_cast<uint32_t>(f2bf(a3)) << 16));
  } else {
    float4* p = reinterpret_cast<float4*>(dst) + i;
    if (accumulate) {
      const float4 o = *p;
      s.x += o.x;
      s.y += o.y;
      s.z += o.z;
      s.w += o.w;
    }
    *p = s;
  }
}

}  // namespace

// n % 4 == 0; slab 16-B aligned, dst 8-B (bf16) / 16-B (fp32) aligned.  The slab is scratch: with
// fewer column blocks than CUs and >= 32 splits the first pass overwrites chunk rows with their sums.
TONY_API int tony_splitk_reduce(const float* slab, int splits, int64_t n, void* dst, int dst_bf16, int accumulate,
                                int num_cus, hipStream_t stream) {
  if (slab == nullptr || dst == nullptr || splits <= 0 || n <= 0 || (n % 4)) return -1;
  if ((reinterpret_cast<uintptr_t>(slab) & 15) || (reinterpret_cast<uintptr_t>(dst) & (dst_bf16 ? 7 : 15))) return -1;
  const int64_t grid = (n / 4 + kCols - 1) / kCols;
  if (grid > 0x7fffffff) return -2;
  const int cus = num_cus > 0 ? num_cus : 256;
  int64_t rstride = n;
  if (grid < cus && splits >= 32) {  // pass 1: chunks of >= 16 splits spread the columns over ~2 x CUs
    const int want = static_cast<int>(std::min<int64_t>((2 * cus + grid - 1) / grid, splits / 16));
    const int chunk = (splits + want - 1) / want;
    const int groups = (splits + chunk - 1) / chunk;
    float* s = const_cast<float*>(slab);
    splitk_reduce_kernel<false><<<dim3(static_cast<unsigned>(grid), groups), 256, 0, stream>>>(
        slab, splits, chunk, n, n, s, chunk * n, 0);
    TONY_LAUNCH_CHECK();
    rstride = chunk * n;
    splits = groups;
  }
  if (dst_bf16)
    splitk_reduce_kernel<true><<<static_cast<int>(grid), 256, 0, stream>>>(slab, splits, splits, n, rstride, dst, 0,
                                                                          accumulate);
  else
    splitk_reduce_kernel<false><<<static_cast<int>(grid), 256, 0, stream>>>(slab, splits, splits, n, rstride, dst, 0,
                                                                           accumulate);
  TONY_LAUNCH_CHECK();
  return 0;
}
