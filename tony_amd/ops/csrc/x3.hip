// fp32 training on the bf16 matrix cores: the "x3" operand split (ops/x3.py).
//
// An fp32 value x is carried as two bf16 values, hi = bf16(x) and lo = bf16(x - hi), with
// |x - hi - lo| <= 2^-17 |x|.  A product x*w is then hi_x*hi_w + lo_x*hi_w + hi_x*lo_w, dropping
// lo_x*lo_w (<= 2^-16 |x w|): the three bf16 x bf16 products are exact in the MFMA and summed in its
// fp32 accumulator.  Laying the operands out as three channel planes -- activations [hi | lo | hi],
// weights [hi | hi | lo] -- turns the whole fp32 convolution into ONE bf16 implicit GEMM over 3x the
// channels, on the same tuned MFMA kernels as the bf16 step, with the fp32 epilogue of
// mfma_common.h nt_epilogue (flag bit 3).  Per product the error is ~2^-16 relative: coarser than
// fp32's 2^-24, 32x finer than the TF32 (10-bit mantissa) that TensorFlow's fp32 convolutions use on
// tensor-core GPUs.
//
// Planes are padded to cp = round_up(C, 8) channels so every plane starts 16-byte aligned (the 3-channel
// image stem: cp = 8, zero-filled) -- the weight planes use the same cp, so padding columns multiply
// zeros by zeros.
#include "common.h"

using namespace tony;

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ void split1(float x, uint16_t& hi, uint16_t& lo) {
  hi = f2bf(x);
  lo = f2bf(x - bf2f(hi));
}

// src fp32 [rows][C] (row stride lds) -> dst bf16 [rows][3 * cp] (row stride ldd); pattern bit p set:
// plane p holds lo, clear: hi.  One thread per (row, 4-channel group of cp).
__global__ __launch_bounds__(kThreads) void split3_kernel(const float* __restrict__ src, int64_t lds, int64_t rows,
                                                          int C, int cp, uint16_t* __restrict__ dst, int64_t ldd,
                                                          int pattern, int vec, int pst) {
  const int G = cp >> 2;
  const int64_t total = rows * G;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * kThreads) {
    const int64_t r = t / G;
    const int c = static_cast<int>(t - r * G) * 4;
    const float* s = src + r * lds + c;
    float v[4];
    if (vec && c + 4 <= C) {
      const float4 q = *reinterpret_cast<const float4*>(s);
      v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = c + j < C ? s[j] : 0.f;
    }
    uint16_t hi[4], lo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) split1(v[j], hi[j], lo[j]);
    const uint2 H = make_uint2(hi[0] | (static_cast<uint32_t>(hi[1]) << 16), hi[2] | (static_cast<uint32_t>(hi[3]) << 16));
    const uint2 L = make_uint2(lo[0] | (static_cast<uint32_t>(lo[1]) << 16), lo[2] | (static_cast<uint32_t>(lo[3]) << 16));
    uint16_t* d = dst + r * ldd + c;
#pragma unroll
    for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(d + p * pst) = (pattern >> p) & 1 ? L : H;
  }
}

// w fp32 [Co][RS][C] -> dst bf16 [C][RS][3 * Co] with planes [hi | hi | lo] over Co: the backward-data
// weights (csrc/conv.hip tony_conv_dgrad's Wt = W permuted to [C][R][S][Co]) of an x3 conv.
__global__ __launch_bounds__(kThreads) void wt_split3_kernel(const float* __restrict__ w, int Co, int RS, int C,
                                                             uint16_t* __restrict__ dst) {
  const int64_t total = static_cast<int64_t>(C) * RS * Co;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * kThreads) {
    const int co = static_cast<int>(t % Co);
    const int64_t crs = t / Co;
    const int rs = static_cast<int>(crs % RS);
    const int c = static_cast<int>(crs / RS);
    uint16_t hi, lo;
    split1(w[(static_cast<int64_t>(co) * RS + rs) * C + c], hi, lo);
    uint16_t* d = dst + crs * (3 * static_cast<int64_t>(Co)) + co;
    d[0] = hi;
    d[Co] = hi;
    d[2 * Co] = lo;
  }
}

// Both x3 weight layouts of every conv of a model in ONE launch after the optimizer step (ops/wt_cache.py
// X3Weights): the forward planes [Co][RS][3cp] ([hi | hi | lo] over the cp channels, zero past C) and the
// backward-data planes [C][RS][3Co] ([hi | hi | lo] over Co) of the fp32 weight [Co][RS][C] -- instead of
// two split launches per conv per step on the critical path (~190 per Inception-v3 step).  One workgroup
// per 64 (co) x 64 (c) tile of one tap, staged through LDS as fp32 (row padded by one float: the column
// reads of the transposed store are conflict free).
struct XDesc {
  const float* src;  // [Co][RS][C]
  uint16_t* fwd;     // [Co][RS][3cp]
  uint16_t* bwd;     // [C][RS][3Co]
  int co, rs, c, cp;
  int tiles_c, tiles_co;
  int tile_begin;
  int pad;
};

constexpr int XT = 64;

__global__ __launch_bounds__(kThreads) void x3_weights_batch_kernel(const XDesc* __restrict__ descs, int n) {
  __shared__ float tile[XT][XT + 1];
  const int b = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (descs[mid].tile_begin <= b) lo = mid; else hi = mid - 1;
  }
  const XDesc d = descs[lo];
  int t = b - d.tile_begin;
  const int tc = t % d.tiles_c;
  t /= d.tiles_c;
  const int tco = t % d.tiles_co;
  const int tap = t / d.tiles_co;
  const int co0 = tco * XT, c0 = tc * XT;
  // load 64 (co) x 64 (c) fp32; channels past C (the cp padding) read as zero
  for (int v = threadIdx.x; v < XT * (XT / 4); v += kThreads) {
    const int r = v >> 4, c4 = (v & 15) * 4;
    const int co = co0 + r, c = c0 + c4;
    const float* p = d.src + (static_cast<int64_t>(co) * d.rs + tap) * d.c + c;
#pragma unroll
    for (int e = 0; e < 4; ++e) tile[r][c4 + e] = (co < d.co && c + e < d.c) ? p[e] : 0.f;
  }
  __syncthreads();
  // forward planes: row (co, tap), columns c .. c + 3 of each plane
  for (int v = threadIdx.x; v < XT * (XT / 4); v += kThreads) {
    const int r = v >> 4, c4 = (v & 15) * 4;
    const int co = co0 + r, c = c0 + c4;
    if (co >= d.co || c >= d.cp) continue;
    uint16_t h[4], l[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) split1(tile[r][c4 + e], h[e], l[e]);
    const uint2 H = make_uint2(h[0] | (static_cast<uint32_t>(h[1]) << 16), h[2] | (static_cast<uint32_t>(h[3]) << 16));
    const uint2 L = make_uint2(l[0] | (static_cast<uint32_t>(l[1]) << 16), l[2] | (static_cast<uint32_t>(l[3]) << 16));
    uint16_t* q = d.fwd + (static_cast<int64_t>(co) * d.rs + tap) * (3 * d.cp) + c;
    *reinterpret_cast<uint2*>(q) = H;
    *reinterpret_cast<uint2*>(q + d.cp) = H;
    *reinterpret_cast<uint2*>(q + 2 * d.cp) = L;
  }
  // backward-data planes: row (c, tap), columns co .. co + 3 of each plane
  for (int v = threadIdx.x; v < XT * (XT / 4); v += kThreads) {
    const int r = v >> 4, o4 = (v & 15) * 4;
    const int c = c0 + r, co = co0 + o4;
    if (c >= d.c || co >= d.co) continue;
    uint16_t h[4], l[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) split1(tile[o4 + e][r], h[e], l[e]);
    const uint2 H = make_uint2(h[0] | (static_cast<uint32_t>(h[1]) << 16), h[2] | (static_cast<uint32_t>(h[3]) << 16));
    const uint2 L = make_uint2(l[0] | (static_cast<uint32_t>(l[1]) << 16), l[2] | (static_cast<uint32_t>(l[3]) << 16));
    uint16_t* q = d.bwd + (static_cast<int64_t>(c) * d.rs + tap) * (3 * d.co) + co;
    *reinterpret_cast<uint2*>(q) = H;
    *reinterpret_cast<uint2*>(q + d.co) = H;
    *reinterpret_cast<uint2*>(q + 2 * d.co) = L;
  }
}

int grid_for(int64_t work) {
  int64_t g = (work + kThreads - 1) / kThreads;
  if (g > 8192) g = 8192;
  return static_cast<int>(g < 1 ? 1 : g);
}

}  // namespace

TONY_API int tony_x3_split(const void* src, int64_t lds, int64_t rows, int C, int cp, void* dst, int64_t ldd,
                           int pattern, hipStream_t stream) {
  if (src == nullptr || dst == nullptr || rows < 0 || C <= 0 || cp < C || (cp % 8) || lds < C || ldd < 3 * cp ||
      (ldd % 4) || (reinterpret_cast<uintptr_t>(dst) & 7) || pattern < 0 || pattern > 7)
    return -1;
  if (rows == 0) return 0;
  const int vec = (C % 4 == 0) && (lds % 4 == 0) && !(reinterpret_cast<uintptr_t>(src) & 15);
  split3_kernel<<<grid_for(rows * (cp / 4)), kThreads, 0, stream>>>(static_cast<const float*>(src), lds, rows, C, cp,
                                                                     static_cast<uint16_t*>(dst), ldd, pattern, vec, cp);
  TONY_LAUNCH_CHECK();
  return 0;
}

// tony_x3_split of a channel slice into a wider planes buffer: dst = the slice's first column of a
// [rows][3 * pst] planes buffer (plane p at column p * pst); C % 8 == 0 (no padding columns written)
TONY_API int tony_x3_split_slice(const void* src, int64_t lds, int64_t rows, int C, void* dst, int64_t ldd, int pst,
                                 int pattern, hipStream_t stream) {
  if (src == nullptr || dst == nullptr || rows < 0 || C <= 0 || (C % 8) || pst < C || (pst % 4) || lds < C ||
      ldd < 3 * pst || (ldd % 4) || (reinterpret_cast<uintptr_t>(dst) & 7) || pattern < 0 || pattern > 7)
    return -1;
  if (rows == 0) return 0;
  const int vec = (lds % 4 == 0) && !(reinterpret_cast<uintptr_t>(src) & 15);
  split3_kernel<<<grid_for(rows * (C / 4)), kThreads, 0, stream>>>(static_cast<const float*>(src), lds, rows, C, C,
                                                                    static_cast<uint16_t*>(dst), ldd, pattern, vec,
                                                                    pst);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_x3_weights_t(const void* w, int Co, int RS, int C, void* dst, hipStream_t stream) {
  if (w == nullptr || dst == nullptr || Co <= 0 || RS <= 0 || C <= 0 || (Co % 8)) return -1;
  wt_split3_kernel<<<grid_for(static_cast<int64_t>(C) * RS * Co), kThreads, 0, stream>>>(
      static_cast<const float*>(w), Co, RS, C, static_cast<uint16_t*>(dst));
  TONY_LAUNCH_CHECK();
  return 0;
}

// Size in bytes of one x3 weight descriptor (ops/wt_cache.py packs the work list to match).
TONY_API int tony_x3_desc_bytes() { return static_cast<int>(sizeof(XDesc)); }

// descs: device array of n XDesc (tile_begin ascending, Co % 4 == 0 and cp % 8 == 0 for the vector stores);
// total_tiles = sum over descriptors of rs * tiles_c * tiles_co.
TONY_API int tony_x3_weights_batch(const void* descs, int n, int total_tiles, hipStream_t stream) {
  if (n <= 0 || total_tiles <= 0 || descs == nullptr) return -1;
  x3_weights_batch_kernel<<<total_tiles, kThreads, 0, stream>>>(static_cast<const XDesc*>(descs), n);
  TONY_LAUNCH_CHECK();
  return 0;
}
