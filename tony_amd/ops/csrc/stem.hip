// Direct (non-GEMM) forward convolution for 3-channel image stems, with the BatchNorm statistics
// epilogue of the implicit-GEMM kernels (conv.hip tony_conv_fwd flags bit0).
//
// Inception-v3's first layer (128x3x299x299 -> 32, 3x3/2) has a K of 27: an MFMA tile would be
// 70 % padding and the tony GEMM kernels need C % 8 == 0 (zero-padding the input to 8 channels
// measured slower than MIOpen: profiles/r1_rejected_stem_pad8.log).  The layer is bound by its
// 250 MB of HBM traffic, not by math (4.9 GFLOP), so this kernel runs it on the vector ALUs:
// each thread owns kPix output pixels x 32 channels in fp32 registers, the fp32 weight panel
// [R*S*3][32] sits in LDS and is read with wave-uniform ds_read_b128 broadcasts, and the 3
// input channels of each tap are loaded straight from the NHWC image (L1/L2 absorb the 3x3
// window overlap; a workgroup's input rows are first staged into LDS with 16-B loads when they
// form one contiguous range).  Output pixels are assigned so adjacent lanes store adjacent 64-B pixel rows.
// Statistics: per-thread sums over its pixels -> an LDS transpose [32][threads] -> 8 lanes per
// channel -> one sharded atomic per channel per workgroup.
#include "common.h"

namespace {

using namespace tony;

constexpr int kThreads = 256;
constexpr int kCo = 32;
constexpr int kPix = 4;
constexpr int kMaxTaps = 49;                // R*S <= 7x7
constexpr int kRedLd = kThreads + 1;        // padded row of the statistics transpose
constexpr int kPatch = 24576;               // bf16 elements of the staged input rows (48 KB)
static_assert(kCo * kRedLd * 4 <= kPatch * 2, "the statistics transpose reuses the patch buffer");

__global__ __launch_bounds__(kThreads) void stem_fwd_kernel(const uint16_t* __restrict__ x, int H, int W,
                                                            const float* __restrict__ wf, int R, int S, int sh,
                                                            int sw, int ph, int pw, uint16_t* __restrict__ y, int OH,
                                                            int OW, int64_t ldy, int M, int64_t total,
                                                            float* __restrict__ stats, int64_t sstride) {
  __shared__ __attribute__((aligned(16))) uint16_t patch[kPatch];
  float* red = reinterpret_cast<float*>(patch);  // after the FMAs: statistics transpose [kCo][kRedLd]

  const int ohw = OH * OW;
  // The workgroup's pixels are consecutive output rows of one image (unless it straddles two):
  // their input rows are one contiguous NHWC byte range, staged into LDS with 16-B loads instead
  // of 3 x 2-B gathers per tap and lane.  Straddling / oversized ranges read global memory.
  const int m_first = blockIdx.x * kPix * kThreads;
  const int m_last = min(M, m_first + kPix * kThreads) - 1;
  const int n0 = m_first / ohw, n1 = m_last / ohw;
  const int ya = max(0, (m_first - n0 * ohw) / OW * sh - ph);
  const int yb = min(H - 1, (m_last - n1 * ohw) / OW * sh - ph + R - 1);
  const int64_t e0a = ((static_cast<int64_t>(n0) * H + ya) * W * 3) & ~static_cast<int64_t>(7);
  const int64_t e1r = (((static_cast<int64_t>(n0) * H + yb + 1) * W * 3) + 7) & ~static_cast<int64_t>(7);
  const bool staged = n0 == n1 && ya <= yb && e1r - e0a <= kPatch;
  if (staged) {
    for (int64_t k = e0a + threadIdx.x * 8; k < e1r; k += kThreads * 8) {
      uint16_t* d = patch + (k - e0a);
      if (k + 8 <= total) {
        *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(x + k);
      } else {
        for (int j = 0; j < 8; ++j) d[j] = k + j < total ? x[k + j] : 0;
      }
    }
  }
  __syncthreads();

  int64_t xb[kPix];
  int iy0[kPix], ix0[kPix];
  bool valid[kPix];
#pragma unroll
  for (int p = 0; p < kPix; ++p) {
    const int m = (blockIdx.x * kPix + p) * kThreads + threadIdx.x;
    valid[p] = m < M;
    const int mm = valid[p] ? m : 0;
    const int n = mm / ohw, rem = mm - n * ohw;
    const int oy = rem / OW, ox = rem - oy * OW;
    iy0[p] = oy * sh - ph;
    ix0[p] = ox * sw - pw;
    xb[p] = static_cast<int64_t>(n) * H * W * 3;
  }

  float acc[kPix][kCo];
#pragma unroll
  for (int p = 0; p < kPix; ++p)
#pragma unroll
    for (int c = 0; c < kCo; ++c) acc[p][c] = 0.f;

  // taps flattened and software-pipelined one ahead: the 3 x kPix input loads of tap t+1 are in
  // flight while tap t's 96 x kPix FMAs (v_pk_fma_f32) run (only 2 waves per SIMD at ~200 VGPRs)
  auto load_tap = [&](int t, float (&v)[kPix][3]) {
    const int r = t / S, s = t - (t / S) * S;
#pragma unroll
    for (int p = 0; p < kPix; ++p) {
      const int iy = iy0[p] + r, ix = ix0[p] + s;
      const bool in = valid[p] && static_cast<unsigned>(iy) < static_cast<unsigned>(H) &&
                      static_cast<unsigned>(ix) < static_cast<unsigned>(W);
      // clamped address: out-of-image taps load pixel (0,0) of the same image and are zeroed, so
      // no load can leave the tensor even if the compiler hoists it above the select
      const int64_t off = xb[p] + (static_cast<int64_t>(in ? iy : 0) * W + (in ? ix : 0)) * 3;
      if (staged) {  // in-image taps of this workgroup's pixels lie in [e0a, e1r) by construction
        const uint16_t* src = patch + (in ? off - e0a : 0);
#pragma unroll
        for (int c = 0; c < 3; ++c) v[p][c] = in ? bf2f(src[c]) : 0.f;
      } else {
        const uint16_t* src = x + off;
#pragma unroll
        for (int c = 0; c < 3; ++c) v[p][c] = in ? bf2f(src[c]) : 0.f;
      }
    }
  };
  const int RS = R * S;
  float v[kPix][3];
  load_tap(0, v);
  for (int t = 0; t < RS; ++t) {
    float vn[kPix][3];
    load_tap(t + 1 < RS ? t + 1 : t, vn);
    // wave-uniform fp32 weights [tap][c][co] from global memory: scalar loads into SGPRs that the
    // v_pk_fma_f32 take as operands (no LDS traffic in the inner loop)
    const float4* wk = reinterpret_cast<const float4*>(wf + t * 3 * kCo);
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int q = 0; q < kCo / 4; ++q) {
        const float4 wv = wk[c * (kCo / 4) + q];
#pragma unroll
        for (int p = 0; p < kPix; ++p) {
          acc[p][4 * q + 0] = fmaf(v[p][c], wv.x, acc[p][4 * q + 0]);
          acc[p][4 * q + 1] = fmaf(v[p][c], wv.y, acc[p][4 * q + 1]);
          acc[p][4 * q + 2] = fmaf(v[p][c], wv.z, acc[p][4 * q + 2]);
          acc[p][4 * q + 3] = fmaf(v[p][c], wv.w, acc[p][4 * q + 3]);
        }
      }
#pragma unroll
    for (int p = 0; p < kPix; ++p)
#pragma unroll
      for (int c = 0; c < 3; ++c) v[p][c] = vn[p][c];
  }

#pragma unroll
  for (int p = 0; p < kPix; ++p) {
    if (!valid[p]) continue;
    const int m = (blockIdx.x * kPix + p) * kThreads + threadIdx.x;
    uint4* dst = reinterpret_cast<uint4*>(y + static_cast<int64_t>(m) * ldy);
#pragma unroll
    for (int q = 0; q < kCo / 8; ++q) dst[q] = bf16x8::from_float(&acc[p][8 * q]).raw;
  }

  if (stats == nullptr) return;  // uniform over the workgroup
  __syncthreads();  // every lane is done reading the patch: it becomes the statistics transpose
  float* st = stats + shard_off(blockIdx.x, sstride);
  constexpr int kSeg = kThreads / kCo;  // lanes per channel in the final sum (8, adjacent lanes)
  constexpr int kLen = kThreads / kSeg;
#pragma unroll
  for (int which = 0; which < 2; ++which) {  // 0: sum, 1: sum of squares (of the fp32 accumulators)
#pragma unroll
    for (int c = 0; c < kCo; ++c) {
      float t = 0.f;
#pragma unroll
      for (int p = 0; p < kPix; ++p) {
        const float a = valid[p] ? acc[p][c] : 0.f;
        t = which ? fmaf(a, a, t) : t + a;
      }
      red[c * kRedLd + threadIdx.x] = t;
    }
    __syncthreads();
    const int c = threadIdx.x / kSeg, seg = threadIdx.x - c * kSeg;
    float t = 0.f;
    for (int j = 0; j < kLen; ++j) t += red[c * kRedLd + seg * kLen + j];
#pragma unroll
    for (int o = 1; o < kSeg; o <<= 1) t += __shfl_xor(t, o, 64);
    if (seg == 0) atomicAdd(st + which * kCo + c, t);
    __syncthreads();  // red is rewritten by the next pass
  }
}

}  // namespace

// Y[N*OH*OW, 32] (row stride ldy) = conv(X [N,H,W,3] dense NHWC bf16, W fp32 [R][S][3][32]).
// flags bit0: per-channel [sum | sumsq] of Y into stats (zero on entry; kStatShards copies sstride
// floats apart when sstride > 0), the layout tony_conv_fwd uses.
TONY_API int tony_stem_fwd(const void* x, int N, int H, int W, int C, const void* w, int Co, int R, int S, int sh,
                           int sw, int ph, int pw, void* y, int OH, int OW, int64_t ldy, int flags, float* stats,
                           int64_t sstride, hipStream_t stream) {
  if (C != 3 || Co != kCo || (reinterpret_cast<uintptr_t>(w) & 15) || R <= 0 || S <= 0 || R * S > kMaxTaps || sh <= 0 || sw <= 0 || ph < 0 || pw < 0 ||
      sstride < 0 || ldy < kCo || (ldy % 8) || (reinterpret_cast<uintptr_t>(y) & 15))
    return -1;
  if (OH != (H + 2 * ph - R) / sh + 1 || OW != (W + 2 * pw - S) / sw + 1 || OH <= 0 || OW <= 0) return -1;
  const int64_t M = static_cast<int64_t>(N) * OH * OW;
  if (M > 0x7fffffff - kPix * kThreads) return -1;  // 32-bit pixel index in the kernel
  if ((flags & 1) && stats == nullptr) return -1;
  const int64_t per = static_cast<int64_t>(kPix) * kThreads;
  const int grid = static_cast<int>((M + per - 1) / per);
  stem_fwd_kernel<<<grid, kThreads, 0, stream>>>(static_cast<const uint16_t*>(x), H, W,
                                                 static_cast<const float*>(w), R, S, sh, sw, ph, pw,
                                                 static_cast<uint16_t*>(y), OH, OW, ldy, static_cast<int>(M),
                                                 static_cast<int64_t>(N) * H * W * 3, (flags & 1) ? stats : nullptr,
                                                 sstride);
  return 0;
}
