// NHWC pooling for Inception-v3, bf16, 8 channels (16 B) per lane.
//
// * avg 3x3, stride 1, pad 1, count_include_pad: y = (1/9) * box(x).  The
//   stencil is symmetric, so the backward dx = (1/9) * box(dy) is the SAME kernel.
// * avg KxK, stride S, no padding (aux head, global pool): direct window sum; backward gathers
//   over the covering windows like the max-pool backward.
// * max KxK, stride S, no padding: forward writes y and, per output element and
//   channel, the argmax offset inside its window as one byte; backward is a
//   gather over the <= ceil(K/S)^2 windows covering each input (no atomics).
//
// A lane owns one (n, h, w) site x 8 channels; neighbouring lanes own the next
// channel groups of the same site, so every wavefront access is a contiguous
// span of the NHWC image and the 3x3 neighbourhood re-reads hit L1/L2.
#include <algorithm>

#include "common.h"

using namespace tony;

namespace {

constexpr int kThreads = 256;

// The 3x3/s1/p1 window sum / 9 of 8 channels at (n, h, w), group cg: all 9 taps loaded before the first
// is summed (clamped to the image, so every address is valid; an out-of-image tap is then masked out):
// the per-tap `continue` made each load wait on the last, which left the fp32 form (2 x 16 B per tap)
// latency-bound at 104 us per 35x35 layer
template <class T>
__device__ __forceinline__ void box3_sum(const T* __restrict__ x, int64_t n, int h, int w, int H, int W, int64_t ldx,
                                         uint32_t cg, float (&acc)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  V8<T> v[9];
#pragma unroll
  for (int dh = 0; dh < 3; ++dh) {
    const int hh = min(max(h + dh - 1, 0), H - 1);
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
      const int ww = min(max(w + dw - 1, 0), W - 1);
      v[dh * 3 + dw] = V8<T>::load(x + ((n * H + hh) * W + ww) * ldx + cg * 8);
    }
  }
#pragma unroll
  for (int dh = 0; dh < 3; ++dh) {
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
      const bool in = (static_cast<unsigned>(h + dh - 1) < static_cast<unsigned>(H)) &&
                      (static_cast<unsigned>(w + dw - 1) < static_cast<unsigned>(W));
      float f[8];
      v[dh * 3 + dw].to_float(f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += in ? f[j] : 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] *= (1.f / 9.f);
}

// ACC: y += box3(x) / 9 (the avg pool's input gradient added into another consumer's, ops/residual.py
// GradJoin: no separate add kernel over the block input)
template <class T, bool ACC = false>
__global__ __launch_bounds__(kThreads) void box3_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                        int N, int H, int W, int C, int64_t ldx, int64_t ldy) {
  // 32-bit index math (the host checks the element count fits): 64-bit div/mod are long
  // instruction sequences and made these memory-bound kernels ALU-bound
  const uint32_t CG = C >> 3;
  const uint32_t total = static_cast<uint32_t>(N) * H * W * CG;
  const uint32_t stride = gridDim.x * kThreads;
  for (uint32_t t = blockIdx.x * kThreads + threadIdx.x; t < total; t += stride) {
    const uint32_t cg = t % CG;
    const uint32_t site = t / CG;
    const int w = static_cast<int>(site % W);
    const uint32_t nh = site / W;
    const int h = static_cast<int>(nh % H);
    float acc[8];
    box3_sum(x, nh / H, h, w, H, W, ldx, cg, acc);
    T* dst = y + static_cast<int64_t>(site) * ldy + cg * 8;
    if (ACC) {
      float o[8];
      V8<T>::load(dst).to_float(o);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += o[j];
    }
    V8<T>::from_float(acc).store(dst);
  }
}

// fp32 avg pool straight to the x3 operand planes of its only consumer conv (ops/x3.py split_act layout:
// [hi | lo | hi] over cp = C channels per row, hi = bf16(v), lo = bf16(v - hi)): the fp32 pooled map is
// never stored or re-read by a split pass.  Rows of y3 are ldy elements apart, plane p starts at column
// p * ps (ps = C: a plane tensor of its own; ps > C: a slice of wider planes, ops/fused.py x3 head)
__global__ __launch_bounds__(kThreads) void box3_x3_kernel(const float* __restrict__ x, uint16_t* __restrict__ y3,
                                                           int N, int H, int W, int C, int64_t ldx, int64_t ldy,
                                                           int64_t ps) {
  const uint32_t CG = C >> 3;
  const uint32_t total = static_cast<uint32_t>(N) * H * W * CG;
  const uint32_t stride = gridDim.x * kThreads;
  for (uint32_t t = blockIdx.x * kThreads + threadIdx.x; t < total; t += stride) {
    const uint32_t cg = t % CG;
    const uint32_t site = t / CG;
    const int w = static_cast<int>(site % W);
    const uint32_t nh = site / W;
    const int h = static_cast<int>(nh % H);
    float acc[8], lo[8];
    box3_sum(x, nh / H, h, w, H, W, ldx, cg, acc);
    const bf16x8 hi = bf16x8::from_float(acc);
    float hf[8];
    hi.to_float(hf);
#pragma unroll
    for (int j = 0; j < 8; ++j) lo[j] = acc[j] - hf[j];
    uint16_t* d = y3 + static_cast<int64_t>(site) * ldy + cg * 8;
    store8(d, hi);
    store8(d + ps, bf16x8::from_float(lo));
    store8(d + 2 * ps, hi);
  }
}

// KT = 3: the window's 9 loads are issued before the first is consumed (the runtime-K loop waits on
// each in turn); 0: any K
// P: zero-padding of the window (torch's max_pool2d padding: padded taps never win; ResNet's stem pool
// is 3x3/2 p1).  With P > 0 each tap is bounds-checked and an out-of-image tap is skipped.
template <int KT, class T = uint16_t>
__global__ __launch_bounds__(kThreads) void maxpool_fwd_kernel(const T* __restrict__ x,
                                                               T* __restrict__ y, uint8_t* __restrict__ arg,
                                                               int N, int H, int W, int C, int OH, int OW, int K,
                                                               int S, int P, int64_t ldx, int64_t ldy) {
  const uint32_t CG = C >> 3;
  const uint32_t total = static_cast<uint32_t>(N) * OH * OW * CG;
  const uint32_t stride = gridDim.x * kThreads;
  for (uint32_t t = blockIdx.x * kThreads + threadIdx.x; t < total; t += stride) {
    const uint32_t cg = t % CG;
    const uint32_t site = t / CG;
    const int ow = static_cast<int>(site % OW);
    const uint32_t nh = site / OW;
    const int oh = static_cast<int>(nh % OH);
    const int64_t n = nh / OH;
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      bi[j] = 0;
    }
    auto take = [&](const V8<T>& raw, uint8_t idx) {
      float f[8];
      raw.to_float(f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (f[j] > best[j] || (f[j] != f[j])) {  // NaN propagates like torch
          best[j] = f[j];
          bi[j] = idx;
        }
      }
    };
    const int h0 = oh * S - P, w0 = ow * S - P;
    if constexpr (KT > 0) {
      if (P == 0) {
        const T* base = x + ((n * H + h0) * W + w0) * ldx + cg * 8;
        const int64_t row = static_cast<int64_t>(W) * ldx;
        V8<T> raw[KT * KT];
#pragma unroll
        for (int kh = 0; kh < KT; ++kh)
#pragma unroll
          for (int kw = 0; kw < KT; ++kw) raw[kh * KT + kw] = V8<T>::load(base + kh * row + kw * ldx);
#pragma unroll
        for (int k = 0; k < KT * KT; ++k) take(raw[k], static_cast<uint8_t>(k));
        } else {  // padded: the in-image taps' loads all issued up front, then consumed
        V8<T> raw[KT * KT];
        bool ok[KT * KT];
#pragma unroll
        for (int kh = 0; kh < KT; ++kh)
#pragma unroll
          for (int kw = 0; kw < KT; ++kw) {
            const int hh = h0 + kh, ww = w0 + kw;
            ok[kh * KT + kw] = static_cast<unsigned>(hh) < static_cast<unsigned>(H) &&
                               static_cast<unsigned>(ww) < static_cast<unsigned>(W);
            if (ok[kh * KT + kw]) raw[kh * KT + kw] = V8<T>::load(x + ((n * H + hh) * W + ww) * ldx + cg * 8);
          }
#pragma unroll
        for (int k = 0; k < KT * KT; ++k)
          if (ok[k]) take(raw[k], static_cast<uint8_t>(k));
      }
    } else {
      for (int kh = 0; kh < K; ++kh) {
        const int hh = h0 + kh;
        if (static_cast<unsigned>(hh) >= static_cast<unsigned>(H)) continue;
        for (int kw = 0; kw < K; ++kw) {
          const int ww = w0 + kw;
          if (static_cast<unsigned>(ww) >= static_cast<unsigned>(W)) continue;
          take(V8<T>::load(x + ((n * H + hh) * W + ww) * ldx + cg * 8), static_cast<uint8_t>(kh * K + kw));
        }
      }
    }
    V8<T>::from_float(best).store(y + static_cast<int64_t>(site) * ldy + cg * 8);
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (static_cast<uint32_t>(bi[3]) << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (static_cast<uint32_t>(bi[7]) << 24);
    *reinterpret_cast<uint2*>(arg + static_cast<int64_t>(site) * C + cg * 8) = packed;
  }
}

// KxK / stride S windows known at compile time (3x3/2: every pool of Inception-v3 and ResNet-50): a dX
// pixel is covered by at most NW = ceil(K / S) windows per dimension; all NW x NW candidates (argmax
// bytes + dY) are loaded before the first is tested -- clamped to the output grid, an out-of-range
// candidate is masked out -- instead of the generic loop's load -> compare -> next-window chain, which
// left the 35x35 / 147x147 backward pools latency-bound (75-135 us per call in the step).
template <int KT, int ST, class T>
__global__ __launch_bounds__(kThreads) void maxpool_bwd_kst_kernel(const T* __restrict__ dy,
                                                                   const uint8_t* __restrict__ arg,
                                                                   T* __restrict__ dx, int N, int H, int W, int C,
                                                                   int OH, int OW, int P, int64_t lddy, int64_t lddx,
                                                                   int accum) {
  constexpr int NW = (KT + ST - 1) / ST;
  const uint32_t CG = C >> 3;
  const uint32_t total = static_cast<uint32_t>(N) * H * W * CG;
  const uint32_t stride = gridDim.x * kThreads;
  for (uint32_t t = blockIdx.x * kThreads + threadIdx.x; t < total; t += stride) {
    const uint32_t cg = t % CG;
    const uint32_t site = t / CG;
    const int w = static_cast<int>(site % W);
    const uint32_t nh = site / W;
    const int h = static_cast<int>(nh % H);
    const int64_t n = nh / H;
    const int hp = h + P, wp = w + P;
    const int oh_lo = hp >= KT ? (hp - KT + ST) / ST : 0;
    const int ow_lo = wp >= KT ? (wp - KT + ST) / ST : 0;
    const int oh_hi = min(OH - 1, hp / ST), ow_hi = min(OW - 1, wp / ST);
    uint2 pk[NW][NW];
    V8<T> g[NW][NW];
#pragma unroll
    for (int a = 0; a < NW; ++a)
#pragma unroll
      for (int b = 0; b < NW; ++b) {
        const int oh = min(oh_lo + a, OH - 1), ow = min(ow_lo + b, OW - 1);
        const int64_t osite = (n * OH + oh) * OW + ow;
        pk[a][b] = *reinterpret_cast<const uint2*>(arg + osite * C + cg * 8);
        g[a][b] = V8<T>::load(dy + osite * lddy + cg * 8);
      }
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int a = 0; a < NW; ++a)
#pragma unroll
      for (int b = 0; b < NW; ++b) {
        const int oh = oh_lo + a, ow = ow_lo + b;
        const bool ok = oh <= oh_hi && ow <= ow_hi;
        const int local = (hp - oh * ST) * KT + (wp - ow * ST);
        float f[8];
        g[a][b].to_float(f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t word = j < 4 ? pk[a][b].x : pk[a][b].y;
          const int bb = (word >> (8 * (j & 3))) & 0xff;
          acc[j] += (ok && bb == local) ? f[j] : 0.f;
        }
      }
    T* d = dx + static_cast<int64_t>(site) * lddx + cg * 8;
    if (accum) {
      float o[8];
      V8<T>::load(d).to_float(o);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += o[j];
    }
    V8<T>::from_float(acc).store(d);
  }
}

template <class T>
__global__ __launch_bounds__(kThreads) void maxpool_bwd_kernel(const T* __restrict__ dy,
                                                               const uint8_t* __restrict__ arg,
                                                               T* __restrict__ dx, int N, int H, int W, int C,
                                                               int OH, int OW, int K, int S, int P, int64_t lddy,
                                                               int64_t lddx, int accum = 0) {
  // accum: dx += the pooled gradient (a tensor with several consumers, ops/residual.py GradJoin)
  const uint32_t CG = C >> 3;
  const uint32_t total = static_cast<uint32_t>(N) * H * W * CG;
  const uint32_t stride = gridDim.x * kThreads;
  for (uint32_t t = blockIdx.x * kThreads + threadIdx.x; t < total; t += stride) {
    const uint32_t cg = t % CG;
    const uint32_t site = t / CG;
    const int w = static_cast<int>(site % W);
    const uint32_t nh = site / W;
    const int h = static_cast<int>(nh % H);
    const int64_t n = nh / H;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // windows oh with oh*S - P <= h <= oh*S - P + K - 1 (hp = h + P: the padded coordinate)
    const int hp = h + P, wp = w + P;
    const int oh_lo = hp >= K ? (hp - K + S) / S : 0;
    const int oh_hi = min(OH - 1, hp / S);
    const int ow_lo = wp >= K ? (wp - K + S) / S : 0;
    const int ow_hi = min(OW - 1, wp / S);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int local = (hp - oh * S) * K + (wp - ow * S);
        const int64_t osite = (n * OH + oh) * OW + ow;
        const uint2 packed = *reinterpret_cast<const uint2*>(arg + osite * C + cg * 8);
        float g[8];
        V8<T>::load(dy + osite * lddy + cg * 8).to_float(g);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t word = j < 4 ? packed.x : packed.y;
          const int b = (word >> (8 * (j & 3))) & 0xff;
          if (b == local) acc[j] += g[j];
        }
      }
    }
    T* d = dx + static_cast<int64_t>(site) * lddx + cg * 8;
    if (accum) {
      float o[8];
      V8<T>::load(d).to_float(o);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += o[j];
    }
    V8<T>::from_float(acc).store(d);
  }
}

// Max-pool backward fused with the BatchNorm-backward reduction of the layer that fed the pool
// (Inception's stem: conv -> BN -> ReLU -> maxpool 3x3/2 at 147x147x64 and 71x71x192, whose BN
// backward then needs dsum[c] = sum dY', dsumx[c] = sum dY' xhat over 354 / 155 MB of Z and dY).
// The pool backward produces every dY element anyway: reading Z beside it and reducing there
// replaces the separate reduce kernel's two full passes by one.  Workgroup-contiguous site ranges,
// one fixed 8-channel group per thread (the BN kernels' RowMap), partial sums folded in LDS and
// added once per workgroup into the sharded [dsum | dsumx] buffer.
__global__ __launch_bounds__(kThreads) void maxpool_bwd_bnred_kernel(
    const uint16_t* __restrict__ dy, const uint8_t* __restrict__ arg, uint16_t* __restrict__ dx, int N, int H,
    int W, int C, int OH, int OW, int K, int S, int P, int64_t lddy, int64_t lddx, int64_t sites_per_block,
    const uint16_t* __restrict__ z, int64_t ldz, const float* __restrict__ mean, const float* __restrict__ invstd,
    const void* gamma, const void* beta, int pb, int relu, float* __restrict__ dsum, int64_t sstride) {
  __shared__ float red[2 * kThreads * 8];
  const int CG = C >> 3, RPI = kThreads / CG;
  const int cg = threadIdx.x % CG, rsub = threadIdx.x / CG;
  const bool active = rsub < RPI;
  float a[8], b[8], p0[8], p1[8], p2[8], p3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = b[j] = 0.f;
    const int c = cg * 8 + j;
    const float mu = mean[c], is = invstd[c];
    const float g = gamma == nullptr ? 1.f : pb ? bf2f(static_cast<const uint16_t*>(gamma)[c])
                                                : static_cast<const float*>(gamma)[c];
    const float be = beta == nullptr ? 0.f : pb ? bf2f(static_cast<const uint16_t*>(beta)[c])
                                                : static_cast<const float*>(beta)[c];
    p0[j] = is;
    p1[j] = -mu * is;
    p2[j] = g * is;
    p3[j] = be - g * is * mu;
  }
  const int64_t total = static_cast<int64_t>(N) * H * W;
  const int64_t s0 = static_cast<int64_t>(blockIdx.x) * sites_per_block;
  const int64_t s1 = min(total, s0 + sites_per_block);
  if (active) {
    // (n, h, w) walked incrementally (one 32-bit decomposition per lane: 64-bit divisions are emulated)
    const uint32_t first = static_cast<uint32_t>(s0 + rsub);
    int w = static_cast<int>(first % static_cast<uint32_t>(W));
    const uint32_t nh0 = first / static_cast<uint32_t>(W);
    int h = static_cast<int>(nh0 % static_cast<uint32_t>(H));
    int64_t n = nh0 / static_cast<uint32_t>(H);
    for (int64_t site = s0 + rsub; site < s1; site += RPI) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      const int hp = h + P, wp = w + P;  // the padded coordinate
      const int oh_lo = hp >= K ? (hp - K + S) / S : 0;
      const int oh_hi = min(OH - 1, hp / S);
      const int ow_lo = wp >= K ? (wp - K + S) / S : 0;
      const int ow_hi = min(OW - 1, wp / S);
      for (int oh = oh_lo; oh <= oh_hi; ++oh) {
        for (int ow = ow_lo; ow <= ow_hi; ++ow) {
          const int local = (hp - oh * S) * K + (wp - ow * S);
          const int64_t osite = (n * OH + oh) * OW + ow;
          const uint2 packed = *reinterpret_cast<const uint2*>(arg + osite * C + cg * 8);
          float g[8];
          load8(dy + osite * lddy + cg * 8).to_float(g);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const uint32_t word = j < 4 ? packed.x : packed.y;
            if (((word >> (8 * (j & 3))) & 0xff) == static_cast<uint32_t>(local)) acc[j] += g[j];
          }
        }
      }
      const bf16x8 o = bf16x8::from_float(acc);
      if (dx != nullptr) store8(dx + site * lddx + cg * 8, o);  // none: the BN apply gathers it again
      float d[8], zf[8];
      o.to_float(d);  // the stored bf16 values, as a separate reduce kernel would read them
      load8(z + site * ldz + cg * 8).to_float(zf);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = (relu && fmaf(zf[j], p2[j], p3[j]) <= 0.f) ? 0.f : d[j];
        a[j] += v;
        b[j] = fmaf(v, fmaf(zf[j], p0[j], p1[j]), b[j]);
      }
      for (w += RPI; w >= W;) {
        w -= W;
        if (++h == H) {
          h = 0;
          ++n;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[rsub * C + cg * 8 + j] = a[j];
      red[kThreads * 8 + rsub * C + cg * 8 + j] = b[j];
    }
  }
  __syncthreads();
  float* ds = dsum + shard_off(blockIdx.x, sstride);
  for (int c = threadIdx.x; c < C; c += kThreads) {
    float sa = 0.f, sb = 0.f;
    for (int k = 0; k < RPI; ++k) {
      sa += red[k * C + c];
      sb += red[kThreads * 8 + k * C + c];
    }
    atomicAdd(ds + c, sa);
    atomicAdd(ds + C + c, sb);
  }
}

// avg KxK, stride S, no padding (Inception aux head 5x5/s3; K = H = W is the global average pool).
template <class T>
__global__ __launch_bounds__(kThreads) void avgpool_fwd_kernel(const T* __restrict__ x,
                                                               T* __restrict__ y, int N, int H, int W, int C,
                                                               int OH, int OW, int K, int S, int64_t ldx,
                                                               int64_t ldy) {
  const uint32_t CG = C >> 3;
  const uint32_t total = static_cast<uint32_t>(N) * OH * OW * CG;
  const uint32_t stride = gridDim.x * kThreads;
  const float inv = 1.f / static_cast<float>(K * K);
  for (uint32_t t = blockIdx.x * kThreads + threadIdx.x; t < total; t += stride) {
    const uint32_t cg = t % CG;
    const uint32_t site = t / CG;
    const int ow = static_cast<int>(site % OW);
    const uint32_t nh = site / OW;
    const int oh = static_cast<int>(nh % OH);
    const int64_t n = nh / OH;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < K; ++r) {
      const int64_t row = (n * H + oh * S + r) * W + ow * S;
      for (int s = 0; s < K; ++s) {
        float v[8];
        V8<T>::load(x + (row + s) * ldx + cg * 8).to_float(v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= inv;
    V8<T>::from_float(acc).store(y + static_cast<int64_t>(site) * ldy + cg * 8);
  }
}

// dx[h, w] = (1/K^2) * sum of dy over the <= ceil(K/S)^2 windows covering (h, w): a gather, no atomics
template <class T>
__global__ __launch_bounds__(kThreads) void avgpool_bwd_kernel(const T* __restrict__ dy,
                                                               T* __restrict__ dx, int N, int H, int W, int C,
                                                               int OH, int OW, int K, int S, int64_t lddy,
                                                               int64_t lddx) {
  const uint32_t CG = C >> 3;
  const uint32_t total = static_cast<uint32_t>(N) * H * W * CG;
  const uint32_t stride = gridDim.x * kThreads;
  const float inv = 1.f / static_cast<float>(K * K);
  for (uint32_t t = blockIdx.x * kThreads + threadIdx.x; t < total; t += stride) {
    const uint32_t cg = t % CG;
    const uint32_t site = t / CG;
    const int w = static_cast<int>(site % W);
    const uint32_t nh = site / W;
    const int h = static_cast<int>(nh % H);
    const int64_t n = nh / H;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int oh_lo = h >= K ? (h - K + S) / S : 0;
    const int oh_hi = min(OH - 1, h / S);
    const int ow_lo = w >= K ? (w - K + S) / S : 0;
    const int ow_hi = min(OW - 1, w / S);
    for (int oh = oh_lo; oh <= oh_hi; ++oh)
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        float g[8];
        V8<T>::load(dy + ((n * OH + oh) * OW + ow) * lddy + cg * 8).to_float(g);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += g[j];
      }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= inv;
    V8<T>::from_float(acc).store(dx + static_cast<int64_t>(site) * lddx + cg * 8);
  }
}

int grid_for(int64_t work) {
  int64_t g = (work + kThreads - 1) / kThreads;
  if (g > 16384) g = 16384;
  return static_cast<int>(g < 1 ? 1 : g);
}

}  // namespace

// y (or dx) = box3x3(x) / 9 over NHWC rows with row strides ldx / ldy.
TONY_API int tony_avgpool3_s1p1(const void* x, void* y, int N, int H, int W, int C, int64_t ldx, int64_t ldy,
                                hipStream_t stream) {
  if (C % 8 || ldx % 8 || ldy % 8 || static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff) return -1;
  box3_kernel<uint16_t><<<grid_for(static_cast<int64_t>(N) * H * W * (C / 8)), kThreads, 0, stream>>>(
      static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), N, H, W, C, ldx, ldy);
  TONY_LAUNCH_CHECK();
  return 0;
}

// Max pool KxK / stride S / zero-padding P (P < K: every window holds an in-image tap), NHWC bf16
// with row strides; argmax: one byte per output element (the winning tap kh*K + kw).
TONY_API int tony_maxpool_fwd(const void* x, void* y, void* argmax, int N, int H, int W, int C, int K, int S, int P,
                              int64_t ldx, int64_t ldy, hipStream_t stream) {
  if (C % 8 || ldx % 8 || ldy % 8 || K * K > 255 || P < 0 || 2 * P >= K + 1 || H + 2 * P < K || W + 2 * P < K ||
      S < 1)
    return -1;
  if (static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff) return -1;
  const int OH = (H + 2 * P - K) / S + 1, OW = (W + 2 * P - K) / S + 1;
  (K == 3 ? maxpool_fwd_kernel<3, uint16_t> : maxpool_fwd_kernel<0, uint16_t>)<<<grid_for(static_cast<int64_t>(N) * OH * OW * (C / 8)), kThreads, 0, stream>>>(
      static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), static_cast<uint8_t*>(argmax), N, H, W, C, OH, OW,
      K, S, P, ldx, ldy);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_maxpool_bwd(const void* dy, const void* argmax, void* dx, int N, int H, int W, int C, int K, int S,
                              int P, int64_t lddy, int64_t lddx, hipStream_t stream) {
  if (C % 8 || lddy % 8 || lddx % 8 || P < 0 || 2 * P >= K + 1 || H + 2 * P < K || W + 2 * P < K || S < 1)
    return -1;
  if (static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff) return -1;
  const int OH = (H + 2 * P - K) / S + 1, OW = (W + 2 * P - K) / S + 1;
  if (K == 3 && S == 2)
    maxpool_bwd_kst_kernel<3, 2, uint16_t><<<grid_for(static_cast<int64_t>(N) * H * W * (C / 8)), kThreads, 0, stream>>>(
        static_cast<const uint16_t*>(dy), static_cast<const uint8_t*>(argmax), static_cast<uint16_t*>(dx), N, H, W, C,
        OH, OW, P, lddy, lddx, 0);
  else
    maxpool_bwd_kernel<uint16_t><<<grid_for(static_cast<int64_t>(N) * H * W * (C / 8)), kThreads, 0, stream>>>(
        static_cast<const uint16_t*>(dy), static_cast<const uint8_t*>(argmax), static_cast<uint16_t*>(dx), N, H, W, C,
        OH, OW, K, S, P, lddy, lddx);
  TONY_LAUNCH_CHECK();
  return 0;
}

// tony_maxpool_bwd adding into dx (dx += the pooled gradient)
TONY_API int tony_maxpool_bwd_acc(const void* dy, const void* argmax, void* dx, int N, int H, int W, int C, int K,
                                  int S, int P, int64_t lddy, int64_t lddx, hipStream_t stream) {
  if (C % 8 || lddy % 8 || lddx % 8 || P < 0 || 2 * P >= K + 1 || H + 2 * P < K || W + 2 * P < K || S < 1)
    return -1;
  if (static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff) return -1;
  const int OH = (H + 2 * P - K) / S + 1, OW = (W + 2 * P - K) / S + 1;
  if (K == 3 && S == 2)
    maxpool_bwd_kst_kernel<3, 2, uint16_t><<<grid_for(static_cast<int64_t>(N) * H * W * (C / 8)), kThreads, 0, stream>>>(
        static_cast<const uint16_t*>(dy), static_cast<const uint8_t*>(argmax), static_cast<uint16_t*>(dx), N, H, W, C,
        OH, OW, P, lddy, lddx, 1);
  else
    maxpool_bwd_kernel<uint16_t><<<grid_for(static_cast<int64_t>(N) * H * W * (C / 8)), kThreads, 0, stream>>>(
        static_cast<const uint16_t*>(dy), static_cast<const uint8_t*>(argmax), static_cast<uint16_t*>(dx), N, H, W, C,
        OH, OW, K, S, P, lddy, lddx, 1);
  TONY_LAUNCH_CHECK();
  return 0;
}

// tony_maxpool_bwd + the BN-backward reduction of Z (the pool input's BN input, rows = dX pixels):
// [dsum | dsumx] (kStatShards copies sstride floats apart, zeroed) accumulate sum dY', sum dY' xhat.
// Padding P as tony_maxpool_bwd; dx == nullptr: the reduction only (bn_act.hip tony_bn_bwd_pool_apply
// gathers dY again, so it is never stored).
TONY_API int tony_maxpool_bwd_bnred(const void* dy, const void* argmax, void* dx, int N, int H, int W, int C, int K,
                                    int S, int P, int64_t lddy, int64_t lddx, const void* z, int64_t ldz,
                                    const float* mean, const float* invstd, const void* gamma, const void* beta, int pb,
                                    int relu, float* dsum, int64_t sstride, int num_cus, hipStream_t stream) {
  if (C % 8 || C > 2048 || lddy % 8 || lddx % 8 || ldz % 8 || P < 0 || 2 * P >= K + 1 || H + 2 * P < K ||
      W + 2 * P < K || S < 1 || z == nullptr || mean == nullptr || invstd == nullptr || dsum == nullptr ||
      (reinterpret_cast<uintptr_t>(z) & 15) || sstride < 0)
    return -1;
  const int64_t total = static_cast<int64_t>(N) * H * W;
  if (total * (C / 8) > 0x7fffffff) return -1;
  const int OH = (H + 2 * P - K) / S + 1, OW = (W + 2 * P - K) / S + 1;
  // 4 workgroups per CU: 16 measured slower (187 vs 166 us at ResNet's 112x112x64 stem)
  const int64_t blocks = std::min<int64_t>(4 * static_cast<int64_t>(num_cus > 0 ? num_cus : 256),
                                           (total + 63) / 64);
  const int64_t per = (total + blocks - 1) / blocks;
  maxpool_bwd_bnred_kernel<<<static_cast<int>((total + per - 1) / per), kThreads, 0, stream>>>(
      static_cast<const uint16_t*>(dy), static_cast<const uint8_t*>(argmax), static_cast<uint16_t*>(dx), N, H, W, C,
      OH, OW, K, S, P, lddy, lddx, per, static_cast<const uint16_t*>(z), ldz, mean, invstd, gamma, beta, pb, relu, dsum,
      sstride);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_avgpool_fwd(const void* x, void* y, int N, int H, int W, int C, int K, int S, int64_t ldx,
                              int64_t ldy, hipStream_t stream) {
  if (C % 8 || ldx % 8 || ldy % 8 || K < 1 || S < 1 || H < K || W < K) return -1;
  if (static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff) return -1;
  const int OH = (H - K) / S + 1, OW = (W - K) / S + 1;
  avgpool_fwd_kernel<uint16_t><<<grid_for(static_cast<int64_t>(N) * OH * OW * (C / 8)), kThreads, 0, stream>>>(
      static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), N, H, W, C, OH, OW, K, S, ldx, ldy);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_avgpool_bwd(const void* dy, void* dx, int N, int H, int W, int C, int K, int S, int64_t lddy,
                              int64_t lddx, hipStream_t stream) {
  if (C % 8 || lddy % 8 || lddx % 8 || K < 1 || S < 1 || H < K || W < K) return -1;
  if (static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff) return -1;
  const int OH = (H - K) / S + 1, OW = (W - K) / S + 1;
  avgpool_bwd_kernel<uint16_t><<<grid_for(static_cast<int64_t>(N) * H * W * (C / 8)), kThreads, 0, stream>>>(
      static_cast<const uint16_t*>(dy), static_cast<uint16_t*>(dx), N, H, W, C, OH, OW, K, S, lddy, lddx);
  TONY_LAUNCH_CHECK();
  return 0;
}

// ---- fp32 forms (the x3 fp32 step, ops/x3.py): the same kernels on float rows ----------------------
TONY_API int tony_avgpool3_s1p1_f32(const void* x, void* y, int N, int H, int W, int C, int64_t ldx, int64_t ldy,
                                    hipStream_t stream) {
  if (C % 8 || ldx % 4 || ldy % 4 || static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff) return -1;
  box3_kernel<float><<<grid_for(static_cast<int64_t>(N) * H * W * (C / 8)), kThreads, 0, stream>>>(
      static_cast<const float*>(x), static_cast<float*>(y), N, H, W, C, ldx, ldy);
  TONY_LAUNCH_CHECK();
  return 0;
}

// fp32 x -> the x3 planes [N*H*W][3C] of box3x3(x) / 9 (C % 8 == 0)
TONY_API int tony_avgpool3_s1p1_x3(const void* x, void* y3, int N, int H, int W, int C, int64_t ldx,
                                   hipStream_t stream) {
  if (C % 8 || ldx % 4 || (reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(y3) & 15) ||
      static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff)
    return -1;
  box3_x3_kernel<<<grid_for(static_cast<int64_t>(N) * H * W * (C / 8)), kThreads, 0, stream>>>(
      static_cast<const float*>(x), static_cast<uint16_t*>(y3), N, H, W, C, ldx, 3 * C, C);
  TONY_LAUNCH_CHECK();
  return 0;
}

// the same into channels [0, C) of wider planes: rows ldy3 elements apart, plane p at column p * pstride
TONY_API int tony_avgpool3_s1p1_x3p(const void* x, void* y3, int N, int H, int W, int C, int64_t ldx, int64_t ldy3,
                                    int64_t pstride, hipStream_t stream) {
  if (C % 8 || ldx % 4 || ldy3 % 8 || pstride % 8 || pstride < C || ldy3 < 2 * pstride + C ||
      (reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(y3) & 15) ||
      static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff)
    return -1;
  box3_x3_kernel<<<grid_for(static_cast<int64_t>(N) * H * W * (C / 8)), kThreads, 0, stream>>>(
      static_cast<const float*>(x), static_cast<uint16_t*>(y3), N, H, W, C, ldx, ldy3, pstride);
  TONY_LAUNCH_CHECK();
  return 0;
}

// y += box3x3(x) / 9 (fp32 / bf16 rows: ``f32``)
TONY_API int tony_avgpool3_s1p1_acc(const void* x, void* y, int N, int H, int W, int C, int64_t ldx, int64_t ldy,
                                    int f32, hipStream_t stream) {
  if (C % 8 || ldx % 8 || ldy % 8 || static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff) return -1;
  const int g = grid_for(static_cast<int64_t>(N) * H * W * (C / 8));
  if (f32)
    box3_kernel<float, true><<<g, kThreads, 0, stream>>>(static_cast<const float*>(x), static_cast<float*>(y), N, H,
                                                          W, C, ldx, ldy);
  else
    box3_kernel<uint16_t, true><<<g, kThreads, 0, stream>>>(static_cast<const uint16_t*>(x),
                                                             static_cast<uint16_t*>(y), N, H, W, C, ldx, ldy);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_maxpool_fwd_f32(const void* x, void* y, void* argmax, int N, int H, int W, int C, int K, int S,
                                  int P, int64_t ldx, int64_t ldy, hipStream_t stream) {
  if (C % 8 || ldx % 4 || ldy % 4 || K * K > 255 || P < 0 || 2 * P >= K + 1 || H + 2 * P < K || W + 2 * P < K ||
      S < 1)
    return -1;
  if (static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff) return -1;
  const int OH = (H + 2 * P - K) / S + 1, OW = (W + 2 * P - K) / S + 1;
  (K == 3 ? maxpool_fwd_kernel<3, float> : maxpool_fwd_kernel<0, float>)<<<grid_for(static_cast<int64_t>(N) * OH * OW * (C / 8)), kThreads, 0, stream>>>(
      static_cast<const float*>(x), static_cast<float*>(y), static_cast<uint8_t*>(argmax), N, H, W, C, OH, OW, K, S,
      P, ldx, ldy);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_maxpool_bwd_f32(const void* dy, const void* argmax, void* dx, int N, int H, int W, int C, int K,
                                  int S, int P, int64_t lddy, int64_t lddx, hipStream_t stream) {
  if (C % 8 || lddy % 4 || lddx % 4 || P < 0 || 2 * P >= K + 1 || H + 2 * P < K || W + 2 * P < K || S < 1)
    return -1;
  if (static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff) return -1;
  const int OH = (H + 2 * P - K) / S + 1, OW = (W + 2 * P - K) / S + 1;
  if (K == 3 && S == 2)
    maxpool_bwd_kst_kernel<3, 2, float><<<grid_for(static_cast<int64_t>(N) * H * W * (C / 8)), kThreads, 0, stream>>>(
        static_cast<const float*>(dy), static_cast<const uint8_t*>(argmax), static_cast<float*>(dx), N, H, W, C, OH,
        OW, P, lddy, lddx, 0);
  else
    maxpool_bwd_kernel<float><<<grid_for(static_cast<int64_t>(N) * H * W * (C / 8)), kThreads, 0, stream>>>(
        static_cast<const float*>(dy), static_cast<const uint8_t*>(argmax), static_cast<float*>(dx), N, H, W, C, OH,
        OW, K, S, P, lddy, lddx);
  TONY_LAUNCH_CHECK();
  return 0;
}

// tony_maxpool_bwd_f32 adding into dx (the x3 blocks' block-input gradient join, ops/pool.py)
TONY_API int tony_maxpool_bwd_acc_f32(const void* dy, const void* argmax, void* dx, int N, int H, int W, int C, int K,
                                  int S, int P, int64_t lddy, int64_t lddx, hipStream_t stream) {
  if (C % 8 || lddy % 4 || lddx % 4 || P < 0 || 2 * P >= K + 1 || H + 2 * P < K || W + 2 * P < K || S < 1)
    return -1;
  if (static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff) return -1;
  const int OH = (H + 2 * P - K) / S + 1, OW = (W + 2 * P - K) / S + 1;
  if (K == 3 && S == 2)
    maxpool_bwd_kst_kernel<3, 2, float><<<grid_for(static_cast<int64_t>(N) * H * W * (C / 8)), kThreads, 0, stream>>>(
        static_cast<const float*>(dy), static_cast<const uint8_t*>(argmax), static_cast<float*>(dx), N, H, W, C, OH,
        OW, P, lddy, lddx, 1);
  else
    maxpool_bwd_kernel<float><<<grid_for(static_cast<int64_t>(N) * H * W * (C / 8)), kThreads, 0, stream>>>(
        static_cast<const float*>(dy), static_cast<const uint8_t*>(argmax), static_cast<float*>(dx), N, H, W, C, OH,
        OW, K, S, P, lddy, lddx, 1);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_avgpool_fwd_f32(const void* x, void* y, int N, int H, int W, int C, int K, int S, int64_t ldx,
                                  int64_t ldy, hipStream_t stream) {
  if (C % 8 || ldx % 4 || ldy % 4 || K < 1 || S < 1 || H < K || W < K) return -1;
  if (static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff) return -1;
  const int OH = (H - K) / S + 1, OW = (W - K) / S + 1;
  avgpool_fwd_kernel<float><<<grid_for(static_cast<int64_t>(N) * OH * OW * (C / 8)), kThreads, 0, stream>>>(
      static_cast<const float*>(x), static_cast<float*>(y), N, H, W, C, OH, OW, K, S, ldx, ldy);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_avgpool_bwd_f32(const void* dy, void* dx, int N, int H, int W, int C, int K, int S, int64_t lddy,
                                  int64_t lddx, hipStream_t stream) {
  if (C % 8 || lddy % 4 || lddx % 4 || K < 1 || S < 1 || H < K || W < K) return -1;
  if (static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff) return -1;
  const int OH = (H - K) / S + 1, OW = (W - K) / S + 1;
  avgpool_bwd_kernel<float><<<grid_for(static_cast<int64_t>(N) * H * W * (C / 8)), kThreads, 0, stream>>>(
      static_cast<const float*>(dy), static_cast<float*>(dx), N, H, W, C, OH, OW, K, S, lddy, lddx);
  TONY_LAUNCH_CHECK();
  return 0;
}
