// NHWC BatchNorm (+ optional ReLU) for training and inference, bf16 activations.
//
// This is the fused "BN+ReLU" of every Inception-v3 BasicConv2d and ResNet
// conv-bn-relu.  Layout is NHWC flattened to [M, C]
// rows (M = N*H*W) with a row stride `ld` so a branch output can be written
// straight into its channel slice of an Inception concat buffer (H7).
//
// Forward  = stats kernel (per-channel sum / sum-of-squares, fp32, LDS tree +
//            one device atomic per channel per workgroup) + apply kernel
//            (normalise, affine, ReLU, bf16 store).  Every workgroup of the
//            apply kernel rebuilds scale/shift for all C channels in LDS from
//            the sums, so no finalize launch is needed.
// Backward = reduce kernel (sum dy', sum dy'*xhat with the ReLU mask
//            recomputed from x, so y is never re-read) + apply kernel.
//
// Thread map: one 16-byte (8-channel) vector per lane; a 256-thread workgroup
// covers RPI = 256/(C/8) rows per iteration, so a wavefront always reads a
// contiguous 1 KiB span of the row-major image (fully coalesced for any C%8==0).
#include <algorithm>
#include <cstdlib>

#include "common.h"

using namespace tony;

namespace {

constexpr int kThreads = 256;
constexpr int kMaxC = 2048;
// Per-channel tables and block reductions live in dynamic LDS sized to the layer's C (not kMaxC):
// a 17x17 / 35x35 layer's BN kernel then takes ~1-16 KB instead of 16-40 KB, so it co-resides with
// the LDS-heavy MFMA kernels of the other streams (wgrad 144 KB per CU) and runs at full occupancy.
extern __shared__ __attribute__((aligned(16))) float bn_dyn[];
inline size_t bn_lds_table(int C, int rows) { return static_cast<size_t>(rows) * C * sizeof(float); }
inline size_t bn_lds_reduce(int C) {  // block_reduce_add: [2][RPI][C]
  return static_cast<size_t>(2) * (kThreads / (C / 8)) * C * sizeof(float);
}
inline size_t bn_lds_bred(int C) { return std::max(bn_lds_table(C, 4), bn_lds_reduce(C)); }

struct RowMap {
  int CG, RPI, cg, rsub;
  bool active;
  __device__ RowMap(int C) {
    CG = C >> 3;
    RPI = kThreads / CG;
    cg = threadIdx.x % CG;
    rsub = threadIdx.x / CG;
    active = rsub < RPI;
  }
};

// Column segments of a multi-output BN pass -- the 1x1 splits of a fused Inception head (ops/fused.py):
// columns [end[s-1], end[s]) of the [M, C] tensor live in tensor p[s] (its column 0) with row stride
// ld[s], so ONE launch normalises (or back-propagates) every split.  n == 0: the plain pointer.
struct Segs {
  int n = 0;
  int end[4] = {0, 0, 0, 0};
  void* p[4] = {nullptr, nullptr, nullptr, nullptr};
  int64_t ld[4] = {0, 0, 0, 0};
  template <class T>
  __device__ __forceinline__ void resolve(int col, T*& base, int64_t& ld_out) const {
    int s = 0, start = 0;
    while (s + 1 < n && col >= end[s]) {
      start = end[s];
      ++s;
    }
    base = static_cast<T*>(p[s]) + (col - start);
    ld_out = ld[s];
  }
};

__device__ __forceinline__ float load_param(const void* p, int idx, int is_bf16, float dflt) {
  if (p == nullptr) return dflt;
  return is_bf16 ? bf2f(static_cast<const uint16_t*>(p)[idx]) : static_cast<const float*>(p)[idx];
}

// accumulate=1 adds into an existing gradient (flat grad buffer, zeroed once per step)
__device__ __forceinline__ void store_param(void* p, int idx, int is_bf16, float v, int accumulate) {
  if (p == nullptr) return;
  if (is_bf16) {
    uint16_t* q = static_cast<uint16_t*>(p) + idx;
    *q = f2bf(accumulate ? bf2f(*q) + v : v);
  } else {
    float* q = static_cast<float*>(p) + idx;
    *q = accumulate ? *q + v : v;
  }
}

// Reduce per-thread partials over the RPI row-lanes in LDS and add one value
// per channel into global `out` (2*C floats: [sum | sum2]).
__device__ __forceinline__ void block_reduce_add(float* red, const RowMap& rm, int C,
                                                 const float* a, const float* b, float* out_a, float* out_b) {
  if (rm.active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[rm.rsub * C + rm.cg * 8 + j] = a[j];
      red[rm.RPI * C + rm.rsub * C + rm.cg * 8 + j] = b[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kThreads) {
    float sa = 0.f, sb = 0.f;
    for (int k = 0; k < rm.RPI; ++k) {
      sa += red[k * C + c];
      sb += red[rm.RPI * C + k * C + c];
    }
    atomicAdd(out_a + c, sa);
    atomicAdd(out_b + c, sb);
  }
}

template <class T>
__global__ __launch_bounds__(kThreads) void bn_fwd_stats_kernel(
    const T* __restrict__ x, int64_t M, int C, int64_t ldx, int64_t rows_per_block,
    float* __restrict__ sum, float* __restrict__ sumsq, int64_t sstride) {
  float* red = bn_dyn;  // bn_lds_reduce(C) bytes
  RowMap rm(C);
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  if (rm.active) {
    const T* base = x + rm.cg * 8;
    int64_t r = r0 + rm.rsub;
    const int64_t step = rm.RPI;
    for (; r + 3 * step < r1; r += 4 * step) {
      V8<T> v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = V8<T>::load(base + (r + u * step) * ldx);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float f[8];
        v[u].to_float(f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] += f[j];
          q[j] = fmaf(f[j], f[j], q[j]);
        }
      }
    }
    for (; r < r1; r += step) {
      float f[8];
      V8<T>::load(base + r * ldx).to_float(f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += f[j];
        q[j] = fmaf(f[j], f[j], q[j]);
      }
    }
  }
  const int64_t so = shard_off(blockIdx.x, sstride);
  block_reduce_add(red, rm, C, s, q, sum + so, sumsq + so);
}

// mode 0: training (stats from sums, saves mean/invstd, updates running stats)
// mode 1: inference (stats from running_mean / running_var)
// RES: y = act(bn(x) + res)  (ResNet bottleneck tail: BN + identity add + ReLU in one pass)
// mask (RES form, optional): one byte per 8 channels of a row (bit j: y > 0 for channel 8 * cg + j,
// row stride ldm bytes) -- the ReLU mask the backward needs, 1/16 of the bytes of re-reading y
// X3 (T = float, the fp32 step of ops/x3.py): y is written as the bf16 [hi | lo | hi] planes the next
// convolution reads (row stride ldy >= 3C in bf16 elements, plane p at column p * C) instead of fp32 --
// for a layer whose only consumer is another x3 conv, the fp32 y and the split pass over it are never made
template <bool RES, class T = uint16_t, bool X3 = false>
__global__ __launch_bounds__(kThreads) void bn_fwd_apply_kernel(
    const T* __restrict__ x, int64_t M, int C, int64_t ldx, int64_t rows_per_block,
    const T* __restrict__ res, int64_t ldr,
    T* __restrict__ y, int64_t ldy, const float* __restrict__ sum, const float* __restrict__ sumsq,
    int64_t sstride, const void* gamma, const void* beta, int param_bf16, float eps, int relu, int mode,
    float* __restrict__ save_mean, float* __restrict__ save_invstd,
    float* __restrict__ running_mean, float* __restrict__ running_var, float momentum, Segs segs,
    uint8_t* __restrict__ mask = nullptr, int64_t ldm = 0, uint16_t* __restrict__ p3 = nullptr, int64_t ldp = 0,
    int64_t pst = 0) {
  float* scale = bn_dyn;  // [C] then shift [C]: bn_lds_table(C, 2) bytes
  float* shift = bn_dyn + C;
  const float inv_m = 1.f / static_cast<float>(M);
  for (int c = threadIdx.x; c < C; c += kThreads) {
    float mean, invstd;
    if (mode == 0) {
      mean = shard_sum(sum, c, sstride) * inv_m;
      float var = fmaxf(shard_sum(sumsq, c, sstride) * inv_m - mean * mean, 0.f);
      invstd = rsqrtf(var + eps);
      if (blockIdx.x == 0) {
        save_mean[c] = mean;
        save_invstd[c] = invstd;
        if (running_mean != nullptr) {
          const float unbiased = M > 1 ? var * (static_cast<float>(M) / static_cast<float>(M - 1)) : var;
          running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
          running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
        }
      }
    } else {
      mean = running_mean[c];
      invstd = rsqrtf(running_var[c] + eps);
    }
    const float g = load_param(gamma, c, param_bf16, 1.f);
    const float b = load_param(beta, c, param_bf16, 0.f);
    scale[c] = g * invstd;
    shift[c] = b - mean * g * invstd;
  }
  __syncthreads();
  RowMap rm(C);
  if (!rm.active) return;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = scale[rm.cg * 8 + j];
    sh[j] = shift[rm.cg * 8 + j];
  }
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  const int64_t step = rm.RPI;
  int64_t r = r0 + rm.rsub;
  T* yb = y + rm.cg * 8;
  int64_t ldyt = ldy;
  if (segs.n > 0) segs.resolve(rm.cg * 8, yb, ldyt);
  auto body = [&](const V8<T>& v, const V8<T>& rv, int64_t row) {
    float f[8], q[8];
    v.to_float(f);
    if (RES) rv.to_float(q);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = fmaf(f[j], sc[j], sh[j]);
      if (RES) t += q[j];
      f[j] = relu ? relu_f(t) : t;
    }
    if constexpr (X3) {
      const V8<uint16_t> hi = V8<uint16_t>::from_float(f);
      float hf[8], lo[8];
      hi.to_float(hf);
#pragma unroll
      for (int j = 0; j < 8; ++j) lo[j] = f[j] - hf[j];
      uint16_t* d = reinterpret_cast<uint16_t*>(y) + row * ldy + rm.cg * 8;
      hi.store(d);
      V8<uint16_t>::from_float(lo).store(d + C);
      hi.store(d + 2 * C);
      return;
    }
    const V8<T> out = V8<T>::from_float(f);
    out.store(yb + row * ldyt);
    // also the x3 planes of y (a concat slot's slice of the block's planes); fp32 rows only -- compiled out of
    // the bf16 kernel (the runtime test alone cost it 18 VGPRs: 100 -> 118, one wave per SIMD fewer)
    if constexpr (!X3 && std::is_same<T, float>::value) {
      if (p3 != nullptr) {
        const V8<uint16_t> hi = V8<uint16_t>::from_float(f);
        float hf[8], lo[8];
        hi.to_float(hf);
#pragma unroll
        for (int j = 0; j < 8; ++j) lo[j] = f[j] - hf[j];
        uint16_t* d = p3 + row * ldp + rm.cg * 8;
        hi.store(d);
        V8<uint16_t>::from_float(lo).store(d + pst);
        hi.store(d + 2 * pst);
      }
    }
    if (RES && mask != nullptr) {  // the stored values' sign, exactly what re-reading y would test
      float g[8];
      out.to_float(g);
      unsigned b = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) b |= (g[j] > 0.f ? 1u : 0u) << j;
      mask[row * ldm + rm.cg] = static_cast<uint8_t>(b);
    }
  };
  V8<T> none{};
  for (; r + 3 * step < r1; r += 4 * step) {
    V8<T> v[4], rv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v[u] = V8<T>::load(x + (r + u * step) * ldx + rm.cg * 8);
      if (RES) rv[u] = V8<T>::load(res + (r + u * step) * ldr + rm.cg * 8);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) body(v[u], RES ? rv[u] : none, r + u * step);
  }
  for (; r < r1; r += step)
    body(V8<T>::load(x + r * ldx + rm.cg * 8), RES ? V8<T>::load(res + r * ldr + rm.cg * 8) : none, r);
}

// Backward reduction: dsums[c] = sum(dy'), dsums[C+c] = sum(dy' * xhat),
// where dy' = dy masked by the ReLU (recomputed from x), or -- YMASK, the
// residual form where the ReLU followed an add -- masked by the saved output y.
// Per-channel coefficients are built once per workgroup in LDS (xhat = x*p0 + p1,
// pre-activation = x*p2 + p3), so no lane waits on scattered parameter loads.
// MB (with YMASK): ym is the forward's byte mask (bn_fwd_apply_kernel mask, row stride ldym bytes)
// instead of y
template <bool YMASK, class T = uint16_t, bool MB = false>
__global__ __launch_bounds__(kThreads) void bn_bwd_reduce_kernel(
    const T* __restrict__ x, int64_t ldx, const T* __restrict__ dy, int64_t lddy,
    const T* __restrict__ ym, int64_t ldym,
    int64_t M, int C, int64_t rows_per_block, const float* __restrict__ mean,
    const float* __restrict__ invstd, const void* gamma, const void* beta, int param_bf16,
    int relu, float* __restrict__ dsum, float* __restrict__ dsumx, int64_t sstride, Segs segs) {
  float* red = bn_dyn;  // coefficient table [4][C] first, then the block reduction (bn_lds_bred)
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const float mu = mean[c], is = invstd[c];
    const float g = load_param(gamma, c, param_bf16, 1.f), be = load_param(beta, c, param_bf16, 0.f);
    red[c] = is;
    red[C + c] = -mu * is;
    red[2 * C + c] = g * is;
    red[3 * C + c] = be - g * is * mu;
  }
  __syncthreads();
  RowMap rm(C);
  float a[8], b[8];
  float p0[8], p1[8], p2[8], p3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = b[j] = 0.f;
    const int c = (rm.active ? rm.cg * 8 : 0) + j;
    p0[j] = red[c];
    p1[j] = red[C + c];
    p2[j] = red[2 * C + c];
    p3[j] = red[3 * C + c];
  }
  __syncthreads();  // the table is dead: red is reused by block_reduce_add
  if (rm.active) {
    const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
    const int64_t r1 = min(M, r0 + rows_per_block);
    const int64_t step = rm.RPI;
    const uint8_t* mbp = reinterpret_cast<const uint8_t*>(ym) + rm.cg;
    auto body = [&](const V8<T>& xv, const V8<T>& gv, const V8<T>& yv, unsigned mbits) {
      float xf[8], gf[8], yf[8];
      xv.to_float(xf);
      gv.to_float(gf);
      if (YMASK && !MB) yv.to_float(yf);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = fmaf(xf[j], p0[j], p1[j]);
        float d = gf[j];
        if (YMASK && MB) {
          if (!((mbits >> j) & 1u)) d = 0.f;
        } else if (YMASK) {
          if (yf[j] <= 0.f) d = 0.f;
        } else if (relu && fmaf(xf[j], p2[j], p3[j]) <= 0.f) {
          d = 0.f;
        }
        a[j] += d;
        b[j] = fmaf(d, xh, b[j]);
      }
    };
    V8<T> none{};
    const T* db = dy + rm.cg * 8;
    int64_t lddt = lddy;
    if (segs.n > 0) {
      T* b;
      segs.resolve(rm.cg * 8, b, lddt);
      db = b;
    }
    int64_t r = r0 + rm.rsub;
    for (; r + 3 * step < r1; r += 4 * step) {
      V8<T> xv[4], gv[4], yv[4];
      unsigned mb[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        xv[u] = V8<T>::load(x + (r + u * step) * ldx + rm.cg * 8);
        gv[u] = V8<T>::load(db + (r + u * step) * lddt);
        if (YMASK && MB) mb[u] = mbp[(r + u * step) * ldym];
        else if (YMASK) yv[u] = V8<T>::load(ym + (r + u * step) * ldym + rm.cg * 8);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) body(xv[u], gv[u], (YMASK && !MB) ? yv[u] : none, mb[u]);
    }
    for (; r < r1; r += step)
      body(V8<T>::load(x + r * ldx + rm.cg * 8), V8<T>::load(db + r * lddt),
           (YMASK && !MB) ? V8<T>::load(ym + r * ldym + rm.cg * 8) : none, (YMASK && MB) ? mbp[r * ldym] : 0u);
  }
  const int64_t so = shard_off(blockIdx.x, sstride);
  block_reduce_add(red, rm, C, a, b, dsum + so, dsumx + so);
}

// dx = k*(dy' - dsum/M - xhat*dsumx/M) folded per channel into dx = dy'*q0 + x*q1 + q2 (LDS table,
// with the ReLU test x*q3 + q4 > 0).  YMASK: mask dy by the saved output y and also write the
// masked dy -- the gradient of the residual branch -- to dres (when non-null).
// X3 (T = float, the fp32 step of ops/x3.py): dx is written straight as the bf16 [hi | lo | hi] planes
// of the next convolution's backward (row stride lddx = 3C, plane p at column p * C): the fp32 dx and
// the separate split pass over it (x3.hip split3_kernel) are never made.
template <bool YMASK, class T = uint16_t, bool X3 = false, bool MB = false>
__global__ __launch_bounds__(kThreads) void bn_bwd_apply_kernel(
    const T* __restrict__ x, int64_t ldx, const T* __restrict__ dy, int64_t lddy,
    const T* __restrict__ ym, int64_t ldym, T* __restrict__ dres, int64_t lddr,
    T* __restrict__ dx, int64_t lddx, int64_t M, int C, int64_t rows_per_block,
    const float* __restrict__ mean, const float* __restrict__ invstd, const void* gamma,
    const void* beta, int param_bf16, int relu, const float* __restrict__ dsum,
    const float* __restrict__ dsumx, int64_t sstride, void* dgamma, void* dbeta, int accumulate, Segs segs,
    int64_t pstride = 0) {
  float* tab = bn_dyn;  // [5][C]: bn_lds_table(C, 5) bytes
  const float inv_m = 1.f / static_cast<float>(M);
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const float g = load_param(gamma, c, param_bf16, 1.f), be = load_param(beta, c, param_bf16, 0.f);
    const float ds = shard_sum(dsum, c, sstride), dsx = shard_sum(dsumx, c, sstride);
    const float mu = mean[c], is = invstd[c];
    const float k = g * is, am = ds * inv_m, bm = dsx * inv_m;
    // dx = k*(d - am - (x - mu)*is*bm)
    tab[0 * C + c] = k;
    tab[1 * C + c] = -k * bm * is;
    tab[2 * C + c] = k * (bm * is * mu - am);
    tab[3 * C + c] = k;               // pre-activation = x*k + (be - k*mu)
    tab[4 * C + c] = be - k * mu;
    if (blockIdx.x == 0) {
      store_param(dbeta, c, param_bf16, ds, accumulate);
      store_param(dgamma, c, param_bf16, dsx, accumulate);
    }
  }
  __syncthreads();
  RowMap rm(C);
  if (!rm.active) return;
  float q0[8], q1[8], q2[8], q3[8], q4[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = rm.cg * 8 + j;
    q0[j] = tab[0 * C + c];
    q1[j] = tab[1 * C + c];
    q2[j] = tab[2 * C + c];
    q3[j] = tab[3 * C + c];
    q4[j] = tab[4 * C + c];
  }
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  const int64_t step = rm.RPI;
  const uint8_t* mbp = reinterpret_cast<const uint8_t*>(ym) + rm.cg;
  auto body = [&](const V8<T>& xv, const V8<T>& gv, const V8<T>& yv, int64_t row, unsigned mbits) {
    float xf[8], gf[8], yf[8], o[8];
    xv.to_float(xf);
    gv.to_float(gf);
    if (YMASK && !MB) yv.to_float(yf);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float d = gf[j];
      if (YMASK) {
        if (MB ? !((mbits >> j) & 1u) : yf[j] <= 0.f) d = 0.f;
        gf[j] = d;
      } else if (relu && fmaf(xf[j], q3[j], q4[j]) <= 0.f) {
        d = 0.f;
      }
      o[j] = fmaf(d, q0[j], fmaf(xf[j], q1[j], q2[j]));
    }
    if constexpr (X3) {
      float lo[8];
      const V8<uint16_t> hi = V8<uint16_t>::from_float(o);
      float hf[8];
      hi.to_float(hf);
#pragma unroll
      for (int j = 0; j < 8; ++j) lo[j] = o[j] - hf[j];
      uint16_t* d = reinterpret_cast<uint16_t*>(dx) + row * lddx + rm.cg * 8;
      const int64_t ps = pstride > 0 ? pstride : C;  // a slice of wider planes (ops/fused.py x3 head)
      hi.store(d);
      V8<uint16_t>::from_float(lo).store(d + ps);
      hi.store(d + 2 * ps);
    } else {
      V8<T>::from_float(o).store(dx + row * lddx + rm.cg * 8);
    }
    if (YMASK && dres != nullptr) V8<T>::from_float(gf).store(dres + row * lddr + rm.cg * 8);
  };
  V8<T> none{};
  const T* db = dy + rm.cg * 8;
  int64_t lddt = lddy;
  if (segs.n > 0) {
    T* b;
    segs.resolve(rm.cg * 8, b, lddt);
    db = b;
  }
  int64_t r = r0 + rm.rsub;
  for (; r + 3 * step < r1; r += 4 * step) {
    V8<T> xv[4], gv[4], yv[4];
    unsigned mb[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      xv[u] = V8<T>::load(x + (r + u * step) * ldx + rm.cg * 8);
      gv[u] = V8<T>::load(db + (r + u * step) * lddt);
      if (YMASK && MB) mb[u] = mbp[(r + u * step) * ldym];
      else if (YMASK) yv[u] = V8<T>::load(ym + (r + u * step) * ldym + rm.cg * 8);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) body(xv[u], gv[u], (YMASK && !MB) ? yv[u] : none, r + u * step, mb[u]);
  }
  for (; r < r1; r += step)
    body(V8<T>::load(x + r * ldx + rm.cg * 8), V8<T>::load(db + r * lddt),
         (YMASK && !MB) ? V8<T>::load(ym + r * ldym + rm.cg * 8) : none, r, (YMASK && MB) ? mbp[r * ldym] : 0u);
}

// ---- one-launch BN(+ReLU) backward: reduce -> grid barrier -> apply ------------------------------
// The two-kernel backward (reduce, then apply) reads x and dy twice from HBM and pays two launches
// per layer (x 96 layers per Inception step).  Here a workgroup reduces its rows, all workgroups
// meet at a grid barrier (an atomic arrival counter in the zeroed statistics workspace), and each
// then applies to the SAME rows it just reduced -- the second read mostly hits the L2 / MALL.
// The grid is at most 1 workgroup per CU with <= 40 KB of LDS each, so every workgroup of the
// launch is resident on an otherwise idle GPU (4 fit per CU), also beside two more such launches on
// the branch streams: no workgroup can wait on one that never gets a CU.  Opt-in
// (TONY_BN_ONEPASS=1, TONY_BN_ONEPASS_MAX_MB: the layers it applies to, ops/_lib.py).  Arrival is a release atomic by one lane after __syncthreads; the wait polls
// with an acquire load at agent scope (vector memory, never the scalar cache).
__device__ __forceinline__ void grid_barrier(unsigned* counter) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    while (__hip_atomic_load(counter, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < gridDim.x)
      __builtin_amdgcn_s_sleep(1);
  }
  __syncthreads();
}

__device__ __forceinline__ float shard_sum_acquire(const float* p, int c, int64_t sstride) {
  float s = 0.f;
  const int n = sstride == 0 ? 1 : kStatShards;
  for (int k = 0; k < n; ++k)
    s += __hip_atomic_load(p + k * sstride + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return s;
}

__global__ __launch_bounds__(kThreads) void bn_bwd_onepass_kernel(
    const uint16_t* __restrict__ x, int64_t ldx, const uint16_t* __restrict__ dy, int64_t lddy,
    uint16_t* __restrict__ dx, int64_t lddx, int64_t M, int C, int64_t rows_per_block,
    const float* __restrict__ mean, const float* __restrict__ invstd, const void* gamma, const void* beta,
    int param_bf16, int relu, float* __restrict__ dsum, float* __restrict__ dsumx, int64_t sstride,
    void* dgamma, void* dbeta, int accumulate, unsigned* counter) {
  __shared__ float lds[5 * kMaxC];  // phase 1: coefficient table [4][C] then the block reduction; phase 2: [5][C]
  RowMap rm(C);
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  const int64_t step = rm.RPI;
  // ---- phase 1: dsum[c] = sum dy', dsumx[c] = sum dy' * xhat over this workgroup's rows
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const float mu = mean[c], is = invstd[c];
    const float g = load_param(gamma, c, param_bf16, 1.f), be = load_param(beta, c, param_bf16, 0.f);
    lds[c] = is;
    lds[kMaxC + c] = -mu * is;
    lds[2 * kMaxC + c] = g * is;
    lds[3 * kMaxC + c] = be - g * is * mu;
  }
  __syncthreads();
  float a[8], b[8], p0[8], p1[8], p2[8], p3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = b[j] = 0.f;
    const int c = (rm.active ? rm.cg * 8 : 0) + j;
    p0[j] = lds[c];
    p1[j] = lds[kMaxC + c];
    p2[j] = lds[2 * kMaxC + c];
    p3[j] = lds[3 * kMaxC + c];
  }
  __syncthreads();
  if (rm.active) {
    auto red_body = [&](const bf16x8& xv, const bf16x8& gv) {
      float xf[8], gf[8];
      xv.to_float(xf);
      gv.to_float(gf);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = fmaf(xf[j], p0[j], p1[j]);
        const float d = (relu && fmaf(xf[j], p2[j], p3[j]) <= 0.f) ? 0.f : gf[j];
        a[j] += d;
        b[j] = fmaf(d, xh, b[j]);
      }
    };
    int64_t r = r0 + rm.rsub;
    for (; r + 3 * step < r1; r += 4 * step) {
      bf16x8 xv[4], gv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        xv[u] = load8(x + (r + u * step) * ldx + rm.cg * 8);
        gv[u] = load8(dy + (r + u * step) * lddy + rm.cg * 8);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) red_body(xv[u], gv[u]);
    }
    for (; r < r1; r += step) red_body(load8(x + r * ldx + rm.cg * 8), load8(dy + r * lddy + rm.cg * 8));
  }
  const int64_t so = shard_off(blockIdx.x, sstride);
  block_reduce_add(lds, rm, C, a, b, dsum + so, dsumx + so);
  grid_barrier(counter);
  // ---- phase 2: dx = dy'*q0 + x*q1 + q2 with the completed sums
  const float inv_m = 1.f / static_cast<float>(M);
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const float g = load_param(gamma, c, param_bf16, 1.f), be = load_param(beta, c, param_bf16, 0.f);
    const float ds = shard_sum_acquire(dsum, c, sstride), dsx = shard_sum_acquire(dsumx, c, sstride);
    const float mu = mean[c], is = invstd[c];
    const float k = g * is, am = ds * inv_m, bm = dsx * inv_m;
    lds[c] = k;
    lds[kMaxC + c] = -k * bm * is;
    lds[2 * kMaxC + c] = k * (bm * is * mu - am);
    lds[3 * kMaxC + c] = k;
    lds[4 * kMaxC + c] = be - k * mu;
    if (blockIdx.x == 0) {
      store_param(dbeta, c, param_bf16, ds, accumulate);
      store_param(dgamma, c, param_bf16, dsx, accumulate);
    }
  }
  __syncthreads();
  if (!rm.active) return;
  float q0[8], q1[8], q2[8], q3[8], q4[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = rm.cg * 8 + j;
    q0[j] = lds[c];
    q1[j] = lds[kMaxC + c];
    q2[j] = lds[2 * kMaxC + c];
    q3[j] = lds[3 * kMaxC + c];
    q4[j] = lds[4 * kMaxC + c];
  }
  auto app_body = [&](const bf16x8& xv, const bf16x8& gv, int64_t row) {
    float xf[8], gf[8], o[8];
    xv.to_float(xf);
    gv.to_float(gf);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = (relu && fmaf(xf[j], q3[j], q4[j]) <= 0.f) ? 0.f : gf[j];
      o[j] = fmaf(d, q0[j], fmaf(xf[j], q1[j], q2[j]));
    }
    store8(dx + row * lddx + rm.cg * 8, bf16x8::from_float(o));
  };
  int64_t r = r0 + rm.rsub;
  for (; r + 3 * step < r1; r += 4 * step) {
    bf16x8 xv[4], gv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      xv[u] = load8(x + (r + u * step) * ldx + rm.cg * 8);
      gv[u] = load8(dy + (r + u * step) * lddy + rm.cg * 8);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) app_body(xv[u], gv[u], r + u * step);
  }
  for (; r < r1; r += step) app_body(load8(x + r * ldx + rm.cg * 8), load8(dy + r * lddy + rm.cg * 8), r);
}

// Grid sizing: enough workgroups to cover 256 CUs several times over, but each
// workgroup streams >= `min_iters` row groups so the per-WG LDS epilogue and
// atomics stay amortised.
void plan_rows(int64_t M, int C, int min_iters, int max_blocks, int64_t* rpb, int* grid, bool fill = false) {
  const int RPI = kThreads / (C / 8);
  // fill: small images (Inception's 17x17 / 8x8 layers: M = 37k / 8k rows) would get fewer
  // workgroups than the cap at the default depth; trade per-workgroup iterations for workgroups.
  // Measured (tools/bn_bench.py): pays for the backward reduction (-121 us/step), costs the apply
  // kernels (+180 us/step), so only the reduction asks for it.
  const int64_t want = max_blocks < 1024 ? max_blocks : 1024;
  while (fill && min_iters > 1 &&
         (M + static_cast<int64_t>(RPI) * min_iters - 1) / (static_cast<int64_t>(RPI) * min_iters) < want)
    min_iters >>= 1;
  int64_t g = (M + static_cast<int64_t>(RPI) * min_iters - 1) / (static_cast<int64_t>(RPI) * min_iters);
  if (g > max_blocks) g = max_blocks;
  if (g < 1) g = 1;
  int64_t r = (M + g - 1) / g;
  r = ((r + RPI - 1) / RPI) * RPI;
  *rpb = r;
  *grid = static_cast<int>((M + r - 1) / r);
}

bool bad_c(int C) { return C <= 0 || C % 8 != 0 || C > kMaxC; }

// workgroup cap of the backward reduction (TONY_BN_RED_WGS, default 512 = 2 per CU)
int red_wgs() {
  static const int v = [] {
    const char* e = getenv("TONY_BN_RED_WGS");
    const int n = e != nullptr ? atoi(e) : 0;
    return n > 0 ? n : 512;
  }();
  return v;
}

// Training BN + ReLU fused with the KxK / stride-S max pool that follows it (Inception's stem:
// conv -> BN -> ReLU -> maxpool 3x3/2 at 147x147 and 71x71).  The full-resolution activation is
// never written: each lane normalises the 9 window inputs of its 8 channels on the fly (scale /
// shift rebuilt per workgroup from the conv epilogue's statistics, as in bn_fwd_apply_kernel),
// rounds them to bf16 (so max and argmax match the unfused pair exactly) and writes the pooled
// value and the window argmax byte.  The backward needs only Z (the BN backward recomputes the ReLU
// mask from it) and the argmax.
// KT: the pool window when known at compile time (3: Inception's stem pools) -- the window's 9 loads
// are then all issued before the first is used (the runtime-K loop waited on each load in turn:
// latency-bound at ~2.4 TB/s, 190 / 130 us per step at the two stem pools) and their addresses are
// row / column offsets of one base pointer; 0: any K.
template <int KT>
__global__ __launch_bounds__(kThreads) void bn_relu_maxpool_kernel(
    const uint16_t* __restrict__ z, int64_t ldz, const float* __restrict__ sum, const float* __restrict__ sumsq,
    int64_t sstride, const void* gamma, const void* beta, int param_bf16, float eps,
    float* __restrict__ save_mean, float* __restrict__ save_invstd, float* __restrict__ running_mean,
    float* __restrict__ running_var, float momentum, uint16_t* __restrict__ y, int64_t ldy,
    uint8_t* __restrict__ arg, int N, int H, int W, int C, int OH, int OW, int K, int S, int P) {
  float* scale = bn_dyn;  // [C] then shift [C]: bn_lds_table(C, 2) bytes
  float* shift = bn_dyn + C;
  const int64_t M = static_cast<int64_t>(N) * H * W;
  const float inv_m = 1.f / static_cast<float>(M);
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const float mean = shard_sum(sum, c, sstride) * inv_m;
    const float var = fmaxf(shard_sum(sumsq, c, sstride) * inv_m - mean * mean, 0.f);
    const float invstd = rsqrtf(var + eps);
    if (blockIdx.x == 0) {
      save_mean[c] = mean;
      save_invstd[c] = invstd;
      if (running_mean != nullptr) {
        const float unbiased = M > 1 ? var * (static_cast<float>(M) / static_cast<float>(M - 1)) : var;
        running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
      }
    }
    const float g = load_param(gamma, c, param_bf16, 1.f);
    const float b = load_param(beta, c, param_bf16, 0.f);
    scale[c] = g * invstd;
    shift[c] = b - mean * g * invstd;
  }
  __syncthreads();
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
    float sc[8], sh[8], best[8];
    uint8_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = scale[cg * 8 + j];
      sh[j] = shift[cg * 8 + j];
      best[j] = -__builtin_huge_valf();
      bi[j] = 0;
    }
    auto take = [&](const bf16x8& raw, uint8_t idx) {
      float f[8];
      raw.to_float(f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = bf2f(f2bf(relu_f(fmaf(f[j], sc[j], sh[j]))));  // the bf16 activation
        if (v > best[j] || (v != v)) {
          best[j] = v;
          bi[j] = idx;
        }
      }
    };
    // P > 0 (ResNet's 3x3/2 p1 stem pool): out-of-image taps are skipped -- every window holds an
    // in-image tap (P < K) and the ReLU outputs are >= 0, so a padded tap could never win anyway
    const int h0 = oh * S - P, w0 = ow * S - P;
    if constexpr (KT > 0) {
      if (P == 0) {
        const uint16_t* base = z + ((n * H + h0) * W + w0) * ldz + cg * 8;
        const int64_t row = static_cast<int64_t>(W) * ldz;
        bf16x8 raw[KT * KT];
#pragma unroll
        for (int kh = 0; kh < KT; ++kh)
#pragma unroll
          for (int kw = 0; kw < KT; ++kw) raw[kh * KT + kw] = load8(base + kh * row + kw * ldz);
#pragma unroll
        for (int k = 0; k < KT * KT; ++k) take(raw[k], static_cast<uint8_t>(k));
      } else {
        bf16x8 raw[KT * KT];
        bool ok[KT * KT];
#pragma unroll
        for (int kh = 0; kh < KT; ++kh)
#pragma unroll
          for (int kw = 0; kw < KT; ++kw) {
            const int hh = h0 + kh, ww = w0 + kw;
            ok[kh * KT + kw] = static_cast<unsigned>(hh) < static_cast<unsigned>(H) &&
                               static_cast<unsigned>(ww) < static_cast<unsigned>(W);
            if (ok[kh * KT + kw]) raw[kh * KT + kw] = load8(z + ((n * H + hh) * W + ww) * ldz + cg * 8);
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
          take(load8(z + ((n * H + hh) * W + ww) * ldz + cg * 8), static_cast<uint8_t>(kh * K + kw));
        }
      }
    }
    store8(y + static_cast<int64_t>(site) * ldy + cg * 8, bf16x8::from_float(best));
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (static_cast<uint32_t>(bi[3]) << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (static_cast<uint32_t>(bi[7]) << 24);
    *reinterpret_cast<uint2*>(arg + static_cast<int64_t>(site) * C + cg * 8) = packed;
  }
}

// BN(+ReLU) backward apply of the layer a KxK / stride-S max pool (padding P) read, with the pool's
// backward gathered in: each lane's dY[site, 8 channels] is summed from the <= ceil(K/S)^2 windows
// that cover the site and chose it (argmax byte == the site's window position), exactly as
// csrc/pool.hip maxpool_bwd_kernel writes it, and goes straight into dZ = dY'*q0 + Z*q1 + q2 -- the
// full-resolution dY (354 / 248 MB at Inception's two stem pools, 205 MB at ResNet's) is never
// stored nor read back.  The sums come from the pool backward's fused reduction (pool.hip
// maxpool_bwd_bnred_kernel with no dX store).  Rows per workgroup, thread map and the per-channel
// coefficient table in LDS as in bn_bwd_apply_kernel.
__global__ __launch_bounds__(kThreads) void bn_bwd_pool_apply_kernel(
    const uint16_t* __restrict__ dyp, int64_t lddy, const uint8_t* __restrict__ arg, int N, int H, int W, int C,
    int OH, int OW, int K, int S, int P, const uint16_t* __restrict__ z, int64_t ldz, uint16_t* __restrict__ dz,
    int64_t lddz, int64_t rows_per_block, const float* __restrict__ mean, const float* __restrict__ invstd,
    const void* gamma, const void* beta, int param_bf16, int relu, const float* __restrict__ dsum, int64_t sstride,
    void* dgamma, void* dbeta, int accumulate) {
  const int64_t M = static_cast<int64_t>(N) * H * W;
  const float inv_m = 1.f / static_cast<float>(M);
  float* tab = bn_dyn;  // [5][C] per workgroup (bn_bwd_apply_kernel's table): the sharded sums are read
                        // C times per workgroup, not 8 x 2 x kStatShards times per lane
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const float g = load_param(gamma, c, param_bf16, 1.f), be = load_param(beta, c, param_bf16, 0.f);
    const float ds = shard_sum(dsum, c, sstride), dsx = shard_sum(dsum + C, c, sstride);
    const float mu = mean[c], is = invstd[c];
    const float k = g * is, am = ds * inv_m, bm = dsx * inv_m;
    tab[0 * C + c] = k;
    tab[1 * C + c] = -k * bm * is;
    tab[2 * C + c] = k * (bm * is * mu - am);
    tab[3 * C + c] = k;
    tab[4 * C + c] = be - k * mu;
    if (blockIdx.x == 0) {
      store_param(dbeta, c, param_bf16, ds, accumulate);
      store_param(dgamma, c, param_bf16, dsx, accumulate);
    }
  }
  __syncthreads();
  RowMap rm(C);
  if (!rm.active) return;
  float q0[8], q1[8], q2[8], q3[8], q4[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = rm.cg * 8 + j;
    q0[j] = tab[0 * C + c];
    q1[j] = tab[1 * C + c];
    q2[j] = tab[2 * C + c];
    q3[j] = tab[3 * C + c];
    q4[j] = tab[4 * C + c];
  }
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  // (n, h, w) of the site walked incrementally: one 32-bit decomposition per lane, not four 64-bit
  // divisions per row (emulated: they made this kernel ALU-bound at 1.9 TB/s)
  const uint32_t first = static_cast<uint32_t>(r0 + rm.rsub);
  int w = static_cast<int>(first % static_cast<uint32_t>(W));
  const uint32_t nh0 = first / static_cast<uint32_t>(W);
  int h = static_cast<int>(nh0 % static_cast<uint32_t>(H));
  int64_t n = nh0 / static_cast<uint32_t>(H);
  for (int64_t site = r0 + rm.rsub; site < r1; site += rm.RPI) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int hp = h + P, wp = w + P;  // windows oh with oh*S <= hp <= oh*S + K - 1
    const int oh_lo = hp >= K ? (hp - K + S) / S : 0, oh_hi = min(OH - 1, hp / S);
    const int ow_lo = wp >= K ? (wp - K + S) / S : 0, ow_hi = min(OW - 1, wp / S);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const uint32_t local = static_cast<uint32_t>((hp - oh * S) * K + (wp - ow * S));
        const int64_t osite = (n * OH + oh) * OW + ow;
        const uint2 packed = *reinterpret_cast<const uint2*>(arg + osite * C + rm.cg * 8);
        float g[8];
        V8<uint16_t>::load(dyp + osite * lddy + rm.cg * 8).to_float(g);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t word = j < 4 ? packed.x : packed.y;
          if (((word >> (8 * (j & 3))) & 0xffu) == local) acc[j] += g[j];
        }
      }
    }
    float d[8], xf[8], o[8];
    V8<uint16_t>::from_float(acc).to_float(d);  // the bf16 dY the unfused pool backward would store
    V8<uint16_t>::load(z + site * ldz + rm.cg * 8).to_float(xf);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float dd = (relu && fmaf(xf[j], q3[j], q4[j]) <= 0.f) ? 0.f : d[j];
      o[j] = fmaf(dd, q0[j], fmaf(xf[j], q1[j], q2[j]));
    }
    V8<uint16_t>::from_float(o).store(dz + site * lddz + rm.cg * 8);
    for (w += rm.RPI; w >= W;) {
      w -= W;
      if (++h == H) {
        h = 0;
        ++n;
      }
    }
  }
}

}  // namespace

// ---- composable entry points (the fused conv heads call these on channel sub-ranges) ----
//
// Statistics buffers: sum/sumsq (and dsum/dsumx) point into shard 0 of a buffer holding
// kStatShards copies `sstride` floats apart (sstride = 0: one copy).  Producers add into the
// copy of their block index; consumers sum all copies (common.h).

TONY_API int tony_stat_shards() { return kStatShards; }

// sum/sumsq[C] (zero on entry: the caller zeroes them, ops/arena.py) accumulate over the M rows of x.
TONY_API int tony_bn_stats(const void* x, int64_t M, int C, int64_t ldx, float* sum, float* sumsq, int64_t sstride,
                           hipStream_t stream) {
  if (bad_c(C) || (ldx % 8) || sstride < 0) return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 8, 512, &rpb, &grid);  // few WGs: C atomics per WG contend per channel
  bn_fwd_stats_kernel<uint16_t><<<grid, kThreads, bn_lds_reduce(C), stream>>>(static_cast<const uint16_t*>(x), M, C, ldx, rpb, sum, sumsq,
                                                      sstride);
  TONY_LAUNCH_CHECK();
  return 0;
}

// mode 0 (train): normalise with the batch stats in sum/sumsq, save mean/invstd,
// update running stats; mode 1 (eval): use running_mean/var.
TONY_API int tony_bn_apply(const void* x, int64_t M, int C, int64_t ldx, void* y, int64_t ldy, const float* sum,
                           const float* sumsq, int64_t sstride, const void* gamma, const void* beta, int param_bf16,
                           float eps, int relu, int mode, float* save_mean, float* save_invstd, float* running_mean,
                           float* running_var, float momentum, hipStream_t stream) {
  if (bad_c(C) || (ldx % 8) || (ldy % 8) || sstride < 0) return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 4, 8192, &rpb, &grid);
  bn_fwd_apply_kernel<false, uint16_t><<<grid, kThreads, bn_lds_table(C, 2), stream>>>(
      static_cast<const uint16_t*>(x), M, C, ldx, rpb, nullptr, 0, static_cast<uint16_t*>(y), ldy, sum, sumsq,
      sstride, gamma, beta, param_bf16, eps, relu, mode, save_mean, save_invstd, running_mean, running_var, momentum, Segs{});
  TONY_LAUNCH_CHECK();
  return 0;
}

// y = act(bn(x) + res): the bottleneck tail (conv3 -> BN -> + identity -> ReLU) in one pass.
TONY_API int tony_bn_apply_res(const void* x, int64_t M, int C, int64_t ldx, const void* res, int64_t ldr, void* y,
                               int64_t ldy, const float* sum, const float* sumsq, int64_t sstride, const void* gamma,
                               const void* beta, int param_bf16, float eps, int relu, int mode, float* save_mean,
                               float* save_invstd, float* running_mean, float* running_var, float momentum,
                               hipStream_t stream) {
  if (bad_c(C) || (ldx % 8) || (ldy % 8) || (ldr % 8) || res == nullptr || sstride < 0) return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 4, 8192, &rpb, &grid);
  bn_fwd_apply_kernel<true, uint16_t><<<grid, kThreads, bn_lds_table(C, 2), stream>>>(
      static_cast<const uint16_t*>(x), M, C, ldx, rpb, static_cast<const uint16_t*>(res), ldr,
      static_cast<uint16_t*>(y), ldy, sum, sumsq, sstride, gamma, beta, param_bf16, eps, relu, mode, save_mean,
      save_invstd, running_mean, running_var, momentum, Segs{});
  TONY_LAUNCH_CHECK();
  return 0;
}

// tony_bn_apply_res that also writes the forward's ReLU byte mask (M x C/8 bytes, row stride ldm)
TONY_API int tony_bn_apply_res_m(const void* x, int64_t M, int C, int64_t ldx, const void* res, int64_t ldr, void* y,
                                 int64_t ldy, const float* sum, const float* sumsq, int64_t sstride, const void* gamma,
                                 const void* beta, int param_bf16, float eps, int relu, int mode, float* save_mean,
                                 float* save_invstd, float* running_mean, float* running_var, float momentum,
                                 void* mask, int64_t ldm, hipStream_t stream) {
  if (bad_c(C) || (ldx % 8) || (ldy % 8) || (ldr % 8) || res == nullptr || sstride < 0 || mask == nullptr ||
      ldm < C / 8)
    return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 4, 8192, &rpb, &grid);
  bn_fwd_apply_kernel<true, uint16_t><<<grid, kThreads, bn_lds_table(C, 2), stream>>>(
      static_cast<const uint16_t*>(x), M, C, ldx, rpb, static_cast<const uint16_t*>(res), ldr,
      static_cast<uint16_t*>(y), ldy, sum, sumsq, sstride, gamma, beta, param_bf16, eps, relu, mode, save_mean,
      save_invstd, running_mean, running_var, momentum, Segs{}, static_cast<uint8_t*>(mask), ldm);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_bn_bwd_reduce(const void* x, int64_t ldx, const void* dy, int64_t lddy, int64_t M, int C,
                                const float* mean, const float* invstd, const void* gamma, const void* beta,
                                int param_bf16, int relu, float* dsum, float* dsumx, int64_t sstride,
                                hipStream_t stream) {
  if (bad_c(C) || (ldx % 8) || (lddy % 8) || sstride < 0) return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 8, red_wgs(), &rpb, &grid, true);  // few WGs: C atomics per WG contend per channel
  bn_bwd_reduce_kernel<false, uint16_t><<<grid, kThreads, bn_lds_bred(C), stream>>>(
      static_cast<const uint16_t*>(x), ldx, static_cast<const uint16_t*>(dy), lddy, nullptr, 0, M, C, rpb, mean,
      invstd, gamma, beta, param_bf16, relu, dsum, dsumx, sstride, Segs{});
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_bn_bwd_apply(const void* x, int64_t ldx, const void* dy, int64_t lddy, void* dx, int64_t lddx,
                               int64_t M, int C, const float* mean, const float* invstd, const void* gamma,
                               const void* beta, int param_bf16, int relu, const float* dsum, const float* dsumx,
                               int64_t sstride, void* dgamma, void* dbeta, int accumulate, hipStream_t stream) {
  if (bad_c(C) || (ldx % 8) || (lddy % 8) || (lddx % 8) || sstride < 0) return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 4, 8192, &rpb, &grid);
  bn_bwd_apply_kernel<false, uint16_t><<<grid, kThreads, bn_lds_table(C, 5), stream>>>(
      static_cast<const uint16_t*>(x), ldx, static_cast<const uint16_t*>(dy), lddy, nullptr, 0, nullptr, 0,
      static_cast<uint16_t*>(dx), lddx, M, C, rpb, mean, invstd, gamma, beta, param_bf16, relu, dsum, dsumx, sstride,
      dgamma, dbeta, accumulate, Segs{});
  TONY_LAUNCH_CHECK();
  return 0;
}

// ---- multi-output forms: the splits of a fused Inception head (ops/fused.py) in ONE launch ------
// Segment s covers columns [e[s-1], e[s]) of the [M, C] BN tensor x (C = e[n-1]); its output (apply)
// / input gradient (backward) lives at p[s] with row stride l[s].  n = 1..4, every e[s] % 8 == 0,
// every p[s] 16-byte aligned and every l[s] % 8 == 0.
namespace {
bool make_segs(Segs& sg, int C, int n, int e0, int e1, int e2, int e3, void* p0, void* p1, void* p2, void* p3,
               int64_t l0, int64_t l1, int64_t l2, int64_t l3) {
  if (n < 1 || n > 4) return false;
  const int e[4] = {e0, e1, e2, e3};
  void* p[4] = {p0, p1, p2, p3};
  const int64_t l[4] = {l0, l1, l2, l3};
  int prev = 0;
  sg.n = n;
  for (int s = 0; s < n; ++s) {
    if (e[s] <= prev || (e[s] % 8) || p[s] == nullptr || (reinterpret_cast<uintptr_t>(p[s]) & 15) || (l[s] % 8) ||
        l[s] < e[s] - prev)
      return false;
    sg.end[s] = e[s];
    sg.p[s] = p[s];
    sg.ld[s] = l[s];
    prev = e[s];
  }
  return prev == C;
}
}  // namespace

TONY_API int tony_bn_apply_segs(const void* x, int64_t M, int C, int64_t ldx, int n, int e0, int e1, int e2, int e3,
                                void* p0, void* p1, void* p2, void* p3, int64_t l0, int64_t l1, int64_t l2, int64_t l3,
                                const float* sum, const float* sumsq, int64_t sstride, const void* gamma,
                                const void* beta, int param_bf16, float eps, int relu, int mode, float* save_mean,
                                float* save_invstd, float* running_mean, float* running_var, float momentum,
                                hipStream_t stream) {
  Segs sg;
  if (bad_c(C) || (ldx % 8) || sstride < 0 || !make_segs(sg, C, n, e0, e1, e2, e3, p0, p1, p2, p3, l0, l1, l2, l3))
    return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 4, 8192, &rpb, &grid);
  bn_fwd_apply_kernel<false, uint16_t><<<grid, kThreads, bn_lds_table(C, 2), stream>>>(
      static_cast<const uint16_t*>(x), M, C, ldx, rpb, nullptr, 0, static_cast<uint16_t*>(sg.p[0]), sg.ld[0], sum, sumsq, sstride, gamma, beta,
      param_bf16, eps, relu, mode, save_mean, save_invstd, running_mean, running_var, momentum, sg);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_bn_bwd_reduce_segs(const void* x, int64_t ldx, int n, int e0, int e1, int e2, int e3, void* p0,
                                     void* p1, void* p2, void* p3, int64_t l0, int64_t l1, int64_t l2, int64_t l3,
                                     int64_t M, int C, const float* mean, const float* invstd, const void* gamma,
                                     const void* beta, int param_bf16, int relu, float* dsum, float* dsumx,
                                     int64_t sstride, hipStream_t stream) {
  Segs sg;
  if (bad_c(C) || (ldx % 8) || sstride < 0 || !make_segs(sg, C, n, e0, e1, e2, e3, p0, p1, p2, p3, l0, l1, l2, l3))
    return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 8, red_wgs(), &rpb, &grid, true);
  bn_bwd_reduce_kernel<false, uint16_t><<<grid, kThreads, bn_lds_bred(C), stream>>>(
      static_cast<const uint16_t*>(x), ldx, static_cast<const uint16_t*>(sg.p[0]), sg.ld[0], nullptr, 0, M, C, rpb, mean, invstd, gamma, beta,
      param_bf16, relu, dsum, dsumx, sstride, sg);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_bn_bwd_apply_segs(const void* x, int64_t ldx, int n, int e0, int e1, int e2, int e3, void* p0,
                                    void* p1, void* p2, void* p3, int64_t l0, int64_t l1, int64_t l2, int64_t l3,
                                    void* dx, int64_t lddx, int64_t M, int C, const float* mean, const float* invstd,
                                    const void* gamma, const void* beta, int param_bf16, int relu, const float* dsum,
                                    const float* dsumx, int64_t sstride, void* dgamma, void* dbeta, int accumulate,
                                    hipStream_t stream) {
  Segs sg;
  if (bad_c(C) || (ldx % 8) || (lddx % 8) || sstride < 0 ||
      !make_segs(sg, C, n, e0, e1, e2, e3, p0, p1, p2, p3, l0, l1, l2, l3))
    return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 4, 8192, &rpb, &grid);
  bn_bwd_apply_kernel<false, uint16_t><<<grid, kThreads, bn_lds_table(C, 5), stream>>>(
      static_cast<const uint16_t*>(x), ldx, static_cast<const uint16_t*>(sg.p[0]), sg.ld[0], nullptr, 0, nullptr, 0, static_cast<uint16_t*>(dx),
      lddx, M, C, rpb, mean, invstd, gamma, beta, param_bf16, relu, dsum, dsumx, sstride, dgamma, dbeta, accumulate,
      sg);
  TONY_LAUNCH_CHECK();
  return 0;
}

// ---- fp32 forms (the x3 fp32 step, ops/x3.py): same kernels on float rows, same arguments -------
TONY_API int tony_bn_stats_f32(const void* x, int64_t M, int C, int64_t ldx, float* sum, float* sumsq,
                               int64_t sstride, hipStream_t stream) {
  if (bad_c(C) || (ldx % 4) || sstride < 0) return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 8, 512, &rpb, &grid);
  bn_fwd_stats_kernel<float><<<grid, kThreads, bn_lds_reduce(C), stream>>>(static_cast<const float*>(x), M, C, ldx,
                                                                           rpb, sum, sumsq, sstride);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_bn_apply_f32(const void* x, int64_t M, int C, int64_t ldx, void* y, int64_t ldy, const float* sum,
                               const float* sumsq, int64_t sstride, const void* gamma, const void* beta, int param_bf16,
                               float eps, int relu, int mode, float* save_mean, float* save_invstd,
                               float* running_mean, float* running_var, float momentum, hipStream_t stream) {
  if (bad_c(C) || (ldx % 4) || (ldy % 4) || sstride < 0) return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 4, 8192, &rpb, &grid);
  bn_fwd_apply_kernel<false, float><<<grid, kThreads, bn_lds_table(C, 2), stream>>>(
      static_cast<const float*>(x), M, C, ldx, rpb, nullptr, 0, static_cast<float*>(y), ldy, sum, sumsq, sstride,
      gamma, beta, param_bf16, eps, relu, mode, save_mean, save_invstd, running_mean, running_var, momentum, Segs{});
  TONY_LAUNCH_CHECK();
  return 0;
}

// tony_bn_apply_f32 that ALSO writes y's x3 planes: p3 = the channel-c0 column of a [M][3 * pst] bf16 planes
// buffer (row stride ldp, plane p at column p * pst) -- a concat slot producer filling its slice of the
// block output's planes, so the next block's x3 convs need no split pass over the fp32 concat
TONY_API int tony_bn_apply_f32_p3(const void* x, int64_t M, int C, int64_t ldx, void* y, int64_t ldy, void* p3,
                                  int64_t ldp, int64_t pst, const float* sum, const float* sumsq, int64_t sstride,
                                  const void* gamma, const void* beta, int param_bf16, float eps, int relu, int mode,
                                  float* save_mean, float* save_invstd, float* running_mean, float* running_var,
                                  float momentum, hipStream_t stream) {
  if (bad_c(C) || (ldx % 4) || (ldy % 4) || sstride < 0 || p3 == nullptr || pst < C || ldp < 3 * pst || (ldp % 8) ||
      (pst % 8) || (reinterpret_cast<uintptr_t>(p3) & 15))
    return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 4, 8192, &rpb, &grid);
  bn_fwd_apply_kernel<false, float><<<grid, kThreads, bn_lds_table(C, 2), stream>>>(
      static_cast<const float*>(x), M, C, ldx, rpb, nullptr, 0, static_cast<float*>(y), ldy, sum, sumsq, sstride,
      gamma, beta, param_bf16, eps, relu, mode, save_mean, save_invstd, running_mean, running_var, momentum, Segs{},
      nullptr, 0, static_cast<uint16_t*>(p3), ldp, pst);
  TONY_LAUNCH_CHECK();
  return 0;
}

// tony_bn_apply_f32 writing y as its x3 planes (bf16 [M][3C], row stride ldy3 >= 3C): bn_fwd_apply_kernel X3
TONY_API int tony_bn_apply_f32_x3(const void* x, int64_t M, int C, int64_t ldx, void* y3, int64_t ldy3,
                                  const float* sum, const float* sumsq, int64_t sstride, const void* gamma,
                                  const void* beta, int param_bf16, float eps, int relu, int mode, float* save_mean,
                                  float* save_invstd, float* running_mean, float* running_var, float momentum,
                                  hipStream_t stream) {
  if (bad_c(C) || (ldx % 4) || ldy3 < 3 * C || (ldy3 % 8) || sstride < 0 || (reinterpret_cast<uintptr_t>(y3) & 15))
    return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 4, 8192, &rpb, &grid);
  bn_fwd_apply_kernel<false, float, true><<<grid, kThreads, bn_lds_table(C, 2), stream>>>(
      static_cast<const float*>(x), M, C, ldx, rpb, nullptr, 0, static_cast<float*>(y3), ldy3, sum, sumsq, sstride,
      gamma, beta, param_bf16, eps, relu, mode, save_mean, save_invstd, running_mean, running_var, momentum, Segs{});
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_bn_bwd_reduce_f32(const void* x, int64_t ldx, const void* dy, int64_t lddy, int64_t M, int C,
                                    const float* mean, const float* invstd, const void* gamma, const void* beta,
                                    int param_bf16, int relu, float* dsum, float* dsumx, int64_t sstride,
                                    hipStream_t stream) {
  if (bad_c(C) || (ldx % 4) || (lddy % 4) || sstride < 0) return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 8, red_wgs(), &rpb, &grid, true);
  bn_bwd_reduce_kernel<false, float><<<grid, kThreads, bn_lds_bred(C), stream>>>(
      static_cast<const float*>(x), ldx, static_cast<const float*>(dy), lddy, nullptr, 0, M, C, rpb, mean, invstd,
      gamma, beta, param_bf16, relu, dsum, dsumx, sstride, Segs{});
  TONY_LAUNCH_CHECK();
  return 0;
}

// tony_bn_bwd_apply_f32 writing dx as the x3 planes (bf16 [M][3C], row stride lddx >= 3C): X3 above
TONY_API int tony_bn_bwd_apply_f32_x3(const void* x, int64_t ldx, const void* dy, int64_t lddy, void* dx3,
                                      int64_t lddx, int64_t M, int C, const float* mean, const float* invstd,
                                      const void* gamma, const void* beta, int param_bf16, int relu, const float* dsum,
                                      const float* dsumx, int64_t sstride, void* dgamma, void* dbeta, int accumulate,
                                      hipStream_t stream) {
  if (bad_c(C) || (ldx % 4) || (lddy % 4) || (lddx % 8) || lddx < 3 * static_cast<int64_t>(C) || sstride < 0 ||
      (reinterpret_cast<uintptr_t>(dx3) & 15))
    return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 4, 8192, &rpb, &grid);
  bn_bwd_apply_kernel<false, float, true><<<grid, kThreads, bn_lds_table(C, 5), stream>>>(
      static_cast<const float*>(x), ldx, static_cast<const float*>(dy), lddy, nullptr, 0, nullptr, 0,
      static_cast<float*>(dx3), lddx, M, C, rpb, mean, invstd, gamma, beta, param_bf16, relu, dsum, dsumx, sstride,
      dgamma, dbeta, accumulate, Segs{});
  TONY_LAUNCH_CHECK();
  return 0;
}

// the x3 planes of dx as channels [0, C) of wider planes: plane p at column p * pstride (pstride >= C), so
// the BN backward of one split of a fused x3 head writes its slice of the head's dZ planes
TONY_API int tony_bn_bwd_apply_f32_x3p(const void* x, int64_t ldx, const void* dy, int64_t lddy, void* dx3,
                                       int64_t lddx, int64_t pstride, int64_t M, int C, const float* mean,
                                       const float* invstd, const void* gamma, const void* beta, int param_bf16,
                                       int relu, const float* dsum, const float* dsumx, int64_t sstride, void* dgamma,
                                       void* dbeta, int accumulate, hipStream_t stream) {
  if (bad_c(C) || (ldx % 4) || (lddy % 4) || (lddx % 8) || (pstride % 8) || pstride < C ||
      lddx < 2 * pstride + C || sstride < 0 || (reinterpret_cast<uintptr_t>(dx3) & 15))
    return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 4, 8192, &rpb, &grid);
  bn_bwd_apply_kernel<false, float, true><<<grid, kThreads, bn_lds_table(C, 5), stream>>>(
      static_cast<const float*>(x), ldx, static_cast<const float*>(dy), lddy, nullptr, 0, nullptr, 0,
      static_cast<float*>(dx3), lddx, M, C, rpb, mean, invstd, gamma, beta, param_bf16, relu, dsum, dsumx, sstride,
      dgamma, dbeta, accumulate, Segs{}, pstride);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_bn_bwd_apply_f32(const void* x, int64_t ldx, const void* dy, int64_t lddy, void* dx, int64_t lddx,
                                   int64_t M, int C, const float* mean, const float* invstd, const void* gamma,
                                   const void* beta, int param_bf16, int relu, const float* dsum, const float* dsumx,
                                   int64_t sstride, void* dgamma, void* dbeta, int accumulate, hipStream_t stream) {
  if (bad_c(C) || (ldx % 4) || (lddy % 4) || (lddx % 4) || sstride < 0) return -1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 4, 8192, &rpb, &grid);
  bn_bwd_apply_kernel<false, float><<<grid, kThreads, bn_lds_table(C, 5), stream>>>(
      static_cast<const float*>(x), ldx, static_cast<const float*>(dy), lddy, nullptr, 0, nullptr, 0,
      static_cast<float*>(dx), lddx, M, C, rpb, mean, invstd, gamma, beta, param_bf16, relu, dsum, dsumx, sstride,
      dgamma, dbeta, accumulate, Segs{});
  TONY_LAUNCH_CHECK();
  return 0;
}

// ---- one-call forms used by BatchNormAct2d: the workspace holds kStatShards x 2C floats, zeroed ----

TONY_API int tony_bn_fwd_train(const void* x, int64_t M, int C, int64_t ldx, void* y, int64_t ldy,
                               const void* gamma, const void* beta, int param_bf16, float eps,
                               int relu, float* sums_ws, float* save_mean, float* save_invstd,
                               float* running_mean, float* running_var, float momentum,
                               hipStream_t stream) {
  const int64_t ss = 2 * static_cast<int64_t>(C);
  int rc = tony_bn_stats(x, M, C, ldx, sums_ws, sums_ws + C, ss, stream);
  if (rc) return rc;
  return tony_bn_apply(x, M, C, ldx, y, ldy, sums_ws, sums_ws + C, ss, gamma, beta, param_bf16, eps, relu, 0,
                       save_mean, save_invstd, running_mean, running_var, momentum, stream);
}

TONY_API int tony_bn_fwd_infer(const void* x, int64_t M, int C, int64_t ldx, void* y, int64_t ldy,
                               const void* gamma, const void* beta, int param_bf16, float eps,
                               int relu, const float* running_mean, const float* running_var,
                               hipStream_t stream) {
  return tony_bn_apply(x, M, C, ldx, y, ldy, nullptr, nullptr, 0, gamma, beta, param_bf16, eps, relu, 1, nullptr,
                       nullptr, const_cast<float*>(running_mean), const_cast<float*>(running_var), 0.f, stream);
}

// One-launch backward (bn_bwd_onepass_kernel) when ``counter`` (a zeroed uint32, e.g. the word after
// the statistics workspace) is given and ``num_cus`` > 0; the reduce + apply pair otherwise.
TONY_API int tony_bn_bwd_onepass(const void* x, int64_t ldx, const void* dy, int64_t lddy, void* dx, int64_t lddx,
                                 int64_t M, int C, const float* mean, const float* invstd, const void* gamma,
                                 const void* beta, int param_bf16, int relu, float* dsums_ws, void* dgamma,
                                 void* dbeta, int accumulate, unsigned* counter, int num_cus, hipStream_t stream) {
  if (bad_c(C) || (ldx % 8) || (lddy % 8) || (lddx % 8) || counter == nullptr || num_cus <= 0 || M <= 0) return -1;
  const int64_t ss = 2 * static_cast<int64_t>(C);
  int64_t rpb;
  int grid;
  // <= 1 workgroup per CU (40 KB of LDS, 4 waves): all co-resident even with two more of these kernels
  // spinning at their barriers on the branch streams (4 fit per CU by LDS), so no cycle of waiting grids
  plan_rows(M, C, 4, num_cus, &rpb, &grid);
  bn_bwd_onepass_kernel<<<grid, kThreads, 0, stream>>>(
      static_cast<const uint16_t*>(x), ldx, static_cast<const uint16_t*>(dy), lddy, static_cast<uint16_t*>(dx), lddx,
      M, C, rpb, mean, invstd, gamma, beta, param_bf16, relu, dsums_ws, dsums_ws + C, ss, dgamma, dbeta, accumulate,
      counter);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_bn_bwd(const void* x, int64_t ldx, const void* dy, int64_t lddy, void* dx,
                         int64_t lddx, int64_t M, int C, const float* mean, const float* invstd,
                         const void* gamma, const void* beta, int param_bf16, int relu,
                         float* dsums_ws, void* dgamma, void* dbeta, int accumulate, hipStream_t stream) {
  const int64_t ss = 2 * static_cast<int64_t>(C);
  int rc = tony_bn_bwd_reduce(x, ldx, dy, lddy, M, C, mean, invstd, gamma, beta, param_bf16, relu, dsums_ws,
                              dsums_ws + C, ss, stream);
  if (rc) return rc;
  return tony_bn_bwd_apply(x, ldx, dy, lddy, dx, lddx, M, C, mean, invstd, gamma, beta, param_bf16, relu, dsums_ws,
                           dsums_ws + C, ss, dgamma, dbeta, accumulate, stream);
}

// Backward of y = relu(bn(x) + res): dy' = dy * (y > 0); dres = dy' (if dres != null); dx = bn_bwd(dy').
TONY_API int tony_bn_bwd_res(const void* x, int64_t ldx, const void* dy, int64_t lddy, const void* y, int64_t ldy,
                             void* dx, int64_t lddx, void* dres, int64_t lddr, int64_t M, int C, const float* mean,
                             const float* invstd, const void* gamma, const void* beta, int param_bf16,
                             float* dsums_ws, void* dgamma, void* dbeta, int accumulate, hipStream_t stream) {
  if (bad_c(C) || (ldx % 8) || (lddy % 8) || (ldy % 8) || (lddx % 8) || (lddr % 8) || y == nullptr) return -1;
  const int64_t ss = 2 * static_cast<int64_t>(C);
  int64_t rpb;
  int grid;
  plan_rows(M, C, 8, 512, &rpb, &grid);
  bn_bwd_reduce_kernel<true, uint16_t><<<grid, kThreads, bn_lds_bred(C), stream>>>(
      static_cast<const uint16_t*>(x), ldx, static_cast<const uint16_t*>(dy), lddy, static_cast<const uint16_t*>(y),
      ldy, M, C, rpb, mean, invstd, gamma, beta, param_bf16, 1, dsums_ws, dsums_ws + C, ss, Segs{});
  TONY_LAUNCH_CHECK();
  plan_rows(M, C, 4, 8192, &rpb, &grid);
  bn_bwd_apply_kernel<true, uint16_t><<<grid, kThreads, bn_lds_table(C, 5), stream>>>(
      static_cast<const uint16_t*>(x), ldx, static_cast<const uint16_t*>(dy), lddy, static_cast<const uint16_t*>(y),
      ldy, static_cast<uint16_t*>(dres), lddr, static_cast<uint16_t*>(dx), lddx, M, C, rpb, mean, invstd, gamma, beta,
      param_bf16, 1, dsums_ws, dsums_ws + C, ss, dgamma, dbeta, accumulate, Segs{});
  TONY_LAUNCH_CHECK();
  return 0;
}

// tony_bn_bwd_res with the forward's byte mask (tony_bn_apply_res_m) in place of y
TONY_API int tony_bn_bwd_res_m(const void* x, int64_t ldx, const void* dy, int64_t lddy, const void* mask, int64_t ldm,
                               void* dx, int64_t lddx, void* dres, int64_t lddr, int64_t M, int C, const float* mean,
                               const float* invstd, const void* gamma, const void* beta, int param_bf16,
                               float* dsums_ws, void* dgamma, void* dbeta, int accumulate, hipStream_t stream) {
  if (bad_c(C) || (ldx % 8) || (lddy % 8) || (lddx % 8) || (lddr % 8) || mask == nullptr || ldm < C / 8) return -1;
  const int64_t ss = 2 * static_cast<int64_t>(C);
  const auto* mb = static_cast<const uint16_t*>(mask);  // reinterpreted as bytes inside (MB)
  int64_t rpb;
  int grid;
  plan_rows(M, C, 8, 512, &rpb, &grid);
  bn_bwd_reduce_kernel<true, uint16_t, true><<<grid, kThreads, bn_lds_bred(C), stream>>>(
      static_cast<const uint16_t*>(x), ldx, static_cast<const uint16_t*>(dy), lddy, mb, ldm, M, C, rpb, mean, invstd,
      gamma, beta, param_bf16, 1, dsums_ws, dsums_ws + C, ss, Segs{});
  TONY_LAUNCH_CHECK();
  plan_rows(M, C, 4, 8192, &rpb, &grid);
  bn_bwd_apply_kernel<true, uint16_t, false, true><<<grid, kThreads, bn_lds_table(C, 5), stream>>>(
      static_cast<const uint16_t*>(x), ldx, static_cast<const uint16_t*>(dy), lddy, mb, ldm,
      static_cast<uint16_t*>(dres), lddr, static_cast<uint16_t*>(dx), lddx, M, C, rpb, mean, invstd, gamma, beta,
      param_bf16, 1, dsums_ws, dsums_ws + C, ss, dgamma, dbeta, accumulate, Segs{});
  TONY_LAUNCH_CHECK();
  return 0;
}

// Training BN(+ReLU) of z [N,H,W,C] (pixel stride ldz) from the sharded conv-epilogue statistics,
// fused with a KxK / stride-S max pool: writes the pooled y [N,OH,OW,C] (pixel stride ldy) and the
// argmax bytes [N,OH,OW,C]; saves mean / invstd and updates the running statistics.
TONY_API int tony_bn_relu_maxpool(const void* z, int64_t ldz, const float* sum, const float* sumsq, int64_t sstride,
                                  const void* gamma, const void* beta, int param_bf16, float eps, float* save_mean,
                                  float* save_invstd, float* running_mean, float* running_var, float momentum,
                                  void* y, int64_t ldy, void* argmax, int N, int H, int W, int C, int K, int S,
                                  int P, hipStream_t stream) {
  if (bad_c(C) || (ldz % 8) || (ldy % 8) || sstride < 0 || K * K > 255 || P < 0 || 2 * P >= K + 1 ||
      H + 2 * P < K || W + 2 * P < K || S < 1)
    return -1;
  if (static_cast<int64_t>(N) * H * W * (C / 8) > 0x7fffffff) return -1;
  const int OH = (H + 2 * P - K) / S + 1, OW = (W + 2 * P - K) / S + 1;
  int64_t work = static_cast<int64_t>(N) * OH * OW * (C / 8);
  int64_t grid = (work + kThreads - 1) / kThreads;
  if (grid > 16384) grid = 16384;
  const auto kern = K == 3 ? bn_relu_maxpool_kernel<3> : bn_relu_maxpool_kernel<0>;
  kern<<<static_cast<int>(grid < 1 ? 1 : grid), kThreads, bn_lds_table(C, 2), stream>>>(
      static_cast<const uint16_t*>(z), ldz, sum, sumsq, sstride, gamma, beta, param_bf16, eps, save_mean, save_invstd,
      running_mean, running_var, momentum, static_cast<uint16_t*>(y), ldy, static_cast<uint8_t*>(argmax), N, H, W, C,
      OH, OW, K, S, P);
  TONY_LAUNCH_CHECK();
  return 0;
}

// dZ of conv -> BN -> ReLU -> maxpool KxK/S (padding P) from the POOLED gradient dYp [N*OH*OW, C] (row
// stride lddy) and the pool's argmax bytes (bn_bwd_pool_apply_kernel); dsum = [dsum | dsumx] from
// pool.hip tony_maxpool_bwd_bnred (sharded, sstride floats apart); dgamma / dbeta stored (or added).
TONY_API int tony_bn_bwd_pool_apply(const void* dyp, int64_t lddy, const void* argmax, int N, int H, int W, int C, int K,
                                    int S, int P, const void* z, int64_t ldz, void* dz, int64_t lddz, const float* mean,
                                    const float* invstd, const void* gamma, const void* beta, int param_bf16, int relu,
                                    const float* dsum, int64_t sstride, void* dgamma, void* dbeta, int accumulate,
                                    hipStream_t stream) {
  if (bad_c(C) || (lddy % 8) || (ldz % 8) || (lddz % 8) || K < 1 || S < 1 || P < 0 || 2 * P >= K + 1 ||
      H + 2 * P < K || W + 2 * P < K || z == nullptr || dz == nullptr || dyp == nullptr || argmax == nullptr ||
      mean == nullptr || invstd == nullptr || dsum == nullptr || sstride < 0)
    return -1;
  const int64_t M = static_cast<int64_t>(N) * H * W;
  if (M * (C / 8) > 0x7fffffff) return -1;
  const int OH = (H + 2 * P - K) / S + 1, OW = (W + 2 * P - K) / S + 1;
  int64_t rpb;
  int grid;
  plan_rows(M, C, 4, 8192, &rpb, &grid);
  bn_bwd_pool_apply_kernel<<<grid, kThreads, bn_lds_table(C, 5), stream>>>(
      static_cast<const uint16_t*>(dyp), lddy, static_cast<const uint8_t*>(argmax), N, H, W, C, OH, OW, K, S, P,
      static_cast<const uint16_t*>(z), ldz, static_cast<uint16_t*>(dz), lddz, rpb, mean, invstd, gamma, beta,
      param_bf16, relu, dsum, sstride, dgamma, dbeta, accumulate);
  TONY_LAUNCH_CHECK();
  return 0;
}
