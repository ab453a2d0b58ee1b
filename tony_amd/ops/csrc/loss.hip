// Fused softmax cross-entropy forward/backward with optional label smoothing
// (SURVEY.md §2.7 H9).  One 256-thread workgroup per row; the row is held in
// registers (K <= 256*kPerThread) so the max / sum-exp / target passes read the
// logits from HBM exactly once.  Backward recomputes the softmax from the saved
// log-sum-exp, so no [N,K] probability tensor is ever materialised.
#include "common.h"

using namespace tony;

namespace {

constexpr int kThreads = 256;
constexpr int kPerThread = 16;  // K <= 4096

template <bool kBf16>
__device__ __forceinline__ float ld(const void* p, int64_t i) {
  if constexpr (kBf16) return bf2f(static_cast<const uint16_t*>(p)[i]);
  return static_cast<const float*>(p)[i];
}

__device__ __forceinline__ float block_reduce(float v, float* sh, bool is_max) {
  v = is_max ? wave_max(v) : wave_sum(v);
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  __syncthreads();
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  float r = sh[0];
#pragma unroll
  for (int k = 1; k < kThreads / kWave; ++k) r = is_max ? fmaxf(r, sh[k]) : r + sh[k];
  return r;
}

template <bool kBf16>
__global__ __launch_bounds__(kThreads) void xent_fwd_kernel(const void* __restrict__ logits, int64_t ld_,
                                                            int K, const int64_t* __restrict__ labels,
                                                            float smoothing, float* __restrict__ loss,
                                                            float* __restrict__ lse_out) {
  __shared__ float sh[kThreads / kWave];
  const int64_t row = blockIdx.x;
  const int64_t base = row * ld_;
  float v[kPerThread];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < kPerThread; ++j) {
    const int k = threadIdx.x + j * kThreads;
    v[j] = k < K ? ld<kBf16>(logits, base + k) : -INFINITY;
    mx = fmaxf(mx, v[j]);
  }
  mx = block_reduce(mx, sh, true);
  float se = 0.f, sx = 0.f;
#pragma unroll
  for (int j = 0; j < kPerThread; ++j) {
    const int k = threadIdx.x + j * kThreads;
    if (k < K) {
      se += __expf(v[j] - mx);
      sx += v[j];
    }
  }
  se = block_reduce(se, sh, false);
  sx = block_reduce(sx, sh, false);
  if (threadIdx.x == 0) {
    const float lse = mx + __logf(se);
    const int64_t t = labels[row];
    const float xt = (t >= 0 && t < K) ? ld<kBf16>(logits, base + t) : lse;
    // loss = -(1-s) * log p_t - s/K * sum_k log p_k
    loss[row] = (1.f - smoothing) * (lse - xt) + smoothing * (lse - sx / static_cast<float>(K));
    lse_out[row] = lse;
  }
}

template <bool kBf16>
__global__ __launch_bounds__(kThreads) void xent_bwd_kernel(const void* __restrict__ logits, int64_t ld_,
                                                            int K, const int64_t* __restrict__ labels,
                                                            float smoothing, const float* __restrict__ lse,
                                                            const float* __restrict__ gout,
                                                            void* __restrict__ dlogits, int64_t ldd) {
  const int64_t row = blockIdx.x;
  const float l = lse[row];
  const float go = gout[row];
  const int64_t t = labels[row];
  const float off = smoothing / static_cast<float>(K);
  for (int k = threadIdx.x; k < K; k += kThreads) {
    const float p = __expf(ld<kBf16>(logits, row * ld_ + k) - l);
    const float target = (k == t ? 1.f - smoothing : 0.f) + off;
    const float d = (p - target) * go;
    if constexpr (kBf16)
      static_cast<uint16_t*>(dlogits)[row * ldd + k] = f2bf(d);
    else
      static_cast<float*>(dlogits)[row * ldd + k] = d;
  }
}

}  // namespace

TONY_API int tony_xent_fwd(const void* logits, int is_bf16, int64_t N, int K, int64_t ld_,
                           const int64_t* labels, float smoothing, float* loss, float* lse,
                           hipStream_t stream) {
  if (K <= 0 || K > kThreads * kPerThread) return -1;
  if (is_bf16)
    xent_fwd_kernel<true><<<N, kThreads, 0, stream>>>(logits, ld_, K, labels, smoothing, loss, lse);
  else
    xent_fwd_kernel<false><<<N, kThreads, 0, stream>>>(logits, ld_, K, labels, smoothing, loss, lse);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_xent_bwd(const void* logits, int is_bf16, int64_t N, int K, int64_t ld_,
                           const int64_t* labels, float smoothing, const float* lse, const float* gout,
                           void* dlogits, int64_t ldd, hipStream_t stream) {
  if (K <= 0) return -1;
  if (is_bf16)
    xent_bwd_kernel<true><<<N, kThreads, 0, stream>>>(logits, ld_, K, labels, smoothing, lse, gout, dlogits, ldd);
  else
    xent_bwd_kernel<false><<<N, kThreads, 0, stream>>>(logits, ld_, K, labels, smoothing, lse, gout, dlogits, ldd);
  TONY_LAUNCH_CHECK();
  return 0;
}
