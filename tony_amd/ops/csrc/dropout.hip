// Dropout with a counter-based mask: keep(element e of step t) = hash(seed, t, e) >= p, where t is
// a step counter; both live in device memory (rng = [seed, t]).  No generator state is consumed on the host, so a
// step captured once and replayed (hipGraph replay or the native plan, csrc/plan.hip) draws a NEW
// mask on every replay: tony_counter_bump, issued right after the forward on the same stream, is a
// node of the captured step and advances t on the device.  (A philox draw from torch's generator
// would replay the capture-time seed/offset unless hipGraph replay's generator prologue runs, which
// the native plan does not call.)
//
// Forward: y = x * keep / (1 - p), plus a 1-bit keep mask (8 elements per byte) for the backward:
// dx = dy * keep / (1 - p).  Each thread owns 8 consecutive elements: two splitmix64 draws give 16
// bits per element, compared against p * 65536.
#include "common.h"

using namespace tony;

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const uint16_t* p) { return bf2f(*p); }
__device__ __forceinline__ void st1(float* p, float v) { *p = v; }
__device__ __forceinline__ void st1(uint16_t* p, float v) { *p = f2bf(v); }

template <typename T>
__global__ __launch_bounds__(kThreads) void dropout_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                               uint8_t* __restrict__ mask, int64_t n, uint32_t thr,
                                                               float scale, const int64_t* __restrict__ rng) {
  const int64_t g = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;  // group of 8 elements
  const int64_t e0 = g * 8;
  if (e0 >= n) return;
  const uint64_t key = mix64(static_cast<uint64_t>(rng[0]) ^ mix64(static_cast<uint64_t>(rng[1]) + 0x632be59bd9b4e019ull));
  const uint64_t h0 = mix64(key + 2 * static_cast<uint64_t>(g)), h1 = mix64(key + 2 * static_cast<uint64_t>(g) + 1);
  unsigned bits = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const uint32_t r = static_cast<uint32_t>(((e < 4 ? h0 : h1) >> (16 * (e & 3))) & 0xffffu);
    bits |= (r >= thr ? 1u : 0u) << e;
  }
  mask[g] = static_cast<uint8_t>(bits);
  float v[8];
  if (e0 + 8 <= n) {
    V8<T>::load(x + e0).to_float(v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = ((bits >> e) & 1u) ? v[e] * scale : 0.f;
    V8<T>::from_float(v).store(y + e0);
  } else {
    for (int e = 0; e < 8 && e0 + e < n; ++e) st1(y + e0 + e, ((bits >> e) & 1u) ? ld1(x + e0 + e) * scale : 0.f);
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void dropout_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx,
                                                               const uint8_t* __restrict__ mask, int64_t n,
                                                               float scale) {
  const int64_t g = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  const int64_t e0 = g * 8;
  if (e0 >= n) return;
  const unsigned bits = mask[g];
  if (e0 + 8 <= n) {
    float v[8];
    V8<T>::load(dy + e0).to_float(v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = ((bits >> e) & 1u) ? v[e] * scale : 0.f;
    V8<T>::from_float(v).store(dx + e0);
  } else {
    for (int e = 0; e < 8 && e0 + e < n; ++e) st1(dx + e0 + e, ((bits >> e) & 1u) ? ld1(dy + e0 + e) * scale : 0.f);
  }
}

__global__ void counter_bump_kernel(int64_t* rng) { rng[1] += 1; }

}  // namespace

// x / y: n contiguous elements (bf16 when is_bf16, else fp32), 16-byte aligned; mask: ceil(n / 8) bytes.
// rng: device int64 [seed, step counter]
TONY_API int tony_dropout_fwd(const void* x, void* y, void* mask, int64_t n, int is_bf16, float p, const int64_t* rng,
                              hipStream_t stream) {
  if (n <= 0) return 0;
  if (!(p >= 0.f && p < 1.f)) return -1;
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) return -3;
  const uint32_t thr = static_cast<uint32_t>(p * 65536.f + 0.5f);
  const float scale = 1.f / (1.f - p);
  const int64_t groups = (n + 7) / 8;
  const int blocks = ceil_div(groups, kThreads);
  if (is_bf16)
    dropout_fwd_kernel<uint16_t><<<blocks, kThreads, 0, stream>>>(static_cast<const uint16_t*>(x),
                                                                  static_cast<uint16_t*>(y),
                                                                  static_cast<uint8_t*>(mask), n, thr, scale, rng);
  else
    dropout_fwd_kernel<float><<<blocks, kThreads, 0, stream>>>(static_cast<const float*>(x), static_cast<float*>(y),
                                                               static_cast<uint8_t*>(mask), n, thr, scale, rng);
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int tony_dropout_bwd(const void* dy, void* dx, const void* mask, int64_t n, int is_bf16, float p,
                              hipStream_t stream) {
  if (n <= 0) return 0;
  if (!(p >= 0.f && p < 1.f)) return -1;
  if ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(dx)) & 15) return -3;
  const float scale = 1.f / (1.f - p);
  const int blocks = ceil_div((n + 7) / 8, kThreads);
  if (is_bf16)
    dropout_bwd_kernel<uint16_t><<<blocks, kThreads, 0, stream>>>(static_cast<const uint16_t*>(dy),
                                                                  static_cast<uint16_t*>(dx),
                                                                  static_cast<const uint8_t*>(mask), n, scale);
  else
    dropout_bwd_kernel<float><<<blocks, kThreads, 0, stream>>>(static_cast<const float*>(dy), static_cast<float*>(dx),
                                                               static_cast<const uint8_t*>(mask), n, scale);
  TONY_LAUNCH_CHECK();
  return 0;
}

// rng[1] += 1 on the stream (one thread): the next forward draws the next step's mask
TONY_API int tony_counter_bump(int64_t* rng, hipStream_t stream) {
  counter_bump_kernel<<<1, 1, 0, stream>>>(rng);
  TONY_LAUNCH_CHECK();
  return 0;
}
