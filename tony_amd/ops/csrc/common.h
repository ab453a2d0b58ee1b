// Shared helpers for the tony_amd CDNA4 (gfx950) kernels.
//
// All kernels in this directory are written directly for gfx950: 64-lane
// wavefronts, 16-byte vector memory ops, bf16 stored as raw uint16 bits and
// converted with the hardware cvt (v_cvt_pk_bf16_f32 keeps NaN a NaN).
// Every host entry point is `extern "C"` and takes the HIP stream explicitly so
// the Python side (ctypes) can launch on torch's current stream and the calls
// are capturable into HIP graphs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TONY_API extern "C" __attribute__((visibility("default")))

namespace tony {

static constexpr int kWave = 64;  // CDNA wavefront width (never 32)

// BatchNorm statistics ([sum | sumsq] or the backward [dsum | dsumx]) are accumulated by many
// workgroups with float atomics.  Same-address float atomics serialise at the memory side, so
// with one copy a 5,000-tile conv spends more time in its statistics epilogue than in its MFMAs
// (measured: 682112x80x64 GEMM 51 us without, 266 us with one copy).  Producers therefore add
// into one of kStatShards copies spaced `sstride` floats apart (shard = tile or block index mod
// kStatShards) and consumers sum the copies; sstride == 0 means a single, unsharded copy.
static constexpr int kStatShards = 8;

__device__ __forceinline__ float shard_sum(const float* p, int c, int64_t sstride) {
  if (sstride == 0) return p[c];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kStatShards; ++k) s += p[k * sstride + c];
  return s;
}

__device__ __forceinline__ int64_t shard_off(int idx, int64_t sstride) {
  return sstride == 0 ? 0 : static_cast<int64_t>(idx % kStatShards) * sstride;
}

// ReLU that keeps a NaN a NaN (torch.relu semantics).  fmaxf(NaN, 0) is 0 on CDNA (IEEE maxNum), which
// once turned a NaN produced upstream into a silently all-zero activation instead of a visible error.
__device__ __forceinline__ float relu_f(float t) { return t < 0.f ? 0.f : t; }

__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = static_cast<__bf16>(f);  // lowers to v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(uint16_t, b);
}

// 8 bf16 <-> one 16-byte vector register quad.
struct bf16x8 {
  uint4 raw;
  __device__ __forceinline__ void to_float(float* f) const {
    const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __uint_as_float(w[i] << 16);
      f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static bf16x8 from_float(const float* f) {
    bf16x8 r;
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      w[i] = static_cast<uint32_t>(f2bf(f[2 * i])) |
             (static_cast<uint32_t>(f2bf(f[2 * i + 1])) << 16);
    }
    r.raw = make_uint4(w[0], w[1], w[2], w[3]);
    return r;
  }
};

__device__ __forceinline__ bf16x8 load8(const uint16_t* p) {
  bf16x8 r;
  r.raw = *reinterpret_cast<const uint4*>(p);
  return r;
}
__device__ __forceinline__ void store8(uint16_t* p, const bf16x8& v) {
  *reinterpret_cast<uint4*>(p) = v.raw;
}

// 8 consecutive elements of a bf16 (uint16_t) or fp32 tensor as 8 floats: the element-type
// abstraction of the kernels that serve both the bf16 step and the fp32 x3 step (ops/x3.py)
template <class T>
struct V8;
template <>
struct V8<uint16_t> {
  bf16x8 b;
  __device__ __forceinline__ static V8 load(const uint16_t* p) { return V8{load8(p)}; }
  __device__ __forceinline__ void store(uint16_t* p) const { store8(p, b); }
  __device__ __forceinline__ void to_float(float* f) const { b.to_float(f); }
  __device__ __forceinline__ static V8 from_float(const float* f) { return V8{bf16x8::from_float(f)}; }
};
template <>
struct V8<float> {
  float4 lo, hi;
  __device__ __forceinline__ static V8 load(const float* p) {
    return V8{*reinterpret_cast<const float4*>(p), *reinterpret_cast<const float4*>(p + 4)};
  }
  __device__ __forceinline__ void store(float* p) const {
    *reinterpret_cast<float4*>(p) = lo;
    *reinterpret_cast<float4*>(p + 4) = hi;
  }
  __device__ __forceinline__ void to_float(float* f) const {
    f[0] = lo.x, f[1] = lo.y, f[2] = lo.z, f[3] = lo.w, f[4] = hi.x, f[5] = hi.y, f[6] = hi.z, f[7] = hi.w;
  }
  __device__ __forceinline__ static V8 from_float(const float* f) {
    return V8{make_float4(f[0], f[1], f[2], f[3]), make_float4(f[4], f[5], f[6], f[7])};
  }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

inline int ceil_div(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

}  // namespace tony

// Error code convention for the C ABI: 0 ok, negative = argument error,
// positive = hipError_t from the launch.
#define TONY_LAUNCH_CHECK()                         \
  do {                                              \
    hipError_t _e = hipGetLastError();              \
    if (_e != hipSuccess) return static_cast<int>(_e); \
  } while (0)
