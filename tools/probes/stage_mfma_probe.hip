// Issue cost of operand staging beside MFMAs on gfx950: per step each wave issues NM
// v_mfma_f32_16x16x32_bf16 (register operands, 4 accumulators) and NL 1-KiB loads of an
// L2-resident buffer, staged
//   mode 0: by LDS-DMA (global_load_lds_dwordx4, M0 per piece), vmcnt(NL) keeps one step in flight
//   mode 1: through VGPRs (global_load_dwordx4, then ds_write_b128 of the previous step's data)
//   mode 2: no loads (the MFMA floor)
// 8-wave workgroups, one per CU.  Prints ns per step and cycles per step per SIMD at 2.1 GHz.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/stage_mfma_probe.hip -o tools/probes/stage_mfma_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8_t;
typedef __attribute__((__vector_size__(4 * sizeof(float)))) float f32x4;

__device__ __forceinline__ void glds16(const void* src, uint32_t m0) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory", "m0");
}

template <int MODE, int NL, int NM>
__global__ __launch_bounds__(512) void probe(const uint4* __restrict__ buf, uint32_t mask, int iters,
                                             float* __restrict__ sink) {
  __shared__ __attribute__((aligned(16))) uint4 lds[4096];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t base = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) void*)lds)) +
      ((wave * NL) & 63) * 1024);
  uint32_t idx = (blockIdx.x * 8192u + threadIdx.x) & mask;
  bf16x8_t a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = static_cast<__bf16>(0.001f * (lane + j));
    b[j] = static_cast<__bf16>(0.002f * (lane - j));
  }
  f32x4 acc[4] = {};
  uint4 v[NL];
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int j = 0; j < NL; ++j) glds16(buf + ((idx + j * 512u) & mask), base + j * 1024);
    } else if constexpr (MODE == 1) {
      if (it > 0) {
#pragma unroll
        for (int j = 0; j < NL; ++j) lds[((wave * NL + j) & 63) * 64 + lane] = v[j];
      }
#pragma unroll
      for (int j = 0; j < NL; ++j) v[j] = buf[(idx + j * 512u) & mask];
    }
#pragma unroll
    for (int m = 0; m < NM; ++m) acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[m & 3], 0, 0, 0);
    if constexpr (MODE == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NL) : "memory");
    idx = (idx + NL * 512u) & mask;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float s = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
  if (MODE == 1) s += static_cast<float>(lds[threadIdx.x].x);
  if (s == 1234.5f) sink[0] = s;
}

template <int MODE, int NL, int NM>
void run(const uint4* buf, uint32_t mask, float* sink, int iters) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  probe<MODE, NL, NM><<<256, 512>>>(buf, mask, 10, sink);
  (void)hipEventRecord(e0);
  probe<MODE, NL, NM><<<256, 512>>>(buf, mask, iters, sink);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double ns = ms * 1e6 / iters;
  printf("mode %d  NL %d  NM %2d: %7.1f ns/step  %6.0f cyc/step/SIMD @2.1GHz (2 waves)  MFMA floor %4d cyc  %6.1f GB/s/CU\n",
         MODE, NL, NM, ns, ns * 2.1, 2 * NM * 16, (MODE == 2 ? 0.0 : 8.0 * NL * 1024 / ns));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
}

int main() {
  const uint32_t nvec = 1u << 16;
  uint4* buf;
  float* sink;
  (void)hipMalloc(&buf, nvec * sizeof(uint4));
  (void)hipMalloc(&sink, 64);
  (void)hipMemset(buf, 1, nvec * sizeof(uint4));
  const int it = 20000;
  run<2, 4, 24>(buf, nvec - 1, sink, it);
  run<0, 4, 24>(buf, nvec - 1, sink, it);
  run<1, 4, 24>(buf, nvec - 1, sink, it);
  run<0, 2, 24>(buf, nvec - 1, sink, it);
  run<1, 2, 24>(buf, nvec - 1, sink, it);
  run<0, 4, 48>(buf, nvec - 1, sink, it);
  run<1, 4, 48>(buf, nvec - 1, sink, it);
  run<2, 4, 48>(buf, nvec - 1, sink, it);
  run<0, 8, 48>(buf, nvec - 1, sink, it);
  run<1, 8, 48>(buf, nvec - 1, sink, it);
  (void)hipFree(buf);
  (void)hipFree(sink);
  return 0;
}
