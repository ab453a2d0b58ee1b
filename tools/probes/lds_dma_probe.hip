// Per-CU fill bandwidth of the three ways a tile reaches LDS on gfx950, from an L2-resident buffer:
//   mode 0: global_load_lds_dwordx4 (LDS-DMA, the conv / GEMM kernels' staging)
//   mode 1: global_load_dwordx4 into VGPRs, then ds_write_b128 (register staging)
//   mode 2: global_load_dwordx4 into VGPRs only (the vector-memory path without LDS)
// 8-wave (512-thread) workgroups, NL 16-B loads per lane in flight per batch, `grid` workgroups.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/lds_dma_probe.hip -o /tmp/lds_dma_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ void glds16(const void* src, uint32_t m0) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory", "m0");
}

template <int MODE, int NL>
__global__ __launch_bounds__(512) void probe(const uint4* __restrict__ buf, uint32_t mask, int iters,
                                             uint32_t* __restrict__ sink) {
  __shared__ __attribute__((aligned(16))) uint4 lds[4096];  // 64 KB: 64 slots of 1 KB
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t base = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) void*)lds)) +
      ((wave * NL) & 63) * 1024);
  uint32_t idx = (blockIdx.x * 8192u + threadIdx.x) & mask;
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int j = 0; j < NL; ++j) glds16(buf + ((idx + j * 512u) & mask), base + (j & 63) * 1024);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NL) : "memory");
    } else {
      uint4 v[NL];
#pragma unroll
      for (int j = 0; j < NL; ++j) v[j] = buf[(idx + j * 512u) & mask];
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        if constexpr (MODE == 1)
          lds[((wave * NL + j) & 63) * 64 + lane] = v[j];
        else
          acc ^= v[j].x ^ v[j].w;
      }
    }
    idx = (idx + NL * 512u) & mask;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (MODE == 1) acc = lds[threadIdx.x].x;
  if (acc == 0x12345678u) sink[0] = acc;  // keeps the loads alive
}

template <int MODE, int NL>
void run(const uint4* buf, uint32_t mask, uint32_t* sink, int grid, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  probe<MODE, NL><<<grid, 512>>>(buf, mask, 10, sink);
  hipEventRecord(a);
  probe<MODE, NL><<<grid, 512>>>(buf, mask, iters, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double bytes = double(grid) * 512 * NL * 16 * iters;
  printf("mode %d NL %2d grid %4d: %8.3f ms  %7.1f GB/s chip  %6.1f GB/s per CU  %5.1f B/clk/CU @2.4GHz\n", MODE, NL,
         grid, ms, bytes / ms / 1e6, bytes / ms / 1e6 / 256, bytes / ms / 1e6 / 256 / 2.4);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main() {
  const uint32_t nvec = 1u << 16;  // 1 MB: L2-resident in every XCD
  uint4* buf;
  uint32_t* sink;
  hipMalloc(&buf, nvec * sizeof(uint4));
  hipMalloc(&sink, 64);
  hipMemset(buf, 1, nvec * sizeof(uint4));
  const int iters = 4000;
  for (int grid : {256, 512}) {
    run<0, 4>(buf, nvec - 1, sink, grid, iters);
    run<0, 8>(buf, nvec - 1, sink, grid, iters);
    run<1, 4>(buf, nvec - 1, sink, grid, iters);
    run<1, 8>(buf, nvec - 1, sink, grid, iters);
    run<2, 8>(buf, nvec - 1, sink, grid, iters);
  }
  hipFree(buf);
  hipFree(sink);
  return 0;
}
