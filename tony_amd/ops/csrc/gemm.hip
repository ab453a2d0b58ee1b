// bf16 MFMA GEMM, C[M,N] = A[M,K] * B[N,K]^T (both operands K-contiguous),
// fp32 accumulation, bf16 output, optional fused per-column sum / sum-of-squares
// epilogue (the BatchNorm statistics of a conv output).
//
// Used for NHWC 1x1 convolutions (forward: A = X[NHW, Cin], B = W[Cout, Cin];
// backward-data: A = dY[NHW, Cout], B = W^T[Cin, Cout]) and the classifier FC.
//
// CDNA4 structure:
//  * 256 threads = 4 wave64s in a 2x2 arrangement; each wave owns a
//    (BM/2)x(BN/2) output block built from v_mfma_f32_16x16x32_bf16 tiles.
//  * BK = 64; A/B tiles staged global->VGPR->LDS with 16-byte loads, two LDS
//    buffers, one barrier per K-step: the next tile's global loads are issued
//    before the MFMAs of the current tile so HBM latency hides under compute.
//  * LDS rows are 128 B; the 16-byte chunk c of row r is stored at c^(r&7), which
//    makes every ds_read_b128 lane group of the MFMA operand read hit 16
//    distinct 4-bank slots (conflict free) -- see the bank map in the comment
//    of `lds_off`.
//  * Workgroup ids are remapped so that consecutive output tiles (which share
//    an A row-panel) are dispatched onto the same XCD and hit its private L2.
#include "common.h"

using namespace tony;

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int BK = 64;

// Element offset of 16-byte chunk `ch` (0..7) of LDS row `row` (64 bf16 = 128 B).
// Bank check for one ds_read_b128 lane group (rows r, chunks c fixed per half):
// bank slot = ((r&1)*32 + (c^(r&7))*4) mod 64 -> 16 distinct slots for 16 rows.
__device__ __forceinline__ int lds_off(int row, int ch) { return row * BK + ((ch ^ (row & 7)) << 3); }

// Bijective XCD-aware remap: workgroups dispatched round-robin over 8 XCDs get
// contiguous tile ids per XCD.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, local = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

template <int ROWS>
__device__ __forceinline__ void load_tile(uint4* regs, const uint16_t* __restrict__ G, int64_t ld, int row0,
                                          int nrows, int k0, int K) {
  constexpr int VEC = ROWS * BK / 8 / kThreads;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const int v = threadIdx.x + i * kThreads;
    const int row = v >> 3, ch = v & 7;
    const int gr = row0 + row, gk = k0 + ch * 8;
    if (gr < nrows && gk < K)
      regs[i] = *reinterpret_cast<const uint4*>(G + static_cast<int64_t>(gr) * ld + gk);
    else
      regs[i] = make_uint4(0, 0, 0, 0);
  }
}

template <int ROWS>
__device__ __forceinline__ void store_tile(uint16_t* lds, const uint4* regs) {
  constexpr int VEC = ROWS * BK / 8 / kThreads;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const int v = threadIdx.x + i * kThreads;
    const int row = v >> 3, ch = v & 7;
    *reinterpret_cast<uint4*>(lds + lds_off(row, ch)) = regs[i];
  }
}

template <int BM, int BN>
__global__ __launch_bounds__(kThreads) void gemm_nt_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                           const uint16_t* __restrict__ B, int64_t ldb,
                                                           uint16_t* __restrict__ C, int64_t ldc, int M, int N,
                                                           int K, float* __restrict__ stats, int tiles_n) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int AV = BM * BK / 8 / kThreads, BV = BN * BK / 8 / kThreads;
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * (BM + BN) * BK];

  const int nwg = gridDim.x;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tm = wg / tiles_n, tn = wg % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[AV], rb[BV];
  const int nk = (K + BK - 1) / BK;
  load_tile<BM>(ra, A, lda, m0, M, 0, K);
  load_tile<BN>(rb, B, ldb, n0, N, 0, K);
  store_tile<BM>(smem, ra);
  store_tile<BN>(smem + BM * BK, rb);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    uint16_t* As = smem + (kt & 1) * (BM + BN) * BK;
    uint16_t* Bs = As + BM * BK;
    const bool more = kt + 1 < nk;
    if (more) {
      load_tile<BM>(ra, A, lda, m0, M, (kt + 1) * BK, K);
      load_tile<BN>(rb, B, ldb, n0, N, (kt + 1) * BK, K);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WM + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8_t*>(As + lds_off(r, ch));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WN + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(Bs + lds_off(r, ch));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      uint16_t* An = smem + ((kt + 1) & 1) * (BM + BN) * BK;
      store_tile<BM>(An, ra);
      store_tile<BN>(An + BM * BK, rb);
    }
    __syncthreads();
  }

  // Epilogue: C/D map of 16x16 MFMA: col = lane&15, row = (lane>>4)*4 + r.
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * WN + j * 16 + (lane & 15);
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rowb = m0 + wm * WM + i * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[i][j][r];
        s += v;
        q = fmaf(v, v, q);
        if (rowb + r < M && col < N) C[static_cast<int64_t>(rowb + r) * ldc + col] = f2bf(v);
      }
    }
    if (stats != nullptr) {
      // rows >= M were zero-filled, so they add nothing to the column sums
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (lane < 16 && col < N) {
        atomicAdd(stats + col, s);
        atomicAdd(stats + N + col, q);
      }
    }
  }
}

template <int BM, int BN>
int launch(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N,
           int64_t K, float* stats, hipStream_t stream) {
  const int tiles_m = ceil_div(M, BM), tiles_n = ceil_div(N, BN);
  const int64_t tiles = static_cast<int64_t>(tiles_m) * tiles_n;
  if (tiles > 0x7fffffff) return -2;
  gemm_nt_kernel<BM, BN><<<static_cast<int>(tiles), kThreads, 0, stream>>>(
      static_cast<const uint16_t*>(A), lda, static_cast<const uint16_t*>(B), ldb, static_cast<uint16_t*>(C), ldc,
      static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), stats, tiles_n);
  TONY_LAUNCH_CHECK();
  return 0;
}

}  // namespace

// flags bit0: compute column statistics into stats[2N] (zeroed here).
TONY_API int tony_gemm_bf16(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                            int64_t ldb, int64_t ldc, int flags, float* stats, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return -1;
  if ((K % 8) || (lda % 8) || (ldb % 8)) return -1;
  if (M > 0x7fffffff || N > 0x7fffffff) return -1;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return -1;
  float* st = (flags & 1) ? stats : nullptr;
  if (st != nullptr) (void)hipMemsetAsync(st, 0, sizeof(float) * 2 * N, stream);
  if (N <= 64) return launch<256, 64>(A, lda, B, ldb, C, ldc, M, N, K, st, stream);
  return launch<128, 128>(A, lda, B, ldb, C, ldc, M, N, K, st, stream);
}
