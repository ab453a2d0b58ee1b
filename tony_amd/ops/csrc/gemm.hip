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
#include <type_traits>
#include <cstdlib>

#include "igemm.h"

using namespace tony;
using namespace tony::mfma;
using namespace tony::glds;

namespace {

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
                                                           int K, float* __restrict__ stats, int64_t sstride,
                                                           int epi, int tiles_n) {
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

  // Epilogue (mfma_common.h): BN column statistics from the fp32 accumulators, then the bf16
  // tile staged through LDS and written back with 16-byte coalesced stores.
  // epi bit0: BN statistics into stats (sharded); bit1: stats holds [scale | shift] for the folded
  // inference BN (H5), bit2: ReLU after it
  // bit5: C = tile + (stats as bf16 rows) masked by (sstride as a byte-mask pointer), see tony_gemm_bf16
  const bool am = (epi & 32) != 0;
  nt_epilogue<BM, BN, TM, TN>(acc, smem, C, ldc, M, N, m0, n0,
                               (epi & 1) ? stats + shard_off(tm, sstride) : nullptr,
                               (epi & 2) ? stats : nullptr, (epi & 4) != 0, RowMap{}, (epi & 8) != 0,
                               (epi & 48) != 0, am ? reinterpret_cast<const uint16_t*>(stats) : nullptr,
                               am ? reinterpret_cast<const uint8_t*>(sstride) : nullptr);
}

template <int BM, int BN>
int launch(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N,
           int64_t K, float* stats, int64_t sstride, int epi, hipStream_t stream) {
  const int tiles_m = ceil_div(M, BM), tiles_n = ceil_div(N, BN);
  const int64_t tiles = static_cast<int64_t>(tiles_m) * tiles_n;
  if (tiles > 0x7fffffff) return -2;
  gemm_nt_kernel<BM, BN><<<static_cast<int>(tiles), kThreads, 0, stream>>>(
      static_cast<const uint16_t*>(A), lda, static_cast<const uint16_t*>(B), ldb, static_cast<uint16_t*>(C), ldc,
      static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), stats, sstride, epi, tiles_n);
  TONY_LAUNCH_CHECK();
  return 0;
}

template <int BM>
int launch_bm(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N,
              int64_t K, float* st, int64_t sstride, int epi, int64_t bn, hipStream_t stream) {
  if constexpr (BM == 256) {  // 8 x TN accumulators per wave: only narrow column tiles fit the registers
    if (bn <= 32) return launch<256, 32>(A, lda, B, ldb, C, ldc, M, N, K, st, sstride, epi, stream);
    if (bn <= 64) return launch<256, 64>(A, lda, B, ldb, C, ldc, M, N, K, st, sstride, epi, stream);
    return -3;
  } else {
    switch (bn) {
      case 32: return launch<BM, 32>(A, lda, B, ldb, C, ldc, M, N, K, st, sstride, epi, stream);
      case 64: return launch<BM, 64>(A, lda, B, ldb, C, ldc, M, N, K, st, sstride, epi, stream);
      case 96: return launch<BM, 96>(A, lda, B, ldb, C, ldc, M, N, K, st, sstride, epi, stream);
      case 128: return launch<BM, 128>(A, lda, B, ldb, C, ldc, M, N, K, st, sstride, epi, stream);
      case 160: return launch<BM, 160>(A, lda, B, ldb, C, ldc, M, N, K, st, sstride, epi, stream);
      default: return launch<BM, 192>(A, lda, B, ldb, C, ldc, M, N, K, st, sstride, epi, stream);
    }
  }
}

}  // namespace

// flags bit0: compute column statistics into stats[2N] (zero on entry; kStatShards copies sstride
// floats apart when sstride > 0, common.h); bit1: C = bf16(acc * stats[col] + stats[N + col]) (folded
// inference BN), bit2: ReLU after it; bit4: C += the product; bit5: C = the product + S masked by
// Mk, with S = stats read as a bf16 [M, ldc] matrix and Mk = sstride read as the address of its ReLU
// byte mask [M, ldc / 8] (ops/residual.py MaskedGrad: a residual tail's d(identity), never
// materialised); bits 8..15: tile variant (kNtVariants, mfma_common.h); bits 16..19: stream-K grid in CUs (LDS-DMA
// variants, igemm.h SplitK; tony_splitk_workspace).
// The BN-apply-in-the-consumer prototype (profiles/r5_bn_apply_in_consumer_ab.md): C = relu(A *
// scale + shift) . B^T with the per-channel affine + ReLU applied to each A chunk in LDS as it lands
// (igemm.h X3Planes::atab, table [scale[K] | shift[K]] fp32), on the 128 x 128 three-slot LDS-DMA tile
// (variant 12); flags as tony_gemm_bf16 (bits 0-4).  Measured against bn apply + GEMM by
// tools/bn_consumer_bench.py.
TONY_API int tony_gemm_bf16_bnact(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                                  int64_t ldb, int64_t ldc, int flags, float* stats, int64_t sstride, const float* table,
                                  hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || sstride < 0 || table == nullptr) return -1;
  if ((K % 8) || (lda % 8) || (ldb % 8) || M > 0x7fffffff || N > 0x7fffffff) return -1;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return -1;
  const int epi = flags & 31;
  if (((epi & 1) && (epi & 2)) || ((epi & 16) && (epi & 3)) || ((epi & 3) && stats == nullptr)) return -1;
  X3Planes xp{};
  xp.atab = table;
  return run_glds(gemm_gather(A, lda, M, K), B, ldb, C, ldc, M, N, epi, stats, sstride, kGldsFirst + 1, stream,
                  RowMap{}, BTaps{}, 0, xp);
}

TONY_API int tony_gemm_bf16(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                            int64_t ldb, int64_t ldc, int flags, float* stats, int64_t sstride, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || sstride < 0) return -1;
  if ((K % 8) || (lda % 8) || (ldb % 8)) return -1;
  if (M > 0x7fffffff || N > 0x7fffffff) return -1;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return -1;
  // bit0: st is accumulated into with atomics (the caller hands it over zeroed, ops/arena.py);
  // bit1: st = [scale | shift] of the folded inference BN, bit2: ReLU after it (H5)
  const int epi = flags & 63;  // bit3: fp32 output; bit4: C += the product (nt_epilogue accum)
  if ((epi & 1) && (epi & 2)) return -1;
  if ((epi & 16) && (epi & 3)) return -1;  // no statistics / folded BN on an accumulating store
  if ((epi & 32) && ((epi & 31) || stats == nullptr || sstride == 0 || (ldc % 8) ||
                     (reinterpret_cast<uintptr_t>(stats) & 15)))
    return -1;
  if ((epi & 3) && stats == nullptr) return -1;
  float* st = stats;
  const int v = (flags >> 8) & 0xff;
  if (((flags >> 16) & 15) && !(v >= kGldsFirst && v < kGldsFirst + kNumGlds)) return -3;  // stream-K: LDS-DMA only
  if (v >= kGldsFirst && v < kGldsFirst + kNumGlds)  // LDS-DMA kernel on A as a 1x1 "conv" (igemm.h)
    return run_glds(gemm_gather(A, lda, M, K), B, ldb, C, ldc, M, N, epi, st, sstride, v, stream, RowMap{}, BTaps{},
                    (flags >> 16) & 15);
  if (v >= kNumNtVariants) return -1;
  if (v == 0) {
    if (N <= 64) return launch<256, 64>(A, lda, B, ldb, C, ldc, M, N, K, st, sstride, epi, stream);
    return launch<128, 128>(A, lda, B, ldb, C, ldc, M, N, K, st, sstride, epi, stream);
  }
  const int64_t bn = pick_bn(N, kNtVariants[v].cap);
  switch (kNtVariants[v].bm) {
    case 64: return launch_bm<64>(A, lda, B, ldb, C, ldc, M, N, K, st, sstride, epi, bn, stream);
    case 128: return launch_bm<128>(A, lda, B, ldb, C, ldc, M, N, K, st, sstride, epi, bn, stream);
    default: return launch_bm<256>(A, lda, B, ldb, C, ldc, M, N, K, st, sstride, epi, bn, stream);
  }
}

// ---------------------------------------------------------------------------
// Weight-gradient GEMM ("TN", split-K): C[N1,N2] += sum_m A[m,n1] * B[m,n2]
// with A = dY[M, Cout] and B = X[M, Cin] (both row-major over m).  For a 1x1
// conv this is dW = dY^T X: a huge reduction (M = N*H*W up to ~2.8M rows) into
// a tiny output, so M is split across workgroups and partial tiles are added
// into an fp32 workspace with device-scope atomics (one wave instruction adds
// four 64-byte row segments).
//
// Both MFMA operands need 8 consecutive m per lane while memory holds rows of
// m, so tiles are staged row-major ([m][col], 256 B rows) and read with
// gfx950's transposing LDS read ds_read_b64_tr_b16: a 16-lane group reads a
// 4-row x 16-column block and lane i receives column i.  The 16-byte chunk c of
// LDS row r is stored at c ^ s(r), s(r) = 2*((r&3) | ((r>>3)&1)<<2), so the
// eight rows a 32-lane half reads in one instruction land on 8 disjoint
// chunk pairs = all 64 banks once (conflict free).
// ---------------------------------------------------------------------------
namespace {

constexpr int TBM = 128;   // n1 (Cout) per tile
constexpr int TBN = 128;   // n2 (Cin) per tile

__device__ __forceinline__ void tn_load(uint4* regs, const uint16_t* __restrict__ G, int64_t ld, int64_t m0,
                                        int64_t m1, int c0, int ncols) {
  // tile = TBK rows x 128 cols = 512 chunks of 16 B; 256 threads x 2
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = threadIdx.x + i * kThreads;
    const int row = v >> 4, ch = v & 15;
    const int64_t gm = m0 + row;
    const int gc = c0 + ch * 8;
    if (gm < m1 && gc < ncols)
      regs[i] = *reinterpret_cast<const uint4*>(G + gm * ld + gc);
    else
      regs[i] = make_uint4(0, 0, 0, 0);
  }
}

__device__ __forceinline__ void tn_store(uint16_t* lds, const uint4* regs) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = threadIdx.x + i * kThreads;
    const int row = v >> 4, ch = v & 15;
    *reinterpret_cast<uint4*>(lds + tr_off(row, ch)) = regs[i];
  }
}

// The same split-K TN GEMM with both operand stages written straight into a 3-slot LDS ring by
// LDS-DMA (mfma_common.h glds16): two stages in flight behind the MFMAs instead of one, no VGPR
// staging.  Lane-linear LDS image; the tr_off swizzle moves to the source side (lane l of a row
// fetches logical chunk (l & 15) ^ tr_swz(row)).  Slab mode only.
constexpr int kTnStages = 3;

__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_tn_glds_kernel(
    const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb, int64_t M, int N1,
    int N2, int tiles_n2, int ntiles, int64_t rows_per_split, float* __restrict__ slab, SplitFold fold) {
  constexpr int TILE = TBK * 128, STAGE = 2 * TILE;
  __shared__ __attribute__((aligned(16))) uint16_t smem[kTnStages * STAGE];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wg % ntiles, split = wg / ntiles;
  const int t1 = tile / tiles_n2, t2 = tile % tiles_n2;
  const int n1_0 = t1 * TBM, n2_0 = t2 * TBN;
  const int64_t m_begin = static_cast<int64_t>(split) * rows_per_split;
  const int64_t m_end = min(M, m_begin + rows_per_split);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  const int r0 = threadIdx.x >> 4;
  const int ch = (threadIdx.x & 15) ^ tr_swz(r0);  // tr_swz(r0 + 16) == tr_swz(r0)
  const bool aok = n1_0 + ch * 8 < N1, bok = n2_0 + ch * 8 < N2;
  const uint16_t* ap = A + n1_0 + ch * 8;
  const uint16_t* bp = B + n2_0 + ch * 8;
  // row pointers advance by TBK rows per stage (no 64-bit m * ld product per DMA)
  int am = static_cast<int>(m_begin) + r0;
  const int mend = static_cast<int>(m_end);
  const uint16_t* apm = ap + (m_begin + r0) * lda;
  const uint16_t* bpm = bp + (m_begin + r0) * ldb;
  const int64_t astep = TBK * lda, bstep = TBK * ldb;
  const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(smem) + (4 * wave) * 256);
  constexpr uint32_t kRow16 = 16 * 256, kStageB = STAGE * 2, kTileB = TILE * 2;
  auto issue = [&](int slot) {
    const uint32_t As = base + slot * kStageB, Bs = As + kTileB;
    const void* z = &kZeroChunk;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool mok = am + 16 * i < mend;
      glds16(aok & mok ? static_cast<const void*>(apm + i * 16 * lda) : z, As + i * kRow16);
      glds16(bok & mok ? static_cast<const void*>(bpm + i * 16 * ldb) : z, Bs + i * kRow16);
    }
    am += TBK;
    apm += astep;
    bpm += bstep;
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = static_cast<int>((m_end - m_begin + TBK - 1) / TBK);
  issue(0);
  issue(1);
  const int kgrp = lane >> 4;
  // unrolled by the ring length: compile-time slots, so the fragment reads use immediate offsets
  auto step = [&](auto slot_c) {
    constexpr int SLOT = decltype(slot_c)::value;
    // stage kt landed here (4 DMAs per stage, stage kt+1's may still fly) and, after the barrier,
    // everywhere; stage kt-1's slot is free for stage kt+2 (zero fills past the end)
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue((SLOT + 2) % kTnStages);
    const uint16_t* As = smem + SLOT * STAGE;
    const uint16_t* Bs = As + TILE;
    bf16x8_t af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = tr_frag(As, kgrp, wm * 64 + i * 16, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = tr_frag(Bs, kgrp, wn * 64 + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  };
  static_assert(kTnStages == 3, "the K loop is unrolled by the ring length");
  int kt = 0;
  for (; kt + 3 <= nk; kt += 3) {
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
  }
  if (kt < nk) step(std::integral_constant<int, 0>{});
  if (kt + 1 < nk) step(std::integral_constant<int, 1>{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (fold.flags & 4) {  // the splits meet in-launch (splitk_tree_fold)
    splitk_tree_fold<4, 4, kThreads>(acc, slab, N2, n1_0 + wm * 64, N1, n2_0 + wn * 64, N2, tile, split,
                                     gridDim.x / ntiles, fold);
    return;
  }
  float* dst = slab + static_cast<int64_t>(split) * N1 * N2;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n2_0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = n1_0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (row < N1 && col < N2) dst[static_cast<int64_t>(row) * N2 + col] = acc[i][j][r];
      }
    }
  }
  if (fold.counters != nullptr)
    splitk_fold_tile<TBM, TBN>(slab, static_cast<int64_t>(N1) * N2, gridDim.x / ntiles, N2, n1_0, N1, n2_0, N2, tile,
                               fold);
}

bool tn_glds_enabled() {
  static const bool on = [] {
    const char* e = getenv("TONY_WGRAD_GLDS");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

__global__ __launch_bounds__(kThreads) void gemm_tn_splitk_kernel(
    const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb,
    float* __restrict__ C, int64_t ldc, int64_t M, int N1, int N2, int tiles_n2, int ntiles,
    int64_t rows_per_split, float* __restrict__ slab, SplitFold fold) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * 2 * TBK * 128];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wg % ntiles, split = wg / ntiles;
  const int t1 = tile / tiles_n2, t2 = tile % tiles_n2;
  const int n1_0 = t1 * TBM, n2_0 = t2 * TBN;
  const int64_t m_begin = static_cast<int64_t>(split) * rows_per_split;
  const int64_t m_end = min(M, m_begin + rows_per_split);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = static_cast<int>((m_end - m_begin + TBK - 1) / TBK);
  uint4 ra[2], rb[2];
  if (nk > 0) {
    tn_load(ra, A, lda, m_begin, m_end, n1_0, N1);
    tn_load(rb, B, ldb, m_begin, m_end, n2_0, N2);
    tn_store(smem, ra);
    tn_store(smem + TBK * 128, rb);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const uint16_t* As = smem + (kt & 1) * 2 * TBK * 128;
    const uint16_t* Bs = As + TBK * 128;
    const bool more = kt + 1 < nk;
    if (more) {
      const int64_t mn = m_begin + static_cast<int64_t>(kt + 1) * TBK;
      tn_load(ra, A, lda, mn, m_end, n1_0, N1);
      tn_load(rb, B, ldb, mn, m_end, n2_0, N2);
    }
    const int kgrp = lane >> 4;
    bf16x8_t af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = tr_frag(As, kgrp, wm * 64 + i * 16, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = tr_frag(Bs, kgrp, wn * 64 + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (more) {
      uint16_t* An = smem + ((kt + 1) & 1) * 2 * TBK * 128;
      tn_store(An, ra);
      tn_store(An + TBK * 128, rb);
    }
    __syncthreads();
  }
  // acc[i][j] element r: row n1 = .. + (lane>>4)*4 + r, col n2 = .. + (lane&15).
  if (slab != nullptr && (fold.flags & 4)) {  // the splits meet in-launch (splitk_tree_fold)
    splitk_tree_fold<4, 4, kThreads>(acc, slab, N2, n1_0 + wm * 64, N1, n2_0 + wn * 64, N2, tile, split,
                                     gridDim.x / ntiles, fold);
    return;
  }
  // slab mode: this split's dense [N1][N2] partial with plain stores (tony_splitk_reduce sums them)
  float* dst = slab != nullptr ? slab + static_cast<int64_t>(split) * N1 * N2 : C;
  const int64_t ld = slab != nullptr ? N2 : ldc;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n2_0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = n1_0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (row < N1 && col < N2) {
          if (slab != nullptr)
            dst[static_cast<int64_t>(row) * ld + col] = acc[i][j][r];
          else
            atomicAdd(dst + static_cast<int64_t>(row) * ld + col, acc[i][j][r]);
        }
      }
    }
  }
  if (slab != nullptr && fold.counters != nullptr)
    splitk_fold_tile<TBM, TBN>(slab, static_cast<int64_t>(N1) * N2, gridDim.x / ntiles, N2, n1_0, N1, n2_0, N2, tile,
                               fold);
}

}  // namespace

// C (fp32, [N1, N2], zero on entry) = A^T B ; A [M, N1] (lda), B [M, N2] (ldb).  With a slab
// (slab_cap floats >= splits * N1*N2) the M splits store dense partials there instead of atomics
// into C; *splits_out gets the split count for tony_splitk_reduce.
TONY_API int tony_gemm_tn_bf16(const void* A, const void* B, float* C, int64_t M, int64_t N1, int64_t N2,
                               int64_t lda, int64_t ldb, int64_t ldc, float* slab, int64_t slab_cap,
                               int* splits_out, int num_cus, unsigned* fold_counters, void* fold_dst, int fold_flags,
                               hipStream_t stream) {
  if (M <= 0 || N1 <= 0 || N2 <= 0 || (slab == nullptr && C == nullptr)) return -1;
  if (fold_counters != nullptr && (slab == nullptr || fold_dst == nullptr || (reinterpret_cast<uintptr_t>(fold_dst) & 7)))
    return -1;
  const SplitFold fold{fold_counters, fold_dst, fold_flags};
  if ((N1 % 8) || (N2 % 8) || (lda % 8) || (ldb % 8)) return -1;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return -1;
  // C is accumulated into with atomics: the caller hands it over zeroed (ops/arena.py)
  const int tiles_n1 = ceil_div(N1, TBM), tiles_n2 = ceil_div(N2, TBN);
  const int ntiles = tiles_n1 * tiles_n2;
  // enough workgroups for ~2 per CU, each reducing >= 8 K-steps
  const int target = 2 * (num_cus > 0 ? num_cus : 256);
  int64_t splits = (target + ntiles - 1) / ntiles;
  const int64_t max_splits = (M + 8 * TBK - 1) / (8 * TBK);
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int64_t rows = (M + splits - 1) / splits;
  rows = (rows + TBK - 1) / TBK * TBK;
  splits = (M + rows - 1) / rows;
  const int64_t grid = splits * ntiles;
  if (grid > 0x7fffffff) return -2;
  if (slab != nullptr && splits * N1 * N2 > slab_cap) return -4;  // caller's bound is off
  // the tree fold's workspace: one TBM x TBN fp32 slot per workgroup, 32-bit byte offsets
  if ((fold_flags & 4) && (fold_counters == nullptr || slab == nullptr || grid * TBM * TBN > slab_cap ||
                           grid * TBM * TBN * 4 > 0x7fffffff))
    return -3;
  if (splits_out != nullptr) *splits_out = static_cast<int>(splits);
  if (slab != nullptr && tn_glds_enabled())
    gemm_tn_glds_kernel<<<static_cast<int>(grid), kThreads, 0, stream>>>(
        static_cast<const uint16_t*>(A), lda, static_cast<const uint16_t*>(B), ldb, M, static_cast<int>(N1),
        static_cast<int>(N2), tiles_n2, ntiles, rows, slab, fold);
  else
    gemm_tn_splitk_kernel<<<static_cast<int>(grid), kThreads, 0, stream>>>(
        static_cast<const uint16_t*>(A), lda, static_cast<const uint16_t*>(B), ldb, C, ldc, M, static_cast<int>(N1),
        static_cast<int>(N2), tiles_n2, ntiles, rows, slab, fold);
  TONY_LAUNCH_CHECK();
  return 0;
}
