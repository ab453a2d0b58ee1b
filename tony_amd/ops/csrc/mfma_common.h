// Building blocks shared by the MFMA GEMM (gemm.hip) and the implicit-GEMM
// convolutions (conv.hip): operand typedefs, LDS swizzles, the XCD-aware tile
// remap and the transposed-LDS fragment read.
#pragma once

#include "common.h"

namespace tony {
namespace mfma {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

constexpr int kThreads = 256;
constexpr int BK = 64;  // K depth of one NT K-step (LDS rows of 64 bf16 = 128 B)

// Element offset of 16-byte chunk `ch` (0..7) of LDS row `row` (64 bf16 = 128 B).
// Bank check for one ds_read_b128 lane group (rows r, chunks c fixed per half):
// bank slot = ((r&1)*32 + (c^(r&7))*4) mod 64 -> 16 distinct slots for 16 rows.
__device__ __forceinline__ int lds_off(int row, int ch) { return row * BK + ((ch ^ (row & 7)) << 3); }

// Bijective XCD-aware remap: workgroups dispatched round-robin over 8 XCDs get
// contiguous tile ids per XCD (tiles sharing an operand panel share an L2).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, local = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

// ---- "TN" operands: tiles staged row-major over the reduction dim ([m][col], 256-B rows) and read
// with gfx950's transposing LDS read ds_read_b64_tr_b16.  Chunk c of LDS row r lives at c ^ s(r),
// s(r) = 2*((r&3) | ((r>>3)&1)<<2): the eight rows a 32-lane half reads in one instruction land on
// 8 disjoint chunk pairs = all 64 banks once (conflict free).
constexpr int TBK = 32;    // reduction rows per TN K-step
__device__ __forceinline__ int tr_swz(int row) { return (((row & 3) | (((row >> 3) & 1) << 2)) << 1); }
__device__ __forceinline__ int tr_off(int row, int ch) { return row * 128 + ((ch ^ tr_swz(row)) << 3); }

// MFMA operand fragment (8 consecutive reduction rows for one column) via two transposed reads.
__device__ __forceinline__ bf16x8_t tr_frag(const uint16_t* lds, int kgrp, int col0, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3;
  const int col = col0 + 4 * p;          // this lane supplies row q, columns 4p..4p+3
  const int ch = col >> 3, half = (col >> 2) & 1;
  const int r0 = kgrp * 8 + q;
  const uint16_t* a0 = lds + tr_off(r0, ch) + half * 4;
  const uint16_t* a1 = lds + tr_off(r0 + 4, ch) + half * 4;
  v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a0));
  v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a1));
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  v8i16 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, r);
}

// ---- LDS-DMA staging (global_load_lds_dwordx4): a wave instruction writes 64 x 16 B lane-linearly
// from the wave-uniform LDS byte address in M0.  Issued from inline asm so that hipcc neither counts
// it nor makes every ds_read wait vmcnt(0) for it (it cannot tell LDS-DMA targets apart); the
// kernel waits with its own counted s_waitcnt vmcnt(N) + s_barrier.  Out-of-range lanes fetch the
// 16 zero bytes of kZeroChunk.
__device__ const uint4 kZeroChunk = {0u, 0u, 0u, 0u};

// M0 is declared clobbered rather than saved and restored around every DMA: the compiler
// re-materialises it only where it needs it, which the K loops do not (2 fewer SALU per DMA; a K-step
// issues 4-6 of them beside 12-24 MFMAs).
__device__ __forceinline__ void glds16(const void* src, uint32_t lds_wave_base) {
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off"
      :
      : "v"(src), "s"(lds_wave_base)
      : "memory", "m0");
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const void*)p));
}

// ---- split-K fold: the LAST workgroup of a tile sums every split's partial (no combine launch) ----
// A slab-mode split-K kernel stores its partial tile to slab[split * n + ...]; each workgroup then
// announces its arrival on a per-tile counter (release), and the workgroup that arrives last
// (acquire) sums the `splits` partials of its tile in split order -- deterministic whichever
// workgroup that is -- and writes the result into dst: fp32 or bf16, stored or added.
struct SplitFold {
  unsigned* counters;  // one per tile, zero on entry; nullptr: the caller runs tony_splitk_reduce
  void* dst;
  int flags;           // bit0: dst is bf16; bit1: add into dst; bit2: tree fold (splitk_tree_fold)
};

template <int TR, int TC>
__device__ __forceinline__ void splitk_fold_tile(const float* __restrict__ slab, int64_t n, int splits, int64_t ld,
                                                 int r0, int rlim, int c0, int clim, int tile, const SplitFold& f) {
  __shared__ int s_last;
  __threadfence();  // this thread's partial stores are visible device-wide before the arrival below
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(f.counters + tile, 1u) == static_cast<unsigned>(splits - 1);
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  constexpr int C4 = TC / 4;
  const bool bf16 = f.flags & 1, acc = f.flags & 2;
  for (int v = threadIdx.x; v < TR * C4; v += kThreads) {
    const int row = r0 + v / C4, col = c0 + (v % C4) * 4;
    if (row >= rlim || col >= clim) continue;
    const int64_t off = static_cast<int64_t>(row) * ld + col;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 0; k < splits; ++k) {
      const float4 a = *reinterpret_cast<const float4*>(slab + k * n + off);
      s.x += a.x;
      s.y += a.y;
      s.z += a.z;
      s.w += a.w;
    }
    if (bf16) {
      uint2* p = reinterpret_cast<uint2*>(static_cast<uint16_t*>(f.dst) + off);
      if (acc) {
        const uint2 o = *p;
        s.x += __uint_as_float(o.x << 16);
        s.y += __uint_as_float(o.x & 0xffff0000u);
        s.z += __uint_as_float(o.y << 16);
        s.w += __uint_as_float(o.y & 0xffff0000u);
      }
      *p = make_uint2(static_cast<uint32_t>(f2bf(s.x)) | (static_cast<uint32_t>(f2bf(s.y)) << 16),
                      static_cast<uint32_t>(f2bf(s.z)) | (static_cast<uint32_t>(f2bf(s.w)) << 16));
    } else {
      float4* p = reinterpret_cast<float4*>(static_cast<float*>(f.dst) + off);
      if (acc) {
        const float4 o = *p;
        s.x += o.x;
        s.y += o.y;
        s.z += o.z;
        s.w += o.w;
      }
      *p = s;
    }
  }
}

// ---- split-K tree fold: the splits of a tile meet pairwise inside the launch -------------------------
// SplitFold flags bit2.  The splits of a tile are the leaves of a binary tree over the split index.
// Every workgroup first stores its accumulators to its own workspace slot (write-through sc1 stores);
// at each level the two workgroups holding sibling subtrees take a ticket on their node.  The first
// publishes its slot on the node and retires; the second -- which holds a ticket after the first, so
// the first is already past its K loop and only storing: the wait is bounded by construction -- adds
// the published slot into its own (sc1 loads) and climbs.  The root converts its slot into dst.  Each
// node adds left + right subtree sums, so the result does not depend on arrival order.  No separate
// combine launch, no fences (the stream-K hand-off of igemm.h), and the partial reads are spread over
// the splits instead of the last arriver reading all of them (splitk_fold_tile, 5x slower:
// profiles/r2_rejected_splitk_fold_bn_onepass_prof.md).  The level loop works slot to slot, one
// fragment at a time: holding the accumulators in registers across it cost the kernels 86-148 VGPRs
// (the MFMA results moved out of AGPRs next to the partner's loaded copy).
// Workspace (ws, >= gridDim.x * TM * TN * NT * 4 floats): slot (tile, split) holds the accumulators
// lane-linearly -- fragment f of thread t at ((slot * TM * TN + f) * NT + t) * 16 bytes: 16-byte
// coalesced accesses, each thread touching only its own elements.
// counters: [ntiles][2 * splits] tickets then as many slot words (4 * gridDim.x words), zero on entry;
// the second arriver of a node re-arms both.
// acc[i][j][r] is row r0 + i * 16 + (lane >> 4) * 4 + r, column c0 + j * 16 + (lane & 15) of dst (the
// wave's origin folded into r0, c0 by the caller).  Returns true in the workgroup that wrote dst.
template <int TM, int TN, int NT>
__device__ __forceinline__ bool splitk_tree_fold(f32x4 (&acc)[TM][TN], float* __restrict__ ws, int64_t ld, int r0,
                                                 int rlim, int c0, int clim, int tile, int split, int splits,
                                                 const SplitFold& f) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  constexpr int FR = TM * TN;
  constexpr int SLOT = FR * NT * 16;  // bytes per slot
  __shared__ int s_word;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(ws, 0, 0x7fffffff, 0x00020000);
  // (< 2 * splits nodes per tile: sum over levels of ceil(splits / 2^(L+1)) <= splits - 1 + log2 splits)
  unsigned* cnt = f.counters + static_cast<int64_t>(tile) * 2 * splits;
  unsigned* rdy = cnt + 2 * static_cast<int64_t>(gridDim.x);
  const int vt = threadIdx.x * 16;
  const int own = (tile * splits + split) * SLOT;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs, vt, own + (i * TN + j) * NT * 16, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int level_base = 0;
  for (int L = 0; (1 << L) < splits; ++L) {
    const int nodes = (splits + (2 << L) - 1) >> (L + 1);
    const int sib = ((split >> L) ^ 1) << L;
    if (sib < splits) {  // else the sibling subtree is empty: this sum climbs as it is
      const int node = level_base + (split >> (L + 1));
      __syncthreads();  // every wave's slot stores have drained (each waited on its own)
      if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add(cnt + node, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == 0) {  // first: publish the slot and retire
          __hip_atomic_store(rdy + node, static_cast<unsigned>(split + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s_word = -2;
        } else {
          unsigned v = 0;
          for (unsigned spins = 0;
               (v = __hip_atomic_load(rdy + node, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0 && spins < (1u << 24);
               ++spins)
            __builtin_amdgcn_s_sleep(1);
          __hip_atomic_store(cnt + node, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
          __hip_atomic_store(rdy + node, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s_word = static_cast<int>(v) - 1;  // -1: timed out (the sum climbs without the partner)
        }
      }
      __syncthreads();
      const int p = __builtin_amdgcn_readfirstlane(s_word);
      __syncthreads();  // every wave has p before s_word is reused
      if (p == -2) return false;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the poll
      if (p >= 0) {
        const int pb = (tile * splits + p) * SLOT;
#pragma unroll
        for (int k = 0; k < FR; ++k) {
          const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vt, own + k * NT * 16, 16));
          const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vt, pb + k * NT * 16, 16));
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, a + b), rs, vt, own + k * NT * 16, 16);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    level_base += nodes;
  }
  const bool bf16 = f.flags & 1, add = f.flags & 2;
  const int lane = threadIdx.x & 63;
  const int lrow = r0 + (lane >> 4) * 4, lcol = c0 + (lane & 15);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const f32x4 v4 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vt, own + (i * TN + j) * NT * 16, 16));
      const int col = lcol + j * 16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = lrow + i * 16 + r;
        if (row >= rlim || col >= clim) continue;
        const int64_t e = static_cast<int64_t>(row) * ld + col;
        float v = v4[r];
        if (bf16) {
          uint16_t* q = static_cast<uint16_t*>(f.dst) + e;
          if (add) v += __uint_as_float(static_cast<uint32_t>(*q) << 16);
          *q = f2bf(v);
        } else {
          float* q = static_cast<float*>(f.dst) + e;
          *q = add ? *q + v : v;
        }
      }
    }
  return true;
}

// Column tile for a cap: the output channels split evenly over ceil(N/cap) tiles, rounded up to
// the 32-column granule of the 2x2 wave layout (16-wide MFMA per wave), so no MFMA work is spent on
// padding columns for Cout = 32..384 (Inception's 48/80/96/160/192/320/384).
inline int64_t pick_bn(int64_t N, int64_t cap) {
  const int64_t ntn = (N + cap - 1) / cap;
  return ((N + ntn - 1) / ntn + 31) / 32 * 32;
}

// Tile variants (flags bits 8..15), picked per shape by the Python autotuner (ops/tune.py):
// 0 = built-in heuristic; 1.. = (rows per tile, column-tile cap) from kNtVariants.
struct NtVariant {
  int bm, cap;
};
constexpr NtVariant kNtVariants[] = {{0, 0},    {64, 192},  {128, 192}, {256, 64}, {64, 96},
                                     {128, 96}, {128, 128}, {64, 128},  {256, 32}};
constexpr int kNumNtVariants = sizeof(kNtVariants) / sizeof(kNtVariants[0]);

// Output-row remap of the NT epilogue: GEMM row m -> output pixel.  Identity when qw == 0; else
// m = (n, qy, qx) over an [N][QH][QW] sub-grid of an [N][H][W] image and the pixel is
// n*HW + (qy*sy + y0)*W + qx*sx + x0 (one phase of a stride-2 backward-data conv).
struct RowMap {
  int qw = 0, qhw = 0;  // sub-grid width and height*width
  int W = 0, HW = 0;    // image width and height*width
  int sy = 1, sx = 1, y0 = 0, x0 = 0;
  __device__ __forceinline__ int64_t pixel(int m) const {
    if (qw == 0) return m;
    const int n = m / qhw, rem = m - n * qhw;
    const int qy = rem / qw, qx = rem - qy * qw;
    return static_cast<int64_t>(n) * HW + (qy * sy + y0) * W + qx * sx + x0;
  }
};

// NT epilogue: optional per-column BN statistics from the fp32 accumulators, then the bf16 tile
// staged through LDS (rows padded by 16 B) and written with 16-byte coalesced stores.
// acc layout of 16x16 MFMA: col = lane&15, row = (lane>>4)*4 + r.
// With ``aff`` ([scale N | shift N] fp32, the folded inference BatchNorm) the stored value is
// act(acc * scale[col] + shift[col]) (act = ReLU when ``relu``): conv + BN + ReLU in one pass (H5).
// ``f32out`` (the fp32 "x3" path, ops/x3.py): C is an fp32 [M, ldc] matrix and the accumulators are
// stored as they are -- 4 rows x 16 columns (64 contiguous bytes per row) per store instruction.
// NWM: waves along M (the 2 x NWM wave grid of an NWM * 128-thread workgroup; 2 = the 4-wave kernels)
template <int BM, int BN, int TM, int TN, int LDS_ELEMS = 2 * (BM + BN) * BK, int NWM = 2>
__device__ __forceinline__ void nt_epilogue(f32x4 (&acc)[TM][TN], uint16_t* smem, uint16_t* __restrict__ C,
                                            int64_t ldc, int M, int N, int m0, int n0, float* __restrict__ stats,
                                            const float* __restrict__ aff = nullptr, bool relu = false,
                                            const RowMap rm = RowMap{}, bool f32out = false, bool accum = false,
                                            const uint16_t* __restrict__ asrc = nullptr,
                                            const uint8_t* __restrict__ amask = nullptr) {
  // accum: C += the tile (bf16: the stored bf16 tile and C's old value summed in fp32 and rounded once,
  // as the separate add kernel it replaces did) -- a backward-data GEMM adding its dX into the gradient
  // another consumer of the same input already wrote (ResNet's identity path, ops/residual.py)
  // asrc / amask (bf16 C-shaped, row stride ldc, and its ReLU byte mask, row stride ldc / 8): C = the
  // tile + asrc masked by amask -- the other consumer's gradient dY * (y > 0) of a residual tail read
  // where it lies instead of materialised first (ops/residual.py MaskedGrad); C's old value is unused
  constexpr int WM = BM / NWM, WN = BN / 2, NT = 128 * NWM;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  if (stats != nullptr) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * WN + j * 16 + (lane & 15);
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[i][j][r];
          s += v;
          q = fmaf(v, v, q);
        }
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
  if (f32out) {
    float* Cf = reinterpret_cast<float*>(C);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * WN + j * 16 + (lane & 15);
      float sc = 1.f, sh = 0.f;
      if (aff != nullptr) {
        sc = aff[min(col, N - 1)];
        sh = aff[N + min(col, N - 1)];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
          if (row >= M || col >= N) continue;
          float v = acc[i][j][r];
          if (aff != nullptr) v = fmaf(v, sc, sh);
          float* cp = Cf + rm.pixel(row) * ldc + col;
          *cp = (relu ? relu_f(v) : v) + (accum ? *cp : 0.f);
        }
    }
    return;
  }
  constexpr int LDC = BN + 8;
  static_assert(BM * LDC <= LDS_ELEMS, "C staging tile must fit in the LDS buffers");
  uint16_t* Cs = smem;  // the K loop ended with a barrier: both buffers are free
  if (aff != nullptr) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * WN + j * 16 + (lane & 15);
      const int gcol = min(n0 + col, N - 1);
      const float sc = aff[gcol], sh = aff[N + gcol];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * WM + i * 16 + (lane >> 4) * 4 + r;
          const float v = fmaf(acc[i][j][r], sc, sh);
          Cs[row * LDC + col] = f2bf(relu ? relu_f(v) : v);
        }
    }
  } else {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * WM + i * 16 + (lane >> 4) * 4 + r;
          const int col = wn * WN + j * 16 + (lane & 15);
          Cs[row * LDC + col] = f2bf(acc[i][j][r]);
        }
  }
  __syncthreads();
  constexpr int CHUNKS = BM * BN / 8;
  for (int v = threadIdx.x; v < CHUNKS; v += NT) {
    const int row = v / (BN / 8), ch = v % (BN / 8);
    const int grow = m0 + row, gcol = n0 + ch * 8;
    if (grow >= M || gcol >= N) continue;
    const uint16_t* src = Cs + row * LDC + ch * 8;
    uint16_t* dst = C + rm.pixel(grow) * ldc + gcol;
    if (gcol + 8 <= N && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
      if (accum) {
        float a[8], b[8];
        load8(src).to_float(a);
        if (asrc != nullptr) {
          const int64_t pix = rm.pixel(grow);
          load8(asrc + pix * ldc + gcol).to_float(b);
          const unsigned bits = amask[pix * (ldc >> 3) + (gcol >> 3)];
#pragma unroll
          for (int e = 0; e < 8; ++e) a[e] += ((bits >> e) & 1u) ? b[e] : 0.f;
        } else {
          load8(dst).to_float(b);
#pragma unroll
          for (int e = 0; e < 8; ++e) a[e] += b[e];
        }
        store8(dst, bf16x8::from_float(a));
      } else {
        *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
      }
    } else if (accum && asrc != nullptr) {
      const int64_t pix = rm.pixel(grow);
      const unsigned bits = amask[pix * (ldc >> 3) + (gcol >> 3)];
      const uint16_t* as = asrc + pix * ldc + gcol;
      for (int e = 0; e < 8 && gcol + e < N; ++e)
        dst[e] = f2bf(bf2f(src[e]) + (((bits >> e) & 1u) ? bf2f(as[e]) : 0.f));
    } else {
      for (int e = 0; e < 8 && gcol + e < N; ++e) dst[e] = accum ? f2bf(bf2f(src[e]) + bf2f(dst[e])) : src[e];
    }
  }
}

}  // namespace mfma
}  // namespace tony
