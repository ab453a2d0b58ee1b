// The implicit-GEMM operand gather shared by the conv kernels (conv.hip) and the LDS-DMA
// NT kernel that both the convolutions and the 1x1-conv / FC GEMMs (gemm.hip) use.
//
// GEMM view: C[m, n] = sum_k A[m, k] B[n, k], m = (image, oy, ox) over [N][OH][OW], k = (r, s, c) over
// the filter taps and source channels.  A plain row-major A[M, K] (row stride lda) is the special
// case of a 1 x M "image" with K channels and a 1x1 filter (gemm_gather below).
#pragma once

#include <algorithm>
#include <cstdlib>
#include <tuple>
#include <type_traits>

#include "mfma_common.h"

namespace tony {
// Split-K workspace of the next LDS-DMA NT launches made by this host thread (tony_splitk_workspace,
// conv.hip): the fp32 partial tiles and one arrival counter per output tile (zero on first use; the
// last arriver re-arms it).  A launch that asks for splits without a big enough workspace runs unsplit.
struct SplitWs {
  float* slab = nullptr;
  int64_t slab_floats = 0;
  unsigned* cnt = nullptr;
  int64_t ncnt = 0;
};
SplitWs& splitk_ws();
}  // namespace tony

namespace tony {
namespace glds {  // (named: the launchers below are defined in their own translation units, glds*.hip)

using namespace tony::mfma;

// stream-K of conv_glds_kernel (see the kernel): workgroups own equal ranges of the (tile, K-step)
// iterations; the contributors of a tile shared by several workgroups fold their fp32 partials
// through the slab, the last arriver (per-tile ticket) summing them in K order
struct SplitK {
  float* slab = nullptr;    // 2 partial tiles per workgroup
  unsigned* cnt = nullptr;  // per tile: a ticket counter, then (ntiles further) a done counter
  int ntiles = 0;
  int stream = 0;
};

struct Gather {
  const uint16_t* src;  // source image, pixel-major: pixel p at src + p * ld
  int64_t ld;           // elements per pixel row (>= Cs; a channel slice of a concat buffer is fine)
  int Hs, Ws, Cs;       // source spatial dims and channels
  int OH, OW;           // the GEMM row space: m -> (n, oy, ox) over [N][OH][OW]
  int R, S;             // filter taps
  int sh, sw;           // stride of the output grid in source pixels
  int offh, offw;       // source coord = o*stride + off + sign*tap
  int sign;             // +1 convolution, -1 transposed (dgrad)
  int K;                // R * S * Cs
  int halo_images;      // batch count N (the halo-tile path walks images x tile rows x tile columns)
};

struct RowState {
  int pix;   // n * Hs * Ws
  int iy0;   // oy*sh + offh
  int ix0;   // ox*sw + offw
  bool ok;   // row < M
  const uint16_t* base;  // src + (pix + iy0 * Ws + ix0) * ld: the row's source at tap (0, 0), channel 0
                         // (outside the image for padded rows; only dereferenced with a tap in bounds)
  __device__ __forceinline__ void set_base(const struct Gather& g);
};

__device__ __forceinline__ void RowState::set_base(const Gather& g) {
  base = g.src + (static_cast<int64_t>(pix) + static_cast<int64_t>(iy0) * g.Ws + ix0) * g.ld;
}

// position of a K chunk: channel c of tap (r, s)
struct TapPos {
  int c, r, s;
  // element offset of this chunk from a row's tap-(0, 0) source (RowState::base): one product per
  // K-step shared by all of a thread's rows instead of a 64-bit (pix + iy * Ws + ix) * ld per row
  __device__ __forceinline__ int off(const struct Gather& g) const {
    return g.sign * (r * g.Ws + s) * static_cast<int>(g.ld) + c;
  }
  __device__ __forceinline__ void init(int k, const Gather& g) {
    c = k % g.Cs;
    const int tap = k / g.Cs;
    r = tap / g.S;
    s = tap - r * g.S;
  }
  __device__ __forceinline__ void advance(int dk, const Gather& g) {
    c += dk;
    while (c >= g.Cs) {
      c -= g.Cs;
      if (++s == g.S) {
        s = 0;
        ++r;
      }
    }
  }
};

// Where the B (filter) row of K-chunk tap (a, b) starts, for the uniform-tap loop: S == 0, the row is
// contiguous over the taps (a conv's [Co][R][S][Ci] / a GEMM's B); else the taps of one residue class
// of a strided dgrad read the FULL transposed filter Wt [Ci][R][S][Co] at r = r0 + sy * a,
// s = s0 + sx * b (row stride R * S * Co) -- no per-class weight copies.
struct BTaps {
  int r0 = 0, s0 = 0, sy = 1, sx = 1, S = 0;
};

// The x3 (fp32) operands of conv_glds_kernel X3 (ops/x3.py): A holds [hi | lo | hi] planes of Cs channels
// per pixel (the lo plane alo elements after the hi one), B rows hold per tap [hi | hi | lo] planes (btap
// elements per tap, the lo plane blo after the hi one).  The kernel stages A hi / lo and B hi / lo once per
// K-step and issues the three products hi*hi + lo*hi + hi*lo on the same accumulators (K = R * S * Cs),
// instead of running the three planes as 3x the K with the hi planes staged twice.
struct X3Planes {
  int alo = 0, blo = 0, btap = 0;
  // AT (conv_glds_kernel): [scale | shift] per A channel (K floats each): the A operand is BN-applied +
  // ReLU'd in LDS as it lands -- relu(a * scale[k] + shift[k]) -- the "apply in the consumer" prototype
  // (profiles/r5_bn_apply_in_consumer_ab.md); 1x1 (GEMM) operands only
  const float* atab = nullptr;
};

// Every residue class of a strided dgrad in ONE launch (tony_conv_dgrad_strided): the classes' tile
// ranges sit end to end in the grid, each padded to a multiple of 8 workgroups so that the XCD remap
// runs per class -- every XCD gets an eighth of every class (the classes differ up to 4x in taps, so a
// whole-grid remap would hand the 4-tap class to two XCDs and the 1-tap class to two others), the
// tap-heaviest class dispatched first; the <= 7 pad workgroups per class exit at once.  Each
// workgroup swaps in its class's gather, row map, tap set and row count before the K loop.
// n == 0: a single GEMM (the kernel's own arguments).  One launch instead of sh * sw: the classes'
// tiles fill the CUs together instead of four small grids running one after another.
struct ClassDesc {
  Gather g;
  RowMap rm;
  BTaps bt;
  int M = 0;
  int begin = 0, tiles = 0;  // first workgroup (a multiple of 8) and tile count (set by run_glds)
};
constexpr int kMaxClasses = 4;
struct MultiClass {
  int n = 0;
  ClassDesc c[kMaxClasses];
};

// A[M, K] row-major (row stride lda) as a Gather: one 1 x M image with K channels, 1x1 filter.
inline Gather gemm_gather(const void* A, int64_t lda, int64_t M, int64_t K) {
  return Gather{static_cast<const uint16_t*>(A), lda, 1, static_cast<int>(M), static_cast<int>(K), 1,
                static_cast<int>(M), 1, 1, 1, 1, 0, 0, 1, static_cast<int>(K), 1};
}

// ---- forward / stride-1 dgrad with LDS-DMA staging and wide wave tiles (variants 11..15) -------
// conv_nt_kernel stages both operands through VGPRs (global_load -> ds_write_b128) and its 32x48
// wave tiles read 5 fragments per 6 MFMAs: per 64-deep K-step the LDS array carries ~420 cycles
// (the 13-cycle ds_write_b128 transfer dominates) against 192 MFMA cycles per SIMD.  Here
//   * every 16-byte chunk goes global -> LDS by global_load_lds_dwordx4 (no VGPR round trip, no
//     ds_write): a wave instruction fills 1 KB of LDS rows (8 rows of 128 B at KB = 64, 16 rows of
//     64 B at KB = 32) lane-linearly; the LDS swizzle is applied on the SOURCE side -- the lane that
//     lands on physical chunk p of row r fetches logical chunk p ^ swz(r) -- so the fragment reads
//     stay conflict-free;
//   * padding taps, rows past M and columns past N / K fetch the 16 zero bytes of kZeroChunk;
//   * ST stages ring in LDS, ST - 1 of them in flight behind the MFMAs; completion is one counted
//     `s_waitcnt vmcnt` + s_barrier per K-step (hipcc does not see the DMAs, see glds16);
//   * 2x2 waves of (BM/2) x (BN/2): 64x64 wave tiles read 8 fragments per 16 MFMAs.
// Measured on MI355X (tools/variant_bench.py): what matters most is resident waves -- a 3-stage
// 96 KB ring at one workgroup per CU ran 1.5x slower than a 2-stage 64 KB one at two -- so the
// 32-deep K-steps (KB = 32) exist to keep 2-3 stages in flight at 2-3 workgroups per CU.
// Each thread owns one K chunk column for the whole loop, so the tap walk (TapPos) is per thread,
// as in conv_nt_kernel.  Row groups that do not divide evenly over the 4 waves are re-fetched by a
// wave with a spare instruction slot (identical bytes to the same LDS row: benign, and it keeps the
// per-wave DMA count a compile-time constant for the vmcnt wait).
constexpr int kGldsFirst = 11;
// TONY_GLDS_UNI=0 in the environment keeps the general loop for every shape (A/B measurements)
inline bool glds_uni_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("TONY_GLDS_UNI");
    return !(e != nullptr && e[0] == '0');
  }();
  return on;
}
struct GldsVariant {
  int bm, cap, stages, kb, nwm;  // nwm: waves along M (workgroup = 2 x nwm waves)
  bool il = false;               // interleaved DMA issue (conv_glds_kernel IL; UNI shapes only)
  bool pf = false;               // fragment prefetch (conv_glds_kernel PF)
  int wpe = 0;                   // > 0: register budget for wpe waves per SIMD (conv_glds_occ_kernel)
};
// 11-15: 4-wave 64/128-row tiles at 2-3 workgroups per CU; 16-19: 8-wave 256-row tiles at one (16-18)
// or two (19) workgroups per CU -- each B (weight) tile is shared by 256 rows, so the LDS-DMA intake
// per MFMA is 1.3-1.45x lower than the 128-row tiles' (the conv K loops are intake-latency bound:
// profiles/r3s2_pmc_glds_conv.md), and the ring is deeper per tile
constexpr GldsVariant kGldsVariants[] = {
    {128, 128, 2, 64, 2}, {128, 128, 3, 32, 2}, {128, 128, 4, 32, 2}, {128, 192, 3, 32, 2}, {64, 128, 4, 32, 2},
    {256, 192, 4, 32, 4}, {256, 128, 3, 64, 4}, {256, 192, 5, 32, 4}, {256, 128, 3, 32, 4},
    // 20-24: the interleaved-issue forms of the most-picked tiles (11-19 above)
    {128, 128, 3, 32, 2, true}, {128, 192, 3, 32, 2, true}, {128, 128, 2, 64, 2, true},
    {256, 192, 4, 32, 4, true}, {256, 128, 3, 32, 4, true},
    // 25-31: several workgroups per CU (conv_glds_occ_kernel: a register budget of wpe waves per SIMD and a
    // ring that fits the LDS wpe * 64 / (2 * nwm) times)
    {256, 128, 3, 32, 4, false, false, 4}, {256, 128, 3, 32, 4, true, false, 4}, {128, 128, 3, 32, 2, false, false, 3},
    {128, 128, 3, 32, 2, true, false, 3}, {128, 192, 3, 32, 2, false, false, 2}, {64, 128, 4, 32, 2, false, false, 3},
    {64, 128, 3, 32, 2, false, false, 4}};
// (measured and dropped in round 6: fragment-prefetch forms of 11 / 12 / 14 / 15 / 17-19, PF below -- at most
// 1.09x on one 17x17 layer, flat on the step; the 256 x 192 forms spilled: profiles/r6_conv_pf_scaling.log)
// (measured and dropped in round 5: the 256 x 192 tile on a two-slot ring of 64-deep stages, half the
// barriers per K -- plain 0.93-0.97x of variant 23, interleaved 0.6x; profiles/r5_conv_limits.md)
constexpr int kNumGlds = sizeof(kGldsVariants) / sizeof(kGldsVariants[0]);

template <int N>
__device__ __forceinline__ void glds_wait_barrier() {  // this thread's DMAs but the last N landed, then all waves
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// LDS layout of a KB-deep operand tile: row r holds KB bf16 (KB / 8 chunks of 16 B); logical chunk c
// sits at physical chunk c ^ swz(r).  KB = 64: lds_off's (r & 7).  KB = 32 (4 chunks, 4 rows per
// 256-B bank period): s[(r >> 2) & 3] with s = {0, 2, 3, 1} puts the 16 (row, chunk) pairs of every
// ds_read_b128 lane group ({0-3,12-15,20-27}, ...) on 16 distinct 16-B bank slots.
template <int KB>
__device__ __forceinline__ int gswz(int row) {
  if constexpr (KB == 64) return row & 7;
  else return (0x1320 >> (((row >> 2) & 3) * 4)) & 3;  // {0, 2, 3, 1}
}
template <int KB>
__device__ __forceinline__ int goff(int row, int ch) {
  return row * KB + ((ch ^ gswz<KB>(row)) << 3);
}

// UNI (Cs % KB == 0, every Inception / ResNet layer past the stem): each lane's channel walk
// crosses into the next filter tap at the same K-step, so the tap (r, s) is wave-uniform.  A DMA's
// source then only moves KB channels per step (one 64-bit add; zero-fill lanes point at kZeroChunk
// with a zero increment) and its bounds are re-derived once per tap in a scalar branch, instead of
// the per-step TapPos walk + im2col address + bounds math: the general loop spends ~65 VALU
// instructions per K-step against 12-24 MFMAs, more VALU issue than the MFMAs leave free.
// IL (UNI only): the next stage's DMAs are issued one piece at a time BETWEEN the MFMA groups of the
// current stage (after its fragments are read) instead of all at once right after the barrier -- a
// global_load_lds costs the issuing wave ~60-185 cycles of issue, which then overlaps the matrix pipe
// working off the MFMAs already issued (MI355X_MICROARCH.md, LDS-DMA piece issue cost).
// PF: the fragments of K-substep k+1 are read from LDS into a second register set while substep k's MFMAs
// issue, so no MFMA waits on a ds_read issued after the barrier (profiles/r5_conv_limits.md: the read ->
// MFMA dependency at the head of every step held the plain loop at ~2x the MFMA + DMA issue floor).  A
// stage's slot is refilled right after the barrier that follows its last fragment read (every wave then
// holds those fragments in registers), so all ST slots carry DMAs: one stage more in flight per ring.
// FT: the stream-K segments (SplitK, bit 0) / every-residue-class launches (MultiClass, bit 1) compiled in.
// 0, the workgroup runs exactly one whole tile with none of their state: the round-5 kernels carried both in every
// launch and grew from 122 to 240 VGPRs (256 x 128) / 168 to 256 + spills (256 x 192), SGPRs 85 -> 106,
// which halved the resident workgroups and cost the bf16 step 0.5-1.4 ms (profiles/r6_regression_bisect.md).
template <int BM, int BN, int ST, int KB, bool UNI, int NWM, bool IL, bool X3, bool AT, bool PF, int FT>
__device__ __forceinline__ void conv_glds_body(Gather g, const uint16_t* __restrict__ B, int64_t ldb,
                                               uint16_t* __restrict__ C, int64_t ldc, int M, int N,
                                               float* __restrict__ stats, int64_t sstride, int epi,
                                               int tiles_n, RowMap rmap, BTaps bt, SplitK sk,
                                               X3Planes xp, MultiClass mc) {
  constexpr int NW = 2 * NWM;                 // waves: NWM along M x 2 along N
  constexpr int WM = BM / NWM, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int CPR = KB / 8;                // 16-B chunks per LDS row
  constexpr int RPI = 64 / CPR;              // rows per DMA instruction (1 KB)
  constexpr int AG = BM / RPI, BG = BN / RPI;  // row groups per operand tile
  constexpr int AI = (AG + NW - 1) / NW, BI = (BG + NW - 1) / NW;  // DMA instructions per wave and stage
  constexpr int PL = X3 ? 2 : 1;             // staged planes per operand: X3 [hi | lo]
  constexpr int STAGE = PL * (BM + BN) * KB; // elements
  constexpr int KSUB = KB / 32;              // MFMA K-steps per stage
  constexpr int NDMA = PL * (AI + BI);       // DMA instructions per thread and stage
  static_assert(BM % RPI == 0 && BN % RPI == 0 && BN % 32 == 0 && ST >= 2 && (KB == 32 || KB == 64), "tile shape");
  static_assert(!X3 || (UNI && !IL), "the fused x3 planes run the plain uniform-tap loop");
  static_assert(!AT || (UNI && !IL && !X3), "the A transform runs in the plain uniform-tap loop");
  static_assert(!PF || (!IL && !X3 && !AT), "the fragment prefetch runs the plain loop");
  static_assert(BM * (BN + 8) <= ST * STAGE, "the epilogue's C tile fits in the ring");
  __shared__ __attribute__((aligned(16))) uint16_t smem[ST * STAGE];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int G = gridDim.x;
  int w = 0;
  if ((FT & 2) && mc.n > 0) {  // (uniform; static indices only, so the descriptors stay scalar kernel-argument loads)
    const int b = blockIdx.x;
    int sel = 0;
#pragma unroll
    for (int i = 1; i < kMaxClasses; ++i)
      if (i < mc.n && b >= mc.c[i].begin) sel = i;
#pragma unroll
    for (int i = 0; i < kMaxClasses; ++i)
      if (i == sel) {
        g = mc.c[i].g;
        rmap = mc.c[i].rm;
        bt = mc.c[i].bt;
        M = mc.c[i].M;
        w = xcd_remap(b - mc.c[i].begin, (mc.c[i].tiles + 7) & ~7);
        if (w >= mc.c[i].tiles) return;  // pad workgroup (before any barrier)
      }
  } else {
    w = xcd_remap(blockIdx.x, G);
  }
  const int K = g.K;
  // (>= 1: a strided dgrad's tap-less residue class has K = 0 and must still write its zero tile)
  const int nk_all = max(1, (K + KB - 1) / KB);
  // Work: the (tile, K-step) iterations.  Plain: workgroup w = one whole tile.  Stream-K (sk.stream):
  // the tiles x nk_all iterations cut into gridDim.x equal contiguous ranges, one per workgroup (the
  // grid sized to what the CUs hold at once, so the last tiles do not run as a near-empty second
  // wave); a workgroup walks its range tile segment by tile segment.  A segment that is a whole tile
  // runs the epilogue itself; the segments of a shared tile meet in SplitK's fold.  Neighbouring
  // ranges share a tile, so the remap keeps them on one XCD.
  const int64_t T = static_cast<int64_t>(tiles_n) * ((M + BM - 1) / BM) * nk_all;
  const bool streamk = (FT & 1) && sk.stream;
  int64_t it = streamk ? static_cast<int64_t>(w) * T / G : static_cast<int64_t>(w) * nk_all;
  const int64_t it_end = streamk ? static_cast<int64_t>(w + 1) * T / G : it + nk_all;
  for (bool first_seg = true; it < it_end; first_seg = false) {
  if ((FT & 1) && !first_seg) __syncthreads();  // the previous segment's epilogue is done with the LDS
  const int tile = static_cast<int>(it / nk_all);
  const int kt0 = static_cast<int>(it - static_cast<int64_t>(tile) * nk_all);
  const int nk = static_cast<int>(min(static_cast<int64_t>(nk_all - kt0), it_end - it));
  it += nk;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kstart = kt0 * KB;
  const int kend = min(K, (kt0 + nk) * KB);
  const int rin = lane / CPR;                     // row within the instruction's row group
  const int ck = (lane % CPR) ^ gswz<KB>(rin);    // logical K chunk this lane fetches (row groups are
                                                  // RPI-aligned, so swz(row) == swz(rin))

  RowState rs[AI];
  int agrp[AI];
  const int ohw = g.OH * g.OW;
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    agrp[i] = min(wave + NW * i, AG - 1);
    const int m = m0 + agrp[i] * RPI + rin;
    rs[i].ok = m < M;
    const int mm = rs[i].ok ? m : 0;
    const int n = mm / ohw, rem = mm - n * ohw;
    const int oy = rem / g.OW, ox = rem - oy * g.OW;
    rs[i].pix = n * g.Hs * g.Ws;
    rs[i].iy0 = oy * g.sh + g.offh;
    rs[i].ix0 = ox * g.sw + g.offw;
    rs[i].set_base(g);
  }
  const uint16_t* brow[BI];
  bool bok[BI];
  int bgrp[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    bgrp[i] = min(wave + NW * i, BG - 1);
    const int n = n0 + bgrp[i] * RPI + rin;
    bok[i] = n < N;
    brow[i] = B + static_cast<int64_t>(bok[i] ? n : 0) * ldb;
  }
  TapPos tp;
  tp.init(ck * 8 + kstart, g);
  int kb = ck * 8 + kstart;  // this thread's K column of the next stage to issue
  const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  constexpr uint32_t kGroupB = RPI * KB * 2;  // bytes per row group
  constexpr uint32_t kStageB = STAGE * 2, kBOff = PL * BM * KB * 2;
  constexpr uint32_t kALo = BM * KB * 2, kBLo = BN * KB * 2;  // X3: the lo plane's tile after the hi one
  uint32_t aoff[AI], boff[BI];  // wave-uniform byte offsets of this wave's row groups
#pragma unroll
  for (int i = 0; i < AI; ++i) aoff[i] = __builtin_amdgcn_readfirstlane(agrp[i] * kGroupB);
#pragma unroll
  for (int i = 0; i < BI; ++i) boff[i] = __builtin_amdgcn_readfirstlane(kBOff + bgrp[i] * kGroupB);

  const uint16_t* zc = reinterpret_cast<const uint16_t*>(&kZeroChunk);
  const uint16_t* ap[AI];
  const uint16_t* bp[BI];
  int ainc[AI], binc[BI];
  int alo[AI], blo[BI];  // X3: element offset of the lo plane from the hi source (0 for zero-fill lanes)
  int ur = 0, us = 0, uleft = 0;
  auto set_tap = [&]() {  // UNI: sources of tap (ur, us) for this thread's DMAs
    const bool tap_ok = ur < g.R;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int iy = rs[i].iy0 + g.sign * ur, ix = rs[i].ix0 + g.sign * us;
      const bool ok = tap_ok & rs[i].ok & (static_cast<unsigned>(iy) < static_cast<unsigned>(g.Hs)) &
                      (static_cast<unsigned>(ix) < static_cast<unsigned>(g.Ws));
      ap[i] = ok ? g.src + (static_cast<int64_t>(rs[i].pix) + iy * g.Ws + ix) * g.ld + ck * 8 : zc;
      ainc[i] = ok ? KB : 0;
      alo[i] = ok ? xp.alo : 0;
    }
    if (!tap_ok) {  // K is exhausted (K = R * S * Cs): the ring's tail stages fetch zeros
#pragma unroll
      for (int i = 0; i < BI; ++i) {
        bp[i] = zc;
        binc[i] = 0;
        blo[i] = 0;
      }
    } else if (X3) {  // this tap's hi plane in the filter row ([hi | hi | lo] per tap)
      const int toff = (ur * g.S + us) * xp.btap + ck * 8;
#pragma unroll
      for (int i = 0; i < BI; ++i) {
        bp[i] = bok[i] ? brow[i] + toff : zc;
        binc[i] = bok[i] ? KB : 0;
        blo[i] = bok[i] ? xp.blo : 0;
      }
    } else if (bt.S != 0) {  // a strided dgrad's residue class: this tap's slice of the full filter row
      const int toff = ((bt.r0 + bt.sy * ur) * bt.S + bt.s0 + bt.sx * us) * g.Cs + ck * 8;
#pragma unroll
      for (int i = 0; i < BI; ++i) {
        bp[i] = bok[i] ? brow[i] + toff : zc;
        binc[i] = bok[i] ? KB : 0;
      }
    }
    uleft = g.Cs / KB;
  };
  if constexpr (UNI) {
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      bp[i] = bok[i] ? brow[i] + ck * 8 : zc;
      binc[i] = bok[i] ? KB : 0;
    }
    if (kstart == 0) {
      set_tap();
    } else {  // a later split: start at tap (ur, us), channel c0 of it (KB-aligned: Cs % KB == 0)
      const int tap = kstart / g.Cs, c0 = kstart - tap * g.Cs;
      ur = tap / g.S;
      us = tap - ur * g.S;
      if (bt.S == 0 && !X3) {
#pragma unroll
        for (int i = 0; i < BI; ++i) bp[i] += binc[i] / KB * kstart;  // the filter row is contiguous over K
      }
      set_tap();
      const int steps = c0 / KB;
#pragma unroll
      for (int i = 0; i < AI; ++i) ap[i] += ainc[i] * steps;
      if (bt.S != 0 || X3) {
#pragma unroll
        for (int i = 0; i < BI; ++i) bp[i] += binc[i] * steps;
      }
      uleft -= steps;
    }
  }
  int left = nk;  // real stages still to issue; the ring's tail past them fetches zeros

  // UNI: piece p < AI + BI of a stage's DMAs (A rows first), then the per-stage pointer / tap advance
  auto issue_piece = [&](uint32_t st0, int p, bool live) {
#pragma unroll
    for (int i = 0; i < AI; ++i)
      if (p == i) {
        glds16(live ? ap[i] : zc, st0 + aoff[i]);
        ap[i] += ainc[i];
      }
#pragma unroll
    for (int i = 0; i < BI; ++i)
      if (p == AI + i) {
        glds16(live ? bp[i] : zc, st0 + boff[i]);
        bp[i] += binc[i];
      }
  };
  auto issue_advance = [&]() {
    if (--uleft == 0) {
      if (++us == g.S) {
        us = 0;
        ++ur;
      }
      set_tap();
    }
  };
  auto issue = [&](int slot) {
    const uint32_t st0 = base + slot * kStageB;
    const bool live = left-- > 0;
    if constexpr (UNI) {
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        glds16(live ? ap[i] : zc, st0 + aoff[i]);
        if constexpr (X3) glds16(live ? ap[i] + alo[i] : zc, st0 + aoff[i] + kALo);
        ap[i] += ainc[i];
      }
#pragma unroll
      for (int i = 0; i < BI; ++i) {
        glds16(live ? bp[i] : zc, st0 + boff[i]);
        if constexpr (X3) glds16(live ? bp[i] + blo[i] : zc, st0 + boff[i] + kBLo);
        bp[i] += binc[i];
      }
      if (--uleft == 0) {
        if (++us == g.S) {
          us = 0;
          ++ur;
        }
        set_tap();
      }
      return;
    }
    const void* z = &kZeroChunk;
    const int toff = tp.off(g);
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int iy = rs[i].iy0 + g.sign * tp.r, ix = rs[i].ix0 + g.sign * tp.s;
      const bool ok = live & rs[i].ok & (tp.r < g.R) & (static_cast<unsigned>(iy) < static_cast<unsigned>(g.Hs)) &
                      (static_cast<unsigned>(ix) < static_cast<unsigned>(g.Ws));
      const uint16_t* src = rs[i].base + toff;
      glds16(ok ? static_cast<const void*>(src) : z, st0 + aoff[i]);
    }
    const bool kok = live & (kb < kend);
#pragma unroll
    for (int i = 0; i < BI; ++i) glds16((kok & bok[i]) ? static_cast<const void*>(brow[i] + kb) : z, st0 + boff[i]);
    tp.advance(KB, g);
    kb += KB;
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (PF) {
    bf16x8_t fa[2][TM], fb[2][TN];
    // fragments of substep kk of the stage at As into register set BUF
    auto rd = [&](auto bufc, const uint16_t* As, int kk) {
      constexpr int BUF = decltype(bufc)::value;
      const uint16_t* Bs = As + BM * KB;
      const int ch = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[BUF][i] = *reinterpret_cast<const bf16x8_t*>(As + goff<KB>(wm * WM + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[BUF][j] = *reinterpret_cast<const bf16x8_t*>(Bs + goff<KB>(wn * WN + j * 16 + (lane & 15), ch));
    };
    auto mm = [&](auto bufc) {
      constexpr int BUF = decltype(bufc)::value;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[BUF][i], fb[BUF][j], acc[i][j], 0, 0, 0);
    };
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
#pragma unroll
    for (int s = 0; s < ST; ++s) issue(s);
    glds_wait_barrier<(ST - 1) * NDMA>();
    int slot = 0;
    rd(B0{}, smem, 0);
    // stage kt + 1 starts: every wave holds stage kt's last fragments (lgkmcnt) and stage kt + 1 has
    // landed in every wave (vmcnt: the ST - 2 younger stages may fly); stage kt + ST goes into kt's slot
    auto boundary = [&]() -> const uint16_t* {
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"((ST - 2) * NDMA) : "memory");
      issue(slot);
      slot = slot + 1 == ST ? 0 : slot + 1;
      return smem + slot * STAGE;
    };
    if constexpr (KSUB == 1) {
      int kt = 0;
      for (; kt + 2 <= nk; kt += 2) {
        rd(B1{}, boundary(), 0);
        mm(B0{});
        rd(B0{}, boundary(), 0);
        mm(B1{});
      }
      if (kt < nk) {
        rd(B1{}, boundary(), 0);
        mm(B0{});
      }
    } else {
      static_assert(KSUB == 2, "64-deep stages: two substeps");
      for (int kt = 0; kt < nk; ++kt) {
        rd(B1{}, smem + slot * STAGE, 1);
        mm(B0{});
        rd(B0{}, boundary(), 0);
        mm(B1{});
      }
    }
  } else {
#pragma unroll
  for (int s = 0; s < ST - 1; ++s) issue(s);
  int slot = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt has landed everywhere and every wave is done reading stage kt - 1, whose slot takes
    // stage kt + ST - 1 (past the end: zero fills, which keeps the per-thread DMA count uniform)
    if constexpr (AT) {
      // this thread's own A chunks of the stage have landed (its vmcnt): BN-apply + ReLU them in place
      // before the barrier publishes the stage (each row group by its owner wave only: a spare-slot
      // re-fetch holds the same bytes and must not be transformed twice).  1x1 operands: K = channels.
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((ST - 2) * NDMA) : "memory");
      const int c = kstart + kt * KB + ck * 8;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        if (wave + NW * i < AG && c < K) {
          uint4* pv = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(smem) + slot * kStageB + aoff[i] + lane * 16);
          const float4 s0 = *reinterpret_cast<const float4*>(xp.atab + c);
          const float4 s1 = *reinterpret_cast<const float4*>(xp.atab + c + 4);
          const float4 h0 = *reinterpret_cast<const float4*>(xp.atab + K + c);
          const float4 h1 = *reinterpret_cast<const float4*>(xp.atab + K + c + 4);
          const uint4 v = *pv;
          const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
          const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
          uint32_t o[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float lo = fmaxf(fmaf(__uint_as_float(w[q] << 16), sc[2 * q], sh[2 * q]), 0.f);
            const float hi = fmaxf(fmaf(__uint_as_float(w[q] & 0xffff0000u), sc[2 * q + 1], sh[2 * q + 1]), 0.f);
            o[q] = static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
          }
          *pv = make_uint4(o[0], o[1], o[2], o[3]);
        }
      }
      __builtin_amdgcn_s_barrier();
    } else {
      glds_wait_barrier<(ST - 2) * NDMA>();
    }
    const int fill = slot == 0 ? ST - 1 : slot - 1;
    const uint16_t* As = smem + slot * STAGE;
    const uint16_t* Bs = As + PL * BM * KB;
    if constexpr (IL && UNI) {
      // every fragment of the stage first, then MFMA row groups with one DMA piece after each
      constexpr int NP = AI + BI;
      const uint32_t st0 = base + fill * kStageB;
      bf16x8_t af[KSUB][TM], bfr[KSUB][TN];
#pragma unroll
      for (int kk = 0; kk < KSUB; ++kk) {
        const int ch = kk * 4 + (lane >> 4);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[kk][j] = *reinterpret_cast<const bf16x8_t*>(Bs + goff<KB>(wn * WN + j * 16 + (lane & 15), ch));
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[kk][i] = *reinterpret_cast<const bf16x8_t*>(As + goff<KB>(wm * WM + i * 16 + (lane & 15), ch));
      }
      int p = 0;
      const bool live = left-- > 0;
#pragma unroll
      for (int kk = 0; kk < KSUB; ++kk)
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
          // pieces spread over the KSUB * TM groups (the first groups take the extra ones)
          constexpr int G = KSUB * TM;
          const int g0 = kk * TM + i;
          const int pe = (g0 + 1) * NP / G;
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (; p < pe; ++p) issue_piece(st0, p, live);
          __builtin_amdgcn_sched_barrier(0);
        }
      issue_advance();
      slot = slot + 1 == ST ? 0 : slot + 1;
      continue;
    }
    issue(fill);
    if constexpr (X3) {
      // both A planes' fragments held, the B planes streamed column by column (peak 2 TM + 2 fragments
      // live, not 2 (TM + TN): the 256-row 8-wave tiles spilled otherwise); 3 MFMAs per (i, j):
      // hi*hi + lo*hi + hi*lo, each fragment read once per K-step
      const uint16_t* Al = As + BM * KB;
      const uint16_t* Bl = Bs + BN * KB;
#pragma unroll
      for (int kk = 0; kk < KSUB; ++kk) {
        const int ch = kk * 4 + (lane >> 4);
        bf16x8_t ah[TM], al[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          ah[i] = *reinterpret_cast<const bf16x8_t*>(As + goff<KB>(wm * WM + i * 16 + (lane & 15), ch));
          al[i] = *reinterpret_cast<const bf16x8_t*>(Al + goff<KB>(wm * WM + i * 16 + (lane & 15), ch));
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int bo = goff<KB>(wn * WN + j * 16 + (lane & 15), ch);
          const bf16x8_t bh = *reinterpret_cast<const bf16x8_t*>(Bs + bo);
          const bf16x8_t bl = *reinterpret_cast<const bf16x8_t*>(Bl + bo);
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl, acc[i][j], 0, 0, 0);
          }
        }
      }
      slot = slot + 1 == ST ? 0 : slot + 1;
      continue;
    }
#pragma unroll
    for (int kk = 0; kk < KSUB; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8_t*>(As + goff<KB>(wm * WM + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(Bs + goff<KB>(wn * WN + j * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    slot = slot + 1 == ST ? 0 : slot + 1;
  }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's zero fills land before LDS is reused
  __syncthreads();
  if ((FT & 1) && nk != nk_all) {
    // a shared tile: take the tile's ticket first.  Every contributor but the last stores its fp32
    // partial to its slot (part 0: the workgroup's first segment, 1: its last) and counts itself done;
    // the last waits for the others' done count -- they hold tickets, so they are past their K loops
    // and only storing: the wait is bounded by construction -- then sums the contributors in K order,
    // its own accumulators in their place (the same sum whichever contributor is last), and runs the
    // epilogue.  Hand-off with write-through (sc1) 16-B buffer stores and sc1 loads (MI355X guide,
    // in-launch split-K reduction, sc1 form): no agent release -- a `buffer_wbl2` per workgroup writes
    // back the XCD L2's dirty lines (measured: the fold with release / acquire fences doubled a 17x17
    // conv) -- and no acquire.  Every storing wave drains its stores before the barrier that precedes
    // lane 0's done add; the reducer's waves load after the barrier that follows its poll.
    constexpr int NT = 128 * NWM, FR = TM * TN;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(sk.slab, 0, 0x7fffffff, 0x00020000);
    const int64_t t0 = static_cast<int64_t>(tile) * nk_all;
    const int w_first = static_cast<int>(((t0 + 1) * G - 1) / T);  // the workgroups holding the tile's
    const int w_last = static_cast<int>(((t0 + nk_all) * G - 1) / T);  // first / last iteration
    const unsigned others = static_cast<unsigned>(w_last - w_first);
    unsigned* cnt = sk.cnt + tile;
    unsigned* done = sk.cnt + sk.ntiles + tile;
    int* flag = reinterpret_cast<int*>(smem);
    if (threadIdx.x == 0)
      *flag = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == others;
    __syncthreads();
    const bool last = *flag != 0;
    __syncthreads();  // every wave has read the flag before the epilogue stages C over it
    if (!last) {
      const int mine = (2 * w + (first_seg ? 0 : 1)) * FR;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), prs,
                                                 ((mine + i * TN + j) * NT + threadIdx.x) * 16, 0, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    if (threadIdx.x == 0) {
      for (unsigned spins = 0; __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < others &&
                               spins < (1u << 24);
           ++spins)
        __builtin_amdgcn_s_sleep(1);
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed for the next launch
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the poll
    f32x4 own[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        own[i][j] = acc[i][j];
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    for (int c = w_first; c <= w_last; ++c) {
      if (c == w) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] += own[i][j];
        continue;
      }
      // contributor c holds this tile in its first segment iff its range starts inside the tile
      const int slot_c = (2 * c + ((static_cast<int64_t>(c) * T / G) >= t0 ? 0 : 1)) * FR;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     prs, ((slot_c + i * TN + j) * NT + threadIdx.x) * 16, 0, 16));
    }
  }
  const bool am = (epi & 32) != 0;  // masked-source accumulate (tony_gemm_bf16 flags bit5)
  nt_epilogue<BM, BN, TM, TN, ST * STAGE, NWM>(acc, smem, C, ldc, M, N, m0, n0,
                                           (epi & 1) ? stats + shard_off(tm, sstride) : nullptr,
                                           (epi & 2) ? stats : nullptr, (epi & 4) != 0, rmap, (epi & 8) != 0,
                                           (epi & 48) != 0, am ? reinterpret_cast<const uint16_t*>(stats) : nullptr,
                                           am ? reinterpret_cast<const uint8_t*>(sstride) : nullptr);
  if constexpr (!(FT & 1)) break;  // one whole tile per workgroup
  }
}

#define TONY_GLDS_PARAMS                                                                                      \
  Gather g, const uint16_t* __restrict__ B, int64_t ldb, uint16_t* __restrict__ C, int64_t ldc, int M, int N,   \
      float* __restrict__ stats, int64_t sstride, int epi, int tiles_n, RowMap rmap, BTaps bt, SplitK sk,       \
      X3Planes xp, MultiClass mc
#define TONY_GLDS_ARGS g, B, ldb, C, ldc, M, N, stats, sstride, epi, tiles_n, rmap, bt, sk, xp, mc
template <int BM, int BN, int ST, int KB, bool UNI, int NWM = 2, bool IL = false, bool X3 = false, bool AT = false,
          bool PF = false, int FT = 0>
__global__ __launch_bounds__(128 * NWM) void conv_glds_kernel(TONY_GLDS_PARAMS) {
  conv_glds_body<BM, BN, ST, KB, UNI, NWM, IL, X3, AT, PF, FT>(TONY_GLDS_ARGS);
}
// The same loop with a register budget for WPE waves per SIMD (amdgpu_waves_per_eu): WPE * 64 / (2 * NWM)
// workgroups share a CU, so one workgroup's barrier / DMA-landing waits are covered by another's MFMAs
// instead of idling the SIMD (the plain form takes up to 256 VGPRs: two waves per SIMD, one 8-wave
// workgroup per CU, all eight waves meeting at every K-step's barrier: profiles/r5_conv_limits.md)
template <int BM, int BN, int ST, int KB, bool UNI, int NWM, bool IL, int WPE, int FT = 0>
__global__ __launch_bounds__(128 * NWM) __attribute__((amdgpu_waves_per_eu(WPE))) void conv_glds_occ_kernel(
    TONY_GLDS_PARAMS) {
  conv_glds_body<BM, BN, ST, KB, UNI, NWM, IL, false, false, false, FT>(TONY_GLDS_ARGS);
}
#undef TONY_GLDS_PARAMS
#undef TONY_GLDS_ARGS

constexpr int64_t kStreamMaxTiles = 4096;  // counters of a stream-K launch's workspace (ops/_lib.py)
inline int num_cus_of_current() {
  static int cached[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 256;
  if (cached[dev] == 0) {
    int n = 0;
    cached[dev] = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
  }
  return cached[dev];
}

// B rows n = [K] at row stride ldb (the conv weights [Co][R][S][Ci]: ldb = K)
// stream_m > 0: stream-K over stream_m x (CUs) workgroups (SplitK above) when this thread's workspace
// (tony_splitk_workspace) holds 2 partial tiles per workgroup and a counter per tile, else the plain
// launch (same result)
// The fused x3 forms (X3Planes): tiles whose ring of [A hi | A lo | B hi | B lo] stages fits the LDS, the
// plain uniform-tap loop only.  Variant codes kX3First.. of tony_conv_fwd / tony_conv_dgrad.
struct X3Variant {
  int bm, cap, stages, kb, nwm;
};
constexpr int kX3First = 32;
// (no 256 x 160 / 192 tile: 8 waves of 64 x 96 hold 96 accumulator + 40 fragment registers and spilled)
constexpr X3Variant kX3Variants[] = {{256, 128, 2, 32, 4}, {128, 192, 3, 32, 2}, {128, 128, 4, 32, 2},
                                     {128, 128, 2, 64, 2}, {256, 128, 3, 32, 4}, {64, 128, 4, 32, 2}};
constexpr int kNumX3 = sizeof(kX3Variants) / sizeof(kX3Variants[0]);

// Variant families, each compiled in a translation unit of its own (glds_p0..3.hip, glds_x3.hip) so that the
// build runs them in parallel and every kernel instance lives in exactly one code object: case index
// v - kGldsFirst 0-4 (4-wave tiles), 5-8 (8-wave 256-row tiles), 9-13 (interleaved issue), 14-20 (several
// workgroups per CU); the fused x3 forms.
constexpr int glds_part(int c) { return c <= 4 ? 0 : c <= 8 ? 1 : c <= 13 ? 2 : 3; }

// B rows n = [K] at row stride ldb (the conv weights [Co][R][S][Ci]: ldb = K)
// stream_m > 0: stream-K over stream_m x (CUs) workgroups (SplitK above) when this thread's workspace
// (tony_splitk_workspace) holds 2 partial tiles per workgroup and a counter per tile, else the plain
// launch (same result).  Defined in glds.hip.
int run_glds(const Gather& g, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N, int epi,
             float* st, int64_t sstride, int v, hipStream_t stream, RowMap rmap = RowMap{}, BTaps bt = BTaps{},
             int stream_m = 0, X3Planes xp = X3Planes{}, const MultiClass* classes = nullptr);
// the fused x3 forms (codes kX3First..; xp describes the planes)
int run_glds_x3(const Gather& g, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N, int epi,
                float* st, int64_t sstride, int v, hipStream_t stream, RowMap rmap, BTaps bt, int stream_m,
                X3Planes xp);
// one family's launcher (glds_launch.h, instantiated once per family)
template <bool XF, int PART>
int run_glds_part(const Gather& g, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N, int epi,
                  float* st, int64_t sstride, int v, hipStream_t stream, RowMap rmap, BTaps bt, int stream_m,
                  X3Planes xp, const MultiClass* classes);

}  // namespace glds
}  // namespace tony
