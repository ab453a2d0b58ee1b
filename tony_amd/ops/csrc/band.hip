// Band kernel for the 1-D (1 x T / T x 1) stride-1 convolutions of Inception's 17x17 and 8x8 blocks,
// forward and backward-data (tile variant kBandVariant of tony_conv_fwd / tony_conv_dgrad).
//
// Why (profiles/r6_pmc_conv_lean.md): the implicit-GEMM tiles gather every input pixel once per tap
// (a 17x17 1x7 conv streams ~99 MB of A through L2 for 14 MB of unique input) and stall at s_waitcnt /
// barrier with the MFMA pipe 14 % busy.  Here the GEMM rows of a workgroup are L whole "lines" of the
// output -- image rows for a 1 x T filter, image columns for T x 1 -- so the input it needs is the same
// L lines, each padded by T - 1 positions: one halo of L x (wd + T - 1) pixels per 32-channel K chunk,
// read once and used by all T taps straight out of LDS (the A fragment of tap t is the halo shifted by t
// positions).  A K chunk is then T x 32 deep: 7x the MFMAs per staging round of the im2col tile, one
// pair of barriers per round.  The next chunk's halo and filter slice are loaded into registers while
// the current one computes (the direct kernel's pattern, conv.hip conv_direct_kernel).
//
// GEMM view (as conv_nt_kernel): m = (line, position), k = (tap, channel), B = the filter rows
// [N][T][Cs] (forward: W in KRSC; backward-data: Wt = W^T [C][R][S][Co] with the taps flipped through
// g.sign = -1).  Source coordinate along the line = o + off + sign * t (igemm.h Gather).
#include <algorithm>

#include "igemm.h"

using namespace tony;
using namespace tony::mfma;
using namespace tony::glds;

namespace {

constexpr int kBandThreads = 512;  // 8 waves: 4 along M (64 rows each) x 2 along N
constexpr int kKC = 32;            // channels per K chunk (one MFMA K slice per tap)
constexpr int kAP = kKC + 16;      // LDS elements per halo pixel (32-B pad: conflict-free ds_read_b128 groups)
constexpr int kBM = 256;           // GEMM rows per workgroup (L lines x wd positions, the rest padding)
constexpr int kMaxHaloPx = 512;    // L x (wd + T - 1) <= this (4 chunks per thread)
constexpr int kNA = kMaxHaloPx * (kKC / 8) / kBandThreads;

struct BandArgs {
  const uint16_t* src;
  int64_t ld;          // source elements per pixel
  const uint16_t* B;   // [N][T][Cs]
  uint16_t* C;
  int64_t ldc;         // output elements per pixel
  float* stats;        // [sum | sumsq] of the output per channel (nullable)
  int64_t sstride;
  int N, Cs;
  int lines, per_img;  // total lines, lines per image
  int wd, hp, L;       // output positions per line, halo positions per line, lines per tile
  int h0;              // source position of halo position 0
  int win;             // source positions per line
  int64_t s_img, s_line, s_pos;  // source element strides: image, line within an image, position
  int64_t o_img, o_line, o_pos;  // output element strides
  int sign;
  int ntn;             // N tiles
};

template <int T, int BN>
__global__ __launch_bounds__(kBandThreads) void conv_band_kernel(BandArgs a) {
  constexpr int BP = T * kKC + 16;  // LDS elements per filter row (32-B pad)
  constexpr int TN = BN / 32;       // 16-wide column blocks per wave (2 waves along N)
  constexpr int NB = (BN * T * (kKC / 8) + kBandThreads - 1) / kBandThreads;
  extern __shared__ __attribute__((aligned(16))) uint16_t bsm[];
  const int hpx = a.L * a.hp;  // halo pixels of this tile's lines (<= kMaxHaloPx, checked by the host)
  uint16_t* ha = bsm;              // halo: [L * hp][kAP]
  uint16_t* hb = bsm + hpx * kAP;  // filter slice: [BN][BP] (96-B pixel pitch: 16-B aligned)

  const int tn = blockIdx.x % a.ntn;
  const int tm = blockIdx.x / a.ntn;
  const int line0 = tm * a.L, n0 = tn * BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave & 3, wn = wave >> 2;
  const int kq = lane >> 4;

  // per-thread A chunks (tile-invariant parts): halo pixel -> source element offset of its line base and
  // position; -1 = zero (outside the line or past the last line)
  int64_t asrc[kNA];
  int adst[kNA];
#pragma unroll
  for (int i = 0; i < kNA; ++i) {
    const int v = i * kBandThreads + threadIdx.x;
    const int px = v >> 2, c8 = v & 3;
    asrc[i] = -1;
    adst[i] = -1;
    if (px < hpx) {
      const int ln = px / a.hp, p = px - ln * a.hp;
      const int gl = line0 + ln, sp = a.h0 + p;
      adst[i] = px * kAP + c8 * 8;
      if (gl < a.lines && static_cast<unsigned>(sp) < static_cast<unsigned>(a.win)) {
        const int img = gl / a.per_img, li = gl - img * a.per_img;
        asrc[i] = img * a.s_img + li * a.s_line + sp * a.s_pos + c8 * 8;
      }
    }
  }
  // per-thread B chunks: filter row n0 + row, tap t, 8 channels c8 of the chunk
  int64_t bsrc[NB];
  int bdst[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int v = i * kBandThreads + threadIdx.x;
    const int row = v / (T * 4), rem = v - row * (T * 4);
    const int t = rem >> 2, c8 = rem & 3;
    bsrc[i] = -1;
    bdst[i] = -1;
    if (row < BN) {
      bdst[i] = row * BP + t * kKC + c8 * 8;
      if (n0 + row < a.N) bsrc[i] = static_cast<int64_t>(n0 + row) * T * a.Cs + t * a.Cs + c8 * 8;
    }
  }
  uint4 ra[kNA], rb[NB];
  auto fetch = [&](int c0) {  // chunk c0's halo and filter slice into registers
#pragma unroll
    for (int i = 0; i < kNA; ++i)
      ra[i] = asrc[i] >= 0 ? *reinterpret_cast<const uint4*>(a.src + asrc[i] + c0) : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int i = 0; i < NB; ++i)
      rb[i] = bsrc[i] >= 0 ? *reinterpret_cast<const uint4*>(a.B + bsrc[i] + c0) : make_uint4(0u, 0u, 0u, 0u);
  };
  auto stage = [&]() {
#pragma unroll
    for (int i = 0; i < kNA; ++i)
      if (adst[i] >= 0) *reinterpret_cast<uint4*>(ha + adst[i]) = ra[i];
#pragma unroll
    for (int i = 0; i < NB; ++i)
      if (bdst[i] >= 0) *reinterpret_cast<uint4*>(hb + bdst[i]) = rb[i];
  };

  // this lane's A rows: halo pixel of (line, position) at tap 0 (rows past the tile's lines read line 0:
  // finite garbage, masked in the epilogue)
  int abase[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = wm * 64 + i * 16 + (lane & 15);
    const int ln = m / a.wd, p = m - ln * a.wd;
    abase[i] = (m < a.L * a.wd ? ln * a.hp + p : 0) * kAP + kq * 8;
  }
  f32x4 acc[4][TN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = a.Cs / kKC;
  fetch(0);
  for (int ch = 0; ch < nchunks; ++ch) {
    __syncthreads();  // every wave is done with the previous chunk
    stage();
    __syncthreads();
    if (ch + 1 < nchunks) fetch((ch + 1) * kKC);  // in flight during the MFMAs
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int tt = a.sign > 0 ? t : T - 1 - t;  // halo shift of tap t
      bf16x8_t af[4], bfr[TN];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8_t*>(ha + abase[i] + tt * kAP);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(hb + (wn * (BN / 2) + j * 16 + (lane & 15)) * BP + t * kKC + kq * 8);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  // epilogue: valid rows are positions of real lines of this tile
  bool rv[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int m = wm * 64 + i * 16 + kq * 4 + q;
      rv[i][q] = m < a.L * a.wd && line0 + m / a.wd < a.lines;
    }
  if (a.stats != nullptr) {
    float* st = a.stats + shard_off(blockIdx.x, a.sstride);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * (BN / 2) + j * 16 + (lane & 15);
      float sm = 0.f, sq = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float v = rv[i][q] ? acc[i][j][q] : 0.f;
          sm += v;
          sq = fmaf(v, v, sq);
        }
      sm += __shfl_xor(sm, 16, 64);
      sm += __shfl_xor(sm, 32, 64);
      sq += __shfl_xor(sq, 16, 64);
      sq += __shfl_xor(sq, 32, 64);
      if (lane < 16 && col < a.N) {
        atomicAdd(st + col, sm);
        atomicAdd(st + a.N + col, sq);
      }
    }
  }
  __syncthreads();  // halo and filter slice are dead: they become the C staging tile
  constexpr int LDC = BN + 8;
  uint16_t* cs = bsm;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        cs[(wm * 64 + i * 16 + kq * 4 + q) * LDC + wn * (BN / 2) + j * 16 + (lane & 15)] = f2bf(acc[i][j][q]);
  __syncthreads();
  for (int v = threadIdx.x; v < kBM * (BN / 8); v += kBandThreads) {
    const int m = v / (BN / 8), c8 = v - m * (BN / 8);
    if (m >= a.L * a.wd || n0 + c8 * 8 >= a.N) continue;
    const int ln = m / a.wd, p = m - ln * a.wd;
    const int gl = line0 + ln;
    if (gl >= a.lines) continue;
    const int img = gl / a.per_img, li = gl - img * a.per_img;
    uint16_t* dst = a.C + img * a.o_img + li * a.o_line + p * a.o_pos + n0 + c8 * 8;
    *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(cs + m * LDC + c8 * 8);
  }
}

template <int T, int BN>
int launch_band(const BandArgs& a, int grid, hipStream_t stream) {
  constexpr size_t kMaxLds = (static_cast<size_t>(kMaxHaloPx) * kAP + static_cast<size_t>(BN) * (T * kKC + 16)) * 2;
  static_assert(kMaxLds <= 163840, "LDS");
  // this launch's halo + filter slice, at least the C staging tile (2-3 workgroups per CU on 17x17 / 8x8)
  const size_t lds = std::max((static_cast<size_t>(a.L) * a.hp * kAP + static_cast<size_t>(BN) * (T * kKC + 16)) * 2,
                              static_cast<size_t>(kBM) * (BN + 8) * 2);
  const void* fn = reinterpret_cast<const void*>(&conv_band_kernel<T, BN>);
  static int ok = 0;  // per instance: the dynamic-LDS attribute set
  if (ok == 0)
    ok = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kMaxLds)) == hipSuccess
             ? 1
             : -1;
  if (ok < 0 || lds > kMaxLds) return -3;
  conv_band_kernel<T, BN><<<grid, kBandThreads, lds, stream>>>(a);
  TONY_LAUNCH_CHECK();
  return 0;
}

}  // namespace

namespace tony {

// The band kernel for this conv (forward or backward-data, bf16 output, optional BN statistics), or -3
// when the shape / epilogue is not one it takes (the caller's tuner skips it then).
int run_band(const Gather& g, const void* B, void* C, int64_t ldc, int64_t N, int epi, float* st, int64_t sstride,
             hipStream_t stream) {
  if ((epi & ~1) || ((epi & 1) && st == nullptr) || g.sh != 1 || g.sw != 1 || (g.Cs % kKC) || (g.ld % 8) ||
      (ldc % 8) || N <= 0 || N > 0x7fffffff || g.halo_images <= 0 || (reinterpret_cast<uintptr_t>(C) & 15) ||
      (reinterpret_cast<uintptr_t>(B) & 15) || (reinterpret_cast<uintptr_t>(g.src) & 15))
    return -3;
  const bool along_w = g.R == 1 && g.S > 1;
  const bool along_h = g.S == 1 && g.R > 1;
  if (!along_w && !along_h) return -3;
  const int T = along_w ? g.S : g.R;
  if (T != 3 && T != 7) return -3;
  BandArgs a{};
  a.src = static_cast<const uint16_t*>(g.src);
  a.ld = g.ld;
  a.B = static_cast<const uint16_t*>(B);
  a.C = static_cast<uint16_t*>(C);
  a.ldc = ldc;
  a.stats = (epi & 1) ? st : nullptr;
  a.sstride = sstride;
  a.N = static_cast<int>(N);
  a.Cs = g.Cs;
  a.sign = g.sign;
  a.s_img = static_cast<int64_t>(g.Hs) * g.Ws * g.ld;
  a.o_img = static_cast<int64_t>(g.OH) * g.OW * ldc;
  if (along_w) {  // lines = image rows; the filter has one row, so no offset along H
    if (g.offh != 0 || g.Hs != g.OH) return -3;
    a.per_img = g.OH;
    a.wd = g.OW;
    a.win = g.Ws;
    a.h0 = g.offw + (g.sign < 0 ? -(T - 1) : 0);
    a.s_line = static_cast<int64_t>(g.Ws) * g.ld;
    a.s_pos = g.ld;
    a.o_line = static_cast<int64_t>(g.OW) * ldc;
    a.o_pos = ldc;
  } else {  // lines = image columns
    if (g.offw != 0 || g.Ws != g.OW) return -3;
    a.per_img = g.OW;
    a.wd = g.OH;
    a.win = g.Hs;
    a.h0 = g.offh + (g.sign < 0 ? -(T - 1) : 0);
    a.s_line = g.ld;
    a.s_pos = static_cast<int64_t>(g.Ws) * g.ld;
    a.o_line = ldc;
    a.o_pos = static_cast<int64_t>(g.OW) * ldc;
  }
  // every source position a tap reads must lie in [h0, h0 + hp): stride 1, so o + off + sign*t spans it
  a.hp = a.wd + T - 1;
  a.L = kBM / a.wd;
  if (a.L < 1 || a.L * a.hp > kMaxHaloPx) return -3;
  const int64_t lines = static_cast<int64_t>(g.halo_images) * a.per_img;
  if (lines > 0x7fffffff) return -2;
  a.lines = static_cast<int>(lines);
  const int bn = (N % 96 == 0) ? 96 : 64;
  a.ntn = static_cast<int>((N + bn - 1) / bn);
  const int64_t grid = (lines + a.L - 1) / a.L * a.ntn;
  if (grid > 0x7fffffff) return -2;
  if (T == 7) return bn == 96 ? launch_band<7, 96>(a, static_cast<int>(grid), stream)
                              : launch_band<7, 64>(a, static_cast<int>(grid), stream);
  return bn == 96 ? launch_band<3, 96>(a, static_cast<int>(grid), stream)
                  : launch_band<3, 64>(a, static_cast<int>(grid), stream);
}

}  // namespace tony
