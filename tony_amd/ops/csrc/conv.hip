// Implicit-GEMM NHWC convolutions on MFMA, bf16 in, fp32 accumulate.
//
// Forward   Y[m, co] = sum_k A[m, k] W[co, k],  m = (n, oy, ox), k = (r, s, ci)
//           A[m, k]  = X[n, oy*sh - ph + r, ox*sw - pw + s, ci]   (zero outside the image)
// Dgrad     dX[m, ci] = sum_k dY[n, iy + ph - r, ix + pw - s, co] Wt[ci, k], k = (r, s, co)
//           (stride 1; Wt = W permuted to [Ci][R][S][Co])
// Wgrad     dW[co, k] = sum_m dY[m, co] A[m, k]                   (split-K over m, fp32 atomics)
//
// The GEMM cores are those of gemm.hip (256 threads = 2x2 wave64s, 16x16x32 bf16 MFMA, BK = 64,
// register-staged double-buffered LDS with an XOR swizzle, XCD-aware tile order, BN statistics
// in the forward epilogue); only the operand that is an image changes: instead of a row-major
// matrix it is gathered on the fly ("im2col in the loader").  With Cin % 8 == 0 every 16-byte
// chunk of a K row is 8 channels of ONE filter tap, so each chunk is one aligned 16-byte load
// from one input pixel (or zero for padding).  The tap/channel position of a thread's chunk is
// advanced incrementally per K-step (no divisions in the loop); the per-row pixel coordinates are
// decoded once per tile (forward/dgrad) or advanced incrementally with the row (wgrad).
#include <atomic>
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "igemm.h"

using namespace tony;
using namespace tony::mfma;
using namespace tony::glds;

namespace tony {
// band.hip: the 1 x T / T x 1 stride-1 convs (forward / backward-data) on whole-line halo tiles
int run_band(const Gather& g, const void* B, void* C, int64_t ldc, int64_t N, int epi, float* st, int64_t sstride,
             hipStream_t stream);
}  // namespace tony

namespace {

__device__ __forceinline__ uint4 gather16(const Gather& g, const RowState& rs, const TapPos& t, int toff) {
  const int iy = rs.iy0 + g.sign * t.r, ix = rs.ix0 + g.sign * t.s;
  if (rs.ok && t.r < g.R && static_cast<unsigned>(iy) < static_cast<unsigned>(g.Hs) &&
      static_cast<unsigned>(ix) < static_cast<unsigned>(g.Ws))
    return *reinterpret_cast<const uint4*>(rs.base + toff);  // toff = t.off(g)
  return make_uint4(0, 0, 0, 0);
}

template <int ROWS>
__device__ __forceinline__ void load_rows(uint4* regs, const uint16_t* __restrict__ G, int64_t ld, int row0, int nrows,
                                          int k0, int K) {
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
__device__ __forceinline__ void store_rows(uint16_t* lds, const uint4* regs) {
  constexpr int VEC = ROWS * BK / 8 / kThreads;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const int v = threadIdx.x + i * kThreads;
    const int row = v >> 3, ch = v & 7;
    *reinterpret_cast<uint4*>(lds + lds_off(row, ch)) = regs[i];
  }
}

// One residue class of a strided backward-data conv (tony_conv_dgrad_strided): the dX pixels
// (iy, ix) with iy % sh == py, ix % sw == px only receive the filter taps r = r0 + sh*a,
// s = s0 + sw*b, so they form a stride-1 transposed conv over the class's sub-grid with that
// reduced filter.  The A operand is the usual flipped-tap gather of dY (Gather over the taps (a, b));
// B rows are read straight out of the full transposed filter Wt [Ci][R][S][Co] at the class's taps
// (no per-class weight copies), and the epilogue scatters GEMM rows back to the class's pixels.
// BatchNorm-backward reduction fused into a backward-data epilogue.  The dgrad of conv L+1 produces
// dY_L, the output gradient of layer L's BN(+ReLU), whose backward first reduces
//   dsum[c] = sum dY', dsumx[c] = sum dY' * xhat,  xhat = (Z - mean) * invstd,
//   dY' = dY masked by ReLU(gamma * xhat + beta) > 0 (relu)
// over every pixel (csrc/bn_act.hip bn_bwd_reduce_kernel).  When layer L's output feeds ONLY conv
// L+1, the dgrad epilogue has every dY tile at hand: it reads the matching Z tile, accumulates the two
// sums (from the bf16-rounded dY it stores, as the reduce kernel would read it) and adds them into
// the sharded [dsum | dsumx] buffer -- the separate 2-pass reduce over Z and dY disappears.
struct BnRed {
  const uint16_t* z = nullptr;  // Z of layer L (rows = the dgrad's output pixels), nullptr = off
  int64_t ldz = 0;
  const float* mean = nullptr;
  const float* invstd = nullptr;
  const void* gamma = nullptr;
  const void* beta = nullptr;
  int pb = 0;                   // gamma / beta are bf16
  int relu = 0;
  float* dsum = nullptr;        // [dsum C | dsumx C], kStatShards copies sstride floats apart (zeroed)
  int64_t sstride = 0;
  int done = 0;                 // host side: set by the launcher when the chosen kernel reduced
};

__device__ __forceinline__ float bnr_param(const void* p, int c, int pb, float dflt) {
  if (p == nullptr) return dflt;
  return pb ? bf2f(static_cast<const uint16_t*>(p)[c]) : static_cast<const float*>(p)[c];
}

// per-channel (xhat = z*p0 + p1, pre-activation = z*p2 + p3) of channel c
__device__ __forceinline__ void bnr_coef(const BnRed& br, int c, float& p0, float& p1, float& p2, float& p3) {
  const float mu = br.mean[c], is = br.invstd[c];
  const float g = bnr_param(br.gamma, c, br.pb, 1.f), be = bnr_param(br.beta, c, br.pb, 0.f);
  p0 = is;
  p1 = -mu * is;
  p2 = g * is;
  p3 = be - g * is * mu;
}

struct Phase {
  int R, S;      // taps of the full filter: Wt row layout [R][S][Co]
  int r0, s0;    // the class's first tap
  int tsy, tsx;  // tap step (= conv stride)
  RowMap rows;   // GEMM row -> dX pixel
  BnRed bnr;     // fused BN-backward reduction of the dgrad output (any dgrad, strided or not)
};

// The BN-backward reduction over a finished NT-epilogue tile (bf16 dY in Cs, rows x BN, row pitch
// BN + 8): thread t owns 8 channels (t % (BN/8)) of every (256/(BN/8))-th row, its partial sums meet
// in LDS behind the C tile, one sharded atomic per column and workgroup.
template <int BM, int BN>
__device__ void bnred_tile(const uint16_t* Cs, float* red, int M, int N, int m0, int n0, const RowMap& rm,
                           const BnRed& br, int shard) {
  constexpr int LDC = BN + 8, NCH = BN / 8, RSTEP = kThreads / NCH;
  const int ch = threadIdx.x % NCH, rsub = threadIdx.x / NCH;
  const int gcol = n0 + ch * 8;
  float a[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = b[j] = 0.f;
  if (rsub < RSTEP && gcol < N) {
    float p0[8], p1[8], p2[8], p3[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) bnr_coef(br, gcol + j, p0[j], p1[j], p2[j], p3[j]);
    for (int row = rsub; row < BM && m0 + row < M; row += RSTEP) {
      float d[8], z[8];
      bf16x8 dv, zv;
      dv.raw = *reinterpret_cast<const uint4*>(Cs + row * LDC + ch * 8);
      zv.raw = *reinterpret_cast<const uint4*>(br.z + rm.pixel(m0 + row) * br.ldz + gcol);
      dv.to_float(d);
      zv.to_float(z);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = (br.relu && fmaf(z[j], p2[j], p3[j]) <= 0.f) ? 0.f : d[j];
        a[j] += v;
        b[j] = fmaf(v, fmaf(z[j], p0[j], p1[j]), b[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[j * kThreads + threadIdx.x] = a[j];
    red[(8 + j) * kThreads + threadIdx.x] = b[j];
  }
  __syncthreads();
  float* ds = br.dsum + shard_off(shard, br.sstride);
  for (int q = threadIdx.x; q < 2 * BN; q += kThreads) {
    const int which = q / BN, c = q - which * BN;
    if (n0 + c >= N) continue;
    const int cg = c / 8, j = c % 8;
    float sum = 0.f;
    for (int r = 0; r < RSTEP; ++r) sum += red[(which * 8 + j) * kThreads + r * NCH + cg];
    atomicAdd(ds + which * N + n0 + c, sum);
  }
}

// B rows [row0, row0 + ROWS) x this thread's K chunk, where the K position is the thread's A tap
// (the A and B chunk columns of conv_nt_kernel coincide: both are threadIdx.x & 7)
template <int ROWS>
__device__ __forceinline__ void load_rows_phase(uint4* regs, const uint16_t* __restrict__ B, const Phase& ph,
                                                const Gather& g, const TapPos& t, int row0, int nrows) {
  constexpr int VEC = ROWS * BK / 8 / kThreads;
  // 32-bit offsets (the filter has far fewer than 2^31 elements): no 64-bit products per K-step
  const int ldb = ph.R * ph.S * g.Cs;
  const int koff = ((ph.r0 + ph.tsy * t.r) * ph.S + ph.s0 + ph.tsx * t.s) * g.Cs + t.c;
  const bool kok = t.r < g.R;
  const uint16_t* Bk = B + koff;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const int gr = row0 + ((threadIdx.x + i * kThreads) >> 3);
    if (kok && gr < nrows)
      regs[i] = *reinterpret_cast<const uint4*>(Bk + gr * ldb);
    else
      regs[i] = make_uint4(0, 0, 0, 0);
  }
}

// C[M, N] = gather(A)[M, K] * B[N, K]^T  (forward and stride-1 dgrad; PH: one class of a strided dgrad)
template <int BM, int BN, bool PH = false>
__global__ __launch_bounds__(kThreads) void conv_nt_kernel(Gather g, const uint16_t* __restrict__ B,
                                                           uint16_t* __restrict__ C, int64_t ldc, int M, int N,
                                                           float* __restrict__ stats, int64_t sstride,
                                                           int epi, int tiles_n, Phase ph) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int AV = BM * BK / 8 / kThreads, BV = BN * BK / 8 / kThreads;
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * (BM + BN) * BK];

  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = wg / tiles_n, tn = wg % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int K = g.K;

  // rows of the A tile this thread loads: (tid >> 3) + 32 i ; its chunk column: tid & 7
  RowState rs[AV];
  const int ohw = g.OH * g.OW;
#pragma unroll
  for (int i = 0; i < AV; ++i) {
    const int m = m0 + (threadIdx.x >> 3) + i * (kThreads / 8);
    rs[i].ok = m < M;
    const int mm = rs[i].ok ? m : 0;
    const int n = mm / ohw, rem = mm - n * ohw;
    const int oy = rem / g.OW, ox = rem - oy * g.OW;
    rs[i].pix = n * g.Hs * g.Ws;
    rs[i].iy0 = oy * g.sh + g.offh;
    rs[i].ix0 = ox * g.sw + g.offw;
    rs[i].set_base(g);
  }
  TapPos tp;
  tp.init((threadIdx.x & 7) * 8, g);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[AV], rb[BV];
  const int nk = (K + BK - 1) / BK;
  {
    const int toff = tp.off(g);
#pragma unroll
    for (int i = 0; i < AV; ++i) ra[i] = gather16(g, rs[i], tp, toff);
  }
  if constexpr (PH)
    load_rows_phase<BN>(rb, B, ph, g, tp, n0, N);
  else
    load_rows<BN>(rb, B, K, n0, N, 0, K);
  store_rows<BM>(smem, ra);
  store_rows<BN>(smem + BM * BK, rb);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    uint16_t* As = smem + (kt & 1) * (BM + BN) * BK;
    uint16_t* Bs = As + BM * BK;
    const bool more = kt + 1 < nk;
    if (more) {
      tp.advance(BK, g);
      const int toff = tp.off(g);
#pragma unroll
      for (int i = 0; i < AV; ++i) ra[i] = gather16(g, rs[i], tp, toff);
      if constexpr (PH)
        load_rows_phase<BN>(rb, B, ph, g, tp, n0, N);
      else
        load_rows<BN>(rb, B, K, n0, N, (kt + 1) * BK, K);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8_t*>(As + lds_off(wm * WM + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8_t*>(Bs + lds_off(wn * WN + j * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      uint16_t* An = smem + ((kt + 1) & 1) * (BM + BN) * BK;
      store_rows<BM>(An, ra);
      store_rows<BN>(An + BM * BK, rb);
    }
    __syncthreads();
  }
  // epi bit0: BN statistics into stats (sharded); bit1: stats holds [scale | shift] for the folded
  // inference BN (H5), bit2: ReLU after it
  nt_epilogue<BM, BN, TM, TN>(acc, smem, C, ldc, M, N, m0, n0,
                               (epi & 1) ? stats + shard_off(tm, sstride) : nullptr,
                               (epi & 2) ? stats : nullptr, (epi & 4) != 0, PH ? ph.rows : RowMap{}, (epi & 8) != 0,
                               (epi & 16) != 0);
  if (ph.bnr.z != nullptr) {  // uniform: the C tile is still in LDS, the fold area lies behind it
    constexpr int CS_ELEMS = (BM * (BN + 8) + 7) / 8 * 8;
    static_assert(CS_ELEMS * 2 + 16 * kThreads * 4 <= 2 * (BM + BN) * BK * 2, "BN-reduce fold area fits");
    bnred_tile<BM, BN>(smem, reinterpret_cast<float*>(smem + CS_ELEMS), M, N, m0, n0, PH ? ph.rows : RowMap{},
                       ph.bnr, tm);
  }
}

template <int BM, int BN, bool PH>
int launch_nt(const Gather& g, const void* B, void* C, int64_t ldc, int64_t M, int64_t N, float* stats,
              int64_t sstride, int epi, const Phase& ph, hipStream_t stream) {
  const int tiles_m = ceil_div(M, BM), tiles_n = ceil_div(N, BN);
  const int64_t tiles = static_cast<int64_t>(tiles_m) * tiles_n;
  if (tiles > 0x7fffffff) return -2;
  conv_nt_kernel<BM, BN, PH><<<static_cast<int>(tiles), kThreads, 0, stream>>>(
      g, static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C), ldc, static_cast<int>(M), static_cast<int>(N),
      stats, sstride, epi, tiles_n, ph);
  TONY_LAUNCH_CHECK();
  return 0;
}

template <int BM, bool PH = false>
int launch_nt_bm(const Gather& g, const void* B, void* C, int64_t ldc, int64_t M, int64_t N, float* st,
                 int64_t sstride, int epi, int64_t bn, hipStream_t stream, const Phase& ph = Phase{}) {
  if constexpr (BM == 256) {  // 8 x TN accumulators per wave: only narrow column tiles fit the registers
    if (bn <= 32) return launch_nt<256, 32, PH>(g, B, C, ldc, M, N, st, sstride, epi, ph, stream);
    if (bn <= 64) return launch_nt<256, 64, PH>(g, B, C, ldc, M, N, st, sstride, epi, ph, stream);
    return -3;
  } else {
    switch (bn) {
      case 32: return launch_nt<BM, 32, PH>(g, B, C, ldc, M, N, st, sstride, epi, ph, stream);
      case 64: return launch_nt<BM, 64, PH>(g, B, C, ldc, M, N, st, sstride, epi, ph, stream);
      case 96: return launch_nt<BM, 96, PH>(g, B, C, ldc, M, N, st, sstride, epi, ph, stream);
      case 128: return launch_nt<BM, 128, PH>(g, B, C, ldc, M, N, st, sstride, epi, ph, stream);
      case 160: return launch_nt<BM, 160, PH>(g, B, C, ldc, M, N, st, sstride, epi, ph, stream);
      default: return launch_nt<BM, 192, PH>(g, B, C, ldc, M, N, st, sstride, epi, ph, stream);
    }
  }
}

// ---- 3x3 stride-1 convs with few channels (Cin 32 / 64): halo tiles instead of im2col -----------
// The im2col loader of conv_nt_kernel fetches every input pixel 9 times (once per tap) through
// L2; for Cin = 32/64 (Inception's 147x147 stem layers, ResNet's 56x56 layers, and their dgrads)
// that gather, not the MFMAs, bounds the kernel.  Here a workgroup computes a 2-D block of
// HT x WT = 8 x 16 output pixels (128 GEMM rows) x BN output channels: it loads the (HT+2) x (WT+2)
// input patch once into LDS (zeros outside the image), the BN x 9*Cin weight panel once, and reads
// the MFMA A fragments straight out of the patch at the 9 tap offsets.  LDS pixel rows and weight
// rows are padded by 32 B: with ds_read_b128's lane groups ({0-3,12-15,20-27}, ...) that is the
// smallest pad for which every group's 16 addresses hit distinct 4-bank sets (a 16-B pad measured
// SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = 38 %).
// Same GEMM view as conv_nt_kernel (m = (n, oy, ox), k = (r, s, c)); the dgrad is the same kernel
// on dY with flipped taps (g.sign = -1) and the transposed weights.
constexpr int kHaloH = 8, kHaloW = 16;  // 16 x 16 measured no faster (one-shot load phase dominates)
constexpr int kHaloVariant = 9;  // tile-variant id the autotuner uses for this path (ops/tune.py)

template <int CS, int BN>
__global__ __launch_bounds__(kThreads) void conv_halo_kernel(Gather g, const uint16_t* __restrict__ B,
                                                            uint16_t* __restrict__ C, int64_t ldc, int N,
                                                            float* __restrict__ stats, int64_t sstride, int epi,
                                                            int tiles_x, int tiles_y) {
  constexpr int R = 3, S = 3;
  constexpr int HH = kHaloH + R - 1, HW = kHaloW + S - 1;
  constexpr int PSTR = CS + 16;                // LDS elements per halo pixel (32-B pad)
  constexpr int KK = R * S * CS;               // GEMM K
  constexpr int KP = KK + 16;                  // LDS elements per weight row (32-B pad)
  constexpr int HALO = HH * HW * PSTR;
  constexpr int WTS = BN * KP;
  constexpr int BM = kHaloH * kHaloW;          // 128 rows
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int LDC = BN + 8;
  static_assert(BM * LDC <= HALO + WTS, "the C staging tile reuses the patch + weight panel");
  __shared__ __attribute__((aligned(16))) uint16_t smem[HALO + WTS];
  uint16_t* halo = smem;
  uint16_t* wts = smem + HALO;

  // block -> (n, tile y, tile x, column tile); consecutive blocks share an image row band
  int b = blockIdx.x;
  const int ntn = N / BN;
  const int tn = b % ntn;
  b /= ntn;
  const int tx = b % tiles_x;
  b /= tiles_x;
  const int ty = b % tiles_y;
  const int n = b / tiles_y;
  const int oy0 = ty * kHaloH, ox0 = tx * kHaloW, n0 = tn * BN;
  const int hy0 = oy0 + g.offh - (g.sign < 0 ? R - 1 : 0);
  const int hx0 = ox0 + g.offw - (g.sign < 0 ? S - 1 : 0);
  const int64_t pix0 = static_cast<int64_t>(n) * g.Hs * g.Ws;

  // stage the input patch and the weight panel (all loads in flight together, one barrier)
  constexpr int HCH = HH * HW * (CS / 8);
  for (int v = threadIdx.x; v < HCH; v += kThreads) {
    const int c8 = v % (CS / 8), px = v / (CS / 8);
    const int hy = px / HW, hx = px - hy * HW;
    const int iy = hy0 + hy, ix = hx0 + hx;
    uint4 val = make_uint4(0, 0, 0, 0);
    if (static_cast<unsigned>(iy) < static_cast<unsigned>(g.Hs) && static_cast<unsigned>(ix) < static_cast<unsigned>(g.Ws))
      val = *reinterpret_cast<const uint4*>(g.src + (pix0 + iy * g.Ws + ix) * g.ld + c8 * 8);
    *reinterpret_cast<uint4*>(halo + px * PSTR + c8 * 8) = val;
  }
  constexpr int WCH = BN * (KK / 8);
  for (int v = threadIdx.x; v < WCH; v += kThreads) {
    const int k8 = v % (KK / 8), row = v / (KK / 8);
    *reinterpret_cast<uint4*>(wts + row * KP + k8 * 8) =
        *reinterpret_cast<const uint4*>(B + static_cast<int64_t>(n0 + row) * KK + k8 * 8);
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int kq = lane >> 4;  // which 8-element quarter of a 32-deep K slice this lane holds
  int abase[TM];             // halo pixel of this lane's A row, tap (0, 0)
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rl = wm * WM + i * 16 + (lane & 15);
    abase[i] = ((rl / kHaloW) * HW + (rl % kHaloW)) * PSTR + kq * 8;
  }
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int s2 = 0; s2 < S; ++s2) {
      const int rr = g.sign > 0 ? r : R - 1 - r, ss = g.sign > 0 ? s2 : S - 1 - s2;
      const int aoff = (rr * HW + ss) * PSTR;
#pragma unroll
      for (int cb = 0; cb < CS / 32; ++cb) {
        const int k0 = (r * S + s2) * CS + cb * 32 + kq * 8;
        bf16x8_t af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8_t*>(halo + abase[i] + aoff + cb * 32);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8_t*>(wts + (wn * WN + j * 16 + (lane & 15)) * KP + k0);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  }

  // epilogue: rows outside the output image (partial edge blocks) hold real sums of halo data, so
  // they are masked out of the statistics and the stores
  bool rv[TM][4];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rl = wm * WM + i * 16 + (lane >> 4) * 4 + q;
      rv[i][q] = (oy0 + rl / kHaloW < g.OH) & (ox0 + rl % kHaloW < g.OW);
    }
  if ((epi & 1) && stats != nullptr) {
    float* st = stats + shard_off(blockIdx.x, sstride);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * WN + j * 16 + (lane & 15);
      float sm = 0.f, sq = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
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
      if (lane < 16) {
        atomicAdd(st + col, sm);
        atomicAdd(st + N + col, sq);
      }
    }
  }
  __syncthreads();  // everyone is done with patch and weights: they become the C staging tile
  uint16_t* Cs = smem;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = wm * WM + i * 16 + (lane >> 4) * 4 + q;
        const int col = wn * WN + j * 16 + (lane & 15);
        Cs[row * LDC + col] = f2bf(acc[i][j][q]);
      }
  __syncthreads();
  for (int v = threadIdx.x; v < BM * (BN / 8); v += kThreads) {
    const int row = v / (BN / 8), ch = v % (BN / 8);
    const int oy = oy0 + row / kHaloW, ox = ox0 + row % kHaloW;
    if (oy >= g.OH || ox >= g.OW) continue;
    uint16_t* dst = C + ((static_cast<int64_t>(n) * g.OH + oy) * g.OW + ox) * ldc + n0 + ch * 8;
    *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(Cs + row * LDC + ch * 8);
  }
}

// The halo kernel for this shape, or -3 when it does not apply (caller falls back to a tile variant).
int run_halo(const Gather& g, const void* B, void* C, int64_t ldc, int64_t N, int epi, float* st, int64_t sstride,
             hipStream_t stream) {
  if (g.R != 3 || g.S != 3 || g.sh != 1 || g.sw != 1 || (epi & 6) || (ldc % 8) ||
      (reinterpret_cast<uintptr_t>(C) & 15) || (reinterpret_cast<uintptr_t>(B) & 15))
    return -3;
  const int tiles_x = ceil_div(g.OW, kHaloW), tiles_y = ceil_div(g.OH, kHaloH);
  const auto launch = [&](auto cs, auto bn, int64_t images) -> int {
    constexpr int CS = decltype(cs)::value, BN = decltype(bn)::value;
    const int64_t grid = images * tiles_y * tiles_x * (N / BN);
    if (grid > 0x7fffffff) return -2;
    conv_halo_kernel<CS, BN><<<static_cast<int>(grid), kThreads, 0, stream>>>(
        g, static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C), ldc, static_cast<int>(N), st, sstride, epi,
        tiles_x, tiles_y);
    TONY_LAUNCH_CHECK();
    return 0;
  };
  const int64_t images = g.halo_images;
  if (images <= 0) return -3;
  if (g.Cs == 32 && N % 64 == 0) return launch(std::integral_constant<int, 32>{}, std::integral_constant<int, 64>{}, images);
  if (g.Cs == 32 && N % 32 == 0) return launch(std::integral_constant<int, 32>{}, std::integral_constant<int, 32>{}, images);
  if (g.Cs == 64 && N % 32 == 0) return launch(std::integral_constant<int, 64>{}, std::integral_constant<int, 32>{}, images);
  return -3;
}

// ---- 3x3 stride-1 convs with 32 / 64 channels on both sides: persistent direct kernel ---------
// Inception's 149x149 / 147x147 stem layers (and their dgrads, ResNet's 56x56 3x3s) move ~0.2-0.5
// GB each for 50-100 GFLOP: they must run at HBM speed.  The halo kernel above re-stages the weight
// panel for every 8x16 tile and serialises load -> barrier -> MFMA -> epilogue inside each
// workgroup, so it is latency bound (~300 TF/s).  Here a persistent workgroup
//   * stages the [CO][9*CS] weight panel in LDS ONCE,
//   * walks 8 x TW output tiles (b, b + grid, ...), the NEXT tile's (8+2) x (TW+2) input halo in
//     flight in registers while the current one computes (one LDS write + two barriers per tile),
//   * computes D[co][px] = W . X^T (weights = MFMA A operand, halo pixels = B operand), so each lane
//     ends with 4 consecutive channels of one pixel and stores them straight to global memory (8 B):
//     no LDS staging of the output and no barrier in the epilogue,
//   * keeps the BN statistics in registers over all its tiles (one sharded atomic per channel).
constexpr int kDirectVariant = 10;  // tile-variant id the autotuner uses for this path (ops/tune.py)
constexpr int kBandVariant = 40;    // band.hip run_band (ops/tune.py BAND_CODE)
constexpr int kDirH = 8;

template <int CS, int CO, int TW>
struct DirectCfg {
  static constexpr int R = 3, S = 3, TH = kDirH;
  static constexpr int HH = TH + R - 1, HW = TW + S - 1;
  static constexpr int PSTR = CS + 16;  // halo pixel pitch: 32-B pad, conflict-free ds_read_b128 groups
  static constexpr int K = R * S * CS;
  static constexpr int KP = K + 16;     // weight row pitch
  static constexpr int HALO = HH * HW * PSTR;
  static constexpr int WTS = CO * KP;
  static constexpr int WPX = TH * TW / 4;  // pixels per wave
  static constexpr int PB = WPX / 16, CB = CO / 16;
  static constexpr int HCH = HH * HW * (CS / 8);  // 16-byte chunks of a halo
  static constexpr int PFN = (HCH + kThreads - 1) / kThreads;
  static constexpr size_t kLds = static_cast<size_t>(HALO + WTS) * sizeof(uint16_t) + CO * 4 * sizeof(float);
};

// F32: fp32 output (the x3 fp32 step, ops/x3.py: CS = 3 planes x 32 channels) -- 16 B per lane and channel block
template <int CS, int CO, int TW, bool F32 = false>
__global__ __launch_bounds__(kThreads) void conv_direct_kernel(Gather g, const uint16_t* __restrict__ B,
                                                              uint16_t* __restrict__ C, int64_t ldc,
                                                              float* __restrict__ stats, int64_t sstride,
                                                              int tiles_x, int tiles_y, int ntiles, BnRed bnr) {
  using D = DirectCfg<CS, CO, TW>;
  extern __shared__ __attribute__((aligned(16))) uint16_t dsm[];
  uint16_t* halo = dsm;
  uint16_t* wts = dsm + D::HALO;
  // the fused BN-backward reduction (dgrad): per channel xhat = z*p0 + p1, pre-activation z*p2 + p3
  float4* coef = reinterpret_cast<float4*>(dsm + D::HALO + D::WTS);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kq = lane >> 4;
  if (bnr.z != nullptr)
    for (int c = threadIdx.x; c < CO; c += kThreads) {
      float4 q;
      bnr_coef(bnr, c, q.x, q.y, q.z, q.w);
      coef[c] = q;
    }

  // weight panel [CO][K] -> LDS rows of KP (once per workgroup)
  for (int v = threadIdx.x; v < CO * (D::K / 8); v += kThreads) {
    const int row = v / (D::K / 8), k8 = v - row * (D::K / 8);
    *reinterpret_cast<uint4*>(wts + row * D::KP + k8 * 8) =
        *reinterpret_cast<const uint4*>(B + static_cast<int64_t>(row) * D::K + k8 * 8);
  }

  uint4 pf[D::PFN];
  // tile-invariant part of each prefetch chunk: halo (row, column) packed in one word and the element
  // offset from the halo origin -- per tile only a wave-uniform base pointer changes (no 64-bit
  // (pix + iy * Ws + ix) * ld product per chunk and tile)
  int pyx[D::PFN], poff[D::PFN];
#pragma unroll
  for (int i = 0; i < D::PFN; ++i) {
    const int v = i * kThreads + threadIdx.x;
    const int hp = v / (CS / 8), c8 = v - hp * (CS / 8);
    const int hy = hp / D::HW, hx = hp - hy * D::HW;
    pyx[i] = v < D::HCH ? (hy << 16) | hx : 0x7fff0000;  // past the halo: never in bounds
    poff[i] = (hy * g.Ws + hx) * static_cast<int>(g.ld) + c8 * 8;
  }
  auto tile_origin = [&](int t, int& n, int& oy0, int& ox0) {
    const int tx = t % tiles_x, rest = t / tiles_x;
    const int ty = rest % tiles_y;
    n = rest / tiles_y;
    oy0 = ty * D::TH;
    ox0 = tx * TW;
  };
  auto prefetch = [&](int t) {  // the halo of tile t into registers (zeros outside the image)
    int n, oy0, ox0;
    tile_origin(t, n, oy0, ox0);
    const int hy0 = oy0 + g.offh - (g.sign < 0 ? D::R - 1 : 0);
    const int hx0 = ox0 + g.offw - (g.sign < 0 ? D::S - 1 : 0);
    const uint16_t* hb = g.src + ((static_cast<int64_t>(n) * g.Hs + hy0) * g.Ws + hx0) * g.ld;
#pragma unroll
    for (int i = 0; i < D::PFN; ++i) {
      const int iy = hy0 + (pyx[i] >> 16), ix = hx0 + (pyx[i] & 0xffff);
      pf[i] = make_uint4(0u, 0u, 0u, 0u);
      if (static_cast<unsigned>(iy) < static_cast<unsigned>(g.Hs) && static_cast<unsigned>(ix) < static_cast<unsigned>(g.Ws))
        pf[i] = *reinterpret_cast<const uint4*>(hb + poff[i]);
    }
  };

  float ssum[D::CB][4], ssq[D::CB][4];
#pragma unroll
  for (int c = 0; c < D::CB; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) ssum[c][r] = ssq[c][r] = 0.f;

  if (blockIdx.x < ntiles) prefetch(blockIdx.x);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    __syncthreads();  // every wave is done reading the previous halo
#pragma unroll
    for (int i = 0; i < D::PFN; ++i) {
      const int v = i * kThreads + threadIdx.x;
      if (v < D::HCH) {
        const int hp = v / (CS / 8), c8 = v - hp * (CS / 8);
        *reinterpret_cast<uint4*>(halo + hp * D::PSTR + c8 * 8) = pf[i];
      }
    }
    __syncthreads();
    if (t + static_cast<int>(gridDim.x) < ntiles) prefetch(t + gridDim.x);  // in flight during the MFMAs

    int pbase[D::PB];  // halo element offset of this lane's pixel in each 16-pixel block, tap (0, 0)
#pragma unroll
    for (int b = 0; b < D::PB; ++b) {
      const int p = wave * D::WPX + b * 16 + (lane & 15);
      pbase[b] = ((p / TW) * D::HW + (p % TW)) * D::PSTR + kq * 8;
    }
    f32x4 acc[D::PB][D::CB];
#pragma unroll
    for (int b = 0; b < D::PB; ++b)
#pragma unroll
      for (int c = 0; c < D::CB; ++c) acc[b][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < D::R; ++r)
#pragma unroll
      for (int s2 = 0; s2 < D::S; ++s2) {
        const int rr = g.sign > 0 ? r : D::R - 1 - r, ss = g.sign > 0 ? s2 : D::S - 1 - s2;
        const int hoff = (rr * D::HW + ss) * D::PSTR;
#pragma unroll
        for (int cb = 0; cb < CS / 32; ++cb) {
          const int k0 = (r * D::S + s2) * CS + cb * 32 + kq * 8;
          bf16x8_t wf[D::CB], xf[D::PB];
#pragma unroll
          for (int c = 0; c < D::CB; ++c)
            wf[c] = *reinterpret_cast<const bf16x8_t*>(wts + (c * 16 + (lane & 15)) * D::KP + k0);
#pragma unroll
          for (int b = 0; b < D::PB; ++b) xf[b] = *reinterpret_cast<const bf16x8_t*>(halo + pbase[b] + hoff + cb * 32);
#pragma unroll
          for (int b = 0; b < D::PB; ++b)
#pragma unroll
            for (int c = 0; c < D::CB; ++c)
              acc[b][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[c], xf[b], acc[b][c], 0, 0, 0);
        }
      }

    // epilogue: lane holds channels c*16 + 4kq .. +3 of pixel b*16 + (lane & 15): one 8-byte store
    int n, oy0, ox0;
    tile_origin(t, n, oy0, ox0);
#pragma unroll
    for (int b = 0; b < D::PB; ++b) {
      const int p = wave * D::WPX + b * 16 + (lane & 15);
      const int oy = oy0 + p / TW, ox = ox0 + p % TW;
      if (oy >= g.OH || ox >= g.OW) continue;
      const int64_t pix = (static_cast<int64_t>(n) * g.OH + oy) * g.OW + ox;
      uint16_t* dst = C + pix * ldc + kq * 4;
#pragma unroll
      for (int c = 0; c < D::CB; ++c) {
        const f32x4 a = acc[b][c];
        if constexpr (F32)
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + pix * ldc + c * 16 + kq * 4) =
              make_float4(a[0], a[1], a[2], a[3]);
        else
          *reinterpret_cast<uint2*>(dst + c * 16) =
              make_uint2(static_cast<uint32_t>(f2bf(a[0])) | (static_cast<uint32_t>(f2bf(a[1])) << 16),
                         static_cast<uint32_t>(f2bf(a[2])) | (static_cast<uint32_t>(f2bf(a[3])) << 16));
        if (stats != nullptr) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            ssum[c][r] += a[r];
            ssq[c][r] = fmaf(a[r], a[r], ssq[c][r]);
          }
        } else if (!F32 && bnr.z != nullptr) {  // dY' and dY' * xhat of the bf16 values just stored
          const uint2 zr = *reinterpret_cast<const uint2*>(
              bnr.z + ((static_cast<int64_t>(n) * g.OH + oy) * g.OW + ox) * bnr.ldz + c * 16 + kq * 4);
          const float zf[4] = {__uint_as_float(zr.x << 16), __uint_as_float(zr.x & 0xffff0000u),
                               __uint_as_float(zr.y << 16), __uint_as_float(zr.y & 0xffff0000u)};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float4 q = coef[c * 16 + kq * 4 + r];
            const float d = (bnr.relu && fmaf(zf[r], q.z, q.w) <= 0.f) ? 0.f : bf2f(f2bf(a[r]));
            ssum[c][r] += d;
            ssq[c][r] = fmaf(d, fmaf(zf[r], q.x, q.y), ssq[c][r]);
          }
        }
      }
    }
  }
  if (stats == nullptr && (F32 || bnr.z == nullptr)) return;
  if (stats == nullptr) {  // BN-backward reduction: [dsum | dsumx] of this workgroup's pixels
    stats = bnr.dsum;
    sstride = bnr.sstride;
  }
  float* st = stats + shard_off(blockIdx.x, sstride);
#pragma unroll
  for (int c = 0; c < D::CB; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a = ssum[c][r], q = ssq[c][r];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {  // sum over the 16 pixels of the lane's quarter
        a += __shfl_xor(a, o, 64);
        q += __shfl_xor(q, o, 64);
      }
      if ((lane & 15) == 0) {
        atomicAdd(st + c * 16 + kq * 4 + r, a);
        atomicAdd(st + CO + c * 16 + kq * 4 + r, q);
      }
    }
}

// The direct kernel for this shape, or -3 when it does not apply.
int run_direct(const Gather& g, const void* B, void* C, int64_t ldc, int64_t N, int epi, float* st, int64_t sstride,
               hipStream_t stream, const BnRed& bnr = BnRed{}) {
  const bool f32 = (epi & 8) != 0;
  if (g.R != 3 || g.S != 3 || g.sh != 1 || g.sw != 1 || (epi & 22) || (ldc % 4) || g.halo_images <= 0 ||
      (reinterpret_cast<uintptr_t>(C) & (f32 ? 15 : 7)) || (reinterpret_cast<uintptr_t>(B) & 15) ||
      (f32 && bnr.z != nullptr))
    return -3;
  const auto launch = [&](auto cs, auto co, auto tw, auto f32c) -> int {
    constexpr int CS = decltype(cs)::value, CO = decltype(co)::value, TW = decltype(tw)::value;
    constexpr bool F32 = decltype(f32c)::value;
    using D = DirectCfg<CS, CO, TW>;
    const void* fn = reinterpret_cast<const void*>(&conv_direct_kernel<CS, CO, TW, F32>);
    static int per_cu = 0;  // per template instance: resident workgroups per CU (occupancy query)
    if (per_cu == 0) {
      if (D::kLds > 65536 &&
          hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(D::kLds)) != hipSuccess)
        return -3;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kThreads, D::kLds) != hipSuccess || per_cu <= 0)
        per_cu = -1;
    }
    if (per_cu < 0) return -3;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess)
      return -3;
    const int tiles_x = ceil_div(g.OW, TW), tiles_y = ceil_div(g.OH, kDirH);
    const int64_t ntiles = static_cast<int64_t>(g.halo_images) * tiles_x * tiles_y;
    if (ntiles > 0x7fffffff) return -2;
    const int grid = static_cast<int>(std::min<int64_t>(ntiles, static_cast<int64_t>(per_cu) * cus));
    conv_direct_kernel<CS, CO, TW, F32><<<grid, kThreads, D::kLds, stream>>>(
        g, static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C), ldc, st, sstride, tiles_x, tiles_y,
        static_cast<int>(ntiles), bnr);
    TONY_LAUNCH_CHECK();
    return 0;
  };
  using I = std::integral_constant<int, 32>;
  using I64 = std::integral_constant<int, 64>;
  using I96 = std::integral_constant<int, 96>;
  using I16 = std::integral_constant<int, 16>;
  using BF = std::false_type;
  if (f32) {  // the x3 planes of a 32-channel input (weights [CO][9][3 x 32] + halo in LDS: 130 / 150 KB)
    if (g.Cs == 96 && N == 32) return launch(I96{}, I{}, I{}, std::true_type{});
    if (g.Cs == 96 && N == 64) return launch(I96{}, I64{}, I16{}, std::true_type{});
    return -3;
  }
  if (g.Cs == 32 && N == 32) return launch(I{}, I{}, I{}, BF{});
  if (g.Cs == 32 && N == 64) return launch(I{}, I64{}, I16{}, BF{});  // 8 x 32 tiles: 258 VGPRs, 1 wave/SIMD
  if (g.Cs == 64 && N == 32) return launch(I64{}, I{}, I16{}, BF{});
  if (g.Cs == 64 && N == 64) return launch(I64{}, I64{}, I16{}, BF{});
  return -3;
}

int run_nt(const Gather& g, const void* B, void* C, int64_t ldc, int64_t M, int64_t N, int flags, float* stats,
           int64_t sstride, hipStream_t stream, const Phase& bph = Phase{}) {
  // flags bit0: statistics accumulated into stats (the caller zeroes it, ops/arena.py);
  // bit1: stats = [scale | shift] of the folded inference BN, bit2: ReLU after it (H5)
  // bit3: fp32 output (the x3 path, ops/x3.py): only the variants whose epilogue is nt_epilogue
  // bit4: C += the product (nt_epilogue's accum: a dgrad adding into a gradient already written)
  const int epi = flags & 31;
  if ((epi & 1) && (epi & 2)) return -1;
  if ((epi & 3) && stats == nullptr) return -1;
  if ((epi & 16) && ((epi & 3) || bph.bnr.z != nullptr)) return -1;
  float* st = stats;
  const int v = (flags >> 8) & 0xff;
  if (((flags >> 16) & 15) && !(v >= kGldsFirst && v < kGldsFirst + kNumGlds)) return -3;  // stream-K: LDS-DMA only
  if (((epi & 24) && v == kHaloVariant) || ((epi & 16) && v == kDirectVariant)) return -3;
  if (v == kHaloVariant) return bph.bnr.z != nullptr ? -3 : run_halo(g, B, C, ldc, N, epi, st, sstride, stream);
  if (v == kBandVariant) return bph.bnr.z != nullptr ? -3 : run_band(g, B, C, ldc, N, epi, st, sstride, stream);
  if (v == kDirectVariant) return run_direct(g, B, C, ldc, N, epi, st, sstride, stream, bph.bnr);
  if (v >= kGldsFirst && v < kGldsFirst + kNumGlds)
    return bph.bnr.z != nullptr ? -3
                                : run_glds(g, B, g.K, C, ldc, M, N, epi, st, sstride, v, stream, RowMap{}, BTaps{},
                                           (flags >> 16) & 15);
  if (v >= kNumNtVariants) return -1;
  if (v == 0) {
    const int64_t bn = pick_bn(N, 192);
    return bn <= 64 ? launch_nt_bm<256>(g, B, C, ldc, M, N, st, sstride, epi, bn, stream, bph)
                    : launch_nt_bm<128>(g, B, C, ldc, M, N, st, sstride, epi, bn, stream, bph);
  }
  const int64_t bn = pick_bn(N, kNtVariants[v].cap);
  switch (kNtVariants[v].bm) {
    case 64: return launch_nt_bm<64>(g, B, C, ldc, M, N, st, sstride, epi, bn, stream, bph);
    case 128: return launch_nt_bm<128>(g, B, C, ldc, M, N, st, sstride, epi, bn, stream, bph);
    default: return launch_nt_bm<256>(g, B, C, ldc, M, N, st, sstride, epi, bn, stream, bph);
  }
}

// One residue class of a strided dgrad with tile variant v (flags bits 8..15 of tony_conv_dgrad_strided).
int run_nt_phase(const Gather& g, const void* B, void* C, int64_t ldc, int64_t M, int64_t N, int v, const Phase& ph,
                 hipStream_t stream, int epi = 0) {
  // the LDS-DMA kernels: class taps read out of the full filter (BTaps), rows scattered back to the class's
  // dX pixels by the epilogue's row map; a fused BN-backward reduction (BnRed) has the NT kernel's epilogue only
  if (v >= kGldsFirst && ph.bnr.z != nullptr) v = 0;
  if (v >= kGldsFirst)
    return run_glds(g, B, static_cast<int64_t>(ph.R) * ph.S * g.Cs, C, ldc, M, N, epi, nullptr, 0, v, stream, ph.rows,
                    BTaps{ph.r0, ph.s0, ph.tsy, ph.tsx, ph.S});
  if (v == kBandVariant) return -3;  // (stride 1 only)
  if (v == kHaloVariant || v == kDirectVariant || v >= kNumNtVariants) return -1;
  if (v == 0) {
    const int64_t bn = pick_bn(N, 192);
    return bn <= 64 ? launch_nt_bm<256, true>(g, B, C, ldc, M, N, nullptr, 0, epi, bn, stream, ph)
                    : launch_nt_bm<128, true>(g, B, C, ldc, M, N, nullptr, 0, epi, bn, stream, ph);
  }
  const int64_t bn = pick_bn(N, kNtVariants[v].cap);
  switch (kNtVariants[v].bm) {
    case 64: return launch_nt_bm<64, true>(g, B, C, ldc, M, N, nullptr, 0, epi, bn, stream, ph);
    case 128: return launch_nt_bm<128, true>(g, B, C, ldc, M, N, nullptr, 0, epi, bn, stream, ph);
    default: return launch_nt_bm<256, true>(g, B, C, ldc, M, N, nullptr, 0, epi, bn, stream, ph);
  }
}

// ---------------------------------------------------------------- wgrad --
constexpr int WTBM = 128;  // Cout per tile
constexpr int WTBN = 128;  // K = (r, s, ci) per tile

// rows m of the reduction, tracked as (n, oy, ox) and advanced by TBK per K-step
struct MRow {
  int n, oy, ox;
  int64_t m;
  __device__ __forceinline__ void init(int64_t m_, const Gather& g) {
    m = m_;
    const int ohw = g.OH * g.OW;
    n = static_cast<int>(m_ / ohw);
    const int rem = static_cast<int>(m_ - static_cast<int64_t>(n) * ohw);
    oy = rem / g.OW;
    ox = rem - oy * g.OW;
  }
  __device__ __forceinline__ void advance(int dm, const Gather& g) {
    m += dm;
    ox += dm;
    while (ox >= g.OW) {
      ox -= g.OW;
      if (++oy == g.OH) {
        oy = 0;
        ++n;
      }
    }
  }
};

// One workgroup = a (TBM x 128) tile of dW over Cout x (r, s, ci), reducing WK rows of m per stage
// (WK/32 MFMA K-steps per barrier) over its split of the M rows.  TBM follows Cout (32 / 64 / 128)
// so the 3-channel-free stems (Cout 32/64) waste no MFMA rows; both operand tiles are staged in
// 256-B LDS rows and read with the transposing ds_read (tr_frag).
constexpr int WK = 32;  // 64-row stages measured slower: 2x LDS + VGPRs halve the waves hiding the gather

// INC: the im2col row walk is incremental.  The general walk re-derives every row's source address
// per stage (MRow's wrap loop + 64-bit (n * Hs * Ws + iy * Ws + ix) * ld products): ~24 quarter-rate
// v_mul_lo_u32 / v_mad_u64_u32 per stage against 16 MFMAs, so the loop was VALU-bound.  With INC
// each row keeps its source coordinates (ix, iy) and 32-bit element offset e; a WK-row advance adds
// wave-uniform deltas (WkStep) -- at most one output-row carry and one image carry per stage when
// OH * OW >= WK + OW -- and the dY rows advance by a pointer add: no multiply in the loop.
struct WkStep {
  int dx, dy, de;      // base advance: (WK % OW) columns, (WK / OW) rows
  int cx, cy, ce;      // extra when the column wraps (ox >= OW)
  int img_y, img_e;    // extra when the row wraps past the image (oy >= OH)
};

// the two rows (r, r + 16) of a WK-row stage that one thread fetches, walked incrementally
struct IncRows {
  int ix[2], iy[2], ie[2];  // source coordinates and element offset (pixel * ld + c) per row
  int xlim, ylim;           // carry thresholds: ix >= xlim <=> ox >= OW, iy >= ylim <=> oy >= OH
  __device__ __forceinline__ void init(const MRow* mr, const Gather& g, const TapPos& tp) {
    xlim = g.OW * g.sw + g.offw + tp.s;
    ylim = g.OH * g.sh + g.offh + tp.r;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ix[i] = mr[i].ox * g.sw + g.offw + tp.s;
      iy[i] = mr[i].oy * g.sh + g.offh + tp.r;
      ie[i] = ((mr[i].n * g.Hs + iy[i]) * g.Ws + ix[i]) * static_cast<int>(g.ld) + tp.c;
    }
  }
  __device__ __forceinline__ bool in_image(int i, const Gather& g) const {
    return (static_cast<unsigned>(iy[i]) < static_cast<unsigned>(g.Hs)) &
           (static_cast<unsigned>(ix[i]) < static_cast<unsigned>(g.Ws));
  }
  __device__ __forceinline__ void advance(const WkStep& ws) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ix[i] += ws.dx;
      iy[i] += ws.dy;
      ie[i] += ws.de;
      if (ix[i] >= xlim) {
        ix[i] += ws.cx;
        iy[i] += ws.cy;
        ie[i] += ws.ce;
      }
      if (iy[i] >= ylim) {
        iy[i] += ws.img_y;
        ie[i] += ws.img_e;
      }
    }
  }
};

// x3 (fp32) weight gradients: the three bf16 plane products dW = dYh^T Xh + dYh^T Xl + dYl^T Xh of
// ops/x3.py as ONE split-K launch.  Split s covers rows (s / npairs) * rows_per_split.. of plane pair
// q = s % npairs, reading dY and X at the element offsets dy_off[q] / x_off[q] (the plane's first
// channel), and stores its partials into slab split s, so one tony_splitk_reduce sums all three.
// npairs = 1, offsets 0: the plain wgrad.
struct PlanePairs {
  int npairs, sp;
  int dy_off[3], x_off[3];
};

template <int TBM, bool INC>
__global__ __launch_bounds__(kThreads) void conv_wgrad_kernel(const uint16_t* __restrict__ dY, int64_t lddy,
                                                              Gather g, float* __restrict__ C, int64_t M, int Co,
                                                              int tiles_n2, int ntiles, int64_t rows_per_split,
                                                              float* __restrict__ slab, SplitFold fold, WkStep ws,
                                                              PlanePairs pp) {
  constexpr int TM = TBM / 32;                 // 16-row MFMA tiles per wave along Cout (2 waves)
  constexpr int A_CH = TBM / 8;                // 16-B chunks per dY row in the tile
  constexpr int AV = (WK * A_CH + kThreads - 1) / kThreads;
  constexpr int BV = WK * 16 / kThreads;       // gathered X: WK rows x 16 chunks
  constexpr int TILE = WK * 128;               // elements per staged operand
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * 2 * TILE];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wg % ntiles, split = wg / ntiles;
  // the pairs of one row range are neighbours in the grid (pair = split % npairs), so the workgroups
  // running together read the same dY / X rows (dYh is shared by pairs 0 and 1, Xh by 0 and 2) out of
  // L2 instead of three planes' worth of distinct rows (the stem's 177 MB planes thrashed it: 577 vs
  // 3 x 111 us as three launches).  Wave-uniform selects, no dynamic index into the argument array.
  const int pair = split % pp.npairs;
  dY += pair == 0 ? pp.dy_off[0] : pair == 1 ? pp.dy_off[1] : pp.dy_off[2];
  g.src += pair == 0 ? pp.x_off[0] : pair == 1 ? pp.x_off[1] : pp.x_off[2];
  const int t1 = tile / tiles_n2, t2 = tile % tiles_n2;
  const int n1_0 = t1 * TBM, n2_0 = t2 * WTBN;
  const int64_t m_begin = static_cast<int64_t>(split / pp.npairs) * rows_per_split;
  const int64_t m_end = min(M, m_begin + rows_per_split);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int K = g.K;

  // B (gathered X): this thread's chunk column tid & 15, rows (tid >> 4) + 16 i
  const int bch = threadIdx.x & 15;
  const int brow = threadIdx.x >> 4;
  const int kcol = n2_0 + bch * 8;
  const bool kok = kcol < K;
  TapPos tp;
  tp.init(kok ? kcol : 0, g);
  MRow mr[BV];
#pragma unroll
  for (int i = 0; i < BV; ++i) mr[i].init(m_begin + brow + 16 * i, g);
  // A (dY): chunk v = tid + 256 i -> row v / A_CH, chunk v % A_CH
  int64_t arow_m = m_begin;
  static_assert(!INC || BV == 2, "IncRows walks two rows per thread");
  IncRows inc;
  if constexpr (INC) inc.init(mr, g, tp);

  auto load_b = [&](uint4* regs) {
    if constexpr (INC) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (kok && mr[0].m + 16 * i < m_end && inc.in_image(i, g))
          regs[i] = *reinterpret_cast<const uint4*>(g.src + inc.ie[i]);
        else
          regs[i] = make_uint4(0, 0, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < BV; ++i) {
      const MRow& q = mr[i];
      const int iy = q.oy * g.sh + g.offh + tp.r, ix = q.ox * g.sw + g.offw + tp.s;
      if (kok && q.m < m_end && static_cast<unsigned>(iy) < static_cast<unsigned>(g.Hs) &&
          static_cast<unsigned>(ix) < static_cast<unsigned>(g.Ws))
        regs[i] = *reinterpret_cast<const uint4*>(
            g.src + (static_cast<int64_t>(q.n) * g.Hs * g.Ws + iy * g.Ws + ix) * g.ld + tp.c);
      else
        regs[i] = make_uint4(0, 0, 0, 0);
    }
  };
  auto load_a = [&](uint4* regs) {
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int v = threadIdx.x + i * kThreads;
      const int row = v / A_CH, ch = v % A_CH;
      const int64_t m = arow_m + row;
      const int col = n1_0 + ch * 8;
      if (v < WK * A_CH && col < Co && m < m_end)
        regs[i] = *reinterpret_cast<const uint4*>(dY + m * lddy + col);
      else
        regs[i] = make_uint4(0, 0, 0, 0);
    }
  };
  auto store_a = [&](uint16_t* lds, const uint4* regs) {
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int v = threadIdx.x + i * kThreads;
      if (v < WK * A_CH) *reinterpret_cast<uint4*>(lds + tr_off(v / A_CH, v % A_CH)) = regs[i];
    }
  };
  auto store_b = [&](uint16_t* lds, const uint4* regs) {
#pragma unroll
    for (int i = 0; i < BV; ++i) *reinterpret_cast<uint4*>(lds + tr_off(brow + 16 * i, bch)) = regs[i];
  };

  f32x4 acc[TM][4];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = static_cast<int>((m_end - m_begin + WK - 1) / WK);
  uint4 ra[AV], rb[BV];
  if (nk > 0) {
    load_a(ra);
    load_b(rb);
    store_a(smem, ra);
    store_b(smem + TILE, rb);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const uint16_t* As = smem + (kt & 1) * 2 * TILE;
    const uint16_t* Bs = As + TILE;
    const bool more = kt + 1 < nk;
    if (more) {
      if constexpr (INC) {
        mr[0].m += WK;  // only the row index is read in INC mode
        inc.advance(ws);
      } else {
#pragma unroll
        for (int i = 0; i < BV; ++i) mr[i].advance(WK, g);
      }
      arow_m += WK;
      load_a(ra);
      load_b(rb);
    }
#pragma unroll
    for (int sub = 0; sub < WK / 32; ++sub) {
      const int kgrp = (lane >> 4) + sub * 4;  // 8-row group within the WK-row stage
      bf16x8_t af[TM], bfr[4];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = tr_frag(As, kgrp, wm * (TBM / 2) + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = tr_frag(Bs, kgrp, wn * 64 + j * 16, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      uint16_t* An = smem + ((kt + 1) & 1) * 2 * TILE;
      store_a(An, ra);
      store_b(An + TILE, rb);
    }
    __syncthreads();
  }
  if (slab != nullptr && (fold.flags & 4)) {  // the splits meet in-launch (splitk_tree_fold)
    splitk_tree_fold<TM, 4, kThreads>(acc, slab, K, n1_0 + wm * (TBM / 2), Co, n2_0 + wn * 64, K, tile, split,
                                      gridDim.x / ntiles, fold);
    return;
  }
  // slab mode: this split's partial tile with plain stores (tony_splitk_reduce sums the splits);
  // otherwise fp32 atomics into C
  float* dst = slab != nullptr ? slab + static_cast<int64_t>(split) * Co * K : C;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n2_0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = n1_0 + wm * (TBM / 2) + i * 16 + (lane >> 4) * 4 + r;
        if (row < Co && col < K) {
          if (slab != nullptr)
            dst[static_cast<int64_t>(row) * K + col] = acc[i][j][r];
          else
            atomicAdd(dst + static_cast<int64_t>(row) * K + col, acc[i][j][r]);
        }
      }
    }
  }
  if (slab != nullptr && fold.counters != nullptr)
    splitk_fold_tile<TBM, WTBN>(slab, static_cast<int64_t>(Co) * K, gridDim.x / ntiles, K, n1_0, Co, n2_0, K, tile,
                                fold);
}

// ---- wgrad with LDS-DMA staging: the same tiles and split-K plan as conv_wgrad_kernel<TBM>, but each operand stage is written straight into LDS by
// global_load_lds_dwordx4 (no VGPR staging) into a ring of 3 stages, so two stages are always in
// flight behind the MFMAs instead of one.  The LDS image is lane-linear (a wave instruction fills
// 4 rows of 256 B); the tr_off swizzle is applied on the SOURCE side: lane l of a row fetches
// logical chunk (l & 15) ^ tr_swz(row), which is where tr_frag looks for it.  Out-of-range rows /
// columns / taps fetch 16 zero bytes.  The DMAs are issued from inline asm, so hipcc neither
// counts them nor makes the ds_reads of the current slot wait for the DMAs into the other slots
// (it cannot tell LDS-DMA targets apart and would emit vmcnt(0) there); completion is one counted
// `s_waitcnt vmcnt(4)` + a raw s_barrier per stage (a __syncthreads() would drain the ring).
constexpr int kWgStages = 3;

// PF: the fragments of K-step k+1 are read from LDS into a second register set while step k's MFMAs issue
// (the transposing reads no longer sit between every barrier and its MFMAs); a stage's slot is refilled as
// soon as every wave holds its fragments, so all three slots carry DMAs.  +28 VGPRs (TBM 96): still three
// workgroups per CU (LDS-bound).
template <int TBM, bool INC, bool PF = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_wgrad_glds_kernel(const uint16_t* __restrict__ dY, int64_t lddy,
                                                                   Gather g, int64_t M, int Co, int tiles_n2,
                                                                   int ntiles, int64_t rows_per_split,
                                                                   float* __restrict__ slab, SplitFold fold,
                                                                   WkStep ws, PlanePairs pp) {
  constexpr int TM = TBM / 32;
  constexpr int TILE = WK * 128;           // elements per staged operand (32 rows x 256 B)
  constexpr int STAGE = 2 * TILE;          // A then B
  __shared__ __attribute__((aligned(16))) uint16_t smem[kWgStages * STAGE];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wg % ntiles, split = wg / ntiles;
  // the pairs of one row range are neighbours in the grid (pair = split % npairs), so the workgroups
  // running together read the same dY / X rows (dYh is shared by pairs 0 and 1, Xh by 0 and 2) out of
  // L2 instead of three planes' worth of distinct rows (the stem's 177 MB planes thrashed it: 577 vs
  // 3 x 111 us as three launches).  Wave-uniform selects, no dynamic index into the argument array.
  const int pair = split % pp.npairs;
  dY += pair == 0 ? pp.dy_off[0] : pair == 1 ? pp.dy_off[1] : pp.dy_off[2];
  g.src += pair == 0 ? pp.x_off[0] : pair == 1 ? pp.x_off[1] : pp.x_off[2];
  const int t1 = tile / tiles_n2, t2 = tile % tiles_n2;
  const int n1_0 = t1 * TBM, n2_0 = t2 * WTBN;
  const int64_t m_begin = static_cast<int64_t>(split / pp.npairs) * rows_per_split;
  const int64_t m_end = min(M, m_begin + rows_per_split);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int K = g.K;

  // this thread fetches rows r0 and r0 + 16 of every stage, logical chunk ch of each
  const int r0 = threadIdx.x >> 4;
  const int ch = (threadIdx.x & 15) ^ tr_swz(r0);  // tr_swz(r0 + 16) == tr_swz(r0)
  const int acol = n1_0 + ch * 8;
  // A rows keep the 256-B LDS stride of tr_off; with TBM < 128 the chunks past the tile are zeros
  const bool acol_ok = (ch < TBM / 8) & (acol < Co);
  const int kcol = n2_0 + ch * 8;
  const bool kok = kcol < K;
  TapPos tp;
  tp.init(kok ? kcol : 0, g);
  MRow mr[2];
  mr[0].init(m_begin + r0, g);
  mr[1].init(m_begin + r0 + 16, g);
  int64_t am = m_begin + r0;  // A row of the next stage to issue (second row: + 16)
  // wave-uniform LDS byte addresses: instruction i of this wave fills rows 4 * (wave + 4 i) .. + 3
  const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(smem) + (4 * wave) * 256);
  constexpr uint32_t kRow16 = 16 * 256, kStageB = STAGE * 2, kTileB = TILE * 2;

  // INC state: rows r0 and r0 + 16 of the next stage
  IncRows inc;
  const uint16_t* ap = dY + (m_begin + r0) * lddy + acol;
  int am32 = static_cast<int>(m_begin) + r0;
  const int mend32 = static_cast<int>(m_end);
  if constexpr (INC) inc.init(mr, g, tp);

  auto issue = [&](int slot) {
    const uint32_t As = base + slot * kStageB, Bs = As + kTileB;
    const void* z = &kZeroChunk;
    if constexpr (INC) {
      const int64_t row16 = 16 * lddy;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool ok = acol_ok & (am32 + 16 * i < mend32);
        glds16(ok ? static_cast<const void*>(ap + i * row16) : z, As + i * kRow16);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool ok = kok & (am32 + 16 * i < mend32) & inc.in_image(i, g);
        glds16(ok ? static_cast<const void*>(g.src + inc.ie[i]) : z, Bs + i * kRow16);
      }
      inc.advance(ws);
      am32 += WK;
      ap += WK * lddy;
      return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t m = am + 16 * i;
      const bool ok = acol_ok & (m < m_end);
      glds16(ok ? static_cast<const void*>(dY + m * lddy + acol) : z, As + i * kRow16);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const MRow& q = mr[i];
      const int iy = q.oy * g.sh + g.offh + tp.r, ix = q.ox * g.sw + g.offw + tp.s;
      const bool ok = kok & (q.m < m_end) & (static_cast<unsigned>(iy) < static_cast<unsigned>(g.Hs)) &
                      (static_cast<unsigned>(ix) < static_cast<unsigned>(g.Ws));
      const uint16_t* src = g.src + (static_cast<int64_t>(q.n) * g.Hs * g.Ws + iy * g.Ws + ix) * g.ld + tp.c;
      glds16(ok ? static_cast<const void*>(src) : z, Bs + i * kRow16);
    }
    am += WK;
    mr[0].advance(WK, g);
    mr[1].advance(WK, g);
  };

  f32x4 acc[TM][4];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = static_cast<int>((m_end - m_begin + WK - 1) / WK);
  if constexpr (PF) {
    const int kgrp = lane >> 4;
    bf16x8_t fa[2][TM], fb[2][4];
    auto rd = [&](auto slotc, auto bufc) {
      constexpr int SLOT = decltype(slotc)::value, BUF = decltype(bufc)::value;
      const uint16_t* As = smem + SLOT * STAGE;
      const uint16_t* Bs = As + TILE;
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[BUF][i] = tr_frag(As, kgrp, wm * (TBM / 2) + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[BUF][j] = tr_frag(Bs, kgrp, wn * 64 + j * 16, lane);
    };
    // K-step kt on ring slot SLOT with its fragments in register set BUF: stage kt + 1 has landed in every
    // wave and every wave holds step kt's fragments, so slot SLOT takes stage kt + 3
    auto pstep = [&](auto slotc, auto bufc) {
      constexpr int SLOT = decltype(slotc)::value, BUF = decltype(bufc)::value;
      asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      issue(SLOT);
      rd(std::integral_constant<int, (SLOT + 1) % kWgStages>{}, std::integral_constant<int, 1 - BUF>{});
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[BUF][i], fb[BUF][j], acc[i][j], 0, 0, 0);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    issue(0);
    issue(1);
    issue(2);
    asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    rd(I0{}, I0{});
    int kt = 0;
    for (; kt + 6 <= nk; kt += 6) {  // (slot, register set) repeat every 6 steps
      pstep(I0{}, I0{});
      pstep(I1{}, I1{});
      pstep(I2{}, I0{});
      pstep(I0{}, I1{});
      pstep(I1{}, I0{});
      pstep(I2{}, I1{});
    }
    if (kt < nk) pstep(I0{}, I0{});
    if (kt + 1 < nk) pstep(I1{}, I1{});
    if (kt + 2 < nk) pstep(I2{}, I0{});
    if (kt + 3 < nk) pstep(I0{}, I1{});
    if (kt + 4 < nk) pstep(I1{}, I0{});
  } else {
  issue(0);
  issue(1);
  // one K-step on ring slot SLOT (= kt % 3).  The loop is unrolled by the ring length so that the
  // slot is a compile-time constant: the fragment reads then address LDS as a per-lane offset (loop
  // invariant) plus an immediate, instead of re-deriving 16 addresses from the slot every step.
  const int kgrp = lane >> 4;
  auto step = [&](auto slot_c) {
    constexpr int SLOT = decltype(slot_c)::value;
    // stage kt has landed in this wave (4 DMAs per stage; stage kt+1's 4 may still fly) and, after
    // the barrier, in every wave; every wave is also done reading stage kt-1, whose slot is refilled
    // with stage kt+2 (past the end: zero / unread fills, which keeps the count uniform)
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue((SLOT + 2) % kWgStages);
    const uint16_t* As = smem + SLOT * STAGE;
    const uint16_t* Bs = As + TILE;
    bf16x8_t af[TM], bfr[4];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = tr_frag(As, kgrp, wm * (TBM / 2) + i * 16, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = tr_frag(Bs, kgrp, wn * 64 + j * 16, lane);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  };
  static_assert(kWgStages == 3, "the K loop is unrolled by the ring length");
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;
  int kt = 0;
  for (; kt + 3 <= nk; kt += 3) {
    step(S0{});
    step(S1{});
    step(S2{});
  }
  if (kt < nk) step(S0{});
  if (kt + 1 < nk) step(S1{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the workgroup retires
  if (fold.flags & 4) {  // the splits meet in-launch (splitk_tree_fold)
    splitk_tree_fold<TM, 4, kThreads>(acc, slab, K, n1_0 + wm * (TBM / 2), Co, n2_0 + wn * 64, K, tile, split,
                                      gridDim.x / ntiles, fold);
    return;
  }
  float* dst = slab + static_cast<int64_t>(split) * Co * K;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n2_0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = n1_0 + wm * (TBM / 2) + i * 16 + (lane >> 4) * 4 + r;
        if (row < Co && col < K) dst[static_cast<int64_t>(row) * K + col] = acc[i][j][r];
      }
    }
  }
  if (fold.counters != nullptr)
    splitk_fold_tile<TBM, WTBN>(slab, static_cast<int64_t>(Co) * K, gridDim.x / ntiles, K, n1_0, Co, n2_0, K, tile,
                                fold);
}

// ---- x3 (fp32) weight gradient with the plane pairs fused -------------------------------------------
// dW = dYh^T Xh + dYh^T Xl + dYl^T Xh (ops/x3.py) in ONE pass over the rows: every K-step stages the four
// operand planes of its WK rows -- dY hi / lo ([WK][TBM] each, 256-B rows) and the im2col rows of X hi /
// lo ([WK][128]) -- by LDS-DMA into a ST-slot ring and issues the three products on the same
// accumulators.  Against the plane-pair form of conv_wgrad_glds_kernel (each pair a full pass, three
// times the address walk, the DMAs and the fragment reads for the same MFMAs), the per-step im2col
// walk, bounds checks and pointer selects are shared by all three products: VALU per MFMA drops ~3x
// (the pair form's K loop issued 49 VALU + 21 SALU per 12 MFMAs: issue-bound, profiles/r5_streamk_ab.md
// PMC) and the operand intake per MFMA by a third.  The lo planes sit dplane / xplane elements after
// the hi ones in the same rows.  Slab mode: one partial per split, tony_splitk_reduce sums them.
template <int TBM, int ST, bool INC>
__global__ __launch_bounds__(kThreads) void conv_wgrad_x3f_kernel(const uint16_t* __restrict__ dY, int64_t lddy,
                                                                  Gather g, int64_t M, int Co, int tiles_n2,
                                                                  int ntiles, int64_t rows_per_split,
                                                                  float* __restrict__ slab, WkStep ws, int dplane,
                                                                  int xplane) {
  constexpr int TM = TBM / 32;
  constexpr int TILE = WK * 128;           // elements per staged plane (32 rows x 256 B)
  constexpr int STAGE = 4 * TILE;          // Ah, Al, Bh, Bl
  constexpr int NDMA = 8;                  // per thread and stage: 2 rows x 4 planes
  static_assert(ST == 2 || ST == 3, "ring of 2 or 3 stages");
  __shared__ __attribute__((aligned(16))) uint16_t smem[ST * STAGE];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wg % ntiles, split = wg / ntiles;
  const int t1 = tile / tiles_n2, t2 = tile % tiles_n2;
  const int n1_0 = t1 * TBM, n2_0 = t2 * WTBN;
  const int64_t m_begin = static_cast<int64_t>(split) * rows_per_split;
  const int64_t m_end = min(M, m_begin + rows_per_split);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int K = g.K;

  const int r0 = threadIdx.x >> 4;
  const int ch = (threadIdx.x & 15) ^ tr_swz(r0);  // tr_swz(r0 + 16) == tr_swz(r0)
  const int acol = n1_0 + ch * 8;
  const bool acol_ok = (ch < TBM / 8) & (acol < Co);
  const int kcol = n2_0 + ch * 8;
  const bool kok = kcol < K;
  TapPos tp;
  tp.init(kok ? kcol : 0, g);
  MRow mr[2];
  mr[0].init(m_begin + r0, g);
  mr[1].init(m_begin + r0 + 16, g);
  int64_t am = m_begin + r0;
  const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(smem) + (4 * wave) * 256);
  constexpr uint32_t kRow16 = 16 * 256, kStageB = STAGE * 2, kTileB = TILE * 2;
  IncRows inc;
  const uint16_t* ap = dY + (m_begin + r0) * lddy + acol;
  int am32 = static_cast<int>(m_begin) + r0;
  const int mend32 = static_cast<int>(m_end);
  if constexpr (INC) inc.init(mr, g, tp);

  auto issue = [&](int slot) {
    const uint32_t Ah = base + slot * kStageB, Al = Ah + kTileB, Bh = Al + kTileB, Bl = Bh + kTileB;
    const void* z = &kZeroChunk;
    if constexpr (INC) {
      const int64_t row16 = 16 * lddy;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool ok = acol_ok & (am32 + 16 * i < mend32);
        const uint16_t* a = ap + i * row16;
        glds16(ok ? static_cast<const void*>(a) : z, Ah + i * kRow16);
        glds16(ok ? static_cast<const void*>(a + dplane) : z, Al + i * kRow16);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool ok = kok & (am32 + 16 * i < mend32) & inc.in_image(i, g);
        const uint16_t* b = g.src + inc.ie[i];
        glds16(ok ? static_cast<const void*>(b) : z, Bh + i * kRow16);
        glds16(ok ? static_cast<const void*>(b + xplane) : z, Bl + i * kRow16);
      }
      inc.advance(ws);
      am32 += WK;
      ap += WK * lddy;
      return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t m = am + 16 * i;
      const bool ok = acol_ok & (m < m_end);
      const uint16_t* a = dY + m * lddy + acol;
      glds16(ok ? static_cast<const void*>(a) : z, Ah + i * kRow16);
      glds16(ok ? static_cast<const void*>(a + dplane) : z, Al + i * kRow16);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const MRow& q = mr[i];
      const int iy = q.oy * g.sh + g.offh + tp.r, ix = q.ox * g.sw + g.offw + tp.s;
      const bool ok = kok & (q.m < m_end) & (static_cast<unsigned>(iy) < static_cast<unsigned>(g.Hs)) &
                      (static_cast<unsigned>(ix) < static_cast<unsigned>(g.Ws));
      const uint16_t* b = g.src + (static_cast<int64_t>(q.n) * g.Hs * g.Ws + iy * g.Ws + ix) * g.ld + tp.c;
      glds16(ok ? static_cast<const void*>(b) : z, Bh + i * kRow16);
      glds16(ok ? static_cast<const void*>(b + xplane) : z, Bl + i * kRow16);
    }
    am += WK;
    mr[0].advance(WK, g);
    mr[1].advance(WK, g);
  };

  f32x4 acc[TM][4];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = static_cast<int>((m_end - m_begin + WK - 1) / WK);
#pragma unroll
  for (int s = 0; s < ST - 1; ++s) issue(s);
  const int kgrp = lane >> 4;
  auto step = [&](auto slot_c) {
    constexpr int SLOT = decltype(slot_c)::value;
    // stage kt has landed in this wave (the ST - 2 younger stages' DMAs may still fly) and, after the
    // barrier, in every wave; every wave is also done reading the slot refilled next
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((ST - 2) * NDMA) : "memory");
    __builtin_amdgcn_s_barrier();
    issue((SLOT + ST - 1) % ST);
    const uint16_t* Ahs = smem + SLOT * STAGE;
    const uint16_t* Als = Ahs + TILE;
    const uint16_t* Bhs = Als + TILE;
    const uint16_t* Bls = Bhs + TILE;
    bf16x8_t ah[TM], al[TM], bh[4], bl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bh[j] = tr_frag(Bhs, kgrp, wn * 64 + j * 16, lane);
#pragma unroll
    for (int i = 0; i < TM; ++i) ah[i] = tr_frag(Ahs, kgrp, wm * (TBM / 2) + i * 16, lane);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) bl[j] = tr_frag(Bls, kgrp, wn * 64 + j * 16, lane);
#pragma unroll
    for (int i = 0; i < TM; ++i) al[i] = tr_frag(Als, kgrp, wm * (TBM / 2) + i * 16, lane);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;
  int kt = 0;
  if constexpr (ST == 3) {
    for (; kt + 3 <= nk; kt += 3) {
      step(S0{});
      step(S1{});
      step(S2{});
    }
    if (kt < nk) step(S0{});
    if (kt + 1 < nk) step(S1{});
  } else {
    for (; kt + 2 <= nk; kt += 2) {
      step(S0{});
      step(S1{});
    }
    if (kt < nk) step(S0{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the workgroup retires
  float* dst = slab + static_cast<int64_t>(split) * Co * K;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n2_0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = n1_0 + wm * (TBM / 2) + i * 16 + (lane >> 4) * 4 + r;
        if (row < Co && col < K) dst[static_cast<int64_t>(row) * K + col] = acc[i][j][r];
      }
    }
  }
}

// ---- 3x3 stride-1 weight gradient with 32 / 64 channels on both sides: persistent direct kernel --
// The implicit-GEMM wgrad (above) gathers the im2col rows of X through L2 for each of the 9 taps and,
// with Cout = 32 / 64, runs 16-row MFMA tiles with a thin A panel: Inception's 149x149 / 147x147
// stem layers (51 / 102 GFLOP) ran at ~100 TF/s, serialised at the very end of the backward pass.
// Here a persistent workgroup walks 8 x 16 output-pixel tiles (b, b + grid, ...), stages the tile's
// dY [128 px][CO] and the (8+2) x (16+2) input halo [px][CS] in LDS ONCE (the next tile's in flight
// in registers), and computes every tap's dW_t[co][ci] = sum_px dY[px][co] X[px + t][ci] from LDS:
// MFMA A = dY^T (co x 32 px), B = the tap-shifted halo pixels (32 px x ci), both read with the
// transposing ds_read_b64_tr_b16 (rows = pixels).  The 9 * CS/16 (tap, ci-block) pairs are dealt to
// the 4 waves; each pair's CO/16 accumulator blocks stay in registers over all the workgroup's tiles,
// and the workgroup stores its [CO][9][CS] partial once (tony_splitk_reduce sums the workgroups).
// LDS rows are CS / CO bf16 = 2 or 4 blocks of 16 columns, block b of row r at b ^ wd_swz(r): any 8
// rows {r0..r0+3, r0+8..r0+11} a transposing read touches land on 8 distinct 32-B bank slots.
constexpr int kWdH = 8, kWdW = 16, kWdPix = kWdH * kWdW;

template <int NCB>
__device__ __forceinline__ int wd_swz(int row) {
  if constexpr (NCB == 2) return (row >> 3) & 1;
  else return ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
}
template <int C>
__device__ __forceinline__ int wd_off(int row, int col) {  // element offset of (row, col), col % 4 == 0
  return row * C + ((((col >> 4) ^ wd_swz<C / 16>(row))) << 4) + (col & 15);
}
// MFMA operand of 8 consecutive LDS rows (row0 + 0..7 of this lane's k-group) x 16 columns
template <int C>
__device__ __forceinline__ bf16x8_t wd_frag(const uint16_t* lds, int row0, int col0, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3;
  const int col = col0 + 4 * p;
  v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(lds + wd_off<C>(row0 + q, col)));
  v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(lds + wd_off<C>(row0 + 4 + q, col)));
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  v8i16 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, r);
}

template <int CS, int CO>
struct WdCfg {
  static constexpr int HH = kWdH + 2, HW = kWdW + 2;
  static constexpr int HALO = HH * HW * CS;         // elements
  static constexpr int DYT = kWdPix * CO;
  static constexpr int HV = (HH * HW * CS / 8 + kThreads - 1) / kThreads;  // 16-B chunks per thread
  static constexpr int DV = kWdPix * CO / 8 / kThreads;
  static constexpr int NP = 9 * (CS / 16);          // (tap, ci block) pairs
  static constexpr int PPW = (NP + 3) / 4;          // pairs per wave
  static constexpr int CB = CO / 16;
};

template <int CS, int CO>
__global__ __launch_bounds__(kThreads) void conv_wgrad_direct_kernel(const uint16_t* __restrict__ dY, int64_t lddy,
                                                                     Gather g, float* __restrict__ slab,
                                                                     int tiles_x, int tiles_y, int ntiles) {
  using D = WdCfg<CS, CO>;
  __shared__ __attribute__((aligned(16))) uint16_t smem[D::HALO + D::DYT];
  uint16_t* halo = smem;
  uint16_t* dyl = smem + D::HALO;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kq = lane >> 4;

  f32x4 acc[D::PPW][D::CB];
#pragma unroll
  for (int i = 0; i < D::PPW; ++i)
#pragma unroll
    for (int j = 0; j < D::CB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 hv[D::HV], dv[D::DV];
  auto fetch = [&](int tile) {
    const int tx = tile % tiles_x, rest = tile / tiles_x;
    const int ty = rest % tiles_y, img = rest / tiles_y;
    const int oy0 = ty * kWdH, ox0 = tx * kWdW;
#pragma unroll
    for (int i = 0; i < D::HV; ++i) {
      const int v = threadIdx.x + i * kThreads;
      const int hp = v / (CS / 8), c8 = v % (CS / 8);
      const int hy = hp / D::HW, hx = hp - hy * D::HW;
      const int iy = oy0 + hy + g.offh, ix = ox0 + hx + g.offw;
      hv[i] = (hp < D::HH * D::HW && static_cast<unsigned>(iy) < static_cast<unsigned>(g.Hs) &&
               static_cast<unsigned>(ix) < static_cast<unsigned>(g.Ws))
                  ? *reinterpret_cast<const uint4*>(
                        g.src + ((static_cast<int64_t>(img) * g.Hs + iy) * g.Ws + ix) * g.ld + c8 * 8)
                  : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int i = 0; i < D::DV; ++i) {
      const int v = threadIdx.x + i * kThreads;
      const int px = v / (CO / 8), c8 = v % (CO / 8);
      const int oy = oy0 + px / kWdW, ox = ox0 + px % kWdW;
      dv[i] = (oy < g.OH && ox < g.OW)
                  ? *reinterpret_cast<const uint4*>(
                        dY + ((static_cast<int64_t>(img) * g.OH + oy) * g.OW + ox) * lddy + c8 * 8)
                  : make_uint4(0u, 0u, 0u, 0u);
    }
  };

  if (static_cast<int>(blockIdx.x) < ntiles) fetch(blockIdx.x);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    __syncthreads();  // every wave is done with the previous tile's LDS
#pragma unroll
    for (int i = 0; i < D::HV; ++i) {
      const int v = threadIdx.x + i * kThreads;
      const int hp = v / (CS / 8), c8 = v % (CS / 8);
      if (hp < D::HH * D::HW) *reinterpret_cast<uint4*>(halo + wd_off<CS>(hp, c8 * 8)) = hv[i];
    }
#pragma unroll
    for (int i = 0; i < D::DV; ++i) {
      const int v = threadIdx.x + i * kThreads;
      *reinterpret_cast<uint4*>(dyl + wd_off<CO>(v / (CO / 8), (v % (CO / 8)) * 8)) = dv[i];
    }
    __syncthreads();
    if (tile + static_cast<int>(gridDim.x) < ntiles) fetch(tile + gridDim.x);
#pragma unroll
    for (int ks = 0; ks < kWdPix / 32; ++ks) {
      const int p0 = ks * 32 + kq * 8;       // this lane's 8 pixels: one half row of the tile
      const int py = p0 / kWdW, px = p0 % kWdW;
      bf16x8_t af[D::CB];
#pragma unroll
      for (int i = 0; i < D::CB; ++i) af[i] = wd_frag<CO>(dyl, p0, i * 16, lane);
#pragma unroll
      for (int pp = 0; pp < D::PPW; ++pp) {
        const int pair = wave + 4 * pp;
        if (pair >= D::NP) break;  // wave-uniform
        const int t = pair / (CS / 16), j = pair % (CS / 16);
        const int r = t / 3, sx = t - r * 3;
        const bf16x8_t bfr = wd_frag<CS>(halo, (py + r) * D::HW + px + sx, j * 16, lane);
#pragma unroll
        for (int i = 0; i < D::CB; ++i) acc[pp][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[pp][i], 0, 0, 0);
      }
    }
  }
  // this workgroup's partial dW [CO][9][CS] (every (tap, ci block, co block) has one owner wave)
  constexpr int K = 9 * CS;
  float* out = slab + static_cast<int64_t>(blockIdx.x) * CO * K;
#pragma unroll
  for (int pp = 0; pp < D::PPW; ++pp) {
    const int pair = wave + 4 * pp;
    if (pair >= D::NP) break;
    const int t = pair / (CS / 16), j = pair % (CS / 16);
#pragma unroll
    for (int i = 0; i < D::CB; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        out[static_cast<int64_t>(i * 16 + kq * 4 + rr) * K + t * CS + j * 16 + (lane & 15)] = acc[pp][i][rr];
  }
}

bool wgrad_glds_enabled() {
  static const bool on = [] {
    const char* e = getenv("TONY_WGRAD_GLDS");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

// TONY_WGRAD_PF: 1 = the fragment-prefetch K loop of conv_wgrad_glds_kernel (PF), 0 = the plain one;
// tony_wgrad_pf(-1) reads it, 0 / 1 sets it (tests)
std::atomic<int>& wgrad_pf_flag() {
  static std::atomic<int> f{[] {
    const char* e = getenv("TONY_WGRAD_PF");
    return (e != nullptr && e[0] == '1') ? 1 : 0;
  }()};
  return f;
}
bool wgrad_pf_enabled() { return wgrad_pf_flag().load(std::memory_order_relaxed) != 0; }

bool wgrad_inc_enabled() {  // TONY_WGRAD_INC=0: the general row walk (A/B measurements)
  static const bool on = [] {
    const char* e = getenv("TONY_WGRAD_INC");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

// the WK-row advance of the incremental im2col walk; false when the walk does not apply (element
// offsets or rows past int32, or images so small that one stage can wrap more than one image)
bool wgrad_inc_step(const Gather& g, int64_t M, WkStep* ws) {
  const int64_t images = M / (static_cast<int64_t>(g.OH) * g.OW) + 1;
  const int64_t src_elems = images * g.Hs * g.Ws * g.ld;
  if (!wgrad_inc_enabled() || src_elems >= (int64_t{1} << 30) || M >= (int64_t{1} << 30) ||
      static_cast<int64_t>(g.OH) * g.OW < WK + g.OW)
    return false;
  const int q = WK / g.OW, rem = WK % g.OW, ld = static_cast<int>(g.ld);
  ws->dx = rem * g.sw;
  ws->dy = q * g.sh;
  ws->de = (rem * g.sw + q * g.sh * g.Ws) * ld;
  ws->cx = -g.OW * g.sw;
  ws->cy = g.sh;
  ws->ce = (g.sh * g.Ws - g.OW * g.sw) * ld;
  ws->img_y = -g.OH * g.sh;
  ws->img_e = (g.Hs - g.OH * g.sh) * g.Ws * ld;
  return true;
}

template <int TBM>
int launch_wgrad(const void* dy, int64_t lddy, const Gather& g, float* dw, float* slab, int64_t slab_cap,
                 int* splits_out, int64_t M, int Co, int num_cus, const SplitFold& fold, hipStream_t stream,
                 PlanePairs pp = PlanePairs{1, 1, {0, 0, 0}, {0, 0, 0}}) {
  const int tiles_n1 = ceil_div(Co, TBM), tiles_n2 = ceil_div(g.K, WTBN);
  const int ntiles = tiles_n1 * tiles_n2;
  const int npairs = pp.npairs;
  // enough workgroups for ~2 per CU (over all plane pairs), each reducing >= 8 stages of WK rows
  const int target = 2 * (num_cus > 0 ? num_cus : 256);
  int64_t splits = (target + static_cast<int64_t>(ntiles) * npairs - 1) / (static_cast<int64_t>(ntiles) * npairs);
  const int64_t max_splits = (M + 8 * WK - 1) / (8 * WK);
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int64_t rows = (M + splits - 1) / splits;
  rows = (rows + WK - 1) / WK * WK;
  splits = (M + rows - 1) / rows;  // per plane pair
  pp.sp = static_cast<int>(splits);
  const int64_t grid = splits * npairs * ntiles;
  if (grid > 0x7fffffff) return -2;
  if (slab != nullptr && splits * npairs * Co * static_cast<int64_t>(g.K) > slab_cap) return -4;  // caller's bound is off
  if (npairs > 1 && (slab == nullptr || fold.counters != nullptr)) return -1;  // the pairs meet in the slab
  // the tree fold's workspace: one TBM x WTBN fp32 slot per workgroup, 32-bit byte offsets
  if ((fold.flags & 4) && (fold.counters == nullptr || slab == nullptr || grid * TBM * WTBN > slab_cap ||
                           grid * TBM * WTBN * 4 > 0x7fffffff))
    return -3;
  if (splits_out != nullptr) *splits_out = static_cast<int>(splits * npairs);
  // LDS-DMA staging pays for the 128-row Cout tiles only (measured: Cout <= 64 tiles, whose A rows
  // are half / quarter zero chunks, run 4-8 % slower than the register-staged kernel)
  WkStep ws{};
  const bool inc = wgrad_inc_step(g, M, &ws);
  const auto* dyp = static_cast<const uint16_t*>(dy);
  if (TBM >= 96 && slab != nullptr && wgrad_glds_enabled()) {
    if (inc && wgrad_pf_enabled())
      conv_wgrad_glds_kernel<TBM, true, true><<<static_cast<int>(grid), kThreads, 0, stream>>>(
          dyp, lddy, g, M, Co, tiles_n2, ntiles, rows, slab, fold, ws, pp);
    else if (inc)
      conv_wgrad_glds_kernel<TBM, true><<<static_cast<int>(grid), kThreads, 0, stream>>>(
          dyp, lddy, g, M, Co, tiles_n2, ntiles, rows, slab, fold, ws, pp);
    else
      conv_wgrad_glds_kernel<TBM, false><<<static_cast<int>(grid), kThreads, 0, stream>>>(
          dyp, lddy, g, M, Co, tiles_n2, ntiles, rows, slab, fold, ws, pp);
  } else if (inc) {
    conv_wgrad_kernel<TBM, true><<<static_cast<int>(grid), kThreads, 0, stream>>>(
        dyp, lddy, g, dw, M, Co, tiles_n2, ntiles, rows, slab, fold, ws, pp);
  } else {
    conv_wgrad_kernel<TBM, false><<<static_cast<int>(grid), kThreads, 0, stream>>>(
        dyp, lddy, g, dw, M, Co, tiles_n2, ntiles, rows, slab, fold, ws, pp);
  }
  TONY_LAUNCH_CHECK();
  return 0;
}

// TONY_X3_WGRAD_FUSED: 0 = the plane-pair form, 1 = fused planes on a 3-slot ring (one workgroup per CU),
// 2 = fused on a 2-slot ring (two per CU; default).  tony_x3_wgrad_mode overrides it (tests, A/B).
std::atomic<int> g_x3f_mode{-1};

int x3f_mode() {
  int m = g_x3f_mode.load(std::memory_order_relaxed);
  if (m < 0) {
    const char* e = getenv("TONY_X3_WGRAD_FUSED");
    m = e == nullptr ? 2 : atoi(e);
    g_x3f_mode.store(m, std::memory_order_relaxed);
  }
  return m;
}

// the fused x3 weight gradient (conv_wgrad_x3f_kernel): Cout tiles of 64 / 96 / 128 rows, splits for
// ~1 (3-slot ring) or ~2 (2-slot) workgroups per CU, each reducing >= 8 stages of WK rows
int launch_wgrad_x3f(const void* dy, int64_t lddy, const Gather& g, float* slab, int64_t slab_cap, int* splits_out,
                     int64_t M, int Co, int num_cus, int dplane, int xplane, hipStream_t stream) {
  const int tbm = Co <= 64 ? 64 : (ceil_div(Co, 96) * 96 < ceil_div(Co, 128) * 128 ? 96 : 128);
  const int ring = x3f_mode() == 1 ? 3 : 2;
  const int tiles_n1 = ceil_div(Co, tbm), tiles_n2 = ceil_div(g.K, WTBN);
  const int ntiles = tiles_n1 * tiles_n2;
  const int target = (ring == 3 ? 1 : 2) * (num_cus > 0 ? num_cus : 256);
  int64_t splits = (target + ntiles - 1) / ntiles;
  const int64_t max_splits = (M + 8 * WK - 1) / (8 * WK);
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int64_t rows = (M + splits - 1) / splits;
  rows = (rows + WK - 1) / WK * WK;
  splits = (M + rows - 1) / rows;
  const int64_t grid = splits * ntiles;
  if (grid > 0x7fffffff) return -2;
  if (slab == nullptr || splits * Co * static_cast<int64_t>(g.K) > slab_cap) return -4;
  if (splits_out != nullptr) *splits_out = static_cast<int>(splits);
  WkStep ws{};
  const bool inc = wgrad_inc_step(g, M, &ws);
  const auto* dyp = static_cast<const uint16_t*>(dy);
  const auto go = [&](auto tb, auto st) {
    constexpr int TB = decltype(tb)::value, S = decltype(st)::value;
    if (inc)
      conv_wgrad_x3f_kernel<TB, S, true><<<static_cast<int>(grid), kThreads, 0, stream>>>(
          dyp, lddy, g, M, Co, tiles_n2, ntiles, rows, slab, ws, dplane, xplane);
    else
      conv_wgrad_x3f_kernel<TB, S, false><<<static_cast<int>(grid), kThreads, 0, stream>>>(
          dyp, lddy, g, M, Co, tiles_n2, ntiles, rows, slab, ws, dplane, xplane);
  };
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  switch (tbm) {
    case 64: ring == 3 ? go(std::integral_constant<int, 64>{}, I3{}) : go(std::integral_constant<int, 64>{}, I2{}); break;
    case 96: ring == 3 ? go(std::integral_constant<int, 96>{}, I3{}) : go(std::integral_constant<int, 96>{}, I2{}); break;
    default: ring == 3 ? go(std::integral_constant<int, 128>{}, I3{}) : go(std::integral_constant<int, 128>{}, I2{}); break;
  }
  TONY_LAUNCH_CHECK();
  return 0;
}

// Cout tile rows of the split-K wgrad: 32 / 64 for thin layers; above, 96 where it pads Cout less than
// 128 does (Inception's 160 / 192 / 288 / 448-channel layers: 25-37% of the 128-row tiles' MFMA rows
// were zero padding at 160 / 192), else 128.  TONY_WGRAD_TBM96=0: always 128 (A/B).
int wgrad_tbm(int Co) {
  static const bool t96 = [] {
    const char* e = getenv("TONY_WGRAD_TBM96");
    return e == nullptr || e[0] != '0';
  }();
  if (Co <= 32) return 32;
  if (Co <= 64) return 64;
  return t96 && ceil_div(Co, 96) * 96 < ceil_div(Co, 128) * 128 ? 96 : 128;
}

bool bad_geom(int C, int64_t ld, const void* p) {
  return C <= 0 || (C % 8) || (ld % 8) || (reinterpret_cast<uintptr_t>(p) & 15);
}

}  // namespace

namespace tony {
SplitWs& splitk_ws() {
  static thread_local SplitWs ws;
  return ws;
}
}  // namespace tony

// The stream-K workspace of this host thread's next LDS-DMA conv / GEMM launches (flags bits 16..19 =
// m of tony_conv_fwd / tony_conv_dgrad / tony_gemm_bf16: a grid of m x CUs workgroups): slab_floats
// fp32 for the partial tiles (2 per workgroup) and ncnt uint32 per-tile arrival counters, zero on
// first use (each launch's last arrivers re-arm theirs).  Kernels that may run at the same time
// (other streams) must not share one workspace.  All zero: none (stream-K launches then run plain).
TONY_API int tony_splitk_workspace(float* slab, int64_t slab_floats, unsigned* cnt, int64_t ncnt) {
  if (slab_floats < 0 || ncnt < 0 || (reinterpret_cast<uintptr_t>(slab) & 15)) return -1;
  tony::splitk_ws() = tony::SplitWs{slab, slab_floats, cnt, ncnt};
  return 0;
}

// Y[N*OH*OW, Co] (row stride ldy) = conv(X [N,H,W,C] pixel stride ldx, W [Co][R][S][C]).
// flags bit0: per-channel sum / sum-of-squares of Y into stats[2*Co] (zero on entry; kStatShards
// copies sstride floats apart when sstride > 0); bits 8..15: tile variant (run_nt).
// the fused x3 codes (igemm.h kX3Variants): the operand has C = 3 cp channels per pixel ([hi | lo | hi]
// planes, ops/x3.py) and the filter rows [hi | hi | lo] per tap; the kernel reduces K = R * S * cp with three
// products per K-step.  -3: not an x3 code, or a shape it does not take.
int run_x3(Gather g, const void* B, int Cx, void* C, int64_t ldc, int64_t M, int64_t N, int flags, float* stats,
           int64_t sstride, hipStream_t stream) {
  const int v = (flags >> 8) & 0xff;
  if (v < kX3First || v >= kX3First + kNumX3 || Cx % 3 || (Cx / 3) % 8) return -3;
  const int epi = flags & 31;
  if ((epi & 1) && (epi & 2)) return -1;
  if ((epi & 3) && stats == nullptr) return -1;
  if ((epi & 16) && (epi & 3)) return -1;
  const int cp = Cx / 3;
  g.Cs = cp;
  g.K = g.R * g.S * cp;
  return run_glds_x3(g, B, static_cast<int64_t>(g.R) * g.S * Cx, C, ldc, M, N, epi, stats, sstride, v, stream,
                        RowMap{}, BTaps{}, (flags >> 16) & 15, X3Planes{cp, 2 * cp, 3 * cp});
}

TONY_API int tony_conv_fwd(const void* x, int N, int H, int W, int C, int64_t ldx, const void* w, int Co, int R,
                           int S, int sh, int sw, int ph, int pw, void* y, int OH, int OW, int64_t ldy, int flags,
                           float* stats, int64_t sstride, hipStream_t stream) {
  if (bad_geom(C, ldx, x) || (reinterpret_cast<uintptr_t>(w) & 15) || Co <= 0 || R <= 0 || S <= 0 || sstride < 0)
    return -1;
  if (OH != (H + 2 * ph - R) / sh + 1 || OW != (W + 2 * pw - S) / sw + 1 || OH <= 0 || OW <= 0) return -1;
  const int64_t M = static_cast<int64_t>(N) * OH * OW;
  if (M > 0x7fffffff || static_cast<int64_t>(N) * H * W > 0x7fffffff) return -1;
  Gather g{static_cast<const uint16_t*>(x), ldx, H, W, C, OH, OW, R, S, sh, sw, -ph, -pw, 1, R * S * C, N};
  const int v = (flags >> 8) & 0xff;
  if (v >= kX3First && v < kX3First + kNumX3) return run_x3(g, w, C, y, ldy, M, Co, flags, stats, sstride, stream);
  return run_nt(g, w, y, ldy, M, Co, flags, stats, sstride, stream);
}

// dX[N*H*W, C] (row stride lddx) of a stride-1 conv: dY [N,OH,OW,Co] (pixel stride lddy),
// Wt = W permuted to [C][R][S][Co].  flags bits 8..15: tile variant (run_nt).
TONY_API int tony_conv_dgrad(const void* dy, int N, int OH, int OW, int Co, int64_t lddy, const void* wt, int C,
                             int R, int S, int ph, int pw, void* dx, int H, int W, int64_t lddx, int flags,
                             BnRed* bnr, hipStream_t stream) {
  if (bad_geom(Co, lddy, dy) || (reinterpret_cast<uintptr_t>(wt) & 15) || C <= 0) return -1;
  if (OH != H + 2 * ph - R + 1 || OW != W + 2 * pw - S + 1) return -1;  // stride 1 only
  const int64_t M = static_cast<int64_t>(N) * H * W;
  if (M > 0x7fffffff || static_cast<int64_t>(N) * OH * OW > 0x7fffffff) return -1;
  Gather g{static_cast<const uint16_t*>(dy), lddy, OH, OW, Co, H, W, R, S, 1, 1, ph, pw, -1, R * S * Co, N};
  Phase bph{};
  if (bnr != nullptr) {
    bnr->done = 0;
    if (bnr->z != nullptr) {
      if (bnr->mean == nullptr || bnr->invstd == nullptr || bnr->dsum == nullptr || (bnr->ldz % 8) ||
          (reinterpret_cast<uintptr_t>(bnr->z) & 15) || (C % 8))
        return -1;
      bph.bnr = *bnr;
    }
  }
  const int fl = flags & 0xfff18;  // variant + stream-K (bits 16..19) + fp32 output (bit3) + accumulate (bit4)
  if ((fl & 16) && bph.bnr.z != nullptr) return -1;
  const int v = (fl >> 8) & 0xff;
  if (v >= kX3First && v < kX3First + kNumX3)  // fused x3 planes of dY / Wt (no fused BN reduction)
    return bph.bnr.z != nullptr ? -3 : run_x3(g, wt, Co, dx, lddx, M, C, fl, nullptr, 0, stream);
  const int rc = run_nt(g, wt, dx, lddx, M, C, fl, nullptr, 0, stream, bph);
  if (rc == -3 && bph.bnr.z != nullptr)  // the chosen variant has no fused reduction: plain dgrad
    return run_nt(g, wt, dx, lddx, M, C, fl, nullptr, 0, stream);
  if (rc == 0 && bph.bnr.z != nullptr) bnr->done = 1;
  return rc;
}

// TONY_DGRAD_ONE_LAUNCH=0 (or tony_dgrad_one_launch(0)): one launch per residue class (A/B and the
// numerics test of the MultiClass launch)
static std::atomic<int>& dgrad_one_launch_flag() {
  static std::atomic<int> on{[] {
    const char* e = std::getenv("TONY_DGRAD_ONE_LAUNCH");
    return (e != nullptr && e[0] == '0') ? 0 : 1;
  }()};
  return on;
}
static bool dgrad_one_launch() { return dgrad_one_launch_flag().load(std::memory_order_relaxed) != 0; }
TONY_API int tony_wgrad_pf(int on) {
  const int prev = wgrad_pf_flag().load();
  if (on >= 0) wgrad_pf_flag().store(on ? 1 : 0);
  return prev;
}

TONY_API int tony_dgrad_one_launch(int on) {
  const int prev = dgrad_one_launch_flag().load();
  if (on >= 0) dgrad_one_launch_flag().store(on ? 1 : 0);
  return prev;
}

// dX[N*H*W, C] (row stride lddx) of a STRIDED conv (stride sh x sw, padding ph, pw): one MFMA
// implicit-GEMM launch per residue class (iy % sh, ix % sw) of dX, each a stride-1 transposed conv
// over the class's sub-grid with the class's taps of Wt = W permuted to [C][R][S][Co] (Phase).
// Every dX pixel is written exactly once (classes with no taps write zeros).  flags bits 8..15:
// tile variant (run_nt_phase); bit4: dX += the product (a projection shortcut's dgrad adding into the
// gradient the block's first conv already wrote, ops/residual.py GradJoin) -- the classes with no
// taps then add nothing and are not launched (3 of the 4 classes of a 1x1 / 2 shortcut).
TONY_API int tony_conv_dgrad_strided(const void* dy, int N, int OH, int OW, int Co, int64_t lddy, const void* wt,
                                     int C, int R, int S, int sh, int sw, int ph, int pw, void* dx, int H, int W,
                                     int64_t lddx, int flags, BnRed* bnr, hipStream_t stream) {
  if (bad_geom(Co, lddy, dy) || (reinterpret_cast<uintptr_t>(wt) & 15) || C <= 0 || C % 8 || (lddx % 8) ||
      (reinterpret_cast<uintptr_t>(dx) & 15))
    return -1;
  BnRed br{};
  if (bnr != nullptr) {
    bnr->done = 0;
    if (bnr->z != nullptr) {
      if (bnr->mean == nullptr || bnr->invstd == nullptr || bnr->dsum == nullptr || (bnr->ldz % 8) ||
          (reinterpret_cast<uintptr_t>(bnr->z) & 15))
        return -1;
      br = *bnr;  // every residue class adds its pixels' sums
    }
  }
  if (sh < 1 || sw < 1 || sh > 4 || sw > 4 || ph < 0 || pw < 0 || ph >= R || pw >= S) return -1;
  if (OH != (H + 2 * ph - R) / sh + 1 || OW != (W + 2 * pw - S) / sw + 1 || OH <= 0 || OW <= 0) return -1;
  if (static_cast<int64_t>(N) * H * W > 0x7fffffff || static_cast<int64_t>(N) * OH * OW > 0x7fffffff) return -1;
  const int v = (flags >> 8) & 0xff;
  const int acc = flags & 16;
  if (acc && br.z != nullptr) return -1;
  if ((flags >> 16) & 15) return -3;  // no stream-K for the residue classes
  // the LDS-DMA variants without a fused BN reduction: every class in one launch (MultiClass)
  const bool one = v >= kGldsFirst && v < kGldsFirst + kNumGlds && br.z == nullptr && sh * sw <= kMaxClasses &&
                   Co % kGldsVariants[v - kGldsFirst].kb == 0 && dgrad_one_launch();
  MultiClass mc{};
  for (int py = 0; py < sh; ++py) {
    for (int px = 0; px < sw; ++px) {
      const int QH = H > py ? (H - py + sh - 1) / sh : 0, QW = W > px ? (W - px + sw - 1) / sw : 0;
      const int64_t M = static_cast<int64_t>(N) * QH * QW;
      if (M == 0) continue;
      // taps r = r0 + sh*a reach the pixels iy = sh*qy + py:  oy = (iy + ph - r) / sh = qy + cy - a
      const int r0 = (py + ph) % sh, s0 = (px + pw) % sw;
      int Ra = r0 < R ? (R - r0 + sh - 1) / sh : 0, Sb = s0 < S ? (S - s0 + sw - 1) / sw : 0;
      const int cy = (py + ph - r0) / sh, cx = (px + pw - s0) / sw;
      if (Ra == 0 || Sb == 0) {
        if (acc) continue;  // adds zero
        Ra = 0, Sb = 1;     // no taps: the GEMM has K = 0 and writes zeros
      }
      Gather g{static_cast<const uint16_t*>(dy), lddy, OH, OW, Co, QH, QW, Ra, Sb, 1, 1, cy, cx, -1, Ra * Sb * Co, N};
      Phase phz{R, S, r0, s0, sh, sw, RowMap{}};
      phz.rows.qw = QW;
      phz.rows.qhw = QH * QW;
      phz.rows.W = W;
      phz.rows.HW = H * W;
      phz.rows.sy = sh;
      phz.rows.sx = sw;
      phz.rows.y0 = py;
      phz.rows.x0 = px;
      phz.bnr = br;
      if (one) {
        mc.c[mc.n++] = ClassDesc{g, phz.rows, BTaps{r0, s0, sh, sw, S}, static_cast<int>(M), 0};
        continue;
      }
      const int rc = run_nt_phase(g, wt, dx, lddx, M, C, v, phz, stream, flags & 24);
      if (rc != 0) return rc;
    }
  }
  if (one && mc.n > 0) {
    // (g, M, rmap, bt of the call are placeholders: each workgroup takes its class's)
    // tap-heaviest class first: its tiles run longest (up to 4x the 1-tap class's K)
    std::stable_sort(mc.c, mc.c + mc.n, [](const ClassDesc& a, const ClassDesc& b) { return a.g.K > b.g.K; });
    const ClassDesc& c0 = mc.c[0];
    const int rc = run_glds(c0.g, wt, static_cast<int64_t>(R) * S * Co, dx, lddx, c0.M, C, flags & 24, nullptr, 0, v,
                            stream, c0.rm, c0.bt, 0, X3Planes{}, &mc);
    if (rc != 0) return rc;
  }
  if (br.z != nullptr) bnr->done = 1;
  return 0;
}

// dW (fp32 [Co][R][S][C], zero on entry) = dY^T im2col(X); dY [N*OH*OW, Co] row stride lddy.
// With a slab (slab_cap floats >= splits * Co*R*S*C) the M splits store their partial dW there
// instead of adding into dw with atomics; *splits_out gets the split count.  With fold_counters
// (ceil(Co/TBM) * ceil(K/128) zeroed uint32) the last split of each tile also sums the slab into
// fold_dst (fold_flags bit0 bf16, bit1 accumulate): no tony_splitk_reduce launch.
TONY_API int tony_conv_wgrad(const void* dy, int64_t lddy, const void* x, int N, int H, int W, int C, int64_t ldx,
                             int Co, int R, int S, int sh, int sw, int ph, int pw, int OH, int OW, float* dw,
                             float* slab, int64_t slab_cap, int* splits_out, int num_cus, unsigned* fold_counters,
                             void* fold_dst, int fold_flags, hipStream_t stream) {
  if (bad_geom(C, ldx, x) || (Co % 8) || (lddy % 8) || (reinterpret_cast<uintptr_t>(dy) & 15)) return -1;
  if (OH != (H + 2 * ph - R) / sh + 1 || OW != (W + 2 * pw - S) / sw + 1) return -1;
  const int K = R * S * C;
  const int64_t M = static_cast<int64_t>(N) * OH * OW;
  if (M > 0x7fffffff) return -1;
  Gather g{static_cast<const uint16_t*>(x), ldx, H, W, C, OH, OW, R, S, sh, sw, -ph, -pw, 1, K, 0};
  if (slab == nullptr && dw == nullptr) return -1;
  if (fold_counters != nullptr && (slab == nullptr || fold_dst == nullptr || (K % 4) ||
                                   (reinterpret_cast<uintptr_t>(fold_dst) & 7)))
    return -1;
  const SplitFold fold{fold_counters, fold_dst, fold_flags};
  switch (wgrad_tbm(Co)) {
    case 32: return launch_wgrad<32>(dy, lddy, g, dw, slab, slab_cap, splits_out, M, Co, num_cus, fold, stream);
    case 64: return launch_wgrad<64>(dy, lddy, g, dw, slab, slab_cap, splits_out, M, Co, num_cus, fold, stream);
    case 96: return launch_wgrad<96>(dy, lddy, g, dw, slab, slab_cap, splits_out, M, Co, num_cus, fold, stream);
    default: return launch_wgrad<128>(dy, lddy, g, dw, slab, slab_cap, splits_out, M, Co, num_cus, fold, stream);
  }
}

// x3 weight gradient (ops/x3.py conv_wgrad): dy / x point at the hi planes (channel 0) of the dY and X
// plane tensors, the lo planes start dplane / xplane elements (channels) later; C and Co are the plane
// widths.  Partials of dYh^T Xh, dYh^T Xl and dYl^T Xh into one slab (*splits_out = all of them):
// the caller's tony_splitk_reduce sums the three products.
TONY_API int tony_conv_wgrad_x3(const void* dy, int64_t lddy, const void* x, int N, int H, int W, int C, int64_t ldx,
                                int Co, int R, int S, int sh, int sw, int ph, int pw, int OH, int OW, int dplane,
                                int xplane, float* slab, int64_t slab_cap, int* splits_out, int num_cus,
                                hipStream_t stream) {
  if (bad_geom(C, ldx, x) || (Co % 8) || (lddy % 8) || (reinterpret_cast<uintptr_t>(dy) & 15) || slab == nullptr)
    return -1;
  if ((dplane % 8) || (xplane % 8) || dplane < Co || xplane < C || dplane + Co > lddy || xplane + C > ldx) return -1;
  if (OH != (H + 2 * ph - R) / sh + 1 || OW != (W + 2 * pw - S) / sw + 1) return -1;
  const int K = R * S * C;
  const int64_t M = static_cast<int64_t>(N) * OH * OW;
  if (M > 0x7fffffff) return -1;
  Gather g{static_cast<const uint16_t*>(x), ldx, H, W, C, OH, OW, R, S, sh, sw, -ph, -pw, 1, K, 0};
  const SplitFold fold{nullptr, nullptr, 0};
  if (x3f_mode() > 0 && wgrad_glds_enabled()) {
    const int rc = launch_wgrad_x3f(dy, lddy, g, slab, slab_cap, splits_out, M, Co, num_cus, dplane, xplane, stream);
    if (rc != -3) return rc;
  }
  const PlanePairs pp{3, 1, {0, 0, dplane}, {0, xplane, 0}};
  // thin layers (Co <= 64) on the LDS-DMA kernel's 96-row tiles: its three plane pairs ran 3x slower
  // on the register-staged 32 / 64-row kernel (conv_wgrad_kernel<64>: 304 us per 35x35 layer,
  // profiles/r4_fp32_x3_steady.md) than the padding the 96-row tile wastes
  static const bool thin_glds = [] {
    const char* e = getenv("TONY_X3_WGRAD_THIN_GLDS");
    return e == nullptr || e[0] != '0';
  }();
  const int tbm = wgrad_tbm(Co);
  switch (thin_glds && wgrad_glds_enabled() && tbm < 96 ? 96 : tbm) {
    case 32: return launch_wgrad<32>(dy, lddy, g, nullptr, slab, slab_cap, splits_out, M, Co, num_cus, fold, stream, pp);
    case 64: return launch_wgrad<64>(dy, lddy, g, nullptr, slab, slab_cap, splits_out, M, Co, num_cus, fold, stream, pp);
    case 96: return launch_wgrad<96>(dy, lddy, g, nullptr, slab, slab_cap, splits_out, M, Co, num_cus, fold, stream, pp);
    default: return launch_wgrad<128>(dy, lddy, g, nullptr, slab, slab_cap, splits_out, M, Co, num_cus, fold, stream, pp);
  }
}

// the x3 weight-gradient form (x3f_mode): mode >= 0 sets it, -1 only reads; returns the previous mode
TONY_API int tony_x3_wgrad_mode(int mode) {
  const int prev = x3f_mode();
  if (mode >= 0) g_x3f_mode.store(mode, std::memory_order_relaxed);
  return prev;
}

// dW (fp32 partials, [grid][Co][3][3][C]) of a 3x3 stride-1 conv with C, Co in {32, 64} by the
// persistent direct kernel; *splits = the workgroup count (tony_splitk_reduce sums them).  -3: the
// shape is not one it takes.
TONY_API int tony_conv_wgrad_direct(const void* dy, int64_t lddy, const void* x, int N, int H, int W, int C,
                                    int64_t ldx, int Co, int ph, int pw, int OH, int OW, float* slab,
                                    int64_t slab_cap, int* splits, int num_cus, hipStream_t stream) {
  if (bad_geom(C, ldx, x) || (lddy % 8) || (reinterpret_cast<uintptr_t>(dy) & 15) || slab == nullptr) return -1;
  if ((C != 32 && C != 64) || (Co != 32 && Co != 64) || ph < 0 || pw < 0 || ph > 2 || pw > 2) return -3;
  if (OH != H + 2 * ph - 2 || OW != W + 2 * pw - 2 || OH <= 0 || OW <= 0) return -1;
  if (static_cast<int64_t>(N) * H * W > 0x7fffffff || static_cast<int64_t>(N) * OH * OW > 0x7fffffff) return -1;
  Gather g{static_cast<const uint16_t*>(x), ldx, H, W, C, OH, OW, 3, 3, 1, 1, -ph, -pw, 1, 9 * C, N};
  const int tiles_x = ceil_div(OW, kWdW), tiles_y = ceil_div(OH, kWdH);
  const int64_t nt = static_cast<int64_t>(N) * tiles_x * tiles_y;
  if (nt > 0x7fffffff) return -1;
  const auto launch = [&](auto cs, auto co) -> int {
    constexpr int CS = decltype(cs)::value, CO = decltype(co)::value;
    const void* fn = reinterpret_cast<const void*>(&conv_wgrad_direct_kernel<CS, CO>);
    static int per_cu = 0;  // per instance: resident workgroups per CU
    if (per_cu == 0 && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kThreads, 0) != hipSuccess ||
                        per_cu <= 0))
      per_cu = 1;
    const int grid = static_cast<int>(std::min<int64_t>(nt, static_cast<int64_t>(std::min(per_cu, 2)) *
                                                                (num_cus > 0 ? num_cus : 256)));
    if (static_cast<int64_t>(grid) * CO * 9 * CS > slab_cap) return -4;
    conv_wgrad_direct_kernel<CS, CO><<<grid, kThreads, 0, stream>>>(static_cast<const uint16_t*>(dy), lddy, g, slab,
                                                                    tiles_x, tiles_y, static_cast<int>(nt));
    TONY_LAUNCH_CHECK();
    *splits = grid;
    return 0;
  };
  using I32 = std::integral_constant<int, 32>;
  using I64 = std::integral_constant<int, 64>;
  if (C == 32) return Co == 32 ? launch(I32{}, I32{}) : launch(I32{}, I64{});
  return Co == 32 ? launch(I64{}, I32{}) : launch(I64{}, I64{});
}
