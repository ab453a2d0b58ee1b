// Image-stem convolutions (3-channel input: Inception-v3's 3x3/2, ResNet's 7x7/2) on MFMA:
// forward with the BatchNorm-statistics epilogue of the implicit-GEMM kernels, and the split-K
// weight gradient.  No MIOpen on the stem.
//
// GEMM view (as conv.hip):  Y[m, co] = sum_k A[m, k] W[co, k],  m = (n, oy, ox),  k = (r, s, c),
// A[m, k] = X[n, oy*sh - ph + r, ox*sw - pw + s, c].  With C = 3 a K row is NOT made of 16-byte
// channel chunks (the conv.hip loaders need C % 8 == 0): K = 27 is padded to one 32-deep
// 16x16x32 bf16 MFMA step (7x7: 147 -> 5 steps) and each lane builds its 8-element A fragment
// element by element from the input rows the workgroup staged into LDS.  Because the image is
// dense NHWC, the input rows under a block of consecutive output pixels are ONE contiguous element
// range -- also across an image boundary -- so staging is plain 16-byte loads.
//
// The layer moves 250 MB (Inception, batch 128: 69 MB in, 182 MB out) for 4.9 GFLOP, so it is a
// streaming kernel: one barrier per workgroup, 256 output pixels x Cout per workgroup, the
// statistics + 16-byte store epilogue of the NT kernels (mfma_common.h nt_epilogue).
//
// Weight gradient: dW[co, k] = sum_m dY[m, co] A[m, k] -- a reduction over all 2.8M pixels into
// a Cout x 27 matrix.  A persistent grid of ~2 workgroups per CU walks 256-pixel chunks; per
// chunk the dY rows (16 KB) and the input rows are staged in LDS, every wave reduces 64 pixels
// with the MFMA (A = dY^T: 8 pixels of one channel per lane, B = the same im2col gather as the
// forward), the four waves fold their tiles with LDS float adds at the end, and each workgroup
// stores one partial into the split-K slab that csrc/splitk.hip sums into the gradient slot.
#include <type_traits>
#include "mfma_common.h"

using namespace tony;
using namespace tony::mfma;

namespace {

constexpr int kBM = 256;        // output pixels per forward tile / per wgrad chunk
constexpr int kPatch = 12288;   // bf16 elements of staged input rows (24 KB: 7 rows of a 299-wide
                                // RGB image, 13 rows of a 224-wide one)
constexpr int kPF = kPatch / 8 / kThreads;  // 16-byte prefetch registers per thread
constexpr int kMaxKSteps = 8;   // K = R*S*C <= 256

struct StemGeom {
  const uint16_t* x;     // dense NHWC image [N][H][W][C]
  int H, W, C;
  int R, S, sh, sw, ph, pw;
  int OH, OW;
  int M;                 // N * OH * OW
  int K;                 // R * S * C
  int64_t total;         // N * H * W * C
  float inv_ohw, inv_ow; // 1 / (OH * OW), 1 / OW: pixel index -> (n, oy, ox) without integer division
};

// q = a / b for 0 <= a < 2^24 (exact in fp32): the fp32 quotient is off by at most one, fixed up with
// 24-bit integer products (full rate; a runtime integer division is a ~30-instruction sequence)
__device__ __forceinline__ int fast_div(int a, int b, float inv_b) {
  int q = static_cast<int>(static_cast<float>(a) * inv_b);
  const int r = a - static_cast<int>(__umul24(q, b));
  if (r < 0) --q;
  else if (r >= b) ++q;
  return q;
}

// Element range [e0, e1) of x covering every in-image tap of output pixels m_first..m_last
// (consecutive in m).  e0 is 8-aligned (16-byte loads).  False if it does not fit the patch.
__device__ __forceinline__ bool stage_range(const StemGeom& g, int m_first, int m_last, int64_t& e0, int64_t& e1) {
  const int ohw = g.OH * g.OW;
  const int n0 = m_first / ohw, n1 = m_last / ohw;
  const int ya = max(0, (m_first - n0 * ohw) / g.OW * g.sh - g.ph);
  const int yb = min(g.H - 1, (m_last - n1 * ohw) / g.OW * g.sh - g.ph + g.R - 1);
  e0 = (static_cast<int64_t>(n0) * g.H + ya) * g.W * g.C & ~static_cast<int64_t>(7);
  e1 = ((static_cast<int64_t>(n1) * g.H + yb + 1) * g.W * g.C + 7) & ~static_cast<int64_t>(7);
  if (e1 < e0) e1 = e0;
  return e1 - e0 <= kPatch;
}

// The input rows of the NEXT tile / chunk, loaded into registers while the current one computes
// (one barrier-separated LDS write per tile: the load latency hides behind the MFMA work).
struct RowPrefetch {
  uint4 v[kPF];
  int64_t e0, e1;
  bool staged;
  __device__ __forceinline__ void issue(const StemGeom& g, int m_first, int m_last) {
    staged = stage_range(g, m_first, m_last, e0, e1);
    if (!staged) return;
#pragma unroll
    for (int i = 0; i < kPF; ++i) {
      const int64_t k = e0 + (static_cast<int64_t>(i) * kThreads + threadIdx.x) * 8;
      if (k + 8 <= g.total && k < e1) {
        v[i] = *reinterpret_cast<const uint4*>(g.x + k);
      } else if (k < e1) {
        uint16_t t[8];
        for (int j = 0; j < 8; ++j) t[j] = k + j < g.total ? g.x[k + j] : static_cast<uint16_t>(0);
        v[i] = *reinterpret_cast<const uint4*>(t);
      }
    }
  }
  __device__ __forceinline__ void commit(uint16_t* patch) const {
    if (!staged) return;
#pragma unroll
    for (int i = 0; i < kPF; ++i) {
      const int64_t k = e0 + (static_cast<int64_t>(i) * kThreads + threadIdx.x) * 8;
      if (k < e1) *reinterpret_cast<uint4*>(patch + (k - e0)) = v[i];
    }
  }
};

// One output pixel: element index of its tap (0, 0) relative to the staged range (or to x), and
// its top-left input coordinate.
struct Pix {
  int64_t base;
  int n, oy, ox, iy0, ix0;
  bool ok;
  __device__ __forceinline__ void set(const StemGeom& g, int64_t e0) {
    iy0 = oy * g.sh - g.ph;
    ix0 = ox * g.sw - g.pw;
    // unsigned 24-bit products (full rate) on the unpadded coordinates oy * sh, ox * sw >= 0: the pixel
    // index stays below N * H * W < 2^24 (make_geom) and times C below 2^31; the padding offset is
    // subtracted afterwards
    const unsigned pix = __umul24(__umul24(static_cast<unsigned>(n), g.H) + static_cast<unsigned>(iy0 + g.ph), g.W) +
                         static_cast<unsigned>(ix0 + g.pw);
    base = static_cast<int64_t>(__umul24(pix, g.C)) - (static_cast<int64_t>(g.ph) * g.W + g.pw) * g.C - e0;
  }
  __device__ __forceinline__ void init(const StemGeom& g, int m, int64_t e0) {
    ok = m < g.M;
    const int mm = ok ? m : 0;
    const int ohw = g.OH * g.OW;
    n = fast_div(mm, ohw, g.inv_ohw);  // make_geom guarantees M < 2^24
    const int rem = mm - n * ohw;
    oy = fast_div(rem, g.OW, g.inv_ow);
    ox = rem - oy * g.OW;
    set(g, e0);
  }
  // the next output pixel (m + 1) without divisions
  __device__ __forceinline__ void next(const StemGeom& g, int m_next, int64_t e0) {
    ok = m_next < g.M;
    if (++ox == g.OW) {
      ox = 0;
      if (++oy == g.OH) {
        oy = 0;
        ++n;
      }
    }
    set(g, e0);
  }
};

// GEMM column k inside a pixel's receptive field, packed in one word: element offset (bits 0-19),
// tap row r (20-25), tap column s (26-31).  A K-padding column (k >= K) aliases tap (0, 0): it
// passes the same image-bounds check as a real tap, so it reads either a real, finite input
// element (which the zero weight column cancels) or nothing.  It used to be marked r = 63 and
// skipped only when iy0 + 63 >= H -- for images taller than 63 rows with padding that let pixels of
// the first output rows read the element at input row -ph, outside the staged LDS range (or before
// x), and a NaN found there survived the zero weight (NaN * 0 = NaN) into the BN statistics; the
// fused BN + ReLU then turned the whole activation into zeros (fmaxf(NaN, 0) = 0): the round-2
// "fused ResNet-50 forward collapses to 0" failure of tests/test_ops_gpu.py.
__device__ __forceinline__ uint32_t tap_word(const StemGeom& g, int k) {
  if (k >= g.K) return 0u;
  const int sc = g.S * g.C;
  const int r = k / sc, rem = k - r * sc;
  const int s = rem / g.C;
  const int off = (r * g.W + s) * g.C + (rem - s * g.C);
  return static_cast<uint32_t>(off) | (static_cast<uint32_t>(r) << 20) | (static_cast<uint32_t>(s) << 26);
}

// NP (no padding): every tap of an output pixel lies inside the image, so the gather is one add and
// one load.  Either way the K-padding columns (k >= K) read the pixel's own tap-(0, 0) value, which
// the zero weight columns (forward) cancel and the weight gradient never stores.
template <bool NP>
__device__ __forceinline__ uint16_t tap_value(const StemGeom& g, const uint16_t* src, const Pix& p, uint32_t t) {
  if constexpr (NP) return p.ok ? src[p.base + static_cast<int>(t & 0xfffffu)] : static_cast<uint16_t>(0);
  const int r = (t >> 20) & 63, s = t >> 26;
  const bool in = p.ok && static_cast<unsigned>(p.iy0 + r) < static_cast<unsigned>(g.H) &&
                  static_cast<unsigned>(p.ix0 + s) < static_cast<unsigned>(g.W);
  return in ? src[p.base + static_cast<int>(t & 0xfffffu)] : static_cast<uint16_t>(0);
}

__device__ __forceinline__ bf16x8_t pack8(const uint16_t (&v)[8]) {
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  v8i16 r = {static_cast<short>(v[0]), static_cast<short>(v[1]), static_cast<short>(v[2]), static_cast<short>(v[3]),
             static_cast<short>(v[4]), static_cast<short>(v[5]), static_cast<short>(v[6]), static_cast<short>(v[7])};
  return __builtin_bit_cast(bf16x8_t, r);
}

// ------------------------------------------------------------------------------------ forward --
// Persistent: workgroup b computes tiles b, b + grid, ...; each wave owns 64 rows x all BN columns
// of a 256-pixel tile (no duplicated gathers).  The weight fragments (bf16, MFMA-B order) and the
// per-column tap table are built in LDS once per workgroup.  BN statistics accumulate in
// registers over all the workgroup's tiles and are added once (one sharded atomic per column).
template <int BN, bool NP>
__global__ __launch_bounds__(kThreads) void stem_fwd_kernel(StemGeom g, const uint16_t* __restrict__ wk,
                                                            uint16_t* __restrict__ y, int64_t ldy,
                                                            float* __restrict__ stats, int64_t sstride) {
  constexpr int TM = 4, TN = BN / 16;
  constexpr int LDC = BN + 8;
  constexpr int STAGE = kPatch > kBM * LDC ? kPatch : kBM * LDC;
  // dynamic LDS: [STAGE] staging | [ksteps * TN * 64 * 8] weight fragments (launch-sized)
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  __shared__ uint32_t taps[kMaxKSteps * 32];
  uint16_t* wl = smem + STAGE;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kq = lane >> 4;
  const int ksteps = (g.K + 31) / 32;
  const int ntiles = (g.M + kBM - 1) / kBM;

  RowPrefetch pf;
  if (blockIdx.x < ntiles) pf.issue(g, blockIdx.x * kBM, min(g.M, (blockIdx.x + 1) * kBM) - 1);
  for (int idx = threadIdx.x; idx < ksteps * TN * 64; idx += kThreads) {
    const int t = idx / (TN * 64), j = (idx / 64) % TN, l = idx % 64;
    const uint16_t* wr = wk + static_cast<int64_t>(j * 16 + (l & 15)) * g.K;
    uint16_t v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = t * 32 + (l >> 4) * 8 + e;
      v[e] = k < g.K ? wr[k] : static_cast<uint16_t>(0);
    }
    *reinterpret_cast<bf16x8_t*>(wl + idx * 8) = pack8(v);
  }
  for (int k = threadIdx.x; k < ksteps * 32; k += kThreads) taps[k] = tap_word(g, k);

  float ssum[TN], ssq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) ssum[j] = ssq[j] = 0.f;

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int m0 = tile * kBM;
    __syncthreads();  // the previous tile's epilogue is done with the staging buffer
    pf.commit(smem);
    const bool staged = pf.staged;
    const int64_t e0 = staged ? pf.e0 : 0;
    __syncthreads();
    if (tile + static_cast<int>(gridDim.x) < ntiles) {  // next tile's rows in flight during this one
      const int nt = tile + gridDim.x;
      pf.issue(g, nt * kBM, min(g.M, (nt + 1) * kBM) - 1);
    }
    Pix px[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) px[i].init(g, m0 + wave * 64 + i * 16 + (lane & 15), e0);
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // staged: the gather reads LDS (in-image taps lie in [e0, e1) by construction); otherwise global
    // memory.  Two inlined copies, so that each keeps its address space.
    auto body = [&](const uint16_t* src) {
      for (int t = 0; t < ksteps; ++t) {
        uint32_t tp[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) tp[e] = taps[t * 32 + kq * 8 + e];
        bf16x8_t bfr[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8_t*>(wl + ((t * TN + j) * 64 + lane) * 8);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          uint16_t v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = tap_value<NP>(g, src, px[i], tp[e]);
          const bf16x8_t af = pack8(v);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
        }
      }
    };
    if (staged)
      body(smem);
    else
      body(g.x);
    __syncthreads();  // every wave is done reading the patch: it becomes the C staging tile
    // rows >= M gathered zeros: they add nothing to the statistics
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float a = acc[i][j][r];
          ssum[j] += a;
          ssq[j] = fmaf(a, a, ssq[j]);
          smem[(wave * 64 + i * 16 + kq * 4 + r) * LDC + j * 16 + (lane & 15)] = f2bf(a);
        }
    __syncthreads();
    constexpr int CH = BN / 8;
    for (int v = threadIdx.x; v < kBM * CH; v += kThreads) {
      const int row = v / CH, ch = v - row * CH;
      if (m0 + row < g.M)
        *reinterpret_cast<uint4*>(y + static_cast<int64_t>(m0 + row) * ldy + ch * 8) =
            *reinterpret_cast<const uint4*>(smem + row * LDC + ch * 8);
    }
  }
  if (stats == nullptr) return;
  float* st = stats + shard_off(blockIdx.x, sstride);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    float a = ssum[j], q = ssq[j];
    a += __shfl_xor(a, 16, 64);
    a += __shfl_xor(a, 32, 64);
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    if (lane < 16) {
      atomicAdd(st + j * 16 + lane, a);
      atomicAdd(st + BN + j * 16 + lane, q);
    }
  }
}

// ------------------------------------------------------------------------------ weight grad --
// Each wave reduces 64 pixels of a 256-pixel chunk into the full CO x KW tile of its column group
// (blockIdx.y: GEMM columns [KW y, KW y + KW) of K, KW = 16 KB).  dY rows sit in LDS with a (CO + 4)-element
// pitch: the 8 rows a lane reads for one A fragment are 8 x pitch apart, which puts the four lane
// quarters on disjoint bank ranges (conflict-free ds_read_u16).  The next chunk's dY rows and input
// rows are loaded into registers while the current chunk computes.
template <int CO, int KB, bool NP>
__global__ __launch_bounds__(kThreads) void stem_wgrad_kernel(StemGeom g, const uint16_t* __restrict__ dy,
                                                              int64_t lddy, float* __restrict__ slab, int64_t n) {
  constexpr int PD = CO + 4;
  constexpr int CB = CO / 16;       // 16-row blocks of dW (output channels)
  constexpr int KW = KB * 16;       // dW columns per column group (blockIdx.y)
  constexpr int DYL = kBM * PD;     // dY staging elements
  constexpr int RED = CO * KW;      // fp32 fold tile
  constexpr int DV = kBM * CO / 8 / kThreads;  // 16-byte dY pieces per thread and chunk
  static_assert(RED * 4 <= (DYL + kPatch) * 2, "the fold tile reuses the staging buffers");
  __shared__ __attribute__((aligned(16))) uint16_t smem[DYL + kPatch];
  uint16_t* dyl = smem;
  uint16_t* patch = smem + DYL;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kq = lane >> 4;
  const int kcol0 = blockIdx.y * KW;
  const int kbn = min(KB, (g.K - kcol0 + 15) / 16);  // column blocks of this group inside K
  uint32_t tp[KB];  // this lane's B column per block is fixed for the whole kernel
#pragma unroll
  for (int b = 0; b < KB; ++b) tp[b] = tap_word(g, kcol0 + b * 16 + (lane & 15));

  f32x4 acc[CB][KB];
#pragma unroll
  for (int i = 0; i < CB; ++i)
#pragma unroll
    for (int j = 0; j < KB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = (g.M + kBM - 1) / kBM;
  RowPrefetch pf;
  uint4 dv[DV];
  auto issue = [&](int chunk) {
    const int m0 = chunk * kBM, rows = min(kBM, g.M - m0);
    pf.issue(g, m0, m0 + rows - 1);
#pragma unroll
    for (int i = 0; i < DV; ++i) {
      const int v = i * kThreads + threadIdx.x, r = v / (CO / 8), c8 = v % (CO / 8);
      dv[i] = r < rows ? *reinterpret_cast<const uint4*>(dy + static_cast<int64_t>(m0 + r) * lddy + c8 * 8)
                       : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  if (blockIdx.x < nchunks) issue(blockIdx.x);
  for (int chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    const int m0 = chunk * kBM;
    __syncthreads();  // the previous chunk's reads are done
#pragma unroll
    for (int i = 0; i < DV; ++i) {  // the padded pitch is 8-byte aligned: two 8-byte LDS writes
      const int v = i * kThreads + threadIdx.x, r = v / (CO / 8), c8 = v % (CO / 8);
      uint2* d = reinterpret_cast<uint2*>(dyl + r * PD + c8 * 8);
      d[0] = make_uint2(dv[i].x, dv[i].y);
      d[1] = make_uint2(dv[i].z, dv[i].w);
    }
    pf.commit(patch);
    const bool staged = pf.staged;
    const int64_t e0 = staged ? pf.e0 : 0;
    __syncthreads();
    if (chunk + static_cast<int>(gridDim.x) < nchunks) issue(chunk + gridDim.x);
    auto body = [&](const uint16_t* src) {
#pragma unroll
      for (int step = 0; step < 2; ++step) {
        const int p0 = wave * 64 + step * 32 + kq * 8;  // this lane's 8 pixels of the chunk
        bf16x8_t af[CB];
#pragma unroll
        for (int i = 0; i < CB; ++i) {
          uint16_t v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = dyl[(p0 + e) * PD + i * 16 + (lane & 15)];
          af[i] = pack8(v);
        }
        Pix px[8];
        px[0].init(g, m0 + p0, e0);
#pragma unroll
        for (int e = 1; e < 8; ++e) {
          px[e] = px[e - 1];
          px[e].next(g, m0 + p0 + e, e0);
        }
#pragma unroll
        for (int j = 0; j < KB; ++j) {
          if (j >= kbn) break;  // wave-uniform: column blocks past K
          uint16_t v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = tap_value<NP>(g, src, px[e], tp[j]);
          const bf16x8_t bfr = pack8(v);
#pragma unroll
          for (int i = 0; i < CB; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
        }
      }
    };
    if (staged)
      body(patch);
    else
      body(g.x);
  }

  // fold the four waves' tiles (LDS float adds) and store this workgroup's partial
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  for (int v = threadIdx.x; v < RED; v += kThreads) red[v] = 0.f;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < CB; ++i)
#pragma unroll
    for (int j = 0; j < KB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (j < kbn) atomicAdd(red + (i * 16 + kq * 4 + r) * KW + j * 16 + (lane & 15), acc[i][j][r]);
  __syncthreads();
  float* out = slab + static_cast<int64_t>(blockIdx.x) * n;
  const int kend = min(g.K, kcol0 + KW);
  for (int v = threadIdx.x; v < RED; v += kThreads) {
    const int co = v / KW, k = kcol0 + (v - co * KW);
    if (k < kend) out[static_cast<int64_t>(co) * g.K + k] = red[v];
  }
}

bool make_geom(StemGeom& g, const void* x, int N, int H, int W, int C, int Co, int R, int S, int sh, int sw, int ph,
               int pw, int OH, int OW) {
  if (x == nullptr || (reinterpret_cast<uintptr_t>(x) & 15) || N <= 0 || C <= 0 || C > 8 || (Co != 32 && Co != 64))
    return false;
  if (R <= 0 || S <= 0 || sh <= 0 || sw <= 0 || ph < 0 || pw < 0 || ph >= R || pw >= S) return false;
  if (OH != (H + 2 * ph - R) / sh + 1 || OW != (W + 2 * pw - S) / sw + 1 || OH <= 0 || OW <= 0) return false;
  const int64_t M = static_cast<int64_t>(N) * OH * OW;
  if (M >= (1 << 24) - kBM) return false;  // pixel indices exact in fp32 (fast_div)
  if (static_cast<int64_t>(N) * H * W >= (1 << 24)) return false;  // 24-bit pixel products (Pix::set)
  if (static_cast<int64_t>(R) * S * C > kMaxKSteps * 32 || (static_cast<int64_t>(R) * W + S) * C >= (1 << 20))
    return false;
  g = StemGeom{static_cast<const uint16_t*>(x), H, W, C, R, S, sh, sw, ph, pw, OH, OW, static_cast<int>(M),
               R * S * C, static_cast<int64_t>(N) * H * W * C, 1.f / static_cast<float>(OH * OW),
               1.f / static_cast<float>(OW)};
  return true;
}

}  // namespace

// Y[N*OH*OW, Co] (row stride ldy) = conv(X [N,H,W,C] dense NHWC bf16, C <= 8, W bf16 [Co][R][S][C]),
// Co = 32 or 64.  flags bit0: per-channel [sum | sumsq] of Y into stats (zero on entry;
// kStatShards copies sstride floats apart when sstride > 0), the layout tony_conv_fwd uses.
TONY_API int tony_stem_fwd(const void* x, int N, int H, int W, int C, const void* w, int Co, int R, int S, int sh,
                           int sw, int ph, int pw, void* y, int OH, int OW, int64_t ldy, int flags, float* stats,
                           int64_t sstride, int num_cus, hipStream_t stream) {
  StemGeom g;
  if (!make_geom(g, x, N, H, W, C, Co, R, S, sh, sw, ph, pw, OH, OW)) return -1;
  if (w == nullptr || y == nullptr || sstride < 0 || ldy < Co || (ldy % 8) || (reinterpret_cast<uintptr_t>(y) & 15))
    return -1;
  if ((flags & 1) && stats == nullptr) return -1;
  float* st = (flags & 1) ? stats : nullptr;
  const int ksteps = (g.K + 31) / 32;
  auto lds = [&](int bn) {
    const int stage = kPatch > kBM * (bn + 8) ? kPatch : kBM * (bn + 8);
    return static_cast<size_t>(stage + ksteps * (bn / 16) * 64 * 8) * sizeof(uint16_t);
  };
  // persistent: exactly the resident workgroups (occupancy query), each walking ~10 tiles at batch
  // 128 -- a grid larger than what fits would leave a tail of late workgroups
  static int occ_cache[2][kMaxKSteps + 1];  // per (Cout, K steps): the LDS size depends on both
  auto grid_for = [&](const void* fn, size_t bytes) {
    int& per_cu = occ_cache[Co == 64][ksteps];
    if (per_cu <= 0 &&
        (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kThreads, bytes) != hipSuccess || per_cu <= 0))
      per_cu = 2;
    return min(ceil_div(g.M, kBM), per_cu * (num_cus > 0 ? num_cus : 256));
  };
  const bool np = ph == 0 && pw == 0;
  const auto launch = [&](auto bn_c, auto np_c) {
    constexpr int BN = decltype(bn_c)::value;
    constexpr bool NP = decltype(np_c)::value;
    const size_t b = lds(BN);
    stem_fwd_kernel<BN, NP><<<grid_for(reinterpret_cast<const void*>(&stem_fwd_kernel<BN, NP>), b), kThreads, b,
                               stream>>>(g, static_cast<const uint16_t*>(w), static_cast<uint16_t*>(y), ldy, st, sstride);
  };
  using std::integral_constant;
  if (Co == 32)
    np ? launch(integral_constant<int, 32>{}, std::true_type{}) : launch(integral_constant<int, 32>{}, std::false_type{});
  else
    np ? launch(integral_constant<int, 64>{}, std::true_type{}) : launch(integral_constant<int, 64>{}, std::false_type{});
  TONY_LAUNCH_CHECK();
  return 0;
}

// Split-K weight gradient of the stem conv: workgroup s stores its partial dW ([Co][R][S][C],
// Co * K floats) to slab + s * Co*K; *splits receives the number of partials (<= 2 * num_cus) for
// tony_splitk_reduce.  dY rows [M][Co] with row stride lddy (16-byte aligned rows).
TONY_API int tony_stem_wgrad(const void* dy, int64_t lddy, const void* x, int N, int H, int W, int C, int Co, int R,
                             int S, int sh, int sw, int ph, int pw, int OH, int OW, float* slab, int64_t slab_cap,
                             int* splits, int num_cus, hipStream_t stream) {
  StemGeom g;
  if (!make_geom(g, x, N, H, W, C, Co, R, S, sh, sw, ph, pw, OH, OW)) return -1;
  if (dy == nullptr || slab == nullptr || splits == nullptr || num_cus <= 0 || lddy < Co || (lddy % 8) ||
      (reinterpret_cast<uintptr_t>(dy) & 15))
    return -1;
  const int64_t n = static_cast<int64_t>(Co) * g.K;
  const int nchunks = ceil_div(g.M, kBM);
  const bool k5 = Co == 64 && g.K > 64 && g.K <= 160;
  // persistent grid = the resident workgroups (occupancy query; <= 2 per CU): a second wave of
  // workgroups would only start when the first finishes its whole share of the chunks
  static int occ[3] = {0, 0, 0};
  const int which = k5 ? 2 : (Co == 64);
  if (occ[which] == 0) {
    const void* fn = k5 ? reinterpret_cast<const void*>(&stem_wgrad_kernel<64, 5, false>)
                        : Co == 64 ? reinterpret_cast<const void*>(&stem_wgrad_kernel<64, 4, false>)
                                   : reinterpret_cast<const void*>(&stem_wgrad_kernel<32, 4, false>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[which], fn, kThreads, 0) != hipSuccess || occ[which] <= 0)
      occ[which] = 1;
  }
  const int gx = min(nchunks, min(2, occ[which]) * num_cus);
  if (static_cast<int64_t>(gx) * n > slab_cap) return -1;
  // column groups of 64 (Inception's K = 27 fits one); a 7x7 RGB stem (K = 147) takes its 160 padded
  // columns in two groups of 5 blocks, so dY and the image are streamed twice instead of three times
  // (one group of 10 blocks spills: 160 accumulator registers)
  const bool np = ph == 0 && pw == 0;
  const auto launch = [&](auto co_c, auto kb_c, auto np_c, int gy) {
    stem_wgrad_kernel<decltype(co_c)::value, decltype(kb_c)::value, decltype(np_c)::value>
        <<<dim3(gx, gy), kThreads, 0, stream>>>(g, static_cast<const uint16_t*>(dy), lddy, slab, n);
  };
  using std::integral_constant;
  using I4 = integral_constant<int, 4>;
  if (k5)
    np ? launch(integral_constant<int, 64>{}, integral_constant<int, 5>{}, std::true_type{}, ceil_div(g.K, 80))
       : launch(integral_constant<int, 64>{}, integral_constant<int, 5>{}, std::false_type{}, ceil_div(g.K, 80));
  else if (Co == 32)
    np ? launch(integral_constant<int, 32>{}, I4{}, std::true_type{}, ceil_div(g.K, 64))
       : launch(integral_constant<int, 32>{}, I4{}, std::false_type{}, ceil_div(g.K, 64));
  else
    np ? launch(integral_constant<int, 64>{}, I4{}, std::true_type{}, ceil_div(g.K, 64))
       : launch(integral_constant<int, 64>{}, I4{}, std::false_type{}, ceil_div(g.K, 64));
  TONY_LAUNCH_CHECK();
  *splits = gx;
  return 0;
}
