// Parameter-server data plane over xGMI peer memory: the paper topology of
// TonY's TF-PS jobs (1 ps + N workers, /root/reference/tony-examples/mnist-tensorflow/
// mnist_distributed.py:206-241) with the gradient fan-in, the optimizer apply and the variable
// fan-out all done by GPU kernels over IPC-mapped windows -- no RCCL reduce/broadcast rings.
//
// Windows (fine-grained device memory, hipIpcGetMemHandle, mapped by the peers):
//
//   every rank   [header 2 MiB: arrival flags [bucket][worker][block] u32 | landed flags
//                 [bucket][block] u32 | error word]
//   ps rank      + receive rows: nworkers x (wire bytes of every bucket this ps owns)
//   worker rank  + landing zone: the whole flat parameter buffer (param dtype)
//
// Per bucket b (owned by ps P) and step s (flag value s + 1, monotonic):
//
//   push   (worker w, its communication stream, as soon as backward finished b's gradients):
//          workgroup c copies chunk c of the gradient -- converted to the wire dtype on the fly --
//          straight into row w of P's receive rows (remote stores over the w<->P link), then
//          publishes arrival[b][w][c] in P's window (system-scope release).
//   apply  (P): workgroup c waits for chunk c of every worker's row (sync) and runs the fused
//          optimizer over it: sum of the rows (fp32) x grad_scale -> SGD / Adam on the fp32 master
//          and state -> the new variables are stored straight into EVERY worker's landing zone
//          (remote stores: P drives its 7 links at once) -> landed[b][c] in each worker's window.
//          Async (TF's default PS): workgroup c applies each worker's row on its own as it
//          arrives and lands the result only in THAT worker's zone (its pull sees its own push
//          and everything applied before it).
//   land   (worker, once per step after backward): workgroup (c, b) waits for landed[b][c] and
//          copies the chunk from the landing zone into the flat parameter buffer (a local copy;
//          the model's kernels keep reading coarse-grained HBM).
//
// Reuse of a row / landing chunk across steps is ordered by the protocol itself: a worker pushes
// b at step s+1 only after it landed b at step s, which P signals only after it read the rows.
// Every wait is bounded (wall clock): a peer that never arrives makes the waiter record an error
// in its own window's error word and exit, and the host raises -- no kernel spins forever.
#include <cstring>
#include <type_traits>

#include <algorithm>

#include "common.h"
#include "optim_math.h"

using namespace tony;

namespace {

constexpr int kMaxRanks = 8;
constexpr int kMaxBuckets = 128;
constexpr int kMaxBlocks = 256;  // workgroups per bucket (one per ~64 KiB: parallel/ps_plane.py blocks_for)
constexpr int kThreads = 256;
constexpr int64_t kArrivalOff = 0;
constexpr int64_t kLandedOff = kArrivalOff + 4LL * kMaxBuckets * kMaxRanks * kMaxBlocks;
constexpr int64_t kErrOff = kLandedOff + 4LL * kMaxBuckets * kMaxBlocks;
constexpr int64_t kHeader = 2 << 20;
static_assert(kErrOff + 64 <= kHeader, "flags + error word fit the header");

__device__ __forceinline__ uint32_t* arrival(uint8_t* win, int b, int w) {
  return reinterpret_cast<uint32_t*>(win + kArrivalOff) + (static_cast<int64_t>(b) * kMaxRanks + w) * kMaxBlocks;
}
__device__ __forceinline__ uint32_t* landed(uint8_t* win, int b) {
  return reinterpret_cast<uint32_t*>(win + kLandedOff) + static_cast<int64_t>(b) * kMaxBlocks;
}

// elements [lo, hi) of an n-element bucket handled by workgroup c of `blocks` (multiples of 8)
__device__ __forceinline__ void chunk_of(int64_t n, int c, int blocks, int64_t* lo, int64_t* hi) {
  const int64_t per = ((n + blocks - 1) / blocks + 7) / 8 * 8;
  *lo = min(n, per * c);
  *hi = min(n, *lo + per);
}

// 8 elements: one 16-byte access in bf16 (the remote landing-zone stores go over xGMI at full width),
// two in fp32
template <bool BF16>
__device__ __forceinline__ void load8(const void* base, int64_t i, float* f) {
  if constexpr (BF16) {
    const uint4 v = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(base) + i);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[2 * k] = __uint_as_float(w[k] << 16);
      f[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  } else {
    const float4 a = *reinterpret_cast<const float4*>(static_cast<const float*>(base) + i);
    const float4 b = *reinterpret_cast<const float4*>(static_cast<const float*>(base) + i + 4);
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
    f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
}

template <bool BF16>
__device__ __forceinline__ void store8(void* base, int64_t i, const float* f) {
  if constexpr (BF16) {
    uint4 v;
    v.x = static_cast<uint32_t>(f2bf(f[0])) | (static_cast<uint32_t>(f2bf(f[1])) << 16);
    v.y = static_cast<uint32_t>(f2bf(f[2])) | (static_cast<uint32_t>(f2bf(f[3])) << 16);
    v.z = static_cast<uint32_t>(f2bf(f[4])) | (static_cast<uint32_t>(f2bf(f[5])) << 16);
    v.w = static_cast<uint32_t>(f2bf(f[6])) | (static_cast<uint32_t>(f2bf(f[7])) << 16);
    *reinterpret_cast<uint4*>(static_cast<uint16_t*>(base) + i) = v;
  } else {
    *reinterpret_cast<float4*>(static_cast<float*>(base) + i) = make_float4(f[0], f[1], f[2], f[3]);
    *reinterpret_cast<float4*>(static_cast<float*>(base) + i + 4) = make_float4(f[4], f[5], f[6], f[7]);
  }
}

__device__ __forceinline__ void publish(uint32_t* flag, uint32_t value) {
  __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Poll *flag until it reaches value or the wall-clock budget runs out (then record the error).
__device__ __forceinline__ bool wait_flag(const uint32_t* flag, uint32_t value, uint64_t t0, uint64_t budget,
                                          int* err) {
  // wrap-safe: the counters are cumulative for the life of a job (a kvstore key of >= 4 MiB adds 1024 per
  // copy, so a u32 wraps after ~4.2M copies); the signed difference orders them while they are < 2^31 apart
  while (static_cast<int32_t>(__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - value) < 0) {
    if (wall_clock64() - t0 > budget) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  return true;
}

// ------------------------------------------------------------------------------------- push --
template <bool SRC_BF16, bool WIRE_BF16>
__global__ __launch_bounds__(kThreads) void ps_push_kernel(const void* __restrict__ g, void* __restrict__ row,
                                                           int64_t n, uint32_t* flags, uint32_t value) {
  int64_t lo, hi;
  chunk_of(n, blockIdx.x, gridDim.x, &lo, &hi);
  for (int64_t i = lo + threadIdx.x * 8; i < hi; i += kThreads * 8) {
    float f[8];
    load8<SRC_BF16>(g, i, f);
    store8<WIRE_BF16>(row, i, f);
  }
  __threadfence_system();  // the chunk is visible to the ps before its arrival flag
  __syncthreads();
  if (threadIdx.x == 0) publish(flags + blockIdx.x, value);
}

// ------------------------------------------------------------------------------------ apply --
struct ApplyArgs {
  const uint8_t* rows;      // receive row of worker 0 for this bucket (local window)
  int64_t row_stride;       // bytes between the rows of consecutive workers
  int nworkers;
  int64_t n;                // elements of the bucket
  float* master;            // fp32 master of the bucket (ps-local)
  float* s0;                // SGD momentum / Adam m
  float* s1;                // Adam v (unused for SGD)
  const float* hp;          // csrc/optim.hip hyper-parameter layout
  void* out[kMaxRanks];     // each worker's landing zone at the bucket (remote)
  void* local_out;          // the ps's own flat parameters at the bucket (may be null)
  uint32_t* arrivals;       // arrival[b][0][0] in the ps window (local)
  uint32_t* landed_at[kMaxRanks];  // landed[b][0] in every worker window (remote)
  uint32_t value;
  uint64_t budget;          // wall-clock ticks a workgroup may wait for a worker
  int* err;                 // the ps window's error word
};

template <int OPT, bool WIRE_BF16, bool PARAM_BF16>
__device__ __forceinline__ void update4(const ApplyArgs& a, int64_t i, const float* g, float* wf_out) {
  const float* hp = a.hp;
  float4 wv = *reinterpret_cast<float4*>(a.master + i);
  float wf[4] = {wv.x, wv.y, wv.z, wv.w};
  float4 mv = *reinterpret_cast<float4*>(a.s0 + i);
  float mf[4] = {mv.x, mv.y, mv.z, mv.w};
  if constexpr (OPT == 0) {
    sgd_update4(wf, mf, g, hp[0], hp[1], hp[2], hp[3], hp[4] != 0.f);
  } else {
    float4 vv = *reinterpret_cast<float4*>(a.s1 + i);
    float vf[4] = {vv.x, vv.y, vv.z, vv.w};
    adam_update4(wf, mf, vf, g, hp[0], hp[1], hp[2], hp[3], hp[4], hp[5], hp[0] / hp[6], rsqrtf(hp[7]),
                 hp[8] != 0.f);
    *reinterpret_cast<float4*>(a.s1 + i) = make_float4(vf[0], vf[1], vf[2], vf[3]);
  }
  *reinterpret_cast<float4*>(a.master + i) = make_float4(wf[0], wf[1], wf[2], wf[3]);
  *reinterpret_cast<float4*>(a.s0 + i) = make_float4(mf[0], mf[1], mf[2], mf[3]);
#pragma unroll
  for (int k = 0; k < 4; ++k) wf_out[k] = wf[k];
}

// elements [i, i + 8): the optimizer on the fp32 master / state, then the new variables stored
// (16-byte bf16 stores) into the ps's own parameters and every worker's landing zone, or only
// worker `only`'s (async)
template <int OPT, bool WIRE_BF16, bool PARAM_BF16>
__device__ __forceinline__ void update8(const ApplyArgs& a, int64_t i, const float* g, int only) {
  float wf[8];
  update4<OPT, WIRE_BF16, PARAM_BF16>(a, i, g, wf);
  update4<OPT, WIRE_BF16, PARAM_BF16>(a, i + 4, g + 4, wf + 4);
  if (a.local_out != nullptr) store8<PARAM_BF16>(a.local_out, i, wf);
  if (only >= 0) {
    store8<PARAM_BF16>(a.out[only], i, wf);
  } else {
    for (int w = 0; w < a.nworkers; ++w) store8<PARAM_BF16>(a.out[w], i, wf);
  }
}

// A rank whose wait timed out has set its window's error word: its later kernels do nothing (no
// flag of a later step can then satisfy an earlier step's wait, and nothing is stored from a
// half-applied step) until the host has raised (XgmiPSPlane marks itself unusable).
__device__ __forceinline__ bool poisoned(const int* err) {
  return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

template <int OPT, bool WIRE_BF16, bool PARAM_BF16>
__global__ __launch_bounds__(kThreads) void ps_apply_sync_kernel(ApplyArgs a) {
  __shared__ int ok;
  const uint64_t t0 = wall_clock64();
  if (threadIdx.x == 0) ok = !poisoned(a.err);
  __syncthreads();
  if (!ok) return;
  if (threadIdx.x < a.nworkers &&
      !wait_flag(a.arrivals + threadIdx.x * kMaxBlocks + blockIdx.x, a.value, t0, a.budget, a.err))
    ok = 0;
  __syncthreads();
  if (!ok) return;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  int64_t lo, hi;
  chunk_of(a.n, blockIdx.x, gridDim.x, &lo, &hi);
  for (int64_t i = lo + threadIdx.x * 8; i < hi; i += kThreads * 8) {
    float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, f[8];
    for (int w = 0; w < a.nworkers; ++w) {
      load8<WIRE_BF16>(a.rows + w * a.row_stride, i, f);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] += f[k];
    }
    update8<OPT, WIRE_BF16, PARAM_BF16>(a, i, g, -1);
  }
  __threadfence_system();  // the new variables reach every landing zone before the flags
  __syncthreads();
  if (threadIdx.x < a.nworkers) publish(a.landed_at[threadIdx.x] + blockIdx.x, a.value);
}

// Asynchronous PS: each worker's push is applied on its own, in the order this workgroup sees them
// arrive, and only that worker's landing zone receives the result.
template <int OPT, bool WIRE_BF16, bool PARAM_BF16>
__global__ __launch_bounds__(kThreads) void ps_apply_async_kernel(ApplyArgs a) {
  __shared__ int next;
  const uint64_t t0 = wall_clock64();
  uint32_t pending = poisoned(a.err) ? 0u : (1u << a.nworkers) - 1u;
  int64_t lo, hi;
  chunk_of(a.n, blockIdx.x, gridDim.x, &lo, &hi);
  while (pending) {
    if (threadIdx.x == 0) {
      next = -1;
      while (next < 0) {
        for (int w = 0; w < a.nworkers && next < 0; ++w)
          if ((pending >> w) & 1u &&
              __hip_atomic_load(a.arrivals + w * kMaxBlocks + blockIdx.x, __ATOMIC_ACQUIRE,
                                __HIP_MEMORY_SCOPE_SYSTEM) >= a.value)
            next = w;
        if (next >= 0) break;
        if (wall_clock64() - t0 > a.budget) {
          __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          next = kMaxRanks;  // give up
          break;
        }
        __builtin_amdgcn_s_sleep(8);
      }
    }
    __syncthreads();
    const int w = next;
    __syncthreads();  // every thread read `next` before thread 0 may overwrite it
    if (w >= kMaxRanks) return;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    for (int64_t i = lo + threadIdx.x * 8; i < hi; i += kThreads * 8) {
      float g[8];
      load8<WIRE_BF16>(a.rows + w * a.row_stride, i, g);
      update8<OPT, WIRE_BF16, PARAM_BF16>(a, i, g, w);
    }
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) publish(a.landed_at[w] + blockIdx.x, a.value);
    pending &= ~(1u << w);
  }
}

// ------------------------------------------------------------------------------------- land --
struct LandEntry {
  int64_t lo;    // first element of the bucket in the flat buffer
  int64_t n;     // elements
  int32_t blocks;
  int32_t bucket;
};

// A bounded persistent grid (<= one workgroup per CU) walks the (bucket, chunk) pairs in table order --
// the order the ps applies them -- waiting for each chunk's landed flag and copying it.  One workgroup per
// chunk (the first form) parked up to nb x 256 spinning workgroups on the GPU: on a GPU shared by a ps
// and workers (the one-GPU rehearsal, tony.amd.ps-share-gpu) two workers' landings of the 12 fp32
// Inception buckets filled every workgroup slot and the ps's apply never got a CU (deadlock until the
// wait budget ran out).  Spinning workgroups are now bounded by the grid, whatever the bucket count.
template <bool PARAM_BF16>
__global__ __launch_bounds__(kThreads) void ps_land_kernel(const LandEntry* __restrict__ tab, int nb, uint8_t* win,
                                                           const uint8_t* landing, uint8_t* dst, uint32_t value,
                                                           uint64_t budget) {
  __shared__ int ok;
  const uint64_t t0 = wall_clock64();
  int* err = reinterpret_cast<int*>(win + kErrOff);
  if (threadIdx.x == 0) ok = !poisoned(err);
  __syncthreads();
  if (!ok) return;
  const int64_t G = gridDim.x;
  int64_t base = 0;  // pairs before entry y
  constexpr int esz = PARAM_BF16 ? 2 : 4;
  for (int y = 0; y < nb; ++y) {
    const LandEntry e = tab[y];
    const int64_t p0 = base + ((static_cast<int64_t>(blockIdx.x) - base) % G + G) % G;  // first pair of ours
    for (int64_t p = p0; p < base + e.blocks; p += G) {
      const int c = static_cast<int>(p - base);
      if (threadIdx.x == 0) ok = wait_flag(landed(win, e.bucket) + c, value, t0, budget, err);
      __syncthreads();
      if (!ok) return;  // (uniform: every thread read ok after the barrier)
      __atomic_thread_fence(__ATOMIC_ACQUIRE);
      int64_t lo, hi;
      chunk_of(e.n, c, e.blocks, &lo, &hi);
      const int64_t b0 = (e.lo + lo) * esz, b1 = (e.lo + hi) * esz;  // 16-byte multiples (lo, hi: x8)
      for (int64_t o = b0 + threadIdx.x * 16; o < b1; o += kThreads * 16)
        *reinterpret_cast<uint4*>(dst + o) = *reinterpret_cast<const uint4*>(landing + o);
      __syncthreads();  // thread 0 rewrites ok for the next pair only after every thread tested this one
    }
    base += e.blocks;
  }
}

uint64_t budget_ticks(double seconds) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) !=
                                              hipSuccess || khz <= 0)
    khz = 100000;  // 100 MHz, the gfx9 constant clock
  return static_cast<uint64_t>(seconds * khz * 1000.0);
}

// The kvstore payload plane (parallel/kvstore.py): one key's bytes between a local tensor and a peer's
// IPC-mapped window (either side may be the peer), 16 B per lane, the < 16 B tail by lane 0 of block 0.
// err (nullable): the error word of the window a preceding kv_wait guarded -- a timed-out wait poisons
// the copy behind it (stale or partial bytes are never moved; the host raises at its next check)
__global__ __launch_bounds__(256) void kv_copy_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                       int64_t bytes, const int* err) {
  if (err != nullptr && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return;
  const int64_t n16 = bytes >> 4;
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(dst);
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n16;
       i += static_cast<int64_t>(gridDim.x) * 256)
    d[i] = s[i];
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (int64_t i = n16 << 4; i < bytes; ++i) dst[i] = src[i];
}

// kvstore hand-off with a device flag: the copy above, then every workgroup publishes its part with a
// system-scope fence and one add to a u32 counter in the consumer's window (a peer's: the adds go over
// xGMI).  The consumer learns the whole copy landed when the counter reaches its expected total
// (kv_copy_blocks per copy, cumulative), without a host synchronisation on either side.
__global__ __launch_bounds__(256) void kv_copy_flag_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                            int64_t bytes, uint32_t* flag) {
  const int64_t n16 = bytes >> 4;
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(dst);
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n16;
       i += static_cast<int64_t>(gridDim.x) * 256)
    d[i] = s[i];
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (int64_t i = n16 << 4; i < bytes; ++i) dst[i] = src[i];
  __threadfence_system();  // this workgroup's bytes are visible to the consumer before its add
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the consumer side: one wave waits (bounded) until *flag reaches target; the stream's next kernel (the
// copy out of the window) then reads bytes that landed.  A timeout records the error word and returns.
__global__ __launch_bounds__(64) void kv_wait_kernel(const uint32_t* flag, uint32_t target, uint64_t budget, int* err) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  wait_flag(flag, target, t0, budget, err);
}

int kv_copy_blocks(int64_t bytes) {
  const int64_t n16 = (bytes >> 4) + 1;
  return static_cast<int>(std::min<int64_t>(1024, (n16 + 255) / 256));
}

}  // namespace

// workgroups of one flagged copy of `bytes` (the consumer's counter target grows by this per copy)
TONY_API int tony_kv_copy_blocks(int64_t bytes) { return bytes <= 0 ? 0 : kv_copy_blocks(bytes); }

// dst <- src and a flag add per workgroup (tony_kv_copy_blocks(bytes) adds in all) into *flag
TONY_API int tony_kv_copy_flag(void* dst, const void* src, int64_t bytes, void* flag, hipStream_t stream) {
  if (dst == nullptr || src == nullptr || flag == nullptr || bytes <= 0 || (reinterpret_cast<uintptr_t>(dst) & 15) ||
      (reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(flag) & 3))
    return -1;
  kv_copy_flag_kernel<<<kv_copy_blocks(bytes), 256, 0, stream>>>(static_cast<const uint8_t*>(src),
                                                                 static_cast<uint8_t*>(dst), bytes,
                                                                 static_cast<uint32_t*>(flag));
  TONY_LAUNCH_CHECK();
  return 0;
}

// stream-ordered wait until the u32 counter at *flag (in this rank's window) reaches target; a wait
// longer than budget_s records the error word of `window` (tony_ps_error reads it)
TONY_API int tony_kv_wait(const void* flag, uint32_t target, void* window, double budget_s, hipStream_t stream) {
  if (flag == nullptr || window == nullptr || (reinterpret_cast<uintptr_t>(flag) & 3)) return -1;
  kv_wait_kernel<<<1, 64, 0, stream>>>(static_cast<const uint32_t*>(flag), target, budget_ticks(budget_s),
                                       reinterpret_cast<int*>(static_cast<uint8_t*>(window) + kErrOff));
  TONY_LAUNCH_CHECK();
  return 0;
}

// dst <- src (bytes), both 16-B aligned device addresses (local memory or a mapped peer window); window
// (nullable): skip the copy when that window's error word is set (a timed-out wait ahead of it)
TONY_API int tony_kv_copy(void* dst, const void* src, int64_t bytes, void* window, hipStream_t stream) {
  if (dst == nullptr || src == nullptr || bytes < 0 || (reinterpret_cast<uintptr_t>(dst) & 15) ||
      (reinterpret_cast<uintptr_t>(src) & 15))
    return -1;
  if (bytes == 0) return 0;
  const int64_t n16 = (bytes >> 4) + 1;
  const int blocks = static_cast<int>(std::min<int64_t>(1024, (n16 + 255) / 256));
  kv_copy_kernel<<<blocks, 256, 0, stream>>>(
      static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst), bytes,
      window == nullptr ? nullptr : reinterpret_cast<const int*>(static_cast<const uint8_t*>(window) + kErrOff));
  TONY_LAUNCH_CHECK();
  return 0;
}

TONY_API int64_t tony_ps_header_bytes() { return kHeader; }
TONY_API int tony_ps_max_buckets() { return kMaxBuckets; }
TONY_API int tony_ps_max_blocks() { return kMaxBlocks; }
TONY_API int tony_ps_land_entry_bytes() { return static_cast<int>(sizeof(LandEntry)); }

// Window of header + payload bytes (fine-grained, zeroed); *handle receives its IPC handle.
TONY_API int tony_ps_window_alloc(int64_t payload, void** window, void* handle) {
  if (payload < 0 || window == nullptr || handle == nullptr) return -1;
  const size_t total = static_cast<size_t>(kHeader + (payload + 65535) / 65536 * 65536);
  hipError_t e = hipExtMallocWithFlags(window, total, hipDeviceMallocFinegrained);
  if (e != hipSuccess) return static_cast<int>(e);
  e = hipMemset(*window, 0, total);
  if (e != hipSuccess) return static_cast<int>(e);
  e = hipIpcGetMemHandle(static_cast<hipIpcMemHandle_t*>(handle), *window);
  return static_cast<int>(e);
}

// Worker: push n elements (multiple of 8) of bucket b's gradient into row `widx` of the ps window.
TONY_API int tony_ps_push(const void* grad, int grad_bf16, void* ps_window, int64_t row_off, int wire_bf16,
                          int64_t n, int bucket, int widx, uint32_t value, int blocks, hipStream_t stream) {
  if (grad == nullptr || ps_window == nullptr || n <= 0 || (n % 8) || bucket < 0 || bucket >= kMaxBuckets ||
      widx < 0 || widx >= kMaxRanks || blocks < 1 || blocks > kMaxBlocks || value == 0 || row_off < 0 ||
      (row_off % 16) || (reinterpret_cast<uintptr_t>(grad) & 15))
    return -1;
  uint8_t* win = static_cast<uint8_t*>(ps_window);
  void* row = win + kHeader + row_off;
  uint32_t* flags = reinterpret_cast<uint32_t*>(win + kArrivalOff) +
                    (static_cast<int64_t>(bucket) * kMaxRanks + widx) * kMaxBlocks;
  const auto go = [&](auto src_c, auto wire_c) {
    ps_push_kernel<decltype(src_c)::value, decltype(wire_c)::value>
        <<<blocks, kThreads, 0, stream>>>(grad, row, n, flags, value);
  };
  using T = std::true_type;
  using F = std::false_type;
  if (grad_bf16)
    wire_bf16 ? go(T{}, T{}) : go(T{}, F{});
  else
    wire_bf16 ? go(F{}, T{}) : go(F{}, F{});
  TONY_LAUNCH_CHECK();
  return 0;
}

// PS: apply bucket b.  landings: nworkers landing-zone base pointers (remote windows, payload
// offset 0 = flat element 0) and worker windows (for the landed flags); lo: the bucket's first
// element in the flat buffer; rows_off: byte offset of worker 0's row of b in this window's payload.
TONY_API int tony_ps_apply(void* ps_window, int64_t rows_off, int64_t row_stride, int nworkers, int wire_bf16,
                           int64_t n, int64_t lo, float* master, float* s0, float* s1, const float* hp, int opt,
                           const uint64_t* worker_windows, void* local_params, int param_bf16, int bucket,
                           uint32_t value, int async_mode, double budget_s, int blocks, hipStream_t stream) {
  if (ps_window == nullptr || nworkers < 1 || nworkers > kMaxRanks || n <= 0 || (n % 8) || lo < 0 || (lo % 8) ||
      master == nullptr || s0 == nullptr || hp == nullptr || (opt == 1 && s1 == nullptr) || opt < 0 || opt > 1 ||
      bucket < 0 || bucket >= kMaxBuckets || value == 0 || blocks < 1 || blocks > kMaxBlocks ||
      (row_stride % 16) || (rows_off % 16) || worker_windows == nullptr)
    return -1;
  if ((reinterpret_cast<uintptr_t>(master) | reinterpret_cast<uintptr_t>(s0)) & 15) return -1;
  uint8_t* win = static_cast<uint8_t*>(ps_window);
  ApplyArgs a{};
  a.rows = win + kHeader + rows_off;
  a.row_stride = row_stride;
  a.nworkers = nworkers;
  a.n = n;
  a.master = master;
  a.s0 = s0;
  a.s1 = s1;
  a.hp = hp;
  const int esz = param_bf16 ? 2 : 4;
  for (int w = 0; w < nworkers; ++w) {
    uint8_t* ww = reinterpret_cast<uint8_t*>(worker_windows[w]);
    if (ww == nullptr) return -1;
    a.out[w] = ww + kHeader + lo * esz;
    a.landed_at[w] = reinterpret_cast<uint32_t*>(ww + kLandedOff) + static_cast<int64_t>(bucket) * kMaxBlocks;
  }
  a.local_out = local_params == nullptr ? nullptr : static_cast<uint8_t*>(local_params) + lo * esz;
  a.arrivals = reinterpret_cast<uint32_t*>(win + kArrivalOff) + static_cast<int64_t>(bucket) * kMaxRanks * kMaxBlocks;
  a.value = value;
  a.budget = budget_ticks(budget_s);
  a.err = reinterpret_cast<int*>(win + kErrOff);
  const auto go = [&](auto opt_c, auto wire_c, auto par_c) {
    constexpr int O = decltype(opt_c)::value;
    constexpr bool W = decltype(wire_c)::value, P = decltype(par_c)::value;
    if (async_mode)
      ps_apply_async_kernel<O, W, P><<<blocks, kThreads, 0, stream>>>(a);
    else
      ps_apply_sync_kernel<O, W, P><<<blocks, kThreads, 0, stream>>>(a);
  };
  using T = std::true_type;
  using F = std::false_type;
  using O0 = std::integral_constant<int, 0>;
  using O1 = std::integral_constant<int, 1>;
  if (opt == 0) {
    if (wire_bf16)
      param_bf16 ? go(O0{}, T{}, T{}) : go(O0{}, T{}, F{});
    else
      param_bf16 ? go(O0{}, F{}, T{}) : go(O0{}, F{}, F{});
  } else {
    if (wire_bf16)
      param_bf16 ? go(O1{}, T{}, T{}) : go(O1{}, T{}, F{});
    else
      param_bf16 ? go(O1{}, F{}, T{}) : go(O1{}, F{}, F{});
  }
  TONY_LAUNCH_CHECK();
  return 0;
}

// Worker: wait for every bucket of `table` (device array of nb LandEntry) to land and copy the
// landing zone into the flat parameters.
TONY_API int tony_ps_land(void* window, const void* table, int nb, void* params, int param_bf16, uint32_t value,
                          double budget_s, hipStream_t stream) {
  if (window == nullptr || table == nullptr || nb < 1 || nb > kMaxBuckets || params == nullptr || value == 0 ||
      (reinterpret_cast<uintptr_t>(params) & 15))
    return -1;
  uint8_t* win = static_cast<uint8_t*>(window);
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess || cus <= 0)
    cus = 64;
  // <= one workgroup per CU (see ps_land_kernel), never more than the pairs can use
  const int grid = std::min<int>(cus, nb * kMaxBlocks);
  const uint64_t budget = budget_ticks(budget_s);
  if (param_bf16)
    ps_land_kernel<true><<<grid, kThreads, 0, stream>>>(static_cast<const LandEntry*>(table), nb, win,
                                                        win + kHeader, static_cast<uint8_t*>(params), value, budget);
  else
    ps_land_kernel<false><<<grid, kThreads, 0, stream>>>(static_cast<const LandEntry*>(table), nb, win,
                                                         win + kHeader, static_cast<uint8_t*>(params), value, budget);
  TONY_LAUNCH_CHECK();
  return 0;
}

// Stream-ordered copy of this window's error word into (pinned) host memory, and its synchronous
// read-and-clear (non-zero: a wait of this rank timed out; the step's variables are invalid).
TONY_API int tony_ps_error_async(void* window, int* host_err, hipStream_t stream) {
  return static_cast<int>(hipMemcpyAsync(host_err, static_cast<uint8_t*>(window) + kErrOff, sizeof(int),
                                         hipMemcpyDeviceToHost, stream));
}
TONY_API int tony_ps_error(void* window, int* err) {
  int* word = reinterpret_cast<int*>(static_cast<uint8_t*>(window) + kErrOff);
  hipError_t e = hipMemcpy(err, word, sizeof(int), hipMemcpyDeviceToHost);
  if (e == hipSuccess && *err != 0) e = hipMemset(word, 0, sizeof(int));
  return static_cast<int>(e);
}
