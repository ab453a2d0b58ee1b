// Intra-node collectives over xGMI peer memory, the hand-written
// alternative to RCCL for one-process-per-GPU jobs: one-shot and two-shot all-reduce,
// reduce-scatter, all-gather and broadcast, bf16 or fp32, fp32 accumulation.
//
// Every rank owns one "window" that all peers map with hipIpcOpenMemHandle:
//
//   [flags: 2 phases x kMaxRanks x kMaxBlocks u32, error word | slot 0 | slot 1 | result 0 | result 1]
//
// Windows are fine-grained device memory (cached; hipDeviceMallocUncached with
// TONY_XGMI_MEM=uncached); every hand-off is a system-scope release (writer) / acquire (reader)
// around a per-workgroup flag barrier.
//
// Reductions PUSH: workgroup b of rank r writes chunk b of its input shard s straight into rank
// s's slot at row r (remote stores over the s<->r link; no copy of the input into the local
// window), meets workgroup b of every peer at a flag barrier, then reduces chunk b of its own shard
// from its own input and the peers' rows of its (local) slot.  Slot parity = epoch & 1, so
// back-to-back calls never overwrite a row a slow peer may still read: a rank can only start call
// k+2 after every peer passed call k+1's barrier, i.e. finished reading call k.
//
//   one-shot  (small): every rank pushes its whole buffer to every peer; each reduces all of it.
//   two-shot  (large): push reduce-scatter -> reduced shard into the local result region ->
//             barrier -> all-gather PULLED from every peer's result region (each GPU reads from all
//             7 links at once instead of one ring neighbour).
//   all-gather / broadcast: the own shard (1/n of the output) / the root's buffer is staged in
//             the local slot and every peer pulls it.
//
// Barriers spin with a bound: a peer that never arrives (crashed rank) makes the kernel record an
// error in the window's error word and exit instead of hanging the GPU; the host raises on it.
#include <cstring>

#include <cstdlib>

#include "common.h"

using namespace tony;

namespace {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 256;  // workgroups per collective launch
constexpr int64_t kFlagBytes = 2LL * kMaxRanks * kMaxBlocks * 4;
constexpr int64_t kHeader = 65536;  // flags (16 KiB) + error word, keeps the slots 64 KiB aligned
static_assert(kFlagBytes + 64 <= kHeader, "flags + error word fit the header");
constexpr int64_t kErrOff = kFlagBytes;
constexpr long kSpinLimit = 1L << 26;  // ~seconds of polling before a barrier gives up

struct Comm {
  uint8_t* win[kMaxRanks];  // window base of every rank as mapped in THIS process
  int rank, nranks;
  int64_t slot_bytes;
  long spin_limit;  // polls before a barrier gives up (kSpinLimit; TONY_XGMI_SPIN_LIMIT overrides)
};

__device__ __forceinline__ uint32_t* flags(uint8_t* w, int phase) {
  return reinterpret_cast<uint32_t*>(w) + phase * kMaxRanks * kMaxBlocks;
}
__device__ __forceinline__ uint8_t* slot(const Comm& c, int r, int which, uint32_t epoch) {
  return c.win[r] + kHeader + (static_cast<int64_t>(which) * 2 + (epoch & 1)) * c.slot_bytes;
}

// Workgroup b of this rank meets workgroup b of every peer.  Every thread's prior stores are made
// system-visible before the flag store; the poll is a system-scope acquire.
__device__ bool peer_barrier(const Comm& c, int phase, uint32_t epoch) {
  __threadfence_system();
  __syncthreads();
  __shared__ int ok;
  if (threadIdx.x == 0) ok = 1;
  __syncthreads();
  const int t = threadIdx.x;
  if (t < c.nranks) {
    uint32_t* remote = flags(c.win[t], phase) + c.rank * kMaxBlocks + blockIdx.x;
    __hip_atomic_store(remote, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = flags(c.win[c.rank], phase) + t * kMaxBlocks + blockIdx.x;
    long spins = 0;
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      if (++spins > c.spin_limit) {
        ok = 0;
        int* err = reinterpret_cast<int*>(c.win[c.rank] + kErrOff);
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  return ok != 0;
}

template <bool BF16>
struct Elem;
template <>
struct Elem<true> {  // 8 bf16 per 16-byte vector
  static constexpr int kVec = 8;
  __device__ static void load(const void* p, float* f) {
    bf16x8 v;
    v.raw = *reinterpret_cast<const uint4*>(p);
    v.to_float(f);
  }
  __device__ static void store(void* p, const float* f) { *reinterpret_cast<uint4*>(p) = bf16x8::from_float(f).raw; }
};
template <>
struct Elem<false> {  // 4 fp32 per 16-byte vector
  static constexpr int kVec = 4;
  __device__ static void load(const void* p, float* f) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    f[0] = v.x;
    f[1] = v.y;
    f[2] = v.z;
    f[3] = v.w;
  }
  __device__ static void store(void* p, const float* f) {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  }
};

// vectors [v0, v1) of a region split into gridDim.x chunks: this workgroup's chunk
__device__ __forceinline__ void chunk(int64_t nvec, int64_t* v0, int64_t* v1) {
  const int64_t per = (nvec + gridDim.x - 1) / gridDim.x;
  *v0 = min(nvec, per * blockIdx.x);
  *v1 = min(nvec, *v0 + per);
}

__device__ __forceinline__ void copy16(uint8_t* dst, const uint8_t* src, int64_t v0, int64_t v1) {
  for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x)
    reinterpret_cast<uint4*>(dst)[v] = reinterpret_cast<const uint4*>(src)[v];
}

// dst vectors [v0,v1) = scale * (sum over ranks p of row p of this rank's slot at off, own input for
// p == rank).  The terms are added in rank order on every rank, so a one-shot all-reduce gives
// bit-identical results everywhere (data-parallel replicas must not drift apart).
template <bool BF16>
__device__ void reduce_rows(const Comm& c, uint32_t epoch, const uint8_t* own, int64_t row_bytes, int64_t off,
                            uint8_t* dst, int64_t v0, int64_t v1, float scale) {
  using E = Elem<BF16>;
  const uint8_t* base = slot(c, c.rank, 0, epoch) + off;
  for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
    float acc[E::kVec], f[E::kVec];
#pragma unroll
    for (int j = 0; j < E::kVec; ++j) acc[j] = 0.f;
    for (int p = 0; p < c.nranks; ++p) {
      E::load(p == c.rank ? own + v * 16 : base + p * row_bytes + v * 16, f);
#pragma unroll
      for (int j = 0; j < E::kVec; ++j) acc[j] += f[j];
    }
#pragma unroll
    for (int j = 0; j < E::kVec; ++j) acc[j] *= scale;
    E::store(dst + v * 16, acc);
  }
}

// kind: 0 all-reduce one-shot, 1 all-reduce two-shot, 2 reduce-scatter, 3 all-gather, 4 broadcast
template <bool BF16>
__global__ __launch_bounds__(512) void xgmi_kernel(Comm c, int kind, const uint8_t* __restrict__ in,
                                                   uint8_t* __restrict__ out, int64_t bytes, int root, float scale,
                                                   uint32_t epoch) {
  const int64_t nvec = bytes / 16;
  int64_t v0, v1;
  uint8_t* my_slot = slot(c, c.rank, 0, epoch);
  if (kind == 0) {  // one-shot: push the whole buffer to row `rank` of every peer's slot
    chunk(nvec, &v0, &v1);
    for (int i = 1; i < c.nranks; ++i) {
      const int p = (c.rank + i) % c.nranks;  // stagger the peers so the 7 links are loaded evenly
      copy16(slot(c, p, 0, epoch) + static_cast<int64_t>(c.rank) * bytes, in, v0, v1);
    }
    if (!peer_barrier(c, 0, epoch)) return;
    reduce_rows<BF16>(c, epoch, in, bytes, 0, out, v0, v1, scale);
    return;
  }
  if (kind == 1 || kind == 2) {  // push reduce-scatter (+ pulled all-gather for two-shot); bytes = full input
    const int64_t svec = nvec / c.nranks;  // vectors per shard
    const int64_t sbytes = svec * 16;
    chunk(svec, &v0, &v1);
    for (int i = 1; i < c.nranks; ++i) {  // shard p of the input -> row `rank` of rank p's slot
      const int p = (c.rank + i) % c.nranks;
      copy16(slot(c, p, 0, epoch) + static_cast<int64_t>(c.rank) * sbytes, in + p * sbytes, v0, v1);
    }
    if (!peer_barrier(c, 0, epoch)) return;
    const int64_t off = static_cast<int64_t>(c.rank) * sbytes;
    if (kind == 2) {
      reduce_rows<BF16>(c, epoch, in + off, sbytes, 0, out, v0, v1, scale);
      return;
    }
    uint8_t* my_res = slot(c, c.rank, 1, epoch);
    reduce_rows<BF16>(c, epoch, in + off, sbytes, 0, my_res + off, v0, v1, scale);
    if (!peer_barrier(c, 1, epoch)) return;
    for (int r = 0; r < c.nranks; ++r) {
      const int p = (c.rank + r) % c.nranks;
      const int64_t o = static_cast<int64_t>(p) * sbytes;
      copy16(out + o, slot(c, p, 1, epoch) + o, v0, v1);
    }
    return;
  }
  if (kind == 3) {  // all-gather: bytes = one rank's shard
    chunk(nvec, &v0, &v1);
    copy16(my_slot, in, v0, v1);
    if (!peer_barrier(c, 0, epoch)) return;
    for (int r = 0; r < c.nranks; ++r) {
      const int p = (c.rank + r) % c.nranks;
      copy16(out + static_cast<int64_t>(p) * bytes, slot(c, p, 0, epoch), v0, v1);
    }
    return;
  }
  // broadcast from root
  chunk(nvec, &v0, &v1);
  if (c.rank == root) copy16(my_slot, in, v0, v1);
  if (!peer_barrier(c, 0, epoch)) return;
  copy16(out, slot(c, root, 0, epoch), v0, v1);
}

}  // namespace

TONY_API int64_t tony_xgmi_header_bytes() { return kHeader; }
TONY_API int tony_xgmi_max_ranks() { return kMaxRanks; }

// Window = header + 4 slots of slot_bytes, zeroed; *handle (64 B) exports it to the peers.
TONY_API int tony_xgmi_alloc(int64_t slot_bytes, void** window, void* handle) {
  if (slot_bytes <= 0 || (slot_bytes % 65536) || window == nullptr || handle == nullptr) return -1;
  const size_t total = static_cast<size_t>(kHeader + 4 * slot_bytes);
  const char* mem = std::getenv("TONY_XGMI_MEM");
  const bool uncached = mem != nullptr && std::strcmp(mem, "uncached") == 0;
  hipError_t e = hipExtMallocWithFlags(window, total, uncached ? hipDeviceMallocUncached : hipDeviceMallocFinegrained);
  if (e != hipSuccess) return static_cast<int>(e);
  e = hipMemset(*window, 0, total);
  if (e != hipSuccess) return static_cast<int>(e);
  e = hipIpcGetMemHandle(static_cast<hipIpcMemHandle_t*>(handle), *window);
  return static_cast<int>(e);
}

TONY_API int tony_xgmi_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return static_cast<int>(hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess));
}

TONY_API int tony_xgmi_close(void* ptr) { return static_cast<int>(hipIpcCloseMemHandle(ptr)); }
TONY_API int tony_xgmi_free(void* window) { return static_cast<int>(hipFree(window)); }
TONY_API int tony_xgmi_handle_bytes() { return static_cast<int>(sizeof(hipIpcMemHandle_t)); }

// Non-zero when a barrier of this rank timed out (a peer never arrived).  Synchronous; the error
// word is cleared after it has been read, so one failure is reported once.
TONY_API int tony_xgmi_error(void* window, int* err) {
  int* word = reinterpret_cast<int*>(static_cast<uint8_t*>(window) + kErrOff);
  hipError_t e = hipMemcpy(err, word, sizeof(int), hipMemcpyDeviceToHost);
  if (e == hipSuccess && *err != 0) e = hipMemset(word, 0, sizeof(int));
  return static_cast<int>(e);
}

// Stream-ordered copy of the error word into host memory (pinned): the host checks it before its
// next collective, so a timed-out barrier fails the run one call later without a device sync.
TONY_API int tony_xgmi_error_async(void* window, int* host_err, hipStream_t stream) {
  return static_cast<int>(hipMemcpyAsync(host_err, static_cast<uint8_t*>(window) + kErrOff, sizeof(int),
                                         hipMemcpyDeviceToHost, stream));
}

// windows: host array of nranks window pointers as mapped in this process (own window at [rank]).
// kind as xgmi_kernel; bytes: input bytes (multiple of 16; for reduce-scatter / two-shot a multiple
// of 16 * nranks; one-shot: nranks * bytes must fit a slot); scale multiplies the reduced sums
// (1/nranks for an average).  blocks: workgroups (<= 256), the SAME on every rank for a call.
TONY_API int tony_xgmi_collective(const uint64_t* windows, int rank, int nranks, int64_t slot_bytes, int kind,
                                  const void* in, void* out, int64_t bytes, int dtype_bf16, int root, float scale,
                                  uint32_t epoch, int blocks, hipStream_t stream) {
  if (nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks || kind < 0 || kind > 4) return -1;
  if (bytes <= 0 || (bytes % 16) || bytes > slot_bytes) return -1;
  if (kind == 0 && bytes * nranks > slot_bytes) return -1;  // one-shot: a row per rank
  if ((kind == 1 || kind == 2) && (bytes % (16LL * nranks))) return -1;
  if (((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) || epoch == 0) return -1;
  if (root < 0 || root >= nranks) return -1;
  Comm c{};
  for (int r = 0; r < nranks; ++r) {
    c.win[r] = reinterpret_cast<uint8_t*>(windows[r]);
    if (c.win[r] == nullptr) return -1;
  }
  c.rank = rank;
  c.nranks = nranks;
  c.slot_bytes = slot_bytes;
  c.spin_limit = kSpinLimit;
  if (const char* lim = std::getenv("TONY_XGMI_SPIN_LIMIT")) {
    const long v = std::strtol(lim, nullptr, 10);
    if (v > 0) c.spin_limit = v;
  }
  if (blocks < 1) blocks = 1;
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  if (dtype_bf16)
    xgmi_kernel<true><<<blocks, 512, 0, stream>>>(c, kind, static_cast<const uint8_t*>(in), static_cast<uint8_t*>(out),
                                                  bytes, root, scale, epoch);
  else
    xgmi_kernel<false><<<blocks, 512, 0, stream>>>(c, kind, static_cast<const uint8_t*>(in),
                                                   static_cast<uint8_t*>(out), bytes, root, scale, epoch);
  TONY_LAUNCH_CHECK();
  return 0;
}
