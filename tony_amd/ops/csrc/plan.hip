// Native step replay: a captured training step re-issued from C++ ("HIP streams and
// graphs instead of a tracing compiler").
//
// Why not hipGraphLaunch: the Inception-v3 step is ~600 kernels over 4 streams (compute, weight
// gradients, two branch streams).  Replayed as an instantiated HIP graph it cost ~11 ms of host time
// per launch and ran 5-10% slower on the GPU than the same step issued eagerly (bench.py
// mode_setup_ms); issued eagerly from Python it costs ~11 ms of host time (autograd + ~600 fast-call
// launches).  Here the step is captured ONCE into a hipGraph (torch.cuda.graph with keep_graph, never
// instantiated), the graph is walked, and its nodes are re-issued in capture order onto the SAME
// streams structure the eager step used:
//   * topological order = capture order (Kahn with the node list index as priority), so the issue
//     order matches the eager step that was measured and tuned;
//   * stream assignment by chain extension with vector clocks: a node goes to the stream whose tail
//     is one of its dependencies (the eager stream it came from, in practice); a fork with no such
//     stream takes a stream whose tail it already (transitively) depends on, so no false dependency
//     is introduced; only when every stream would add one does it take the least recently fed;
//   * cross-stream edges become hipEventRecord / hipStreamWaitEvent pairs, elided when the waiting
//     stream already (transitively) waited for that point -- vector clocks again;
//   * kernel nodes replay with hipModuleLaunchKernel on the node's own argument storage (the graph object
//     stays alive), memset / memcpy nodes with their async calls, empty nodes are folded into the
//     dependency lists.
// Marker kernels (tony_plan_mark) captured at points the host must act on -- a gradient bucket whose
// collective runs outside the graph -- split the plan into segments: tony_plan_replay(h, seg, ..)
// issues the ops up to that marker and forks the marker's stream into the caller's side stream.
#include <algorithm>
#include <array>
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace {

__global__ void plan_marker_kernel(int) {}

constexpr int kMaxStreams = 8;

enum OpKind : int { kKernel = 0, kMemset = 1, kMemcpy = 2, kWait = 3, kRecord = 4, kMarker = 5, kGraph = 6 };

struct Op {
  int kind;
  int stream;
  int event;   // kWait / kRecord / kMarker: index into Plan::events
  int marker;  // kMarker: marker id
  hipKernelNodeParams k;
  hipFunction_t fn;  // the device function (resolved once from the captured host stub)
  hipMemsetParams ms;
  hipMemcpy3DParms mc;
  hipGraphExec_t ex;  // kGraph: a one-node executable graph (nodes without a direct re-issue call)
};

struct Plan {
  std::vector<Op> ops;
  std::vector<hipEvent_t> events;  // [0]: replay start on stream 0; [1..]: cross-stream points
  hipStream_t streams[kMaxStreams] = {};
  int nstreams = 0;
  int used[kMaxStreams] = {};
  std::vector<int> tails;            // per stream: event recorded after its last op (joined at the end)
  std::vector<int> seg_end;          // op index one past each marker (segment k = [seg_end[k-1], seg_end[k]))
  int stats[11] = {};
  int fail_op = -1, fail_kind = -1, fail_stream = -1;  // the op whose issue failed last (tony_plan_failure)
};

int new_event(Plan& p) {
  hipEvent_t e;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return -1;
  p.events.push_back(e);
  return static_cast<int>(p.events.size()) - 1;
}

void destroy(Plan* p) {
  for (hipEvent_t e : p->events) (void)hipEventDestroy(e);
  for (Op& o : p->ops)
    if (o.kind == kGraph && o.ex != nullptr) (void)hipGraphExecDestroy(o.ex);
  delete p;
}

// A node without a direct re-issue call (a copy captured from hipMemcpyAsync is a 1D node whose
// parameters no getter returns) becomes a one-node executable graph: the captured graph cloned, every
// other node removed, instantiated.  Launched with hipGraphLaunch on the node's stream.
hipGraphExec_t single_node_exec(hipGraph_t g, hipGraphNode_t node) {
  hipGraph_t clone = nullptr;
  if (hipGraphClone(&clone, g) != hipSuccess) return nullptr;
  hipGraphNode_t target = nullptr;
  hipGraphExec_t ex = nullptr;
  size_t cn = 0;
  if (hipGraphNodeFindInClone(&target, node, clone) == hipSuccess && hipGraphGetNodes(clone, nullptr, &cn) == hipSuccess) {
    std::vector<hipGraphNode_t> all(cn);
    bool ok = cn == 0 || hipGraphGetNodes(clone, all.data(), &cn) == hipSuccess;
    for (size_t i = 0; ok && i < cn; ++i)
      if (all[i] != target) ok = hipGraphDestroyNode(all[i]) == hipSuccess;
    if (ok && hipGraphInstantiate(&ex, clone, nullptr, nullptr, 0) != hipSuccess) ex = nullptr;
  }
  (void)hipGraphDestroy(clone);
  return ex;
}

hipError_t issue(const Plan& p, const Op& o, hipStream_t side) {
  hipStream_t s = p.streams[o.stream];
  switch (o.kind) {
    case kKernel:
      return hipModuleLaunchKernel(o.fn, o.k.gridDim.x, o.k.gridDim.y, o.k.gridDim.z, o.k.blockDim.x, o.k.blockDim.y,
                                   o.k.blockDim.z, o.k.sharedMemBytes, s, o.k.kernelParams, o.k.extra);
    case kMemset: {
      const hipMemsetParams& m = o.ms;
      if (m.height <= 1) {
        if (m.elementSize == 4) return hipMemsetD32Async(m.dst, static_cast<int>(m.value), m.width, s);
        if (m.elementSize == 2) return hipMemsetD16Async(m.dst, static_cast<unsigned short>(m.value), m.width, s);
        return hipMemsetD8Async(m.dst, static_cast<unsigned char>(m.value), m.width, s);
      }
      if (m.elementSize != 1) return hipErrorNotSupported;
      return hipMemset2DAsync(m.dst, m.pitch, static_cast<int>(m.value), m.width, m.height, s);
    }
    case kMemcpy:
      return hipMemcpy3DAsync(&o.mc, s);
    case kWait:
      return hipStreamWaitEvent(s, p.events[o.event], 0);
    case kRecord:
      return hipEventRecord(p.events[o.event], s);
    case kGraph:
      return hipGraphLaunch(o.ex, s);
    case kMarker: {
      hipError_t e = hipEventRecord(p.events[o.event], s);
      if (e == hipSuccess && side != nullptr) e = hipStreamWaitEvent(side, p.events[o.event], 0);
      return e;
    }
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace

// The marker kernel's launch (captured as a kernel node and recognised by its function).
TONY_API int tony_plan_mark(int id, hipStream_t stream) {
  plan_marker_kernel<<<1, 1, 0, stream>>>(id);
  TONY_LAUNCH_CHECK();
  return 0;
}

// Build a replay plan from a captured graph.  streams[0] must be the stream the replay is issued on
// (the capture's origin stream); streams[1..n) are side streams the plan may use (n <= 8).
// stats (10 ints): kernels, memsets, memcpys, waits, records, streams used, markers, graph nodes,
// placements that had to take a false dependency, empty nodes folded, nodes issued as one-node graphs.
// Returns 0 and the handle in *out; negative: unsupported graph (the caller keeps its own path).
TONY_API int tony_plan_build(void* graph, const uint64_t* streams, int nstreams, uint64_t* out, int* stats) {
  if (graph == nullptr || streams == nullptr || out == nullptr || nstreams < 1 || nstreams > kMaxStreams) return -1;
  hipGraph_t g = static_cast<hipGraph_t>(graph);
  size_t n = 0;
  if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess) return -2;
  std::vector<hipGraphNode_t> nodes(n);
  if (n > 0 && hipGraphGetNodes(g, nodes.data(), &n) != hipSuccess) return -2;
  std::unordered_map<hipGraphNode_t, int> index;
  index.reserve(n * 2);
  for (size_t i = 0; i < n; ++i) index[nodes[i]] = static_cast<int>(i);

  // node types and dependency lists (empty nodes folded: a dependent of an empty node depends on
  // the empty node's own dependencies)
  std::vector<hipGraphNodeType> type(n);
  std::vector<std::vector<int>> deps(n);
  for (size_t i = 0; i < n; ++i) {
    if (hipGraphNodeGetType(nodes[i], &type[i]) != hipSuccess) return -2;
    size_t nd = 0;
    if (hipGraphNodeGetDependencies(nodes[i], nullptr, &nd) != hipSuccess) return -2;
    std::vector<hipGraphNode_t> d(nd);
    if (nd > 0 && hipGraphNodeGetDependencies(nodes[i], d.data(), &nd) != hipSuccess) return -2;
    for (hipGraphNode_t x : d) {
      const auto it = index.find(x);
      if (it == index.end()) return -2;
      deps[i].push_back(it->second);
    }
    switch (type[i]) {
      case hipGraphNodeTypeGraph:
      case hipGraphNodeTypeMemAlloc:
      case hipGraphNodeTypeMemFree:
        return -3 - 100 * static_cast<int>(type[i]);  // a child graph / graph-owned memory: not replayed here
      default:
        break;
    }
  }
  // Kahn, lowest node index first (= capture order)
  std::vector<int> indeg(n, 0);
  std::vector<std::vector<int>> succ(n);
  for (size_t i = 0; i < n; ++i)
    for (int d : deps[i]) {
      succ[d].push_back(static_cast<int>(i));
      ++indeg[i];
    }
  std::vector<int> order;
  order.reserve(n);
  {
    std::vector<int> heap;
    for (size_t i = 0; i < n; ++i)
      if (indeg[i] == 0) heap.push_back(static_cast<int>(i));
    std::make_heap(heap.begin(), heap.end(), std::greater<int>());
    while (!heap.empty()) {
      std::pop_heap(heap.begin(), heap.end(), std::greater<int>());
      const int v = heap.back();
      heap.pop_back();
      order.push_back(v);
      for (int w : succ[v])
        if (--indeg[w] == 0) {
          heap.push_back(w);
          std::push_heap(heap.begin(), heap.end(), std::greater<int>());
        }
    }
  }
  if (order.size() != n) return -4;  // a cycle: not a graph capture

  // resolve empty nodes to their real (transitive) dependencies
  std::vector<std::vector<int>> real(n);
  for (int v : order) {
    std::vector<int> r;
    for (int d : deps[v]) {
      if (type[d] == hipGraphNodeTypeEmpty) r.insert(r.end(), real[d].begin(), real[d].end());
      else r.push_back(d);
    }
    std::sort(r.begin(), r.end());
    r.erase(std::unique(r.begin(), r.end()), r.end());
    real[v] = std::move(r);
  }

  // stream roles (TONY_PLAN_ROLES, default on): the eager step keeps every weight-gradient kernel (wgrad
  // GEMMs, their split-K combines) on the side stream, streams[1], and nothing else there; placing by
  // dependency chains alone put wgrads on the compute stream ahead of the BN / dgrad chain waiting
  // behind them (compute-stream gaps of 4.6 ms per step in the plan's trace vs 0.5 ms eager)
  static const bool roles_on = [] {
    const char* e = std::getenv("TONY_PLAN_ROLES");
    return e == nullptr || e[0] != '0';
  }();
  std::vector<char> side_role(n, 0);
  if (roles_on && nstreams > 1)
    for (size_t i = 0; i < n; ++i) {
      if (type[i] != hipGraphNodeTypeKernel) continue;
      hipKernelNodeParams kp{};
      if (hipGraphKernelNodeGetParams(nodes[i], &kp) != hipSuccess) {
        (void)hipGetLastError();
        continue;
      }
      const char* name = hipKernelNameRefByPtr(kp.func, nullptr);
      (void)hipGetLastError();
      if (name != nullptr && (std::strstr(name, "wgrad") != nullptr || std::strstr(name, "gemm_tn") != nullptr ||
                              std::strstr(name, "splitk_reduce") != nullptr))
        side_role[i] = 1;
    }
  const bool roles = roles_on && nstreams > 1;

  Plan* p = new Plan();
  p->nstreams = nstreams;
  for (int s = 0; s < nstreams; ++s) p->streams[s] = reinterpret_cast<hipStream_t>(streams[s]);
  if (new_event(*p) != 0) {
    destroy(p);
    return -5;
  }
  // vector clocks: pos = ops issued on a stream so far; vc[v][t] = the position on stream t node v
  // has (transitively) waited for; known[s][t] = what stream s has waited for on stream t so far
  std::vector<std::array<int, kMaxStreams>> vc(n);
  std::vector<int> node_stream(n, -1), node_pos(n, -1), rec_event(n, -1);
  int pos[kMaxStreams] = {};
  int last_use[kMaxStreams] = {};
  int known[kMaxStreams][kMaxStreams];
  for (auto& row : known)
    for (int& x : row) x = 0;
  int tick = 0, forced = 0, empties = 0, graphs = 0;
  std::vector<int> at_pos[kMaxStreams];  // node at each position of each stream
  // which nodes need an event recorded after them (a dependent lands on another stream): decided
  // as dependents are placed, so records are appended lazily -- an op list position per node
  std::vector<int> op_after(n, -1);
  void* marker_fn = reinterpret_cast<void*>(&plan_marker_kernel);
  auto fail = [&](int rc) {
    destroy(p);
    return rc;
  };
  // pending record insertions: (op index after which to insert, event) -- ops are built in a first
  // pass without records, then records spliced in
  std::vector<std::pair<int, int>> records;
  std::vector<Op> ops;
  ops.reserve(n * 2);
  for (int v : order) {
    if (type[v] == hipGraphNodeTypeEmpty) {
      ++empties;
      continue;
    }
    std::array<int, kMaxStreams> c{};
    for (int d : real[v]) {
      const std::array<int, kMaxStreams>& cd = vc[d];
      for (int t = 0; t < nstreams; ++t) c[t] = std::max(c[t], cd[t]);
      c[node_stream[d]] = std::max(c[node_stream[d]], node_pos[d] + 1);
    }
    // stream choice: (1) a stream whose tail is a direct dependency -- the OLDEST such tail: a node's
    // own-stream predecessor is captured before the cross-stream producer it was forked from (a
    // weight gradient's previous weight gradient vs the data gradient it reads), so this keeps each
    // eager chain on one stream; (2) a stream whose whole history v already depends on (unused
    // streams included): no false dependency; (3) the least recently fed stream (a false
    // dependency, counted in stats[8])
    int s = -1, best = -1;
    if (roles && side_role[v]) s = 1;  // a weight gradient: the side stream (roles above)
    // (with roles, nothing else goes to the side stream)
    for (int d : real[v]) {
      const int t = node_stream[d];
      if (s >= 0 && roles && side_role[v]) break;
      if (roles && t == 1) continue;
      if (node_pos[d] + 1 == pos[t] && (best < 0 || d < best)) {
        best = d;
        s = t;
      }
    }
    if (s < 0)
      for (int t = 0; t < nstreams; ++t)
        if (!(roles && t == 1) && pos[t] <= c[t]) {
          s = t;
          break;
        }
    if (s < 0) {
      s = 0;
      for (int t = 1; t < nstreams; ++t)
        if (!(roles && t == 1) && last_use[t] < last_use[s]) s = t;
      ++forced;
    }
    // waits for the dependencies on other streams not yet covered by what s has waited for:
    // direct dependencies first (each wait also brings what that point knew), then any transitive
    // point still missing
    auto wait_for = [&](int src, int t) -> bool {
      if (rec_event[src] < 0) {
        const int e = new_event(*p);
        if (e < 0) return false;
        rec_event[src] = e;
        records.emplace_back(op_after[src], e);
      }
      Op w{};
      w.kind = kWait;
      w.stream = s;
      w.event = rec_event[src];
      ops.push_back(w);
      for (int u = 0; u < nstreams; ++u) known[s][u] = std::max(known[s][u], vc[src][u]);
      known[s][t] = std::max(known[s][t], node_pos[src] + 1);
      return true;
    };
    for (int pass = 0; pass < 2; ++pass)
      for (int t = 0; t < nstreams; ++t) {
        if (t == s || c[t] <= known[s][t]) continue;
        int src = -1;
        for (int d : real[v])
          if (node_stream[d] == t && node_pos[d] + 1 == c[t]) src = d;
        if (src < 0 && pass == 1) src = at_pos[t][c[t] - 1];
        if (src < 0) continue;
        if (!wait_for(src, t)) return fail(-5);
      }
    Op o{};
    o.stream = s;
    if (type[v] == hipGraphNodeTypeKernel) {
      if (hipGraphKernelNodeGetParams(nodes[v], &o.k) != hipSuccess) return fail(-2);
      if (o.k.func == marker_fn) {
        o.kind = kMarker;
        o.marker = o.k.kernelParams != nullptr ? *static_cast<int*>(o.k.kernelParams[0]) : -1;
        const int e = new_event(*p);
        if (e < 0) return fail(-5);
        o.event = e;
      } else {
        // `func` is the host stub of a kernel registered by some library of the process (ours,
        // torch's: <<<>>> launches) or already a module function (hipModuleLaunchKernel callers such
        // as hipBLASLt).  Resolving the stub once here also saves hipLaunchKernel's per-launch lookup.
        o.kind = kKernel;
        if (hipGetFuncBySymbol(&o.fn, o.k.func) != hipSuccess) {
          (void)hipGetLastError();
          o.fn = static_cast<hipFunction_t>(o.k.func);
        }
        if (o.k.kernelParams == nullptr && o.k.extra == nullptr && o.k.sharedMemBytes == 0 &&
            o.k.gridDim.x == 0)
          return fail(-7);
      }
    } else if (type[v] == hipGraphNodeTypeMemset) {
      // (a memset node's parameters are always readable)
      o.kind = kMemset;
      if (hipGraphMemsetNodeGetParams(nodes[v], &o.ms) != hipSuccess) return fail(-2);
    } else {
      // copies: a fully described 3D copy is re-issued directly, anything else (1D copies captured
      // from hipMemcpyAsync carry no readable parameters) as a one-node executable graph
      // Every copy goes through the one-node graph by default: re-issuing the getter's parameters with
      // hipMemcpy3DAsync failed (hipErrorInvalidValue) on some captured linear copies -- the fp32 step's
      // D2D copies, round 3's captured collective -- and a hipMemcpyAsync of the same extent failed on
      // others; HIP's own instantiation of the node replays each faithfully (a few copies per step).
      // TONY_PLAN_DIRECT_COPY=1 restores the direct re-issue (A/B).
      static const bool allow_direct = [] {
        const char* e = std::getenv("TONY_PLAN_DIRECT_COPY");
        return e != nullptr && e[0] == '1';
      }();
      bool direct = false;
      if (allow_direct && type[v] == hipGraphNodeTypeMemcpy &&
          hipGraphMemcpyNodeGetParams(nodes[v], &o.mc) == hipSuccess) {
        const hipMemcpy3DParms& m = o.mc;
        const bool src_ok = m.srcArray != nullptr || m.srcPtr.ptr != nullptr;
        const bool dst_ok = m.dstArray != nullptr || m.dstPtr.ptr != nullptr;
        direct = src_ok && dst_ok && m.extent.width > 0 && m.extent.height > 0 && m.extent.depth > 0 &&
                 static_cast<int>(m.kind) >= 0 && static_cast<int>(m.kind) <= 4;
      }
      (void)hipGetLastError();
      if (direct) {
        o.kind = kMemcpy;
      } else {
        o.kind = kGraph;
        o.ex = single_node_exec(g, nodes[v]);
        if (o.ex == nullptr) return fail(-9);
        ++graphs;
      }
    }
    ops.push_back(o);
    op_after[v] = static_cast<int>(ops.size()) - 1;
    node_stream[v] = s;
    node_pos[v] = pos[s]++;
    at_pos[s].push_back(v);
    for (int t = 0; t < nstreams; ++t) c[t] = std::max(c[t], known[s][t]);
    c[s] = node_pos[v] + 1;
    vc[v] = c;
    known[s][s] = c[s];
    last_use[s] = ++tick;
    p->used[s] = 1;
  }
  // splice the records in after their ops (stable: records after the same op keep their order)
  std::sort(records.begin(), records.end());
  p->ops.reserve(ops.size() + records.size());
  size_t r = 0;
  for (size_t i = 0; i < ops.size(); ++i) {
    p->ops.push_back(ops[i]);
    if (ops[i].kind == kMarker) p->seg_end.push_back(static_cast<int>(p->ops.size()));
    while (r < records.size() && records[r].first == static_cast<int>(i)) {
      Op rec{};
      rec.kind = kRecord;
      rec.stream = ops[i].stream;
      rec.event = records[r].second;
      p->ops.push_back(rec);
      ++r;
    }
  }
  // marker segment ends must point past the records spliced after the marker op as well
  {
    int k = 0;
    for (size_t i = 0; i < p->ops.size(); ++i)
      if (p->ops[i].kind == kMarker) p->seg_end[k++] = static_cast<int>(i) + 1;
  }
  p->seg_end.push_back(static_cast<int>(p->ops.size()));
  // per side stream: one tail event joined into stream 0 at the end of the replay
  p->tails.assign(nstreams, -1);
  for (int s = 1; s < nstreams; ++s)
    if (p->used[s]) {
      const int e = new_event(*p);
      if (e < 0) return fail(-5);
      p->tails[s] = e;
    }
  int* st = p->stats;
  for (const Op& o : p->ops) {
    if (o.kind == kKernel) ++st[0];
    else if (o.kind == kMemset) ++st[1];
    else if (o.kind == kMemcpy) ++st[2];
    else if (o.kind == kWait) ++st[3];
    else if (o.kind == kRecord) ++st[4];
    else if (o.kind == kMarker) ++st[6];
  }
  for (int s = 0; s < nstreams; ++s) st[5] += p->used[s];
  st[7] = static_cast<int>(n);
  st[8] = forced;
  st[9] = empties;
  st[10] = graphs;
  if (stats != nullptr) std::memcpy(stats, st, sizeof(p->stats));
  *out = reinterpret_cast<uint64_t>(p);
  return 0;
}

// Issue segment `seg` of the plan (0..markers; a plan without markers has the one segment 0), or
// every segment when seg < 0.  Segment 0 starts by forking stream 0 into every used side stream;
// the last segment ends by joining them back into stream 0.  A segment ending in a marker forks the
// marker's stream into `side` (may be null) so work the host enqueues there follows the marker.
TONY_API int tony_plan_replay(void* handle, int seg, hipStream_t side) {
  Plan* p = static_cast<Plan*>(handle);
  if (p == nullptr) return -1;
  const int nseg = static_cast<int>(p->seg_end.size());
  if (seg >= nseg) return -1;
  const int first = seg < 0 ? 0 : seg, last = seg < 0 ? nseg - 1 : seg;
  hipError_t e = hipSuccess;
  if (first == 0) {
    e = hipEventRecord(p->events[0], p->streams[0]);
    for (int s = 1; s < p->nstreams && e == hipSuccess; ++s)
      if (p->used[s]) e = hipStreamWaitEvent(p->streams[s], p->events[0], 0);
  }
  const int lo = first == 0 ? 0 : p->seg_end[first - 1];
  const int hi = p->seg_end[last];
  for (int i = lo; i < hi && e == hipSuccess; ++i) {
    e = issue(*p, p->ops[i], side);
    if (e != hipSuccess) {
      p->fail_op = i;
      p->fail_kind = p->ops[i].kind;
      p->fail_stream = p->ops[i].stream;
    }
  }
  if (e == hipSuccess && last == nseg - 1) {
    for (int s = 1; s < p->nstreams && e == hipSuccess; ++s)
      if (p->tails[s] >= 0) {
        e = hipEventRecord(p->events[p->tails[s]], p->streams[s]);
        if (e == hipSuccess) e = hipStreamWaitEvent(p->streams[0], p->events[p->tails[s]], 0);
      }
  }
  return static_cast<int>(e);
}

// out[3] = (op index, op kind, stream) of the last failed issue (-1s: none)
TONY_API int tony_plan_failure(void* handle, int* out) {
  Plan* p = static_cast<Plan*>(handle);
  if (p == nullptr || out == nullptr) return -1;
  out[0] = p->fail_op;
  out[1] = p->fail_kind;
  out[2] = p->fail_stream;
  return 0;
}

TONY_API int tony_plan_segments(void* handle) {
  Plan* p = static_cast<Plan*>(handle);
  return p == nullptr ? -1 : static_cast<int>(p->seg_end.size());
}

// Stream of each op, kind and marker id (tests / tracing): out has 3 ints per op; returns the op count.
TONY_API int tony_plan_ops(void* handle, int* out, int cap) {
  Plan* p = static_cast<Plan*>(handle);
  if (p == nullptr) return -1;
  const int n = static_cast<int>(p->ops.size());
  for (int i = 0; i < n && i < cap; ++i) {
    out[3 * i] = p->ops[i].kind;
    out[3 * i + 1] = p->ops[i].stream;
    out[3 * i + 2] = p->ops[i].kind == kMarker ? p->ops[i].marker : p->ops[i].event;
  }
  return n;
}

TONY_API int tony_plan_destroy(void* handle) {
  Plan* p = static_cast<Plan*>(handle);
  if (p == nullptr) return -1;
  destroy(p);
  return 0;
}
