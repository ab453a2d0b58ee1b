"""Weight gradients on a second HIP stream, overlapped with the data-gradient chain.

In a layer's backward the weight gradient (split-K wgrad GEMM + slab combine, summed into the
flat gradient buffer) and the data gradient (dgrad GEMM, then the previous layer's BN backward,
...) are independent: only the data gradient is on the critical path of the backward.  Inception-v3
and ResNet-50 backward passes are ~500 launches, half of them small latency-bound kernels (the
17x17 and 8x8 BN kernels, 5-15 us at a few waves per CU) that leave most of the 256 CUs idle.  With
``begin(device)`` active, ops hand their in-place weight-gradient work to ``run()``: it is issued
on a per-device side stream that first waits for the current stream (so dZ / x are ready) and the
trainer's ``end()`` joins the side stream back before the optimizer reads the gradients.  Inside a
HIP-graph capture the fork/join become graph edges and the two chains are parallel graph branches.

Memory safety: operands produced on the current stream (dZ, saved activations) would be recycled
by the caching allocator as soon as the backward node returns, while the side stream may still read
them; ``run`` keeps them referenced until ``end()`` (after the join), so no block is reused early.

Only weight gradients accumulated in place (``_lib.grad_slot``) go to the side stream: a gradient
returned to autograd would be consumed on the current stream without a dependency.  Autotuning
(tune.py, conv._choose) times kernels on the current stream and must not race a side stream, so
the trainer begins overlapping only after its first (tuning) step.  ``TONY_WGRAD_STREAM=0`` turns
the overlap off.

Reference parity: TonY delegates the backward to the framework; the overlap of
independent gradient work is the MI355X-native counterpart of cuDNN/NCCL stream overlap there.
"""
from __future__ import annotations

import os
import threading
from typing import Callable, Dict, List, Optional

import torch

from . import _lib

ENABLED = os.environ.get("TONY_WGRAD_STREAM", "1") != "0"

_lock = threading.Lock()
_streams: Dict[int, torch.cuda.Stream] = {}
_active: List[Optional[torch.cuda.Stream]] = [None]
_keep: List[torch.Tensor] = []
_issued = [0]


def _side(device: torch.device) -> torch.cuda.Stream:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _streams.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=torch.device("cuda", idx))
        _streams[idx] = s
    return s


# ---- parallel model branches (Inception blocks) -------------------------------------------------
# With branches on, ``parallel(*thunks)`` runs the first thunk on the current stream and each other
# one on its own branch stream (forked from the current stream, joined back after), so the 2-3
# independent conv chains of an Inception block execute concurrently; autograd then replays each
# branch's backward on the stream its forward ran on.  Tensors that cross streams are kept
# referenced until ``end()`` (``keep``), which joins every stream used into the current one.
# On by default since round 2: with the faster kernels the Inception step is no longer host-bound, and
# branch streams measured 15.05 vs 15.66 ms/step (alternating A/B on MI355X,
# profiles/r2s3_branch_streams_ab.log).  TONY_BRANCH_STREAMS=0 runs every branch on one stream.
BRANCHES_ENABLED = os.environ.get("TONY_BRANCH_STREAMS", "1") != "0"
_branch_pool: Dict[int, List[torch.cuda.Stream]] = {}
_branches_on = [False]
_used: Dict[int, torch.cuda.Stream] = {}


def _branch_streams(device: torch.device, n: int) -> List[torch.cuda.Stream]:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    pool = _branch_pool.setdefault(idx, [])
    while len(pool) < n:
        pool.append(torch.cuda.Stream(device=torch.device("cuda", idx)))
    return pool[:n]


def plan_streams(device, branches: int = 3) -> List[torch.cuda.Stream]:
    """The side streams a natively replayed step may use (ops/plan.py): the weight-gradient stream
    and ``branches`` branch streams -- the same streams (and so the same hardware queues) as the
    eager step's."""
    device = torch.device(device)
    return [_side(device), *_branch_streams(device, branches)]


def begin(device, branches: bool = False) -> bool:
    """Route in-place weight gradients to the side stream (and, with ``branches``, model branches to
    branch streams) until ``end()``; False when disabled."""
    device = torch.device(device)
    if not ENABLED or device.type != "cuda":
        return False
    _active[0] = _side(device)
    _issued[0] = 0
    _branches_on[0] = branches and BRANCHES_ENABLED
    return True


def branches_active() -> bool:
    return _branches_on[0]


def keep(*tensors) -> None:
    """Hold tensors (read or written on another stream than the one that allocated them) until end()."""
    if _branches_on[0] or _active[0] is not None:
        with _lock:
            _keep.extend(t for t in tensors if isinstance(t, torch.Tensor))


# TONY_MAIN_FIRST=1: ``parallel`` issues its first thunk (the block's longest chain, on the current
# stream) before the branch thunks instead of after them.  Autograd runs backward nodes in reverse creation
# order, so the longest chain's backward is then issued LAST: at a block input with several consumers
# (ops/residual.py GradJoin, Inception's reduction blocks) the short branches park / accumulate their dX
# first and the long chain adds into it as it finishes, instead of the short branches' dgrads queueing
# behind the long chain's (profiles/r6_lean_crit_path_eager.txt: ~0.25 ms idle at Mixed_6a).  Measured
# slower: GPU time with the host ahead 13.42-13.45 vs 13.28-13.32 ms eager, plan even
# (profiles/r6_ab_main_first.log) -- opt-in
MAIN_FIRST = os.environ.get("TONY_MAIN_FIRST", "0") == "1"


def parallel(*thunks):
    """Results of the independent ``thunks``; concurrently on branch streams when branches are on."""
    if not _branches_on[0] or len(thunks) < 2:
        return [f() for f in thunks]
    main = current(torch.cuda.current_device())
    side = _branch_streams(main.device, len(thunks) - 1)
    outs = [None] * len(thunks)
    if MAIN_FIRST:
        for s in side:  # every branch starts from the current stream's position before the first thunk
            fork(main, s)
        outs[0] = thunks[0]()
    for i, (f, s) in enumerate(zip(thunks[1:], side), 1):
        if not MAIN_FIRST:
            fork(main, s)
        torch.cuda.set_stream(s)
        try:
            outs[i] = f()
        finally:
            torch.cuda.set_stream(main)
        _used[id(s)] = s
    if not MAIN_FIRST:
        outs[0] = thunks[0]()
    for s in side:
        fork(s, main)
    keep(*[o for o in outs if isinstance(o, torch.Tensor)])
    return outs


def active() -> bool:
    return _active[0] is not None


# Work is handed to the side stream in batches of BATCH ops: one fork (event record + stream wait,
# ~10 us of host time) and one stream switch per batch instead of per op.  A batch forks from the
# current stream's position at flush time -- later than each op needs, never earlier.
# Measured: 1 (16.34 ms) beat 4 (16.77 ms) while the step was GPU-bound at 16 ms (round 1); with the
# GPU at 14 ms the host issue cost matters: 2 measured 13.90 / 13.89 ms/step vs 14.1-15.1 at 1
# (profiles/r2s3_host_levers_ab.log).  Round 6 (lean conv kernels, GPU at 13.3-13.4 ms, eager host 11.4-15 ms):
# 3 measured 13.265 ms/step mean over 4 repetitions vs 13.755 at 2 (whose host went bound in one of them), GPU
# time with the host ahead 13.36 vs 13.40 (profiles/r6_ab_wgrad_batch_eager.log).  The fp32 (x3) step, whose
# weight gradients are three products deep, takes 4: 0.3 % faster, 0.7 % with TONY_X3_WGRAD_OCC=0.5
# (profiles/r6_ab_fp32_wb4.log) -- parallel/trainer.py picks it per model (set_batch) unless the env says.
BATCH = int(os.environ.get("TONY_WGRAD_BATCH", "3"))
BATCH_FROM_ENV = "TONY_WGRAD_BATCH" in os.environ


def set_batch(n: int) -> None:
    """Weight-gradient ops per side-stream fork from here on (TONY_WGRAD_BATCH, when set, wins)."""
    global BATCH
    if not BATCH_FROM_ENV:
        BATCH = max(1, int(n))
_pending: List[tuple] = []  # (fn, the stream that queued it)
# ...except for big operands: a batch forks from the current stream when it is flushed, so a pending
# op waits for whatever the compute stream was given in between (the next layer's BN backward and
# data gradient).  At the end of an Inception backward that is the serial stem chain: the 149x149
# layer's wgrad sat behind the 147x147 layer's BN backward, and the optimizer waited ~350 us on it
# (profiles/r2s4_step_tail_trace.txt).  Ops whose first kept operand (the conv-output gradient) is at
# least URGENT_BYTES are issued at once.  TONY_WGRAD_URGENT_MB=0 turns this off.
URGENT_BYTES = int(os.environ.get("TONY_WGRAD_URGENT_MB", "64")) << 20


# A fork costs host time on every weight gradient, branch and bucket (~150 per Inception step), so it
# avoids the convenience wrappers: Stream.wait_stream() creates a new HIP event per call, and even a
# pooled torch.cuda.Event's record + wait_event is ~7.6 us of host time (tools/host_micro.py).  Here
# ONE fast-call (csrc/streams.hip tony_fork) records a pooled timing-free HIP event on the producer
# and makes the consumer wait on it (a recorded event may be recorded again once the wait on it is
# enqueued); the current stream is switched with the raw setter.
_ev_next = [0]
_EV_RING = 256
_RAW: Dict[int, List[int]] = {}
_FORK = [None]


def _raw_ring(device_index: int) -> List[int]:
    ring = _RAW.get(device_index)
    if ring is None:
        import ctypes

        buf = (ctypes.c_uint64 * _EV_RING)()
        with torch.cuda.device(device_index):
            _lib.check(_lib.lib().tony_event_pool(_EV_RING, buf), "tony_event_pool")
        ring = _RAW[device_index] = list(buf)
        _FORK[0] = _lib.lib().tony_fork
    return ring


_BY_HANDLE: Dict[int, torch.cuda.Stream] = {}


def current(device_index: int) -> torch.cuda.Stream:
    """torch.cuda.current_stream(device) without its ~2.6 us of host time (tools/host_micro.py): the
    raw current handle (one C call) maps to the Stream object seen the first time (torch never
    destroys its pooled streams, so a handle names one stream for the whole process)."""
    h = _lib._RAW_STREAM(device_index) if _lib._RAW_STREAM is not None else None
    s = _BY_HANDLE.get(h) if h is not None else None
    if s is None:
        s = torch.cuda.current_stream(device_index)
        if h is not None:
            _BY_HANDLE[h] = s
    return s


def fork(producer: torch.cuda.Stream, consumer: torch.cuda.Stream) -> None:
    """``consumer`` waits for everything enqueued on ``producer`` so far (no host block).  A stream is
    never made to wait on itself: inside a capture HIP records that as the stream joining its own
    capture, and hipStreamEndCapture then recurses through the self-join until the host stack overflows
    (x3 InceptionE, both split convs of a join on one branch stream: tools/x3_capture_diag.py --bt)."""
    if producer.cuda_stream == consumer.cuda_stream:
        return
    ring = _RAW.get(producer.device_index) or _raw_ring(producer.device_index)
    i = _ev_next[0]
    _ev_next[0] = i + 1
    rc = _FORK[0](ring[i % _EV_RING], producer.cuda_stream, consumer.cuda_stream)
    if rc:
        _lib.check(rc, "tony_fork")


_DEBUG = os.environ.get("TONY_STREAMS_DEBUG", "0") == "1"
_ALL_SRCS = os.environ.get("TONY_FLUSH_ALL_SRCS", "1") != "0"


def _flush(side: torch.cuda.Stream) -> None:
    with _lock:
        work = list(_pending)
        _pending.clear()
    if not work:
        return
    cur = current(side.device_index)
    # the side stream waits for every stream that queued work of this batch: a backward node of an
    # Inception branch runs on its branch stream, so a batch may hold a weight gradient whose dZ is
    # still being produced on another stream than the one flushing (waiting on the flushing stream
    # alone raced: x3 block D, tools/x3_block_diag.py)
    srcs = {}
    for _, src in work:
        srcs.setdefault(src.cuda_stream, src)
    srcs.setdefault(cur.cuda_stream, cur)
    if _DEBUG:
        st = []
        for src in srcs.values():
            torch.cuda.set_stream(src)
            st.append((hex(src.cuda_stream), torch.cuda.is_current_stream_capturing()))
        torch.cuda.set_stream(cur)
        print(f"[streams] flush {len(work)} cur={hex(cur.cuda_stream)} side={hex(side.cuda_stream)} srcs={st}",
              flush=True)
    for src in (srcs.values() if _ALL_SRCS else [cur]):
        fork(src, side)
    torch.cuda.set_stream(side)
    try:
        for fn, _ in work:
            out = fn()
            assert out is None, "only in-place gradient work may run on the side stream"
    finally:
        torch.cuda.set_stream(cur)


# The last TAIL weight gradients of a backward pass run on the current stream instead.  The
# backward ends with the stem layers (147x147 / 149x149 maps: the largest wgrads of the step) while
# the data-gradient chain has almost nothing left to do; queued behind the side stream's backlog
# they would run alone after it, with the compute stream idle until the join.  The count is taken
# from the previous step (the backward order is fixed); TONY_WGRAD_TAIL=0 keeps all on the side.
TAIL = int(os.environ.get("TONY_WGRAD_TAIL", "0"))
_tail_from = [-1]  # index of the first weight gradient of a step that runs inline (-1: none)


def run(fn: Callable[[], object], *keep: torch.Tensor):
    """Run ``fn`` (which must write its result in place and return None) on the side stream when one
    is active -- possibly deferred to the next batch flush or ``end()`` -- else right here.  ``keep``:
    tensors ``fn`` reads that the caller may drop."""
    side = _active[0]
    if side is None:
        return fn()
    if 0 <= _tail_from[0] <= _issued[0]:  # the step's tail: on the current stream
        with _lock:
            _issued[0] += 1
        return fn()
    urgent = URGENT_BYTES > 0 and bool(keep) and keep[0].numel() * keep[0].element_size() >= URGENT_BYTES
    src = current(side.device_index)  # the stream fn's operands are produced on
    with _lock:
        _pending.append((fn, src))
        _keep.extend(keep)
        _issued[0] += 1
        full = len(_pending) >= BATCH or urgent
    if full:
        _flush(side)
    return None


def fence_into(stream: torch.cuda.Stream) -> None:
    """Make ``stream`` wait for everything issued so far on the weight-gradient side stream and the
    branch streams (deferred work is issued first), without making the compute streams wait."""
    side = _active[0]
    if side is None:
        return
    _flush(side)
    for s in [side, *_used.values()]:
        if s is stream:
            continue
        fork(s, stream)


def end() -> int:
    """Issue the deferred work, join the side stream into the current stream and release the kept
    operands; returns how many ops ran on the side stream this step."""
    side = _active[0]
    _active[0] = None
    _branches_on[0] = False
    if side is not None:
        _flush(side)
        cur = current(side.device_index)
        fork(side, cur)
        for s in _used.values():  # backward kernels of branch nodes ran on these
            fork(s, cur)
        _used.clear()
    with _lock:
        _keep.clear()
        n, _issued[0] = _issued[0], 0
    _tail_from[0] = n - TAIL if 0 < TAIL < n else -1
    return n
