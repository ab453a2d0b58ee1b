"""Gradient buckets that launch their communication while backward is still running.

Shared engine of the three gradient data planes: the colocated / dedicated
parameter server (ps.py, TF between-graph PS), PyTorch-DDP and Horovod's DistributedOptimizer
(ddp.py, hvd.py).  Reference: Horovod overlaps its fused all-reduce with backward
(``EX/horovod-on-tony/tensorflow2_mnist.py:73``); TF-PS workers push each variable's gradient as
soon as it is computed (``EX/mnist-tensorflow/mnist_distributed.py:206-241``).

Readiness.  A bucket is a contiguous slice of the flat gradient buffer (parallel/flat.py) covering
whole parameters, cut in reverse registration order (the order backward produces them).  Its
gradients are complete when every parameter in it has been written.  Two producers report that:

* the fused HIP ops (conv / BN / fused heads / residual), which add parameter gradients straight
  into the flat buffer and return None to autograd, call ``_lib.grads_ready(*params)`` at the end
  of their backward node (after the node's data-gradient kernels are enqueued, so nothing of that
  node still reads the old parameters when the bucket's apply rewrites them);
* every other parameter goes through AccumulateGrad, whose post-accumulate hook reports it (the
  hook also fires, with nothing accumulated, right after a fused node returned None for a
  parameter: such a repeat report is ignored).

Ordering.  Buckets launch strictly in index order (a ready bucket waits for its predecessors), so
every rank issues its collectives in the same sequence -- the RCCL/NCCL requirement -- whatever
order the gradients land in.  A parameter reported twice in one step (used twice in the graph, its
gradient still accumulating) after its bucket launched raises: that would ship a partial gradient.

Streams.  A launch forks a dedicated communication stream from the current compute stream AND the
weight-gradient side stream (ops/streams.py), so the collective sees every gradient write of the
bucket without making the compute streams wait for anything; ``end()`` joins the communication
stream back into the compute stream.  On CPU (gloo tests) launches simply run inline.

xGMI sizing.  A ring reduce-scatter / all-reduce on 8 MI355X moves (N-1)/N of a bucket over every
one of the 7 links per phase; at ~50-100 GB/s achieved per link an 8 MB bf16 bucket costs ~20-40 us,
well past the launch-latency regime yet small enough that the last bucket (stem gradients, exposed
after backward) is short.  ``TONY_BUCKET_MB`` overrides the default.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import torch

from ..ops import _lib, streams
from .flat import FlatParams

DEFAULT_BUCKET_MB = float(os.environ.get("TONY_BUCKET_MB", "8"))


@dataclass
class Bucket:
    index: int
    lo: int
    hi: int
    params: List[int] = field(default_factory=list)
    pending: int = 0
    launched: bool = False
    work: object = None

    @property
    def numel(self) -> int:
        return self.hi - self.lo


def make_buckets(flat: FlatParams, bucket_mb: float, multiple: int = 1) -> List[Bucket]:
    """Partition ``flat`` into buckets of about ``bucket_mb`` MB in reverse parameter order.

    Bucket boundaries are parameter offsets (plus the tail padding in bucket 0); every bucket
    length must be a multiple of ``multiple`` (the reduce-scatter split), which FlatParams
    guarantees when its slot alignment is a multiple of it."""
    cap = max(1, int(bucket_mb * 2 ** 20 // flat.grad.element_size()))
    ends = [s.offset for s in flat.slots[1:]] + [flat.numel]
    out: List[Bucket] = []
    cur: Optional[Bucket] = None
    for i in reversed(range(len(flat.slots))):
        s = flat.slots[i]
        if cur is None:
            cur = Bucket(len(out), s.offset, ends[i])
        cur.lo = s.offset
        cur.params.append(i)
        if cur.hi - cur.lo >= cap:
            out.append(cur)
            cur = None
    if cur is not None:
        out.append(cur)
    for b in out:
        if b.numel % multiple:
            raise ValueError(f"bucket [{b.lo}, {b.hi}) is not a multiple of {multiple} elements: build FlatParams "
                             f"with align a multiple of {multiple}")
    return out


class GradBucketEngine:
    """Counts outstanding gradients per bucket and calls ``launch_fn(bucket)`` in bucket order.

    ``launch_fn`` runs with the communication stream current (GPU) and must only enqueue work;
    ``end()`` launches whatever is left (all buckets when overlap is off) and joins."""

    def __init__(self, flat: FlatParams, buckets: List[Bucket], launch_fn: Callable[[Bucket], None]):
        self.flat = flat
        self.buckets = buckets
        self.launch_fn = launch_fn
        self.bucket_of: List[int] = [0] * len(flat.slots)
        for b in buckets:
            for i in b.params:
                self.bucket_of[i] = b.index
        self._index: Dict[int, int] = {id(p): i for i, p in enumerate(flat.params)}
        self._seen: List[bool] = [False] * len(flat.slots)
        self.device = flat.device
        self.comm: Optional[torch.cuda.Stream] = None
        self._dev_index = -1
        if self.device.type == "cuda":
            self.comm = torch.cuda.Stream(device=self.device)
            self._dev_index = self.comm.device_index
        self._hooks: Dict[int, object] = {}
        self.attached = False  # listening (the hooks of fused-reported parameters are dropped after a step)
        self._inplace = [False] * len(flat.slots)  # reported by a fused op: its AccumulateGrad hook is dropped
        esz = flat.grad.element_size()
        self._slot_ptr = [flat.grad.data_ptr() + s.offset * esz for s in flat.slots]
        self.armed = False
        self.overlap = False
        # native step replay (ops/plan.py): during the capture of a step each bucket's launch point is
        # captured as a plan marker instead; replays then issue the plan segment by segment and the
        # bucket's collective after each (``replay_launch``), in ``marked`` order
        self.capture_markers = False
        self.marked: List[int] = []
        self._next = 0
        self.launches = 0
        self.launched_during_backward = 0  # buckets issued before end() (the overlap actually happened)
        self.log: Optional[List[str]] = None  # set to a list to record the launch / ready sequence (tests)
        # called (during backward) by the first gradient report of an un-armed step; it must call
        # begin() -- DDP / Horovod arm themselves this way, the PS trainer arms explicitly
        self.auto_arm: Optional[Callable[[], None]] = None

    # -- wiring ---------------------------------------------------------------------------------
    def attach(self) -> None:
        """Listen to the fused ops' in-place gradient reports and to AccumulateGrad hooks."""
        if self.attached:
            return
        self.attached = True
        _lib.add_grad_listener(self)
        for i, p in enumerate(self.flat.params):
            self._hooks[i] = p.register_post_accumulate_grad_hook(lambda p, i=i: self._on_accumulate(i, p))

    def detach(self) -> None:
        self.attached = False
        _lib.remove_grad_listener(self)
        for h in self._hooks.values():
            h.remove()
        self._hooks = {}

    # -- per step -------------------------------------------------------------------------------
    def begin(self, overlap: bool = True, markers: bool = False) -> None:
        """Arm for one backward pass; with ``overlap`` False nothing launches before ``end()``.
        ``markers`` (inside a step capture only): record each bucket's launch point as a plan marker."""
        for b in self.buckets:
            b.pending, b.launched, b.work = len(b.params), False, None
        self._seen = [False] * len(self.flat.slots)
        self._next = 0
        self.launched_during_backward = 0
        self.armed = True
        capturing = self.device.type == "cuda" and torch.cuda.is_current_stream_capturing()
        self.capture_markers = bool(markers) and capturing and self.comm is not None
        if self.capture_markers:
            self.marked = []
        self.overlap = (bool(overlap) and not capturing) or self.capture_markers

    def end_capture(self) -> None:
        """Close a marker capture: join the communication stream back (the capture must end joined)
        and disarm without launching anything; ``marked`` keeps the bucket of each marker."""
        if not self.capture_markers:
            return
        self.capture_markers = False
        self.armed = False
        self._drop_inplace_hooks()
        streams.fork(self.comm, streams.current(self._dev_index))

    def replay_launch(self, b: Bucket) -> None:
        """Launch bucket ``b`` on the communication stream after a plan segment (the plan already
        forked the marker's stream into it)."""
        b.launched = True
        self._next = max(self._next, b.index + 1)
        self.launches += 1
        self.launched_during_backward += 1
        if self.log is not None:
            self.log.append(f"launch:{b.index}")
        cur = streams.current(self._dev_index)
        torch.cuda.set_stream(self.comm)
        try:
            self.launch_fn(b)
        finally:
            torch.cuda.set_stream(cur)

    def cancel(self) -> None:
        """Disarm without launching anything (a gradient-accumulation pass)."""
        self.armed = False

    def ready(self, params) -> None:
        """``_lib.grads_ready`` listener: these parameters' gradients are fully written."""
        if not self.armed:
            if self.auto_arm is None or not any(id(p) in self._index for p in params):
                return
            self.auto_arm()
        for p in params:
            i = self._index.get(id(p))
            if i is not None:
                self._inplace[i] = True
                self._mark(i)
        self._drain()

    def _on_accumulate(self, i: int, p: torch.Tensor) -> None:
        g = p.grad
        if g is not None and g.data_ptr() != self._slot_ptr[i]:
            view = self.flat.slots[i].view(self.flat.grad)
            view.copy_(g)  # user code replaced .grad (e.g. zero_grad(set_to_none=True))
            p.grad = view
        if not self.armed:
            if self.auto_arm is None:
                return
            self.auto_arm()
        if self._seen[i]:
            # AccumulateGrad runs (and fires this hook) even when a fused op returned None for the
            # parameter after accumulating in place and reporting it: nothing new was written
            return
        self._mark(i)
        self._drain()

    def _mark(self, i: int) -> None:
        b = self.buckets[self.bucket_of[i]]
        if self._seen[i]:
            if b.launched:
                raise RuntimeError(f"gradient of {self.flat.slots[i].name} written again after its bucket "
                                   f"{b.index} launched (parameter used twice in the graph?)")
            return
        self._seen[i] = True
        b.pending -= 1
        if self.log is not None:
            self.log.append(f"ready:{self.flat.slots[i].name}")

    def _drain(self) -> None:
        if not self.overlap:
            return
        while self._next < len(self.buckets) and self.buckets[self._next].pending <= 0:
            self._launch(self.buckets[self._next])
            self.launched_during_backward += 1

    def _launch(self, b: Bucket) -> None:
        if b.launched:
            return
        b.launched = True
        self._next = max(self._next, b.index + 1)
        self.launches += 1
        if self.log is not None:
            self.log.append(f"launch:{b.index}")
        if self.comm is None:
            self.launch_fn(b)
            return
        cur = streams.current(self._dev_index)
        streams.fork(cur, self.comm)
        streams.fence_into(self.comm)  # the weight-gradient side stream's writes, too
        if self.capture_markers:  # step capture: the launch point becomes a plan marker
            from ..ops import plan

            plan.mark(len(self.marked), self.comm)
            self.marked.append(b.index)
            return
        torch.cuda.set_stream(self.comm)
        try:
            self.launch_fn(b)
        finally:
            torch.cuda.set_stream(cur)

    def _drop_inplace_hooks(self) -> None:
        """Parameters the fused ops report themselves need no AccumulateGrad hook: each Python hook
        call costs ~10 us of host time on the backward's critical issue path (x ~300 parameters)."""
        for i, done in enumerate(self._inplace):
            h = self._hooks.pop(i, None) if done else None
            if h is not None:
                h.remove()

    def end(self, finish: Optional[Callable[[], None]] = None) -> None:
        """Launch the remaining buckets in order, then ``finish`` (enqueued on the communication stream
        after every bucket: e.g. the PS plane's landing of the new variables), and make the current
        stream wait for all of it."""
        self._drop_inplace_hooks()
        for b in self.buckets:
            if not b.launched:
                self._launch(b)
        self.armed = False
        if finish is not None:
            if self.comm is None:
                finish()
            else:
                cur = torch.cuda.current_stream(self.device)
                torch.cuda.set_stream(self.comm)
                try:
                    finish()
                finally:
                    torch.cuda.set_stream(cur)
        if self.comm is not None:
            streams.fork(self.comm, streams.current(self._dev_index))
