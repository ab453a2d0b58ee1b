"""One training step = forward + loss + backward + PS push/apply/pull, optionally
captured once into a HIP graph and replayed.

Graph capture removes the per-kernel host launch cost of the ~1,500 kernels an
Inception-v3 step issues (convs, fused BN, pools, concats, the optimizer and
the collectives): the whole step becomes one ``hipGraphLaunch``.  Inputs live in
static device buffers that the caller refreshes (``x.copy_(batch)``) between
replays; optimizer hyper-parameters are device-resident (ops/optim.py), so a
replay always uses the current learning rate.
"""
from __future__ import annotations

import gc
import os
import time
from typing import Callable

import torch

from ..ops import streams, wt_cache
from ..ops.arena import for_device
from ..utils.tracing import heartbeat, trace_range
from .ps import ParameterServer

# Python garbage collection in the eager loop.  Every step builds and drops an autograd graph of
# ~900 nodes plus their contexts; the cyclic collector's generation-2 passes then walk the whole heap
# (model, tensors, tuning caches) at unpredictable steps -- host stalls of ms on a loop whose host
# issue time is within ~10% of the GPU's.  "freeze" (default): after the first (tuning) step the
# long-lived heap is moved to the permanent generation (gc.freeze) so collections only see the
# step's own garbage; "off": no automatic collection, one full pass every GC_EVERY steps; "auto":
# Python's default.
GC_MODE = os.environ.get("TONY_GC", "freeze").lower()
GC_EVERY = int(os.environ.get("TONY_GC_EVERY", "200"))

# How a captured step is re-issued: "plan" (default) walks the captured hipGraph once and replays it
# from C++ onto the eager step's streams (ops/plan.py, csrc/plan.hip); "graph" instantiates it and
# calls hipGraphLaunch.  A graph the native replay cannot issue falls back to "graph".
REPLAY = os.environ.get("TONY_REPLAY", "plan").lower()
# weight-gradient ops per side-stream fork inside a captured step (eager issue uses streams.BATCH).  4 since
# round 6: with the lean conv kernels one op per fork left the plan 0.8 ms behind eager (14.19 vs 13.40 ms);
# 2 / 3 / 4 ops per fork 13.63 / 13.61 / 13.56 ms (profiles/r6_plan_wgrad_batch.log)
PLAN_WGRAD_BATCH = int(os.environ.get("TONY_PLAN_WGRAD_BATCH", "4"))

# Opt-in: measured slower on MI355X (bench 16.9 vs 15.7 ms/step; the compute queue's gaps grew from
# 3.3 to 5.9 ms under rocprofv3), so the step stays on the caller's stream by default.
PRIO_STREAM = os.environ.get("TONY_PRIO_STREAM", "0") == "1"


# the fp32 model's weight planes split once per step in one launch (ops/wt_cache.py X3Weights);
# TONY_X3_WCACHE=0: split per conv and pass (A/B)
X3_WCACHE = os.environ.get("TONY_X3_WCACHE", "1") != "0"

class Trainer:
    def __init__(self, model: torch.nn.Module, ps: ParameterServer, loss_fn: Callable, use_graph: bool = False,
                 warmup_eager: int = 3, graph_collectives: bool | None = None, overlap_wgrad: bool = True,
                 branch_streams: bool = True, overlap_comm: bool = True):
        self.model = model
        self.ps = ps
        # eager weight-gradient forks: 4 ops per fork for the fp32 (x3) model, 3 for bf16 (ops/streams.py BATCH)
        streams.set_batch(4 if getattr(model, "x3", False) else 3)
        self.loss_fn = loss_fn
        self.use_graph = use_graph
        self.warmup_eager = warmup_eager
        # With >1 rank the PS push/apply/pull (RCCL reduce-scatter, one fused optimizer launch,
        # RCCL all-gather) runs eagerly after the replayed forward+backward graph: three
        # launches, so nothing is lost, and no communicator state is baked into the graph
        # (RCCL's graph-capture support differs across releases).  One rank: all in the graph.
        self.graph_collectives = (ps.world == 1) if graph_collectives is None else graph_collectives
        self.overlap_wgrad = overlap_wgrad
        self.overlap_comm = overlap_comm
        self.phase_events = None
        self.branch_streams = branch_streams
        self._tuned = False
        self.side_ops = 0
        self.host_fwd_s = self.host_bwd_s = 0.0
        self.graph = None
        self.plan = None
        self.plan_error = None
        self.plan_buckets = False
        self.replay_kind = None
        self.static_x = None
        self.static_y = None
        self.static_loss = None
        self._eager_steps = 0
        self._prio = None
        dev = ps.flat.device
        # one zero-fill per step for every fused kernel's fp32 accumulators (ops/arena.py)
        self.arena = for_device(dev) if dev.type == "cuda" else None
        # transposed conv weights for the dgrads, refreshed by one batched launch per step (ops/wt_cache.py)
        # (one cache per trainer, active only inside its steps: nothing else can read a stale copy)
        self.wt = wt_cache.TransposedWeights(dev) if dev.type == "cuda" else None
        if self.wt is not None:
            self.wt.enabled = True
        # the fp32 (x3) model's weight planes, split in one launch after each optimizer step
        self.wx3 = wt_cache.X3Weights(dev) if dev.type == "cuda" and X3_WCACHE else None
        if self.wx3 is not None:
            self.wx3.enabled = True

    def _mark(self, i: int) -> None:
        ev = self.phase_events
        if ev is not None and not torch.cuda.is_current_stream_capturing():
            ev[i].record()

    def enable_phase_timing(self) -> None:
        """Record GPU events at step start / after forward / after backward / after the PS step."""
        self.phase_events = [torch.cuda.Event(enable_timing=True) for _ in range(4)]

    def phase_ms(self):
        """(forward, backward, exposed PS push/apply/pull) GPU ms of the last eager step."""
        ev = self.phase_events
        ev[3].synchronize()
        return tuple(ev[i].elapsed_time(ev[i + 1]) for i in range(3))

    def _body(self, x, y, ps_step: bool = True):
        t0 = time.perf_counter()
        self._mark(0)
        self.ps.zero_grad()
        if ps_step:
            # arm the gradient buckets: each bucket's push/apply/pull is enqueued on the communication
            # stream as soon as backward has written its gradients (parallel/buckets.py); not in the
            # first (autotuning) step, whose kernel timings must not race the communication stream
            self.ps.begin_step(overlap=self.overlap_comm and self._tuned)
        # weight gradients on a second stream, overlapped with the data-gradient chain, and the model's
        # independent branches on branch streams (ops/streams.py); not in the first step, whose
        # autotuning times kernels on the current stream
        overlap = self.overlap_wgrad and self._tuned and streams.begin(self.ps.flat.device,
                                                                        branches=self.branch_streams)
        t1 = t0
        try:
            with trace_range("forward"):
                out = self.model(x)
                loss = self.loss_fn(out, y)
            t1 = time.perf_counter()
            self._mark(1)
            with trace_range("backward"):
                loss.backward()
        finally:
            if overlap:
                self.side_ops = streams.end()  # every stream joined before the PS reads the gradients
        self._mark(2)
        # host seconds spent issuing the forward / the backward (eager steps; the GPU runs behind)
        self.host_fwd_s, self.host_bwd_s = t1 - t0, time.perf_counter() - t1
        self._tuned = True
        if ps_step:
            self._ps_step()
            self._mark(3)
        return loss

    def _ps_step(self):
        with trace_range("ps push/apply/pull"):
            self.ps.step()
        if self.wt is not None:
            self.wt.refresh()  # the dgrads of the next step read the updated weights
        if self.wx3 is not None:
            self.wx3.refresh()  # ... and the x3 convs their weight planes

    def _eager_step(self, x, y):
        if self.arena is not None:
            with self.arena:
                loss = self._body(x, y)
        else:
            loss = self._body(x, y)
        heartbeat()
        self._gc_tick()
        return loss.detach()

    def _gc_tick(self) -> None:
        """GC policy of the eager loop (GC_MODE): called once per step, after the step is issued."""
        n = self._gc_steps = getattr(self, "_gc_steps", 0) + 1
        if GC_MODE == "freeze":
            if n == 1:
                gc.collect()
                gc.freeze()
        elif GC_MODE == "off":
            if n == 1:
                gc.collect()
                gc.freeze()
                gc.disable()
            elif n % GC_EVERY == 0:
                gc.collect()

    def _compute_stream(self):
        """The high-priority stream the step's critical chain runs on (None: the caller's stream).

        The weight gradients and the bucketed communication run on their own default-priority
        streams.  At equal priority the command processor hands freed CUs to whichever queue
        dispatched first, so a wide split-K wgrad grid issued just before a data-gradient kernel
        (the side stream forks at every layer) occupies the CUs that dgrad -- the critical path --
        waits for (rocprofv3: 50-100 us gaps on the compute queue after each BN backward).  With the
        compute queue at the higher priority, the side stream's workgroups only fill what it leaves
        idle.  Opt-in (``TONY_PRIO_STREAM=1``): it measured slower (see PRIO_STREAM)."""
        if not PRIO_STREAM or self.ps.flat.device.type != "cuda":
            return None
        if self._prio is None:
            lo, hi = torch.cuda.Stream.priority_range()  # (lowest, highest): e.g. (0, -1)
            self._prio = torch.cuda.Stream(device=self.ps.flat.device, priority=hi) if hi != lo else False
        return self._prio or None

    def step(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        wt_cache.activate(self.wt, self.wx3)
        try:
            s = self._compute_stream()
            if s is None:
                return self._step(x, y)
            cur = torch.cuda.current_stream(s.device)
            s.wait_stream(cur)  # inputs written on the caller's stream
            with torch.cuda.stream(s):
                loss = self._step(x, y)
            cur.wait_stream(s)  # the caller may read the loss / parameters on its stream
            return loss
        finally:
            wt_cache.activate(None)

    def _step(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        if not self.use_graph:
            return self._eager_step(x, y)
        if self.graph is None:
            if self._eager_steps < self.warmup_eager:
                # warm up on a side stream (allocator pools, MIOpen solution search)
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    loss = self._eager_step(x, y)
                torch.cuda.current_stream().wait_stream(s)
                self._eager_steps += 1
                return loss
            self._capture(x, y)
        if x.data_ptr() != self.static_x.data_ptr():
            self.static_x.copy_(x, non_blocking=True)
        if y.data_ptr() != self.static_y.data_ptr():
            self.static_y.copy_(y, non_blocking=True)
        self._refresh_hp()
        if self.plan is not None and self.plan_buckets:
            self._replay_overlapped()
            heartbeat()
            return self.static_loss
        if self.plan is not None:
            self.plan.replay()
        else:
            self.graph.replay()
        if self.graph_collectives:
            self.ps.steps += 1
            for opt in self.ps.optimizers.values():
                opt.step_count += 1
        else:
            self._ps_step()  # eager push/apply/pull; ps.step() advances the counters itself
        heartbeat()
        return self.static_loss

    def _replay_overlapped(self):
        """Several ranks: the plan segment by segment, each gradient bucket's push / apply / pull
        issued on the communication stream right after the segment that completes it -- the eager
        step's overlap of communication with backward, at the plan's host cost."""
        eng = self.ps.engine
        self.ps.begin_step(overlap=True)
        for k, bi in enumerate(eng.marked):
            self.plan.replay(k, eng.comm)
            eng.replay_launch(eng.buckets[bi])
        self.plan.replay(len(eng.marked))
        self._ps_step()  # the buckets not complete before the end of backward, the join, the weight cache

    def _refresh_hp(self):
        for opt in self.ps.optimizers.values():
            opt.step_count += 1
            opt._push_hp()
            opt.step_count -= 1

    def _capture(self, x, y):
        self.static_x = x
        self.static_y = y
        torch.cuda.synchronize()
        native = REPLAY == "plan"
        g = torch.cuda.CUDAGraph(keep_graph=True) if native else torch.cuda.CUDAGraph()
        self._refresh_hp()
        inside = self.graph_collectives
        # several ranks + native replay: the buckets' launch points are captured as plan markers, so
        # replays can overlap the collectives (which stay outside the graph) with backward
        eng = getattr(self.ps, "engine", None)
        # (``attached``, not ``_hooks``: after the first step every fused-reported parameter's hook is
        # dropped, and testing the hooks disabled the markers -- buckets then all launched after backward)
        markers = native and not inside and self.overlap_comm and eng is not None and eng.comm is not None \
            and eng.attached and os.environ.get("TONY_PLAN_MARKERS", "1") != "0"  # =0: round 3's failing form

        def body():
            if markers:
                eng.begin(overlap=True, markers=True)
            out = self._body(self.static_x, self.static_y, ps_step=inside)
            if markers:
                eng.end_capture()
            return out

        # weight gradients join the side stream PLAN_WGRAD_BATCH ops per fork inside the capture (round 4
        # measured one per fork best, 13.61 vs 13.68 ms, profiles/r4_ab_plan_wgrad_batch.log; with round 6's
        # kernels four per fork: 13.56 vs 14.19 ms, profiles/r6_plan_wgrad_batch.log)
        batch, streams.BATCH = streams.BATCH, PLAN_WGRAD_BATCH
        try:
            with torch.cuda.graph(g):
                if self.arena is not None:
                    with self.arena:  # its one fill is a node of the graph; the slices keep their addresses
                        loss = body()
                else:
                    loss = body()
                self.static_loss = loss.detach()
        finally:
            streams.BATCH = batch
        if inside:
            self.ps.steps -= 1  # the capture itself did not train
            for opt in self.ps.optimizers.values():
                opt.step_count -= 1
        self.graph = g
        self.plan = None
        self.plan_buckets = False
        self.replay_kind = "graph"
        if native:
            from ..ops.plan import PlanUnsupported, StepPlan

            dev = self.ps.flat.device
            try:
                # the compute stream the step is issued on, then the weight-gradient side stream and
                # the branch streams: the streams the eager step runs on
                self.plan = StepPlan(g, [streams.current(dev.index), *streams.plan_streams(dev)])
                self.replay_kind = "plan"
                if markers:
                    ids = [m for k, _, m in self.plan.ops() if k == 5]
                    self.plan_buckets = ids == list(range(len(eng.marked))) and \
                        self.plan.segments == len(eng.marked) + 1
                    if not self.plan_buckets:  # markers out of order: replay whole, buckets after
                        self.plan_error = f"plan markers {ids} vs buckets {eng.marked}"
            except PlanUnsupported as e:
                self.plan_error = str(e)
                g.instantiate()
        if self.wt is not None:
            self.wt.frozen = True  # the captured refresh() holds the current work list
        if self.wx3 is not None:
            self.wx3.frozen = True
