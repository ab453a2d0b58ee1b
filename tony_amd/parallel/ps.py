"""Parameter-server training with TF ParameterServerStrategy semantics, MI355X-native.

TonY runs TF PS jobs as ``ps`` + ``worker`` tasks wired together by ``TF_CONFIG``
(reference: ``T/runtime/TFRuntime.java:45-59``, ``EX/mnist-tensorflow/mnist_distributed.py:206-241``):
the ``ps`` tasks hold the variables and apply the optimizer; workers pull the
variables, compute gradients and push them back.  TF itself is not part of this
stack, so this module implements those semantics directly on HBM and xGMI.

Every gradient exchange is BUCKETED and OVERLAPPED with backward (parallel/buckets.py): the flat
gradient buffer is cut into ~8 MB buckets in reverse layer order; as soon as the last gradient of
a bucket is written (reported by the fused HIP ops or AccumulateGrad) the bucket's push, apply and
pull are enqueued on a communication stream while backward keeps running on the compute streams.
Only the last bucket (the stem's gradients) is exposed after backward.

``mode="colocated"`` (default, the benchmark topology)
    One PS shard per GPU process.  Each bucket is split evenly over the shards (rank r owns the
    r-th piece of every bucket: TF's ``replica_device_setter`` spreads variables over ps tasks, here
    balanced to the byte).  Per bucket:
    push  = ``reduce_scatter`` of the bucket (each shard receives the sum of its piece from every
            worker over all 7 xGMI links);
    apply = one fused HIP optimizer launch over the piece of the shard's fp32 master copy, writing
            the new bf16 variables straight into this rank's piece of the flat parameter buffer;
    pull  = in-place ``all_gather`` of the bucket's pieces into every worker's flat parameters.
``mode="dedicated"``
    The paper topology (1 ps + N workers).  PS ranks own the variables and run no model; bucket b
    belongs to ps task ``b % n_ps`` (round-robin placement, ``replica_device_setter``).
    ``plane="xgmi"`` (default on GPUs, parallel/ps_plane.py + csrc/ps_plane.hip): per bucket the
    workers store their gradients straight into the owner's IPC-mapped receive rows (push), the
    owner GPU applies the fused optimizer chunk by chunk as the rows land and stores the new
    variables straight into every worker's landing window (apply + pull in one kernel), and each
    worker copies its landing window into its parameters after backward.  ``sync=False`` gives an
    *asynchronous* PS on the same plane: every worker's push is applied on its own as it arrives
    (no averaging, no waiting for the others' pushes before applying it) and lands only in that
    worker's window.  Unlike TF's unbounded async PS it is bounded-staleness-1: the ps issues one
    apply kernel per bucket and step, which finishes once it has applied every worker's push of
    that step, so a fast worker can run at most one step ahead of the slowest; the optimizer's step
    counter (Adam's bias correction) advances once per ps step, not per applied push.  ``plane="rccl"`` (and CPU / gloo runs): push =
    ``reduce`` to the owner, apply, pull = ``broadcast``; async = point-to-point send/recv of the
    whole flat gradient with the PS polling the outstanding receives.

Gradients are averaged over workers (TF SyncReplicasOptimizer semantics) by the optimizer's
``grad_scale``.  ``wire_dtype=torch.float32`` pushes and sums fp32 gradients (the reference TF job
is fp32 end to end) even when the gradient buffer the kernels accumulate into is bf16.
"""
from __future__ import annotations

import math
import os
import time
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..ops.optim import FlatAdam, FlatSGD
from . import collectives as coll
from .buckets import DEFAULT_BUCKET_MB, Bucket, GradBucketEngine, make_buckets
from .flat import FlatParams


def make_optimizer(kind: str, master: torch.Tensor, lr: float, momentum: float = 0.9, weight_decay: float = 0.0,
                   **kw):
    kind = kind.lower()
    if kind in ("sgd", "momentum"):
        return FlatSGD(master, lr, momentum=momentum, weight_decay=weight_decay, nesterov=kw.get("nesterov", False))
    if kind in ("adam", "adamw"):
        return FlatAdam(master, lr, betas=kw.get("betas", (0.9, 0.999)), eps=kw.get("eps", 1e-8),
                        weight_decay=weight_decay, decoupled=(kind == "adamw"))
    raise ValueError(f"unknown optimizer {kind!r}")


def _wait(work) -> None:
    """Make the current stream wait for an async collective (no host block on RCCL)."""
    if work is not None:
        work.wait()


class ParameterServer:
    """Owns the variables of a model (sharded or dedicated) and runs bucketed push/apply/pull."""

    def __init__(self, model: torch.nn.Module, optimizer: str = "sgd", lr: float = 0.1, momentum: float = 0.9,
                 weight_decay: float = 0.0, mode: str = "colocated", sync: bool = True, ps_ranks=(0,),
                 group=None, dtype=torch.bfloat16, device=None, wire_dtype: Optional[torch.dtype] = None,
                 bucket_mb: float = DEFAULT_BUCKET_MB, bucketed_single: bool = False, plane: str = "auto",
                 **opt_kw):
        self.mode = mode
        self.sync = sync
        self.group = group
        self.world = coll.world(group)
        self.rank = coll.rank(group)
        if mode == "colocated":
            self.ps_ranks = list(range(self.world))
            self.worker_ranks = list(range(self.world))
        elif mode == "dedicated":
            self.ps_ranks = sorted(ps_ranks)
            self.worker_ranks = [r for r in range(self.world) if r not in self.ps_ranks]
            if not self.worker_ranks:
                raise ValueError("dedicated PS needs at least one worker rank")
            if not sync and len(self.ps_ranks) != 1:
                raise ValueError("asynchronous PS supports exactly one ps task")
        else:
            raise ValueError(f"unknown PS mode {mode!r}")
        self.is_ps = self.rank in self.ps_ranks
        self._begun = False
        self.is_worker = self.rank in self.worker_ranks
        n_split = self.world if mode == "colocated" else 1
        # every bucket must split into n_split pieces of whole 16-byte vectors (8 bf16)
        align = 64 * (8 * n_split) // math.gcd(64, 8 * n_split)
        self.flat = FlatParams(model, dtype=dtype, device=device, world=n_split, align=align)
        self.wire_dtype = wire_dtype or self.flat.grad.dtype
        # every rank starts from rank 0's variables
        coll.broadcast(self.flat.data, src=0, group=group)
        self.buckets: List[Bucket] = make_buckets(self.flat, bucket_mb, multiple=8 * n_split)
        self.steps = 0
        self.push_bytes = 0
        self.optimizers: Dict[int, object] = {}
        # per bucket: (offset into this rank's master shard, length) -- None where this rank owns nothing
        self._master_range: List[Optional[tuple]] = [None] * len(self.buckets)
        f = self.flat
        if mode == "colocated":
            # master pieces in flat order (ascending lo): with one rank the master shard IS the flat
            # buffer's layout and the whole update is one fused launch
            pieces, m = [], 0
            for b in sorted(self.buckets, key=lambda b: b.lo):
                p = b.numel // n_split
                self._master_range[b.index] = (m, p)
                pieces.append(f.data[b.lo + self.rank * p:b.lo + (self.rank + 1) * p])
                m += p
            master = torch.cat(pieces).float()
            opt = make_optimizer(optimizer, master, lr, momentum, weight_decay, **opt_kw)
            opt.grad_scale = 1.0 / len(self.worker_ranks)
            self.optimizers[self.rank] = opt
            self._gshard = torch.zeros(m, dtype=self.wire_dtype, device=f.device) if self.world > 1 else None
        elif sync:
            m, pieces = 0, []
            for b in self.buckets:
                if self._owner(b) == self.rank:
                    self._master_range[b.index] = (m, b.numel)
                    pieces.append(f.data[b.lo:b.hi])
                    m += b.numel
            if pieces:
                master = torch.cat(pieces).float()
                opt = make_optimizer(optimizer, master, lr, momentum, weight_decay, **opt_kw)
                opt.grad_scale = 1.0 / len(self.worker_ranks)
                self.optimizers[self.rank] = opt
        else:  # asynchronous: the single ps task owns the whole buffer (masters in flat order)
            if self.is_ps:
                opt = make_optimizer(optimizer, f.data.float().clone(), lr, momentum, weight_decay, **opt_kw)
                self.optimizers[self.rank] = opt
                for b in self.buckets:
                    self._master_range[b.index] = (b.lo, b.numel)
        if plane == "auto":
            # tony.amd.ps-plane (TONY_PS_PLANE) selects the GPU data plane; CPU tensors always take the
            # collective path (gloo)
            plane = os.environ.get("TONY_PS_PLANE", "xgmi") if f.device.type == "cuda" else "rccl"
        self.plane_kind = plane if mode == "dedicated" and self.world > 1 else "rccl"
        if self.plane_kind not in ("xgmi", "rccl"):
            raise ValueError(f"unknown PS data plane {plane!r}")
        if self.plane_kind == "xgmi" and f.device.type != "cuda":
            raise ValueError("the xGMI PS data plane needs GPU tensors")
        self.plane = None
        if self.plane_kind == "xgmi":
            from .ps_plane import XgmiPSPlane

            if not sync:
                for opt in self.optimizers.values():
                    opt.grad_scale = 1.0  # async: every push is applied on its own
            from .ps_plane import PSPlaneError

            try:
                self.plane = XgmiPSPlane(f, self.buckets, self._owner, self.ps_ranks, self.worker_ranks, self.rank,
                                         self.wire_dtype, group=group, sync=sync)
                coll._STATUS["ps_plane"] = "verified"
            except PSPlaneError as e:  # the init-time canary failed on some rank: every rank gets here
                import warnings

                warnings.warn(f"{e}; the parameter server falls back to the collective (RCCL) data plane",
                              RuntimeWarning)
                coll._STATUS["ps_plane"] = f"failed: {e}"
                self.plane_kind = "rccl"
                for opt in self.optimizers.values():
                    opt.grad_scale = 1.0 / len(self.worker_ranks) if sync else 1.0
        self._wire = None
        if self.world > 1 and self.wire_dtype != f.grad.dtype and self.plane is None:
            self._wire = torch.zeros(f.numel, dtype=self.wire_dtype, device=f.device)
        self.engine = GradBucketEngine(f, self.buckets, self._launch)
        # one rank: nothing to communicate, so nothing to overlap -- the step is ONE fused apply over
        # the whole shard after backward, with no per-parameter readiness bookkeeping on the host
        # (``bucketed_single`` keeps the bucket engine: tests of the overlap machinery on one GPU)
        self.single = mode == "colocated" and self.world == 1 and not bucketed_single
        if (mode == "colocated" or sync or self.plane is not None) and not self.single and \
                not (self.plane is not None and not self.is_worker):
            self.engine.attach()

    # -- helpers ---------------------------------------------------------------
    def zero_grad(self):
        self.flat.zero_grad()

    @property
    def params(self):
        return self.flat.params

    def _owner(self, b: Bucket) -> int:
        return self.ps_ranks[b.index % len(self.ps_ranks)]

    @property
    def comm_stream(self):
        return self.engine.comm

    # -- the PS step -----------------------------------------------------------
    def begin_step(self, overlap: bool = True):
        """Arm the bucket engine before the forward: with ``overlap`` each bucket's push/apply/pull is
        enqueued as soon as backward completes its gradients."""
        if self.plane is not None:
            if self.is_worker:
                self.engine.begin(overlap)  # pushes launch from backward; the ps's hp go out in step()
            return
        if self.mode == "dedicated" and not self.sync:
            return
        for opt in self.optimizers.values():
            opt.begin_step()
        if self.single:
            self._begun = True
            return
        if self.mode == "dedicated" and not self.is_worker:
            self.flat.grad.zero_()  # a PS-only rank contributes nothing to the pushed sums
            overlap = False         # and runs no backward: all buckets go in order from step()
        self.engine.begin(overlap)

    def step(self):
        """Finish push (gradients) -> apply (fused optimizer on the PS) -> pull (variables)."""
        if self.plane is not None:
            self._step_plane()
            self.steps += 1
            return
        if self.mode == "dedicated" and not self.sync:
            self._step_dedicated_async_worker()
            self.steps += 1
            return
        if self.single:
            if not self._begun:
                self.begin_step()
            self._begun = False
            opt = self.optimizers[self.rank]
            self._apply(opt, self.flat.grad, 0, self.flat.data)
            self.steps += 1
            return
        if not self.engine.armed:
            self.begin_step(overlap=False)
        self.engine.end()
        self.steps += 1

    @property
    def overlapped_buckets(self) -> int:
        """Buckets of the last step whose communication was issued while backward was running."""
        return self.engine.launched_during_backward

    def _step_plane(self):
        """One step on the xGMI data plane.  Worker: the remaining pushes, then the landing of every
        bucket's new variables (on the communication stream), joined into the compute stream.  PS:
        the previous step's applies must be done before this step's hyper-parameters go to the
        device (Adam's bias corrections change every step), then one apply per owned bucket, in
        bucket order -- each waits on the GPU for its rows, so the host is not in the loop."""
        pl = self.plane
        if self.is_worker:
            if not self.engine.armed:
                self.engine.begin(False)
            self.engine.end(finish=lambda: pl.land(self.steps))
            return
        # no host synchronisation: this step's hyper-parameters reach the device by a copy ordered on
        # the stream after the previous step's applies, and every apply waits on the GPU for its rows,
        # so the ps host runs ahead like the workers' 
        opt = self.optimizers.get(self.rank)
        if opt is None:
            return
        opt.begin_step()
        for b in self.buckets:
            if self._owner(b) == self.rank:
                m, _ = self._master_range[b.index]
                pl.apply(b, self.steps, opt, m, local_params=self.flat.data)
        pl.end_step()

    def _wire_grad(self, b: Bucket) -> torch.Tensor:
        g = self.flat.grad[b.lo:b.hi]
        if self._wire is not None:
            w = self._wire[b.lo:b.hi]
            w.copy_(g)
            return w
        return g

    def _launch(self, b: Bucket):
        """Enqueue bucket b's push / apply / pull (the communication stream is current)."""
        f = self.flat
        if self.plane is not None:  # worker: straight into the owner's receive rows (push)
            self.plane.push(b, self.steps)
            return
        opt = self.optimizers.get(self.rank)
        if self.mode == "colocated":
            m, p = self._master_range[b.index]
            own = f.data[b.lo + self.rank * p:b.lo + (self.rank + 1) * p]
            if self.world == 1:
                self._apply(opt, f.grad[b.lo:b.hi], m, own)
                return
            g = self._wire_grad(b)
            gs = self._gshard[m:m + p]
            _wait(coll.reduce_scatter_flat(gs, g, group=self.group, async_op=True))     # push
            self._apply(opt, gs, m, own)                                                  # apply (HIP)
            _wait(coll.all_gather_flat(f.data[b.lo:b.hi], own, group=self.group, async_op=True))  # pull
            self.push_bytes += g.numel() * g.element_size()
            return
        owner = self._owner(b)
        g = self._wire_grad(b)
        _wait(dist.reduce(g, dst=owner, group=self.group, async_op=True))                # push
        if self.rank == owner:
            m, _ = self._master_range[b.index]
            self._apply(opt, g, m, f.data[b.lo:b.hi])                                     # apply
        _wait(dist.broadcast(f.data[b.lo:b.hi], src=owner, group=self.group, async_op=True))  # pull
        if self.is_worker:
            self.push_bytes += g.numel() * g.element_size()

    def _apply(self, opt, grad: torch.Tensor, m: int, out: torch.Tensor):
        if out.dtype == torch.bfloat16 or not out.is_cuda:
            opt.apply_range(grad, m, out_bf16=out)
        else:  # fp32 variables (reference-precision runs): the master range IS the new value
            opt.apply_range(grad, m, out_bf16=None)
            out.copy_(opt.w[m:m + out.numel()])

    def _step_dedicated_async_worker(self):
        f = self.flat
        ps = self.ps_ranks[0]
        dist.send(f.grad, dst=ps, group=self.group)
        dist.recv(f.data, src=ps, group=self.group)

    def serve_async(self, total_pushes: int, poll_s: float = 0.0005):
        """Run the asynchronous PS loop on the ps rank: apply each worker push on arrival."""
        if not self.is_ps or self.sync or self.mode != "dedicated":
            raise RuntimeError("serve_async runs on the ps rank of an async dedicated PS")
        f = self.flat
        opt = self.optimizers[self.rank]
        opt.grad_scale = 1.0  # async: every push is applied on its own
        if total_pushes % len(self.worker_ranks):
            raise ValueError("total_pushes must be steps x number of workers")
        per_worker = total_pushes // len(self.worker_ranks)
        if coll._is_gloo(self.group):
            # gloo cannot poll a pending irecv; it can receive from ANY source instead
            buf = torch.empty_like(f.grad)
            for done in range(total_pushes):
                w = dist.recv(buf, group=self.group)  # returns the sender's global rank
                opt.begin_step()
                self._apply(opt, buf, 0, f.data)
                dist.send(f.data, dst=w, group=self.group)
            self.steps = total_pushes
            return
        bufs = {w: torch.empty_like(f.grad) for w in self.worker_ranks}
        got = {w: 0 for w in self.worker_ranks}
        reqs = {w: dist.irecv(bufs[w], src=w, group=self.group) if per_worker else None for w in self.worker_ranks}
        done = 0
        while done < total_pushes:
            progressed = False
            for w, req in list(reqs.items()):
                if req is None or not req.is_completed():
                    continue
                req.wait()
                opt.begin_step()
                self._apply(opt, bufs[w], 0, f.data)        # apply on arrival
                dist.send(f.data, dst=w, group=self.group)  # the worker's pull
                done += 1
                got[w] += 1
                progressed = True
                # each worker pushes exactly per_worker times: repost only for its own next push
                reqs[w] = dist.irecv(bufs[w], src=w, group=self.group) if got[w] < per_worker else None
            if not progressed:
                time.sleep(poll_s)
        self.steps = done

    # -- checkpoint ------------------------------------------------------------
    def layout(self) -> dict:
        """What a shard checkpoint is only valid for (restoring under another layout is refused)."""
        return {"mode": self.mode, "world": self.world, "ps_ranks": list(self.ps_ranks), "numel": self.flat.numel,
                "buckets": [(b.lo, b.hi) for b in self.buckets]}

    def state_dict(self):
        """This rank's part of the PS state: the bf16/fp32 variables plus the fp32 master and
        optimizer state of the shard it owns (every rank saves its own file, utils/checkpoint.py)."""
        sd = {"steps": self.steps, "flat": self.flat.data.detach().clone(), "layout": self.layout(),
              "rank": self.rank, "shards": {}}
        for r, opt in self.optimizers.items():
            sd["shards"][r] = {"master": opt.w.detach().clone(), "opt": opt.state_dict()}
        return sd

    def load_state_dict(self, sd):
        if sd.get("layout") is None:
            raise ValueError("PS checkpoint has no 'layout' record (an older format whose shard order cannot be "
                             "verified): refusing to load it")
        if sd["layout"] != self.layout():
            raise ValueError(f"PS checkpoint layout {sd['layout']} does not match this job's {self.layout()}")
        self.steps = int(sd["steps"])
        self.flat.data.copy_(sd["flat"])
        for r, opt in self.optimizers.items():
            s = sd["shards"][r]
            opt.w.copy_(s["master"])
            opt.load_state_dict(s["opt"])
