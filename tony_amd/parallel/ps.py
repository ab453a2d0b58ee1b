"""Parameter-server training with TF ParameterServerStrategy semantics, MI355X-native.

TonY runs TF PS jobs as ``ps`` + ``worker`` tasks wired together by ``TF_CONFIG``
(reference: ``T/runtime/TFRuntime.java:45-59``, ``EX/mnist-tensorflow/mnist_distributed.py:206-241``):
the ``ps`` tasks hold the variables and apply the optimizer; workers pull the
variables, compute gradients and push them back.  TF itself is not part of this
stack, so this module implements those semantics directly on HBM and xGMI:

``mode="colocated"`` (default, the benchmark topology)
    One PS shard per GPU process.  Variables are partitioned over the shards
    (contiguous ranges of the flat buffer: TF's ``replica_device_setter``
    round-robin with a byte-balanced split).  A step is:
    push  = ``reduce_scatter`` of the flat bf16 gradient (each shard receives
            the sum of its range from every worker, over all 7 xGMI links);
    apply = ONE fused HIP optimizer launch over the shard's fp32 master copy,
            which also emits the bf16 copy;
    pull  = ``all_gather`` of the bf16 shards into every worker's flat params.
``mode="dedicated"``
    The paper topology (1 ps + N workers).  PS ranks own the variables and run
    no model; workers push with ``reduce`` to the owning PS and pull with
    ``broadcast``.  ``sync=False`` gives TF's default *asynchronous* PS: each
    worker's push is applied on arrival (point-to-point send/recv, PS polls
    the outstanding receives) and the worker pulls the post-apply variables.

Gradients are averaged over workers (TF SyncReplicasOptimizer semantics) by the
optimizer's ``grad_scale``.
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist

from ..ops.optim import FlatAdam, FlatSGD
from . import collectives as coll
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


class ParameterServer:
    """Owns the variables of a model (sharded or dedicated) and runs push/apply/pull."""

    def __init__(self, model: torch.nn.Module, optimizer: str = "sgd", lr: float = 0.1, momentum: float = 0.9,
                 weight_decay: float = 0.0, mode: str = "colocated", sync: bool = True, ps_ranks=(0,),
                 group=None, dtype=torch.bfloat16, device=None, **opt_kw):
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
        self.is_worker = self.rank in self.worker_ranks
        n_shards = len(self.ps_ranks)
        self.flat = FlatParams(model, dtype=dtype, device=device, world=n_shards)
        # every rank starts from PS shard 0's init: broadcast rank 0's variables
        coll.broadcast(self.flat.data, src=0, group=group)
        self.optimizers = {}
        for i, r in enumerate(self.ps_ranks):
            if r == self.rank:
                master = self.flat.shard(self.flat.data, i).float().clone()
                opt = make_optimizer(optimizer, master, lr, momentum, weight_decay, **opt_kw)
                opt.grad_scale = 1.0 / len(self.worker_ranks)
                self.optimizers[i] = opt
        self.steps = 0
        self.push_bytes = 0

    # -- helpers ---------------------------------------------------------------
    def zero_grad(self):
        self.flat.zero_grad()

    @property
    def params(self):
        return self.flat.params

    def _shard_index(self) -> int:
        return self.ps_ranks.index(self.rank)

    # -- the PS step -----------------------------------------------------------
    def step(self):
        """push (gradients) -> apply (fused optimizer on the PS) -> pull (variables)."""
        if self.mode == "colocated":
            self._step_colocated()
        elif self.sync:
            self._step_dedicated_sync()
        else:
            self._step_dedicated_async_worker()
        self.steps += 1

    def _step_colocated(self):
        f = self.flat
        i = self._shard_index()
        g_shard = f.shard(f.grad, i)
        coll.reduce_scatter_flat(g_shard, f.grad, group=self.group)       # push
        self.optimizers[i].step(g_shard, out_bf16=f.shard(f.data, i))       # apply (HIP)
        coll.all_gather_flat(f.data, f.shard(f.data, i), group=self.group)  # pull
        self.push_bytes += f.grad.numel() * f.grad.element_size()

    def _step_dedicated_sync(self):
        f = self.flat
        for i, ps in enumerate(self.ps_ranks):
            g = f.shard(f.grad, i)
            if self.is_ps and not self.is_worker:
                g.zero_()  # PS contributes nothing to the gradient sum
            dist.reduce(g, dst=ps, group=self.group)                          # push
            if self.rank == ps:
                self.optimizers[i].step(g, out_bf16=f.shard(f.data, i))       # apply
            dist.broadcast(f.shard(f.data, i), src=ps, group=self.group)      # pull

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
        opt = self.optimizers[0]
        opt.grad_scale = 1.0  # async: every push is applied on its own
        if total_pushes % len(self.worker_ranks):
            raise ValueError("total_pushes must be steps x number of workers")
        per_worker = total_pushes // len(self.worker_ranks)
        if coll._is_gloo(self.group):
            # gloo cannot poll a pending irecv; it can receive from ANY source instead
            buf = torch.empty_like(f.grad)
            for done in range(total_pushes):
                w = dist.recv(buf, group=self.group)  # returns the sender's global rank
                opt.step(buf, out_bf16=f.data)
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
                opt.step(bufs[w], out_bf16=f.data)          # apply on arrival
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
    def state_dict(self):
        sd = {"steps": self.steps, "flat": self.flat.data.detach().clone(), "shards": {}}
        for i, opt in self.optimizers.items():
            sd["shards"][i] = {"master": opt.w.detach().clone(), "opt": opt.state_dict()}
        return sd

    def load_state_dict(self, sd):
        self.steps = int(sd["steps"])
        self.flat.data.copy_(sd["flat"])
        for i, opt in self.optimizers.items():
            s = sd["shards"][i]
            opt.w.copy_(s["master"])
            opt.load_state_dict(s["opt"])
