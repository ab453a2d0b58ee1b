"""Data-parallel gradient all-reduce: flat buckets, launched during backward.

Covers the synchronous-DP rows of SURVEY.md §2.6: PyTorch DDP (the reference's
``EX/mnist-pytorch/mnist_distributed.py:113-126`` averages every parameter
with its own all_reduce on CPU tensors and a fresh group per call), TF
MultiWorkerMirroredStrategy and Horovod's DistributedOptimizer all reduce to
"average the gradients over the data-parallel ranks every step".

MI355X design:

* parameters and gradients live in ONE flat buffer (:class:`FlatParams`), so a
  bucket is a contiguous slice of the gradient buffer: no pack/unpack copies,
  one RCCL ``all_reduce`` per bucket;
* buckets are cut in reverse registration order (the order backward produces
  gradients) and sized for xGMI: a ring all-reduce on 8 GPUs moves
  2*(N-1)/N of the bucket over each of the 7 links, so ~32 MB buckets keep
  every launch well past the latency-bound regime (a few us at 150 GB/s per
  link) while still giving the collective stream work to overlap with the
  remaining backward kernels;
* a bucket is launched (``async_op=True``, RCCL's own stream waits on the
  compute stream only for that bucket) from the post-accumulate-grad hook of
  its last parameter; a callback queued on the autograd engine launches the
  leftovers (parameters whose gradient is written in place by a fused kernel
  never fire the hook) and joins every bucket before ``backward()`` returns;
* averaging uses ``ReduceOp.AVG`` on RCCL (one pass) and SUM + scale on gloo.
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.distributed as dist

from . import collectives as coll
from .flat import FlatParams

DEFAULT_BUCKET_MB = 32


@dataclass
class Bucket:
    lo: int
    hi: int
    params: List[int] = field(default_factory=list)
    pending: int = 0
    work: Optional[object] = None
    launched: bool = False


class BucketedAllReduce:
    """Average ``flat.grad`` over ``group`` in buckets overlapped with backward."""

    def __init__(self, flat: FlatParams, bucket_mb: float = DEFAULT_BUCKET_MB, group=None, average: bool = True,
                 compression: Optional[torch.dtype] = None):
        self.flat = flat
        self.group = group
        self.world = coll.world(group)
        self.average = average
        self.compression = compression
        cap = max(1, int(bucket_mb * 2 ** 20 // flat.grad.element_size()))
        self.buckets: List[Bucket] = []
        self.bucket_of: List[int] = [0] * len(flat.slots)
        cur: Optional[Bucket] = None
        ends = [s.offset for s in flat.slots[1:]] + [flat.numel]
        for i in reversed(range(len(flat.slots))):
            s = flat.slots[i]
            if cur is None:
                cur = Bucket(s.offset, ends[i])
            cur.lo = s.offset
            cur.params.append(i)
            self.bucket_of[i] = len(self.buckets)
            if cur.hi - cur.lo >= cap:
                self.buckets.append(cur)
                cur = None
        if cur is not None:
            self.buckets.append(cur)
        self.buckets[0].hi = flat.numel  # tail padding rides with the first bucket
        self.enabled = True
        self.passes_per_reduce = 1   # gradient accumulation: reduce on every k-th backward
        self._pass = 0
        self._armed = False
        self._active = False
        self._hooks = []
        self.launches = 0

    # -- backward integration -----------------------------------------------------------
    def register_hooks(self) -> None:
        for i, p in enumerate(self.flat.params):
            self._hooks.append(p.register_post_accumulate_grad_hook(lambda p, i=i: self._on_grad(i, p)))

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []

    def _arm(self) -> None:
        self._armed = True
        k = max(1, int(self.passes_per_reduce))
        self._active = self.enabled and self._pass % k == k - 1
        for b in self.buckets:
            b.pending, b.work, b.launched = len(b.params), None, False
        torch.autograd.Variable._execution_engine.queue_callback(self.finish)

    def _on_grad(self, i: int, p: torch.Tensor) -> None:
        if self.world == 1:
            return
        if not self._armed:
            self._arm()
        view = self.flat.slots[i].view(self.flat.grad)
        if p.grad is not None and p.grad.data_ptr() != view.data_ptr():
            view.copy_(p.grad)  # user code replaced .grad (e.g. zero_grad(set_to_none=True))
            p.grad = view
        if not self._active:
            return
        b = self.buckets[self.bucket_of[i]]
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    def _launch(self, b: Bucket) -> None:
        if b.launched:
            return
        b.launched = True
        g = self.flat.grad[b.lo:b.hi]
        if self.compression is not None and g.dtype != self.compression:
            wire = g.to(self.compression)
            b.work = (self._all_reduce(wire), wire, g)
        else:
            b.work = (self._all_reduce(g), None, g)
        self.launches += 1

    def _all_reduce(self, t: torch.Tensor):
        if self.average and dist.get_backend(self.group) == "nccl":
            return dist.all_reduce(t, op=dist.ReduceOp.AVG, group=self.group, async_op=True)
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def finish(self) -> None:
        """Launch the remaining buckets and join them all (runs at the end of backward)."""
        if self.world == 1:
            self._armed = False
            return
        self._pass += 1
        if not self._active:
            self._armed = False
            return
        for b in self.buckets:
            self._launch(b)
        scale_needed = self.average and dist.get_backend(self.group) != "nccl"
        for b in self.buckets:
            work, wire, g = b.work
            work.wait()
            if wire is not None:
                if scale_needed:
                    wire.div_(self.world)
                g.copy_(wire)
            elif scale_needed:
                g.div_(self.world)
            b.work = None
        self._armed = False

    def all_reduce_now(self) -> None:
        """Synchronous path for callers that fill ``flat.grad`` themselves (no hooks)."""
        if self.world == 1:
            return
        self._armed, self._active = True, True
        for b in self.buckets:
            b.launched = False
        self.finish()
        self._pass -= 1  # not a backward pass


class DistributedDataParallel(torch.nn.Module):
    """DDP over a flat parameter buffer: broadcast rank 0's weights, average grads in buckets.

    ``model(x)`` / ``loss.backward()`` work as usual; when ``backward`` returns
    the gradients (``p.grad`` = views of ``self.flat.grad``) are averaged.  Use
    :meth:`no_sync` for gradient accumulation steps.
    """

    def __init__(self, module: torch.nn.Module, bucket_mb: float = DEFAULT_BUCKET_MB, group=None,
                 dtype: Optional[torch.dtype] = None, device=None, compression: Optional[torch.dtype] = None,
                 broadcast_buffers: bool = True):
        super().__init__()
        self.module = module
        dtypes = {p.dtype for p in module.parameters() if p.requires_grad}
        if dtype is None:
            if len(dtypes) != 1:
                raise TypeError(f"parameters have mixed dtypes {dtypes}; pass dtype=")
            dtype = dtypes.pop()
        self.group = group
        self.flat = FlatParams(module, dtype=dtype, device=device, world=1)
        coll.broadcast(self.flat.data, src=0, group=group)
        self.broadcast_buffers = broadcast_buffers
        if broadcast_buffers:
            for b in module.buffers():
                coll.broadcast(b, src=0, group=group)
        self.reducer = BucketedAllReduce(self.flat, bucket_mb, group, average=True, compression=compression)
        self.reducer.register_hooks()

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        old = self.reducer.enabled
        self.reducer.enabled = False
        try:
            yield
        finally:
            self.reducer.enabled = old

    def zero_grad(self, set_to_none: bool = False):  # noqa: ARG002 - grads are views of one buffer
        self.flat.zero_grad()
        self.flat.rebind_grads()
