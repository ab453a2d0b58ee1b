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
  gradients) and sized for xGMI (parallel/buckets.py);
* a bucket launches as soon as all its gradients are written -- reported by the
  fused HIP ops, which accumulate parameter gradients in place and never reach
  AccumulateGrad (``_lib.grads_ready``), and by post-accumulate-grad hooks for
  every other parameter -- on a dedicated communication stream forked from the
  compute and weight-gradient streams, strictly in bucket order so all ranks
  issue the same collective sequence;
* the first report of a backward pass arms the reducer and queues ``finish`` on
  the autograd engine, which launches the leftovers and joins the communication
  stream before ``backward()`` returns (no host block on RCCL);
* averaging uses ``ReduceOp.AVG`` on RCCL (one pass) and SUM + scale on gloo.
"""
from __future__ import annotations

import contextlib
from typing import List, Optional

import torch

from . import collectives as coll
from .buckets import DEFAULT_BUCKET_MB, Bucket, GradBucketEngine, make_buckets
from .flat import FlatParams


class BucketedAllReduce:
    """Average ``flat.grad`` over ``group`` in buckets overlapped with backward."""

    def __init__(self, flat: FlatParams, bucket_mb: float = DEFAULT_BUCKET_MB, group=None, average: bool = True,
                 compression: Optional[torch.dtype] = None, predivide: float = 1.0):
        self.flat = flat
        # Horovod's gradient_predivide_factor f: scale by 1/f before a SUM, by f/size after
        self.predivide = float(predivide)
        if self.predivide <= 0:
            raise ValueError("gradient_predivide_factor must be positive")
        self.group = group
        self.world = coll.world(group)
        self.average = average
        self.compression = compression
        self.buckets: List[Bucket] = make_buckets(flat, bucket_mb)
        self.engine = GradBucketEngine(flat, self.buckets, self._launch)
        self.engine.auto_arm = self._arm
        self.enabled = True
        self.passes_per_reduce = 1   # gradient accumulation: reduce on every k-th backward
        self._pass = 0
        self._active = False

    @property
    def launches(self) -> int:
        return self.engine.launches

    @property
    def overlapped_buckets(self) -> int:
        return self.engine.launched_during_backward

    # -- backward integration -----------------------------------------------------------
    def register_hooks(self) -> None:
        self.engine.attach()

    def remove_hooks(self) -> None:
        self.engine.detach()

    def _arm(self) -> None:
        k = max(1, int(self.passes_per_reduce))
        self._active = self.world > 1 and self.enabled and self._pass % k == k - 1
        self.engine.begin(overlap=self._active)
        torch.autograd.Variable._execution_engine.queue_callback(self.finish)

    def _launch(self, b: Bucket) -> None:
        """Enqueue bucket b's all-reduce (the communication stream is current on the GPU).  Goes through
        parallel/collectives.py, so TONY_COLLECTIVE=hip (tony.amd.collective) runs it on the xGMI
        kernels and RCCL stays the A/B baseline; a fallback to RCCL is counted there."""
        g = self.flat.grad[b.lo:b.hi]
        wire = g.to(self.compression) if self.compression is not None and g.dtype != self.compression else g
        if self.predivide != 1.0:
            if wire is g:
                wire = g.clone()
            wire.mul_(1.0 / self.predivide)
        plain_avg = self.average and self.predivide == 1.0
        work = coll.all_reduce(wire, group=self.group, async_op=True, average=plain_avg)
        if work is not None:
            work.wait()  # the comm stream waits, not the host
        if self.average and not plain_avg:
            wire.mul_(self.predivide / self.world)
        if wire is not g:
            g.copy_(wire)

    def finish(self) -> None:
        """Launch the remaining buckets and join them (runs at the end of backward)."""
        self._pass += 1
        if not self._active:
            self.engine.cancel()
            return
        self.engine.end()

    def all_reduce_now(self) -> None:
        """Synchronous path for callers that fill ``flat.grad`` themselves (no hooks)."""
        if self.world == 1:
            return
        self._active = True
        self.engine.begin(overlap=False)
        self.engine.end()


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
