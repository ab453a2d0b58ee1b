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


def begin(device) -> bool:
    """Route in-place weight gradients to the side stream until ``end()``; False when disabled."""
    device = torch.device(device)
    if not ENABLED or device.type != "cuda":
        return False
    _active[0] = _side(device)
    _issued[0] = 0
    return True


def active() -> bool:
    return _active[0] is not None


def run(fn: Callable[[], object], *keep: torch.Tensor):
    """Run ``fn`` (which must write its result in place and return None) on the side stream when one
    is active, else right here.  ``keep``: tensors ``fn`` reads that the caller may drop."""
    side = _active[0]
    if side is None:
        return fn()
    side.wait_stream(torch.cuda.current_stream(side.device))
    with torch.cuda.stream(side):
        out = fn()
    assert out is None, "only in-place gradient work may run on the side stream"
    with _lock:
        _keep.extend(keep)
        _issued[0] += 1
    return None


def end() -> int:
    """Join the side stream into the current stream and release the kept operands; returns how many
    ops ran on the side stream this step."""
    side = _active[0]
    _active[0] = None
    if side is not None:
        torch.cuda.current_stream(side.device).wait_stream(side)
    with _lock:
        _keep.clear()
        n, _issued[0] = _issued[0], 0
    return n
