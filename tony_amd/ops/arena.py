"""Per-step zero-initialised fp32 scratch for the fused kernels' accumulators.

Every fused BN / GEMM / conv launch accumulates into small fp32 buffers with atomics -- BatchNorm
sums in GEMM epilogues, BN-backward reductions, split-K weight gradients -- and each of those
buffers must start at zero.  Zeroing each one is a fill launch (≈5 µs apiece, ~250 per
Inception-v3 step).  The trainer instead opens a ``StepArena`` per step: one fill zeroes the
arena, and the ops carve their accumulators out of it in call order (a HIP-graph replay reuses the
captured addresses, and the one fill is a node of the graph).  The kernels never zero their own
accumulators: callers hand them zeroed memory (``zeros_f32``), from the arena when one is open,
else from ``torch.zeros``.
"""
from __future__ import annotations

import threading
from typing import Dict, Optional

import torch

_ALIGN = 64  # floats (256 B): every slice 16-B aligned for the kernels' vector loads
# process-wide, not thread-local: autograd runs the backward of CUDA ops on its own device thread,
# and those kernels' accumulators belong to the same step
_CURRENT: list = [None]
_lock = threading.Lock()


def _norm(device) -> torch.device:
    """'cuda' and 'cuda:<current>' are the same device: compare with the index filled in."""
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


class StepArena:
    def __init__(self, device, capacity: int = 0):
        self.device = _norm(device)
        self.buf: Optional[torch.Tensor] = None
        self.capacity = 0
        self.offset = 0
        self.used_last = 0
        self.need = 0
        self.active = False
        self.misses = 0
        if capacity:
            self._alloc(capacity)

    def _alloc(self, n: int) -> None:
        n = (n + _ALIGN - 1) // _ALIGN * _ALIGN
        self.buf = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.capacity = n

    def begin_step(self) -> None:
        """Zero what the previous step used (one fill) and start carving from the top."""
        capturing = self.device.type == "cuda" and torch.cuda.is_current_stream_capturing()
        if self.need > self.capacity and not capturing:
            self._alloc(int(self.need * 1.1))  # grew last step: fresh buffer is already zero
        elif self.buf is not None:
            # zero the whole extent used so far (inside a graph capture: everything, as a node)
            n = self.capacity if capturing else min(self.capacity, max(self.used_last, self.offset))
            if n:
                self.buf[:n].zero_()
        self.offset = 0
        self.need = 0
        self.active = True
        _CURRENT[0] = self

    def end_step(self) -> None:
        self.used_last = min(self.offset, self.capacity)
        self.active = False
        if _CURRENT[0] is self:
            _CURRENT[0] = None

    def take(self, n: int) -> Optional[torch.Tensor]:
        n_al = (n + _ALIGN - 1) // _ALIGN * _ALIGN
        with _lock:  # the forward (caller thread) and backward (autograd thread) both carve
            start, end = self.offset, self.offset + n_al
            self.offset = end        # keep counting past a miss: `need` sizes the next step's arena
            self.need = max(self.need, end)
        if self.buf is None or end > self.capacity:
            self.misses += 1
            return None
        return self.buf[start:start + n]

    def __enter__(self):
        self.begin_step()
        return self

    def __exit__(self, *exc):
        self.end_step()
        return False


def current() -> Optional[StepArena]:
    a = _CURRENT[0]
    return a if a is not None and a.active else None


def zeros_f32(n: int, device) -> torch.Tensor:
    """A zeroed fp32 accumulator of n floats: an arena slice when a step arena is open, else torch.zeros."""
    a = current()
    if a is not None and a.device == _norm(device):
        t = a.take(n)
        if t is not None:
            return t
    return torch.zeros(n, dtype=torch.float32, device=device)


_ARENAS: Dict[torch.device, StepArena] = {}


def for_device(device) -> StepArena:
    d = _norm(device)
    if d not in _ARENAS:
        _ARENAS[d] = StepArena(d)
    return _ARENAS[d]
