"""Zero-copy channel concatenation for the Inception blocks.

A block allocates its NHWC output [N, sum C_i, H, W] once and hands each branch's LAST layer a
``Slot`` (the buffer + its channel offset); the fused BN-apply / max-pool kernels write that branch
straight into its channel slice (row stride = the concat width), so the ``torch.cat`` copy of every
block output disappears.  ``assemble(buf, parts)`` then returns the buffer as the block output with
an autograd node whose backward hands each branch the matching (strided) slice of the gradient --
exactly what ``torch.cat``'s backward does, and what the BN-backward kernels read in place.

A branch whose last op could not write into its slot (a CPU tensor, an unsupported shape falling
back to stock PyTorch) simply returns its own tensor; ``assemble`` copies it in, so the fast path
is an optimisation, never a correctness condition.  The slot views are written through raw device
pointers (no autograd version bumps), which is what makes handing out views of one buffer to
several custom Functions legal.
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

import torch

from . import tape

# TONY_X3_CONCAT_PLANES (default on; =0 off): an fp32 block output also carries its x3 operand planes (ops/x3.py), filled
# slice by slice by the producers that write its slots (the BN apply kernels write both forms) and, for
# the slices no producer covered (max-pool branches, fallbacks), by one slice split in ``assemble`` -- so
# the next block's convs find the planes already made instead of splitting the whole fp32 concat
# (fp32 step 31.79 vs 31.88 ms, profiles/r5_ab_x3_concat_planes.log).
X3_PLANES = os.environ.get("TONY_X3_CONCAT_PLANES", "1") != "0"


class Slot:
    """Channel slice [c0, c0 + c) of a channels_last concat buffer, as a destination for a kernel."""

    __slots__ = ("buf", "c0")

    def __init__(self, buf: torch.Tensor, c0: int):
        self.buf = buf
        self.c0 = c0

    def view(self, c: int) -> torch.Tensor:
        return self.buf[:, self.c0:self.c0 + c]

    def matches(self, n, c, h, w, dtype, device) -> bool:
        b = self.buf
        return (b.shape[0] == n and b.shape[2] == h and b.shape[3] == w and self.c0 + c <= b.shape[1]
                and b.dtype == dtype and b.device == device)


def take(slot: Optional[Slot], n, c, h, w, like: torch.Tensor) -> Optional[torch.Tensor]:
    """The slice a kernel should write its [n, c, h, w] output into, or None (allocate normally)."""
    if slot is None or not slot.matches(n, c, h, w, like.dtype, like.device):
        return None
    return slot.view(c)


def concat_buffer(n, c, h, w, like: torch.Tensor) -> torch.Tensor:
    buf = torch.empty((n, c, h, w), dtype=like.dtype, device=like.device, memory_format=torch.channels_last)
    if X3_PLANES and like.dtype == torch.float32 and like.is_cuda and c % 8 == 0:
        buf._tony_p3 = torch.empty((n, h, w, 3 * c), dtype=torch.bfloat16, device=like.device)
        buf._tony_p3_cov = set()  # channel offsets of the slices whose planes a producer wrote
    return buf


def planes_of(slot: Optional[Slot], c: int):
    """(pointer, row stride, plane stride) of slot's slice of its buffer's x3 planes, or None."""
    if slot is None or c % 8 or slot.c0 % 8:
        return None
    p3 = getattr(slot.buf, "_tony_p3", None)
    if p3 is None:
        return None
    ctot = slot.buf.shape[1]
    return p3.data_ptr() + 2 * slot.c0, 3 * ctot, ctot


def planes_written(slot: Slot) -> None:
    slot.buf._tony_p3_cov.add(slot.c0)


def _finish_planes(buf: torch.Tensor, widths, out: torch.Tensor) -> None:
    """Split the slices no producer covered into buf's planes and hang them on the block output, where
    ops/x3.split_act finds them."""
    from . import _lib
    from .x3 import ACT

    p3, cov = buf._tony_p3, buf._tony_p3_cov
    n, ctot, h, w = buf.shape
    L, st = _lib.lib(), _lib.stream_ptr(buf.device)
    c0 = 0
    for c in widths:
        if c0 not in cov:
            if c % 8:
                return  # cannot split this slice in place: the consumers split the whole concat
            rc = L.tony_x3_split_slice(buf.data_ptr() + 4 * c0, ctot, n * h * w, c, p3.data_ptr() + 2 * c0, 3 * ctot,
                                       ctot, ACT, st)
            _lib.check(rc, "tony_x3_split_slice")
        c0 += c
    out._tony_x3 = (out._version, p3.permute(0, 3, 1, 2), ctot)


class _AssembleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, buf_holder, *parts):
        buf = buf_holder.buf
        c0 = 0
        for p in parts:
            dst = buf[:, c0:c0 + p.shape[1]]
            if p.data_ptr() != dst.data_ptr() or p.stride() != dst.stride():
                dst.data.copy_(p)  # this branch did not write in place (fallback path)
            c0 += p.shape[1]
        if c0 != buf.shape[1]:
            raise ValueError(f"concat parts cover {c0} of {buf.shape[1]} channels")
        ctx.widths = [p.shape[1] for p in parts]
        return buf

    @staticmethod
    def backward(ctx, dbuf):
        from . import streams

        streams.keep(dbuf)  # its slices feed branch-stream backward nodes
        grads, c0 = [], 0
        for c in ctx.widths:
            grads.append(dbuf[:, c0:c0 + c])
            c0 += c
        return (None, *grads)


def assemble(buf: torch.Tensor, parts: Sequence[torch.Tensor]) -> torch.Tensor:
    """The block output ``buf`` (= cat(parts, 1)), with the parts already written into it in place."""
    out = tape.apply(_AssembleFn, Slot(buf, 0), *parts)
    if getattr(buf, "_tony_p3", None) is not None and out.is_cuda:
        _finish_planes(buf, [p.shape[1] for p in parts], out)
    return out
