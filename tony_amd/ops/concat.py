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

from typing import Optional, Sequence

import torch

from . import tape


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
    return torch.empty((n, c, h, w), dtype=like.dtype, device=like.device, memory_format=torch.channels_last)


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
    return tape.apply(_AssembleFn, Slot(buf, 0), *parts)
