"""Dropout whose mask survives step replay (HIP kernels in csrc/dropout.hip).

``torch.nn.Dropout`` draws its mask from the CUDA generator's philox state.  Under
``CUDAGraph.replay()`` the generator's replay prologue refreshes the captured seed/offset, but the
native step plan (ops/plan.py) re-issues the captured kernels itself, so every replay would reuse
the capture-time mask.  Here the mask is a pure function of (seed, step counter, element) with the
counter held in device memory and bumped by a one-thread kernel right after the forward on the same
stream -- both are nodes of a captured step, so eager steps, graph replays and plan replays all draw
a fresh mask per step.  ``seed`` and ``counter`` are buffers: they follow ``.to(device)`` and the
model's ``state_dict`` (a resumed job continues the same mask sequence).

Reference parity: Inception-v3's classifier dropout (keep 0.8 / p 0.5 in the TF-slim model the
reference's TF-PS job family trains; SURVEY.md §2.7 H17 workload).
"""
from __future__ import annotations

import torch
from torch import nn

from . import _lib


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, rng):
        L = _lib.lib()
        xc = x.contiguous()
        n = xc.numel()
        is_bf16 = int(xc.dtype == torch.bfloat16)
        if not is_bf16 and xc.dtype != torch.float32:
            raise TypeError(f"dropout kernel takes bf16/fp32, got {xc.dtype}")
        if rng.device != x.device or rng.dtype != torch.int64 or rng.numel() != 2:
            raise ValueError("dropout rng state must be an int64 [seed, counter] tensor on the input's device")
        y = torch.empty_like(xc)
        mask = torch.empty((n + 7) // 8, dtype=torch.uint8, device=x.device)
        s = _lib.stream_ptr(x.device)
        _lib.check(L.tony_dropout_fwd(xc.data_ptr(), y.data_ptr(), mask.data_ptr(), n, is_bf16, float(p),
                                      rng.data_ptr(), s), "tony_dropout_fwd")
        _lib.check(L.tony_counter_bump(rng.data_ptr(), s), "tony_counter_bump")
        ctx.save_for_backward(mask)
        ctx.p = p
        return y

    @staticmethod
    def backward(ctx, gy):
        L = _lib.lib()
        (mask,) = ctx.saved_tensors
        g = gy.contiguous()
        dx = torch.empty_like(g)
        _lib.check(L.tony_dropout_bwd(g.data_ptr(), dx.data_ptr(), mask.data_ptr(), g.numel(),
                                      int(g.dtype == torch.bfloat16), float(ctx.p), _lib.stream_ptr(g.device)),
                   "tony_dropout_bwd")
        return dx, None, None


def dropout(x: torch.Tensor, p: float, rng: torch.Tensor) -> torch.Tensor:
    """Training-mode dropout of a CUDA tensor with the counter-based mask; advances ``rng[1]``."""
    return _DropoutFn.apply(x, p, rng)


class Dropout(nn.Module):
    """Drop-in for ``nn.Dropout`` (training: zero with probability p, scale the rest by 1/(1-p)).

    ``rng`` = [seed, step counter] (int64, non-persistent: the model's ``state_dict`` keeps the stock
    keys; ``named_buffers`` -- what the jobs' checkpoints store -- includes it, so a resumed job
    continues the same mask sequence).  The seed is drawn from torch's CPU generator, so
    ``torch.manual_seed`` makes the sequence reproducible."""

    def __init__(self, p: float = 0.5):
        super().__init__()
        if not 0.0 <= p < 1.0:
            raise ValueError(f"dropout probability must be in [0, 1), got {p}")
        self.p = float(p)
        seed = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64)
        self.register_buffer("rng", torch.cat([seed, torch.zeros(1, dtype=torch.int64)]), persistent=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not self.training or self.p == 0.0:
            return x
        if not x.is_cuda:  # CPU (control-plane tests): torch's dropout, same expectation
            return nn.functional.dropout(x, self.p, True)
        return _DropoutFn.apply(x, self.p, self.rng)

    def extra_repr(self) -> str:
        return f"p={self.p}"
