"""Flat parameter / gradient buffers.

Every trainable tensor of a model becomes a view into one contiguous buffer
(and its ``.grad`` a view into a second one).  This is what lets the hot path
run ONE fused optimizer launch over a whole shard, ONE reduce-scatter /
all-gather / all-reduce per bucket, and a single memset to zero gradients —
instead of per-tensor launches.  The layout is padded so every shard of a
``world``-way split is a multiple of ``align`` elements (16-byte vector loads
in the HIP kernels need multiples of 8 bf16).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch


@dataclass
class Slot:
    name: str
    offset: int
    numel: int
    shape: torch.Size
    channels_last: bool = False  # 4-D conv weight kept in [Co][R][S][Ci] memory order

    def view(self, buf: torch.Tensor) -> torch.Tensor:
        flat = buf[self.offset:self.offset + self.numel]
        if self.channels_last:
            co, ci, r, s = self.shape
            return flat.view(co, r, s, ci).permute(0, 3, 1, 2)
        return flat.view(self.shape)


class FlatParams:
    def __init__(self, module: torch.nn.Module, dtype=torch.bfloat16, device=None, world: int = 1,
                 align: int = 64, grad_dtype=None):
        params = [(n, p) for n, p in module.named_parameters() if p.requires_grad]
        if not params:
            raise ValueError("module has no trainable parameters")
        device = torch.device(device) if device is not None else params[0][1].device
        self.slots = []
        off = 0
        for name, p in params:
            # conv weights of a channels_last model stay channels_last: the implicit-GEMM convs read
            # them as [Co][R][S][Ci] and write dW in that order, with no per-step transposes
            cl = p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last) and not p.is_contiguous()
            self.slots.append(Slot(name, off, p.numel(), p.shape, cl))
            off += (p.numel() + align - 1) // align * align  # keep every view 16B aligned
        self.numel_unpadded = off
        chunk = world * align
        self.numel = (off + chunk - 1) // chunk * chunk
        self.world = world
        self.dtype = dtype
        self.device = device
        self.data = torch.zeros(self.numel, dtype=dtype, device=device)
        self.grad = torch.zeros(self.numel, dtype=grad_dtype or dtype, device=device)
        self.params = []
        with torch.no_grad():
            for slot, (_, p) in zip(self.slots, params):
                view = slot.view(self.data)
                view.copy_(p.detach().to(device=device, dtype=dtype))
                p.data = view
                p.grad = slot.view(self.grad)
                self.params.append(p)

    @property
    def shard_numel(self) -> int:
        return self.numel // self.world

    def shard(self, buf: torch.Tensor, rank: int) -> torch.Tensor:
        n = self.shard_numel
        return buf[rank * n:(rank + 1) * n]

    def zero_grad(self):
        self.grad.zero_()

    def rebind_grads(self):
        """Re-point ``p.grad`` at the flat buffer (after user code replaced them)."""
        for slot, p in zip(self.slots, self.params):
            p.grad = slot.view(self.grad)

    def master_copy(self, rank: int = 0) -> torch.Tensor:
        return self.shard(self.data, rank).float().clone()
