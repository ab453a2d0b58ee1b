"""Fused softmax cross-entropy (HIP kernels in csrc/loss.hip)."""
from __future__ import annotations

import torch

from . import _lib


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, smoothing):
        L = _lib.lib()
        if logits.stride(1) != 1:
            logits = logits.contiguous()
        labels = labels.contiguous().to(torch.int64)
        n, k = logits.shape
        is_bf16 = int(logits.dtype == torch.bfloat16)
        if not is_bf16 and logits.dtype != torch.float32:
            raise TypeError(f"cross_entropy kernel takes bf16/fp32 logits, got {logits.dtype}")
        loss = torch.empty(n, dtype=torch.float32, device=logits.device)
        lse = torch.empty(n, dtype=torch.float32, device=logits.device)
        rc = L.tony_xent_fwd(logits.data_ptr(), is_bf16, n, k, logits.stride(0), labels.data_ptr(), float(smoothing),
                             loss.data_ptr(), lse.data_ptr(), _lib.stream_ptr(logits.device))
        _lib.check(rc, "tony_xent_fwd")
        ctx.save_for_backward(logits, labels, lse)
        ctx.smoothing = smoothing
        return loss

    @staticmethod
    def backward(ctx, gout):
        L = _lib.lib()
        logits, labels, lse = ctx.saved_tensors
        n, k = logits.shape
        gout = gout.float().contiguous()
        if gout.numel() != n:
            gout = gout.expand(n).contiguous()
        d = torch.empty((n, k), dtype=logits.dtype, device=logits.device)
        rc = L.tony_xent_bwd(logits.data_ptr(), int(logits.dtype == torch.bfloat16), n, k, logits.stride(0),
                             labels.data_ptr(), float(ctx.smoothing), lse.data_ptr(), gout.data_ptr(), d.data_ptr(), k,
                             _lib.stream_ptr(logits.device))
        _lib.check(rc, "tony_xent_bwd")
        return d, None, None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, label_smoothing: float = 0.0,
                  reduction: str = "mean") -> torch.Tensor:
    """Softmax cross-entropy; per-row losses are fp32 whatever the logits dtype."""
    if logits.is_cuda:
        per_row = _XentFn.apply(logits, labels, label_smoothing)
    else:
        per_row = torch.nn.functional.cross_entropy(logits.float(), labels, reduction="none",
                                                    label_smoothing=label_smoothing)
    if reduction == "mean":
        return per_row.mean()
    if reduction == "sum":
        return per_row.sum()
    return per_row
