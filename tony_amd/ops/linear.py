"""Fully-connected layers on the MFMA GEMM kernels (csrc/gemm.hip), SURVEY.md §2.7 H8.

``Linear`` is an ``nn.Linear`` (same parameters, same state dict) whose forward runs, for CUDA
bf16 inputs, on tony_amd's kernels instead of hipBLASLt:

forward   Y = X W^T + b        tony_gemm_bf16 with the bias as the epilogue's per-column shift
                               (the folded-affine epilogue, scale = 1): one launch, no bias pass
backward  dX = dY W            tony_gemm_bf16 on the transposed weight
          dW = dY^T X          split-K TN GEMM (tony_gemm_tn_bf16), summed straight into the flat
                               gradient slot when one exists (parallel/ FlatParams)
          db = sum_rows(dY)

The classifier heads of Inception-v3 (2048 -> 1000, aux 768 -> 1000) and ResNet-50 (2048 -> 1000)
use it; the reference jobs' heads are the Keras/TF ``Dense`` layers of
/root/reference/tony-examples/mnist-tensorflow/mnist_distributed.py:110-124.
"""
from __future__ import annotations

import os

import torch
from torch import nn

from . import _lib, tape, tune
from .gemm import wgrad_tn

_BF16 = torch.bfloat16
# TONY_LINEAR_TUNE=0: the GEMM's built-in tile heuristic (A/B)
TUNE = os.environ.get("TONY_LINEAR_TUNE", "1") != "0"


def supported(x: torch.Tensor, weight: torch.Tensor) -> bool:
    """Whether the tony GEMMs take this layer: CUDA bf16, 2-D input, both feature dims % 8 == 0."""
    return (x.is_cuda and x.dtype == _BF16 and weight.dtype == _BF16 and x.dim() == 2
            and weight.shape[1] % 8 == 0 and weight.shape[0] % 8 == 0 and x.shape[1] == weight.shape[1])


def _affine(bias: torch.Tensor | None, n: int, device) -> torch.Tensor:
    """[scale | shift] fp32 for the GEMM epilogue: scale 1, shift = bias (0 without one)."""
    aff = torch.zeros(2 * n, dtype=torch.float32, device=device)
    aff[:n] = 1.0
    if bias is not None:
        aff[n:] = bias.float()
    return aff


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        L = _lib.lib()
        if x.stride(1) != 1 or x.data_ptr() % 16 or x.stride(0) % 8:
            x = x.contiguous()
        w = weight if weight.is_contiguous() else weight.contiguous()
        m, k = x.shape
        n = w.shape[0]
        y = torch.empty((m, n), dtype=x.dtype, device=x.device)
        aff = _affine(bias, n, x.device)
        # per-shape tile variant (ops/tune.py): the classifier's M = batch rows leave the default 128 x 192
        # tiles at 6 workgroups for the whole K = 2048 reduction
        vf = tune.gemm_flags(x, w, y, m, n, k, x.stride(0), False) if TUNE else 0
        rc = L.tony_gemm_bf16(x.data_ptr(), w.data_ptr(), y.data_ptr(), m, n, k, x.stride(0), k, n, 2 | vf,
                              aff.data_ptr(), 0, _lib.stream_ptr(x.device))
        _lib.check(rc, "tony_gemm_bf16 (linear)")
        ctx.save_for_backward(x, w)
        ctx.has_bias = bias is not None
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        weight, bias = ctx.params
        L, dev = _lib.lib(), x.device
        st = _lib.stream_ptr(dev)
        if dy.stride(1) != 1 or dy.data_ptr() % 16 or dy.stride(0) % 8:
            dy = dy.contiguous()
        m, k = x.shape
        n = w.shape[0]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            wt = w.t().contiguous()  # [in][out]: the NT GEMM's B operand
            dx = torch.empty((m, k), dtype=x.dtype, device=dev)
            vf = tune.gemm_flags(dy, wt, dx, m, k, n, dy.stride(0), False) if TUNE else 0
            rc = L.tony_gemm_bf16(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), m, k, n, dy.stride(0), n, k, vf, 0, 0,
                                  st)
            _lib.check(rc, "tony_gemm_bf16 (linear dgrad)")
        if ctx.needs_input_grad[1]:
            gw = _lib.grad_slot(weight)
            if gw is not None and gw.is_contiguous():
                wgrad_tn(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), m, n, k, dev, dst=gw)
            else:
                dw = wgrad_tn(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), m, n, k, dev).to(weight.dtype)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.float().sum(0)
            gb = _lib.grad_slot(bias)
            if gb is not None:
                gb.add_(db.to(gb.dtype))
                db = None
            else:
                db = db.to(bias.dtype)
        _lib.report_inplace((weight, bias), (dw, db))
        return dx, dw, db


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """``F.linear`` on the MFMA GEMMs when ``supported``, else PyTorch's."""
    if supported(x, weight):
        return tape.apply(_LinearFn, x, weight, bias)
    return nn.functional.linear(x, weight, bias)


class Linear(nn.Linear):
    """``nn.Linear`` whose CUDA bf16 forward/backward run on tony_amd's MFMA GEMMs (see module doc)."""

    def forward(self, x):
        return linear(x, self.weight, self.bias)
