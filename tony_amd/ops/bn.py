"""Fused BatchNorm(+ReLU) on NHWC bf16 activations (HIP kernels in csrc/bn_act.hip).

``bn_act(x, weight, bias, running_mean, running_var, training, momentum, eps, relu)``
is a drop-in for ``relu(batch_norm(x, ...))`` on channels_last tensors.  The
HIP path is taken for CUDA bf16 tensors; CPU tensors use the PyTorch reference
(so the control-plane / local-mode tests run on a CPU-only container).  A CUDA
tensor of another dtype is an error, not a silent fallback.
"""
from __future__ import annotations

import os

import torch

from . import _lib, tape
from .arena import zeros_f32


def _rows_view_uncached(shape, stride):
    if len(shape) == 4:
        n, c, h, w = shape
        sn, sc, sh, sw = stride
        if sc != 1 and c > 1:
            return None
        # strides of size-1 dims are arbitrary: derive the row stride from the
        # innermost non-trivial spatial / batch dim
        if h * w == 1:
            ld = sn if n > 1 else c
        elif w == 1:
            ld = sh
            if n > 1 and sn != h * ld:
                return None
        else:
            ld = sw
            if (h > 1 and sh != w * ld) or (n > 1 and sn != h * w * ld):
                return None
        if ld < c:
            return None
        return n * h * w, c, ld
    if len(shape) == 2:
        m, c = shape
        if stride[1] != 1:
            return None
        return m, c, stride[0] if m > 1 else c
    return None


# The row view depends only on (shape, strides): memoised, since every fused op asks it for each
# operand on every call (~600 times per Inception step; the uncached walk is ~2 us of Python).
# TONY_HOST_MEMO=0 turns the host-side memos of ops/ off (A/B of the host issue time).
HOST_MEMO = os.environ.get("TONY_HOST_MEMO", "1") != "0"
_RV_CACHE: dict = {}


def _rows_view(t: torch.Tensor):
    """Return (M, C, ld) when ``t``'s memory is M rows of C channels with row
    stride ``ld`` (channels_last 4D, a channel slice of one, or 2D [M, C])."""
    if not HOST_MEMO:
        return _rows_view_uncached(t.shape, t.stride())
    key = (t.shape, t.stride())
    r = _RV_CACHE.get(key, _RV_CACHE)
    if r is _RV_CACHE:
        if len(_RV_CACHE) > 4096:
            _RV_CACHE.clear()
        r = _RV_CACHE[key] = _rows_view_uncached(*key)
    return r


def _as_rows(t: torch.Tensor):
    rv = _rows_view(t)
    if rv is None or rv[2] % 8 != 0 or t.data_ptr() % 16 != 0:
        t = t.contiguous(memory_format=torch.channels_last) if t.dim() == 4 else t.contiguous()
        rv = _rows_view(t)
    return t, rv


class MaskedGrad:
    """A residual tail's d(identity) = dY * (y > 0) left unmaterialised: the dY rows (bf16, dense
    channels_last) and the forward's ReLU byte mask (_res_mask).  The conv consumer that runs second
    reads both in its dgrad epilogue (csrc/gemm.hip flags bit5) -- the tail's backward then writes dZ
    only, one activation-sized store fewer per identity block -- and anything else materialises it."""

    __slots__ = ("dy", "mask")

    def __init__(self, dy: torch.Tensor, mask: torch.Tensor):
        self.dy, self.mask = dy, mask

    @property
    def device(self):
        return self.dy.device

    @property
    def is_cuda(self):
        return self.dy.is_cuda

    def materialize(self) -> torch.Tensor:
        n, c, h, w = self.dy.shape
        shifts = torch.arange(8, device=self.mask.device, dtype=torch.uint8)
        bits = ((self.mask.unsqueeze(-1) >> shifts) & 1).reshape(n * h * w, c)  # channel 8 * j + e
        rows = self.dy.permute(0, 2, 3, 1).reshape(n * h * w, c)
        return (rows * bits.to(rows.dtype)).view(n, h, w, c).permute(0, 3, 1, 2)


def _accum_ok(t: torch.Tensor, x_shape) -> bool:
    """``t`` can take a dgrad epilogue's accumulating store: bf16, x's shape, dense channels_last rows."""
    if t.dtype != torch.bfloat16 or tuple(t.shape) != tuple(x_shape) or t.data_ptr() % 16:
        return False
    rv = _rows_view(t)
    return rv is not None and rv[2] == t.shape[1]


def _empty_like_rows(x: torch.Tensor) -> torch.Tensor:
    if x.dim() == 4:
        return torch.empty(x.shape, dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    return torch.empty(x.shape, dtype=x.dtype, device=x.device)


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, training, momentum, eps, relu):
        L = _lib.lib()
        _lib.check_f32_stats(running_mean, running_var)
        x, (M, C, ldx) = _as_rows(x)
        y = _empty_like_rows(x)
        _, _, ldy = _rows_view(y)
        pb = int(weight is not None and weight.dtype == torch.bfloat16)
        stream = _lib.stream_ptr(x.device)
        if training:
            ws = zeros_f32(_lib.stat_floats(C), x.device)  # STAT_SHARDS x [sum | sumsq]
            mean = torch.empty(C, dtype=torch.float32, device=x.device)
            invstd = torch.empty(C, dtype=torch.float32, device=x.device)
            rc = L.tony_bn_fwd_train(x.data_ptr(), M, C, ldx, y.data_ptr(), ldy, _lib.ptr(weight), _lib.ptr(bias),
                                     pb, float(eps), int(relu), ws.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                                     _lib.ptr(running_mean), _lib.ptr(running_var), float(momentum), stream)
            _lib.check(rc, "tony_bn_fwd_train")
        else:
            mean = running_mean
            invstd = torch.rsqrt(running_var.float() + eps)
            rc = L.tony_bn_fwd_infer(x.data_ptr(), M, C, ldx, y.data_ptr(), ldy, _lib.ptr(weight), _lib.ptr(bias),
                                     pb, float(eps), int(relu), running_mean.data_ptr(), running_var.data_ptr(),
                                     stream)
            _lib.check(rc, "tony_bn_fwd_infer")
        ctx.save_for_backward(x, weight, bias, mean, invstd)
        ctx.params = (weight, bias)  # the Parameter objects (for in-place grad accumulation)
        ctx.relu = relu
        ctx.pb = pb
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        x, weight, bias, mean, invstd = ctx.saved_tensors
        M, C, ldx = _rows_view(x)
        dy, (_, _, lddy) = _as_rows(dy)
        dx = _empty_like_rows(x)
        _, _, lddx = _rows_view(dx)
        ws = zeros_f32(_lib.bn_bwd_ws_floats(C), x.device)
        gw, gb = _lib.grad_slot(ctx.params[0]), _lib.grad_slot(ctx.params[1])
        inplace = gw is not None and gb is not None
        if inplace:
            dw, db = gw, gb
        else:
            dw = torch.empty_like(weight) if weight is not None else None
            db = torch.empty_like(bias) if bias is not None else None
        _lib.bn_bwd(x, ldx, dy, lddy, dx, lddx, M, C, mean, invstd, weight, bias, ctx.pb, ctx.relu, ws, dw, db,
                    inplace, x.device)
        if inplace:
            dw = db = None  # already added into param.grad
        _lib.report_inplace(ctx.params, (dw, db))
        return dx, dw, db, None, None, None, None, None, None


def bn_act_reference(x, weight, bias, running_mean, running_var, training, momentum, eps, relu):
    y = torch.nn.functional.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    return torch.relu(y) if relu else y


def bn_act(x, weight, bias, running_mean, running_var, training=True, momentum=0.1, eps=1e-5, relu=True):
    if x.is_cuda:
        if x.dtype != torch.bfloat16:
            raise TypeError(f"bn_act HIP kernel takes bf16 activations, got {x.dtype}")
        return tape.apply(_BNActFn, x, weight, bias, running_mean, running_var, training, momentum, eps, relu)
    return bn_act_reference(x, weight, bias, running_mean, running_var, training, momentum, eps, relu)


class BatchNormAct2d(torch.nn.BatchNorm2d):
    """BatchNorm2d fused with an optional ReLU, NHWC bf16 on the GPU."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, relu=True, **kw):
        super().__init__(num_features, eps=eps, momentum=momentum, **kw)
        self.relu = relu

    def forward(self, x):
        training = self.training or not self.track_running_stats
        if self.training and self.track_running_stats and self.momentum is None:
            # only needed for cumulative averaging; skipping it saves one
            # launch per BN layer per step on the fixed-momentum hot path
            self.num_batches_tracked.add_(1)
        return bn_act(x, self.weight, self.bias, self.running_mean if self.track_running_stats else None,
                      self.running_var if self.track_running_stats else None, training, self.momentum, self.eps,
                      self.relu)
