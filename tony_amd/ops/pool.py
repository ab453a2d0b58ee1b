"""NHWC pooling kernels (csrc/pool.hip): avg 3x3/s1/p1, avg KxK/sS and max KxK/sS with zero padding."""
from __future__ import annotations

import torch

from . import _lib, concat, streams, tape
from .bn import _as_rows, _rows_view


def _nhwc_empty(n, c, h, w, like):
    return torch.empty((n, c, h, w), dtype=like.dtype, device=like.device, memory_format=torch.channels_last)


def _fn(name: str, t: torch.Tensor):
    """The bf16 entry point or its fp32 form (``_f32``: the x3 fp32 step, ops/x3.py) for ``t``'s dtype."""
    return getattr(_lib.lib(), name + "_f32" if t.dtype == torch.float32 else name)


def _ok(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) and x.shape[1] % 8 == 0


def _dense_rows(t: torch.Tensor, shape) -> bool:
    """``t`` (bf16 or fp32) has ``shape`` as dense 16-B aligned channels_last rows: an accumulating store fits."""
    if tuple(t.shape) != tuple(shape) or t.data_ptr() % 16:
        return False
    rv = _rows_view(t)
    return rv is not None and rv[2] == t.shape[1]


def _box3(src, n, c, h, w, ld_src):
    out = _nhwc_empty(n, c, h, w, src)
    rc = _fn("tony_avgpool3_s1p1", src)(src.data_ptr(), out.data_ptr(), n, h, w, c, ld_src, c,
                                        _lib.stream_ptr(src.device))
    _lib.check(rc, "tony_avgpool3_s1p1")
    return out


_LAST_PLANES = [None]


class _AvgPool3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, planes_only=False):
        x, (_, c, ld) = _as_rows(x)
        n, _, h, w = x.shape
        ctx.join = getattr(x, "_tony_join", None)  # ops/residual.py GradJoin: x has other consumers
        if planes_only:
            # fp32 x, read only by one x3 conv: the pooled map goes straight to its operand planes
            # (ops/x3.py split_act layout), the fp32 map is never stored
            y3 = torch.empty((n * h * w, 3 * c), dtype=torch.bfloat16, device=x.device)
            rc = _lib.lib().tony_avgpool3_s1p1_x3(x.data_ptr(), y3.data_ptr(), n, h, w, c, ld,
                                                  _lib.stream_ptr(x.device))
            _lib.check(rc, "tony_avgpool3_s1p1_x3")
            _LAST_PLANES[0] = y3.view(n, h, w, 3 * c).permute(0, 3, 1, 2)
            return torch.empty_strided((n, c, h, w), (0, 0, 0, 0), dtype=x.dtype, device=x.device)  # shape only
        return _box3(x, n, c, h, w, ld)

    @staticmethod
    def backward(ctx, dy):
        dy, (_, c, ld) = _as_rows(dy)
        n, _, h, w = dy.shape
        join = ctx.join if ctx.needs_input_grad[0] else None
        pend = join.take() if join is not None else None
        if pend is not None and pend.dtype == dy.dtype and _dense_rows(pend, (n, c, h, w)):
            # another consumer of x already wrote its gradient: box(dy)/9 is added into it in-kernel
            rc = _lib.lib().tony_avgpool3_s1p1_acc(dy.data_ptr(), pend.data_ptr(), n, h, w, c, ld, c,
                                                   int(dy.dtype == torch.float32), _lib.stream_ptr(dy.device))
            _lib.check(rc, "tony_avgpool3_s1p1_acc")
            dx = pend
        else:
            dx = _box3(dy, n, c, h, w, ld)  # symmetric stencil: dx = box(dy)/9
            if pend is not None:
                dx = pend.add_(dx)
        if join is not None:
            dx = join.settle(dx)
        streams.keep(dx)  # may be consumed on another (branch) stream
        return dx, None


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, slot=None, p=0):
        x, (_, c, ld) = _as_rows(x)
        n, _, h, w = x.shape
        oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        y = concat.take(slot, n, c, oh, ow, x)  # straight into the block's concat buffer
        if y is None:
            y = _nhwc_empty(n, c, oh, ow, x)
        arg = torch.empty((n, oh, ow, c), dtype=torch.uint8, device=x.device)
        rc = _fn("tony_maxpool_fwd", x)(x.data_ptr(), y.data_ptr(), arg.data_ptr(), n, h, w, c, k, s, p, ld,
                                         _rows_view(y)[2], _lib.stream_ptr(x.device))
        _lib.check(rc, "tony_maxpool_fwd")
        ctx.save_for_backward(arg)
        ctx.shape = (n, c, h, w, k, s, p)
        ctx.join = getattr(x, "_tony_join", None)  # ops/residual.py GradJoin: x has other consumers
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        n, c, h, w, k, s, p = ctx.shape
        dy, (_, _, lddy) = _as_rows(dy)
        join = ctx.join if ctx.needs_input_grad[0] else None
        pend = join.take() if join is not None else None
        if pend is not None and pend.dtype == dy.dtype and _dense_rows(pend, (n, c, h, w)):
            # another consumer of x already wrote its gradient: the pool's is added into it in-kernel
            rc = _fn("tony_maxpool_bwd_acc", dy)(dy.data_ptr(), arg.data_ptr(), pend.data_ptr(), n, h, w, c, k, s, p,
                                                  lddy, c, _lib.stream_ptr(dy.device))
            _lib.check(rc, "tony_maxpool_bwd_acc")
            dx = pend
        else:
            dx = _nhwc_empty(n, c, h, w, dy)
            rc = _fn("tony_maxpool_bwd", dy)(dy.data_ptr(), arg.data_ptr(), dx.data_ptr(), n, h, w, c, k, s, p, lddy,
                                             c, _lib.stream_ptr(dy.device))
            _lib.check(rc, "tony_maxpool_bwd")
            if pend is not None:
                dx = pend.add_(dx)
        if join is not None:
            dx = join.settle(dx)
        streams.keep(dx)  # may be consumed on another (branch) stream
        return dx, None, None, None, None


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s):
        x, (_, c, ld) = _as_rows(x)
        n, _, h, w = x.shape
        oh, ow = (h - k) // s + 1, (w - k) // s + 1
        y = _nhwc_empty(n, c, oh, ow, x)
        rc = _fn("tony_avgpool_fwd", x)(x.data_ptr(), y.data_ptr(), n, h, w, c, k, s, ld, c,
                                         _lib.stream_ptr(x.device))
        _lib.check(rc, "tony_avgpool_fwd")
        ctx.shape = (n, c, h, w, k, s)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, c, h, w, k, s = ctx.shape
        dy, (_, _, lddy) = _as_rows(dy)
        dx = _nhwc_empty(n, c, h, w, dy)
        rc = _fn("tony_avgpool_bwd", dy)(dy.data_ptr(), dx.data_ptr(), n, h, w, c, k, s, lddy, c,
                                         _lib.stream_ptr(dy.device))
        _lib.check(rc, "tony_avgpool_bwd")
        return dx, None, None


def avg_pool(x: torch.Tensor, k: int, s: int) -> torch.Tensor:
    """avg_pool2d(x, k, s) (no padding) on channels_last bf16 / fp32; k = H = W is the global average pool."""
    if _ok(x):
        return tape.apply(_AvgPoolFn, x, k, s)
    return torch.nn.functional.avg_pool2d(x, k, s)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """adaptive_avg_pool2d(x, 1) flattened to [N, C]."""
    if x.shape[2] == x.shape[3]:
        return torch.flatten(avg_pool(x, x.shape[2], 1), 1)
    return torch.flatten(torch.nn.functional.adaptive_avg_pool2d(x, 1), 1)


def avg_pool3x3_s1(x: torch.Tensor, planes_only: bool = False) -> torch.Tensor:
    """avg_pool2d(x, 3, 1, 1, count_include_pad=True) on channels_last bf16 / fp32.  ``planes_only`` (fp32
    x): the output feeds one x3 conv only -- a shape-only tensor comes back whose operand planes
    ops/x3.split_act finds cached on it (never read as fp32)."""
    if _ok(x):
        planes_only = planes_only and x.dtype == torch.float32 and not tape.recording()
        _LAST_PLANES[0] = None
        y = tape.apply(_AvgPool3Fn, x, planes_only)
        planes = _LAST_PLANES[0]
        if planes is not None:
            _LAST_PLANES[0] = None
            y._tony_x3 = (y._version, planes, x.shape[1])
        return y
    return torch.nn.functional.avg_pool2d(x, 3, 1, 1, count_include_pad=True)


def max_pool(x: torch.Tensor, k: int = 3, s: int = 2, slot=None, padding: int = 0) -> torch.Tensor:
    """max_pool2d(x, k, s, padding) on channels_last bf16 (into a concat.Slot when given); padded taps
    never win (torch semantics), e.g. ResNet's 3x3/2 p1 stem pool."""
    if _ok(x) and 2 * padding <= k:
        return tape.apply(_MaxPoolFn, x, k, s, slot, padding)
    return torch.nn.functional.max_pool2d(x, k, s, padding)
