"""BN + residual add + ReLU in one pass (the ResNet bottleneck tail), optionally behind a 1x1 MFMA GEMM.

``y = relu(bn(z) + identity)`` is three memory passes in the textbook graph
(BN apply, add, ReLU) plus their three backward passes.  Here:

forward   stats(z) [from the GEMM epilogue when z comes from the fused 1x1 conv]
          -> ONE apply pass reading z and identity, writing y
backward  ONE reduce pass (dy masked by y > 0, sums for dgamma/dbeta) and ONE
          apply pass writing both dz and d(identity) = dy * (y > 0)

``conv1x1_bn_add_relu`` fuses the bottleneck's conv3 as well: Z = x . W^T with
the BN statistics in the GEMM epilogue (csrc/gemm.hip), the backward-data GEMM
and split-K wgrad GEMM of ops/fused.py, and parameter gradients accumulated in
place into the flat gradient buffer when the trainer enabled it.
"""
from __future__ import annotations

import os

import torch

from . import _lib, streams, tape, tune, wt_cache
from .arena import zeros_f32
from .bn import MaskedGrad, _as_rows, _empty_like_rows, _rows_view
from .fused import _cl_empty
from .gemm import wgrad_tn

_BF16 = torch.bfloat16


class GradJoin:
    """The gradient meeting point of a tensor with two consumers: a ResNet block feeds its input x to
    conv1 AND to the residual add (identity blocks) or the downsample conv (projection blocks).
    Autograd would sum the two gradients with a separate add kernel (3 passes over a 51-205 MB
    activation per block).  Instead the consumer whose backward runs first parks its gradient here and
    returns None for x; the second one adds its dX into that tensor in the dgrad epilogue
    (csrc/mfma_common.h nt_epilogue accum) and returns the sum.  Set by models/resnet.py on x as
    ``_tony_join``, one per forward; both consumers of x are then join-aware:

    * the residual op (produces d(identity) with its own kernel): ``park(grad)`` -> what to return for x;
    * a conv (ops/conv.py _conv_bn_backward, ops/fused.py _HeadFn): ``take()`` before its dgrad -- a
      parked gradient to accumulate into, or None, and then ``settle(dx)`` -> what to return."""

    __slots__ = ("pending", "stream", "ran", "n")

    def __init__(self, n: int = 2):
        self.pending = None
        self.stream = None
        self.ran = 0  # consumers whose backward has started
        self.n = n    # consumers of the tensor (Inception's reduction blocks: 3)

    def _hold(self, grad: torch.Tensor) -> None:
        self.pending = grad
        self.stream = torch.cuda.current_stream(grad.device) if grad.is_cuda else None

    def _ordered(self, g):
        """``g`` (parked on self.stream) usable on the current stream."""
        if self.stream is not None:
            cur = streams.current(g.device.index)
            # (by handle: current_stream() returns a new Stream object per call)
            if cur.cuda_stream != self.stream.cuda_stream:
                streams.fork(self.stream, cur)
                if isinstance(g, MaskedGrad):
                    streams.keep(g.dy, g.mask)
                else:
                    streams.keep(g)
        return g

    def wants_masked(self) -> bool:
        """The caller (a residual tail) runs first and another consumer follows: it may park a MaskedGrad."""
        return MASKED_JOIN and self.pending is None and self.ran + 1 < self.n

    def park_masked(self, dy: torch.Tensor, mask: torch.Tensor):
        self.ran += 1
        self._hold(MaskedGrad(dy, mask))
        return None

    def park(self, grad):
        self.ran += 1
        if self.pending is not None:  # a conv consumer ran first and parked its dX
            p = self._ordered(self.pending)
            grad = (p.materialize() if isinstance(p, MaskedGrad) else p).add_(grad)
            self.pending = None
        if grad is None or self.ran >= self.n:
            return grad
        self._hold(grad)
        return None

    def take(self, masked_ok: bool = False):
        """The parked gradient (None: this consumer is the first); a MaskedGrad only for ``masked_ok``
        callers, materialised for the others."""
        self.ran += 1
        g, self.pending = self.pending, None
        if g is None:
            return None
        g = self._ordered(g)
        return g.materialize() if isinstance(g, MaskedGrad) and not masked_ok else g

    def settle(self, dx):
        if dx is None or self.ran >= self.n:
            return dx
        self._hold(dx)
        return None


# TONY_MASKED_JOIN=0: the residual tail writes d(identity) for the GradJoin instead of parking dY and its
# ReLU mask for the conv consumer's dgrad epilogue to read (MaskedGrad)
MASKED_JOIN = os.environ.get("TONY_MASKED_JOIN", "1") != "0"

# TONY_RES_MASK=0: the residual BN backward re-reads y for its ReLU mask instead of the forward's byte
# mask (1 bit per element: y is a 51-205 MB activation read twice per block backward)
RES_MASK = os.environ.get("TONY_RES_MASK", "1") != "0"


def _res_mask(M: int, C: int, dev):
    """The byte mask of a residual BN forward (bit j of byte [m, c // 8]: y[m, c] > 0), or None."""
    if not RES_MASK or C % 8:
        return None
    return torch.empty((M, C // 8), dtype=torch.uint8, device=dev)


def _bn_stats_and_apply(L, z, ldz, M, C, res, ldr, y, ldy, gamma, beta, pb, eps, training, momentum, running_mean,
                        running_var, stats, stream, mask=None):
    _lib.check_f32_stats(running_mean, running_var)
    dev = z.device
    if training:
        mean = torch.empty(C, dtype=torch.float32, device=dev)
        invstd = torch.empty(C, dtype=torch.float32, device=dev)
    else:
        mean = running_mean
        invstd = torch.rsqrt(running_var.float() + eps)
    args = (z.data_ptr(), M, C, ldz, res.data_ptr(), ldr, y.data_ptr(), ldy,
            _lib.ptr(stats) if training else 0, _lib.ptr(stats) + 4 * C if training else 0,
            2 * C if training else 0, _lib.ptr(gamma), _lib.ptr(beta), pb, float(eps), 1, 0 if training else 1,
            _lib.ptr(mean) if training else 0, _lib.ptr(invstd) if training else 0,
            _lib.ptr(running_mean), _lib.ptr(running_var), float(momentum))
    if mask is not None:
        rc = L.tony_bn_apply_res_m(*args, mask.data_ptr(), C // 8, stream)
    else:
        rc = L.tony_bn_apply_res(*args, stream)
    _lib.check(rc, "tony_bn_apply_res")
    return mean, invstd


def _bwd_res(L, z, ldz, dy, y, M, C, mean, invstd, gamma, beta, pb, params, stream, want_dres=True):
    """``y``: the forward output, or its byte mask (uint8 [M, C/8], _res_mask) for the ReLU test."""
    dev = z.device
    dy, (_, _, lddy) = _as_rows(dy)
    if y.dtype == torch.uint8:
        return _bwd_res_mask(L, z, ldz, dy, lddy, y, M, C, mean, invstd, gamma, beta, pb, params, stream, want_dres)
    _, _, ldy = _rows_view(y)
    dz = _empty_like_rows(y)
    _, _, lddz = _rows_view(dz)
    dres = _empty_like_rows(y) if want_dres else None
    ws = zeros_f32(_lib.stat_floats(C), dev)
    gg, gb = _lib.grad_slot(params[0]), _lib.grad_slot(params[1])
    inplace = gg is not None and gb is not None
    dgamma = gg if inplace else torch.empty_like(gamma)
    dbeta = gb if inplace else torch.empty_like(beta)
    rc = L.tony_bn_bwd_res(z.data_ptr(), ldz, dy.data_ptr(), lddy, y.data_ptr(), ldy, dz.data_ptr(), lddz,
                           _lib.ptr(dres), lddz, M, C, mean.data_ptr(), invstd.data_ptr(), _lib.ptr(gamma),
                           _lib.ptr(beta), pb, ws.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), int(inplace),
                           stream)
    _lib.check(rc, "tony_bn_bwd_res")
    return dz, dres, (None, None) if inplace else (dgamma, dbeta)


def _bwd_res_mask(L, z, ldz, dy, lddy, mask, M, C, mean, invstd, gamma, beta, pb, params, stream, want_dres):
    dev = z.device
    n, _, h, w = z.shape
    dz = _cl_empty(n, C, h, w, dev)
    dres = _cl_empty(n, C, h, w, dev) if want_dres else None
    ws = zeros_f32(_lib.stat_floats(C), dev)
    gg, gb = _lib.grad_slot(params[0]), _lib.grad_slot(params[1])
    inplace = gg is not None and gb is not None
    dgamma = gg if inplace else torch.empty_like(gamma)
    dbeta = gb if inplace else torch.empty_like(beta)
    rc = L.tony_bn_bwd_res_m(z.data_ptr(), ldz, dy.data_ptr(), lddy, mask.data_ptr(), C // 8, dz.data_ptr(), C,
                             _lib.ptr(dres), C, M, C, mean.data_ptr(), invstd.data_ptr(), _lib.ptr(gamma),
                             _lib.ptr(beta), pb, ws.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), int(inplace),
                             stream)
    _lib.check(rc, "tony_bn_bwd_res_m")
    return dz, dres, (None, None) if inplace else (dgamma, dbeta)


class _BNAddReLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, res, gamma, beta, running_mean, running_var, training, momentum, eps):
        L = _lib.lib()
        stream = _lib.stream_ptr(z.device)
        z, (M, C, ldz) = _as_rows(z)
        res, (_, _, ldr) = _as_rows(res)
        y = _empty_like_rows(z)
        _, _, ldy = _rows_view(y)
        pb = int(gamma.dtype == _BF16)
        stats = None
        if training:
            stats = zeros_f32(_lib.stat_floats(C), z.device)
            rc = L.tony_bn_stats(z.data_ptr(), M, C, ldz, stats.data_ptr(), stats.data_ptr() + 4 * C, 2 * C,
                                 stream)
            _lib.check(rc, "tony_bn_stats")
        mask = _res_mask(M, C, z.device) if training and ldz == C else None
        mean, invstd = _bn_stats_and_apply(L, z, ldz, M, C, res, ldr, y, ldy, gamma, beta, pb, eps, training,
                                           momentum, running_mean, running_var, stats, stream, mask)
        ctx.save_for_backward(z, y if mask is None else mask, gamma, beta, mean, invstd)
        ctx.params = (gamma, beta)
        ctx.pb = pb
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        z, y, gamma, beta, mean, invstd = ctx.saved_tensors
        M, C, ldz = _rows_view(z)
        dz, dres, (dg, db) = _bwd_res(L, z, ldz, dy, y, M, C, mean, invstd, gamma, beta, ctx.pb, ctx.params,
                                      _lib.stream_ptr(z.device))
        _lib.report_inplace(ctx.params, (dg, db))
        return dz, dres, dg, db, None, None, None, None, None


class _Conv1x1BNAddReLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, res, gamma, beta, running_mean, running_var, training, momentum, eps):
        L = _lib.lib()
        dev = x.device
        stream = _lib.stream_ptr(dev)
        x, (M, cin, ldx) = _as_rows(x)
        res, (_, _, ldr) = _as_rows(res)
        n, _, h, w = x.shape
        cout = weight.shape[0]
        w2 = weight.reshape(cout, cin)
        if w2.stride(0) != cin or w2.stride(1) != 1:
            w2 = w2.contiguous()
        Z = _cl_empty(n, cout, h, w, dev)
        stats = zeros_f32(_lib.stat_floats(cout), dev)
        rc = L.tony_gemm_bf16(x.data_ptr(), w2.data_ptr(), Z.data_ptr(), M, cout, cin, ldx, cin, cout,
                              (1 if training else 0) | tune.gemm_flags(x, w2, Z, M, cout, cin, ldx, training),
                              stats.data_ptr(), 2 * cout, stream)
        _lib.check(rc, "tony_gemm_bf16")
        y = _cl_empty(n, cout, h, w, dev)
        pb = int(gamma.dtype == _BF16)
        mask = _res_mask(M, cout, dev) if training else None
        mean, invstd = _bn_stats_and_apply(L, Z, cout, M, cout, res, ldr, y, cout, gamma, beta, pb, eps, training,
                                           momentum, running_mean, running_var, stats, stream, mask)
        ctx.save_for_backward(x, weight, Z, y if mask is None else mask, gamma, beta, mean, invstd)
        ctx.params = (weight, gamma, beta)
        ctx.pb = pb
        ctx.join = getattr(res, "_tony_join", None)
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        x, weight, Z, y, gamma, beta, mean, invstd = ctx.saved_tensors
        dev = x.device
        stream = _lib.stream_ptr(dev)
        M, cin, ldx = _rows_view(x)
        n, _, h, w = x.shape
        cout = weight.shape[0]
        masked = False
        if ctx.join is not None and y.dtype == torch.uint8 and ctx.join.wants_masked():
            dy, (_, _, lddy) = _as_rows(dy)
            masked = lddy == cout and dy.data_ptr() % 16 == 0 and tuple(dy.shape) == (n, cout, h, w)
        dZ, dres, (dg, db) = _bwd_res(L, Z, cout, dy, y, M, cout, mean, invstd, gamma, beta, ctx.pb, ctx.params[1:],
                                      stream, want_dres=not masked)
        gw = _lib.grad_slot(ctx.params[0])
        dw = None
        if gw is not None and dg is None:  # dW summed straight into the flat gradient slot (side stream)
            streams.run(lambda: wgrad_tn(dZ.data_ptr(), cout, x.data_ptr(), ldx, M, cout, cin, dev, dst=gw), dZ, x)
        dx = None
        if ctx.needs_input_grad[0]:
            wt = wt_cache.transposed(weight).reshape(cin, cout)
            dx = _cl_empty(n, cin, h, w, dev)
            rc = L.tony_gemm_bf16(dZ.data_ptr(), wt.data_ptr(), dx.data_ptr(), M, cin, cout, cout, cout, cin,
                                  tune.gemm_flags(dZ, wt, dx, M, cin, cout, cout, False), 0, 0, stream)
            _lib.check(rc, "tony_gemm_bf16")
        if gw is None or dg is not None:
            dw = wgrad_tn(dZ.data_ptr(), cout, x.data_ptr(), ldx, M, cout, cin, dev).to(weight.dtype)
            dw = dw.reshape(weight.shape)
        _lib.report_inplace(ctx.params, (dw, dg, db))
        if masked:  # conv1's dgrad epilogue adds dY * mask to its dX (GradJoin, MaskedGrad)
            dres = ctx.join.park_masked(dy, y)
        elif ctx.join is not None:  # conv1's dgrad adds its dX into it, or it already ran (GradJoin)
            dres = ctx.join.park(dres)
        return dx, dw, dres, dg, db, None, None, None, None, None


def bn_add_relu_reference(z, res, gamma, beta, running_mean, running_var, training, momentum, eps):
    return torch.relu(torch.nn.functional.batch_norm(z, running_mean, running_var, gamma, beta, training, momentum,
                                                     eps) + res)


def bn_add_relu(z, res, gamma, beta, running_mean, running_var, training=True, momentum=0.1, eps=1e-5):
    if z.is_cuda:
        if z.dtype != _BF16:
            raise TypeError("bn_add_relu HIP kernel takes bf16 activations")
        return tape.apply(_BNAddReLUFn, z, res, gamma, beta, running_mean, running_var, training, momentum, eps)
    return bn_add_relu_reference(z, res, gamma, beta, running_mean, running_var, training, momentum, eps)


def conv1x1_bn_add_relu(x, weight, res, gamma, beta, running_mean, running_var, training=True, momentum=0.1,
                        eps=1e-5):
    if x.is_cuda:
        if x.dtype != _BF16:
            raise TypeError("conv1x1_bn_add_relu HIP path takes bf16 activations")
        return tape.apply(_Conv1x1BNAddReLUFn, x, weight, res, gamma, beta, running_mean, running_var, training, momentum,
                                         eps)
    z = torch.nn.functional.conv2d(x, weight)
    return bn_add_relu_reference(z, res, gamma, beta, running_mean, running_var, training, momentum, eps)
