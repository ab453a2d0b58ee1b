"""Fused "conv head": every 1x1 conv that reads the same input, as ONE MFMA GEMM.

An Inception block feeds its input x to several branches whose first layer is
a 1x1 conv + BN + ReLU, plus an avg-pool branch (avgpool 3x3/s1/p1 -> 1x1 conv
-> BN -> ReLU).  Per-channel BN and per-pixel 1x1 convs compose cleanly, so the
MI355X-native schedule is:

forward
    Z = x . [W_1 | W_2 | ... | W_pool]^T          one MFMA GEMM, N = sum(C_i);
                                                  BN sums/sum-squares of every
                                                  column come out of its epilogue
    y_i = relu(bn_i(Z[:, slice_i]))               apply kernels read channel slices
    P   = avgpool3x3(Z[:, pool])                  linear ops commute: conv(avg(x)) ==
    y_p = relu(bn_p(P))                           avg(conv(x)), and the pool now runs
                                                  on pool_ch (32..192) channels
                                                  instead of Cin (192..2048)
backward
    dZ[:, slice_i] = bn_bwd_i(dy_i)               written into one [M, sum C_i] buffer
    dZ[:, pool]    = avgpool3x3(bn_bwd_p(dy_p))   (the box stencil is self-adjoint)
    dx = dZ . W                                   ONE backward-data GEMM: the input
    dW = dZ^T x                                   gradient needs no per-branch adds

Compared with the textbook graph this removes the separate BN statistics pass
of each head conv, 2-3 gradient-accumulation adds of the block input per block,
the avg-pool over Cin channels, and turns 3-4 small GEMMs into one wide one.
A single-split head is simply conv1x1 + BN + ReLU with epilogue statistics.
"""
from __future__ import annotations

import os
from typing import Sequence

import torch
from torch import nn

from . import _lib, concat, streams, tape, tune, wt_cache
from .arena import zeros_f32
from .bn import MaskedGrad, _accum_ok, _as_rows, _rows_view
from .gemm import wgrad_tn

_BF16 = torch.bfloat16


def _cl_empty(n, c, h, w, device, dtype=_BF16):
    return torch.empty((n, c, h, w), dtype=dtype, device=device, memory_format=torch.channels_last)


def _off(t: torch.Tensor, elems: int) -> int:
    return t.data_ptr() + elems * t.element_size()


# TONY_BN_SEGS=0: one BN apply / reduce / apply launch per head split instead of one per head
SEGS = os.environ.get("TONY_BN_SEGS", "1") != "0"


def _seg_ends(splits):
    """Cumulative column ends of up to 4 splits, padded to 4 values (the C ABI's fixed arity)."""
    ends, e = [], 0
    for c in splits:
        e += c
        ends.append(e)
    return ends + [0] * (4 - len(ends))


def _seg_args(tensors):
    """(4 data pointers, 4 row strides) of up to 4 per-split row tensors, zero-padded."""
    ptr = [t.data_ptr() for t in tensors] + [0] * (4 - len(tensors))
    ld = [_rows_view(t)[2] for t in tensors] + [0] * (4 - len(tensors))
    return ptr, ld


class _HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, gamma, beta, running_mean, running_var, splits, npool, training, momentum, eps,
                slots=None):
        L = _lib.lib()
        _lib.check_f32_stats(running_mean, running_var)
        dev = x.device
        stream = _lib.stream_ptr(dev)
        ctx.join = getattr(x, "_tony_join", None)  # ops/residual.py GradJoin: x has a second consumer
        x, (M, cin, ldx) = _as_rows(x)
        n, _, h, w = x.shape
        ctot = weight.shape[0]
        w2 = weight.reshape(ctot, cin)
        if w2.stride(0) != cin or w2.stride(1) != 1:
            w2 = w2.contiguous()
        pb = int(gamma.dtype == _BF16)
        Z = _cl_empty(n, ctot, h, w, dev)
        # the GEMM epilogue accumulates [sum | sumsq] into it (STAT_SHARDS copies, stride 2*ctot)
        stats = zeros_f32(_lib.stat_floats(ctot), dev)
        ss = 2 * ctot
        rc = L.tony_gemm_bf16(x.data_ptr(), w2.data_ptr(), Z.data_ptr(), M, ctot, cin, ldx, cin, ctot,
                              (1 if training else 0) | tune.gemm_flags(x, w2, Z, M, ctot, cin, ldx, training),
                              stats.data_ptr(), ss, stream)
        _lib.check(rc, "tony_gemm_bf16")
        if training:
            mean = torch.empty(ctot, dtype=torch.float32, device=dev)
            invstd = torch.empty(ctot, dtype=torch.float32, device=dev)
        else:
            mean = running_mean
            invstd = torch.rsqrt(running_var.float() + eps)
        mode = 0 if training else 1
        outs = []
        slots = slots or ()
        for k, ci in enumerate(splits):
            # a final branch output goes straight into the block's concat buffer (ops/concat.py)
            y = concat.take(slots[k] if k < len(slots) else None, n, ci, h, w, x)
            if y is None:
                y = _cl_empty(n, ci, h, w, dev)
            outs.append(y)
        # every split normalised by ONE launch (csrc/bn_act.hip segment table), else one per split
        csum = sum(splits)
        rc = -1
        if SEGS and 1 <= len(splits) <= 4:
            ptr, ld = _seg_args(outs)
            ends = _seg_ends(splits)
            rc = L.tony_bn_apply_segs(Z.data_ptr(), M, csum, ctot, len(splits), *ends, *ptr, *ld, stats.data_ptr(),
                                      _off(stats, ctot), ss, gamma.data_ptr(), beta.data_ptr(), pb, float(eps), 1,
                                      mode, mean.data_ptr() if training else 0, invstd.data_ptr() if training else 0,
                                      _lib.ptr(running_mean), _lib.ptr(running_var), float(momentum), stream)
        c0 = 0
        for y, ci in zip(outs, splits):
            if rc != 0:
                rc2 = L.tony_bn_apply(_off(Z, c0), M, ci, ctot, y.data_ptr(), _rows_view(y)[2], _off(stats, c0),
                                      _off(stats, ctot + c0), ss, _off(gamma, c0), _off(beta, c0), pb, float(eps), 1,
                                      mode, _off(mean, c0) if training else 0, _off(invstd, c0) if training else 0,
                                      _off(running_mean, c0), _off(running_var, c0), float(momentum), stream)
                _lib.check(rc2, "tony_bn_apply")
            c0 += ci
        P = None
        if npool:
            P = _cl_empty(n, npool, h, w, dev)
            rc = L.tony_avgpool3_s1p1(_off(Z, c0), P.data_ptr(), n, h, w, npool, ctot, npool, stream)
            _lib.check(rc, "tony_avgpool3_s1p1")
            pstats = None
            if training:  # statistics of the pooled tensor (the GEMM's columns c0.. are pre-pool)
                pstats = zeros_f32(_lib.stat_floats(npool), dev)
                rc = L.tony_bn_stats(P.data_ptr(), M, npool, npool, pstats.data_ptr(), _off(pstats, npool),
                                     2 * npool, stream)
                _lib.check(rc, "tony_bn_stats")
            k = len(splits)
            y = concat.take(slots[k] if k < len(slots) else None, n, npool, h, w, x)
            if y is None:
                y = _cl_empty(n, npool, h, w, dev)
            rc = L.tony_bn_apply(P.data_ptr(), M, npool, npool, y.data_ptr(), _rows_view(y)[2], _lib.ptr(pstats),
                                 _off(pstats, npool) if training else 0, 2 * npool if training else 0,
                                 _off(gamma, c0), _off(beta, c0), pb,
                                 float(eps), 1, mode,
                                 _off(mean, c0) if training else 0, _off(invstd, c0) if training else 0,
                                 _off(running_mean, c0), _off(running_var, c0), float(momentum), stream)
            _lib.check(rc, "tony_bn_apply")
            outs.append(y)
        ctx.save_for_backward(x, weight, gamma, beta, mean, invstd, Z, P)
        ctx.params = (weight, gamma, beta)
        ctx.splits = tuple(splits)
        ctx.npool = npool
        ctx.pb = pb
        return tuple(outs)

    @staticmethod
    def backward(ctx, *douts):
        L = _lib.lib()
        x, weight, gamma, beta, mean, invstd, Z, P = ctx.saved_tensors
        dev = x.device
        stream = _lib.stream_ptr(dev)
        M, cin, ldx = _rows_view(x)
        n, _, h, w = x.shape
        ctot = weight.shape[0]
        pb = ctx.pb
        dZ = _cl_empty(n, ctot, h, w, dev)
        # each split's BN-backward reduction accumulates into its slice (STAT_SHARDS copies, stride 2*ctot)
        dsum = zeros_f32(_lib.stat_floats(ctot), dev)
        ss = 2 * ctot
        gw, gg, gb = (_lib.grad_slot(p) for p in ctx.params)
        inplace = gw is not None and gg is not None and gb is not None
        acc = int(inplace)
        dgamma = gg if inplace else torch.empty_like(gamma)
        dbeta = gb if inplace else torch.empty_like(beta)
        dys = [_as_rows(dy)[0] for dy in douts[:len(ctx.splits)]]
        rc = -1
        if SEGS and 1 <= len(ctx.splits) <= 4:  # every split's reduce / apply in ONE launch each
            ptr, ld = _seg_args(dys)
            ends = _seg_ends(ctx.splits)
            csum = sum(ctx.splits)
            rc = L.tony_bn_bwd_reduce_segs(Z.data_ptr(), ctot, len(ctx.splits), *ends, *ptr, *ld, M, csum,
                                           mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(), pb,
                                           1, dsum.data_ptr(), _off(dsum, ctot), ss, stream)
            if rc == 0:
                rc = L.tony_bn_bwd_apply_segs(Z.data_ptr(), ctot, len(ctx.splits), *ends, *ptr, *ld, dZ.data_ptr(),
                                              ctot, M, csum, mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(),
                                              beta.data_ptr(), pb, 1, dsum.data_ptr(), _off(dsum, ctot), ss,
                                              dgamma.data_ptr(), dbeta.data_ptr(), acc, stream)
                _lib.check(rc, "tony_bn_bwd_apply_segs")
        c0 = 0
        for ci, dy in zip(ctx.splits, dys):
            if rc == 0:
                break
            lddy = _rows_view(dy)[2]
            rc2 = L.tony_bn_bwd_reduce(_off(Z, c0), ctot, dy.data_ptr(), lddy, M, ci, _off(mean, c0),
                                       _off(invstd, c0), _off(gamma, c0), _off(beta, c0), pb, 1, _off(dsum, c0),
                                       _off(dsum, ctot + c0), ss, stream)
            _lib.check(rc2, "tony_bn_bwd_reduce")
            rc2 = L.tony_bn_bwd_apply(_off(Z, c0), ctot, dy.data_ptr(), lddy, _off(dZ, c0), ctot, M, ci,
                                      _off(mean, c0), _off(invstd, c0), _off(gamma, c0), _off(beta, c0), pb, 1,
                                      _off(dsum, c0), _off(dsum, ctot + c0), ss, _off(dgamma, c0), _off(dbeta, c0),
                                      acc, stream)
            _lib.check(rc2, "tony_bn_bwd_apply")
            c0 += ci
        c0 = sum(ctx.splits)  # the pool branch's columns follow the splits
        if ctx.npool:
            npool = ctx.npool
            dy, (_, _, lddy) = _as_rows(douts[len(ctx.splits)])
            dP = _cl_empty(n, npool, h, w, dev)
            rc = L.tony_bn_bwd_reduce(P.data_ptr(), npool, dy.data_ptr(), lddy, M, npool, _off(mean, c0),
                                      _off(invstd, c0), _off(gamma, c0), _off(beta, c0), pb, 1, _off(dsum, c0),
                                      _off(dsum, ctot + c0), ss, stream)
            _lib.check(rc, "tony_bn_bwd_reduce")
            rc = L.tony_bn_bwd_apply(P.data_ptr(), npool, dy.data_ptr(), lddy, dP.data_ptr(), npool, M, npool,
                                     _off(mean, c0), _off(invstd, c0), _off(gamma, c0), _off(beta, c0), pb, 1,
                                     _off(dsum, c0), _off(dsum, ctot + c0), ss, _off(dgamma, c0), _off(dbeta, c0),
                                     acc, stream)
            _lib.check(rc, "tony_bn_bwd_apply")
            rc = L.tony_avgpool3_s1p1(dP.data_ptr(), _off(dZ, c0), n, h, w, npool, npool, ctot, stream)
            _lib.check(rc, "tony_avgpool3_s1p1")
        if inplace:  # dW summed straight into the flat gradient slot ([ctot][cin] = the slot's order),
            # issued first so that it overlaps the dgrad GEMM on the weight-gradient stream
            streams.run(lambda: wgrad_tn(dZ.data_ptr(), ctot, x.data_ptr(), ldx, M, ctot, cin, dev, dst=gw), dZ, x)
        dx = None
        join = getattr(ctx, "join", None) if ctx.needs_input_grad[0] else None
        pend = join.take(masked_ok=True) if join is not None else None
        if ctx.needs_input_grad[0]:
            wt = wt_cache.transposed(weight).reshape(cin, ctot)  # [Cin, Ctot]
            dx = _cl_empty(n, cin, h, w, dev)
            vf = tune.gemm_flags(dZ, wt, dx, M, cin, ctot, ctot, False)  # timing runs write dx, never pend
            if isinstance(pend, MaskedGrad):
                # the residual tail parked dY and its ReLU mask: the epilogue writes dX + dY * mask (bit 5;
                # the source rows ride in the stats argument, the mask's address in sstride)
                if tuple(pend.dy.shape) == tuple(x.shape) and pend.mask.shape == (M, cin // 8):
                    rc = L.tony_gemm_bf16(dZ.data_ptr(), wt.data_ptr(), dx.data_ptr(), M, cin, ctot, ctot, ctot, cin,
                                          vf | 32, pend.dy.data_ptr(), pend.mask.data_ptr(), stream)
                    if rc == 0:
                        pend = None
                        vf = None
                if pend is not None:
                    pend = pend.materialize()
        if ctx.needs_input_grad[0] and vf is not None:
            if pend is not None and _accum_ok(pend, x.shape):
                # x's other consumer (the identity path) already wrote its gradient: the epilogue adds
                # dX into it (bit 4) -- no separate add kernel
                dx = pend
                vf |= 16
            rc = L.tony_gemm_bf16(dZ.data_ptr(), wt.data_ptr(), dx.data_ptr(), M, cin, ctot, ctot, ctot, cin,
                                  vf, 0, 0, stream)
            _lib.check(rc, "tony_gemm_bf16")
            if pend is not None and dx is not pend:
                dx = pend.add_(dx)
            elif pend is None and join is not None:
                dx = join.settle(dx)  # first of the two: parked for the other consumer
        if inplace:
            _lib.report_inplace(ctx.params, (None, None, None))
            return dx, None, None, None, None, None, None, None, None, None, None, None
        dw32 = wgrad_tn(dZ.data_ptr(), ctot, x.data_ptr(), ldx, M, ctot, cin, dev)
        dw = dw32.to(weight.dtype).reshape(weight.shape)
        return dx, dw, dgamma, dbeta, None, None, None, None, None, None, None, None


def head_reference(x, weight, gamma, beta, running_mean, running_var, splits, npool, training, momentum, eps):
    """PyTorch fp32-capable reference of the fused head (CPU path and tests)."""
    z = torch.nn.functional.conv2d(x, weight)
    outs = []
    c0 = 0
    for ci in splits:
        sl = slice(c0, c0 + ci)
        outs.append(torch.relu(torch.nn.functional.batch_norm(
            z[:, sl], running_mean[sl] if running_mean is not None else None,
            running_var[sl] if running_var is not None else None, gamma[sl], beta[sl], training, momentum, eps)))
        c0 += ci
    if npool:
        sl = slice(c0, c0 + npool)
        # contiguous NCHW on purpose: this PyTorch-ROCm build's channels_last
        # avg_pool2d backward returns wrong gradients on the GPU
        p = torch.nn.functional.avg_pool2d(z[:, sl].contiguous(), 3, 1, 1, count_include_pad=True)
        outs.append(torch.relu(torch.nn.functional.batch_norm(
            p, running_mean[sl] if running_mean is not None else None,
            running_var[sl] if running_var is not None else None, gamma[sl], beta[sl], training, momentum, eps)))
    return tuple(outs)


class FusedHead(nn.Module):
    """Parallel 1x1 conv+BN+ReLU branches (and an optional avgpool->1x1 branch) on one input."""

    def __init__(self, cin: int, couts: Sequence[int], pool_cout: int = 0, eps: float = 1e-3,
                 momentum: float = 0.1):
        super().__init__()
        self.splits = tuple(int(c) for c in couts)
        self.npool = int(pool_cout)
        total = sum(self.splits) + self.npool
        self.conv = nn.Conv2d(cin, total, 1, bias=False)
        self.bn = nn.BatchNorm2d(total, eps=eps, momentum=momentum)

    def forward(self, x, slots=None, planes=None):
        """One output per split (+ the pool branch); ``slots`` (per output, None or a concat.Slot)
        lets final branch outputs land directly in the block's concat buffer.  fp32 input: the x3 head
        (ops/x3.py head), where ``planes[k]`` hands split k over as the next conv's operand planes only."""
        training = self.training
        args = (x, self.conv.weight, self.bn.weight, self.bn.bias, self.bn.running_mean, self.bn.running_var,
                self.splits, self.npool, training, self.bn.momentum, self.bn.eps)
        if x.is_cuda and x.dtype == torch.float32:
            from . import x3

            return x3.head(*args, slots=slots, planes=planes)
        if x.is_cuda and x.dtype != torch.float64:
            if x.dtype != _BF16:
                raise TypeError("FusedHead HIP path takes bf16 (or fp32: x3) activations")
            return tape.apply(_HeadFn, *args, tuple(slots) if slots else None)
        return head_reference(*args)
