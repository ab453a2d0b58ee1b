"""fp32 training on the bf16 matrix cores: the x3 operand split (csrc/x3.hip).

The reference's TF-PS job trains in fp32 (``tony-examples/mnist-tensorflow/mnist_distributed.py:64-124``).
MI355X's matrix cores are bf16/fp8 machines (fp32 MFMA runs at 1/16 of the bf16 rate), so the fp32
step keeps every tensor -- activations, gradients, BN statistics, variables -- in fp32 and only the
convolution / GEMM *products* go through the bf16 MFMAs, each fp32 operand split as hi + lo:

    x * w  ~=  hi_x*hi_w + lo_x*hi_w + hi_x*lo_w        (lo_x*lo_w <= 2^-16 |x w| dropped)

With activations laid out as channel planes [hi | lo | hi] and weights as [hi | hi | lo] (``split``),
that sum is ONE implicit GEMM over 3x the channels on the same tuned kernels as the bf16 step, with
the fp32 epilogue (flag bit 3 of tony_conv_fwd / tony_conv_dgrad / tony_gemm_bf16).  Weight gradients
are the three plane pairs through the bf16 split-K wgrad kernels, summed in fp32.  BatchNorm, pooling
and the loss run on fp32 rows (the ``*_f32`` entry points of csrc/bn_act.hip, csrc/pool.hip,
csrc/loss.hip).  Products are accurate to ~2^-16 relative (fp32: 2^-24; the TF32 that TensorFlow's
fp32 convolutions default to on tensor-core GPUs: 2^-11); accumulation is fp32 throughout.

``ConvBNActX3`` is the layer (conv + BN + ReLU); ``inception_v3(precision="fp32")`` builds the whole
model from it (models/inception_v3.py).
"""
from __future__ import annotations

import ctypes
import os
from typing import Tuple

import torch

from . import _lib, concat, streams, tune, wt_cache
from .arena import zeros_f32
from .bn import _as_rows, _rows_view

ACT = 0b010  # activation / gradient planes: [hi | lo | hi]
WGT = 0b100  # weight planes:                [hi | hi | lo]
_F32 = torch.float32
_BF16 = torch.bfloat16


def cp_of(c: int) -> int:
    """Channels per plane: C rounded up to 8 (16-byte aligned planes; the 3-channel image: 8)."""
    return (c + 7) // 8 * 8


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def split_rows(src: torch.Tensor, rows: int, c: int, ld: int, pattern: int) -> torch.Tensor:
    """bf16 [rows, 3 * cp] planes of the fp32 rows ``src`` ([rows][c] at row stride ld)."""
    cp = cp_of(c)
    out = torch.empty((rows, 3 * cp), dtype=_BF16, device=src.device)
    rc = _lib.lib().tony_x3_split(src.data_ptr(), ld, rows, c, cp, out.data_ptr(), 3 * cp, pattern,
                                  _lib.stream_ptr(src.device))
    _lib.check(rc, "tony_x3_split")
    return out


def split_act(x: torch.Tensor) -> Tuple[torch.Tensor, int]:
    """fp32 NHWC activation (channels_last 4D, a channel slice of one, or [M, C]) -> bf16 planes as a
    channels_last [N, 3cp, H, W] tensor (2D input: [M, 3cp]); also returns cp.  The planes are kept on
    ``x`` (keyed by its version counter): an Inception block input feeds 3-4 branch heads, which then
    share one split of it instead of making one each."""
    hit = getattr(x, "_tony_x3", None)
    if hit is not None and hit[0] == x._version:
        return hit[1], hit[2]
    src = x
    x, (m, c, ld) = _rows4(x)
    out = split_rows(x, m, c, ld, ACT)
    cp = cp_of(c)
    if x.dim() == 4:
        n, _, h, w = x.shape
        out = out.view(n, h, w, 3 * cp).permute(0, 3, 1, 2)
    # only activations made inside the step (grad_fn set): a persistent input -- the trainer's static
    # batch, refilled by copy_ between replays of a captured step -- must be split inside the capture
    if x is src and src.grad_fn is not None:
        src._tony_x3 = (src._version, out, cp)
    return out, cp


def _rows4(x: torch.Tensor):
    if x.dtype != _F32:
        raise TypeError(f"x3 path: fp32 activations expected, got {x.dtype}")
    return _as_rows(x)  # (rows, (M, C, ld)); the RGB image (C = 3): dense channels_last, ld = 3


def split_weight(w: torch.Tensor) -> torch.Tensor:
    """fp32 conv weight [Co, C, R, S] -> bf16 [Co][R][S][3cp] planes [hi | hi | lo] (KRSC memory)."""
    co, c, r, s = w.shape
    wk = w.permute(0, 2, 3, 1)
    wk = wk if wk.is_contiguous() else wk.contiguous()
    return split_rows(wk, co * r * s, c, c, WGT)


def split_weight_t(w: torch.Tensor) -> torch.Tensor:
    """fp32 conv weight [Co, C, R, S] -> bf16 [C][R][S][3Co] planes [hi | hi | lo] (the dgrad operand)."""
    co, c, r, s = w.shape
    wk = w.permute(0, 2, 3, 1)
    wk = wk if wk.is_contiguous() else wk.contiguous()
    out = torch.empty((c, r, s, 3 * co), dtype=_BF16, device=w.device)
    rc = _lib.lib().tony_x3_weights_t(wk.data_ptr(), co, r * s, c, out.data_ptr(), _lib.stream_ptr(w.device))
    _lib.check(rc, "tony_x3_weights_t")
    return out


def _cl(n, c, h, w, dev, dtype=_F32):
    return torch.empty((n, c, h, w), dtype=dtype, device=dev, memory_format=torch.channels_last)


# ---- convolution passes ---------------------------------------------------------------------------
def conv_fwd(x3: torch.Tensor, cp: int, w3: torch.Tensor, wshape, stride, padding, stats=None) -> torch.Tensor:
    """fp32 Z = conv(x, w) from the planes x3 [N, 3cp, H, W] and w3 [Co][R][S][3cp]; with ``stats``
    (zeroed, _lib.stat_floats(Co)) the epilogue adds the BN [sum | sumsq] of Z."""
    n, _, h, w = x3.shape
    co, _, r, s = wshape
    (sh, sw), (ph, pw) = _pair(stride), _pair(padding)
    oh, ow = (h + 2 * ph - r) // sh + 1, (w + 2 * pw - s) // sw + 1
    z = _cl(n, co, oh, ow, x3.device)
    ldx = 3 * cp  # dense planes (split_act)
    L, st = _lib.lib(), _lib.stream_ptr(x3.device)
    base = 8 | (1 if stats is not None else 0)

    def launch(vf, stats_t):
        return L.tony_conv_fwd(x3.data_ptr(), n, h, w, 3 * cp, ldx, w3.data_ptr(), co, r, s, sh, sw, ph, pw,
                               z.data_ptr(), oh, ow, co, (base if stats_t is not None else 8) | vf,
                               _lib.ptr(stats_t), 2 * co, st)

    key = ("x3_fwd", tuple(x3.shape), ldx, tuple(wshape), (sh, sw), (ph, pw), stats is not None)
    vf = tune.cached(key)
    if vf is None:
        scratch = torch.zeros(_lib.stat_floats(co), device=x3.device) if stats is not None else None
        vf = tune.pick(key, lambda v: launch(v, scratch), tune.X3_VARIANTS + (tune.X3F_VARIANTS if cp % 32 == 0 else ()))
    _lib.check(launch(vf, stats), "tony_conv_fwd (x3)")
    return z


def _accum_f32_ok(t, x_shape) -> bool:
    """``t`` can take the fp32 dgrad epilogue's accumulating store: fp32, x's shape, dense channels_last."""
    if t is None or t.dtype != _F32 or tuple(t.shape) != tuple(x_shape) or t.data_ptr() % 16:
        return False
    rv = _rows_view(t)
    return rv is not None and rv[2] == t.shape[1]


def conv_dgrad(d3: torch.Tensor, wt3: torch.Tensor, co: int, x_shape, wshape, stride, padding,
               accum: torch.Tensor | None = None) -> torch.Tensor:
    """fp32 dX from the dZ planes d3 [N, 3Co, OH, OW] and wt3 [C][R][S][3Co].  ``accum``: an fp32 gradient
    of x's shape (dense channels_last) that dX is added into by the epilogue (flag bit 4) and returned --
    a tensor with several consumers (ops/residual.py GradJoin) needs no add kernel."""
    n, c, h, w = x_shape
    _, _, r, s = wshape
    (sh, sw), (ph, pw) = _pair(stride), _pair(padding)
    _, _, oh, ow = d3.shape
    acc = 16 if _accum_f32_ok(accum, x_shape) else 0
    dx = accum if acc else _cl(n, c, h, w, d3.device)
    L, st = _lib.lib(), _lib.stream_ptr(d3.device)
    ldd = 3 * co
    def launch(vf, out=dx, flags=8):
        if (sh, sw) == (1, 1):
            return L.tony_conv_dgrad(d3.data_ptr(), n, oh, ow, 3 * co, ldd, wt3.data_ptr(), c, r, s, ph, pw,
                                     out.data_ptr(), h, w, c, flags | vf, None, st)
        return L.tony_conv_dgrad_strided(d3.data_ptr(), n, oh, ow, 3 * co, ldd, wt3.data_ptr(), c, r, s, sh, sw,
                                         ph, pw, out.data_ptr(), h, w, c, flags | vf, None, st)
    name = "tony_conv_dgrad (x3)" if (sh, sw) == (1, 1) else "tony_conv_dgrad_strided (x3)"
    key = ("x3_dgrad", tuple(d3.shape), tuple(x_shape), tuple(wshape), (sh, sw), (ph, pw))
    variants = tuple(v for v in tune.X3_VARIANTS if v != 9)  # fp32 epilogue: NT / LDS-DMA / direct kernels
    from .conv import STRIDED_GLDS

    if (sh, sw) != (1, 1):  # the strided dgrad refuses stream-K forms
        variants = tuple(v for v in variants if (v < 11 or STRIDED_GLDS) and v < 256)  # v + 256 m: stream-K
    elif co % 32 == 0:  # the fused-plane tiles (stride-1 dgrad: the gather runs over dY's Co planes)
        variants = variants + tune.X3F_VARIANTS
    vf = tune.cached(key)
    if vf is None:  # timed into a scratch output: an accumulating call must add exactly once
        scratch = _cl(n, c, h, w, d3.device) if acc else dx
        vf = tune.pick(key, lambda v: launch(v, scratch), variants)
    rc = launch(vf, dx, 8 | acc)
    if rc == -3 and acc:  # the chosen variant has no accumulating store (the direct kernel): add after
        dx = _cl(n, c, h, w, d3.device)
        rc = launch(vf, dx, 8)
        acc = 0
    _lib.check(rc, name)
    if accum is not None and not acc:
        return accum.add_(dx)
    return dx


def conv_wgrad(d3: torch.Tensor, x3: torch.Tensor, cp: int, wshape, stride, padding, dst=None):
    """fp32 dW [Co, C, R, S] (channels_last memory [Co][R][S][C]) = the three plane products
    hi_d*hi_x + hi_d*lo_x + lo_d*hi_x: ONE split-K wgrad launch whose splits come in three plane-pair
    groups (csrc/conv.hip tony_conv_wgrad_x3) and one combine of all their partials -- not three
    launches, three combines and an fp32 accumulator fill (profiles/r3s2_fp32_x3_steady.md).
    ``dst``: an fp32 gradient slot in [Co][R][S][C] memory (C a multiple of 8) that the combine adds
    dW into; returns None then."""
    from .gemm import splitk_combine, wgrad_cus, x3_occ

    co, c, r, s = wshape
    dev = d3.device
    d3, (_, _, lddy) = _as_rows(d3)
    x3, (_, _, ldx) = _as_rows(x3)
    n, _, h, w = x3.shape
    _, _, oh, ow = d3.shape
    (sh, sw), (ph, pw) = _pair(stride), _pair(padding)
    L = _lib.lib()
    if WGRAD_DIRECT and cp == c and c in (32, 64) and co in (32, 64) and (r, s) == (3, 3) and (sh, sw) == (1, 1):
        return _wgrad_direct3(d3, lddy, x3, ldx, n, h, w, c, co, ph, pw, oh, ow, dst)
    tbm = 32 if co <= 32 else 64 if co <= 64 else 128  # csrc/conv.hip wgrad tile rows
    ntiles = -(-co // tbm) * -(-(r * s * cp) // 128)
    occ = x3_occ(n * oh * ow)
    acc = splitk_combine(
        lambda slab, cap, sp, fc, fd, ff: L.tony_conv_wgrad_x3(
            d3.data_ptr(), lddy, x3.data_ptr(), n, h, w, cp, ldx, co, r, s, sh, sw, ph, pw, oh, ow, co, cp, slab, cap,
            sp, wgrad_cus(dev, occ), _lib.stream_ptr(dev)),
        co * r * s * cp, ntiles, dev, dst if cp == c else None, occ, pairs=3)
    if acc is None:
        return None
    dw = acc.view(co, r, s, cp)
    if cp != c:
        dw = dw[..., :c].contiguous()
    dw = dw.permute(0, 3, 1, 2)
    if dst is not None:  # the stem's padded planes: add the unpadded dW into the slot
        dst.add_(dw)
        return None
    return dw


# The 32 / 64-channel 3x3 stride-1 layers (the 147x147 / 149x149 stem): the bf16 step's persistent direct
# wgrad kernel (csrc/conv.hip conv_wgrad_direct_kernel) once per plane pair into three slab regions, one
# combine over all partials -- the split-K implicit GEMM's 32-row tiles took 759 us per layer for the
# three pairs (profiles/r4_fp32_x3_steady.md).  TONY_X3_WGRAD_DIRECT=0: the split-K path (A/B).
WGRAD_DIRECT = os.environ.get("TONY_X3_WGRAD_DIRECT", "1") != "0"


def _wgrad_direct3(d3, lddy, x3, ldx, n, h, w, c, co, ph, pw, oh, ow, dst=None):
    L = _lib.lib()
    cus = _lib.num_cus(d3.device)
    nel = co * 9 * c
    part = 2 * cus * nel  # one launch's partials (<= 2 workgroups per CU)
    slab = torch.empty(3 * part, dtype=_F32, device=d3.device)
    splits = ctypes.c_int(0)
    st = _lib.stream_ptr(d3.device)
    # hi_d * hi_x + hi_d * lo_x + lo_d * hi_x: plane offsets (elements) of d3 [hi | lo | hi], x3 [hi | lo | hi]
    for k, (do, xo) in enumerate(((0, 0), (0, c), (co, 0))):
        rc = L.tony_conv_wgrad_direct(d3.data_ptr() + 2 * do, lddy, x3.data_ptr() + 2 * xo, n, h, w, c, ldx, co,
                                      ph, pw, oh, ow, slab.data_ptr() + 4 * k * part, part,
                                      ctypes.addressof(splits), cus, st)
        _lib.check(rc, "tony_conv_wgrad_direct (x3)")
        if k < 2 and splits.value * nel != part:  # pack the three launches' partials back to back
            part = splits.value * nel
    out = dst if dst is not None else torch.empty(nel, dtype=_F32, device=d3.device)
    rc = L.tony_splitk_reduce(slab.data_ptr(), 3 * splits.value, nel, out.data_ptr(), int(out.dtype == _BF16),
                              int(dst is not None), cus, st)
    _lib.check(rc, "tony_splitk_reduce (x3 direct)")
    if dst is not None:
        return None
    return out.view(co, 3, 3, c).permute(0, 3, 1, 2)


# ---- BatchNorm on fp32 rows -------------------------------------------------------------------------
def _apply_f32(L, x_ptr, m, c, ldx, y, slot, tail):
    """tony_bn_apply_f32 of ``c`` channels into ``y``; when y is a concat slot whose buffer carries x3
    planes (ops/concat.X3_PLANES), the same pass also writes the slot's slice of the planes."""
    p3 = concat.planes_of(slot, c) if slot is not None and y.data_ptr() == slot.view(c).data_ptr() else None
    if p3 is not None:
        rc = L.tony_bn_apply_f32_p3(x_ptr, m, c, ldx, y.data_ptr(), _rows_view(y)[2], *p3, *tail)
        _lib.check(rc, "tony_bn_apply_f32_p3")
        concat.planes_written(slot)
        return
    _lib.check(L.tony_bn_apply_f32(x_ptr, m, c, ldx, y.data_ptr(), _rows_view(y)[2], *tail), "tony_bn_apply_f32")


def bn_apply(z: torch.Tensor, stats, gamma, beta, rmean, rvar, eps, momentum, relu, training, out=None, slot=None):
    """y = act(BN(z)) in fp32; training: batch statistics from ``stats`` (sharded [sum | sumsq]),
    running statistics updated.  ``out``: a channel slice of a block's concat buffer (ops/concat.py) to
    write y into (``slot``: that slice's Slot).  Returns (y, mean, invstd)."""
    n, co, oh, ow = z.shape
    m = n * oh * ow
    y = out if out is not None else _cl(n, co, oh, ow, z.device)
    mean = torch.empty(co, dtype=_F32, device=z.device)
    invstd = torch.empty(co, dtype=_F32, device=z.device)
    _apply_f32(_lib.lib(), z.data_ptr(), m, co, co, y, slot if out is not None else None,
               (_lib.ptr(stats), None if stats is None else stats.data_ptr() + 4 * co,
                2 * co if stats is not None else 0, gamma.data_ptr(), beta.data_ptr(), 0, float(eps), int(relu),
                0 if training else 1, mean.data_ptr(), invstd.data_ptr(), _lib.ptr(rmean), _lib.ptr(rvar),
                float(momentum), _lib.stream_ptr(z.device)))
    return y, mean, invstd


def bn_apply_planes(z: torch.Tensor, stats, gamma, beta, rmean, rvar, eps, momentum, relu, training):
    """bn_apply writing y as its x3 operand planes (bf16 channels_last [N, 3Co, OH, OW], split_act's layout;
    Co a multiple of 8).  Returns (planes, mean, invstd)."""
    n, co, oh, ow = z.shape
    m = n * oh * ow
    y3 = torch.empty((n, oh, ow, 3 * co), dtype=_BF16, device=z.device).permute(0, 3, 1, 2)
    mean = torch.empty(co, dtype=_F32, device=z.device)
    invstd = torch.empty(co, dtype=_F32, device=z.device)
    rc = _lib.lib().tony_bn_apply_f32_x3(z.data_ptr(), m, co, co, y3.data_ptr(), 3 * co, _lib.ptr(stats),
                                         None if stats is None else stats.data_ptr() + 4 * co,
                                         2 * co if stats is not None else 0, gamma.data_ptr(), beta.data_ptr(), 0,
                                         float(eps), int(relu), 0 if training else 1, mean.data_ptr(),
                                         invstd.data_ptr(), _lib.ptr(rmean), _lib.ptr(rvar), float(momentum),
                                         _lib.stream_ptr(z.device))
    _lib.check(rc, "tony_bn_apply_f32_x3")
    return y3, mean, invstd


def bn_backward(z, dy, mean, invstd, gamma, beta, relu, planes: bool = False, dgamma=None, dbeta=None):
    """(dZ, dgamma, dbeta) of y = act(BN(z)) on fp32 rows; ``planes``: dZ comes back as its x3 planes
    (bf16 channels_last [N, 3Co, OH, OW], split_act's layout) written by the apply kernel itself --
    the fp32 dZ and a split pass over it are never made (Co is a multiple of 8, so cp = Co).
    ``dgamma`` / ``dbeta``: fp32 gradient slots the kernel adds into (returned as None then)."""
    n, co, oh, ow = z.shape
    m = n * oh * ow
    dy, (_, _, lddy) = _as_rows(dy)
    dev = z.device
    sums = zeros_f32(_lib.stat_floats(co), dev)  # a slice of the step arena's one fill
    if planes and co % 8 == 0:
        dz = _cl(n, 3 * co, oh, ow, dev, _BF16)
        apply, ldo = L_apply_x3, 3 * co
    else:
        dz = _cl(n, co, oh, ow, dev)
        apply, ldo = None, co
    slots = dgamma is not None and dbeta is not None
    if not slots:
        dgamma = torch.empty(co, dtype=_F32, device=dev)
        dbeta = torch.empty(co, dtype=_F32, device=dev)
    L, st = _lib.lib(), _lib.stream_ptr(dev)
    rc = L.tony_bn_bwd_reduce_f32(z.data_ptr(), co, dy.data_ptr(), lddy, m, co, mean.data_ptr(), invstd.data_ptr(),
                                  gamma.data_ptr(), beta.data_ptr(), 0, int(relu), sums.data_ptr(),
                                  sums.data_ptr() + 4 * co, 2 * co, st)
    _lib.check(rc, "tony_bn_bwd_reduce_f32")
    fn = L.tony_bn_bwd_apply_f32_x3 if apply is not None else L.tony_bn_bwd_apply_f32
    rc = fn(z.data_ptr(), co, dy.data_ptr(), lddy, dz.data_ptr(), ldo, m, co, mean.data_ptr(), invstd.data_ptr(),
            gamma.data_ptr(), beta.data_ptr(), 0, int(relu), sums.data_ptr(), sums.data_ptr() + 4 * co, 2 * co,
            dgamma.data_ptr(), dbeta.data_ptr(), int(slots), st)
    _lib.check(rc, "tony_bn_bwd_apply_f32")
    return (dz, None, None) if slots else (dz, dgamma, dbeta)


L_apply_x3 = "tony_bn_bwd_apply_f32_x3"


class _ConvBNActX3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, gamma, beta, rmean, rvar, stride, padding, training, momentum, eps, relu, slot=None,
                planes_only=False):
        x3, cp = split_act(x)
        w3 = wt_cache.x3_planes(weight)  # split once per step after the optimizer (ops/wt_cache.py)
        if w3 is None:
            w3 = split_weight(weight)
        co = weight.shape[0]
        stats = zeros_f32(_lib.stat_floats(co), x.device) if training else None
        z = conv_fwd(x3, cp, w3, weight.shape, stride, padding, stats)
        n, _, oh, ow = z.shape
        if planes_only and slot is None and co % 8 == 0:
            # the only consumer is another x3 conv: BN writes its operand planes, the fp32 y is never made
            y3, mean, invstd = bn_apply_planes(z, stats, gamma, beta, rmean, rvar, eps, momentum, relu, training)
            _LAST_PLANES[0] = y3
            y = torch.empty_strided((n, co, oh, ow), (0, 0, 0, 0), dtype=_F32, device=z.device)  # shape only
        else:
            y, mean, invstd = bn_apply(z, stats, gamma, beta, rmean, rvar, eps, momentum, relu, training,
                                       out=concat.take(slot, n, co, oh, ow, z), slot=slot)
        ctx.save_for_backward(x3, weight, gamma, beta, z, mean, invstd)
        ctx.conf = (cp, tuple(x.shape), stride, padding, relu, x.requires_grad)
        ctx.join = getattr(x, "_tony_join", None)  # ops/residual.py GradJoin: x has other consumers
        return y

    @staticmethod
    def backward(ctx, dy):
        x3, weight, gamma, beta, z, mean, invstd = ctx.saved_tensors
        cp, x_shape, stride, padding, relu, need_dx = ctx.conf
        # in-place gradient slots (the trainer's flat fp32 gradients): BN's dgamma / dbeta are added by
        # the apply kernel, dW by the wgrad combine -- on the weight-gradient side stream when one is
        # active (ops/streams.py), overlapped with the data-gradient chain as in the bf16 step
        gw, gg, gb = _lib.grad_slot(weight), _lib.grad_slot(gamma), _lib.grad_slot(beta)
        gw = gw if gw is not None and gw.dtype == _F32 and gw.is_contiguous(memory_format=torch.channels_last) \
            else None
        bn_slots = gg is not None and gb is not None and gg.dtype == _F32 and gb.dtype == _F32
        d3, dgamma, dbeta = bn_backward(z, dy, mean, invstd, gamma, beta, relu, planes=True,
                                        dgamma=gg if bn_slots else None, dbeta=gb if bn_slots else None)
        if d3.dtype == _F32:  # Co not a multiple of 8: fp32 dZ, split here
            d3, _ = split_act(d3)
        if gw is not None:
            dw = streams.run(lambda: conv_wgrad(d3, x3, cp, weight.shape, stride, padding, dst=gw), d3, x3)
        else:
            dw = conv_wgrad(d3, x3, cp, weight.shape, stride, padding)
        dx = None
        if need_dx and ctx.needs_input_grad[0]:
            join = ctx.join
            pend = join.take() if join is not None else None  # another consumer's parked dX: add into it
            wt3 = wt_cache.x3_planes_t(weight)
            if wt3 is None:
                wt3 = split_weight_t(weight)
            dx = conv_dgrad(d3, wt3, weight.shape[0], x_shape, weight.shape, stride, padding, accum=pend)
            if join is not None:
                dx = join.settle(dx)
            streams.keep(dx)  # may be consumed on another (branch) stream
        _lib.report_inplace((weight, gamma, beta), (dw, dgamma, dbeta))
        return dx, dw, dgamma, dbeta, None, None, None, None, None, None, None, None, None, None


_LAST_PLANES = [None]


def conv_bn_act(x, weight, gamma, beta, rmean, rvar, stride=1, padding=0, training=True, momentum=0.1, eps=1e-3,
                relu=True, slot=None, planes_only=False):
    """``planes_only``: the output feeds only other x3 convs -- it comes back as a shape-only tensor whose
    operand planes split_act finds cached on it (never read as fp32: no pool, concat or loss may take it)."""
    _LAST_PLANES[0] = None
    y = _ConvBNActX3Fn.apply(x, weight, gamma, beta, rmean, rvar, stride, padding, training, momentum, eps, relu,
                             slot, planes_only)
    planes = _LAST_PLANES[0]
    if planes is not None:
        _LAST_PLANES[0] = None
        y._tony_x3 = (y._version, planes, weight.shape[0])
    return y


# ---- the fused 1x1 head of an Inception block (ops/fused.py FusedHead) on x3 planes -------------------
def _o(t: torch.Tensor, elems: int) -> int:
    return t.data_ptr() + elems * t.element_size()


class _HeadX3Fn(torch.autograd.Function):
    """FusedHead in fp32: every 1x1 conv that reads the block input as ONE x3 GEMM (N = sum of the splits
    + the pool branch's width) with the BN statistics in its epilogue; per split a BN apply that writes
    either the fp32 output (a concat slot) or only the operand planes of the next conv; the pool branch
    pooled after its 1x1 (they commute) on pool_ch channels instead of Cin.  Backward: every split's BN
    backward writes its slice of ONE [M, 3 * Ctot] dZ plane tensor (tony_bn_bwd_apply_f32_x3p; the pool
    branch through the self-adjoint box filter, tony_avgpool3_s1p1_x3p), then one x3 dgrad (K = 3 Ctot,
    no per-branch accumulation into dX) and one fused x3 wgrad.  Against the textbook graph's 3-4 head
    convs: one dgrad writing the Cin-wide fp32 dX once instead of 3-4 read-modify-write passes, no box
    filter over Cin fp32 channels in either direction, and 3-4x fewer launches."""

    @staticmethod
    def forward(ctx, x, weight, gamma, beta, rmean, rvar, splits, npool, training, momentum, eps, slots, planes):
        L = _lib.lib()
        dev = x.device
        st = _lib.stream_ptr(dev)
        x3, cp = split_act(x)
        w3 = wt_cache.x3_planes(weight)
        if w3 is None:
            w3 = split_weight(weight)
        ctot = weight.shape[0]
        stats = zeros_f32(_lib.stat_floats(ctot), dev) if training else None
        z = conv_fwd(x3, cp, w3, weight.shape, 1, 0, stats)
        n, _, h, w = z.shape
        m = n * h * w
        mean = torch.empty(ctot, dtype=_F32, device=dev)
        invstd = torch.empty(ctot, dtype=_F32, device=dev)
        mode = 0 if training else 1
        ss = 2 * ctot

        def sp(e):  # split statistics: sums at column e, sums of squares at ctot + e (none in inference)
            return (_o(stats, e), _o(stats, ctot + e), ss) if training else (None, None, 0)

        outs, plist = [], []
        c0 = 0
        for k, ci in enumerate(splits):
            slot = slots[k] if slots and k < len(slots) else None
            if planes and k < len(planes) and planes[k] and slot is None:
                y3 = torch.empty((n, h, w, 3 * ci), dtype=_BF16, device=dev).permute(0, 3, 1, 2)
                rc = L.tony_bn_apply_f32_x3(_o(z, c0), m, ci, ctot, y3.data_ptr(), 3 * ci, *sp(c0), _o(gamma, c0),
                                            _o(beta, c0), 0, float(eps), 1, mode, _o(mean, c0), _o(invstd, c0),
                                            _o(rmean, c0), _o(rvar, c0), float(momentum), st)
                _lib.check(rc, "tony_bn_apply_f32_x3 (head)")
                plist.append((k, y3, ci))
                outs.append(torch.empty_strided((n, ci, h, w), (0, 0, 0, 0), dtype=_F32, device=dev))  # shape only
            else:
                y = concat.take(slot, n, ci, h, w, z)
                if y is None:
                    y = _cl(n, ci, h, w, dev)
                _apply_f32(L, _o(z, c0), m, ci, ctot, y, slot,
                           (*sp(c0), _o(gamma, c0), _o(beta, c0), 0, float(eps), 1, mode, _o(mean, c0),
                            _o(invstd, c0), _o(rmean, c0), _o(rvar, c0), float(momentum), st))
                outs.append(y)
            c0 += ci
        p = None
        if npool:
            p = _cl(n, npool, h, w, dev)
            rc = L.tony_avgpool3_s1p1_f32(_o(z, c0), p.data_ptr(), n, h, w, npool, ctot, npool, st)
            _lib.check(rc, "tony_avgpool3_s1p1_f32 (head)")
            pstats = None
            if training:  # the pool branch's statistics are of the pooled columns
                pstats = zeros_f32(_lib.stat_floats(npool), dev)
                rc = L.tony_bn_stats_f32(p.data_ptr(), m, npool, npool, pstats.data_ptr(), _o(pstats, npool),
                                         2 * npool, st)
                _lib.check(rc, "tony_bn_stats_f32 (head pool)")
            k = len(splits)
            slot = slots[k] if slots and k < len(slots) else None
            y = concat.take(slot, n, npool, h, w, z)
            if y is None:
                y = _cl(n, npool, h, w, dev)
            _apply_f32(L, p.data_ptr(), m, npool, npool, y, slot,
                       (_lib.ptr(pstats), _o(pstats, npool) if training else 0, 2 * npool if training else 0,
                        _o(gamma, c0), _o(beta, c0), 0, float(eps), 1, mode, _o(mean, c0), _o(invstd, c0),
                        _o(rmean, c0), _o(rvar, c0), float(momentum), st))
            outs.append(y)
        ctx.save_for_backward(x3, weight, gamma, beta, z, p, mean, invstd)
        ctx.conf = (cp, tuple(x.shape), tuple(splits), npool, x.requires_grad)
        ctx.join = getattr(x, "_tony_join", None)
        _LAST_HEAD_PLANES[:] = plist
        return tuple(outs)

    @staticmethod
    def backward(ctx, *douts):
        x3, weight, gamma, beta, z, p, mean, invstd = ctx.saved_tensors
        cp, x_shape, splits, npool, need_dx = ctx.conf
        L = _lib.lib()
        dev = z.device
        st = _lib.stream_ptr(dev)
        n, ctot, h, w = z.shape
        m = n * h * w
        gw, gg, gb = _lib.grad_slot(weight), _lib.grad_slot(gamma), _lib.grad_slot(beta)
        gw = gw if gw is not None and gw.dtype == _F32 and gw.is_contiguous(memory_format=torch.channels_last) \
            else None
        bn_slots = gg is not None and gb is not None and gg.dtype == _F32 and gb.dtype == _F32
        dgamma = gg if bn_slots else torch.empty(ctot, dtype=_F32, device=dev)
        dbeta = gb if bn_slots else torch.empty(ctot, dtype=_F32, device=dev)
        acc = int(bn_slots)
        d3 = _cl(n, 3 * ctot, h, w, dev, _BF16)  # [hi | lo | hi] planes of dZ, ctot channels each
        dsum = zeros_f32(_lib.stat_floats(ctot), dev)
        ss = 2 * ctot
        c0 = 0
        for k, ci in enumerate(splits):
            dy = douts[k]
            if dy is None:
                dy = torch.zeros((n, ci, h, w), dtype=_F32, device=dev).contiguous(memory_format=torch.channels_last)
            dy, (_, _, lddy) = _as_rows(dy)
            rc = L.tony_bn_bwd_reduce_f32(_o(z, c0), ctot, dy.data_ptr(), lddy, m, ci, _o(mean, c0), _o(invstd, c0),
                                          _o(gamma, c0), _o(beta, c0), 0, 1, _o(dsum, c0), _o(dsum, ctot + c0), ss, st)
            _lib.check(rc, "tony_bn_bwd_reduce_f32 (head)")
            rc = L.tony_bn_bwd_apply_f32_x3p(_o(z, c0), ctot, dy.data_ptr(), lddy, _o(d3, c0), 3 * ctot, ctot, m, ci,
                                             _o(mean, c0), _o(invstd, c0), _o(gamma, c0), _o(beta, c0), 0, 1,
                                             _o(dsum, c0), _o(dsum, ctot + c0), ss, _o(dgamma, c0), _o(dbeta, c0), acc,
                                             st)
            _lib.check(rc, "tony_bn_bwd_apply_f32_x3p (head)")
            c0 += ci
        if npool:
            dy = douts[len(splits)]
            if dy is None:
                dy = torch.zeros((n, npool, h, w), dtype=_F32, device=dev).contiguous(memory_format=torch.channels_last)
            dy, (_, _, lddy) = _as_rows(dy)
            dp = _cl(n, npool, h, w, dev)
            rc = L.tony_bn_bwd_reduce_f32(p.data_ptr(), npool, dy.data_ptr(), lddy, m, npool, _o(mean, c0),
                                          _o(invstd, c0), _o(gamma, c0), _o(beta, c0), 0, 1, _o(dsum, c0),
                                          _o(dsum, ctot + c0), ss, st)
            _lib.check(rc, "tony_bn_bwd_reduce_f32 (head pool)")
            rc = L.tony_bn_bwd_apply_f32(p.data_ptr(), npool, dy.data_ptr(), lddy, dp.data_ptr(), npool, m, npool,
                                         _o(mean, c0), _o(invstd, c0), _o(gamma, c0), _o(beta, c0), 0, 1, _o(dsum, c0),
                                         _o(dsum, ctot + c0), ss, _o(dgamma, c0), _o(dbeta, c0), acc, st)
            _lib.check(rc, "tony_bn_bwd_apply_f32 (head pool)")
            # the pool's input gradient (box3 is self-adjoint) straight into the pool columns of the dZ planes
            rc = L.tony_avgpool3_s1p1_x3p(dp.data_ptr(), _o(d3, c0), n, h, w, npool, npool, 3 * ctot, ctot, st)
            _lib.check(rc, "tony_avgpool3_s1p1_x3p (head pool)")
        wshape = weight.shape
        if gw is not None:
            dw = streams.run(lambda: conv_wgrad(d3, x3, cp, wshape, 1, 0, dst=gw), d3, x3)
        else:
            dw = conv_wgrad(d3, x3, cp, wshape, 1, 0)
        dx = None
        if need_dx and ctx.needs_input_grad[0]:
            join = ctx.join
            pend = join.take() if join is not None else None
            wt3 = wt_cache.x3_planes_t(weight)
            if wt3 is None:
                wt3 = split_weight_t(weight)
            dx = conv_dgrad(d3, wt3, ctot, x_shape, wshape, 1, 0, accum=pend)
            if join is not None:
                dx = join.settle(dx)
            streams.keep(dx)
        _lib.report_inplace((weight, gamma, beta), (dw, None if bn_slots else dgamma, None if bn_slots else dbeta))
        return (dx, dw, None if bn_slots else dgamma, None if bn_slots else dbeta) + (None,) * 9


_LAST_HEAD_PLANES = []


def head(x, weight, gamma, beta, rmean, rvar, splits, npool, training, momentum, eps, slots=None, planes=None):
    """The fp32 FusedHead (ops/fused.py): one output per split (+ the pool branch).  ``planes[k]``: split k
    feeds only x3 convs -- it comes back as a shape-only tensor carrying its operand planes (conv_bn_act
    planes_only); ``slots[k]``: write split k's fp32 output into a block's concat buffer."""
    _LAST_HEAD_PLANES[:] = []
    outs = _HeadX3Fn.apply(x, weight, gamma, beta, rmean, rvar, tuple(splits), int(npool), training, momentum, eps,
                           tuple(slots) if slots else None, tuple(planes) if planes else None)
    for k, y3, ci in _LAST_HEAD_PLANES:
        outs[k]._tony_x3 = (outs[k]._version, y3, ci)
    _LAST_HEAD_PLANES[:] = []
    return outs


# ---- the classifier: an x3 GEMM --------------------------------------------------------------------
class _LinearX3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        n, k = x.shape
        out_f = weight.shape[0]
        x3 = split_rows(x.contiguous(), n, k, k, ACT)
        w3 = split_rows(weight.contiguous(), out_f, k, k, WGT)
        kp = 3 * cp_of(k)
        y = torch.empty((n, out_f), dtype=_F32, device=x.device)
        rc = _lib.lib().tony_gemm_bf16(x3.data_ptr(), w3.data_ptr(), y.data_ptr(), n, out_f, kp, kp, kp, out_f, 8, None,
                                       0, _lib.stream_ptr(x.device))
        _lib.check(rc, "tony_gemm_bf16 (x3 linear)")
        if bias is not None:
            y += bias
        ctx.save_for_backward(x3, weight)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x3, weight = ctx.saved_tensors
        out_f, k = weight.shape
        n = dy.shape[0]
        dev = dy.device
        L, st = _lib.lib(), _lib.stream_ptr(dev)
        dy = dy.contiguous().float()
        d3 = split_rows(dy, n, out_f, out_f, ACT)
        cpo = cp_of(out_f)
        # dX [n, k] = dY [n, out] . W [out, k]: B = W^T planes [k][3 out]
        wt3 = split_rows(weight.t().contiguous(), k, out_f, out_f, WGT)
        dx = torch.empty((n, k), dtype=_F32, device=dev)
        rc = L.tony_gemm_bf16(d3.data_ptr(), wt3.data_ptr(), dx.data_ptr(), n, k, 3 * cpo, 3 * cpo, 3 * cpo, k, 8,
                              None, 0, st)
        _lib.check(rc, "tony_gemm_bf16 (x3 linear dgrad)")
        # dW [out, k] = dY^T X: the three plane products through the split-K TN GEMM
        from .gemm import wgrad_tn

        cpk = cp_of(k)
        acc = torch.zeros(out_f * cpk, dtype=_F32, device=dev)
        for do, xo in ((0, 0), (0, cpk), (cpo, 0)):
            wgrad_tn(d3.data_ptr() + 2 * do, 3 * cpo, x3.data_ptr() + 2 * xo, 3 * cpk, n, out_f, cpk, dev, dst=acc)
        dw = acc.view(out_f, cpk)[:, :k]
        db = dy.sum(0) if ctx.has_bias else None
        return dx, dw, db


class LinearX3(torch.nn.Linear):
    """fp32 nn.Linear whose products run as an x3 bf16 GEMM (the classifier of the fp32 model)."""

    def forward(self, x):
        return _LinearX3Fn.apply(x, self.weight, self.bias)


class ConvBNActX3(torch.nn.Module):
    """Conv2d (no bias) + BatchNorm2d + ReLU, fp32, on the x3 split kernels (same parameters and
    state-dict keys as models/layers.ConvBNAct)."""

    fused = False  # models/layers.conv_bn_act_maxpool: no fused BN + pool kernel on this path
    x3 = True

    def __init__(self, cin, cout, k, stride=1, padding=0, eps=1e-3, momentum=0.1, relu=True):
        super().__init__()
        kk = _pair(k)
        self.conv = torch.nn.Conv2d(cin, cout, kk, stride, padding, bias=False)
        self.bn = torch.nn.BatchNorm2d(cout, eps=eps, momentum=momentum)
        self.relu = relu
        self.is_1x1 = kk == (1, 1) and _pair(stride) == (1, 1) and _pair(padding) == (0, 0)

    def forward(self, x, slot=None, planes_only=False):
        """``slot`` (ops/concat.Slot): write the output into a block's fp32 concat buffer; ``planes_only``:
        the output feeds only other x3 convs (conv_bn_act)."""
        c, bn = self.conv, self.bn
        return conv_bn_act(x, c.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var, c.stride, c.padding,
                           self.training, bn.momentum, bn.eps, self.relu, slot, planes_only)


__all__ = ["ConvBNActX3", "LinearX3", "conv_bn_act", "split_act", "split_weight", "split_weight_t", "cp_of"]
