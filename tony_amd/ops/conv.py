"""NHWC implicit-GEMM convolutions on MFMA (csrc/conv.hip) and the fused conv + BN(+ReLU) layer.

``conv2d(x, weight, stride, padding)`` is a drop-in for ``F.conv2d`` on channels_last bf16 CUDA
tensors with ``Cin % 8 == 0``: forward, backward-data (every stride) and split-K backward-weight
are tony_amd kernels.  Image stems (``Cin < 8``, e.g. the 3-channel Inception-v3 / ResNet-50 first
layers) run forward and backward-weight on the MFMA stem kernels of csrc/stem.hip.

``conv_bn_act(x, weight, bn...)`` fuses the BatchNorm that follows: the forward GEMM epilogue
produces the per-channel sums of its output, so the separate statistics pass over the conv
output disappears; the apply kernel normalises (+ReLU); the backward is the fused BN backward
followed by the dgrad / wgrad GEMMs on dZ.  Parameter gradients are accumulated in place into the
flat gradient buffer when ``_lib.set_inplace_grads`` is on (the trainer's default).

Per-shape selection.  Every (pass, shape) a tony kernel covers runs on it -- including strided
backward-data (one MFMA launch per residue class of dX).  ``TONY_MIOPEN_CANDIDATES=1`` turns MIOpen
into a per-shape autotune candidate (the first eager call times both on the real operands and
caches the faster: A/B studies, test oracle).  Decisions made before a HIP-graph capture are
replayed by the capture; ``choices()`` records every pass, MIOpen ones included.
"""
from __future__ import annotations

import ctypes
import os
import weakref
from typing import Callable, Dict, Tuple

import torch

from . import _lib, concat, streams, tape, tune, wt_cache
from .arena import zeros_f32
from .bn import HOST_MEMO, _accum_ok, _as_rows, _rows_view
from .gemm import occ_choices, splitk_combine, wgrad_cus, wgrad_tn

_BF16 = torch.bfloat16
AUTOTUNE = os.environ.get("TONY_CONV_AUTOTUNE", "1") != "0"
_CHOICE: Dict[Tuple, str] = {}


def _pair(v):
    if type(v) is tuple:
        return v
    return tuple(v) if isinstance(v, (tuple, list)) else (int(v), int(v))


# Image stems (3-channel input) run on the MFMA stem kernels of csrc/stem.hip: forward with the BN
# statistics epilogue and the split-K weight gradient.  TONY_STEM=0 sends them back to MIOpen (A/B).
STEM = os.environ.get("TONY_STEM", "1") != "0"
# Fewest output pixels a conv needs to run on the tony kernels.  Every shape does (1): small-M layers
# (ResNet's 7x7 maps at per-GPU batch 16, the whole-model tests at 64x64) pick their tile variant by
# autotuning like every other shape (64-row variants for few rows), so no conv falls to MIOpen --
# runtime multi-backend dispatch on the hot path.  TONY_CONV_MIN_ROWS=2048 restores the round-2
# MIOpen cutoff for A/B runs.
MIN_ROWS = int(os.environ.get("TONY_CONV_MIN_ROWS", "1"))


_SUP_CACHE: dict = {}


def supported(x: torch.Tensor, weight: torch.Tensor, stride=1, padding=0, dilation=1, groups=1,
              min_rows: int = 0) -> bool:
    """Whether the tony kernels take this conv (``min_rows``: fewest output pixels, default MIN_ROWS)."""
    if not HOST_MEMO:
        return _supported(x, weight, stride, padding, dilation, groups, min_rows)
    key = (x.shape, x.dtype, x.device, weight.shape, weight.dtype, _pair(stride), _pair(padding), _pair(dilation),
           groups, min_rows)
    r = _SUP_CACHE.get(key)
    if r is None:
        if len(_SUP_CACHE) > 4096:
            _SUP_CACHE.clear()
        r = _SUP_CACHE[key] = _supported(x, weight, stride, padding, dilation, groups, min_rows)
    return r


def _supported(x, weight, stride, padding, dilation, groups, min_rows) -> bool:
    if not (x.is_cuda and x.dtype == _BF16 and weight.dtype == _BF16 and x.dim() == 4 and groups == 1
            and _pair(dilation) == (1, 1) and x.shape[1] % 8 == 0 and weight.shape[0] % 8 == 0
            and weight.shape[1] == x.shape[1]):
        return False
    if fullcover(x.shape, weight.shape, stride, padding):
        return True
    oh, ow = out_hw(x.shape[2], x.shape[3], weight.shape[2], weight.shape[3], stride, padding)
    return x.shape[0] * oh * ow >= (min_rows or MIN_ROWS)


def fullcover(x_shape, w_shape, stride=1, padding=0) -> bool:
    """A conv whose filter covers its whole unpadded input -- one output pixel per image, e.g. the
    Inception-v3 aux head's 5x5 conv on a 5x5 map: a plain GEMM over images (``_gemm_*``)."""
    return (_pair(padding) == (0, 0) and tuple(w_shape[2:]) == tuple(x_shape[2:]) and x_shape[1] % 8 == 0
            and w_shape[0] % 8 == 0 and w_shape[1] == x_shape[1])


def stem_supported(x: torch.Tensor, weight: torch.Tensor, stride=1, padding=0, dilation=1, groups=1) -> bool:
    """Whether the MFMA stem kernels (csrc/stem.hip) take this conv: dense NHWC bf16 input with fewer
    than 8 channels (an image), 32 or 64 output channels, padding smaller than the filter."""
    (ph, pw) = _pair(padding)
    return (x.is_cuda and x.dtype == _BF16 and weight.dtype == _BF16 and x.dim() == 4 and groups == 1
            and _pair(dilation) == (1, 1) and 0 < x.shape[1] < 8 and weight.shape[0] in (32, 64)
            and weight.shape[1] == x.shape[1] and ph < weight.shape[2] and pw < weight.shape[3]
            and x.is_contiguous(memory_format=torch.channels_last) and x.numel() < 2 ** 31
            and x.data_ptr() % 16 == 0)


def out_hw(h, w, r, s, stride, padding):
    (sh, sw), (ph, pw) = _pair(stride), _pair(padding)
    return (h + 2 * ph - r) // sh + 1, (w + 2 * pw - s) // sw + 1


def _krsc(weight: torch.Tensor) -> torch.Tensor:
    """[Co, Ci, R, S] -> memory [Co][R][S][Ci] (free for channels_last weights)."""
    w = weight.permute(0, 2, 3, 1)
    return w if w.is_contiguous() else w.contiguous()


def _crsk(weight: torch.Tensor) -> torch.Tensor:
    """[Co, Ci, R, S] -> memory [Ci][R][S][Co] (the dgrad operand)."""
    return weight.permute(1, 2, 3, 0).contiguous()


def _cl_empty(n, c, h, w, device):
    return torch.empty((n, c, h, w), dtype=_BF16, device=device, memory_format=torch.channels_last)


# ---------------------------------------------------------------------------- tony kernels --
def conv_fwd(x: torch.Tensor, weight: torch.Tensor, stride=1, padding=0, stats: torch.Tensor | None = None,
             vflags: int | None = None):
    """Y = conv(x, w); with ``stats`` (zeroed, ``_lib.stat_floats(Cout)`` floats) the epilogue accumulates
    [sum | sumsq] of Y into its STAT_SHARDS copies.  ``vflags``: tile variant bits (None: autotuned)."""
    if HOST_MEMO and vflags is None:  # steady state: the shape's geometry and tuned variant are memoised
        plan = _FWD_PLAN.get((x.shape, x.stride(), x.dtype, x.device, weight.shape, weight.stride(), weight.dtype,
                              stride, padding, stats is not None))
        if plan is not None and x.data_ptr() % 16 == 0:
            n, h, w, C, ldx, co, r, s, sh, sw, ph, pw, oh, ow, vf = plan
            y = _cl_empty(n, co, oh, ow, x.device)
            wk = _krsc(weight)
            rc = _lib.lib().tony_conv_fwd(x.data_ptr(), n, h, w, C, ldx, wk.data_ptr(), co, r, s, sh, sw, ph, pw,
                                          y.data_ptr(), oh, ow, co, (1 if stats is not None else 0) | vf,
                                          _lib.ptr(stats), 2 * co, _lib.stream_ptr(x.device))
            _lib.check(rc, "tony_conv_fwd")
            return y
    if x.shape[1] < 8:  # image stem (csrc/stem.hip)
        return stem_fwd(x, weight, stride, padding, stats)
    key0 = (x.shape, x.stride(), x.dtype, x.device, weight.shape, weight.stride(), weight.dtype, stride, padding,
            stats is not None)
    x, (_, C, ldx) = _as_rows(x)
    n, _, h, w = x.shape
    co, _, r, s = weight.shape
    _lib.check_stat_buffer(stats, co)
    (sh, sw), (ph, pw) = _pair(stride), _pair(padding)
    oh, ow = out_hw(h, w, r, s, stride, padding)
    y = _cl_empty(n, co, oh, ow, x.device)
    wk = _krsc(weight)
    L, st = _lib.lib(), _lib.stream_ptr(x.device)

    def launch(vf, stats_t):
        return L.tony_conv_fwd(x.data_ptr(), n, h, w, C, ldx, wk.data_ptr(), co, r, s, sh, sw, ph, pw, y.data_ptr(),
                               oh, ow, co, (1 if stats_t is not None else 0) | vf, _lib.ptr(stats_t), 2 * co, st)

    if vflags is None:
        key = ("conv_fwd", tuple(x.shape), ldx, tuple(weight.shape), (sh, sw), (ph, pw), stats is not None)
        vflags = tune.cached(key)
        if vflags is None:  # first call of this shape: time the variants (statistics into a scratch buffer)
            scratch = torch.zeros(_lib.stat_floats(co), device=x.device) if stats is not None else None
            vflags = tune.pick(key, lambda vf: launch(vf, scratch), tune.CONV_VARIANTS)
        if (HOST_MEMO and key0[1] == x.stride() and x.dtype == _BF16 and weight.dtype == _BF16
                and not torch.cuda.is_current_stream_capturing()):
            _FWD_PLAN[key0] = (n, h, w, C, ldx, co, r, s, sh, sw, ph, pw, oh, ow, vflags)
    _lib.check(launch(vflags, stats), "tony_conv_fwd")
    return y


# conv_fwd: (x shape / strides / dtype / device, w shape / strides / dtype, stride, padding, stats) -> launch
# geometry.  Everything the geometry or the kernel's operand contract depends on is in the key.
_FWD_PLAN: Dict[Tuple, Tuple] = {}


def stem_fwd(x: torch.Tensor, weight: torch.Tensor, stride=1, padding=0, stats: torch.Tensor | None = None):
    """Forward of an image-stem conv on MFMA (csrc/stem.hip: K = R*S*C padded to 32-deep steps, the
    input rows staged in LDS), optional BN statistics epilogue in the ``conv_fwd`` layout."""
    if not stem_supported(x, weight, stride, padding):
        raise ValueError(f"stem_fwd: unsupported conv x={tuple(x.shape)} w={tuple(weight.shape)}")
    n, c, h, w = x.shape
    co, _, r, s = weight.shape
    _lib.check_stat_buffer(stats, co)
    (sh, sw), (ph, pw) = _pair(stride), _pair(padding)
    oh, ow = out_hw(h, w, r, s, stride, padding)
    y = _cl_empty(n, co, oh, ow, x.device)
    wk = _krsc(weight)
    rc = _lib.lib().tony_stem_fwd(x.data_ptr(), n, h, w, c, wk.data_ptr(), co, r, s, sh, sw, ph, pw, y.data_ptr(),
                                  oh, ow, co, 1 if stats is not None else 0, _lib.ptr(stats),
                                  2 * co if stats is not None else 0, _lib.num_cus(x.device),
                                  _lib.stream_ptr(x.device))
    _lib.check(rc, "tony_stem_fwd")
    return y


def stem_wgrad(dy: torch.Tensor, x: torch.Tensor, weight_shape, stride=1, padding=0, dst=None):
    """dW of an image-stem conv (csrc/stem.hip split-K MFMA kernel + csrc/splitk.hip combine): fp32
    memory [Co][R][S][C] returned as a [Co, C, R, S] view, or added into ``dst`` (a gradient slot in
    that memory order; returns None)."""
    dy, (_, co, lddy) = _as_rows(dy)
    n, c, h, w = x.shape
    _, _, r, s = weight_shape
    (sh, sw), (ph, pw) = _pair(stride), _pair(padding)
    L, dev = _lib.lib(), x.device
    cus = _lib.num_cus(dev)
    nel = co * r * s * c
    slab = torch.empty(2 * cus * nel, dtype=torch.float32, device=dev)
    splits = ctypes.c_int(0)
    st = _lib.stream_ptr(dev)
    rc = L.tony_stem_wgrad(dy.data_ptr(), lddy, x.data_ptr(), n, h, w, c, co, r, s, sh, sw, ph, pw, dy.shape[2],
                           dy.shape[3], slab.data_ptr(), slab.numel(), ctypes.addressof(splits), cus, st)
    _lib.check(rc, "tony_stem_wgrad")
    out = dst if dst is not None else torch.empty(nel, dtype=torch.float32, device=dev)
    rc = L.tony_splitk_reduce(slab.data_ptr(), splits.value, nel, out.data_ptr(), int(out.dtype == _BF16),
                              int(dst is not None), cus, st)
    _lib.check(rc, "tony_splitk_reduce")
    return None if dst is not None else out.view(co, r, s, c).permute(0, 3, 1, 2)


# strided backward-data residue classes on the LDS-DMA tile variants (csrc/igemm.h BTaps); =0: only the
# register-staged NT variants 0-8 (A/B)
STRIDED_GLDS = os.environ.get("TONY_STRIDED_GLDS", "1") != "0"


def dgrad_supported(x_shape, weight: torch.Tensor, stride=1, padding=0) -> bool:
    """Whether a tony kernel computes this conv's input gradient (every stride <= 4, Cin % 8 == 0)."""
    (sh, sw), (ph, pw) = _pair(stride), _pair(padding)
    r, s = weight.shape[2], weight.shape[3]
    return x_shape[1] % 8 == 0 and 1 <= sh <= 4 and 1 <= sw <= 4 and 0 <= ph < r and 0 <= pw < s


def conv_dgrad(dy: torch.Tensor, weight: torch.Tensor, x_shape, stride=1, padding=0,
               vflags: int | None = None, bnr: "_lib.BnRed | None" = None,
               accum: torch.Tensor | None = None) -> torch.Tensor:
    """dX of conv(x, w): stride 1 is one implicit-GEMM transposed conv; a strided conv is one
    launch per residue class of dX (csrc/conv.hip tony_conv_dgrad_strided, no MIOpen).  With ``bnr``
    the epilogue also accumulates the BN-backward reduction of the layer whose output x is
    (``bnr.done`` tells whether the chosen kernel did).  ``accum``: a bf16 channels_last gradient of
    x's shape (dense rows) that dX is added into by the epilogue (flag bit 4) and returned -- the
    separate add kernel of a tensor with two consumers (ResNet's identity path, ops/residual.py)."""
    if not dgrad_supported(x_shape, weight, stride, padding):
        raise ValueError(f"conv_dgrad: unsupported x={tuple(x_shape)} w={tuple(weight.shape)} stride={stride} "
                         f"padding={padding}")
    n, c, h, w = x_shape
    co, _, r, s = weight.shape
    dy, (_, _, lddy) = _as_rows(dy)
    (sh, sw), (ph, pw) = _pair(stride), _pair(padding)
    dx = _cl_empty(n, c, h, w, dy.device)
    wt = wt_cache.transposed(weight)
    L, st = _lib.lib(), _lib.stream_ptr(dy.device)

    if (sh, sw) == (1, 1):
        def launch(vf, br=None):
            return L.tony_conv_dgrad(dy.data_ptr(), n, dy.shape[2], dy.shape[3], co, lddy, wt.data_ptr(), c, r, s, ph,
                                     pw, dx.data_ptr(), h, w, c, vf, None if br is None else ctypes.addressof(br), st)
        name = "tony_conv_dgrad"
    else:
        def launch(vf, br=None):
            if (vf >> 8) & 0xff in (9, 10, tune.BAND_CODE):  # the halo / direct / band variants are stride-1 only
                return -3
            if not STRIDED_GLDS and (vf >> 8) & 0xff >= 11:  # A/B: the register-staged NT kernel only
                return -3
            return L.tony_conv_dgrad_strided(dy.data_ptr(), n, dy.shape[2], dy.shape[3], co, lddy, wt.data_ptr(), c,
                                             r, s, sh, sw, ph, pw, dx.data_ptr(), h, w, c, vf,
                                             None if br is None else ctypes.addressof(br), st)
        name = "tony_conv_dgrad_strided"

    # variants are timed without the fused reduction (it must run exactly once)
    vf = vflags if vflags is not None else tune.pick(("conv_dgrad", tuple(dy.shape), lddy, tuple(weight.shape),
                                                         (sh, sw), (ph, pw)), launch, tune.CONV_VARIANTS)
    if accum is not None and bnr is None and _accum_ok(accum, x_shape):
        plain = dx
        dx = accum
        rc = launch(vf | 16)
        if rc == 0:
            return dx
        if rc != -3:  # -3: the chosen tile variant has its own epilogue (halo / direct): add after
            _lib.check(rc, name)
        dx = plain
        _lib.check(launch(vf), name)
        accum.add_(dx)
        return accum
    _lib.check(launch(vf, bnr), name)
    if accum is not None:
        accum.add_(dx)
        return accum
    return dx



class BnCtx:
    """What a consumer's backward-data kernel needs to fuse layer L's BN-backward reduction
    (csrc/conv.hip BnRed): L's BN input Z and its batch statistics / affine.  Attached by
    ``_ConvBNActFn.forward`` to its output (``_tony_bnr``) and picked up by the conv that consumes it."""
    __slots__ = ("Z", "ldz", "mean", "invstd", "gamma", "beta", "pb", "relu", "C", "__weakref__")

    def __init__(self, Z, ldz, mean, invstd, gamma, beta, pb, relu):
        self.Z, self.ldz, self.mean, self.invstd = Z, ldz, mean, invstd
        self.gamma, self.beta, self.pb, self.relu, self.C = gamma, beta, pb, int(relu), Z.shape[1]


# TONY_BN_FUSED_REDUCE = 1 (every eligible layer) | 0 (never) | auto (default: layers whose Z is at
# least FUSED_REDUCE_MIN_BYTES).  Fusing every eligible layer measured a net loss on MI355X: the
# dgrad epilogues grow by the Z reads + fold, and for the small 35x35 / 17x17 layers the separate
# apply pass loses the warm caches the reduce leaves (Z + dY fit the 256 MB Infinity Cache):
# 15.88 vs 15.60 ms/step (profiles/r2s3_rejected_bn_reduce_in_dgrad_ab.log).  The stem layers' Z
# (85-182 MB, twice that with dY) does not stay cached, so there the fused form saves a full pass.
# Measured again with the "auto" threshold + the fused pool backward: 15.34 / 15.05 vs 14.98 / 14.98
# ms/step (profiles/r2s3_rejected_bn_reduce_in_dgrad_ab.log): off by default.
_FR = os.environ.get("TONY_BN_FUSED_REDUCE", "0").lower()
FUSED_REDUCE = _FR != "0"
FUSED_REDUCE_MIN_BYTES = 0 if _FR == "1" else int(os.environ.get("TONY_BN_FUSED_REDUCE_MIN_MB", "64")) << 20
FUSED_REDUCE_HITS = [0]  # BN backward passes that used a dgrad-fused reduction (tests, bench record)
# TONY_POOL_BNRED=1: the stem max-pool backward also reduces the BN-backward sums (one kernel
# instead of two); opt-in, measured no faster end to end (see _FR above)
POOL_BNRED = os.environ.get("TONY_POOL_BNRED", "0") == "1"
# TONY_POOL_BN_GATHER=1: the conv -> BN -> ReLU -> max-pool backward never writes the full-resolution dY:
# the pooled gradient is gathered twice, in the BN reduction (csrc/pool.hip maxpool_bwd_bnred_kernel
# without the store) and in the BN apply (csrc/bn_act.hip bn_bwd_pool_apply_kernel).  Opt-in: it saves
# 3 passes over dY but the gathers are latency-bound -- 161 + 166 us vs 103 (pool backward) + 96
# (reduce) + 107 (apply) at ResNet's 112x112x64 stem, end to end within noise on both models
# (profiles/r3s2_rejected_pool_bn_gather.log)
POOL_BN_GATHER = os.environ.get("TONY_POOL_BN_GATHER", "0") == "1"


def _dgrad_fused_bn(ctx, dy, weight, x_shape, stride, padding):
    """dX of the layer's conv; when its input is the output of a BN layer (``ctx.bnc_in``) the dgrad
    also reduces that layer's BN-backward sums and tags dX with them (``_tony_bnsums``): if autograd
    hands dX unchanged to that layer's backward, it skips its reduce kernel (``_bn_presums``)."""
    bnc = getattr(ctx, "bnc_in", None)
    if (bnc is None or not FUSED_REDUCE or tuple(bnc.Z.shape) != tuple(x_shape)
            or bnc.Z.numel() * bnc.Z.element_size() < FUSED_REDUCE_MIN_BYTES):
        return _dgrad(dy, weight, x_shape, stride, padding)
    sums = zeros_f32(_lib.stat_floats(bnc.C), dy.device)
    br = _lib.BnRed(bnc.Z.data_ptr(), bnc.ldz, bnc.mean.data_ptr(), bnc.invstd.data_ptr(), _lib.ptr(bnc.gamma),
                    _lib.ptr(bnc.beta), bnc.pb, bnc.relu, sums.data_ptr(), 2 * bnc.C, 0)
    dx = _dgrad(dy, weight, x_shape, stride, padding, br)
    if br.done:
        dx._tony_bnsums = (bnc, sums, dx._version)
    return dx


def _bn_presums(ctx, dy):
    """The [dsum | dsumx] a consumer's dgrad reduced for THIS layer, if ``dy`` is exactly that dgrad's
    output (same tensor, never modified: a gradient summed from several consumers does not qualify)."""
    pre = getattr(dy, "_tony_bnsums", None)
    if pre is None or pre[0] is not getattr(ctx, "bnc_self", None) or dy._version != pre[2]:
        return None
    FUSED_REDUCE_HITS[0] += 1
    return pre[1]


# csrc/conv.hip conv_wgrad_direct_kernel: 3x3 stride-1 convs with 32 / 64 channels in and out (the
# 147x147 / 149x149 stem layers); a candidate of the per-shape wgrad choice (TONY_WGRAD_DIRECT=0: never)
WGRAD_DIRECT = os.environ.get("TONY_WGRAD_DIRECT", "1") != "0"


def wgrad_direct_supported(c, co, r, s, sh, sw) -> bool:
    return c in (32, 64) and co in (32, 64) and (r, s) == (3, 3) and (sh, sw) == (1, 1)


def _wgrad_direct(dy, lddy, x, ldx, co, ph, pw, dst=None):
    """dW of a 3x3 stride-1 conv by the direct kernel: [Co][3][3][C] fp32 partials per workgroup,
    summed by tony_splitk_reduce into ``dst`` (added; returns None) or a new fp32 tensor."""
    n, c, h, w = x.shape
    L, dev = _lib.lib(), x.device
    cus = _lib.num_cus(dev)
    nel = co * 9 * c
    slab = torch.empty(2 * cus * nel, dtype=torch.float32, device=dev)
    splits = ctypes.c_int(0)
    st = _lib.stream_ptr(dev)
    rc = L.tony_conv_wgrad_direct(dy.data_ptr(), lddy, x.data_ptr(), n, h, w, c, ldx, co, ph, pw, dy.shape[2],
                                  dy.shape[3], slab.data_ptr(), slab.numel(), ctypes.addressof(splits), cus, st)
    _lib.check(rc, "tony_conv_wgrad_direct")
    out = dst if dst is not None else torch.empty(nel, dtype=torch.float32, device=dev)
    rc = L.tony_splitk_reduce(slab.data_ptr(), splits.value, nel, out.data_ptr(), int(out.dtype == _BF16),
                              int(dst is not None), cus, st)
    _lib.check(rc, "tony_splitk_reduce")
    return None if dst is not None else out


def conv_wgrad(dy: torch.Tensor, x: torch.Tensor, weight_shape, stride=1, padding=0, dst=None,
               impl: str | None = None):
    """fp32 dW with memory [Co][R][S][Ci] (returned as a [Co, Ci, R, S] channels_last view), or, with
    ``dst`` (a gradient slot in [Co][R][S][Ci] memory order), dW added into dst (returns None).

    The M = N*OH*OW reduction is split over ~2 workgroups per CU whose partial dW tiles are stored
    to a slab; the last split of each tile sums them (gemm.splitk_combine) -- no fp32 atomics."""
    dy, (_, co, lddy) = _as_rows(dy)
    x, (_, c, ldx) = _as_rows(x)
    n, _, h, w = x.shape
    _, _, r, s = weight_shape
    (sh, sw), (ph, pw) = _pair(stride), _pair(padding)
    L, dev = _lib.lib(), x.device
    tbm = 32 if co <= 32 else 64 if co <= 64 else 128  # csrc/conv.hip tony_conv_wgrad tile rows
    ntiles = -(-co // tbm) * -(-(r * s * c) // 128)

    def run(occ, dst_=None):
        if occ == "direct":
            return _wgrad_direct(dy, lddy, x, ldx, co, ph, pw, dst_)
        return splitk_combine(
            lambda slab, cap, sp, fc, fd, ff: L.tony_conv_wgrad(
                dy.data_ptr(), lddy, x.data_ptr(), n, h, w, c, ldx, co, r, s, sh, sw, ph, pw, dy.shape[2],
                dy.shape[3], 0, slab, cap, sp, wgrad_cus(dev, occ), fc, fd, ff, _lib.stream_ptr(dev)),
            co * r * s * c, ntiles, dev, dst_, occ)

    choices = occ_choices(n * dy.shape[2] * dy.shape[3])
    if WGRAD_DIRECT and wgrad_direct_supported(c, co, r, s, sh, sw):
        choices = ("direct",) + tuple(choices)
    if impl is not None:  # tests: a fixed path ("direct" or an occupancy)
        occ = impl
    else:
        occ = tune.pick_choice(("wgrad_occ", tuple(dy.shape), lddy, tuple(x.shape), ldx, tuple(weight_shape), sh,
                                sw, ph, pw), choices, run)
    out = run(occ, dst)
    return None if out is None else out.view(co, r, s, c).permute(0, 3, 1, 2)


# ------------------------------------------------------- whole-input filters: plain GEMMs --
def _dense_rows(x: torch.Tensor) -> torch.Tensor:
    """x with every image one contiguous [H*W*C] row (dense channels_last)."""
    x = _as_rows(x)[0]
    return x if _rows_view(x)[2] == x.shape[1] else x.contiguous(memory_format=torch.channels_last)


def _gemm_fwd(x, weight, stats=None):
    """Y[n, co] = X[n, (r, s, c)] . W[co, (r, s, c)]^T on the MFMA NT GEMM (+ BN statistics epilogue)."""
    x = _dense_rows(x)
    n = x.shape[0]
    co = weight.shape[0]
    k = x[0].numel()
    _lib.check_stat_buffer(stats, co)
    wk = _krsc(weight).reshape(co, k)
    y = _cl_empty(n, co, 1, 1, x.device)
    # tuned like every other GEMM: with only n = batch rows (one tile row) the tile variant and the
    # stream-K forms (the K = R*S*C reduction spread over the CUs) decide whether 6 or 256 CUs work
    vf = tune.gemm_flags(x, wk, y, n, co, k, k, stats is not None, tune.SMALL_GEMM_VARIANTS)
    rc = _lib.lib().tony_gemm_bf16(x.data_ptr(), wk.data_ptr(), y.data_ptr(), n, co, k, k, k, co,
                                   (1 if stats is not None else 0) | vf, _lib.ptr(stats),
                                   2 * co if stats is not None else 0, _lib.stream_ptr(x.device))
    _lib.check(rc, "tony_gemm_bf16 (whole-input conv)")
    return y


def _gemm_dgrad(dy, weight, x_shape):
    """dX[n, (r, s, c)] = dY[n, co] . W[co, (r, s, c)] (NT GEMM on the transposed weight)."""
    dy, (_, co, lddy) = _as_rows(dy)
    n, c, h, w = x_shape
    k = c * h * w
    wt = _krsc(weight).reshape(co, k).t().contiguous()  # [(r, s, c)][co]
    dx = _cl_empty(n, c, h, w, dy.device)
    if lddy != co:
        dy = dy.contiguous(memory_format=torch.channels_last)
        lddy = co
    vf = tune.gemm_flags(dy, wt, dx, n, k, co, lddy, False, tune.SMALL_GEMM_VARIANTS)
    rc = _lib.lib().tony_gemm_bf16(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), n, k, co, lddy, co, k, vf, 0, 0,
                                   _lib.stream_ptr(dy.device))
    _lib.check(rc, "tony_gemm_bf16 (whole-input conv dgrad)")
    return dx


def _gemm_wgrad(dy, x, weight_shape, dst=None):
    """dW[co, (r, s, c)] = dY^T X, added into ``dst`` or returned [Co, C, R, S].  The reduction is over
    the batch only (n = 128 rows) and the output is large (Co x R*S*C): an NT GEMM over the transposed
    operands (dW = dY^T . (X^T)^T, K = n) writes each dW element once from one workgroup -- no split-K
    slab, no combine launch -- into the gradient slot directly (epilogue accumulate, fp32 or bf16)."""
    dy, (_, co, lddy) = _as_rows(dy)
    x = _dense_rows(x)
    n = x.shape[0]
    k = x[0].numel()
    if n % 8 == 0 and (dst is None or dst.dtype in (torch.float32, _BF16)):
        dev = x.device
        dyt = torch.as_strided(dy, (co, n), (1, lddy)).contiguous()         # [co][n]
        xt = x.permute(0, 2, 3, 1).reshape(n, k).t().contiguous()           # [(r, s, c)][n] (NHWC memory)
        out = dst if dst is not None else torch.empty(co * k, dtype=torch.float32, device=dev)
        base = (8 if out.dtype == torch.float32 else 0) | (16 if dst is not None else 0)
        scratch = torch.empty(co * k, dtype=_BF16, device=dev)  # the tuner's timing runs write here
        vf = tune.gemm_flags(dyt, xt, scratch, co, k, n, n, False, tune.SMALL_GEMM_VARIANTS)
        L, st = _lib.lib(), _lib.stream_ptr(dev)
        rc = L.tony_gemm_bf16(dyt.data_ptr(), xt.data_ptr(), out.data_ptr(), co, k, n, n, n, k, base | vf, 0, 0, st)
        if rc == -3:  # the tuned variant has no fp32 / accumulating epilogue: the default one has both
            rc = L.tony_gemm_bf16(dyt.data_ptr(), xt.data_ptr(), out.data_ptr(), co, k, n, n, n, k, base, 0, 0, st)
        _lib.check(rc, "tony_gemm_bf16 (whole-input conv wgrad)")
        if dst is not None:
            return None
        _, c, r, s = weight_shape
        return out.view(co, r, s, c).permute(0, 3, 1, 2)
    out = wgrad_tn(dy.data_ptr(), lddy, x.data_ptr(), k, n, co, k, x.device, dst=dst)
    if out is None:
        return None
    _, c, r, s = weight_shape
    return out.view(co, r, s, c).permute(0, 3, 1, 2)


# --------------------------------------------------------------------------------- MIOpen --
def _miopen_fwd(x, weight, stride, padding, stats=None):
    y = torch.nn.functional.conv2d(x, weight, None, _pair(stride), _pair(padding))
    if not y.is_contiguous(memory_format=torch.channels_last):
        y = y.contiguous(memory_format=torch.channels_last)
    if stats is not None:
        M, co, ld = _rows_view(y)
        _lib.check_stat_buffer(stats, co)
        rc = _lib.lib().tony_bn_stats(y.data_ptr(), M, co, ld, stats.data_ptr(), stats.data_ptr() + 4 * co, 2 * co,
                                      _lib.stream_ptr(y.device))
        _lib.check(rc, "tony_bn_stats")
    return y


def _miopen_dgrad(dy, weight, x_shape, stride, padding):
    xs = torch.empty(x_shape, dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
    return torch.ops.aten.convolution_backward(dy, xs, weight, None, _pair(stride), _pair(padding), (1, 1), False,
                                               (0, 0), 1, (True, False, False))[0]


def _miopen_wgrad(dy, x, weight, stride, padding):
    return torch.ops.aten.convolution_backward(dy, x, weight, None, _pair(stride), _pair(padding), (1, 1), False,
                                               (0, 0), 1, (False, True, False))[1]


# ------------------------------------------------------------------------------ selection --
def _time(fn: Callable[[], object], reps: int = 5) -> float:
    return tune.time_ms(fn, reps)


# MIOpen is a per-shape autotune candidate only when TONY_MIOPEN_CANDIDATES=1 (A/B studies and as a
# test oracle); by default every conv pass tony_amd has a kernel for runs on it, and MIOpen serves
# only what has none (recorded as such in choices(), so bench's conv_impl shows every MIOpen use).
MIOPEN_CANDIDATES = os.environ.get("TONY_MIOPEN_CANDIDATES", "0") == "1"


def _choose(key: Tuple, candidates: Dict[str, Callable[[], object]], default: str = "tony",
            weight: Dict[str, float] | None = None) -> str:
    """Fastest candidate for ``key`` (cached); ``weight`` scales a candidate's measured time."""
    c = _CHOICE.get(key)
    if c is not None:
        return c
    if not MIOPEN_CANDIDATES and len(candidates) > 1:
        candidates = {k: v for k, v in candidates.items() if k != "miopen"}
    if not AUTOTUNE or len(candidates) == 1 or torch.cuda.is_current_stream_capturing():
        c = default if default in candidates else next(iter(candidates))
    else:
        times = {name: _time(fn) * (weight or {}).get(name, 1.0) for name, fn in candidates.items()}
        c = min(times, key=times.get)
    _CHOICE[key] = c
    return c


def _record_unsupported(pas: str, x_shape, w_shape, stride, padding) -> None:
    """Count a conv pass no tony kernel takes (MIOpen) in choices()."""
    _CHOICE.setdefault((pas, tuple(x_shape), tuple(w_shape), _pair(stride), _pair(padding)), "miopen")


def choices() -> Dict[Tuple, str]:
    """The per-(pass, shape) implementation decisions made so far (for logs / profiles)."""
    return dict(_CHOICE)


def _fwd(x, weight, stride, padding, stats):
    key = ("fwd", tuple(x.shape), tuple(weight.shape), stride, padding, stats is not None)
    if fullcover(x.shape, weight.shape, stride, padding):
        _CHOICE.setdefault(key, "gemm")
        return _gemm_fwd(x, weight, stats)
    impl = _CHOICE.get(key)
    if impl is None:
        co = weight.shape[0]
        scratch = torch.zeros(_lib.stat_floats(co), dtype=torch.float32, device=x.device) if stats is not None \
            else None
        impl = _choose(key, {"tony": lambda: conv_fwd(x, weight, stride, padding, scratch),
                             "miopen": lambda: _miopen_fwd(x, weight, stride, padding, scratch)})
    return conv_fwd(x, weight, stride, padding, stats) if impl == "tony" else \
        _miopen_fwd(x, weight, stride, padding, stats)


def _dgrad(dy, weight, x_shape, stride, padding, bnr=None, accum=None):
    """dX (``accum``: added into that gradient and returned, see conv_dgrad)."""
    if accum is not None:
        impl = _CHOICE.get(("dgrad", tuple(dy.shape), tuple(weight.shape), stride, padding))
        if impl == "tony":
            return conv_dgrad(dy, weight, x_shape, stride, padding, accum=accum)
        return accum.add_(_dgrad(dy, weight, x_shape, stride, padding))
    key = ("dgrad", tuple(dy.shape), tuple(weight.shape), stride, padding)
    if fullcover(x_shape, weight.shape, stride, padding):
        _CHOICE.setdefault(key, "gemm")
        return _gemm_dgrad(dy, weight, x_shape)
    impl = _CHOICE.get(key)  # steady state: no candidate closures to build
    if impl == "tony":
        return conv_dgrad(dy, weight, x_shape, stride, padding, bnr=bnr)
    if impl == "miopen":
        return _miopen_dgrad(dy, weight, x_shape, stride, padding)
    cands = {"miopen": lambda: _miopen_dgrad(dy, weight, x_shape, stride, padding)}
    if dgrad_supported(x_shape, weight, stride, padding):
        cands["tony"] = lambda: conv_dgrad(dy, weight, x_shape, stride, padding)
    impl = _choose(key, cands)
    return conv_dgrad(dy, weight, x_shape, stride, padding, bnr=bnr) if impl == "tony" else \
        _miopen_dgrad(dy, weight, x_shape, stride, padding)


MIOPEN_WGRAD_WEIGHT = float(os.environ.get("TONY_MIOPEN_WGRAD_WEIGHT", "1.6"))
# TONY_WGRAD_IMPL=tony|miopen pins the weight-gradient implementation (autotuned per shape otherwise)
WGRAD_IMPL = os.environ.get("TONY_WGRAD_IMPL", "")


def _wgrad(dy, x, weight, stride, padding):
    """dW accumulated into the parameter's gradient slot (returns None) or returned for autograd."""
    key = ("wgrad", tuple(dy.shape), tuple(weight.shape), stride, padding)
    impl = _CHOICE.get(key) or WGRAD_IMPL or None
    if fullcover(x.shape, weight.shape, stride, padding):
        impl = "gemm"
        _CHOICE.setdefault(key, impl)
    elif x.shape[1] % 8:  # image stem: the MFMA stem kernel, or MIOpen if it does not take the shape
        impl = "stem" if STEM and stem_supported(x, weight, stride, padding) else "miopen"
        _CHOICE.setdefault(key, impl)
    if impl is None:
        # With the weight gradients on the side stream (ops/streams.py) their GPU time hides behind the
        # data-gradient chain, while MIOpen's costs 3 more launches (output fill, fp32->bf16 cast, add
        # into the slot) and ~40 us of host time each: MIOpen must win by a margin to be picked.
        impl = _choose(key, {"tony": lambda: conv_wgrad(dy, x, weight.shape, stride, padding),
                             "miopen": lambda: _miopen_wgrad(dy, x, weight, stride, padding)},
                       weight={"miopen": MIOPEN_WGRAD_WEIGHT if streams.ENABLED else 1.0})
    gw = _lib.grad_slot(weight)
    if impl == "gemm":
        if gw is not None and gw.is_contiguous(memory_format=torch.channels_last):
            return streams.run(lambda: _gemm_wgrad(dy, x, weight.shape, dst=gw), dy, x)
        return _accumulate_wgrad(weight, _gemm_wgrad(dy, x, weight.shape))
    if impl == "stem":
        if gw is not None and gw.is_contiguous(memory_format=torch.channels_last):
            return streams.run(lambda: stem_wgrad(dy, x, weight.shape, stride, padding, dst=gw), dy, x)
        return _accumulate_wgrad(weight, stem_wgrad(dy, x, weight.shape, stride, padding))
    if impl == "tony":
        if gw is not None and gw.is_contiguous(memory_format=torch.channels_last):
            # summed straight into the slot (on the weight-gradient stream when one is active)
            return streams.run(lambda: conv_wgrad(dy, x, weight.shape, stride, padding, dst=gw), dy, x)
        return _accumulate_wgrad(weight, conv_wgrad(dy, x, weight.shape, stride, padding))
    if gw is None:
        return _miopen_wgrad(dy, x, weight, stride, padding)

    def into_slot():
        gw.add_(_miopen_wgrad(dy, x, weight, stride, padding))

    return streams.run(into_slot, dy, x)


def _accumulate_wgrad(weight, dw32):
    """Add dW (a [Co, Ci, R, S] view of fp32 memory [Co][R][S][Ci]) into the parameter's flat
    gradient slot in place and return None, or return it (bf16) for autograd to accumulate."""
    gw = _lib.grad_slot(weight)
    if gw is None:
        return dw32.to(weight.dtype)
    # same memory order as the slot: channels_last slots (FlatParams keeps conv weights that way)
    # take dW as is; an NCHW-contiguous slot gets an NCHW-ordered copy
    src = dw32 if gw.is_contiguous(memory_format=torch.channels_last) else dw32.contiguous()
    rc = _lib.lib().tony_add_f32(gw.data_ptr(), int(gw.dtype == _BF16), src.data_ptr(), src.numel(),
                                 _lib.stream_ptr(weight.device))
    _lib.check(rc, "tony_add_f32")
    return None


# ------------------------------------------------------------------------------- autograd --
class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride, padding):
        y = _fwd(x, weight, stride, padding, None)
        ctx.save_for_backward(x, weight)
        ctx.params = (weight,)
        ctx.stride, ctx.padding = stride, padding
        ctx.bnc_in = getattr(x, "_tony_bnr", None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy = _as_rows(dy)[0]
        dw = _wgrad(dy, x, weight, ctx.stride, ctx.padding)  # first: overlaps the dgrad on the side stream
        dx = _dgrad_fused_bn(ctx, dy, weight, x.shape, ctx.stride, ctx.padding) if ctx.needs_input_grad[0] else None
        streams.keep(dx)  # may be consumed on another (branch) stream
        _lib.report_inplace(ctx.params, (dw,))
        return dx, dw, None, None


def conv2d(x, weight, stride=1, padding=0):
    if supported(x, weight, stride, padding):
        return tape.apply(_ConvFn, x, weight, _pair(stride), _pair(padding))
    if x.is_cuda:
        _record_unsupported("fwd", x.shape, weight.shape, stride, padding)
    return torch.nn.functional.conv2d(x, weight, None, stride, padding)


class _ConvBNActFn(torch.autograd.Function):
    """Z = conv(x) with BN sums from the GEMM epilogue; y = act(bn(Z)); backward through both."""

    @staticmethod
    def forward(ctx, x, weight, gamma, beta, running_mean, running_var, stride, padding, training, momentum, eps,
                relu, slot=None):
        L = _lib.lib()
        _lib.check_f32_stats(running_mean, running_var)
        dev = x.device
        stream = _lib.stream_ptr(dev)
        co = weight.shape[0]
        stats = zeros_f32(_lib.stat_floats(co), dev) if training else None
        Z = _fwd(x, weight, stride, padding, stats)
        M, _, ldz = _rows_view(Z)
        y = concat.take(slot, *Z.shape, Z)  # write straight into the block's concat buffer (ops/concat.py)
        if y is None:
            y = torch.empty_like(Z)
        _, _, ldy = _rows_view(y)
        pb = int(gamma.dtype == _BF16)
        if training:
            mean = torch.empty(co, dtype=torch.float32, device=dev)
            invstd = torch.empty(co, dtype=torch.float32, device=dev)
        else:
            mean = running_mean
            invstd = torch.rsqrt(running_var.float() + eps)
        rc = L.tony_bn_apply(Z.data_ptr(), M, co, ldz, y.data_ptr(), ldy, _lib.ptr(stats),
                             _lib.ptr(stats) + 4 * co if training else 0, 2 * co if training else 0,
                             gamma.data_ptr(), beta.data_ptr(), pb,
                             float(eps), int(relu), 0 if training else 1, _lib.ptr(mean) if training else 0,
                             _lib.ptr(invstd) if training else 0, _lib.ptr(running_mean), _lib.ptr(running_var),
                             float(momentum), stream)
        _lib.check(rc, "tony_bn_apply")
        ctx.save_for_backward(x, weight, gamma, beta, mean, invstd, Z)
        ctx.params = (weight, gamma, beta)
        ctx.cfg = (stride, padding, relu, pb)
        ctx.bnc_in = getattr(x, "_tony_bnr", None)
        ctx.join = getattr(x, "_tony_join", None)  # ops/residual.py GradJoin: x has a second consumer
        ctx.bnc_self = None
        if training and slot is None:  # a consumer conv's dgrad may reduce this layer's BN backward
            ctx.bnc_self = BnCtx(Z, ldz, mean, invstd, gamma, beta, pb, relu)
            y._tony_bnr = ctx.bnc_self
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, gamma, beta, mean, invstd, Z = ctx.saved_tensors
        dx, dw, dgamma, dbeta = _conv_bn_backward(ctx, x, weight, gamma, beta, mean, invstd, Z, dy)
        return dx, dw, dgamma, dbeta, None, None, None, None, None, None, None, None, None


def _bn_grad_slots(ctx, gamma, beta):
    """(dgamma, dbeta, inplace): the flat-buffer gradient slots when the trainer made them, else new."""
    gg, gb = _lib.grad_slot(ctx.params[1]), _lib.grad_slot(ctx.params[2])
    inplace = gg is not None and gb is not None
    return (gg if inplace else torch.empty_like(gamma)), (gb if inplace else torch.empty_like(beta)), inplace


def _conv_bn_backward(ctx, x, weight, gamma, beta, mean, invstd, Z, dy, presums=None, done=None):
    """BN(+ReLU) backward from Z (the ReLU mask is recomputed from it), then the conv's wgrad (side
    stream when active) and dgrad; parameter gradients go straight into their flat slots.
    ``presums``: the BN reduction already computed by the kernel that produced dy.  ``done``: the BN
    backward already ran (dZ, dgamma, dbeta, inplace), e.g. fused with a max-pool backward."""
    stride, padding, relu, pb = ctx.cfg
    dev = x.device
    if done is not None:
        dZ, dgamma, dbeta, inplace = done
    else:
        M, co, ldz = _rows_view(Z)
        if presums is None:
            presums = _bn_presums(ctx, dy)  # reduced by the consumer's dgrad epilogue
        dy, (_, _, lddy) = _as_rows(dy)
        dZ = torch.empty_like(Z)
        ws = None if presums is not None else zeros_f32(_lib.bn_bwd_ws_floats(co), dev)
        dgamma, dbeta, inplace = _bn_grad_slots(ctx, gamma, beta)
        _lib.bn_bwd(Z, ldz, dy, lddy, dZ, ldz, M, co, mean, invstd, gamma, beta, pb, relu, ws, dgamma, dbeta, inplace,
                    dev, sums=presums)
    dw = _wgrad(dZ, x, weight, stride, padding)  # first: overlaps the dgrad on the side stream
    join = getattr(ctx, "join", None) if ctx.needs_input_grad[0] else None
    pend = join.take() if join is not None else None
    if pend is not None:
        # x's other consumer already wrote its gradient: dX is added into it (ops/residual.py GradJoin)
        dx = _dgrad(dZ, weight, x.shape, stride, padding, accum=pend)
    else:
        dx = _dgrad_fused_bn(ctx, dZ, weight, x.shape, stride, padding) if ctx.needs_input_grad[0] else None
        if join is not None:
            dx = join.settle(dx)  # first of the two: parked for the other consumer
    streams.keep(dx)  # may be consumed on another (branch) stream
    if inplace:
        dgamma = dbeta = None
    _lib.report_inplace(ctx.params, (dw, dgamma, dbeta))  # after the dgrad: the bucket may now be applied
    return dx, dw, dgamma, dbeta


class _ConvBNActPoolFn(torch.autograd.Function):
    """maxpool_KxK/S(relu(bn(conv(x)))) in training: the conv epilogue produces the BN sums and one
    kernel normalises + ReLUs + pools (csrc/bn_act.hip bn_relu_maxpool_kernel), so the
    full-resolution activation is never written or re-read.  Backward: max-pool backward through
    the saved argmax, then the BN + conv backward of _ConvBNActFn."""

    @staticmethod
    def forward(ctx, x, weight, gamma, beta, running_mean, running_var, stride, padding, momentum, eps, k, s, p=0):
        L = _lib.lib()
        _lib.check_f32_stats(running_mean, running_var)
        dev = x.device
        co = weight.shape[0]
        stats = zeros_f32(_lib.stat_floats(co), dev)
        Z = _fwd(x, weight, stride, padding, stats)
        _, _, ldz = _rows_view(Z)
        n, _, h, w = Z.shape
        oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        y = _cl_empty(n, co, oh, ow, dev)
        arg = torch.empty((n, oh, ow, co), dtype=torch.uint8, device=dev)
        mean = torch.empty(co, dtype=torch.float32, device=dev)
        invstd = torch.empty(co, dtype=torch.float32, device=dev)
        pb = int(gamma.dtype == _BF16)
        rc = L.tony_bn_relu_maxpool(Z.data_ptr(), ldz, stats.data_ptr(), stats.data_ptr() + 4 * co, 2 * co,
                                    gamma.data_ptr(), beta.data_ptr(), pb, float(eps), mean.data_ptr(),
                                    invstd.data_ptr(), _lib.ptr(running_mean), _lib.ptr(running_var), float(momentum),
                                    y.data_ptr(), co, arg.data_ptr(), n, h, w, co, k, s, p, _lib.stream_ptr(dev))
        _lib.check(rc, "tony_bn_relu_maxpool")
        ctx.save_for_backward(x, weight, gamma, beta, mean, invstd, Z, arg)
        ctx.params = (weight, gamma, beta)
        ctx.cfg = (stride, padding, True, pb)
        ctx.pool = (k, s, p)
        ctx.bnc_in = getattr(x, "_tony_bnr", None)
        return y

    @staticmethod
    def backward(ctx, dyp):
        x, weight, gamma, beta, mean, invstd, Z, arg = ctx.saved_tensors
        k, s, p = ctx.pool
        n, co, h, w = Z.shape
        dyp, (_, _, lddy) = _as_rows(dyp)
        if POOL_BN_GATHER:
            # the full-resolution dY is never made: the pool backward's gather runs twice, once reducing
            # the BN sums beside Z (no store) and once inside the BN apply that writes dZ
            L, dev = _lib.lib(), Z.device
            _, _, ldz = _rows_view(Z)
            stream = _lib.stream_ptr(dev)
            sums = zeros_f32(_lib.stat_floats(co), dev)
            rc = L.tony_maxpool_bwd_bnred(dyp.data_ptr(), arg.data_ptr(), None, n, h, w, co, k, s, p, lddy, co,
                                          Z.data_ptr(), ldz, mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(),
                                          beta.data_ptr(), ctx.cfg[3], 1, sums.data_ptr(), 2 * co, _lib.num_cus(dev),
                                          stream)
            _lib.check(rc, "tony_maxpool_bwd_bnred")
            dZ = torch.empty_like(Z)
            dgamma, dbeta, inplace = _bn_grad_slots(ctx, gamma, beta)
            rc = L.tony_bn_bwd_pool_apply(dyp.data_ptr(), lddy, arg.data_ptr(), n, h, w, co, k, s, p, Z.data_ptr(), ldz,
                                          dZ.data_ptr(), ldz, mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(),
                                          beta.data_ptr(), ctx.cfg[3], 1, sums.data_ptr(), 2 * co, dgamma.data_ptr(),
                                          dbeta.data_ptr(), int(inplace), stream)
            _lib.check(rc, "tony_bn_bwd_pool_apply")
            dx, dw, dgamma, dbeta = _conv_bn_backward(ctx, x, weight, gamma, beta, mean, invstd, Z, None,
                                                      done=(dZ, dgamma, dbeta, inplace))
            return dx, dw, dgamma, dbeta, None, None, None, None, None, None, None, None, None
        dy = _cl_empty(n, co, h, w, Z.device)
        if not POOL_BNRED:
            rc = _lib.lib().tony_maxpool_bwd(dyp.data_ptr(), arg.data_ptr(), dy.data_ptr(), n, h, w, co, k, s, p, lddy,
                                             co, _lib.stream_ptr(Z.device))
            _lib.check(rc, "tony_maxpool_bwd")
            dx, dw, dgamma, dbeta = _conv_bn_backward(ctx, x, weight, gamma, beta, mean, invstd, Z, dy)
            return dx, dw, dgamma, dbeta, None, None, None, None, None, None, None, None, None
        # the pool backward also reduces the BN backward sums (csrc/pool.hip maxpool_bwd_bnred_kernel):
        # the separate two-pass reduce over Z and dY (354 / 155 MB each at the Inception stem) disappears
        _, _, ldz = _rows_view(Z)
        sums = zeros_f32(_lib.stat_floats(co), Z.device)
        rc = _lib.lib().tony_maxpool_bwd_bnred(dyp.data_ptr(), arg.data_ptr(), dy.data_ptr(), n, h, w, co, k, s, p,
                                               lddy, co, Z.data_ptr(), ldz, mean.data_ptr(), invstd.data_ptr(),
                                               gamma.data_ptr(), beta.data_ptr(), ctx.cfg[3], 1, sums.data_ptr(),
                                               2 * co, _lib.num_cus(Z.device), _lib.stream_ptr(Z.device))
        _lib.check(rc, "tony_maxpool_bwd_bnred")
        dx, dw, dgamma, dbeta = _conv_bn_backward(ctx, x, weight, gamma, beta, mean, invstd, Z, dy, presums=sums)
        return dx, dw, dgamma, dbeta, None, None, None, None, None, None, None, None, None


def conv_bn_act_pool(x, weight, gamma, beta, running_mean, running_var, stride=1, padding=0, momentum=0.1,
                     eps=1e-3, k=3, s=2, pool_padding=0):
    """max_pool2d(relu(batch_norm(conv2d(x))), k, s, pool_padding) in training mode, fused (see
    _ConvBNActPoolFn)."""
    return tape.apply(_ConvBNActPoolFn, x, weight, gamma, beta, running_mean, running_var, _pair(stride), _pair(padding),
                                  momentum, eps, k, s, pool_padding)


def conv_bn_act(x, weight, gamma, beta, running_mean, running_var, stride=1, padding=0, training=True,
                momentum=0.1, eps=1e-3, relu=True, slot=None):
    """relu(bn(conv(x))); with a ``concat.Slot`` the result is written into that channel slice."""
    if supported(x, weight, stride, padding) or (STEM and stem_supported(x, weight, stride, padding)):
        return tape.apply(_ConvBNActFn, x, weight, gamma, beta, running_mean, running_var, _pair(stride), _pair(padding),
                                  training, momentum, eps, relu, slot)
    if x.is_cuda:
        _record_unsupported("fwd", x.shape, weight.shape, stride, padding)
    z = torch.nn.functional.conv2d(x, weight, None, stride, padding)
    y = torch.nn.functional.batch_norm(z, running_mean, running_var, gamma, beta, training, momentum, eps)
    return torch.relu(y) if relu else y


# ------------------------------------------------------------------------------ inference --
_AFF: Dict[int, Tuple] = {}


def folded_bn(gamma, beta, running_mean, running_var, eps) -> torch.Tensor:
    """[scale | shift] fp32 of an inference BatchNorm (y = z * scale + shift), cached per gamma TENSOR
    (keyed by id, but a hit requires the entry's weak references to still be these very tensors: a
    new module's gamma at a recycled id / address never hits an old entry) until any of the four
    tensors changes (version counters)."""
    ver = (beta._version, running_mean._version, running_var._version, gamma._version, float(eps))
    hit = _AFF.get(id(gamma))
    if (hit is not None and hit[0] == ver and hit[2]() is gamma and hit[3]() is beta
            and hit[4]() is running_mean and hit[5]() is running_var):
        return hit[1]
    scale = gamma.float() * torch.rsqrt(running_var.float() + eps)
    aff = torch.cat([scale, beta.float() - running_mean.float() * scale]).contiguous()
    if len(_AFF) > 4096:
        _AFF.clear()
    _AFF[id(gamma)] = (ver, aff, weakref.ref(gamma), weakref.ref(beta), weakref.ref(running_mean),
                       weakref.ref(running_var))
    return aff


def conv_bn_act_infer(x, weight, gamma, beta, running_mean, running_var, stride=1, padding=0, eps=1e-3,
                      relu=True, slot=None):
    """Inference conv + BatchNorm(running statistics) + ReLU in ONE kernel: the
    BN folds into a per-channel scale / shift applied to the fp32 accumulators in the MFMA epilogue
    (implicit-GEMM conv, or the NT GEMM for 1x1 / stride-1 convs), so the activation is written once
    and never re-read.  No autograd (call under ``torch.no_grad()``); with a ``concat.Slot`` the
    output goes straight into the block's concat buffer."""
    x, (M, C, ldx) = _as_rows(x)
    n, _, h, w = x.shape
    co, _, r, s = weight.shape
    (sh, sw), (ph, pw) = _pair(stride), _pair(padding)
    oh, ow = out_hw(h, w, r, s, stride, padding)
    aff = folded_bn(gamma, beta, running_mean, running_var, eps)
    y = concat.take(slot, n, co, oh, ow, x)
    if y is None:
        y = _cl_empty(n, co, oh, ow, x.device)
    _, _, ldy = _rows_view(y)
    L, st = _lib.lib(), _lib.stream_ptr(x.device)
    epi = 2 | (4 if relu else 0)
    wk = _krsc(weight)
    if (r, s, sh, sw, ph, pw) == (1, 1, 1, 1, 0, 0):
        rc = L.tony_gemm_bf16(x.data_ptr(), wk.data_ptr(), y.data_ptr(), M, co, C, ldx, C, ldy, epi,
                              aff.data_ptr(), 0, st)
        _lib.check(rc, "tony_gemm_bf16 (folded BN)")
        return y
    rc = L.tony_conv_fwd(x.data_ptr(), n, h, w, C, ldx, wk.data_ptr(), co, r, s, sh, sw, ph, pw, y.data_ptr(), oh,
                         ow, ldy, epi, aff.data_ptr(), 0, st)
    _lib.check(rc, "tony_conv_fwd (folded BN)")
    return y

