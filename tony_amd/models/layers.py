"""Building blocks shared by the reference models (NHWC / channels_last, bf16).

``ConvBNAct`` is the unit every CNN in tony_amd is made of: a bias-free conv
(MIOpen implicit GEMM, or the tony_amd MFMA GEMM for 1x1/stride-1 convs) followed
by the fused BN(+ReLU) HIP kernel.  ``fused=False`` builds the stock
nn.BatchNorm2d + nn.ReLU pair instead; it exists only as the comparator for the
"stock PyTorch-ROCm" baseline column and for CPU tests.
"""
from __future__ import annotations

import torch
from torch import nn

import os

from ..ops import conv as conv_ops
from ..ops import tape
from ..ops.bn import BatchNormAct2d
from ..ops.fused import _HeadFn

# TONY_CONV=miopen keeps the spatial convs on MIOpen (A/B comparisons); default: tony_amd's kernels
USE_TONY_CONV = os.environ.get("TONY_CONV", "tony").lower() != "miopen"


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


class ConvBNAct(nn.Module):
    def __init__(self, cin, cout, kernel_size, stride=1, padding=0, eps=1e-3, relu=True, fused=True,
                 momentum=0.1):
        super().__init__()
        k = _pair(kernel_size)
        s = _pair(stride)
        p = _pair(padding)
        self.conv = nn.Conv2d(cin, cout, k, s, p, bias=False)
        self.is_1x1 = k == (1, 1) and s == (1, 1) and p == (0, 0)
        self.fused = fused
        if fused:
            self.bn = BatchNormAct2d(cout, eps=eps, momentum=momentum, relu=relu)
        else:
            self.bn = nn.BatchNorm2d(cout, eps=eps, momentum=momentum)
            self.act = nn.ReLU(inplace=True) if relu else nn.Identity()

    # training hot path: the route (fused head / implicit-GEMM conv + BN) and the op's arguments are
    # resolved once per input layout (~6 us of support checks and module attribute lookups per call,
    # ~94 layers per Inception step); _apply (to / cuda / cast_model replace buffers) drops them
    _ROUTE_HEAD, _ROUTE_CONV = 1, 2

    def _apply(self, fn, *a, **k):
        self.__dict__.pop("_routes", None)
        return super()._apply(fn, *a, **k)

    def _route(self, x):
        c, bn = self.conv, self.bn
        if self.is_1x1 and bn.relu:
            return (self._ROUTE_HEAD, (c.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                       (c.out_channels,), 0))
        if USE_TONY_CONV and (conv_ops.supported(x, c.weight, c.stride, c.padding)
                              or (conv_ops.STEM and conv_ops.stem_supported(x, c.weight, c.stride, c.padding))):
            return (self._ROUTE_CONV, (c.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                       conv_ops._pair(c.stride), conv_ops._pair(c.padding)))
        return None

    def forward(self, x, slot=None):
        """``slot`` (ops/concat.Slot): write the output into a block's concat buffer when the fused
        kernels run (ignored on the stock / CPU path, where the block copies it in)."""
        if self.training and self.fused and x.is_cuda:
            routes = self.__dict__.get("_routes")
            if routes is None:
                routes = self.__dict__["_routes"] = {}
            key = (x.shape, x.stride(), x.dtype, x.data_ptr() % 16 == 0)
            r = routes.get(key, routes)
            if r is routes:
                r = routes[key] = self._route(x)
            if r is not None:
                bn = self.bn
                if r[0] == self._ROUTE_HEAD:
                    return tape.apply(_HeadFn, x, *r[1], True, bn.momentum, bn.eps,
                                      (slot,) if slot is not None else None)[0]
                return tape.apply(conv_ops._ConvBNActFn, x, *r[1], True, bn.momentum, bn.eps, bn.relu, slot)
        if (self.fused and x.is_cuda and not self.training and not torch.is_grad_enabled()
                and conv_ops.supported(x, self.conv.weight, self.conv.stride, self.conv.padding, min_rows=1)
                and (self.is_1x1 or USE_TONY_CONV)):
            # inference: BN folded into the conv's MFMA epilogue, one kernel per layer (ops/conv.py)
            bn, c = self.bn, self.conv
            return conv_ops.conv_bn_act_infer(x, c.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                              c.stride, c.padding, bn.eps, bn.relu, slot)
        if self.fused and self.is_1x1 and self.bn.relu and x.is_cuda:
            # MFMA GEMM with BN statistics in its epilogue + fused apply (ops/fused.py)
            bn = self.bn
            return tape.apply(_HeadFn, x, self.conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                 (self.conv.out_channels,), 0, self.training, bn.momentum, bn.eps,
                                 (slot,) if slot is not None else None)[0]
        if self.fused and x.is_cuda and USE_TONY_CONV and (
                conv_ops.supported(x, self.conv.weight, self.conv.stride, self.conv.padding)
                or (conv_ops.STEM and conv_ops.stem_supported(x, self.conv.weight, self.conv.stride,
                                                              self.conv.padding))):
            # implicit-GEMM conv with BN statistics in its epilogue + fused apply (ops/conv.py)
            bn, c = self.bn, self.conv
            return conv_ops.conv_bn_act(x, c.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var, c.stride,
                                        c.padding, self.training, bn.momentum, bn.eps, bn.relu, slot)
        if self.fused and x.is_cuda:
            conv_ops._record_unsupported("fwd", x.shape, self.conv.weight.shape, self.conv.stride, self.conv.padding)
        y = self.conv(x)
        if self.fused:
            return self.bn(y)
        return self.act(self.bn(y))


def conv_bn_act_maxpool(layer: "ConvBNAct", x, k: int = 3, s: int = 2, padding: int = 0):
    """max_pool(layer(x), k, s, padding); in fused training on the tony conv path (implicit GEMM, or the
    MFMA image stem) one kernel does BN + ReLU + pool, so the full-resolution activation is never
    materialised (ops/conv.py conv_bn_act_pool) -- Inception's stem pools and ResNet's 7x7 stem + 3x3/2 p1
    pool alike."""
    from ..ops.pool import max_pool

    c, bn = layer.conv, layer.bn
    if (layer.fused and layer.training and x.is_cuda and bn.relu and not layer.is_1x1 and USE_TONY_CONV
            and (torch.is_grad_enabled() or tape.recording())
            and (conv_ops.supported(x, c.weight, c.stride, c.padding)
                 or (conv_ops.STEM and conv_ops.stem_supported(x, c.weight, c.stride, c.padding)))):
        return conv_ops.conv_bn_act_pool(x, c.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var, c.stride,
                                         c.padding, bn.momentum, bn.eps, k, s, padding)
    y = layer(x)
    tony_pool = layer.fused or getattr(layer, "x3", False)
    return max_pool(y, k, s, padding=padding) if tony_pool else nn.functional.max_pool2d(y, k, s, padding)


def cast_model(model: nn.Module, dtype: torch.dtype, device=None) -> nn.Module:
    """``model.to(device, dtype)`` that keeps BatchNorm running statistics (and the batch
    counter) in fp32: the fused BN kernels accumulate them in fp32, in place."""
    if device is not None:
        model.to(device)
    for m in model.modules():
        for name, p in m.named_parameters(recurse=False):
            if p.is_floating_point():
                p.data = p.data.to(dtype)
        if isinstance(m, nn.modules.batchnorm._BatchNorm):
            continue
        for name, b in m.named_buffers(recurse=False):
            if b.is_floating_point():
                setattr(m, name, b.to(dtype))
    return model


def init_weights(model: nn.Module, seed: int = 0):
    """Deterministic random init (truncated-normal-ish convs, zero biases)."""
    g = torch.Generator().manual_seed(seed)
    for m in model.modules():
        if isinstance(m, (nn.Conv2d, nn.Linear)):
            fan_in = m.weight[0].numel()
            std = (2.0 / fan_in) ** 0.5 if isinstance(m, nn.Conv2d) else 0.01
            with torch.no_grad():
                m.weight.copy_(torch.randn(m.weight.shape, generator=g).clamp_(-2, 2) * std)
                if m.bias is not None:
                    m.bias.zero_()
        elif isinstance(m, nn.BatchNorm2d):
            with torch.no_grad():
                m.weight.fill_(1.0)
                m.bias.zero_()
    return model
