"""ResNet-50 (v1.5) for the horovod-on-tony config (BASELINE.json: "ResNet-50 ring-allreduce bf16
on 8xMI355X"), NHWC / bf16, built from tony_amd's fused ops.

Bottleneck schedule with ``fused=True`` (the default on the GPU):

conv1  1x1 s1      MFMA GEMM with BN statistics in the epilogue + fused BN/ReLU apply
conv2  3x3 s1|s2   tony_amd MFMA implicit GEMM (BN statistics epilogue) -> fused BN+ReLU apply
conv3  1x1 s1      MFMA GEMM (+stats) -> ONE pass: BN apply + identity add + ReLU
                   (ops/residual.py); its backward writes d(conv3 out) and
                   d(identity) in the same pass
downsample         1x1 s1|s2 conv (tony_amd implicit GEMM; strided dgrad per residue class) -> fused BN

Architecture: torchvision's resnet50 (stride on the 3x3, "v1.5"); layer
widths 64/128/256/512 x4, blocks [3, 4, 6, 3], 7x7/s2 stem + 3x3/s2 p1 max pool (fused with the stem's
BN + ReLU in one kernel when training, ops/conv.py conv_bn_act_pool),
global average pool, 1000-way FC (MFMA GEMMs, ops/linear.py).  The 7x7/s2 stem runs on the
MFMA stem kernels (csrc/stem.hip).  ``fused=False`` is the stock PyTorch
module graph (the comparator and the CPU path).
"""
from __future__ import annotations

import os

import torch
from torch import nn

from ..ops import conv as conv_ops
from ..ops.bn import BatchNormAct2d
from ..ops.linear import Linear
from ..ops.pool import global_avg_pool
from ..ops.residual import GradJoin, bn_add_relu, conv1x1_bn_add_relu
from .layers import ConvBNAct, conv_bn_act_maxpool, init_weights


# TONY_RESNET_JOIN=0: let autograd sum the block input gradients (A/B)
JOIN = os.environ.get("TONY_RESNET_JOIN", "1") != "0"
# TONY_RESNET_DS_TONY=0: the projection shortcut as nn.Conv2d (MIOpen) + fused BN (A/B)
DS_TONY = os.environ.get("TONY_RESNET_DS_TONY", "1") != "0"


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1, fused=True, eps=1e-5):
        super().__init__()
        cout = width * self.expansion
        self.fused = fused
        self.conv1 = ConvBNAct(cin, width, 1, fused=fused, eps=eps)
        self.conv2 = ConvBNAct(width, width, 3, stride=stride, padding=1, fused=fused, eps=eps)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout, eps=eps)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(
                nn.Conv2d(cin, cout, 1, stride=stride, bias=False),
                BatchNormAct2d(cout, eps=eps, relu=False) if fused else nn.BatchNorm2d(cout, eps=eps))

    def forward(self, x):
        ds_tony = (self.downsample is not None and self.fused and x.is_cuda and self.training and DS_TONY
                   and conv_ops.supported(x, self.downsample[0].weight, self.downsample[0].stride,
                                          self.downsample[0].padding))
        if (self.fused and x.is_cuda and self.training and JOIN and torch.is_grad_enabled()
                and x.dtype == torch.bfloat16 and (self.downsample is None or ds_tony)):
            # x feeds conv1 and the identity add (or the downsample conv), both join-aware fused ops:
            # their gradients meet in one tensor (GradJoin), no add kernel
            x._tony_join = GradJoin()
        if self.downsample is None:
            identity = x
        elif ds_tony:
            # the projection shortcut on the tony kernels: 1x1/s conv with the BN statistics in its
            # epilogue + BN apply (no ReLU), strided dgrad per residue class -- not MIOpen
            c, bn = self.downsample[0], self.downsample[1]
            identity = conv_ops.conv_bn_act(x, c.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                            c.stride, c.padding, True, bn.momentum, bn.eps, relu=False)
        else:
            identity = self.downsample(x)
        out = self.conv2(self.conv1(x))
        bn = self.bn3
        if self.fused and out.is_cuda:
            return conv1x1_bn_add_relu(out, self.conv3.weight, identity, bn.weight, bn.bias, bn.running_mean,
                                       bn.running_var, self.training, bn.momentum, bn.eps)
        if self.fused:
            return bn_add_relu(self.conv3(out), identity, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                               self.training, bn.momentum, bn.eps)
        return torch.relu(bn(self.conv3(out)) + identity)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, fused=True, eps=1e-5):
        super().__init__()
        self.fused = fused
        self.stem = ConvBNAct(3, 64, 7, stride=2, padding=3, fused=fused, eps=eps)
        blocks = []
        cin = 64
        for i, n in enumerate(layers):
            width = 64 * 2 ** i
            for j in range(n):
                blocks.append(Bottleneck(cin, width, stride=2 if (j == 0 and i > 0) else 1, fused=fused, eps=eps))
                cin = width * Bottleneck.expansion
        self.blocks = nn.Sequential(*blocks)
        self.fc = (Linear if fused else nn.Linear)(cin, num_classes)

    def forward(self, x):
        if self.fused:
            # one kernel: BN + ReLU + 3x3/2 p1 max pool over the stem conv's output (training), the
            # padded tony max pool otherwise -- no stock pooling kernel on the fused path
            x = conv_bn_act_maxpool(self.stem, x, 3, 2, padding=1)
        else:
            x = torch.nn.functional.max_pool2d(self.stem(x), 3, 2, 1)
        x = self.blocks(x)
        x = global_avg_pool(x) if self.fused else x.mean((2, 3))
        return self.fc(x)


def resnet50(num_classes: int = 1000, fused: bool = True, seed: int = 0) -> ResNet:
    m = ResNet((3, 4, 6, 3), num_classes, fused=fused)
    init_weights(m, seed)
    # zero-init the last BN gamma of each block (standard large-batch ResNet recipe)
    for b in m.blocks:
        nn.init.zeros_(b.bn3.weight)
    return m
