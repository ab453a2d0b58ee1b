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

from ..ops.bn import BatchNormAct2d
from ..ops.linear import Linear
from ..ops.pool import global_avg_pool
from ..ops.residual import GradJoin, bn_add_relu, conv1x1_bn_add_relu
from .layers import ConvBNAct, conv_bn_act_maxpool, init_weights


# TONY_RESNET_JOIN=0: let autograd sum the identity-block input gradients (A/B)
JOIN = os.environ.get("TONY_RESNET_JOIN", "1") != "0"


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
        if self.fused and self.downsample is None and x.is_cuda and JOIN and torch.is_grad_enabled():
            # x feeds conv1 and the identity add: their gradients meet in one tensor (GradJoin), no add
            x._tony_join = GradJoin()
        identity = self.downsample(x) if self.downsample is not None else x
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
