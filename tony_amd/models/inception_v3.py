"""Inception-v3 (Szegedy et al. 2015), NHWC / bf16, for the TF-PS headline benchmark.

The topology is the standard 299x299 Inception-v3 used by the TF-slim /
tf_cnn_benchmarks job that TonY's paper runs as a parameter-server job
(BASELINE.json config "Inception-v3 TF ParameterServerStrategy"): stem of five
3x3/1x1 convs and two max-pools, 3x Inception-A (35x35), reduction-B,
4x Inception-C with factorised 1x7/7x1 convs (17x17), the auxiliary head,
reduction-D, 2x Inception-E with split 1x3/3x1 branches (8x8), global average
pool, dropout and a 1000-way classifier.  BN epsilon is 1e-3 as in TF.

Every conv is a ``ConvBNAct`` (conv + fused HIP BN+ReLU kernel).  With
``fused=True`` the 1x1 convs that read a block's input -- including the avg-pool
branch's 1x1, commuted in front of the pool -- are one ``FusedHead`` MFMA GEMM
with BN statistics in its epilogue (ops/fused.py).  ``fused=False`` builds the
textbook graph on stock PyTorch ops (the comparator).  Parameter count (with
aux head) is 27,161,264 either way.
"""
from __future__ import annotations

import os

import torch
from torch import nn

from ..ops.concat import Slot, assemble, concat_buffer
from ..ops.dropout import Dropout as TonyDropout
from ..ops.pool import avg_pool, avg_pool3x3_s1, global_avg_pool, max_pool
from ..ops import conv as conv_ops
from ..ops import streams, tape
from ..ops.fused import FusedHead
from ..ops.residual import GradJoin
from ..ops.linear import Linear
from ..ops.x3 import ConvBNActX3, LinearX3, split_act
from .layers import ConvBNAct, conv_bn_act_maxpool, init_weights


# TONY_INCEPTION_JOIN=0: let autograd sum the gradients of tensors with several consumers (A/B)
JOIN = os.environ.get("TONY_INCEPTION_JOIN", "1") != "0"


def _join(t: torch.Tensor, n: int) -> None:
    """``t`` feeds ``n`` join-aware fused ops (convs / heads / max pool): their input gradients meet in one
    tensor, each added by its producer's epilogue (ops/residual.py GradJoin) -- no autograd add kernels.
    fp32 tensors: the x3 model's (ops/x3.py ConvBNActX3 adds in its fp32 dgrad epilogue)."""
    if JOIN and t.is_cuda and t.dtype in (torch.bfloat16, torch.float32) and torch.is_grad_enabled() \
            and t.requires_grad:
        t._tony_join = GradJoin(n)


def _x3_input(x: torch.Tensor) -> None:
    """Split an fp32 block input into its x3 planes once, on the current stream, before the branches fork:
    every branch's first conv reuses them (ops/x3.split_act caches them on x) instead of racing to make
    them on its own branch stream."""
    if x.is_cuda and x.dtype == torch.float32:
        split_act(x)


# TONY_X3_PLANES=0: intra-chain x3 layers hand over the fp32 y (A/B, diagnosis)
X3_PLANES = os.environ.get("TONY_X3_PLANES", "1") != "0"
X3_BLOCKS = os.environ.get("TONY_X3_BLOCKS", "1") != "0"
# TONY_X3_HEADS=0: the fp32 blocks keep the textbook head convs (one x3 conv per branch) instead of the
# fused x3 head (ops/x3.py head: one GEMM, one dgrad, one wgrad per block input)
X3_HEADS = os.environ.get("TONY_X3_HEADS", "1") != "0"


def _inner(m, x):
    """A layer whose output only the next conv of its chain reads: an fp32 x3 layer hands it over as the
    conv operand planes alone (ops/x3.conv_bn_act planes_only: no fp32 y, no split pass)."""
    return m(x, planes_only=True) if (X3_PLANES and isinstance(m, ConvBNActX3)) else m(x)


def _seq_inner(seq, x):
    """An nn.Sequential (or one layer) whose output only convs read (every layer planes-only)."""
    for m in (list(seq) if isinstance(seq, nn.Sequential) else [seq]):
        x = _inner(m, x)
    return x


def _seq(seq, x, slot):
    """Run an nn.Sequential of ConvBNAct whose last layer writes into ``slot``."""
    mods = list(seq) if isinstance(seq, nn.Sequential) else [seq]
    for m in mods[:-1]:
        x = _inner(m, x)
    return mods[-1](x, slot=slot)


def _slots(buf, widths):
    out, c0 = [], 0
    for w in widths:
        out.append(Slot(buf, c0))
        c0 += w
    return out


class _Block(nn.Module):
    """A set of parallel branches whose outputs are concatenated on channels.  ``x3``: the fp32 model
    (ops/x3.py) -- the textbook graph with every conv + BN + ReLU, pool and classifier on the fp32 /
    x3-split kernels."""

    def __init__(self, fused, x3=False):
        super().__init__()
        self.fused = fused and not x3
        self.x3 = x3
        # the fp32 blocks' fast form (concat slots, branch streams, joins); TONY_X3_BLOCKS=0: the torch.cat
        # graph whatever TONY_X3_HEADS says (the fused heads live in the fast form only)
        self.x3_fast = x3 and X3_BLOCKS
        # the fused-head layout (ops/fused.py FusedHead, models/convert.py): the bf16 model and the fp32 one
        self.heads = self.fused or (self.x3_fast and X3_HEADS)

    def avgpool(self, x, planes_only=False):
        """``planes_only``: the x3 pool branch, read by its 1x1 conv only (ops/pool.avg_pool3x3_s1)."""
        if self.fused or self.x3:
            return avg_pool3x3_s1(x, planes_only and self.x3 and X3_PLANES)
        return nn.functional.avg_pool2d(x, 3, 1, 1, count_include_pad=True)

    def maxpool(self, x):
        return max_pool(x, 3, 2) if (self.fused or self.x3) else nn.functional.max_pool2d(x, 3, 2)

    def c(self, cin, cout, k, s=1, p=0):
        if self.x3:
            return ConvBNActX3(cin, cout, k, s, p, eps=1e-3)
        return ConvBNAct(cin, cout, k, s, p, eps=1e-3, fused=self.fused)


class InceptionA(_Block):
    def __init__(self, cin, pool_ch, fused=True, x3=False):
        super().__init__(fused, x3)
        if self.heads:
            # b1 1x1/64, b5 1x1/48, b3 1x1/64 and the pool branch's 1x1 share one GEMM
            self.head = FusedHead(cin, (64, 48, 64), pool_cout=pool_ch)
            self.b5 = self.c(48, 64, 5, p=2)
            self.b3 = nn.Sequential(self.c(64, 96, 3, p=1), self.c(96, 96, 3, p=1))
        else:
            self.b1 = self.c(cin, 64, 1)
            self.b5 = nn.Sequential(self.c(cin, 48, 1), self.c(48, 64, 5, p=2))
            self.b3 = nn.Sequential(self.c(cin, 64, 1), self.c(64, 96, 3, p=1), self.c(96, 96, 3, p=1))
            self.bp = self.c(cin, pool_ch, 1)
        self.out_channels = 64 + 64 + 96 + pool_ch

    def forward(self, x):
        if self.fused:  # every branch writes its slice of one output buffer (ops/concat.py)
            n, _, h, w = x.shape
            buf = concat_buffer(n, self.out_channels, h, w, x)
            s1, s5, s3, sp = _slots(buf, (64, 64, 96, self.out_channels - 224))
            y1, y5, y3, yp = self.head(x, slots=(s1, None, None, sp))
            # the double-3x3 chain on this stream, the 5x5 beside it (ops/streams.py)
            o3, o5 = streams.parallel(lambda: _seq(self.b3, y3, s3), lambda: self.b5(y5, slot=s5))
            streams.keep(y5, y3)
            return assemble(buf, [y1, o5, o3, yp])
        if self.x3_fast and self.heads:  # the x3 head, then the chains on their streams
            n, _, h, w = x.shape
            buf = concat_buffer(n, self.out_channels, h, w, x)
            s1, s5, s3, sp = _slots(buf, (64, 64, 96, self.out_channels - 224))
            y1, y5, y3, yp = self.head(x, slots=(s1, None, None, sp), planes=(False, True, True))
            o3, o5 = streams.parallel(lambda: _seq(self.b3, y3, s3), lambda: self.b5(y5, slot=s5))
            streams.keep(y5, y3)
            return assemble(buf, [y1, o5, o3, yp])
        if self.x3_fast:  # branches on their streams, each writing its slice of one fp32 buffer
            n, _, h, w = x.shape
            buf = concat_buffer(n, self.out_channels, h, w, x)
            s1, s5, s3, sp = _slots(buf, (64, 64, 96, self.out_channels - 224))
            _x3_input(x)
            if self.training:
                _join(x, 4)  # the three 1x1 convs and the pool branch's avg pool
            o3, o1, o5, op = streams.parallel(lambda: _seq(self.b3, x, s3), lambda: self.b1(x, slot=s1),
                                              lambda: _seq(self.b5, x, s5),
                                              lambda: self.bp(self.avgpool(x, planes_only=True), slot=sp))
            streams.keep(x)
            return assemble(buf, [o1, o5, o3, op])
        p = self.avgpool(x)
        return torch.cat([self.b1(x), self.b5(x), self.b3(x), self.bp(p)], 1)


class InceptionB(_Block):  # 35x35 -> 17x17 reduction
    def __init__(self, cin, fused=True, x3=False):
        super().__init__(fused, x3)
        self.b3 = self.c(cin, 384, 3, s=2)
        self.bd = nn.Sequential(self.c(cin, 64, 1), self.c(64, 96, 3, p=1), self.c(96, 96, 3, s=2))
        self.out_channels = 384 + 96 + cin

    def forward(self, x):
        if self.fused:
            n, c, h, w = x.shape
            buf = concat_buffer(n, self.out_channels, (h - 3) // 2 + 1, (w - 3) // 2 + 1, x)
            s3, sd, sp = _slots(buf, (384, 96, c))
            if self.training:
                _join(x, 3)  # the double-3x3 chain's 1x1 head, the 3x3/2 conv, the max pool
            od, o3, op = streams.parallel(lambda: _seq(self.bd, x, sd), lambda: self.b3(x, slot=s3),
                                          lambda: max_pool(x, 3, 2, slot=sp))
            streams.keep(x)
            return assemble(buf, [o3, od, op])
        if self.x3_fast:
            n, c, h, w = x.shape
            buf = concat_buffer(n, self.out_channels, (h - 3) // 2 + 1, (w - 3) // 2 + 1, x)
            s3, sd, sp = _slots(buf, (384, 96, c))
            _x3_input(x)
            if self.training:
                _join(x, 3)  # the double-3x3 chain's 1x1, the 3x3/2 conv, the max pool
            od, o3, op = streams.parallel(lambda: _seq(self.bd, x, sd), lambda: self.b3(x, slot=s3),
                                          lambda: max_pool(x, 3, 2, slot=sp))
            streams.keep(x)
            return assemble(buf, [o3, od, op])
        return torch.cat([self.b3(x), self.bd(x), self.maxpool(x)], 1)


class InceptionC(_Block):  # 17x17 with factorised 7x7
    def __init__(self, cin, c7, fused=True, x3=False):
        super().__init__(fused, x3)
        if self.heads:
            self.head = FusedHead(cin, (192, c7, c7), pool_cout=192)
            self.b7 = nn.Sequential(self.c(c7, c7, (1, 7), p=(0, 3)), self.c(c7, 192, (7, 1), p=(3, 0)))
            self.bd = nn.Sequential(self.c(c7, c7, (7, 1), p=(3, 0)), self.c(c7, c7, (1, 7), p=(0, 3)),
                                    self.c(c7, c7, (7, 1), p=(3, 0)), self.c(c7, 192, (1, 7), p=(0, 3)))
        else:
            self.b1 = self.c(cin, 192, 1)
            self.b7 = nn.Sequential(self.c(cin, c7, 1), self.c(c7, c7, (1, 7), p=(0, 3)),
                                    self.c(c7, 192, (7, 1), p=(3, 0)))
            self.bd = nn.Sequential(self.c(cin, c7, 1), self.c(c7, c7, (7, 1), p=(3, 0)),
                                    self.c(c7, c7, (1, 7), p=(0, 3)), self.c(c7, c7, (7, 1), p=(3, 0)),
                                    self.c(c7, 192, (1, 7), p=(0, 3)))
            self.bp = self.c(cin, 192, 1)
        self.out_channels = 768

    def forward(self, x):
        if self.fused:
            n, _, h, w = x.shape
            buf = concat_buffer(n, 768, h, w, x)
            s1, s7, sd, sp = _slots(buf, (192, 192, 192, 192))
            y1, y7, yd, yp = self.head(x, slots=(s1, None, None, sp))
            od, o7 = streams.parallel(lambda: _seq(self.bd, yd, sd), lambda: _seq(self.b7, y7, s7))
            streams.keep(y7, yd)
            return assemble(buf, [y1, o7, od, yp])
        if self.x3_fast and self.heads:
            n, _, h, w = x.shape
            buf = concat_buffer(n, 768, h, w, x)
            s1, s7, sd, sp = _slots(buf, (192, 192, 192, 192))
            y1, y7, yd, yp = self.head(x, slots=(s1, None, None, sp), planes=(False, True, True))
            od, o7 = streams.parallel(lambda: _seq(self.bd, yd, sd), lambda: _seq(self.b7, y7, s7))
            streams.keep(y7, yd)
            return assemble(buf, [y1, o7, od, yp])
        if self.x3_fast:
            n, _, h, w = x.shape
            buf = concat_buffer(n, 768, h, w, x)
            s1, s7, sd, sp = _slots(buf, (192, 192, 192, 192))
            _x3_input(x)
            if self.training:
                _join(x, 4)  # the three 1x1 convs and the pool branch's avg pool
            od, o7, o1, op = streams.parallel(lambda: _seq(self.bd, x, sd), lambda: _seq(self.b7, x, s7),
                                              lambda: self.b1(x, slot=s1),
                                              lambda: self.bp(self.avgpool(x, planes_only=True), slot=sp))
            streams.keep(x)
            return assemble(buf, [o1, o7, od, op])
        p = self.avgpool(x)
        return torch.cat([self.b1(x), self.b7(x), self.bd(x), self.bp(p)], 1)


class InceptionD(_Block):  # 17x17 -> 8x8 reduction
    def __init__(self, cin, fused=True, x3=False):
        super().__init__(fused, x3)
        if self.heads:
            self.head = FusedHead(cin, (192, 192))
            self.b3 = self.c(192, 320, 3, s=2)
            self.b7 = nn.Sequential(self.c(192, 192, (1, 7), p=(0, 3)), self.c(192, 192, (7, 1), p=(3, 0)),
                                    self.c(192, 192, 3, s=2))
        else:
            self.b3 = nn.Sequential(self.c(cin, 192, 1), self.c(192, 320, 3, s=2))
            self.b7 = nn.Sequential(self.c(cin, 192, 1), self.c(192, 192, (1, 7), p=(0, 3)),
                                    self.c(192, 192, (7, 1), p=(3, 0)), self.c(192, 192, 3, s=2))
        self.out_channels = 320 + 192 + cin

    def forward(self, x):
        if self.fused:
            n, c, h, w = x.shape
            buf = concat_buffer(n, self.out_channels, (h - 3) // 2 + 1, (w - 3) // 2 + 1, x)
            s3, s7, sp = _slots(buf, (320, 192, c))
            if self.training:
                _join(x, 2)  # the fused 1x1 head and the max pool
            t3, t7 = self.head(x)
            o7, o3, op = streams.parallel(lambda: _seq(self.b7, t7, s7), lambda: self.b3(t3, slot=s3),
                                          lambda: max_pool(x, 3, 2, slot=sp))
            streams.keep(x, t3, t7)
            return assemble(buf, [o3, o7, op])
        if self.x3_fast and self.heads:
            n, c, h, w = x.shape
            buf = concat_buffer(n, self.out_channels, (h - 3) // 2 + 1, (w - 3) // 2 + 1, x)
            s3, s7, sp = _slots(buf, (320, 192, c))
            if self.training:
                _join(x, 2)  # the x3 head and the max pool
            t3, t7 = self.head(x, planes=(True, True))
            o7, o3, op = streams.parallel(lambda: _seq(self.b7, t7, s7), lambda: self.b3(t3, slot=s3),
                                          lambda: max_pool(x, 3, 2, slot=sp))
            streams.keep(x, t3, t7)
            return assemble(buf, [o3, o7, op])
        if self.x3_fast:
            n, c, h, w = x.shape
            buf = concat_buffer(n, self.out_channels, (h - 3) // 2 + 1, (w - 3) // 2 + 1, x)
            s3, s7, sp = _slots(buf, (320, 192, c))
            _x3_input(x)
            if self.training:
                _join(x, 3)  # the two 1x1 convs and the max pool
            o7, o3, op = streams.parallel(lambda: _seq(self.b7, x, s7), lambda: _seq(self.b3, x, s3),
                                          lambda: max_pool(x, 3, 2, slot=sp))
            streams.keep(x)
            return assemble(buf, [o3, o7, op])
        return torch.cat([self.b3(x), self.b7(x), self.maxpool(x)], 1)


class InceptionE(_Block):  # 8x8 with split 1x3 / 3x1 branches
    def __init__(self, cin, fused=True, x3=False):
        super().__init__(fused, x3)
        fused = self.heads
        if fused:
            self.head = FusedHead(cin, (320, 384, 448), pool_cout=192)
        else:
            self.b1 = self.c(cin, 320, 1)
            self.b3 = self.c(cin, 384, 1)
            self.bd = nn.Sequential(self.c(cin, 448, 1), self.c(448, 384, 3, p=1))
            self.bp = self.c(cin, 192, 1)
        self.b3a = self.c(384, 384, (1, 3), p=(0, 1))
        self.b3b = self.c(384, 384, (3, 1), p=(1, 0))
        if fused:
            self.bd = self.c(448, 384, 3, p=1)
        self.bda = self.c(384, 384, (1, 3), p=(0, 1))
        self.bdb = self.c(384, 384, (3, 1), p=(1, 0))
        self.out_channels = 2048

    def forward(self, x):
        if self.fused:
            n, _, h, w = x.shape
            buf = concat_buffer(n, 2048, h, w, x)
            s1, sa, sb, sda, sdb, sp = _slots(buf, (320, 384, 384, 384, 384, 192))
            y1, t, d, yp = self.head(x, slots=(s1, None, None, sp))
            if self.training:
                _join(t, 2)  # the 1x3 and 3x1 splits

            def dbl():
                dd = self.bd(d)
                if self.training:
                    _join(dd, 2)
                return self.bda(dd, slot=sda), self.bdb(dd, slot=sdb)

            (oda, odb), oa, ob = streams.parallel(dbl, lambda: self.b3a(t, slot=sa), lambda: self.b3b(t, slot=sb))
            streams.keep(t, d)
            return assemble(buf, [y1, oa, ob, oda, odb, yp])
        elif self.x3_fast and self.heads:
            n, _, h, w = x.shape
            buf = concat_buffer(n, 2048, h, w, x)
            s1, sa, sb, sda, sdb, sp = _slots(buf, (320, 384, 384, 384, 384, 192))
            y1, t, d, yp = self.head(x, slots=(s1, None, None, sp), planes=(False, True, True))
            if self.training:
                _join(t, 2)  # the 1x3 and 3x1 splits

            def dbl():
                dd = _inner(self.bd, d)  # read by the two split convs only: operand planes
                if self.training:
                    _join(dd, 2)
                return self.bda(dd, slot=sda), self.bdb(dd, slot=sdb)

            (oda, odb), oa, ob = streams.parallel(dbl, lambda: self.b3a(t, slot=sa), lambda: self.b3b(t, slot=sb))
            streams.keep(t, d)
            return assemble(buf, [y1, oa, ob, oda, odb, yp])
        elif self.x3_fast:
            n, _, h, w = x.shape
            buf = concat_buffer(n, 2048, h, w, x)
            s1, sa, sb, sda, sdb, sp = _slots(buf, (320, 384, 384, 384, 384, 192))
            _x3_input(x)
            if self.training:
                _join(x, 4)  # the three 1x1 convs and the pool branch's avg pool

            def split(head, a, b, sa_, sb_):
                t = _seq_inner(head, x)  # read by the two split convs only: operand planes
                _x3_input(t)
                if self.training:
                    _join(t, 2)  # the 1x3 and 3x1 splits
                return a(t, slot=sa_), b(t, slot=sb_)

            (oda, odb), (oa, ob), y1, yp = streams.parallel(
                lambda: split(self.bd, self.bda, self.bdb, sda, sdb), lambda: split(self.b3, self.b3a, self.b3b, sa, sb),
                lambda: self.b1(x, slot=s1), lambda: self.bp(self.avgpool(x, planes_only=True), slot=sp))
            streams.keep(x)
            return assemble(buf, [y1, oa, ob, oda, odb, yp])
        else:
            y1 = self.b1(x)
            t = self.b3(x)
            d = self.bd(x)
            yp = self.bp(self.avgpool(x))
        return torch.cat([y1, self.b3a(t), self.b3b(t), self.bda(d), self.bdb(d), yp], 1)


class InceptionAux(_Block):
    def __init__(self, cin, num_classes, fused=True, x3=False):
        super().__init__(fused, x3)
        self.conv0 = self.c(cin, 128, 1)
        self.conv1 = self.c(128, 768, 5)
        self.fc = (LinearX3 if x3 else Linear if self.fused else nn.Linear)(768, num_classes)

    def forward(self, x):
        tony = self.fused or self.x3
        x = avg_pool(x, 5, 3) if tony else nn.functional.avg_pool2d(x, 5, 3)
        x = self.conv1(_inner(self.conv0, x))
        x = global_avg_pool(x) if tony else torch.flatten(nn.functional.adaptive_avg_pool2d(x, 1), 1)
        return self.fc(x)


class InceptionV3(nn.Module):
    def __init__(self, num_classes=1000, aux_logits=True, dropout=0.5, fused=True, x3=False):
        super().__init__()
        fused = fused and not x3
        if x3:
            c = lambda cin, cout, k, s=1, p=0: ConvBNActX3(cin, cout, k, s, p, eps=1e-3)  # noqa: E731
        else:
            c = lambda cin, cout, k, s=1, p=0: ConvBNAct(cin, cout, k, s, p, eps=1e-3, fused=fused)  # noqa: E731
        kw = {"fused": fused, "x3": x3}
        self.stem = nn.ModuleList([c(3, 32, 3, s=2), c(32, 32, 3), c(32, 64, 3, p=1)])
        self.stem2 = nn.ModuleList([c(64, 80, 1), c(80, 192, 3)])
        self.mixed_5 = nn.Sequential(InceptionA(192, 32, **kw), InceptionA(256, 64, **kw), InceptionA(288, 64, **kw))
        self.mixed_6a = InceptionB(288, **kw)
        self.mixed_6 = nn.Sequential(InceptionC(768, 128, **kw), InceptionC(768, 160, **kw),
                                     InceptionC(768, 160, **kw), InceptionC(768, 192, **kw))
        self.aux = InceptionAux(768, num_classes, **kw) if aux_logits else None
        self.mixed_7 = nn.Sequential(InceptionD(768, **kw), InceptionE(1280, **kw), InceptionE(2048, **kw))
        # tony dropout (device-side step counter: fresh masks under plan / graph replay) on the tony paths
        self.dropout = TonyDropout(dropout) if (fused or x3) else nn.Dropout(dropout)
        self.fc = (LinearX3 if x3 else Linear if fused else nn.Linear)(2048, num_classes)
        self.fused = fused
        self.x3 = x3

    def _stem_fwd(self, x):
        # the last conv of each group feeds a 3x3/2 max pool; fused training runs BN + ReLU + pool as
        # one kernel there (models/layers.py conv_bn_act_maxpool)
        for m in self.stem[:-1]:
            x = _inner(m, x)
        x = conv_bn_act_maxpool(self.stem[-1], x, 3, 2)
        for m in self.stem2[:-1]:
            x = _inner(m, x)
        return conv_bn_act_maxpool(self.stem2[-1], x, 3, 2)

    def _segments(self):
        """(callable, params) per tape segment: the stem, then every Inception block (ops/tape.py)."""
        segs = getattr(self, "_tape_segs", None)
        if segs is None:
            stem = (self.stem, self.stem2)
            segs = [(self._stem_fwd, [p for m in stem for p in m.parameters()], [b for m in stem for b in m.buffers()])]
            for blk in (*self.mixed_5, self.mixed_6a, *self.mixed_6):
                segs.append((blk, list(blk.parameters()), list(blk.buffers())))
            tail = [(blk, list(blk.parameters()), list(blk.buffers())) for blk in self.mixed_7]
            segs = self._tape_segs = (segs, tail)
        return segs

    def forward(self, x):
        # tape segments need every op of a block on the tony kernels: the 8x8 convs are at batch >= 32
        if (self.fused and self.training and x.is_cuda and tape.ENABLED and torch.is_grad_enabled()
                and x.shape[0] * 64 >= conv_ops.MIN_ROWS):
            # each block = one autograd node replaying its ops' backward from a tape (ops/tape.py)
            head, tail = self._segments()
            for run, params, bufs in head:
                x = tape.segment(run, x, params, bufs)
            aux = self.aux(x) if self.aux is not None else None
            for run, params, bufs in tail:
                x = tape.segment(run, x, params, bufs)
        else:
            x = self._stem_fwd(x)
            x = self.mixed_6(self.mixed_6a(self.mixed_5(x)))
            aux = self.aux(x) if (self.aux is not None and self.training) else None
            x = self.mixed_7(x)
        if self.fused or self.x3:
            x = global_avg_pool(x)
        else:
            x = torch.flatten(nn.functional.adaptive_avg_pool2d(x, 1), 1)
        logits = self.fc(self.dropout(x))
        return (logits, aux) if aux is not None else logits


def inception_v3(num_classes=1000, aux_logits=True, fused=True, seed=0, precision: str = "bf16") -> InceptionV3:
    """``precision="fp32"``: the fp32 model on the x3-split kernels (ops/x3.py); "bf16": the bf16 model
    (``fused`` picks the tony kernels or the stock comparator)."""
    if precision not in ("bf16", "fp32"):
        raise ValueError(f"precision must be bf16 or fp32, not {precision!r}")
    return init_weights(InceptionV3(num_classes, aux_logits, fused=fused, x3=precision == "fp32"), seed)
