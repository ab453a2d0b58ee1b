#!/usr/bin/env python3
"""Per-layer numerics of the x3 (fp32) conv + BN + ReLU at a small batch: every Inception-v3 conv shape,
ConvBNActX3 forward / backward twice against a float64 PyTorch reference of the same layer (conv, training
BatchNorm, ReLU), and stock fp32 PyTorch against the same reference.

Two float64 references: with its own ReLU mask, and through the x3 run's mask (y > 0 of the x3 output).
The x3 forward is ~4e-6 from float64 (hi*hi + hi*lo + lo*hi products), so wherever |y| is that small the
mask bit can differ, and each flipped element moves dbeta / dX / dW by a whole dy: ~1e-3 per layer against
the own-mask reference (stock fp32, ~1e-7 from float64, flips almost none).  Through the same mask the
x3 gradients are pinned at ~1e-5 -- the kernels' own precision, what tests/test_x3_gpu.py asserts.
Flags layers whose same-mask error exceeds --tol.

usage: python tools/x3_layer_check.py [--batch 2] [--tol 1e-4] [--only 8x8]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    return float((a.double() - b.double()).norm() / (b.double().norm() + 1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--tol", type=float, default=1e-4)
    ap.add_argument("--only", default="", help="substring filter on the shape string")
    a = ap.parse_args()
    from conv_bench import collect_shapes  # noqa: E402 (tools/ on the path)

    from tony_amd.ops.x3 import ConvBNActX3

    dev = torch.device("cuda", 0)
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    bad = 0
    for (n, cin, h, w, cout, k, s, p), _ in collect_shapes("inception_v3", a.batch).items():
        tag = f"{n}x{cin}x{h}x{w}->{cout} k{k[0]}x{k[1]} s{s[0]} p{p[0]},{p[1]}"
        if a.only and a.only not in tag:
            continue
        torch.manual_seed(1)
        m = ConvBNActX3(cin, cout, k, s, p).to(dev).train()
        x = torch.randn(n, cin, h, w, device=dev).contiguous(memory_format=torch.channels_last)
        need_dx = cin > 3  # (the stem's input has no gradient in the model)
        x.requires_grad_(need_dx)
        ref = torch.nn.Sequential(torch.nn.Conv2d(cin, cout, k, s, p, bias=False),
                                  torch.nn.BatchNorm2d(cout, eps=1e-3), torch.nn.ReLU()).double().to(dev).train()
        with torch.no_grad():
            ref[0].weight.copy_(m.conv.weight)
        xr = x.detach().double().requires_grad_(need_dx)
        yr = ref(xr)
        g = torch.randn(yr.shape, device=dev, dtype=torch.float64)
        yr.backward(g)
        own = [xr.grad.clone() if need_dx else yr.new_zeros(1), ref[0].weight.grad.clone(),
               ref[1].bias.grad.clone()]
        outs = []
        for _ in range(2):
            for t in (x, m.conv.weight, m.bn.weight, m.bn.bias):
                t.grad = None
            y = m(x)
            y.backward(g.float().contiguous(memory_format=torch.channels_last))
            torch.cuda.synchronize()
            outs.append([y.detach().clone(), x.grad.clone() if need_dx else y.new_zeros(1), m.conv.weight.grad.clone(),
                         m.bn.weight.grad.clone(), m.bn.bias.grad.clone()])
        # the float64 reference through the x3 run's ReLU mask
        for t in (xr, ref[0].weight, ref[1].weight, ref[1].bias):
            t.grad = None
        mask = (outs[1][0] > 0).double()
        pre = ref[1](ref[0](xr))
        (pre * mask).backward(g)
        want = [yr, xr.grad if need_dx else yr.new_zeros(1), ref[0].weight.grad, ref[1].weight.grad, ref[1].bias.grad]
        errs = [rel(o, r) for o, r in zip(outs[1], want)]
        own_errs = [rel(outs[1][1], own[0]) if need_dx else 0.0, rel(outs[1][2], own[1]), rel(outs[1][4], own[2])]
        # stock PyTorch in fp32 against the same float64 reference: the floor any fp32 implementation sees
        # (a ReLU mask bit flips wherever |y| is below the forward's rounding, and dbeta / dX / dW take it)
        t32 = torch.nn.Sequential(torch.nn.Conv2d(cin, cout, k, s, p, bias=False),
                                  torch.nn.BatchNorm2d(cout, eps=1e-3), torch.nn.ReLU()).to(dev).train()
        with torch.no_grad():
            t32[0].weight.copy_(m.conv.weight)
        x32 = x.detach().clone().requires_grad_(need_dx)
        t32(x32).backward(g.float())
        e32 = [rel(x32.grad, own[0]) if need_dx else 0.0, rel(t32[0].weight.grad, own[1]),
               rel(t32[1].bias.grad, own[2])]
        rerun = max(rel(u, v) for u, v in zip(outs[1], outs[0]))
        flag = max(errs) > a.tol or rerun > a.tol
        bad += flag
        print(f"[{time.strftime('%H:%M:%S')}] {'BAD ' if flag else 'ok  '}{tag:44s} y {errs[0]:.1e} dx {errs[1]:.1e} "
              f"dW {errs[2]:.1e} dg {errs[3]:.1e} db {errs[4]:.1e} rerun {rerun:.1e} | own mask: x3 dx {own_errs[0]:.1e} "
              f"dW {own_errs[1]:.1e} db {own_errs[2]:.1e}, torch fp32 dx {e32[0]:.1e} dW {e32[1]:.1e} db {e32[2]:.1e}",
              flush=True)
    print(f"{bad} layer shapes above {a.tol}")
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
