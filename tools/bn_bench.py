#!/usr/bin/env python3
"""Time the fused BN kernels on every Inception-v3 BN shape (bs128) and report achieved HBM GB/s.

    python tools/bn_bench.py [--batch 128] [--reps 20] [--f32]

--f32: the fp32 step's forms (ops/x3.py): fp32 rows, the apply writing y, the backward apply writing the
x3 dZ planes [hi | lo | hi] (bf16, 3C per row) as the step does.

Shapes come from forward hooks on the stock model (one entry per BN layer, M = N*H*W rows of C
channels).  Per shape: stats (read x), apply (read x, write y), bwd_reduce (read x, dy),
bwd_apply (read x, dy, write dx); the total is the per-step BN cost of the model.
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def bn_shapes(batch):
    from tony_amd.models.inception_v3 import inception_v3

    m = inception_v3(fused=False).train()
    shapes = []

    def hook(mod, inp, out):
        n, c, h, w = inp[0].shape
        shapes.append((batch * h * w, c))

    for mm in m.modules():
        if isinstance(mm, torch.nn.BatchNorm2d):
            mm.register_forward_hook(hook)
    with torch.no_grad():
        m(torch.randn(2, 3, 299, 299))
    return collections.Counter(shapes)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--f32", action="store_true")
    args = ap.parse_args()
    from tony_amd.ops import _lib

    L = _lib.lib()
    dev = torch.device("cuda", 0)
    stream = _lib.stream_ptr(dev)
    shapes = bn_shapes(args.batch)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def tm(fn):
        fn()
        ev0.record()
        for _ in range(args.reps):
            fn()
        ev1.record()
        ev1.synchronize()
        return ev0.elapsed_time(ev1) * 1000.0 / args.reps  # us

    tot = collections.Counter()
    print(f"{'M':>9} {'C':>5} {'n':>3} | {'stats us':>9} {'GB/s':>6} | {'apply us':>9} {'GB/s':>6} | "
          f"{'bred us':>9} {'GB/s':>6} | {'bapp us':>9} {'GB/s':>6}")
    for (M, C), cnt in sorted(shapes.items(), key=lambda kv: -kv[0][0] * kv[0][1]):
        f32 = args.f32
        if f32 and C % 8:
            continue
        dt = torch.float32 if f32 else torch.bfloat16
        x = torch.randn(M, C, device=dev).to(dt)
        dy = torch.randn(M, C, device=dev).to(dt)
        y = torch.empty_like(x)
        d3 = torch.empty(M, 3 * C, device=dev, dtype=torch.bfloat16) if f32 else None
        g = torch.ones(C, device=dev)
        b = torch.zeros(C, device=dev)
        ws = torch.zeros(_lib.stat_floats(C), device=dev)
        ss = 2 * C
        mean = torch.zeros(C, device=dev)
        inv = torch.ones(C, device=dev)
        rm = torch.zeros(C, device=dev)
        rv = torch.ones(C, device=dev)
        B = M * C * x.element_size()
        sfx = "_f32" if f32 else ""
        stats_fn, apply_fn, red_fn = (getattr(L, f"tony_bn_stats{sfx}"), getattr(L, f"tony_bn_apply{sfx}"),
                                      getattr(L, f"tony_bn_bwd_reduce{sfx}"))
        t_s = tm(lambda: stats_fn(x.data_ptr(), M, C, C, ws.data_ptr(), ws.data_ptr() + 4 * C, ss, stream))
        t_a = tm(lambda: apply_fn(x.data_ptr(), M, C, C, y.data_ptr(), C, ws.data_ptr(), ws.data_ptr() + 4 * C,
                                  ss, g.data_ptr(), b.data_ptr(), 0, 1e-3, 1, 0, mean.data_ptr(), inv.data_ptr(),
                                  rm.data_ptr(), rv.data_ptr(), 0.1, stream))
        t_r = tm(lambda: red_fn(x.data_ptr(), C, dy.data_ptr(), C, M, C, mean.data_ptr(),
                                inv.data_ptr(), g.data_ptr(), b.data_ptr(), 0, 1, ws.data_ptr(),
                                ws.data_ptr() + 4 * C, ss, stream))
        if f32:  # the step's backward apply: dZ as its x3 planes
            t_p = tm(lambda: L.tony_bn_bwd_apply_f32_x3(x.data_ptr(), C, dy.data_ptr(), C, d3.data_ptr(), 3 * C, M, C,
                                                        mean.data_ptr(), inv.data_ptr(), g.data_ptr(), b.data_ptr(), 0,
                                                        1, ws.data_ptr(), ws.data_ptr() + 4 * C, ss, 0, 0, 0, stream))
            bp = 2 * B + M * 3 * C * 2
        else:
            t_p = tm(lambda: L.tony_bn_bwd_apply(x.data_ptr(), C, dy.data_ptr(), C, y.data_ptr(), C, M, C,
                                                 mean.data_ptr(), inv.data_ptr(), g.data_ptr(), b.data_ptr(), 0, 1,
                                                 ws.data_ptr(), ws.data_ptr() + 4 * C, ss, 0, 0, 0, stream))
            bp = 3 * B
        print(f"{M:>9} {C:>5} {cnt:>3} | {t_s:9.1f} {B / t_s / 1e3:6.0f} | {t_a:9.1f} {2 * B / t_a / 1e3:6.0f} | "
              f"{t_r:9.1f} {2 * B / t_r / 1e3:6.0f} | {t_p:9.1f} {bp / t_p / 1e3:6.0f}")
        tot["bapp_bytes"] += cnt * bp
        tot["stats"] += cnt * t_s
        tot["apply"] += cnt * t_a
        tot["bwd_reduce"] += cnt * t_r
        tot["bwd_apply"] += cnt * t_p
        tot["bytes"] += cnt * B
        del x, dy, y
    print("per-step totals (us):", {k: round(v, 1) for k, v in tot.items() if "bytes" not in k},
          f"activation bytes {tot['bytes'] / 1e9:.2f} GB")
    gb = tot["bytes"] / 1e3
    print(f"effective GB/s: stats {gb / tot['stats']:.0f}  apply {2 * gb / tot['apply']:.0f}  "
          f"bwd_reduce {2 * gb / tot['bwd_reduce']:.0f}  bwd_apply {tot['bapp_bytes'] / 1e3 / tot['bwd_apply']:.0f}")


if __name__ == "__main__":
    main()
