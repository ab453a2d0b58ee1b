"""Per-layer conv timing for a model's conv shapes (MIOpen via PyTorch), NHWC bf16.

Collects every nn.Conv2d call of the model at the given batch, de-duplicates shapes, and times
forward, backward-data and backward-weight separately with HIP events.  Prints a table sorted by
total time with achieved TFLOP/s, i.e. where MIOpen leaves the MFMA units idle.

usage: python tools/conv_bench.py [--model inception_v3] [--batch 128] [--iters 20] [--find]
"""
import argparse
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def collect_shapes(model_name, batch):
    from tony_amd.models.inception_v3 import inception_v3
    from tony_amd.models.resnet import resnet50

    m = inception_v3(fused=False) if model_name == "inception_v3" else resnet50(fused=False)
    res = 299 if model_name == "inception_v3" else 224
    shapes = collections.Counter()

    def hook(mod, inp, out):
        x = inp[0]
        shapes[(batch, x.shape[1], x.shape[2], x.shape[3], mod.out_channels, mod.kernel_size, mod.stride,
                mod.padding)] += 1

    for mod in m.modules():
        if isinstance(mod, torch.nn.Conv2d):
            mod.register_forward_hook(hook)
    m.train()
    with torch.no_grad():
        m(torch.randn(2, 3, res, res))
    return shapes


def time_ms(fn, iters):
    """GPU time per call: a spin kernel keeps the GPU busy while the host enqueues the calls, so
    Python / ctypes launch overhead is not measured (tony_amd.ops.tune.time_ms)."""
    from tony_amd.ops.tune import time_ms as gpu_time_ms

    return gpu_time_ms(fn, iters)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="inception_v3")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--find", action="store_true")
    ap.add_argument("--json", default=None)
    ap.add_argument("--tony", action="store_true", help="time tony_amd's implicit-GEMM kernels instead")
    ap.add_argument("--skip-1x1", action="store_true")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = a.find
    dev = torch.device("cuda")
    rows = []
    from tony_amd.ops import conv as tc

    for (n, cin, h, w, cout, k, s, p), count in collect_shapes(a.model, a.batch).items():
        if a.skip_1x1 and k == (1, 1):
            continue
        x = torch.randn(n, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = torch.randn(cout, cin, *k, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = torch.nn.functional.conv2d(x, wt, None, s, p)
        dy = torch.randn_like(y)
        oh, ow = y.shape[2], y.shape[3]
        flop = 2.0 * n * oh * ow * cout * cin * k[0] * k[1]
        if a.tony:
            if not tc.supported(x, wt):
                continue
            if tc.fullcover(x.shape, wt.shape, s, p):  # the model's dispatch: whole-input filters are GEMMs
                f = time_ms(lambda: tc._gemm_fwd(x, wt), a.iters)
                d = time_ms(lambda: tc._gemm_dgrad(dy, wt, x.shape), a.iters)
                g = time_ms(lambda: tc._gemm_wgrad(dy, x, wt.shape), a.iters)
            else:
                f = time_ms(lambda: tc.conv_fwd(x, wt, s, p), a.iters)
                d = time_ms(lambda: tc.conv_dgrad(dy, wt, x.shape, s, p), a.iters)
                g = time_ms(lambda: tc.conv_wgrad(dy, x, wt.shape, s, p), a.iters)
        else:
            f = time_ms(lambda: torch.nn.functional.conv2d(x, wt, None, s, p), a.iters)
            d = time_ms(lambda: torch.ops.aten.convolution_backward(dy, x, wt, None, s, p, (1, 1), False, (0, 0),
                                                                    1, (True, False, False)), a.iters)
            g = time_ms(lambda: torch.ops.aten.convolution_backward(dy, x, wt, None, s, p, (1, 1), False, (0, 0),
                                                                    1, (False, True, False)), a.iters)
        rows.append(dict(shape=f"{n}x{cin}x{h}x{w}->{cout} k{k[0]}x{k[1]} s{s[0]} p{p[0]},{p[1]}", count=count,
                         fwd_ms=f, dgrad_ms=d, wgrad_ms=g, total_ms=count * (f + d + g),
                         fwd_tf=flop / f / 1e9, dgrad_tf=flop / d / 1e9, wgrad_tf=flop / g / 1e9))
        del x, wt, y, dy
    rows.sort(key=lambda r: -r["total_ms"])
    tot = sum(r["total_ms"] for r in rows)
    print(f"model {a.model} batch {a.batch} {'tony' if a.tony else 'MIOpen'} find={a.find}: {len(rows)} shapes, "
          f"{tot:.2f} ms/step in convs")
    print("| shape | n | fwd ms (TF/s) | dgrad ms (TF/s) | wgrad ms (TF/s) | total ms |")
    print("|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['shape']} | {r['count']} | {r['fwd_ms']:.3f} ({r['fwd_tf']:.0f}) | {r['dgrad_ms']:.3f} "
              f"({r['dgrad_tf']:.0f}) | {r['wgrad_ms']:.3f} ({r['wgrad_tf']:.0f}) | {r['total_ms']:.3f} |")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
