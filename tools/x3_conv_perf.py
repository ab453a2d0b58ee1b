"""Per-layer speed of the x3 (fp32) conv passes at the step's batch: forward, backward-data and backward-weight
of each distinct Inception-v3 conv shape on the x3 path (ops/x3.py), tuned as in the step, reported as
the bf16-MFMA-equivalent TF/s (three bf16 products per fp32 product) next to the bf16 pass of the same
shape -- what the fp32 row pays per layer over the bf16 step.

usage: python tools/x3_conv_perf.py [--batch 128] [--iters 10] [--top 20]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    from conv_bench import collect_shapes

    from tony_amd.ops import conv as tc
    from tony_amd.ops import tune, x3

    dev = torch.device("cuda", 0)
    shapes = collect_shapes("inception_v3", a.batch)
    rows = []
    for (n, c, h, w, co, k, st, p), cnt in shapes.items():
        if c < 8 or c % 8:
            continue  # the image stem has its own kernels
        torch.manual_seed(0)
        x = torch.randn(n, c, h, w, device=dev).contiguous(memory_format=torch.channels_last)
        wt = torch.randn(co, c, *k, device=dev) / (c * k[0] * k[1]) ** 0.5
        x3p, cp = x3.split_act(x)
        w3 = x3.split_weight(wt)
        z = x3.conv_fwd(x3p, cp, w3, wt.shape, st, p)
        d3, _ = x3.split_act(torch.randn_like(z).contiguous(memory_format=torch.channels_last))
        wtt = x3.split_weight_t(wt)
        fwd = tune.time_ms(lambda: x3.conv_fwd(x3p, cp, w3, wt.shape, st, p), a.iters)
        dgr = tune.time_ms(lambda: x3.conv_dgrad(d3, wtt, co, x.shape, wt.shape, st, p), a.iters)
        wgr = tune.time_ms(lambda: x3.conv_wgrad(d3, x3p, cp, wt.shape, st, p), a.iters)
        xb, wb = x.to(torch.bfloat16), wt.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        stats = None
        bf = tune.time_ms(lambda: tc.conv_fwd(xb, wb, st, p, stats), a.iters)
        oh, ow = z.shape[2], z.shape[3]
        flop = 2.0 * n * oh * ow * co * c * k[0] * k[1]
        tf = lambda ms: 3 * flop / (ms * 1e-3) / 1e12  # noqa: E731
        rows.append((cnt * (fwd + dgr + wgr), f"{n}x{c}x{h}x{w}->{co} k{k[0]}x{k[1]} s{st[0]}", cnt, fwd, dgr, wgr,
                     tf(fwd), tf(dgr), tf(wgr), bf, flop / (bf * 1e-3) / 1e12))
        print(f"{rows[-1][1]:34s} x{cnt}  fwd {fwd * 1e3:7.1f}us ({rows[-1][6]:4.0f}) dgrad {dgr * 1e3:7.1f}us "
              f"({rows[-1][7]:4.0f}) wgrad {wgr * 1e3:7.1f}us ({rows[-1][8]:4.0f} TF/s eq)  | bf16 fwd "
              f"{bf * 1e3:6.1f}us ({rows[-1][10]:4.0f} TF/s)  x3/bf16 fwd {fwd / bf:4.2f}", flush=True)
    tot = sum(r[0] for r in rows)
    print(f"total x3 conv time over the model's conv shapes (x occurrences): {tot:.3f} ms")


if __name__ == "__main__":
    main()
