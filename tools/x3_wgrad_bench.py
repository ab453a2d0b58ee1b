"""A/B of the x3 (fp32) weight-gradient forms (csrc/conv.hip tony_conv_wgrad_x3) on Inception-v3 layers.

Mode 0: the three plane pairs as split groups of conv_wgrad_glds_kernel; 1 / 2: conv_wgrad_x3f_kernel
(all four planes per K-step) on a 3- / 2-slot LDS ring.  Times x3.conv_wgrad (kernel + split combine).

usage: python tools/x3_wgrad_bench.py [--batch 128] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (C, H, W, Co, (R, S), stride, (ph, pw))
LAYERS = [(192, 17, 17, 192, (1, 7), 1, (0, 3)), (160, 17, 17, 160, (7, 1), 1, (3, 0)),
          (128, 17, 17, 128, (1, 7), 1, (0, 3)), (768, 17, 17, 192, (1, 1), 1, (0, 0)),
          (64, 35, 35, 96, (3, 3), 1, (1, 1)), (96, 35, 35, 96, (3, 3), 1, (1, 1)),
          (288, 35, 35, 384, (3, 3), 2, (0, 0)), (448, 8, 8, 384, (3, 3), 1, (1, 1)),
          (2048, 8, 8, 448, (1, 1), 1, (0, 0)), (80, 73, 73, 192, (3, 3), 1, (0, 0))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from tony_amd.ops import _lib, tune, x3

    dev = torch.device("cuda", 0)
    L = _lib.lib()
    prev = L.tony_x3_wgrad_mode(-1)
    tot = [0.0, 0.0, 0.0]
    print(f"batch {a.batch}: x3.conv_wgrad us per call (pairs / fused ring3 / fused ring2)")
    for c, h, w, co, k, s, p in LAYERS:
        xf = torch.randn(a.batch, c, h, w, device=dev).contiguous(memory_format=torch.channels_last)
        oh, ow = (h + 2 * p[0] - k[0]) // s + 1, (w + 2 * p[1] - k[1]) // s + 1
        dyf = torch.randn(a.batch, co, oh, ow, device=dev).contiguous(memory_format=torch.channels_last)
        xp, cp = x3.split_act(xf)
        dp, _ = x3.split_act(dyf)
        ts = []
        for mode in (0, 1, 2):
            L.tony_x3_wgrad_mode(mode)
            ts.append(tune.time_ms(lambda: x3.conv_wgrad(dp, xp, cp, (co, c) + k, s, p), a.iters))
        for i, t in enumerate(ts):
            tot[i] += t
        flop = 3 * 2.0 * a.batch * oh * ow * co * c * k[0] * k[1]
        print(f"{c:4d}x{h}x{w}->{co:4d} k{k[0]}x{k[1]} s{s}: " +
              " / ".join(f"{t * 1e3:7.1f}" for t in ts) +
              f"   ({flop / (min(ts) * 1e-3) / 1e12:5.0f} TF/s best, ring2 {ts[0] / ts[2]:.2f}x, ring3 {ts[0] / ts[1]:.2f}x)",
              flush=True)
    L.tony_x3_wgrad_mode(prev)
    print("total: " + " / ".join(f"{t * 1e3:.1f}" for t in tot) + " us")


if __name__ == "__main__":
    main()
