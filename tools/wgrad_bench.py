"""Weight-gradient paths of the 3x3 stride-1 32/64-channel convs (Inception stem, ResNet-50 layer1):
the direct kernel (csrc/conv.hip conv_wgrad_direct_kernel) vs the split-K implicit GEMM at each
occupancy, HIP-event timed, the slab combine included.

usage: python tools/wgrad_bench.py [--batch 128]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(32, 149, 149, 32, 0), (32, 147, 147, 64, 1), (64, 56, 56, 64, 1), (64, 35, 35, 64, 1)]
# implicit-GEMM wgrad shapes of Inception-v3 (Cin, H, W, Cout, (R, S), (ph, pw)), stride 1
MIXED = [(64, 35, 35, 96, (3, 3), (1, 1)), (96, 35, 35, 96, (3, 3), (1, 1)), (48, 35, 35, 64, (5, 5), (2, 2)),
         (128, 17, 17, 128, (1, 7), (0, 3)), (160, 17, 17, 160, (7, 1), (3, 0)), (192, 17, 17, 192, (1, 7), (0, 3)),
         (384, 8, 8, 384, (1, 3), (0, 1)), (448, 8, 8, 384, (3, 3), (1, 1)), (80, 73, 73, 192, (3, 3), (0, 0))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    args = ap.parse_args()
    from tony_amd.ops import tune
    from tony_amd.ops.conv import conv_wgrad

    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    for c, h, w, co, p in SHAPES:
        x = torch.randn(args.batch, c, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        oh, ow = h + 2 * p - 2, w + 2 * p - 2
        dy = torch.randn(args.batch, co, oh, ow, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        slot = torch.zeros(co * 9 * c, device=dev)
        flop = 2.0 * args.batch * oh * ow * co * 9 * c
        row = []
        for impl in ("direct", 1, 2, 4):
            ms = tune.time_ms(lambda: conv_wgrad(dy, x, (co, c, 3, 3), 1, p, dst=slot, impl=impl), 5)
            row.append(f"{impl}: {ms * 1e3:6.1f} us ({flop / ms / 1e9:4.0f} TF/s)")
        print(f"{args.batch}x{c}x{h}x{w}->{co} p{p}  " + " | ".join(row), flush=True)


def mixed(batch):
    from tony_amd.ops import tune
    from tony_amd.ops.conv import conv_wgrad

    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    for c, h, w, co, (r, s), (ph, pw) in MIXED:
        x = torch.randn(batch, c, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        oh, ow = h + 2 * ph - r + 1, w + 2 * pw - s + 1
        dy = torch.randn(batch, co, oh, ow, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        slot = torch.zeros(co * r * s * c, device=dev)
        flop = 2.0 * batch * oh * ow * co * r * s * c
        row = []
        for impl in (1, 2, 4):
            ms = tune.time_ms(lambda: conv_wgrad(dy, x, (co, c, r, s), 1, (ph, pw), dst=slot, impl=impl), 5)
            row.append(f"occ {impl}: {ms * 1e3:6.1f} us ({flop / ms / 1e9:4.0f} TF/s)")
        print(f"{batch}x{c}x{h}x{w}->{co} k{r}x{s}  " + " | ".join(row), flush=True)


if __name__ == "__main__":
    if "--mixed" in sys.argv:
        sys.argv.remove("--mixed")
        mixed(128)
        sys.exit(0)
    main()
