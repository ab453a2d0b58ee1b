"""Does a conv kernel's throughput scale with the number of busy CUs?  One LDS-DMA tile variant, one
layer shape, batch 32..512: the grid grows from a fraction of the 256 CUs to several waves of them.
If the time per image stays flat once the grid covers the CUs, the kernel is limited per CU (issue /
latency); if it keeps falling, a partly filled grid is what costs.

usage: python tools/conv_scaling.py [--variant 23] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(192, 17, 17, 192, (1, 7), (0, 3)), (160, 17, 17, 160, (7, 1), (3, 0)), (96, 35, 35, 96, (3, 3), (1, 1)),
          (448, 8, 8, 384, (3, 3), (1, 1))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="23,19,15,11")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from tony_amd.ops import _lib, tune
    from tony_amd.ops import conv as C

    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    for cin, h, w, co, k, p in SHAPES:
        for v in [int(s) for s in a.variants.split(",")]:
            row = []
            for n in (32, 64, 128, 256, 512):
                x = torch.randn(n, cin, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
                wt = (0.05 * torch.randn(co, cin, *k, device=dev)).to(torch.bfloat16).contiguous(memory_format=cl)
                stats = torch.zeros(_lib.stat_floats(co), device=dev)
                try:
                    C.conv_fwd(x, wt, 1, p, stats, v << 8)
                    t = tune.time_ms(lambda: C.conv_fwd(x, wt, 1, p, stats, v << 8), a.iters)
                except Exception as e:  # noqa: BLE001 - variant not applicable
                    row.append(f"n{n}: n/a")
                    continue
                flop = 2.0 * n * h * w * co * cin * k[0] * k[1]  # stride 1, same padding
                row.append(f"n{n} {t * 1e3:6.1f}us {flop / (t * 1e-3) / 1e12:4.0f}TF/s")
            print(f"{cin}x{h}x{w}->{co} k{k[0]}x{k[1]} v{v}: " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
