"""Per-variant timing of the implicit-GEMM conv kernels on chosen Inception-v3 shapes (NHWC bf16):
forward with the BN-statistics epilogue (as the model runs it) and backward-data, every tile
variant of csrc/mfma_common.h kNtVariants (+ 9 = the halo-tile path), HIP-event timed.

usage: python tools/variant_bench.py [--batch 128] [--shapes stem|all]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (Cin, H, W, Cout, (R, S), stride, (ph, pw))
STEM = [(32, 149, 149, 32, (3, 3), 1, (0, 0)), (32, 147, 147, 64, (3, 3), 1, (1, 1)),
        (80, 73, 73, 192, (3, 3), 1, (0, 0)), (64, 35, 35, 96, (3, 3), 1, (1, 1)),
        (192, 17, 17, 192, (1, 7), 1, (0, 3)), (288, 35, 35, 384, (3, 3), 2, (0, 0))]
# the other heavy Inception-v3 spatial convs (the 1x1s run through gemm.hip)
MIXED = [(96, 35, 35, 96, (3, 3), 1, (1, 1)), (48, 35, 35, 64, (5, 5), 1, (2, 2)),
         (128, 17, 17, 128, (1, 7), 1, (0, 3)), (160, 17, 17, 160, (7, 1), 1, (3, 0)),
         (192, 17, 17, 320, (3, 3), 2, (0, 0)), (384, 8, 8, 384, (1, 3), 1, (0, 1)),
         (448, 8, 8, 384, (3, 3), 1, (1, 1))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", choices=("stem", "mixed", "all"), default="all")
    args = ap.parse_args()
    from tony_amd.ops import _lib, tune
    from tony_amd.ops import conv as C

    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    shapes = {"stem": STEM, "mixed": MIXED, "all": STEM + MIXED}[args.shapes]
    for cin, h, w, co, (r, s), st, pad in shapes:
        x = torch.randn(args.batch, cin, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        wt = (0.05 * torch.randn(co, cin, r, s, device=dev)).to(torch.bfloat16).contiguous(memory_format=cl)
        y = C.conv_fwd(x, wt, st, pad)
        dy = torch.randn_like(y).contiguous(memory_format=cl)
        stats = torch.zeros(_lib.stat_floats(co), device=dev)
        oh, ow = y.shape[2], y.shape[3]
        flop = 2.0 * args.batch * oh * ow * co * cin * r * s
        print(f"{args.batch}x{cin}x{h}x{w}->{co} k{r}x{s} s{st} p{pad}  ({flop / 1e9:.0f} GFLOP)")
        for v in tune.NT_VARIANTS:
            row = []
            for name, fn in (("fwd", lambda: C.conv_fwd(x, wt, st, pad, None, v << 8)),
                             ("fwd+stats", lambda: C.conv_fwd(x, wt, st, pad, stats, v << 8)),
                             ("dgrad", lambda: C.conv_dgrad(dy, wt, x.shape, st, pad, v << 8))):
                try:
                    ms = tune.time_ms(fn, args.iters)
                    row.append(f"{name} {ms * 1000:7.1f} us ({flop / ms / 1e9:4.0f} TF/s)")
                except Exception as e:  # noqa: BLE001 - a variant that does not apply to the shape
                    row.append(f"{name}    n/a ({type(e).__name__})")
            print(f"  v{v}: " + " | ".join(row))


if __name__ == "__main__":
    main()
