"""Per-variant timing of the NT GEMM (csrc/gemm.hip: register-staged tiles 1-8, LDS-DMA kernels 11-15
from igemm.h) on the Inception-v3 1x1-conv shapes at batch 128: the fused-head forwards (N = the
concatenated 1x1 outputs of a block) and their backward-data GEMMs.

usage: python tools/gemm_bench.py [--iters 10] [--resnet]   (--resnet: the ResNet-50 bottleneck 1x1s)
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (M, N, K, label)
SHAPES = [(128 * 35 * 35, 176, 192, "Mixed_5b head fwd"), (128 * 35 * 35, 192, 176, "Mixed_5b head dgrad"),
          (128 * 35 * 35, 176, 288, "Mixed_5d head fwd"), (128 * 17 * 17, 768, 768, "Mixed_6c head fwd"),
          (128 * 17 * 17, 768, 768, "Mixed_6c head dgrad"), (128 * 8 * 8, 1344, 1280, "Mixed_7b head fwd"),
          (128 * 8 * 8, 1280, 1344, "Mixed_7b head dgrad"), (128 * 73 * 73, 80, 64, "Conv2d_3b fwd"),
          (128 * 73 * 73, 64, 80, "Conv2d_3b dgrad"), (128 * 8 * 8, 1344, 2048, "Mixed_7c head fwd")]
M1, M2, M3, M4 = 128 * 56 * 56, 128 * 28 * 28, 128 * 14 * 14, 128 * 7 * 7
RESNET = [(M1, 64, 256, "s1 conv1 fwd/conv3 dgrad"), (M1, 64, 64, "s1 b1 conv1 fwd/dgrad"),
          (M1, 256, 64, "s1 conv3 fwd/conv1 dgrad"), (M2, 128, 512, "s2 conv1 fwd"), (M2, 512, 128, "s2 conv3 fwd"),
          (M3, 256, 1024, "s3 conv1 fwd"), (M3, 1024, 256, "s3 conv3 fwd"), (M4, 512, 2048, "s4 conv1 fwd"),
          (M4, 2048, 512, "s4 conv3 fwd")]
VARIANTS = list(range(9)) + list(range(11, 16))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--resnet", action="store_true")
    args = ap.parse_args()
    from tony_amd.ops import _lib, tune

    dev = torch.device("cuda", 0)
    L = _lib.lib()
    st = _lib.stream_ptr(dev)
    for m, n, k, label in (RESNET if args.resnet else SHAPES):
        a = torch.randn(m, k, device=dev).to(torch.bfloat16)
        b = (0.05 * torch.randn(n, k, device=dev)).to(torch.bfloat16)
        c = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        stats = torch.zeros(_lib.stat_floats(n), device=dev)
        flop = 2.0 * m * n * k
        row = []
        for v in VARIANTS:
            def run(v=v):
                return L.tony_gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, k, k, n, 1 | (v << 8),
                                        stats.data_ptr(), 2 * n, st)
            if run() != 0:
                continue
            ms = tune.time_ms(run, args.iters)
            row.append((ms, v))
        best = min(row)
        gbs = 2.0 * (m * k + n * k + m * n) / best[0] / 1e6
        print(f"{label:26s} M={m:7d} N={n:5d} K={k:5d}  best v{best[1]:2d} {best[0] * 1e3:7.1f} us "
              f"({flop / best[0] / 1e9:4.0f} TF/s, {gbs:5.0f} GB/s) | " +
              " ".join(f"v{v}:{ms * 1e3:.0f}" for ms, v in row), flush=True)


if __name__ == "__main__":
    main()
