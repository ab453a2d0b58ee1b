#!/usr/bin/env python3
"""A short program for one rocprofv3 --pmc pass over the LDS-DMA implicit-GEMM conv kernel
(igemm.h conv_glds_kernel) on three Inception-v3 shapes at batch 128, 5 launches each, one tile
variant pinned per shape (the autotuner's usual pick), nothing else on the GPU.

  rocprofv3 --pmc <<=8 SQ counters>> --kernel-trace -d out -o run --output-format csv -- python3 tools/pmc_glds.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    from tony_amd.ops import _lib
    from tony_amd.ops.conv import conv_fwd

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)

    def nhwc(t):
        return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    cases = [  # (N, Cin, H, W, Cout, k, pad, variant)
        (128, 64, 35, 35, 96, (3, 3), (1, 1), 12),
        (128, 160, 17, 17, 160, (7, 1), (3, 0), 14),
        (128, 80, 73, 73, 192, (3, 3), (0, 0), 14),
    ]
    for n, ci, h, w, co, k, p, v in cases:
        x = nhwc(torch.randn(n, ci, h, w, device=dev))
        wt = nhwc(torch.randn(co, ci, *k, device=dev) / (ci * k[0] * k[1]) ** 0.5)
        stats = torch.zeros(_lib.stat_floats(co), device=dev)
        for _ in range(5):
            stats.zero_()
            conv_fwd(x, wt, 1, p, stats, vflags=v << 8)
        torch.cuda.synchronize()
    print("ok")
    return 0


if __name__ == "__main__":
    sys.exit(main())
