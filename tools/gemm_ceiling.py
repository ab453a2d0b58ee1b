#!/usr/bin/env python3
"""Calibration of the implicit-GEMM conv kernels against the vendor GEMM library on the same GEMM
shapes: per Inception-v3 conv shape (batch 128) the time of every LDS-DMA tile variant of
tony_conv_fwd (igemm.h 11-24) and of torch.matmul (hipBLASLt) on the equivalent dense GEMM
[M = N*OH*OW, K = R*S*Cin] x [K, Cout] -- the library gets a materialised im2col matrix, i.e. an upper
bound on what a tuned GEMM does with these skinny-N shapes.  Prints TF/s per row.

usage: python tools/gemm_ceiling.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASES = [  # (N, Cin, H, W, Cout, (R, S), (ph, pw))
    (128, 64, 35, 35, 96, (3, 3), (1, 1)),
    (128, 96, 35, 35, 96, (3, 3), (1, 1)),
    (128, 160, 17, 17, 160, (7, 1), (3, 0)),
    (128, 192, 17, 17, 192, (1, 7), (0, 3)),
    (128, 768, 17, 17, 192, (1, 1), (0, 0)),
    (128, 448, 8, 8, 384, (3, 3), (1, 1)),
    (128, 80, 73, 73, 192, (3, 3), (0, 0)),
]


def main() -> int:
    from tony_amd.ops import _lib, tune
    from tony_amd.ops.conv import conv_fwd

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)

    def nhwc(t):
        return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    print("| shape | M x N x K | best tony (variant) | hipBLASLt GEMM | tony / BLAS |")
    print("|---|---|---|---|---|")
    for n, ci, h, w, co, (r, s), (ph, pw) in CASES:
        oh, ow = h + 2 * ph - r + 1, w + 2 * pw - s + 1
        m, k = n * oh * ow, r * s * ci
        flop = 2.0 * m * co * k
        x = nhwc(torch.randn(n, ci, h, w, device=dev))
        wt = nhwc(torch.randn(co, ci, r, s, device=dev) / k ** 0.5)
        stats = torch.zeros(_lib.stat_floats(co), device=dev)
        best = (float("inf"), None)
        per = []
        for v in range(11, 25):
            try:
                t = tune.time_ms(lambda: conv_fwd(x, wt, 1, (ph, pw), stats, vflags=v << 8), 10)
            except Exception:  # noqa: BLE001 - variant does not take the shape
                continue
            per.append(f"{v}:{flop / t / 1e9:.0f}")
            best = min(best, (t, v))
        a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        b = torch.randn(k, co, device=dev, dtype=torch.bfloat16)
        tb = tune.time_ms(lambda: torch.matmul(a, b), 10)
        bt = torch.randn(co, k, device=dev, dtype=torch.bfloat16)
        tbt = tune.time_ms(lambda: torch.matmul(a, bt.t()), 10)
        tb = min(tb, tbt)
        print(f"| {ci}->{co} {r}x{s} {h}x{w} | {m} x {co} x {k} | {best[0] * 1e3:.1f} us "
              f"({flop / best[0] / 1e9:.0f} TF/s, v{best[1]}) | {tb * 1e3:.1f} us ({flop / tb / 1e9:.0f} TF/s) | "
              f"{tb / best[0]:.2f} |")
        print(f"|  per variant TF/s: {' '.join(per)} | | | | |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
