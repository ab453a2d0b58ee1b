#!/usr/bin/env python3
"""A short program for hardware-counter passes (rocprofv3 --pmc): runs a handful of tony_amd's hot
kernels on Inception-v3 shapes (batch 128), 5 launches each, with nothing else on the GPU.

  rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES ... --kernel-trace -d out -- python3 tools/pmc_probe.py

Kernels: implicit-GEMM conv forward (35x35 64->96 3x3), LDS-DMA wgrad (17x17 192->192 1x7),
1x1 GEMM with BN-statistics epilogue (35x35 288->64... as the fused head), BN backward, halo 3x3.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    from tony_amd.ops import _lib
    from tony_amd.ops.conv import conv_dgrad, conv_fwd, conv_wgrad

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)

    def nhwc(t):
        return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    cases = {
        "conv_fwd_35x35_64to96_3x3": (128, 64, 35, 35, 96, (3, 3), (1, 1)),
        "conv_wgrad_17x17_192to192_1x7": (128, 192, 17, 17, 192, (1, 7), (0, 3)),
        "conv_halo_147x147_32to64_3x3": (128, 32, 147, 147, 64, (3, 3), (1, 1)),
    }
    for name, (n, ci, h, w, co, k, p) in cases.items():
        x = nhwc(torch.randn(n, ci, h, w, device=dev))
        wt = nhwc(torch.randn(co, ci, *k, device=dev) / (ci * k[0] * k[1]) ** 0.5)
        stats = torch.zeros(_lib.stat_floats(co), device=dev)
        for _ in range(5):
            if name.startswith("conv_fwd"):
                stats.zero_()
                conv_fwd(x, wt, 1, p, stats, vflags=0)
            elif name.startswith("conv_wgrad"):
                dy = nhwc(torch.randn(n, co, h, w, device=dev)) if _ == 0 else dy
                conv_wgrad(dy, x, wt.shape, 1, p)
            else:
                stats.zero_()
                conv_fwd(x, wt, 1, p, stats, vflags=9 << 8)
        torch.cuda.synchronize()
        print(f"pmc_probe: {name} done", flush=True)
    # BN backward (fused BN+ReLU of a 35x35x288 activation)
    from tony_amd.ops.bn import bn_act

    z = nhwc(torch.randn(128, 288, 35, 35, device=dev)).requires_grad_(True)
    g = torch.nn.Parameter(torch.ones(288, device=dev))
    b = torch.nn.Parameter(torch.zeros(288, device=dev))
    rm, rv = torch.zeros(288, device=dev), torch.ones(288, device=dev)
    for _ in range(5):
        y = bn_act(z, g, b, rm, rv, True, 0.1, 1e-3, True)
        y.backward(torch.ones_like(y))
    torch.cuda.synchronize()
    print("pmc_probe: bn fwd/bwd done", flush=True)
    _ = conv_dgrad
    return 0


if __name__ == "__main__":
    sys.exit(main())
