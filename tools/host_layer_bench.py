#!/usr/bin/env python3
"""Host issue cost of one fused layer: forward + backward of a ConvBNAct layer (and a 1x1 fused head)
at a tiny batch, so the GPU work is negligible and the wall time per iteration is the Python +
HIP-runtime cost of issuing it (what bounds the eager Inception step when the box's CPU is slow).

usage: python tools/host_layer_bench.py [--iters 300]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=300)
    args = ap.parse_args()
    from tony_amd.models.layers import ConvBNAct, cast_model
    from tony_amd.ops import _lib, streams

    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    cases = {
        "conv1x7_bn_relu": (ConvBNAct(192, 192, (1, 7), padding=(0, 3)), (4, 192, 17, 17)),
        "conv3x3_bn_relu": (ConvBNAct(64, 96, 3, padding=1), (4, 64, 35, 35)),
        "head1x1_bn_relu": (ConvBNAct(192, 64, 1), (4, 192, 35, 35)),
    }
    for name, (layer, shape) in cases.items():
        layer = cast_model(layer, torch.bfloat16, dev).to(memory_format=cl)
        layer.train()
        # gradients land in existing .grad slots (as with the flat PS buffers): allocate them once
        for p in layer.parameters():
            p.grad = torch.zeros_like(p)
        x = torch.randn(shape, device=dev).to(torch.bfloat16).contiguous(memory_format=cl).requires_grad_(True)

        def it():
            streams.begin(dev)
            y = layer(x)
            y.backward(torch.ones_like(y))
            streams.end()

        for _ in range(20):
            it()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            it()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{name}: host {1e6 * (t1 - t0) / args.iters:7.1f} us/iter (fwd+bwd issue), "
              f"wall {1e6 * (t2 - t0) / args.iters:7.1f} us/iter", flush=True)


if __name__ == "__main__":
    main()
