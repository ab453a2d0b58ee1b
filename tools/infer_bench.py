#!/usr/bin/env python3
"""Inference throughput of Inception-v3 / ResNet-50 (bf16, NHWC, eval mode, one MI355X).

Compares the folded-BN path (conv + BN + ReLU as ONE MFMA kernel per layer, BN scale/shift applied to
the accumulators in the epilogue: SURVEY.md §2.7 H5, ops/conv.py conv_bn_act_infer -- taken under
``torch.no_grad()``) with the same model's eval forward with autograd on (conv kernel, then a
separate BN-apply kernel).  Synthetic inputs, random-init weights; prints one JSON line per path.

Usage: python tools/infer_bench.py [--model inception_v3] [--batch 256] [--iters 30]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="inception_v3", choices=["inception_v3", "resnet50"])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    if a.model == "inception_v3":
        from tony_amd.models.inception_v3 import inception_v3
        m, res = inception_v3(seed=0), 299
    else:
        from tony_amd.models.resnet import resnet50
        m, res = resnet50(seed=0), 224
    m = m.to(dev).to(memory_format=torch.channels_last)
    for p in m.parameters():
        p.data = p.data.to(torch.bfloat16)
    m.eval()
    x = torch.randn(a.batch, 3, res, res, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    def run(folded: bool) -> float:
        ctx = torch.no_grad() if folded else torch.enable_grad()
        with ctx:
            for _ in range(3):
                out = m(x)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(a.iters):
                out = m(x)
            torch.cuda.synchronize()
        del out
        return (time.perf_counter() - t) / a.iters

    for folded in (True, False):
        dt = run(folded)
        print(json.dumps({"metric": f"{a.model} inference images/sec", "value": round(a.batch / dt, 1),
                          "ms_per_batch": round(1000 * dt, 3), "batch": a.batch, "dtype": "bf16",
                          "path": "folded BN epilogue (no_grad)" if folded else "conv + separate BN apply"}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
