#!/usr/bin/env python3
"""NT GEMM / conv forward kernels on Inception-v3 shapes: time, TFLOP/s, and the cost of the BN-stats
epilogue (flags bit0) -- per tile variant (flags bits 8..15, 0 = built-in heuristic).

usage: python tools/nt_bench.py [--variants 0,1,2,...] [--reps 20]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

# 1x1 convs as GEMMs (M, N, K) at bs128 and the spatial convs (N, H, W, C, Co, R, S, stride, pad)
GEMMS = [(682112, 80, 64), (156800, 224, 192), (156800, 288, 256), (156800, 288, 288), (36992, 768, 768),
         (36992, 1344, 768), (8192, 1344, 1280), (8192, 1344, 2048), (156800, 192, 224), (36992, 768, 1344)]
CONVS = [(128, 71, 71, 80, 192, 3, 3, 1, 0), (128, 35, 35, 48, 64, 5, 5, 1, 2), (128, 35, 35, 64, 96, 3, 3, 1, 1),
         (128, 35, 35, 96, 96, 3, 3, 1, 1), (128, 17, 17, 160, 160, 1, 7, 1, 3), (128, 17, 17, 192, 192, 7, 1, 3, 0),
         (128, 17, 17, 128, 192, 7, 1, 3, 0), (128, 8, 8, 448, 384, 3, 3, 1, 1), (128, 8, 8, 384, 384, 1, 3, 0, 1),
         (128, 147, 147, 32, 64, 3, 3, 1, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    from tony_amd.ops import _lib

    L = _lib.lib()
    dev = torch.device("cuda", 0)
    st = _lib.stream_ptr(dev)
    variants = [int(v) for v in args.variants.split(",")]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def tm(fn):
        rc = fn()
        if rc != 0:
            return float("nan")
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1000.0 / args.reps

    hdr = " ".join(f"v{v}:nostat v{v}:stat" for v in variants)
    print(f"GEMM M,N,K | {hdr}   (us, TF/s of the best)")
    for M, N, K in GEMMS:
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        b = torch.randn(N, K, device=dev).to(torch.bfloat16)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        s = torch.zeros(_lib.stat_floats(N), device=dev)
        row, best = [], 1e30
        for v in variants:
            for f in (0, 1):
                t = tm(lambda: L.tony_gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, K, K, N,
                                                f | (v << 8), s.data_ptr(), 2 * N, st))
                best = min(best, t)
                row.append(f"{t:8.1f}")
        print(f"{M},{N},{K} | {' '.join(row)} | {2 * M * N * K / best / 1e6:.0f} TF/s")
    print(f"\nCONV n,h,w,c,co,r,s,p | {hdr}")
    for n, h, w, c, co, r, s_, ph, pw in CONVS:
        x = torch.randn(n, h, w, c, device=dev).to(torch.bfloat16)
        wt = torch.randn(co, r, s_, c, device=dev).to(torch.bfloat16)
        oh, ow = h + 2 * ph - r + 1, w + 2 * pw - s_ + 1
        y = torch.empty(n, oh, ow, co, device=dev, dtype=torch.bfloat16)
        sv = torch.zeros(_lib.stat_floats(co), device=dev)
        row, best = [], 1e30
        for v in variants:
            for f in (0, 1):
                t = tm(lambda: L.tony_conv_fwd(x.data_ptr(), n, h, w, c, c, wt.data_ptr(), co, r, s_, 1, 1, ph, pw,
                                               y.data_ptr(), oh, ow, co, f | (v << 8), sv.data_ptr(), 2 * co,
                                               st))
                best = min(best, t)
                row.append(f"{t:8.1f}")
        fl = 2.0 * n * oh * ow * co * r * s_ * c
        print(f"{n},{h},{w},{c},{co},{r},{s_},{ph},{pw} | {' '.join(row)} | {fl / best / 1e6:.0f} TF/s")


if __name__ == "__main__":
    main()
