"""A/B of BatchNorm's forward apply folded into its consumer GEMM.

Today: bn apply + ReLU writes y (csrc/bn_act.hip, one pass over z), then the 1x1 GEMM reads y.
Prototype: the GEMM reads z and applies relu(z * scale + shift) to each A chunk in LDS as it lands
(igemm.h X3Planes::atab, tony_gemm_bf16_bnact, the 128 x 128 three-slot LDS-DMA tile).  For each
consumer shape: the two-pass form on the same tile (variant 12), the two-pass form with the tuned best
tile, and the fused form; plus a numerics check of fused vs two-pass.

usage: python tools/bn_consumer_bench.py [--iters 30]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (label, M, K = the BN'd channels read, N)
SHAPES = [("Inception 17x17 block head (768 -> 768)", 128 * 17 * 17, 768, 768),
          ("Inception 35x35 block head (288 -> 224)", 128 * 35 * 35, 288, 224),
          ("Inception 8x8 block head (2048 -> 1344)", 128 * 8 * 8, 2048, 1344),
          ("ResNet-50 conv1 56x56 (256 -> 64)", 128 * 56 * 56, 256, 64),
          ("ResNet-50 conv3 56x56 (64 -> 256)", 128 * 56 * 56, 64, 256),
          ("ResNet-50 conv1 14x14 (1024 -> 256)", 128 * 14 * 14, 1024, 256)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    from tony_amd.ops import _lib, tune

    dev = torch.device("cuda", 0)
    L, st = _lib.lib(), _lib.stream_ptr(dev)
    print("shape | bn apply us | GEMM v12 us | two-pass v12 us | tuned GEMM us | two-pass tuned us | fused v12 us "
          "| fused vs two-pass tuned | max rel diff")
    for label, m, k, n in SHAPES:
        z = (torch.randn(m, k, device=dev) * 2).to(torch.bfloat16)
        w = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.bfloat16)
        scale = torch.rand(k, device=dev) + 0.5
        shift = torch.randn(k, device=dev) * 0.2
        tab = torch.cat([scale, shift]).contiguous()
        y = torch.empty(m, k, device=dev, dtype=torch.bfloat16)
        c1 = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        c2 = torch.empty_like(c1)
        zeros, ones = torch.zeros(k, device=dev), torch.ones(k, device=dev)

        def bn():  # the apply pass (mode 1: running mean 0, var 1, eps 0, gamma = scale, beta = shift):
            # y = relu(z * scale + shift), the same pass the training step's bn_fwd_apply makes
            rc = L.tony_bn_apply(z.data_ptr(), m, k, k, y.data_ptr(), k, None, None, 0, scale.data_ptr(),
                                 shift.data_ptr(), 0, 0.0, 1, 1, None, None, zeros.data_ptr(), ones.data_ptr(), 0.0, st)
            assert rc == 0, rc

        def gemm(v, src=y, out=c1):
            return L.tony_gemm_bf16(src.data_ptr(), w.data_ptr(), out.data_ptr(), m, n, k, k, k, n, v << 8, None, 0, st)

        def fused():
            rc = L.tony_gemm_bf16_bnact(z.data_ptr(), w.data_ptr(), c2.data_ptr(), m, n, k, k, k, n, 0, None, 0,
                                        tab.data_ptr(), st)
            assert rc == 0, rc

        bn()
        best_v, best_t = 12, float("inf")
        for v in tune._BASE:
            if v >= 9 and v < 11:
                continue
            if gemm(v) != 0:
                continue
            t = tune.time_ms(lambda: gemm(v), a.iters)
            if t < best_t:
                best_v, best_t = v, t
        t_bn = tune.time_ms(bn, a.iters)
        t_g12 = tune.time_ms(lambda: gemm(12), a.iters)
        t_two12 = tune.time_ms(lambda: (bn(), gemm(12)), a.iters)
        t_two = tune.time_ms(lambda: (bn(), gemm(best_v)), a.iters)
        t_f = tune.time_ms(fused, a.iters)
        gemm(12)
        fused()
        torch.cuda.synchronize()
        diff = ((c1.float() - c2.float()).abs().max() / c1.float().abs().max()).item()
        print(f"{label} | {t_bn * 1e3:.1f} | {t_g12 * 1e3:.1f} | {t_two12 * 1e3:.1f} | {best_t * 1e3:.1f} (v{best_v}) | "
              f"{t_two * 1e3:.1f} | {t_f * 1e3:.1f} | {t_two / t_f:.2f}x | {diff:.2e}", flush=True)


if __name__ == "__main__":
    main()
