"""Time the image-stem conv (Inception-v3: 128x3x299x299 -> 32, 3x3/2; --resnet: 7x7/2 p3 -> 64 at
224x224), NHWC bf16, MIOpen vs the MFMA stem kernels of csrc/stem.hip:

  miopen : F.conv2d forward (+ a tony statistics pass) and MIOpen backward-weight (the TONY_STEM=0 path)
  mfma   : tony_stem_fwd (statistics epilogue) and tony_stem_wgrad + split-K combine (the default path)

Prints per-pass microseconds, the HBM bytes each pass must move and the implied TB/s, plus the
numerics of the MFMA kernels against fp32.

usage: python tools/stem_bench.py [--batch 128] [--iters 20] [--resnet]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def gpu_ms(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--resnet", action="store_true")
    args = ap.parse_args()
    from tony_amd.ops import _lib
    from tony_amd.ops import conv as C

    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    hw, co, k, s, p = (224, 64, 7, 2, 3) if args.resnet else (299, 32, 3, 2, 0)
    x = torch.randn(args.batch, 3, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (0.1 * torch.randn(co, 3, k, k, device=dev)).to(torch.bfloat16).contiguous(memory_format=cl)
    y = torch.nn.functional.conv2d(x, w, None, s, p)
    dy = torch.randn_like(y).contiguous(memory_format=cl)
    stats = torch.zeros(_lib.stat_floats(co), device=dev)
    slot = torch.zeros_like(w)

    res = {
        "miopen fwd+stats": gpu_ms(lambda: C._miopen_fwd(x, w, s, p, stats), args.iters),
        "miopen wgrad": gpu_ms(lambda: C._miopen_wgrad(dy, x, w, s, p), args.iters),
        "mfma fwd": gpu_ms(lambda: C.stem_fwd(x, w, s, p), args.iters),
        "mfma fwd+stats": gpu_ms(lambda: C.stem_fwd(x, w, s, p, stats), args.iters),
        "mfma wgrad (into slot)": gpu_ms(lambda: C.stem_wgrad(dy, x, w.shape, s, p, dst=slot), args.iters),
    }
    xb, yb = x.numel() * 2, y.numel() * 2
    moved = {"miopen fwd+stats": xb + 2 * yb, "miopen wgrad": xb + yb, "mfma fwd": xb + yb,
             "mfma fwd+stats": xb + yb, "mfma wgrad (into slot)": xb + yb}
    for name, ms in res.items():
        print(f"{name:>24}: {ms * 1000:8.1f} us  ({moved[name] / ms / 1e9:5.2f} TB/s of {moved[name] / 1e6:.0f} MB)")
    ref = torch.nn.functional.conv2d(x.float(), w.float(), None, s, p)
    got = C.stem_fwd(x, w, s, p).float()
    dwr = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), s, p)
    dwg = C.stem_wgrad(dy, x, w.shape, s, p).float()
    print("fwd rel err", ((got - ref).norm() / ref.norm()).item(),
          "wgrad rel err", ((dwg - dwr).norm() / dwr.norm()).item())


if __name__ == "__main__":
    main()
