"""Time the Inception-v3 3-channel stem conv (128x3x299x299 -> 32, 3x3/2) two ways, NHWC bf16:

  miopen : F.conv2d forward + MIOpen backward-weight (what the 3-channel stem runs on today);
  direct : csrc/stem.hip, the 27-tap direct kernel with the statistics epilogue (the shipped path);
  pad8   : input zero-padded to 8 channels (one copy) + tony implicit-GEMM forward (with the BN
           statistics epilogue) + tony split-K backward-weight on the padded operands.

usage: python tools/stem_bench.py [--batch 128] [--iters 20]
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
    args = ap.parse_args()
    from tony_amd.ops import _lib
    from tony_amd.ops import conv as C

    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    x = torch.randn(args.batch, 3, 299, 299, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (0.1 * torch.randn(32, 3, 3, 3, device=dev)).to(torch.bfloat16).contiguous(memory_format=cl)
    y = torch.nn.functional.conv2d(x, w, None, 2, 0)
    dy = torch.randn_like(y).contiguous(memory_format=cl)

    x8 = torch.zeros(args.batch, 8, 299, 299, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
    w8 = torch.zeros(32, 8, 3, 3, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
    w8[:, :3] = w
    stats = torch.zeros(_lib.stat_floats(32), device=dev)

    def pad():
        x8[:, :3].copy_(x)

    res = {
        "miopen fwd": gpu_ms(lambda: C._miopen_fwd(x, w, 2, 0), args.iters),
        "miopen fwd+stats": gpu_ms(lambda: C._miopen_fwd(x, w, 2, 0, stats), args.iters),
        "miopen wgrad": gpu_ms(lambda: C._miopen_wgrad(dy, x, w, 2, 0), args.iters),
        "pad 3->8": gpu_ms(pad, args.iters),
        "tony fwd+stats (pad8)": gpu_ms(lambda: C.conv_fwd(x8, w8, 2, 0, stats), args.iters),
        "tony wgrad (pad8)": gpu_ms(lambda: C.conv_wgrad(dy, x8, w8.shape, 2, 0), args.iters),
        "direct fwd (stem.hip)": gpu_ms(lambda: C.stem_fwd(x, w, 2, 0), args.iters),
        "direct fwd+stats (stem.hip)": gpu_ms(lambda: C.stem_fwd(x, w, 2, 0, stats), args.iters),
    }
    # numerics of the padded path vs the fp32 reference
    ref = torch.nn.functional.conv2d(x.float(), w.float(), None, 2, 0)
    got = C.conv_fwd(x8, w8, 2, 0).float()
    dwr = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), 2, 0)
    dwg = C.conv_wgrad(dy, x8, w8.shape, 2, 0)[:, :3].float()
    for k, v in res.items():
        print(f"{k:>24}: {v * 1000:8.1f} us")
    print(f"miopen total {1000 * (res['miopen fwd+stats'] + res['miopen wgrad']):.1f} us; pad8 total "
          f"{1000 * (res['pad 3->8'] + res['tony fwd+stats (pad8)'] + res['tony wgrad (pad8)']):.1f} us")
    got_d = C.stem_fwd(x, w, 2, 0).float()
    print("direct fwd rel err", ((got_d - ref).norm() / ref.norm()).item())
    print("fwd max rel err", ((got - ref).abs().max() / ref.abs().max()).item(),
          "wgrad max rel err", ((dwg - dwr).abs().max() / dwr.abs().max()).item())


if __name__ == "__main__":
    main()
