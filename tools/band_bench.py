#!/usr/bin/env python3
"""The band kernel (csrc/band.hip, variant 40) against the tuner's best other variant on every 1 x T / T x 1
conv shape of Inception-v3 at the step's batch: forward (with BN statistics) and backward-data, us and TF/s.

usage: python tools/band_bench.py [--batch 128]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    from conv_bench import collect_shapes

    from tony_amd.ops import _lib, tune
    from tony_amd.ops import conv as C

    dev = torch.device("cuda", 0)
    tot_b = tot_o = 0.0
    for (n, c, h, w, co, k, s, p), cnt in collect_shapes("inception_v3", a.batch).items():
        if s != (1, 1) or (k[0] != 1 and k[1] != 1) or k == (1, 1):
            continue
        x = torch.randn(n, c, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(co, c, *k, device=dev) / (c * k[0] * k[1]) ** 0.5).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        stats = torch.zeros(_lib.stat_floats(co), device=dev)
        y = C.conv_fwd(x, wt, 1, p, stats, vflags=0)
        dy = torch.randn_like(y)
        flop = 2.0 * n * y.shape[2] * y.shape[3] * co * c * k[0] * k[1]
        row = []
        for name, fn in (("fwd", lambda vf: C.conv_fwd(x, wt, 1, p, stats, vflags=vf)),
                         ("dgrad", lambda vf: C.conv_dgrad(dy, wt, x.shape, 1, p, vflags=vf))):
            tb = tune.time_ms(lambda: fn(40 << 8), 10)
            best, bv = float("inf"), None
            for v in tune.NT_VARIANTS:
                try:
                    t = tune.time_ms(lambda: fn(v << 8), 10)
                except Exception:  # noqa: BLE001 - a variant that does not take the shape
                    continue
                if t < best:
                    best, bv = t, v
            row.append(f"{name} band {tb * 1e3:6.1f} us ({flop / tb / 1e9:4.0f} TF/s) vs best {bv} "
                       f"{best * 1e3:6.1f} us ({best / tb:4.2f}x)")
            tot_b += cnt * tb
            tot_o += cnt * best
        print(f"{n}x{c}x{h}x{w}->{co} k{k[0]}x{k[1]} x{cnt}: " + " | ".join(row), flush=True)
    print(f"total over the model's 1-D conv shapes (fwd + dgrad, x occurrences): band {tot_b:.3f} ms vs best "
          f"other {tot_o:.3f} ms")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
