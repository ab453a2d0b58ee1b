"""Stream-K A/B of the LDS-DMA NT kernels (csrc/igemm.h SplitK) on the small-spatial Inception-v3 layers.

For every shape and pass (forward + BN statistics, stride-1 backward-data, and the 1x1 layers' GEMM),
each LDS-DMA tile variant is timed as a plain launch (one workgroup per tile) and in stream-K form over
m x CUs workgroups; the table shows the best plain and the best stream-K time per m and pass, and the
variant that achieved each.

usage: python tools/splitk_bench.py [--batch 128] [--iters 20] [--ms 1,2,3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (Cin, H, W, Cout, (R, S), (ph, pw))
CONV = [(192, 17, 17, 192, (1, 7), (0, 3)), (160, 17, 17, 160, (7, 1), (3, 0)), (128, 17, 17, 128, (1, 7), (0, 3)),
        (160, 17, 17, 192, (7, 1), (3, 0)), (384, 8, 8, 384, (1, 3), (0, 1)), (448, 8, 8, 384, (3, 3), (1, 1)),
        (64, 35, 35, 96, (3, 3), (1, 1)), (96, 35, 35, 96, (3, 3), (1, 1))]
# 1x1 layers as GEMMs (M = batch * H * W): (K = Cin, N = Cout)
GEMM = [(17, 768, 192), (17, 768, 768), (8, 2048, 448), (8, 2048, 384), (8, 1280, 320), (8, 1280, 1152),
        (35, 288, 64)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--ms", default="1,2,3")
    a = ap.parse_args()
    from tony_amd.ops import _lib, tune
    from tony_amd.ops import conv as C

    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    L = _lib.lib()
    splits = [int(s) for s in a.ms.split(",")]
    base = [v for v in tune._BASE if v >= 11]

    def best(fn):
        out = {}
        for s in [0] + splits:
            t_best, v_best = float("inf"), None
            for v in base:
                vf = (v << 8) | (s << 16)
                try:
                    if fn(vf) != 0:
                        continue
                    t = tune.time_ms(lambda: fn(vf), a.iters)
                except Exception:  # noqa: BLE001 - variant not applicable
                    continue
                if t < t_best:
                    t_best, v_best = t, v
            out[s] = (t_best, v_best)
        return out

    def report(name, flop, res):
        t1, v1 = res[0]
        cells = [f"{name:44s} plain {t1 * 1e3:6.1f} us v{v1} ({flop / t1 / 1e9:4.0f} TF/s)"]
        for s in splits:
            t, v = res[s]
            if v is None:
                cells.append(f"m{s}    n/a")
            else:
                cells.append(f"m{s} {t * 1e3:6.1f} us v{v} ({t1 / t:4.2f}x)")
        print(" | ".join(cells), flush=True)

    print(f"batch {a.batch}; best LDS-DMA variant per split count (tune.time_ms, {a.iters} reps)")
    for cin, h, w, co, (r, s), pad in CONV:
        x = torch.randn(a.batch, cin, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        wt = (0.05 * torch.randn(co, cin, r, s, device=dev)).to(torch.bfloat16).contiguous(memory_format=cl)
        y = C.conv_fwd(x, wt, 1, pad)
        dy = torch.randn_like(y).contiguous(memory_format=cl)
        stats = torch.zeros(_lib.stat_floats(co), device=dev)
        flop = 2.0 * a.batch * y.shape[2] * y.shape[3] * co * cin * r * s
        tag = f"{cin}x{h}x{w}->{co} k{r}x{s}"

        def fwd(vf):
            C.conv_fwd(x, wt, 1, pad, stats, vf)
            return 0

        def dgr(vf):
            C.conv_dgrad(dy, wt, x.shape, 1, pad, vf)
            return 0

        report(tag + " fwd+stats", flop, best(fwd))
        report(tag + " dgrad", flop, best(dgr))
    st = _lib.stream_ptr(dev)
    for hw, k, n in GEMM:
        m = a.batch * hw * hw
        A = torch.randn(m, k, device=dev).to(torch.bfloat16)
        B = (0.05 * torch.randn(n, k, device=dev)).to(torch.bfloat16)
        Cm = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        stats = torch.zeros(_lib.stat_floats(n), device=dev)

        def gemm(vf):
            return L.tony_gemm_bf16(A.data_ptr(), B.data_ptr(), Cm.data_ptr(), m, n, k, k, k, n, 1 | vf,
                                    stats.data_ptr(), 2 * n, st)

        report(f"gemm {hw}x{hw} M={m} K={k} N={n} +stats", 2.0 * m * n * k, best(gemm))


if __name__ == "__main__":
    main()
