"""Every tile variant of the fp32 (x3) strided backward-data on one shape, pinned through the autotuner's
cache: run-to-run spread over REPS runs and the distance to variant 0.
usage: python tools/x3_dgrad_variants.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from tony_amd.ops import tune, x3

    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    reps = int(os.environ.get("REPS", "6"))
    for n, c, h, w, co, (r, s), st, p in [(2, 192, 17, 17, 192, (3, 3), 2, 0), (2, 192, 17, 17, 320, (3, 3), 2, 0),
                                          (4, 192, 17, 17, 192, (3, 3), 2, 0)]:
        torch.manual_seed(0)
        oh, ow = (h - r) // st + 1, (w - s) // st + 1
        d = torch.randn(n, co, oh, ow, device=dev).contiguous(memory_format=cl)
        d3, _ = x3.split_act(d)
        wt = torch.randn(co, c, r, s, device=dev) / (c * r * s) ** 0.5
        wt3 = x3.split_weight_t(wt)
        key = ("x3_dgrad", tuple(d3.shape), (n, c, h, w), tuple(wt.shape), (st, st), (p, p))
        ref = None
        for v in [v for v in tune.NT_VARIANTS if v not in (9, 10)]:
            tune._CACHE[key] = v
            outs = []
            for _ in range(reps):
                junk = torch.randn(n, c, h, w, device=dev)  # varies what a fresh allocation holds
                del junk
                outs.append(x3.conv_dgrad(d3, wt3, co, (n, c, h, w), wt.shape, st, p).clone())
            torch.cuda.synchronize()
            if ref is None:
                ref = outs[0]
            spread = max(rel(o, outs[0]) for o in outs)
            print(f"{c}->{co} n{n} variant {v}: run-to-run {spread:.1e}  vs variant 0 {rel(outs[0], ref):.1e}",
                  flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
