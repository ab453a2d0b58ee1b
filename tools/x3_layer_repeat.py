"""Repeatability of single fp32 (x3) conv + BN + ReLU layers: the same inputs N times, rel. difference of
every output / gradient against the first run (a nondeterministic kernel or an uninitialised read shows
up as run-to-run differences far above the fp32 atomics' ~1e-7).
usage: python tools/x3_layer_repeat.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

SHAPES = [  # (N, C, H, W, Co, k, stride, padding)
    (2, 64, 17, 17, 192, (1, 1), 1, 0), (2, 192, 17, 17, 192, (1, 7), 1, (0, 3)),
    (2, 192, 17, 17, 192, (7, 1), 1, (3, 0)), (2, 192, 17, 17, 192, (3, 3), 2, 0),
    (2, 192, 17, 17, 320, (3, 3), 2, 0), (2, 64, 17, 17, 64, (1, 1), 1, 0), (2, 64, 17, 17, 384, (3, 3), 2, 0)]


def main():
    from tony_amd.ops.x3 import ConvBNActX3

    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    reps = int(os.environ.get("REPS", "6"))
    for n, c, h, w, co, k, s, p in SHAPES:
        torch.manual_seed(0)
        layer = ConvBNActX3(c, co, k, s, p).to(dev).to(memory_format=cl).train()
        x0 = torch.randn(n, c, h, w, device=dev).contiguous(memory_format=cl)
        outs = []
        for _ in range(reps):
            for q in layer.parameters():
                q.grad = None
            x = x0.clone().requires_grad_(True)
            y = layer(x * 1.0)
            g = torch.randn(y.shape, device=dev, generator=torch.Generator(dev).manual_seed(1)).contiguous(memory_format=cl)
            y.backward(g)
            torch.cuda.synchronize()
            outs.append([y.detach().clone(), x.grad.clone()] + [q.grad.clone() for q in layer.parameters()])
        errs = [max(rel(a, b) for a, b in zip(o, outs[0])) for o in outs[1:]]
        names = ["y", "dx", "dw", "dgamma", "dbeta"]
        worst = [max(rel(o[i], outs[0][i]) for o in outs[1:]) for i in range(len(names))]
        print(f"{c}->{co} k{k} s{s}: run-to-run max {' '.join(f'{e:.1e}' for e in errs)} | per output "
              f"{dict(zip(names, [f'{e:.1e}' for e in worst]))}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
