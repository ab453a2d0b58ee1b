#!/usr/bin/env python3
"""Host-side (Python) profile of eager Inception-v3 training steps: where the ~15 ms of host issue
time per step goes (ctypes launches, autograd nodes, MIOpen calls, allocator).  GPU box only.

Usage: python tools/host_profile.py [--steps 5] [--batch 128]
"""
import argparse
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--bwd", action="store_true", help="profile the autograd (backward) thread instead")
    args = ap.parse_args()
    from tony_amd.models.inception_v3 import inception_v3
    from tony_amd.ops import cross_entropy
    from tony_amd.parallel.ps import ParameterServer
    from tony_amd.parallel.trainer import Trainer

    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    model = inception_v3(seed=0).to(dev).to(memory_format=torch.channels_last).train()
    ps = ParameterServer(model, optimizer="sgd", lr=0.045, momentum=0.9, weight_decay=4e-5, device=dev)

    def loss_fn(out, y):
        return cross_entropy(out[0], y) + 0.4 * cross_entropy(out[1], y)

    x = torch.randn((args.batch, 3, 299, 299), device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (args.batch,), device=dev)
    tr = Trainer(model, ps, loss_fn, use_graph=False)
    for _ in range(3):
        tr.step(x, y)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    if args.bwd:
        # the backward runs on autograd's device thread: start the profiler there, from the first
        # custom Function backward of the profiled steps (cProfile hooks only the calling thread)
        on = [False]
        import tony_amd.ops as ops_pkg
        fns = set()
        for mod in list(sys.modules.values()):
            if mod is None or not getattr(mod, "__name__", "").startswith(ops_pkg.__name__):
                continue
            for v in vars(mod).values():
                if isinstance(v, type) and issubclass(v, torch.autograd.Function) and "backward" in vars(v):
                    fns.add(v)

        def wrap(orig):
            def bw(ctx, *a):
                if not on[0]:
                    on[0] = True
                    pr.enable()
                return orig(ctx, *a)
            return staticmethod(bw)

        for f in fns:
            f.backward = wrap(f.backward)
        for _ in range(args.steps):
            tr.step(x, y)
        torch.cuda.synchronize()
    else:
        pr.enable()
        for _ in range(args.steps):
            tr.step(x, y)
        pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(args.top)
    st.sort_stats("cumulative").print_stats(args.top)


if __name__ == "__main__":
    main()
