#!/usr/bin/env python3
"""Force one NT tile variant everywhere (tune.pick returns it whenever the kernel accepts it) and
compare the fused model's forward against the stock fp32 graph, for every variant: a variant that
is wrong for some shape the model hits shows up as a large relative error (autotuning picks
variants by timing, so such a bug would otherwise surface only when that variant happens to win).

usage: python tools/variant_sweep_model.py [--model resnet50|inception_v3] [--batch 4] [--res 64]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--res", type=int, default=64)
    args = ap.parse_args()
    from tony_amd.models.layers import cast_model
    from tony_amd.ops import conv, tune

    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    if args.model == "resnet50":
        from tony_amd.models.resnet import resnet50 as build_fn
        kw = {"num_classes": 10}
    else:
        from tony_amd.models.inception_v3 import inception_v3 as build_fn
        kw = {"num_classes": 10}

    def build(fused, dtype):
        torch.manual_seed(0)
        return cast_model(build_fn(fused=fused, **kw), dtype, dev).to(memory_format=cl)

    fused = build(True, torch.bfloat16)
    ref = build(False, torch.float32)
    ref.load_state_dict({k: v.float() for k, v in fused.state_dict().items()}, strict=False)
    torch.manual_seed(1)
    x = torch.randn(args.batch, 3, args.res, args.res, device=dev).contiguous(memory_format=cl)
    with torch.no_grad():
        pass
    yr = ref(x)
    yr = yr[0] if isinstance(yr, tuple) else yr
    orig_pick = tune.pick
    for v in [None] + list(tune.NT_VARIANTS):
        tune._CACHE.clear()
        conv._CHOICE.clear()
        conv._FWD_PLAN.clear()
        if v is not None:
            def forced(key, launch, variants=tune.NT_VARIANTS, v=v):
                return (v << 8) if launch(v << 8) == 0 else 0
            tune.pick = forced
        else:
            tune.pick = orig_pick
        y = fused(x.to(torch.bfloat16))
        y = y[0] if isinstance(y, tuple) else y
        torch.cuda.synchronize()
        rel = ((y.float() - yr).norm() / yr.norm()).item()
        print(f"variant {'auto' if v is None else v:>4}: rel err to fp32 {rel:.4f}", flush=True)
    tune.pick = orig_pick


if __name__ == "__main__":
    main()
