#!/usr/bin/env python3
"""Census of the x3 activation splits (ops/x3.split_rows on activations) in one fp32 Inception-v3 training
step: shape and the model call site of each, to find splits the plane caches miss.

usage: python tools/x3_split_census.py [--batch 128]
"""
import collections
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    from tony_amd.models.inception_v3 import inception_v3
    from tony_amd.ops import streams, x3
    from tony_amd.ops.loss import cross_entropy

    batch = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 32
    dev = torch.device("cuda", 0)
    model = inception_v3(fused=False, seed=0, precision="fp32").to(dev).to(memory_format=torch.channels_last).train()
    xb = torch.randn(batch, 3, 299, 299, device=dev).contiguous(memory_format=torch.channels_last)
    yb = torch.randint(0, 1000, (batch,), device=dev)
    census = collections.Counter()
    real = x3.split_rows

    def spy(src, rows, c, ld, pattern):
        if pattern == x3.ACT:
            site = [f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in traceback.extract_stack()[-7:-1]
                    if "tony_amd" in f.filename or "torch" not in f.filename]
            census[(rows, c, " <- ".join(site[-4:]))] += 1
        return real(src, rows, c, ld, pattern)

    x3.split_rows = spy

    def step():
        on = streams.begin(dev, branches=True)
        try:
            out = model(xb)
            logits, aux = out if isinstance(out, tuple) else (out, None)
            loss = cross_entropy(logits, yb) + (0.4 * cross_entropy(aux, yb) if aux is not None else 0)
            loss.backward()
        finally:
            if on:
                streams.end()

    step()  # tuning
    census.clear()
    step()
    torch.cuda.synchronize()
    total = 0
    for (rows, c, site), k in sorted(census.items(), key=lambda t: -t[0][0] * t[0][1]):
        total += k
        print(f"{k:3d} x rows={rows:8d} c={c:5d}  {site}")
    print(f"activation splits per step: {total}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
