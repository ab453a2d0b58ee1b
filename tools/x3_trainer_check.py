#!/usr/bin/env python3
"""Where does the x3 (fp32) Inception-v3 trained through Trainer + ParameterServer leave the plain autograd
reference?  One process, one GPU, batch 2: gradients of (a) a plain forward/backward twice (determinism),
(b) forward/backward under the Trainer's arena + weight caches, and (c) the update of one Trainer step on a
one-rank ParameterServer against the SGD-momentum update built from (a).  Prints the worst / best
parameters of each comparison.

usage: python tools/x3_trainer_check.py [--steps 1]
"""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")

B, CLASSES = 2, 1000
LR, MU, WD = 0.1, 0.9, 4e-5
PRECISION = "fp32"


def say(msg):
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)


def data(dev, w=0):
    g = torch.Generator(device=dev).manual_seed(77 + w)
    x = torch.randn((B, 3, 299, 299), generator=g, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, CLASSES, (B,), generator=g, device=dev)
    return x, y


def model(dev):
    from tony_amd.models.inception_v3 import inception_v3

    torch.manual_seed(0)
    m = inception_v3(num_classes=CLASSES, precision=PRECISION, seed=0).to(dev).to(memory_format=torch.channels_last)
    m.dropout.p = 0.0
    return m.train()


def loss_fn(out, y):
    from tony_amd.ops import cross_entropy

    logits, aux = out
    return cross_entropy(logits, y) + 0.4 * cross_entropy(aux, y)


def grads(m, x, y, ctx=None):
    for p in m.parameters():
        p.grad = None
    if ctx is None:
        loss_fn(m(x), y).backward()
    else:
        with ctx():
            loss_fn(m(x), y).backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().clone() for n, p in m.named_parameters()}


def compare(tag, a, b, top=6):
    rows = []
    num = den = 0.0
    for n in a:
        d = (a[n] - b[n]).double().norm().item()
        r = b[n].double().norm().item()
        num += d * d
        den += r * r
        rows.append((d / (r + 1e-30), n, a[n].numel()))
    rows.sort(reverse=True)
    say(f"{tag}: total rel err {(num / den) ** 0.5:.3e}")
    for e, n, k in rows[:top]:
        say(f"   worst {e:.3e} {n} ({k})")
    for e, n, k in rows[-3:]:
        say(f"   best  {e:.3e} {n} ({k})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--det-only", action="store_true", help="only the plain-backward-twice comparison")
    a = ap.parse_args()
    global PRECISION
    PRECISION = a.precision
    dev = torch.device("cuda", 0)
    x, y = data(dev)
    ref = model(dev)
    w0 = {n: p.detach().clone() for n, p in ref.named_parameters()}
    g1 = grads(ref, x, y)
    say("reference backward 1 done")
    g2 = grads(ref, x, y)
    compare("plain backward twice", g2, g1)
    # backward order (the top of the network first): where the two runs start to disagree
    names = list(g1)[::-1]
    shown = 0
    for n in names:
        e = ((g2[n] - g1[n]).double().norm() / (g1[n].double().norm() + 1e-30)).item()
        if e > 1e-4 or shown < 12:
            say(f"   backward order: {e:.3e} {n}")
            shown += 1
        if shown >= 40:
            break
    g2b = grads(ref, x, y)
    compare("plain backward 3 vs 2 (both after the autotuning call)", g2b, g2)
    if a.det_only:
        return 0

    from contextlib import contextmanager

    from tony_amd.ops import wt_cache
    from tony_amd.ops.arena import for_device

    wt, wx3 = wt_cache.TransposedWeights(dev), wt_cache.X3Weights(dev)
    wt.enabled = wx3.enabled = True
    arena = for_device(dev)

    @contextmanager
    def cached():
        wt_cache.activate(wt, wx3)
        try:
            with arena:
                yield
        finally:
            wt_cache.activate(None)

    g3 = grads(ref, x, y, cached)
    compare("under arena + weight caches", g3, g1)

    from tony_amd.parallel.ps import ParameterServer
    from tony_amd.parallel.trainer import Trainer

    m = model(dev)
    ps = ParameterServer(m, optimizer="sgd", lr=LR, momentum=MU, weight_decay=WD, dtype=torch.float32, device=dev,
                         wire_dtype=torch.float32)
    tr = Trainer(m, ps, loss_fn, use_graph=False)
    tr.step(x, y)
    torch.cuda.synchronize()
    du = {n: (p.detach() - w0[n]) for n, p in m.named_parameters()}
    want = {n: -LR * (g1[n] + WD * w0[n]) for n in g1}
    compare("Trainer + PS step 0 update vs reference update", du, want)
    # the gradient the PS saw: its flat gradient buffer, if the parameters still expose .grad
    gs = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    if len(gs) == len(g1):
        compare("Trainer step 0 gradients vs reference", gs, g1)
    else:
        say(f"{len(gs)} of {len(g1)} parameters expose .grad after the step")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
