"""Diagnose the fp32 (x3) Inception blocks' fast form: (joins on/off) x (branch streams on/off) against the
plain graph, per block, rel. error of the output, dX and every parameter gradient.
usage: python tools/x3_block_diag.py [A B C D E]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from tony_amd.models import inception_v3 as I
    from tony_amd.ops import streams

    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    mk = {"A": lambda: I.InceptionA(64, 32, x3=True), "B": lambda: I.InceptionB(64, x3=True),
          "C": lambda: I.InceptionC(64, 32, x3=True), "D": lambda: I.InceptionD(64, x3=True),
          "E": lambda: I.InceptionE(64, x3=True)}
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    for name in (sys.argv[1:] or list(mk)):
        torch.manual_seed(0)
        blk = mk[name]().to(dev).to(memory_format=cl).train()
        x0 = torch.randn(2, 64, 17, 17, device=dev).contiguous(memory_format=cl)

        masks = []

        def hook(mod, inp, out):
            masks.append((out.detach() > 0).clone())

        if os.environ.get("DIAG_MASKS") and hasattr(blk, "b7"):
            blk.b7[2].register_forward_hook(hook)  # needs TONY_X3_PLANES=0 (an fp32 output to look at)

        def run(join, br):
            I.JOIN = join
            for p in blk.parameters():
                p.grad = None
            x = x0.clone().requires_grad_(True)
            on = br and streams.begin(x.device, branches=True)
            try:
                y = blk(x * 1.0)
                g = torch.randn(y.shape, device=dev, generator=torch.Generator(dev).manual_seed(1))
                y.backward(g.contiguous(memory_format=cl))
            finally:
                if on:
                    streams.end()
            torch.cuda.synchronize()
            return y.detach().clone(), x.grad.clone(), [p.grad.clone() for p in blk.parameters()]

        ref = run(False, False)
        configs = [(False, False)] * int(os.environ.get("DIAG_REPS", "0")) or \
            [(False, False), (False, False), (True, False), (False, True), (True, True)]
        for join, br in configs:
            out = run(join, br)
            worst = max(rel(a, b) for a, b in zip(out[2], ref[2]))
            if os.environ.get("DIAG_PARAMS") and worst > 1e-4:
                names = [nm for nm, _ in blk.named_parameters()]
                bad = [f"{nm} {rel(a, b):.1e}" for nm, a, b in zip(names, out[2], ref[2]) if rel(a, b) > 1e-4]
                print("   differing:", "; ".join(bad), flush=True)
            flips = int((masks[-1] != masks[0]).sum()) if masks else -1
            print(f"block {name} join={join} streams={br}: y {rel(out[0], ref[0]):.2e} dx {rel(out[1], ref[1]):.2e} "
                  f"worst param grad {worst:.2e} b7[2] ReLU flips vs ref {flips}", flush=True)
    I.JOIN = True
    return 0


if __name__ == "__main__":
    sys.exit(main())
