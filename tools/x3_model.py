"""Where does the fp32 (x3) Inception-v3 backward leave the float64 textbook graph?  Block outputs'
gradients and every parameter gradient of one step, in network order (norm-relative error)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def nrel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    from tony_amd.models.inception_v3 import inception_v3
    from tony_amd.ops import cross_entropy
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ours = inception_v3(precision="fp32", seed=3).to(dev).to(memory_format=torch.channels_last).train()
    ref = inception_v3(fused=False, seed=3).to(dev).double().train()
    ours.dropout.p = ref.dropout.p = 0.0
    outs = {}

    def hook(tag):
        def f(mod, inp, out):
            o = out[0] if isinstance(out, tuple) else out
            o.retain_grad()
            outs.setdefault(tag, []).append(o)
        return f

    for m, tagm in ((ours, "o"), (ref, "r")):
        for name, blk in [("mixed_5.%d" % i, b) for i, b in enumerate(m.mixed_5)] + [("mixed_6a", m.mixed_6a)] + \
                [("mixed_6.%d" % i, b) for i, b in enumerate(m.mixed_6)] + [("aux", m.aux)] + \
                [("mixed_7.%d" % i, b) for i, b in enumerate(m.mixed_7)] + [("fc", m.fc)]:
            blk.register_forward_hook(hook((tagm, name)))
    x = torch.randn(4, 3, 299, 299, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (4,), device=dev)
    lo, ao = ours(x)
    lr_, ar = ref(x.double().contiguous())
    loss_o = cross_entropy(lo, y) + 0.4 * cross_entropy(ao, y)
    loss_r = F.cross_entropy(lr_, y) + 0.4 * F.cross_entropy(ar, y)
    loss_o.backward()
    loss_r.backward()
    print("loss", loss_o.item(), loss_r.item())
    names = [k[1] for k in outs if k[0] == "o"]
    for n in names:
        o, r = outs[("o", n)][0], outs[("r", n)][0]
        print(f"{n:10s} out {nrel(o.detach(), r.detach()):.3g}  grad {nrel(o.grad, r.grad):.3g}")
    for (name, po), pr in zip(ours.named_parameters(), ref.parameters()):
        e = nrel(po.grad, pr.grad)
        if e > 1e-3:
            print(f"  {name:40s} {e:.3g}")


if __name__ == "__main__":
    main()
