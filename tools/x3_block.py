"""One Inception block of the fp32 (x3) model against its float64 twin: every sub-layer's output and
output gradient (norm-relative), the block input gradient.
usage: python tools/x3_block.py [block, e.g. mixed_7.2] [batch]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def nrel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    from tony_amd.models.inception_v3 import inception_v3
    blk_name = sys.argv[1] if len(sys.argv) > 1 else "mixed_7.2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.device("cuda", 0)
    ours = inception_v3(precision="fp32", seed=3).to(dev).to(memory_format=torch.channels_last).train()
    ref = inception_v3(fused=False, seed=3).to(dev).double().train()
    bo, br = ours.get_submodule(blk_name), ref.get_submodule(blk_name)
    cin = {"mixed_7.2": 2048, "mixed_7.1": 1280, "mixed_7.0": 768}.get(blk_name, 768)
    hw = 8 if blk_name in ("mixed_7.1", "mixed_7.2") else 17
    outs = {}

    def hook(tag):
        def f(mod, inp, out):
            out.retain_grad()
            outs[tag] = out
        return f

    for tagm, b in (("o", bo), ("r", br)):
        for name, m in b.named_modules():
            if name and name.count(".") <= 1 and hasattr(m, "forward") and (hasattr(m, "conv") or hasattr(m, "bn")):
                m.register_forward_hook(hook((tagm, name)))
    torch.manual_seed(0)
    x = torch.randn(n, cin, hw, hw, device=dev).contiguous(memory_format=torch.channels_last).requires_grad_()
    xr = x.detach().double().contiguous().requires_grad_()
    yo, yr = bo(x), br(xr)
    g = torch.randn_like(yr)
    yo.backward(g.float().contiguous(memory_format=torch.channels_last))
    yr.backward(g)
    print(f"{blk_name}: out {nrel(yo.detach(), yr.detach()):.3g}  dx {nrel(x.grad, xr.grad):.3g}")
    for k in sorted(k for k in outs if k[0] == "o"):
        o, r = outs[k], outs[("r", k[1])]
        print(f"  {k[1]:10s} out {nrel(o.detach(), r.detach()):.3g}  dout {nrel(o.grad, r.grad):.3g}")
    for (name, po), pr in zip(bo.named_parameters(), br.parameters()):
        print(f"  param {name:24s} {nrel(po.grad, pr.grad):.3g}")


if __name__ == "__main__":
    main()
