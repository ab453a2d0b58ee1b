"""Piecewise check of one x3 (fp32) conv + BN + ReLU layer against float64: Z, the BN backward dZ and
the weight gradient (from OUR dZ, so a wrong dZ and a wrong wgrad are told apart).
usage: python tools/x3_layer.py N C H W Co R S ph pw [stride]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    e = (a - b).abs()
    return e.max().item() / b.abs().max().item(), int((e > 1e-3 * b.abs().max()).sum())


def main():
    a = [int(v) for v in sys.argv[1:]]
    n, c, h, w, co, r, s, ph, pw = a[:9]
    st = a[9] if len(a) > 9 else 1
    from tony_amd.ops import x3
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    x = torch.randn(n, c, h, w, device=dev).contiguous(memory_format=torch.channels_last)
    wt = torch.randn(co, c, r, s, device=dev) / (c * r * s) ** 0.5
    x3p, cp = x3.split_act(x)
    w3 = x3.split_weight(wt)
    z = x3.conv_fwd(x3p, cp, w3, wt.shape, st, (ph, pw))
    zr = F.conv2d(x.double().cpu(), wt.double().cpu(), None, st, (ph, pw))
    print("Z", rel(z, zr))
    g = torch.randn_like(z).contiguous(memory_format=torch.channels_last)
    d3, _ = x3.split_act(g)
    dw = x3.conv_wgrad(d3, x3p, cp, wt.shape, st, (ph, pw))
    xr = x.double().cpu().requires_grad_()
    wr = wt.double().cpu().requires_grad_()
    F.conv2d(xr, wr, None, st, (ph, pw)).backward(g.double().cpu())
    print("dW", rel(dw, wr.grad))
    dx = x3.conv_dgrad(d3, x3.split_weight_t(wt), co, x.shape, wt.shape, st, (ph, pw))
    print("dX", rel(dx, xr.grad))
    for name, (dd, xx) in {"hh": (d3[:, 0:co], x3p[:, 0:cp]), "hl": (d3[:, 0:co], x3p[:, cp:2 * cp]),
                           "lh": (d3[:, co:2 * co], x3p[:, 0:cp])}.items():
        from tony_amd.ops.conv import conv_wgrad
        part = conv_wgrad(dd, xx, (co, cp, r, s), st, (ph, pw))
        xr2 = xx.double().cpu()
        wr2 = torch.zeros(co, cp, r, s, dtype=torch.float64, requires_grad=True)
        F.conv2d(xr2, wr2, None, st, (ph, pw)).backward(dd.double().cpu())
        print("  plane", name, rel(part, wr2.grad))


if __name__ == "__main__" and sys.argv[1:2] != ["bn"]:
    main()


def bn_check():
    """BN(+ReLU) forward / backward on fp32 rows (x3.bn_apply / x3.bn_backward) vs float64."""
    a = [int(v) for v in sys.argv[2:]]
    n, co, h, w = a[:4]
    from tony_amd.ops import _lib, x3
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    z = (torch.randn(n, co, h, w, device=dev) * 3 + 1).contiguous(memory_format=torch.channels_last)
    gamma = torch.empty(co, device=dev).uniform_(0.5, 1.5)
    beta = torch.empty(co, device=dev).uniform_(-0.2, 0.2)
    stats = torch.zeros(_lib.stat_floats(co), device=dev)
    zs = z.double()
    s = zs.sum((0, 2, 3))
    s2 = (zs * zs).sum((0, 2, 3))
    stats.view(-1, 2 * co)[0, :co] = s.float()
    stats.view(-1, 2 * co)[0, co:] = s2.float()
    rm, rv = torch.zeros(co, device=dev), torch.ones(co, device=dev)
    y, mean, invstd = x3.bn_apply(z, stats, gamma, beta, rm, rv, 1e-3, 0.1, True, True)
    zr = z.double().cpu().requires_grad_()
    gr, br = gamma.double().cpu().requires_grad_(), beta.double().cpu().requires_grad_()
    yr = torch.relu(F.batch_norm(zr, None, None, gr, br, True, 0.0, 1e-3))
    print("BN y", rel(y, yr))
    g = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
    dz, dgamma, dbeta = x3.bn_backward(z, g, mean, invstd, gamma, beta, True)
    yr.backward(g.double().cpu())
    print("BN dz", rel(dz, zr.grad), "dgamma", rel(dgamma, gr.grad), "dbeta", rel(dbeta, br.grad))


if __name__ == "__main__" and sys.argv[1:2] == ["bn"]:
    bn_check()
