"""Element-wise check of one conv wgrad shape against an fp64 CPU reference (max error location).
usage: python tools/diag/wgrad_elem.py N C H W Co R S ph pw [stride]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    a = [int(v) for v in sys.argv[1:]]
    n, c, h, w, co, r, s, ph, pw = a[:9]
    st = a[9] if len(a) > 9 else 1
    from tony_amd.ops.conv import conv_wgrad
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    x = torch.randn(n, c, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    oh, ow = (h + 2 * ph - r) // st + 1, (w + 2 * pw - s) // st + 1
    dy = torch.randn(n, co, oh, ow, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dw = conv_wgrad(dy, x, (co, c, r, s), st, (ph, pw)).double().cpu()
    xr = x.double().cpu().requires_grad_()
    wr = torch.zeros(co, c, r, s, dtype=torch.float64, requires_grad=True)
    F.conv2d(xr, wr, None, st, (ph, pw)).backward(dy.double().cpu())
    ref = wr.grad
    err = (dw - ref).abs()
    i = int(err.argmax())
    idx = torch.unravel_index(torch.tensor(i), err.shape)
    print(f"shape {a}: max abs err {err.max().item():.4g} at (co, c, r, s) = {tuple(int(t) for t in idx)}; "
          f"max |ref| {ref.abs().max().item():.4g}; elements > 1e-2*max: {(err > 1e-2 * ref.abs().max()).sum().item()}"
          f" of {err.numel()}")
    bad = (err > 1e-2 * ref.abs().max()).nonzero()
    if len(bad):
        print("  bad taps (r, s):", sorted(set((int(b[2]), int(b[3])) for b in bad))[:10],
              "co range", int(bad[:, 0].min()), int(bad[:, 0].max()), "c range", int(bad[:, 1].min()),
              int(bad[:, 1].max()))


if __name__ == "__main__":
    main()
