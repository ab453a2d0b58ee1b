"""Compare fused vs stock ResNet-50 block by block on the GPU (bf16 vs fp32)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tony_amd.models.layers import cast_model  # noqa: E402
from tony_amd.models.resnet import resnet50  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    fused = cast_model(resnet50(num_classes=10, fused=True), torch.bfloat16, dev).to(
        memory_format=torch.channels_last)
    stock = resnet50(num_classes=10, fused=False).to(dev, torch.float32).to(memory_format=torch.channels_last)
    for b in list(fused.blocks) + list(stock.blocks):
        torch.nn.init.constant_(b.bn3.weight, 0.5)
    stock.load_state_dict({k: v.float() for k, v in fused.state_dict().items()})
    x = torch.randn(4, 3, 64, 64, device=dev).contiguous(memory_format=torch.channels_last)
    xf, xs = x.to(torch.bfloat16), x
    xf, xs = fused.stem(xf), stock.stem(xs)
    print("stem", rel(xf, xs), xf.float().norm().item(), xs.norm().item())
    xf = torch.nn.functional.max_pool2d(xf, 3, 2, 1)
    xs = torch.nn.functional.max_pool2d(xs, 3, 2, 1)
    for i, (bf, bs) in enumerate(zip(fused.blocks, stock.blocks)):
        a1, s1 = bf.conv1(xf), bs.conv1(xs)
        a2, s2 = bf.conv2(a1), bs.conv2(s1)
        idf = bf.downsample(xf) if bf.downsample is not None else xf
        ids = bs.downsample(xs) if bs.downsample is not None else xs
        yf, ys = bf(xf), bs(xs)
        print(f"block {i}: conv1 {rel(a1, s1):.3g} conv2 {rel(a2, s2):.3g} id {rel(idf, ids):.3g} "
              f"out {rel(yf, ys):.3g} |yf| {yf.float().norm().item():.3g} |ys| {ys.norm().item():.3g}")
        xf, xs = yf, ys
    print("logits", rel(fused(x.to(torch.bfloat16)), stock(x)))
    # isolated op at the failing block's shapes
    from tony_amd.ops.residual import bn_add_relu, conv1x1_bn_add_relu

    for (n, cin, h, w, cout) in [(4, 128, 8, 8, 512), (4, 64, 16, 16, 256), (4, 256, 4, 4, 1024)]:
        xi = torch.randn(n, cin, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wi = (torch.randn(cout, cin, 1, 1, device=dev) / cin ** 0.5).to(torch.bfloat16)
        ri = torch.randn(n, cout, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        g = torch.full((cout,), 0.5, device=dev, dtype=torch.bfloat16)
        b = torch.zeros(cout, device=dev, dtype=torch.bfloat16)
        rm, rv = torch.zeros(cout, device=dev), torch.ones(cout, device=dev)
        y = conv1x1_bn_add_relu(xi, wi, ri, g, b, rm, rv, True, 0.1, 1e-5)
        z = torch.nn.functional.conv2d(xi.float(), wi.float())
        yr = torch.relu(torch.nn.functional.batch_norm(z, None, None, g.float(), b.float(), True, 0.1, 1e-5)
                        + ri.float())
        y2 = bn_add_relu(z.to(torch.bfloat16).contiguous(memory_format=torch.channels_last), ri, g, b, rm, rv,
                         True, 0.1, 1e-5)
        from tony_amd.ops.gemm import gemm_nt

        zg = gemm_nt(xi.permute(0, 2, 3, 1).reshape(-1, cin), wi.reshape(cout, cin))
        print(f"op {n}x{cin}x{h}x{w}->{cout}: conv1x1_bn_add_relu {rel(y, yr):.3g} bn_add_relu {rel(y2, yr):.3g} "
              f"gemm {rel(zg, z.permute(0, 2, 3, 1).reshape(-1, cout)):.3g} finite {torch.isfinite(y.float()).all().item()}")


if __name__ == "__main__":
    main()
