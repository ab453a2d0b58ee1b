"""Per-layer A/B of ConvBNAct inside Inception-v3: tony implicit-GEMM conv path vs MIOpen path on the
same inputs (training-mode forward), to localise a layer whose outputs disagree."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tony_amd.models import layers  # noqa: E402
from tony_amd.models.inception_v3 import inception_v3  # noqa: E402
from tony_amd.models.layers import cast_model  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = cast_model(inception_v3(num_classes=10, fused=True, seed=0), torch.bfloat16, dev).to(
        memory_format=torch.channels_last)
    model.dropout.p = 0.0
    orig = layers.ConvBNAct.forward
    names = {m: n for n, m in model.named_modules()}
    rows = []

    def both(self, x):
        layers.USE_TONY_CONV = True
        rm, rv = self.bn.running_mean.clone(), self.bn.running_var.clone()
        a = orig(self, x)
        self.bn.running_mean.copy_(rm)
        self.bn.running_var.copy_(rv)
        layers.USE_TONY_CONV = False
        b = orig(self, x)
        layers.USE_TONY_CONV = True
        rel = ((a.float() - b.float()).norm() / (b.float().norm() + 1e-9)).item()
        c = self.conv
        rows.append((rel, names.get(self, "?"), tuple(x.shape), tuple(x.stride()), c.kernel_size, c.stride,
                     c.padding, c.out_channels))
        return b

    layers.ConvBNAct.forward = both
    x = torch.randn(8, 3, 299, 299, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        model(x)
    for r in sorted(rows, reverse=True)[:25]:
        print(f"{r[0]:.4f} {r[1]} in {r[2]} stride {r[3]} k{r[4]} s{r[5]} p{r[6]} co {r[7]}")


if __name__ == "__main__":
    main()
