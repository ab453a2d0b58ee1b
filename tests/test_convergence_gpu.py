"""bf16 (tony_amd HIP kernels) vs fp32 (stock PyTorch-ROCm) training: the same reduced Inception
network, the same initial weights and the same fixed synthetic data, trained 200 steps through the
real parameter-server step (Trainer + ParameterServer + fused SGD-momentum).  The reference TF-PS
Inception job trains in fp32 (EX/mnist-tensorflow/mnist_distributed.py:64-124); this pins that the
bf16 fast path follows the fp32 loss curve -- the "AMP equivalence" the headline number rests on.
"""
import pytest
import torch
from torch import nn

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


class _Reduced(nn.Module):
    """Inception-v3 pieces whose fused and stock forms have identical parameters: the 3-channel
    stem, a 3x3 (halo kernel), a 1x1 (MFMA GEMM head), reduction-B (strided 3x3 fwd + strided
    dgrad, max-pool branch, zero-copy concat) and a factorised 1x7 / 7x1 pair, then the classifier."""

    def __init__(self, fused: bool, classes: int = 10):
        super().__init__()
        from tony_amd.models import inception_v3 as iv3
        from tony_amd.models.layers import ConvBNAct

        def c(cin, cout, k, s=1, p=0):
            return ConvBNAct(cin, cout, k, s, p, eps=1e-3, fused=fused)

        self.fused = fused
        self.stem = nn.Sequential(c(3, 32, 3, 2), c(32, 64, 3, 1, 1), c(64, 64, 1))
        self.b = iv3.InceptionB(64, fused=fused)
        self.c7 = nn.Sequential(c(self.b.out_channels, 128, (1, 7), 1, (0, 3)), c(128, 192, (7, 1), 1, (3, 0)))
        self.fc = nn.Linear(192, classes)

    def forward(self, x):
        from tony_amd.ops.pool import global_avg_pool

        x = self.c7(self.b(self.stem(x)))
        x = global_avg_pool(x) if self.fused else torch.flatten(nn.functional.adaptive_avg_pool2d(x, 1), 1)
        return self.fc(x)


def _data(dev, n=128, classes=10, hw=71):
    g = torch.Generator().manual_seed(123)
    x = torch.randn(n, 3, hw, hw, generator=g)
    proj = torch.randn(classes, 3, generator=g)
    # learnable labels: the class whose colour projection of the image mean is largest
    y = (x.mean((2, 3)) @ proj.t()).argmax(1)
    return x.to(dev), y.to(dev)


def _curve(fused: bool, steps: int, dev):
    from tony_amd.models.layers import init_weights
    from tony_amd.ops import cross_entropy
    from tony_amd.parallel.ps import ParameterServer
    from tony_amd.parallel.trainer import Trainer

    dtype = torch.bfloat16 if fused else torch.float32
    ref = init_weights(_Reduced(fused=False), seed=7)
    model = _Reduced(fused=fused)
    model.load_state_dict(ref.state_dict())  # identical initial weights for both precisions
    model = model.to(dev).to(memory_format=torch.channels_last).train()
    ps = ParameterServer(model, optimizer="sgd", lr=0.02, momentum=0.9, weight_decay=1e-4, dtype=dtype, device=dev)

    def loss_fn(out, y):
        return cross_entropy(out, y) if fused else nn.functional.cross_entropy(out.float(), y)

    tr = Trainer(model, ps, loss_fn, use_graph=False)
    x, y = _data(dev)
    x = x.to(dtype).contiguous(memory_format=torch.channels_last)
    losses = [float(tr.step(x, y).float().item()) for _ in range(steps)]
    return torch.tensor(losses)


def test_bf16_fused_training_follows_fp32_loss_curve(cuda):
    steps = 200
    l16 = _curve(True, steps, cuda)
    l32 = _curve(False, steps, cuda)
    assert torch.isfinite(l16).all() and torch.isfinite(l32).all()
    # both learn: the last 20 steps average well below the first step's loss
    assert l32[-20:].mean() < 0.5 * l32[0] and l16[-20:].mean() < 0.5 * l16[0], (l16[-5:], l32[-5:])
    # the curves agree: windowed means within 15% (relative to fp32) + 0.05 absolute at every quarter
    for end in (50, 100, 150, 200):
        a, b = l16[end - 10:end].mean().item(), l32[end - 10:end].mean().item()
        assert abs(a - b) <= 0.15 * b + 0.05, (end, a, b)
    print("bf16 loss:", [round(v, 4) for v in l16[::25].tolist()])
    print("fp32 loss:", [round(v, 4) for v in l32[::25].tolist()])
