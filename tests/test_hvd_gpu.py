"""Horovod API on the GPU: DistributedOptimizer's fused HIP SGD apply == torch.optim.SGD (1 rank)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(fused, steps=3):
    import tony_amd.hvd as hvd
    from tony_amd.models.layers import ConvBNAct, init_weights
    from tony_amd.ops import cross_entropy
    from tony_amd.ops.pool import global_avg_pool

    dev = torch.device("cuda", 0)

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.c1 = ConvBNAct(16, 32, 3, 1, 1)
            self.c2 = ConvBNAct(32, 64, 3, 2, 1)
            self.fc = torch.nn.Linear(64, 10)

        def forward(self, x):
            return self.fc(global_avg_pool(self.c2(self.c1(x))))

    model = init_weights(Net(), seed=3).to(dev).to(memory_format=torch.channels_last).train()
    for p in model.parameters():
        p.data = p.data.to(torch.bfloat16)
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters(), fused=fused)
    assert bool(opt._fused) == fused
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn((8, 16, 20, 20), generator=g, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), generator=g, device=dev)
    for _ in range(steps):
        opt.zero_grad()
        cross_entropy(model(x), y).backward()
        opt.step()
    torch.cuda.synchronize()
    return torch.cat([p.detach().float().reshape(-1) for p in model.parameters()])


def test_distributed_optimizer_fused_sgd_matches_torch_sgd(cuda, monkeypatch):
    import tony_amd.hvd as hvd

    monkeypatch.setenv("HOROVOD_RANK", "0")
    monkeypatch.setenv("HOROVOD_SIZE", "1")
    hvd.init()
    try:
        a = _train(fused=True)
        b = _train(fused=False)   # torch SGD on the bf16 parameters
    finally:
        hvd.shutdown()
    # the fused path keeps an fp32 master copy; torch's bf16 in-place update rounds every step
    assert ((a - b).abs() <= 2e-2 + 2e-2 * b.abs()).all(), (a - b).abs().max().item()
