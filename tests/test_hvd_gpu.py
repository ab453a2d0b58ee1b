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


def test_fused_sgd_reseeds_master_after_external_weight_change(cuda, monkeypatch):
    """the fused SGD's fp32 master must follow weights changed outside ``step`` (a model
    load_state_dict / broadcast_parameters after the optimizer was built), and its state_dict /
    load_state_dict must carry the momentum (torch.optim.SGD's format)."""
    import tony_amd.hvd as hvd
    from tony_amd.ops import cross_entropy

    monkeypatch.setenv("HOROVOD_RANK", "0")
    monkeypatch.setenv("HOROVOD_SIZE", "1")
    hvd.init()
    dev = torch.device("cuda", 0)
    try:
        def net(seed):
            torch.manual_seed(seed)
            m = torch.nn.Sequential(torch.nn.Linear(64, 32), torch.nn.ReLU(), torch.nn.Linear(32, 16)).to(dev)
            return m.to(torch.bfloat16)

        g = torch.Generator(device=dev).manual_seed(1)
        x = torch.randn((8, 64), generator=g, device=dev).to(torch.bfloat16)
        y = torch.randint(0, 16, (8,), generator=g, device=dev)

        def step(model, opt):
            opt.zero_grad()
            cross_entropy(model(x), y).backward()
            opt.step()

        fused_model = net(0)
        fused = hvd.DistributedOptimizer(torch.optim.SGD(fused_model.parameters(), lr=0.1, momentum=0.9),
                                         named_parameters=fused_model.named_parameters(), fused=True)
        assert fused._fused
        new_weights = net(1).state_dict()
        fused_model.load_state_dict(new_weights)  # after the optimizer snapshotted its master
        step(fused_model, fused)
        ref_model = net(1)
        ref = torch.optim.SGD(ref_model.parameters(), lr=0.1, momentum=0.9)
        step(ref_model, ref)
        for a, b in zip(fused_model.parameters(), ref_model.parameters()):
            assert torch.allclose(a.float(), b.float(), rtol=2e-2, atol=2e-3), "master was not re-seeded"
        # momentum round trip through torch's state_dict format
        step(fused_model, fused)
        sd = fused.state_dict()
        assert len(sd["state"]) == 4 and all("momentum_buffer" in v for v in sd["state"].values())
        other = hvd.DistributedOptimizer(torch.optim.SGD(net(2).parameters(), lr=0.1, momentum=0.9), fused=True)
        other.load_state_dict(sd)
        for (fa, oa), (fb, ob) in zip(fused._fused, other._fused):
            assert torch.equal(oa.v, ob.v)
    finally:
        hvd.shutdown()
