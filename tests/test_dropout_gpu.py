"""Dropout with a device-side step counter (ops/dropout.py, csrc/dropout.hip).

The mask is a function of (seed, counter, element) and the counter is bumped by a kernel captured
with the step, so the native plan replay and hipGraph replay draw a new mask every step -- the same
sequence of masks an eager run draws (torch's philox dropout replays the capture-time mask
under the plan)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype,n", [(torch.bfloat16, 1 << 20), (torch.float32, 1 << 20), (torch.bfloat16, 1003),
                                     (torch.float32, 37)])
def test_dropout_kernel_matches_mask(cuda, dtype, n):
    from tony_amd.ops.dropout import dropout

    p = 0.5
    rng = torch.tensor([1234, 0], dtype=torch.int64, device=cuda)
    x = (torch.rand(n, device=cuda) + 0.5).to(dtype)  # no zeros: y == 0 <=> dropped
    x.requires_grad_(True)
    y = dropout(x, p, rng)
    keep = y.detach() != 0
    ref = torch.where(keep, x.detach().float() / (1 - p), torch.zeros((), device=cuda))
    torch.testing.assert_close(y.float(), ref, rtol=1e-2 if dtype == torch.bfloat16 else 1e-6, atol=0)
    if n >= 1 << 16:
        assert abs(keep.float().mean().item() - (1 - p)) < 0.01
    gy = torch.randn(n, device=cuda).to(dtype)
    y.backward(gy)
    gref = torch.where(keep, gy.float() / (1 - p), torch.zeros((), device=cuda))
    torch.testing.assert_close(x.grad.float(), gref, rtol=1e-2 if dtype == torch.bfloat16 else 1e-6, atol=0)
    assert int(rng[1].item()) == 1  # one forward = one bump


def test_dropout_counter_gives_fresh_deterministic_masks(cuda):
    from tony_amd.ops.dropout import dropout

    x = torch.ones(1 << 16, device=cuda, dtype=torch.bfloat16)
    rng = torch.tensor([99, 0], dtype=torch.int64, device=cuda)
    m1, m2 = (dropout(x, 0.3, rng) != 0 for _ in range(2))
    assert not torch.equal(m1, m2)
    rng2 = torch.tensor([99, 0], dtype=torch.int64, device=cuda)
    assert torch.equal(dropout(x, 0.3, rng2) != 0, m1)  # (seed, counter) fixes the mask
    rng3 = torch.tensor([100, 0], dtype=torch.int64, device=cuda)
    assert not torch.equal(dropout(x, 0.3, rng3) != 0, m1)
    assert abs(m1.float().mean().item() - 0.7) < 0.02


def _train(replay, monkeypatch, steps=5):
    import tony_amd.parallel.trainer as trainer_mod
    from tony_amd.models import inception_v3 as iv3
    from tony_amd.models.layers import init_weights
    from tony_amd.ops import cross_entropy
    from tony_amd.ops.dropout import Dropout
    from tony_amd.ops.pool import global_avg_pool
    from tony_amd.parallel.ps import ParameterServer

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.block = iv3.InceptionA(64, 32)
            self.drop = Dropout(0.5)
            self.fc = torch.nn.Linear(self.block.out_channels, 10)
            self.seen = None

        def forward(self, x):
            h = self.drop(global_avg_pool(self.block(x)))
            self.seen = h  # under replay: the captured (static) tensor the replays rewrite
            return self.fc(h)

    monkeypatch.setattr(trainer_mod, "REPLAY", replay or "plan")
    dev = torch.device("cuda", 0)
    model = init_weights(Net(), seed=0).to(dev).to(memory_format=torch.channels_last).train()
    model.drop.rng[0] = 4242
    ps = ParameterServer(model, optimizer="sgd", lr=0.05, momentum=0.9, device=dev)
    tr = trainer_mod.Trainer(model, ps, lambda o, y: cross_entropy(o, y), use_graph=replay is not None,
                             warmup_eager=1, graph_collectives=True if replay else None)
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn((16, 64, 35, 35), generator=g, device=dev).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), generator=g, device=dev)
    masks = []
    for _ in range(steps):
        tr.step(x, y)
        torch.cuda.synchronize()
        masks.append((model.seen != 0).clone())
    return masks, int(model.drop.rng[1].item()), tr


@pytest.mark.parametrize("replay", ["plan", "graph"])
def test_replayed_step_draws_a_new_mask_every_step(cuda, monkeypatch, replay):
    me, ce, _ = _train(None, monkeypatch)
    mr, cr, tr = _train(replay, monkeypatch)
    assert tr.replay_kind == replay, tr.plan_error
    assert ce == cr == len(me)  # one bump per executed forward (the capture itself executes nothing)
    for a, b in zip(mr, mr[1:]):
        assert not torch.equal(a, b), "a replay reused the previous step's dropout mask"
    for i, (a, b) in enumerate(zip(me, mr)):
        # same (seed, counter) -> same mask; values differ only where a kept activation is exactly 0
        agree = (a == b).float().mean().item()
        assert agree > 0.99, (i, agree)
