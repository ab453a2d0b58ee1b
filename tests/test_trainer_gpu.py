"""The HIP-graph trainer: a replayed step must train exactly like the eager step, whether the
PS push/apply/pull is captured inside the graph (1 rank) or runs eagerly after it (>1 rank)."""
import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu


class _Tiny(nn.Module):
    def __init__(self):
        super().__init__()
        from tony_amd.models.layers import ConvBNAct
        from tony_amd.ops.fused import FusedHead

        self.c1 = ConvBNAct(16, 32, 3, 1, 1)
        self.head = FusedHead(32, (32, 16), pool_cout=16)
        self.fc = nn.Linear(64, 10)

    def forward(self, x):
        a, b, p = self.head(self.c1(x))
        z = torch.cat([a, b, p], 1)
        return self.fc(torch.flatten(nn.functional.adaptive_avg_pool2d(z, 1), 1))


class _Block(nn.Module):
    """One Inception block (fused head, parallel branches, zero-copy concat) + classifier."""

    def __init__(self, kind="A"):
        super().__init__()
        from tony_amd.models import inception_v3 as iv3

        self.block = {"A": lambda: iv3.InceptionA(64, 32), "B": lambda: iv3.InceptionB(64),
                      "C": lambda: iv3.InceptionC(64, 32), "D": lambda: iv3.InceptionD(64),
                      "E": lambda: iv3.InceptionE(64)}[kind]()
        self.fc = nn.Linear(self.block.out_channels, 10)

    def forward(self, x):
        from tony_amd.ops.pool import global_avg_pool

        return self.fc(global_avg_pool(self.block(x)))


def _train(mode, steps=4, overlap=True, net=_Tiny, shape=(32, 16, 24, 24)):
    from tony_amd.models.layers import init_weights
    from tony_amd.ops import cross_entropy
    from tony_amd.parallel.ps import ParameterServer
    from tony_amd.parallel.trainer import Trainer

    dev = torch.device("cuda", 0)
    model = init_weights(net(), seed=0).to(dev).to(memory_format=torch.channels_last).train()
    ps = ParameterServer(model, optimizer="sgd", lr=0.05, momentum=0.9, device=dev)
    use_graph = mode != "eager"
    tr = Trainer(model, ps, lambda o, y: cross_entropy(o, y), use_graph=use_graph, warmup_eager=1,
                 graph_collectives=(mode == "graph_in") if use_graph else None, overlap_wgrad=overlap)
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(shape, generator=g, device=dev).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (shape[0],), generator=g, device=dev)
    losses = [float(tr.step(x, y).float().item()) for _ in range(steps)]
    torch.cuda.synchronize()
    if overlap and mode == "eager" and steps > 1:
        assert tr.side_ops > 0, "no weight gradient ran on the side stream"
    return losses, ps.flat.data.float().clone(), ps.steps


@pytest.mark.parametrize("mode,kind", [("eager", "A"), ("graph_in", "A"), ("eager", "B"), ("eager", "C"),
                                       ("eager", "D"), ("eager", "E")])
def test_wgrad_stream_overlap_matches_serial(cuda, mode, kind):
    """Weight gradients on the side stream and block branches on branch streams (ops/streams.py)
    train exactly like the serial single-stream step."""
    hw = {"A": 35, "B": 35, "C": 17, "D": 17, "E": 8}[kind]
    kw = dict(net=lambda: _Block(kind), shape=(max(8, 2048 // (hw * hw)), 64, hw, hw), steps=5)
    ls, ps_, _ = _train(mode, overlap=False, **kw)
    lo, po, _ = _train(mode, overlap=True, **kw)
    for a, b in zip(lo, ls):
        assert abs(a - b) <= 1e-2 * max(1.0, abs(b)), (lo, ls)
    err = (po - ps_).abs().max().item()
    assert err < 1e-2, err


def test_graph_replay_matches_eager(cuda):
    le, pe, se = _train("eager")
    for mode in ("graph_in", "graph_out"):
        lg, pg, sg = _train(mode)
        assert sg == se == 4, mode
        for a, b in zip(lg, le):
            assert abs(a - b) <= 2e-2 * max(1.0, abs(b)), (mode, lg, le)
        err = (pg - pe).abs().max().item()
        assert err < 2e-2, (mode, err)


def test_transpose_batch_matches_permute(cuda):
    from tony_amd.ops.wt_cache import TransposedWeights

    torch.manual_seed(0)
    shapes = [(192, 160, 7, 1), (48, 288, 1, 1), (80, 64, 3, 3), (2048 // 8, 72, 1, 3), (32, 32, 3, 3)]
    ws = [nn.Parameter(torch.randn(s, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
          for s in shapes]
    c = TransposedWeights(torch.device("cuda", 0))
    c.enabled = True
    for w in ws:
        assert torch.equal(c.get(w), w.permute(1, 2, 3, 0).contiguous())
    with torch.no_grad():
        for w in ws:
            w.mul_(-2.0).add_(1.0)  # the "optimizer step"
    c.refresh()
    torch.cuda.synchronize()
    for w in ws:
        assert torch.equal(c.get(w), w.permute(1, 2, 3, 0).contiguous())


def test_trainer_matches_plain_loop(cuda):
    """Trainer (arena, cached transposed weights) vs a plain PS loop with none of its machinery."""
    from tony_amd.models.layers import init_weights
    from tony_amd.ops import cross_entropy
    from tony_amd.parallel.ps import ParameterServer

    le, pe, _ = _train("eager")
    dev = torch.device("cuda", 0)
    model = init_weights(_Tiny(), seed=0).to(dev).to(memory_format=torch.channels_last).train()
    ps = ParameterServer(model, optimizer="sgd", lr=0.05, momentum=0.9, device=dev)
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn((32, 16, 24, 24), generator=g, device=dev).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,), generator=g, device=dev)
    losses = []
    for _ in range(4):
        ps.zero_grad()
        loss = cross_entropy(model(x), y)
        loss.backward()
        ps.step()
        losses.append(float(loss.float().item()))
    for a, b in zip(losses, le):
        assert abs(a - b) <= 2e-2 * max(1.0, abs(b)), (losses, le)
    assert (ps.flat.data.float() - pe).abs().max().item() < 2e-2


@pytest.mark.parametrize("block", ["A", "B", "C", "D", "E"])
def test_zero_copy_concat_matches_copy_path(cuda, block, monkeypatch):
    """Inception blocks writing branch outputs straight into the concat buffer == the copy path."""
    from tony_amd.models import inception_v3 as iv3
    from tony_amd.models.layers import init_weights
    from tony_amd.ops import concat

    mk = {"A": (lambda: iv3.InceptionA(192, 32), 35), "B": (lambda: iv3.InceptionB(288), 35),
          "C": (lambda: iv3.InceptionC(768, 128), 17), "D": (lambda: iv3.InceptionD(768), 17),
          "E": (lambda: iv3.InceptionE(1280), 8)}[block]
    cin = {"A": 192, "B": 288, "C": 768, "D": 768, "E": 1280}[block]
    torch.manual_seed(0)
    x0 = torch.randn(16, cin, mk[1], mk[1], device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)

    def run(zero_copy):
        m = init_weights(mk[0](), seed=1).to(cuda).to(memory_format=torch.channels_last).train()
        for p in m.parameters():
            p.data = p.data.to(torch.bfloat16)
        if not zero_copy:
            monkeypatch.setattr(concat, "take", lambda *a, **k: None)
        x = x0.clone().requires_grad_(True)
        y = m(x)
        g = torch.randn(y.shape, device=cuda, generator=torch.Generator(device=cuda).manual_seed(3))
        (y.float() * g).sum().backward()
        monkeypatch.undo()
        return y.detach().float(), x.grad.float()

    y1, g1 = run(True)
    y2, g2 = run(False)
    # the two paths may pick different autotuned kernels: allow one bf16 ulp of the output scale
    assert ((y1 - y2).abs() <= 5e-2 + 2 ** -7 * y2.abs()).all().item(), (y1 - y2).abs().max().item()
    # input gradients pass 2-5 bf16 conv+BN backward layers whose BN statistics are summed with
    # float atomics (order-dependent): a few % relative difference is rounding, not a wrong slice
    assert ((g1 - g2).norm() / g2.norm()).item() < 4e-2
