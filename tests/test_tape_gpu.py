"""Tape segments (ops/tape.py) vs per-op autograd on the fused bf16 Inception-v3: the same training
step with the stem / every Inception block replayed from a tape must give the same logits, the same
loss and the same parameter gradients (returned through autograd -- no flat gradient slots here --
and, with the branch and weight-gradient streams on, replayed on the streams the forward used)."""
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _step(model, x, w, use_tape, streams_on):
    from tony_amd.ops import streams, tape

    model.zero_grad(set_to_none=True)
    tape.ENABLED = use_tape
    try:
        on = streams_on and streams.begin(x.device, branches=True)
        logits, aux = model(x)
        loss = (logits.float() * w).sum() + 0.4 * (aux.float() * w).sum()
        loss.backward()
        if on:
            streams.end()
    finally:
        tape.ENABLED = False
    torch.cuda.synchronize()
    return logits.float(), {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("streams_on", [False, True])
def test_tape_segments_match_autograd(cuda, streams_on):
    from tony_amd.models.inception_v3 import inception_v3
    from tony_amd.models.layers import cast_model

    torch.manual_seed(0)
    m = cast_model(inception_v3(num_classes=100, fused=True, seed=3), torch.bfloat16, cuda)
    m = m.to(memory_format=torch.channels_last).train()
    m.dropout.p = 0.0
    x = torch.randn(32, 3, 299, 299, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(32, 100, device=cuda)
    _step(m, x, w, False, False)  # autotuning happens here, outside the compared steps
    state = {k: v.clone() for k, v in m.state_dict().items()}
    # the BN statistics are float atomics (order-dependent): two autograd runs set the noise floor
    runs = []
    for use_tape in (False, False, True):
        m.load_state_dict(state)  # the BN running statistics moved
        runs.append(_step(m, x, w, use_tape, streams_on))
    (l0, g0), (l1, g1), (lt, gt) = runs

    def rel(a, b):
        return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()

    assert set(gt) == set(g0) and len(gt) > 200, (len(gt), len(g0), sorted(set(gt) ^ set(g0))[:10])
    floor_l = rel(l1, l0)
    assert rel(lt, l0) <= 3 * floor_l + 1e-3, (rel(lt, l0), floor_l)
    worst = max((rel(gt[n], g0[n]) - 3 * rel(g1[n], g0[n]), n) for n in g0)
    assert worst[0] < 2e-2, f"gradient further from autograd than 3x run-to-run noise: {worst}"
