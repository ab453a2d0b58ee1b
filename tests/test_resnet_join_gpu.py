"""ResNet blocks: the consumer of the block input whose backward runs second adds its dX into the
gradient the first one parked, in its dgrad epilogue (ops/residual.py GradJoin, csrc/mfma_common.h accum)
instead of autograd's add kernel -- the block input gradient must match the unjoined graph's (to bf16 rounding: the BN
statistics are summed with atomics, so two runs may differ in the last bit; a lost contribution
of either consumer is off by far more)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _close_but_flips(a, b):
    """Elementwise within 1e-2, except where a ReLU of the block took the other side between the two
    runs (its BN statistics are summed with atomics: a pre-activation within their last bit of 0
    can flip) -- a handful of elements, against a lost consumer contribution that moves them all."""
    bad = ~torch.isclose(a, b, rtol=1e-2, atol=1e-2)
    assert bad.float().mean().item() < 1e-3, f"{int(bad.sum())} of {bad.numel()} elements differ"
    assert ((a - b).norm() / b.norm()).item() < 5e-3


@pytest.mark.parametrize("shape", [(4, 256, 14, 14, 1, 64), (2, 512, 7, 9, 1, 128), (4, 64, 16, 16, 1, 64),
                                   (4, 256, 16, 16, 2, 128)],
                         ids=["identity-256", "identity-512", "projection-s1", "projection-s2"])
@pytest.mark.parametrize("masked", [True, False], ids=["masked", "dres"])
def test_identity_block_join_matches_autograd_sum(cuda, shape, masked, monkeypatch):
    from tony_amd.models import resnet
    from tony_amd.models.layers import cast_model, init_weights

    n, c, h, w, stride, width = shape
    torch.manual_seed(0)
    blk = cast_model(init_weights(resnet.Bottleneck(c, width, stride=stride), 5), torch.bfloat16, cuda)
    blk = blk.to(memory_format=torch.channels_last).train()
    torch.nn.init.constant_(blk.bn3.weight, 0.5)  # non-degenerate residual branch
    x0 = _cl(torch.randn(n, c, h, w, device=cuda)).to(torch.bfloat16)
    oh, ow = (h - 1) // stride + 1, (w - 1) // stride + 1
    g = _cl(torch.randn(n, 4 * width, oh, ow, device=cuda)).to(torch.bfloat16)
    grads = {}
    from tony_amd.ops import residual

    # the joined run parks the residual tail's dY + ReLU mask for conv1's dgrad epilogue (MaskedGrad),
    # which must read them there: no materialised fallback
    if masked:
        from tony_amd.ops.bn import MaskedGrad

        def _no_materialize(self):
            raise AssertionError("MaskedGrad materialised: the dgrad epilogue did not take it")
        monkeypatch.setattr(MaskedGrad, "materialize", _no_materialize)
    for join in (False, True):
        monkeypatch.setattr(resnet, "JOIN", join)
        monkeypatch.setattr(resnet, "DS_TONY", True)
        monkeypatch.setattr(residual, "MASKED_JOIN", masked)
        blk.zero_grad(set_to_none=True)
        x = (x0 * 1).requires_grad_(True)  # a non-leaf copy per run (the join rides on the tensor)
        x.retain_grad()
        y = blk(x)
        y.backward(g)
        grads[join] = (x.grad.float().clone(), [p.grad.float().clone() for p in blk.parameters()])
    _close_but_flips(grads[True][0], grads[False][0])
    # parameter gradients by norm: between two runs a pre-activation within the atomically summed BN
    # statistics' last bit of 0 may take the other side of a ReLU and move single dW elements
    for a, b in zip(grads[True][1], grads[False][1]):
        assert ((a - b).norm() / b.norm().clamp_min(1e-12)).item() < 2e-2


@pytest.mark.parametrize("block", ["B", "D", "E"])
def test_inception_block_join_matches_autograd_sum(cuda, block, monkeypatch):
    """Inception's reduction blocks (input -> 1x1 head / 3x3-s2 conv / max pool: 3 or 2 consumers) and
    the E block's 1x3 / 3x1 splits: the joined input gradient matches autograd's sum."""
    from tony_amd.models import inception_v3 as iv3
    from tony_amd.models.layers import cast_model, init_weights

    torch.manual_seed(0)
    cin, hw, make = {"B": (288, 35, lambda: iv3.InceptionB(288)), "D": (768, 17, lambda: iv3.InceptionD(768)),
                     "E": (1280, 8, lambda: iv3.InceptionE(1280))}[block]
    blk = cast_model(init_weights(make(), 7), torch.bfloat16, cuda).to(memory_format=torch.channels_last).train()
    x0 = _cl(torch.randn(8, cin, hw, hw, device=cuda)).to(torch.bfloat16)
    grads = {}
    for join in (False, True):
        monkeypatch.setattr(iv3, "JOIN", join)
        blk.zero_grad(set_to_none=True)
        x = (x0 * 1).requires_grad_(True)
        y = blk(x)
        g = _cl(torch.randn(y.shape, device=cuda, generator=torch.Generator(device=cuda).manual_seed(1))).to(y.dtype)
        y.backward(g)
        torch.cuda.synchronize()
        grads[join] = (x.grad.float().clone(), [p.grad.float().clone() for p in blk.parameters()])
    a, b = grads[True][0], grads[False][0]
    assert ((a - b).norm() / b.norm()).item() < 1e-2
    for pa, pb in zip(grads[True][1], grads[False][1]):
        assert ((pa - pb).norm() / pb.norm().clamp_min(1e-12)).item() < 2e-2
