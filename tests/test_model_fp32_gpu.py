"""Whole-model numerics: the fused bf16 Inception-v3 (every tony_amd HIP kernel on its hot path) vs the
stock fp32 PyTorch graph with identical weights (models/convert.py), one training step: logits, aux
logits and EVERY parameter gradient.  A 94-layer random-init net amplifies bf16 rounding, so the
yardstick is the stock graph run in bf16: the fused model must be about as close to fp32 as stock
bf16 is, layer by layer.
"""
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def test_inception_v3_train_step_matches_fp32_every_gradient(cuda):
    from tony_amd.models.convert import fused_grads_to_stock, stock_to_fused
    from tony_amd.models.inception_v3 import inception_v3
    from tony_amd.models.layers import cast_model

    torch.manual_seed(0)
    ref = inception_v3(num_classes=100, fused=False, seed=0)
    fused = inception_v3(num_classes=100, fused=True, seed=1)
    fused.load_state_dict(stock_to_fused(ref.state_dict(), fused))
    stock16 = inception_v3(num_classes=100, fused=False, seed=2)
    stock16.load_state_dict(ref.state_dict())
    models = {}
    for name, m, dt in (("ref", ref, torch.float32), ("fused", fused, torch.bfloat16),
                        ("stock16", stock16, torch.bfloat16)):
        m = cast_model(m, dt, cuda).to(memory_format=torch.channels_last).train()
        m.dropout.p = 0.0  # identical masks are impossible across graphs: no dropout
        models[name] = m
    # batch 32: the 8x8 layers still have 2048 GEMM rows, so every conv takes the tony kernels
    x = torch.randn(32, 3, 299, 299, device=cuda).contiguous(memory_format=torch.channels_last)
    w = torch.randn(32, 100, device=cuda)
    outs = {}
    for name, m in models.items():
        xi = x if name == "ref" else x.to(torch.bfloat16)
        logits, aux = m(xi)
        ((logits.float() * w).sum() + 0.4 * (aux.float() * w).sum()).backward()
        outs[name] = (logits.float(), aux.float())

    def rel(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()

    for i, what in enumerate(("logits", "aux")):
        rk, rs = rel(outs["fused"][i], outs["ref"][i]), rel(outs["stock16"][i], outs["ref"][i])
        assert rk < 1.5 * rs + 0.02, f"{what}: fused {rk:.4f} vs stock-bf16 {rs:.4f}"
    gk = fused_grads_to_stock(models["fused"], models["ref"])
    worst = []
    for name, p in models["ref"].named_parameters():
        gr = p.grad
        gs = dict(models["stock16"].named_parameters())[name].grad
        ek, es = rel(gk[name], gr), rel(gs, gr)
        worst.append((ek - (2.0 * es + 0.05), name, ek, es))
    worst.sort(reverse=True)
    bad = [w for w in worst if w[0] > 0]
    assert not bad, "gradients further from fp32 than 2x stock-bf16 + 0.05: " + ", ".join(
        f"{n} fused {ek:.3f} stock16 {es:.3f}" for _, n, ek, es in bad[:8])
    print("worst 5 (name, fused rel err, stock-bf16 rel err):",
          [(n, round(ek, 4), round(es, 4)) for _, n, ek, es in worst[:5]])
