"""ops/bn.py MaskedGrad: a residual tail's d(identity) = dY * (y > 0) held as dY + the forward's ReLU byte
mask (bit j of byte [m, c // 8] is channel 8 * (c // 8) + j); materialize() must reproduce the masked dY."""
import torch


def test_masked_grad_materialize_matches_dense_mask():
    from tony_amd.ops.bn import MaskedGrad

    torch.manual_seed(0)
    n, c, h, w = 2, 24, 3, 5
    dy = torch.randn(n, c, h, w).contiguous(memory_format=torch.channels_last)
    y = torch.randn(n, c, h, w)
    dense = (y > 0).permute(0, 2, 3, 1).reshape(n * h * w, c)  # rows [m, c]
    mask = torch.zeros(n * h * w, c // 8, dtype=torch.uint8)
    for j in range(8):
        mask |= dense.view(-1, c // 8, 8)[:, :, j].to(torch.uint8) << j
    out = MaskedGrad(dy, mask).materialize()
    assert out.shape == dy.shape
    torch.testing.assert_close(out, dy * (y > 0))


def test_grad_join_materializes_masked_for_plain_takers():
    from tony_amd.ops.bn import MaskedGrad
    from tony_amd.ops.residual import GradJoin

    dy = torch.ones(1, 8, 1, 2).contiguous(memory_format=torch.channels_last)
    mask = torch.tensor([[0b00000101], [0b11111111]], dtype=torch.uint8)
    j = GradJoin()
    assert j.wants_masked()
    assert j.park_masked(dy, mask) is None
    g = j.take()  # a taker without masked_ok gets a tensor
    assert not isinstance(g, MaskedGrad)
    assert g[0, :, 0, 0].tolist() == [1, 0, 1, 0, 0, 0, 0, 0] and g[0, :, 0, 1].tolist() == [1] * 8
    j2 = GradJoin()
    j2.park_masked(dy, mask)
    assert isinstance(j2.take(masked_ok=True), MaskedGrad)
