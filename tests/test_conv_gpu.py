"""Implicit-GEMM conv kernels (csrc/conv.hip) vs PyTorch fp32 references, and the fused conv+BN layer."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (N, Cin, H, W, Cout, (R, S), stride, (ph, pw)) -- the Inception-v3 / ResNet-50 conv shapes, shrunk in N
SHAPES = [
    (4, 32, 37, 37, 64, (3, 3), 1, (1, 1)),
    (2, 64, 35, 35, 96, (3, 3), 1, (1, 1)),
    (2, 48, 35, 35, 64, (5, 5), 1, (2, 2)),
    (2, 128, 17, 17, 192, (1, 7), 1, (0, 3)),
    (2, 160, 17, 17, 160, (7, 1), 1, (3, 0)),
    (2, 384, 8, 8, 384, (1, 3), 1, (0, 1)),
    (2, 448, 8, 8, 384, (3, 3), 1, (1, 1)),
    (2, 288, 35, 35, 384, (3, 3), 2, (0, 0)),
    (2, 64, 56, 56, 64, (3, 3), 1, (1, 1)),
    (2, 128, 28, 28, 128, (3, 3), 2, (1, 1)),
    (3, 32, 149, 149, 32, (3, 3), 1, (0, 0)),
    (2, 80, 73, 73, 192, (3, 3), 1, (0, 0)),
    # strided backward-data: one tony launch per residue class of dX (no MIOpen)
    (2, 96, 35, 35, 96, (3, 3), 2, (0, 0)),        # Mixed_6a double-3x3 tail
    (2, 192, 17, 17, 320, (3, 3), 2, (0, 0)),      # Mixed_7a
    (2, 256, 56, 56, 512, (1, 1), 2, (0, 0)),      # ResNet downsample: odd classes get no taps (zeros)
    (2, 64, 57, 57, 64, (3, 3), 2, (1, 1)),        # odd size + padding
    (2, 32, 20, 20, 48, (5, 5), 3, (2, 2)),        # stride 3: nine classes
    # tiny output images (OH * OW < 32 + OW): the wgrad's general row walk, not the incremental one
    (5, 128, 5, 5, 128, (3, 3), 1, (0, 0)),
    (3, 128, 12, 9, 160, (3, 3), 2, (1, 1)),
]


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("shape", SHAPES, ids=[f"{s[1]}x{s[2]}k{s[5][0]}{s[5][1]}s{s[6]}" for s in SHAPES])
def test_conv_fwd_dgrad_wgrad(cuda, shape):
    from tony_amd.ops.conv import conv_dgrad, conv_fwd, conv_wgrad

    n, ci, h, w, co, (r, s), st, (ph, pw) = shape
    torch.manual_seed(0)
    x = _nhwc(torch.randn(n, ci, h, w, device=cuda)).to(torch.bfloat16)
    wt = _nhwc(torch.randn(co, ci, r, s, device=cuda) / (ci * r * s) ** 0.5).to(torch.bfloat16)
    xr, wr = x.float().requires_grad_(True), wt.float().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, None, st, (ph, pw))
    from tony_amd.ops import _lib

    stats = torch.zeros(_lib.stat_floats(co), device=cuda)  # accumulated into: zero on entry
    y = conv_fwd(x, wt, st, (ph, pw), stats)
    stats = _lib.fold_stats(stats, co)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, yr) < 1e-2, f"fwd rel {_rel(y, yr):.4f}"
    torch.testing.assert_close(stats[:co], yr.sum((0, 2, 3)), rtol=2e-2, atol=2e-2 * (yr.numel() / co) ** 0.5)
    torch.testing.assert_close(stats[co:], (yr * yr).sum((0, 2, 3)), rtol=2e-2, atol=1.0)
    dy = _nhwc(torch.randn_like(yr)).to(torch.bfloat16)
    yr.backward(dy.float())
    dx = conv_dgrad(dy, wt, x.shape, st, (ph, pw))
    assert _rel(dx, xr.grad) < 1e-2, f"dgrad rel {_rel(dx, xr.grad):.4f}"
    dw = conv_wgrad(dy, x, wt.shape, st, (ph, pw))
    assert dw.shape == wt.shape
    assert _rel(dw, wr.grad) < 1e-2, f"wgrad rel {_rel(dw, wr.grad):.4f}"


ACC_SHAPES = [SHAPES[1], SHAPES[8], SHAPES[7], SHAPES[14], SHAPES[16], SHAPES[18]]


@pytest.mark.parametrize("shape", ACC_SHAPES, ids=[f"{s[1]}x{s[2]}k{s[5][0]}{s[5][1]}s{s[6]}" for s in ACC_SHAPES])
def test_conv_dgrad_accumulates_into_gradient(cuda, shape):
    """conv_dgrad(accum=g) returns g + dX, summed in the epilogue (flag bit 4) -- stride 1 and the
    strided per-residue-class launches, whose tap-less classes are then skipped (g kept there)."""
    from tony_amd.ops.conv import conv_dgrad

    n, ci, h, w, co, (r, s), st, (ph, pw) = shape
    torch.manual_seed(1)
    oh, ow = (h + 2 * ph - r) // st + 1, (w + 2 * pw - s) // st + 1
    wt = _nhwc(torch.randn(co, ci, r, s, device=cuda) / (ci * r * s) ** 0.5).to(torch.bfloat16)
    dy = _nhwc(torch.randn(n, co, oh, ow, device=cuda)).to(torch.bfloat16)
    g = _nhwc(torch.randn(n, ci, h, w, device=cuda)).to(torch.bfloat16)
    ref = g.float() + conv_dgrad(dy, wt, (n, ci, h, w), st, (ph, pw)).float()
    ptr = g.data_ptr()
    out = conv_dgrad(dy, wt, (n, ci, h, w), st, (ph, pw), accum=g)
    assert out.data_ptr() == ptr
    # one bf16 rounding of the fp32 sum vs the add of two bf16 tensors: within 2 bf16 ulps
    torch.testing.assert_close(out.float(), ref, rtol=1.6e-2, atol=1.6e-2)


def test_conv_on_channel_slice_input(cuda):
    """The input may be a channel slice of a concat buffer (pixel stride > C)."""
    from tony_amd.ops.conv import conv_fwd

    big = _nhwc(torch.randn(2, 96, 17, 17, device=cuda)).to(torch.bfloat16)
    x = big[:, 32:96]
    wt = _nhwc(torch.randn(48, 64, 3, 3, device=cuda) * 0.05).to(torch.bfloat16)
    y = conv_fwd(x, wt, 1, 1)
    yr = torch.nn.functional.conv2d(x.float(), wt.float(), None, 1, 1)
    assert _rel(y, yr) < 1e-2


@pytest.mark.parametrize("relu", [True, False])
def test_conv_bn_act_fused_matches_reference(cuda, relu):
    from tony_amd.ops import _lib
    from tony_amd.ops.conv import conv_bn_act

    torch.manual_seed(1)
    n, ci, h, w, co = 4, 64, 35, 35, 96
    x = _nhwc(torch.randn(n, ci, h, w, device=cuda)).to(torch.bfloat16)
    conv = torch.nn.Conv2d(ci, co, 3, 1, 1, bias=False).to(cuda)
    bn = torch.nn.BatchNorm2d(co, eps=1e-3).to(cuda)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    wt = _nhwc(conv.weight.detach()).to(torch.bfloat16).requires_grad_(True)
    g = bn.weight.detach().to(torch.bfloat16).requires_grad_(True)
    b = bn.bias.detach().to(torch.bfloat16).requires_grad_(True)
    rm, rv = torch.zeros(co, device=cuda), torch.ones(co, device=cuda)
    _lib.set_inplace_grads(False)
    try:
        xk = x.detach().requires_grad_(True)
        y = conv_bn_act(xk, wt, g, b, rm, rv, 1, 1, True, 0.1, 1e-3, relu)
        xr = x.float().requires_grad_(True)
        wr, gr, br = wt.detach().float().requires_grad_(True), g.detach().float().requires_grad_(True), \
            b.detach().float().requires_grad_(True)
        rm_r, rv_r = torch.zeros(co, device=cuda), torch.ones(co, device=cuda)
        yr = torch.nn.functional.batch_norm(torch.nn.functional.conv2d(xr, wr, None, 1, 1), rm_r, rv_r, gr, br,
                                            True, 0.1, 1e-3)
        yr = torch.relu(yr) if relu else yr
        assert _rel(y, yr) < 2e-2
        torch.testing.assert_close(rm, rm_r, rtol=2e-2, atol=2e-3)
        dy = _nhwc(torch.randn_like(yr)).to(torch.bfloat16)
        y.backward(dy)
        yr.backward(dy.float())
        assert _rel(xk.grad, xr.grad) < 3e-2
        assert _rel(wt.grad, wr.grad) < 3e-2
        assert _rel(g.grad, gr.grad) < 3e-2 and _rel(b.grad, br.grad) < 3e-2
    finally:
        _lib.set_inplace_grads(True)


def test_inception_tony_convs_match_miopen_convs(cuda):
    """The same fused Inception-v3 with its spatial convs on tony_amd's kernels vs on MIOpen (A/B in one
    model): forward logits and a weight gradient must agree to bf16 rounding."""
    from tony_amd.models import layers
    from tony_amd.models.inception_v3 import inception_v3
    from tony_amd.models.layers import cast_model

    torch.manual_seed(0)
    model = cast_model(inception_v3(num_classes=10, fused=True, seed=0), torch.bfloat16, cuda).to(
        memory_format=torch.channels_last)
    # Per layer, on the layer's real input (a random-init 90-layer net amplifies bf16 rounding differences
    # between any two kernels, so whole-model logits are no test): every ConvBNAct runs both ways.
    orig = layers.ConvBNAct.forward
    names = {m: n for n, m in model.named_modules()}
    rels = []

    def both(self, x, slot=None):  # slot ignored: the block copies the (MIOpen) result into its buffer
        saved = self.bn.running_mean.clone(), self.bn.running_var.clone()
        layers.USE_TONY_CONV = True
        a = orig(self, x)
        self.bn.running_mean.copy_(saved[0])
        self.bn.running_var.copy_(saved[1])
        layers.USE_TONY_CONV = False
        b = orig(self, x)
        rels.append((_rel(a, b), names.get(self, "?")))
        return b

    old = layers.USE_TONY_CONV
    layers.ConvBNAct.forward = both
    try:
        with torch.no_grad():
            model(_nhwc(torch.randn(8, 3, 299, 299, device=cuda)).to(torch.bfloat16))
    finally:
        layers.ConvBNAct.forward = orig
        layers.USE_TONY_CONV = old
    assert len(rels) > 40
    worst = max(rels)
    assert worst[0] < 2e-2, f"layer {worst[1]} differs by {worst[0]:.4f}"


@pytest.mark.parametrize("cfg", [(4, 64, 35, 35, 96, (3, 3), 1, (1, 1)), (2, 160, 17, 17, 192, (7, 1), 1, (3, 0)),
                                 (2, 288, 35, 35, 384, (3, 3), 2, (0, 0)), (3, 256, 9, 9, 80, (1, 1), 1, (0, 0)),
                                 (1, 384, 8, 8, 384, (1, 3), 1, (0, 1))])
@pytest.mark.parametrize("relu", [True, False])
def test_conv_bn_act_infer_folded_epilogue(cuda, cfg, relu):
    """Inference conv + BN(running stats) + ReLU in one kernel (H5) vs fp32 conv2d + batch_norm."""
    from tony_amd.ops import concat
    from tony_amd.ops.conv import conv_bn_act_infer

    n, ci, h, w, co, k, st, pad = cfg
    torch.manual_seed(11)
    x = torch.randn(n, ci, h, w, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(co, ci, *k, device=cuda) * (ci * k[0] * k[1]) ** -0.5).to(torch.bfloat16)
    wt = wt.contiguous(memory_format=torch.channels_last)
    g, b = torch.rand(co, device=cuda) + 0.5, torch.randn(co, device=cuda) * 0.1
    rm, rv = torch.randn(co, device=cuda) * 0.1, torch.rand(co, device=cuda) + 0.5
    with torch.no_grad():
        ref = torch.nn.functional.conv2d(x.float(), wt.float(), None, st, pad)
        ref = torch.nn.functional.batch_norm(ref, rm, rv, g, b, False, 0.0, 1e-3)
        ref = torch.relu(ref) if relu else ref
        y = conv_bn_act_infer(x, wt, g, b, rm, rv, st, pad, 1e-3, relu)
        assert y.is_contiguous(memory_format=torch.channels_last)
        torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
        # straight into a channel slice of a wider concat buffer
        buf = concat.concat_buffer(n, co + 32, ref.shape[2], ref.shape[3], x)
        ys = conv_bn_act_infer(x, wt, g, b, rm, rv, st, pad, 1e-3, relu, slot=concat.Slot(buf, 32))
        assert ys.data_ptr() == buf[:, 32:].data_ptr()
        torch.testing.assert_close(buf[:, 32:].float(), ref, rtol=2e-2, atol=2e-2)


def test_inception_eval_folded_matches_unfolded(cuda):
    """Inception-v3 eval under no_grad (folded-BN epilogues) == eval with autograd on (separate BN apply)."""
    from tony_amd.models.inception_v3 import inception_v3

    m = inception_v3(seed=3).to(cuda).to(memory_format=torch.channels_last)
    for p in m.parameters():
        p.data = p.data.to(torch.bfloat16)
    m.train()
    x = torch.randn(8, 3, 299, 299, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    m(x)  # one training forward: non-trivial running statistics
    m.eval()
    with torch.no_grad():
        y_fold = m(x).float()
    y_ref = m(x).float().detach()
    err = ((y_fold - y_ref).norm() / y_ref.norm()).item()
    assert err < 3e-2, err


@pytest.mark.parametrize("shape", [(2, 32, 37, 35, 32, 0), (2, 32, 19, 21, 64, 1), (2, 64, 17, 33, 64, 1),
                                   (1, 64, 9, 9, 32, 0), (3, 32, 24, 16, 64, 1)])
def test_halo_tile_conv3x3(cuda, shape):
    """The halo-tile 3x3 kernel (tile variant 9, csrc/conv.hip conv_halo_kernel) for fwd (+BN statistics)
    and dgrad vs fp32 references, including partial edge blocks and both paddings."""
    from tony_amd.ops import _lib
    from tony_amd.ops.conv import conv_dgrad, conv_fwd

    n, ci, h, w, co, p = shape
    torch.manual_seed(5)
    x = _nhwc(torch.randn(n, ci, h, w, device=cuda)).to(torch.bfloat16)
    wt = _nhwc(torch.randn(co, ci, 3, 3, device=cuda) / (ci * 9) ** 0.5).to(torch.bfloat16)
    xr, wr = x.float().requires_grad_(True), wt.float()
    yr = torch.nn.functional.conv2d(xr, wr, None, 1, p)
    stats = torch.zeros(_lib.stat_floats(co), device=cuda)
    y = conv_fwd(x, wt, 1, p, stats, vflags=9 << 8)
    assert _rel(y, yr) < 1e-2, f"halo fwd rel {_rel(y, yr):.4f}"
    st = _lib.fold_stats(stats, co)
    torch.testing.assert_close(st[:co], yr.sum((0, 2, 3)), rtol=2e-2, atol=2e-2 * (yr.numel() / co) ** 0.5)
    torch.testing.assert_close(st[co:], (yr * yr).sum((0, 2, 3)), rtol=2e-2, atol=1.0)
    dy = _nhwc(torch.randn_like(yr)).to(torch.bfloat16)
    yr.backward(dy.float())
    if co in (32, 64):  # dgrad runs the kernel with Cin' = co
        dx = conv_dgrad(dy, wt, x.shape, 1, p, vflags=9 << 8)
        assert _rel(dx, xr.grad) < 1e-2, f"halo dgrad rel {_rel(dx, xr.grad):.4f}"


@pytest.mark.parametrize("mode", ["gather", "dy", "bnred"])
@pytest.mark.parametrize("shape", [(2, 32, 37, 37, 64, 1), (2, 80, 35, 35, 192, 0)])  # M >= MIN_ROWS: both paths on tony kernels
def test_conv_bn_act_pool_fused_matches_unfused(cuda, shape, mode, monkeypatch):
    """conv -> BN -> ReLU -> maxpool 3x3/2 as one BN+ReLU+pool kernel == conv_bn_act then max_pool
    (outputs, running statistics, input / weight / gamma / beta gradients).  Backward modes: the pooled
    gradient gathered inside the BN reduce and apply (default), the full-resolution dY written by the
    pool backward, and that dY with the BN reduction fused into the pool backward."""
    from tony_amd.ops import conv as conv_mod
    from tony_amd.ops.conv import conv_bn_act, conv_bn_act_pool

    monkeypatch.setattr(conv_mod, "POOL_BN_GATHER", mode == "gather")
    monkeypatch.setattr(conv_mod, "POOL_BNRED", mode == "bnred")
    from tony_amd.ops.pool import max_pool

    n, ci, h, w, co, p = shape
    torch.manual_seed(6)
    x0 = _nhwc(torch.randn(n, ci, h, w, device=cuda)).to(torch.bfloat16)
    w0 = _nhwc(torch.randn(co, ci, 3, 3, device=cuda) / (ci * 9) ** 0.5).to(torch.bfloat16)
    g0 = (torch.rand(co, device=cuda) + 0.5)
    b0 = torch.randn(co, device=cuda) * 0.1

    def run(fused):
        x = x0.clone().requires_grad_(True)
        wt = torch.nn.Parameter(w0.clone())
        g, b = torch.nn.Parameter(g0.clone()), torch.nn.Parameter(b0.clone())
        rm, rv = torch.zeros(co, device=cuda), torch.ones(co, device=cuda)
        if fused:
            y = conv_bn_act_pool(x, wt, g, b, rm, rv, 1, p, 0.1, 1e-3, 3, 2)
        else:
            y = max_pool(conv_bn_act(x, wt, g, b, rm, rv, 1, p, True, 0.1, 1e-3, True), 3, 2)
        gy = torch.randn(y.shape, device=cuda, generator=torch.Generator(device=cuda).manual_seed(2))
        (y.float() * gy).sum().backward()
        return y.detach().float(), rm, rv, x.grad.float(), wt.grad.float(), g.grad.float(), b.grad.float()

    fu, ref = run(True), run(False)
    assert torch.equal(fu[0], ref[0]), "pooled outputs differ"
    torch.testing.assert_close(fu[1], ref[1], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(fu[2], ref[2], rtol=1e-5, atol=1e-6)
    for a, b, what in zip(fu[3:], ref[3:], ("dx", "dw", "dgamma", "dbeta")):
        assert _rel(a, b) < 2e-2, f"{what} rel {_rel(a, b):.4f}"


# (N, H, W, (R, S), stride, (ph, pw), Cout): Inception-v3's 3x3/2 stem (shrunk in N and H/W, with a
# partial last workgroup and workgroups straddling two images), ResNet's 7x7/2 p3 stem (5 K steps,
# 3 wgrad column groups) at 45x33 / 56x56 / 64x64 (the whole-model test's shape) / 224x224, and
# padded 3x3 stems at stride 2 and stride 1.  Images taller than 63 rows with padding are the case
# the round-2 K-padding-column bug read outside the staged rows (csrc/stem.hip tap_word).
STEM_SHAPES = [(2, 299, 299, (3, 3), 2, (0, 0), 32), (3, 37, 41, (3, 3), 2, (0, 0), 32),
               (2, 45, 33, (7, 7), 2, (3, 3), 64), (4, 64, 64, (3, 3), 2, (1, 1), 32),
               (3, 56, 56, (7, 7), 2, (3, 3), 64), (4, 64, 64, (7, 7), 2, (3, 3), 64),
               (2, 224, 224, (7, 7), 2, (3, 3), 64), (4, 64, 64, (3, 3), 1, (1, 1), 32),
               (2, 80, 72, (3, 3), 1, (1, 1), 64)]


@pytest.mark.parametrize("shape", STEM_SHAPES, ids=[f"{s[1]}x{s[2]}k{s[3][0]}s{s[4]}c{s[6]}" for s in STEM_SHAPES])
def test_stem_fwd_wgrad_mfma(cuda, shape):
    """csrc/stem.hip: MFMA stem forward (+ BN statistics epilogue) and split-K weight gradient vs fp32."""
    from tony_amd.ops import _lib
    from tony_amd.ops.conv import stem_fwd, stem_supported, stem_wgrad

    n, h, w, k, s, p, co = shape
    torch.manual_seed(3)
    x = _nhwc(torch.randn(n, 3, h, w, device=cuda)).to(torch.bfloat16)
    wt = _nhwc(0.2 * torch.randn(co, 3, *k, device=cuda)).to(torch.bfloat16)
    assert stem_supported(x, wt, s, p)
    stats = torch.zeros(_lib.stat_floats(co), device=cuda)
    y = stem_fwd(x, wt, s, p, stats)
    xr = x.float().requires_grad_(False)
    wr = wt.float().requires_grad_(True)
    ref = torch.nn.functional.conv2d(xr, wr, None, s, p)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, ref) < 1e-2
    st = _lib.fold_stats(stats, co)
    torch.testing.assert_close(st[:co], ref.sum((0, 2, 3)), rtol=1e-3, atol=ref.numel() / co * 1e-4)
    torch.testing.assert_close(st[co:], (ref * ref).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    dy = _nhwc(torch.randn_like(ref)).to(torch.bfloat16)
    ref.backward(dy.float())
    dw = stem_wgrad(dy, x, wt.shape, s, p)
    assert dw.shape == wt.shape and _rel(dw, wr.grad) < 1e-2
    # accumulate into a bf16 channels_last gradient slot
    slot = _nhwc(torch.ones_like(wt))
    assert stem_wgrad(dy, x, wt.shape, s, p, dst=slot) is None
    assert _rel(slot.float() - 1.0, wr.grad) < 2e-2


@pytest.mark.parametrize("shape", STEM_SHAPES[3:], ids=[f"{s[1]}x{s[2]}k{s[3][0]}s{s[4]}p{s[5][0]}" for s in STEM_SHAPES[3:]])
def test_stem_ignores_nan_outside_the_image(cuda, shape):
    """Regression for the round-2 stem bug: the padded stem must never read an element outside the image.
    The image sits inside a NaN-filled allocation (global memory around it is NaN) and an all-NaN image
    of the same shape runs first (the staged-row LDS of every CU is left full of NaN).  Any read outside
    the input's in-image taps then shows up as a non-finite output row or statistic."""
    from tony_amd.ops import _lib
    from tony_amd.ops.conv import stem_fwd, stem_wgrad

    n, h, w, k, s, p, co = shape
    torch.manual_seed(5)
    numel = n * h * w * 3
    pad = 64 * 1024  # elements of NaN on each side (more than the widest tap reach)
    buf = torch.full((numel + 2 * pad,), float("nan"), dtype=torch.bfloat16, device=cuda)
    x = buf[pad:pad + numel].view(n, h, w, 3).permute(0, 3, 1, 2)  # channels_last view inside the NaN sea
    x.copy_(torch.randn(n, 3, h, w, device=cuda))
    assert x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0
    wt = _nhwc(0.2 * torch.randn(co, 3, *k, device=cuda)).to(torch.bfloat16)
    poison = torch.full_like(x, float("nan")).contiguous(memory_format=torch.channels_last)
    stem_fwd(poison, wt, s, p, torch.zeros(_lib.stat_floats(co), device=cuda))  # NaN into the LDS staging
    stats = torch.zeros(_lib.stat_floats(co), device=cuda)
    y = stem_fwd(x, wt, s, p, stats)
    torch.cuda.synchronize()
    assert torch.isfinite(y.float()).all(), "stem forward read outside the image"
    assert torch.isfinite(stats).all(), "stem statistics read outside the image"
    ref = torch.nn.functional.conv2d(x.float(), wt.float(), None, s, p)
    assert _rel(y, ref) < 1e-2
    dy = _nhwc(torch.randn_like(ref)).to(torch.bfloat16)
    stem_wgrad(dy, poison, wt.shape, s, p)  # NaN into the wgrad kernel's LDS
    dw = stem_wgrad(dy, x, wt.shape, s, p)
    assert torch.isfinite(dw).all(), "stem weight gradient read outside the image"
    wr = wt.float().requires_grad_(True)
    torch.nn.functional.conv2d(x.float(), wr, None, s, p).backward(dy.float())
    assert _rel(dw, wr.grad) < 1e-2


def test_fused_relu_propagates_nan(cuda):
    """The fused BN+ReLU keeps a NaN a NaN (torch.relu semantics): an upstream NaN must surface as a
    non-finite activation, not as the silent all-zero output fmaxf(NaN, 0) = 0 produced in round 2."""
    from tony_amd.ops.bn import bn_act

    x = _nhwc(torch.randn(2, 16, 4, 4, device=cuda)).to(torch.bfloat16)
    x[0, 3, 1, 1] = float("nan")
    g, b = torch.ones(16, device=cuda), torch.zeros(16, device=cuda)
    y = bn_act(x, g, b, None, None, True, 0.1, 1e-5, True)
    assert torch.isnan(y[:, 3].float()).all(), "NaN in channel 3's statistics must reach its outputs"
    assert torch.isfinite(y[:, 2].float()).all()


@pytest.mark.parametrize("shape", [(4, 64, 64), (2, 224, 224)], ids=["64", "224"])
def test_resnet_stem_conv_bn_relu_padded_pool_fused(cuda, shape):
    """ResNet's stem as ONE conv + BN + ReLU + 3x3/2 p1 max-pool fusion (MFMA stem kernel + the padded
    bn_relu_maxpool kernel) == conv_bn_act then the padded max pool (outputs, running stats, gradients)."""
    from tony_amd.ops import _lib
    from tony_amd.ops.conv import conv_bn_act, conv_bn_act_pool
    from tony_amd.ops.pool import max_pool

    n, h, w = shape
    co = 64
    torch.manual_seed(9)
    x0 = _nhwc(torch.randn(n, 3, h, w, device=cuda)).to(torch.bfloat16)
    w0 = _nhwc(torch.randn(co, 3, 7, 7, device=cuda) / (3 * 49) ** 0.5).to(torch.bfloat16)
    g0 = (torch.rand(co, device=cuda) + 0.5)
    b0 = torch.randn(co, device=cuda) * 0.1

    def run(fused):
        _lib.set_inplace_grads(False)
        wt = torch.nn.Parameter(w0.clone())
        g, b = torch.nn.Parameter(g0.clone()), torch.nn.Parameter(b0.clone())
        rm, rv = torch.zeros(co, device=cuda), torch.ones(co, device=cuda)
        if fused:
            y = conv_bn_act_pool(x0, wt, g, b, rm, rv, 2, 3, 0.1, 1e-5, 3, 2, 1)
        else:
            y = max_pool(conv_bn_act(x0, wt, g, b, rm, rv, 2, 3, True, 0.1, 1e-5, True), 3, 2, padding=1)
        gy = torch.randn(y.shape, device=cuda, generator=torch.Generator(device=cuda).manual_seed(3))
        (y.float() * gy).sum().backward()
        _lib.set_inplace_grads(True)
        return y.detach().float(), rm, rv, wt.grad.float(), g.grad.float(), b.grad.float()

    fu, ref = run(True), run(False)
    assert fu[0].shape == (n, co, (h // 2 + 1) // 2, (w // 2 + 1) // 2)
    assert torch.isfinite(fu[0]).all()
    # the stem kernel adds its BN statistics with float atomics in workgroup-completion order, so the
    # two runs' means differ in the last bits and a few outputs round to the neighbouring bf16
    differ = (fu[0] != ref[0]).float().mean().item()
    assert differ < 1e-3, f"{differ:.2%} of the pooled outputs differ"
    torch.testing.assert_close(fu[0], ref[0], rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(fu[1], ref[1], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(fu[2], ref[2], rtol=1e-4, atol=1e-5)
    for a, b, what in zip(fu[3:], ref[3:], ("dw", "dgamma", "dbeta")):
        assert _rel(a, b) < 2e-2, f"{what} rel {_rel(a, b):.4f}"


def test_stem_conv_bn_act_layer_fwd_bwd(cuda):
    """The fused ConvBNAct layer on a 3-channel input (MFMA stem forward + wgrad, no MIOpen) vs fp32."""
    from tony_amd.ops import _lib
    from tony_amd.ops import conv as C

    torch.manual_seed(4)
    n, h, w, co = 4, 75, 75, 32
    x = _nhwc(torch.randn(n, 3, h, w, device=cuda)).to(torch.bfloat16)
    wt = _nhwc(0.2 * torch.randn(co, 3, 3, 3, device=cuda)).to(torch.bfloat16).requires_grad_(True)
    g = torch.empty(co, device=cuda).uniform_(0.5, 1.5).to(torch.bfloat16).requires_grad_(True)
    b = torch.empty(co, device=cuda).uniform_(-0.2, 0.2).to(torch.bfloat16).requires_grad_(True)
    rm, rv = torch.zeros(co, device=cuda), torch.ones(co, device=cuda)
    _lib.set_inplace_grads(False)
    saved = C.AUTOTUNE, C.STEM
    C.AUTOTUNE, C.STEM = False, True  # route the stem to the fused layer and its MFMA kernels
    try:
        y = C.conv_bn_act(x, wt, g, b, rm, rv, 2, 0, True, 0.1, 1e-3, True)
        key = [k for k in C._CHOICE if k[0] == "fwd" and k[1] == tuple(x.shape) and k[2] == (co, 3, 3, 3)]
        assert not key or C._CHOICE[key[0]] == "tony"
        assert "miopen" not in {v for k, v in C._CHOICE.items() if k[1] == tuple(x.shape)}
        wr, gr, br = (t.detach().float().requires_grad_(True) for t in (wt, g, b))
        rm_r, rv_r = torch.zeros(co, device=cuda), torch.ones(co, device=cuda)
        yr = torch.relu(torch.nn.functional.batch_norm(torch.nn.functional.conv2d(x.float(), wr, None, 2, 0), rm_r,
                                                       rv_r, gr, br, True, 0.1, 1e-3))
        assert _rel(y, yr) < 2e-2
        torch.testing.assert_close(rm, rm_r, rtol=2e-2, atol=2e-3)
        dy = _nhwc(torch.randn_like(yr)).to(torch.bfloat16)
        y.backward(dy)
        yr.backward(dy.float())
        assert _rel(wt.grad, wr.grad) < 3e-2
        assert _rel(g.grad, gr.grad) < 3e-2 and _rel(b.grad, br.grad) < 3e-2
    finally:
        C.AUTOTUNE, C.STEM = saved
        _lib.set_inplace_grads(True)


# (N, Cin, H, W, Cout, padding): the shapes of the persistent direct 3x3 kernel (tile variant 10),
# with partial edge tiles in both directions and several tiles per workgroup
DIRECT_SHAPES = [(3, 32, 37, 45, 32, (0, 0)), (4, 32, 37, 37, 64, (1, 1)), (2, 64, 29, 35, 32, (1, 1)),
                 (2, 64, 24, 20, 64, (1, 1)), (64, 32, 19, 21, 32, (1, 1))]


@pytest.mark.parametrize("shape", DIRECT_SHAPES, ids=[f"{s[1]}->{s[4]}_{s[2]}x{s[3]}p{s[5][0]}" for s in DIRECT_SHAPES])
def test_conv_direct_variant(cuda, shape):
    """csrc/conv.hip conv_direct_kernel (variant 10): forward + BN statistics and backward-data vs fp32."""
    from tony_amd.ops import _lib
    from tony_amd.ops.conv import conv_dgrad, conv_fwd

    n, c, h, w, co, p = shape
    torch.manual_seed(11)
    x = _nhwc(torch.randn(n, c, h, w, device=cuda)).to(torch.bfloat16)
    wt = _nhwc(0.1 * torch.randn(co, c, 3, 3, device=cuda)).to(torch.bfloat16)
    stats = torch.zeros(_lib.stat_floats(co), device=cuda)
    y = conv_fwd(x, wt, 1, p, stats, vflags=10 << 8)
    xr = x.float().requires_grad_(True)
    ref = torch.nn.functional.conv2d(xr, wt.float(), None, 1, p)
    assert _rel(y, ref) < 1e-2
    st = _lib.fold_stats(stats, co)
    torch.testing.assert_close(st[:co], ref.detach().sum((0, 2, 3)), rtol=2e-3, atol=ref.numel() / co * 2e-4)
    torch.testing.assert_close(st[co:], (ref.detach() ** 2).sum((0, 2, 3)), rtol=2e-3, atol=1e-1)
    dy = _nhwc(torch.randn_like(ref)).to(torch.bfloat16)
    ref.backward(dy.float())
    dx = conv_dgrad(dy, wt, x.shape, 1, p, vflags=10 << 8)
    assert _rel(dx, xr.grad) < 1e-2


@pytest.mark.parametrize("shape", DIRECT_SHAPES + [(2, 64, 21, 40, 64, (2, 2)), (1, 32, 3, 3, 64, (1, 1))],
                         ids=lambda s: f"{s[1]}->{s[4]}_{s[2]}x{s[3]}p{s[5][0]}")
def test_conv_wgrad_direct(cuda, shape):
    """csrc/conv.hip conv_wgrad_direct_kernel (3x3 stride 1, C / Co in {32, 64}) vs fp32, returned and
    added into a bf16 gradient slot."""
    from tony_amd.ops.conv import conv_wgrad

    n, c, h, w, co, p = shape
    torch.manual_seed(12)
    x = _nhwc(torch.randn(n, c, h, w, device=cuda)).to(torch.bfloat16)
    wt = _nhwc(0.1 * torch.randn(co, c, 3, 3, device=cuda)).to(torch.bfloat16)
    xr, wr = x.float(), wt.float().requires_grad_(True)
    ref = torch.nn.functional.conv2d(xr, wr, None, 1, p)
    dy = _nhwc(torch.randn_like(ref)).to(torch.bfloat16)
    ref.backward(dy.float())
    dw = conv_wgrad(dy, x, wt.shape, 1, p, impl="direct")
    assert _rel(dw, wr.grad) < 5e-3, f"direct wgrad rel {_rel(dw, wr.grad):.5f}"
    slot = torch.full((co * 9 * c,), 0.5, device=cuda, dtype=torch.bfloat16)
    assert conv_wgrad(dy, x, wt.shape, 1, p, dst=slot, impl="direct") is None
    want = 0.5 + wr.grad.permute(0, 2, 3, 1).reshape(-1)
    assert _rel(slot, want) < 1e-2


# (N, Cin, H, W, Cout, (R, S), padding): LDS-DMA kernel shapes -- partial row / column tiles, K not a
# multiple of 64, Cin < 64 (several taps per K-step), 1x1
GLDS_SHAPES = [(2, 64, 35, 35, 96, (3, 3), (1, 1)), (2, 48, 17, 19, 64, (5, 5), (2, 2)),
               (2, 160, 17, 17, 192, (1, 7), (0, 3)), (3, 448, 8, 8, 384, (3, 3), (1, 1)),
               (2, 88, 13, 11, 40, (1, 1), (0, 0)), (1, 32, 9, 9, 32, (3, 3), (0, 0)),
               # channel counts that are multiples of both K-step depths (the uniform-tap loop of
               # igemm.h: every lane crosses into the next tap at the same step) incl. a 1x1
               (2, 64, 17, 19, 64, (5, 5), (2, 2)), (3, 128, 9, 7, 192, (1, 1), (0, 0)),
               (2, 192, 11, 13, 128, (3, 1), (1, 0))]


@pytest.mark.parametrize("v", range(11, 32))
@pytest.mark.parametrize("shape", GLDS_SHAPES, ids=[f"{s[1]}->{s[4]}_{s[2]}x{s[3]}k{s[5][0]}{s[5][1]}" for s in GLDS_SHAPES])
def test_conv_glds_variants(cuda, shape, v):
    """csrc/conv.hip conv_glds_kernel (variants 11-15: 4 waves; 16-19: 8 waves, 256-row tiles; 20-24: the
    interleaved-issue forms, uniform-tap shapes only; 25-31: several workgroups per CU, conv_glds_occ_kernel,
    26 / 28 interleaved): forward + BN statistics, stride-1 backward-data."""
    from tony_amd.ops import _lib
    from tony_amd.ops.conv import conv_dgrad, conv_fwd

    n, c, h, w, co, (r, s), p = shape
    il_kb = 64 if v == 22 else 32  # the K-step depth a uniform-tap (interleaved) variant needs
    if v in (20, 21, 22, 23, 24, 26, 28) and (c % il_kb or co % il_kb):
        pytest.skip("interleaved-issue variants take uniform-tap shapes only (fwd Cin, dgrad Cout)")
    torch.manual_seed(v)
    x = _nhwc(torch.randn(n, c, h, w, device=cuda)).to(torch.bfloat16)
    wt = _nhwc(torch.randn(co, c, r, s, device=cuda) / (c * r * s) ** 0.5).to(torch.bfloat16)
    stats = torch.zeros(_lib.stat_floats(co), device=cuda)
    y = conv_fwd(x, wt, 1, p, stats, vflags=v << 8)
    xr = x.float().requires_grad_(True)
    ref = torch.nn.functional.conv2d(xr, wt.float(), None, 1, p)
    assert _rel(y, ref) < 1e-2
    st = _lib.fold_stats(stats, co)
    torch.testing.assert_close(st[:co], ref.detach().sum((0, 2, 3)), rtol=2e-3, atol=ref.numel() / co * 2e-4)
    torch.testing.assert_close(st[co:], (ref.detach() ** 2).sum((0, 2, 3)), rtol=2e-3, atol=1e-1)
    dy = _nhwc(torch.randn_like(ref)).to(torch.bfloat16)
    ref.backward(dy.float())
    dx = conv_dgrad(dy, wt, x.shape, 1, p, vflags=v << 8)
    assert _rel(dx, xr.grad) < 1e-2


STRIDED_GLDS = [(2, 288, 35, 35, 384, (3, 3), 2, (0, 0)), (2, 192, 17, 17, 320, (3, 3), 2, (0, 0)),
                (2, 96, 35, 35, 96, (3, 3), 2, (0, 0)), (2, 256, 28, 28, 512, (1, 1), 2, (0, 0)),
                (2, 64, 57, 57, 64, (3, 3), 2, (1, 1)), (3, 128, 12, 9, 160, (3, 3), 2, (1, 1)),
                (2, 64, 20, 20, 64, (5, 5), 3, (2, 2))]


@pytest.mark.parametrize("v", range(11, 32))
@pytest.mark.parametrize("shape", STRIDED_GLDS, ids=[f"{s[1]}->{s[4]}_{s[2]}k{s[5][0]}s{s[6]}" for s in STRIDED_GLDS])
def test_strided_dgrad_glds_variants(cuda, shape, v):
    """Strided backward-data on the LDS-DMA kernels (igemm.h BTaps: each residue class reads its taps out
    of the full transposed filter; the epilogue's row map scatters rows to the class's dX pixels), every
    tile variant, plain and accumulating into a gradient (flag bit 4)."""
    from tony_amd.ops.conv import conv_dgrad

    n, ci, h, w, co, (r, s), st, (ph, pw) = shape
    if co % (64 if v in (11, 17, 22) else 32):
        pytest.skip("the LDS-DMA strided dgrad takes uniform-tap shapes (Cout a multiple of the K-step)")
    torch.manual_seed(v)
    xr = torch.randn(n, ci, h, w, device=cuda, requires_grad=True)
    wt = _nhwc(torch.randn(co, ci, r, s, device=cuda) / (ci * r * s) ** 0.5).to(torch.bfloat16)
    yr = torch.nn.functional.conv2d(xr, wt.float(), None, st, (ph, pw))
    dy = _nhwc(torch.randn_like(yr)).to(torch.bfloat16)
    yr.backward(dy.float())
    dx = conv_dgrad(dy, wt, (n, ci, h, w), st, (ph, pw), vflags=v << 8)
    assert _rel(dx, xr.grad) < 1e-2, f"dgrad rel {_rel(dx, xr.grad):.4f}"
    g = _nhwc(torch.randn(n, ci, h, w, device=cuda)).to(torch.bfloat16)
    ref = g.float() + dx.float()
    out = conv_dgrad(dy, wt, (n, ci, h, w), st, (ph, pw), vflags=v << 8, accum=g)
    torch.testing.assert_close(out.float(), ref, rtol=1.6e-2, atol=1.6e-2)


@pytest.mark.parametrize("v", [12, 16, 19, 23, 24, 25, 26])
@pytest.mark.parametrize("shape", STRIDED_GLDS[:6], ids=[f"{s[1]}->{s[4]}_{s[2]}k{s[5][0]}" for s in STRIDED_GLDS[:6]])
def test_strided_dgrad_one_launch_matches_per_class(cuda, shape, v):
    """csrc/igemm.h MultiClass: every residue class of a stride-2 dgrad in one launch is bit-identical to
    one launch per class (same tiles, same K order), plain and accumulating."""
    from tony_amd.ops import _lib
    from tony_amd.ops.conv import conv_dgrad

    n, ci, h, w, co, (r, s), st, (ph, pw) = shape
    if co % 32:
        pytest.skip("uniform-tap shapes only")
    torch.manual_seed(v)
    wt = _nhwc(torch.randn(co, ci, r, s, device=cuda) / (ci * r * s) ** 0.5).to(torch.bfloat16)
    oh, ow = (h + 2 * ph - r) // st + 1, (w + 2 * pw - s) // st + 1
    dy = _nhwc(torch.randn(n, co, oh, ow, device=cuda)).to(torch.bfloat16)
    g = _nhwc(torch.randn(n, ci, h, w, device=cuda)).to(torch.bfloat16)
    L = _lib.lib()
    prev = L.tony_dgrad_one_launch(-1)
    outs = []
    try:
        for one in (1, 0):
            L.tony_dgrad_one_launch(one)
            outs.append((conv_dgrad(dy, wt, (n, ci, h, w), st, (ph, pw), vflags=v << 8),
                         conv_dgrad(dy, wt, (n, ci, h, w), st, (ph, pw), vflags=v << 8, accum=g.clone())))
    finally:
        L.tony_dgrad_one_launch(prev)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


def test_bn_reduce_fused_into_dgrad(cuda):
    """A chain conv-BN-ReLU -> conv-BN-ReLU (strided) -> conv-BN-ReLU: each BN backward's reduction
    comes from the next conv's dgrad epilogue (csrc/conv.hip BnRed: NT kernel, strided residue classes,
    direct kernel) instead of a separate kernel; gradients match the unfused run and fp32."""
    from tony_amd.ops import _lib
    from tony_amd.ops import conv as C

    torch.manual_seed(12)
    dims = [(32, 32, 1, 1), (32, 64, 2, 0), (64, 64, 1, 1)]  # (cin, cout, stride, pad), 3x3 each
    x = _nhwc(torch.randn(16, 32, 37, 37, device=cuda)).to(torch.bfloat16)  # >= conv.MIN_ROWS pixels per layer
    ws = [_nhwc(0.1 * torch.randn(co, ci, 3, 3, device=cuda)).to(torch.bfloat16) for ci, co, _, _ in dims]
    gs = [torch.empty(co, device=cuda).uniform_(0.5, 1.5).to(torch.bfloat16) for _, co, _, _ in dims]
    bs = [torch.empty(co, device=cuda).uniform_(-0.2, 0.2).to(torch.bfloat16) for _, co, _, _ in dims]

    def run(fused, fp32=False):
        C.FUSED_REDUCE = fused  # every eligible layer (the default fuses only >= 64 MB layers)
        C.FUSED_REDUCE_MIN_BYTES = 0
        params = [t.detach().clone().float() if fp32 else t.detach().clone() for t in ws + gs + bs]
        for p in params:
            p.requires_grad_(True)
        h = x.float() if fp32 else x
        for i, (ci, co, st, pd) in enumerate(dims):
            w, g, b = params[i], params[3 + i], params[6 + i]
            rm, rv = torch.zeros(co, device=cuda), torch.ones(co, device=cuda)
            if fp32:
                h = torch.relu(torch.nn.functional.batch_norm(torch.nn.functional.conv2d(h, w, None, st, pd), rm, rv,
                                                              g, b, True, 0.1, 1e-3))
            else:
                h = C.conv_bn_act(h, w, g, b, rm, rv, st, pd, True, 0.1, 1e-3, True)
        torch.manual_seed(13)
        dy = torch.randn(h.shape, device=cuda)
        (h.float() * dy).sum().backward()
        return [p.grad.float() for p in params]

    _lib.set_inplace_grads(False)
    saved = C.FUSED_REDUCE, C.FUSED_REDUCE_MIN_BYTES
    try:
        hits0 = C.FUSED_REDUCE_HITS[0]
        fused = run(True)
        # layer 1's reduction always fuses (strided dgrad); layer 2's unless the autotuner picked the halo
        # variant (no fused epilogue: the separate reduce runs)
        assert C.FUSED_REDUCE_HITS[0] - hits0 >= 1, "the inner BN backward passes use the fused reduction"
        plain = run(False)
        ref = run(False, fp32=True)
    finally:
        C.FUSED_REDUCE, C.FUSED_REDUCE_MIN_BYTES = saved
        _lib.set_inplace_grads(True)
    for i, (a, b, r) in enumerate(zip(fused, plain, ref)):
        assert _rel(a, b) < 2e-3, f"param {i}: fused vs unfused {_rel(a, b):.2e}"
        # bf16 chain vs fp32: the fused path is no further from fp32 than the unfused one
        assert _rel(a, r) < 1.2 * _rel(b, r) + 1e-2, f"param {i}: fused {_rel(a, r):.2e} unfused {_rel(b, r):.2e}"


SPLITK_SHAPES = [(8, 192, 17, 17, 192, (1, 7), (0, 3)), (8, 160, 17, 17, 160, (7, 1), (3, 0)),
                 (16, 384, 8, 8, 384, (3, 1), (1, 0)), (16, 448, 8, 8, 384, (3, 3), (1, 1))]


@pytest.mark.parametrize("m", [1, 2, 3])
@pytest.mark.parametrize("v", [11, 12, 14, 17, 20, 23])
@pytest.mark.parametrize("shape", SPLITK_SHAPES, ids=[f"{s[1]}->{s[4]}_{s[2]}k{s[5][0]}x{s[5][1]}" for s in SPLITK_SHAPES])
def test_conv_glds_streamk(cuda, shape, v, m):
    """Stream-K form of the LDS-DMA conv (igemm.h SplitK: m x CUs workgroups own equal ranges of the
    (tile, K-step) iterations; the contributors of a shared tile fold their partials, the last arriver
    summing them in K order and running the epilogue).  At batch 8 every tile is shared by many
    workgroups (>= 4 K-steps each): forward + BN statistics and stride-1 backward-data against fp32,
    deterministic (two runs bit-identical) and equal to the plain kernel within fp32 reassociation."""
    from tony_amd.ops import _lib
    from tony_amd.ops.conv import conv_dgrad, conv_fwd

    n, c, h, w, co, (r, s), p = shape
    kb = 64 if v in (11, 17, 22) else 32
    if c % kb or co % kb:
        pytest.skip("uniform-tap shapes only for this variant")
    vf = (v << 8) | (m << 16)
    torch.manual_seed(v + 7 * m)
    x = _nhwc(torch.randn(n, c, h, w, device=cuda)).to(torch.bfloat16)
    wt = _nhwc(torch.randn(co, c, r, s, device=cuda) / (c * r * s) ** 0.5).to(torch.bfloat16)
    stats = torch.zeros(_lib.stat_floats(co), device=cuda)
    y = conv_fwd(x, wt, 1, p, stats, vflags=vf)
    y2 = conv_fwd(x, wt, 1, p, None, vflags=vf)
    y1 = conv_fwd(x, wt, 1, p, None, vflags=v << 8)
    assert torch.equal(y, y2), "the fold must not depend on which contributor arrives last"
    assert (y.float() - y1.float()).abs().max().item() <= 2 ** -6 * y1.float().abs().max().item()
    xr = x.float().requires_grad_(True)
    ref = torch.nn.functional.conv2d(xr, wt.float(), None, 1, p)
    assert _rel(y, ref) < 1e-2
    st = _lib.fold_stats(stats, co)
    torch.testing.assert_close(st[:co], ref.detach().sum((0, 2, 3)), rtol=2e-3, atol=ref.numel() / co * 2e-4)
    torch.testing.assert_close(st[co:], (ref.detach() ** 2).sum((0, 2, 3)), rtol=2e-3, atol=1e-1)
    dy = _nhwc(torch.randn_like(ref)).to(torch.bfloat16)
    ref.backward(dy.float())
    dx = conv_dgrad(dy, wt, x.shape, 1, p, vflags=vf)
    assert _rel(dx, xr.grad) < 1e-2
    g = _nhwc(torch.randn(n, c, h, w, device=cuda)).to(torch.bfloat16)
    want = g.float() + dx.float()
    out = conv_dgrad(dy, wt, x.shape, 1, p, vflags=vf, accum=g)
    torch.testing.assert_close(out.float(), want, rtol=1.6e-2, atol=1.6e-2)


@pytest.mark.parametrize("m", [1, 3])
def test_gemm_glds_streamk_reuses_rearmed_counters(cuda, m):
    """The 1x1 GEMM path (tony_gemm_bf16 on the LDS-DMA kernel) in stream-K form through ONE persistent
    workspace, three launches in a row: each launch's last arrivers re-arm the tile counters, so the
    next launch reads a clean ticket sequence; an 8x8 head GEMM (M = 1024, K = 2048) with BN stats."""
    from tony_amd.ops import _lib

    L = _lib.lib()
    M, N, K = 1024, 448, 2048
    torch.manual_seed(m)
    a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    b = (torch.randn(N, K, device=cuda) / K ** 0.5).to(torch.bfloat16)
    ref = a.float() @ b.float().t()
    slab = torch.empty(_lib.splitk_slab_floats(m, _lib.num_cus(cuda)), device=cuda)
    cnt = torch.zeros(2 * _lib.SPLITK_MAX_TILES, dtype=torch.int32, device=cuda)
    raw = L.tony_gemm_bf16.__wrapped__
    st = _lib.stream_ptr(cuda)
    outs = []
    try:
        _lib.check(L.tony_splitk_workspace(slab.data_ptr(), slab.numel(), cnt.data_ptr(), cnt.numel()), "ws")
        for _ in range(3):
            c = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
            stats = torch.zeros(_lib.stat_floats(N), device=cuda)
            _lib.check(raw(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, K, K, N,
                           1 | (14 << 8) | (m << 16), stats.data_ptr(), 2 * N, st), "gemm stream-K")
            outs.append((c, stats))
        torch.cuda.synchronize()
    finally:
        L.tony_splitk_workspace(0, 0, 0, 0)
    assert int(cnt.abs().sum()) == 0, "counters re-armed to zero"
    for c, stats in outs:
        assert torch.equal(c, outs[0][0])
        assert _rel(c, ref) < 1e-2
        torch.testing.assert_close(_lib.fold_stats(stats, N)[:N], ref.sum(0), rtol=2e-3, atol=M * 2e-3)


# (N, Cin, H, W, Cout, (R, S), padding): wgrad shapes on the LDS-DMA wgrad kernel (Cout > 64: 96 / 128-row
# tiles) with the incremental row walk -- K steps not a multiple of the 6-step unroll, 1x1, 3x3, 1x7
WGRAD_PF_SHAPES = [(4, 64, 35, 35, 96, (3, 3), (1, 1)), (3, 160, 17, 17, 192, (1, 7), (0, 3)),
                   (2, 192, 17, 17, 160, (1, 1), (0, 0)), (5, 96, 11, 13, 128, (3, 3), (0, 0))]


@pytest.mark.parametrize("shape", WGRAD_PF_SHAPES, ids=[f"{s[1]}->{s[4]}_{s[2]}x{s[3]}k{s[5][0]}{s[5][1]}" for s in WGRAD_PF_SHAPES])
def test_wgrad_fragment_prefetch_matches_plain(cuda, shape):
    """conv.hip conv_wgrad_glds_kernel PF (tony_wgrad_pf): the fragment-prefetch K loop issues the same MFMAs
    in the same order as the plain loop -- bit-identical dW -- and matches the fp32 reference."""
    from tony_amd.ops import _lib
    from tony_amd.ops.conv import conv_wgrad

    n, c, h, w, co, (r, s), p = shape
    torch.manual_seed(1)
    x = _nhwc(torch.randn(n, c, h, w, device=cuda)).to(torch.bfloat16)
    wt = torch.randn(co, c, r, s, device=cuda)
    oh, ow = h + 2 * p[0] - r + 1, w + 2 * p[1] - s + 1
    dy = _nhwc(torch.randn(n, co, oh, ow, device=cuda)).to(torch.bfloat16)
    L = _lib.lib()
    prev = L.tony_wgrad_pf(-1)
    try:
        outs = []
        for pf in (0, 1):
            L.tony_wgrad_pf(pf)
            outs.append(conv_wgrad(dy, x, wt.shape, 1, p, impl=1).float().clone())
    finally:
        L.tony_wgrad_pf(prev)
    torch.testing.assert_close(outs[1], outs[0], rtol=0, atol=0)
    xr = x.float().requires_grad_(False)
    wr = torch.zeros_like(wt, requires_grad=True)
    torch.nn.functional.conv2d(xr, wr, None, 1, p).backward(dy.float())
    assert _rel(outs[1], wr.grad) < 1e-2


BAND_SHAPES = [(4, 192, 17, 17, 192, (1, 7), (0, 3)), (4, 160, 17, 17, 192, (7, 1), (3, 0)),
               (3, 128, 17, 17, 160, (1, 7), (0, 3)), (5, 384, 8, 8, 384, (1, 3), (0, 1)),
               (5, 384, 8, 8, 384, (3, 1), (1, 0)), (2, 192, 11, 13, 128, (3, 1), (1, 0)),
               (2, 64, 9, 20, 96, (1, 7), (0, 3)), (3, 96, 17, 17, 64, (1, 7), (0, 0))]


@pytest.mark.parametrize("shape", BAND_SHAPES, ids=[f"{s[1]}->{s[4]}_{s[2]}x{s[3]}k{s[5][0]}{s[5][1]}p{s[6][0]}{s[6][1]}"
                                                    for s in BAND_SHAPES])
def test_conv_band_variant(cuda, shape):
    """csrc/band.hip (tile variant 40): the 1 x T / T x 1 stride-1 convs on whole-line halo tiles --
    forward with BN statistics and backward-data against fp32 PyTorch; N not a multiple of the column tile,
    partial last line tiles, "valid" padding; other shapes are declined (-3)."""
    from tony_amd.ops import _lib
    from tony_amd.ops.conv import conv_dgrad, conv_fwd

    n, c, h, w, co, (r, s), p = shape
    torch.manual_seed(c + co)
    x = _nhwc(torch.randn(n, c, h, w, device=cuda)).to(torch.bfloat16)
    wt = _nhwc(torch.randn(co, c, r, s, device=cuda) / (c * r * s) ** 0.5).to(torch.bfloat16)
    stats = torch.zeros(_lib.stat_floats(co), device=cuda)
    y = conv_fwd(x, wt, 1, p, stats, vflags=40 << 8)
    xr = x.float().requires_grad_(True)
    ref = torch.nn.functional.conv2d(xr, wt.float(), None, 1, p)
    assert _rel(y, ref) < 1e-2
    st = _lib.fold_stats(stats, co)
    torch.testing.assert_close(st[:co], ref.detach().sum((0, 2, 3)), rtol=2e-3, atol=ref.numel() / co * 2e-4)
    torch.testing.assert_close(st[co:], (ref.detach() ** 2).sum((0, 2, 3)), rtol=2e-3, atol=1e-1)
    dy = _nhwc(torch.randn_like(ref)).to(torch.bfloat16)
    ref.backward(dy.float())
    if p[0] * 2 + 1 == r and p[1] * 2 + 1 == s:  # "same" padding: the dgrad is a band conv too
        dx = conv_dgrad(dy, wt, x.shape, 1, p, vflags=40 << 8)
        assert _rel(dx, xr.grad) < 1e-2


def test_conv_band_declines_other_shapes(cuda):
    """A 3x3 conv, a strided 1x7 and an fp32 (x3) output are not band shapes: -3, nothing launched."""
    from tony_amd.ops import _lib

    L = _lib.lib()
    st = _lib.stream_ptr(torch.device(cuda))
    x = _nhwc(torch.randn(2, 64, 17, 17, device=cuda)).to(torch.bfloat16)
    wk = torch.randn(64, 3, 3, 64, device=cuda).to(torch.bfloat16)
    y = torch.empty(2 * 17 * 17 * 64, device=cuda, dtype=torch.float32)
    assert L.tony_conv_fwd(x.data_ptr(), 2, 17, 17, 64, 64, wk.data_ptr(), 64, 3, 3, 1, 1, 1, 1, y.data_ptr(), 17,
                           17, 64, 40 << 8, None, 0, st) == -3
    w7 = torch.randn(64, 1, 7, 64, device=cuda).to(torch.bfloat16)
    assert L.tony_conv_fwd(x.data_ptr(), 2, 17, 17, 64, 64, w7.data_ptr(), 64, 1, 7, 2, 2, 0, 3, y.data_ptr(), 9,
                           9, 64, 40 << 8, None, 0, st) == -3
    assert L.tony_conv_fwd(x.data_ptr(), 2, 17, 17, 64, 64, w7.data_ptr(), 64, 1, 7, 1, 1, 0, 3, y.data_ptr(), 17,
                           17, 64, (40 << 8) | 8, None, 0, st) == -3
    torch.cuda.synchronize()
