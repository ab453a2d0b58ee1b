"""Step arena: zeroed fp32 accumulators carved per step, one fill per step (ops/arena.py)."""
import torch

from tony_amd.ops.arena import StepArena, current, zeros_f32


def test_arena_grows_then_serves_zeroed_slices():
    a = StepArena("cpu")
    with a:  # first step: nothing allocated yet -> every take misses, the need is recorded
        t1 = zeros_f32(10, "cpu")
        t2 = zeros_f32(100, "cpu")
        assert a.misses == 2 and current() is a
    assert current() is None
    for step in range(3):
        with a:
            x = zeros_f32(10, "cpu")
            y = zeros_f32(100, "cpu")
            assert x.abs().sum() == 0 and y.abs().sum() == 0     # zeroed by this step's single fill
            assert x.data_ptr() == a.buf.data_ptr()                # carved from the arena, in call order
            assert y.data_ptr() == a.buf.data_ptr() + 64 * 4       # 256-B aligned slices
            x += 5
            y -= 1                                                 # dirtied: the next step must re-zero
    assert a.misses == 2
    t = zeros_f32(7, "cpu")  # outside a step: plain zeros
    assert t.abs().sum() == 0 and t.data_ptr() != a.buf.data_ptr()
    del t1, t2


def test_side_stream_inactive_runs_inline():
    """ops/streams.py: without a CUDA device (or before begin()) gradient work runs right here."""
    from tony_amd.ops import streams

    assert streams.begin("cpu") is False and not streams.active()
    acc = torch.zeros(4)

    def work():
        acc.add_(1.0)

    assert streams.run(work, acc) is None
    assert acc.tolist() == [1.0] * 4
    assert streams.end() == 0


def test_tune_cache_roundtrip(tmp_path):
    """ops/tune.py save/load: tile variants, split plans and tony-vs-MIOpen choices survive a JSON round
    trip with their tuple keys intact (bench.py --tune-cache)."""
    from tony_amd.ops import conv, tune

    saved_t, saved_c = dict(tune._CACHE), dict(conv._CHOICE)
    try:
        tune._CACHE.clear()
        conv._CHOICE.clear()
        tune._CACHE[("conv_fwd", (128, 64, 35, 35), 64, (96, 64, 3, 3), (1, 1), (1, 1), True)] = 4
        tune._CACHE[("wgrad_occ", (128, 96, 35, 35), 96, (128, 64, 35, 35), 64, (96, 64, 3, 3), 1, 1, 1, 1)] = 2
        conv._CHOICE[("wgrad", (128, 96, 35, 35), (96, 64, 3, 3), (1, 1), (1, 1))] = "tony"
        path = str(tmp_path / "tune.json")
        assert tune.save(path) == 3
        want_t, want_c = dict(tune._CACHE), dict(conv._CHOICE)
        tune._CACHE.clear()
        conv._CHOICE.clear()
        assert tune.load(path) == 3
        assert tune._CACHE == want_t and conv._CHOICE == want_c
        assert tune.cached(("conv_fwd", (128, 64, 35, 35), 64, (96, 64, 3, 3), (1, 1), (1, 1), True)) == 4 << 8
    finally:
        tune._CACHE.clear()
        tune._CACHE.update(saved_t)
        conv._CHOICE.clear()
        conv._CHOICE.update(saved_c)


def test_rows_view_memo_matches_uncached_walk():
    """ops/bn.py memoises the (shape, strides) -> (M, C, ld) row view: every layout the fused ops see
    (channels_last, channel slices of a concat buffer, 2D, size-1 dims, non-row layouts) must give
    the uncached answer, on the first (miss) and second (hit) call."""
    import torch

    from tony_amd.ops import bn

    cl = torch.channels_last
    base = torch.empty(3, 24, 5, 7).contiguous(memory_format=cl)
    cases = [base, base[:, 8:16], base[:, :8], torch.empty(4, 16, 1, 1).contiguous(memory_format=cl),
             torch.empty(1, 8, 1, 9).contiguous(memory_format=cl), torch.empty(2, 8, 3, 3),  # NCHW: no row view
             torch.empty(6, 40), torch.empty(6, 40)[:, :16], torch.empty(6, 40).t()]
    for t in cases:
        want = bn._rows_view_uncached(t.shape, t.stride())
        assert bn._rows_view(t) == want
        assert bn._rows_view(t) == want


def test_conv_pair_fast_path():
    from tony_amd.ops.conv import _pair

    assert _pair(3) == (3, 3) and _pair((1, 2)) == (1, 2) and _pair([2, 1]) == (2, 1)


def test_wgrad_split_plans(monkeypatch):
    """ops/gemm.py: the weight-gradient split plan (workgroups per CU) -- the default for every layer,
    the stem-size override above WGRAD_BIG_ROWS reduction rows, fractional plans rounded to whole CUs."""
    from tony_amd.ops import _lib, gemm

    monkeypatch.setattr(_lib, "num_cus", lambda device: 256)
    assert gemm.wgrad_cus("cpu", 0.5) == 128 and gemm.wgrad_cus("cpu", 2) == 512
    assert gemm.wgrad_cus("cpu", 0.001) == 1
    monkeypatch.setattr(gemm, "WGRAD_OCC", (0.5,))
    monkeypatch.setattr(gemm, "WGRAD_OCC_BIG", (2,))
    monkeypatch.setattr(gemm, "WGRAD_BIG_ROWS", 600000)
    assert gemm.occ_choices(128 * 35 * 35) == (0.5,)     # mid-network layer: one workgroup per 2 CUs
    assert gemm.occ_choices(128 * 73 * 73) == (2,)       # the stem's 73x73 / 147x147 layers
    monkeypatch.setattr(gemm, "WGRAD_OCC_BIG", ())
    assert gemm.occ_choices(128 * 147 * 147) == (0.5,)   # override off
    monkeypatch.setattr(gemm, "X3_WGRAD_OCC", 1.0)
    monkeypatch.setattr(gemm, "X3_WGRAD_OCC_BIG", 2.0)
    assert gemm.x3_occ(128 * 17 * 17) == 1.0 and gemm.x3_occ(128 * 147 * 147) == 2.0
    assert gemm._occ_list("0.5,1,2") == (0.5, 1, 2) and gemm._occ_list("") == ()
