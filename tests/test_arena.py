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
