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
