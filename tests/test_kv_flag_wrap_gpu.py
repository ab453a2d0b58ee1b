"""Wrap-safe device flag waits (csrc/ps_plane.hip wait_flag): the kvstore / PS-plane arrival
counters are cumulative u32s for the life of a job (a >= 4 MiB kvstore key adds 1024 per copy, so they wrap
after ~4.2M copies).  ``tony_kv_wait`` must order counter and target by their signed difference: a target
just past the wrap is NOT reached by a counter just before it (the old ``flag < value`` test let that wait
pass at once, and the copy behind it read bytes that had not landed), and a wrapped counter does reach a
target just before the wrap."""
import ctypes

import pytest
import torch

from tony_amd.ops import _lib

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(120)]


@pytest.fixture()
def window():
    L = _lib.lib()
    torch.cuda.init()
    win = ctypes.c_void_p()
    handle = (ctypes.c_uint8 * L.tony_xgmi_handle_bytes())()
    _lib.check(L.tony_ps_window_alloc(4096, ctypes.byref(win), handle), "tony_ps_window_alloc")
    yield L, win.value, win.value + L.tony_ps_header_bytes()  # (lib, window, a flag word in its payload)
    torch.cuda.synchronize()
    L.tony_xgmi_free(win.value)


def _set(L, flag, value):
    v = value - (1 << 32) if value >= (1 << 31) else value
    src = torch.tensor([v, 0, 0, 0], dtype=torch.int32, device="cuda")
    _lib.check(L.tony_kv_copy(flag, src.data_ptr(), 4, None, _lib.stream_ptr(src.device)), "tony_kv_copy")
    torch.cuda.synchronize()


def _wait_errs(L, win, flag, target, budget=0.2):
    _lib.check(L.tony_kv_wait(flag, target, win, budget, _lib.stream_ptr(torch.device("cuda"))), "tony_kv_wait")
    torch.cuda.synchronize()
    err = ctypes.c_int(0)
    _lib.check(L.tony_ps_error(win, ctypes.byref(err)), "tony_ps_error")  # reads and clears
    return err.value


@pytest.mark.parametrize("counter,target,reached", [
    (0x00000100, 0x00000100, True),   # equal
    (0xFFFFFFF0, 0xFFFFFF00, True),   # ahead, no wrap
    (0x00000005, 0xFFFFFFF0, True),   # the counter wrapped past a target just before the wrap
    (0x00000180, 0x00000100, True),   # both past the wrap
    (0xFFFFFF00, 0x00000100, False),  # the target is past the wrap, the counter 512 short of it
    (0x000000FF, 0x00000100, False),  # one short
], ids=["equal", "ahead", "wrapped-counter", "both-wrapped", "target-past-wrap", "one-short"])
def test_flag_wait_orders_wrapped_counters(window, counter, target, reached):
    L, win, flag = window
    _set(L, flag, counter)
    assert _wait_errs(L, win, flag, target) == (0 if reached else 1)
