"""xGMI peer-memory collectives (csrc/xgmi.hip): 2-4 ranks as processes sharing the test box's GPU.

The single-GPU box cannot exercise real xGMI links; this checks the IPC window exchange, the push
reduce-scatter into peer windows, the per-workgroup flag barriers, the slot parity protocol (1,000
back-to-back calls, alternating parities with changing data), odd sizes and slot-sized pieces
against exact values, and that a rank whose peer skips a call gets XgmiError instead of a result.
A peer killed outright is not staged here: the survivor's push would store into the dead process's
freed window (a GPU fault on a shared box); the skipped call exercises the same bounded barrier.
"""
import multiprocessing as mp
import socket

import pytest

from gpu_ranks import placement

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(180)]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3, 4], ids=lambda w: placement(w))
def test_xgmi_collectives(world, monkeypatch):
    import xgmi_worker as W

    # barriers give up after ~1 s of polling (the default is minutes): the skipped-call case below
    monkeypatch.setenv("TONY_XGMI_SPIN_LIMIT", str(1 << 20))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=W.run, args=(r, world, port, q, world == 2)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = dict(q.get(timeout=150) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert "error" not in out[r], out[r]
        bad = [k for k, v in out[r].items() if not v]
        assert not bad, (r, bad)
    if world == 2:
        assert out[0]["skip_raises"] is True
