"""The dedicated parameter server on the xGMI data plane (csrc/ps_plane.hip, parallel/ps_plane.py): 1 ps +
2-3 workers as processes sharing the test box's one GPU.

Checks the window exchange, push into the ps's receive rows, the apply-as-rows-land kernel (sync: sum of
every worker's chunk; async: each worker's chunk on its own), the landing of the new variables in every
worker's window and the copy into the flat parameters, against exact expectations; and a fused conv net
trained through the Trainer whose pushes launch during backward (the overlap the bucket engine logs).
The one-GPU box has no real xGMI link: this proves the protocol, not the link bandwidth.
"""
import multiprocessing as mp
import socket

import pytest

from gpu_ranks import placement

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(240)]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = dict(q.get(timeout=200) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    errors = {r: out[r]["error"] for r in range(world) if "error" in out[r]}
    assert not errors, "\n".join(f"rank {r}: {e}" for r, e in errors.items())
    return out


@pytest.mark.parametrize("world,sync,wire", [(3, True, None), (4, True, "fp32"), (3, False, None)],
                         ids=[f"sync-2w-bf16-{placement(3)}", f"sync-3w-fp32wire-{placement(4)}", f"async-2w-{placement(3)}"])
def test_ps_plane_push_apply_land(world, sync, wire, monkeypatch):
    import torch

    import ps_plane_worker as W

    monkeypatch.setenv("TONY_PS_SPIN_S", "60")
    out = _spawn(W.run, world, sync, torch.float32 if wire == "fp32" else None)
    for r in range(world):
        bad = [k for k, v in out[r].items() if v is False]
        assert not bad, (r, bad, out[r])
    assert out[0]["pushed"] == 0 and all(out[r]["pushed"] > 0 for r in range(1, world))


@pytest.mark.parametrize("where", [placement(3)])
def test_ps_plane_trainer_overlap(where, monkeypatch):
    monkeypatch.setenv("TONY_PS_SPIN_S", "20")
    monkeypatch.setenv("TONY_PS_PLANE_TRACE", "1")
    out = _spawn(__import__("ps_plane_worker").run_overlap, 3)
    for r in range(1, 3):
        assert out[r]["loss_finite"] and out[r]["overlapped"], out[r]
    for r in range(3):
        assert out[r]["workers_agree"] and out[r]["ps_matches_workers"], out[r]
    # the ps's variables follow a single-process reference of the sync-PS step (mean of the workers'
    # gradients, SGD-momentum on fp32 masters)
    assert out[0]["matches_reference"], out[0]["update_rel_err_vs_reference"]
