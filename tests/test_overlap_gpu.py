"""Gradient communication overlapped with backward on the FUSED models (parallel/buckets.py).

The fused HIP ops accumulate parameter gradients in place and never reach AccumulateGrad, so the
bucket engine learns of them through ``_lib.grads_ready``.  These tests check, on the GPU:

* one rank: the PS applies each bucket on the communication stream while backward runs, and the
  result equals the serial (apply-after-backward) step;
* two ranks sharing the box's GPU over gloo (the 1-GPU stand-in for 2 MI355X over RCCL): the first
  bucket's push is issued before backward has reported its last gradient, params are identical on
  both ranks and equal the non-overlapped run; DDP's flat gradients are identical across ranks.
"""
import multiprocessing as mp
import socket

import pytest

from gpu_ranks import placement
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(240)]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("kind", ["A", "C"])
def test_ps_overlap_one_rank_matches_serial(cuda, kind):
    import overlap_worker as W

    a = W.ps_run(0, kind, overlap=True, bucket_mb=0.05)
    b = W.ps_run(0, kind, overlap=False, bucket_mb=0.05)
    assert a["n_buckets"] > 2
    assert a["overlapped"] >= a["n_buckets"] - 1, (a["overlapped"], a["n_buckets"])
    assert b["overlapped"] == 0
    err = (a["params"] - b["params"]).abs().max().item()
    assert err < 1e-2, err
    # bucket 0 (the classifier + last layers) was launched before the first layers reported
    log = a["log"]
    assert log.index("launch:0") < max(i for i, e in enumerate(log) if e.startswith("ready:"))


@pytest.mark.parametrize("kind,collective", [("A", "rccl"), ("A", "hip")], ids=[f"process-group-{placement(2)}", f"xgmi-kernels-{placement(2)}"])
def test_two_ranks_overlap_ps_and_ddp(cuda, kind, collective, monkeypatch):
    """collective=hip: the colocated PS push / pull and DDP's bucket all-reduce run on the xGMI
    peer-memory kernels (TONY_COLLECTIVE=hip routes every data plane through parallel/collectives.py;
    gloo then only carries the window-handle exchange)."""
    import overlap_worker as W

    monkeypatch.setenv("TONY_COLLECTIVE", collective)

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _port()
    procs = [ctx.Process(target=W.run, args=(r, world, port, q, kind, 0.05)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = dict(q.get(timeout=200) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert "error" not in out[r], out[r]["error"]
        for v in out[r].values():
            if not isinstance(v, dict):
                continue
            for k in ("params", "grad"):
                if k in v:
                    v[k] = torch.from_numpy(v[k])
    o0, o1 = out[0]["ps_overlap"], out[1]["ps_overlap"]
    assert o0["n_buckets"] > 2
    assert o0["overlapped"] >= o0["n_buckets"] - 1
    log = o0["log"]
    assert log.index("launch:0") < max(i for i, e in enumerate(log) if e.startswith("ready:"))
    assert torch.equal(o0["params"], o1["params"])               # every rank pulled the same variables
    err = (o0["params"] - out[0]["ps_serial"]["params"]).abs().max().item()
    assert err < 1e-2, err
    # the natively replayed step (ops/plan.py) with the buckets issued between plan segments
    p0, p1 = out[0]["ps_plan"], out[1]["ps_plan"]
    assert p0["replay"] == "plan" and p0["plan_buckets"], p0["plan_error"]
    assert p0["overlapped"] >= p0["n_buckets"] - 1, (p0["overlapped"], p0["n_buckets"])
    assert torch.equal(p0["params"], p1["params"])
    err = (p0["params"] - out[0]["ps_serial"]["params"]).abs().max().item()
    assert err < 1e-2, err
    d0, d1 = out[0]["ddp"], out[1]["ddp"]
    assert d0["launches"] == d0["n_buckets"] and d0["overlapped"] >= d0["n_buckets"] - 1
    assert torch.equal(d0["grad"], d1["grad"])                    # averaged gradients identical on both ranks
    assert d0["grad"].abs().sum().item() > 0
    # ... and equal to the mean of the gradients each rank computes alone (a rank counted twice or
    # dropped, or a missing / double 1/world scale, moves every parameter's gradient by >= 30 %).  The
    # local gradients come from a second backward whose BN statistics are fp32 atomics: a bf16
    # pre-activation that rounds to the other side of its ReLU moves one small conv's weight gradient by
    # a few % (measured 4.1 % once), so per tensor < 0.1 and the whole gradient's cosine > 0.999
    ga, gw = [], []
    for name, g in d0["named"].items():
        g = torch.from_numpy(g)
        want = sum(torch.from_numpy(out[r]["ddp"]["local"][name]) for r in range(world)) / world
        err = (g - want).norm().item() / max(want.norm().item(), 1e-12)
        assert err < 0.1, (name, err)
        ga.append(g.double().flatten())
        gw.append(want.double().flatten())
    ga, gw = torch.cat(ga), torch.cat(gw)
    assert (ga @ gw / (ga.norm() * gw.norm())).item() > 0.999
    assert abs(ga.norm().item() / gw.norm().item() - 1) < 0.02  # the scale: 1/world applied exactly once
    if collective == "hip":  # every bucket push / pull / all-reduce ran on the xGMI kernels
        for r in range(world):
            for name in ("ps_overlap", "ps_plan", "ps_serial", "ddp"):
                assert out[r][name]["train_fallbacks"] == 0, (r, name, "a bucket collective fell back to gloo")
