"""Reference precision through the parameter server (verdict r5 #3): the x3 (fp32) Inception-v3 trained by
2 workers through the ParameterServer -- colocated shards (2 ranks) and the dedicated paper topology over the
xGMI PS plane (1 ps + 2 workers) -- matches a single-process reference of the same sync-PS steps (each
worker's batch forward / backward, gradients averaged, fp32 SGD-momentum with L2 decay) to within 6x the
reference's own run-to-run spread: two fp32 runs of a 95-BN-layer network at batch 2 are not bitwise equal
(atomic BN statistics flip ReLU mask bits, the depth amplifies it: ~5 % after one step), so a fixed 1e-3
bound would test the network's conditioning, not the parameter server.
On the one-GPU box the ranks share cuda:0 (gloo); on a multi-GPU node each owns a device over RCCL."""
import multiprocessing as mp
import os
import socket

import pytest

from gpu_ranks import placement

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(420)]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode,world", [("colocated", 2), ("dedicated", 3)],
                         ids=[f"colocated-{placement(2)}", f"dedicated-1ps2w-{placement(3)}"])
def test_x3_inception_through_ps_matches_reference(mode, world, monkeypatch):
    import x3_ps_worker as W

    from gpu_ranks import distinct

    if mode == "dedicated" and not distinct(world):
        # three processes on one GPU: the xGMI plane's apply kernels and landings wait on the GPU for their
        # peers (the host stays out of the loop), and with the x3 step's streams in all three processes a
        # worker's queue was observed to make no progress until its peers' wait budgets expired
        # (profiles/r6_x3_ps_dedicated_shared_gpu.log); with one compute stream per process it passed once
        # and stalled once (profiles/r6_x3_ps_dedicated_xgmi_few_streams.log).  So on a shared GPU the
        # rehearsal checks the dedicated PS semantics on the collective plane (reduce -> apply -> broadcast,
        # no kernel waits on a peer); tests/test_ps_plane_gpu.py rehearses the xGMI plane's protocol with a
        # small net, and a node with a GPU per rank runs this test on the xGMI plane.  X3PS_PLANE=xgmi
        # reproduces the shared-GPU stall.
        monkeypatch.setenv("TONY_PS_PLANE", os.environ.get("X3PS_PLANE", "rccl"))

    monkeypatch.setenv("TONY_PS_SPIN_S", os.environ.get("TONY_PS_SPIN_S", "300"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=W.run, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = dict(q.get(timeout=400) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    errors = {r: out[r]["error"] for r in out if "error" in out[r]}
    assert not errors, "\n".join(f"rank {r}: {e}" for r, e in errors.items())
    first = 0 if mode == "colocated" else 1
    r = out[first]
    assert r["loss_finite"] and r["workers"] == 2, r
    assert r["update_norm"] > 0, r
    # the PS run against the reference, per step, with the reference's own run-to-run spread as the yardstick
    # (a gradient not averaged, a bucket applied twice or a stale pull is an O(1) error at step 0)
    # (observed at step 0: PS 0.058-0.17 against a spread of 0.055-0.061 -- the divergence of a chaotic
    # system is itself a random draw, hence the factor; a missing 1/n or a dropped worker is >= 0.5)
    for err, spread in zip(r["update_rel_err_per_step"], r["ref_spread_per_step"]):
        assert err < max(1e-3, 6 * spread), r
    assert r["update_rel_err_per_step"][0] < 0.3, r
