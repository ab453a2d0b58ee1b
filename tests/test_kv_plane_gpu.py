"""The kvstore server modes with their payloads on the GPU plane (parallel/kvstore.py _KvPlane): a
scheduler, one server and two workers as processes on the box's GPU (the server shares it, as TonY's
0-GPU servers would share a worker's).  Values are checked against the closed-form SGD result -- the
same numbers the gloo-payload CPU test (tests/test_dist_cpu.py) pins -- and the pushes / pulls must have
gone over the plane."""
import multiprocessing as mp
import socket

import pytest
import torch

import dist_workers as W

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("kind", ["dist_sync", "dist_async"])
def test_kvstore_server_modes_move_payloads_on_the_gpu_plane(kind):
    port, steps = _port(), 3
    args = [("scheduler", 0, 1, 2, port, kind, steps, "cuda"), ("server", 0, 1, 2, port, kind, steps, "cuda"),
            ("worker", 0, 1, 2, port, kind, steps, "cuda"), ("worker", 1, 1, 2, port, kind, steps, "cuda")]
    ctx = mp.get_context("spawn")
    with ctx.Pool(len(args)) as pool:
        outs = [r.get(110) for r in [pool.apply_async(W.kv_rank, a) for a in args]]
    workers = [o for o in outs if o["role"] == "worker"]
    assert sorted(o["rank"] for o in workers) == [0, 1]
    n = 1000003
    ramp = torch.arange(n, dtype=torch.float32) / n
    for o in workers:
        assert o["k7"] == [1.0, 1.0]
        # every push and pull of "w" / "big" rode the plane (the key-7 pull too)
        assert o["plane_ops"] == [2 * steps, 2 * steps + 1], o["plane_ops"]
    if kind == "dist_sync":
        for o in workers:
            for s, w in enumerate(o["seen"]):
                torch.testing.assert_close(w, torch.full((3,), -0.75 * (s + 1)))
            # big: w -= 0.5 * (1 + 2) / 2 * ramp per round
            torch.testing.assert_close(o["big"], -0.75 * steps * ramp, rtol=1e-5, atol=1e-6)
    else:
        final = min(float(o["seen"][-1][0]) for o in workers)
        assert final == pytest.approx(-2.25)


def test_kvstore_plane_bulk_keys_sync_timed():
    """64 MB of keys (8 x 8 MB) per round through dist_sync on the GPU plane: the host never waits for a
    payload (device flags, ``tony_kv_copy_flag`` / ``tony_kv_wait``), every push / pull rides the plane,
    and the values follow the closed-form SGD result.  Prints the per-round time and per-push latency."""
    port, steps, keys, mb = _port(), 4, 8, 8
    args = [("scheduler", 0, 1, 2, port, "dist_sync", steps, keys, mb),
            ("server", 0, 1, 2, port, "dist_sync", steps, keys, mb),
            ("worker", 0, 1, 2, port, "dist_sync", steps, keys, mb),
            ("worker", 1, 1, 2, port, "dist_sync", steps, keys, mb)]
    ctx = mp.get_context("spawn")
    with ctx.Pool(len(args)) as pool:
        outs = [r.get(110) for r in [pool.apply_async(W.kv_bulk_rank, a) for a in args]]
    workers = [o for o in outs if o["role"] == "worker"]
    for o in workers:
        assert o["plane_ops"] == [steps * keys, steps * keys], o["plane_ops"]
        n = o["n"]
        ramp = torch.arange(0, n, n // 64, dtype=torch.float32) / n
        # per round: w -= 0.5 * (grad_0 + grad_1) / 2, grad_r = ramp * (r + 1) + k
        torch.testing.assert_close(o["v0"], -0.5 * steps * (1.5 * ramp), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(o["vlast"], -0.5 * steps * (1.5 * ramp + keys - 1), rtol=1e-5, atol=1e-5)
        steady = sorted(o["times"][1:])[len(o["times"][1:]) // 2]
        print(f"worker {o['rank']}: round of {keys} x {mb} MB push + pull: {steady * 1e3:.2f} ms "
              f"({steady * 1e3 / keys:.3f} ms per key push+pull, {2 * keys * mb / 1024 / steady:.1f} GB/s "
              f"moved per worker); all rounds {[round(t * 1e3, 2) for t in o['times']]}")


def test_kvstore_plane_async_pull_pull_never_torn():
    """Two plane pulls of one key in a row with no push between them: the second reply must
    not land in the landing area while the first is still being copied out -- worker 1 pushes all along,
    and every tensor worker 0 pulls is one whole version of the key."""
    port, rounds = _port(), 12
    args = [("scheduler", 0, 1, 2, port, rounds), ("server", 0, 1, 2, port, rounds),
            ("worker", 0, 1, 2, port, rounds), ("worker", 1, 1, 2, port, rounds)]
    ctx = mp.get_context("spawn")
    with ctx.Pool(len(args)) as pool:
        outs = [r.get(110) for r in [pool.apply_async(W.kv_pullpull_rank, a) for a in args]]
    puller = [o for o in outs if o.get("rank") == 0][0]
    assert puller["torn"] == 0, puller
    assert len(puller["ks"]) == 2 * rounds and puller["ks"] == sorted(puller["ks"]), puller["ks"]
    assert puller["plane_ops"][1] == 2 * rounds, puller["plane_ops"]
